// Fused image preprocessing for serving / ImageSet pipelines:
//   uint8 HWC (decoded JPEG/PNG, BGR or RGB) -> bilinear resize (OpenCV
//   INTER_LINEAR pixel-centre convention) -> per-channel (x - mean) / std ->
//   layout change (NCHW fp32, or the NHWC-padded-to-4 bf16 image the ResNet stem
//   conv consumes) in ONE pass over the source pixels.
//
// Replaces the reference's OpenCV JNI resize / toFloatPixels / transpose chain
// (Zs/serving/PreProcessing.scala:24-53, Zs/feature/image/ImageResize.scala,
// ImageChannelNormalize, ImageMatToTensor; SURVEY.md §2.13 "OpenCV JNI").
#include "common.h"

namespace zoo {

// one thread per output pixel; all channels of that pixel
template <int LAYOUT>  // 0: NCHW fp32, 1: NHWC4 bf16 (channels padded to 4 with zeros)
__global__ void resize_normalize_kernel(const uint8_t* __restrict__ in, void* __restrict__ out, int N, int Hi,
                                        int Wi, int C, int Ho, int Wo, float m0, float m1, float m2, float s0,
                                        float s1, float s2, int swap_rb) {
  const long total = (long)N * Ho * Wo;
  const float sy = (float)Hi / Ho, sx = (float)Wi / Wo;
  const float mean[3] = {m0, m1, m2};
  const float inv[3] = {1.f / s0, 1.f / s1, 1.f / s2};
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int x = idx % Wo;
    const int y = (idx / Wo) % Ho;
    const int n = idx / ((long)Wo * Ho);
    float fy = (y + 0.5f) * sy - 0.5f, fx = (x + 0.5f) * sx - 0.5f;
    fy = fminf(fmaxf(fy, 0.f), (float)(Hi - 1));
    fx = fminf(fmaxf(fx, 0.f), (float)(Wi - 1));
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = min(y0 + 1, Hi - 1), x1 = min(x0 + 1, Wi - 1);
    const float wy = fy - y0, wx = fx - x0;
    const uint8_t* base = in + (size_t)n * Hi * Wi * C;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C && c < 4; ++c) {
      const float p00 = base[((size_t)y0 * Wi + x0) * C + c], p01 = base[((size_t)y0 * Wi + x1) * C + c];
      const float p10 = base[((size_t)y1 * Wi + x0) * C + c], p11 = base[((size_t)y1 * Wi + x1) * C + c];
      const float top = p00 + (p01 - p00) * wx, bot = p10 + (p11 - p10) * wx;
      const int oc = (swap_rb && C >= 3 && c < 3) ? 2 - c : c;
      const float val = top + (bot - top) * wy;
      v[oc] = oc < 3 ? (val - mean[oc]) * inv[oc] : val;
    }
    if constexpr (LAYOUT == 0) {
      float* o = reinterpret_cast<float*>(out);
      for (int c = 0; c < C && c < 4; ++c) o[(((size_t)n * C + c) * Ho + y) * Wo + x] = v[c];
    } else {
      uint2 pk;
      pk.x = pack2bf(v[0], C > 1 ? v[1] : 0.f);
      pk.y = pack2bf(C > 2 ? v[2] : 0.f, C > 3 ? v[3] : 0.f);
      reinterpret_cast<uint2*>(out)[((size_t)n * Ho + y) * Wo + x] = pk;
    }
  }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_resize_normalize(const void* in, void* out, int N, int Hi, int Wi, int C, int Ho, int Wo,
                                           const float* mean, const float* stdv, int swap_rb, int layout,
                                           hipStream_t st) {
  const long total = (long)N * Ho * Wo;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
  if (layout == 0)
    hipLaunchKernelGGL(resize_normalize_kernel<0>, dim3(blocks), dim3(256), 0, st, (const uint8_t*)in, out, N, Hi, Wi,
                       C, Ho, Wo, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2], swap_rb);
  else
    hipLaunchKernelGGL(resize_normalize_kernel<1>, dim3(blocks), dim3(256), 0, st, (const uint8_t*)in, out, N, Hi, Wi,
                       C, Ho, Wo, mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2], swap_rb);
  return hipGetLastError();
}
