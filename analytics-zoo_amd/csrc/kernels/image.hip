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
#include "geom.h"

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

// ---------------------------------------------------------------------------------------------
// GPU half of the JPEG decoder (host half: csrc/runtime/jpeg.cpp, entropy decode only).
//
// jpeg_idct_kernel: dequantise + 8x8 inverse DCT of every block of every component of the
// batch -> uint8 component planes. One 64-lane wave per 8x8 block (lane = output pixel), the
// separable transform as two 8-tap passes through LDS, 4 blocks per workgroup.

__constant__ float kIdct[64];   // kIdct[x * 8 + u] = C(u) / 2 * cos((2x + 1) u pi / 16)

__global__ __launch_bounds__(256) void jpeg_idct_kernel(const int16_t* __restrict__ coef,
                                                        const int32_t* __restrict__ qt,
                                                        uint8_t* __restrict__ planes, JpegGeom g) {
  __shared__ float t[4][64];
  __shared__ float f[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long blk = (long)blockIdx.x * 4 + w;
  const long nblk = (long)g.N * g.total;
  const bool ok = blk < nblk;
  const int img = ok ? (int)(blk / g.total) : 0;
  const int b = ok ? (int)(blk - (long)img * g.total) : 0;
  int c = 0;
  if (g.ncomp > 1 && b >= g.boff[1]) c = 1;
  if (g.ncomp > 2 && b >= g.boff[2]) c = 2;
  const int y = lane >> 3, x = lane & 7;
  if (ok) f[w][lane] = (float)coef[blk * 64 + lane] * (float)qt[((long)img * g.ncomp + c) * 64 + lane];
  __syncthreads();
  // rows: t[v][x] = sum_u F[v][u] M[x][u]   (lane = v * 8 + x)
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) s = fmaf(f[w][y * 8 + u], kIdct[x * 8 + u], s);
  t[w][lane] = s;
  __syncthreads();
  // columns: out[y][x] = sum_v M[y][v] t[v][x]
  s = 0.f;
#pragma unroll
  for (int v = 0; v < 8; ++v) s = fmaf(kIdct[y * 8 + v], t[w][v * 8 + x], s);
  if (!ok) return;
  const int lb = b - g.boff[c];
  const int by = lb / g.bw[c], bx = lb - by * g.bw[c];
  const int pitch = g.bw[c] * 8;
  const long plane = ((long)img * g.total + g.boff[c]) * 64;   // pixels of the component plane start
  const float v = fminf(fmaxf(rintf(s + 128.f), 0.f), 255.f);
  planes[plane + (long)(by * 8 + y) * pitch + bx * 8 + x] = (uint8_t)v;
}

// One source pixel of the decoded image: Y, chroma upsampled with the triangle ("fancy")
// filter -- bilinear at the co-sited chroma position -- then YCbCr -> RGB (JFIF), rounded.
ZOO_DEV void jpeg_rgb(const uint8_t* __restrict__ planes, const JpegGeom& g, long img_base, int sx, int sy,
                      float* rgb) {
  const uint8_t* yp = planes + img_base + (long)g.boff[0] * 64;
  const float Y = yp[(long)sy * g.bw[0] * 8 + sx];
  if (g.ncomp == 1) {
    rgb[0] = rgb[1] = rgb[2] = Y;
    return;
  }
  float cc[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int c = k + 1;
    const uint8_t* cp = planes + img_base + (long)g.boff[c] * 64;
    const int pitch = g.bw[c] * 8;
    const int cw = (g.w * g.hs[c] + g.hmax - 1) / g.hmax, ch = (g.h * g.vs[c] + g.vmax - 1) / g.vmax;
    float fx = (sx + 0.5f) * g.hs[c] / g.hmax - 0.5f, fy = (sy + 0.5f) * g.vs[c] / g.vmax - 0.5f;
    fx = fminf(fmaxf(fx, 0.f), (float)(cw - 1));
    fy = fminf(fmaxf(fy, 0.f), (float)(ch - 1));
    const int x0 = (int)fx, y0 = (int)fy;
    const int x1 = min(x0 + 1, cw - 1), y1 = min(y0 + 1, ch - 1);
    const float wx = fx - x0, wy = fy - y0;
    const float a = cp[(long)y0 * pitch + x0], bb = cp[(long)y0 * pitch + x1];
    const float d = cp[(long)y1 * pitch + x0], e = cp[(long)y1 * pitch + x1];
    const float top = a + (bb - a) * wx, bot = d + (e - d) * wx;
    cc[k] = rintf(top + (bot - top) * wy);
  }
  const float cb = cc[0] - 128.f, cr = cc[1] - 128.f;
  rgb[0] = fminf(fmaxf(rintf(Y + 1.402f * cr), 0.f), 255.f);
  rgb[1] = fminf(fmaxf(rintf(Y - 0.344136286f * cb - 0.714136286f * cr), 0.f), 255.f);
  rgb[2] = fminf(fmaxf(rintf(Y + 1.772f * cb), 0.f), 255.f);
}

// decoded planes -> bilinear resize (OpenCV pixel-centre convention, as resize_normalize) ->
// (x - mean) / std -> NCHW fp32 or NHWC4 bf16; the RGB image itself is never written
template <int LAYOUT>
__global__ void jpeg_color_resize_kernel(const uint8_t* __restrict__ planes, void* __restrict__ out, JpegGeom g,
                                         int Ho, int Wo, float m0, float m1, float m2, float s0, float s1,
                                         float s2, int swap_rb) {
  const long total = (long)g.N * Ho * Wo;
  const float sy = (float)g.h / Ho, sx = (float)g.w / Wo;
  const float mean[3] = {m0, m1, m2};
  const float inv[3] = {1.f / s0, 1.f / s1, 1.f / s2};
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int x = idx % Wo;
    const int y = (idx / Wo) % Ho;
    const int n = idx / ((long)Wo * Ho);
    float fy = (y + 0.5f) * sy - 0.5f, fx = (x + 0.5f) * sx - 0.5f;
    fy = fminf(fmaxf(fy, 0.f), (float)(g.h - 1));
    fx = fminf(fmaxf(fx, 0.f), (float)(g.w - 1));
    const int y0 = (int)fy, x0 = (int)fx;
    const int y1 = min(y0 + 1, g.h - 1), x1 = min(x0 + 1, g.w - 1);
    const float wy = fy - y0, wx = fx - x0;
    const long base = (long)n * g.total * 64;
    float p00[3], p01[3], p10[3], p11[3];
    jpeg_rgb(planes, g, base, x0, y0, p00);
    jpeg_rgb(planes, g, base, x1, y0, p01);
    jpeg_rgb(planes, g, base, x0, y1, p10);
    jpeg_rgb(planes, g, base, x1, y1, p11);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float top = p00[c] + (p01[c] - p00[c]) * wx, bot = p10[c] + (p11[c] - p10[c]) * wx;
      const int oc = swap_rb ? 2 - c : c;
      v[oc] = (top + (bot - top) * wy - mean[oc]) * inv[oc];
    }
    if constexpr (LAYOUT == 0) {
      float* o = reinterpret_cast<float*>(out);
#pragma unroll
      for (int c = 0; c < 3; ++c) o[(((size_t)n * 3 + c) * Ho + y) * Wo + x] = v[c];
    } else if constexpr (LAYOUT == 1) {
      uint2 pk;
      pk.x = pack2bf(v[0], v[1]);
      pk.y = pack2bf(v[2], 0.f);
      reinterpret_cast<uint2*>(out)[((size_t)n * Ho + y) * Wo + x] = pk;
    } else {   // 2: plain decoded RGB uint8 HWC (Ho == h, Wo == w: no resize, no normalise)
      uint8_t* o = reinterpret_cast<uint8_t*>(out) + (((size_t)n * Ho + y) * Wo + x) * 3;
      o[0] = (uint8_t)p00[0];
      o[1] = (uint8_t)p00[1];
      o[2] = (uint8_t)p00[2];
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

static bool g_idct_ready = false;

extern "C" hipError_t zoo_jpeg_idct(const int16_t* coef, const int32_t* qt, uint8_t* planes, const JpegGeom* g,
                                    hipStream_t st) {
  if (!g_idct_ready) {
    float m[64];
    for (int x = 0; x < 8; ++x)
      for (int u = 0; u < 8; ++u)
        m[x * 8 + u] = (u == 0 ? 0.70710678118654752f : 1.f) * 0.5f * cosf((2 * x + 1) * u * 3.14159265358979f / 16.f);
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(kIdct), m, sizeof(m));
    if (e != hipSuccess) return e;
    g_idct_ready = true;
  }
  const long nblk = (long)g->N * g->total;
  if (nblk <= 0) return hipSuccess;
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((unsigned)((nblk + 3) / 4)), dim3(256), 0, st, coef, qt, planes, *g);
  return hipGetLastError();
}

extern "C" hipError_t zoo_jpeg_color_resize(const uint8_t* planes, void* out, const JpegGeom* g, int Ho, int Wo,
                                            const float* mean, const float* stdv, int swap_rb, int layout,
                                            hipStream_t st) {
  const long total = (long)g->N * Ho * Wo;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65536) blocks = 65536;
  if (blocks < 1) blocks = 1;
#define ZOO_JCR(L)                                                                                           \
  hipLaunchKernelGGL(jpeg_color_resize_kernel<L>, dim3(blocks), dim3(256), 0, st, planes, out, *g, Ho, Wo,   \
                     mean[0], mean[1], mean[2], stdv[0], stdv[1], stdv[2], swap_rb)
  if (layout == 0) ZOO_JCR(0);
  else if (layout == 1) ZOO_JCR(1);
  else ZOO_JCR(2);
#undef ZOO_JCR
  return hipGetLastError();
}
