// Max RoI pooling on channels-last features (Faster R-CNN, BigDL RoiPooling / Caffe ROIPooling
// semantics): each RoI (batch index, x1, y1, x2, y2 in image pixels) is scaled to the feature
// map with round(), split into pooled_h x pooled_w bins of fractional size, and each bin is
// max-reduced per channel (empty bin -> 0). The argmax (flat h*W+w) is kept for the backward,
// which scatters dy to it with fp32 atomics (bins of different RoIs can share a pixel).
//
// One thread per (roi, ph, pw, c) output element: c is fastest, so a wave reads 64 (or fewer)
// consecutive channels of one feature pixel -- coalesced NHWC rows.
//
// Reference: ObjectDetectionConfig.scala:38-46 (frcnn-vgg16 / frcnn-pvanet), BigDL
// nn.RoiPooling.
#include "common.h"

namespace zoo {

template <typename T>
ZOO_DEV float roi_ld(const T* p, size_t i);
template <>
ZOO_DEV float roi_ld<float>(const float* p, size_t i) { return p[i]; }
template <>
ZOO_DEV float roi_ld<bf16_t>(const bf16_t* p, size_t i) { return bf2f(p[i]); }

template <typename T>
__global__ void roi_pool_fwd_kernel(const T* __restrict__ f, const float* __restrict__ rois, T* __restrict__ out,
                                    int* __restrict__ argmax, int B, int R, int H, int W, int C, int PH, int PW,
                                    float scale) {
  const size_t n = (size_t)R * PH * PW * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int pw = (int)(t % PW);
    t /= PW;
    const int ph = (int)(t % PH);
    const int r = (int)(t / PH);
    const float* ro = rois + (size_t)r * 5;
    const int b = min(max((int)ro[0], 0), B - 1);   // never index outside the batch
    const int x1 = (int)roundf(ro[1] * scale), y1 = (int)roundf(ro[2] * scale);
    const int x2 = (int)roundf(ro[3] * scale), y2 = (int)roundf(ro[4] * scale);
    const int rw = max(x2 - x1 + 1, 1), rh = max(y2 - y1 + 1, 1);
    const float bw = (float)rw / PW, bh = (float)rh / PH;
    int hs = (int)floorf(ph * bh) + y1, he = (int)ceilf((ph + 1) * bh) + y1;
    int ws = (int)floorf(pw * bw) + x1, we = (int)ceilf((pw + 1) * bw) + x1;
    hs = min(max(hs, 0), H); he = min(max(he, 0), H);
    ws = min(max(ws, 0), W); we = min(max(we, 0), W);
    float best = 0.f;
    int arg = -1;
    if (hs < he && ws < we) {
      best = -3.4e38f;
      const T* fb = f + (size_t)b * H * W * C + c;
      for (int h = hs; h < he; ++h)
        for (int w = ws; w < we; ++w) {
          const float v = roi_ld(fb, ((size_t)h * W + w) * C);
          if (v > best) { best = v; arg = h * W + w; }
        }
    }
    if constexpr (sizeof(T) == 4) out[i] = best;
    else out[i] = f2bf(best);
    if (argmax) argmax[i] = arg;
  }
}

template <typename T>
__global__ void roi_pool_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ argmax,
                                    const float* __restrict__ rois, float* __restrict__ df, int B, int R, int H, int W,
                                    int C, int PH, int PW) {
  const size_t n = (size_t)R * PH * PW * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int a = argmax[i];
    if (a < 0) continue;
    const int c = (int)(i % C);
    const int r = (int)(i / ((size_t)C * PW * PH));
    const int b = min(max((int)rois[(size_t)r * 5], 0), B - 1);
    atomicAdd(df + ((size_t)b * H * W + a) * C + c, roi_ld(dy, i));
  }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_roi_pool(const void* f, const float* rois, void* out, int* argmax, const void* dy,
                                   float* df, int B, int R, int H, int W, int C, int PH, int PW, float scale, int backward,
                                   int bf16, hipStream_t st) {
  const size_t n = (size_t)R * PH * PW * C;
  const int g = (int)((n + 255) / 256 < 8192 ? ((n + 255) / 256 > 0 ? (n + 255) / 256 : 1) : 8192);
  if (!backward) {
    if (bf16)
      hipLaunchKernelGGL(roi_pool_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)f, rois,
                         (bf16_t*)out, argmax, B, R, H, W, C, PH, PW, scale);
    else
      hipLaunchKernelGGL(roi_pool_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)f, rois, (float*)out,
                         argmax, B, R, H, W, C, PH, PW, scale);
  } else {
    if (bf16)
      hipLaunchKernelGGL(roi_pool_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)dy, argmax, rois, df,
                         B, R, H, W, C, PH, PW);
    else
      hipLaunchKernelGGL(roi_pool_bwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)dy, argmax, rois, df, B,
                         R, H, W, C, PH, PW);
  }
  return hipGetLastError();
}
