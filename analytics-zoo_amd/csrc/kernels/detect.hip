// Detection kernels: IoU suppression bitmask for greedy NMS.
//
// Boxes arrive sorted by descending score. Block (rb, cb) holds 64 "row" boxes
// of tile rb and compares each with the 64 "column" boxes of tile cb (staged in
// LDS); lane i sets bit j of mask[row][cb] when IoU(row, col) > threshold and
// col > row. The greedy pass over the bitmask (O(N * N/64) word ops) runs on
// the host in ops.cpp. Replaces the DetectionOutputSSD / Proposal NMS of the
// reference (BigDL Nms, used by SSDGraph.scala:193-215 and FRCNN's Proposal).
#include "common.h"

namespace zoo {

constexpr int NMS_T = 64;

ZOO_DEV float iou4(const float4 a, const float4 b) {
  const float ix1 = fmaxf(a.x, b.x), iy1 = fmaxf(a.y, b.y);
  const float ix2 = fminf(a.z, b.z), iy2 = fminf(a.w, b.w);
  const float iw = fmaxf(ix2 - ix1, 0.f), ih = fmaxf(iy2 - iy1, 0.f);
  const float inter = iw * ih;
  const float ua = fmaxf(a.z - a.x, 0.f) * fmaxf(a.w - a.y, 0.f) + fmaxf(b.z - b.x, 0.f) * fmaxf(b.w - b.y, 0.f) -
                   inter;
  return ua > 0.f ? inter / ua : 0.f;
}

__global__ __launch_bounds__(NMS_T) void nms_mask_kernel(const float4* __restrict__ boxes, int n, float thresh,
                                                         unsigned long long* __restrict__ mask, int words) {
  const int rb = blockIdx.y, cb = blockIdx.x;
  if (cb < rb) return;  // only columns at or after the row tile can be suppressed
  __shared__ float4 cols[NMS_T];
  const int c0 = cb * NMS_T;
  const int ncol = min(NMS_T, n - c0);
  if ((int)threadIdx.x < ncol) cols[threadIdx.x] = boxes[c0 + threadIdx.x];
  __syncthreads();
  const int row = rb * NMS_T + threadIdx.x;
  if (row >= n) return;
  const float4 me = boxes[row];
  unsigned long long bits = 0ull;
  const int j0 = cb == rb ? (int)threadIdx.x + 1 : 0;
  for (int j = j0; j < ncol; ++j)
    if (iou4(me, cols[j]) > thresh) bits |= 1ull << j;
  mask[(size_t)row * words + cb] = bits;
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_nms_mask(const float* boxes, int n, float thresh, unsigned long long* mask,
                                   hipStream_t st) {
  const int words = (n + NMS_T - 1) / NMS_T;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(nms_mask_kernel, dim3(words, words), dim3(NMS_T), 0, st,
                     reinterpret_cast<const float4*>(boxes), n, thresh, mask, words);
  return hipGetLastError();
}
