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

// ---------------------------------------------------------------------------
// SSD / MultiBox ground-truth matching (MultiBoxLoss.scala matching; BboxUtil IoU):
// per image, every prior takes its best-IoU ground truth; every ground truth claims
// its best prior (ties -> lowest prior index, as argmax); claimed priors are forced
// positive (the last claiming ground truth wins, as sequential assignment); priors
// below `overlap` become background. Outputs the encoded regression targets and labels.
//   gt   [B, G, 5] (label, x1, y1, x2, y2), rows >= count[b] ignored
//   priors [P, 4] centre-size; loc_t [B, P, 4]; conf_t [B, P] (int64)
// ---------------------------------------------------------------------------
namespace zoo {

ZOO_DEV float box_iou(float ax1, float ay1, float ax2, float ay2, float bx1, float by1, float bx2, float by2) {
  const float iw = fmaxf(fminf(ax2, bx2) - fmaxf(ax1, bx1), 0.f);
  const float ih = fmaxf(fminf(ay2, by2) - fmaxf(ay1, by1), 0.f);
  const float inter = iw * ih;
  const float u = (ax2 - ax1) * (ay2 - ay1) + (bx2 - bx1) * (by2 - by1) - inter;
  return inter / fmaxf(u, 1e-12f);
}

__global__ __launch_bounds__(256) void ssd_match_iou_kernel(const float* __restrict__ gt, const int* __restrict__ count,
                                                            const float4* __restrict__ priors, int G, int P,
                                                            int* __restrict__ best_gt, float* __restrict__ best_iou,
                                                            unsigned long long* __restrict__ gt_best) {
  const int b = blockIdx.y, p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const float4 pr = priors[p];
  const float px1 = pr.x - pr.z * 0.5f, py1 = pr.y - pr.w * 0.5f, px2 = pr.x + pr.z * 0.5f,
              py2 = pr.y + pr.w * 0.5f;
  const int n = count[b];
  float bi = -1.f;
  int bg = 0;
  for (int g = 0; g < n; ++g) {
    const float* r = gt + ((size_t)b * G + g) * 5;
    const float iou = box_iou(r[1], r[2], r[3], r[4], px1, py1, px2, py2);
    if (iou > bi) { bi = iou; bg = g; }
    // per-gt argmax over priors: max IoU, then the lowest prior index
    const unsigned long long key = ((unsigned long long)__float_as_uint(fmaxf(iou, 0.f)) << 32) |
                                   (unsigned long long)(0xFFFFFFFFu - (unsigned)p);
    atomicMax(gt_best + (size_t)b * G + g, key);
  }
  best_gt[(size_t)b * P + p] = bg;
  best_iou[(size_t)b * P + p] = bi;
}

__global__ __launch_bounds__(256) void ssd_match_encode_kernel(
    const float* __restrict__ gt, const int* __restrict__ count, const float4* __restrict__ priors, int G, int P,
    const int* __restrict__ best_gt, const float* __restrict__ best_iou,
    const unsigned long long* __restrict__ gt_best, float overlap, float v0, float v1, int bg_label,
    float* __restrict__ loc_t, long long* __restrict__ conf_t) {
  const int b = blockIdx.y, p = blockIdx.x * 256 + threadIdx.x;
  if (p >= P) return;
  const int n = count[b];
  int g = best_gt[(size_t)b * P + p];
  float iou = best_iou[(size_t)b * P + p];
  for (int k = 0; k < n; ++k) {
    const unsigned bp = 0xFFFFFFFFu - (unsigned)(gt_best[(size_t)b * G + k] & 0xFFFFFFFFull);
    if ((int)bp == p) { g = k; iou = 2.f; }
  }
  float4* lt = reinterpret_cast<float4*>(loc_t) + (size_t)b * P + p;
  if (n == 0) {
    *lt = make_float4(0.f, 0.f, 0.f, 0.f);
    conf_t[(size_t)b * P + p] = bg_label;
    return;
  }
  const float* r = gt + ((size_t)b * G + g) * 5;
  const float4 pr = priors[p];
  const float cx = (r[1] + r[3]) * 0.5f, cy = (r[2] + r[4]) * 0.5f;
  const float w = fmaxf(r[3] - r[1], 1e-12f), h = fmaxf(r[4] - r[2], 1e-12f);
  *lt = make_float4((cx - pr.x) / (pr.z * v0), (cy - pr.y) / (pr.w * v0), __logf(w / pr.z) / v1,
                    __logf(h / pr.w) / v1);
  conf_t[(size_t)b * P + p] = iou < overlap ? bg_label : (long long)r[0];
}

}  // namespace zoo

extern "C" hipError_t zoo_ssd_match(const float* gt, const int* count, const float* priors, int B, int G, int P,
                                    float overlap, float v0, float v1, int bg_label, int* best_gt, float* best_iou,
                                    unsigned long long* gt_best, float* loc_t, long long* conf_t, hipStream_t st) {
  using namespace zoo;
  const dim3 grid((P + 255) / 256, B);
  hipMemsetAsync(gt_best, 0, (size_t)B * G * sizeof(unsigned long long), st);
  hipLaunchKernelGGL(ssd_match_iou_kernel, grid, dim3(256), 0, st, gt, count, (const float4*)priors, G, P, best_gt,
                     best_iou, gt_best);
  hipLaunchKernelGGL(ssd_match_encode_kernel, grid, dim3(256), 0, st, gt, count, (const float4*)priors, G, P,
                     best_gt, best_iou, gt_best, overlap, v0, v1, bg_label, loc_t, conf_t);
  return hipGetLastError();
}
