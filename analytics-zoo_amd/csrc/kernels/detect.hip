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

// ---- hard negative mining (MultiBoxLoss.scala: 3:1 negatives by confidence loss) ----------
// One 1024-thread block per image. k = ceil(ratio * #positives) (<= P - 1) priors with the
// largest loss among neg_ce (= ce, 0 on positives) are selected: the exact k-th largest value by
// a 4-pass 8-bit MSB-first radix select over the loss bits (losses are >= 0, so their bit
// patterns order like the values), then every prior above it plus the first (by prior index)
// ones equal to it. Output: pos | neg as a byte mask. Replaces argsort(argsort()) ranking.
constexpr int MINE_T = 1024;

__global__ __launch_bounds__(MINE_T) void ssd_mine_kernel(const float* __restrict__ ce,
                                                         const long long* __restrict__ conf_t, int P, int bg,
                                                         float ratio, unsigned char* __restrict__ sel) {
  __shared__ unsigned hist[256];
  __shared__ unsigned s_prefix, s_mask;
  __shared__ int s_npos, s_rem, s_base;
  __shared__ int scan[MINE_T];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* c = ce + (size_t)b * P;
  const long long* lab = conf_t + (size_t)b * P;
  unsigned char* out = sel + (size_t)b * P;
  if (tid == 0) { s_npos = 0; s_prefix = 0u; s_mask = 0u; }
  __syncthreads();
  int np = 0;
  for (int p = tid; p < P; p += MINE_T) np += lab[p] != bg;
  atomicAdd(&s_npos, np);
  __syncthreads();
  int k = (int)ceilf(ratio * (float)s_npos);
  if (k > P - 1) k = P - 1;
  if (k <= 0) {
    for (int p = tid; p < P; p += MINE_T) out[p] = lab[p] != bg;
    return;
  }
  if (tid == 0) s_rem = k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = tid; i < 256; i += MINE_T) hist[i] = 0u;
    __syncthreads();
    const unsigned pre = s_prefix, msk = s_mask;
    for (int p = tid; p < P; p += MINE_T) {
      const float v = lab[p] != bg ? 0.f : fmaxf(c[p], 0.f);
      const unsigned u = __float_as_uint(v);
      if ((u & msk) == pre) atomicAdd(&hist[(u >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int rem = s_rem, d = 255;
      for (; d > 0; --d) {
        if ((int)hist[d] >= rem) break;
        rem -= (int)hist[d];
      }
      s_rem = rem;
      s_prefix = pre | ((unsigned)d << shift);
      s_mask = msk | (255u << shift);
    }
    __syncthreads();
  }
  const unsigned thr = s_prefix;
  const int need_eq = s_rem;          // ties at the threshold still to take, lowest prior index first
  if (tid == 0) s_base = 0;
  __syncthreads();
  for (int p0 = 0; p0 < P; p0 += MINE_T) {
    const int p = p0 + tid;
    bool pos = false, gt = false, eq = false;
    if (p < P) {
      pos = lab[p] != bg;
      const unsigned u = __float_as_uint(pos ? 0.f : fmaxf(c[p], 0.f));
      gt = u > thr;
      eq = u == thr;
    }
    scan[tid] = eq ? 1 : 0;
    __syncthreads();
    for (int off = 1; off < MINE_T; off <<= 1) {       // inclusive Hillis-Steele scan
      const int v = tid >= off ? scan[tid - off] : 0;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    const int before = s_base + scan[tid] - (eq ? 1 : 0);
    if (p < P) out[p] = (pos || gt || (eq && before < need_eq)) ? 1 : 0;
    __syncthreads();
    if (tid == MINE_T - 1) s_base += scan[tid];
    __syncthreads();
  }
}

// ---- SSD conv4_3 NormalizeScale: y = x / (||x||_2 + eps) * w over the channels (NHWC) ------
// one wave per row, 8-channel bf16 chunks (C % 8 == 0); the backward folds dw per block into a
// partial row (fixed-order column sums afterwards: deterministic)
__global__ __launch_bounds__(256) void l2norm_scale_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                               bf16_t* __restrict__ y, float* __restrict__ rn, long R,
                                                               int C, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int cpr = C >> 3;
  const bf16_t* xr = x + row * C;
  float s = 0.f;
  for (int ch = lane; ch < cpr; ch += 64) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + ch * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s = fmaf(v[e], v[e], s);
  }
  s = warp_sum(s);
  const float n = sqrtf(s) + eps;
  const float inv = 1.f / n;
  if (lane == 0) rn[row] = n;
  for (int ch = lane; ch < cpr; ch += 64) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + ch * 8), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] * inv * w[ch * 8 + e];
    *reinterpret_cast<uint4*>(y + row * C + ch * 8) = pack8(v);
  }
}

__global__ __launch_bounds__(256) void l2norm_scale_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                               const float* __restrict__ w, const float* __restrict__ rn,
                                                               bf16_t* __restrict__ dx, float* __restrict__ dwp, long R,
                                                               int C, float eps, int rows_per_block) {
  extern __shared__ float l2_dw[];          // [4 waves][C]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int cpr = C >> 3;
  for (int i = threadIdx.x; i < 4 * C; i += 256) l2_dw[i] = 0.f;
  __syncthreads();
  const long r0 = (long)blockIdx.x * rows_per_block;
  const long r1 = r0 + rows_per_block < R ? r0 + rows_per_block : R;
  for (long row = r0 + wv; row < r1; row += 4) {
    const bf16_t* xr = x + row * C;
    const bf16_t* dr = dy + row * C;
    const float n = rn[row], inv = 1.f / n, sq = n - eps;
    float dot = 0.f;
    for (int ch = lane; ch < cpr; ch += 64) {
      float xv[8], dv[8];
      unpack8(*reinterpret_cast<const uint4*>(xr + ch * 8), xv);
      unpack8(*reinterpret_cast<const uint4*>(dr + ch * 8), dv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dot = fmaf(w[ch * 8 + e] * dv[e], xv[e], dot);
        l2_dw[wv * C + ch * 8 + e] += dv[e] * xv[e] * inv;     // this wave's lanes own disjoint columns
      }
    }
    dot = warp_sum(dot);
    const float k = sq > 0.f ? dot / (n * n * sq) : 0.f;
    for (int ch = lane; ch < cpr; ch += 64) {
      float xv[8], dv[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(xr + ch * 8), xv);
      unpack8(*reinterpret_cast<const uint4*>(dr + ch * 8), dv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = w[ch * 8 + e] * dv[e] * inv - xv[e] * k;
      *reinterpret_cast<uint4*>(dx + row * C + ch * 8) = pack8(o);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += 256)
    dwp[(size_t)blockIdx.x * C + i] = ((l2_dw[i] + l2_dw[C + i]) + l2_dw[2 * C + i]) + l2_dw[3 * C + i];
}

__global__ __launch_bounds__(256) void colsum_rows_kernel(const float* __restrict__ part, int nb, int n,
                                                          float* __restrict__ out) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= n) return;
  float s = 0.f;
  for (int b = 0; b < nb; ++b) s += part[(size_t)b * n + col];
  out[col] += s;
}

}  // namespace zoo

extern "C" hipError_t zoo_ssd_mine(const float* ce, const long long* conf_t, int B, int P, int bg, float ratio,
                                   unsigned char* sel, hipStream_t st) {
  hipLaunchKernelGGL(zoo::ssd_mine_kernel, dim3(B), dim3(zoo::MINE_T), 0, st, ce, conf_t, P, bg, ratio, sel);
  return hipGetLastError();
}

extern "C" hipError_t zoo_l2norm_scale_fwd(const void* x, const float* w, void* y, float* rn, long R, int C, float eps,
                                           hipStream_t st) {
  const long blocks = (R + 3) / 4;
  hipLaunchKernelGGL(zoo::l2norm_scale_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const zoo::bf16_t*)x, w,
                     (zoo::bf16_t*)y, rn, R, C, eps);
  return hipGetLastError();
}

extern "C" int zoo_l2norm_scale_bwd_blocks(long R) {
  long rpb = (R + 511) / 512;
  if (rpb < 16) rpb = 16;
  return (int)((R + rpb - 1) / rpb);
}

// dw (fp32 [C]) += sum over rows; part: zoo_l2norm_scale_bwd_blocks(R) x C floats
extern "C" hipError_t zoo_l2norm_scale_bwd(const void* dy, const void* x, const float* w, const float* rn, void* dx,
                                           float* dw, float* part, long R, int C, float eps, hipStream_t st) {
  const int nb = zoo_l2norm_scale_bwd_blocks(R);
  const int rpb = (int)((R + nb - 1) / nb);
  const size_t lds = (size_t)4 * C * sizeof(float);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(zoo::l2norm_scale_bwd_kernel, dim3(nb), dim3(256), lds, st, (const zoo::bf16_t*)dy,
                     (const zoo::bf16_t*)x, w, rn, (zoo::bf16_t*)dx, part, R, C, eps, rpb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(zoo::colsum_rows_kernel, dim3((C + 255) / 256), dim3(256), 0, st, part, nb, C, dw);
  return hipGetLastError();
}

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
