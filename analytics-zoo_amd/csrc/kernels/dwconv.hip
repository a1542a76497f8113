// Depthwise convolution for NHWC bf16 activations on gfx950 (MobileNet v1/v2,
// separable convs): groups == channels, one R x S filter per channel.
//
// A depthwise conv does R*S MACs per output element, far too little work for
// the matrix cores: it is an HBM-streaming kernel. Every thread owns 8
// consecutive channels of one output pixel (16-byte loads of activations AND
// weights: the filter is stored tap-major [R*S][C], so the 8 channels of one
// tap are contiguous), accumulates in fp32 and fuses bias + activation.
//
//   fwd   y[n,p,q,c]  = act(sum_rs x[n, p*sh-ph+r, q*sw-pw+s, c] * w[r,s,c] + b[c])
//   dgrad dx[n,h,w,c] = sum over the taps that reach (h, w) (gather form: no atomics)
//   wgrad dw[r,s,c]  += sum_pixels dy * x  (per-thread register partials, wave shuffle fold,
//                        block fold in LDS, one deterministic partial row per block, then a
//                        column-sum kernel -- no global atomics)
//
// Reference: BigDL SpatialSeparableConvolution / SpatialConvolution(nGroup) behind
// Zs/pipeline/api/keras/layers/SeparableConvolution2D.scala and the MobileNet
// configs of ImageClassificationConfig.scala.
#include <stdlib.h>

#include "common.h"

namespace zoo {

struct DwGeom {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw;
};

__global__ __launch_bounds__(256) void dwconv_fwd_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                                                        const float* __restrict__ bias, bf16_t* __restrict__ Y,
                                                        DwGeom g, int act) {
  const int cpr = g.C >> 3;
  const size_t total = (size_t)g.N * g.P * g.Q * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % cpr);
    size_t t = i / cpr;
    const int q = (int)(t % g.Q); t /= g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = bias ? bias[chunk * 8 + e] : 0.f;
    const bf16_t* xb = X + (size_t)n * g.H * g.W * g.C + chunk * 8;
    for (int r = 0; r < g.R; ++r) {
      const int ih = p * g.sh - g.ph + r;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int s = 0; s < g.S; ++s) {
        const int iw = q * g.sw - g.pw + s;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float xv[8], wv[8];
        unpack8(*reinterpret_cast<const uint4*>(xb + ((size_t)ih * g.W + iw) * g.C), xv);
        unpack8(*reinterpret_cast<const uint4*>(Wt + (size_t)(r * g.S + s) * g.C + chunk * 8), wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += xv[e] * wv[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = apply_act(acc[e], act);
    *reinterpret_cast<uint4*>(Y + i * 8) = pack8(acc);
  }
}

__global__ __launch_bounds__(256) void dwconv_dgrad_kernel(const bf16_t* __restrict__ dY,
                                                          const bf16_t* __restrict__ Wt, bf16_t* __restrict__ dX,
                                                          DwGeom g) {
  const int cpr = g.C >> 3;
  const size_t total = (size_t)g.N * g.H * g.W * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % cpr);
    size_t t = i / cpr;
    const int w = (int)(t % g.W); t /= g.W;
    const int h = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const bf16_t* db = dY + (size_t)n * g.P * g.Q * g.C + chunk * 8;
    for (int r = 0; r < g.R; ++r) {
      const int ph = h + g.ph - r;  // = p * sh
      if (ph < 0 || ph % g.sh) continue;
      const int p = ph / g.sh;
      if (p >= g.P) continue;
      for (int s = 0; s < g.S; ++s) {
        const int qw = w + g.pw - s;
        if (qw < 0 || qw % g.sw) continue;
        const int q = qw / g.sw;
        if (q >= g.Q) continue;
        float dv[8], wv[8];
        unpack8(*reinterpret_cast<const uint4*>(db + ((size_t)p * g.Q + q) * g.C), dv);
        unpack8(*reinterpret_cast<const uint4*>(Wt + (size_t)(r * g.S + s) * g.C + chunk * 8), wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += dv[e] * wv[e];
      }
    }
    *reinterpret_cast<uint4*>(dX + i * 8) = pack8(acc);
  }
}

// wgrad: thread layout [row lane][chunk] over output pixels; RS_MAX taps in registers. Each
// block folds its waves' partial sums into an LDS [RS][C] accumulator and writes ONE
// deterministic partial row (no global atomics); dwconv_wgrad_reduce_kernel adds the rows.
template <int RS_MAX>
__global__ __launch_bounds__(256) void dwconv_wgrad_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                                                          float* __restrict__ partial, DwGeom g, int rows_per_block) {
  extern __shared__ __align__(16) float dw_red[];   // [RS][C]
  const int cpr = g.C >> 3;
  const int RS = g.R * g.S;
  for (int i = threadIdx.x; i < RS * g.C; i += 256) dw_red[i] = 0.f;
  __syncthreads();
  // chunk lanes per wave row: cpr rounded up to a power of two (<= 64) so that the lanes
  // sharing a chunk are a power-of-two stride apart for the shuffle fold; surplus lanes
  // carry zeros
  int lanes = 1;
  while (lanes < cpr && lanes < 64) lanes <<= 1;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rstep_w = 64 / lanes;          // pixel rows per wave step
  const int my_row = lane / lanes, ch0 = lane - my_row * lanes;
  const int M = g.N * g.P * g.Q;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const int nchunk_iter = (cpr + lanes - 1) / lanes;
  for (int it = 0; it < nchunk_iter; ++it) {
    const int chunk = ch0 + it * lanes;
    const bool cok = chunk < cpr;
    float acc[RS_MAX][8];
#pragma unroll
    for (int t = 0; t < RS_MAX; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
    for (int m = r0 + wid * rstep_w + my_row; cok && m < r1; m += 4 * rstep_w) {
      const int n = m / (g.P * g.Q);
      const int pq = m - n * g.P * g.Q;
      const int p = pq / g.Q, q = pq - (pq / g.Q) * g.Q;
      float dv[8];
      unpack8(*reinterpret_cast<const uint4*>(dY + (size_t)m * g.C + chunk * 8), dv);
      const bf16_t* xb = X + (size_t)n * g.H * g.W * g.C + chunk * 8;
#pragma unroll
      for (int t = 0; t < RS_MAX; ++t) {
        if (t >= RS) break;
        const int r = t / g.S, s = t - (t / g.S) * g.S;
        const int ih = p * g.sh - g.ph + r, iw = q * g.sw - g.pw + s;
        if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) continue;
        float xv[8];
        unpack8(*reinterpret_cast<const uint4*>(xb + ((size_t)ih * g.W + iw) * g.C), xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[t][e] += dv[e] * xv[e];
      }
    }
    // fold the wave's pixel rows (lanes with the same chunk are `lanes` apart), then the
    // block's waves in LDS (4 LDS atomics per value: the waves of the block)
#pragma unroll
    for (int t = 0; t < RS_MAX; ++t) {
      if (t >= RS) break;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = acc[t][e];
        for (int o = lanes; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
        acc[t][e] = v;
      }
      if (my_row == 0 && cok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(dw_red + t * g.C + chunk * 8 + e, acc[t][e]);
      }
    }
  }
  __syncthreads();
  float* dst = partial + (size_t)blockIdx.x * RS * g.C;
  for (int i = threadIdx.x; i < RS * g.C; i += 256) dst[i] = dw_red[i];
}

// 3x3 wgrad (every MobileNet / separable-conv layer), stride 1 or 2: a thread owns one 8-channel
// chunk and walks down an output column q over a segment of rows, keeping the 3 input rows its
// taps touch in registers as a sliding window (stride 1: one new row per output row, not 3 --
// the horizontal neighbours are the adjacent threads' loads, L1 hits), with the next row and
// dY prefetched while the current row's 72 FMAs run. Blocks = (chunk group of CB chunks) x
// (image, row segment); lanes of a wave that share a chunk fold by xor-shuffles, the 4 waves in
// fixed order through LDS, and each block writes its columns of ONE partial row per (image,
// segment): deterministic, no atomics. (The per-pixel-row kernel above divided every pixel index
// and reloaded all 9 taps: 2.1 ms of a 5.95 ms MobileNet-v1 b64 step,
// profiles/r3/mobilenet_train_b64_r3.md.)
constexpr int DW3_CBMAX = 32;

ZOO_DEV void dw3_unpack4(uint2 v, float* f) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}

// chunks here are 4 channels (8-byte loads): 36 fp32 accumulators + a 5-row window of packed
// bf16 keep the kernel at ~100 VGPRs (8-channel chunks needed 218 -> 2 waves / SIMD)
template <int SH>
__global__ __launch_bounds__(256) void dwconv_wgrad3_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                                                           float* __restrict__ partial, DwGeom g, int cb_log2,
                                                           int nseg, int rps) {
  __shared__ float red[4 * DW3_CBMAX * 36];
  const int CB = 1 << cb_log2;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cl = tid & (CB - 1), ql = tid >> cb_log2, qlanes = 256 >> cb_log2;
  const int cg = blockIdx.x, ns = blockIdx.y;
  const int n = ns / nseg, seg = ns - n * nseg;
  const int p0 = seg * rps, p1 = min(g.P, p0 + rps);
  const int chunk = cg * CB + cl;
  const bf16_t* xb = X + (size_t)n * g.H * g.W * g.C + chunk * 4;
  const bf16_t* db = dY + (size_t)n * g.P * g.Q * g.C + chunk * 4;
  const uint2 z2 = make_uint2(0, 0);
  float acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[t][e] = 0.f;

  for (int q = ql; q < g.Q; q += qlanes) {
    const int iw0 = q * SH - g.pw;
    const bool c0 = (unsigned)iw0 < (unsigned)g.W, c1 = (unsigned)(iw0 + 1) < (unsigned)g.W,
               c2 = (unsigned)(iw0 + 2) < (unsigned)g.W;
#define DW3_LD(IH, R)                                                                              \
  do {                                                                                             \
    const int ih_ = (IH);                                                                          \
    const bool rok_ = (unsigned)ih_ < (unsigned)g.H;                                               \
    const bf16_t* rp_ = xb + ((size_t)(rok_ ? ih_ : 0) * g.W + iw0) * g.C;                         \
    R[0] = (rok_ && c0) ? *reinterpret_cast<const uint2*>(rp_) : z2;                               \
    R[1] = (rok_ && c1) ? *reinterpret_cast<const uint2*>(rp_ + g.C) : z2;                         \
    R[2] = (rok_ && c2) ? *reinterpret_cast<const uint2*>(rp_ + 2 * g.C) : z2;                     \
  } while (0)
    uint2 w0[3], w1[3], w2[3], n1[3], n2[3];
    int ih = p0 * SH - g.ph;
    DW3_LD(ih, w0);
    DW3_LD(ih + 1, w1);
    DW3_LD(ih + 2, w2);
    uint2 dyv = *reinterpret_cast<const uint2*>(db + ((size_t)p0 * g.Q + q) * g.C);
    for (int p = p0; p < p1; ++p) {
      // prefetch the next output row's new input rows and dY
      const bool more = p + 1 < p1;
      uint2 ndy = z2;
      if (more) {
        if (SH == 1) {
          DW3_LD(ih + 3, n2);
        } else {
          DW3_LD(ih + 3, n1);
          DW3_LD(ih + 4, n2);
        }
        ndy = *reinterpret_cast<const uint2*>(db + ((size_t)(p + 1) * g.Q + q) * g.C);
      }
      float dv[4];
      dw3_unpack4(dyv, dv);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        float a[4], b[4], c[4];
        dw3_unpack4(w0[s], a);
        dw3_unpack4(w1[s], b);
        dw3_unpack4(w2[s], c);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[s][e] = fmaf(dv[e], a[e], acc[s][e]);
          acc[3 + s][e] = fmaf(dv[e], b[e], acc[3 + s][e]);
          acc[6 + s][e] = fmaf(dv[e], c[e], acc[6 + s][e]);
        }
      }
      if (more) {
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          if (SH == 1) {
            w0[s] = w1[s];
            w1[s] = w2[s];
            w2[s] = n2[s];
          } else {
            w0[s] = w2[s];
            w1[s] = n1[s];
            w2[s] = n2[s];
          }
        }
        dyv = ndy;
        ih += SH;
      }
    }
#undef DW3_LD
  }
  // lanes sharing a chunk are CB apart inside the wave: fixed xor tree, then lanes < CB
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = acc[t][e];
      for (int o = CB; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[t][e] = v;
    }
  if (lane < CB) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) red[(wv * DW3_CBMAX + lane) * 36 + t * 4 + e] = acc[t][e];
  }
  __syncthreads();
  float* dst = partial + (size_t)ns * 9 * g.C;
  for (int i = tid; i < CB * 36; i += 256) {
    const int c = i / 36, k = i - c * 36, t = k >> 2, e = k & 3;
    const float v = ((red[(0 * DW3_CBMAX + c) * 36 + k] + red[(1 * DW3_CBMAX + c) * 36 + k]) +
                     red[(2 * DW3_CBMAX + c) * 36 + k]) + red[(3 * DW3_CBMAX + c) * 36 + k];
    dst[t * g.C + (cg * CB + c) * 4 + e] = v;
  }
}

// dW[i] += sum over the nb partial rows (16 columns x 16 row slices per block)
__global__ __launch_bounds__(256) void dwconv_wgrad_reduce_kernel(const float* __restrict__ partial, int nb, int n,
                                                                 float* __restrict__ dW) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, part = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (col < n)
    for (int b = part; b < nb; b += 16) s += partial[(size_t)b * n + col];
  red[part][cl] = s;
  __syncthreads();
  if (part != 0 || col >= n) return;
#pragma unroll
  for (int k = 1; k < 16; ++k) s += red[k][cl];
  dW[col] += s;
}

static int dw_grid(size_t total) {
  const size_t b = (total + 255) / 256;
  return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_dwconv_fwd(const void* X, const void* W, const float* bias, void* Y, const int* gi, int act,
                                     hipStream_t st) {
  DwGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], gi[11]};
  const size_t total = (size_t)g.N * g.P * g.Q * (g.C / 8);
  hipLaunchKernelGGL(dwconv_fwd_kernel, dim3(dw_grid(total)), dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)W,
                     bias, (bf16_t*)Y, g, act);
  return hipGetLastError();
}

extern "C" hipError_t zoo_dwconv_dgrad(const void* dY, const void* W, void* dX, const int* gi, hipStream_t st) {
  DwGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], gi[11]};
  const size_t total = (size_t)g.N * g.H * g.W * (g.C / 8);
  hipLaunchKernelGGL(dwconv_dgrad_kernel, dim3(dw_grid(total)), dim3(256), 0, st, (const bf16_t*)dY,
                     (const bf16_t*)W, (bf16_t*)dX, g);
  return hipGetLastError();
}

// requires R*S <= 9 (the caller falls back otherwise). `partial` holds >= dwconv_wgrad_blocks()
// rows of R*S*C floats.
static int dw_wgrad_rpb(int M) {
  // <= 256 blocks (bounded partial buffer), >= 64 pixels per block
  int rpb = (M + 255) / 256;
  return rpb < 64 ? 64 : rpb;
}

struct Dw3Plan {
  bool ok;
  int cb_log2, nseg, rps;
};

static Dw3Plan dw3_plan(const DwGeom& g) {
  Dw3Plan pl{false, 0, 1, 1};
  static const bool on = true;
  if (!on || g.R != 3 || g.S != 3 || g.sh != g.sw || (g.sh != 1 && g.sh != 2) || g.C % 8) return pl;
  const int cpr = g.C / 4;                       // 4-channel chunks
  int qlt = 1;                                   // q lanes wanted: the row width, <= 32
  while (qlt < g.Q && qlt < 32) qlt <<= 1;
  int cb = 256 / qlt;
  int cbmax = 1;                                 // largest power of two dividing cpr
  while (cbmax < DW3_CBMAX && cpr % (cbmax * 2) == 0) cbmax <<= 1;
  if (cb > cbmax) cb = cbmax;
  int l2 = 0;
  while ((1 << l2) < cb) ++l2;
  const int groups = (cpr / cb) * g.N;
  int nseg = (2048 + groups - 1) / groups;       // ~2048 blocks
  if (nseg > g.P) nseg = g.P;
  if (nseg < 1) nseg = 1;
  const int rps = (g.P + nseg - 1) / nseg;
  pl.ok = true;
  pl.cb_log2 = l2;
  pl.rps = rps;
  pl.nseg = (g.P + rps - 1) / rps;
  return pl;
}

extern "C" int zoo_dwconv_wgrad_blocks(const int* gi) {
  DwGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], gi[11]};
  const Dw3Plan pl = dw3_plan(g);
  if (pl.ok) return g.N * pl.nseg;
  const int M = gi[0] * gi[4] * gi[5];
  const int rpb = dw_wgrad_rpb(M);
  return (M + rpb - 1) / rpb;
}

extern "C" hipError_t zoo_dwconv_wgrad(const void* X, const void* dY, float* dW, float* partial, const int* gi,
                                       hipStream_t st) {
  DwGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], gi[11]};
  const Dw3Plan pl = dw3_plan(g);
  if (pl.ok) {
    const dim3 grid(g.C / 4 >> pl.cb_log2, g.N * pl.nseg);
    if (g.sh == 1)
      hipLaunchKernelGGL(dwconv_wgrad3_kernel<1>, grid, dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)dY, partial,
                         g, pl.cb_log2, pl.nseg, pl.rps);
    else
      hipLaunchKernelGGL(dwconv_wgrad3_kernel<2>, grid, dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)dY, partial,
                         g, pl.cb_log2, pl.nseg, pl.rps);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int n = 9 * g.C;
    hipLaunchKernelGGL(dwconv_wgrad_reduce_kernel, dim3((n + 15) / 16), dim3(256), 0, st, partial, g.N * pl.nseg, n,
                       dW);
    return hipGetLastError();
  }
  const int M = g.N * g.P * g.Q;
  const int rpb = dw_wgrad_rpb(M);
  const int blocks = (M + rpb - 1) / rpb;
  const int n = g.R * g.S * g.C;
  const size_t lds = (size_t)n * 4;
  if (lds > 160 * 1024) return hipErrorInvalidValue;
#define ZOO_DW_WG(RSM)                                                                                        \
  do {                                                                                                       \
    auto k = &dwconv_wgrad_kernel<RSM>;                                                                      \
    if (lds > 64 * 1024)                                                                                     \
      hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, st, (const bf16_t*)X, (const bf16_t*)dY, partial, g, rpb); \
  } while (0)
  if (g.R * g.S <= 1) ZOO_DW_WG(1);
  else if (g.R * g.S <= 4) ZOO_DW_WG(4);
  else ZOO_DW_WG(9);
#undef ZOO_DW_WG
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(dwconv_wgrad_reduce_kernel, dim3((n + 15) / 16), dim3(256), 0, st, partial, blocks, n, dW);
  return hipGetLastError();
}
