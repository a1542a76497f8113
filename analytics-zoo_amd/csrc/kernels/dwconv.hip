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

extern "C" int zoo_dwconv_wgrad_blocks(const int* gi) {
  const int M = gi[0] * gi[4] * gi[5];
  const int rpb = dw_wgrad_rpb(M);
  return (M + rpb - 1) / rpb;
}

extern "C" hipError_t zoo_dwconv_wgrad(const void* X, const void* dY, float* dW, float* partial, const int* gi,
                                       hipStream_t st) {
  DwGeom g{gi[0], gi[1], gi[2], gi[3], gi[4], gi[5], gi[6], gi[7], gi[8], gi[9], gi[10], gi[11]};
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
