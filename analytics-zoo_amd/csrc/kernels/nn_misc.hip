// LayerNorm and embedding kernels (gfx950).
//
// * LayerNorm forward/backward over the last dimension (InternalLayerNorm,
//   Zs/pipeline/api/keras/layers/internal/InternalLayerNorm.scala:26-97; BERT's
//   normalisation). One wave per row, 8 elements per lane
//   per step (16-byte vector loads of bf16), fp32 statistics, gamma/beta grads
//   reduced per workgroup in LDS and added with one fp32 atomic per column.
// * Embedding gather (LookupTable forward, Embedding.scala:82-100) and sorted-
//   free scatter-add backward with fp32 atomics into the (flat) gradient buffer
//   (HK9). Rows are gathered 16 bytes per lane; each row's gradient add is a
//   contiguous row segment (Guideline 12 atomic shaping).
#include "common.h"

namespace zoo {

template <typename T>
ZOO_DEV void ld8(const T* p, float* f);
template <>
ZOO_DEV void ld8<bf16_t>(const bf16_t* p, float* f) { unpack8(*reinterpret_cast<const uint4*>(p), f); }
template <>
ZOO_DEV void ld8<float>(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
template <typename T>
ZOO_DEV void st8(T* p, const float* f);
template <>
ZOO_DEV void st8<bf16_t>(bf16_t* p, const float* f) { *reinterpret_cast<uint4*>(p) = pack8(f); }
template <>
ZOO_DEV void st8<float>(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(f[4], f[5], f[6], f[7]);
}

// Dropout keep-mask: a counter-based hash of (seed, element index), so backward regenerates the
// mask instead of storing it (da = keep * dout * scale). i8 = index of the element's 8-element
// chunk in the flat tensor, e = element within the chunk. Shared by dropout_add_kernel and the
// fused residual-dropout LayerNorm forward, which must draw identical masks.
ZOO_DEV uint32_t drop_fmix(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}
ZOO_DEV uint32_t drop_base(size_t i8, uint32_t s1) { return drop_fmix((uint32_t)(i8 >> 29) ^ s1); }
ZOO_DEV bool drop_keep(size_t i8, int e, uint32_t s0, uint32_t base, uint32_t thresh) {
  return drop_fmix(((uint32_t)(i8 << 3) + e) * 0x9E3779B1u ^ s0 ^ base) >= thresh;
}

struct DropArgs {
  const bf16_t* A;  // dropout branch (nullptr: plain LayerNorm)
  bf16_t* S;        // residual sum out = X + keep * A * scale (the LayerNorm input saved for backward)
  uint32_t thresh, s0, s1;
  float scale;
  const uint32_t* off;  // per-step device seed offset (g_seed_off) or null
};

// ---------------------------------------------------------------- LayerNorm
template <typename T>
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const T* __restrict__ X, const float* __restrict__ g,
                                                            const float* __restrict__ b, T* __restrict__ Y,
                                                            float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                            int rows, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = X + (size_t)row * D;
  float s = 0.f, ss = 0.f;
  for (int c = lane * 8; c < D; c += 512) {
    float v[8];
    ld8(x + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) { s += v[e]; ss += v[e] * v[e]; }
  }
  s = warp_sum(s);
  ss = warp_sum(ss);
  const float mu = s / D;
  const float var = fmaxf(ss / D - mu * mu, 0.f);
  const float rs = rsqrtf(var + eps);
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
  T* y = Y + (size_t)row * D;
  for (int c = lane * 8; c < D; c += 512) {
    float v[8];
    ld8(x + c, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (v[e] - mu) * rs * (g ? g[c + e] : 1.f) + (b ? b[c + e] : 0.f);
    st8(y + c, v);
  }
}

// Row-resident variant for D <= NCH*512: one wave per row keeps its NCH x 8
// values in registers between the statistics and the normalise pass (the row
// is read once), and gamma/beta are read with 16-byte vector loads.
//
// DROP (bf16 only): the Transformer residual LayerNorm(x + dropout(a)) in one pass -- the sum is
// formed in registers, rounded to bf16 and stored (S, the tensor LayerNorm backward reads) and
// normalised from the rounded values, so no separate dropout_add pass writes S and reads it back.
template <typename T, int NCH, bool DROP = false>
__global__ __launch_bounds__(256) void layernorm_fwd_reg_kernel(const T* __restrict__ X, const float* __restrict__ g,
                                                                const float* __restrict__ b, T* __restrict__ Y,
                                                                float* __restrict__ mean_out,
                                                                float* __restrict__ rstd_out, int rows, int D,
                                                                float eps, DropArgs dr) {
  if (dr.A && dr.off) dr.s0 ^= *dr.off;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = X + (size_t)row * D;
  float v[NCH][8];
  float s = 0.f, ss = 0.f;
  uint32_t dbase = 0;
  if constexpr (DROP) dbase = drop_base(((size_t)row * D) >> 3, dr.s1);
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < D) {
      ld8(x + c, v[k]);
      if constexpr (DROP) {
        float a[8];
        ld8(dr.A + (size_t)row * D + c, a);
        const size_t i8 = ((size_t)row * D + c) >> 3;
        // the hash base depends on i8 >> 29 only: recompute it for chunks past a 2^29 boundary
        const uint32_t bs = (i8 >> 29) == ((((size_t)row * D) >> 3) >> 29) ? dbase : drop_base(i8, dr.s1);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[k][e] += drop_keep(i8, e, dr.s0, bs, dr.thresh) ? a[e] * dr.scale : 0.f;
        const uint4 pk = pack8(v[k]);
        *reinterpret_cast<uint4*>(dr.S + (size_t)row * D + c) = pk;
        unpack8(pk, v[k]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[k][e] = 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { s += v[k][e]; ss += v[k][e] * v[k][e]; }
  }
  s = warp_sum(s);
  ss = warp_sum(ss);
  const float mu = s / D;
  const float var = fmaxf(ss / D - mu * mu, 0.f);
  const float rs = rsqrtf(var + eps);
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
  T* y = Y + (size_t)row * D;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c >= D) continue;
    float gg[8], bb[8];
    if (g) {
      const float4 g0 = *reinterpret_cast<const float4*>(g + c), g1 = *reinterpret_cast<const float4*>(g + c + 4);
      gg[0] = g0.x; gg[1] = g0.y; gg[2] = g0.z; gg[3] = g0.w; gg[4] = g1.x; gg[5] = g1.y; gg[6] = g1.z; gg[7] = g1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) gg[e] = 1.f;
    }
    if (b) {
      const float4 b0 = *reinterpret_cast<const float4*>(b + c), b1 = *reinterpret_cast<const float4*>(b + c + 4);
      bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w; bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) bb[e] = 0.f;
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[k][e] - mu) * rs * gg[e] + bb[e];
    st8(y + c, o);
  }
}

// Register-resident LayerNorm backward (D <= 64*8*NCH): each wave keeps its row of x/dy in
// registers for both passes, gamma once per thread (float4), and the dgamma/dbeta partials
// of every row the wave visits in registers; the 4 waves fold them through LDS once and
// the block adds [D] partials to global with one atomic per column. Replaces per-element
// LDS atomics (the generic kernel below).
template <typename T, int NCH>
__global__ __launch_bounds__(256) void layernorm_bwd_reg_kernel(const T* __restrict__ dY, const T* __restrict__ X,
                                                                const float* __restrict__ g,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd, T* __restrict__ dX,
                                                                float* __restrict__ dg, float* __restrict__ db,
                                                                int rows, int D) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* part = reinterpret_cast<float*>(smem);  // [4 waves][2][D]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gg[NCH][8], pg[NCH][8], pb[NCH][8];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) { gg[k][e] = 1.f; pg[k][e] = 0.f; pb[k][e] = 0.f; }
    if (g && c < D) {
      const float4 g0 = *reinterpret_cast<const float4*>(g + c), g1 = *reinterpret_cast<const float4*>(g + c + 4);
      gg[k][0] = g0.x; gg[k][1] = g0.y; gg[k][2] = g0.z; gg[k][3] = g0.w;
      gg[k][4] = g1.x; gg[k][5] = g1.y; gg[k][6] = g1.z; gg[k][7] = g1.w;
    }
  }
  for (int row = blockIdx.x * 4 + wid; row < rows; row += gridDim.x * 4) {
    const T* x = X + (size_t)row * D;
    const T* dy = dY + (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float xh[NCH][8], gv[NCH][8];
    float a = 0.f, bsum = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < D) {
        ld8(x + c, xh[k]);
        ld8(dy + c, gv[k]);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) { xh[k][e] = 0.f; gv[k][e] = 0.f; }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xh[k][e] = c < D ? (xh[k][e] - mu) * rs : 0.f;
        const float gy = gv[k][e] * gg[k][e];
        a += gy * xh[k][e];
        bsum += gy;
        pg[k][e] += gv[k][e] * xh[k][e];
        pb[k][e] += gv[k][e];
      }
    }
    a = warp_sum(a) / D;
    bsum = warp_sum(bsum) / D;
    T* dx = dX + (size_t)row * D;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c >= D) continue;
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = rs * (gv[k][e] * gg[k][e] - bsum - xh[k][e] * a);
      st8(dx + c, o);
    }
  }
  if (!dg && !db) return;
  // fold the 4 waves' partials, one global atomic per column per block
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c >= D) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      part[(wid * 2) * D + c + e] = pg[k][e];
      part[(wid * 2 + 1) * D + c + e] = pb[k][e];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { sg += part[(w * 2) * D + i]; sb += part[(w * 2 + 1) * D + i]; }
    if (dg) atomicAdd(dg + i, sg);
    if (db) atomicAdd(db + i, sb);
  }
}

// bf16 LayerNorm backward, v2: 4-element (8-byte) chunks so D = 768 maps onto all 64 lanes
// (3 chunks each; the 8-element layout left half the wave idle on its second chunk), two rows
// per wave iteration with all of both rows' loads issued before the first reduction (twice the
// bytes in flight per wave), and the dgamma / dbeta block partials stored plainly
// (part[block][2][D]) for an ordered fold instead of ~10^6 contended global atomics.
template <int NCH>
__global__ __launch_bounds__(256) void layernorm_bwd_v2_kernel(const bf16_t* __restrict__ dY,
                                                               const bf16_t* __restrict__ X,
                                                               const float* __restrict__ g,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd, bf16_t* __restrict__ dX,
                                                               float* __restrict__ part, int rows, int D,
                                                               const bf16_t* __restrict__ dY2, DropArgs dr) {
  if (dr.S && dr.off) dr.s0 ^= *dr.off;  // backward: dr.S (dA) marks the dropout branch
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][2][D]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const float invD = 1.f / (float)D;
  float gg[NCH][4], pg[NCH][4], pb[NCH][4];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) { gg[k][e] = 1.f; pg[k][e] = 0.f; pb[k][e] = 0.f; }
    if (g && c < D) {
      const float4 g0 = *reinterpret_cast<const float4*>(g + c);
      gg[k][0] = g0.x; gg[k][1] = g0.y; gg[k][2] = g0.z; gg[k][3] = g0.w;
    }
  }
  const int pairs = (rows + 1) >> 1;
  for (int pr = blockIdx.x * 4 + wid; pr < pairs; pr += gridDim.x * 4) {
    const int r0 = pr * 2;
    const bool has1 = r0 + 1 < rows;
    uint2 xv[2][NCH], dv[2][NCH], d2[2][NCH];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = (k * 64 + lane) * 4;
        const bool ok = c < D && (h == 0 || has1);
        const size_t off = (size_t)(r0 + h) * D + c;
        xv[h][k] = ok ? *reinterpret_cast<const uint2*>(X + off) : make_uint2(0u, 0u);
        dv[h][k] = ok ? *reinterpret_cast<const uint2*>(dY + off) : make_uint2(0u, 0u);
        d2[h][k] = ok && dY2 ? *reinterpret_cast<const uint2*>(dY2 + off) : make_uint2(0u, 0u);
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !has1) break;
      const int row = r0 + h;
      const float mu = mean[row], rs = rstd[row];
      float xh[NCH][4], gv[NCH][4];
      float a = 0.f, bsum = 0.f;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = (k * 64 + lane) * 4;
        xh[k][0] = bf2f((bf16_t)(xv[h][k].x & 0xFFFFu)); xh[k][1] = bf2f((bf16_t)(xv[h][k].x >> 16));
        xh[k][2] = bf2f((bf16_t)(xv[h][k].y & 0xFFFFu)); xh[k][3] = bf2f((bf16_t)(xv[h][k].y >> 16));
        gv[k][0] = bf2f((bf16_t)(dv[h][k].x & 0xFFFFu)); gv[k][1] = bf2f((bf16_t)(dv[h][k].x >> 16));
        gv[k][2] = bf2f((bf16_t)(dv[h][k].y & 0xFFFFu)); gv[k][3] = bf2f((bf16_t)(dv[h][k].y >> 16));
        if (dY2) {  // second output gradient (a residual consumer's, LayerNorm GradAdd), summed in fp32
          gv[k][0] += bf2f((bf16_t)(d2[h][k].x & 0xFFFFu)); gv[k][1] += bf2f((bf16_t)(d2[h][k].x >> 16));
          gv[k][2] += bf2f((bf16_t)(d2[h][k].y & 0xFFFFu)); gv[k][3] += bf2f((bf16_t)(d2[h][k].y >> 16));
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[k][e] = c < D ? (xh[k][e] - mu) * rs : 0.f;
          const float gy = gv[k][e] * gg[k][e];
          a = fmaf(gy, xh[k][e], a);
          bsum += gy;
          pg[k][e] = fmaf(gv[k][e], xh[k][e], pg[k][e]);
          pb[k][e] += gv[k][e];
        }
      }
      a = warp_sum(a) * invD;
      bsum = warp_sum(bsum) * invD;
#pragma unroll
      for (int k = 0; k < NCH; ++k) {
        const int c = (k * 64 + lane) * 4;
        if (c >= D) continue;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (gv[k][e] * gg[k][e] - bsum - xh[k][e] * a);
        const uint2 pk = make_uint2(pack2bf(o[0], o[1]), pack2bf(o[2], o[3]));
        *reinterpret_cast<uint2*>(dX + (size_t)row * D + c) = pk;
        if (dr.S) {
          // the residual-dropout branch's gradient from the same rounded values: dA = keep * dX * scale
          // (dr.S carries dA here; the mask of zoo_dropout_add for this (p, seed))
          const size_t E = (size_t)row * D + c;  // 4-aligned: one 8-element hash chunk
          const size_t i8 = E >> 3;
          const uint32_t bs = drop_base(i8, dr.s1);
          const float q[4] = {bf2f((bf16_t)(pk.x & 0xFFFFu)), bf2f((bf16_t)(pk.x >> 16)), bf2f((bf16_t)(pk.y & 0xFFFFu)),
                              bf2f((bf16_t)(pk.y >> 16))};
          float d[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) d[e] = drop_keep(i8, (int)(E & 7) + e, dr.s0, bs, dr.thresh) ? q[e] * dr.scale : 0.f;
          *reinterpret_cast<uint2*>(dr.S + E) = make_uint2(pack2bf(d[0], d[1]), pack2bf(d[2], d[3]));
        }
      }
    }
  }
  if (!part) return;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = (k * 64 + lane) * 4;
    if (c >= D) continue;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red[(wid * 2) * D + c + e] = pg[k][e];
      red[(wid * 2 + 1) * D + c + e] = pb[k][e];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) {
    const int w2 = i >= D ? 1 : 0, col = i - w2 * D;
    part[(size_t)blockIdx.x * 2 * D + i] =
        ((red[(0 * 2 + w2) * D + col] + red[(1 * 2 + w2) * D + col]) + red[(2 * 2 + w2) * D + col]) +
        red[(3 * 2 + w2) * D + col];
  }
}

// Ordered two-level fold of the block partials: level 1 sums groups of 32 partial rows per
// column (64 columns x one group per workgroup, 4 independent chains), level 2 adds the group
// sums in order into dg / db. (A single pass with one thread per column was latency-bound:
// ~150 us for 1024 partial rows.)
constexpr int LN_FOLD_G = 32;

__global__ __launch_bounds__(64) void layernorm_part_fold1_kernel(const float* __restrict__ part, int nb, int n2,
                                                                  float* __restrict__ lvl) {
  const int col = blockIdx.x * 64 + threadIdx.x;
  if (col >= n2) return;
  const int b0 = blockIdx.y * LN_FOLD_G, b1 = min(nb, b0 + LN_FOLD_G);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int b = b0;
  for (; b + 3 < b1; b += 4) {
    s0 += part[(size_t)b * n2 + col];
    s1 += part[(size_t)(b + 1) * n2 + col];
    s2 += part[(size_t)(b + 2) * n2 + col];
    s3 += part[(size_t)(b + 3) * n2 + col];
  }
  for (; b < b1; ++b) s0 += part[(size_t)b * n2 + col];
  lvl[(size_t)blockIdx.y * n2 + col] = (s0 + s1) + (s2 + s3);
}

// one wave per column: lane l reads group l's sum (ng <= 64), fixed-order shuffle tree
__global__ __launch_bounds__(256) void layernorm_part_fold2_kernel(const float* __restrict__ lvl, int ng, int D,
                                                                   float* __restrict__ dg, float* __restrict__ db) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= 2 * D) return;
  const float s = warp_sum(lane < ng ? lvl[(size_t)lane * 2 * D + i] : 0.f);
  if (lane != 0) return;
  if (i < D) {
    if (dg) dg[i] += s;
  } else if (db) {
    db[i - D] += s;
  }
}

// ---------------------------------------------------------------- Dropout (+ residual add)
// out = x + keep(i) * a * scale  (x optional); see drop_keep above.

__global__ __launch_bounds__(256) void dropout_add_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ X,
                                                          bf16_t* __restrict__ Out, size_t n8, uint32_t thresh,
                                                          float scale, uint32_t s0, uint32_t s1,
                                                          const uint32_t* __restrict__ soff) {
  if (soff) s0 ^= *soff;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    float a[8], o[8];
    unpack8(reinterpret_cast<const uint4*>(A)[i], a);
    if (X) unpack8(reinterpret_cast<const uint4*>(X)[i], o);
    const uint32_t base = drop_base(i, s1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = drop_keep(i, e, s0, base, thresh) ? a[e] * scale : 0.f;
      o[e] = X ? o[e] + v : v;
    }
    reinterpret_cast<uint4*>(Out)[i] = pack8(o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const T* __restrict__ dY, const T* __restrict__ X,
                                                            const float* __restrict__ g, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, T* __restrict__ dX,
                                                            float* __restrict__ dg, float* __restrict__ db, int rows,
                                                            int D, int rows_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sdg = reinterpret_cast<float*>(smem);  // [D]
  float* sdb = sdg + D;                          // [D]
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) sdg[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  for (int row = r0 + wid; row < r1; row += 4) {
    const T* x = X + (size_t)row * D;
    const T* dy = dY + (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float a = 0.f, bsum = 0.f;  // sum(dy*g*xhat), sum(dy*g)
    for (int c = lane * 8; c < D; c += 512) {
      float xv[8], gv[8];
      ld8(x + c, xv);
      ld8(dy + c, gv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (xv[e] - mu) * rs;
        const float gg = gv[e] * (g ? g[c + e] : 1.f);
        a += gg * xh;
        bsum += gg;
        atomicAdd(&sdg[c + e], gv[e] * xh);  // LDS atomics
        atomicAdd(&sdb[c + e], gv[e]);
      }
    }
    a = warp_sum(a) / D;
    bsum = warp_sum(bsum) / D;
    T* dx = dX + (size_t)row * D;
    for (int c = lane * 8; c < D; c += 512) {
      float xv[8], gv[8], o[8];
      ld8(x + c, xv);
      ld8(dy + c, gv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (xv[e] - mu) * rs;
        o[e] = rs * (gv[e] * (g ? g[c + e] : 1.f) - bsum - xh * a);
      }
      st8(dx + c, o);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < D; i += blockDim.x) {
    if (dg) atomicAdd(dg + i, sdg[i]);
    if (db) atomicAdd(db + i, sdb[i]);
  }
}

// ---------------------------------------------------------------- Embedding
// out[i][:] = table[idx[i]][:]   (rows with idx < 0 or == padding produce zeros)
template <typename T>
__global__ __launch_bounds__(256) void embedding_fwd_kernel(const T* __restrict__ table, const int64_t* __restrict__ idx,
                                                            T* __restrict__ out, int n, int D, int V, int64_t pad) {
  const int vec = 16 / sizeof(T);
  const int cpr = D / vec;
  const size_t total = (size_t)n * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / cpr), c = (int)(i % cpr);
    const int64_t id = idx[r];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (id >= 0 && id < V && id != pad) v = reinterpret_cast<const uint4*>(table + (size_t)id * D)[c];
    reinterpret_cast<uint4*>(out + (size_t)r * D)[c] = v;
  }
}

// grad_table[idx[i]][:] += scale * dout[i][:]  (fp32 accumulate), two forms:
//
// * tiny tables (V <= EMB_LDS_ROWS: token-type / segment embeddings, where thousands of
//   tokens hit the same few rows and per-element global atomics serialise on a handful of
//   addresses; 3x torch index_add_ at V = 2): a workgroup owns a 16-column slice and a chunk of >= 16V tokens,
//   accumulates into an LDS copy of its [V][16] slice (LDS atomics), then flushes every
//   touched row with one global atomic per element -- the global atomic count drops by the
//   tokens-per-row ratio of the chunk;
// * large tables (word embeddings: ids spread, little contention): one element per thread,
//   coalesced atomics (as fast as torch's index_add_ on these shapes, tools/emb_bench.py).
constexpr int EMB_LDS_ROWS = 32, EMB_SLICE = 16;

template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_lds_kernel(const T* __restrict__ dout,
                                                                const int64_t* __restrict__ idx,
                                                                float* __restrict__ gtable, int n, int D, int V,
                                                                int64_t pad, float scale, int chunk) {
  __shared__ float tab[EMB_LDS_ROWS * EMB_SLICE];
  __shared__ unsigned char touched[EMB_LDS_ROWS];
  const int c0 = blockIdx.x * EMB_SLICE;
  const int t0 = blockIdx.y * chunk, t1 = min(n, t0 + chunk);
  for (int i = threadIdx.x; i < V * EMB_SLICE; i += 256) tab[i] = 0.f;
  for (int i = threadIdx.x; i < V; i += 256) touched[i] = 0;
  __syncthreads();
  const int col = threadIdx.x & (EMB_SLICE - 1), lane_t = threadIdx.x / EMB_SLICE;  // 16 token lanes
  const bool colok = c0 + col < D;
  constexpr int LANES = 256 / EMB_SLICE, U = 8;  // 8 tokens per lane in flight per round
  for (int rb = t0 + lane_t; rb < t1; rb += LANES * U) {
    int id[U];
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int r = rb + u * LANES;
      const int64_t x = r < t1 ? idx[r] : -1;
      id[u] = (x < 0 || x >= V || x == pad) ? -1 : (int)x;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = (size_t)(rb + u * LANES) * D + c0 + col;
      if (id[u] >= 0 && colok) {
        if constexpr (sizeof(T) == 4) v[u] = dout[off];
        else v[u] = bf2f(dout[off]);
      } else {
        v[u] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (id[u] < 0) continue;
      atomicAdd(&tab[id[u] * EMB_SLICE + col], v[u]);
      if (col == 0) touched[id[u]] = 1;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < V * EMB_SLICE; i += 256) {
    const int row = i / EMB_SLICE, c = i % EMB_SLICE;
    if (touched[row] && c0 + c < D) atomicAdd(gtable + (size_t)row * D + c0 + c, tab[i] * scale);
  }
}

// one element per thread, consecutive lanes on consecutive columns: every wave-wide
// atomic instruction covers one contiguous 256-byte row segment
template <typename T>
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const T* __restrict__ dout, const int64_t* __restrict__ idx,
                                                            float* __restrict__ gtable, int n, int D, int V,
                                                            int64_t pad, float scale) {
  const size_t total = (size_t)n * D;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / D), c = (int)(i % D);
    const int64_t id = idx[r];
    if (id < 0 || id >= V || id == pad) continue;
    float v;
    if constexpr (sizeof(T) == 4) v = dout[i];
    else v = bf2f(dout[i]);
    atomicAdd(gtable + (size_t)id * D + c, v * scale);
  }
}

static int mgrid(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b ? b : 1);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_layernorm_fwd(const void* X, int f32, const float* g, const float* b, void* Y, float* mean,
                                        float* rstd, int rows, int D, float eps, hipStream_t st) {
  const int blocks = (rows + 3) / 4;
  // gamma/beta are read as float4 by the register-resident kernels
  const bool al = ((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(b)) & 15) == 0;
#define ZOO_LN_REG(T, NCH)                                                                                   \
  hipLaunchKernelGGL((layernorm_fwd_reg_kernel<T, NCH>), dim3(blocks), dim3(256), 0, st, (const T*)X, g, b, \
                     (T*)Y, mean, rstd, rows, D, eps, DropArgs{})
  if (al && D <= 2048) {
    if (f32) {
      if (D <= 512) ZOO_LN_REG(float, 1);
      else if (D <= 1024) ZOO_LN_REG(float, 2);
      else ZOO_LN_REG(float, 4);
    } else {
      if (D <= 512) ZOO_LN_REG(bf16_t, 1);
      else if (D <= 1024) ZOO_LN_REG(bf16_t, 2);
      else ZOO_LN_REG(bf16_t, 4);
    }
    return hipGetLastError();
  }
#undef ZOO_LN_REG
  if (f32)
    hipLaunchKernelGGL(layernorm_fwd_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)X, g, b, (float*)Y,
                       mean, rstd, rows, D, eps);
  else
    hipLaunchKernelGGL(layernorm_fwd_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)X, g, b,
                       (bf16_t*)Y, mean, rstd, rows, D, eps);
  return hipGetLastError();
}

// Y = LayerNorm(S), S = X + dropout(A) (stored): the fused Transformer residual LayerNorm. bf16,
// D % 8 == 0, D <= 2048, 16-byte aligned gamma / beta. Draws the mask zoo_dropout_add draws for
// the same (n, p, seed), so its backward is zoo_dropout_add(dS, nullptr, ...).
extern "C" hipError_t zoo_dropout_add_layernorm_fwd(const void* A, const void* X, const float* g, const float* b,
                                                    void* S, void* Y, float* mean, float* rstd, int rows, int D,
                                                    float eps, float p, uint64_t seed, hipStream_t st) {
  if (D % 8 || D > 2048 || (((reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(b)) & 15) != 0))
    return hipErrorInvalidValue;
  const double t = (double)p * 4294967296.0;
  DropArgs dr;
  dr.A = (const bf16_t*)A;
  dr.S = (bf16_t*)S;
  dr.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  dr.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dr.s0 = (uint32_t)seed;
  dr.s1 = (uint32_t)(seed >> 32);
  dr.off = g_seed_off;
  const int blocks = (rows + 3) / 4;
#define ZOO_LN_DROP(NCH)                                                                                    \
  hipLaunchKernelGGL((layernorm_fwd_reg_kernel<bf16_t, NCH, true>), dim3(blocks), dim3(256), 0, st,        \
                     (const bf16_t*)X, g, b, (bf16_t*)Y, mean, rstd, rows, D, eps, dr)
  if (D <= 512) ZOO_LN_DROP(1);
  else if (D <= 1024) ZOO_LN_DROP(2);
  else ZOO_LN_DROP(4);
#undef ZOO_LN_DROP
  return hipGetLastError();
}

static int ln_v2_nch(int D) {
  static const bool on = true;
  if (!on || D % 4 || D > 64 * 4 * 4) return 0;
  return (D + 255) / 256;                      // 4-element chunks per lane
}

static int ln_v2_blocks(int rows) {
  int b = ((rows + 1) / 2 + 7) / 8;            // >= 2 row pairs per wave
  return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

// fp32 scratch floats the bf16 v2 backward needs for its dgamma / dbeta partials (0: none)
extern "C" size_t zoo_layernorm_bwd_part_floats(int rows, int D, int f32) {
  if (f32 || !ln_v2_nch(D)) return 0;
  const int nb = ln_v2_blocks(rows);
  return ((size_t)nb + (nb + LN_FOLD_G - 1) / LN_FOLD_G) * 2 * D;
}

// dY2 (nullable): a second output gradient added to dY inside the bf16 v2 kernel; the other
// paths return hipErrorNotSupported for it (the caller then adds it first)
// deferred dgamma / dbeta fold (zoo_layernorm_defer_fold(1)): the v2 backward leaves its block
// partials in `part` and the caller folds them later with zoo_layernorm_fold -- on the
// weight-gradient side stream, off the data-gradient chain
static int g_ln_defer_fold = 0;
extern "C" void zoo_layernorm_defer_fold(int on) { g_ln_defer_fold = on ? 1 : 0; }
extern "C" int zoo_layernorm_bwd_v2_blocks(int rows, int D, int f32) {
  return (f32 || !ln_v2_nch(D)) ? 0 : ln_v2_blocks(rows);
}
extern "C" hipError_t zoo_layernorm_fold(float* part, int rows, int D, float* dg, float* db, hipStream_t st) {
  const int blocks = ln_v2_blocks(rows);
  const int ng = (blocks + LN_FOLD_G - 1) / LN_FOLD_G;
  float* lvl = part + (size_t)blocks * 2 * D;
  hipLaunchKernelGGL(layernorm_part_fold1_kernel, dim3((2 * D + 63) / 64, ng), dim3(64), 0, st, part, blocks, 2 * D,
                     lvl);
  hipLaunchKernelGGL(layernorm_part_fold2_kernel, dim3((2 * D + 3) / 4), dim3(256), 0, st, lvl, ng, D, dg, db);
  return hipGetLastError();
}

static hipError_t ln_bwd_impl(const void* dY, const void* X, int f32, const float* g, const float* mean,
                              const float* rstd, void* dX, float* dg, float* db, int rows, int D, float* part,
                              const void* dY2, const DropArgs& dr, hipStream_t st) {
  const int nch = f32 ? 0 : ln_v2_nch(D);
  const bool v2 = nch && (reinterpret_cast<uintptr_t>(g) & 15) == 0;
  if ((dY2 || dr.S) && !v2) return hipErrorNotSupported;
  if (v2) {
    const int blocks = ln_v2_blocks(rows);
    float* pp = (dg || db) ? part : nullptr;
    if ((dg || db) && !part) return hipErrorInvalidValue;
    const size_t lds = (size_t)8 * D * sizeof(float);
#define ZOO_LNB2(N)                                                                                              \
  hipLaunchKernelGGL((layernorm_bwd_v2_kernel<N>), dim3(blocks), dim3(256), lds, st, (const bf16_t*)dY,         \
                     (const bf16_t*)X, g, mean, rstd, (bf16_t*)dX, pp, rows, D, (const bf16_t*)dY2, dr)
    if (nch == 1) ZOO_LNB2(1);
    else if (nch == 2) ZOO_LNB2(2);
    else if (nch == 3) ZOO_LNB2(3);
    else ZOO_LNB2(4);
#undef ZOO_LNB2
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !pp || g_ln_defer_fold) return e;   // deferred: zoo_layernorm_fold
    const int ng = (blocks + LN_FOLD_G - 1) / LN_FOLD_G;
    float* lvl = pp + (size_t)blocks * 2 * D;
    hipLaunchKernelGGL(layernorm_part_fold1_kernel, dim3((2 * D + 63) / 64, ng), dim3(64), 0, st, pp, blocks, 2 * D,
                       lvl);
    hipLaunchKernelGGL(layernorm_part_fold2_kernel, dim3((2 * D + 3) / 4), dim3(256), 0, st, lvl, ng, D, dg, db);
    return hipGetLastError();
  }
  const bool al = (reinterpret_cast<uintptr_t>(g) & 15) == 0 && (f32 ? D % 4 == 0 : D % 8 == 0);
  if (al && D <= 2048 && (f32 ? D % 8 == 0 : true)) {
    // ~512 blocks of 4 waves; each wave loops over rows, so the dgamma/dbeta partials are
    // folded once per block instead of once per row
    int blocks = (rows + 3) / 4;
    if (blocks > 512) blocks = 512;
    const size_t psm = (size_t)8 * D * sizeof(float);
#define ZOO_LNB_REG(TT, NCH)                                                                                   \
  hipLaunchKernelGGL((layernorm_bwd_reg_kernel<TT, NCH>), dim3(blocks), dim3(256), psm, st, (const TT*)dY,   \
                     (const TT*)X, g, mean, rstd, (TT*)dX, dg, db, rows, D)
    if (f32) {
      if (D <= 512) ZOO_LNB_REG(float, 1);
      else if (D <= 1024) ZOO_LNB_REG(float, 2);
      else ZOO_LNB_REG(float, 4);
    } else {
      if (D <= 512) ZOO_LNB_REG(bf16_t, 1);
      else if (D <= 1024) ZOO_LNB_REG(bf16_t, 2);
      else ZOO_LNB_REG(bf16_t, 4);
    }
#undef ZOO_LNB_REG
    return hipGetLastError();
  }
  int rpb = (rows + 511) / 512;
  if (rpb < 4) rpb = 4;
  const int blocks = (rows + rpb - 1) / rpb;
  const size_t smem = (size_t)2 * D * sizeof(float);
  if (f32)
    hipLaunchKernelGGL(layernorm_bwd_kernel<float>, dim3(blocks), dim3(256), smem, st, (const float*)dY,
                       (const float*)X, g, mean, rstd, (float*)dX, dg, db, rows, D, rpb);
  else
    hipLaunchKernelGGL(layernorm_bwd_kernel<bf16_t>, dim3(blocks), dim3(256), smem, st, (const bf16_t*)dY,
                       (const bf16_t*)X, g, mean, rstd, (bf16_t*)dX, dg, db, rows, D, rpb);
  return hipGetLastError();
}

extern "C" hipError_t zoo_layernorm_bwd(const void* dY, const void* X, int f32, const float* g, const float* mean,
                                        const float* rstd, void* dX, float* dg, float* db, int rows, int D,
                                        float* part, const void* dY2, hipStream_t st) {
  return ln_bwd_impl(dY, X, f32, g, mean, rstd, dX, dg, db, rows, D, part, dY2, DropArgs{}, st);
}

// backward of zoo_dropout_add_layernorm_fwd: dX (= the residual input's gradient) and, from the
// same rounded values, dA = keep * dX / (1 - p) for the dropout branch -- no second pass over dX.
// bf16 v2 kernel only (hipErrorNotSupported otherwise: the caller runs zoo_dropout_add on dX).
extern "C" hipError_t zoo_layernorm_bwd_drop(const void* dY, const void* X, const float* g, const float* mean,
                                             const float* rstd, void* dX, void* dA, float* dg, float* db, int rows,
                                             int D, float* part, const void* dY2, float p, uint64_t seed,
                                             hipStream_t st) {
  const double t = (double)p * 4294967296.0;
  DropArgs dr;
  dr.A = nullptr;
  dr.S = (bf16_t*)dA;
  dr.thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  dr.scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  dr.s0 = (uint32_t)seed;
  dr.s1 = (uint32_t)(seed >> 32);
  dr.off = g_seed_off;
  return ln_bwd_impl(dY, X, 0, g, mean, rstd, dX, dg, db, rows, D, part, dY2, dr, st);
}

extern "C" hipError_t zoo_embedding_fwd(const void* table, int f32, const int64_t* idx, void* out, int n, int D, int V,
                                        int64_t pad, hipStream_t st) {
  const int vec = f32 ? 4 : 8;
  if (f32)
    hipLaunchKernelGGL(embedding_fwd_kernel<float>, dim3(mgrid((size_t)n * D / vec)), dim3(256), 0, st,
                       (const float*)table, idx, (float*)out, n, D, V, pad);
  else
    hipLaunchKernelGGL(embedding_fwd_kernel<bf16_t>, dim3(mgrid((size_t)n * D / vec)), dim3(256), 0, st,
                       (const bf16_t*)table, idx, (bf16_t*)out, n, D, V, pad);
  return hipGetLastError();
}

extern "C" hipError_t zoo_embedding_bwd(const void* dout, int f32, const int64_t* idx, float* gtable, int n, int D,
                                        int V, int64_t pad, float scale, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (V <= EMB_LDS_ROWS) {
    const int slices = (D + EMB_SLICE - 1) / EMB_SLICE;
    // short chunks (>= 8 tokens per table row, >= 128 tokens): the kernel is latency-bound,
    // so many small workgroups beat few long ones; the flush is V x 16 atomics per chunk
    int chunk = 16 * V > 128 ? 16 * V : 128;
    if ((n + chunk - 1) / chunk > 65535) chunk = (n + 65534) / 65535;  // grid.y limit
    const int chunks = (n + chunk - 1) / chunk;
    const dim3 grid(slices, chunks);
    if (f32)
      hipLaunchKernelGGL(embedding_bwd_lds_kernel<float>, grid, dim3(256), 0, st, (const float*)dout, idx, gtable, n,
                         D, V, pad, scale, chunk);
    else
      hipLaunchKernelGGL(embedding_bwd_lds_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)dout, idx, gtable,
                         n, D, V, pad, scale, chunk);
    return hipGetLastError();
  }
  if (f32)
    hipLaunchKernelGGL(embedding_bwd_kernel<float>, dim3(mgrid((size_t)n * D)), dim3(256), 0, st, (const float*)dout,
                       idx, gtable, n, D, V, pad, scale);
  else
    hipLaunchKernelGGL(embedding_bwd_kernel<bf16_t>, dim3(mgrid((size_t)n * D)), dim3(256), 0, st,
                       (const bf16_t*)dout, idx, gtable, n, D, V, pad, scale);
  return hipGetLastError();
}

extern "C" hipError_t zoo_dropout_add(const void* A, const void* X, void* Out, size_t n, float p, uint64_t seed,
                                      hipStream_t st) {
  const double t = (double)p * 4294967296.0;
  const uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  const float scale = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const size_t n8 = n / 8;
  size_t blocks = (n8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(dropout_add_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)A,
                     (const bf16_t*)X, (bf16_t*)Out, n8, thresh, scale, (uint32_t)seed, (uint32_t)(seed >> 32),
                     g_seed_off);
  return hipGetLastError();
}
