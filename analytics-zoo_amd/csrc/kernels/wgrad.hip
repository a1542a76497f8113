// Convolution / Linear weight gradient on CDNA4 matrix cores (gfx950).
//
//   dW[k][(r,s,c)] += sum_m dY[m][k] * im2col(X)[m][(r,s,c)]
//
// The reduction runs over output pixels m, and BOTH operands are stored
// m-major (NHWC), i.e. not K-contiguous per lane as the MFMA operand maps
// want. Instead of an explicit transpose pass, the tiles are staged [m][col]
// in LDS and read with gfx950's hardware transposing read ds_read_b64_tr_b16
// (cdna_hip_programming.md T10): two 4x16 transposed reads give a lane the 8
// consecutive-k values of its v_mfma_f32_16x16x32_bf16 operand fragment.
//
// The pixel dimension (up to N*P*Q = 802816 for ResNet-50 stage 1 at batch 256)
// is split over workgroups; each adds its fp32 partial tile into dW with
// global float atomics (shaped 64 B per 16-lane row segment).
//
// Reference parity: the weight-gradient half of BigDL SpatialConvolution /
// Linear accGradParameters.
#include <stdlib.h>

#include "common.h"
#include "geom.h"

namespace zoo {



constexpr int WG_BM = 128, WG_BN = 128, WG_BK = 64;

typedef __attribute__((address_space(3))) void wg_lds_void;
typedef __attribute__((address_space(1))) const void wg_gl_void;
__device__ __attribute__((aligned(16))) bf16_t wg_zero_page[8];

// XOR swizzle on 16-column (32-byte) blocks; rows {0..3, 8..11} (one
// half-wave of transposed reads) map to 8 distinct bank groups.
ZOO_DEV int wg_f(int row) { return (row & 3) | (((row >> 3) & 1) << 2); }
ZOO_DEV int wg_off(int row, int col) {  // element offset in a [64][128] bf16 tile
  return row * 128 + ((((col >> 4) ^ wg_f(row)) & 7) << 4) + (col & 15);
}
// [64][64] tile (the dY tile of K <= 64 convs): two 128-byte rows per 64-bank row, so the
// even and the odd rows of {0..3, 8..11} each need 4 distinct 32-byte slots
ZOO_DEV int wg_f64(int row) { return ((row >> 1) & 1) | (((row >> 3) & 1) << 1); }
ZOO_DEV int wg_off64(int row, int col) {
  return row * 64 + ((((col >> 4) ^ wg_f64(row)) & 3) << 4) + (col & 15);
}

// BMT: output-channel tile (128, or 64 for K <= 64 convs, which would waste half of a
// 128-row tile's MFMA work).
template <int VEC, bool DMA, int BMT>
__global__ __launch_bounds__(256, 2) void wgrad_kernel(const bf16_t* __restrict__ X,
                                                        const bf16_t* __restrict__ dY,
                                                        float* __restrict__ dW, float* __restrict__ part,
                                                        WgradGeom g) {
  static_assert(BMT == 128 || (BMT == 64 && !DMA), "64-row tiles use register staging");
  constexpr int NIW = BMT / 32;  // 16-row MFMA tiles per wave (wave tile BMT/2 x 64)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);  // [2][64 m][BMT k-out]
  bf16_t* Bs = As + 2 * WG_BK * BMT;             // [2][64 m][128 (r,s,c)]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_m = (g.K + BMT - 1) / BMT;
  const int tiles_n = (g.Ktot + WG_BN - 1) / WG_BN;
  const int tiles = tiles_m * tiles_n;
  const int split = blockIdx.x / tiles;
  const int tile = blockIdx.x - split * tiles;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int k0 = tm * BMT, c0 = tn * WG_BN;
  const int mstart = split * g.m_per_split;
  const int mend = min(g.M, mstart + g.m_per_split);
  if (mstart >= mend) return;
  const int nk = (mend - mstart + WG_BK - 1) / WG_BK;

  // staging: thread -> 8-column chunk `ch` (16 per 128-wide row), rows rb + 16*i
  // LDS-DMA (VEC 8): a wave writes 4 rows x 256 B lane-linearly (lane -> 16-byte slot lane&15
  // of row lane>>4), so each lane loads the logical 8-column chunk that the swizzle puts in
  // its slot; wg_f depends on row bits 0,1,3 only -> one chunk per thread for all its rows
  const int rb = tid >> 4;  // 0..15
  const int ch = DMA ? 2 * ((((tid & 15) >> 1) ^ wg_f(rb)) & 7) + (tid & 1) : (tid & 15);

  // dY columns (output channels) for this thread's chunk; 64-row tiles: 8 chunks per row,
  // rows arb + 32*i (i < 2)
  const int ach = BMT == 128 ? ch : (tid & 7);
  const int arb = BMT == 128 ? rb : (tid >> 3);
  const int ycol = k0 + ach * 8;
  const bool ycol_ok = ycol < g.K;
  // im2col column decode for the X chunk (fixed for the whole block)
  const int xcol = c0 + ch * 8;
  int xr[2], xs[2], xc[2];
  bool xok[2];
  if constexpr (VEC == 8) {
    const int rs = xcol / g.C;
    xc[0] = xcol - rs * g.C;
    xr[0] = rs / g.S;
    xs[0] = rs - xr[0] * g.S;
    xok[0] = xcol < g.Ktot;
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int pos = (xcol >> 2) + h;
      xr[h] = pos / g.S;
      xs[h] = pos - xr[h] * g.S;
      xc[h] = 0;
      xok[h] = pos * 4 < g.Ktot;
    }
  }

  uint4 ra[4], rbv[4];
  const int PQ = g.P * g.Q;
  // incremental pixel decode: row i of the staging pattern sits at pixel
  // m = mstart + kt*BK + rb + 16i; each k-tile advances it by BK = dn*PQ + dp*Q + dq
  // (no integer division inside the loop)
  const int dn = WG_BK / PQ, dp = (WG_BK % PQ) / g.Q, dq = (WG_BK % PQ) % g.Q;
  int pn[4], pp[4], pqq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mstart + rb + 16 * i;
    const int mm = m < g.M ? m : 0;
    pn[i] = mm / PQ;
    const int pq = mm - pn[i] * PQ;
    pp[i] = pq / g.Q;
    pqq[i] = pq - pp[i] * g.Q;
  }
  auto advance = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      pqq[i] += dq; pp[i] += dp; pn[i] += dn;
      if (pqq[i] >= g.Q) { pqq[i] -= g.Q; ++pp[i]; }
      if (pp[i] >= g.P) { pp[i] -= g.P; ++pn[i]; }
    }
  };

  auto dma16 = [&](const bf16_t* src, bf16_t* dst) {
    __builtin_amdgcn_global_load_lds((wg_gl_void*)src, (wg_lds_void*)dst, 16, 0, 0);
  };
  auto load_tile = [&](int kt) {
    bf16_t* adst = As + (kt & 1) * WG_BK * BMT + (wid * 4) * BMT;
    bf16_t* bdst = Bs + (kt & 1) * WG_BK * WG_BN + (wid * 4) * WG_BN;
    (void)adst; (void)bdst;
    if constexpr (BMT == 64) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int m = mstart + kt * WG_BK + arb + 32 * i;
        ra[i] = (m < mend && ycol_ok) ? *reinterpret_cast<const uint4*>(dY + (size_t)m * g.K + ycol)
                                      : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mstart + kt * WG_BK + rb + 16 * i;
      const bool mok = m < mend;
      if constexpr (BMT == 64) {
      } else if constexpr (DMA) {
        dma16(mok && ycol_ok ? dY + (size_t)m * g.K + ycol : wg_zero_page, adst + 16 * i * BMT);
      } else {
        ra[i] = (mok && ycol_ok) ? *reinterpret_cast<const uint4*>(dY + (size_t)m * g.K + ycol)
                                 : make_uint4(0, 0, 0, 0);
      }
      const int n = mok ? pn[i] : 0, p = mok ? pp[i] : 0, q = mok ? pqq[i] : 0;
      const bf16_t* xb = X + (size_t)n * g.H * g.W * g.C;
      if constexpr (VEC == 8) {
        const int ih = p * g.sh - g.ph + xr[0] * g.dh;
        const int iw = q * g.sw - g.pw + xs[0] * g.dw;
        const bool ok = mok && xok[0] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        if constexpr (DMA) {
          dma16(ok ? xb + (ih * g.W + iw) * g.C + xc[0] : wg_zero_page, bdst + 16 * i * WG_BN);
        } else {
          rbv[i] = ok ? *reinterpret_cast<const uint4*>(xb + (ih * g.W + iw) * g.C + xc[0])
                      : make_uint4(0, 0, 0, 0);
        }
      } else {
        uint2 v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ih = p * g.sh - g.ph + xr[h] * g.dh;
          const int iw = q * g.sw - g.pw + xs[h] * g.dw;
          const bool ok = mok && xok[h] && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          v[h] = ok ? *reinterpret_cast<const uint2*>(xb + (ih * g.W + iw) * 4) : make_uint2(0, 0);
        }
        rbv[i] = make_uint4(v[0].x, v[0].y, v[1].x, v[1].y);
      }
    }
    advance();
  };

  auto store_tile = [&](int buf) {
    bf16_t* a = As + buf * WG_BK * BMT;
    bf16_t* b = Bs + buf * WG_BK * WG_BN;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rb + 16 * i;
      if constexpr (BMT == 128) *reinterpret_cast<uint4*>(a + wg_off(row, ch * 8)) = ra[i];
      *reinterpret_cast<uint4*>(b + wg_off(row, ch * 8)) = rbv[i];
    }
    if constexpr (BMT == 64) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *reinterpret_cast<uint4*>(a + wg_off64(arb + 32 * i, ach * 8)) = ra[i];
    }
  };

  f32x4 acc[NIW][4];
#pragma unroll
  for (int i = 0; i < NIW; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addressing: group gq = lane>>4 holds k = 8*gq..8*gq+7 of a
  // 32-deep k-step; lane i = 4q+p of the group addresses row q, columns 4p..4p+3
  const int gq = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;

  auto read_frag = [&](const bf16_t* base, int kk, int colbase, bool narrow) -> bf16x8 {
    const int row0 = kk * 32 + gq * 8 + tq;
    typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
    const int o0 = narrow ? wg_off64(row0, colbase + 4 * tp) : wg_off(row0, colbase + 4 * tp);
    const int o1 = narrow ? wg_off64(row0 + 4, colbase + 4 * tp) : wg_off(row0 + 4, colbase + 4 * tp);
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + o0));
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + o1));
    typedef short i16x8 __attribute__((ext_vector_type(8)));
    i16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(bf16x8, v);
  };

  auto compute = [&](int buf) {
    const bf16_t* a = As + buf * WG_BK * BMT;
    const bf16_t* b = Bs + buf * WG_BK * WG_BN;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[NIW], bfg[4];
#pragma unroll
      for (int i = 0; i < NIW; ++i) af[i] = read_frag(a, kk, wm * (BMT / 2) + i * 16, BMT == 64);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfg[j] = read_frag(b, kk, wn * 64 + j * 16, false);
#pragma unroll
      for (int i = 0; i < NIW; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfg[j], acc[i][j]);
    }
  };

  if constexpr (DMA) {
    load_tile(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) load_tile(kt + 1);
      compute(kt & 1);
      if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) load_tile(kt + 1);
      compute(cur);
      if (more) store_tile(cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: C/D map of 16x16x32 -> row = 4*(lane>>4)+reg (k-out), col = lane&15.
  // part != null: plain stores of this split's tile into part[split][K][Ktot] (folded in a
  // fixed order by wgrad_fold_kernel: deterministic, no atomics); otherwise fp32 atomics
  // into dW (a single split is one adder per element, hence also deterministic)
  const int fr = lane & 15, fq = lane >> 4;
  float* const pdst = part ? part + (size_t)split * g.K * g.Ktot : nullptr;
#pragma unroll
  for (int i = 0; i < NIW; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = c0 + wn * 64 + j * 16 + fr;
      if (col >= g.Ktot) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = k0 + wm * (BMT / 2) + i * 16 + fq * 4 + r;
        if (row < g.K) {
          if (pdst) pdst[(size_t)row * g.Ktot + col] = acc[i][j][r];
          else atomicAdd(dW + (size_t)row * g.ldw + col, acc[i][j][r]);
        }
      }
    }
}

// Ordered fold of the per-split partials. Level 1 (splits > kFoldGroup): blockIdx.y = group g
// sums splits [g*G, (g+1)*G) in order into lvl1[g]; level 2 sums the groups in order and adds
// into dW. 4 columns per thread (Ktot % 4 == 0). Parallel over splits as well as elements, so
// layers with hundreds of splits and small weights (ResNet stage 1) fold in microseconds.
constexpr int kFoldGroup = 16;
__global__ __launch_bounds__(256) void wgrad_fold1_kernel(const float* __restrict__ part, float* __restrict__ lvl1,
                                                         size_t n4, int splits) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int s0 = blockIdx.y * kFoldGroup, s1 = min(splits, s0 + kFoldGroup);
  const float4* p = reinterpret_cast<const float4*>(part) + i;
  // two interleaved partial sums keep loads in flight (fixed order: deterministic)
  float4 s = p[(size_t)s0 * n4], t = make_float4(0.f, 0.f, 0.f, 0.f);
  int sp = s0 + 1;
  for (; sp + 1 < s1; sp += 2) {
    const float4 v = p[(size_t)sp * n4], u = p[(size_t)(sp + 1) * n4];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
  }
  if (sp < s1) {
    const float4 v = p[(size_t)sp * n4];
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  reinterpret_cast<float4*>(lvl1)[(size_t)blockIdx.y * n4 + i] = s;
}

__global__ __launch_bounds__(256) void wgrad_fold_kernel(const float* __restrict__ part, float* __restrict__ dW,
                                                        int K, int Ktot, int ldw, int splits) {
  const int q = Ktot >> 2;
  const size_t n4 = (size_t)K * q;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(i / q), c4 = (int)(i - (size_t)k * q) * 4;
    const float4* p = reinterpret_cast<const float4*>(part) + i;
    float4 s = p[0], t = make_float4(0.f, 0.f, 0.f, 0.f);
    int sp = 1;
    for (; sp + 1 < splits; sp += 2) {
      const float4 v = p[(size_t)sp * n4], u = p[(size_t)(sp + 1) * n4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    if (sp < splits) {
      const float4 v = p[(size_t)sp * n4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
    float* d = dW + (size_t)k * ldw + c4;
    d[0] += s.x; d[1] += s.y; d[2] += s.z; d[3] += s.w;
  }
}


// ---------------------------------------------------------------------------------------------
// Band weight gradient: the 64-output-channel stride-1 convs of ResNet stage 1 (3x3 64->64, the
// 1x1 64->64 / 256->64) and the space-to-depth stem (4x4, 16 -> 64 channels).
//
// wgrad_kernel above tiles dW into 64 x 128 column blocks and gathers the im2col operand per
// tile, so a 3x3 conv's activation lines are fetched 9x (once per tap) and its dY tile once per
// column block; at these shapes (M = 0.8 - 3.2 M pixels, dW only 64 x 256..576) that made the
// stage-1 3x3 weight gradients 234-511 us and the stem's 408 us -- the last kernel of the step
// (profiles/r5/resnet50_b256_critical_path_final_r5.md rows 330-360).
// Here a workgroup owns ALL of dW (64 x R*S*C fp32 in the accumulators of its 8 waves) and walks
// bands of TP output rows of one image: the band's dY rows [TP*Q][64] and the input halo
// [(TP+R-1) x (Q+S-1)][C] are staged into LDS once (each activation line is read ~(TP+R-1)/TP
// times, each dY line once), and every tap's B fragments are transposed reads
// (ds_read_b64_tr_b16) of the shifted halo rows -- a lane addresses its own row, so the tap shift
// is only an address offset. The next band's global loads are issued into registers before this
// band's MFMAs (register double buffer; LDS single-buffered). Each workgroup writes its dW
// partial once; wgrad_fold*_kernel sum the partials in a fixed order (deterministic).
// Waves: 2 halves of the 64 output channels x 4 groups of the 16-column blocks of dW.
template <int C>
ZOO_DEV int wb_xoff(int row, int col) {   // element offset of (halo row, channel) in LDS
  if constexpr (C == 16) {
    // 32-byte rows; 128 bytes of padding per 8 rows put rows h and h+8 of a transposed read
    // half-wave on different bank halves
    return row * 16 + (row >> 3) * 64 + col;
  } else if constexpr (C == 64) {
    return row * 64 + ((((col >> 4) ^ wg_f64(row)) & 3) << 4) + (col & 15);
  } else {
    return row * C + ((((col >> 4) ^ wg_f(row)) & (C / 16 - 1)) << 4) + (col & 15);
  }
}
template <int C>
constexpr int wb_xelems(int rows) {
  return C == 16 ? rows * 16 + ((rows + 7) >> 3) * 64 : rows * C;
}

template <int R, int S, int C, int TP, int Q>
struct WbCfg {
  static constexpr int NT = 512;
  static constexpr int HC = Q + S - 1, HR = TP + R - 1, HROWS = HR * HC;
  static constexpr int NPX = (TP * Q + 31) / 32 * 32;       // band pixels, padded to 32-pixel K-steps
  static constexpr int DY_PIECES = NPX * 8;                 // 16-byte pieces of the dY band
  static constexpr int X_PIECES = HROWS * (C / 8);
  static constexpr int PPT = (DY_PIECES + X_PIECES + NT - 1) / NT;
  static constexpr int NCB = R * S * C / 16, NCBW = NCB / 4;
  static constexpr int DY_ELEMS = NPX * 64, X_ELEMS = wb_xelems<C>(HROWS);
  static constexpr size_t SMEM = (size_t)(DY_ELEMS + X_ELEMS) * 2;
  static_assert(NCB % 4 == 0, "dW columns must split into 4 groups of 16-column blocks");
  static_assert(C == 16 || C % 64 == 0, "C = 16 or a multiple of 64");
  static_assert(SMEM <= 160 * 1024, "band does not fit in LDS");
};

template <int R, int S, int C, int TP, int Q>
__global__ __launch_bounds__(512, 1) void wgrad_band_kernel(const bf16_t* __restrict__ X,
                                                             const bf16_t* __restrict__ dY,
                                                             float* __restrict__ part, WgradGeom g) {
  using Cfg = WbCfg<R, S, C, TP, Q>;
  constexpr int NT = Cfg::NT, HC = Cfg::HC, HROWS = Cfg::HROWS, NPX = Cfg::NPX, PPT = Cfg::PPT;
  constexpr int DYP = Cfg::DY_PIECES, TOTAL = Cfg::DY_PIECES + Cfg::X_PIECES, NCBW = Cfg::NCBW;
  constexpr int KTOT = R * S * C;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* dyl = reinterpret_cast<bf16_t*>(smem);
  bf16_t* xl = dyl + Cfg::DY_ELEMS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bands_per_img = (g.P + TP - 1) / TP;
  const int nbands = g.N * bands_per_img;

  uint4 st[PPT];
  // piece -> (global source or zero) for band b
  auto gload = [&](int b) {
    const int n = b / bands_per_img, p0 = (b - n * bands_per_img) * TP;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int pid = tid + i * NT;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (pid < DYP) {
        const int row = pid >> 3, j = pid & 7;
        const int pr = row / Q, pc = row - pr * Q;
        if (row < TP * Q && p0 + pr < g.P)
          v = *reinterpret_cast<const uint4*>(dY + ((size_t)(n * g.P + p0 + pr) * Q + pc) * 64 + 8 * j);
      } else if (pid < TOTAL) {
        const int q = pid - DYP;
        const int row = q / (C / 8), j = q - row * (C / 8);
        const int hr = row / HC, hc = row - hr * HC;
        const int ih = p0 - g.ph + hr, iw = hc - g.pw;
        if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
          v = *reinterpret_cast<const uint4*>(X + ((size_t)(n * g.H + ih) * g.W + iw) * C + 8 * j);
      }
      st[i] = v;
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int pid = tid + i * NT;
      if (pid < DYP) {
        const int row = pid >> 3, j = pid & 7;
        *reinterpret_cast<uint4*>(dyl + wg_off64(row, 8 * j)) = st[i];
      } else if (pid < TOTAL) {
        const int q = pid - DYP;
        const int row = q / (C / 8), j = q - row * (C / 8);
        *reinterpret_cast<uint4*>(xl + wb_xoff<C>(row, 8 * j)) = st[i];
      }
    }
  };

  f32x4 acc[2][NCBW];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < NCBW; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kb0 = 2 * (w & 1), cb0 = (w >> 1) * NCBW;
  const int gq = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  auto tr = [&](const bf16_t* base, int o0, int o1) -> bf16x8 {
    const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + o0));
    const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(base + o1));
    i16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(bf16x8, v);
  };
  auto compute = [&]() {
#pragma unroll 1
    for (int ks = 0; ks < NPX / 32; ++ks) {
      // this lane's two pixel rows of the K-step (transposed-read rows q and q + 4 of group gq)
      const int i0 = ks * 32 + gq * 8 + tq, i1 = i0 + 4;
      int pr0 = i0 / Q, pr1 = i1 / Q;
      int h0 = pr0 * HC + (i0 - pr0 * Q), h1 = pr1 * HC + (i1 - pr1 * Q);
      // padding pixels of the last K-step: their dY rows are zero, any halo row will do
      h0 = i0 < TP * Q ? h0 : 0;
      h1 = i1 < TP * Q ? h1 : 0;
      bf16x8 af[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int col = (kb0 + a) * 16 + 4 * tp;
        af[a] = tr(dyl, wg_off64(i0, col), wg_off64(i1, col));
      }
#pragma unroll
      for (int c = 0; c < NCBW; ++c) {
        const int colg = (cb0 + c) * 16;                 // dW column block: tap (r, s), channels cc..cc+15
        const int tap = colg / C, cc = colg - tap * C;
        const int r = tap / S, s = tap - r * S;
        const int sh = r * HC + s;
        const bf16x8 bfr = tr(xl, wb_xoff<C>(h0 + sh, cc + 4 * tp), wb_xoff<C>(h1 + sh, cc + 4 * tp));
        acc[0][c] = mfma16(af[0], bfr, acc[0][c]);
        acc[1][c] = mfma16(af[1], bfr, acc[1][c]);
      }
    }
  };

  int band = blockIdx.x;
  if (band < nbands) gload(band);
  for (; band < nbands; band += gridDim.x) {
    __syncthreads();              // the previous band's fragment reads are done
    lstore();
    __syncthreads();
    if (band + (int)gridDim.x < nbands) gload(band + gridDim.x);   // in flight during the MFMAs
    compute();
  }
  // this workgroup's partial: row = output channel kb*16 + 4*(lane>>4) + e, col = block*16 + (lane&15)
  float* dst = part + (size_t)blockIdx.x * 64 * KTOT;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < NCBW; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        dst[(size_t)((kb0 + a) * 16 + gq * 4 + e) * KTOT + (cb0 + c) * 16 + li] = acc[a][c][e];
}

}  // namespace zoo

using namespace zoo;

// split plan of the pixel reduction: sets g->m_per_split, returns the number of splits
static int wgrad_bm(const WgradGeom& g) {
  static const int narrow = 1;
  return (narrow && g.K <= 64) ? 64 : 128;
}

extern "C" int zoo_wgrad_plan(WgradGeom* gp) {
  WgradGeom& g = *gp;
  const int bm = wgrad_bm(g);
  const int tiles = ((g.K + bm - 1) / bm) * ((g.Ktot + WG_BN - 1) / WG_BN);
  // split the pixel reduction so that ~target workgroups are in flight, >= min_pix pixels each.
  // 512 (one occupancy-full wave of 2 per CU) rather than 1024: the side-stream weight gradients
  // then hold fewer CUs at a time next to the compute stream and write half the partials
  // (ResNet-50 b256 +0.7 %, profiles/r5/ab_wgrad_wg_r5.log)
  static const int target = 512;
  static const int min_pix = 512;
  int splits = (target + tiles - 1) / tiles;
  const int max_splits = (g.M + min_pix - 1) / min_pix;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int mps = (g.M + splits - 1) / splits;
  mps = (mps + WG_BK - 1) / WG_BK * WG_BK;
  splits = (g.M + mps - 1) / mps;
  g.m_per_split = mps;
  return splits;
}

// part: null (fp32 atomics into dW) or [splits][K][Ktot] scratch from zoo_wgrad_plan
extern "C" hipError_t zoo_wgrad(const void* X, const void* dY, float* dW, float* part, const WgradGeom* gin,
                                hipStream_t st) {
  WgradGeom g = *gin;
  const int bm = wgrad_bm(g);
  const int tiles = ((g.K + bm - 1) / bm) * ((g.Ktot + WG_BN - 1) / WG_BN);
  const int splits = zoo_wgrad_plan(&g);
  if (splits <= 1) part = nullptr;
  const size_t smem = (size_t)2 * WG_BK * (bm + WG_BN) * sizeof(bf16_t);
  // LDS-DMA staging: slower in round 2 (bench 8912 vs 9045 img/s with register staging), ahead
  // by 0.1-0.4 % in five round-5 pairs on the side stream (profiles/r5/ab_wgrad_wg_r5.log)
  constexpr bool dma = true;
  if (g.C == 4) {
    if (bm == 64)
      hipLaunchKernelGGL((wgrad_kernel<4, false, 64>), dim3(tiles * splits), dim3(256), smem, st,
                         (const bf16_t*)X, (const bf16_t*)dY, dW, part, g);
    else
      hipLaunchKernelGGL((wgrad_kernel<4, false, 128>), dim3(tiles * splits), dim3(256), smem, st,
                         (const bf16_t*)X, (const bf16_t*)dY, dW, part, g);
  } else if (bm == 64) {
    hipLaunchKernelGGL((wgrad_kernel<8, false, 64>), dim3(tiles * splits), dim3(256), smem, st, (const bf16_t*)X,
                       (const bf16_t*)dY, dW, part, g);
  } else if (dma) {
    hipLaunchKernelGGL((wgrad_kernel<8, true, 128>), dim3(tiles * splits), dim3(256), smem, st, (const bf16_t*)X,
                       (const bf16_t*)dY, dW, part, g);
  } else {
    hipLaunchKernelGGL((wgrad_kernel<8, false, 128>), dim3(tiles * splits), dim3(256), smem, st, (const bf16_t*)X,
                       (const bf16_t*)dY, dW, part, g);
  }
  if (part) {
    const size_t n4 = (size_t)g.K * (g.Ktot / 4);
    const int blocks = (int)((n4 + 255) / 256 < 4096 ? (n4 + 255) / 256 : 4096);
    const float* src = part;
    int n = splits;
    if (splits > kFoldGroup) {  // level 1 in place of the first groups' slots: group g -> slot g
      const int groups = (splits + kFoldGroup - 1) / kFoldGroup;
      float* lvl1 = part + (size_t)splits * g.K * g.Ktot;  // scratch after the partials
      hipLaunchKernelGGL(wgrad_fold1_kernel, dim3((unsigned)((n4 + 255) / 256), groups), dim3(256), 0, st, part,
                         lvl1, n4, splits);
      src = lvl1;
      n = groups;
    }
    hipLaunchKernelGGL(wgrad_fold_kernel, dim3(blocks), dim3(256), 0, st, src, dW, g.K, g.Ktot, g.ldw, n);
  }
  return hipGetLastError();
}

// final fold of a TRANSPOSED band partial: the 1x1 64 -> 256 convs run the band kernel with the
// operands swapped (64-channel X in the dY role, 256-channel dY in the X role), so the partials are
// dW^T [64][Ktot]; this sums the n partial rows in order and adds element (c, k) into dW[k][c]
__global__ __launch_bounds__(256) void wgrad_fold_t_kernel(const float* __restrict__ part, float* __restrict__ dW,
                                                          int Ktot, int ldw, int splits) {
  const int n = 64 * Ktot;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int c = i / Ktot, k = i - c * Ktot;
    float s = part[i], t = 0.f;
    int sp = 1;
    for (; sp + 1 < splits; sp += 2) {
      s += part[(size_t)sp * n + i];
      t += part[(size_t)(sp + 1) * n + i];
    }
    if (sp < splits) s += part[(size_t)sp * n + i];
    dW[(size_t)k * ldw + c] += s + t;
  }
}

// band weight gradient (wgrad_band_kernel): stride-1, K = 64 output channels, one of the shapes
// instantiated below. Returns the number of partial rows it needs (0 = not handled); with
// part != null it also runs the kernel and the ordered fold into dW.
template <int R, int S, int C, int TP, int Q>
static int wb_run(const WgradGeom& g, const void* X, const void* dY, float* dW, float* part, hipStream_t st,
                  bool transposed = false) {
  using Cfg = WbCfg<R, S, C, TP, Q>;
  auto kfn = &wgrad_band_kernel<R, S, C, TP, Q>;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)Cfg::SMEM);
    attr = true;
  }
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const int nbands = g.N * ((g.P + TP - 1) / TP);
  static const int target = 0;
  int G = target > 0 ? target : ncu;
  if (G > nbands) G = nbands;
  if (!part) return G + (G > kFoldGroup ? (G + kFoldGroup - 1) / kFoldGroup : 0);
  hipLaunchKernelGGL(kfn, dim3(G), dim3(Cfg::NT), Cfg::SMEM, st, (const bf16_t*)X, (const bf16_t*)dY, part, g);
  const int Ktot = R * S * C;
  const size_t n4 = (size_t)64 * (Ktot / 4);
  const int blocks = (int)((n4 + 255) / 256 < 4096 ? (n4 + 255) / 256 : 4096);
  const float* src = part;
  int n = G;
  if (G > kFoldGroup) {
    const int groups = (G + kFoldGroup - 1) / kFoldGroup;
    float* lvl1 = part + (size_t)G * 64 * Ktot;
    hipLaunchKernelGGL(wgrad_fold1_kernel, dim3((unsigned)((n4 + 255) / 256), groups), dim3(256), 0, st, part, lvl1,
                       n4, G);
    src = lvl1;
    n = groups;
  }
  if (transposed)
    hipLaunchKernelGGL(wgrad_fold_t_kernel, dim3((64 * Ktot + 255) / 256), dim3(256), 0, st, src, dW, Ktot, g.ldw, n);
  else
    hipLaunchKernelGGL(wgrad_fold_kernel, dim3(blocks), dim3(256), 0, st, src, dW, 64, Ktot, g.ldw, n);
  return G;
}

// 0: not a band shape; else the number of [64][Ktot] fp32 partial rows the call needs (part ==
// null), or runs it (part != null)
extern "C" int zoo_wgrad_band(const WgradGeom* gp, const void* X, const void* dY, float* dW, float* part,
                              hipStream_t st) {
  // 1: every band shape; 2: only the 64-output-channel ones (A/B of the transposed 64 -> 256 case)
  static const int on = [] {
    const char* e = getenv("ZOO_WGRAD_BAND");
    return e ? atoi(e) : 1;
  }();
  const WgradGeom& g = *gp;
  if (!on || g.sh != 1 || g.sw != 1 || g.dh != 1 || g.dw != 1 || g.P != g.H + 2 * g.ph - g.R + 1 ||
      g.Q != g.W + 2 * g.pw - g.S + 1)
    return 0;
  if (on == 1 && g.K == 256 && g.R == 1 && g.S == 1 && g.C == 64 && g.ph == 0 && g.pw == 0 && g.Q == 56) {
    // 1x1 64 -> 256 (stage-1 conv3 and projection shortcut): dW^T = X^T dY is the 256-channel
    // band shape with the operands swapped; the fold writes it back transposed. wgrad256's
    // im2col kernel took 180-580 us per call there on the side stream, the last work of the step
    // (profiles/r6/ab4_prof_rn_step_r6.md rows 320-368)
    WgradGeom t = g;
    t.C = 256;
    t.K = 64;
    t.Ktot = 256;
    return wb_run<1, 1, 256, 4, 56>(t, dY, X, dW, part, st, true);
  }
  if (g.K != 64) return 0;
  if (g.R == 4 && g.S == 4 && g.C == 16 && g.ph == 0 && g.pw == 0 && g.Q == 112)
    return wb_run<4, 4, 16, 4, 112>(g, X, dY, dW, part, st);
  if (g.R == 3 && g.S == 3 && g.C == 64 && g.ph == 1 && g.pw == 1 && g.Q == 56)
    return wb_run<3, 3, 64, 4, 56>(g, X, dY, dW, part, st);
  if (g.R == 1 && g.S == 1 && g.C == 64 && g.ph == 0 && g.pw == 0 && g.Q == 56)
    return wb_run<1, 1, 64, 4, 56>(g, X, dY, dW, part, st);
  if (g.R == 1 && g.S == 1 && g.C == 256 && g.ph == 0 && g.pw == 0 && g.Q == 56)
    return wb_run<1, 1, 256, 4, 56>(g, X, dY, dW, part, st);
  return 0;
}
