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

}  // namespace zoo

using namespace zoo;

// split plan of the pixel reduction: sets g->m_per_split, returns the number of splits
static int wgrad_bm(const WgradGeom& g) {
  static const int narrow = [] {
    const char* e = getenv("ZOO_WGRAD_BM64");
    return e ? atoi(e) : 1;
  }();
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
  static const int target = [] {
    const char* e = getenv("ZOO_WGRAD_WG");
    return e ? atoi(e) : 512;
  }();
  static const int min_pix = [] {
    const char* e = getenv("ZOO_WGRAD_MINPIX");
    return e ? atoi(e) : 512;
  }();
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
  static const bool dma = [] {
    // LDS-DMA staging: slower in round 2 (bench 8912 vs 9045 img/s with register staging), ahead
    // by 0.1-0.4 % in five round-5 pairs on the side stream (profiles/r5/ab_wgrad_wg_r5.log)
    const char* e = getenv("ZOO_WGRAD_DMA");
    return e ? atoi(e) != 0 : true;
  }();
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
