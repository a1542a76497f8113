// Implicit-GEMM convolution / GEMM on CDNA4 matrix cores (gfx950).
//
// One kernel template covers every "K-contiguous" GEMM in the framework:
//   * conv forward (NHWC activations, weights [Cout][R][S][Cin])
//   * conv data-gradient (a transposed conv: input dilation = forward stride,
//     weights pre-flipped to [Cin][R][S][Cout] by `flip_weights_kernel`)
//   * 1x1 convs and Linear layers (A is a plain row-major [M][K] matrix)
//
// Replaces the reference's MKL im2col+sgemm / MKL-DNN conv primitives
// (BigDL SpatialConvolution, used by Zs/pipeline/api/keras/layers/Convolution2D.scala:86-110
// and Dense.scala) — see SURVEY.md §2.16 HK1/HK3/HK5.
//
// Tiling: BM=128 rows (output pixels) x BN={64,128} cols (output channels) x
// BK=64, 256 threads = 4 waves in a 2x2 grid, each wave owns a 64 x BN/2 tile
// computed with v_mfma_f32_16x16x32_bf16 (8 bf16 per lane per operand).
// A/B tiles are register-staged (the im2col gather needs per-lane addresses and
// zero-fill for padding) into a double-buffered, XOR-swizzled LDS image; the
// global loads of tile k+1 are in flight while tile k is on the MFMA pipe.
// The epilogue stages the fp32 accumulators through LDS so that every global
// store is a full 16-byte row segment, and optionally fuses bias, residual add,
// activation and per-channel BatchNorm statistics (sum, sum of squares).
#include <stdlib.h>

#include "common.h"
#include "geom.h"
#include "bnmask.h"

namespace zoo {



constexpr int IG_BM = 128, IG_BK = 64, IG_NT = 256;

typedef __attribute__((address_space(3))) void ig_lds_void;
typedef __attribute__((address_space(1))) const void ig_gl_void;
// zero page for LDS-DMA of out-of-range rows / padding taps
__device__ __attribute__((aligned(16))) bf16_t ig_zero_page[8];

ZOO_DEV int ig_swz(int row) { return (row >> 1) & 7; }

// LEAN: the plain-conv epilogue (bf16 output, optional BN statistics; no bias / residual /
// activation / fp32 output / row remap / fused BN-backward): the tile is staged through LDS
// as bf16 (half the LDS of the fp32 staging, so 6 instead of 4 workgroups fit per CU) and
// stored with precomputed row pointers. The general epilogue was instruction-issue bound on
// the memory-bound 1x1 convolutions (rocprofv3: SQ_ACTIVE_INST_ANY ~ the whole wave lifetime
// at 3.4 resident waves per SIMD, profiles/conv1x1_r2.md).
// EPI: 0 general epilogue; 1 LEAN (above); 2 backward epilogue (no bias / activation / fp32
// output: residual-gradient add, producer ReLU mask and fused BN-backward sums) with the
// per-column BN constants hoisted out of the row loop.
template <int VEC, bool IS1x1, bool LDIL, int BN, bool DMA, int EPI>
__global__ __launch_bounds__(256, 2) void igemm_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wm, bf16_t* __restrict__ Y,
    float* __restrict__ Yf, const float* __restrict__ bias, const bf16_t* __restrict__ resid,
    float* __restrict__ stats, ConvGeom g, int act, BwdStats bs) {
  constexpr int BM = IG_BM, BK = IG_BK;
  constexpr int WN = BN / 2;      // wave tile width
  constexpr int NJ = WN / 16;     // 16-wide n tiles per wave
  constexpr int NI = 4;           // 16-high m tiles per wave (wave tile height 64)
  constexpr int B_ROWS_PER_THREAD = BN / 32;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  // single-K-tile GEMMs (1x1 convs with C <= 64) need no second stage buffer:
  // the launcher then sizes LDS for one stage, which raises occupancy
  const int nbuf = g.ldb > BK ? 2 : 1;
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + nbuf * BM * BK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int ntn = (g.K + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / ntn, tn = bid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- staging assignment: thread -> (16-byte k-chunk, rows) ----
  // DMA staging writes LDS lane-linearly (lane -> 16-byte slot lane&7 of row lane>>3 of the
  // wave's 8-row group), so the XOR swizzle is applied by choosing which k-chunk each lane
  // loads; ig_swz depends on row bits 1..3 only, so it is the same for all rows of a thread
  const int rbase = tid >> 3;  // 0..31
  const int cc = DMA ? ((tid & 7) ^ ig_swz(rbase)) : (tid & 7);

  // per-row precompute for the A (activation) gather
  int a_base[4], a_ih[4], a_iw[4];
  bool a_ok[4];
  const int PQ = g.P * g.Q;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rbase + 32 * i;
    a_ok[i] = m < g.M;
    const int mm = a_ok[i] ? m : 0;
    if constexpr (IS1x1) {
      a_base[i] = mm * g.C;
      a_ih[i] = a_iw[i] = 0;
    } else {
      const int n = mm / PQ;
      const int pq = mm - n * PQ;
      const int p = pq / g.Q;
      const int q = pq - p * g.Q;
      a_base[i] = n * g.H * g.W * g.C;
      a_ih[i] = p * g.sh - g.ph;
      a_iw[i] = q * g.sw - g.pw;
    }
  }
  // k position of this thread's chunk (VEC==8 path): (kr, ks, kc)
  int kr = 0, ks = 0, kc = cc * 8;
  if constexpr (!IS1x1 && VEC == 8) {
    while (kc >= g.C) { kc -= g.C; if (++ks == g.S) { ks = 0; ++kr; } }
  }

  uint4 ra[4], rb[B_ROWS_PER_THREAD];
  const int nk = (g.ldb + BK - 1) / BK;

  // LDS-DMA: per-lane 16-byte global source, wave-uniform LDS base (lane-linear image)
  auto dma16 = [&](const bf16_t* src, bf16_t* dst) {
    __builtin_amdgcn_global_load_lds((ig_gl_void*)src, (ig_lds_void*)dst, 16, 0, 0);
  };
  auto load_tile = [&](int kt) {
    const int k = kt * BK + cc * 8;
    // wave-uniform LDS row-group bases of this tile's buffer (DMA path)
    bf16_t* adst = As + (kt & 1) * BM * BK + (wid * 8) * BK;
    bf16_t* bdst = Bs + (kt & 1) * BN * BK + (wid * 8) * BK;
    (void)adst; (void)bdst;
    // ---- A ----
    if constexpr (IS1x1) {
      const bool kok = k < g.Ktot;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (DMA) {
          dma16(a_ok[i] && kok ? X + a_base[i] + k : ig_zero_page, adst + (32 * i) * BK);
        } else {
          ra[i] = (a_ok[i] && kok) ? *reinterpret_cast<const uint4*>(X + a_base[i] + k)
                                   : make_uint4(0, 0, 0, 0);
        }
      }
    } else if constexpr (VEC == 8) {
      const bool kok = kr < g.R;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int ih = a_ih[i] + kr * g.dh, iw = a_iw[i] + ks * g.dw;
        bool ok = a_ok[i] && kok;
        if constexpr (LDIL) {
          ok = ok && ih >= 0 && iw >= 0 && (ih % g.lh) == 0 && (iw % g.lw) == 0;
          ih /= g.lh; iw /= g.lw;
          ok = ok && ih < g.H && iw < g.W;
        } else {
          ok = ok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        }
        if constexpr (DMA) {
          dma16(ok ? X + a_base[i] + (ih * g.W + iw) * g.C + kc : ig_zero_page, adst + (32 * i) * BK);
        } else {
          ra[i] = ok ? *reinterpret_cast<const uint4*>(X + a_base[i] + (ih * g.W + iw) * g.C + kc)
                     : make_uint4(0, 0, 0, 0);
        }
      }
    } else {  // VEC == 4: C == 4, each 8-element chunk spans two filter taps
      const int pos0 = k >> 2;
      uint2 lo[4], hi[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pos = pos0 + h;
        const int r = pos / g.S, s = pos - (pos / g.S) * g.S;
        const bool kok = r < g.R;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ih = a_ih[i] + r * g.dh, iw = a_iw[i] + s * g.dw;
          const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
          const uint2 v = ok ? *reinterpret_cast<const uint2*>(X + a_base[i] + (ih * g.W + iw) * 4)
                             : make_uint2(0, 0);
          if (h == 0) lo[i] = v; else hi[i] = v;
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) ra[i] = make_uint4(lo[i].x, lo[i].y, hi[i].x, hi[i].y);
    }
    // ---- B (weights, row-major [K][ldb]) ----
    const bool kokb = k < g.ldb;
#pragma unroll
    for (int i = 0; i < B_ROWS_PER_THREAD; ++i) {
      const int n = n0 + rbase + 32 * i;
      if constexpr (DMA) {
        dma16(n < g.K && kokb ? Wm + (size_t)n * g.ldb + k : ig_zero_page, bdst + (32 * i) * BK);
      } else {
        rb[i] = (n < g.K && kokb) ? *reinterpret_cast<const uint4*>(Wm + (size_t)n * g.ldb + k)
                                  : make_uint4(0, 0, 0, 0);
      }
    }
    // advance the incremental k decode for the next tile
    if constexpr (!IS1x1 && VEC == 8) {
      kc += BK;
      while (kc >= g.C) { kc -= g.C; if (++ks == g.S) { ks = 0; ++kr; } }
    }
  };

  auto store_tile = [&](int buf) {
    bf16_t* a = As + buf * BM * BK;
    bf16_t* b = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = rbase + 32 * i;
      *reinterpret_cast<uint4*>(a + row * BK + ((cc ^ ig_swz(row)) << 3)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_ROWS_PER_THREAD; ++i) {
      const int row = rbase + 32 * i;
      *reinterpret_cast<uint4*>(b + row * BK + ((cc ^ ig_swz(row)) << 3)) = rb[i];
    }
  };

  f32x4 acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;

  auto compute = [&](int buf) {
    const bf16_t* a = As + buf * BM * BK;
    const bf16_t* b = Bs + buf * BN * BK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;
      bf16x8 af[NI], bfg[NJ];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const bf16x8*>(a + row * BK + ((chunk ^ ig_swz(row)) << 3));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * WN + j * 16 + fr;
        bfg[j] = *reinterpret_cast<const bf16x8*>(b + row * BK + ((chunk ^ ig_swz(row)) << 3));
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(af[i], bfg[j], acc[i][j]);
    }
  };

  // ---- EPI 2 operand prefetch (1x1 dgrads: a short K loop, often one tile) ----
  // The backward epilogue's global operands (residual gradient, producer y, ReLU mask) do not
  // depend on the GEMM: for 1x1 layers their first batch of loads is issued here, so it is in
  // flight together with the operand DMA instead of after the MFMAs (ZOO_EPI2_BATCH=0: off).
  constexpr int E2_CPR = BN / 8, E2_RSTEP = IG_NT / E2_CPR;
  constexpr int E2_NP = BM / E2_RSTEP, E2_PB = E2_NP < 4 ? E2_NP : 4;
  const int e2_ch = tid % E2_CPR, e2_rr0 = tid / E2_CPR, e2_col0 = n0 + e2_ch * 8;
  const bool e2_fast = EPI == 2 && e2_col0 < g.K && g.M - m0 >= BM && !bs.zgelu && !bs.unbatched;
  size_t e2_off[E2_PB];
  uint4 e2_rv[E2_PB], e2_yv[E2_PB], e2_zv[E2_PB];
  unsigned e2_mb[E2_PB];
  auto e2_fetch = [&](int p0) {
#pragma unroll
    for (int u = 0; u < E2_PB; ++u) {
      const int m = m0 + e2_rr0 + (p0 + u) * E2_RSTEP;
      if (g.omap) {
        const int n = m / PQ, pq = m - n * PQ;
        const int p = pq / g.Q, q = pq - p * g.Q;
        e2_off[u] = ((size_t)(n * g.oH + g.oh0 + g.osh * p) * g.oW + g.ow0 + g.osw * q) * g.K + e2_col0;
      } else {
        e2_off[u] = (size_t)m * g.K + e2_col0;
      }
      e2_rv[u] = e2_yv[u] = e2_zv[u] = uint4{0u, 0u, 0u, 0u};
      e2_mb[u] = 0u;
      if (resid) e2_rv[u] = *reinterpret_cast<const uint4*>(resid + e2_off[u]);
      if (bs.sums) e2_yv[u] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + e2_off[u]);
      if (bs.zmode == 2) e2_mb[u] = reinterpret_cast<const uint8_t*>(bs.z)[e2_off[u] >> 3];
      else if (bs.zmode == 0 && bs.z)
        e2_zv[u] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.z) + e2_off[u]);
    }
  };
  // only for 1-2 K-tiles: across a longer K loop the held registers and the extra in-flight
  // loads cost more than they hide (conv3 dgrad, Ktot 256: 161 -> 178 us; conv1, Ktot 64:
  // 303 -> 275 us, profiles/r3/epilogue_batching_r3.md)
  const bool e2_early = IS1x1 && e2_fast && g.ldb <= 2 * BK;
  if constexpr (EPI == 2 && IS1x1) {
    if (e2_early) e2_fetch(0);
  }

  // ---- main loop: one barrier per K tile, loads of tile k+1 overlap MFMA on tile k ----
  if constexpr (DMA) {
    // tile k+1 streams into the other LDS buffer (free since the previous barrier)
    // while tile k is on the MFMA pipe; vmcnt(0) + barrier publish it
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

  if constexpr (EPI == 1) {
    // bf16 staging, pitch BN+4 elements: the 4 row groups of a ds_write_b16 land 8 banks apart
    constexpr int LD16 = BN + 4;
    bf16_t* C16 = reinterpret_cast<bf16_t*>(smem);
    float* wst = reinterpret_cast<float*>(smem + ((BM * LD16 * 2 + 15) / 16) * 16);  // [2 wm][BN][2]
    if (stats) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float q = bf2f(f2bf(acc[i][j][r]));
            a += q;
            b += q * q;
          }
        a += __shfl_xor(a, 16, 64);
        b += __shfl_xor(b, 16, 64);
        a += __shfl_xor(a, 32, 64);
        b += __shfl_xor(b, 32, 64);
        if (fq == 0) {
          const int col = wn * WN + j * 16 + fr;
          wst[(wm * BN + col) * 2 + 0] = a;
          wst[(wm * BN + col) * 2 + 1] = b;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          C16[(wm * 64 + i * 16 + fq * 4 + r) * LD16 + wn * WN + j * 16 + fr] = f2bf(acc[i][j][r]);
    __syncthreads();
    constexpr int CPR = BN / 8, RSTEP = IG_NT / CPR;
    const int ch = tid % CPR, rr0 = tid / CPR;
    const int col0 = n0 + ch * 8;
    if (col0 < g.K) {
      const int rend = min(BM, g.M - m0);
      bf16_t* yp = Y + (size_t)(m0 + rr0) * g.K + col0;
      const bf16_t* cp = C16 + rr0 * LD16 + ch * 8;
      for (int rr = rr0; rr < rend; rr += RSTEP, yp += (size_t)RSTEP * g.K, cp += RSTEP * LD16) {
        const uint2 lo = *reinterpret_cast<const uint2*>(cp);
        const uint2 hi = *reinterpret_cast<const uint2*>(cp + 4);
        *reinterpret_cast<uint4*>(yp) = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    }
    if (stats && tid < BN && n0 + tid < g.K) {
      const float a = wst[tid * 2] + wst[(BN + tid) * 2];
      const float b = wst[tid * 2 + 1] + wst[(BN + tid) * 2 + 1];
      if (g.stat_slots == kStatPartial) {
        float* const dst = stats + (size_t)tm * 2 * g.K;
        dst[n0 + tid] = a;
        dst[g.K + n0 + tid] = b;
      } else {
        float* const dst = g.stat_slots > 0 ? slot_ptr(stats, 2 * g.K, g.stat_slots) : stats;
        atomicAdd(dst + n0 + tid, a);
        atomicAdd(dst + g.K + n0 + tid, b);
      }
    }
    return;
  }

  // ---- epilogue: stage fp32 tile in LDS, then row-contiguous 16-byte stores ----
  constexpr int EPI_LD = BN + 4;  // fp32 pitch: rows r and r+4 land 16 banks apart
  float* Cs = reinterpret_cast<float*>(smem);
  // Plain forward conv with BN statistics (no bias/residual/activation): reduce the
  // statistics straight from the accumulators (bf16-rounded, as stored) -- column
  // sums over the wave's 64 rows need two cross-lane steps -- and park the two
  // row-waves' partials next to the staging tile; no extra barrier is needed.
  const bool reg_stats = stats && !bias && !resid && act == 0 && !Yf && !g.omap;
  float* wstat = Cs + BM * EPI_LD;  // [2 wm][BN][2]
  if (reg_stats) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float q = bf2f(f2bf(acc[i][j][r]));
          a += q;
          b += q * q;
        }
      a += __shfl_xor(a, 16, 64);
      b += __shfl_xor(b, 16, 64);
      a += __shfl_xor(a, 32, 64);
      b += __shfl_xor(b, 32, 64);
      if (fq == 0) {
        const int col = wn * WN + j * 16 + fr;
        wstat[(wm * BN + col) * 2 + 0] = a;
        wstat[(wm * BN + col) * 2 + 1] = b;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = wm * 64 + i * 16 + fq * 4 + r;
        const int col = wn * WN + j * 16 + fr;
        Cs[row * EPI_LD + col] = acc[i][j][r];
      }
  __syncthreads();

  constexpr int CPR = BN / 8;            // 8-column chunks per row
  constexpr int RSTEP = IG_NT / CPR;     // rows handled per pass
  const int ch = tid % CPR;
  const int rr0 = tid / CPR;
  const int col0 = n0 + ch * 8;
  const bool col_ok = col0 < g.K;        // K % 8 == 0 is required by the launcher
  float bsv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bsv[e] = (bias && col_ok) ? bias[col0 + e] : 0.f;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }

  if constexpr (EPI == 2) {
    float mu[8], iv[8], msc[8], msh[8];
    const bool bnsum = bs.sums && !bs.zgelu;
    if (bnsum && col_ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { mu[e] = bs.mean[col0 + e]; iv[e] = bs.inv[col0 + e]; }
    }
    bnm_coeffs(bs, col0, col_ok && !bs.zgelu, msc, msh);
    const int rend = min(BM, g.M - m0);
    // Full tiles: the global loads (residual gradient, producer y, mask) of PB passes are all
    // issued before the first of their stores, so each wave keeps PB x 2-3 16-byte loads in
    // flight instead of one pass's worth (the row loop is otherwise latency-bound: a stage-1
    // conv1 dgrad moved ~1.4 GB at 3.9 TB/s). Each element is still read before it is written
    // by the same lane, so an in-place residual (resid == Y) stays correct.
    constexpr int NP = E2_NP, PB = E2_PB;
    static_assert(E2_RSTEP == RSTEP, "EPI 2 prefetch geometry");
    if (e2_fast) {
#pragma unroll
      for (int p0 = 0; p0 < NP; p0 += PB) {
        if (!(p0 == 0 && e2_early)) e2_fetch(p0);  // batch 0 may be in flight since the prologue
        const size_t* offs = e2_off;
        const uint4* rv = e2_rv;
        const uint4* yv = e2_yv;
        const uint4* zv = e2_zv;
        const unsigned* mb = e2_mb;
#pragma unroll
        for (int u = 0; u < PB; ++u) {
          const int rr = rr0 + (p0 + u) * RSTEP;
          const float4 lo = *reinterpret_cast<const float4*>(Cs + rr * EPI_LD + ch * 8);
          const float4 hi = *reinterpret_cast<const float4*>(Cs + rr * EPI_LD + ch * 8 + 4);
          float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          if (resid) {
            float r8[8];
            unpack8(rv[u], r8);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += r8[e];
          }
          float yy[8];
          unpack8(yv[u], yy);
          bnm_apply_pre(bs, yy, msc, msh, mb[u], zv[u], v);
          const uint4 pk = pack8(v);
          *reinterpret_cast<uint4*>(Y + offs[u]) = pk;
          if (bnsum) {
            float q[8];
            unpack8(pk, q);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              s1[e] += q[e];
              s2[e] += q[e] * (yy[e] - mu[e]) * iv[e];
            }
          }
        }
      }
    } else
    for (int rr = rr0; col_ok && rr < rend; rr += RSTEP) {
      const int m = m0 + rr;
      float v[8];
      const float4 lo = *reinterpret_cast<const float4*>(Cs + rr * EPI_LD + ch * 8);
      const float4 hi = *reinterpret_cast<const float4*>(Cs + rr * EPI_LD + ch * 8 + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
      v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
      size_t off;
      if (g.omap) {
        const int n = m / PQ, pq = m - n * PQ;
        const int p = pq / g.Q, q = pq - p * g.Q;
        off = ((size_t)(n * g.oH + g.oh0 + g.osh * p) * g.oW + g.ow0 + g.osw * q) * g.K + col0;
      } else {
        off = (size_t)m * g.K + col0;
      }
      if (resid) {
        float rv[8];
        unpack8(*reinterpret_cast<const uint4*>(resid + off), rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rv[e];
      }
      float yy[8];
      if (bnsum) unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off), yy);
      if (bs.zgelu) {
        float zz[8];
        unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.z) + off), zz);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu_grad_f(zz[e]);
      } else {
        bnm_apply(bs, off, yy, msc, msh, v);
      }
      const uint4 pk = pack8(v);
      *reinterpret_cast<uint4*>(Y + off) = pk;
      if (bs.sums) {
        float q[8];
        unpack8(pk, q);
        if (bs.zgelu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) s1[e] += q[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += q[e];
            s2[e] += q[e] * (yy[e] - mu[e]) * iv[e];
          }
        }
      }
    }
  } else
  for (int rr = rr0; rr < BM; rr += RSTEP) {
    const int m = m0 + rr;
    if (m >= g.M || !col_ok) continue;
    float v[8];
    const float4 lo = *reinterpret_cast<const float4*>(Cs + rr * EPI_LD + ch * 8);
    const float4 hi = *reinterpret_cast<const float4*>(Cs + rr * EPI_LD + ch * 8 + 4);
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    size_t off;
    if (g.omap) {
      const int n = m / PQ, pq = m - (m / PQ) * PQ;
      const int p = pq / g.Q, q = pq - (pq / g.Q) * g.Q;
      off = ((size_t)(n * g.oH + g.oh0 + g.osh * p) * g.oW + g.ow0 + g.osw * q) * g.K + col0;
    } else {
      off = (size_t)m * g.K + col0;
    }
    if (resid) {
      float rv[8];
      unpack8(*reinterpret_cast<const uint4*>(resid + off), rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += rv[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e] + bsv[e], act);
    if (Yf) {
      *reinterpret_cast<float4*>(Yf + off) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(Yf + off + 4) = make_float4(v[4], v[5], v[6], v[7]);
    }
    float yy[8];
    if (bs.sums) {  // fused BN-backward: mask with the producer's ReLU, accumulate (dy, dy*xhat)
      unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off), yy);
      float msc[8], msh[8];
      bnm_coeffs(bs, col0, true, msc, msh);
      bnm_apply(bs, off, yy, msc, msh, v);
    }
    if (Y) {
      const uint4 pk = pack8(v);
      *reinterpret_cast<uint4*>(Y + off) = pk;
      if (stats && !reg_stats) {  // statistics of the values actually stored (bf16-rounded)
        float q[8];
        unpack8(pk, q);
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] += q[e]; s2[e] += q[e] * q[e]; }
      } else if (bs.sums) {
        float q[8];
        unpack8(pk, q);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          s1[e] += q[e];
          s2[e] += q[e] * (yy[e] - bs.mean[col0 + e]) * bs.inv[col0 + e];
        }
      }
    }
  }

  if (reg_stats) {
    if (tid < BN && n0 + tid < g.K) {
      const float a = wstat[tid * 2] + wstat[(BN + tid) * 2];
      const float b = wstat[tid * 2 + 1] + wstat[(BN + tid) * 2 + 1];
      if (g.stat_slots == kStatPartial) {
        float* const dst = stats + (size_t)tm * 2 * g.K;
        dst[n0 + tid] = a;
        dst[g.K + n0 + tid] = b;
      } else {
        float* const dst = g.stat_slots > 0 ? slot_ptr(stats, 2 * g.K, g.stat_slots) : stats;
        atomicAdd(dst + n0 + tid, a);
        atomicAdd(dst + g.K + n0 + tid, b);
      }
    }
    return;
  }
  float* const sacc = stats ? stats : bs.sums;
  if (sacc) {
    // threads sharing a column chunk: tid % CPR equal. Reduce within the wave
    // (lanes differing in bits >= log2(CPR)), then across waves through LDS.
    __syncthreads();
    float* red = Cs;  // reuse: [4 waves][BN][2]
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    }
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wid * BN + ch * 8 + e) * 2 + 0] = s1[e];
        red[(wid * BN + ch * 8 + e) * 2 + 1] = s2[e];
      }
    }
    __syncthreads();
    if (tid < BN) {
      const int col = n0 + tid;
      if (col < g.K) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) { a += red[(w * BN + tid) * 2]; b += red[(w * BN + tid) * 2 + 1]; }
        if (g.stat_slots == kStatPartial) {
          float* const dst = sacc + (size_t)tm * 2 * g.K;
          dst[col] = a;
          dst[g.K + col] = b;
        } else {
          float* const dst = g.stat_slots > 0 ? slot_ptr(sacc, 2 * g.K, g.stat_slots) : sacc;
          atomicAdd(dst + col, a);
          atomicAdd(dst + g.K + col, b);
        }
      }
    }
  }
}

// Wt[c][t][u][k] = W[k][r0 + sh*(Ra-1-t)][s0 + sw*(Sb-1-u)][c]
// (flipped sub-filter of one output-parity class of a strided conv's dgrad;
//  r0=s0=0, sh=sw=1, Ra=R, Sb=S is the plain flipped filter). W rows have leading dim ldw.
__global__ void flip_weights_kernel(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wt, int K, int R, int S,
                                    int C, int ldw, int r0, int s0, int Ra, int Sb, int sh, int sw, int ldt) {
  const int total = C * Ra * Sb * K;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    int t = idx;
    const int k = t % K; t /= K;
    const int u = t % Sb; t /= Sb;
    const int v = t % Ra; t /= Ra;
    const int c = t;
    const int r = r0 + sh * (Ra - 1 - v), s = s0 + sw * (Sb - 1 - u);
    Wt[(size_t)c * ldt + (v * Sb + u) * K + k] = W[(size_t)k * ldw + (r * S + s) * C + c];
  }
}

// All the flipped (sub-)filters a training step's dgrads need, in ONE launch (once per
// optimizer step instead of one launch per conv per backward). Descriptor d owns blocks
// [blk0, blk0 + nblk); the descriptor table is sorted by blk0.
__global__ __launch_bounds__(256) void flip_weights_batched_kernel(const FlipDesc* __restrict__ descs, int n) {
  int lo = 0, hi = n - 1;
  const int b = blockIdx.x;
  while (lo < hi) {  // last descriptor with blk0 <= b (uniform across the block)
    const int mid = (lo + hi + 1) >> 1;
    if (descs[mid].blk0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const FlipDesc d = descs[lo];
  if (d.R == 1 && d.S == 1 && d.Ra == 1 && d.Sb == 1) {
    // 1x1 filters (every transformer linear): a plain [K][C] -> [C][K] transpose through a
    // 64x64 LDS tile, both global sides coalesced 4-byte pairs (the element loop below reads W
    // with a stride of ldw per lane: 595 us per BERT-base step, profiles/r3/bert_base_train_b128_r3.md)
    __shared__ bf16_t tl[64][66];
    const int tk = (d.K + 63) >> 6, tc = (d.C + 63) >> 6;
    const bf16_t* W = static_cast<const bf16_t*>(d.W);
    bf16_t* Wt = static_cast<bf16_t*>(d.Wt);
    const int tid = threadIdx.x, pr = tid >> 5, pc = (tid & 31) * 2;   // 8 rows x 32 pairs per pass
    for (int t = b - d.blk0; t < tk * tc; t += d.nblk) {
      const int k0 = (t / tc) * 64, c0 = (t % tc) * 64;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = pr + 8 * i, k = k0 + r, c = c0 + pc;
        bf16_t v0 = bf16_t(0), v1 = bf16_t(0);
        if (k < d.K) {
          const bf16_t* src = W + (size_t)k * d.ldw + c;
          if (c + 1 < d.C) {
            v0 = src[0];
            v1 = src[1];
          } else if (c < d.C) {
            v0 = src[0];
          }
        }
        tl[r][pc] = v0;
        tl[r][pc + 1] = v1;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = pr + 8 * i, c = c0 + r, k = k0 + pc;
        if (c < d.C) {
          bf16_t* dst = Wt + (size_t)c * d.ldt + k;
          if (k + 1 < d.K) {
            dst[0] = tl[pc][r];
            dst[1] = tl[pc + 1][r];
          } else if (k < d.K) {
            dst[0] = tl[pc][r];
          }
        }
      }
      __syncthreads();
    }
    return;
  }
  const int total = d.C * d.Ra * d.Sb * d.K;
  const int step = d.nblk * blockDim.x;
  for (int idx = (b - d.blk0) * blockDim.x + threadIdx.x; idx < total; idx += step) {
    int t = idx;
    const int k = t % d.K; t /= d.K;
    const int u = t % d.Sb; t /= d.Sb;
    const int v = t % d.Ra; t /= d.Ra;
    const int c = t;
    const int r = d.r0 + d.sh * (d.Ra - 1 - v), s = d.s0 + d.sw * (d.Sb - 1 - u);
    static_cast<bf16_t*>(d.Wt)[(size_t)c * d.ldt + (v * d.Sb + u) * d.K + k] =
        static_cast<const bf16_t*>(d.W)[(size_t)k * d.ldw + (r * d.S + s) * d.C + c];
  }
}

size_t igemm_smem_bytes(int BN, int nbuf = 2, bool lean = false) {
  const size_t main_bytes = (size_t)nbuf * (IG_BM + BN) * IG_BK * sizeof(bf16_t);
  const size_t epi_bytes = lean ? ((size_t)IG_BM * (BN + 4) * sizeof(bf16_t) + 15) / 16 * 16 +
                                      (size_t)2 * BN * 2 * sizeof(float)
                                : (size_t)IG_BM * (BN + 4) * sizeof(float) + (size_t)2 * BN * 2 * sizeof(float);
  return main_bytes > epi_bytes ? main_bytes : epi_bytes;
}

template <int VEC, bool IS1x1, bool LDIL, int BN, bool DMA, int EPI>
static hipError_t launch_ig1(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* Yf, const float* bias,
                             const bf16_t* resid, float* stats, const ConvGeom& g, int act, const BwdStats& bs,
                             hipStream_t st) {
  const int tiles = ((g.M + IG_BM - 1) / IG_BM) * ((g.K + BN - 1) / BN);
  const size_t smem = igemm_smem_bytes(BN, g.ldb > IG_BK ? 2 : 1, EPI == 1);
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&igemm_kernel<VEC, IS1x1, LDIL, BN, DMA, EPI>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)igemm_smem_bytes(BN, 2, EPI == 1));
    attr_set = true;
  }
  hipLaunchKernelGGL((igemm_kernel<VEC, IS1x1, LDIL, BN, DMA, EPI>), dim3(tiles), dim3(IG_NT), smem, st, X, W,
                     Y, Yf, bias, resid, stats, g, act, bs);
  return hipGetLastError();
}

template <int VEC, bool IS1x1, bool LDIL, int BN, bool DMA>
static hipError_t launch_ig(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* Yf, const float* bias,
                            const bf16_t* resid, float* stats, const ConvGeom& g, int act, const BwdStats& bs,
                            hipStream_t st) {
  static const bool lean_ok = true;
  const bool lean = lean_ok && Y && !Yf && !bias && !resid && act == 0 && !g.omap && !bs.sums;
  if (lean) return launch_ig1<VEC, IS1x1, LDIL, BN, DMA, 1>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  const bool bwd = lean_ok && Y && !Yf && !bias && act == 0 && !stats;
  if (bwd) return launch_ig1<VEC, IS1x1, LDIL, BN, DMA, 2>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  return launch_ig1<VEC, IS1x1, LDIL, BN, DMA, 0>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
}

template <int VEC, bool IS1x1, bool LDIL, bool DMA>
static hipError_t launch_ig_bn(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* Yf, const float* bias,
                               const bf16_t* resid, float* stats, const ConvGeom& g, int act, const BwdStats& bs,
                               hipStream_t st) {
  static const int force_bn = 0;
  if (force_bn == 64) return launch_ig<VEC, IS1x1, LDIL, 64, DMA>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  if (force_bn == 128) return launch_ig<VEC, IS1x1, LDIL, 128, DMA>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  // BN=64 tiles (lower VGPR/LDS footprint, more workgroups in flight) win while
  // there are plenty of them; few large tiles win when the grid is small
  // (tools/gemm_bench.py sweep on ResNet-50 shapes)
  if (g.K <= 64) return launch_ig<VEC, IS1x1, LDIL, 64, DMA>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  const long tiles64 = (long)((g.M + IG_BM - 1) / IG_BM) * ((g.K + 63) / 64);
  if (tiles64 >= 1536) return launch_ig<VEC, IS1x1, LDIL, 64, DMA>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  return launch_ig<VEC, IS1x1, LDIL, 128, DMA>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
}

}  // namespace zoo

using namespace zoo;

extern "C" int zoo_igemm2_eligible(const ConvGeom* g, int epi);
extern "C" hipError_t zoo_igemm2(const void* X, const void* W, void* Y, float* Yf, const float* bias,
                                 const void* resid, float* stats, const ConvGeom* g, int act, const BwdStats* bsp,
                                 hipStream_t st);

extern "C" int zoo_pw_eligible(const ConvGeom* g, int route, const BwdStats* bs);
extern "C" int zoo_pw_stem_eligible(const ConvGeom* g, int route);
extern "C" hipError_t zoo_pw_stem(const void* X, const void* W, void* Y, float* stats, const ConvGeom* g,
                                  hipStream_t st);
extern "C" hipError_t zoo_pw(const void* X, const void* W, void* Y, const void* resid, float* stats,
                             const ConvGeom* g, int epi, const BwdStats* bsp, hipStream_t st);

extern "C" int zoo_c3_grid(const ConvGeom* g, int epi, const BwdStats* bs);
extern "C" hipError_t zoo_c3(const void* X, const void* W, void* Y, const void* resid, float* stats,
                             const ConvGeom* g, int epi, const BwdStats* bsp, hipStream_t st);

extern "C" hipError_t zoo_igemm(const void* X, const void* W, void* Y, float* Yf, const float* bias,
                                const void* resid, float* stats, const ConvGeom* g, int act, const BwdStats* bsp,
                                hipStream_t st) {
  if (bsp && (bsp->pro_y || bsp->resid_half || bsp->pro_fwd)) {
    // the BN-backward prologue and the half-resolution residual exist only in pw.hip (the caller
    // materialises dy / the full-size residual otherwise)
    const int epi = igemm_epi(Y, Yf, bias, resid, act, g->omap, bsp->sums, stats);
    if (zoo_pw_eligible(g, igemm_route_epi(epi, bsp->zgelu), bsp)) return zoo_pw(X, W, Y, resid, stats, g, epi, bsp, st);
    return hipErrorInvalidValue;
  }
  {
    // stride-1 3x3 64 -> 64 channel convs (ResNet stage 1): the persistent streaming kernel (c3.hip)
    const int epi = igemm_epi(Y, Yf, bias, resid, act, g->omap, bsp && bsp->sums, stats);
    if (zoo_c3_grid(g, epi, bsp) > 0) return zoo_c3(X, W, Y, resid, stats, g, epi, bsp, st);
  }
  {
    // memory-bound 1x1 shapes: the persistent streaming kernel (pw.hip)
    const int epi = igemm_epi(Y, Yf, bias, resid, act, g->omap, bsp && bsp->sums, stats);
    const int route = igemm_route_epi(epi, bsp && bsp->zgelu);
    if (zoo_pw_eligible(g, route, bsp)) return zoo_pw(X, W, Y, resid, stats, g, epi, bsp, st);
    // the space-to-depth ResNet stem (4x4, 16 -> 64) on the same persistent kernel with a gathered operand
    static const bool stem_on = true;
    if (stem_on && !(bsp && bsp->sums) && zoo_pw_stem_eligible(g, route)) return zoo_pw_stem(X, W, Y, stats, g, st);
  }
  // whole-64-channel K-tiles: the large-tile second-generation kernel (igemm2.hip)
  if (zoo_igemm2_eligible(g, igemm_route_epi(igemm_epi(Y, Yf, bias, resid, act, g->omap, bsp && bsp->sums, stats),
                                             bsp && bsp->zgelu)))
    return zoo_igemm2(X, W, Y, Yf, bias, resid, stats, g, act, bsp, st);
  BwdStats bs = bsp ? *bsp : BwdStats{nullptr, nullptr, nullptr, nullptr, nullptr};
  const bf16_t* x = (const bf16_t*)X;
  const bf16_t* w = (const bf16_t*)W;
  bf16_t* y = (bf16_t*)Y;
  const bf16_t* rs = (const bf16_t*)resid;
  const bool is1x1 = g->R == 1 && g->S == 1 && g->sh == 1 && g->sw == 1 && g->ph == 0 && g->pw == 0 &&
                     g->lh == 1 && g->lw == 1 && g->H == g->P && g->W == g->Q;
  const bool ldil = g->lh > 1 || g->lw > 1;
  // LDS-DMA staging (global_load_lds) for the 16-byte-vector paths; ZOO_IGEMM_DMA=0 selects
  // the register-staged variant
  static const bool dma = true;
  if (g->C == 4) return launch_ig_bn<4, false, false, false>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
  if (dma) {
    if (is1x1) return launch_ig_bn<8, true, false, true>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
    if (ldil) return launch_ig_bn<8, false, true, true>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
    return launch_ig_bn<8, false, false, true>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
  }
  if (is1x1) return launch_ig_bn<8, true, false, false>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
  if (ldil) return launch_ig_bn<8, false, true, false>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
  return launch_ig_bn<8, false, false, false>(x, w, y, Yf, bias, rs, stats, *g, act, bs, st);
}

extern "C" hipError_t zoo_flip_weights(const void* W, void* Wt, int K, int R, int S, int C, int ldw, int r0,
                                       int s0, int Ra, int Sb, int sh, int sw, int ldt, hipStream_t st) {
  const int total = C * Ra * Sb * K;
  const int blocks = (total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048;
  hipLaunchKernelGGL(flip_weights_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, (const bf16_t*)W,
                     (bf16_t*)Wt, K, R, S, C, ldw, r0, s0, Ra, Sb, sh, sw, ldt);
  return hipGetLastError();
}

// descs: device array of n FlipDesc sorted by blk0; nblocks = last.blk0 + last.nblk
extern "C" hipError_t zoo_flip_weights_batched(const void* descs, int n, int nblocks, hipStream_t st) {
  if (n <= 0 || nblocks <= 0) return hipSuccess;
  hipLaunchKernelGGL(flip_weights_batched_kernel, dim3(nblocks), dim3(256), 0, st, (const FlipDesc*)descs, n);
  return hipGetLastError();
}
