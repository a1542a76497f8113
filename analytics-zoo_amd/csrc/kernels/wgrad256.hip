// Linear / 1x1-conv weight gradient on CDNA4 matrix cores (gfx950), large-tile form:
//
//   dW[n][k] (fp32, row stride ldw) += sum_m dY[m][n] * X[m][k]      dY [M, N], X [M, K] bf16
//
// Both operands are m-major (the reduction runs down their rows), so neither is
// K-contiguous per lane as the MFMA operand maps want. The tiles are staged into LDS
// as-is with LDS-DMA (global_load_lds, 16 B per lane, no VGPRs) and read back with the
// hardware transposing read ds_read_b64_tr_b16 (cdna_hip_programming.md T10): two 4x16
// transposed reads give a lane the 8 consecutive-m values of its v_mfma_f32_16x16x32_bf16
// operand fragment.
//
// Structure (the schedule of gemm256.hip, i.e. cdna_hip_programming.md §5 "256² 8-phase"):
//   * 256 (n) x 256 (k) output tile, 64-row m-steps, 8 waves as 2 (n) x 4 (k); each wave
//     owns 128 x 64 outputs = 8 x 4 tiles of 16x16 (128 accumulator registers).
//   * each m-step is four 16 KiB half-tiles (A = dY halves by the waves' upper / lower
//     64-row quadrant, B = X halves by their left / right 32-column quadrant), staged one
//     per phase 5-6 phases ahead; counted `s_waitcnt vmcnt(8)` + one raw s_barrier per
//     phase, never a drain inside the loop.
//   * LDS image of a half-tile: blocks of [8 m-rows][16 columns] (256 B, rows 32 B apart);
//     the 8-row blocks of odd m-block index store their rows 0-3 <-> 4-7 swapped, so the
//     two 16-lane groups of a half-wave (m-blocks 2g, 2g+1) read opposite 128-byte halves
//     of the bank row: conflict-free. The swizzle is applied through the per-lane DMA
//     SOURCE row (the DMA image is lane-linear).
//   * the reduction (M up to 10^6 for ResNet stage 1, 16384 for BERT) is split over
//     workgroups so ~one wave of 256 workgroups fills the chip; each split stores its
//     fp32 tile in MFMA-fragment order (1 KiB fully coalesced per wave store) and an
//     ordered fold kernel sums the splits into dW (deterministic, no atomics). A single
//     split accumulates straight into dW. When the live part of the split tiles is small
//     (<= ZOO_WGRAD256_ATOMIC_MB of added bytes, default 32 MB: the 64/128-channel ResNet
//     shapes) and the deterministic mode is off, the splits add their tiles into dW with fp32
//     atomics instead: no partial buffer, no fold launch (the r4 folds moved up to 64 MB per
//     call through HBM beside the data-gradient chain).
//
// Reference parity: the weight-gradient half of BigDL Linear / SpatialConvolution
// accGradParameters, as wgrad.hip.
#include "common.h"
#include "geom.h"

namespace zoo {

typedef __attribute__((address_space(3))) void w2_lds_void;
typedef __attribute__((address_space(1))) const void w2_gl_void;
typedef __attribute__((address_space(3))) i16x4 w2_lds_i16x4;

constexpr int W2_T = 256, W2_BM = 64, W2_NT = 512, W2_HALF = 16384;

ZOO_DEV void w2_vm8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
ZOO_DEV void w2_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
ZOO_DEV void w2_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

struct W2Geom {
  int M, N, K;        // reduction rows, dY columns (dW rows), X columns (dW cols)
  int ldy, ldx, ldw;  // leading dims (elements); ldy, ldx % 8 == 0
  int m_per_split, splits, tiles_n, tiles_k;
  int atomic;         // splits > 1 without partials: every split adds its tile into dW with fp32 atomics
};

// implicit-GEMM (im2col) form of the X operand for convolutions: X[m][k] with m = output
// pixel (n, p, q) and k = (r * S + s) * C + c reads x[n][p*sh - ph + r*dh][q*sw - pw + s*dw][c]
// of the NHWC input (zero outside). C % 8 == 0, so a lane's 16-byte chunk never straddles taps.
struct W2Conv {
  int H, W, C, P, Q, S;
  int sh, sw, ph, pw, dh, dw;
};

// one fragment = two transposed 4-row reads of an 8-row block (rows 0-3 -> elements 0-3)
ZOO_DEV bf16x8 w2_frag(const char* blk, int lo_off, int hi_off) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w2_lds_i16x4*)(blk + lo_off));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w2_lds_i16x4*)(blk + hi_off));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  i16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

template <bool PP, bool IMPL>
__global__ __launch_bounds__(W2_NT, 1) void wgrad256_kernel(const bf16_t* __restrict__ dY,
                                                            const bf16_t* __restrict__ X, float* __restrict__ dW,
                                                            float* __restrict__ part, W2Geom g,
                                                            const bf16_t* __restrict__ zpage, W2Conv cv) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;

  const int tiles = g.tiles_n * g.tiles_k;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles, tile = bid - split * tiles;
  const int n0 = (tile / g.tiles_k) * W2_T, k0 = (tile % g.tiles_k) * W2_T;
  const int ms = split * g.m_per_split;
  const int me = min(g.M, ms + g.m_per_split);
  const int nk = (me - ms + W2_BM - 1) / W2_BM;

  // ---- per-lane DMA source (lane-linear 1 KiB per wave instruction) ----
  const int slot = (lane >> 1) & 7, c8 = (lane & 1) * 8;
  // A (dY) half h, instruction j: LDS block (q = j, mb = w): [nb16 = lane>>4][slot][16]
  const int a_mb = w;
  const int a_row = a_mb * 8 + (slot ^ ((a_mb & 1) << 2));
  int a_col[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) a_col[h][j] = n0 + j * 128 + h * 64 + (lane >> 4) * 16 + c8;
  // B (X) half h, instruction j: idx = j*8 + w -> wn' = idx>>2, m-block pair mbp = idx&3;
  // [mb = 2 mbp + (lane>>5)][nb16 = (lane>>4)&1][slot][16]
  int b_row[2], b_col[2][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = j * 8 + w, mb = 2 * (idx & 3) + (lane >> 5);
    b_row[j] = mb * 8 + (slot ^ ((mb & 1) << 2));
#pragma unroll
    for (int h = 0; h < 2; ++h) b_col[h][j] = k0 + (idx >> 2) * 64 + h * 32 + ((lane >> 4) & 1) * 16 + c8;
  }

  // IMPL: per (half, instruction) the lane's k chunk is one fixed tap (r, s) and channel c;
  // its pixel (n, p, q) advances by 64 rows per staged m-step without integer division
  int xoff_h[2][2], xoff_w[2][2], xc[2][2], pn[2][2], pp[2][2], pq[2][2];
  int adv_n = 0, adv_p = 0, adv_q = 0;
  if constexpr (IMPL) {
    const int PQ = cv.P * cv.Q;
    adv_n = W2_BM / PQ;
    adv_p = (W2_BM % PQ) / cv.Q;
    adv_q = (W2_BM % PQ) % cv.Q;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int k = b_col[h][j];
        const int t = k / cv.C;
        const int r = t / cv.S;
        xc[h][j] = k - t * cv.C;
        // a k beyond K gets an offset that fails the row bounds test
        xoff_h[h][j] = k < g.K ? r * cv.dh - cv.ph : -(1 << 28);
        xoff_w[h][j] = (t - r * cv.S) * cv.dw - cv.pw;
        const int m = ms + b_row[j];
        const int mm = m < g.M ? m : 0;
        pn[h][j] = mm / PQ;
        const int rem = mm - pn[h][j] * PQ;
        pp[h][j] = rem / cv.Q;
        pq[h][j] = rem - pp[h][j] * cv.Q;
      }
  }

  auto half_base = [&](int buf, int op, int h) -> char* {
    return smem + (((buf * 2 + op) * 2 + h) * W2_HALF);
  };

  auto stage = [&](int kt, int op, int h) {
    char* hb = half_base(kt & 1, op, h);
    const int mrow0 = ms + kt * W2_BM;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16_t* src;
      if (op == 0) {
        const int m = mrow0 + a_row, n = a_col[h][j];
        src = (m < me && n < g.N) ? dY + (size_t)m * g.ldy + n : zpage;
      } else if constexpr (IMPL) {
        const int m = mrow0 + b_row[j];
        const int hi = pp[h][j] * cv.sh + xoff_h[h][j], wi = pq[h][j] * cv.sw + xoff_w[h][j];
        const bool ok = m < me && (unsigned)hi < (unsigned)cv.H && (unsigned)wi < (unsigned)cv.W;
        src = ok ? X + (((size_t)pn[h][j] * cv.H + hi) * cv.W + wi) * cv.C + xc[h][j] : zpage;
        pq[h][j] += adv_q; pp[h][j] += adv_p; pn[h][j] += adv_n;
        if (pq[h][j] >= cv.Q) { pq[h][j] -= cv.Q; ++pp[h][j]; }
        if (pp[h][j] >= cv.P) { pp[h][j] -= cv.P; ++pn[h][j]; }
      } else {
        const int m = mrow0 + b_row[j], k = b_col[h][j];
        src = (m < me && k < g.K) ? X + (size_t)m * g.ldx + k : zpage;
      }
      __builtin_amdgcn_global_load_lds((w2_gl_void*)src, (w2_lds_void*)(hb + (j * 8 + w) * 1024), 16, 0, 0);
    }
  };

  // ---- transposed fragment reads ----
  // lane: group gq = lane>>4 takes m rows 8gq..8gq+7 of a 32-row k-step (= m-block 4kb+gq);
  // inside the group lane 4tq+tp addresses row tq (and 4+tq) columns 4tp..4tp+3
  const int gq = lane >> 4, tq = (lane >> 2) & 3, tp = lane & 3;
  const int sw = (gq & 1) << 2;  // odd m-blocks store rows 0-3 <-> 4-7 swapped
  const int lo_off = ((tq ^ sw) * 32) + tp * 8, hi_off = (((4 + tq) ^ sw) * 32) + tp * 8;
  // A frag (half h, wave row wm, 16-col block i, k-step kb): block wm*8 + 4kb+gq, column block i
  auto read_a = [&](int buf, int h, int i, int kb) -> bf16x8 {
    const char* blk = half_base(buf, 0, h) + (wm * 8 + 4 * kb + gq) * 1024 + i * 256;
    return w2_frag(blk, lo_off, hi_off);
  };
  // B frag (half h, wave col wn, 16-col block j, k-step kb)
  auto read_b = [&](int buf, int h, int j, int kb) -> bf16x8 {
    const char* blk = half_base(buf, 1, h) + wn * 4096 + (4 * kb + gq) * 512 + j * 256;
    return w2_frag(blk, lo_off, hi_off);
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];

  if (nk > 0) {
    stage(0, 0, 0);
    stage(0, 1, 0);
    stage(0, 1, 1);
    stage(0, 0, 1);
    if (nk > 1) {
      stage(1, 0, 0);
      stage(1, 1, 0);
      w2_vm8();
    } else {
      w2_vm0();
    }
  }
  __builtin_amdgcn_s_barrier();
  // PP (ping-pong): the two wave rows run one barrier apart, so on every SIMD (one wave of
  // each row) one wave issues its LDS reads / DMA while the other runs its MFMAs; every
  // phase then has a second barrier after its MFMAs (cdna_hip_programming.md §5 256²
  // template). Hazards shift by half a phase: reads still come >= 1 barrier after every
  // wave's retiring wait, restaging stays >= 1.5 phases after the last read.
  if (PP && wm == 1) __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fa[i][kb] = read_a(buf, 0, i, kb);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fb0[j][kb] = read_b(buf, 0, j, kb);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fb1[j][kb] = read_b(buf, 1, j, kb);
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fa[i][kb] = read_a(buf, 1, i, kb);
      }
      // stage one half-tile: P0 -> B1(kt+1), P1 -> A1(kt+1), P2 -> A0(kt+2), P3 -> B0(kt+2)
      const int skt = p < 2 ? kt + 1 : kt + 2;
      const bool valid = skt < nk;
      if (valid) stage(skt, p == 1 || p == 2 ? 0 : 1, p == 0 || p == 1 ? 1 : 0);
      if (valid) w2_vm8(); else w2_vm0();
      __builtin_amdgcn_s_barrier();
      w2_lgkm0();
      const int qa = p >= 2 ? 1 : 0;
      const int qb = (p == 1 || p == 2) ? 1 : 0;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qa][qb][i][j] = mfma16(fa[i][kb], qb ? fb1[j][kb] : fb0[j][kb], acc[qa][qb][i][j]);
      __builtin_amdgcn_s_setprio(0);
      if (PP) __builtin_amdgcn_s_barrier();
    }
  }
  if (PP && wm == 0) __builtin_amdgcn_s_barrier();

  // ---- epilogue ----
  // fragment (qa, qb, i, j) reg r <-> dW row n0 + wm*128 + qa*64 + i*16 + 4*(lane>>4) + r,
  //                                   col k0 + wn*64 + qb*32 + j*16 + (lane&15)
  if (part) {
    // fragment order: [split][tile][wave][qa][qb][i][j][lane] float4
    // fragments wholly outside dW (tile overhang: N or K not a multiple of 256) are neither
    // stored nor read by the fold -- half the partial traffic on 128-channel shapes
    f32x4* dst = reinterpret_cast<f32x4*>(part) + ((size_t)(split * tiles + tile) * 8 + w) * 32 * 64 + lane;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const bool live = k0 + wn * 64 + qb * 32 + j * 16 < g.K && n0 + wm * 128 + qa * 64 + i * 16 < g.N;
            if (live) dst[(((qa * 2 + qb) * 4 + i) * 2 + j) * 64] = acc[qa][qb][i][j];
          }
  } else {
    const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int col = k0 + wn * 64 + qb * 32 + j * 16 + fr;
            const int row = n0 + wm * 128 + qa * 64 + i * 16 + fq * 4;
            if (col < g.K) {
              if (g.atomic) {
                // no-return global_atomic_add_f32 (-munsafe-fp-atomics), executed at the memory
                // side: one 16-lane x 4-row wave instruction per accumulator register
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  if (row + r < g.N) atomicAdd(dW + (size_t)(row + r) * g.ldw + col, acc[qa][qb][i][j][r]);
              } else {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                  if (row + r < g.N) dW[(size_t)(row + r) * g.ldw + col] += acc[qa][qb][i][j][r];
              }
            }
          }
  }
}

// Ordered fold of the split partials into dW: thread = one fragment lane (float4) of one
// tile; sums splits 0..S-1 in order, then adds its 4 rows x 1 column into dW.
__global__ __launch_bounds__(256) void wgrad256_fold_kernel(const float* __restrict__ part, float* __restrict__ dW,
                                                           W2Geom g) {
  const int tiles = g.tiles_n * g.tiles_k;
  const size_t per_tile = (size_t)8 * 32 * 64;  // float4 slots per tile
  const size_t total = per_tile * tiles;
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int tile = (int)(idx / per_tile);
  const int rem = (int)(idx - (size_t)tile * per_tile);
  const int w = rem >> 11, f = (rem >> 6) & 31, lane = rem & 63;
  const int j = f & 1, i = (f >> 1) & 3, qb = (f >> 3) & 1, qa = f >> 4;
  const int wm = w >> 2, wn = w & 3;
  const int n0 = (tile / g.tiles_k) * W2_T, k0 = (tile % g.tiles_k) * W2_T;
  const int col = k0 + wn * 64 + qb * 32 + j * 16 + (lane & 15);
  const int row = n0 + wm * 128 + qa * 64 + i * 16 + (lane >> 4) * 4;
  if (col >= g.K || row >= g.N) return;  // slot never written (see the partial store)
  const f32x4* p = reinterpret_cast<const f32x4*>(part) + idx;
  // 4 independent partial sums keep 4 loads in flight (the splits are summed in a fixed
  // order per lane, so the result stays deterministic)
  f32x4 s = p[0], s1 = f32x4{0.f, 0.f, 0.f, 0.f}, s2 = s1, s3 = s1;
  int sp = 1;
  for (; sp + 3 < g.splits; sp += 4) {
    s += p[(size_t)sp * total];
    s1 += p[(size_t)(sp + 1) * total];
    s2 += p[(size_t)(sp + 2) * total];
    s3 += p[(size_t)(sp + 3) * total];
  }
  for (; sp < g.splits; ++sp) s += p[(size_t)sp * total];
  s += (s1 + s2) + s3;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (row + r < g.N) dW[(size_t)(row + r) * g.ldw + col] += s[r];
}

}  // namespace zoo

using namespace zoo;

static const bf16_t* w2_zero_page() {
  static bf16_t* z = nullptr;
  if (!z) {
    hipMalloc(&z, 4096);
    hipMemset(z, 0, 4096);
  }
  return z;
}

// split plan: ~one workgroup per CU (256), >= 4 m-steps per split. Returns the number of
// splits and fills m_per_split; the caller provides part (splits * tiles * 256 KiB) when > 1.
// target override (> 0) for the calls made while it is set: conv weight gradients use fewer,
// longer splits (ZOO_WGRAD256_CONV_WG, default 128). With the weight-gradient side stream they
// run beside the memory-bound BatchNorm passes, where half the split-K partial traffic beat the
// extra parallelism: ResNet-50 b256 12,149-12,179 -> 12,278-12,314 img/s; BERT's linear weight
// gradients, beside compute-bound GEMMs, stay at 256 (15.73 vs 16.06 ms at 128).
static int g_w256_target = 0;
extern "C" void zoo_wgrad256_target(int t) { g_w256_target = t; }

extern "C" int zoo_wgrad256_plan(int M, int N, int K, int* m_per_split) {
  const int tiles = ((N + W2_T - 1) / W2_T) * ((K + W2_T - 1) / W2_T);
  static const int target_default = 256;
  const int target = g_w256_target > 0 ? g_w256_target : target_default;
  int splits = (target + tiles / 2) / tiles;
  const int max_splits = (M + 4 * W2_BM - 1) / (4 * W2_BM);
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  int mps = (M + splits - 1) / splits;
  mps = (mps + W2_BM - 1) / W2_BM * W2_BM;
  splits = (M + mps - 1) / mps;
  *m_per_split = mps;
  return splits;
}

// split-K by fp32 atomics (no partials) for this plan? Never in the deterministic mode (set
// by the host through zoo_wgrad256_set_atomic(0)); the added bytes are splits x the live
// (N x K) part of the output.
static int g_w256_atomic = 1;
extern "C" void zoo_wgrad256_set_atomic(int on) { g_w256_atomic = on; }

static bool w2_atomic(int splits, int N, int K) {
  static const double mb_max = 32.0;
  return g_w256_atomic && splits > 1 && (double)splits * N * K * 4 / 1e6 <= mb_max;
}

extern "C" size_t zoo_wgrad256_part_floats(int M, int N, int K) {
  int mps = 0;
  const int splits = zoo_wgrad256_plan(M, N, K, &mps);
  const size_t tiles = (size_t)((N + W2_T - 1) / W2_T) * ((K + W2_T - 1) / W2_T);
  if (w2_atomic(splits, N, K)) return 0;
  return splits > 1 ? (size_t)splits * tiles * W2_T * W2_T : 0;
}

// dW[N][K] (row stride ldw) += dY[M][N]^T X[M][K]; part: zoo_wgrad256_part_floats() fp32 scratch
extern "C" hipError_t zoo_wgrad256(const void* dY, const void* X, float* dW, float* part, int M, int N, int K,
                                   int ldy, int ldx, int ldw, hipStream_t st) {
  W2Geom g;
  g.M = M; g.N = N; g.K = K; g.ldy = ldy; g.ldx = ldx; g.ldw = ldw;
  g.tiles_n = (N + W2_T - 1) / W2_T;
  g.tiles_k = (K + W2_T - 1) / W2_T;
  g.splits = zoo_wgrad256_plan(M, N, K, &g.m_per_split);
  g.atomic = w2_atomic(g.splits, N, K) ? 1 : 0;
  if (g.splits > 1 && !g.atomic && !part) return hipErrorInvalidValue;
  if (g.atomic || g.splits <= 1) part = nullptr;
  const int tiles = g.tiles_n * g.tiles_k;
  const size_t smem = 4 * 2 * W2_HALF;  // 2 buffers x (A, B) x 2 halves = 128 KiB
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad256_kernel<false, false>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad256_kernel<false, true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  const W2Conv cv{};
  hipLaunchKernelGGL((wgrad256_kernel<false, false>), dim3(tiles * g.splits), dim3(W2_NT), smem, st, (const bf16_t*)dY,
                     (const bf16_t*)X, dW, part, g, w2_zero_page(), cv);
  if (g.splits > 1 && !g.atomic) {
    const size_t total = (size_t)tiles * 8 * 32 * 64;
    hipLaunchKernelGGL(wgrad256_fold_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, part, dW, g);
  }
  return hipGetLastError();
}

// convolution weight gradient on the same kernel, X staged as the implicit im2col matrix:
// dW[Cout][(r*S + s)*C + c] (row stride ldw) += sum over output pixels; dY = [Nb*P*Q][Cout]
// contiguous, x = NHWC [Nb][H][W][C] with C % 8 == 0. part: zoo_wgrad256_part_floats(M, Cout,
// R*S*C) fp32 scratch.
extern "C" hipError_t zoo_wgrad256_conv(const void* dY, const void* X, float* dW, float* part, int Nb, int H, int W,
                                        int C, int Cout, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                        int dh, int dw, int ldw, hipStream_t st) {
  if (C % 8 || Cout % 8) return hipErrorInvalidValue;
  W2Geom g;
  g.M = Nb * P * Q; g.N = Cout; g.K = R * S * C;
  g.ldy = Cout; g.ldx = 0; g.ldw = ldw;
  g.tiles_n = (g.N + W2_T - 1) / W2_T;
  g.tiles_k = (g.K + W2_T - 1) / W2_T;
  g.splits = zoo_wgrad256_plan(g.M, g.N, g.K, &g.m_per_split);
  g.atomic = w2_atomic(g.splits, g.N, g.K) ? 1 : 0;
  if (g.splits > 1 && !g.atomic && !part) return hipErrorInvalidValue;
  if (g.atomic || g.splits <= 1) part = nullptr;
  const W2Conv cv{H, W, C, P, Q, S, sh, sw, ph, pw, dh, dw};
  const int tiles = g.tiles_n * g.tiles_k;
  const size_t smem = 4 * 2 * W2_HALF;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&wgrad256_kernel<false, true>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    attr = true;
  }
  hipLaunchKernelGGL((wgrad256_kernel<false, true>), dim3(tiles * g.splits), dim3(W2_NT), smem, st, (const bf16_t*)dY,
                     (const bf16_t*)X, dW, part, g, w2_zero_page(), cv);
  if (g.splits > 1 && !g.atomic) {
    const size_t total = (size_t)tiles * 8 * 32 * 64;
    hipLaunchKernelGGL(wgrad256_fold_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, part, dW, g);
  }
  return hipGetLastError();
}
