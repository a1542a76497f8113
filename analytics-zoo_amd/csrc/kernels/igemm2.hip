// Implicit-GEMM convolution / GEMM, second generation: large tiles, full-line LDS-DMA
// staging, counted-vmcnt software pipeline (gfx950 / MI355X).
//
//   Y[m][n] = epilogue( sum_k A[m][k] * W[n][k] )      m = output pixel (n,p,q), n = Cout,
//                                                      k = (r, s, c) filter tap x channel
//
// Scope: every conv / linear whose reduction runs over whole 64-channel slices (C % 64 == 0),
// i.e. all ResNet-50 convs but the stem, transformer linears, and the parity-decomposed
// dgrads built on them (zoo/ops/_kern.py conv_dgrad). Each 64-deep K-tile is then ONE filter
// tap (r, s) and a contiguous 64-channel run, so the tap decode is wave-uniform scalar work
// and every staged row is one full 128-byte line of the NHWC activation.
//
// Why a second kernel (profiles/PERF.md "Why the conv GEMMs stop at ~500 TF/s"): igemm.hip's
// 128x64 tiles with 64x32 wave tiles need 0.75 LDS fragment reads per MFMA plus 24 KiB of
// staging per 64 MFMAs, which makes the LDS array -- not the matrix cores -- the bound. Here:
//   * wave tile 64x64 (or 128x64): 0.5 fragment reads per v_mfma_f32_16x16x32_bf16;
//   * block tiles 128x128 / 256x128 / 256x64 / 256x256 chosen per shape on the host;
//   * A and B staged with global_load_lds (16 B per lane, no VGPRs, no ds_write): one wave
//     instruction moves 8 rows x 128 B -- whole cache lines, so the TA sees 8 lines per
//     instruction instead of 16 half lines;
//   * LDS image [row][128 B] with the 16-byte chunk XOR-swizzled by (row & 7). The DMA image
//     is lane-linear, so the swizzle is applied through the per-lane SOURCE chunk (each row's
//     8 lanes still fetch its whole line, permuted); fragment reads apply the same XOR. With the
//     ds_read_b128 lane groups of MI355X_MICROARCH.md §LDS every 16-lane group of a 16x16x32
//     fragment read lands on 16 distinct 16-byte bank slots: conflict-free;
//   * STAGES-deep LDS ring: tile kt+STAGES-1 is issued at the top of iteration kt; the end of
//     the iteration waits with a counted `s_waitcnt vmcnt((STAGES-2) * DMA-per-tile)` and a raw
//     s_barrier, so with STAGES=3 one tile stays in flight across every barrier and the main
//     loop never drains the memory queue (cdna_hip_programming.md "Pipelining across barriers");
//   * all LDS is one extern __shared__ array and the loop issues no VGPR-destination global
//     load (the two .s traps of cdna_hip_programming.md §5 item 4).
// Epilogue: per wave, 16-row slices of the fp32 accumulators go through a wave-private LDS
// patch and leave as row-contiguous 16-byte stores, with the same fusions as igemm.hip:
// EPI 1 = plain conv + BN statistics (the forward of every conv->BN unit), EPI 2 = backward
// (residual-gradient add, producer ReLU mask, fused BN-backward sums, strided output remap),
// EPI 0 = general (bias, activation, residual, fp32 output, statistics, remap);
// EPI 3 = bf16 output + bias + none / ReLU / GELU (the transformer linears' forward).
//
// Reference parity: the MKL-DNN convolution / inner-product primitives behind BigDL
// SpatialConvolution and Linear (Zs/pipeline/api/keras/layers/Convolution2D.scala:86-110,
// Dense.scala).
#include <stdlib.h>

#include "common.h"
#include "geom.h"
#include "bnmask.h"

namespace zoo {

typedef __attribute__((address_space(3))) void i2_lds_void;
typedef __attribute__((address_space(1))) const void i2_gl_void;

// zero page read by the DMA for rows beyond M / N and for padding taps
__device__ __attribute__((aligned(64))) bf16_t i2_zero_page[32];

template <int N>
ZOO_DEV void i2_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int NWM, int NWN, int TM, int TN>
struct I2Cfg {
  static constexpr int NW = NWM * NWN, NT = NW * 64;
  static constexpr int WTM = TM * 16, WTN = TN * 16;  // wave tile
  static constexpr int BM = NWM * WTM, BN = NWN * WTN;  // block tile
  // DMA instructions per wave per K-tile. A tile whose rows do not split evenly over the waves
  // (BM = 224 with 8 waves: 28 pieces) gives every wave the same count and sends the pieces past
  // BM -- zero-page reads -- to a per-wave junk slot, so every wave's vmcnt count stays uniform
  static constexpr int A_PW = (BM + 8 * NW - 1) / (8 * NW), B_PW = BN / (8 * NW);
  static constexpr bool A_RAG = A_PW * 8 * NW != BM;
  static constexpr int DPT = A_PW + B_PW;
  static constexpr int STAGE_BYTES = (BM + BN) * 128;
  static constexpr int JUNK_BYTES = A_RAG ? NW * 1024 : 0;
  static constexpr int EPI_PITCH = WTN + 4;  // fp32 patch pitch (16-byte aligned rows)
  static constexpr int EPI_BYTES = NW * 16 * EPI_PITCH * 4 + NWM * BN * 2 * 4;
  static_assert(B_PW * 8 * NW == BN, "B tile rows must split into 8-row DMA groups");
};

// A-operand modes: I2_AM_IMPLICIT stages BM im2col rows per K-tile (any tap geometry);
// I2_AM_1X1 the same rows of a 1x1 conv / GEMM; I2_AM_BAND (stride-1 3x3, pad 1) stages the
// block's input rows ONCE per 64-channel slice -- a band of TP = BM / Q output rows of one
// image needs (TP + 2) x (Q + 2) halo pixels -- and reads all nine taps' A fragments from that
// LDS patch, so each activation line is fetched ~1.3x instead of 9x per conv (the small-channel
// ResNet stage-1/2 3x3 convs, which the per-tap gather left L2/LDS-DMA bound at ~300 TF/s).
// Slice s+1's patch streams into the second patch buffer during slice s's K-tiles.
enum I2AMode : int { I2_AM_IMPLICIT = 0, I2_AM_1X1 = 1, I2_AM_BAND = 2 };

template <int NWM, int NWN, int TM, int TN, int STAGES, int AM, int EPI>
__global__ __launch_bounds__(64 * NWM * NWN, AM == I2_AM_BAND ? 1 : 2) void igemm2_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wm, bf16_t* __restrict__ Y, float* __restrict__ Yf,
    const float* __restrict__ bias, const bf16_t* __restrict__ resid, float* __restrict__ stats, ConvGeom g, int act,
    BwdStats bs) {
  using Cfg = I2Cfg<NWM, NWN, TM, TN>;
  constexpr int NW = Cfg::NW, WTM = Cfg::WTM, WTN = Cfg::WTN, BM = Cfg::BM, BN = Cfg::BN;
  constexpr int A_PW = Cfg::A_PW, B_PW = Cfg::B_PW, DPT = Cfg::DPT, SB = Cfg::STAGE_BYTES;
  constexpr bool IS1x1 = AM == I2_AM_1X1;
  constexpr bool BAND = AM == I2_AM_BAND;
  static_assert(BAND || A_PW * 8 * NW >= BM, "A tile rows must be covered by the 8-row DMA groups");
  static_assert(BAND || BM % 8 == 0, "A tile rows must split into 8-row DMA groups");

  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / NWN, wn = w - (w / NWN) * NWN;

  const int ntn = (g.K + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / ntn, tn = bid - tm * ntn;
  const int PQ = g.P * g.Q;
  // band mode: m-tile tm = (image, band of TP output rows); rows of the next image are not ours
  const int TP = BAND ? BM / g.Q : 0;
  const int nbands = BAND ? (g.P + TP - 1) / TP : 1;
  const int b_img = BAND ? tm / nbands : 0;
  const int b_p0 = BAND ? (tm - b_img * nbands) * TP : 0;
  const int m0 = BAND ? b_img * PQ + b_p0 * g.Q : tm * BM, n0 = tn * BN;
  const int mlim = BAND ? min(g.M, b_img * PQ + PQ) : g.M;
  const int nk = g.Ktot >> 6;  // C % 64 == 0: one 64-deep K-tile per (tap, 64-channel slice)

  // ---- staging assignment: lane -> row lr of each 8-row group, global 16-byte chunk gc ----
  const int lr = lane >> 3;
  const int gc = (lane & 7) ^ lr;  // XOR swizzle through the source (LDS image lane-linear)

  // band geometry: patch row pr = pi * PW2 + pj holds input pixel (b_p0 - 1 + pi, pj - 1);
  // a slice buffer is PROWS (multiple of 8) rows x 128 B; then the B ring, then a 1 KiB junk
  // slot per wave for DMA pieces past the patch end (keeps every wave's vmcnt count uniform)
  const int PW2 = g.Q + 2;
  const int prow_n = BAND ? (TP + 2) * PW2 : 0;
  const int npiece = (prow_n + 7) >> 3;
  const int nslice = g.C >> 6;
  const int pbytes = npiece * 1024;
  const int bring = BAND ? (nslice > 1 ? 2 : 1) * pbytes : 0;  // B ring offset
  char* const junk = smem + bring + STAGES * BN * 128 + w * 1024;
  auto stage_piece = [&](int j, int cs, int buf) {
    const bf16_t* src = i2_zero_page;
    char* dst = junk;
    if (j < npiece) {
      const int pr = j * 8 + lr;
      const int pi = pr / PW2, pj = pr - pi * PW2;
      const int ih = b_p0 - 1 + pi, iw = pj - 1;
      if (pr < prow_n && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
        src = X + (((size_t)b_img * g.H + ih) * g.W + iw) * g.C + cs * 64 + gc * 8;
      dst = smem + buf * pbytes + j * 1024;
    }
    __builtin_amdgcn_global_load_lds((i2_gl_void*)src, (i2_lds_void*)dst, 16, 0, 0);
  };
  // per lane: patch row of its pixel's window origin for each of its TM row tiles
  int a_pb[BAND ? TM : 1];
  if constexpr (BAND) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int t = wm * WTM + i * 16 + (lane & 15);  // < BM = TP * Q
      const int pp = t / g.Q;
      a_pb[i] = pp * PW2 + (t - pp * g.Q);
    }
  }

  int a_base[A_PW], a_ih[A_PW], a_iw[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    if constexpr (BAND) break;
    const int prow = (i * NW + w) * 8;   // first tile row of this DMA piece (>= BM: junk piece)
    const int m = m0 + prow + lr;
    const bool ok = prow < BM && m < g.M;
    if constexpr (IS1x1) {
      a_base[i] = ok ? m * g.C + gc * 8 : -1;
      a_ih[i] = a_iw[i] = 0;
    } else {
      const int mm = ok ? m : 0;
      const int n = mm / PQ, pq = mm - n * PQ;
      const int p = pq / g.Q, q = pq - p * g.Q;
      a_base[i] = n * g.H * g.W * g.C + gc * 8;
      a_ih[i] = ok ? p * g.sh - g.ph : -(1 << 28);  // invalid rows never pass the bounds check
      a_iw[i] = q * g.sw - g.pw;
    }
  }
  const bf16_t* b_src[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int n = n0 + (i * NW + w) * 8 + lr;
    b_src[i] = n < g.K ? Wm + (size_t)n * g.ldb + gc * 8 : nullptr;
  }

  // tap decode of the NEXT tile to stage (wave-uniform)
  int st_r = 0, st_s = 0, st_c = 0, st_k = 0;
  // band mode: K-tiles run slice-major (all nine taps of 64-channel slice 0, then slice 1, ...)
  // so one patch slice serves nine consecutive tiles; weights are [K][tap][C]
  int sb_tap = 0, sb_cs = 0;
  auto stage_b = [&](int buf) {
    char* sb = smem + bring + buf * (BN * 128) + w * 1024;
    const int koff = sb_tap * g.C + sb_cs * 64;
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const bf16_t* src = b_src[i] ? b_src[i] + koff : i2_zero_page;
      __builtin_amdgcn_global_load_lds((i2_gl_void*)src, (i2_lds_void*)(sb + i * NW * 1024), 16, 0, 0);
    }
    if (++sb_tap == 9) { sb_tap = 0; ++sb_cs; }
  };
  auto stage = [&](int buf) {
    char* sa = smem + buf * SB + w * 1024;
    char* sb = smem + buf * SB + BM * 128 + w * 1024;
    char* const ajunk = smem + STAGES * SB + w * 1024;
#pragma unroll
    for (int i = 0; i < A_PW; ++i) {
      char* adst = (Cfg::A_RAG && (i * NW + w) * 8 >= BM) ? ajunk : sa + i * NW * 1024;
      const bf16_t* src;
      if constexpr (IS1x1) {
        src = a_base[i] >= 0 ? X + a_base[i] + st_k : i2_zero_page;
      } else {
        const int ih = a_ih[i] + st_r * g.dh, iw = a_iw[i] + st_s * g.dw;
        const bool ok = (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        src = ok ? X + a_base[i] + (ih * g.W + iw) * g.C + st_c : i2_zero_page;
      }
      __builtin_amdgcn_global_load_lds((i2_gl_void*)src, (i2_lds_void*)adst, 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_PW; ++i) {
      const bf16_t* src = b_src[i] ? b_src[i] + st_k : i2_zero_page;
      __builtin_amdgcn_global_load_lds((i2_gl_void*)src, (i2_lds_void*)(sb + i * NW * 1024), 16, 0, 0);
    }
    st_k += 64;
    if constexpr (!IS1x1) {
      st_c += 64;
      if (st_c == g.C) {
        st_c = 0;
        if (++st_s == g.S) { st_s = 0; ++st_r; }
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: lane -> tile row (lane & 15), chunk kk*4 + (lane >> 4), XOR (row & 7)
  const int rl = (lane & 15) * 128;
  const int co0 = (((lane >> 4)) ^ (lane & 7)) << 4;
  const int co1 = ((4 + (lane >> 4)) ^ (lane & 7)) << 4;
  auto compute = [&](int buf) {
    const char* ab = smem + buf * SB + (wm * WTM) * 128 + rl;
    const char* bb = smem + buf * SB + (BM + wn * WTN) * 128 + rl;
    // all fragment reads of the tile up front (the kk = 1 reads overlap the kk = 0 MFMAs)
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int co = kk ? co1 : co0;
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[kk][j] = *reinterpret_cast<const bf16x8*>(bb + j * 2048 + co);
#pragma unroll
      for (int i = 0; i < TM; ++i) af[kk][i] = *reinterpret_cast<const bf16x8*>(ab + i * 2048 + co);
    }
    // (no s_setprio: it made hipcc wait for all 16 reads before the first MFMA)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[kk][i], bfr[kk][j], acc[i][j]);

  };
  // band mode: A fragments from the patch slice `pbuf` at tap offset toff (patch rows); the
  // chunk XOR uses the patch row actually addressed (rows are stored swizzled by their own index)
  auto compute_band = [&](int buf, int pbuf, int toff) {
    const char* pa = smem + pbuf * pbytes;
    const char* bb = smem + bring + buf * (BN * 128) + (wn * WTN) * 128 + rl;
    bf16x8 af[2][TM], bfr[2][TN];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int co = kk ? co1 : co0;
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[kk][j] = *reinterpret_cast<const bf16x8*>(bb + j * 2048 + co);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pr = a_pb[i] + toff;
        af[kk][i] = *reinterpret_cast<const bf16x8*>(pa + pr * 128 + (((kk * 4 + (lane >> 4)) ^ (pr & 7)) << 4));
      }
    }
    // every fragment read is issued before the first MFMA (counted lgkmcnt waits then retire
    // them in order); left alone, hipcc recycles 3-4 fragment registers and drains the LDS
    // queue (lgkmcnt(0)) every 2-4 MFMAs, exposing the LDS latency ~7x per K-tile
    __builtin_amdgcn_sched_barrier(0);
    if (g.dbg & 1) return;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[kk][i], bfr[kk][j], acc[i][j]);
  };

  // ---- main loop ----
  if constexpr (BAND) {
    // prologue: patch slice 0 (all waves, junk-padded to a uniform count), then B tiles
    const int rounds0 = (npiece + NW - 1) / NW;
    for (int r = 0; r < rounds0; ++r) stage_piece(r * NW + w, 0, 0);
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nk) stage_b(s);
    if (STAGES == 3 && nk > 1) i2_wait_vm<B_PW>();
    else i2_wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    int cbuf = 0, sbuf = STAGES - 1;
    int cs = 0, tap = 0, toff = 0, tr = 0, tsc = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const bool issue = kt + STAGES - 1 < nk && !(g.dbg & 4);
      if (issue) stage_b(sbuf);
      // slice cs+1 streams in during taps 0..7 of slice cs (one piece per wave per tap; the
      // wait at the end of tap 8 sees the last of them land before slice cs+1 is read)
      const bool piece = cs + 1 < nslice && tap < 8 && tap * NW < npiece;
      if (piece) stage_piece(tap * NW + w, cs + 1, (cs + 1) & 1);
      if (!(g.dbg & 8)) compute_band(cbuf, cs & 1, toff);
      if constexpr (STAGES == 3) {
        if (issue) {
          if (piece) i2_wait_vm<B_PW + 1>(); else i2_wait_vm<B_PW>();
        } else {
          if (piece) i2_wait_vm<1>(); else i2_wait_vm<0>();
        }
      } else {
        i2_wait_vm<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      cbuf = cbuf + 1 == STAGES ? 0 : cbuf + 1;
      sbuf = sbuf + 1 == STAGES ? 0 : sbuf + 1;
      if (++tap == 9) { tap = 0; ++cs; tr = 0; tsc = 0; toff = 0; }
      else if (++tsc == 3) { tsc = 0; ++tr; toff = tr * PW2; }
      else ++toff;
    }
  }
  // Software-pipelined 2-stage loop (default for the 2-stage tiles; ConvGeom.dbg bit 16 = the
  // plain loop below): the fragment reads of k-half 1 of tile kt run in the MFMA
  // gaps of k-half 0, and the reads of k-half 0 of tile kt+1 in the gaps of k-half 1 -- the
  // barrier sits between the two halves, so no wave ever waits on an LDS read with its MFMA
  // pipe empty (the plain loop issues all 2 x (TM + TN) reads, more than the 4-bit lgkmcnt can
  // track, then its MFMAs: two exposed LDS latencies per K-tile, on every wave at once).
  //   tile kt+2 is staged right after barrier kt into the buffer tile kt vacated (every wave's
  //   reads of it retired by lgkmcnt(0) before that barrier) and must land by barrier kt+1.
  if constexpr (!BAND && STAGES == 2) {
    if (!(g.dbg & 16)) {
      const char* abase = smem + (wm * WTM) * 128 + rl;
      const char* bbase = smem + (BM + wn * WTN) * 128 + rl;
      // A fragments of rows 0..TM-2 single-buffered and replaced in place (row i's next fragment
      // is read one MFMA after row i's last use); the last row and the B fragments double-
      // buffered, so every read of the other half issues in an MFMA gap of this one: 28 fewer
      // VGPRs than two full fragment sets, which the 128-accumulator 256x256 tile cannot spare
      bf16x8 pa[TM - 1], pl[2], pb[2][TN];
      auto rda = [&](int buf, int kk, int i) {
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(abase + buf * SB + i * 2048 + (kk ? co1 : co0));
        if (i == TM - 1) pl[kk] = v; else pa[i] = v;
      };
      auto rdb = [&](int buf, int kk, int j) {
        pb[kk][j] = *reinterpret_cast<const bf16x8*>(bbase + buf * SB + j * 2048 + (kk ? co1 : co0));
      };
      // the TM x TN MFMAs of k-half kk (row-major); when rdo, the other half's fragments from
      // buffer rbuf are read in its gaps: B j after MFMA j, the last A row after MFMA TN, A row
      // i < TM-1 after MFMA (i+1)*TN (hipcc's counted lgkmcnt waits order every use)
      auto half = [&](int kk, bool rdo, int rbuf, int rkk) {
#pragma unroll
        for (int q = 0; q < TM * TN; ++q) {
          const int i = q / TN, j = q - (q / TN) * TN;
          acc[i][j] = mfma16(i == TM - 1 ? pl[kk] : pa[i < TM - 1 ? i : 0], pb[kk][j], acc[i][j]);
          if (rdo) {
            if (q < TN) rdb(rbuf, rkk, q);
            if (q == TN) rda(rbuf, rkk, TM - 1);
            if (q >= TN && q % TN == 0) rda(rbuf, rkk, q / TN - 1);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      stage(0);
      if (nk > 1) stage(1);
      if (nk > 1) i2_wait_vm<DPT>(); else i2_wait_vm<0>();
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int j = 0; j < TN; ++j) rdb(0, 0, j);
#pragma unroll
      for (int i = 0; i < TM; ++i) rda(0, 0, i);
      for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        half(0, true, buf, 1);
        // tile kt+1 (the only DMA in flight) has landed and no wave still reads tile kt
        i2_wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < nk) stage(buf);
        half(1, kt + 1 < nk, buf ^ 1, 0);
      }
      // every wave's ring reads retired before the last barrier and the final half issues none:
      // the epilogue may reuse the ring without another barrier
    }
  }
  int cbuf = 0, sbuf = STAGES - 1;
  const bool plain = !BAND && !(STAGES == 2 && !(g.dbg & 16));
  if constexpr (!BAND) {
    if (plain) {
#pragma unroll
      for (int s = 0; s < STAGES - 1; ++s)
        if (s < nk) stage(s);
      if (STAGES == 3 && nk > 1) i2_wait_vm<DPT>();
      else i2_wait_vm<0>();
      __builtin_amdgcn_s_barrier();
    }
  }
  for (int kt = 0; kt < (plain ? nk : 0); ++kt) {
    const bool issue = kt + STAGES - 1 < nk;
    if (issue) stage(sbuf);
    compute(cbuf);
    // tile kt+1 must have landed (every wave's part) before any wave reads it; with STAGES = 3
    // the tile issued above stays in flight across the barrier
    if constexpr (STAGES == 3) {
      if (issue) i2_wait_vm<DPT>();
      else i2_wait_vm<0>();
    } else {
      i2_wait_vm<0>();
    }
    // every fragment read of this buffer has returned before any wave restages it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cbuf = cbuf + 1 == STAGES ? 0 : cbuf + 1;
    sbuf = sbuf + 1 == STAGES ? 0 : sbuf + 1;
  }

  // ---- epilogue ----
  // every wave is past the last barrier: the operand ring is free. Wave-private fp32 patch of
  // 16 rows x WTN columns; one 16-row accumulator slice at a time.
  constexpr int PITCH = Cfg::EPI_PITCH;
  constexpr int CPR = WTN / 8;            // 8-column chunks per patch row
  constexpr int PPL = 16 * CPR / 64;      // pieces (row, chunk) per lane per slice
  float* patch = reinterpret_cast<float*>(smem) + w * 16 * PITCH;
  float* red = reinterpret_cast<float*>(smem) + NW * 16 * PITCH;  // [NWM][BN][2]
  const int fr = lane & 15, fq = lane >> 4;
  const int ch = lane % CPR;              // constant per lane: (lane + 64 h) % CPR
  const int colt = wn * WTN + ch * 8;     // column inside the block tile
  const int col0 = n0 + colt;
  const bool col_ok = col0 < g.K;         // K % 8 == 0 (launcher)
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  float bsv[8], mu[8], iv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { bsv[e] = 0.f; mu[e] = 0.f; iv[e] = 0.f; }
  if constexpr (EPI == 0 || EPI == 3) {
    if (bias && col_ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bsv[e] = bias[col0 + e];
    }
  }
  float msc[8], msh[8];
  if constexpr (EPI == 0 || EPI == 2) {
    if (bs.sums && !bs.zgelu && col_ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { mu[e] = bs.mean[col0 + e]; iv[e] = bs.inv[col0 + e]; }
    }
    bnm_coeffs(bs, col0, col_ok && bs.sums && !bs.zgelu, msc, msh);
  }
  // EPI 1: stats only; EPI 2: BN-backward sums only; EPI 0: either (stats win)
  const bool want_stats = stats != nullptr || bs.sums != nullptr;

  // EPI 2: the global operands of 16-row slice i + 1 (residual gradient, producer y, ReLU
  // mask / GELU pre-activation) are fetched while slice i is staged and stored, so their
  // latency overlaps the LDS patch round trip instead of serialising every slice
  // (ZOO_EPI2_BATCH=0: loads at the point of use)
  // (tiles with 128 accumulator registers per lane -- 256x256 -- have no room for the
  // prefetch registers: it spilled to scratch there, so they keep the loads at their use)
  // (the 12-wave 256x192 tile runs 3 waves per SIMD: 168 VGPRs, where the prefetch spilled too)
  const bool pre2 = EPI == 2 && TM * TN <= 16 && NW <= 8 && !bs.unbatched;
  uint4 nrv[PPL], nyv[PPL], nzv[PPL];
  unsigned nmb[PPL];
  auto slice_off = [&](int i, int h, bool& ok) -> size_t {
    const int prow = (lane + 64 * h) / CPR;
    const int m = m0 + wm * WTM + i * 16 + prow;
    ok = m < mlim && col_ok;
    if (!ok) return 0;
    if (g.omap) {
      const int n = m / PQ, pq = m - n * PQ;
      const int p = pq / g.Q, q = pq - p * g.Q;
      return ((size_t)(n * g.oH + g.oh0 + g.osh * p) * g.oW + g.ow0 + g.osw * q) * g.K + col0;
    }
    return (size_t)m * g.K + col0;
  };
  auto fetch2 = [&](int i) {
#pragma unroll
    for (int h = 0; h < PPL; ++h) {
      bool ok;
      const size_t off = slice_off(i, h, ok);
      nrv[h] = nyv[h] = nzv[h] = uint4{0u, 0u, 0u, 0u};
      nmb[h] = 0u;
      if (!ok) continue;
      if (resid) nrv[h] = *reinterpret_cast<const uint4*>(resid + off);
      if (bs.sums && !bs.zgelu) nyv[h] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off);
      if (bs.zgelu || (bs.zmode == 0 && bs.z))
        nzv[h] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.z) + off);
      else if (bs.zmode == 2)
        nmb[h] = reinterpret_cast<const uint8_t*>(bs.z)[off >> 3];
    }
  };
  if constexpr (EPI == 2) {
    if (pre2) fetch2(0);
  }

#pragma unroll
  for (int i = 0; i < TM; ++i) {
    uint4 crv[PPL], cyv[PPL], czv[PPL];
    unsigned cmb[PPL];
    if constexpr (EPI == 2) {
      if (pre2) {
#pragma unroll
        for (int h = 0; h < PPL; ++h) { crv[h] = nrv[h]; cyv[h] = nyv[h]; czv[h] = nzv[h]; cmb[h] = nmb[h]; }
        if (i + 1 < TM) fetch2(i + 1);
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) patch[(fq * 4 + r) * PITCH + j * 16 + fr] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int h = 0; h < PPL; ++h) {
      const int pidx = lane + 64 * h;
      const int prow = pidx / CPR;
      const int m = m0 + wm * WTM + i * 16 + prow;
      const float4 lo = *reinterpret_cast<const float4*>(patch + prow * PITCH + ch * 8);
      const float4 hi = *reinterpret_cast<const float4*>(patch + prow * PITCH + ch * 8 + 4);
      if (m >= mlim || !col_ok) continue;
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      size_t off;
      if (EPI != 1 && EPI != 3 && g.omap) {
        const int n = m / PQ, pq = m - n * PQ;
        const int p = pq / g.Q, q = pq - p * g.Q;
        off = ((size_t)(n * g.oH + g.oh0 + g.osh * p) * g.oW + g.ow0 + g.osw * q) * g.K + col0;
      } else {
        off = (size_t)m * g.K + col0;
      }
      if constexpr (EPI == 3) {
        // lean bias / activation epilogue: the activation branch is per 8-column piece
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += bsv[e];
        if (bs.act_pre) {   // training GELU linear: keep the pre-activation for the backward
          const uint4 pk = pack8(v);
          *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(bs.act_pre) + off) = pk;
          unpack8(pk, v);   // the activation of the stored (rounded) value, as the separate pass did
        }
        if (act == ACT_RELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        } else if (act == ACT_GELU) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
        }
        *reinterpret_cast<uint4*>(Y + off) = pack8(v);
      } else if constexpr (EPI == 1) {
        const uint4 pk = pack8(v);
        if (!(BAND && (g.dbg & 2))) *reinterpret_cast<uint4*>(Y + off) = pk;
        if (want_stats) {
          float q[8];
          unpack8(pk, q);
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += q[e]; s2[e] += q[e] * q[e]; }
        }
      } else if constexpr (EPI == 2) {
        if (resid) {
          float rv[8];
          unpack8(pre2 ? crv[h] : *reinterpret_cast<const uint4*>(resid + off), rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += rv[e];
        }
        float yy[8];
        const bool bnsum = bs.sums && !bs.zgelu;
        if (bnsum)
          unpack8(pre2 ? cyv[h] : *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off), yy);
        if (bs.zgelu) {
          float zz[8];
          unpack8(pre2 ? czv[h] : *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.z) + off), zz);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= gelu_grad_f(zz[e]);
        } else if (pre2) {
          bnm_apply_pre(bs, yy, msc, msh, cmb[h], czv[h], v);
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
      } else {
        if (resid) {
          float rv[8];
          unpack8(*reinterpret_cast<const uint4*>(resid + off), rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += rv[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e] + bsv[e], act);
        float yy[8];
        if (bs.sums) {
          unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off), yy);
          bnm_apply(bs, off, yy, msc, msh, v);
        }
        if (Yf) {
          *reinterpret_cast<float4*>(Yf + off) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(Yf + off + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
        if (Y) {
          const uint4 pk = pack8(v);
          *reinterpret_cast<uint4*>(Y + off) = pk;
          float q[8];
          unpack8(pk, q);
          if (stats) {
#pragma unroll
            for (int e = 0; e < 8; ++e) { s1[e] += q[e]; s2[e] += q[e] * q[e]; }
          } else if (bs.sums) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              s1[e] += q[e];
              s2[e] += q[e] * (yy[e] - mu[e]) * iv[e];
            }
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  if (EPI == 3 || !want_stats) return;
  // per-column sums: lanes sharing `ch` differ in bits >= log2(CPR); fold them, then the wave
  // rows of the block through LDS, then one store / atomic per column per block
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
      red[(wm * BN + colt + e) * 2 + 0] = s1[e];
      red[(wm * BN + colt + e) * 2 + 1] = s2[e];
    }
  }
  __syncthreads();
  float* const sacc = stats ? stats : bs.sums;
  for (int c = tid; c < BN; c += Cfg::NT) {
    const int col = n0 + c;
    if (col >= g.K) continue;
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int r = 0; r < NWM; ++r) { a += red[(r * BN + c) * 2]; b += red[(r * BN + c) * 2 + 1]; }
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

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------

// tile configurations (NWM, NWN, TM, TN, STAGES): block = (NWM*TM*16) x (NWN*TN*16)
enum I2Tile : int {
  I2_AUTO = 0,
  I2_128x128 = 1,   // 4 waves (2x2) of 64x64, 2-stage ring: 64 KiB LDS, 2 workgroups / CU
  I2_256x128 = 2,   // 8 waves (4x2) of 64x64, 2-stage: 96 KiB, 1 / CU
  I2_256x128_3 = 3, // 8 waves (4x2) of 64x64, 3-stage: 144 KiB, 1 / CU
  I2_256x64 = 4,    // 4 waves (4x1) of 64x64, 2-stage: 80 KiB, 2 / CU
  I2_256x256 = 5,   // 8 waves (2x4) of 128x64, 2-stage: 128 KiB, 1 / CU
  I2_128x64 = 6,    // 4 waves (2x2) of 64x32, 3-stage: 72 KiB, 2 / CU
  I2_128x128_3 = 7, // 4 waves (2x2) of 64x64, 3-stage: 96 KiB, 1 / CU
  // band mode (I2_AM_BAND, 224 = 4 x 56 or 8 x 28 output pixels; LDS = patch slice(s) + B ring)
  I2_B224x64 = 8,   // 4 waves (2x2) of 112x32, 3-stage: 45 KiB patch + 24 KiB ring, 2 / CU
  I2_B224x128 = 9,  // 8 waves (2x4) of 112x32, 3-stage: 2 x 38 KiB patches + 48 KiB ring, 1 / CU
  I2_B224x128w = 10,// 4 waves (2x2) of 112x64, 3-stage (A/B of the wider wave tile)
  I2_224x256 = 11,  // 8 waves (2x4) of 112x64, 2-stage: 120 KiB + junk slots, 1 / CU (wave quantization)
  I2_256x192 = 12,  // 12 waves (4x3) of 64x64, 2-stage: 112 KiB + junk slots, 1 / CU: a 768-wide output
                    // is 4 column tiles, so 16384 rows make 256 tiles -- one full round on 256 CUs
};

static bool i2_is_band(int tile) { return tile >= I2_B224x64 && tile <= I2_B224x128w; }

// selectors set through zoo_igemm2_set / zoo_igemm2_tile_set / zoo_igemm2_band_set (tests, A/B tools)
static int g_i2_mode = 1;  // 0: off, 1: on
static int g_i2_tile = 0;  // 0 auto, else I2Tile
// band tiles off since the two-stream backward: ResNet-50 b256 12,273 / 12,267 img/s off vs
// 12,239 / 12,205 on, same box (scripts/r4/knobs.sh); kept for the stride-1 band tests
static int g_i2_band = 0;
// 256x192 tiles for outputs that are a multiple of 192 wide: 0 off, 1 forward-type epilogues,
// 2 also the backward epilogues (BN / GELU backward). Off by default: faster alone (BERT linears
// 63.5 / 23.9 / 67.7 us vs 70.9 / 26.1 / 74.1 us) but the BERT training step loses 1.2 % with them
// (15.58 ms off vs 15.76 mode 1 / 15.73 mode 2, profiles/r6/ab6_bert_*_r6.log): 256 tiles take
// every CU, so the side-stream weight gradients beside the data-gradient chain find no free CU,
// where the 224-row tiles leave 34 of them (setter zoo_igemm2_w192_set for serial / inference use)
static int g_i2_w192 = 0;

static int i2_mode() { return g_i2_mode; }
static int i2_tile_force() { return g_i2_tile; }
static int i2_band_mode() { return g_i2_band; }

static int i2_bm(int tile) {
  switch (tile) {
    case I2_128x128: case I2_128x64: case I2_128x128_3: return 128;
    case I2_B224x64: case I2_B224x128: case I2_B224x128w: case I2_224x256: return 224;
    default: return 256;
  }
}
static int i2_bn(int tile) {
  switch (tile) {
    case I2_256x64: case I2_128x64: case I2_B224x64: return 64;
    case I2_256x256: case I2_224x256: return 256;
    case I2_256x192: return 192;
    default: return 128;
  }
}
static int i2_nw(int tile) {
  switch (tile) {
    case I2_256x128: case I2_256x128_3: case I2_256x256: case I2_B224x128: case I2_224x256: return 8;
    case I2_256x192: return 12;
    default: return 4;
  }
}

// band geometry of a tile on this conv: rows per band, bands per image, LDS patch slice bytes
struct I2Band {
  int tp, nbands, pbytes;
};
static I2Band i2_band_geom(const ConvGeom& g, int bm) {
  I2Band b;
  b.tp = bm / g.Q;
  b.nbands = (g.P + b.tp - 1) / b.tp;
  b.pbytes = (((b.tp + 2) * (g.Q + 2) + 7) / 8) * 1024;
  return b;
}

// m-tiles of a tile on this conv (band tiles: images x bands)
static long i2_tiles_m(const ConvGeom& g, int tile) {
  if (i2_is_band(tile)) return (long)g.N * i2_band_geom(g, i2_bm(tile)).nbands;
  return (g.M + i2_bm(tile) - 1) / i2_bm(tile);
}

template <int NWM, int NWN, int TM, int TN, int STAGES, int AM, int EPI>
static hipError_t i2_launch(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* Yf, const float* bias,
                            const bf16_t* resid, float* stats, const ConvGeom& g, int act, const BwdStats& bs,
                            hipStream_t st) {
  using Cfg = I2Cfg<NWM, NWN, TM, TN>;
  const int ntn = (g.K + Cfg::BN - 1) / Cfg::BN;
  long tiles;
  size_t smem;
  if constexpr (AM == I2_AM_BAND) {
    const I2Band b = i2_band_geom(g, Cfg::BM);
    tiles = (long)g.N * b.nbands * ntn;
    smem = (size_t)(g.C > 64 ? 2 : 1) * b.pbytes + (size_t)STAGES * Cfg::BN * 128 + (size_t)Cfg::NW * 1024;
  } else {
    tiles = (long)((g.M + Cfg::BM - 1) / Cfg::BM) * ntn;
    smem = (size_t)STAGES * Cfg::STAGE_BYTES + Cfg::JUNK_BYTES;
  }
  if (smem < (size_t)Cfg::EPI_BYTES) smem = Cfg::EPI_BYTES;
  if (smem > 160 * 1024) return hipErrorInvalidValue;
  auto kfn = &igemm2_kernel<NWM, NWN, TM, TN, STAGES, AM, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    // band smem depends on the conv's width: allow the whole LDS once
    hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize,
                        AM == I2_AM_BAND ? 160 * 1024 : (int)smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kfn, dim3((unsigned)tiles), dim3(Cfg::NT), smem, st, X, W, Y, Yf, bias, resid, stats, g, act, bs);
  return hipGetLastError();
}

template <int NWM, int NWN, int TM, int TN, int STAGES, int AM>
static hipError_t i2_epi(int epi, const bf16_t* X, const bf16_t* W, bf16_t* Y, float* Yf, const float* bias,
                         const bf16_t* resid, float* stats, const ConvGeom& g, int act, const BwdStats& bs,
                         hipStream_t st) {
  if (epi == 1) return i2_launch<NWM, NWN, TM, TN, STAGES, AM, 1>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  if (epi == 2) return i2_launch<NWM, NWN, TM, TN, STAGES, AM, 2>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  if constexpr (AM != I2_AM_BAND) {
    if (epi == 3) return i2_launch<NWM, NWN, TM, TN, STAGES, AM, 3>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
  }
  return i2_launch<NWM, NWN, TM, TN, STAGES, AM, 0>(X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
}

template <int AM>
static hipError_t i2_tile(int tile, int epi, const bf16_t* X, const bf16_t* W, bf16_t* Y, float* Yf,
                          const float* bias, const bf16_t* resid, float* stats, const ConvGeom& g, int act,
                          const BwdStats& bs, hipStream_t st) {
  if constexpr (AM == I2_AM_BAND) {
    switch (tile) {
      case I2_B224x64: return i2_epi<2, 2, 7, 2, 3, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_B224x128: return i2_epi<2, 4, 7, 2, 3, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_B224x128w: return i2_epi<2, 2, 7, 4, 3, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      default: return hipErrorInvalidValue;
    }
  } else {
    switch (tile) {
      case I2_128x128: return i2_epi<2, 2, 4, 4, 2, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_256x128: return i2_epi<4, 2, 4, 4, 2, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_256x128_3: return i2_epi<4, 2, 4, 4, 3, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_256x64: return i2_epi<4, 1, 4, 4, 2, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_256x256: return i2_epi<2, 4, 8, 4, 2, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_128x64: return i2_epi<2, 2, 4, 2, 3, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_128x128_3: return i2_epi<2, 2, 4, 4, 3, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_224x256: return i2_epi<2, 4, 7, 4, 2, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      case I2_256x192: return i2_epi<4, 3, 4, 4, 2, AM>(epi, X, W, Y, Yf, bias, resid, stats, g, act, bs, st);
      default: return hipErrorInvalidValue;
    }
  }
}

// band tile for a stride-1 3x3 conv (pad 1, no dilation, same-size output), or 0: the output
// width must divide the 224-pixel tile into whole rows with bands no taller than the image
// (Q = 56 -> 4 rows, Q = 28 -> 8 rows), the LDS patch + ring must fit, and each of the 8 DMA
// rounds of a slice must cover its patch (npiece <= 8 * waves)
static int i2_band_choose(const ConvGeom& g, int epi) {
  if (!i2_band_mode()) return 0;
  if (!(g.R == 3 && g.S == 3 && g.sh == 1 && g.sw == 1 && g.ph == 1 && g.pw == 1 && g.dh == 1 && g.dw == 1 &&
        g.lh == 1 && g.lw == 1 && g.H == g.P && g.W == g.Q && !g.omap && g.C % 64 == 0 && g.Q > 0))
    return 0;
  if (epi == 3 || epi == 4) return 0;
  if (224 % g.Q != 0 || 224 / g.Q > g.P) return 0;
  static const int forced = 0;
  const int t = forced >= I2_B224x64 ? forced : (g.K <= 64 ? I2_B224x64 : I2_B224x128);
  const I2Band b = i2_band_geom(g, 224);
  const size_t smem = (size_t)(g.C > 64 ? 2 : 1) * b.pbytes + 3 * (size_t)i2_bn(t) * 128 + (size_t)i2_nw(t) * 1024;
  if (smem > 160 * 1024 || (g.C > 64 && b.pbytes / 1024 > 8 * i2_nw(t))) return 0;
  return t;
}

// shape + epilogue -> tile, or 0 = "leave it to igemm.hip" (tools/igemm2_bench.py on the
// ResNet-50 b256 convs with the model's own epilogues, round 3, profiles/r3/igemm2_r3.md):
//   * stride-1 3x3 convs over 56- or 28-wide maps: the band tiles (patch reuse of the 9 taps);
//   * N (output channels) < 256: igemm.hip's 128x{64,128} tiles are as fast or faster;
//   * a short reduction (Ktot < 256 forward, < 1024 for the BN-backward epilogue) is bound by
//     the epilogue, where igemm.hip's row-pointer epilogues win (the GELU-backward form of EPI 2,
//     routing class 4, follows the forward rule: igemm.hip took 162 us vs ~77 us for BERT's
//     16384x3072x768 FFN dgrad, profiles/r3/bert_base_train_b128_r3.md);
//   * otherwise 256x256 (8 waves of 128x64) while >= 160 tiles fill the chip, else 128x128.
static int i2_choose(const ConvGeom& g, int epi) {
  const int bt = i2_band_choose(g, epi);
  if (bt > 0) return bt;
  const int f = i2_tile_force();
  if (f > 0 && !i2_is_band(f)) return f;
  auto tiles = [&](int t) { return i2_tiles_m(g, t) * ((g.K + i2_bn(t) - 1) / i2_bn(t)); };
  // narrowest output the large-tile kernel takes (ZOO_I2_KMIN; the 128x128 tile serves 128-wide
  // outputs such as the ResNet stage-2 3x3 convs when set to 128)
  static const int kmin = 256;
  if (g.K < kmin) return 0;
  if (epi == 4) {
    // GELU-backward dgrad (BERT FFN): ZOO_I2_GELU_TILE picks its tile (A/B of the 128x128
    // tile, whose EPI 2 prefetches the next slice's pre-activation, against 256x256)
    static const int gt = 0;
    if (gt > 0 && g.Ktot >= 256) return gt;
  }
  if (epi == 2 && g.Ktot < 1024) return 0;
  if (epi != 2 && g.Ktot < 256) return 0;
  if (tiles(I2_256x256) >= 160) {
    // wave quantization: one 256x256 workgroup per CU, so a grid of t tiles takes ceil(t / CUs)
    // rounds. 224-row tiles cost 7/8 of a 256-row round: take them when they finish in fewer
    // round-equivalents (BERT / ResNet stage 3-4: 196 tiles of 256 rows fill 77 % of the CUs,
    // 224 tiles of 224 rows 88 %; BERT linears 16384x{2304,768}x768 and x768x3072 -5..-7 %, ResNet-50
    // fwd/dgrad conv sweep -1..-2 %, profiles/r4/ab/q224_*). ZOO_I2_Q224=0: always 256x256.
    // 192-wide tiles (12 waves) cost 3/4 of a round and split 768- and 2304-wide outputs exactly:
    // BERT's 16384 x 768 x {768, 3072} and 16384 x 2304 x 768 linears 65.6-65.7 us vs 70.9-76.9 us
    // (tools/gemm_bench.py --bert --tiles, profiles/r6/ab5_gemm_tiles_r6.log)
    static int ncu = 0;
    if (!ncu) {
      int dev = 0;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      if (ncu <= 0) ncu = 256;
    }
    auto rounds = [&](int t) { return (double)((tiles(t) + ncu - 1) / ncu) * (i2_bm(t) * i2_bn(t)) / (256.0 * 256.0); };
    int best = I2_256x256;
    double cbest = rounds(I2_256x256);
    static const bool q224 = true;
    if (q224 && epi != 4 && rounds(I2_224x256) < 0.97 * cbest) {
      best = I2_224x256;
      cbest = rounds(I2_224x256);
    }
    const int w192 = g_i2_w192;
    if (w192 > 0 && g.K % 192 == 0 && (w192 > 1 || (epi != 2 && epi != 4)) && rounds(I2_256x192) < 0.97 * cbest)
      best = I2_256x192;
    return best;
  }
  return I2_128x128;
}

}  // namespace zoo

using namespace zoo;

// eligibility: whole 64-channel K-tiles, plain (non-input-dilated) conv, 16-byte rows, and a
// shape / epilogue where the large tiles win
extern "C" int zoo_igemm2_eligible(const ConvGeom* g, int epi) {
  if (i2_mode() == 0) return 0;
  return g->C % 64 == 0 && g->lh == 1 && g->lw == 1 && g->K % 8 == 0 && g->ldb % 8 == 0 &&
         g->Ktot == g->R * g->S * g->C && g->ldb >= g->Ktot && i2_choose(*g, epi) > 0;
}

// m-tile height the dispatcher will use for this geometry and epilogue; 0 = not taken by igemm2
extern "C" int zoo_igemm2_bm(const ConvGeom* g, int epi) {
  if (!zoo_igemm2_eligible(g, epi)) return 0;
  return i2_bm(i2_choose(*g, epi));
}

// number of m-tiles (rows of a partial-statistics buffer [tiles_m][2K]); 0 = not taken by igemm2
extern "C" int zoo_igemm2_tiles_m(const ConvGeom* g, int epi) {
  if (!zoo_igemm2_eligible(g, epi)) return 0;
  return (int)i2_tiles_m(*g, i2_choose(*g, epi));
}

extern "C" void zoo_igemm2_set(int mode, int tile) {
  if (mode >= 0) g_i2_mode = mode;
  if (tile >= 0) g_i2_tile = tile;
}

extern "C" void zoo_igemm2_w192_set(int mode) {
  if (mode >= 0) g_i2_w192 = mode;
}

// band tiles on / off (-1: leave)
extern "C" void zoo_igemm2_band_set(int on) {
  if (on >= 0) g_i2_band = on;
}

extern "C" hipError_t zoo_igemm2(const void* X, const void* W, void* Y, float* Yf, const float* bias,
                                 const void* resid, float* stats, const ConvGeom* g, int act, const BwdStats* bsp,
                                 hipStream_t st) {
  BwdStats bs = bsp ? *bsp : BwdStats{nullptr, nullptr, nullptr, nullptr, nullptr};
  const int epi = igemm_epi(Y, Yf, bias, resid, act, g->omap, bs.sums, stats);
  const int route = igemm_route_epi(epi, bs.zgelu != 0);
  if (!zoo_igemm2_eligible(g, route)) return hipErrorNotSupported;
  const bool is1x1 = g->R == 1 && g->S == 1 && g->sh == 1 && g->sw == 1 && g->ph == 0 && g->pw == 0 &&
                     g->H == g->P && g->W == g->Q;
  const int tile = i2_choose(*g, route);
  const bf16_t* x = (const bf16_t*)X;
  const bf16_t* w = (const bf16_t*)W;
  if (i2_is_band(tile)) {
    ConvGeom gb = *g;
    gb.dbg = 0;
    return i2_tile<I2_AM_BAND>(tile, epi, x, w, (bf16_t*)Y, Yf, bias, (const bf16_t*)resid, stats, gb, act, bs, st);
  }
  static const int pipe = 1;
  ConvGeom gp = *g;
  gp.dbg = pipe ? 0 : 16;  // bit 16: the plain (unpipelined) 2-stage loop
  if (is1x1)
    return i2_tile<I2_AM_1X1>(tile, epi, x, w, (bf16_t*)Y, Yf, bias, (const bf16_t*)resid, stats, gp, act, bs, st);
  return i2_tile<I2_AM_IMPLICIT>(tile, epi, x, w, (bf16_t*)Y, Yf, bias, (const bf16_t*)resid, stats, gp, act, bs,
                                 st);
}
