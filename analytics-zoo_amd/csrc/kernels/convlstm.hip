// One launch per ConvLSTM2D / ConvLSTM3D time step (gfx950): the recurrent convolution as an MFMA implicit
// GEMM with the LSTM cell in its epilogue.
//
// Gate-interleaved layout: the gate weights (and the input convolution's output, the gate
// gradients and the saved activations) are ordered column 4j + g = gate g (i, f, cand, o) of
// hidden channel j. A 16x16x32 MFMA accumulator gives each lane one pixel and 4 CONSECUTIVE rows,
// so with D = W . X^T (rows = gate columns, columns = pixels) a lane holds all four gate
// pre-activations of one (pixel, channel): the cell update needs no data exchange, no LDS and
// no second pass over gate tensors.
//
// Forward, step t:   g = gx_t + conv(h_{t-1}, Wh)  ->  i, f, cand, o;  c_t = f c_{t-1} + i cand;
//                    h_t = o act(c_t)  (h_t also stored bf16 in the padded NHWC history slot that
//                    step t + 1's conv reads). Step 0 (h_{-1} = 0) skips the GEMM.
// Backward, step t:  dh_t = dout_t + conv(dgb_{t+1}, flip(Wh)) (the recurrent data gradient, rows =
//                    hidden channels) and the step's cell backward in the same epilogue: gate
//                    gradients fp32 (the input conv's gradient) + bf16 (dgb_t, the operand of the
//                    next dgrad and of ONE batched weight-gradient conv over all steps), dc_{t-1}.
//
// Four waves per workgroup, 16 pixels per wave, all gate rows per wave (NI = rows / 16 <= 16).
// The workgroup stages the step's weights in LDS once (rows padded by 16 B: conflict-free 16-byte
// reads; from L2 when they exceed 128 KiB); the reduction Q*R*S*Cx is walked 32 deep with the
// activation fragments gathered straight from global (zero outside the image) CL_PF chunks ahead.
// Sized for the latency-bound recurrent step (M = B*D*H*W of a few thousand pixels, 4F <= 256
// gate rows).
// ConvLSTM3D is the same kernel with a depth axis (D slices, Q depth taps).
// Reference: InternalConvLSTM2D.scala / InternalConvLSTM3D.scala (Zs/pipeline/api/keras/layers),
// SURVEY.md §2.16 HK11.
#include "common.h"
#include "lstm.h"

namespace zoo {

struct CLArgs {
  const bf16_t* X;   // conv input [B][D][H][W][Cx] (null: no GEMM -- the step's recurrent term is 0)
  const bf16_t* Wt;  // weights [Nr][ldw], row n = output row, k = ((q * R + r) * S + s) * Cx + channel
  int B, D, H, Wd, Cx, Q, R, S, ldw, Nr, M, F, iact, act;   // ConvLSTM2D: D = Q = 1
  // forward
  const float* gx;      // [M][F][4] input-conv gate pre-activations (bias included)
  const bf16_t* gxb;    // or the same as bf16 (the input conv's own output; gx null)
  const float* cprev;   // [M][F] or null
  float* h;             // [M][F]
  float* c;             // [M][F]
  float* acts;          // [M][F][4] activated gates (saved for backward)
  bf16_t* hb;           // [M][ldh] next history slot
  int ldh;
  // backward
  const float* dout;    // [M][F] or null
  const float* cc;      // c_t [M][F]
  float* dc;            // in: dc_{t+1} contribution (null when dc_in is false), out: dc_{t-1}
  int dc_in;
  float* dg;            // [M][F][4] fp32 gate gradients (null: only the bf16 copy dgb)
  bf16_t* dgb;          // [M][ldg] bf16 gate gradients
  int ldg;
  // reduction range (32-deep chunks [c_beg, c_beg + c_cnt); c_cnt 0: all) and the K-split partial
  // sums [M][16 NI] fp32 (the persistent kernel's PART 1 stores them, PART 2 adds them)
  int c_beg, c_cnt;
  float* part;
};

constexpr int CL_WAVES = 4;   // 4 waves x 16 pixels per workgroup
constexpr int CL_PF = 4;      // activation chunks in flight per wave (one-tile kernels)
constexpr int CL_PPF = 4;     // ... in the persistent kernel (8 measured 3-5 % slower: ab24)

// reduction chunks of 32, padded to whole prefetch groups (the padding is zero in LDS and never loaded)
template <int PF>
__host__ __device__ inline int cl_kcp(int KD) { return ((KD + 31) / 32 + PF - 1) / PF * PF; }
// LDS row pitch: whole 256-B blocks, the 16-B units of row n XOR-swizzled by n & 15 -- conflict-free
// ds_read_b128 for the fragment reads (lane: row lane & 15, unit 4 c + (lane >> 4)) under gfx950's
// 4 x 16-lane groups; the earlier +16 B row padding left 2-way conflicts in every group
// (SQ_LDS_BANK_CONFLICT 3.7x the LDS-active cycles, profiles/r6/ab23_pmc2_sum_r6.txt)
template <int PF>
__host__ __device__ inline int cl_kdp(int KD) { return cl_kcp<PF>(KD) * 32; }

// acc[j][i] (rows 16 i .. 16 i + 15, this lane's pixel m0 + 16 j) = W[rows] . X_patch(m0 + 16 j)
// LDSW: the workgroup's weights staged once in LDS (rows padded to cl_kdp); else read from L2.
// MJ pixel blocks per wave share every weight fragment: at large M (a 32^3 ConvLSTM3D volume,
// 262k pixels per step) the kernel is bound by the L2 reads of weights the wave re-reads per
// 32-deep chunk (221 KiB per 16 pixels); MJ = 2 halves them per MFMA
// TAPU (Cx % 32 == 0: every 32-deep chunk lies in ONE tap): the chunk's tap offset is
// wave-uniform, walked incrementally in chunk order in scalar registers, and the lane adds only
// its own pixel's bounds checks to it. The general gather divides k by Cx, R * S and S per lane
// per chunk: with 4 - 8 MFMAs per chunk the step kernels were bound by that integer VALU work.
template <int NI, int MJ, bool LDSW, bool TAPU, int PF, bool KS>
ZOO_DEV void cl_gemm_impl(const CLArgs& a, int m0, f32x4 (&acc)[MJ][NI], int lane, const bf16_t* wl) {
  bool mok[MJ];
  int px[MJ], py[MJ], pz[MJ], pb[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) {
    const int m = m0 + 16 * j;
    mok[j] = m < a.M;
    const int mm = mok[j] ? m : 0;
    px[j] = mm % a.Wd;
    py[j] = (mm / a.Wd) % a.H;
    pz[j] = (mm / (a.Wd * a.H)) % a.D;
    pb[j] = mm / (a.Wd * a.H * a.D);
  }
  const int KD = a.Q * a.R * a.S * a.Cx;
  // this range's chunks (KS: the K-split's [c_beg, c_beg + c_cnt); else all)
  const int cb0 = KS ? a.c_beg : 0, KC = KS ? a.c_cnt : (KD + 31) / 32;
  const int kdp = cl_kdp<PF>(KC * 32);
  const int pq = a.Q / 2, ph = a.R / 2, pw = a.S / 2;
  const int kq = 8 * (lane >> 4), nr = lane & 15;
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  const bf16_t* X = a.X;
  const int Cx = a.Cx, RS = a.R * a.S, S = a.S, D = a.D, H = a.H, Wd = a.Wd;
  // branch-free: every lane loads from an in-bounds address (clamped) and zeroes the value when
  // the tap is outside the image / reduction -- a predicated load in a divergent branch made the
  // compiler wait for ALL outstanding loads (vmcnt(0)) before each chunk, serialising the prefetch
  auto load_act = [=](int j, int c) __attribute__((always_inline)) -> uint4 {
    int k = (cb0 + c) * 32 + kq;
    const bool kin = mok[j] && c < KC && k < KD;
    k = kin ? k : 0;
    const int tap = k / Cx, ch = k - tap * Cx;
    const int q = tap / RS, rs = tap - q * RS;
    const int r = rs / S, s = rs - r * S;
    const int zz = pz[j] + q - pq, yy = py[j] + r - ph, xx = px[j] + s - pw;
    const bool ok = kin && zz >= 0 && zz < D && yy >= 0 && yy < H && xx >= 0 && xx < Wd;
    const int zc = ok ? zz : pz[j], yc = ok ? yy : py[j], xc = ok ? xx : px[j];
    const uint4 v = *reinterpret_cast<const uint4*>(X + ((((size_t)pb[j] * D + zc) * H + yc) * Wd + xc) * Cx + ch);
    return ok ? v : z4;
  };
  // the next chunk's tap (TAPU), from the range's first chunk; it_c = chunk index in the range
  const int CB = Cx >> 5, tap0 = cb0 / (CB > 0 ? CB : 1);
  int it_c = 0, it_cb = cb0 - tap0 * CB, it_s = tap0 % S, it_r = (tap0 / S) % a.R, it_q = tap0 / RS;
  int t_dq = 0, t_dr = 0, t_ds = 0, t_off = 0;
  bool t_in = false;
  auto next_tap = [&]() __attribute__((always_inline)) {
    t_in = (!KS || it_c < KC) && it_q < a.Q;
    ++it_c;
    t_dq = it_q - pq;
    t_dr = it_r - ph;
    t_ds = it_s - pw;
    t_off = ((t_dq * H + t_dr) * Wd + t_ds) * Cx + it_cb * 32;
    if (++it_cb == CB) {
      it_cb = 0;
      if (++it_s == S) {
        it_s = 0;
        if (++it_r == a.R) {
          it_r = 0;
          ++it_q;
        }
      }
    }
  };
  // the lane's own pixel, channel kq (always in bounds), as an element offset from X
  size_t pbase[MJ];
#pragma unroll
  for (int j = 0; j < MJ; ++j) pbase[j] = ((((size_t)pb[j] * D + pz[j]) * H + py[j]) * Wd + px[j]) * Cx + kq;
  // by-value captures (as load_act): by-reference captured arrays went to scratch
  auto load_tap = [=](int j, int dq, int dr, int ds, int off, bool tin) __attribute__((always_inline)) -> uint4 {
    const int zz = pz[j] + dq, yy = py[j] + dr, xx = px[j] + ds;
    const bool ok = tin && mok[j] && (unsigned)zz < (unsigned)D && (unsigned)yy < (unsigned)H &&
                    (unsigned)xx < (unsigned)Wd;
    const uint4 v = *reinterpret_cast<const uint4*>(X + pbase[j] + (ok ? off : 0));
    return ok ? v : z4;
  };
  uint4 pre[MJ][PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    if constexpr (TAPU) {
      next_tap();
#pragma unroll
      for (int j = 0; j < MJ; ++j) pre[j][u] = load_tap(j, t_dq, t_dr, t_ds, t_off, t_in);
    } else {
#pragma unroll
      for (int j = 0; j < MJ; ++j) pre[j][u] = load_act(j, u);
    }
  }
  // whole prefetch groups (chunks past KC read zeros): a straight-line body, so the in-order
  // vmcnt waits only for the chunk being consumed
  const int KCp = cl_kcp<PF>(KC * 32);
  for (int c0 = 0; c0 < KCp; c0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int c = c0 + u;
      const int k = c * 32 + kq;   // in the range (LDS image); the weight row's k is (cb0 + c) * 32 + kq
      uint4 wv[NI];   // every row block's weight fragment first (one LDS wait), then the MFMAs
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int n = 16 * i + nr;
        if (LDSW) {
          wv[i] = *reinterpret_cast<const uint4*>(wl + (size_t)n * kdp + (((k >> 3) ^ nr) << 3));   // zero padded
        } else {
          const int kg = cb0 * 32 + k;
          const bool ok = n < a.Nr && c < KC && kg < KD;
          const uint4 t = *reinterpret_cast<const uint4*>(a.Wt + (size_t)(ok ? n : 0) * a.ldw + (ok ? kg : 0));
          wv[i] = ok ? t : z4;
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the fragment reads batched ahead of the MFMAs
      if constexpr (TAPU) next_tap();   // chunk c + PF
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const bf16x8 bv = __builtin_bit_cast(bf16x8, pre[j][u]);
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[j][i] = mfma16(__builtin_bit_cast(bf16x8, wv[i]), bv, acc[j][i]);
        // refill this slot after its use: the in-order vmcnt then waits only for this chunk's load
        if constexpr (TAPU)
          pre[j][u] = load_tap(j, t_dq, t_dr, t_ds, t_off, t_in);
        else
          pre[j][u] = load_act(j, c + PF);
      }
    }
  }
}

template <int NI, int MJ, bool LDSW, int PF, bool KS = false>
ZOO_DEV void cl_gemm(const CLArgs& a, int m0, f32x4 (&acc)[MJ][NI], int lane, const bf16_t* wl) {
#pragma unroll
  for (int j = 0; j < MJ; ++j)
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (!a.X) return;
  if ((a.Cx & 31) == 0)
    cl_gemm_impl<NI, MJ, LDSW, true, PF, KS>(a, m0, acc, lane, wl);
  else
    cl_gemm_impl<NI, MJ, LDSW, false, PF, KS>(a, m0, acc, lane, wl);
}

// stage rows [0, 16 NI) of the weights (zero beyond Nr / KD) into LDS, pitch cl_kdp(KD), swizzled.
// CP: channel-blocked forward rows -- LDS row 16 i + 4 quad + g <- gate-interleaved row
// 4 (quad NI + i) + g (cl_fwd_tile_cp)
template <int NI, int PF, bool CP = false>
ZOO_DEV void cl_stage(const CLArgs& a, bf16_t* wl) {
  if (!a.X) return;
  const int KD = a.Q * a.R * a.S * a.Cx;
  const int KC = a.c_cnt > 0 ? a.c_cnt : (KD + 31) / 32, kb = a.c_beg * 32, kdp = cl_kdp<PF>(KC * 32);
  const int per_row = kdp / 8, total = 16 * NI * per_row;
  // batches of 8 independent 16-byte loads in flight per thread before their LDS stores (a
  // load-store-load loop would pay one L2 round trip per element: ~20 us for 73 KB)
  constexpr int BATCH = 8;
  const bf16_t* Wt = a.Wt;
  const int ldw = a.ldw, Nr = a.Nr;
  for (int e0 = threadIdx.x; e0 < total; e0 += BATCH * blockDim.x) {
    uint4 v[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int e = e0 + u * blockDim.x;
      const int n = e / per_row, k = (e - n * per_row) * 8;
      const int src = CP ? 4 * (((n >> 2) & 3) * NI + (n >> 4)) + (n & 3) : n;
      v[u] = e < total && src < Nr && k < KC * 32 && kb + k < KD
                 ? *reinterpret_cast<const uint4*>(Wt + (size_t)src * ldw + kb + k)
                 : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int e = e0 + u * blockDim.x;
      const int n = e / per_row, k = (e - n * per_row) * 8;
      if (e < total) *reinterpret_cast<uint4*>(wl + (size_t)n * kdp + (((k >> 3) ^ (n & 15)) << 3)) = v[u];
    }
  }
  __syncthreads();
}

// The epilogue operands do not depend on the GEMM: they are loaded BEFORE it (every lane, clamped
// addresses, no branch) so their latency hides behind the reduction; loading them between the
// stores of the epilogue made each channel wait for its own round trip (the stores may alias the
// loads): 11 us of a 23 us step.
// K-split partial sums, [M][16 NI] fp32 in the accumulator layout (lane: pixel, 4 consecutive rows)
template <int NI, int MJ, int PART>
ZOO_DEV void cl_part(const CLArgs& a, int m0, int lane, f32x4 (&acc)[MJ][NI]) {
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      float4* pp = reinterpret_cast<float4*>(a.part + (size_t)m * (16 * NI) + 16 * i + 4 * (lane >> 4));
      if constexpr (PART == 1) {
        *pp = make_float4(acc[jb][i][0], acc[jb][i][1], acc[jb][i][2], acc[jb][i][3]);
      } else {
        const float4 v = *pp;
        acc[jb][i][0] += v.x;
        acc[jb][i][1] += v.y;
        acc[jb][i][2] += v.z;
        acc[jb][i][3] += v.w;
      }
    }
  }
}

// one wave's MJ pixel blocks of the forward step; cofs = the first hidden channel of the wave's rows
// (a row group of the persistent kernel; 0 otherwise). STAGE: stage the weights first (LDSW).
// PART (K-split, CLArgs::part): 1 = store this reduction range's sums and stop, 2 = add them, then
// the cell
template <int NI, int MJ, bool LDSW, bool STAGE, int PF, int PART = 0>
ZOO_DEV void cl_fwd_tile(const CLArgs& a, int m0, int lane, bf16_t* wl, int cofs) {
  if constexpr (PART == 1) {
    if (LDSW && STAGE) cl_stage<NI, PF>(a, wl);
    f32x4 acc[MJ][NI];
    cl_gemm<NI, MJ, LDSW, PF, true>(a, m0, acc, lane, wl);
    cl_part<NI, MJ, 1>(a, m0, lane, acc);
    return;
  }
  const int F = a.F;
  const float* __restrict__ gx = a.gx;
  const float* __restrict__ cprev = a.cprev;
  float4 g4[MJ][NI];
  float cp[MJ][NI];
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    const int mc = m < a.M ? m : a.M - 1;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = cofs + 4 * i + (lane >> 4);   // rows 16 i + 4 (lane >> 4) + q = gate q of channel j
      const size_t e = (size_t)mc * F + (j < F ? j : F - 1);
      if (a.gxb) {
        const uint2 u = *reinterpret_cast<const uint2*>(a.gxb + 4 * e);
        g4[jb][i] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
      } else {
        g4[jb][i] = *reinterpret_cast<const float4*>(gx + 4 * e);
      }
      cp[jb][i] = cprev ? cprev[e] : 0.f;
    }
  }
  if (LDSW && STAGE) cl_stage<NI, PF>(a, wl);
  f32x4 acc[MJ][NI];
  cl_gemm<NI, MJ, LDSW, PF, PART != 0>(a, m0, acc, lane, wl);
  if constexpr (PART == 2) cl_part<NI, MJ, 2>(a, m0, lane, acc);
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = cofs + 4 * i + (lane >> 4);
      if (j >= F) continue;
      const size_t e = (size_t)m * F + j;
      const float4 g = g4[jb][i];
      const float ig = lstm_act(acc[jb][i][0] + g.x, a.iact), fg = lstm_act(acc[jb][i][1] + g.y, a.iact);
      const float cg = lstm_act(acc[jb][i][2] + g.z, a.act), og = lstm_act(acc[jb][i][3] + g.w, a.iact);
      const float cn = fg * cp[jb][i] + ig * cg;
      const float hn = og * lstm_act(cn, a.act);
      a.c[e] = cn;
      a.h[e] = hn;
      a.hb[(size_t)m * a.ldh + j] = f2bf(hn);
      *reinterpret_cast<float4*>(a.acts + 4 * e) = make_float4(ig, fg, cg, og);
    }
  }
}

// Persistent forward step, channel-blocked rows (cl_stage CP: row 16 i + 4 quad + g = gate g of
// channel cofs + quad NI + i), so a lane's NI channels are consecutive and the cell operands /
// results move as 16-byte vectors -- with the gate-interleaved rows (channels quad + 4 i) every
// channel was its own 2 - 8 byte access, 56 memory instructions per 16 pixels against the half
// reduction's 14 gathers (K-split). Launcher: NI % 4 == 0, 4 F = 16 NI x row groups.
template <int NI, int MJ, int PF, int PART>
ZOO_DEV void cl_fwd_tile_cp(const CLArgs& a, int m0, int lane, bf16_t* wl, int cofs) {
  static_assert(NI % 4 == 0, "channel-blocked forward: 4 | NI");
  f32x4 acc[MJ][NI];
  if constexpr (PART == 1) {
    cl_gemm<NI, MJ, true, PF, true>(a, m0, acc, lane, wl);
    cl_part<NI, MJ, 1>(a, m0, lane, acc);
    return;
  }
  const int F = a.F;
  const int j0 = cofs + (lane >> 4) * NI;   // the lane's NI consecutive channels
  float4 g4[MJ][NI];
  float cp[MJ][NI];
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb, mc = m < a.M ? m : a.M - 1;
    const size_t e0 = (size_t)mc * F + j0;
    if (a.gxb) {
#pragma unroll
      for (int i = 0; i < NI; i += 2) {
        const uint4 u = *reinterpret_cast<const uint4*>(a.gxb + 4 * (e0 + i));
        g4[jb][i] = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
        g4[jb][i + 1] = make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u),
                                    __uint_as_float(u.w << 16), __uint_as_float(u.w & 0xffff0000u));
      }
    } else {
#pragma unroll
      for (int i = 0; i < NI; ++i) g4[jb][i] = *reinterpret_cast<const float4*>(a.gx + 4 * (e0 + i));
    }
#pragma unroll
    for (int i = 0; i < NI; i += 4) {
      const float4 c4 = a.cprev ? *reinterpret_cast<const float4*>(a.cprev + e0 + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      cp[jb][i] = c4.x;
      cp[jb][i + 1] = c4.y;
      cp[jb][i + 2] = c4.z;
      cp[jb][i + 3] = c4.w;
    }
  }
  cl_gemm<NI, MJ, true, PF, PART != 0>(a, m0, acc, lane, wl);
  if constexpr (PART == 2) cl_part<NI, MJ, 2>(a, m0, lane, acc);
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    if (m >= a.M) continue;
    const size_t e = (size_t)m * F + j0;
    float cn[NI], hn[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const float4 g = g4[jb][i];
      const float ig = lstm_act(acc[jb][i][0] + g.x, a.iact), fg = lstm_act(acc[jb][i][1] + g.y, a.iact);
      const float cg = lstm_act(acc[jb][i][2] + g.z, a.act), og = lstm_act(acc[jb][i][3] + g.w, a.iact);
      cn[i] = fg * cp[jb][i] + ig * cg;
      hn[i] = og * lstm_act(cn[i], a.act);
      *reinterpret_cast<float4*>(a.acts + 4 * (e + i)) = make_float4(ig, fg, cg, og);
    }
#pragma unroll
    for (int i = 0; i < NI; i += 4) {
      *reinterpret_cast<float4*>(a.c + e + i) = make_float4(cn[i], cn[i + 1], cn[i + 2], cn[i + 3]);
      *reinterpret_cast<float4*>(a.h + e + i) = make_float4(hn[i], hn[i + 1], hn[i + 2], hn[i + 3]);
      *reinterpret_cast<uint2*>(a.hb + (size_t)m * a.ldh + j0 + i) =
          make_uint2((uint32_t)f2bf(hn[i]) | ((uint32_t)f2bf(hn[i + 1]) << 16),
                     (uint32_t)f2bf(hn[i + 2]) | ((uint32_t)f2bf(hn[i + 3]) << 16));
    }
  }
}

template <int NI, int MJ, bool LDSW>
__global__ __launch_bounds__(64 * CL_WAVES) void convlstm_fwd_kernel(CLArgs a) {
  extern __shared__ __attribute__((aligned(16))) char cl_smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(cl_smem);
  const int lane = threadIdx.x & 63;
  const int m0 = (blockIdx.x * CL_WAVES + (threadIdx.x >> 6)) * 16 * MJ + (lane & 15);
  cl_fwd_tile<NI, MJ, LDSW, true, CL_PF>(a, m0, lane, wl, 0);
}

// backward: operands of every (row block, channel) up front while NI <= 4 (the data-gradient rows
// are the hidden channels: <= 64); wider row counts load them per row block
// rofs = the wave's first data-gradient row (hidden channel): a row group of the persistent kernel
template <int NI, int MJ, bool LDSW, bool STAGE, int PF, int PART = 0>
ZOO_DEV void cl_bwd_tile(const CLArgs& a, int m0, int lane, bf16_t* wl, int rofs) {
  if constexpr (PART == 1) {
    if (LDSW && STAGE) cl_stage<NI, PF>(a, wl);
    f32x4 acc[MJ][NI];
    cl_gemm<NI, MJ, LDSW, PF, true>(a, m0, acc, lane, wl);
    cl_part<NI, MJ, 1>(a, m0, lane, acc);
    return;
  }
  constexpr bool PRE = NI * MJ <= 4;
  constexpr int NP = PRE ? NI : 1, MP = PRE ? MJ : 1;
  const int F = a.F;
  const float* __restrict__ acts = a.acts;
  const float* __restrict__ cc = a.cc;
  const float* __restrict__ dout = a.dout;
  const float* __restrict__ cprev = a.cprev;
  const float* __restrict__ dcin = a.dc_in ? a.dc : nullptr;
  float4 av[MP][NP][4];
  float cv[MP][NP][4], ov[MP][NP][4], dv[MP][NP][4], pv[MP][NP][4];
  // F % 4 == 0: a lane's 4 rows are 4 consecutive channels, all < F or all >= F -- one 16-byte
  // access per operand instead of four 4-byte ones (the epilogue's memory instructions rivalled the
  // K-split half reduction's gathers)
  const bool f4 = (F & 3) == 0;
  auto ld4 = [](const float* p, size_t e) -> float4 {
    return p ? *reinterpret_cast<const float4*>(p + e) : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto load_ops = [&](int jb, int i, int sj, int slot) {
    const int m = m0 + 16 * jb;
    const int mc = m < a.M ? m : a.M - 1;
    if (f4) {
      const int j0 = rofs + 16 * i + 4 * (lane >> 4);
      const size_t e0 = (size_t)mc * F + (j0 < F ? j0 : F - 4);
      const float4 c4 = ld4(cc, e0), o4 = ld4(dout, e0), d4 = ld4(dcin, e0), p4 = ld4(cprev, e0);
      const float c4a[4] = {c4.x, c4.y, c4.z, c4.w}, o4a[4] = {o4.x, o4.y, o4.z, o4.w};
      const float d4a[4] = {d4.x, d4.y, d4.z, d4.w}, p4a[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        av[sj][slot][q] = *reinterpret_cast<const float4*>(acts + 4 * (e0 + q));
        cv[sj][slot][q] = c4a[q];
        ov[sj][slot][q] = o4a[q];
        dv[sj][slot][q] = d4a[q];
        pv[sj][slot][q] = p4a[q];
      }
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = rofs + 16 * i + 4 * (lane >> 4) + q;   // row = hidden channel of the data gradient
      const size_t e = (size_t)mc * F + (j < F ? j : F - 1);
      av[sj][slot][q] = *reinterpret_cast<const float4*>(acts + 4 * e);
      cv[sj][slot][q] = cc[e];
      ov[sj][slot][q] = dout ? dout[e] : 0.f;
      dv[sj][slot][q] = dcin ? dcin[e] : 0.f;
      pv[sj][slot][q] = cprev ? cprev[e] : 0.f;
    }
  };
  if constexpr (PRE) {
#pragma unroll
    for (int jb = 0; jb < MJ; ++jb)
#pragma unroll
      for (int i = 0; i < NI; ++i) load_ops(jb, i, jb, i);
  }
  if (LDSW && STAGE) cl_stage<NI, PF>(a, wl);
  f32x4 acc[MJ][NI];
  cl_gemm<NI, MJ, LDSW, PF, PART != 0>(a, m0, acc, lane, wl);
  if constexpr (PART == 2) cl_part<NI, MJ, 2>(a, m0, lane, acc);
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int slot = PRE ? i : 0, sj = PRE ? jb : 0;
      if constexpr (!PRE) load_ops(jb, i, 0, 0);
      const int jq0 = rofs + 16 * i + 4 * (lane >> 4);
      if (f4 && jq0 >= F) continue;
      uint32_t gw[8];
      float dcn[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = jq0 + q;
        if (!f4 && j >= F) continue;
        const size_t e = (size_t)m * F + j;
        const float ig = av[sj][slot][q].x, fg = av[sj][slot][q].y, cg = av[sj][slot][q].z, og = av[sj][slot][q].w;
        const float tc = lstm_act(cv[sj][slot][q], a.act);
        const float dh = acc[jb][i][q] + ov[sj][slot][q];
        const float dcv = dh * og * lstm_dact(tc, a.act) + dv[sj][slot][q];
        const float cpv = pv[sj][slot][q];
        const float d0 = dcv * cg * lstm_dact(ig, a.iact), d1 = dcv * cpv * lstm_dact(fg, a.iact);
        const float d2 = dcv * ig * lstm_dact(cg, a.act), d3 = dh * tc * lstm_dact(og, a.iact);
        if (a.dg) *reinterpret_cast<float4*>(a.dg + 4 * e) = make_float4(d0, d1, d2, d3);
        gw[2 * q] = (uint32_t)f2bf(d0) | ((uint32_t)f2bf(d1) << 16);
        gw[2 * q + 1] = (uint32_t)f2bf(d2) | ((uint32_t)f2bf(d3) << 16);
        dcn[q] = dcv * fg;
        if (!f4) {
          *reinterpret_cast<uint2*>(a.dgb + (size_t)m * a.ldg + 4 * j) = make_uint2(gw[2 * q], gw[2 * q + 1]);
          a.dc[e] = dcn[q];   // this lane read dc_{t+1}[e] before: in place
        }
      }
      if (f4) {   // 4 channels x 4 gates bf16 = 32 contiguous bytes; dc as one float4
        uint4* gp = reinterpret_cast<uint4*>(a.dgb + (size_t)m * a.ldg + 4 * jq0);
        gp[0] = make_uint4(gw[0], gw[1], gw[2], gw[3]);
        gp[1] = make_uint4(gw[4], gw[5], gw[6], gw[7]);
        *reinterpret_cast<float4*>(a.dc + (size_t)m * F + jq0) = make_float4(dcn[0], dcn[1], dcn[2], dcn[3]);
      }
    }
  }
}

template <int NI, int MJ, bool LDSW>
__global__ __launch_bounds__(64 * CL_WAVES) void convlstm_bwd_kernel(CLArgs a) {
  extern __shared__ __attribute__((aligned(16))) char cl_smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(cl_smem);
  const int lane = threadIdx.x & 63;
  const int m0 = (blockIdx.x * CL_WAVES + (threadIdx.x >> 6)) * 16 * MJ + (lane & 15);
  cl_bwd_tile<NI, MJ, LDSW, true, CL_PF>(a, m0, lane, wl, 0);
}

// Persistent variant for the large steps (a 32^3 ConvLSTM3D volume: 262k pixels per step) whose
// weights exceed LDS: the rows are split into RG groups whose weights do fit (forward: 64 of the
// 128 gate rows = 16 hidden channels, all four gates; backward: 16 of the 32 data-gradient rows),
// one workgroup of CL_PW waves per CU stages its group's weights ONCE and walks pixel tiles. The
// one-tile-per-workgroup kernels either re-read the weights from L2 per 32-deep chunk (221 KiB per
// 16 pixels) or re-stage all of them per 64-pixel workgroup. Workgroup b: XCD b & 7; the RG
// workgroups of consecutive b >> 3 share an XCD and walk the same tiles (the activation gather of
// the second group hits that XCD's L2). Launcher: G % (8 RG) == 0.
// K-split (PART 1 / 2, RG = 1): all rows, the reduction halved over two launches whose weights each
// fit LDS -- the activations are gathered once per step instead of once per row group (the
// row-group split doubled the gathers, which bound the backward step: 3.5M wave-loads per step
// against 3.5M MFMAs, profiles/r6/ab23_pmc*_sum_r6.txt); the first launch stores its fp32 sums, the
// second adds them before the cell.
constexpr int CL_PW = 8;
template <int NI, int MJ, bool BWD, int PART, bool CP>
__global__ __launch_bounds__(64 * CL_PW) void convlstm_pers_kernel(CLArgs a, int RG) {
  extern __shared__ __attribute__((aligned(16))) char cl_smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(cl_smem);
  const int b = blockIdx.x, G = gridDim.x;
  const int xcd = b & 7, li = b >> 3;
  const int rg = li % RG, wi = (li / RG) * 8 + xcd, NW = G / RG;
  const int r0 = rg * 16 * NI;
  CLArgs ag = a;
  ag.Wt = a.Wt + (size_t)r0 * a.ldw;
  ag.Nr = a.Nr - r0;
  cl_stage<NI, CL_PPF, CP>(ag, wl);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int TPX = 16 * MJ * CL_PW;
  const int ntiles = (a.M + TPX - 1) / TPX;
  for (int t = wi; t < ntiles; t += NW) {   // uniform per workgroup: no barrier inside
    const int m0 = (t * CL_PW + wv) * 16 * MJ + (lane & 15);
    if constexpr (BWD)
      cl_bwd_tile<NI, MJ, true, false, CL_PPF, PART>(ag, m0, lane, wl, r0);
    else if constexpr (CP)
      cl_fwd_tile_cp<NI, MJ, CL_PPF, PART>(ag, m0, lane, wl, r0 / 4);
    else
      cl_fwd_tile<NI, MJ, true, false, CL_PPF, PART>(ag, m0, lane, wl, r0 / 4);
  }
}

// weights in LDS while they fit 128 KiB per workgroup (one workgroup per CU at these grids); else from L2
constexpr size_t CL_LDS_MAX = 128 * 1024;

template <int NI, int MJ, bool LDSW, bool BWD>
static hipError_t cl_launch2(const CLArgs& a, size_t smem, hipStream_t st) {
  const dim3 grid((a.M + 16 * MJ * CL_WAVES - 1) / (16 * MJ * CL_WAVES));
  auto kf = BWD ? &convlstm_bwd_kernel<NI, MJ, LDSW> : &convlstm_fwd_kernel<NI, MJ, LDSW>;
  if (LDSW) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kf),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kf, grid, dim3(64 * CL_WAVES), LDSW ? smem : 0, st, a);
  return hipGetLastError();
}

// pixel blocks per wave: 2 once the step has enough pixels to fill the chip with half the waves
// (>= 64k: 512+ workgroups) and the weights do not fit in LDS (each wave then re-reads them from
// L2 per chunk), while the registers allow it (forward <= 8 row blocks: 242 VGPRs; backward <= 4:
// its epilogue operands spill beyond); small latency-bound steps keep one block per wave
// persistent kernels for the large steps: 1 K-split (else row groups), 2 row groups only, 0 off (A/Bs)
static int g_cl_pers = 1;
// forward K-split also at >= 64k pixels (0: the row-group kernel there: its one launch without the
// fp32 partial round trip ran the 32^3 forward step in 210 vs 260 us, ab22 / ab26 totals)
static int g_cl_fks = 0;
static int g_cl_cp = 1;   // channel-blocked epilogue on the row-group forward (A/B: pers_set bit 3)
static int g_cl_ncu = 0;

template <int NIG, int MJ, bool BWD, int PART = 0, bool CP = false>
static hipError_t cl_launch_pers(const CLArgs& a, int RG, size_t smem, hipStream_t st) {
  auto kf = &convlstm_pers_kernel<NIG, MJ, BWD, PART, CP>;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kf),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
  if (e != hipSuccess) return e;
  if (!g_cl_ncu) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_cl_ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (g_cl_ncu <= 0) g_cl_ncu = 256;
  }
  // one workgroup per CU (the LDS image allows one), a multiple of 8 RG
  const int unit = 8 * RG;
  const int G = (g_cl_ncu / unit > 0 ? g_cl_ncu / unit : 1) * unit;
  hipLaunchKernelGGL(kf, dim3(G), dim3(64 * CL_PW), smem, st, a, RG);
  return hipGetLastError();
}

template <int NI, bool BWD>
static hipError_t cl_launch_dir(const CLArgs& a, hipStream_t st) {
  const int KD = a.Q * a.R * a.S * a.Cx;
  const size_t smem = (size_t)16 * NI * cl_kdp<CL_PF>(KD) * 2;
  const size_t psmem = (size_t)16 * NI * cl_kdp<CL_PPF>(KD) * 2;   // all rows at the persistent padding
  // K-split: all rows, two halves of the reduction (tap-aligned gathers, partial-sum buffer given)
  if constexpr (NI <= (BWD ? 2 : 8) && (BWD || NI % 4 == 0)) {
    // from 32k pixels: one 128-pixel tile per workgroup of the 256-workgroup grid and up
    if (a.X && a.M >= 32768 && smem > CL_LDS_MAX && g_cl_pers == 1 && a.part && (a.Cx & 31) == 0 &&
        (BWD || 4 * a.F == 16 * NI) && (a.ldh % 4) == 0 && (BWD || a.M < 65536 || g_cl_fks)) {
      const int KC = (KD + 31) / 32, KH = (KC + 1) / 2;
      const size_t ks = (size_t)16 * NI * cl_kdp<CL_PPF>(KH * 32) * 2;
      if (ks <= CL_LDS_MAX) {
        // one pixel block per wave except the 1-row-block backward (the cell-backward operands of
        // two blocks and two row blocks spilled; the 8-row-block forward holds one)
        constexpr int MJK = (BWD && NI == 1) ? 2 : 1;
        CLArgs a0 = a, a1 = a;
        a0.c_beg = 0;
        a0.c_cnt = KH;
        a1.c_beg = KH;
        a1.c_cnt = KC - KH;
        // the first half has no epilogue operands: two pixel blocks per wave (more gathers in flight)
        // once there are tiles for every workgroup (at 32k pixels 256-pixel tiles left half the
        // CUs idle: 16^3 3.25 vs 2.97 ms; 32^3 18.41-18.49 vs 18.57-18.60 ms, ab35)
        const hipError_t e = a.M >= 65536 ? cl_launch_pers<NI, 2, BWD, 1, !BWD>(a0, 1, ks, st)
                                          : cl_launch_pers<NI, MJK, BWD, 1, !BWD>(a0, 1, ks, st);
        if (e != hipSuccess) return e;
        return cl_launch_pers<NI, MJK, BWD, 2, !BWD>(a1, 1, ks, st);
      }
    }
  }
  if (a.X && a.M >= 65536 && smem > CL_LDS_MAX && g_cl_pers) {
    if constexpr (NI % 2 == 0 && NI / 2 <= (BWD ? 1 : 5)) {   // register-bound: no spills
      if (psmem / 2 <= CL_LDS_MAX) {
        if constexpr (!BWD && (NI / 2) % 4 == 0) {   // channel-blocked epilogue where the rows allow
          if (4 * a.F == 16 * NI && (a.ldh % 4) == 0 && g_cl_cp)
            return cl_launch_pers<NI / 2, 2, BWD, 0, true>(a, 2, psmem / 2, st);
        }
        return cl_launch_pers<NI / 2, 2, BWD>(a, 2, psmem / 2, st);
      }
    }
    if constexpr (NI % 4 == 0 && NI / 4 <= (BWD ? 1 : 5)) {
      if (psmem / 4 <= CL_LDS_MAX) return cl_launch_pers<NI / 4, 2, BWD>(a, 4, psmem / 4, st);
    }
  }
  if (a.X && smem <= CL_LDS_MAX) return cl_launch2<NI, 1, true, BWD>(a, smem, st);
  if constexpr (NI <= (BWD ? 4 : 8)) {
    if (a.X && a.M >= 65536) return cl_launch2<NI, 2, false, BWD>(a, 0, st);
  }
  return cl_launch2<NI, 1, false, BWD>(a, 0, st);
}

template <int NI>
static hipError_t cl_launch(const CLArgs& a, int bwd, hipStream_t st) {
  return bwd ? cl_launch_dir<NI, true>(a, st) : cl_launch_dir<NI, false>(a, st);
}

}  // namespace zoo

using namespace zoo;

// rows: forward 4F (gate rows), backward the hidden channels of the data gradient (>= F)
extern "C" hipError_t zoo_convlstm_step(const void* X, const void* Wt, int B, int D, int H, int W, int Cx, int Q,
                                        int R, int S, int ldw, int Nr, int F, int iact, int act, const void* gx,
                                        int gx_bf16, const float* cprev, float* h, float* c, float* acts, void* hb, int ldh,
                                        const float* dout, const float* cc, float* dc, int dc_in, float* dg,
                                        void* dgb, int ldg, int bwd, float* part, hipStream_t st) {
  CLArgs a{(const bf16_t*)X, (const bf16_t*)Wt, B, D, H, W, Cx, Q, R, S, ldw, Nr, B * D * H * W, F, iact, act,
           gx_bf16 ? nullptr : (const float*)gx, gx_bf16 ? (const bf16_t*)gx : nullptr, cprev, h, c, acts, (bf16_t*)hb, ldh, dout, cc, dc, dc_in, dg, (bf16_t*)dgb, ldg};
  a.c_beg = 0;
  a.c_cnt = 0;
  a.part = part;   // [M][16 ceil(Nr / 16)] fp32 scratch of the K-split path (null: not taken)
  if (a.M <= 0) return hipSuccess;
  if (a.M >= (1 << 30) / 8) return hipErrorInvalidValue;   // 32-bit pixel indices
  const int ni = (Nr + 15) / 16;
  switch (ni) {
#define CL_CASE(n) \
  case n: return cl_launch<n>(a, bwd, st);
    CL_CASE(1) CL_CASE(2) CL_CASE(3) CL_CASE(4) CL_CASE(5) CL_CASE(6) CL_CASE(7) CL_CASE(8)
    CL_CASE(9) CL_CASE(10) CL_CASE(11) CL_CASE(12) CL_CASE(13) CL_CASE(14) CL_CASE(15) CL_CASE(16)
#undef CL_CASE
    default: return hipErrorInvalidValue;
  }
}

extern "C" void zoo_convlstm_pers_set(int on) {
  g_cl_pers = on & 3;
  g_cl_fks = (on >> 2) & 1;   // 4 | mode: forward K-split at every size (A/B)
  g_cl_cp = ((on >> 3) & 1) ? 0 : 1;   // 8 | mode: gate-interleaved epilogue on the row-group forward
}
