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
  float* dg;            // [M][F][4]
  bf16_t* dgb;          // [M][ldg] bf16 gate gradients
  int ldg;
};

constexpr int CL_WAVES = 4;   // 4 waves x 16 pixels per workgroup
constexpr int CL_PF = 4;      // activation chunks in flight per wave

// reduction chunks of 32, padded to whole prefetch groups (the padding is zero in LDS and never loaded)
ZOO_DEV int cl_kcp(int KD) { return ((KD + 31) / 32 + CL_PF - 1) / CL_PF * CL_PF; }
ZOO_DEV int cl_kdp(int KD) { return cl_kcp(KD) * 32 + 8; }   // LDS row pitch (+16 B: conflict-free)

// acc[j][i] (rows 16 i .. 16 i + 15, this lane's pixel m0 + 16 j) = W[rows] . X_patch(m0 + 16 j)
// LDSW: the workgroup's weights staged once in LDS (rows padded to cl_kdp); else read from L2.
// MJ pixel blocks per wave share every weight fragment: at large M (a 32^3 ConvLSTM3D volume,
// 262k pixels per step) the kernel is bound by the L2 reads of weights the wave re-reads per
// 32-deep chunk (221 KiB per 16 pixels); MJ = 2 halves them per MFMA
template <int NI, int MJ, bool LDSW>
ZOO_DEV void cl_gemm(const CLArgs& a, int m0, f32x4 (&acc)[MJ][NI], int lane, const bf16_t* wl) {
#pragma unroll
  for (int j = 0; j < MJ; ++j)
#pragma unroll
    for (int i = 0; i < NI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (!a.X) return;
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
  const int KD = a.Q * a.R * a.S * a.Cx, KC = (KD + 31) / 32, kdp = cl_kdp(KD);
  const int pq = a.Q / 2, ph = a.R / 2, pw = a.S / 2;
  const int kq = 8 * (lane >> 4), nr = lane & 15;
  const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
  const bf16_t* X = a.X;
  const int Cx = a.Cx, RS = a.R * a.S, S = a.S, D = a.D, H = a.H, Wd = a.Wd;
  // branch-free: every lane loads from an in-bounds address (clamped) and zeroes the value when
  // the tap is outside the image / reduction -- a predicated load in a divergent branch made the
  // compiler wait for ALL outstanding loads (vmcnt(0)) before each chunk, serialising the prefetch
  auto load_act = [=](int j, int c) -> uint4 {
    int k = c * 32 + kq;
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
  uint4 pre[MJ][CL_PF];
#pragma unroll
  for (int u = 0; u < CL_PF; ++u)
#pragma unroll
    for (int j = 0; j < MJ; ++j) pre[j][u] = load_act(j, u);
  // whole prefetch groups (chunks past KC read zeros): a straight-line body, so the in-order
  // vmcnt waits only for the chunk being consumed
  const int KCp = cl_kcp(KD);
  for (int c0 = 0; c0 < KCp; c0 += CL_PF) {
#pragma unroll
    for (int u = 0; u < CL_PF; ++u) {
      const int c = c0 + u;
      const int k = c * 32 + kq;
      uint4 wv[NI];   // every row block's weight fragment first (one LDS wait), then the MFMAs
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int n = 16 * i + nr;
        if (LDSW) {
          wv[i] = *reinterpret_cast<const uint4*>(wl + (size_t)n * kdp + k);   // zero padded rows / k
        } else {
          const bool ok = n < a.Nr && k < KD;
          const uint4 t = *reinterpret_cast<const uint4*>(a.Wt + (size_t)(ok ? n : 0) * a.ldw + (ok ? k : 0));
          wv[i] = ok ? t : z4;
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the fragment reads batched ahead of the MFMAs
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const bf16x8 bv = __builtin_bit_cast(bf16x8, pre[j][u]);
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[j][i] = mfma16(__builtin_bit_cast(bf16x8, wv[i]), bv, acc[j][i]);
        // refill this slot after its use: the in-order vmcnt then waits only for this chunk's load
        pre[j][u] = load_act(j, c + CL_PF);
      }
    }
  }
}

// stage rows [0, 16 NI) of the weights (zero beyond Nr / KD) into LDS, pitch cl_kdp(KD)
template <int NI>
ZOO_DEV void cl_stage(const CLArgs& a, bf16_t* wl) {
  if (!a.X) return;
  const int KD = a.Q * a.R * a.S * a.Cx, kdp = cl_kdp(KD);
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
      v[u] = e < total && n < Nr && k < KD ? *reinterpret_cast<const uint4*>(Wt + (size_t)n * ldw + k)
                                           : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int e = e0 + u * blockDim.x;
      const int n = e / per_row, k = (e - n * per_row) * 8;
      if (e < total) *reinterpret_cast<uint4*>(wl + (size_t)n * kdp + k) = v[u];
    }
  }
  __syncthreads();
}

// The epilogue operands do not depend on the GEMM: they are loaded BEFORE it (every lane, clamped
// addresses, no branch) so their latency hides behind the reduction; loading them between the
// stores of the epilogue made each channel wait for its own round trip (the stores may alias the
// loads): 11 us of a 23 us step.
template <int NI, int MJ, bool LDSW>
__global__ __launch_bounds__(64 * CL_WAVES) void convlstm_fwd_kernel(CLArgs a) {
  extern __shared__ __attribute__((aligned(16))) char cl_smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(cl_smem);
  const int lane = threadIdx.x & 63;
  const int m0 = (blockIdx.x * CL_WAVES + (threadIdx.x >> 6)) * 16 * MJ + (lane & 15);
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
      const int j = 4 * i + (lane >> 4);   // rows 16 i + 4 (lane >> 4) + q = gate q of channel j
      const size_t e = (size_t)mc * F + (j < F ? j : F - 1);
      g4[jb][i] = *reinterpret_cast<const float4*>(gx + 4 * e);
      cp[jb][i] = cprev ? cprev[e] : 0.f;
    }
  }
  if (LDSW) cl_stage<NI>(a, wl);
  f32x4 acc[MJ][NI];
  cl_gemm<NI, MJ, LDSW>(a, m0, acc, lane, wl);
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int j = 4 * i + (lane >> 4);
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

// backward: operands of every (row block, channel) up front while NI <= 4 (the data-gradient rows
// are the hidden channels: <= 64); wider row counts load them per row block
template <int NI, int MJ, bool LDSW>
__global__ __launch_bounds__(64 * CL_WAVES) void convlstm_bwd_kernel(CLArgs a) {
  extern __shared__ __attribute__((aligned(16))) char cl_smem[];
  bf16_t* wl = reinterpret_cast<bf16_t*>(cl_smem);
  constexpr bool PRE = NI * MJ <= 4;
  constexpr int NP = PRE ? NI : 1, MP = PRE ? MJ : 1;
  const int lane = threadIdx.x & 63;
  const int m0 = (blockIdx.x * CL_WAVES + (threadIdx.x >> 6)) * 16 * MJ + (lane & 15);
  const int F = a.F;
  const float* __restrict__ acts = a.acts;
  const float* __restrict__ cc = a.cc;
  const float* __restrict__ dout = a.dout;
  const float* __restrict__ cprev = a.cprev;
  const float* __restrict__ dcin = a.dc_in ? a.dc : nullptr;
  float4 av[MP][NP][4];
  float cv[MP][NP][4], ov[MP][NP][4], dv[MP][NP][4], pv[MP][NP][4];
  auto load_ops = [&](int jb, int i, int sj, int slot) {
    const int m = m0 + 16 * jb;
    const int mc = m < a.M ? m : a.M - 1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = 16 * i + 4 * (lane >> 4) + q;   // row = hidden channel of the data gradient
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
  if (LDSW) cl_stage<NI>(a, wl);
  f32x4 acc[MJ][NI];
  cl_gemm<NI, MJ, LDSW>(a, m0, acc, lane, wl);
#pragma unroll
  for (int jb = 0; jb < MJ; ++jb) {
    const int m = m0 + 16 * jb;
    if (m >= a.M) continue;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int slot = PRE ? i : 0, sj = PRE ? jb : 0;
      if constexpr (!PRE) load_ops(jb, i, 0, 0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = 16 * i + 4 * (lane >> 4) + q;
        if (j >= F) continue;
        const size_t e = (size_t)m * F + j;
        const float ig = av[sj][slot][q].x, fg = av[sj][slot][q].y, cg = av[sj][slot][q].z, og = av[sj][slot][q].w;
        const float tc = lstm_act(cv[sj][slot][q], a.act);
        const float dh = acc[jb][i][q] + ov[sj][slot][q];
        const float dcv = dh * og * lstm_dact(tc, a.act) + dv[sj][slot][q];
        const float cpv = pv[sj][slot][q];
        const float d0 = dcv * cg * lstm_dact(ig, a.iact), d1 = dcv * cpv * lstm_dact(fg, a.iact);
        const float d2 = dcv * ig * lstm_dact(cg, a.act), d3 = dh * tc * lstm_dact(og, a.iact);
        *reinterpret_cast<float4*>(a.dg + 4 * e) = make_float4(d0, d1, d2, d3);
        *reinterpret_cast<uint2*>(a.dgb + (size_t)m * a.ldg + 4 * j) =
            make_uint2((uint32_t)f2bf(d0) | ((uint32_t)f2bf(d1) << 16), (uint32_t)f2bf(d2) | ((uint32_t)f2bf(d3) << 16));
        a.dc[e] = dcv * fg;   // this lane read dc_{t+1}[e] before: in place
      }
    }
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
template <int NI, bool BWD>
static hipError_t cl_launch_dir(const CLArgs& a, hipStream_t st) {
  const int KD = a.Q * a.R * a.S * a.Cx;
  const size_t smem = (size_t)16 * NI * ((((KD + 31) / 32 + CL_PF - 1) / CL_PF * CL_PF) * 32 + 8) * 2;
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
                                        int R, int S, int ldw, int Nr, int F, int iact, int act, const float* gx,
                                        const float* cprev, float* h, float* c, float* acts, void* hb, int ldh,
                                        const float* dout, const float* cc, float* dc, int dc_in, float* dg,
                                        void* dgb, int ldg, int bwd, hipStream_t st) {
  CLArgs a{(const bf16_t*)X, (const bf16_t*)Wt, B, D, H, W, Cx, Q, R, S, ldw, Nr, B * D * H * W, F, iact, act,
           gx, cprev, h, c, acts, (bf16_t*)hb, ldh, dout, cc, dc, dc_in, dg, (bf16_t*)dgb, ldg};
  if (a.M <= 0) return hipSuccess;
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
