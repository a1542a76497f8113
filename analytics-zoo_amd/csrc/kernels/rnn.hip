// Persistent recurrent-cell kernels (SimpleRNN / LSTM / GRU) for gfx950 (HK11).
//
// Reference: the Keras-1 recurrent layers (Zs/pipeline/api/keras/layers/
// LSTM.scala:71-80, GRU.scala, SimpleRNN.scala) unroll the time loop in
// InternalRecurrent.scala:80-140 and run one small GEMM plus a handful of
// elementwise modules per step. Here the input projection of ALL steps is one
// MFMA GEMM on the host side (zoo.ops.linear), and the whole time loop of the
// recurrence runs inside ONE kernel launch:
//
//   * one workgroup owns 16 batch rows (the M=16 of v_mfma_f32_16x16x32_bf16)
//     for every time step, so there is no inter-workgroup synchronisation;
//   * wave w owns hidden-column blocks jb = w*NB .. w*NB+NB-1 and computes the
//     G gate tiles of those columns, so the accumulator lanes of the i/f/c/o
//     (or z/r/h) tiles line up and the cell update is lane-local;
//   * the recurrent weight U lives in VGPRs for the whole sequence when it fits
//     (<= 128 registers per lane), otherwise its fragments stream from L2 every
//     step (U is shared by all workgroups, so it stays L2-resident);
//   * h_{t-1} is exchanged through a double-buffered bf16 tile in LDS (one
//     barrier per step; GRU needs a second one for r*h), c and h stay fp32 in
//     registers, and the xw loads of a step do not depend on the MFMA chain.
//
// Backward (BPTT) is the mirror image: per step the lane-local gate gradients
// are formed, written out (they are d(xw); the host turns them into dW, db, dx
// and dU with plain GEMMs), staged as bf16 in LDS, and dh_{t-1} = dgates . U is
// one more register-resident MFMA chain against U^T.
//
// Layouts (all row-major, fp32 unless noted):
//   xw    [B, T, G*H]   pre-activation input projections (bias included)
//   u     [G*H, H] bf16 recurrent weight, gate-major rows (Keras order
//                       LSTM i,f,c,o; GRU z,r,h)   -- U^T [H, G*H] for backward
//   hseq  [B, T, H]     outputs, in processing order
//   cseq  [B, T, H]     LSTM cell states / GRU_RA candidate recurrent pre-activations (saved)
//   gates [B, T, G*H]   activated gates (saved for backward)
//   dgate [B, T, G*H]   d(pre-activation) = d(xw)
#include "common.h"
#include "geom.h"

namespace zoo {

ZOO_DEV float ract(float x, int a) {
  switch (a) {
    case RA_TANH: return tanhf(x);
    case RA_SIGMOID: return 1.f / (1.f + __expf(-x));
    case RA_HSIG: return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f);
    case RA_RELU: return fmaxf(x, 0.f);
    default: return x;
  }
}

// derivative written in terms of the activation's OUTPUT y
ZOO_DEV float ractd(float y, int a) {
  switch (a) {
    case RA_TANH: return 1.f - y * y;
    case RA_SIGMOID: return y * (1.f - y);
    case RA_HSIG: return (y > 0.f && y < 1.f) ? 0.2f : 0.f;
    case RA_RELU: return y > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

template <int CELL, int H>
struct RnnCfg {
  static constexpr int G = CELL == CELL_LSTM ? 4 : ((CELL == CELL_GRU || CELL == CELL_GRU_RA) ? 3 : 1);
  static constexpr int GH = G * H;
  static constexpr int NBLK = H / 16;             // 16-wide hidden column blocks
  static constexpr int NB = (NBLK + 7) / 8;       // blocks per wave (<= 8 waves)
  static constexpr int NW = NBLK / NB;            // waves per workgroup
  static constexpr int KC = H / 32;               // K chunks over the hidden dim
  static constexpr int LDH = H + 8;               // LDS row stride (bf16): rows 16 B apart in the banks
  // U fragments held in VGPRs when they cost <= 128 registers per lane
  static constexpr bool RES = NB * G * KC * 4 <= 128;
  static_assert(H % 32 == 0 && NBLK % NB == 0 && NW >= 1 && NW <= 8, "unsupported hidden size");
};

ZOO_DEV bf16x8 ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int CELL, int H>
__global__ __launch_bounds__((RnnCfg<CELL, H>::NW * 64)) void rnn_fwd_kernel(RnnArgs a) {
  using C = RnnCfg<CELL, H>;
  constexpr int G = C::G, GH = C::GH, NB = C::NB, KC = C::KC, LDH = C::LDH;
  constexpr int G1 = CELL == CELL_GRU ? 2 : G;  // GRU: the candidate uses (r*h) . U_h in phase 2
  __shared__ __attribute__((aligned(16))) bf16_t hs[2][16 * LDH];
  __shared__ __attribute__((aligned(16))) bf16_t rs[CELL == CELL_GRU ? 16 * LDH : 8];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int b0 = blockIdx.x * 16;
  const int B = a.B, T = a.T;
  const bf16_t* u = static_cast<const bf16_t*>(a.u);

  // U fragment (gate g, hidden block jb, k chunk kc): B-operand column = gate row n
  auto ufrag = [&](int g, int jb, int kc) -> bf16x8 {
    return ld8(u + (size_t)(g * H + jb * 16 + fr) * H + kc * 32 + fq * 8);
  };
  bf16x8 ures[C::RES ? NB : 1][C::RES ? G : 1][C::RES ? KC : 1];
  if constexpr (C::RES) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) ures[nb][g][kc] = ufrag(g, w * NB + nb, kc);
  }

  // initial state: bf16 tile in LDS for the MFMA, fp32 copies in registers
  for (int idx = tid; idx < 16 * H; idx += C::NW * 64) {
    const int r = idx / H, j = idx - r * H, b = b0 + r;
    const float v = (a.h0 != nullptr && b < B) ? a.h0[(size_t)b * H + j] : 0.f;
    hs[0][r * LDH + j] = f2bf(v);
  }
  float hreg[NB][4], creg[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = b0 + fq * 4 + i, j = (w * NB + nb) * 16 + fr;
      const bool ok = b < B;
      hreg[nb][i] = (a.h0 != nullptr && ok) ? a.h0[(size_t)b * H + j] : 0.f;
      creg[nb][i] = (CELL == CELL_LSTM && a.c0 != nullptr && ok) ? a.c0[(size_t)b * H + j] : 0.f;
    }

  for (int t = 0; t < T; ++t) {
    const int cur = t & 1;
    __syncthreads();
    bf16x8 af[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) af[kc] = ld8(&hs[cur][fr * LDH + kc * 32 + fq * 8]);

#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int jb = w * NB + nb, j = jb * 16 + fr;
      float xv[G1][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = b0 + fq * 4 + i;
        const bool ok = b < B;
        const float* xr = a.xw + ((size_t)(ok ? b : 0) * T + t) * GH + j;
#pragma unroll
        for (int g = 0; g < G1; ++g) xv[g][i] = ok ? xr[g * H] : 0.f;
      }
      f32x4 acc[G1];
#pragma unroll
      for (int g = 0; g < G1; ++g) {
        acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          bf16x8 bu;
          if constexpr (C::RES) bu = ures[nb][g][kc]; else bu = ufrag(g, jb, kc);
          acc[g] = mfma16(af[kc], bu, acc[g]);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = fq * 4 + i, b = b0 + row;
        const bool ok = b < B;
        const size_t bt = (size_t)b * T + t;
        if constexpr (CELL == CELL_RNN) {
          const float hn = ract(xv[0][i] + acc[0][i], a.act);
          hreg[nb][i] = hn;
          hs[cur ^ 1][row * LDH + j] = f2bf(hn);
        } else if constexpr (CELL == CELL_LSTM) {
          const float gi = ract(xv[0][i] + acc[0][i], a.iact);
          const float gf = ract(xv[1][i] + acc[1][i], a.iact);
          const float gc = ract(xv[2][i] + acc[2][i], a.act);
          const float go = ract(xv[3][i] + acc[3][i], a.iact);
          const float c = gf * creg[nb][i] + gi * gc;
          const float hn = go * ract(c, a.act);
          creg[nb][i] = c;
          hreg[nb][i] = hn;
          hs[cur ^ 1][row * LDH + j] = f2bf(hn);
          if (ok && a.gates != nullptr) {
            float* gp = a.gates + bt * GH + j;
            gp[0] = gi; gp[H] = gf; gp[2 * H] = gc; gp[3 * H] = go;
          }
          if (ok && a.cseq != nullptr) a.cseq[bt * H + j] = c;
        } else if constexpr (CELL == CELL_GRU_RA) {
          // reset-after GRU: one GEMM for z, r and the candidate's U_n h; the candidate's
          // recurrent pre-activation an = U_n h + b_hn is saved (cseq) for the backward
          const float gz = ract(xv[0][i] + acc[0][i], a.iact);
          const float gr = ract(xv[1][i] + acc[1][i], a.iact);
          const float an = acc[2][i] + (a.bhn != nullptr ? a.bhn[j] : 0.f);
          const float gn = ract(xv[2][i] + gr * an, a.act);
          const float hn = gz * hreg[nb][i] + (1.f - gz) * gn;
          hreg[nb][i] = hn;
          hs[cur ^ 1][row * LDH + j] = f2bf(hn);
          if (ok && a.gates != nullptr) {
            float* gp = a.gates + bt * GH + j;
            gp[0] = gz; gp[H] = gr; gp[2 * H] = gn;
          }
          if (ok && a.cseq != nullptr) a.cseq[bt * H + j] = an;
        } else {  // GRU phase 1: z, r; stage r*h_{t-1} for the candidate GEMM
          const float gz = ract(xv[0][i] + acc[0][i], a.iact);
          const float gr = ract(xv[1][i] + acc[1][i], a.iact);
          creg[nb][i] = gz;  // z parked until the candidate is known
          rs[row * LDH + j] = f2bf(gr * hreg[nb][i]);
          if (ok && a.gates != nullptr) {
            float* gp = a.gates + bt * GH + j;
            gp[0] = gz; gp[H] = gr;
          }
        }
      }
    }

    if constexpr (CELL == CELL_GRU) {
      __syncthreads();  // every column of r*h is needed by every wave
      bf16x8 rf[KC];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) rf[kc] = ld8(&rs[fr * LDH + kc * 32 + fq * 8]);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int jb = w * NB + nb, j = jb * 16 + fr;
        float xh[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = b0 + fq * 4 + i;
          xh[i] = b < B ? a.xw[((size_t)b * T + t) * GH + 2 * H + j] : 0.f;
        }
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          bf16x8 bu;
          if constexpr (C::RES) bu = ures[nb][2][kc]; else bu = ufrag(2, jb, kc);
          acc = mfma16(rf[kc], bu, acc);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = fq * 4 + i, b = b0 + row;
          const float hh = ract(xh[i] + acc[i], a.act);
          const float z = creg[nb][i];
          const float hn = z * hreg[nb][i] + (1.f - z) * hh;
          hreg[nb][i] = hn;
          hs[cur ^ 1][row * LDH + j] = f2bf(hn);
          if (b < B && a.gates != nullptr) a.gates[((size_t)b * T + t) * GH + 2 * H + j] = hh;
        }
      }
    }

    // outputs of step t
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int j = (w * NB + nb) * 16 + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = b0 + fq * 4 + i;
        if (b < B) a.hseq[((size_t)b * T + t) * H + j] = hreg[nb][i];
      }
    }
  }
  if constexpr (CELL == CELL_LSTM) {
    if (a.cT != nullptr) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int j = (w * NB + nb) * 16 + fr;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = b0 + fq * 4 + i;
          if (b < B) a.cT[(size_t)b * H + j] = creg[nb][i];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// backward (BPTT)
// ---------------------------------------------------------------------------
template <int CELL, int H>
__global__ __launch_bounds__((RnnCfg<CELL, H>::NW * 64)) void rnn_bwd_kernel(RnnArgs a) {
  using C = RnnCfg<CELL, H>;
  constexpr int GH = C::GH, NB = C::NB, KC = C::KC, LDH = C::LDH;
  // K of the dh_{t-1} GEMM: every gate column (RNN / LSTM) or z|r (GRU; the
  // candidate's path goes through d(r*h) in a separate GEMM first)
  constexpr int KA = CELL == CELL_GRU ? 2 * H : GH;
  constexpr int KCA = KA / 32;
  constexpr int LDA = KA + 8;
  __shared__ __attribute__((aligned(16))) bf16_t ds[2][16 * LDA];
  __shared__ __attribute__((aligned(16))) bf16_t dsh[CELL == CELL_GRU ? 16 * LDH : 8];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int b0 = blockIdx.x * 16;
  const int B = a.B, T = a.T;
  const bf16_t* ut = static_cast<const bf16_t*>(a.u);

  // U^T fragment: B-operand column = hidden unit j, k = gate rows n0 + fq*8 .. +8
  auto utfrag = [&](int jb, int n0) -> bf16x8 {
    return ld8(ut + (size_t)(jb * 16 + fr) * GH + n0 + fq * 8);
  };
  constexpr bool RES = C::RES;
  constexpr bool GRU = CELL == CELL_GRU;
  bf16x8 ures[RES ? NB : 1][RES ? KCA : 1];
  bf16x8 uhres[(RES && GRU) ? NB : 1][(RES && GRU) ? KC : 1];
  if constexpr (RES) {
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
#pragma unroll
      for (int kc = 0; kc < KCA; ++kc) ures[nb][kc] = utfrag(w * NB + nb, kc * 32);
      if constexpr (GRU) {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) uhres[nb][kc] = utfrag(w * NB + nb, 2 * H + kc * 32);
      }
    }
  }

  float dhrec[NB][4], dcreg[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = b0 + fq * 4 + i, j = (w * NB + nb) * 16 + fr;
      dhrec[nb][i] = 0.f;
      dcreg[nb][i] = (CELL == CELL_LSTM && a.dcT != nullptr && b < B) ? a.dcT[(size_t)b * H + j] : 0.f;
    }

  for (int t = T - 1; t >= 0; --t) {
    const int cur = t & 1;
    float dhd[NB][4];  // GRU: direct dh_{t-1} terms (dh*z, then + d(rh)*r)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int j = (w * NB + nb) * 16 + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = fq * 4 + i, b = b0 + row;
        const bool ok = b < B;
        const size_t bt = (size_t)(ok ? b : 0) * T + t;
        float dh = dhrec[nb][i];
        if (ok && a.dhseq != nullptr) dh += a.dhseq[bt * H + j];
        if (!ok) dh = 0.f;
        if constexpr (CELL == CELL_RNN) {
          const float da = dh * ractd(a.hseq[bt * H + j], a.act);
          if (ok) a.dgates[bt * GH + j] = da;
          ds[cur][row * LDA + j] = f2bf(da);
        } else if constexpr (CELL == CELL_LSTM) {
          const float* gp = a.gates + bt * GH + j;
          const float gi = gp[0], gf = gp[H], gc = gp[2 * H], go = gp[3 * H];
          const float ct = a.cseq[bt * H + j];
          float cp = 0.f;
          if (t > 0) cp = a.cseq[(bt - 1) * H + j];
          else if (a.c0 != nullptr && ok) cp = a.c0[(size_t)b * H + j];
          const float tc = ract(ct, a.act);
          const float dgo = dh * tc * ractd(go, a.iact);
          const float dc = dcreg[nb][i] + dh * go * ractd(tc, a.act);
          const float dgv[4] = {ok ? dc * gc * ractd(gi, a.iact) : 0.f, ok ? dc * cp * ractd(gf, a.iact) : 0.f,
                                ok ? dc * gi * ractd(gc, a.act) : 0.f, ok ? dgo : 0.f};
          dcreg[nb][i] = ok ? dc * gf : 0.f;
          if (ok) {
            float* dp = a.dgates + bt * GH + j;
            dp[0] = dgv[0]; dp[H] = dgv[1]; dp[2 * H] = dgv[2]; dp[3 * H] = dgv[3];
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) ds[cur][row * LDA + g * H + j] = f2bf(dgv[g]);
        } else if constexpr (CELL == CELL_GRU_RA) {
          // h = z h_p + (1 - z) n,  n = act(xn + r an),  an = U_n h_p + b_hn
          const float* gp = a.gates + bt * GH + j;
          const float z = gp[0], r = gp[H], n = gp[2 * H];
          const float an = a.cseq[bt * H + j];
          float hp = 0.f;
          if (t > 0) hp = a.hseq[(bt - 1) * H + j];
          else if (a.h0 != nullptr && ok) hp = a.h0[(size_t)b * H + j];
          const float dn = ok ? dh * (1.f - z) * ractd(n, a.act) : 0.f;
          const float dz = ok ? dh * (hp - n) * ractd(z, a.iact) : 0.f;
          const float dr = ok ? dn * an * ractd(r, a.iact) : 0.f;
          const float dan = dn * r;
          dhd[nb][i] = ok ? dh * z : 0.f;
          if (ok) {
            float* dp = a.dgates + bt * GH + j;
            dp[0] = dz; dp[H] = dr; dp[2 * H] = dn;
            a.dgn[bt * H + j] = dan;
          }
          ds[cur][row * LDA + j] = f2bf(dz);
          ds[cur][row * LDA + H + j] = f2bf(dr);
          ds[cur][row * LDA + 2 * H + j] = f2bf(dan);
        } else {  // GRU phase 1: dz and the candidate's pre-activation gradient
          const float* gp = a.gates + bt * GH + j;
          const float z = gp[0], hh = gp[2 * H];
          float hp = 0.f;
          if (t > 0) hp = a.hseq[(bt - 1) * H + j];
          else if (a.h0 != nullptr && ok) hp = a.h0[(size_t)b * H + j];
          const float dz = ok ? dh * (hp - hh) * ractd(z, a.iact) : 0.f;
          const float dhh = ok ? dh * (1.f - z) * ractd(hh, a.act) : 0.f;
          dhd[nb][i] = dh * z;
          if (ok) {
            a.dgates[bt * GH + j] = dz;
            a.dgates[bt * GH + 2 * H + j] = dhh;
          }
          dsh[row * LDH + j] = f2bf(dhh);
          ds[cur][row * LDA + j] = f2bf(dz);
        }
      }
    }
    __syncthreads();

    if constexpr (GRU) {
      // d(r*h) = dhh . U_h  -> dr and the r-path of dh_{t-1}
      bf16x8 af[KC];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) af[kc] = ld8(&dsh[fr * LDH + kc * 32 + fq * 8]);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        const int jb = w * NB + nb, j = jb * 16 + fr;
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          bf16x8 bu;
          if constexpr (RES) bu = uhres[nb][kc]; else bu = utfrag(jb, 2 * H + kc * 32);
          acc = mfma16(af[kc], bu, acc);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = fq * 4 + i, b = b0 + row;
          const bool ok = b < B;
          const size_t bt = (size_t)(ok ? b : 0) * T + t;
          const float r = a.gates[bt * GH + H + j];
          float hp = 0.f;
          if (t > 0) hp = a.hseq[(bt - 1) * H + j];
          else if (a.h0 != nullptr && ok) hp = a.h0[(size_t)b * H + j];
          const float dr = ok ? acc[i] * hp * ractd(r, a.iact) : 0.f;
          dhd[nb][i] += ok ? acc[i] * r : 0.f;
          if (ok) a.dgates[bt * GH + H + j] = dr;
          ds[cur][row * LDA + H + j] = f2bf(dr);
        }
      }
      __syncthreads();
    }

    // dh_{t-1} = dgates_t . U   (GRU: [dz | dr] . [U_z ; U_r] + the direct terms)
    bf16x8 af[KCA];
#pragma unroll
    for (int kc = 0; kc < KCA; ++kc) af[kc] = ld8(&ds[cur][fr * LDA + kc * 32 + fq * 8]);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int jb = w * NB + nb;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KCA; ++kc) {
        bf16x8 bu;
        if constexpr (RES) bu = ures[nb][kc]; else bu = utfrag(jb, kc * 32);
        acc = mfma16(af[kc], bu, acc);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = acc[i];
        if constexpr (GRU || CELL == CELL_GRU_RA) v += dhd[nb][i];
        dhrec[nb][i] = v;
      }
    }
  }

#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int j = (w * NB + nb) * 16 + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = b0 + fq * 4 + i;
      if (b < B) {
        if (a.dh0 != nullptr) a.dh0[(size_t)b * H + j] = dhrec[nb][i];
        if (CELL == CELL_LSTM && a.dc0 != nullptr) a.dc0[(size_t)b * H + j] = dcreg[nb][i];
      }
    }
  }
}

template <int CELL, int H>
hipError_t launch_rnn(const RnnArgs& a, bool bwd, hipStream_t st) {
  using C = RnnCfg<CELL, H>;
  const dim3 grid((a.B + 15) / 16), block(C::NW * 64);
  if (bwd) hipLaunchKernelGGL((rnn_bwd_kernel<CELL, H>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((rnn_fwd_kernel<CELL, H>), grid, block, 0, st, a);
  return hipGetLastError();
}

template <int CELL>
hipError_t dispatch_h(const RnnArgs& a, int H, bool bwd, hipStream_t st) {
  switch (H) {
    case 32: return launch_rnn<CELL, 32>(a, bwd, st);
    case 64: return launch_rnn<CELL, 64>(a, bwd, st);
    case 128: return launch_rnn<CELL, 128>(a, bwd, st);
    case 256: return launch_rnn<CELL, 256>(a, bwd, st);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace zoo

extern "C" hipError_t zoo_rnn(const zoo::RnnArgs* a, int cell, int H, int bwd, hipStream_t st) {
  if (a->B <= 0 || a->T <= 0) return hipSuccess;
  switch (cell) {
    case zoo::CELL_RNN: return zoo::dispatch_h<zoo::CELL_RNN>(*a, H, bwd != 0, st);
    case zoo::CELL_LSTM: return zoo::dispatch_h<zoo::CELL_LSTM>(*a, H, bwd != 0, st);
    case zoo::CELL_GRU: return zoo::dispatch_h<zoo::CELL_GRU>(*a, H, bwd != 0, st);
    case zoo::CELL_GRU_RA: return zoo::dispatch_h<zoo::CELL_GRU_RA>(*a, H, bwd != 0, st);
    default: return hipErrorInvalidValue;
  }
}
