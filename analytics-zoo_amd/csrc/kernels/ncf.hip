// Fused NeuralCF forward / backward (Zs/models/recommendation/NeuralCF.scala:45-138).
//
// The whole NCF network -- four embedding gathers, the MLP tower over concat(user, item), the
// matrix-factorisation product, concat, Dense(nc) + softmax -- is one kernel per direction, one
// thread per (user, item) record. Layer-by-layer the same step is ~130 launches of tiny GEMMs,
// gathers, concats, fills and copies (profiles/ncf_b65536_r2.md).
//
//   forward   gathers (bf16 tables, 8-byte row chunks) -> h1 = relu(W1 x0 + b1) -> h2 -> h3,
//             mf = mu * mi, logits = Wo [h3, mf] + bo, softmax -> probs [B, nc] fp32.
//             The MLP weights live in LDS (fp32, zero-padded to compile-time caps) and are read
//             as wave-uniform broadcasts; the layer being computed is in registers.
//   backward  recomputes the forward and parks every activation the backward needs in LDS as
//             bf16, transposed per wave ([feature][64 records], the layout the matrix cores
//             read), so nothing but the current layer stays in registers. From dprobs:
//             softmax-backward, then per layer: the wave's dZ is staged next to the parked
//             activations [A, 1] and dW = dZ^T [A, 1] (the ones column is the bias gradient) runs
//             on v_mfma_f32_16x16x32_bf16 with the 64 records as the reduction dimension; the
//             per-record dA = W^T dZ uses transposed weight copies (row dot products again) and
//             the ReLU masks read back from the parked activations. Embedding-row gradients are
//             scattered with fp32 atomics. Waves fold their dW into a block sum in LDS; blocks
//             write deterministic partials that one small kernel adds into the fp32 gradients.
//
// Caps (EC embedding width, H1C/H2C/H3C hidden widths, NCC classes) are template parameters;
// real widths are runtime and every padded weight is zero, so a padded unit is exactly 0 and
// receives exactly 0 gradient. Embedding widths must be multiples of 4.
#include "common.h"
#include "ncf.h"

namespace zoo {

// packed gradient layout: W1 [h1, eu+ei], b1, W2 [h2, h1], b2, W3 [h3, h2], b3, Wo [nc, h3+em], bo
struct NcfOff {
  int w1, b1, w2, b2, w3, b3, wo, bo, n;
  ZOO_DEV __host__ NcfOff(int eu, int ei, int em, int h1, int h2, int h3, int nc) {
    w1 = 0;
    b1 = w1 + h1 * (eu + ei);
    w2 = b1 + h1;
    b2 = w2 + h2 * h1;
    w3 = b2 + h2;
    b3 = w3 + h3 * h2;
    wo = b3 + h3;
    bo = wo + nc * (h3 + em);
    n = bo + nc;
  }
};

constexpr int kNcfRows = 256;     // records per block (4 waves, one record per lane)
constexpr int kPitch = 72;        // bf16 per parked feature row: 64 records + 8 pad (bank spread)

template <int EC, int H1C, int H2C, int H3C, int NCC>
struct NcfCaps {
  static constexpr int X0 = 2 * EC, FIN = H3C + EC;
  static constexpr int W1 = H1C * X0, W2 = H2C * H1C, W3 = H3C * H2C, WO = NCC * FIN;
  // LDS weight image (floats): W1 b1 W2 b2 W3 b3 Wo bo, then (backward) W1^T W2^T W3^T Wo^T
  static constexpr int OW1 = 0, OB1 = W1, OW2 = OB1 + H1C, OB2 = OW2 + W2, OW3 = OB2 + H2C, OB3 = OW3 + W3,
                       OWO = OB3 + H3C, OBO = OWO + WO, NWF = OBO + NCC;
  static constexpr int OT1 = NWF, OT2 = OT1 + W1, OT3 = OT2 + W2, OTO = OT3 + W3, NWT = OTO + WO;
  static constexpr int r16(int v) { return (v + 15) / 16 * 16; }
  static constexpr int mx(int a, int b) { return a > b ? a : b; }
  // parked rows per wave: [x0, 1], [h1, 1], [h2, 1], [h3, mf, 1], then the dZ staging rows
  static constexpr int RX0 = 0, RH1 = RX0 + r16(X0 + 1), RH2 = RH1 + r16(H1C + 1), RFIN = RH2 + r16(H2C + 1),
                       RM = RFIN + r16(FIN + 1), ROWS = RM + r16(mx(mx(H1C, H2C), mx(H3C, NCC)));
  static constexpr size_t lds_fwd() { return (size_t)NWF * 4 + 16 + 4ull * ROWS * kPitch * 2; }
  // weights, then nwg + 1 (trash) partial sums, then the 16-byte aligned per-wave rows
  static constexpr size_t lds_bwd(int nwg) {
    return (size_t)NWT * 4 + (size_t)(nwg + 1) * 4 + 16 + 4ull * ROWS * kPitch * 2;
  }
};

template <typename T>
ZOO_DEV void ncf_load4(const T* p, float* o);
template <>
ZOO_DEV void ncf_load4<float>(const float* p, float* o) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <>
ZOO_DEV void ncf_load4<bf16_t>(const bf16_t* p, float* o) {
  const uint2 v = *reinterpret_cast<const uint2*>(p);
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}

template <typename T, int EC>
ZOO_DEV void ncf_gather(const T* tab, int64_t id, int V, int e, float* o) {
  const bool ok = id >= 0 && id < V;
  const T* p = tab + (ok ? id : 0) * (int64_t)e;
#pragma unroll
  for (int k = 0; k < EC; k += 4) {
    if (ok && k < e) ncf_load4<T>(p + k, o + k);
    else { o[k] = 0.f; o[k + 1] = 0.f; o[k + 2] = 0.f; o[k + 3] = 0.f; }
  }
}

// park N values of this lane's record as rows [0, N) of `rows` (bf16, [feature][kPitch])
template <int N>
ZOO_DEV void ncf_park(bf16_t* rows, int lane, const float* v) {
#pragma unroll
  for (int f = 0; f < N; ++f) rows[f * kPitch + lane] = f2bf(v[f]);
  // the scheduler must not sink the parking stores (their sources would stay live)
  __builtin_amdgcn_sched_barrier(0);
}
// volatile: the compiler would otherwise forward the parked value from the register it was
// stored from, keeping every forward activation live through the backward (and spilling)
ZOO_DEV float ncf_parked(const bf16_t* rows, int f, int lane) {
  return bf2f(*reinterpret_cast<const volatile bf16_t*>(rows + f * kPitch + lane));
}

// one wave: dW[m][n] += sum over its 64 records of dz[m] * a[n] for m < MC, n < NC, plus the
// constant-1 row n = NC of `act` -> bias. Packed destinations: weight row m at woff + m * ld, bias
// at boff + m; activation n maps to weight column n (n < C0, kept if n < T0) or T0 + (n - C0)
// (n >= C0, kept if n - C0 < T1) -- two-segment concat inputs. Rows m >= mrows, dropped columns
// and padding land in the trash slot. `dzr` holds the staged dZ rows, `act` the parked [A, 1].
template <int MC, int NC, int C0>
ZOO_DEV void ncf_wgrad(const bf16_t* dzr, const bf16_t* act, float* sred, int trash, int lane, int mrows, int woff,
                       int ld, int boff, int T0, int T1) {
  constexpr int MP = (MC + 15) / 16 * 16, NP = (NC + 1 + 15) / 16 * 16;
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int nt = 0; nt < NP / 16; ++nt) {
    const int n = nt * 16 + fr;
    const bool seg0 = n < C0;
    const int col = seg0 ? n : T0 + (n - C0);
    const bool colok = seg0 ? (n < T0) : (n < NC && n - C0 < T1);
    const bool isb = n == NC;
#pragma unroll
    for (int mt = 0; mt < MP / 16; ++mt) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 av = *reinterpret_cast<const bf16x8*>(dzr + (mt * 16 + fr) * kPitch + ks * 32 + fq * 8);
        const bf16x8 bv = *reinterpret_cast<const bf16x8*>(act + (nt * 16 + fr) * kPitch + ks * 32 + fq * 8);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mt * 16 + fq * 4 + r;
        const bool rowok = m < MC && m < mrows;
        const int idx = isb ? boff + m : woff + m * ld + col;
        atomicAdd(sred + ((rowok && (isb || colok)) ? idx : trash), acc[r]);
      }
      __builtin_amdgcn_sched_barrier(0);   // one output tile's fragments in flight at a time
    }
  }
}

// dot of a weight row (LDS, fp32, broadcast) with a register vector
template <int N>
ZOO_DEV float ncf_dot(const float* w, const float* x) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < N; ++k) s = fmaf(w[k], x[k], s);
  return s;
}

template <int N>
ZOO_DEV void ncf_unpark(const bf16_t* rows, int lane, float* v) {
#pragma unroll
  for (int f = 0; f < N; ++f) v[f] = bf2f(rows[f * kPitch + lane]);
}

// U independent output rows per rolled iteration: U accumulator chains in flight (one wave per
// SIMD at the benchmark batch, so the FMA latency is hidden by ILP, not by other waves)
template <int N>
struct NcfU {
  static constexpr int v = N % 4 == 0 ? 4 : (N % 2 == 0 ? 2 : 1);
};

// out[j] = relu(B[j] + W[j] . x) for all NOUT (cap) rows -- padded rows are zero weights, so they
// park exactly 0 -- as bf16 rows, the output loop rolled
template <int NIN, int NOUT>
ZOO_DEV void ncf_layer(const float* W, const float* B, const float* x, bf16_t* out, int lane) {
  constexpr int U = NcfU<NOUT>::v;
#pragma unroll 1
  for (int j = 0; j < NOUT; j += U) {
    float s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = B[j + u];
#pragma unroll
    for (int k = 0; k < NIN; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u) s[u] = fmaf(W[(j + u) * NIN + k], x[k], s[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) out[(j + u) * kPitch + lane] = f2bf(fmaxf(s[u], 0.f));
  }
}
template <int NIN, int NOUT>
ZOO_DEV void ncf_layer_from(const float* W, const float* B, const bf16_t* in, bf16_t* out, int lane) {
  float x[NIN];
  ncf_unpark<NIN>(in, lane, x);
  ncf_layer<NIN, NOUT>(W, B, x, out, lane);
}

// dz[k] = relu'(act[k]) * (W^T d)[k] for all NOUT (cap) rows of WT (rows of NIN), parked into out
template <int NIN, int NOUT>
ZOO_DEV void ncf_back(const float* WT, const float* d, const bf16_t* act, bf16_t* out, int lane) {
  constexpr int U = NcfU<NOUT>::v;
#pragma unroll 1
  for (int k = 0; k < NOUT; k += U) {
    float t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = 0.f;
#pragma unroll
    for (int j = 0; j < NIN; ++j)
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = fmaf(WT[(k + u) * NIN + j], d[j], t[u]);
#pragma unroll
    for (int u = 0; u < U; ++u)
      out[(k + u) * kPitch + lane] = f2bf(bf2f(act[(k + u) * kPitch + lane]) > 0.f ? t[u] : 0.f);
  }
}

template <typename T, int EC, int H1C, int H2C, int H3C, int NCC, bool BWD>
__global__ __launch_bounds__(kNcfRows) void ncf_kernel(NcfArgs a) {
  using Cp = NcfCaps<EC, H1C, H2C, H3C, NCC>;
  constexpr int X0 = Cp::X0, FIN = Cp::FIN;
  extern __shared__ __align__(16) unsigned char ncf_smem[];
  float* sw = reinterpret_cast<float*>(ncf_smem);
  float* sred = sw + Cp::NWT;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int eu = a.eu, ei = a.ei, em = a.em, h1 = a.h1, h2 = a.h2, h3 = a.h3, nc = a.nc;

  // ---- weights -> zero-padded fp32 LDS image (rolled: an unrolled copy loop hoards its index
  // math in registers across the kernel)
#pragma unroll 1
  for (int i = tid; i < Cp::NWF; i += kNcfRows) {
    float v = 0.f;
    if (i < Cp::OB1) {
      const int j = i / X0, k = i % X0;
      if (j < h1) {
        if (k < EC) { if (k < eu) v = a.w1[j * (eu + ei) + k]; }
        else if (k - EC < ei) v = a.w1[j * (eu + ei) + eu + (k - EC)];
      }
    } else if (i < Cp::OW2) {
      const int j = i - Cp::OB1;
      if (j < h1 && a.b1) v = a.b1[j];
    } else if (i < Cp::OB2) {
      const int j = (i - Cp::OW2) / H1C, k = (i - Cp::OW2) % H1C;
      if (j < h2 && k < h1) v = a.w2[j * h1 + k];
    } else if (i < Cp::OW3) {
      const int j = i - Cp::OB2;
      if (j < h2 && a.b2) v = a.b2[j];
    } else if (i < Cp::OB3) {
      const int j = (i - Cp::OW3) / H2C, k = (i - Cp::OW3) % H2C;
      if (j < h3 && k < h2) v = a.w3[j * h2 + k];
    } else if (i < Cp::OWO) {
      const int j = i - Cp::OB3;
      if (j < h3 && a.b3) v = a.b3[j];
    } else if (i < Cp::OBO) {
      const int c = (i - Cp::OWO) / FIN, k = (i - Cp::OWO) % FIN;
      if (c < nc) {
        if (k < H3C) { if (k < h3) v = a.wo[c * (h3 + em) + k]; }
        else if (k - H3C < em) v = a.wo[c * (h3 + em) + h3 + (k - H3C)];
      }
    } else {
      const int c = i - Cp::OBO;
      if (c < nc && a.bo) v = a.bo[c];
    }
    sw[i] = v;
  }
  if constexpr (BWD) {
#pragma unroll 1
    for (int i = tid; i <= a.nwg; i += kNcfRows) sred[i] = 0.f;
    __syncthreads();
#pragma unroll 1
    for (int i = tid; i < Cp::NWT - Cp::NWF; i += kNcfRows) {
      int src;
      if (i < Cp::W1) {
        const int k = i / H1C, j = i % H1C;
        src = Cp::OW1 + j * X0 + k;
      } else if (i < Cp::W1 + Cp::W2) {
        const int t = i - Cp::W1, k = t / H2C, j = t % H2C;
        src = Cp::OW2 + j * H1C + k;
      } else if (i < Cp::W1 + Cp::W2 + Cp::W3) {
        const int t = i - Cp::W1 - Cp::W2, k = t / H3C, j = t % H3C;
        src = Cp::OW3 + j * H2C + k;
      } else {
        const int t = i - Cp::W1 - Cp::W2 - Cp::W3, k = t / NCC, c = t % NCC;
        src = Cp::OWO + c * FIN + k;
      }
      sw[Cp::NWF + i] = sw[src];
    }
  }
  __syncthreads();
  const float* W1 = sw + Cp::OW1;
  const float* B1 = sw + Cp::OB1;
  const float* W2 = sw + Cp::OW2;
  const float* B2 = sw + Cp::OB2;
  const float* W3 = sw + Cp::OW3;
  const float* B3 = sw + Cp::OB3;
  const float* WO = sw + Cp::OWO;
  const float* BO = sw + Cp::OBO;

  // per-wave parked rows: every layer's output goes straight to LDS (bf16, [feature][64 records])
  // and the next layer loads its input vector from there, so only one input vector and one
  // running dot product are ever in registers; the output loops stay rolled
  bf16_t* rows = reinterpret_cast<bf16_t*>(BWD ? sred + a.nwg + 1 : sw + Cp::NWF);
  rows = reinterpret_cast<bf16_t*>(reinterpret_cast<uintptr_t>(rows + 7) & ~(uintptr_t)15);
  rows += wv * Cp::ROWS * kPitch;
  bf16_t* const rx0 = rows + Cp::RX0 * kPitch;
  bf16_t* const rh1 = rows + Cp::RH1 * kPitch;
  bf16_t* const rh2 = rows + Cp::RH2 * kPitch;
  bf16_t* const rfin = rows + Cp::RFIN * kPitch;
  bf16_t* const rdz = rows + Cp::RM * kPitch;
  const bf16_t one = f2bf(1.f);

  // ---- forward (one record per thread)
  const int row = blockIdx.x * kNcfRows + tid;
  const bool valid = row < a.B;
  int64_t uid = -1, iid = -1;
  if (valid) {
    uid = a.ids[2 * (int64_t)row] - a.id_off;
    iid = a.ids[2 * (int64_t)row + 1] - a.id_off;
  }
  float mu[EC], mi[EC];
  if (em > 0) {
    ncf_gather<T, EC>(reinterpret_cast<const T*>(a.tmu), uid, a.Vu, em, mu);
    ncf_gather<T, EC>(reinterpret_cast<const T*>(a.tmi), iid, a.Vi, em, mi);
  } else {
#pragma unroll
    for (int k = 0; k < EC; ++k) { mu[k] = 0.f; mi[k] = 0.f; }
  }
  {
    float x0[X0];
    ncf_gather<T, EC>(reinterpret_cast<const T*>(a.tu), uid, a.Vu, eu, x0);
    ncf_gather<T, EC>(reinterpret_cast<const T*>(a.ti), iid, a.Vi, ei, x0 + EC);
    if constexpr (BWD) {
      ncf_park<X0>(rx0, lane, x0);
      rx0[X0 * kPitch + lane] = one;
    }
    ncf_layer<X0, H1C>(W1, B1, x0, rh1, lane);
  }
  rh1[H1C * kPitch + lane] = one;
  ncf_layer_from<H1C, H2C>(W2, B2, rh1, rh2, lane);
  rh2[H2C * kPitch + lane] = one;
  ncf_layer_from<H2C, H3C>(W3, B3, rh2, rfin, lane);
#pragma unroll
  for (int k = 0; k < EC; ++k) rfin[(H3C + k) * kPitch + lane] = f2bf(mu[k] * mi[k]);
  rfin[FIN * kPitch + lane] = one;
  float lg[NCC];
  {
    float fin[FIN];
    ncf_unpark<FIN>(rfin, lane, fin);
    float mxv = -3.4e38f;
#pragma unroll
    for (int c = 0; c < NCC; ++c) {
      lg[c] = BO[c] + ncf_dot<FIN>(WO + c * FIN, fin);
      if (c < nc) mxv = fmaxf(mxv, lg[c]);
    }
    float den = 0.f;
#pragma unroll
    for (int c = 0; c < NCC; ++c) {
      lg[c] = c < nc ? __expf(lg[c] - mxv) : 0.f;
      den += lg[c];
    }
    const float rden = 1.f / den;
#pragma unroll
    for (int c = 0; c < NCC; ++c) lg[c] *= rden;   // probabilities
  }
  if constexpr (!BWD) {
    if (valid)
#pragma unroll
      for (int c = 0; c < NCC; ++c)
        if (c < nc) a.probs[(int64_t)row * nc + c] = lg[c];
    return;
  } else {
    const float* W1T = sw + Cp::OT1;   // [X0][H1C]
    const float* W2T = sw + Cp::OT2;   // [H1C][H2C]
    const float* W3T = sw + Cp::OT3;   // [H2C][H3C]
    const float* WOT = sw + Cp::OTO;   // [FIN][NCC]
    const NcfOff off(eu, ei, em, h1, h2, h3, nc);
    const int trash = a.nwg;

    // ---- softmax backward: dl = p * (dp - sum(p dp)); padded / invalid records give 0
    float dl[NCC];
    float sdp = 0.f;
#pragma unroll
    for (int c = 0; c < NCC; ++c) {
      dl[c] = (valid && c < nc) ? a.dprobs[(int64_t)row * nc + c] : 0.f;
      sdp += lg[c] * dl[c];
    }
#pragma unroll
    for (int c = 0; c < NCC; ++c) dl[c] = lg[c] * (dl[c] - sdp);
    // a wave's LDS operations complete in order: its own parked rows are readable after its
    // stores, and a staging row is only rewritten after the reads that consume it
    ncf_park<NCC>(rdz, lane, dl);
    __builtin_amdgcn_wave_barrier();
    ncf_wgrad<NCC, FIN, H3C>(rdz, rfin, sred, trash, lane, nc, off.wo, h3 + em, off.bo, h3, em);

    // output layer -> dz3 = relu'(h3) * (Wo^T dl)[:h3]; then layers 3, 2 (dz staged in rdz)
    __builtin_amdgcn_wave_barrier();
    ncf_back<NCC, H3C>(WOT, dl, rfin, rdz, lane);
    __builtin_amdgcn_wave_barrier();
    ncf_wgrad<H3C, H2C, H2C>(rdz, rh2, sred, trash, lane, h3, off.w3, h2, off.b3, h2, 0);
    {
      float dz[H3C];
      ncf_unpark<H3C>(rdz, lane, dz);
      __builtin_amdgcn_wave_barrier();
      ncf_back<H3C, H2C>(W3T, dz, rh2, rdz, lane);
    }
    __builtin_amdgcn_wave_barrier();
    ncf_wgrad<H2C, H1C, H1C>(rdz, rh1, sred, trash, lane, h2, off.w2, h1, off.b2, h1, 0);
    {
      float dz[H2C];
      ncf_unpark<H2C>(rdz, lane, dz);
      __builtin_amdgcn_wave_barrier();
      ncf_back<H2C, H1C>(W2T, dz, rh1, rdz, lane);
    }
    __builtin_amdgcn_wave_barrier();
    ncf_wgrad<H1C, X0, EC>(rdz, rx0, sred, trash, lane, h1, off.w1, eu + ei, off.b1, eu, ei);
    // ---- embedding-row gradients, coalesced: the wave's 64 records x [user | item | mf-user |
    // mf-item] columns are staged fp32 in LDS (the parked rows are free now), then scattered one
    // record at a time with the lanes across its columns -- each atomic instruction then touches a
    // few contiguous row segments instead of 64 scattered rows
    constexpr int SP = 4 * EC + 1;
    static_assert(64 * SP * 4 <= Cp::ROWS * kPitch * 2, "staging fits the parked rows");
    float* stg = reinterpret_cast<float*>(rows);
    {
      float dz[H1C];
      ncf_unpark<H1C>(rdz, lane, dz);
      __builtin_amdgcn_wave_barrier();
      constexpr int U = NcfU<X0>::v;
#pragma unroll 1
      for (int k = 0; k < X0; k += U) {
        float t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = 0.f;
#pragma unroll
        for (int j = 0; j < H1C; ++j)
#pragma unroll
          for (int u = 0; u < U; ++u) t[u] = fmaf(W1T[(k + u) * H1C + j], dz[j], t[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) stg[lane * SP + k + u] = t[u];
      }
    }
    // matrix-factorisation rows: d mu = (Wo_mf^T dl) * mi, d mi = (Wo_mf^T dl) * mu
#pragma unroll
    for (int k = 0; k < EC; ++k) {
      const float t = ncf_dot<NCC>(WOT + (H3C + k) * NCC, dl);
      stg[lane * SP + 2 * EC + k] = t * mi[k];
      stg[lane * SP + 3 * EC + k] = t * mu[k];
    }
    __builtin_amdgcn_wave_barrier();
    const int ulo = (int)uid, uhi = (int)(uid >> 32), ilo = (int)iid, ihi = (int)(iid >> 32);
#pragma unroll 1
    for (int r = 0; r < 64; ++r) {
      const int64_t ur = (int64_t)(((uint64_t)(uint32_t)__shfl(uhi, r, 64) << 32) | (uint32_t)__shfl(ulo, r, 64));
      const int64_t ir = (int64_t)(((uint64_t)(uint32_t)__shfl(ihi, r, 64) << 32) | (uint32_t)__shfl(ilo, r, 64));
#pragma unroll
      for (int c0 = 0; c0 < 4 * EC; c0 += 64) {
        const int c = c0 + lane;
        if (c < 4 * EC) {
          const int seg = c / EC, col = c - seg * EC;
          const bool user = (seg & 1) == 0;
          float* g = seg == 0 ? a.gtu : (seg == 1 ? a.gti : (seg == 2 ? a.gtmu : a.gtmi));
          const int e = seg == 0 ? eu : (seg == 1 ? ei : em);
          const int64_t id = user ? ur : ir;
          const int V = user ? a.Vu : a.Vi;
          if (g != nullptr && col < e && id >= 0 && id < V) atomicAdd(g + id * e + col, stg[r * SP + c]);
        }
      }
    }
    __syncthreads();
    float* dst = a.partial + (size_t)blockIdx.x * a.nwg;
    for (int i = tid; i < a.nwg; i += kNcfRows) dst[i] = sred[i];
  }
}

// partial [nblk, nwg] -> column sums added into the 8 packed segments' destinations
struct NcfDst {
  float* p[8];
  int off[9];
};

// 16 columns x 16 partial-row slices per block: ~nwg / 16 blocks keep enough loads in flight
__global__ __launch_bounds__(256) void ncf_reduce_kernel(const float* __restrict__ partial, int nblk, int nwg,
                                                         NcfDst d) {
  __shared__ float red[16][17];
  const int cl = threadIdx.x & 15, part = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (col < nwg)
    for (int b = part; b < nblk; b += 16) s += partial[(size_t)b * nwg + col];
  red[part][cl] = s;
  __syncthreads();
  if (part != 0 || col >= nwg) return;
#pragma unroll
  for (int p = 1; p < 16; ++p) s += red[p][cl];
#pragma unroll
  for (int k = 0; k < 8; ++k)
    if (col >= d.off[k] && col < d.off[k + 1]) {
      if (d.p[k]) d.p[k][col - d.off[k]] += s;
      break;
    }
}

template <typename T, int EC, int H1C, int H2C, int H3C, int NCC>
static hipError_t ncf_launch(const NcfArgs& a, float* const* gdst, hipStream_t st) {
  using Cp = NcfCaps<EC, H1C, H2C, H3C, NCC>;
  const int grid = (a.B + kNcfRows - 1) / kNcfRows;
  if (a.dprobs == nullptr) {
    auto k = &ncf_kernel<T, EC, H1C, H2C, H3C, NCC, false>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kNcfRows), Cp::lds_fwd(), st, a);
    return hipGetLastError();
  }
  const size_t lds = Cp::lds_bwd(a.nwg);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  auto k = &ncf_kernel<T, EC, H1C, H2C, H3C, NCC, true>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3(grid), dim3(kNcfRows), lds, st, a);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const NcfOff o(a.eu, a.ei, a.em, a.h1, a.h2, a.h3, a.nc);
  NcfDst d;
  const int offs[9] = {o.w1, o.b1, o.w2, o.b2, o.w3, o.b3, o.wo, o.bo, o.n};
  for (int i = 0; i < 8; ++i) d.p[i] = gdst[i];
  for (int i = 0; i < 9; ++i) d.off[i] = offs[i];
  hipLaunchKernelGGL(ncf_reduce_kernel, dim3((a.nwg + 15) / 16), dim3(256), 0, st, a.partial, grid, a.nwg, d);
  return hipGetLastError();
}

}  // namespace zoo

using namespace zoo;

// caps: embedding widths <= 20, hidden <= (40, 20, 10), classes <= 8 -- the NeuralCF defaults
// (NeuralCF.scala:45-60, the ml-1m / ml-20m examples); -1 = use the layer-by-layer path
extern "C" int zoo_ncf_tier(int eu, int ei, int em, int h1, int h2, int h3, int nc) {
  if (eu <= 0 || ei <= 0 || em < 0 || h1 <= 0 || h2 <= 0 || h3 <= 0 || nc <= 0) return -1;
  if (eu % 4 || ei % 4 || em % 4) return -1;
  const int e = eu > ei ? (eu > em ? eu : em) : (ei > em ? ei : em);
  if (e <= 20 && h1 <= 40 && h2 <= 20 && h3 <= 10 && nc <= 8) return 0;
  return -1;
}

extern "C" int zoo_ncf_nwg(int eu, int ei, int em, int h1, int h2, int h3, int nc) {
  return NcfOff(eu, ei, em, h1, h2, h3, nc).n;
}

// gdst: 8 fp32 destinations (W1, b1, W2, b2, W3, b3, Wo, bo; null = skip), backward only
extern "C" hipError_t zoo_ncf(const NcfArgs* a, float* const* gdst, int bf16, hipStream_t st) {
  if (zoo_ncf_tier(a->eu, a->ei, a->em, a->h1, a->h2, a->h3, a->nc) < 0 || a->B <= 0) return hipErrorInvalidValue;
  return bf16 ? ncf_launch<bf16_t, 20, 40, 20, 10, 8>(*a, gdst, st) : ncf_launch<float, 20, 40, 20, 10, 8>(*a, gdst, st);
}
