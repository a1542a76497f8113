// Fused scaled-dot-product attention (flash-style) for CDNA4 (gfx950).
//
// Reference op: TransformerLayer.attn / BERT self-attention
//   softmax(Q K^T * scale + mask) V        (TransformerLayer.scala:163-181,
//   SURVEY.md §2.16 HK8), with an optional causal mask (tril(S-L)) and an
//   optional additive per-key mask [B][S] (BERT's (1-mask)*-10000).
// The score matrix is never materialised: per query tile the kernel walks
// 64-key K/V tiles with an online softmax (running max / sum per query row).
//
// Layouts: q/o [B][H][L][D], k/v [B][H][S][D] bf16, D in {64, 128};
// lse [B][H][L] fp32 = ln sum_k exp(logit) (saved for the backward pass).
//
// MFMA orientation (v_mfma_f32_16x16x32_bf16; A lane l: row l&15, k 8(l>>4)+j;
// B lane l: k 8(l>>4)+j, col l&15; C: row 4(l>>4)+r, col l&15):
//   forward  S^T = K Q^T   -> a lane owns ONE query row (col) and 16 keys
//                              (rows), so row max / sum need only 2 shuffles
//            O^T = V^T P^T -> P^T comes straight from the S^T accumulators
//                              (k order permuted identically on both sides:
//                              k-slot (g, j) = key 4g+j (j<4) / 16+4g+j-4),
//                              V^T is read from the row-major V tile with the
//                              hardware transposing ds_read_b64_tr_b16.
//   dK/dV    S = Q K^T, dP = dO V^T (key on the lane, K/V in registers),
//            dV^T += dO^T P, dK^T += Q^T dS  (Q/dO tiles transposed-read)
//   dQ       S^T, dP^T as in the forward, dQ^T += K^T dS^T
// dK/dV and dQ are separate passes (each recomputes P from the saved LSE), so
// no float atomics and no cross-wave transposes are needed.
#include "common.h"

namespace zoo {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// [64][D] bf16 tile, 16-byte chunks XOR-swizzled by row so that the 16 rows of
// a half-wave's row read land in distinct bank groups.
template <int D>
ZOO_DEV int t_off(int row, int col) {
  constexpr int NCH = D / 8;
  return row * D + ((((col >> 3) ^ row) & (NCH - 1)) << 3) + (col & 7);
}

// 16-byte row fragment: A/B operand with k along the tile's columns
template <int D>
ZOO_DEV bf16x8 row_frag(const bf16_t* tile, int row, int col) {
  return *reinterpret_cast<const bf16x8*>(tile + t_off<D>(row, col));
}

// transposed fragment: operand element j of lane-group g = tile[rowk(g,j)][col0 + (l&15)]
// with the permuted k order rowk = base + 4g + j (j<4), base + 16 + 4g + j-4 (j>=4)
template <int D>
ZOO_DEV bf16x8 tr_frag(const bf16_t* tile, int base, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_i16x4*)(tile + t_off<D>(base + 4 * g + tq, col0 + 4 * tp)));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_i16x4*)(tile + t_off<D>(base + 16 + 4 * g + tq, col0 + 4 * tp)));
  typedef short i16x8 __attribute__((ext_vector_type(8)));
  i16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// two accumulator tiles (k = 4g+r and 16+4g+r) -> one bf16 operand fragment
ZOO_DEV bf16x8 pack_frag(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (__bf16)a[0]; r[1] = (__bf16)a[1]; r[2] = (__bf16)a[2]; r[3] = (__bf16)a[3];
  r[4] = (__bf16)b[0]; r[5] = (__bf16)b[1]; r[6] = (__bf16)b[2]; r[7] = (__bf16)b[3];
  return r;
}

ZOO_DEV bf16x8 load_frag(const bf16_t* p, bool ok) {
  uint4 v = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8, v);
}

// Register-staged double-buffered copy of `NT` [64][D] tiles (rows r0.., bounded by nrows)
template <int D, int NT>
struct TileStage {
  static constexpr int PER = 64 * D / 8 / 256;  // 16-byte chunks per thread per tile
  uint4 reg[NT][PER];
  ZOO_DEV void load(const bf16_t* const* src, int r0, int nrows) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int idx = threadIdx.x + 256 * i;
        const int row = idx / (D / 8), ch = idx % (D / 8);
        const int r = r0 + row;
        reg[t][i] = r < nrows ? *reinterpret_cast<const uint4*>(src[t] + (size_t)r * D + ch * 8)
                              : make_uint4(0, 0, 0, 0);
      }
  }
  ZOO_DEV void store(bf16_t* const* dst) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < PER; ++i) {
        const int idx = threadIdx.x + 256 * i;
        const int row = idx / (D / 8), ch = idx % (D / 8);
        *reinterpret_cast<uint4*>(dst[t] + t_off<D>(row, ch * 8)) = reg[t][i];
      }
  }
};

// ---------------------------------------------------------------------------
// forward: block = 4 waves x 32 query rows; 64-key K/V tiles double-buffered
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256, D == 128 ? 1 : 2) void attn_fwd_kernel(const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K,
                                                          const bf16_t* __restrict__ V,
                                                          const float* __restrict__ mask, bf16_t* __restrict__ O,
                                                          float* __restrict__ LSE, int H, int L, int S, float scale,
                                                          int causal) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);  // [2][64][D]
  bf16_t* Vs = Ks + 2 * 64 * D;                  // [2][64][D]
  constexpr int DC = D / 32, DT = D / 16;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int bh = blockIdx.y, b = bh / H;
  const bf16_t* Qp = Q + (size_t)bh * L * D;
  const bf16_t* Kp = K + (size_t)bh * S * D;
  const bf16_t* Vp = V + (size_t)bh * S * D;
  const float* mrow = mask ? mask + (size_t)b * S : nullptr;
  const int qblk = blockIdx.x * 128, q0 = qblk + wid * 32;
  const int coff = S - L;  // causal: key allowed iff key <= q + coff
  const float c2 = scale * kLog2e;

  bf16x8 qf[2][DC];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int dc = 0; dc < DC; ++dc) {
      const int q = q0 + 16 * s + li;
      qf[s][dc] = load_frag(Qp + (size_t)q * D + 32 * dc + 8 * g, q < L);
    }

  f32x4 o[2][DT];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < DT; ++i) o[s][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, lsum[2] = {0.f, 0.f};

  int kv_end = S;
  if (causal) kv_end = min(S, qblk + 127 + coff + 1);
  const int ntiles = kv_end > 0 ? (kv_end + 63) / 64 : 0;

  TileStage<D, 2> st;
  const bf16_t* srcs[2] = {Kp, Vp};
  if (ntiles > 0) {
    st.load(srcs, 0, S);
    bf16_t* d0[2] = {Ks, Vs};
    st.store(d0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, kv0 = t * 64;
    if (t + 1 < ntiles) st.load(srcs, kv0 + 64, S);
    const bf16_t* kt_ = Ks + buf * 64 * D;
    const bf16_t* vt_ = Vs + buf * 64 * D;
    // wave-uniform skip of tiles entirely above this wave's causal diagonal
    const bool active = !(causal && kv0 > q0 + 31 + coff) && q0 < L;
    if (active) {
      f32x4 sc[2][4];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) sc[s][k4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int dc = 0; dc < DC; ++dc) {
          const bf16x8 a = row_frag<D>(kt_, 16 * k4 + li, 32 * dc + 8 * g);
          sc[0][k4] = mfma16(a, qf[0][dc], sc[0][k4]);
          sc[1][k4] = mfma16(a, qf[1][dc], sc[1][k4]);
        }
      // additive key mask for this lane's 16 keys (same for both query subtiles)
      float madd[4][4];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kv0 + 16 * k4 + 4 * g + r;
          madd[k4][r] = key < S ? (mrow ? mrow[key] * kLog2e : 0.f) : -INFINITY;
        }
      bf16x8 pf[2][2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int q = q0 + 16 * s + li;
        float mx = -INFINITY;
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = kv0 + 16 * k4 + 4 * g + r;
            float x = sc[s][k4][r] * c2 + madd[k4][r];
            if (causal && key > q + coff) x = -INFINITY;
            sc[s][k4][r] = x;
            mx = fmaxf(mx, x);
          }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[s], mx);
        const float base = mnew == -INFINITY ? 0.f : mnew;
        const float alpha = exp2f(m[s] - base);
        float sum = 0.f;
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = exp2f(sc[s][k4][r] - base);
            sc[s][k4][r] = p;
            sum += p;
          }
        sum += __shfl_xor(sum, 16, 64);
        sum += __shfl_xor(sum, 32, 64);
        lsum[s] = lsum[s] * alpha + sum;
        m[s] = mnew;
#pragma unroll
        for (int i = 0; i < DT; ++i) o[s][i] *= alpha;
        pf[s][0] = pack_frag(sc[s][0], sc[s][1]);
        pf[s][1] = pack_frag(sc[s][2], sc[s][3]);
      }
#pragma unroll
      for (int i = 0; i < DT; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const bf16x8 a = tr_frag<D>(vt_, 32 * c, 16 * i, lane);
          o[0][i] = mfma16(a, pf[0][c], o[0][i]);
          o[1][i] = mfma16(a, pf[1][c], o[1][i]);
        }
    }
    if (t + 1 < ntiles) {
      bf16_t* dn[2] = {Ks + (buf ^ 1) * 64 * D, Vs + (buf ^ 1) * 64 * D};
      st.store(dn);
    }
    __syncthreads();
  }

  // epilogue: lane owns query row q, d = 16i + 4g .. +3 of every d-tile
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int q = q0 + 16 * s + li;
    if (q >= L) continue;
    const float inv = lsum[s] > 0.f ? 1.f / lsum[s] : 0.f;
    bf16_t* orow = O + ((size_t)bh * L + q) * D;
#pragma unroll
    for (int i = 0; i < DT; ++i) {
      uint2 w;
      w.x = pack2bf(o[s][i][0] * inv, o[s][i][1] * inv);
      w.y = pack2bf(o[s][i][2] * inv, o[s][i][3] * inv);
      *reinterpret_cast<uint2*>(orow + 16 * i + 4 * g) = w;
    }
    if (g == 0) LSE[(size_t)bh * L + q] = lsum[s] > 0.f ? (m[s] + __log2f(lsum[s])) * kLn2 : INFINITY;
  }
}

// delta[row] = sum_d dO[row][d] * O[row][d]  (fp32), 16 lanes per row
template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_t* __restrict__ dO, const bf16_t* __restrict__ O,
                                                         float* __restrict__ delta, int rows) {
  constexpr int LPR = D / 8;  // lanes per row (8 or 16)
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int row = tid / LPR, part = tid % LPR;
  float acc = 0.f;
  if (row < rows) {
    float a[8], b[8];
    unpack8(*reinterpret_cast<const uint4*>(dO + (size_t)row * D + part * 8), a);
    unpack8(*reinterpret_cast<const uint4*>(O + (size_t)row * D + part * 8), b);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += a[e] * b[e];
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < rows && part == 0) delta[row] = acc;
}

// ---------------------------------------------------------------------------
// backward dK/dV: block = 4 waves x 16 keys (64 keys); 64-query Q/dO tiles
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const float* __restrict__ mask, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    const float* __restrict__ delta, bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int H, int L, int S,
    float scale, int causal) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);  // [2][64][D]
  bf16_t* dOs = Qs + 2 * 64 * D;                 // [2][64][D]
  float* lse_s = reinterpret_cast<float*>(dOs + 2 * 64 * D);  // [2][64] (log2 domain)
  float* del_s = lse_s + 2 * 64;                               // [2][64]
  constexpr int DC = D / 32, DT = D / 16;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int bh = blockIdx.y, b = bh / H;
  const bf16_t* Qp = Q + (size_t)bh * L * D;
  const bf16_t* dOp = dO + (size_t)bh * L * D;
  const float* lp = LSE + (size_t)bh * L;
  const float* dp_ = delta + (size_t)bh * L;
  const int kblk = blockIdx.x * 64, key = kblk + wid * 16 + li;
  const int coff = S - L;
  const float c2 = scale * kLog2e;
  const bool key_ok = key < S;
  const float madd = !key_ok ? -INFINITY : (mask ? mask[(size_t)b * S + key] * kLog2e : 0.f);

  bf16x8 kf[DC], vf[DC];
#pragma unroll
  for (int dc = 0; dc < DC; ++dc) {
    kf[dc] = load_frag(K + ((size_t)bh * S + key) * D + 32 * dc + 8 * g, key_ok);
    vf[dc] = load_frag(V + ((size_t)bh * S + key) * D + 32 * dc + 8 * g, key_ok);
  }
  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // causal: query q sees key iff key <= q + coff  ->  first useful q = kblk - coff
  int qstart = 0;
  if (causal) qstart = max(0, (kblk - coff) / 64 * 64);
  const int ntiles = qstart < L ? (L - qstart + 63) / 64 : 0;

  TileStage<D, 2> st;
  const bf16_t* srcs[2] = {Qp, dOp};
  float lse_r = 0.f, del_r = 0.f;
  auto load_rows = [&](int q0) {
    st.load(srcs, q0, L);
    if (threadIdx.x < 64) {
      const int q = q0 + threadIdx.x;
      lse_r = q < L ? lp[q] * kLog2e : INFINITY;
      del_r = q < L ? dp_[q] : 0.f;
    }
  };
  auto store_rows = [&](int buf) {
    bf16_t* d[2] = {Qs + buf * 64 * D, dOs + buf * 64 * D};
    st.store(d);
    if (threadIdx.x < 64) {
      lse_s[buf * 64 + threadIdx.x] = lse_r;
      del_s[buf * 64 + threadIdx.x] = del_r;
    }
  };
  if (ntiles > 0) {
    load_rows(qstart);
    store_rows(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, q0 = qstart + t * 64;
    if (t + 1 < ntiles) load_rows(q0 + 64);
    const bf16_t* qt_ = Qs + buf * 64 * D;
    const bf16_t* ot_ = dOs + buf * 64 * D;
    const float* ls = lse_s + buf * 64;
    const float* ds_ = del_s + buf * 64;
    const bool active = !(causal && kblk + wid * 16 > q0 + 63 + coff);
    if (active) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) sc[q4] = dp[q4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int dc = 0; dc < DC; ++dc) {
          sc[q4] = mfma16(row_frag<D>(qt_, 16 * q4 + li, 32 * dc + 8 * g), kf[dc], sc[q4]);
          dp[q4] = mfma16(row_frag<D>(ot_, 16 * q4 + li, 32 * dc + 8 * g), vf[dc], dp[q4]);
        }
      // P = exp2(s*c2 + mask - lse2), dS = P * (dP - delta); row q = 16q4 + 4g + r
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int qr = 16 * q4 + 4 * g + r;
          float p = exp2f(sc[q4][r] * c2 + madd - ls[qr]);
          if (causal && key > q0 + qr + coff) p = 0.f;
          sc[q4][r] = p;
          dp[q4][r] = p * (dp[q4][r] - ds_[qr]);
        }
      const bf16x8 pf0 = pack_frag(sc[0], sc[1]), pf1 = pack_frag(sc[2], sc[3]);
      const bf16x8 sf0 = pack_frag(dp[0], dp[1]), sf1 = pack_frag(dp[2], dp[3]);
#pragma unroll
      for (int i = 0; i < DT; ++i) {
        dv[i] = mfma16(tr_frag<D>(ot_, 0, 16 * i, lane), pf0, dv[i]);
        dv[i] = mfma16(tr_frag<D>(ot_, 32, 16 * i, lane), pf1, dv[i]);
        dk[i] = mfma16(tr_frag<D>(qt_, 0, 16 * i, lane), sf0, dk[i]);
        dk[i] = mfma16(tr_frag<D>(qt_, 32, 16 * i, lane), sf1, dk[i]);
      }
    }
    if (t + 1 < ntiles) store_rows(buf ^ 1);
    __syncthreads();
  }

  if (!key_ok) return;
  bf16_t* dkr = dK + ((size_t)bh * S + key) * D;
  bf16_t* dvr = dV + ((size_t)bh * S + key) * D;
#pragma unroll
  for (int i = 0; i < DT; ++i) {
    uint2 w;
    w.x = pack2bf(dk[i][0] * scale, dk[i][1] * scale);
    w.y = pack2bf(dk[i][2] * scale, dk[i][3] * scale);
    *reinterpret_cast<uint2*>(dkr + 16 * i + 4 * g) = w;
    w.x = pack2bf(dv[i][0], dv[i][1]);
    w.y = pack2bf(dv[i][2], dv[i][3]);
    *reinterpret_cast<uint2*>(dvr + 16 * i + 4 * g) = w;
  }
}

// ---------------------------------------------------------------------------
// backward dQ: block = 4 waves x 16 query rows (64 rows); K/V tiles as forward
// ---------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const float* __restrict__ mask, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    const float* __restrict__ delta, bf16_t* __restrict__ dQ, int H, int L, int S, float scale, int causal) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Vs = Ks + 2 * 64 * D;
  constexpr int DC = D / 32, DT = D / 16;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, li = lane & 15;
  const int bh = blockIdx.y, b = bh / H;
  const bf16_t* Kp = K + (size_t)bh * S * D;
  const bf16_t* Vp = V + (size_t)bh * S * D;
  const float* mrow = mask ? mask + (size_t)b * S : nullptr;
  const int qblk = blockIdx.x * 64, q0 = qblk + wid * 16, q = q0 + li;
  const int coff = S - L;
  const float c2 = scale * kLog2e;
  const bool q_ok = q < L;

  bf16x8 qf[DC], of[DC];
#pragma unroll
  for (int dc = 0; dc < DC; ++dc) {
    qf[dc] = load_frag(Q + ((size_t)bh * L + q) * D + 32 * dc + 8 * g, q_ok);
    of[dc] = load_frag(dO + ((size_t)bh * L + q) * D + 32 * dc + 8 * g, q_ok);
  }
  const float lse2 = q_ok ? LSE[(size_t)bh * L + q] * kLog2e : INFINITY;
  const float del = q_ok ? delta[(size_t)bh * L + q] : 0.f;
  f32x4 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  int kv_end = S;
  if (causal) kv_end = min(S, qblk + 63 + coff + 1);
  const int ntiles = kv_end > 0 ? (kv_end + 63) / 64 : 0;
  TileStage<D, 2> st;
  const bf16_t* srcs[2] = {Kp, Vp};
  if (ntiles > 0) {
    st.load(srcs, 0, S);
    bf16_t* d0[2] = {Ks, Vs};
    st.store(d0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, kv0 = t * 64;
    if (t + 1 < ntiles) st.load(srcs, kv0 + 64, S);
    const bf16_t* kt_ = Ks + buf * 64 * D;
    const bf16_t* vt_ = Vs + buf * 64 * D;
    const bool active = !(causal && kv0 > q0 + 15 + coff) && q0 < L;
    if (active) {
      f32x4 sc[4], dp[4];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) sc[k4] = dp[k4] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int dc = 0; dc < DC; ++dc) {
          sc[k4] = mfma16(row_frag<D>(kt_, 16 * k4 + li, 32 * dc + 8 * g), qf[dc], sc[k4]);
          dp[k4] = mfma16(row_frag<D>(vt_, 16 * k4 + li, 32 * dc + 8 * g), of[dc], dp[k4]);
        }
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = kv0 + 16 * k4 + 4 * g + r;
          const float madd = key < S ? (mrow ? mrow[key] * kLog2e : 0.f) : -INFINITY;
          float p = exp2f(sc[k4][r] * c2 + madd - lse2);
          if (causal && key > q + coff) p = 0.f;
          dp[k4][r] = p * (dp[k4][r] - del);
        }
      const bf16x8 sf0 = pack_frag(dp[0], dp[1]), sf1 = pack_frag(dp[2], dp[3]);
#pragma unroll
      for (int i = 0; i < DT; ++i) {
        dq[i] = mfma16(tr_frag<D>(kt_, 0, 16 * i, lane), sf0, dq[i]);
        dq[i] = mfma16(tr_frag<D>(kt_, 32, 16 * i, lane), sf1, dq[i]);
      }
    }
    if (t + 1 < ntiles) {
      bf16_t* dn[2] = {Ks + (buf ^ 1) * 64 * D, Vs + (buf ^ 1) * 64 * D};
      st.store(dn);
    }
    __syncthreads();
  }
  if (!q_ok) return;
  bf16_t* dqr = dQ + ((size_t)bh * L + q) * D;
#pragma unroll
  for (int i = 0; i < DT; ++i) {
    uint2 w;
    w.x = pack2bf(dq[i][0] * scale, dq[i][1] * scale);
    w.y = pack2bf(dq[i][2] * scale, dq[i][3] * scale);
    *reinterpret_cast<uint2*>(dqr + 16 * i + 4 * g) = w;
  }
}

}  // namespace zoo

using namespace zoo;

// D = 128 tiles need more than the default 64 KiB of dynamic LDS per block
#define ATTN_LAUNCH(kern, grid, smem, ...)                                                              \
  do {                                                                                                  \
    static const bool lds_ok_ = [] {                                                                    \
      hipFuncSetAttribute(reinterpret_cast<const void*>(&kern), hipFuncAttributeMaxDynamicSharedMemorySize, \
                          96 * 1024);                                                                   \
      return true;                                                                                      \
    }();                                                                                                \
    (void)lds_ok_;                                                                                      \
    hipLaunchKernelGGL(kern, grid, dim3(256), smem, st, __VA_ARGS__);                                   \
  } while (0)

extern "C" hipError_t zoo_attn_fwd(const void* q, const void* k, const void* v, const float* mask, void* o,
                                   float* lse, int B, int H, int L, int S, int D, float scale, int causal,
                                   hipStream_t st) {
  const dim3 grid((L + 127) / 128, B * H);
  const size_t smem = (size_t)4 * 64 * D * sizeof(bf16_t);
  if (D == 64)
    ATTN_LAUNCH(attn_fwd_kernel<64>, grid, smem, (const bf16_t*)q, (const bf16_t*)k,
                       (const bf16_t*)v, mask, (bf16_t*)o, lse, H, L, S, scale, causal);
  else if (D == 128)
    ATTN_LAUNCH(attn_fwd_kernel<128>, grid, smem, (const bf16_t*)q, (const bf16_t*)k,
                       (const bf16_t*)v, mask, (bf16_t*)o, lse, H, L, S, scale, causal);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

extern "C" hipError_t zoo_attn_bwd(const void* dout, const void* q, const void* k, const void* v, const float* mask,
                                   const void* o, const float* lse, float* delta, void* dq, void* dk, void* dv, int B,
                                   int H, int L, int S, int D, float scale, int causal, hipStream_t st) {
  const int rows = B * H * L;
  const int dblocks = (rows * (D / 8) + 255) / 256;
  const size_t smem_kv = (size_t)4 * 64 * D * sizeof(bf16_t);
  const size_t smem_q = smem_kv + 4 * 64 * sizeof(float);
  if (D == 64) {
    hipLaunchKernelGGL(attn_delta_kernel<64>, dim3(dblocks), dim3(256), 0, st, (const bf16_t*)dout,
                       (const bf16_t*)o, delta, rows);
    ATTN_LAUNCH(attn_bwd_dkdv_kernel<64>, dim3((S + 63) / 64, B * H), smem_q,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dk, (bf16_t*)dv, H, L, S, scale, causal);
    ATTN_LAUNCH(attn_bwd_dq_kernel<64>, dim3((L + 63) / 64, B * H), smem_kv,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dq, H, L, S, scale, causal);
  } else if (D == 128) {
    hipLaunchKernelGGL(attn_delta_kernel<128>, dim3(dblocks), dim3(256), 0, st, (const bf16_t*)dout,
                       (const bf16_t*)o, delta, rows);
    ATTN_LAUNCH(attn_bwd_dkdv_kernel<128>, dim3((S + 63) / 64, B * H), smem_q,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dk, (bf16_t*)dv, H, L, S, scale, causal);
    ATTN_LAUNCH(attn_bwd_dq_kernel<128>, dim3((L + 63) / 64, B * H), smem_kv,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dq, H, L, S, scale, causal);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
