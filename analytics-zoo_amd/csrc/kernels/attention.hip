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
// All products run on v_mfma_f32_32x32x16_bf16 (A lane l: row l&31, k 8(l>>5)+j;
// B lane l: k 8(l>>5)+j, col l&31; C reg i: row 8(i>>2)+4(l>>5)+(i&3), col l&31):
//   forward  S^T = K Q^T   -> a lane owns ONE query row (col) and 32 keys
//                              (rows): row max needs one cross-half shuffle
//            O^T = V^T P^T -> P^T comes straight from the S^T accumulators
//                              (k-step s = regs 8s..8s+7, a permuted key order
//                              that the transposed V^T read reproduces with
//                              the hardware ds_read_b64_tr_b16)
//   dK/dV    S = Q K^T, dP = dO V^T (key on the lane, K/V in registers),
//            dV^T += dO^T P, dK^T += Q^T dS  (Q/dO tiles transposed-read)
//   dQ       S^T, dP^T as in the forward, dQ^T += K^T dS^T
// dK/dV and dQ are separate passes (each recomputes P from the saved LSE), so
// no float atomics and no cross-wave transposes are needed.
#include "common.h"

namespace zoo {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// [64][D] bf16 tile, 16-byte chunks XOR-swizzled by row. The swizzle is chosen
// for BOTH reads of the tile (MI355X_MICROARCH.md §LDS lane groups):
//  * ds_read_b128 row fragments (16 rows of a lane group, one logical chunk):
//    the 16 rows must hit 16 distinct 16-byte bank slots;
//  * ds_read_b64_tr_b16 (4 consecutive rows x 4 consecutive chunks per 32-lane
//    half): the 4 rows' chunk groups must land on disjoint bank slots.
// D = 128 (256-B rows): chunk ^= ((row&3)<<2) | ((row>>2)&3)
// D = 64 (128-B rows, two rows per bank line): chunk ^= (((row>>1)&1)<<2) | ((row>>2)&3)
template <int D>
ZOO_DEV int swz(int row) {
  return D == 128 ? (((row & 3) << 2) | ((row >> 2) & 3)) : ((((row >> 1) & 1) << 2) | ((row >> 2) & 3));
}
template <int D>
ZOO_DEV int t_off(int row, int col) {
  return row * D + ((((col >> 3) ^ swz<D>(row)) & (D / 8 - 1)) << 3) + (col & 7);
}

// exp2 straight to v_exp_f32 (no denormal range fix-up: softmax terms that
// small are zero at bf16 anyway)
ZOO_DEV float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 16-byte row fragment: A/B operand with k along the tile's columns
template <int D>
ZOO_DEV bf16x8 row_frag(const bf16_t* tile, int row, int col) {
  return *reinterpret_cast<const bf16x8*>(tile + t_off<D>(row, col));
}

ZOO_DEV bf16x8 load_frag(const bf16_t* p, bool ok) {
  uint4 v = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
  return __builtin_bit_cast(bf16x8, v);
}

// ---------------------------------------------------------------------------
// forward: NW waves x 32 query rows per block on v_mfma_f32_32x32x16_bf16
// (a 32x32x16 MFMA blocks vector issue for 8 of its 32 cycles, leaving 3x the
// room of 16x16x32 for the softmax VALU work, MI355X_MICROARCH.md constants).
//   S^T[key][q] = K Q^T: A = K rows (LDS), B = Q (registers); accumulator reg
//   i of tile kt holds key 32kt + 8(i>>2) + 4h + (i&3) for query q0 + (l&31).
//   O^T[d][q] += V^T P^T: B = P^T packed straight from the accumulators
//   (k-step s = regs 8s..8s+7), A = V^T via ds_read_b64_tr_b16 in the same
//   permuted key order.
// Online softmax in the log2 domain with a deferred max: the running max only
// moves when a tile's max exceeds it by > kDeferTh (P <= 2^kDeferTh stays exact
// in fp32 sums and bf16 operands), so the O rescale is rare and wave-uniform.
// ---------------------------------------------------------------------------
typedef float f32x16 __attribute__((ext_vector_type(16)));

ZOO_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr float kDeferTh = 8.0f;

// A operand of a 32x32x16 MFMA = tile^T: lane (row d = col0 + (l&31), half h) gets
// keys kbase + 8(j>>2) + 4h + (j&3), j = 0..7, of column d
template <int D>
ZOO_DEV bf16x8 tr_frag32(const bf16_t* tile, int kbase, int col0, int lane) {
  const int gq = lane >> 4, h = gq >> 1, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int col = col0 + 16 * (gq & 1) + 4 * tp;
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + t_off<D>(kbase + 4 * h + tq, col)));
  const i16x4 hi =
      __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(tile + t_off<D>(kbase + 8 + 4 * h + tq, col)));
  const uint2 a = __builtin_bit_cast(uint2, lo), b = __builtin_bit_cast(uint2, hi);
  return __builtin_bit_cast(bf16x8, make_uint4(a.x, a.y, b.x, b.y));
}

ZOO_DEV bf16x8 pack8_acc(const f32x16& a, int base) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)a[base + j];
  return r;
}


typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gl_void;
ZOO_DEV void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Stage two [64][D] tiles (rows r0.., clamped to nrows-1: rows past the end
// only ever meet zero probabilities) with LDS-DMA: one wave-instruction writes a
// lane-linear 1-KiB piece, the swizzle is applied on the per-lane SOURCE address
// (position (row, pc) receives logical chunk pc ^ swz(row)). The NW waves of the
// block split the pieces; no staging registers, no ds_write.
// element strides of the forward kernel's operands: [batch, head, row]
struct AttnStrides {
  long qb, qh, ql, kb, kh, kl, vb, vh, vl, ob, oh, ol;
};

// backward element strides (batch, head, row) of q, k, v, dO, O, dQ, dK, dV: the packed training
// path reads q/k/v straight out of the [B, L, 3, H, D] projection and writes dq/dk/dv into its
// gradient, dO / O being [B, L, H, D] (LSE and delta stay contiguous [B*H, L]).
struct AttnBwdStrides {
  long qb, qh, ql, kb, kh, kl, vb, vh, vl, gb, gh, gl, ob, oh, ol;
  long dqb, dqh, dql, dkb, dkh, dkl, dvb, dvh, dvl;
};

// Dropout on the attention probabilities (BERT attention_probs dropout, TransformerLayer.scala
// attnDrop): keep(bh, q, key) is a counter hash of the element coordinates and a per-call seed,
// so the forward and both backward passes regenerate the same mask without storing it.
//   forward   O = (1/l) sum_k keep*scale * exp(s - m) V     (l sums the UNdropped terms)
//   backward  dV += P_drop^T dO ; dS = P * (keep*scale * dP_drop - delta), delta = rowsum(dO*O)
struct AttnDrop {
  uint32_t thresh;  // 0: no dropout
  float scale;      // 1 / (1 - p)
  uint32_t s0, s1;
  const uint32_t* off;  // per-step device seed offset (g_seed_off) or null
};

ZOO_DEV uint32_t attn_fmix(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// keep-factor (scale or 0) of probability (bh, q, key)
ZOO_DEV float attn_keep(const AttnDrop& d, int bh, int q, int key) {
  const uint32_t a = attn_fmix((uint32_t)bh * 0x9E3779B1u ^ d.s1);
  const uint32_t hsh = attn_fmix(((uint32_t)q * 0x85EBCA77u + (uint32_t)key) ^ d.s0 ^ a);
  return hsh >= d.thresh ? d.scale : 0.f;
}

template <int D, int NW>
ZOO_DEV void dma_tiles(const bf16_t* src0, const bf16_t* src1, bf16_t* dst0, bf16_t* dst1, int r0, int nrows,
                       long ld0 = D, long ld1 = D) {
  constexpr int PPT = D / 8;            // 1-KiB pieces per tile
  constexpr int PPW = 2 * PPT / NW;     // pieces per wave
  static_assert((2 * PPT) % NW == 0, "pieces must split evenly over the waves");
  constexpr int RP = 512 / D;           // tile rows per piece
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int rsub = lane / (D / 8), pc = lane % (D / 8);
#pragma unroll
  for (int i = 0; i < PPW; ++i) {
    const int gp = wid * PPW + i;
    const bool second = gp >= PPT;
    const int pp = second ? gp - PPT : gp;
    const int row = pp * RP + rsub;
    const int r = min(r0 + row, nrows - 1);
    const bf16_t* sp = (second ? src1 : src0) + (size_t)r * (second ? ld1 : ld0) + ((pc ^ swz<D>(row)) << 3);
    bf16_t* dp = (second ? dst1 : dst0) + pp * 512;
    __builtin_amdgcn_global_load_lds((gl_void*)sp, (lds_void*)dp, 16, 0, 0);
  }
}

template <int D, int NW, bool HAS_MASK, bool DROP>
__global__ __launch_bounds__(NW * 64, 8 / NW) void attn_fwd_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const float* __restrict__ mask, bf16_t* __restrict__ O, float* __restrict__ LSE, int H, int L, int S,
    float scale, int causal, AttnStrides sd, AttnDrop dd) {
  if (dd.thresh && dd.off) dd.s0 ^= *dd.off;
  constexpr int NTH = NW * 64, KS = D / 16, DT = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);  // [2][64][D]
  bf16_t* Vs = Ks + 2 * 64 * D;                  // [2][64][D]
  float* Ms = reinterpret_cast<float*>(Vs + 2 * 64 * D);  // [2][64] additive mask (log2 units)

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, lr = lane & 31;
  const int bh = blockIdx.y, b = bh / H, hd = bh - b * H;
  // element strides (batch, head, row); rows are D-contiguous. Contiguous [B,H,T,D]
  // tensors and views into a packed [B,T,3,H,D] QKV projection both come through here.
  const bf16_t* Kp = K + b * sd.kb + hd * sd.kh;
  const bf16_t* Vp = V + b * sd.vb + hd * sd.vh;
  const float* mrow = HAS_MASK ? mask + (size_t)b * S : nullptr;
  // causal: heaviest query blocks (largest index) first
  const int qb = causal ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int qblk = qb * 32 * NW, q0 = qblk + wid * 32, q = q0 + lr;
  const int coff = S - L;  // causal: key allowed iff key <= q + coff
  const float c2 = scale * kLog2e;

  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    qf[ks] = load_frag(Q + b * sd.qb + hd * sd.qh + (long)min(q, L - 1) * sd.ql + 16 * ks + 8 * h, q < L);

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[i][r] = 0.f;
  float m = -INFINITY, lsum = 0.f;

  int kv_end = S;
  if (causal) kv_end = min(S, qblk + 32 * NW - 1 + coff + 1);
  const int ntiles = kv_end > 0 ? (kv_end + 63) / 64 : 0;

  float mreg = 0.f;
  auto load_mask = [&](int kv0) {
    if (HAS_MASK && threadIdx.x < 64) {
      const int key = kv0 + threadIdx.x;
      mreg = key < S ? mrow[key] * kLog2e : -INFINITY;
    }
  };
  auto store_mask = [&](int buf) {
    if (HAS_MASK && threadIdx.x < 64) Ms[buf * 64 + threadIdx.x] = mreg;
  };
  if (ntiles > 0) {
    dma_tiles<D, NW>(Kp, Vp, Ks, Vs, 0, S, sd.kl, sd.vl);
    load_mask(0);
    wait_vm0();
    store_mask(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, kv0 = t * 64;
    if (t + 1 < ntiles) {
      dma_tiles<D, NW>(Kp, Vp, Ks + (buf ^ 1) * 64 * D, Vs + (buf ^ 1) * 64 * D, kv0 + 64, S, sd.kl, sd.vl);
      load_mask(kv0 + 64);
    }
    const bf16_t* kt_ = Ks + buf * 64 * D;
    const bf16_t* vt_ = Vs + buf * 64 * D;
    // wave-uniform: skip tiles entirely above this wave's causal diagonal
    if (q0 < L && !(causal && kv0 > q0 + 31 + coff)) {
      f32x16 s[2];
      const f32x16 z16 = {};
      // K fragments one k-step ahead of their MFMAs (keeps LDS latency off the chain)
      bf16x8 ka[2][2];
      ka[0][0] = row_frag<D>(kt_, lr, 8 * h);
      ka[0][1] = row_frag<D>(kt_, 32 + lr, 8 * h);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
          ka[(ks + 1) & 1][0] = row_frag<D>(kt_, lr, 16 * (ks + 1) + 8 * h);
          ka[(ks + 1) & 1][1] = row_frag<D>(kt_, 32 + lr, 16 * (ks + 1) + 8 * h);
        }
        s[0] = mfma32(ka[ks & 1][0], qf[ks], ks == 0 ? z16 : s[0]);
        s[1] = mfma32(ka[ks & 1][1], qf[ks], ks == 0 ? z16 : s[1]);
      }

      // logits in log2 units: x = s*c2 (+ mask); -inf outside [0, S) / above the diagonal
      const bool edge = (kv0 + 64 > S) || (causal && kv0 + 63 > q0 + coff);
      if (HAS_MASK) {
        const float* mk = Ms + buf * 64;
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i4 = 0; i4 < 4; ++i4) {
            const float4 mv = *reinterpret_cast<const float4*>(mk + 32 * kt + 8 * i4 + 4 * h);
            s[kt][4 * i4 + 0] = s[kt][4 * i4 + 0] * c2 + mv.x;
            s[kt][4 * i4 + 1] = s[kt][4 * i4 + 1] * c2 + mv.y;
            s[kt][4 * i4 + 2] = s[kt][4 * i4 + 2] * c2 + mv.z;
            s[kt][4 * i4 + 3] = s[kt][4 * i4 + 3] * c2 + mv.w;
          }
      }
      if (edge) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = kv0 + 32 * kt + 8 * (i >> 2) + 4 * h + (i & 3);
            if (key >= S || (causal && key > q + coff)) s[kt][i] = -INFINITY;
          }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[kt][i]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (!HAS_MASK) mx *= c2;
      const bool upd = mx > m + kDeferTh;
      if (__ballot(upd)) {
        const float mnew = upd ? mx : m;
        const float alpha = mnew == m ? 1.f : fexp2(m - mnew);
        lsum *= alpha;
#pragma unroll
        for (int i = 0; i < DT; ++i) o[i] *= alpha;
        m = mnew;
      }
      const float base = m == -INFINITY ? 0.f : m;
      float ps[4] = {0.f, 0.f, 0.f, 0.f};  // independent partial sums (no serial add chain)
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = HAS_MASK ? fexp2(s[kt][i] - base) : fexp2(s[kt][i] * c2 - base);
          s[kt][i] = p;
          ps[i & 3] += p;
        }
      lsum += (ps[0] + ps[1]) + (ps[2] + ps[3]);
      if (DROP) {  // dropout after the (undropped) normaliser sum
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            s[kt][i] *= attn_keep(dd, bh, q, kv0 + 32 * kt + 8 * (i >> 2) + 4 * h + (i & 3));
      }
      bf16x8 pf[4];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) pf[k4] = pack8_acc(s[k4 >> 1], 8 * (k4 & 1));
      constexpr int NSTEP = 4 * DT;
      bf16x8 fv[2];
      fv[0] = tr_frag32<D>(vt_, 0, 0, lane);
#pragma unroll
      for (int idx = 0; idx < NSTEP; ++idx) {
        if (idx + 1 < NSTEP) fv[(idx + 1) & 1] = tr_frag32<D>(vt_, 16 * ((idx + 1) / DT), 32 * ((idx + 1) % DT), lane);
        o[idx % DT] = mfma32(fv[idx & 1], pf[idx / DT], o[idx % DT]);
      }
    }
    if (t + 1 < ntiles) {
      wait_vm0();
      store_mask(buf ^ 1);
    }
    __syncthreads();
  }

  // epilogue: reg i of o[dt] = O[q][32dt + 8(i>>2) + 4h + (i&3)]
  lsum += __shfl_xor(lsum, 32, 64);
  if (q >= L) return;
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  bf16_t* orow = O + b * sd.ob + hd * sd.oh + (long)q * sd.ol;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      uint2 w;
      w.x = pack2bf(o[dt][4 * i4 + 0] * inv, o[dt][4 * i4 + 1] * inv);
      w.y = pack2bf(o[dt][4 * i4 + 2] * inv, o[dt][4 * i4 + 3] * inv);
      *reinterpret_cast<uint2*>(orow + 32 * dt + 8 * i4 + 4 * h) = w;
    }
  if (h == 0) LSE[(size_t)bh * L + q] = lsum > 0.f ? (m + __log2f(lsum)) * kLn2 : INFINITY;
}

// delta[row] = sum_d dO[row][d] * O[row][d]  (fp32), 16 lanes per row
template <int D>
__global__ __launch_bounds__(256) void attn_delta_kernel(const bf16_t* __restrict__ dO, const bf16_t* __restrict__ O,
                                                         float* __restrict__ delta, int rows, int H, int L,
                                                         AttnBwdStrides sd) {
  constexpr int LPR = D / 8;  // lanes per row (8 or 16)
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int row = tid / LPR, part = tid % LPR;
  float acc = 0.f;
  if (row < rows) {
    const int bh = row / L, l = row - bh * L, b = bh / H, hd = bh - b * H;
    float a[8], c[8];
    unpack8(*reinterpret_cast<const uint4*>(dO + b * sd.gb + hd * sd.gh + (long)l * sd.gl + part * 8), a);
    unpack8(*reinterpret_cast<const uint4*>(O + b * sd.ob + hd * sd.oh + (long)l * sd.ol + part * 8), c);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc += a[e] * c[e];
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < rows && part == 0) delta[row] = acc;
}

// ---------------------------------------------------------------------------
// backward dK/dV on 32x32x16 MFMAs: block = 128 keys (4 key groups of 32) x
// QW query halves; 64-query Q/dO tiles double-buffered by LDS-DMA.
//   S = Q K^T, dP = dO V^T with the key on the lane (K/V fragments in registers,
//   Q/dO row fragments from LDS); reg i of tile qt <-> q = 32qt + 8(i>>2) + 4h + (i&3)
//   dV^T += dO^T P, dK^T += Q^T dS: P / dS packed from the accumulators, dO^T /
//   Q^T transposed-read from the same LDS tiles in that permuted q order.
// ---------------------------------------------------------------------------
template <int D, int QW, bool HAS_MASK, bool DROP>
__global__ __launch_bounds__(256 * QW, 1) void attn_bwd_dkdv_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const float* __restrict__ mask, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    const float* __restrict__ delta, bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int H, int L, int S,
    float scale, int causal, AttnBwdStrides sd, AttnDrop dd) {
  if (dd.thresh && dd.off) dd.s0 ^= *dd.off;
  // QW = 2: 8 waves; wave w owns keys 32(w&3).. and query rows 32(w>>2).. of every
  // 64-row tile (two waves per SIMD); the two q-halves are summed through LDS at the end
  constexpr int KS = D / 16, DT = D / 32, NQT = 2 / QW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);                 // [2][64][D]
  bf16_t* dOs = Qs + 2 * 64 * D;                                // [2][64][D]
  float* lse_s = reinterpret_cast<float*>(dOs + 2 * 64 * D);    // [2][64] (log2 units)
  float* del_s = lse_s + 2 * 64;                                // [2][64]

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, lr = lane & 31;
  const int kg = wid & 3, qh = QW == 2 ? wid >> 2 : 0;
  const int bh = blockIdx.y, b = bh / H, hd = bh - b * H;
  const bf16_t* Qp = Q + b * sd.qb + hd * sd.qh;
  const bf16_t* dOp = dO + b * sd.gb + hd * sd.gh;
  const float* lp = LSE + (size_t)bh * L;
  const float* dp_ = delta + (size_t)bh * L;
  const int kblk = blockIdx.x * 128, kw0 = kblk + kg * 32, key = kw0 + lr;
  const int coff = S - L;
  const float c2 = scale * kLog2e;
  const bool key_ok = key < S;
  const float madd = !key_ok ? -INFINITY : (HAS_MASK ? mask[(size_t)b * S + key] * kLog2e : 0.f);

  bf16x8 kf[KS], vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    kf[ks] = load_frag(K + b * sd.kb + hd * sd.kh + (long)key * sd.kl + 16 * ks + 8 * h, key_ok);
    vf[ks] = load_frag(V + b * sd.vb + hd * sd.vh + (long)key * sd.vl + 16 * ks + 8 * h, key_ok);
  }
  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dk[i][r] = dv[i][r] = 0.f;

  // causal: query q sees key iff key <= q + coff -> first useful q = kblk - coff
  int qstart = 0;
  if (causal) qstart = max(0, (kblk - coff) / 64 * 64);
  const int ntiles = qstart < L ? (L - qstart + 63) / 64 : 0;

  float lse_r = 0.f, del_r = 0.f;
  auto load_rows = [&](int q0, int buf) {
    dma_tiles<D, 4 * QW>(Qp, dOp, Qs + buf * 64 * D, dOs + buf * 64 * D, q0, L, sd.ql, sd.gl);
    if (threadIdx.x < 64) {
      const int q = q0 + threadIdx.x;
      lse_r = q < L ? lp[q] * kLog2e : INFINITY;
      del_r = q < L ? dp_[q] : 0.f;
    }
  };
  auto store_rows = [&](int buf) {
    if (threadIdx.x < 64) {
      lse_s[buf * 64 + threadIdx.x] = lse_r;
      del_s[buf * 64 + threadIdx.x] = del_r;
    }
  };
  if (ntiles > 0) {
    load_rows(qstart, 0);
    wait_vm0();
    store_rows(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, q0 = qstart + t * 64;
    if (t + 1 < ntiles) load_rows(q0 + 64, buf ^ 1);
    const bf16_t* qt_ = Qs + buf * 64 * D;
    const bf16_t* ot_ = dOs + buf * 64 * D;
    const float* ls = lse_s + buf * 64;
    const float* ds_ = del_s + buf * 64;
    const int qlo = 32 * qh;  // first tile row of this wave (QW = 2) or 0
    if (kw0 < S && !(causal && kw0 > q0 + qlo + 32 * NQT - 1 + coff)) {
      f32x16 s[NQT], dp[NQT];
      const f32x16 z16 = {};
      bf16x8 qa[2][NQT], oa[2][NQT];
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt) {
        qa[0][qt] = row_frag<D>(qt_, qlo + 32 * qt + lr, 8 * h);
        oa[0][qt] = row_frag<D>(ot_, qlo + 32 * qt + lr, 8 * h);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
          const int c = 16 * (ks + 1) + 8 * h;
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) {
            qa[(ks + 1) & 1][qt] = row_frag<D>(qt_, qlo + 32 * qt + lr, c);
            oa[(ks + 1) & 1][qt] = row_frag<D>(ot_, qlo + 32 * qt + lr, c);
          }
        }
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) {
          s[qt] = mfma32(qa[ks & 1][qt], kf[ks], ks == 0 ? z16 : s[qt]);
          dp[qt] = mfma32(oa[ks & 1][qt], vf[ks], ks == 0 ? z16 : dp[qt]);
        }
      }
      const bool diag = causal && kw0 + 31 > q0 + qlo + coff;
#pragma unroll
      for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int qr = qlo + 32 * qt + 8 * i4 + 4 * h;
          const float4 l4 = *reinterpret_cast<const float4*>(ls + qr);
          const float4 d4 = *reinterpret_cast<const float4*>(ds_ + qr);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 4 * i4 + r;
            float p = fexp2(s[qt][i] * c2 + (madd - lv[r]));
            if (diag && key > q0 + qr + r + coff) p = 0.f;
            const float kf_ = DROP ? attn_keep(dd, bh, q0 + qr + r, key) : 1.f;
            s[qt][i] = p * kf_;
            dp[qt][i] = p * (dp[qt][i] * kf_ - dv4[r]);
          }
        }
      bf16x8 pf[2 * NQT], sf[2 * NQT];
#pragma unroll
      for (int k4 = 0; k4 < 2 * NQT; ++k4) {
        pf[k4] = pack8_acc(s[k4 >> 1], 8 * (k4 & 1));
        sf[k4] = pack8_acc(dp[k4 >> 1], 8 * (k4 & 1));
      }
      // dO^T / Q^T fragments one step ahead of their MFMAs
      constexpr int NSTEP = 2 * NQT * DT;
      bf16x8 fo[2], fq[2];
      fo[0] = tr_frag32<D>(ot_, qlo, 0, lane);
      fq[0] = tr_frag32<D>(qt_, qlo, 0, lane);
#pragma unroll
      for (int idx = 0; idx < NSTEP; ++idx) {
        if (idx + 1 < NSTEP) {
          const int k4n = (idx + 1) / DT, dtn = (idx + 1) % DT;
          fo[(idx + 1) & 1] = tr_frag32<D>(ot_, qlo + 16 * k4n, 32 * dtn, lane);
          fq[(idx + 1) & 1] = tr_frag32<D>(qt_, qlo + 16 * k4n, 32 * dtn, lane);
        }
        const int k4 = idx / DT, dt = idx % DT;
        dv[dt] = mfma32(fo[idx & 1], pf[k4], dv[dt]);
        dk[dt] = mfma32(fq[idx & 1], sf[k4], dk[dt]);
      }
    }
    if (t + 1 < ntiles) {
      wait_vm0();
      store_rows(buf ^ 1);
    }
    __syncthreads();
  }

  if (QW == 2) {
    // sum the two query halves: waves 4..7 park their partials in the (now idle) tile LDS
    float* red = reinterpret_cast<float*>(smem);  // [4 key groups][DT][16][64 lanes]
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      f32x16* acc = pass == 0 ? dk : dv;
      if (qh == 1) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) red[((kg * DT + dt) * 16 + r) * 64 + lane] = acc[dt][r];
      }
      __syncthreads();
      if (qh == 0) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[dt][r] += red[((kg * DT + dt) * 16 + r) * 64 + lane];
      }
      __syncthreads();
    }
    if (qh == 1) return;
  }
  if (!key_ok) return;
  // reg i of dk[dt] = dK[key][32dt + 8(i>>2) + 4h + (i&3)]
  bf16_t* dkr = dK + b * sd.dkb + hd * sd.dkh + (long)key * sd.dkl;
  bf16_t* dvr = dV + b * sd.dvb + hd * sd.dvh + (long)key * sd.dvl;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      const int d = 32 * dt + 8 * i4 + 4 * h;
      uint2 w;
      w.x = pack2bf(dk[dt][4 * i4 + 0] * scale, dk[dt][4 * i4 + 1] * scale);
      w.y = pack2bf(dk[dt][4 * i4 + 2] * scale, dk[dt][4 * i4 + 3] * scale);
      *reinterpret_cast<uint2*>(dkr + d) = w;
      w.x = pack2bf(dv[dt][4 * i4 + 0], dv[dt][4 * i4 + 1]);
      w.y = pack2bf(dv[dt][4 * i4 + 2], dv[dt][4 * i4 + 3]);
      *reinterpret_cast<uint2*>(dvr + d) = w;
    }
}

template <int D, int QW, bool HAS_MASK, bool DROP>
__global__ __launch_bounds__(256 * QW, 1) void attn_bwd_dkdv_pers_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const float* __restrict__ mask, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    const float* __restrict__ delta, bf16_t* __restrict__ dK, bf16_t* __restrict__ dV, int H, int L, int S,
    float scale, int causal, AttnBwdStrides sd, AttnDrop dd, int BH) {
  if (dd.thresh && dd.off) dd.s0 ^= *dd.off;
  // QW = 2: 8 waves; wave w owns keys 32(w&3).. and query rows 32(w>>2).. of every
  // 64-row tile (two waves per SIMD); the two q-halves are summed through LDS at the end.
  // Persistent over heads: block (x, y) handles heads y, y + gridDim.y, ... of key block x.
  // During the last query tile of a head the NEXT head's first Q/dO tile (LDS-DMA), its
  // LSE / delta rows and its K/V fragments (registers) are already in flight, so a head's
  // prologue latency overlaps the previous head's last tile and dK/dV epilogue (BERT s128
  // has two query tiles per head: the prologue was a third of a block's life).
  constexpr int KS = D / 16, DT = D / 32, NQT = 2 / QW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Qs = reinterpret_cast<bf16_t*>(smem);                 // [2][64][D]
  bf16_t* dOs = Qs + 2 * 64 * D;                                // [2][64][D]
  float* lse_s = reinterpret_cast<float*>(dOs + 2 * 64 * D);    // [2][64] (log2 units)
  float* del_s = lse_s + 2 * 64;                                // [2][64]
  float* red = del_s + 2 * 64;                                  // QW = 2: [4 key groups][DT][16][64 lanes]
  // persistent form (D = 64, QW = 2): the next head's 128 K / V rows staged here during the
  // current head's last tile, [2 x 64 rows][D] each (after the reduction area)
  constexpr bool PRE = D == 64 && QW == 2;
  bf16_t* KsN = reinterpret_cast<bf16_t*>(red + (QW == 2 ? 4 * DT * 16 * 64 : 0));
  bf16_t* VsN = KsN + 2 * 64 * D;

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, lr = lane & 31;
  const int kg = wid & 3, qh = QW == 2 ? wid >> 2 : 0;
  const int kblk = blockIdx.x * 128, kw0 = kblk + kg * 32, key = kw0 + lr;
  const int coff = S - L;
  const float c2 = scale * kLog2e;
  const bool key_ok = key < S;

  // causal: query q sees key iff key <= q + coff -> first useful q = kblk - coff
  int qstart = 0;
  if (causal) qstart = max(0, (kblk - coff) / 64 * 64);
  const int ntiles = qstart < L ? (L - qstart + 63) / 64 : 0;

  bf16x8 kf[KS], vf[KS];
  float madd = 0.f, lse_r = 0.f, del_r = 0.f;
  auto mask_of = [&](int bh_) -> float {
    const int b_ = bh_ / H;
    return !key_ok ? -INFINITY : (HAS_MASK ? mask[(size_t)b_ * S + key] * kLog2e : 0.f);
  };
  // K/V fragments straight from global memory (first head, non-persistent forms)
  auto load_kv = [&](int bh_) {
    const int b_ = bh_ / H, hd_ = bh_ - b_ * H;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = load_frag(K + b_ * sd.kb + hd_ * sd.kh + (long)key * sd.kl + 16 * ks + 8 * h, key_ok);
      vf[ks] = load_frag(V + b_ * sd.vb + hd_ * sd.vh + (long)key * sd.vl + 16 * ks + 8 * h, key_ok);
    }
    madd = mask_of(bh_);
  };
  // persistent form: the next head's K/V rows kblk.. kblk+127 into KsN / VsN (LDS-DMA; rows past
  // S clamp to S-1 -- those keys get p = 0 from madd = -inf and are never stored)
  auto stage_kv = [&](int bh_) {
    const int b_ = bh_ / H, hd_ = bh_ - b_ * H;
    const bf16_t* kp = K + b_ * sd.kb + hd_ * sd.kh;
    const bf16_t* vp = V + b_ * sd.vb + hd_ * sd.vh;
    dma_tiles<D, 4 * QW>(kp, vp, KsN, VsN, kblk, S, sd.kl, sd.vl);
    dma_tiles<D, 4 * QW>(kp, vp, KsN + 64 * D, VsN + 64 * D, kblk + 64, S, sd.kl, sd.vl);
  };
  auto read_kv = [&]() {
    const int kr = kg * 32 + lr;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = row_frag<D>(KsN + (kr >> 6) * 64 * D, kr & 63, 16 * ks + 8 * h);
      vf[ks] = row_frag<D>(VsN + (kr >> 6) * 64 * D, kr & 63, 16 * ks + 8 * h);
    }
  };
  auto load_rows = [&](int bh_, int q0, int buf) {
    const int b_ = bh_ / H, hd_ = bh_ - b_ * H;
    dma_tiles<D, 4 * QW>(Q + b_ * sd.qb + hd_ * sd.qh, dO + b_ * sd.gb + hd_ * sd.gh, Qs + buf * 64 * D,
                         dOs + buf * 64 * D, q0, L, sd.ql, sd.gl);
    if (threadIdx.x < 64) {
      const int q = q0 + threadIdx.x;
      lse_r = q < L ? LSE[(size_t)bh_ * L + q] * kLog2e : INFINITY;
      del_r = q < L ? delta[(size_t)bh_ * L + q] : 0.f;
    }
  };
  auto store_rows = [&](int buf) {
    if (threadIdx.x < 64) {
      lse_s[buf * 64 + threadIdx.x] = lse_r;
      del_s[buf * 64 + threadIdx.x] = del_r;
    }
  };

  int cb = 0;              // buffer holding the current head's first query tile
  bool ready = false;      // the current head's K/V fragments and first tile were prefetched
  for (int bh = blockIdx.y; bh < BH; bh += gridDim.y) {
    const int b = bh / H, hd = bh - b * H;
    const int nbh = bh + gridDim.y;
    const bool pre = PRE && nbh < BH && ntiles > 0;   // prefetch the next head during this one's last tile
    if (ready) {
      read_kv();   // staged during the previous head's last tile (past its closing barrier)
    } else {
      load_kv(bh);
      if (ntiles > 0) {
        load_rows(bh, qstart, cb);
        wait_vm0();
        store_rows(cb);
      } else {
        wait_vm0();
      }
      __syncthreads();
    }
    float maddn = 0.f;
    f32x16 dk[DT], dv[DT];
#pragma unroll
    for (int i = 0; i < DT; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) dk[i][r] = dv[i][r] = 0.f;

    for (int t = 0; t < ntiles; ++t) {
      const int buf = cb ^ (t & 1), q0 = qstart + t * 64;
      if (t + 1 < ntiles) {
        load_rows(bh, q0 + 64, buf ^ 1);
      } else if (pre) {
        load_rows(nbh, qstart, buf ^ 1);
        stage_kv(nbh);
        maddn = mask_of(nbh);
      }
      const bf16_t* qt_ = Qs + buf * 64 * D;
      const bf16_t* ot_ = dOs + buf * 64 * D;
      const float* ls = lse_s + buf * 64;
      const float* ds_ = del_s + buf * 64;
      const int qlo = 32 * qh;  // first tile row of this wave (QW = 2) or 0
      if (kw0 < S && !(causal && kw0 > q0 + qlo + 32 * NQT - 1 + coff)) {
        f32x16 s[NQT], dp[NQT];
        const f32x16 z16 = {};
        bf16x8 qa[2][NQT], oa[2][NQT];
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) {
          qa[0][qt] = row_frag<D>(qt_, qlo + 32 * qt + lr, 8 * h);
          oa[0][qt] = row_frag<D>(ot_, qlo + 32 * qt + lr, 8 * h);
        }
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          if (ks + 1 < KS) {
            const int c = 16 * (ks + 1) + 8 * h;
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt) {
              qa[(ks + 1) & 1][qt] = row_frag<D>(qt_, qlo + 32 * qt + lr, c);
              oa[(ks + 1) & 1][qt] = row_frag<D>(ot_, qlo + 32 * qt + lr, c);
            }
          }
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) {
            s[qt] = mfma32(qa[ks & 1][qt], kf[ks], ks == 0 ? z16 : s[qt]);
            dp[qt] = mfma32(oa[ks & 1][qt], vf[ks], ks == 0 ? z16 : dp[qt]);
          }
        }
        const bool diag = causal && kw0 + 31 > q0 + qlo + coff;
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
          for (int i4 = 0; i4 < 4; ++i4) {
            const int qr = qlo + 32 * qt + 8 * i4 + 4 * h;
            const float4 l4 = *reinterpret_cast<const float4*>(ls + qr);
            const float4 d4 = *reinterpret_cast<const float4*>(ds_ + qr);
            const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = 4 * i4 + r;
              float p = fexp2(s[qt][i] * c2 + (madd - lv[r]));
              if (diag && key > q0 + qr + r + coff) p = 0.f;
              const float kf_ = DROP ? attn_keep(dd, bh, q0 + qr + r, key) : 1.f;
              s[qt][i] = p * kf_;
              dp[qt][i] = p * (dp[qt][i] * kf_ - dv4[r]);
            }
          }
        bf16x8 pf[2 * NQT], sf[2 * NQT];
#pragma unroll
        for (int k4 = 0; k4 < 2 * NQT; ++k4) {
          pf[k4] = pack8_acc(s[k4 >> 1], 8 * (k4 & 1));
          sf[k4] = pack8_acc(dp[k4 >> 1], 8 * (k4 & 1));
        }
        // dO^T / Q^T fragments one step ahead of their MFMAs
        constexpr int NSTEP = 2 * NQT * DT;
        bf16x8 fo[2], fq[2];
        fo[0] = tr_frag32<D>(ot_, qlo, 0, lane);
        fq[0] = tr_frag32<D>(qt_, qlo, 0, lane);
#pragma unroll
        for (int idx = 0; idx < NSTEP; ++idx) {
          if (idx + 1 < NSTEP) {
            const int k4n = (idx + 1) / DT, dtn = (idx + 1) % DT;
            fo[(idx + 1) & 1] = tr_frag32<D>(ot_, qlo + 16 * k4n, 32 * dtn, lane);
            fq[(idx + 1) & 1] = tr_frag32<D>(qt_, qlo + 16 * k4n, 32 * dtn, lane);
          }
          const int k4 = idx / DT, dt = idx % DT;
          dv[dt] = mfma32(fo[idx & 1], pf[k4], dv[dt]);
          dk[dt] = mfma32(fq[idx & 1], sf[k4], dk[dt]);
        }
      }
      if (t + 1 < ntiles || pre) {
        wait_vm0();
        store_rows(buf ^ 1);
      }
      __syncthreads();
    }
    if (pre) cb = cb ^ ((ntiles - 1) & 1) ^ 1;   // the next head's first tile sits in the other buffer

    bool store = key_ok;
    if (QW == 2) {
      // sum the two query halves: waves 4..7 park their partials in the reduction area (its own
      // LDS: the tile buffers already hold the next head's first tile)
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        f32x16* acc = pass == 0 ? dk : dv;
        if (qh == 1) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) red[((kg * DT + dt) * 16 + r) * 64 + lane] = acc[dt][r];
        }
        __syncthreads();
        if (qh == 0) {
#pragma unroll
          for (int dt = 0; dt < DT; ++dt)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[dt][r] += red[((kg * DT + dt) * 16 + r) * 64 + lane];
        }
        __syncthreads();
      }
      store = store && qh == 0;
    }
    if (store) {
      // reg i of dk[dt] = dK[key][32dt + 8(i>>2) + 4h + (i&3)]
      bf16_t* dkr = dK + b * sd.dkb + hd * sd.dkh + (long)key * sd.dkl;
      bf16_t* dvr = dV + b * sd.dvb + hd * sd.dvh + (long)key * sd.dvl;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int d = 32 * dt + 8 * i4 + 4 * h;
          uint2 w;
          w.x = pack2bf(dk[dt][4 * i4 + 0] * scale, dk[dt][4 * i4 + 1] * scale);
          w.y = pack2bf(dk[dt][4 * i4 + 2] * scale, dk[dt][4 * i4 + 3] * scale);
          *reinterpret_cast<uint2*>(dkr + d) = w;
          w.x = pack2bf(dv[dt][4 * i4 + 0], dv[dt][4 * i4 + 1]);
          w.y = pack2bf(dv[dt][4 * i4 + 2], dv[dt][4 * i4 + 3]);
          *reinterpret_cast<uint2*>(dvr + d) = w;
        }
    }
    ready = pre;
    if (pre) madd = maddn;
  }
}

// ---------------------------------------------------------------------------
// backward dQ on 32x32x16 MFMAs: NW waves x 32 query rows; K/V tiles as forward
//   S^T = K Q^T, dP^T = V dO^T (query on the lane: LSE and delta are per-lane
//   scalars), dQ^T += K^T dS^T with K^T transposed-read from the K tile.
// ---------------------------------------------------------------------------
template <int D, int NW, bool HAS_MASK, bool DROP>
__global__ __launch_bounds__(NW * 64, 1) void attn_bwd_dq_kernel(
    const bf16_t* __restrict__ Q, const bf16_t* __restrict__ K, const bf16_t* __restrict__ V,
    const float* __restrict__ mask, const bf16_t* __restrict__ dO, const float* __restrict__ LSE,
    const float* __restrict__ delta, bf16_t* __restrict__ dQ, int H, int L, int S, float scale, int causal,
    AttnBwdStrides sd, AttnDrop dd) {
  if (dd.thresh && dd.off) dd.s0 ^= *dd.off;
  constexpr int NTH = NW * 64, KS = D / 16, DT = D / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* Ks = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Vs = Ks + 2 * 64 * D;
  float* Ms = reinterpret_cast<float*>(Vs + 2 * 64 * D);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, h = lane >> 5, lr = lane & 31;
  const int bh = blockIdx.y, b = bh / H, hd = bh - b * H;
  const bf16_t* Kp = K + b * sd.kb + hd * sd.kh;
  const bf16_t* Vp = V + b * sd.vb + hd * sd.vh;
  const float* mrow = HAS_MASK ? mask + (size_t)b * S : nullptr;
  // causal: heaviest query blocks (largest index) first
  const int qb = causal ? (int)gridDim.x - 1 - (int)blockIdx.x : (int)blockIdx.x;
  const int qblk = qb * 32 * NW, q0 = qblk + wid * 32, q = q0 + lr;
  const int coff = S - L;
  const float c2 = scale * kLog2e;
  const bool q_ok = q < L;

  bf16x8 qf[KS], of[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = load_frag(Q + b * sd.qb + hd * sd.qh + (long)q * sd.ql + 16 * ks + 8 * h, q_ok);
    of[ks] = load_frag(dO + b * sd.gb + hd * sd.gh + (long)q * sd.gl + 16 * ks + 8 * h, q_ok);
  }
  const float lse2 = q_ok ? LSE[(size_t)bh * L + q] * kLog2e : INFINITY;
  const float del = q_ok ? delta[(size_t)bh * L + q] : 0.f;
  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) dq[i][r] = 0.f;

  int kv_end = S;
  if (causal) kv_end = min(S, qblk + 32 * NW - 1 + coff + 1);
  const int ntiles = kv_end > 0 ? (kv_end + 63) / 64 : 0;
  float mreg = 0.f;
  auto load_mask = [&](int kv0) {
    if (threadIdx.x < 64) {
      const int key = kv0 + threadIdx.x;
      mreg = key < S ? (HAS_MASK ? mrow[key] * kLog2e : 0.f) : -INFINITY;
    }
  };
  auto store_mask = [&](int buf) {
    if (threadIdx.x < 64) Ms[buf * 64 + threadIdx.x] = mreg;
  };
  if (ntiles > 0) {
    dma_tiles<D, NW>(Kp, Vp, Ks, Vs, 0, S, sd.kl, sd.vl);
    load_mask(0);
    wait_vm0();
    store_mask(0);
  }
  __syncthreads();

  for (int t = 0; t < ntiles; ++t) {
    const int buf = t & 1, kv0 = t * 64;
    if (t + 1 < ntiles) {
      dma_tiles<D, NW>(Kp, Vp, Ks + (buf ^ 1) * 64 * D, Vs + (buf ^ 1) * 64 * D, kv0 + 64, S, sd.kl, sd.vl);
      load_mask(kv0 + 64);
    }
    const bf16_t* kt_ = Ks + buf * 64 * D;
    const bf16_t* vt_ = Vs + buf * 64 * D;
    if (q0 < L && !(causal && kv0 > q0 + 31 + coff)) {
      f32x16 s[2], dp[2];
      const f32x16 z16 = {};
      bf16x8 ka[2][2], va[2][2];
      ka[0][0] = row_frag<D>(kt_, lr, 8 * h);
      ka[0][1] = row_frag<D>(kt_, 32 + lr, 8 * h);
      va[0][0] = row_frag<D>(vt_, lr, 8 * h);
      va[0][1] = row_frag<D>(vt_, 32 + lr, 8 * h);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if (ks + 1 < KS) {
          const int c = 16 * (ks + 1) + 8 * h;
          ka[(ks + 1) & 1][0] = row_frag<D>(kt_, lr, c);
          ka[(ks + 1) & 1][1] = row_frag<D>(kt_, 32 + lr, c);
          va[(ks + 1) & 1][0] = row_frag<D>(vt_, lr, c);
          va[(ks + 1) & 1][1] = row_frag<D>(vt_, 32 + lr, c);
        }
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          s[kt] = mfma32(ka[ks & 1][kt], qf[ks], ks == 0 ? z16 : s[kt]);
          dp[kt] = mfma32(va[ks & 1][kt], of[ks], ks == 0 ? z16 : dp[kt]);
        }
      }
      const bool diag = causal && kv0 + 63 > q0 + coff;
      const float* mk = Ms + buf * 64;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) {
          const int kr = 32 * kt + 8 * i4 + 4 * h;
          const float4 mv = *reinterpret_cast<const float4*>(mk + kr);
          const float ma[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 4 * i4 + r;
            float p = fexp2(s[kt][i] * c2 + (ma[r] - lse2));
            if (diag && kv0 + kr + r > q + coff) p = 0.f;
            const float kf_ = DROP ? attn_keep(dd, bh, q, kv0 + kr + r) : 1.f;
            dp[kt][i] = p * (dp[kt][i] * kf_ - del);
          }
        }
      bf16x8 sf[4];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) sf[k4] = pack8_acc(dp[k4 >> 1], 8 * (k4 & 1));
      constexpr int NSTEP = 4 * DT;
      bf16x8 fk[2];
      fk[0] = tr_frag32<D>(kt_, 0, 0, lane);
#pragma unroll
      for (int idx = 0; idx < NSTEP; ++idx) {
        if (idx + 1 < NSTEP) fk[(idx + 1) & 1] = tr_frag32<D>(kt_, 16 * ((idx + 1) / DT), 32 * ((idx + 1) % DT), lane);
        dq[idx % DT] = mfma32(fk[idx & 1], sf[idx / DT], dq[idx % DT]);
      }
    }
    if (t + 1 < ntiles) {
      wait_vm0();
      store_mask(buf ^ 1);
    }
    __syncthreads();
  }
  if (!q_ok) return;
  bf16_t* dqr = dQ + b * sd.dqb + hd * sd.dqh + (long)q * sd.dql;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      uint2 w;
      w.x = pack2bf(dq[dt][4 * i4 + 0] * scale, dq[dt][4 * i4 + 1] * scale);
      w.y = pack2bf(dq[dt][4 * i4 + 2] * scale, dq[dt][4 * i4 + 3] * scale);
      *reinterpret_cast<uint2*>(dqr + 32 * dt + 8 * i4 + 4 * h) = w;
    }
}

}  // namespace zoo

using namespace zoo;

template <int D, int NW, bool HM, bool DR>
static void launch_fwd(const void* q, const void* k, const void* v, const float* mask, void* o, float* lse, int B,
                       int H, int L, int S, float scale, int causal, const AttnStrides& sd, const AttnDrop& dd,
                       hipStream_t st) {
  const dim3 grid((L + 32 * NW - 1) / (32 * NW), B * H);
  const size_t smem = (size_t)4 * 64 * D * sizeof(bf16_t) + 2 * 64 * sizeof(float);
  static const bool lds_ok_ = [] {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_fwd_kernel<D, NW, HM, DR>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    return true;
  }();
  (void)lds_ok_;
  hipLaunchKernelGGL((attn_fwd_kernel<D, NW, HM, DR>), grid, dim3(NW * 64), smem, st, (const bf16_t*)q,
                     (const bf16_t*)k, (const bf16_t*)v, mask, (bf16_t*)o, lse, H, L, S, scale, causal, sd, dd);
}

template <int D>
static void launch_fwd_d(const void* q, const void* k, const void* v, const float* mask, void* o, float* lse, int B,
                         int H, int L, int S, float scale, int causal, const AttnStrides& sd, const AttnDrop& dd,
                         hipStream_t st) {
  // 8 waves (256 query rows) share each K/V tile when there are enough rows; dropout is a
  // template flag so the plain kernels keep their register budget (occupancy)
#define ZOO_ATTN_FWD(NW_, HM_, DR_) launch_fwd<D, NW_, HM_, DR_>(q, k, v, mask, o, lse, B, H, L, S, scale, causal, sd, dd, st)
  const bool dr = dd.thresh != 0u;
  if (L >= 256) {
    if (mask) { if (dr) ZOO_ATTN_FWD(8, true, true); else ZOO_ATTN_FWD(8, true, false); }
    else { if (dr) ZOO_ATTN_FWD(8, false, true); else ZOO_ATTN_FWD(8, false, false); }
  } else {
    if (mask) { if (dr) ZOO_ATTN_FWD(4, true, true); else ZOO_ATTN_FWD(4, true, false); }
    else { if (dr) ZOO_ATTN_FWD(4, false, true); else ZOO_ATTN_FWD(4, false, false); }
  }
#undef ZOO_ATTN_FWD
}

static AttnDrop make_drop(float p, uint64_t seed) {
  AttnDrop d;
  d.thresh = p <= 0.f ? 0u : (p >= 1.f ? 0xFFFFFFFFu : (uint32_t)((double)p * 4294967296.0));
  if (p > 0.f && d.thresh == 0u) d.thresh = 1u;
  d.scale = p >= 1.f ? 0.f : 1.f / (1.f - p);
  d.s0 = (uint32_t)seed;
  d.s1 = (uint32_t)(seed >> 32);
  d.off = g_seed_off;
  return d;
}

// strides: 12 element strides (q, k, v, o) x (batch, head, row); nullptr = contiguous [B,H,T,D]
extern "C" hipError_t zoo_attn_fwd(const void* q, const void* k, const void* v, const float* mask, void* o,
                                   float* lse, int B, int H, int L, int S, int D, float scale, int causal,
                                   const long* strides, float pdrop, uint64_t seed, hipStream_t st) {
  const AttnDrop dd = make_drop(pdrop, seed);
  AttnStrides sd;
  if (strides) {
    sd = AttnStrides{strides[0], strides[1], strides[2], strides[3], strides[4], strides[5],
                     strides[6], strides[7], strides[8], strides[9], strides[10], strides[11]};
  } else {
    sd = AttnStrides{(long)H * L * D, (long)L * D, D, (long)H * S * D, (long)S * D, D,
                     (long)H * S * D, (long)S * D, D, (long)H * L * D, (long)L * D, D};
  }
  if (D == 64)
    launch_fwd_d<64>(q, k, v, mask, o, lse, B, H, L, S, scale, causal, sd, dd, st);
  else if (D == 128)
    launch_fwd_d<128>(q, k, v, mask, o, lse, B, H, L, S, scale, causal, sd, dd, st);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int D, bool HM, bool DR, int QW, int NWQ>
static void launch_bwd(const void* dout, const void* q, const void* k, const void* v, const float* mask,
                       const float* lse, const float* delta, void* dq, void* dk, void* dv, int B, int H, int L, int S,
                       float scale, int causal, const AttnBwdStrides& sd, const AttnDrop& dd, hipStream_t st) {
  static const bool lds_ok_ = [] {
    hipError_t e1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_dkdv_kernel<D, QW, HM, DR>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipError_t e2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&attn_bwd_dq_kernel<D, NWQ, HM, DR>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    return e1 == hipSuccess && e2 == hipSuccess;
  }();
  (void)lds_ok_;
  const size_t smem = (size_t)4 * 64 * D * sizeof(bf16_t) + 4 * 64 * sizeof(float);
  // dK/dV: one resident block per CU, persistent over heads (the kernel prefetches the next
  // head); its q-half reduction area follows the tiles
  const size_t smem_kv = smem + (QW == 2 ? (size_t)4 * (D / 32) * 16 * 64 * sizeof(float) : 0) +
                         (D == 64 && QW == 2 ? (size_t)4 * 64 * D * sizeof(bf16_t) : 0);
  static const int ncu = [] {
    int dev = 0, n = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  static const bool pers = true;
  const int nkb = (S + 127) / 128;
  if constexpr (D == 64 && QW == 2) {
    if (pers) {
      static const bool attr = hipFuncSetAttribute(
          reinterpret_cast<const void*>(&attn_bwd_dkdv_pers_kernel<D, QW, HM, DR>),
          hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024) == hipSuccess;
      (void)attr;
      const int gy = std::max(1, std::min(B * H, ncu / std::max(1, nkb)));
      hipLaunchKernelGGL((attn_bwd_dkdv_pers_kernel<D, QW, HM, DR>), dim3(nkb, gy), dim3(256 * QW), smem_kv, st,
                         (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse,
                         delta, (bf16_t*)dk, (bf16_t*)dv, H, L, S, scale, causal, sd, dd, B * H);
    } else {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, QW, HM, DR>), dim3(nkb, B * H), dim3(256 * QW), smem, st,
                         (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse,
                         delta, (bf16_t*)dk, (bf16_t*)dv, H, L, S, scale, causal, sd, dd);
    }
  } else {
    (void)smem_kv;
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, QW, HM, DR>), dim3(nkb, B * H), dim3(256 * QW), smem, st,
                       (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask, (const bf16_t*)dout, lse, delta,
                       (bf16_t*)dk, (bf16_t*)dv, H, L, S, scale, causal, sd, dd);
  }
  hipLaunchKernelGGL((attn_bwd_dq_kernel<D, NWQ, HM, DR>), dim3((L + 32 * NWQ - 1) / (32 * NWQ), B * H),
                     dim3(64 * NWQ), smem, st, (const bf16_t*)q, (const bf16_t*)k, (const bf16_t*)v, mask,
                     (const bf16_t*)dout, lse, delta, (bf16_t*)dq, H, L, S, scale, causal, sd, dd);
}

template <int D>
static void launch_bwd_d(const void* dout, const void* q, const void* k, const void* v, const float* mask,
                         const float* lse, const float* delta, void* dq, void* dk, void* dv, int B, int H, int L,
                         int S, float scale, int causal, const AttnBwdStrides& sd, const AttnDrop& dd,
                         hipStream_t st) {
  // D = 64 fits two waves per SIMD (8-wave blocks); D = 128 keeps one wave per
  // SIMD with the accumulators in AGPRs (the 8-wave form would spill). The dQ pass covers
  // 32 queries per wave: at L <= 128 (BERT s128) an 8-wave block would leave half its waves
  // without queries, so those sequences use 4-wave dQ blocks (two per CU)
  constexpr int QW = D == 64 ? 2 : 1, NWQ = D == 64 ? 8 : 4;
  static const bool small_q = true;
  const bool q4 = D == 64 && small_q && L <= 128;
#define ZOO_ATTN_BWD(HM_, DR_)                                                                                   \
  do {                                                                                                          \
    if (q4)                                                                                                     \
      launch_bwd<D, HM_, DR_, QW, 4>(dout, q, k, v, mask, lse, delta, dq, dk, dv, B, H, L, S, scale, causal, sd,  \
                                     dd, st);                                                                   \
    else                                                                                                        \
      launch_bwd<D, HM_, DR_, QW, NWQ>(dout, q, k, v, mask, lse, delta, dq, dk, dv, B, H, L, S, scale, causal,   \
                                       sd, dd, st);                                                             \
  } while (0)
  const bool dr = dd.thresh != 0u;
  if (mask) { if (dr) ZOO_ATTN_BWD(true, true); else ZOO_ATTN_BWD(true, false); }
  else { if (dr) ZOO_ATTN_BWD(false, true); else ZOO_ATTN_BWD(false, false); }
#undef ZOO_ATTN_BWD
}

// strides: 24 element strides (q, k, v, dO, O, dQ, dK, dV) x (batch, head, row); nullptr = contiguous
extern "C" hipError_t zoo_attn_bwd(const void* dout, const void* q, const void* k, const void* v, const float* mask,
                                   const void* o, const float* lse, float* delta, void* dq, void* dk, void* dv, int B,
                                   int H, int L, int S, int D, float scale, int causal, const long* strides,
                                   float pdrop, uint64_t seed, hipStream_t st) {
  const AttnDrop dd = make_drop(pdrop, seed);
  AttnBwdStrides sd;
  if (strides) {
    long* f = &sd.qb;
    for (int i = 0; i < 24; ++i) f[i] = strides[i];
  } else {
    const long lq[3] = {(long)H * L * D, (long)L * D, D}, lk[3] = {(long)H * S * D, (long)S * D, D};
    sd = AttnBwdStrides{lq[0], lq[1], lq[2], lk[0], lk[1], lk[2], lk[0], lk[1], lk[2], lq[0], lq[1], lq[2],
                        lq[0], lq[1], lq[2], lq[0], lq[1], lq[2], lk[0], lk[1], lk[2], lk[0], lk[1], lk[2]};
  }
  const int rows = B * H * L;
  const int dblocks = (rows * (D / 8) + 255) / 256;
  if (D == 64) {
    hipLaunchKernelGGL(attn_delta_kernel<64>, dim3(dblocks), dim3(256), 0, st, (const bf16_t*)dout,
                       (const bf16_t*)o, delta, rows, H, L, sd);
    launch_bwd_d<64>(dout, q, k, v, mask, lse, delta, dq, dk, dv, B, H, L, S, scale, causal, sd, dd, st);
  } else if (D == 128) {
    hipLaunchKernelGGL(attn_delta_kernel<128>, dim3(dblocks), dim3(256), 0, st, (const bf16_t*)dout,
                       (const bf16_t*)o, delta, rows, H, L, sd);
    launch_bwd_d<128>(dout, q, k, v, mask, lse, delta, dq, dk, dv, B, H, L, S, scale, causal, sd, dd, st);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
