// Shared device helpers for the zoo CDNA4 (gfx950) kernel library.
//
// Everything here is written for MI355X directly: 64-lane wavefronts,
// v_mfma_f32_16x16x32_bf16 matrix cores, 160 KiB LDS per CU and 8 XCDs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ZOO_DEV __device__ __forceinline__

namespace zoo {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;  // raw storage type for bf16 in global memory

constexpr int kWave = 64;

ZOO_DEV float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even f32 -> bf16. Plain cast lowers to v_cvt_pk_bf16_f32 on
// gfx950 and keeps NaNs NaN (MI355X_MICROARCH.md "Correctness boundaries").
ZOO_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

ZOO_DEV uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

ZOO_DEV void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

ZOO_DEV uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2bf(f[0], f[1]);
  r.y = pack2bf(f[2], f[3]);
  r.z = pack2bf(f[4], f[5]);
  r.w = pack2bf(f[6], f[7]);
  return r;
}

// zero a loaded vector on a predicate without a branch or an aggregate select
// (an aggregate `ok ? v : zero` lowers to a scratch-memory select on hipcc)
ZOO_DEV uint4 mask4(uint4 v, bool ok) {
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_uint4(v.x & m, v.y & m, v.z & m, v.w & m);
}
ZOO_DEV uint2 mask2(uint2 v, bool ok) {
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return make_uint2(v.x & m, v.y & m);
}

ZOO_DEV float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

ZOO_DEV float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): blocks b and b+8 share an XCD under round-robin dispatch, so
// give each XCD group a contiguous range of logical tiles -> neighbouring tiles
// (which share operand panels) hit the same L2.
ZOO_DEV int xcd_remap(int orig, int nwg) {
  if (nwg <= 8) return orig;
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + orig / 8;
}

// Contention-spreading per-channel sums (MI355X_MICROARCH.md "Global float
// atomics": every workgroup adding into ONE row runs ~14x below the atomic
// rate). buf = [n2 final][nslot x n2 partial][pad], zero-initialised; a block
// adds its partials into slot blockIdx % nslot and zoo_stats_finalize (a tiny
// follow-up kernel on the same stream) folds the slots into buf[0..n2).
ZOO_DEV float* slot_ptr(float* buf, int n2, int nslot) {
  return buf + (size_t)n2 * (1 + (int)(blockIdx.x % (unsigned)nslot));
}

ZOO_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Activation codes shared with the Python side (zoo/ops/_codes.py).
enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2, ACT_SIGMOID = 3, ACT_TANH = 4 };

// GELU (erf form) on the fast path: erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, under
// fp32 / bf16 output precision) with the hardware exp and reciprocal -- branch-free, ~15 VALU
// ops where ocml's erff runs range-split polynomials (the GELU passes of a BERT step were
// VALU-bound on it: profiles/bert_base_train_b128_r2.md act_kernel_v8 / act_colsum_kernel<2>).
// The Gaussian factor exp(-x^2/2) is shared by the CDF and the density of the derivative.
ZOO_DEV void gelu_parts(float x, float& cdf, float& dens) {
  const float u = x * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, fabsf(u), 1.f));
  const float e = __expf(-u * u);
  const float p =
      t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f), 0.254829592f);
  const float q = 0.5f * p * e;            // 0.5 * erfc(|u|)
  cdf = u < 0.f ? q : 1.f - q;
  dens = 0.39894228040143268f * e;         // phi(x)
}
ZOO_DEV float gelu_f(float x) {
  float c, d;
  gelu_parts(x, c, d);
  return x * c;
}
ZOO_DEV float gelu_grad_f(float x) {
  float c, d;
  gelu_parts(x, c, d);
  return fmaf(x, d, c);
}

ZOO_DEV float apply_act(float x, int act) {
  switch (act) {
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_GELU: return gelu_f(x);
    case ACT_SIGMOID: return 1.f / (1.f + __expf(-x));
    case ACT_TANH: return tanhf(x);
    default: return x;
  }
}

// per-step dropout seed offset (device uint32, set by zoo_set_seed_offset in pointwise.hip): every
// dropout kernel xors it into its host seed, so a hipGraph-captured step that replays baked host
// seeds still draws a fresh mask each step (the host stages a new offset before every replay)
extern const uint32_t* g_seed_off;
// CUs reserved for the weight-gradient side stream while it runs on a CU-masked stream
// (zoo_set_reserved_cus, pw.hip): persistent kernels size their grids to the remaining CUs
extern int g_reserved_cus;

}  // namespace zoo
