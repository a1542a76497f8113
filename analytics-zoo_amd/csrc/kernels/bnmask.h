// Producer ReLU mask of a fused BN-backward dgrad epilogue (BwdStats.zmode, geom.h).
//
// The mask used to be a re-read of the producer's bf16 ReLU output z (2 bytes per element on
// top of the y read the sums need). For a conv->BN->ReLU unit without a residual add the sign
// of z is a function of y alone, so zmode 1 recomputes it from the y values the epilogue loads
// anyway (0 extra bytes); a unit with a residual add stores a 1-bit mask in its forward apply
// (bn_fwd_apply_kernel, 1/8 byte per element) for zmode 2. Shared by igemm.hip / igemm2.hip.
#pragma once
#include "common.h"
#include "geom.h"

namespace zoo {

// per-lane affine of the 8 columns starting at col0 (zmode 1): v = y * sc + sh, exactly the
// coefficients bn_fwd_apply_kernel derives from the same (mean, invstd, gamma, beta)
ZOO_DEV void bnm_coeffs(const BwdStats& bs, int col0, bool ok, float* sc, float* sh) {
#pragma unroll
  for (int e = 0; e < 8; ++e) { sc[e] = 0.f; sh[e] = 0.f; }
  if (bs.zmode != 1 || !ok) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float is = bs.inv[col0 + e], mu = bs.mean[col0 + e];
    sc[e] = bs.mgamma ? bs.mgamma[col0 + e] * is : is;
    sh[e] = (bs.mbeta ? bs.mbeta[col0 + e] : 0.f) - mu * sc[e];
  }
}

// apply the ReLU mask to v[8] at element offset `off` (8-aligned); yy = the producer's y there
// (used by zmode 1 only)
ZOO_DEV void bnm_apply(const BwdStats& bs, size_t off, const float* yy, const float* sc, const float* sh, float* v) {
  if (bs.zmode == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = yy[e] * sc[e] + sh[e] > 0.f ? v[e] : 0.f;
  } else if (bs.zmode == 2) {
    const unsigned b = reinterpret_cast<const uint8_t*>(bs.z)[off >> 3];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (b >> e) & 1u ? v[e] : 0.f;
  } else if (bs.z) {
    float zz[8];
    unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.z) + off), zz);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = zz[e] > 0.f ? v[e] : 0.f;
  }
}

// bnm_apply with the mask operand already loaded (batched epilogues that issue every pass's
// loads before the first store): mbits = the zmode-2 byte, zv = the zmode-0 z chunk
ZOO_DEV void bnm_apply_pre(const BwdStats& bs, const float* yy, const float* sc, const float* sh, unsigned mbits,
                           const uint4& zv, float* v) {
  if (bs.zmode == 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = yy[e] * sc[e] + sh[e] > 0.f ? v[e] : 0.f;
  } else if (bs.zmode == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (mbits >> e) & 1u ? v[e] : 0.f;
  } else if (bs.z) {
    float zz[8];
    unpack8(zv, zz);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = zz[e] > 0.f ? v[e] : 0.f;
  }
}

}  // namespace zoo
