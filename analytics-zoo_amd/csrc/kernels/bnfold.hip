// BatchNorm backward as a PROLOGUE of the unit's own data-gradient GEMM (gfx950).
//
// A training-mode conv -> BN(-> ReLU) unit whose consumer already produced the ReLU-masked
// output gradient g and its per-channel sums S1 = sum g, S2 = sum g * xhat (the consumer's fused
// dgrad epilogue) needs, for its own backward,
//     dy = A o g + B o y + Cc,   A = gamma * inv,  B = -A * inv * S2 / M,
//                                Cc = A * (mean * inv * S2 / M - S1 / M)
// (the BN backward, bn.hip bn_bwd_apply) as the A operand of its dgrad GEMM and as the dY
// operand of its wgrad. Materialising dy costs a pass that reads g and y and writes dy, and the
// dgrad then reads dy again: 8 bytes per element. With the prologue the 1x1 streaming kernel
// (pw.hip, PRO; 64-channel units) reads g and y straight into its operand registers, forms dy
// there with the coefficients below, feeds the MFMAs and writes dy once for the weight gradient:
// 6 bytes per element and one launch (plus its tail) less per unit.
//
// bnfold_coef_kernel:  (A | B | Cc) [3K], dgamma += S2, dbeta += S1
// bnpro_apply_kernel:  dy = A o g + B o y + Cc materialised (shapes the prologue kernel does not
//                      take: the GEMM then reads dy as before)
//
// An algebraic variant that also removed dy from the weight gradient (dW = diag(A) g^T x +
// diag(B) W x^T x + Cc (x) sum x, and dx = g diag(A) W + x W^T diag(B) W + cvec) was measured
// slower: its C x C GEMMs on the data-gradient chain cost what the apply pass did
// (profiles/r5/ab_bnfold_algebraic_r5.md).
// Reference parity: SpatialBatchNormalization.backward after SpatialConvolution in the BigDL
// ResNet-50 bottleneck.
#include "common.h"

namespace zoo {

__global__ __launch_bounds__(256) void bnfold_coef_kernel(int K, const float* __restrict__ gamma,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ inv,
                                                          const float* __restrict__ sums, float invM,
                                                          float* __restrict__ coef, float* __restrict__ dgamma,
                                                          float* __restrict__ dbeta) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const float is = inv[k], a = (gamma ? gamma[k] : 1.f) * is;
  const float m1 = sums[k] * invM, m2 = sums[K + k] * invM;
  coef[k] = a;
  coef[K + k] = -a * is * m2;
  coef[2 * K + k] = a * (mean[k] * is * m2 - m1);
  if (dgamma) dgamma[k] += sums[K + k];
  if (dbeta) dbeta[k] += sums[k];
}

// grid-stride over 8-channel chunks of rows; each thread keeps one fixed chunk's coefficients
// (blockDim.x threads cover the row in chunks: K / 8 <= 256 chunks per row here)
__global__ __launch_bounds__(256) void bnpro_apply_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                                          const float* __restrict__ coef, bf16_t* __restrict__ dy,
                                                          long long rows, int K, int relu) {
  const int cpr = K / 8;                        // chunks per row
  const int rpb = blockDim.x / cpr;             // rows per block step (launcher: cpr <= 256, divides 256)
  const int ch = threadIdx.x % cpr, r0 = threadIdx.x / cpr;
  if (r0 >= rpb) return;
  const int k0 = ch * 8;
  float ca[8], cb[8], cc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ca[e] = coef[k0 + e];
    cb[e] = coef[K + k0 + e];
    cc[e] = coef[2 * K + k0 + e];
  }
  for (long long r = (long long)blockIdx.x * rpb + r0; r < rows; r += (long long)gridDim.x * rpb) {
    const size_t off = (size_t)r * K + k0;
    float gv[8], yv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(g + off), gv);
    unpack8(*reinterpret_cast<const uint4*>(y + off), yv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = ca[e] * gv[e] + cb[e] * yv[e] + cc[e];
      if (relu) o[e] = fmaxf(o[e], 0.f);
    }
    *reinterpret_cast<uint4*>(dy + off) = pack8(o);
  }
}

// any K % 8 == 0: grid-stride over 8-channel chunks (coefficients re-read per chunk)
__global__ __launch_bounds__(256) void bnpro_apply_any_kernel(const bf16_t* __restrict__ g,
                                                              const bf16_t* __restrict__ y,
                                                              const float* __restrict__ coef,
                                                              bf16_t* __restrict__ dy, size_t n8, int K, int relu) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const int k0 = (int)((i * 8) % K);
    float gv[8], yv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(g + i * 8), gv);
    unpack8(*reinterpret_cast<const uint4*>(y + i * 8), yv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o[e] = coef[k0 + e] * gv[e] + coef[K + k0 + e] * yv[e] + coef[2 * K + k0 + e];
      if (relu) o[e] = fmaxf(o[e], 0.f);
    }
    *reinterpret_cast<uint4*>(dy + i * 8) = pack8(o);
  }
}

// the residual unit's apply where the consumer cannot take the EPI 4 prologue (pw.hip):
// z = relu(A y + Cc + R), R = r or rA r + rC (rcoef = rA | - | rC of a projection shortcut's
// BatchNorm), and the unit's 1-bit ReLU mask (bit e of byte i = element 8 i + e > 0)
__global__ __launch_bounds__(256) void bnres_apply_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                                          const bf16_t* __restrict__ r, const float* __restrict__ rcoef,
                                                          bf16_t* __restrict__ z, uint8_t* __restrict__ mask, size_t n8,
                                                          int K) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const int k0 = (int)((i * 8) % K);
    float yv[8], rv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(y + i * 8), yv);
    unpack8(*reinterpret_cast<const uint4*>(r + i * 8), rv);
    unsigned bits = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float res = rcoef ? rcoef[k0 + e] * rv[e] + rcoef[2 * K + k0 + e] : rv[e];
      const float v = coef[k0 + e] * yv[e] + coef[2 * K + k0 + e] + res;
      bits |= (v > 0.f ? 1u : 0u) << e;
      o[e] = fmaxf(v, 0.f);
    }
    *reinterpret_cast<uint4*>(z + i * 8) = pack8(o);
    if (mask) mask[i] = (uint8_t)bits;
  }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_bnres_apply(const void* y, const float* coef, const void* r, const float* rcoef, void* z,
                                      void* mask, size_t n, int K, hipStream_t st) {
  const size_t n8 = n / 8;
  const int blocks = (int)((n8 + 255) / 256 < 4096 ? (n8 + 255) / 256 : 4096);
  hipLaunchKernelGGL(bnres_apply_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, (const bf16_t*)y, coef,
                     (const bf16_t*)r, rcoef, (bf16_t*)z, (uint8_t*)mask, n8, K);
  return hipGetLastError();
}

extern "C" hipError_t zoo_bnfold_coef(int K, const float* gamma, const float* mean, const float* inv,
                                      const float* sums, long long M, float* coef, float* dgamma, float* dbeta,
                                      hipStream_t st) {
  hipLaunchKernelGGL(bnfold_coef_kernel, dim3((K + 255) / 256), dim3(256), 0, st, K, gamma, mean, inv, sums,
                     1.f / (float)M, coef, dgamma, dbeta);
  return hipGetLastError();
}

// relu: max(., 0) of the result (the forward consumer-side apply's fallback, conv_fwd pro_fwd)
extern "C" hipError_t zoo_bnpro_apply(const void* g, const void* y, const float* coef, void* dy, size_t n, int K,
                                      int relu, hipStream_t st) {
  if (K % 8) return hipErrorInvalidValue;
  const long long rows = (long long)(n / K);
  if (rows == 0) return hipSuccess;
  if (K / 8 > 256 || 256 % (K / 8)) {   // not K = 8 * 2^j <= 2048: the generic chunk loop
    const size_t n8 = n / 8;
    size_t b = (n8 + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(bnpro_apply_any_kernel, dim3((unsigned)b), dim3(256), 0, st, (const bf16_t*)g,
                       (const bf16_t*)y, coef, (bf16_t*)dy, n8, K, relu);
    return hipGetLastError();
  }
  const int rpb = 256 / (K / 8);
  long long blocks = (rows + rpb - 1) / rpb;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(bnpro_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)g,
                     (const bf16_t*)y, coef, (bf16_t*)dy, rows, K, relu);
  return hipGetLastError();
}
