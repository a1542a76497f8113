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
// (pw.hip, PRO) reads g and y straight into its operand registers, forms dy there with the
// coefficients below, feeds the MFMAs and writes dy once for the weight gradient: 6 bytes per
// element and one launch (plus its tail) less per unit.
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

// 8 channels per thread; K % 8 == 0
__global__ __launch_bounds__(256) void bnpro_apply_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                                          const float* __restrict__ coef, bf16_t* __restrict__ dy,
                                                          size_t n8, int K) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    const int k0 = (int)((i * 8) % K);
    float gv[8], yv[8], o[8];
    unpack8(*reinterpret_cast<const uint4*>(g + i * 8), gv);
    unpack8(*reinterpret_cast<const uint4*>(y + i * 8), yv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = coef[k0 + e] * gv[e] + coef[K + k0 + e] * yv[e] + coef[2 * K + k0 + e];
    *reinterpret_cast<uint4*>(dy + i * 8) = pack8(o);
  }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_bnfold_coef(int K, const float* gamma, const float* mean, const float* inv,
                                      const float* sums, long long M, float* coef, float* dgamma, float* dbeta,
                                      hipStream_t st) {
  hipLaunchKernelGGL(bnfold_coef_kernel, dim3((K + 255) / 256), dim3(256), 0, st, K, gamma, mean, inv, sums,
                     1.f / (float)M, coef, dgamma, dbeta);
  return hipGetLastError();
}

extern "C" hipError_t zoo_bnpro_apply(const void* g, const void* y, const float* coef, void* dy, size_t n, int K,
                                      hipStream_t st) {
  const size_t n8 = n / 8;
  size_t blocks = (n8 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(bnpro_apply_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)g,
                     (const bf16_t*)y, coef, (bf16_t*)dy, n8, K);
  return hipGetLastError();
}
