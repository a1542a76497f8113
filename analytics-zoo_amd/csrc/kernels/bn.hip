// BatchNorm for NHWC bf16 activations on gfx950 (training + inference), with
// the residual add and ReLU of ResNet bottlenecks fused into the same pass.
//
// Reference: BigDL BatchNormalization / SpatialBatchNormalization as wrapped by
// Zs/pipeline/api/keras/layers/BatchNormalization.scala:85-110.
//
// Forward (training):
//   stats  = (sum x, sum x^2) per channel — normally produced for free by the
//            producing conv's epilogue (igemm.hip); `bn_reduce` exists for the
//            unfused case;
//   apply  = y = relu?( x*scale + shift (+ residual) ), where every workgroup
//            derives scale/shift from the raw sums itself (no finalize launch),
//            and workgroup 0 updates the running statistics and saves
//            mean/invstd for the backward pass.
// Backward:
//   reduce = (sum dy, sum dy*xhat) with dy = dz * [z > 0] (ReLU mask recomputed
//            from the saved output z), one pass over [M][C];
//   apply  = dx = scale*(dy - mean(dy) - xhat*mean(dy*xhat)); optionally also
//            emits dy for the residual branch; workgroup 0 writes dgamma/dbeta.
// All passes move 8 bf16 per lane (16-byte vector loads, Guideline 13).
#include "common.h"

namespace zoo {

// ---------------------------------------------------------------------------
// channel reduction over [M][C]; mode 0: (x, x^2); mode 1: (dy, dy*xhat)
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const bf16_t* __restrict__ A,    // x or dz
                                                        const bf16_t* __restrict__ Z,    // relu output (mode 1, may be null)
                                                        const bf16_t* __restrict__ Xin,  // conv output x (mode 1)
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        float* __restrict__ out,  // [2][C]
                                                        int M, int C, int rows_per_block) {
  const int cpr = C >> 3;  // 8-channel chunks per row
  const int tid = threadIdx.x;
  // threads are laid out [row_lane][chunk]; if C/8 > 256 a thread walks several chunks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* red = reinterpret_cast<float*>(smem);  // [2][C]
  for (int i = tid; i < 2 * C; i += blockDim.x) red[i] = 0.f;
  __syncthreads();

  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const int lanes_per_row = cpr < 256 ? cpr : 256;
  const int row_step = 256 / lanes_per_row;
  const int my_row = tid / lanes_per_row;
  const int my_chunk0 = tid - my_row * lanes_per_row;
  if (my_row < row_step) {
    for (int chunk = my_chunk0; chunk < cpr; chunk += lanes_per_row) {
      float s1[8], s2[8];
      float mu[8], is[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] = 0.f; s2[e] = 0.f;
        if (MODE == 1) { mu[e] = mean[chunk * 8 + e]; is[e] = invstd[chunk * 8 + e]; }
      }
      for (int r = r0 + my_row; r < r1; r += row_step) {
        const size_t off = (size_t)r * C + chunk * 8;
        float a[8];
        unpack8(*reinterpret_cast<const uint4*>(A + off), a);
        if (MODE == 0) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += a[e]; s2[e] += a[e] * a[e]; }
        } else {
          float x[8];
          unpack8(*reinterpret_cast<const uint4*>(Xin + off), x);
          if (Z) {
            float z[8];
            unpack8(*reinterpret_cast<const uint4*>(Z + off), z);
#pragma unroll
            for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += a[e];
            s2[e] += a[e] * (x[e] - mu[e]) * is[e];
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(&red[chunk * 8 + e], s1[e]);  // LDS atomics: cheap, few per thread
        atomicAdd(&red[C + chunk * 8 + e], s2[e]);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += blockDim.x) atomicAdd(out + i, red[i]);
}

// ---------------------------------------------------------------------------
// forward apply (training): stats -> scale/shift in every block
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_fwd_apply_kernel(
    const bf16_t* __restrict__ X, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, const bf16_t* __restrict__ resid, bf16_t* __restrict__ Y,
    float* __restrict__ running_mean, float* __restrict__ running_var, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, int M, int C, float eps, float momentum, int relu, int training) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* sc = reinterpret_cast<float*>(smem);  // [C] scale
  float* sh = sc + C;                           // [C] shift
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mu, is;
    if (training) {
      mu = stats[c] * invM;
      const float var = fmaxf(stats[C + c] * invM - mu * mu, 0.f);
      is = rsqrtf(var + eps);
      if (blockIdx.x == 0) {
        save_mean[c] = mu;
        save_invstd[c] = is;
        if (running_mean) {
          const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
          running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
          running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
        }
      }
    } else {
      mu = running_mean[c];
      is = rsqrtf(running_var[c] + eps);
    }
    const float s = gamma ? gamma[c] * is : is;
    sc[c] = s;
    sh[c] = (beta ? beta[c] : 0.f) - mu * s;
  }
  __syncthreads();
  const int cpr = C >> 3;
  const size_t total = (size_t)M * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % cpr);
    const size_t off = i * 8;
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(X + off), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[chunk * 8 + e] + sh[chunk * 8 + e];
    if (resid) {
      float r[8];
      unpack8(*reinterpret_cast<const uint4*>(resid + off), r);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += r[e];
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    }
    *reinterpret_cast<uint4*>(Y + off) = pack8(v);
  }
}

// ---------------------------------------------------------------------------
// backward apply
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dZ, const bf16_t* __restrict__ Z, const bf16_t* __restrict__ X,
    const float* __restrict__ save_mean, const float* __restrict__ save_invstd,
    const float* __restrict__ gamma, const float* __restrict__ sums,  // [2][C]: sum dy, sum dy*xhat
    bf16_t* __restrict__ dX, bf16_t* __restrict__ dResid, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int M, int C) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* k1 = reinterpret_cast<float*>(smem);  // scale = gamma*invstd
  float* k2 = k1 + C;                          // mean(dy)
  float* k3 = k2 + C;                          // mean(dy*xhat)
  float* mu = k3 + C;
  float* is = mu + C;
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float g = gamma ? gamma[c] : 1.f;
    is[c] = save_invstd[c];
    mu[c] = save_mean[c];
    k1[c] = g * is[c];
    k2[c] = sums[c] * invM;
    k3[c] = sums[C + c] * invM;
    if (blockIdx.x == 0) {
      if (dgamma) dgamma[c] += sums[C + c];
      if (dbeta) dbeta[c] += sums[c];
    }
  }
  __syncthreads();
  const int cpr = C >> 3;
  const size_t total = (size_t)M * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cb = (int)(i % cpr) * 8;
    const size_t off = i * 8;
    float dy[8], x[8];
    unpack8(*reinterpret_cast<const uint4*>(dZ + off), dy);
    unpack8(*reinterpret_cast<const uint4*>(X + off), x);
    if (Z) {
      float z[8];
      unpack8(*reinterpret_cast<const uint4*>(Z + off), z);
#pragma unroll
      for (int e = 0; e < 8; ++e) dy[e] = z[e] > 0.f ? dy[e] : 0.f;
    }
    if (dResid) *reinterpret_cast<uint4*>(dResid + off) = pack8(dy);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cb + e;
      const float xh = (x[e] - mu[c]) * is[c];
      o[e] = k1[c] * (dy[e] - k2[c] - xh * k3[c]);
    }
    *reinterpret_cast<uint4*>(dX + off) = pack8(o);
  }
}

static int grid_for(size_t work, int per_block) {
  size_t b = (work + per_block - 1) / per_block;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_bn_reduce(const void* A, const void* Z, const void* X, const float* mean,
                                    const float* invstd, float* out, int M, int C, int mode,
                                    hipStream_t st) {
  // ~1024 blocks, each owning a contiguous row range
  int blocks = 1024;
  int rpb = (M + blocks - 1) / blocks;
  if (rpb < 8) rpb = 8;
  blocks = (M + rpb - 1) / rpb;
  const size_t smem = (size_t)2 * C * sizeof(float);
  if (mode == 0)
    hipLaunchKernelGGL(bn_reduce_kernel<0>, dim3(blocks), dim3(256), smem, st, (const bf16_t*)A,
                       (const bf16_t*)Z, (const bf16_t*)X, mean, invstd, out, M, C, rpb);
  else
    hipLaunchKernelGGL(bn_reduce_kernel<1>, dim3(blocks), dim3(256), smem, st, (const bf16_t*)A,
                       (const bf16_t*)Z, (const bf16_t*)X, mean, invstd, out, M, C, rpb);
  return hipGetLastError();
}

extern "C" hipError_t zoo_bn_fwd_apply(const void* X, const float* stats, const float* gamma,
                                       const float* beta, const void* resid, void* Y, float* rmean,
                                       float* rvar, float* smean, float* sinv, int M, int C, float eps,
                                       float momentum, int relu, int training, hipStream_t st) {
  const size_t work = (size_t)M * (C / 8);
  hipLaunchKernelGGL(bn_fwd_apply_kernel, dim3(grid_for(work, 256 * 4)), dim3(256), 2 * C * sizeof(float), st,
                     (const bf16_t*)X, stats, gamma, beta, (const bf16_t*)resid, (bf16_t*)Y, rmean, rvar,
                     smean, sinv, M, C, eps, momentum, relu, training);
  return hipGetLastError();
}

extern "C" hipError_t zoo_bn_bwd_apply(const void* dZ, const void* Z, const void* X, const float* smean,
                                       const float* sinv, const float* gamma, const float* sums, void* dX,
                                       void* dResid, float* dgamma, float* dbeta, int M, int C,
                                       hipStream_t st) {
  const size_t work = (size_t)M * (C / 8);
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_for(work, 256 * 4)), dim3(256), 5 * C * sizeof(float), st,
                     (const bf16_t*)dZ, (const bf16_t*)Z, (const bf16_t*)X, smean, sinv, gamma, sums,
                     (bf16_t*)dX, (bf16_t*)dResid, dgamma, dbeta, M, C);
  return hipGetLastError();
}
