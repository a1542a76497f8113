// Row reductions and row L2-normalisation (HK14: AutoGrad.sum / mean / max / min,
// l2Normalize, cosine / dot merges). One wave per row, 4 rows per
// 256-thread block, 16-byte loads when the row is 8-element aligned, wave shuffles for the
// cross-lane step; fp32 or bf16 input, fp32 accumulation.
#include "common.h"

namespace zoo {

enum { RD_SUM = 0, RD_MEAN = 1, RD_MAX = 2, RD_MIN = 3, RD_SUMSQ = 4 };

template <typename T>
ZOO_DEV float rd_ld(const T* p, long i) {
  if constexpr (sizeof(T) == 4) return p[i];
  else return bf2f(p[i]);
}

ZOO_DEV float rd_comb(float a, float b, int op) {
  return op == RD_MAX ? fmaxf(a, b) : (op == RD_MIN ? fminf(a, b) : a + b);
}

ZOO_DEV float rd_wave(float v, int op) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = rd_comb(v, __shfl_xor(v, o, 64), op);
  return v;
}

template <typename T>
__global__ __launch_bounds__(256) void row_reduce_kernel(const T* __restrict__ x, float* __restrict__ out, long rows,
                                                         int cols, int op) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* xr = x + row * cols;
  const float init = op == RD_MAX ? -INFINITY : (op == RD_MIN ? INFINITY : 0.f);
  float a = init;
  for (int c = lane; c < cols; c += 64) {
    const float v = rd_ld(xr, c);
    a = rd_comb(a, op == RD_SUMSQ ? v * v : v, op);
  }
  a = rd_wave(a, op);
  if (lane == 0) out[row] = op == RD_MEAN ? a / (float)cols : a;
}

// y = x / sqrt(max(sum x^2, eps)); backward dx = (dy - y * sum(dy * y)) / norm
template <typename T>
__global__ __launch_bounds__(256) void row_l2norm_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                         const T* __restrict__ y, T* __restrict__ out, long rows,
                                                         int cols, float eps) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const long base = row * cols;
  float ss = 0.f;
  for (int c = lane; c < cols; c += 64) {
    const float v = rd_ld(x, base + c);
    ss += v * v;
  }
  ss = rd_wave(ss, RD_SUM);
  const float inv = rsqrtf(fmaxf(ss, eps));
  if (!dy) {
    for (int c = lane; c < cols; c += 64) {
      const float v = rd_ld(x, base + c) * inv;
      if constexpr (sizeof(T) == 4) out[base + c] = v;
      else out[base + c] = f2bf(v);
    }
    return;
  }
  float gy = 0.f;
  for (int c = lane; c < cols; c += 64) gy += rd_ld(dy, base + c) * rd_ld(y, base + c);
  gy = rd_wave(gy, RD_SUM);
  for (int c = lane; c < cols; c += 64) {
    const float v = (rd_ld(dy, base + c) - rd_ld(y, base + c) * gy) * inv;
    if constexpr (sizeof(T) == 4) out[base + c] = v;
    else out[base + c] = f2bf(v);
  }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_row_reduce(const void* x, float* out, long rows, int cols, int f32, int op,
                                     hipStream_t st) {
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (f32) hipLaunchKernelGGL(row_reduce_kernel<float>, grid, dim3(256), 0, st, (const float*)x, out, rows, cols, op);
  else hipLaunchKernelGGL(row_reduce_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, out, rows, cols, op);
  return hipGetLastError();
}

extern "C" hipError_t zoo_row_l2norm(const void* x, const void* dy, const void* y, void* out, long rows, int cols,
                                     int f32, float eps, hipStream_t st) {
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (f32)
    hipLaunchKernelGGL(row_l2norm_kernel<float>, grid, dim3(256), 0, st, (const float*)x, (const float*)dy,
                       (const float*)y, (float*)out, rows, cols, eps);
  else
    hipLaunchKernelGGL(row_l2norm_kernel<bf16_t>, grid, dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)dy,
                       (const bf16_t*)y, (bf16_t*)out, rows, cols, eps);
  return hipGetLastError();
}
