// MFMA issue-rate probe (gfx950): cycles per v_mfma_f32_16x16x32_bf16 at one wave per SIMD for
// the operand arrangements the conv kernels use, from s_memtime stamps.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_probe tools/mfma_probe.hip && /tmp/mfma_probe
// Variants: 0 = 28 MFMAs per step on 14 accumulators (A 7 frags x 2 halves, B 2 frags), operands
// in registers; 1 = same + one ds_read_b128 per MFMA gap (14 per step, next step's A); 2 = 32x32x16
// reference (7 MFMAs per step on 7 accumulators... same FLOP as 28 16x16x32).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int V>
__global__ __launch_bounds__(256, 1) void probe(const bf16x8* __restrict__ src, float* __restrict__ out,
                                                unsigned long long* __restrict__ cyc, int steps) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;
  bf16x8 a[2][2][7], b[2];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int i = 0; i < 7; ++i) a[0][k][i] = a[1][k][i] = src[(k * 7 + i) * 64 + lane];
  b[0] = src[14 * 64 + lane];
  b[1] = src[15 * 64 + lane];
  for (int i = threadIdx.x; i < 16384; i += 256) reinterpret_cast<float4*>(lds)[i] = make_float4(1.f, 2.f, 3.f, 4.f);
  __syncthreads();
  f32x4 acc[7][2];
#pragma unroll
  for (int i = 0; i < 7; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x16 acc32[7];
#pragma unroll
  for (int i = 0; i < 7; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc32[i][e] = 0.f;
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  // two steps per iteration so the A double buffer is indexed with constants (a runtime
  // index into a register array would put it in scratch memory)
  auto body = [&](const int cur, const int st) {
    if constexpr (V == 2) {
#pragma unroll
      for (int i = 0; i < 7; ++i)
        acc32[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0][0][i], b[0], acc32[i], 0, 0, 0);
    } else {
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int k = 0; k < 28; ++k) {
        const int kk = k / 14, i = (k % 14) / 2, j = k % 2;
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[cur][kk][i], b[j], acc[i][j], 0, 0, 0);
        if (V == 1 && k >= 14) {
          const int ri = (k - 14) >> 1, rk = k & 1;
          a[cur ^ 1][rk][ri] = *reinterpret_cast<const bf16x8*>(lds + ((lane * 16 + ri * 1024 + rk * 64 + st * 128) & 0xffff));
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  for (int st = 0; st < steps; st += 2) {
    body(0, st);
    body(1, st + 1);
  }
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    s += acc[i][0][0] + acc[i][1][1];
    s += acc32[i][0];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int grid = 256, steps = 2000;
  bf16x8* src;
  float* out;
  unsigned long long* cyc;
  hipMalloc(&src, 16 * 64 * sizeof(bf16x8));
  hipMemset(src, 0x3c, 16 * 64 * sizeof(bf16x8));  // ~1.0 bf16 patterns, non-zero
  hipMalloc(&out, grid * 256 * sizeof(float));
  hipMalloc(&cyc, grid * sizeof(unsigned long long));
  unsigned long long h[256];
  const char* names[3] = {"16x16x32, regs only", "16x16x32 + ds_read_b128 per gap", "32x32x16, regs only"};
  for (int v = 0; v < 3; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      if (v == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(256), 65536, 0, src, out, cyc, steps);
      if (v == 1) hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(256), 65536, 0, src, out, cyc, steps);
      if (v == 2) hipLaunchKernelGGL(probe<2>, dim3(grid), dim3(256), 65536, 0, src, out, cyc, steps);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < grid; ++i) m += h[i];
    m /= grid;
    const double per = v == 2 ? m / (steps * 7.0) : m / (steps * 28.0);
    printf("%-34s %8.2f cycles per MFMA (%s)\n", names[v], per, v == 2 ? "32x32x16" : "16x16x32");
  }
  return 0;
}
