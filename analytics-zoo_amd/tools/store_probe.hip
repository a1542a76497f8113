// Store-path probe for the write-heavy 1x1 convolutions (tools/conv1x1_probe.py):
// what does a 128x64-bf16-tile-per-workgroup output pattern achieve on MI355X,
// with / without an LDS round trip and with a matching input read, vs a plain fill?
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/store_probe tools/store_probe.hip && /tmp/store_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int BM = 128, BN = 64;

// MODE bit0: stage through LDS; bit1: read a 128x64 input tile first; bit2: non-temporal stores
template <int MODE>
__global__ __launch_bounds__(256) void tile_store(const uint4* __restrict__ in, uint4* __restrict__ out, int M, int K,
                                                 int Cin) {
  __shared__ uint4 lds[BM * BN / 8];
  const int ntn = K / BN;
  const int tm = blockIdx.x / ntn, tn = blockIdx.x - tm * ntn;
  const int tid = threadIdx.x;
  const int ch = tid % 8, r0 = tid / 8;
  uint4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = make_uint4(tid, i, tm, tn);
  if (MODE & 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = tm * BM + r0 + 32 * i;
      v[i] = in[((size_t)m * Cin) / 8 + ch];
    }
  }
  if (MODE & 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) lds[(r0 + 32 * i) * 8 + (ch ^ (r0 & 7))] = v[i];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = lds[(r0 + 32 * i) * 8 + ((ch + 1) % 8 ^ (r0 & 7))];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = tm * BM + r0 + 32 * i;
    uint4* p = out + ((size_t)m * K + tn * BN) / 8 + ch;
    if (MODE & 4) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      u32x4 w = {v[i].x, v[i].y, v[i].z, v[i].w};
      __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(p));
    } else {
      *p = v[i];
    }
  }
}

__global__ void fill(uint4* out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = make_uint4(1, 2, 3, 4);
}

template <int MODE>
int run(const char* name, const uint4* in, uint4* out, int M, int K, int Cin) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int grid = (M / BM) * (K / BN);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(tile_store<MODE>, dim3(grid), dim3(256), 0, 0, in, out, M, K, Cin);
  hipEventRecord(a);
  const int it = 20;
  for (int i = 0; i < it; ++i) hipLaunchKernelGGL(tile_store<MODE>, dim3(grid), dim3(256), 0, 0, in, out, M, K, Cin);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double us = ms * 1e3 / it;
  const double wbytes = (double)M * K * 2, rbytes = (MODE & 2) ? (double)M * Cin * 2 * (K / BN) : 0;
  printf("%-34s %8.1f us  write %.2f TB/s  total %.2f TB/s\n", name, us, wbytes / us / 1e6, (wbytes + rbytes) / us / 1e6);
  return 0;
}

int main() {
  const int M = 802816, K = 256, Cin = 64;
  uint4 *in, *out;
  CK(hipMalloc(&in, (size_t)M * Cin * 2));
  CK(hipMalloc(&out, (size_t)M * K * 2));
  CK(hipMemset(in, 0, (size_t)M * Cin * 2));
  run<0>("store tiles (regs)", in, out, M, K, Cin);
  run<1>("store tiles (LDS round trip)", in, out, M, K, Cin);
  run<4>("store tiles (nontemporal)", in, out, M, K, Cin);
  run<2>("load A tile + store", in, out, M, K, Cin);
  run<3>("load A + LDS + store", in, out, M, K, Cin);
  run<6>("load A + nt store", in, out, M, K, Cin);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t n = (size_t)M * K * 2 / 16;
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, out, n);
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, out, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("%-34s %8.1f us  write %.2f TB/s\n", "grid-stride fill", ms * 1e3 / 20, (double)M * K * 2 / (ms * 1e3 / 20) / 1e6);
  return 0;
}
