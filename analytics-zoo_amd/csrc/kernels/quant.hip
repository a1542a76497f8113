// int8 quantized inference kernels for CDNA4 (gfx950).
//
// Reference: BigDL `quantize()` (InferenceModelFactory.scala:33,47; ImageModel.scala:133-145;
// SURVEY.md §2.16 HK23): symmetric int8 weights with one scale per output channel,
// activations quantized on the fly, int32 accumulation, fp32 rescale.
//
//   absmax   : one fp32 |x| max of a whole activation tensor (atomicMax on the
//              ordered bit pattern of non-negative floats)
//   im2col_q8: NHWC bf16/fp32 activation -> int8 rows [M = N*P*Q][Kp] with
//              k = (r*S + s)*C + c (the packed weight order), zero padding, Kp = ceil16
//   qgemm    : Y[m][n] = (sum_k A[m][k] * W[n][k]) * sa * sw[n] + bias[n] (+resid) (ReLU)
//              on v_mfma_i32_16x16x64_i8 (64 int8 products per lane-pair per instruction)
#include "common.h"

namespace zoo {

typedef int i32x4 __attribute__((ext_vector_type(4)));

ZOO_DEV float load_act(const void* x, int is_f32, size_t i) {
  return is_f32 ? reinterpret_cast<const float*>(x)[i] : bf2f(reinterpret_cast<const bf16_t*>(x)[i]);
}

__global__ __launch_bounds__(256) void absmax_kernel(const void* __restrict__ x, int is_f32, size_t n,
                                                     float* __restrict__ out) {
  float m = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(load_act(x, is_f32, i)));
  m = warp_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(reinterpret_cast<unsigned int*>(out), __float_as_uint(m));  // m >= 0: uint order == float order
  }
}

// one thread = 4 consecutive k of one row; out int8 [M][Kp]
__global__ __launch_bounds__(256) void im2col_q8_kernel(const void* __restrict__ x, int is_f32,
                                                        const float* __restrict__ amax, int8_t* __restrict__ q,
                                                        int N, int H, int W, int C, int R, int S, int P, int Q,
                                                        int sh, int sw, int ph, int pw, int Kp) {
  const int kq = Kp / 4;
  const size_t total = (size_t)N * P * Q * kq;
  const float inv = amax[0] > 0.f ? 127.f / amax[0] : 0.f;
  const int Ktot = R * S * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t m = i / kq;
    const int k0 = (int)(i - m * kq) * 4;
    const int n = (int)(m / (P * Q));
    const int pq = (int)(m - (size_t)n * P * Q);
    const int p = pq / Q, qq = pq - p * Q;
    uint32_t packed = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = k0 + e;
      int v = 0;
      if (k < Ktot) {
        const int rs = k / C, c = k - rs * C;
        const int r = rs / S, s = rs - r * S;
        const int ih = p * sh - ph + r, iw = qq * sw - pw + s;
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
          const float f = load_act(x, is_f32, (((size_t)n * H + ih) * W + iw) * C + c) * inv;
          v = (int)rintf(fminf(fmaxf(f, -127.f), 127.f));
        }
      }
      packed |= ((uint32_t)(v & 0xff)) << (8 * e);
    }
    reinterpret_cast<uint32_t*>(q + m * Kp)[k0 / 4] = packed;
  }
}

constexpr int QG_BM = 128, QG_BN = 128, QG_BK = 64;

// [128 rows][64 B] tile, 16-byte chunk g of row r stored at chunk g ^ ((r >> 2) & 3)
ZOO_DEV int q_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

__global__ __launch_bounds__(256, 2) void qgemm_kernel(const int8_t* __restrict__ A, const int8_t* __restrict__ Wq,
                                                       const float* __restrict__ amax,
                                                       const float* __restrict__ wscale,
                                                       const float* __restrict__ bias, const void* __restrict__ resid,
                                                       void* __restrict__ Y, int M, int N, int Kp, int relu,
                                                       int out_f32) {
  __shared__ __attribute__((aligned(16))) int8_t As[2][QG_BM * QG_BK];
  __shared__ __attribute__((aligned(16))) int8_t Bs[2][QG_BN * QG_BK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (N + QG_BN - 1) / QG_BN;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (tile / tiles_n) * QG_BM, n0 = (tile % tiles_n) * QG_BN;
  const int nk = (Kp + QG_BK - 1) / QG_BK;

  uint4 ra[2], rb[2];
  auto load = [&](int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, row = idx >> 2, ch = idx & 3;
      const int k = kt * QG_BK + ch * 16;
      const bool kok = k < Kp;
      ra[i] = (m0 + row < M && kok) ? *reinterpret_cast<const uint4*>(A + (size_t)(m0 + row) * Kp + k)
                                    : make_uint4(0, 0, 0, 0);
      rb[i] = (n0 + row < N && kok) ? *reinterpret_cast<const uint4*>(Wq + (size_t)(n0 + row) * Kp + k)
                                    : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = tid + 256 * i, row = idx >> 2, ch = idx & 3;
      *reinterpret_cast<uint4*>(&As[buf][q_off(row, ch)]) = ra[i];
      *reinterpret_cast<uint4*>(&Bs[buf][q_off(row, ch)]) = rb[i];
    }
  };

  i32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = i32x4{0, 0, 0, 0};

  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load(kt + 1);
    i32x4 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      af[i] = *reinterpret_cast<const i32x4*>(&As[buf][q_off(wm * 64 + 16 * i + fr, fg)]);
      bfr[i] = *reinterpret_cast<const i32x4*>(&Bs[buf][q_off(wn * 64 + 16 * i + fr, fg)]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C row = 4*(lane>>4) + r, col = lane & 15
  const float sa = amax[0] / 127.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + 16 * j + fr;
    if (n >= N) continue;
    const float s = sa * wscale[n];
    const float b = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + 16 * i + 4 * fg + r;
        if (m >= M) continue;
        float v = (float)acc[i][j][r] * s + b;
        if (resid) v += bf2f(reinterpret_cast<const bf16_t*>(resid)[(size_t)m * N + n]);
        if (relu) v = fmaxf(v, 0.f);
        if (out_f32)
          reinterpret_cast<float*>(Y)[(size_t)m * N + n] = v;
        else
          reinterpret_cast<bf16_t*>(Y)[(size_t)m * N + n] = f2bf(v);
      }
  }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_absmax(const void* x, int is_f32, size_t n, float* out, hipStream_t st) {
  size_t b = (n + 1023) / 1024;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(absmax_kernel, dim3((unsigned)b), dim3(256), 0, st, x, is_f32, n, out);
  return hipGetLastError();
}

extern "C" hipError_t zoo_im2col_q8(const void* x, int is_f32, const float* amax, void* q, int N, int H, int W,
                                    int C, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int Kp,
                                    hipStream_t st) {
  const size_t total = (size_t)N * P * Q * (Kp / 4);
  size_t b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  hipLaunchKernelGGL(im2col_q8_kernel, dim3((unsigned)b), dim3(256), 0, st, x, is_f32, amax, (int8_t*)q, N, H, W, C,
                     R, S, P, Q, sh, sw, ph, pw, Kp);
  return hipGetLastError();
}

extern "C" hipError_t zoo_qgemm(const void* a, const void* w, const float* amax, const float* wscale,
                                const float* bias, const void* resid, void* y, int M, int N, int Kp, int relu,
                                int out_f32, hipStream_t st) {
  const int tiles = ((M + QG_BM - 1) / QG_BM) * ((N + QG_BN - 1) / QG_BN);
  hipLaunchKernelGGL(qgemm_kernel, dim3(tiles), dim3(256), 0, st, (const int8_t*)a, (const int8_t*)w, amax, wscale,
                     bias, resid, y, M, N, Kp, relu, out_f32);
  return hipGetLastError();
}
