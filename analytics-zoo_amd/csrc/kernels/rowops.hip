// Row-wise ops on gfx950: Softmax / LogSoftmax (forward + backward) and the
// cross-channel local response normalisation (LRN2D / SpatialCrossMapLRN).
//
// Softmax family: one 64-lane wave per row (warp_max / warp_sum over the wave),
// fp32 math, fp32 or bf16 storage. Reference: the Keras Softmax layer
// (Zs/pipeline/api/keras/layers/internal/InternalSoftmax.scala:33-57) and
// LogSoftMax inside BigDL's criteria.
//
// LRN: channels are the innermost (NHWC / [rows][C]) dimension, so the window is
// a contiguous run of one row; one thread per element, the squared-sum window is
// recomputed per element (size <= 9 taps, L1-resident). Reference:
// Zs/pipeline/api/keras/layers/LRN2D.scala (BigDL SpatialCrossMapLRN), HK17.
#include "common.h"

namespace zoo {

template <typename T>
ZOO_DEV float rl(const T* p, size_t i);
template <>
ZOO_DEV float rl<float>(const float* p, size_t i) { return p[i]; }
template <>
ZOO_DEV float rl<bf16_t>(const bf16_t* p, size_t i) { return bf2f(p[i]); }
template <typename T>
ZOO_DEV void rs(T* p, size_t i, float v);
template <>
ZOO_DEV void rs<float>(float* p, size_t i, float v) { p[i] = v; }
template <>
ZOO_DEV void rs<bf16_t>(bf16_t* p, size_t i, float v) { p[i] = f2bf(v); }

// log_out: 0 softmax, 1 log-softmax
template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ X, T* __restrict__ Y, int rows,
                                                          int n, int log_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = X + (size_t)row * n;
  T* y = Y + (size_t)row * n;
  float mx = -INFINITY;
  for (int j = lane; j < n; j += 64) mx = fmaxf(mx, rl(x, j));
  mx = warp_max(mx);
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += __expf(rl(x, j) - mx);
  s = warp_sum(s);
  if (log_out) {
    const float lse = mx + __logf(s);
    for (int j = lane; j < n; j += 64) rs(y, j, rl(x, j) - lse);
  } else {
    const float inv = 1.f / s;
    for (int j = lane; j < n; j += 64) rs(y, j, __expf(rl(x, j) - mx) * inv);
  }
}

// softmax:     dx = y * (dy - sum(dy * y))
// log-softmax: dx = dy - exp(y) * sum(dy)
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ Y, const T* __restrict__ dY,
                                                          T* __restrict__ dX, int rows, int n, int log_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* y = Y + (size_t)row * n;
  const T* dy = dY + (size_t)row * n;
  T* dx = dX + (size_t)row * n;
  float s = 0.f;
  if (log_out) {
    for (int j = lane; j < n; j += 64) s += rl(dy, j);
  } else {
    for (int j = lane; j < n; j += 64) s += rl(dy, j) * rl(y, j);
  }
  s = warp_sum(s);
  if (log_out) {
    for (int j = lane; j < n; j += 64) rs(dx, j, rl(dy, j) - __expf(rl(y, j)) * s);
  } else {
    for (int j = lane; j < n; j += 64) rs(dx, j, rl(y, j) * (rl(dy, j) - s));
  }
}

// S_c = k + alpha/size * sum_{c' in [c-lo, c+hi]} x_c'^2, lo = (size-1)/2, hi = size-1-lo
template <typename T>
ZOO_DEV float lrn_scale(const T* x, int c, int C, int size, float alpha, float k) {
  const int lo = (size - 1) / 2;
  float s = 0.f;
  for (int d = -lo; d < size - lo; ++d) {
    const int cc = c + d;
    if (cc >= 0 && cc < C) {
      const float v = rl(x, cc);
      s += v * v;
    }
  }
  return k + alpha / (float)size * s;
}

template <typename T>
__global__ __launch_bounds__(256) void lrn_fwd_kernel(const T* __restrict__ X, T* __restrict__ Y, size_t rows, int C,
                                                      int size, float alpha, float beta, float k) {
  const size_t total = rows * C;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / C;
    const int c = (int)(i - r * C);
    const T* x = X + r * C;
    rs(Y, i, rl(x, c) * __powf(lrn_scale(x, c, C, size, alpha, k), -beta));
  }
}

// dx_c = dy_c * S_c^-b - 2 a b / size * x_c * sum_{c' : c in win(c')} dy_c' x_c' S_c'^(-b-1)
template <typename T>
__global__ __launch_bounds__(256) void lrn_bwd_kernel(const T* __restrict__ X, const T* __restrict__ dY,
                                                      T* __restrict__ dX, size_t rows, int C, int size, float alpha,
                                                      float beta, float k) {
  const size_t total = rows * C;
  const int lo = (size - 1) / 2, hi = size - 1 - lo;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / C;
    const int c = (int)(i - r * C);
    const T* x = X + r * C;
    const T* dy = dY + r * C;
    float acc = 0.f;
    // c' with c - hi <= c' <= c + lo (c lies in c' 's window [c'-lo, c'+hi])
    for (int cc = c - hi; cc <= c + lo; ++cc) {
      if (cc < 0 || cc >= C) continue;
      const float s = lrn_scale(x, cc, C, size, alpha, k);
      acc += rl(dy, cc) * rl(x, cc) * __powf(s, -beta - 1.f);
    }
    const float sc = lrn_scale(x, c, C, size, alpha, k);
    rs(dX, i, rl(dy, c) * __powf(sc, -beta) - 2.f * alpha * beta / (float)size * rl(x, c) * acc);
  }
}

static int rgrid(size_t work) {
  size_t b = (work + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b ? b : 1);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_softmax_rows(const void* X, void* Y, int rows, int n, int log_out, int is_f32,
                                       hipStream_t st) {
  const int blocks = (rows + 3) / 4;
  if (is_f32)
    hipLaunchKernelGGL(softmax_fwd_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)X, (float*)Y, rows, n,
                       log_out);
  else
    hipLaunchKernelGGL(softmax_fwd_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)X, (bf16_t*)Y,
                       rows, n, log_out);
  return hipGetLastError();
}

extern "C" hipError_t zoo_softmax_rows_bwd(const void* Y, const void* dY, void* dX, int rows, int n, int log_out,
                                           int is_f32, hipStream_t st) {
  const int blocks = (rows + 3) / 4;
  if (is_f32)
    hipLaunchKernelGGL(softmax_bwd_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)Y, (const float*)dY,
                       (float*)dX, rows, n, log_out);
  else
    hipLaunchKernelGGL(softmax_bwd_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)Y,
                       (const bf16_t*)dY, (bf16_t*)dX, rows, n, log_out);
  return hipGetLastError();
}

extern "C" hipError_t zoo_lrn(const void* X, const void* dY, void* out, size_t rows, int C, int size, float alpha,
                              float beta, float k, int backward, int is_f32, hipStream_t st) {
  const size_t total = rows * C;
  if (is_f32) {
    if (backward)
      hipLaunchKernelGGL(lrn_bwd_kernel<float>, dim3(rgrid(total)), dim3(256), 0, st, (const float*)X,
                         (const float*)dY, (float*)out, rows, C, size, alpha, beta, k);
    else
      hipLaunchKernelGGL(lrn_fwd_kernel<float>, dim3(rgrid(total)), dim3(256), 0, st, (const float*)X, (float*)out,
                         rows, C, size, alpha, beta, k);
  } else {
    if (backward)
      hipLaunchKernelGGL(lrn_bwd_kernel<bf16_t>, dim3(rgrid(total)), dim3(256), 0, st, (const bf16_t*)X,
                         (const bf16_t*)dY, (bf16_t*)out, rows, C, size, alpha, beta, k);
    else
      hipLaunchKernelGGL(lrn_fwd_kernel<bf16_t>, dim3(rgrid(total)), dim3(256), 0, st, (const bf16_t*)X,
                         (bf16_t*)out, rows, C, size, alpha, beta, k);
  }
  return hipGetLastError();
}
