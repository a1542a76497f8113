// Pointwise / reduction kernels for the Keras layers, objectives and metrics (gfx950):
//
//   * activations fwd + bwd (HK13): the Keras activation table (relu, relu6, elu, selu, gelu
//     erf/tanh, sigmoid, hard_sigmoid, tanh, softplus, softsign, swish, log_sigmoid,
//     tanh_shrink, exponential, leaky_relu); backward recomputes from x, nothing is stored
//     but the input (Zs/pipeline/api/keras/layers/Activation.scala + BigDL nn activations);
//   * dropout (HK16): counter-hash keep-mask (same hash as nn_misc.hip dropout_add), fp32 and
//     bf16, mask regenerated in backward;
//   * elementwise objectives (HK20): loss and d loss / d pred in ONE pass -- the gradient is
//     written during the forward (mean reduction known up front), the loss sum is a wave
//     reduction + one atomic per block (Zs/pipeline/api/keras/objectives/*.scala:
//     MeanSquaredError, MeanAbsoluteError, BinaryCrossEntropy, Hinge, SquaredHinge, Poisson,
//     MeanAbsolutePercentageError, MeanSquaredLogarithmicError, KullbackLeiblerDivergence,
//     and smooth-L1 / BCE-with-logits);
//   * threshold AUC (HK14): the reference's AUC metric counts TP/FP over fixed thresholds
//     (Zs/pipeline/api/keras/metrics/AUC.scala:128-211); here one pass bins every score
//     into per-block LDS histograms of positives/negatives, merged with global atomics;
//   * SSD box decode (HK21): loc offsets + priors (+ variances) -> corner boxes
//     (Zs/models/image/objectdetection/common/BboxUtil.scala decodeBoxes).
#include "common.h"

namespace zoo {

enum PwAct : int {
  PW_RELU = 0, PW_RELU6, PW_ELU, PW_SELU, PW_GELU, PW_GELU_TANH, PW_SIGMOID, PW_HARD_SIGMOID, PW_TANH,
  PW_SOFTPLUS, PW_SOFTSIGN, PW_SWISH, PW_LOG_SIGMOID, PW_TANH_SHRINK, PW_EXP, PW_LEAKY_RELU
};

ZOO_DEV float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

ZOO_DEV float act_f(float x, int a, float alpha) {
  switch (a) {
    case PW_RELU: return fmaxf(x, 0.f);
    case PW_RELU6: return fminf(fmaxf(x, 0.f), 6.f);
    case PW_ELU: return x > 0.f ? x : alpha * (__expf(x) - 1.f);
    case PW_SELU: return 1.0507009873554805f * (x > 0.f ? x : 1.6732632423543772f * (__expf(x) - 1.f));
    case PW_GELU: return gelu_f(x);
    case PW_GELU_TANH: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case PW_SIGMOID: return sigm(x);
    case PW_HARD_SIGMOID: return fminf(fmaxf(0.2f * x + 0.5f, 0.f), 1.f);
    case PW_TANH: return tanhf(x);
    case PW_SOFTPLUS: return x > 20.f ? x : log1pf(__expf(x));
    case PW_SOFTSIGN: return x / (1.f + fabsf(x));
    case PW_SWISH: return x * sigm(x);
    case PW_LOG_SIGMOID: return x < 0.f ? x - log1pf(__expf(x)) : -log1pf(__expf(-x));
    case PW_TANH_SHRINK: return x - tanhf(x);
    case PW_EXP: return __expf(x);
    case PW_LEAKY_RELU: return x > 0.f ? x : alpha * x;
    default: return x;
  }
}

// d act / dx at x
ZOO_DEV float act_d(float x, int a, float alpha) {
  switch (a) {
    case PW_RELU: return x > 0.f ? 1.f : 0.f;
    case PW_RELU6: return (x > 0.f && x < 6.f) ? 1.f : 0.f;
    case PW_ELU: return x > 0.f ? 1.f : alpha * __expf(x);
    case PW_SELU: return 1.0507009873554805f * (x > 0.f ? 1.f : 1.6732632423543772f * __expf(x));
    case PW_GELU: return gelu_grad_f(x);
    case PW_GELU_TANH: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      const float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * 0.7978845608028654f * (1.f + 0.134145f * x * x);
    }
    case PW_SIGMOID: { const float s = sigm(x); return s * (1.f - s); }
    case PW_HARD_SIGMOID: return (x >= -2.5f && x <= 2.5f) ? 0.2f : 0.f;  // clamp: inclusive ends
    case PW_TANH: { const float t = tanhf(x); return 1.f - t * t; }
    case PW_SOFTPLUS: return sigm(x);
    case PW_SOFTSIGN: { const float d = 1.f + fabsf(x); return 1.f / (d * d); }
    case PW_SWISH: { const float s = sigm(x); return s * (1.f + x * (1.f - s)); }
    case PW_LOG_SIGMOID: return 1.f - sigm(x);
    case PW_TANH_SHRINK: { const float t = tanhf(x); return t * t; }
    case PW_EXP: return __expf(x);
    case PW_LEAKY_RELU: return x > 0.f ? 1.f : alpha;
    default: return 1.f;
  }
}

template <typename T>
ZOO_DEV float ldf(const T* p, size_t i) {
  if constexpr (sizeof(T) == 4) return p[i];
  else return bf2f(p[i]);
}
template <typename T>
ZOO_DEV void stf(T* p, size_t i, float v) {
  if constexpr (sizeof(T) == 4) p[i] = v;
  else p[i] = f2bf(v);
}

// y = act(x)  or (dy != null) dx = dy * act'(x)
template <typename T>
__global__ __launch_bounds__(256) void act_kernel(const T* __restrict__ x, const T* __restrict__ dy, T* __restrict__ out,
                                                  size_t n, int a, float alpha) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = ldf(x, i);
    stf(out, i, dy ? ldf(dy, i) * act_d(v, a, alpha) : act_f(v, a, alpha));
  }
}

// 8 elements per thread with 16-byte loads/stores (n % 8 == 0, 16-byte aligned pointers)
template <typename T>
ZOO_DEV void ld8(const T* p, size_t i8, float* v) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = reinterpret_cast<const float4*>(p)[2 * i8], b = reinterpret_cast<const float4*>(p)[2 * i8 + 1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    unpack8(reinterpret_cast<const uint4*>(p)[i8], v);
  }
}
template <typename T>
ZOO_DEV void st8(T* p, size_t i8, const float* v) {
  if constexpr (sizeof(T) == 4) {
    reinterpret_cast<float4*>(p)[2 * i8] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[2 * i8 + 1] = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    reinterpret_cast<uint4*>(p)[i8] = pack8(v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void act_kernel_v8(const T* __restrict__ x, const T* __restrict__ dy,
                                                     T* __restrict__ out, size_t n8, int a, float alpha) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    float v[8];
    ld8(x, i, v);
    if (dy) {
      float d[8];
      ld8(dy, i, d);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = d[e] * act_d(v[e], a, alpha);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = act_f(v[e], a, alpha);
    }
    st8(out, i, v);
  }
}

ZOO_DEV uint32_t pw_fmix(uint32_t h) {
  h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13; h *= 0xC2B2AE35u; h ^= h >> 16;
  return h;
}

// out = keep(i) ? x * scale : 0 with keep(i) a counter hash of (seed, i)
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ out, size_t n,
                                                      uint32_t thresh, float scale, uint32_t s0, uint32_t s1,
                                                      const uint32_t* __restrict__ soff) {
  if (soff) s0 ^= *soff;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t base = pw_fmix((uint32_t)(i >> 32) ^ s1);
    const uint32_t h = pw_fmix((uint32_t)i * 0x9E3779B1u ^ s0 ^ base);
    stf(out, i, h >= thresh ? ldf(x, i) * scale : 0.f);
  }
}

enum PwLoss : int {
  L_MSE = 0, L_MAE, L_SMOOTH_L1, L_BCE, L_BCE_LOGITS, L_HINGE, L_SQ_HINGE, L_POISSON, L_MAPE, L_MSLE, L_KLD
};

// per-element loss l and dl/dp (p = prediction, t = target)
ZOO_DEV void loss_pt(float p, float t, int k, float beta, float* l, float* d) {
  const float eps = 1e-7f;
  switch (k) {
    case L_MSE: { const float e = p - t; *l = e * e; *d = 2.f * e; break; }
    case L_MAE: { const float e = p - t; *l = fabsf(e); *d = e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f); break; }
    case L_SMOOTH_L1: {
      const float e = p - t, ae = fabsf(e);
      if (ae < beta) { *l = 0.5f * e * e / beta; *d = e / beta; }
      else { *l = ae - 0.5f * beta; *d = e > 0.f ? 1.f : -1.f; }
      break;
    }
    case L_BCE: {
      const float q = fminf(fmaxf(p, eps), 1.f - eps);
      *l = -(t * logf(q) + (1.f - t) * logf(1.f - q));
      *d = (p > eps && p < 1.f - eps) ? (q - t) / (q * (1.f - q)) : 0.f;
      break;
    }
    case L_BCE_LOGITS: {
      *l = fmaxf(p, 0.f) - p * t + log1pf(__expf(-fabsf(p)));
      *d = sigm(p) - t;
      break;
    }
    // (beta is the margin for the hinge losses, the transition point for smooth-L1)
    case L_HINGE: { const float m = beta - p * t; *l = fmaxf(m, 0.f); *d = m > 0.f ? -t : 0.f; break; }
    case L_SQ_HINGE: { const float m = fmaxf(beta - p * t, 0.f); *l = m * m; *d = -2.f * m * t; break; }
    case L_POISSON: { *l = p - t * logf(p + eps); *d = 1.f - t / (p + eps); break; }
    case L_MAPE: {
      const float den = fmaxf(fabsf(t), eps), e = p - t;
      *l = 100.f * fabsf(e) / den;
      *d = 100.f * (e > 0.f ? 1.f : (e < 0.f ? -1.f : 0.f)) / den;
      break;
    }
    case L_MSLE: {
      const float a = logf(fmaxf(p, eps) + 1.f), b = logf(fmaxf(t, eps) + 1.f), e = a - b;
      *l = e * e;
      *d = p > eps ? 2.f * e / (fmaxf(p, eps) + 1.f) : 0.f;
      break;
    }
    case L_KLD: {
      const float tt = fminf(fmaxf(t, eps), 1.f), pp = fminf(fmaxf(p, eps), 1.f);
      *l = tt * logf(tt / pp);
      *d = (p > eps && p < 1.f) ? -tt / pp : 0.f;
      break;
    }
    default: *l = 0.f; *d = 0.f;
  }
}

// loss_sum += sum_i w * l(p_i, t_i);  grad_i = w * dl/dp_i * gscale   (w = 1 / N for mean)
template <typename T>
__global__ __launch_bounds__(256) void loss_kernel(const T* __restrict__ p, const T* __restrict__ t,
                                                   T* __restrict__ grad, float* __restrict__ loss_sum, size_t n,
                                                   int kind, float beta, float w) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float l, d;
    loss_pt(ldf(p, i), ldf(t, i), kind, beta, &l, &d);
    acc += l;
    if (grad) stf(grad, i, d * w);
  }
  acc = warp_sum(acc);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss_sum, ((red[0] + red[1]) + (red[2] + red[3])) * w);
}

// per-block LDS histograms of positives / negatives over `nbins` equal-width score bins in
// [lo, hi]; hist = [2][nbins] float counts (weights)
__global__ __launch_bounds__(256) void auc_hist_kernel(const float* __restrict__ score,
                                                       const float* __restrict__ label, float* __restrict__ hist,
                                                       size_t n, int nbins, float lo, float hi) {
  extern __shared__ float sh[];
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x) sh[i] = 0.f;
  __syncthreads();
  const float inv = (float)nbins / fmaxf(hi - lo, 1e-30f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    int b = (int)((score[i] - lo) * inv);
    b = b < 0 ? 0 : (b >= nbins ? nbins - 1 : b);
    atomicAdd(&sh[(label[i] > 0.5f ? 0 : nbins) + b], 1.f);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x)
    if (sh[i] != 0.f) atomicAdd(hist + i, sh[i]);
}

// boxes[n][j] = corners of prior j shifted by loc[n][j] (center-size coding with variances)
__global__ __launch_bounds__(256) void box_decode_kernel(const float* __restrict__ loc, const float* __restrict__ priors,
                                                         float* __restrict__ boxes, int N, int P, float v0, float v1,
                                                         int clip) {
  const int total = N * P;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int j = i % P;
    const float4 l = reinterpret_cast<const float4*>(loc)[i];
    const float4 pr = reinterpret_cast<const float4*>(priors)[j];  // (cx, cy, w, h)
    const float cx = pr.x + l.x * v0 * pr.z, cy = pr.y + l.y * v0 * pr.w;
    const float w = pr.z * __expf(l.z * v1), h = pr.w * __expf(l.w * v1);
    float4 b = make_float4(cx - 0.5f * w, cy - 0.5f * h, cx + 0.5f * w, cy + 0.5f * h);
    if (clip) {
      b.x = fminf(fmaxf(b.x, 0.f), 1.f); b.y = fminf(fmaxf(b.y, 0.f), 1.f);
      b.z = fminf(fmaxf(b.z, 0.f), 1.f); b.w = fminf(fmaxf(b.w, 0.f), 1.f);
    }
    reinterpret_cast<float4*>(boxes)[i] = b;
  }
}

static int pw_grid(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b ? b : 1);
}

}  // namespace zoo

using namespace zoo;

const uint32_t* zoo::g_seed_off = nullptr;
extern "C" void zoo_set_seed_offset(const uint32_t* p) { zoo::g_seed_off = p; }

extern "C" hipError_t zoo_act(const void* x, const void* dy, void* out, size_t n, int f32, int a, float alpha,
                              hipStream_t st) {
  const bool al = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(dy) |
                    reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (n % 8 == 0 && al) {
    const size_t n8 = n / 8;
    if (f32)
      hipLaunchKernelGGL(act_kernel_v8<float>, dim3(pw_grid(n8)), dim3(256), 0, st, (const float*)x,
                         (const float*)dy, (float*)out, n8, a, alpha);
    else
      hipLaunchKernelGGL(act_kernel_v8<bf16_t>, dim3(pw_grid(n8)), dim3(256), 0, st, (const bf16_t*)x,
                         (const bf16_t*)dy, (bf16_t*)out, n8, a, alpha);
    return hipGetLastError();
  }
  if (f32)
    hipLaunchKernelGGL(act_kernel<float>, dim3(pw_grid(n)), dim3(256), 0, st, (const float*)x, (const float*)dy,
                       (float*)out, n, a, alpha);
  else
    hipLaunchKernelGGL(act_kernel<bf16_t>, dim3(pw_grid(n)), dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)dy,
                       (bf16_t*)out, n, a, alpha);
  return hipGetLastError();
}

extern "C" hipError_t zoo_dropout(const void* x, void* out, size_t n, int f32, float p, uint64_t seed,
                                  hipStream_t st) {
  const uint32_t thresh = p >= 1.f ? 0xFFFFFFFFu : (uint32_t)((double)p * 4294967296.0);
  const float scale = p >= 1.f ? 0.f : 1.f / (1.f - p);
  const uint32_t s0 = (uint32_t)seed, s1 = (uint32_t)(seed >> 32);
  if (f32)
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(pw_grid(n)), dim3(256), 0, st, (const float*)x, (float*)out, n,
                       thresh, scale, s0, s1, g_seed_off);
  else
    hipLaunchKernelGGL(dropout_kernel<bf16_t>, dim3(pw_grid(n)), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)out, n, thresh, scale, s0, s1, g_seed_off);
  return hipGetLastError();
}

extern "C" hipError_t zoo_loss(const void* p, const void* t, void* grad, float* loss_sum, size_t n, int f32, int kind,
                               float beta, float w, hipStream_t st) {
  const int blocks = pw_grid(n) < 2048 ? pw_grid(n) : 2048;
  if (f32)
    hipLaunchKernelGGL(loss_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)p, (const float*)t,
                       (float*)grad, loss_sum, n, kind, beta, w);
  else
    hipLaunchKernelGGL(loss_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)p, (const bf16_t*)t,
                       (bf16_t*)grad, loss_sum, n, kind, beta, w);
  return hipGetLastError();
}

extern "C" hipError_t zoo_auc_hist(const float* score, const float* label, float* hist, size_t n, int nbins, float lo,
                                   float hi, hipStream_t st) {
  const int blocks = pw_grid(n) < 1024 ? pw_grid(n) : 1024;
  hipLaunchKernelGGL(auc_hist_kernel, dim3(blocks), dim3(256), 2 * nbins * sizeof(float), st, score, label, hist, n,
                     nbins, lo, hi);
  return hipGetLastError();
}

extern "C" hipError_t zoo_box_decode(const float* loc, const float* priors, float* boxes, int N, int P, float v0,
                                     float v1, int clip, hipStream_t st) {
  hipLaunchKernelGGL(box_decode_kernel, dim3(pw_grid((size_t)N * P)), dim3(256), 0, st, loc, priors, boxes, N, P, v0,
                     v1, clip);
  return hipGetLastError();
}
