// Losses, fused optimizer updates and small utility kernels (gfx950).
//
//  * softmax + cross-entropy (fused fwd+bwd), with the padding/ignore label of
//    ZooClassNLLCriterion (Zs/pipeline/api/keras/objectives/ZooClassNLLCriterion.scala:28-100)
//  * SGD (momentum / dampening / nesterov / weight decay, BigDL SGD semantics)
//    and Adam (Zs/pipeline/api/keras/optimizers/Adam.scala:59-106, bias corrected)
//    / AdamWeightDecay (AdamWeightDecay.scala:75-124) over ONE flat fp32 master
//    buffer: a single launch updates every parameter of the model and writes
//    the bf16 compute copy in the same pass
//  * global L2-norm partial sums and constant clipping (HK19)
//  * layout/cast helpers (input NCHW fp32 -> NHWC bf16 with channel padding)
#include "common.h"

namespace zoo {

// one wave per row; logits fp32 or bf16
template <typename T>
ZOO_DEV float ld(const T* p, size_t i);
template <>
ZOO_DEV float ld<float>(const float* p, size_t i) { return p[i]; }
template <>
ZOO_DEV float ld<bf16_t>(const bf16_t* p, size_t i) { return bf2f(p[i]); }

template <typename T>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const T* __restrict__ logits,
                                                           const int64_t* __restrict__ labels,
                                                           float* __restrict__ loss_sum,
                                                           float* __restrict__ count,
                                                           T* __restrict__ dlogits, int B, int NC,
                                                           float grad_scale, int ignore_index, int per_row) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* x = logits + (size_t)row * NC;
  float mx = -INFINITY;
  for (int j = lane; j < NC; j += 64) mx = fmaxf(mx, ld(x, j));
  mx = warp_max(mx);
  float s = 0.f;
  for (int j = lane; j < NC; j += 64) s += __expf(ld(x, j) - mx);
  s = warp_sum(s);
  const float lse = mx + __logf(s);
  const int64_t lab = labels[row];
  const bool valid = lab != ignore_index && lab >= 0 && lab < NC;
  if (lane == 0) {
    if (per_row) {  // deterministic mode: per-row terms, summed by the caller in a fixed order
      loss_sum[row] = valid ? lse - ld(x, lab) : 0.f;
      count[row] = valid ? 1.f : 0.f;
    } else if (valid) {
      atomicAdd(loss_sum, lse - ld(x, lab));
      atomicAdd(count, 1.f);
    }
  }
  if (dlogits) {
    const float inv_s = 1.f / s;
    for (int j = lane; j < NC; j += 64) {
      float p = __expf(ld(x, j) - mx) * inv_s;
      if (j == lab) p -= 1.f;
      const float gv = valid ? p * grad_scale : 0.f;
      if constexpr (sizeof(T) == 4) dlogits[(size_t)row * NC + j] = gv;
      else dlogits[(size_t)row * NC + j] = f2bf(gv);
    }
  }
}

// NLL of probabilities (ClassNLLCriterion with log_prob_as_input = false, Zs ClassNLLCriterion /
// keras SparseCategoricalCrossEntropy): loss_i = -log(clamp(p[i, y_i], eps, 1)); one thread per
// row, wave-reduced sums. dp (optional, unscaled) = -1 / p at the label where eps <= p <= 1
// (torch.clamp's pass-through band), 0 elsewhere -- the caller scales it by dloss / count.
template <typename T>
__global__ __launch_bounds__(256) void prob_nll_kernel(const T* __restrict__ probs, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss_sum, float* __restrict__ count,
                                                       float* __restrict__ dp, int B, int NC, float eps,
                                                       int ignore_index, int per_row) {
  // grid-stride over rows; the scalar sums are reduced per block in LDS so a launch issues at
  // most 2 * gridDim same-address atomics (one per wave serialised ~28 us at B = 65536)
  float l = 0.f, c = 0.f;
  for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < B; row += gridDim.x * blockDim.x) {
    const int64_t lab = labels[row];
    const bool valid = lab != ignore_index && lab >= 0 && lab < NC;
    const float p = valid ? ld(probs + (size_t)row * NC, (int)lab) : 1.f;
    const float pc = fminf(fmaxf(p, eps), 1.f);
    const float lr = valid ? -__logf(pc) : 0.f;
    const float cr = valid ? 1.f : 0.f;
    if (dp) {
      const bool pass = valid && p >= eps && p <= 1.f;
      for (int j = 0; j < NC; ++j) dp[(size_t)row * NC + j] = (pass && j == lab) ? -1.f / pc : 0.f;
    }
    if (per_row == 1) {  // (per_row 2: loss_sum / count are the [gridDim] block partials)
      loss_sum[row] = lr;
      count[row] = cr;
    }
    l += lr;
    c += cr;
  }
  if (per_row == 1) return;
  __shared__ float red[2][4];
  l = warp_sum(l);
  c = warp_sum(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = l;
    red[1][w] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    l = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    c = red[1][0] + red[1][1] + red[1][2] + red[1][3];
    if (per_row == 2) {  // block partials, folded in order by prob_nll_finalize_kernel
      loss_sum[blockIdx.x] = l;
      count[blockIdx.x] = c;
    } else if (c > 0.f) {
      atomicAdd(loss_sum, l);
      atomicAdd(count, c);
    }
  }
}

// out[0] = sum(part loss) / max(sum(part count), 1) (or the plain sum), out[1] = count: the
// loss scalar straight from the block partials (no zero-fill of accumulators, no clamp / div
// launches; ordered, so deterministic)
__global__ __launch_bounds__(64) void prob_nll_finalize_kernel(const float* __restrict__ part, int nb,
                                                               float* __restrict__ out, int size_average) {
  float l = 0.f, c = 0.f;
  for (int b = threadIdx.x; b < nb; b += 64) {
    l += part[b];
    c += part[nb + b];
  }
  l = warp_sum(l);
  c = warp_sum(c);
  if (threadIdx.x == 0) {
    out[0] = size_average ? l / fmaxf(c, 1.f) : l;
    out[1] = c;
  }
}

// d loss / d probs of the NLL above, already scaled by the upstream gradient and 1 / count
// (both device scalars): the backward is this one pass, no separate scale kernels
template <typename T>
__global__ __launch_bounds__(256) void prob_nll_grad_kernel(const T* __restrict__ probs,
                                                            const int64_t* __restrict__ labels,
                                                            const float* __restrict__ g, const float* __restrict__ count,
                                                            float* __restrict__ dp, int B, int NC, float eps,
                                                            int ignore_index) {
  const float s = g[0] / fmaxf(count[0], 1.f);
  for (int row = blockIdx.x * blockDim.x + threadIdx.x; row < B; row += gridDim.x * blockDim.x) {
    const int64_t lab = labels[row];
    const bool valid = lab != ignore_index && lab >= 0 && lab < NC;
    const float p = valid ? ld(probs + (size_t)row * NC, (int)lab) : 1.f;
    const bool pass = valid && p >= eps && p <= 1.f;
    const float d = pass ? -s / fminf(fmaxf(p, eps), 1.f) : 0.f;
    for (int j = 0; j < NC; ++j) dp[(size_t)row * NC + j] = j == lab ? d : 0.f;
  }
}

// dlogits * (g / max(count, 1)) in the logits dtype: the softmax-xent backward in one pass (the
// upstream gradient and the count are device scalars; was a div, a mul and a cast launch)
template <typename T>
__global__ __launch_bounds__(256) void xent_grad_scale_kernel(const T* __restrict__ dl, const float* __restrict__ g,
                                                              const float* __restrict__ count, T* __restrict__ out,
                                                              size_t n) {
  const float s = g[0] / fmaxf(count[0], 1.f);
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    if constexpr (sizeof(T) == 4) out[i] = dl[i] * s;
    else out[i] = f2bf(bf2f(dl[i]) * s);
  }
}

// ---------------- optimizers over flat buffers ----------------
// zero_g: the gradient slot is cleared after it is read (the engine's next step then needs no
// fill launch over the flat gradient buffer)
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, float* __restrict__ g,
                                                  float* __restrict__ mom, bf16_t* __restrict__ pbf, size_t n,
                                                  float lr, float momentum, float dampening, float wd,
                                                  int nesterov, float gscale, int first_step, int zero_g,
                                                  const float* __restrict__ hp) {
  if (hp) {  // per-step values from device memory (hipGraph replays of a captured update)
    lr = hp[0];
    first_step = hp[3] != 0.f;
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gscale;
    if (zero_g) g[i] = 0.f;
    float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    if (momentum != 0.f) {
      float b = first_step ? gi : momentum * mom[i] + (1.f - dampening) * gi;
      mom[i] = b;
      gi = nesterov ? gi + momentum * b : b;
    }
    pi -= lr * gi;
    p[i] = pi;
    if (pbf) pbf[i] = f2bf(pi);
  }
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ pbf, size_t n, float lr, float b1,
                                                   float b2, float eps, float wd, float bc1, float bc2,
                                                   float gscale, int decoupled, int zero_g,
                                                   const float* __restrict__ hp) {
  if (hp) {
    lr = hp[0];
    bc1 = hp[1];
    bc2 = hp[2];
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gscale;
    if (zero_g) g[i] = 0.f;
    float pi = p[i];
    if (wd != 0.f && !decoupled) gi += wd * pi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    // Zoo Adam (Adam.scala:93-99): step = lr*sqrt(bc2)/bc1, update = m/(sqrt(v)+eps)
    float upd = mi / (sqrtf(vi) + eps) * (sqrtf(bc2) / bc1);
    if (wd != 0.f && decoupled) upd += wd * pi;
    pi -= lr * upd;
    p[i] = pi;
    if (pbf) pbf[i] = f2bf(pi);
  }
}

// generic "RMSprop / Adagrad / Adadelta / Adamax" family in one kernel
// kind: 0 rmsprop, 1 adagrad, 2 adadelta, 3 adamax
__global__ __launch_bounds__(256) void adaptive_kernel(float* __restrict__ p, float* __restrict__ g,
                                                       float* __restrict__ s1, float* __restrict__ s2,
                                                       bf16_t* __restrict__ pbf, size_t n, int kind, float lr,
                                                       float rho, float rho2, float eps, float wd, float bc1,
                                                       float gscale, int zero_g, const float* __restrict__ hp) {
  if (hp) {
    lr = hp[0];
    bc1 = hp[1];
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float gi = g[i] * gscale;
    if (zero_g) g[i] = 0.f;
    float pi = p[i];
    if (wd != 0.f) gi += wd * pi;
    float upd;
    if (kind == 0) {  // rmsprop
      const float a = rho * s1[i] + (1.f - rho) * gi * gi;
      s1[i] = a;
      upd = lr * gi / (sqrtf(a) + eps);
    } else if (kind == 1) {  // adagrad
      const float a = s1[i] + gi * gi;
      s1[i] = a;
      upd = lr * gi / (sqrtf(a) + eps);
    } else if (kind == 2) {  // adadelta
      const float a = rho * s1[i] + (1.f - rho) * gi * gi;
      const float d = sqrtf(s2[i] + eps) / sqrtf(a + eps) * gi;
      s1[i] = a;
      s2[i] = rho * s2[i] + (1.f - rho) * d * d;
      upd = lr * d;
    } else {  // adamax: s1 = m, s2 = u
      const float mi = rho * s1[i] + (1.f - rho) * gi;  // rho = beta1 here
      const float ui = fmaxf(rho2 * s2[i], fabsf(gi));
      s1[i] = mi;
      s2[i] = ui;
      upd = lr / bc1 * mi / (ui + eps);
    }
    pi -= upd;
    p[i] = pi;
    if (pbf) pbf[i] = f2bf(pi);
  }
}

// sum of squares (global L2 norm) -> atomicAdd into out[0]
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, size_t n, float* __restrict__ out) {
  float s = 0.f;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float v = g[i];
    s += v * v;
  }
  s = warp_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, red[0] + red[1] + red[2] + red[3]);
}

__global__ __launch_bounds__(256) void clip_kernel(float* __restrict__ g, size_t n, float lo, float hi,
                                                   const float* __restrict__ norm_sq, float max_norm) {
  float sc = 1.f;
  if (norm_sq) {
    const float nrm = sqrtf(*norm_sq);
    sc = nrm > max_norm ? max_norm / (nrm + 1e-6f) : 1.f;
  }
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float v = g[i] * sc;
    g[i] = fminf(fmaxf(v, lo), hi);
  }
}

// ---------------- layout / cast helpers ----------------
// NCHW float -> NHWC bf16 with channels padded to Cp (zero fill)
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ X, bf16_t* __restrict__ Y,
                                                           int N, int C, int H, int W, int Cp) {
  const size_t total = (size_t)N * H * W * Cp;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    size_t t = i / Cp;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const float v = c < C ? X[(((size_t)n * C + c) * H + h) * W + w] : 0.f;
    Y[i] = f2bf(v);
  }
}

// NCHW fp32 images -> zero-padded space-to-depth(2) NHWC bf16: Y[n][i][j][(dy*2+dx)*Cp + c] =
// X[n][c][2i+dy-pad][2j+dx-pad]. A 7x7 stride-2 stem conv on X equals a 4x4 stride-1 conv
// on Y (16 channels instead of 4 -> the 16-byte-vector implicit-GEMM path). One thread
// writes the 8 channels of one (pixel, dy): 16 bytes.
__global__ __launch_bounds__(256) void nchw_to_s2d_kernel(const float* __restrict__ X, bf16_t* __restrict__ Y,
                                                          int N, int C, int H, int W, int Cp, int pad, int Hs,
                                                          int Ws) {
  // 32-bit index math (the launcher checks total < 2^31): the 64-bit div / mod of a size_t index
  // are emulated in dozens of instructions each and made this pass ~2.5x its bytes' time
  const unsigned total = (unsigned)N * Hs * Ws * 2;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int dy = (int)(i & 1);
    unsigned t = i >> 1;
    const int j = (int)(t % (unsigned)Ws); t /= (unsigned)Ws;
    const int ii = (int)(t % (unsigned)Hs);
    const int n = (int)(t / (unsigned)Hs);
    const int h = 2 * ii + dy - pad;
    float v[8];
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int w = 2 * j + dx - pad;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        v[dx * 4 + c] = (ok && c < C) ? X[(((size_t)n * C + c) * H + h) * W + w] : 0.f;
    }
    // Cp == 4: the 8 values of (dy, dx=0..1, c=0..3) are contiguous in the output pixel
    *reinterpret_cast<uint4*>(Y + ((((size_t)n * Hs + ii) * Ws + j) * 4 * Cp) + dy * 2 * Cp) = pack8(v);
  }
}

// uint8 NHWC images (the input pipeline's wire format: 1/4 of the fp32 NCHW bytes over PCIe) ->
// normalised, zero-padded space-to-depth(2) NHWC bf16 in one pass: Y[n][i][j][(dy*2+dx)*4 + c] =
// X[n][2i+dy-pad][2j+dx-pad][c] * scale[c] + shift[c] (0 outside the image and for c >= C).
__global__ __launch_bounds__(256) void nhwc_u8_to_s2d_kernel(const uint8_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                             int N, int C, int H, int W, int pad, int Hs, int Ws,
                                                             float4 scale, float4 shift) {
  const unsigned total = (unsigned)N * Hs * Ws * 2;   // 32-bit index math, as nchw_to_s2d_kernel
  const float sc[4] = {scale.x, scale.y, scale.z, scale.w}, sh[4] = {shift.x, shift.y, shift.z, shift.w};
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int dy = (int)(i & 1);
    unsigned t = i >> 1;
    const int j = (int)(t % (unsigned)Ws); t /= (unsigned)Ws;
    const int ii = (int)(t % (unsigned)Hs);
    const int n = (int)(t / (unsigned)Hs);
    const int h = 2 * ii + dy - pad;
    float v[8];
#pragma unroll
    for (int dx = 0; dx < 2; ++dx) {
      const int w = 2 * j + dx - pad;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const uint8_t* px = X + (((size_t)n * H + (ok ? h : 0)) * W + (ok ? w : 0)) * C;
#pragma unroll
      for (int c = 0; c < 4; ++c) v[dx * 4 + c] = (ok && c < C) ? (float)px[c] * sc[c] + sh[c] : 0.f;
    }
    *reinterpret_cast<uint4*>(Y + ((((size_t)n * Hs + ii) * Ws + j) * 16) + dy * 8) = pack8(v);
  }
}

__global__ __launch_bounds__(256) void bf16_to_f32_accum_kernel(const bf16_t* __restrict__ x, float* __restrict__ y,
                                                                 size_t n, int accumulate) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = accumulate ? y[i] + bf2f(x[i]) : bf2f(x[i]);
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// bf16 elementwise add (8 per lane), y = a + b
__global__ __launch_bounds__(256) void add_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ y, size_t n8) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    float x[8], z[8];
    unpack8(reinterpret_cast<const uint4*>(a)[i], x);
    unpack8(reinterpret_cast<const uint4*>(b)[i], z);
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] += z[e];
    reinterpret_cast<uint4*>(y)[i] = pack8(x);
  }
}

static int egrid(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b ? b : 1);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_softmax_xent(const void* logits, int is_f32, const int64_t* labels, float* loss_sum,
                                       float* count, void* dlogits, int B, int NC, float grad_scale,
                                       int ignore_index, int per_row, hipStream_t st) {
  const int blocks = (B + 3) / 4;
  if (is_f32)
    hipLaunchKernelGGL(softmax_xent_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)logits, labels,
                       loss_sum, count, (float*)dlogits, B, NC, grad_scale, ignore_index, per_row);
  else
    hipLaunchKernelGGL(softmax_xent_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)logits, labels,
                       loss_sum, count, (bf16_t*)dlogits, B, NC, grad_scale, ignore_index, per_row);
  return hipGetLastError();
}

// mean softmax cross-entropy in two launches: per-row terms (part: [B] losses, [B] counts), then
// the ordered fold into out = [mean, count] (prob_nll_finalize_kernel); deterministic, no
// accumulator fill, no clamp / div launches
extern "C" hipError_t zoo_softmax_xent_mean(const void* logits, int is_f32, const int64_t* labels, float* part,
                                            float* out, void* dlogits, int B, int NC, int ignore_index,
                                            hipStream_t st) {
  const hipError_t e = zoo_softmax_xent(logits, is_f32, labels, part, part + B, dlogits, B, NC, 1.f, ignore_index, 1, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(prob_nll_finalize_kernel, dim3(1), dim3(64), 0, st, part, B, out, 1);
  return hipGetLastError();
}

extern "C" hipError_t zoo_xent_grad_scale(const void* dl, int is_f32, const float* g, const float* count, void* out,
                                          size_t n, hipStream_t st) {
  const int blocks = egrid(n);
  if (is_f32)
    hipLaunchKernelGGL(xent_grad_scale_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)dl, g, count,
                       (float*)out, n);
  else
    hipLaunchKernelGGL(xent_grad_scale_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)dl, g, count,
                       (bf16_t*)out, n);
  return hipGetLastError();
}

extern "C" hipError_t zoo_prob_nll(const void* probs, int is_f32, const int64_t* labels, float* loss_sum, float* count,
                                   float* dp, int B, int NC, float eps, int ignore_index, int per_row, hipStream_t st) {
  const int rb = (B + 255) / 256;
  const int blocks = per_row ? rb : (rb < 128 ? rb : 128);
  if (is_f32)
    hipLaunchKernelGGL(prob_nll_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)probs, labels, loss_sum,
                       count, dp, B, NC, eps, ignore_index, per_row);
  else
    hipLaunchKernelGGL(prob_nll_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)probs, labels,
                       loss_sum, count, dp, B, NC, eps, ignore_index, per_row);
  return hipGetLastError();
}

// loss scalar + count of the probability NLL in two native launches: [out 2], part: 2 * 128 floats
extern "C" hipError_t zoo_prob_nll_mean(const void* probs, int is_f32, const int64_t* labels, float* part,
                                        float* out, int B, int NC, float eps, int ignore_index, int size_average,
                                        hipStream_t st) {
  const int rb = (B + 255) / 256;
  const int blocks = rb < 128 ? (rb > 0 ? rb : 1) : 128;
  if (is_f32)
    hipLaunchKernelGGL(prob_nll_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)probs, labels, part,
                       part + blocks, (float*)nullptr, B, NC, eps, ignore_index, 2);
  else
    hipLaunchKernelGGL(prob_nll_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)probs, labels, part,
                       part + blocks, (float*)nullptr, B, NC, eps, ignore_index, 2);
  hipLaunchKernelGGL(prob_nll_finalize_kernel, dim3(1), dim3(64), 0, st, part, blocks, out, size_average);
  return hipGetLastError();
}

extern "C" hipError_t zoo_prob_nll_grad(const void* probs, int is_f32, const int64_t* labels, const float* g,
                                        const float* count, float* dp, int B, int NC, float eps, int ignore_index,
                                        hipStream_t st) {
  const int blocks = (B + 255) / 256;
  if (is_f32)
    hipLaunchKernelGGL(prob_nll_grad_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)probs, labels, g,
                       count, dp, B, NC, eps, ignore_index);
  else
    hipLaunchKernelGGL(prob_nll_grad_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)probs, labels, g,
                       count, dp, B, NC, eps, ignore_index);
  return hipGetLastError();
}

// zero_g (optimizer-side gradient clear, ops.cpp optim_zero_grad): g is cleared after it is read
static int g_zero_g = 0;
extern "C" void zoo_optim_zero_grad(int on) { g_zero_g = on ? 1 : 0; }
// device hyper-parameters (ops.cpp optim_device_hparams): while set, the optimizer kernels read
// lr / bias corrections / the first-step flag from this fp32 [4] buffer instead of their scalar
// arguments -- a captured update then follows the schedule on every replay
static const float* g_hp = nullptr;
extern "C" void zoo_optim_device_hparams(const float* hp) { g_hp = hp; }

extern "C" hipError_t zoo_sgd(float* p, const float* g, float* mom, void* pbf, size_t n, float lr, float momentum,
                              float dampening, float wd, int nesterov, float gscale, int first_step,
                              hipStream_t st) {
  hipLaunchKernelGGL(sgd_kernel, dim3(egrid(n)), dim3(256), 0, st, p, const_cast<float*>(g), mom, (bf16_t*)pbf, n, lr,
                     momentum, dampening, wd, nesterov, gscale, first_step, g_zero_g, g_hp);
  return hipGetLastError();
}

extern "C" hipError_t zoo_adam(float* p, const float* g, float* m, float* v, void* pbf, size_t n, float lr, float b1,
                               float b2, float eps, float wd, float bc1, float bc2, float gscale, int decoupled,
                               hipStream_t st) {
  hipLaunchKernelGGL(adam_kernel, dim3(egrid(n)), dim3(256), 0, st, p, const_cast<float*>(g), m, v, (bf16_t*)pbf, n,
                     lr, b1, b2, eps, wd, bc1, bc2, gscale, decoupled, g_zero_g, g_hp);
  return hipGetLastError();
}

extern "C" hipError_t zoo_adaptive(float* p, const float* g, float* s1, float* s2, void* pbf, size_t n, int kind,
                                   float lr, float rho, float rho2, float eps, float wd, float bc1, float gscale,
                                   hipStream_t st) {
  hipLaunchKernelGGL(adaptive_kernel, dim3(egrid(n)), dim3(256), 0, st, p, const_cast<float*>(g), s1, s2, (bf16_t*)pbf,
                     n, kind, lr, rho, rho2, eps, wd, bc1, gscale, g_zero_g, g_hp);
  return hipGetLastError();
}

extern "C" hipError_t zoo_sumsq(const float* g, size_t n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(egrid(n) > 1024 ? 1024 : egrid(n)), dim3(256), 0, st, g, n, out);
  return hipGetLastError();
}

extern "C" hipError_t zoo_clip(float* g, size_t n, float lo, float hi, const float* norm_sq, float max_norm,
                               hipStream_t st) {
  hipLaunchKernelGGL(clip_kernel, dim3(egrid(n)), dim3(256), 0, st, g, n, lo, hi, norm_sq, max_norm);
  return hipGetLastError();
}

extern "C" hipError_t zoo_nchw_to_nhwc(const float* X, void* Y, int N, int C, int H, int W, int Cp, hipStream_t st) {
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(egrid((size_t)N * H * W * Cp)), dim3(256), 0, st, X, (bf16_t*)Y, N, C,
                     H, W, Cp);
  return hipGetLastError();
}

extern "C" hipError_t zoo_nchw_to_s2d(const float* X, void* Y, int N, int C, int H, int W, int pad, int Hs, int Ws,
                                       hipStream_t st) {
  if ((size_t)N * Hs * Ws * 2 >= (1ull << 31)) return hipErrorInvalidValue;   // 32-bit kernel index
  hipLaunchKernelGGL(nchw_to_s2d_kernel, dim3(egrid((size_t)N * Hs * Ws * 2)), dim3(256), 0, st, X, (bf16_t*)Y, N, C,
                     H, W, 4, pad, Hs, Ws);
  return hipGetLastError();
}

extern "C" hipError_t zoo_nhwc_u8_to_s2d(const void* X, void* Y, int N, int C, int H, int W, int pad, int Hs, int Ws,
                                          const float* scale, const float* shift, hipStream_t st) {
  if ((size_t)N * Hs * Ws * 2 >= (1ull << 31)) return hipErrorInvalidValue;   // 32-bit kernel index
  const float4 sc{scale[0], scale[1], scale[2], scale[3]}, sf{shift[0], shift[1], shift[2], shift[3]};
  hipLaunchKernelGGL(nhwc_u8_to_s2d_kernel, dim3(egrid((size_t)N * Hs * Ws * 2)), dim3(256), 0, st,
                     (const uint8_t*)X, (bf16_t*)Y, N, C, H, W, pad, Hs, Ws, sc, sf);
  return hipGetLastError();
}

extern "C" hipError_t zoo_bf16_to_f32(const void* x, float* y, size_t n, int accumulate, hipStream_t st) {
  hipLaunchKernelGGL(bf16_to_f32_accum_kernel, dim3(egrid(n)), dim3(256), 0, st, (const bf16_t*)x, y, n, accumulate);
  return hipGetLastError();
}

extern "C" hipError_t zoo_f32_to_bf16(const float* x, void* y, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(egrid(n)), dim3(256), 0, st, x, (bf16_t*)y, n);
  return hipGetLastError();
}

// Reduce-scatter epilogue of the all-to-all gradient exchange (zoo/parallel/ddp.py): rank r
// received chunk r of every peer's bf16 bucket, recv = [nchunks][cb]; the sum is accumulated in
// fp32 (one bf16 rounding per input instead of one per ring hop) and written as fp32 (sharded
// optimizer input) and/or bf16 (the all-gather payload). 8 elements per thread, cb % 8 == 0.
__global__ __launch_bounds__(256) void sum_chunks_bf16_kernel(const bf16_t* __restrict__ recv, int nchunks,
                                                             size_t cb, float* __restrict__ out32,
                                                             bf16_t* __restrict__ out16, float scale) {
  const size_t n8 = cb / 8;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (size_t)gridDim.x * blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < nchunks; ++c) {
      float v[8];
      unpack8(reinterpret_cast<const uint4*>(recv + (size_t)c * cb)[i], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= scale;
    if (out32) {
      reinterpret_cast<float4*>(out32)[2 * i] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      reinterpret_cast<float4*>(out32)[2 * i + 1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
    if (out16) reinterpret_cast<uint4*>(out16)[i] = pack8(acc);
  }
}

extern "C" hipError_t zoo_sum_chunks_bf16(const void* recv, int nchunks, size_t cb, float* out32, void* out16,
                                          float scale, hipStream_t st) {
  hipLaunchKernelGGL(sum_chunks_bf16_kernel, dim3(egrid(cb / 8)), dim3(256), 0, st, (const bf16_t*)recv, nchunks, cb,
                     out32, (bf16_t*)out16, scale);
  return hipGetLastError();
}

extern "C" hipError_t zoo_add_bf16(const void* a, const void* b, void* y, size_t n, hipStream_t st) {
  hipLaunchKernelGGL(add_bf16_kernel, dim3(egrid(n / 8)), dim3(256), 0, st, (const bf16_t*)a, (const bf16_t*)b,
                     (bf16_t*)y, n / 8);
  return hipGetLastError();
}
