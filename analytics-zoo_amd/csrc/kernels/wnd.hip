// Wide & Deep glue as native kernels (WideAndDeep.scala:113-144; profiles/r3/wide_and_deep_glue_r3.md).
//
// deep_input: the deep tower's input row [indicator | embedding_0 | ... | continuous] built in one
//   pass straight into the bf16 MFMA operand: float ids (the Keras input dtype) are converted in
//   the kernel, each embedding segment gathers its table row, the dense segments are copied. The
//   Select / Flatten / Embedding / concat / bf16-cast chain was ~8 launches and 4 HBM round trips.
//   Backward scatter-adds each embedding segment into its fp32 table gradient (vector atomics:
//   ids repeat across the batch).
// wnd_head: logits = wide + bias + deep, probabilities = softmax(logits), one thread per row
//   (class counts <= 32); backward dlogits = p * (g - sum(g * p)) written to both towers and
//   folded per block into the bias gradient.
#include "common.h"
#include "geom.h"

namespace zoo {

__global__ __launch_bounds__(256) void deep_input_fwd_kernel(const float* __restrict__ ids, int n_ids, DeepSegs segs,
                                                             bf16_t* __restrict__ out, int B, int W) {
  const long total = (long)B * W;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int b = (int)(i / W), c = (int)(i - (long)b * W);
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < DI_MAX_SEG; ++k) {
      if (k >= segs.n) break;
      const DeepSeg& sg = segs.s[k];
      const int j = c - sg.col0;
      if (j >= 0 && j < sg.width) {
        if (sg.emb) {
          const int id = (int)ids[(size_t)b * n_ids + sg.id_col];
          v = (id >= 0 && id < sg.V) ? sg.src[(size_t)id * sg.width + j] : 0.f;
        } else {
          v = sg.src[(size_t)b * sg.ld + j];
        }
      }
    }
    out[i] = f2bf(v);
  }
}

// one thread per (row, column) of the embedding segments only
__global__ __launch_bounds__(256) void deep_input_bwd_kernel(const bf16_t* __restrict__ dout, const float* __restrict__ ids,
                                                             int n_ids, DeepSegs segs, int B, int W) {
  for (int k = 0; k < segs.n; ++k) {
    const DeepSeg& sg = segs.s[k];
    if (!sg.emb || !sg.gsrc) continue;
    const long total = (long)B * sg.width;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
      const int b = (int)(i / sg.width), j = (int)(i - (long)b * sg.width);
      const int id = (int)ids[(size_t)b * n_ids + sg.id_col];
      if (id >= 0 && id < sg.V) atomicAdd(sg.gsrc + (size_t)id * sg.width + j, bf2f(dout[(size_t)b * W + sg.col0 + j]));
    }
  }
}

constexpr int HEAD_MAX_C = 32;

ZOO_DEV float wnd_ld(float v) { return v; }
ZOO_DEV float wnd_ld(bf16_t v) { return bf2f(v); }

template <typename TD>
__global__ __launch_bounds__(256) void wnd_head_fwd_kernel(const float* __restrict__ wide, const TD* __restrict__ deep,
                                                           const float* __restrict__ bias, float* __restrict__ prob,
                                                           int B, int C) {
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  float z[HEAD_MAX_C];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < HEAD_MAX_C; ++c) {
    if (c < C) {
      float v = bias ? bias[c] : 0.f;
      if (wide) v += wide[(size_t)b * C + c];
      if (deep) v += wnd_ld(deep[(size_t)b * C + c]);
      z[c] = v;
      mx = fmaxf(mx, v);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < HEAD_MAX_C; ++c)
    if (c < C) {
      z[c] = __expf(z[c] - mx);
      s += z[c];
    }
  const float inv = 1.f / s;
#pragma unroll
  for (int c = 0; c < HEAD_MAX_C; ++c)
    if (c < C) prob[(size_t)b * C + c] = z[c] * inv;
}

// dlogits = p * (g - <g, p>); dwide fp32, ddeep in the deep tower's dtype; per-block bias
// partials [gridDim][C] (deterministic fold afterwards)
template <typename TD>
__global__ __launch_bounds__(256) void wnd_head_bwd_kernel(const float* __restrict__ prob, const float* __restrict__ g,
                                                           float* __restrict__ dwide, TD* __restrict__ ddeep,
                                                           float* __restrict__ bpart, int B, int C) {
  __shared__ float red[HEAD_MAX_C][8];
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float d[HEAD_MAX_C];
  const bool ok = b < B;
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < HEAD_MAX_C; ++c) {
    d[c] = 0.f;
    if (ok && c < C) dot = fmaf(g[(size_t)b * C + c], prob[(size_t)b * C + c], dot);
  }
#pragma unroll
  for (int c = 0; c < HEAD_MAX_C; ++c)
    if (ok && c < C) {
      const float p = prob[(size_t)b * C + c];
      d[c] = p * (g[(size_t)b * C + c] - dot);
      if (dwide) dwide[(size_t)b * C + c] = d[c];
      if (ddeep) {
        if constexpr (sizeof(TD) == 2) ddeep[(size_t)b * C + c] = f2bf(d[c]);
        else ddeep[(size_t)b * C + c] = d[c];
      }
    }
  if (!bpart) return;
#pragma unroll
  for (int c = 0; c < HEAD_MAX_C; ++c) {
    if (c < C) {
      const float s = warp_sum(d[c]);
      if (lane == 0) red[c][wv] = s;
    }
  }
  __syncthreads();
  if (threadIdx.x < C)
    bpart[(size_t)blockIdx.x * C + threadIdx.x] =
        ((red[threadIdx.x][0] + red[threadIdx.x][1]) + red[threadIdx.x][2]) + red[threadIdx.x][3];
}

__global__ __launch_bounds__(64) void wnd_bias_fold_kernel(const float* __restrict__ bpart, int nb, int C,
                                                           float* __restrict__ gbias) {
  const int c = threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int k = 0; k < nb; ++k) s += bpart[(size_t)k * C + c];
  gbias[c] += s;
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_deep_input(const float* ids, int n_ids, const DeepSegs* segs, void* out, const void* dout,
                                     int B, int W, hipStream_t st) {
  if (segs->n > DI_MAX_SEG) return hipErrorInvalidValue;
  const long total = (long)B * W;
  const int grid = (int)std::min<long>((total + 255) / 256, 4096);
  if (!dout)
    hipLaunchKernelGGL(deep_input_fwd_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, st, ids, n_ids, *segs,
                       (bf16_t*)out, B, W);
  else
    hipLaunchKernelGGL(deep_input_bwd_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, st, (const bf16_t*)dout, ids,
                       n_ids, *segs, B, W);
  return hipGetLastError();
}

extern "C" int zoo_wnd_head_blocks(int B) { return (B + 255) / 256; }

extern "C" hipError_t zoo_wnd_head_fwd(const float* wide, const void* deep, int deep_bf16, const float* bias,
                                       float* prob, int B, int C, hipStream_t st) {
  if (C > HEAD_MAX_C || C < 1) return hipErrorInvalidValue;
  const int nb = zoo_wnd_head_blocks(B);
  if (deep_bf16)
    hipLaunchKernelGGL(wnd_head_fwd_kernel<bf16_t>, dim3(nb), dim3(256), 0, st, wide, (const bf16_t*)deep, bias, prob,
                       B, C);
  else
    hipLaunchKernelGGL(wnd_head_fwd_kernel<float>, dim3(nb), dim3(256), 0, st, wide, (const float*)deep, bias, prob,
                       B, C);
  return hipGetLastError();
}

// gbias (fp32 [C]) += column sums of dlogits; bpart: zoo_wnd_head_blocks(B) * C floats
extern "C" hipError_t zoo_wnd_head_bwd(const float* prob, const float* g, float* dwide, void* ddeep, int deep_bf16,
                                       float* gbias, float* bpart, int B, int C, hipStream_t st) {
  if (C > HEAD_MAX_C || C < 1) return hipErrorInvalidValue;
  const int nb = zoo_wnd_head_blocks(B);
  float* bp = gbias ? bpart : nullptr;
  if (deep_bf16)
    hipLaunchKernelGGL(wnd_head_bwd_kernel<bf16_t>, dim3(nb), dim3(256), 0, st, prob, g, dwide, (bf16_t*)ddeep, bp, B,
                       C);
  else
    hipLaunchKernelGGL(wnd_head_bwd_kernel<float>, dim3(nb), dim3(256), 0, st, prob, g, dwide, (float*)ddeep, bp, B,
                       C);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !gbias) return e;
  hipLaunchKernelGGL(wnd_bias_fold_kernel, dim3(1), dim3(64), 0, st, bpart, nb, C, gbias);
  return hipGetLastError();
}
