// Pooling for NHWC bf16 activations (gfx950).
//
// Reference: BigDL SpatialMaxPooling / SpatialAveragePooling behind
// Zs/pipeline/api/keras/layers/{MaxPooling2D,AveragePooling2D,GlobalAveragePooling2D}.scala
// (SURVEY.md §2.16 HK6). Max pooling records the winning tap (0..R*S-1) as one
// byte per output so the backward pass is a race-free gather (no atomics).
#include "common.h"

namespace zoo {

// 32-bit index math throughout (the launcher checks N*P*Q*C/8 and N*H*W*C/8 < 2^31): the
// 64-bit div/mod of a size_t grid-stride index made the r1 kernels VALU-bound (~2 TB/s)
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                          uint8_t* __restrict__ arg, int N, int H, int W, int C,
                                                          int P, int Q, int R, int S, int sh, int sw, int ph,
                                                          int pw) {
  const int cpr = C >> 3;
  const int total = N * P * Q * cpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int chunk = i % cpr;
    int t = i / cpr;
    const int q = t % Q;
    t /= Q;
    const int p = t % P;
    const int n = t / P;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    const bf16_t* xn = X + (size_t)n * H * W * C + chunk * 8;
    for (int r = 0; r < R; ++r) {
      const int ih = p * sh - ph + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int s = 0; s < S; ++s) {
        const int iw = q * sw - pw + s;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(xn + (ih * W + iw) * C), v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = (uint8_t)(r * S + s); }
      }
    }
    *reinterpret_cast<uint4*>(Y + (size_t)i * 8) = pack8(best);
    if (arg) {
      uint2 pk;
      pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
      pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *reinterpret_cast<uint2*>(arg + (size_t)i * 8) = pk;
    }
  }
}

// gather form: every input pixel sums the gradients of the windows whose argmax it is
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dY,
                                                          const uint8_t* __restrict__ arg, bf16_t* __restrict__ dX,
                                                          int N, int H, int W, int C, int P, int Q, int R, int S,
                                                          int sh, int sw, int ph, int pw) {
  const int cpr = C >> 3;
  const int total = N * H * W * cpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int chunk = i % cpr;
    int t = i / cpr;
    const int w = t % W;
    t /= W;
    const int h = t % H;
    const int n = t / H;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // output rows p with p*sh - ph <= h <= p*sh - ph + R - 1
    const int p_lo = max(0, (h + ph - R + sh) / sh);
    const int p_hi = min(P - 1, (h + ph) / sh);
    const int q_lo = max(0, (w + pw - S + sw) / sw);
    const int q_hi = min(Q - 1, (w + pw) / sw);
    const size_t nb = (size_t)n * P * Q * C + chunk * 8;
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * sh - ph);
      if (r < 0 || r >= R) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * sw - pw);
        if (s < 0 || s >= S) continue;
        const uint32_t tap = (uint32_t)(r * S + s);
        const size_t o = nb + (size_t)(p * Q + q) * C;
        const uint2 ab = *reinterpret_cast<const uint2*>(arg + o);
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dY + o), g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (((ab.x >> (8 * e)) & 0xff) == tap) acc[e] += g[e];
          if (((ab.y >> (8 * e)) & 0xff) == tap) acc[4 + e] += g[4 + e];
        }
      }
    }
    *reinterpret_cast<uint4*>(dX + (size_t)i * 8) = pack8(acc);
  }
}

// Row-per-block variants for a power-of-two C/8 (ResNet stem, every NHWC net with C % 64
// == 0 ...): one block owns one (n, output row) [fwd] or (n, input row) [bwd], so the
// row's window bounds are block-uniform (scalar) and the per-thread index split is a
// shift/mask. The grid-stride kernels above spend ~6 integer divisions per element and
// ran VALU-bound (stem bwd 236 us = 2.4 TB/s at b256).
__global__ __launch_bounds__(256) void maxpool_fwd_row_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                              uint8_t* __restrict__ arg, int H, int W, int C, int P,
                                                              int Q, int R, int S, int sh, int sw, int ph, int pw,
                                                              int lg) {
  const int row = blockIdx.x;  // n * P + p
  const int n = row / P, p = row - n * P;
  const int mask = (C >> 3) - 1;
  const int r_lo = max(0, ph - p * sh), r_hi = min(R, H + ph - p * sh);
  const bf16_t* xn = X + (size_t)n * H * W * C + (size_t)(p * sh - ph) * W * C;
  const size_t ybase = (size_t)row * Q * C;
  for (int j = threadIdx.x; j < (Q << lg); j += 256) {
    const int q = j >> lg, chunk = j & mask;
    const int s_lo = max(0, pw - q * sw), s_hi = min(S, W + pw - q * sw);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    const bf16_t* xq = xn + (q * sw - pw) * C + chunk * 8;
    for (int r = r_lo; r < r_hi; ++r) {
      for (int s = s_lo; s < s_hi; ++s) {
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(xq + (r * W + s) * C), v);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) { best[e] = v[e]; bi[e] = (uint8_t)(r * S + s); }
      }
    }
    const size_t o = ybase + (size_t)j * 8;
    *reinterpret_cast<uint4*>(Y + o) = pack8(best);
    if (arg) {
      uint2 pk;
      pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
      pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
      *reinterpret_cast<uint2*>(arg + o) = pk;
    }
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_row_kernel(const bf16_t* __restrict__ dY,
                                                              const uint8_t* __restrict__ arg,
                                                              bf16_t* __restrict__ dX, int H, int W, int C, int P,
                                                              int Q, int R, int S, int sh, int sw, int ph, int pw,
                                                              int lg) {
  const int row = blockIdx.x;  // n * H + h
  const int n = row / H, h = row - n * H;
  const int mask = (C >> 3) - 1;
  // output rows p with p*sh - ph <= h <= p*sh - ph + R - 1 (block-uniform)
  const int p_lo = max(0, (h + ph - R + sh) / sh);
  const int p_hi = min(P - 1, (h + ph) / sh);
  const size_t nb = (size_t)n * P * Q * C;
  const size_t xbase = (size_t)row * W * C;
  for (int j = threadIdx.x; j < (W << lg); j += 256) {
    const int w = j >> lg, chunk = j & mask;
    const int q_lo = max(0, (w + pw - S + sw) / sw);
    const int q_hi = min(Q - 1, (w + pw) / sw);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * sh - ph);
      if (r < 0 || r >= R) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * sw - pw);
        if (s < 0 || s >= S) continue;
        const uint32_t tap = (uint32_t)(r * S + s);
        const size_t o = nb + (size_t)(p * Q + q) * C + chunk * 8;
        const uint2 ab = *reinterpret_cast<const uint2*>(arg + o);
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dY + o), g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (((ab.x >> (8 * e)) & 0xff) == tap) acc[e] += g[e];
          if (((ab.y >> (8 * e)) & 0xff) == tap) acc[4 + e] += g[4 + e];
        }
      }
    }
    *reinterpret_cast<uint4*>(dX + xbase + (size_t)j * 8) = pack8(acc);
  }
}

// log2 of C/8 when it is a power of two, else -1 (row kernels not applicable)
static int row_lg(int C) {
  const int cpr = C >> 3;
  if (cpr <= 0 || (cpr & (cpr - 1))) return -1;
  int lg = 0;
  while ((1 << lg) < cpr) ++lg;
  return lg;
}

// global average pool [N][HW][C] -> [N][C] (fp32 accumulate, bf16 or fp32 out)
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                      int N, int HW, int C) {
  const int cpr = C >> 3;
  const int total = N * cpr;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int chunk = i % cpr, n = i / cpr;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const bf16_t* base = X + (size_t)n * HW * C + chunk * 8;
    for (int s = 0; s < HW; ++s) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(base + (size_t)s * C), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    *reinterpret_cast<uint4*>(Y + (size_t)n * C + chunk * 8) = pack8(acc);
  }
}

__global__ __launch_bounds__(256) void gap_bwd_kernel(const bf16_t* __restrict__ dY, bf16_t* __restrict__ dX,
                                                      int N, int HW, int C) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * HW * cpr;
  const float inv = 1.f / (float)HW;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % cpr);
    const int n = (int)(i / ((size_t)cpr * HW));
    float g[8];
    unpack8(*reinterpret_cast<const uint4*>(dY + (size_t)n * C + chunk * 8), g);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= inv;
    *reinterpret_cast<uint4*>(dX + i * 8) = pack8(g);
  }
}

// average pooling (AveragePooling2D / SpatialAveragePooling): the divisor is the window
// clipped to the padded input (count_include_pad) or to the valid taps; ceil-mode output
// sizes come in through P / Q
ZOO_DEV int avg_div(int p, int q, int H, int W, int R, int S, int sh, int sw, int ph, int pw, int inc_pad) {
  int h0 = p * sh - ph, w0 = q * sw - pw;
  int h1 = min(h0 + R, H + ph), w1 = min(w0 + S, W + pw);
  if (!inc_pad) {
    h0 = max(h0, 0); w0 = max(w0, 0);
    h1 = min(h1, H); w1 = min(w1, W);
  }
  const int d = (h1 - h0) * (w1 - w0);
  return d > 0 ? d : 1;
}

__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16_t* __restrict__ X, bf16_t* __restrict__ Y,
                                                          int N, int H, int W, int C, int P, int Q, int R, int S,
                                                          int sh, int sw, int ph, int pw, int inc_pad) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * P * Q * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % cpr);
    size_t t = i / cpr;
    const int q = (int)(t % Q); t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < R; ++r) {
      const int ih = p * sh - ph + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int s = 0; s < S; ++s) {
        const int iw = q * sw - pw + s;
        if ((unsigned)iw >= (unsigned)W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const uint4*>(X + (((size_t)n * H + ih) * W + iw) * C + chunk * 8), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    }
    const float inv = 1.f / (float)avg_div(p, q, H, W, R, S, sh, sw, ph, pw, inc_pad);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    *reinterpret_cast<uint4*>(Y + i * 8) = pack8(acc);
  }
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const bf16_t* __restrict__ dY, bf16_t* __restrict__ dX,
                                                          int N, int H, int W, int C, int P, int Q, int R, int S,
                                                          int sh, int sw, int ph, int pw, int inc_pad) {
  const int cpr = C >> 3;
  const size_t total = (size_t)N * H * W * cpr;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int chunk = (int)(i % cpr);
    size_t t = i / cpr;
    const int w = (int)(t % W); t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int p_lo = max(0, (h + ph - R + sh) / sh), p_hi = min(P - 1, (h + ph) / sh);
    const int q_lo = max(0, (w + pw - S + sw) / sw), q_hi = min(Q - 1, (w + pw) / sw);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * sh - ph);
      if (r < 0 || r >= R) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * sw - pw);
        if (s < 0 || s >= S) continue;
        float g[8];
        unpack8(*reinterpret_cast<const uint4*>(dY + (((size_t)n * P + p) * Q + q) * C + chunk * 8), g);
        const float inv = 1.f / (float)avg_div(p, q, H, W, R, S, sh, sw, ph, pw, inc_pad);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += g[e] * inv;
      }
    }
    *reinterpret_cast<uint4*>(dX + i * 8) = pack8(acc);
  }
}

static int pgrid(size_t work) {
  size_t b = (work + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b ? b : 1);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_maxpool_fwd(const void* X, void* Y, void* arg, int N, int H, int W, int C, int P, int Q,
                                      int R, int S, int sh, int sw, int ph, int pw, hipStream_t st) {
  const int lg = row_lg(C);
  if (lg >= 0 && R * S <= 256) {
    hipLaunchKernelGGL(maxpool_fwd_row_kernel, dim3(N * P), dim3(256), 0, st, (const bf16_t*)X, (bf16_t*)Y,
                       (uint8_t*)arg, H, W, C, P, Q, R, S, sh, sw, ph, pw, lg);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(pgrid((size_t)N * P * Q * (C / 8))), dim3(256), 0, st,
                     (const bf16_t*)X, (bf16_t*)Y, (uint8_t*)arg, N, H, W, C, P, Q, R, S, sh, sw, ph, pw);
  return hipGetLastError();
}

extern "C" hipError_t zoo_maxpool_bwd(const void* dY, const void* arg, void* dX, int N, int H, int W, int C, int P,
                                      int Q, int R, int S, int sh, int sw, int ph, int pw, hipStream_t st) {
  const int lg = row_lg(C);
  if (lg >= 0 && R * S <= 256) {
    hipLaunchKernelGGL(maxpool_bwd_row_kernel, dim3(N * H), dim3(256), 0, st, (const bf16_t*)dY,
                       (const uint8_t*)arg, (bf16_t*)dX, H, W, C, P, Q, R, S, sh, sw, ph, pw, lg);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(pgrid((size_t)N * H * W * (C / 8))), dim3(256), 0, st,
                     (const bf16_t*)dY, (const uint8_t*)arg, (bf16_t*)dX, N, H, W, C, P, Q, R, S, sh, sw, ph, pw);
  return hipGetLastError();
}

extern "C" hipError_t zoo_gap_fwd(const void* X, void* Y, int N, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gap_fwd_kernel, dim3(pgrid((size_t)N * (C / 8))), dim3(256), 0, st, (const bf16_t*)X,
                     (bf16_t*)Y, N, HW, C);
  return hipGetLastError();
}

extern "C" hipError_t zoo_gap_bwd(const void* dY, void* dX, int N, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(pgrid((size_t)N * HW * (C / 8))), dim3(256), 0, st, (const bf16_t*)dY,
                     (bf16_t*)dX, N, HW, C);
  return hipGetLastError();
}

extern "C" hipError_t zoo_avgpool_fwd(const void* X, void* Y, int N, int H, int W, int C, int P, int Q, int R, int S,
                                      int sh, int sw, int ph, int pw, int inc_pad, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3(pgrid((size_t)N * P * Q * (C / 8))), dim3(256), 0, st,
                     (const bf16_t*)X, (bf16_t*)Y, N, H, W, C, P, Q, R, S, sh, sw, ph, pw, inc_pad);
  return hipGetLastError();
}

extern "C" hipError_t zoo_avgpool_bwd(const void* dY, void* dX, int N, int H, int W, int C, int P, int Q, int R,
                                      int S, int sh, int sw, int ph, int pw, int inc_pad, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(pgrid((size_t)N * H * W * (C / 8))), dim3(256), 0, st,
                     (const bf16_t*)dY, (bf16_t*)dX, N, H, W, C, P, Q, R, S, sh, sw, ph, pw, inc_pad);
  return hipGetLastError();
}
