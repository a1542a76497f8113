// Kernels behind the Keras layers that round 2 left on PyTorch (VERDICT r2 missing #3-#4):
//
//   * WithinChannelLRN2D  (SpatialWithinChannelLRN): y = x * (1 + alpha * avg_{size x size}(x^2))^-beta
//   * ResizeBilinear      (BigDL nn.ResizeBilinear, TF-legacy sampling, optional align_corners)
//   * UpSampling1D/2D/3D  (nearest repeat over up to three spatial dims)
//   * ConvLSTM2D/3D gates (InternalConvLSTM2D/3D.scala: i, f, o gates, candidate, cell and
//     hidden update fused into one pass per timestep, and its backward)
//
// All activations are channels-last (NHWC / NDHWC) so the channel index is the fastest and
// every warp touches contiguous memory; compute is fp32 for fp32 or bf16 storage. Backward
// passes are gather-form (no atomics) except the bilinear resize, whose 4-tap scatter goes
// through fp32 atomics into a zeroed fp32 buffer.
//
// Reference: Zs/pipeline/api/keras/layers/{WithinChannelLRN2D,ResizeBilinear,UpSampling2D,
// ConvLSTM2D,ConvLSTM3D}.scala and InternalConvLSTM3D.scala:40-218 (SURVEY.md §2.2 K3, §2.16
// HK11/HK15/HK17).
#include "common.h"
#include "lstm.h"

namespace zoo {

template <typename T>
ZOO_DEV float ld(const T* p, size_t i);
template <>
ZOO_DEV float ld<float>(const float* p, size_t i) { return p[i]; }
template <>
ZOO_DEV float ld<bf16_t>(const bf16_t* p, size_t i) { return bf2f(p[i]); }
template <typename T>
ZOO_DEV void st(T* p, size_t i, float v);
template <>
ZOO_DEV void st<float>(float* p, size_t i, float v) { p[i] = v; }
template <>
ZOO_DEV void st<bf16_t>(bf16_t* p, size_t i, float v) { p[i] = f2bf(v); }

#define GRID_STRIDE(i, n) for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); \
                               i += (size_t)gridDim.x * blockDim.x)

// ---------------------------------------------------------------- within-channel LRN
// x [N, H, W, C]; window size x size centred ((size-1)/2 before), zero padded, mean over size^2
template <typename T>
__global__ void wlrn_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int size,
                                float alpha, float beta) {
  const size_t n = (size_t)N * H * W * C;
  const int lo = (size - 1) / 2;
  const float inv = 1.f / (size * size);
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const size_t b = t / H;
    float s = 0.f;
    for (int dh = 0; dh < size; ++dh) {
      const int hh = h - lo + dh;
      if (hh < 0 || hh >= H) continue;
      for (int dw = 0; dw < size; ++dw) {
        const int ww = w - lo + dw;
        if (ww < 0 || ww >= W) continue;
        const float v = ld(x, ((b * H + hh) * W + ww) * C + c);
        s += v * v;
      }
    }
    st(y, i, ld(x, i) * __powf(1.f + alpha * s * inv, -beta));
  }
}

// pass 1 of the backward: q = dy * x * scale^(-beta-1), scale recomputed
template <typename T>
__global__ void wlrn_bwd1_kernel(const T* __restrict__ x, const T* __restrict__ dy, float* __restrict__ q,
                                 float* __restrict__ sc, int N, int H, int W, int C, int size, float alpha, float beta) {
  const size_t n = (size_t)N * H * W * C;
  const int lo = (size - 1) / 2;
  const float inv = 1.f / (size * size);
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const size_t b = t / H;
    float s = 0.f;
    for (int dh = 0; dh < size; ++dh) {
      const int hh = h - lo + dh;
      if (hh < 0 || hh >= H) continue;
      for (int dw = 0; dw < size; ++dw) {
        const int ww = w - lo + dw;
        if (ww < 0 || ww >= W) continue;
        const float v = ld(x, ((b * H + hh) * W + ww) * C + c);
        s += v * v;
      }
    }
    const float scale = 1.f + alpha * s * inv;
    sc[i] = __powf(scale, -beta);
    q[i] = ld(dy, i) * ld(x, i) * __powf(scale, -beta - 1.f);
  }
}

// pass 2: dx_i = dy_i * scale_i^-beta - 2 alpha beta / size^2 * x_i * sum_{j : i in win(j)} q_j
template <typename T>
__global__ void wlrn_bwd2_kernel(const T* __restrict__ x, const T* __restrict__ dy, const float* __restrict__ q,
                                 const float* __restrict__ sc, T* __restrict__ dx, int N, int H, int W, int C,
                                 int size, float alpha, float beta) {
  const size_t n = (size_t)N * H * W * C;
  const int lo = (size - 1) / 2;
  const float k = 2.f * alpha * beta / (size * size);
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const size_t b = t / H;
    float s = 0.f;
    // j's window covers i  <=>  i - (size-1-lo) <= j <= i + lo  (per axis)
    for (int dh = -lo; dh <= size - 1 - lo; ++dh) {
      const int hh = h + dh;
      if (hh < 0 || hh >= H) continue;
      for (int dw = -lo; dw <= size - 1 - lo; ++dw) {
        const int ww = w + dw;
        if (ww < 0 || ww >= W) continue;
        s += q[((b * H + hh) * W + ww) * C + c];
      }
    }
    st(dx, i, ld(dy, i) * sc[i] - k * ld(x, i) * s);
  }
}

// ---------------------------------------------------------------- bilinear resize (NHWC)
// BigDL / TF-legacy sampling: src = dst * scale, scale = in/out or (in-1)/(out-1) (align_corners);
// half-pixel mode (off = 0.5 * scale - 0.5, PyTorch align_corners=False / Caffe bilinear
// deconvolution upsampling): src = max((dst + 0.5) * scale - 0.5, 0)
ZOO_DEV void lerp_idx(int o, int in, float scale, float off, int& lo, int& hi, float& f) {
  float s = o * scale + off;
  s = s < 0.f ? 0.f : s;
  lo = (int)floorf(s);
  lo = lo < in - 1 ? lo : in - 1;
  hi = lo + 1 < in ? lo + 1 : in - 1;
  f = s - lo;
  f = f < 0.f ? 0.f : (f > 1.f ? 1.f : f);
}

template <typename T>
__global__ void resize_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H, int W, int C, int OH,
                                  int OW, float sh, float sw, float oh_off, float ow_off) {
  const size_t n = (size_t)N * OH * OW * C;
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const size_t b = t / OH;
    int h0, h1, w0, w1;
    float fh, fw;
    lerp_idx(oh, H, sh, oh_off, h0, h1, fh);
    lerp_idx(ow, W, sw, ow_off, w0, w1, fw);
    const size_t base = b * H;
    const float a = ld(x, ((base + h0) * W + w0) * C + c), bb = ld(x, ((base + h0) * W + w1) * C + c);
    const float cc = ld(x, ((base + h1) * W + w0) * C + c), d = ld(x, ((base + h1) * W + w1) * C + c);
    const float top = a + (bb - a) * fw, bot = cc + (d - cc) * fw;
    st(y, i, top + (bot - top) * fh);
  }
}

template <typename T>
__global__ void resize_bwd_kernel(const T* __restrict__ dy, float* __restrict__ dx, int N, int H, int W, int C,
                                  int OH, int OW, float sh, float sw, float oh_off, float ow_off) {
  const size_t n = (size_t)N * OH * OW * C;
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const size_t b = t / OH;
    int h0, h1, w0, w1;
    float fh, fw;
    lerp_idx(oh, H, sh, oh_off, h0, h1, fh);
    lerp_idx(ow, W, sw, ow_off, w0, w1, fw);
    const float g = ld(dy, i);
    const size_t base = b * H;
    atomicAdd(dx + ((base + h0) * W + w0) * C + c, g * (1.f - fh) * (1.f - fw));
    atomicAdd(dx + ((base + h0) * W + w1) * C + c, g * (1.f - fh) * fw);
    atomicAdd(dx + ((base + h1) * W + w0) * C + c, g * fh * (1.f - fw));
    atomicAdd(dx + ((base + h1) * W + w1) * C + c, g * fh * fw);
  }
}

// ---------------------------------------------------------------- nearest upsampling
// x [N, D, H, W, C] -> y [N, D*fd, H*fh, W*fw, C]; backward sums each fd x fh x fw block
template <typename T>
__global__ void upsample_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int D, int H, int W, int C,
                                    int fd, int fh, int fw) {
  const int OD = D * fd, OH = H * fh, OW = W * fw;
  const size_t n = (size_t)N * OD * OH * OW * C;
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    t /= OH;
    const int od = (int)(t % OD);
    const size_t b = t / OD;
    y[i] = x[(((b * D + od / fd) * H + oh / fh) * W + ow / fw) * C + c];
  }
}

template <typename T>
__global__ void upsample_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, int N, int D, int H, int W, int C,
                                    int fd, int fh, int fw) {
  const int OH = H * fh, OW = W * fw;
  const size_t n = (size_t)N * D * H * W * C;
  GRID_STRIDE(i, n) {
    const int c = (int)(i % C);
    size_t t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    t /= H;
    const int d = (int)(t % D);
    const size_t b = t / D;
    float s = 0.f;
    for (int a = 0; a < fd; ++a)
      for (int e = 0; e < fh; ++e)
        for (int f = 0; f < fw; ++f)
          s += ld(dy, ((((b * D * fd + d * fd + a) * OH) + h * fh + e) * OW + w * fw + f) * C + c);
    st(dx, i, s);
  }
}

// ---------------------------------------------------------------- ConvLSTM gates
// g = gx + gh ([M, 4F]: i | f | candidate | o); c = f * c_prev + i * act(cand); h = o * act(c)
__global__ void lstm_gates_fwd_kernel(const float* __restrict__ gx, const float* __restrict__ gh,
                                      const float* __restrict__ cprev, float* __restrict__ h, float* __restrict__ c,
                                      float* __restrict__ acts, int M, int F, int iact, int act) {
  const size_t n = (size_t)M * F;
  GRID_STRIDE(idx, n) {
    const size_t m = idx / F;
    const int j = (int)(idx % F);
    const size_t r = m * 4 * F;
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const size_t o = r + q * F + j;
      g[q] = gx[o] + (gh ? gh[o] : 0.f);
    }
    const float ig = lstm_act(g[0], iact), fg = lstm_act(g[1], iact);
    const float cg = lstm_act(g[2], act), og = lstm_act(g[3], iact);
    const float cp = cprev ? cprev[idx] : 0.f;
    const float cn = fg * cp + ig * cg;
    c[idx] = cn;
    h[idx] = og * lstm_act(cn, act);
    acts[r + j] = ig;
    acts[r + F + j] = fg;
    acts[r + 2 * F + j] = cg;
    acts[r + 3 * F + j] = og;
  }
}

// dh (+ dc from the next step) -> pre-activation gate gradients dg [M, 4F] and dc_prev
__global__ void lstm_gates_bwd_kernel(const float* __restrict__ dh, const float* __restrict__ dcn,
                                      const float* __restrict__ acts, const float* __restrict__ cprev,
                                      const float* __restrict__ c, float* __restrict__ dg, float* __restrict__ dcp,
                                      int M, int F, int iact, int act) {
  const size_t n = (size_t)M * F;
  GRID_STRIDE(idx, n) {
    const size_t m = idx / F;
    const int j = (int)(idx % F);
    const size_t r = m * 4 * F;
    const float ig = acts[r + j], fg = acts[r + F + j], cg = acts[r + 2 * F + j], og = acts[r + 3 * F + j];
    const float cn = c[idx];
    const float tc = lstm_act(cn, act);
    const float gh = dh ? dh[idx] : 0.f;
    const float dc = gh * og * lstm_dact(tc, act) + (dcn ? dcn[idx] : 0.f);
    const float cp = cprev ? cprev[idx] : 0.f;
    dg[r + j] = dc * cg * lstm_dact(ig, iact);
    dg[r + F + j] = dc * cp * lstm_dact(fg, iact);
    dg[r + 2 * F + j] = dc * ig * lstm_dact(cg, act);
    dg[r + 3 * F + j] = gh * tc * lstm_dact(og, iact);
    if (dcp) dcp[idx] = dc * fg;
  }
}

// Whole-sequence ConvLSTM step kernels (zoo/pipeline/api/keras/layers/recurrent.py
// _ConvLSTMSeqFn): the forward also writes h_t as bf16 into the padded NHWC conv-input
// history slot the next step's recurrent conv reads (row stride ldh, pad channels untouched =
// 0), so a step is one recurrent conv + this kernel with no Python glue in between.
__global__ void lstm_step_fwd_kernel(const float* __restrict__ gx, const float* __restrict__ gh,
                                     const float* __restrict__ cprev, float* __restrict__ h, float* __restrict__ c,
                                     float* __restrict__ acts, bf16_t* __restrict__ hb, int ldh, int M, int F,
                                     int ldgh, int iact, int act) {
  const size_t n = (size_t)M * F;
  GRID_STRIDE(idx, n) {
    const size_t m = idx / F;
    const int j = (int)(idx % F);
    const size_t r = m * 4 * F;
    float g[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) g[q] = gx[r + q * F + j] + (gh ? gh[m * ldgh + q * F + j] : 0.f);
    const float ig = lstm_act(g[0], iact), fg = lstm_act(g[1], iact);
    const float cg = lstm_act(g[2], act), og = lstm_act(g[3], iact);
    const float cp = cprev ? cprev[idx] : 0.f;
    const float cn = fg * cp + ig * cg;
    const float hn = og * lstm_act(cn, act);
    c[idx] = cn;
    h[idx] = hn;
    hb[m * ldh + j] = f2bf(hn);
    acts[r + j] = ig;
    acts[r + F + j] = fg;
    acts[r + 2 * F + j] = cg;
    acts[r + 3 * F + j] = og;
  }
}

// backward of one step: dh = dout (fp32 [M, F], may be null) + dhr (bf16 recurrent gradient,
// row stride lddh, may be null); writes dg fp32 [M, 4F] (the input conv's gradient slot), dgb
// bf16 [M, lddg] (the recurrent dgrad / wgrad operand) and dc_prev
__global__ void lstm_step_bwd_kernel(const float* __restrict__ dout, const bf16_t* __restrict__ dhr, int lddh,
                                     const float* __restrict__ dcn, const float* __restrict__ acts,
                                     const float* __restrict__ cprev, const float* __restrict__ c,
                                     float* __restrict__ dg, bf16_t* __restrict__ dgb, int lddg,
                                     float* __restrict__ dcp, int M, int F, int iact, int act) {
  const size_t n = (size_t)M * F;
  GRID_STRIDE(idx, n) {
    const size_t m = idx / F;
    const int j = (int)(idx % F);
    const size_t r = m * 4 * F;
    const float ig = acts[r + j], fg = acts[r + F + j], cg = acts[r + 2 * F + j], og = acts[r + 3 * F + j];
    const float tc = lstm_act(c[idx], act);
    const float gh = (dout ? dout[idx] : 0.f) + (dhr ? bf2f(dhr[m * lddh + j]) : 0.f);
    const float dc = gh * og * lstm_dact(tc, act) + (dcn ? dcn[idx] : 0.f);
    const float cp = cprev ? cprev[idx] : 0.f;
    const float d0 = dc * cg * lstm_dact(ig, iact), d1 = dc * cp * lstm_dact(fg, iact);
    const float d2 = dc * ig * lstm_dact(cg, act), d3 = gh * tc * lstm_dact(og, iact);
    dg[r + j] = d0;
    dg[r + F + j] = d1;
    dg[r + 2 * F + j] = d2;
    dg[r + 3 * F + j] = d3;
    if (dgb) {
      bf16_t* o = dgb + m * lddg;
      o[j] = f2bf(d0);
      o[F + j] = f2bf(d1);
      o[2 * F + j] = f2bf(d2);
      o[3 * F + j] = f2bf(d3);
    }
    if (dcp) dcp[idx] = dc * fg;
  }
}

static int grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_wlrn(const void* x, const void* dy, void* out, float* q, float* sc, int N, int H, int W,
                               int C, int size, float alpha, float beta, int bf16, hipStream_t st) {
  const size_t n = (size_t)N * H * W * C;
  const int g = grid_for(n);
  if (!dy) {
    if (bf16)
      hipLaunchKernelGGL(wlrn_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)out, N, H, W,
                         C, size, alpha, beta);
    else
      hipLaunchKernelGGL(wlrn_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, (float*)out, N, H, W, C,
                         size, alpha, beta);
    return hipGetLastError();
  }
  if (bf16) {
    hipLaunchKernelGGL(wlrn_bwd1_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)dy, q,
                       sc, N, H, W, C, size, alpha, beta);
    hipLaunchKernelGGL(wlrn_bwd2_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)dy, q,
                       sc, (bf16_t*)out, N, H, W, C, size, alpha, beta);
  } else {
    hipLaunchKernelGGL(wlrn_bwd1_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, (const float*)dy, q, sc,
                       N, H, W, C, size, alpha, beta);
    hipLaunchKernelGGL(wlrn_bwd2_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)x, (const float*)dy, q, sc,
                       (float*)out, N, H, W, C, size, alpha, beta);
  }
  return hipGetLastError();
}

extern "C" hipError_t zoo_resize_bilinear(const void* in, void* out, int N, int H, int W, int C, int OH, int OW,
                                          int align, int backward, int bf16, hipStream_t st) {
  // align: 0 TF-legacy (BigDL ResizeBilinear), 1 align_corners, 2 half-pixel centres
  const float sh = (align == 1 && OH > 1) ? (float)(H - 1) / (OH - 1) : (float)H / OH;
  const float sw = (align == 1 && OW > 1) ? (float)(W - 1) / (OW - 1) : (float)W / OW;
  const float oh_off = align == 2 ? 0.5f * sh - 0.5f : 0.f, ow_off = align == 2 ? 0.5f * sw - 0.5f : 0.f;
  const size_t n = (size_t)N * OH * OW * C;
  const int g = grid_for(n);
  if (!backward) {
    if (bf16)
      hipLaunchKernelGGL(resize_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)in, (bf16_t*)out, N, H,
                         W, C, OH, OW, sh, sw, oh_off, ow_off);
    else
      hipLaunchKernelGGL(resize_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)in, (float*)out, N, H, W,
                         C, OH, OW, sh, sw, oh_off, ow_off);
  } else {  // in = dy [N, OH, OW, C], out = fp32 dx [N, H, W, C] (zeroed by the caller)
    if (bf16)
      hipLaunchKernelGGL(resize_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)in, (float*)out, N, H,
                         W, C, OH, OW, sh, sw, oh_off, ow_off);
    else
      hipLaunchKernelGGL(resize_bwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)in, (float*)out, N, H, W,
                         C, OH, OW, sh, sw, oh_off, ow_off);
  }
  return hipGetLastError();
}

extern "C" hipError_t zoo_upsample(const void* in, void* out, int N, int D, int H, int W, int C, int fd, int fh, int fw,
                                   int backward, int bf16, hipStream_t st) {
  const size_t n = (size_t)N * D * H * W * C * (backward ? 1 : (size_t)fd * fh * fw);
  const int g = grid_for(n);
  if (!backward) {
    if (bf16)
      hipLaunchKernelGGL(upsample_fwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)in, (bf16_t*)out, N, D,
                         H, W, C, fd, fh, fw);
    else
      hipLaunchKernelGGL(upsample_fwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)in, (float*)out, N, D, H,
                         W, C, fd, fh, fw);
  } else {
    if (bf16)
      hipLaunchKernelGGL(upsample_bwd_kernel<bf16_t>, dim3(g), dim3(256), 0, st, (const bf16_t*)in, (bf16_t*)out, N, D,
                         H, W, C, fd, fh, fw);
    else
      hipLaunchKernelGGL(upsample_bwd_kernel<float>, dim3(g), dim3(256), 0, st, (const float*)in, (float*)out, N, D, H,
                         W, C, fd, fh, fw);
  }
  return hipGetLastError();
}

extern "C" hipError_t zoo_lstm_gates(const float* gx, const float* gh, const float* cprev, float* h, float* c,
                                     float* acts, const float* dh, const float* dcn, float* dg, float* dcp, int M,
                                     int F, int iact, int act, int backward, hipStream_t st) {
  const int g = grid_for((size_t)M * F);
  if (!backward)
    hipLaunchKernelGGL(lstm_gates_fwd_kernel, dim3(g), dim3(256), 0, st, gx, gh, cprev, h, c, acts, M, F, iact, act);
  else
    hipLaunchKernelGGL(lstm_gates_bwd_kernel, dim3(g), dim3(256), 0, st, dh, dcn, acts, cprev, c, dg, dcp, M, F, iact,
                       act);
  return hipGetLastError();
}

extern "C" hipError_t zoo_lstm_step(const float* gx, const float* gh, int ldgh, const float* cprev, float* h,
                                    float* c, float* acts, void* hb, int ldh, const float* dout, const void* dhr,
                                    int lddh, const float* dcn, float* dg, void* dgb, int lddg, float* dcp, int M,
                                    int F, int iact, int act, int backward, hipStream_t st) {
  const int g = grid_for((size_t)M * F);
  if (!backward)
    hipLaunchKernelGGL(lstm_step_fwd_kernel, dim3(g), dim3(256), 0, st, gx, gh, cprev, h, c, acts, (bf16_t*)hb, ldh,
                       M, F, ldgh, iact, act);
  else
    hipLaunchKernelGGL(lstm_step_bwd_kernel, dim3(g), dim3(256), 0, st, dout, (const bf16_t*)dhr, lddh, dcn, acts,
                       cprev, c, dg, (bf16_t*)dgb, lddg, dcp, M, F, iact, act);
  return hipGetLastError();
}
