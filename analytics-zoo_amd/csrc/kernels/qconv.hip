// Static-int8 implicit-GEMM convolution on the gfx950 int8 matrix cores.
//
// Reference: BigDL quantize() int8 inference (InferenceModelFactory.scala:33,47,
// ImageModel.scala:133-145). There the int8 path is MKL-DNN's
// u8s8 convolution with calibrated scales; here it is the bf16 implicit-GEMM kernel
// (igemm.hip) re-targeted at v_mfma_i32_16x16x64_i8, which runs at twice the bf16 MFMA rate
// and reads half the bytes:
//
//   * operands are int8 NHWC activations and int8 [K][R][S][C] weights (C % 16 == 0). Byte
//     for byte the LDS tiles, the LDS-DMA staging (global_load_lds, swizzle through the
//     per-lane source chunk), the im2col address decode and the fragment reads are the bf16
//     kernel's: a 16-byte chunk carries 16 int8 channels instead of 8 bf16 ones, and a lane's
//     16 fragment bytes are k = 16(l>>4)..+15 of the i8 MFMA exactly where they were
//     k = 8(l>>4)..+7 of the bf16 one;
//   * the epilogue is the whole rest of a ResNet unit in one pass:
//       v = acc * colscale[c] + bias[c] (+ resid_q * rscale) -> ReLU -> int8 or bf16,
//     where colscale = s_in * s_w[c] / s_out, bias = folded-BN bias / s_out and
//     rscale = s_resid / s_out (all precomputed on the host from calibration), so an int8
//     output is round-to-nearest + saturate of v.
//
// FP8 (OCP e4m3fn) twin, same kernel body: the operands are e4m3 bytes (per-channel weight
// scale = amax / 448, calibrated per-tensor activation scales), the 128-byte k-step feeds ONE
// v_mfma_scale_f32_16x16x128_f8f6f4 (unit block scales) per fragment pair instead of two i8
// MFMAs -- the K=128 scaled form is the one that runs at the fp8 peak (2x bf16, MI355X_MICROARCH
// "FP8"); a lane's 32 operand bytes are the two consecutive 16-byte chunks 2(l>>4), 2(l>>4)+1 of
// the row (A and B use the same k map, so the reduction pairs them correctly). fp32
// accumulation; the epilogue converts with the hardware e4m3 conversion after clamping to
// +-448 (e4m3fn has no infinity).
#include <type_traits>

#include "common.h"
#include "geom.h"

namespace zoo {

typedef int qi32x4 __attribute__((ext_vector_type(4)));
typedef int qi32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void q_lds_void;
typedef __attribute__((address_space(1))) const void q_gl_void;

constexpr int QC_BM = 128, QC_BK = 128 /* bytes = int8 elements */, QC_NT = 256;
__device__ __attribute__((aligned(16))) int8_t qc_zero_page[16];
// the real zero of an offset-coded (unsigned) activation: padding taps of a QF_IN_U8 input
__device__ __attribute__((aligned(16))) int8_t qc_u8zero_page[16] = {-128, -128, -128, -128, -128, -128, -128, -128,
                                                                    -128, -128, -128, -128, -128, -128, -128, -128};

// Unsigned (offset-coded) int8 activations: a non-negative tensor (post-ReLU) is stored as
// q = clamp(round(x / s), 0, 255) - 128, x = (q + 128) s -- the full 8-bit grid instead of the
// 7 bits a symmetric code leaves a ReLU output. The i8 MFMA sums q * w; the missing
// 128 * sum_k w[n][k] is a per-output-channel constant the host folds into the bias (padding
// taps read -128, the real zero, so the constant holds at the borders too).
constexpr int QF_IN_U8 = 1, QF_OUT_U8 = 2, QF_RES_U8 = 4;

ZOO_DEV int8_t q_sat_u8(float v) {
  const float r = rintf(v);
  return (int8_t)((r > 255.f ? 255.f : (r < 0.f ? 0.f : r)) - 128.f);
}

ZOO_DEV int qc_swz(int row) { return (row >> 1) & 7; }

ZOO_DEV int8_t q_sat(float v) {
  const float r = rintf(v);
  return (int8_t)(r > 127.f ? 127.f : (r < -127.f ? -127.f : r));
}

// 4 floats -> 4 OCP e4m3fn bytes (round to nearest even, clamped to the finite range)
ZOO_DEV uint32_t f8_pack4(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

ZOO_DEV void f8_unpack4(uint32_t w, float* f) {
  f[0] = __builtin_amdgcn_cvt_f32_fp8((int)w, 0);
  f[1] = __builtin_amdgcn_cvt_f32_fp8((int)w, 1);
  f[2] = __builtin_amdgcn_cvt_f32_fp8((int)w, 2);
  f[3] = __builtin_amdgcn_cvt_f32_fp8((int)w, 3);
}

template <bool IS1x1, int BN, bool FP8>
__global__ __launch_bounds__(256, 2) void qconv_kernel(const int8_t* __restrict__ X, const int8_t* __restrict__ Wm,
                                                      void* __restrict__ Y, const float* __restrict__ colscale,
                                                      const float* __restrict__ bias,
                                                      const int8_t* __restrict__ resid, float rscale,
                                                      const float* __restrict__ rvec, ConvGeom g, int relu,
                                                      int out_bf16, int qflags) {
  constexpr int BM = QC_BM, BK = QC_BK;
  constexpr int WN = BN / 2, NJ = WN / 16, NI = 4;
  constexpr int B_ROWS_PER_THREAD = BN / 32;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nbuf = g.ldb > BK ? 2 : 1;
  int8_t* As = reinterpret_cast<int8_t*>(smem);
  int8_t* Bs = As + nbuf * BM * BK;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int ntn = (g.K + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / ntn, tn = bid - tm * ntn;
  const int m0 = tm * BM, n0 = tn * BN;

  // staging: lane -> 16-byte slot (lane & 7) of row (lane >> 3) of the wave's 8-row group;
  // the swizzle is applied by choosing which k-chunk this lane loads
  const int rbase = tid >> 3;
  const int cc = (tid & 7) ^ qc_swz(rbase);

  int a_base[4], a_ih[4], a_iw[4];
  bool a_ok[4];
  const int PQ = g.P * g.Q;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + rbase + 32 * i;
    a_ok[i] = m < g.M;
    const int mm = a_ok[i] ? m : 0;
    if constexpr (IS1x1) {
      a_base[i] = mm * g.C;
      a_ih[i] = a_iw[i] = 0;
    } else {
      const int n = mm / PQ, pq = mm - n * PQ;
      const int p = pq / g.Q, q = pq - p * g.Q;
      a_base[i] = n * g.H * g.W * g.C;
      a_ih[i] = p * g.sh - g.ph;
      a_iw[i] = q * g.sw - g.pw;
    }
  }
  int kr = 0, ks = 0, kc = cc * 16;
  if constexpr (!IS1x1) {
    while (kc >= g.C) { kc -= g.C; if (++ks == g.S) { ks = 0; ++kr; } }
  }
  const int nk = (g.ldb + BK - 1) / BK;
  const int8_t* a_pad = (!FP8 && (qflags & QF_IN_U8)) ? qc_u8zero_page : qc_zero_page;

  auto dma16 = [&](const int8_t* src, int8_t* dst) {
    __builtin_amdgcn_global_load_lds((q_gl_void*)src, (q_lds_void*)dst, 16, 0, 0);
  };
  auto load_tile = [&](int kt) {
    const int k = kt * BK + cc * 16;
    int8_t* adst = As + (kt & 1) * BM * BK + (wid * 8) * BK;
    int8_t* bdst = Bs + (kt & 1) * BN * BK + (wid * 8) * BK;
    if constexpr (IS1x1) {
      const bool kok = k < g.Ktot;
#pragma unroll
      for (int i = 0; i < 4; ++i) dma16(a_ok[i] && kok ? X + a_base[i] + k : a_pad, adst + (32 * i) * BK);
    } else {
      const bool kok = kr < g.R;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ih = a_ih[i] + kr * g.dh, iw = a_iw[i] + ks * g.dw;
        const bool ok = a_ok[i] && kok && (unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W;
        dma16(ok ? X + a_base[i] + (ih * g.W + iw) * g.C + kc : a_pad, adst + (32 * i) * BK);
      }
    }
    const bool kokb = k < g.ldb;
#pragma unroll
    for (int i = 0; i < B_ROWS_PER_THREAD; ++i) {
      const int n = n0 + rbase + 32 * i;
      dma16(n < g.K && kokb ? Wm + (size_t)n * g.ldb + k : qc_zero_page, bdst + (32 * i) * BK);
    }
    if constexpr (!IS1x1) {
      kc += BK;
      while (kc >= g.C) { kc -= g.C; if (++ks == g.S) { ks = 0; ++kr; } }
    }
  };

  typedef typename std::conditional<FP8, f32x4, qi32x4>::type acc_t;
  acc_t acc[NI][NJ];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = acc_t{0, 0, 0, 0};
  const int fr = lane & 15, fq = lane >> 4;

  auto compute = [&](int buf) {
    const int8_t* a = As + buf * BM * BK;
    const int8_t* b = Bs + buf * BN * BK;
    if constexpr (FP8) {
      qi32x8 af[NI], bfg[NJ];
      const int c0 = 2 * fq, c1 = 2 * fq + 1;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        const qi32x4 lo = *reinterpret_cast<const qi32x4*>(a + row * BK + ((c0 ^ qc_swz(row)) << 4));
        const qi32x4 hi = *reinterpret_cast<const qi32x4*>(a + row * BK + ((c1 ^ qc_swz(row)) << 4));
        af[i] = qi32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * WN + j * 16 + fr;
        const qi32x4 lo = *reinterpret_cast<const qi32x4*>(b + row * BK + ((c0 ^ qc_swz(row)) << 4));
        const qi32x4 hi = *reinterpret_cast<const qi32x4*>(b + row * BK + ((c1 ^ qc_swz(row)) << 4));
        bfg[j] = qi32x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfg[j], acc[i][j], 0, 0, 0, 0, 0, 0);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;
      qi32x4 af[NI], bfg[NJ];
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const qi32x4*>(a + row * BK + ((chunk ^ qc_swz(row)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = wn * WN + j * 16 + fr;
        bfg[j] = *reinterpret_cast<const qi32x4*>(b + row * BK + ((chunk ^ qc_swz(row)) << 4));
      }
#pragma unroll
      for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          if constexpr (!FP8) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bfg[j], acc[i][j], 0, 0, 0);
        }
    }
  };

  load_tile(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) load_tile(kt + 1);
    compute(kt & 1);
    if (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue: scaled fp32 tile staged in LDS, then row-contiguous 8-column stores ----
  constexpr int LD = BN + 4;
  float* Cs = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int col = wn * WN + j * 16 + fr;
    const float cs = n0 + col < g.K ? colscale[n0 + col] : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) Cs[(wm * 64 + i * 16 + fq * 4 + r) * LD + col] = (float)acc[i][j][r] * cs;
  }
  __syncthreads();
  constexpr int CPR = BN / 8, RSTEP = QC_NT / CPR;
  const int ch = tid % CPR, rr0 = tid / CPR;
  const int col0 = n0 + ch * 8;
  if (col0 >= g.K) return;
  float bv[8], rv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bv[e] = bias ? bias[col0 + e] : 0.f;
    rv[e] = rvec ? rvec[col0 + e] : rscale;   // per-channel activation scales: s_resid[c] / s_out[c]
  }
  const int rend = min(BM, g.M - m0);
  for (int rr = rr0; rr < rend; rr += RSTEP) {
    const size_t off = (size_t)(m0 + rr) * g.K + col0;
    const float4 lo = *reinterpret_cast<const float4*>(Cs + rr * LD + ch * 8);
    const float4 hi = *reinterpret_cast<const float4*>(Cs + rr * LD + ch * 8 + 4);
    float v[8] = {lo.x + bv[0], lo.y + bv[1], lo.z + bv[2], lo.w + bv[3],
                  hi.x + bv[4], hi.y + bv[5], hi.z + bv[6], hi.w + bv[7]};
    if (resid) {
      const uint2 rq = *reinterpret_cast<const uint2*>(resid + off);
      if constexpr (FP8) {
        float r[8];
        f8_unpack4(rq.x, r);
        f8_unpack4(rq.y, r + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += r[e] * rv[e];
      } else {
        const float ro = (qflags & QF_RES_U8) ? 128.f : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] += ((float)(int8_t)(rq.x >> (8 * e)) + ro) * rv[e];
          v[4 + e] += ((float)(int8_t)(rq.y >> (8 * e)) + ro) * rv[4 + e];
        }
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (out_bf16) {
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(Y) + off) = pack8(v);
    } else if constexpr (FP8) {
      *reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(Y) + off) =
          make_uint2(f8_pack4(v[0], v[1], v[2], v[3]), f8_pack4(v[4], v[5], v[6], v[7]));
    } else if (qflags & QF_OUT_U8) {
      uint2 pk;
      pk.x = (uint32_t)(uint8_t)q_sat_u8(v[0]) | ((uint32_t)(uint8_t)q_sat_u8(v[1]) << 8) |
             ((uint32_t)(uint8_t)q_sat_u8(v[2]) << 16) | ((uint32_t)(uint8_t)q_sat_u8(v[3]) << 24);
      pk.y = (uint32_t)(uint8_t)q_sat_u8(v[4]) | ((uint32_t)(uint8_t)q_sat_u8(v[5]) << 8) |
             ((uint32_t)(uint8_t)q_sat_u8(v[6]) << 16) | ((uint32_t)(uint8_t)q_sat_u8(v[7]) << 24);
      *reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(Y) + off) = pk;
    } else {
      uint2 pk;
      pk.x = (uint32_t)(uint8_t)q_sat(v[0]) | ((uint32_t)(uint8_t)q_sat(v[1]) << 8) |
             ((uint32_t)(uint8_t)q_sat(v[2]) << 16) | ((uint32_t)(uint8_t)q_sat(v[3]) << 24);
      pk.y = (uint32_t)(uint8_t)q_sat(v[4]) | ((uint32_t)(uint8_t)q_sat(v[5]) << 8) |
             ((uint32_t)(uint8_t)q_sat(v[6]) << 16) | ((uint32_t)(uint8_t)q_sat(v[7]) << 24);
      *reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(Y) + off) = pk;
    }
  }
}

// bf16 -> int8 with one per-tensor inverse scale (16 elements per thread, 16-byte stores)
// inv_vec (optional, C % 16 == 0): one inverse scale per channel of the NHWC tensor (last dim C)
__global__ __launch_bounds__(256) void quantize_i8_kernel(const bf16_t* __restrict__ x, int8_t* __restrict__ q,
                                                          size_t n16, float inv_scale, const float* __restrict__ inv_vec,
                                                          int C, int u8) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    float a[8], b[8];
    unpack8(reinterpret_cast<const uint4*>(x)[2 * i], a);
    unpack8(reinterpret_cast<const uint4*>(x)[2 * i + 1], b);
    const int c0 = inv_vec ? (int)((i * 16) % (size_t)C) : 0;
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sa = inv_vec ? inv_vec[c0 + e] : inv_scale, sb = inv_vec ? inv_vec[c0 + 8 + e] : inv_scale;
      const int8_t qa = u8 ? q_sat_u8(a[e] * sa) : q_sat(a[e] * sa);
      const int8_t qb = u8 ? q_sat_u8(b[e] * sb) : q_sat(b[e] * sb);
      w[e >> 2] |= (uint32_t)(uint8_t)qa << (8 * (e & 3));
      w[2 + (e >> 2)] |= (uint32_t)(uint8_t)qb << (8 * (e & 3));
    }
    reinterpret_cast<uint4*>(q)[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// bf16 -> e4m3 with one per-tensor inverse scale
__global__ __launch_bounds__(256) void quantize_f8_kernel(const bf16_t* __restrict__ x, int8_t* __restrict__ q,
                                                          size_t n16, float inv_scale, const float* __restrict__ inv_vec,
                                                          int C) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    float a[8], b[8];
    unpack8(reinterpret_cast<const uint4*>(x)[2 * i], a);
    unpack8(reinterpret_cast<const uint4*>(x)[2 * i + 1], b);
    const int c0 = inv_vec ? (int)((i * 16) % (size_t)C) : 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] *= inv_vec ? inv_vec[c0 + e] : inv_scale;
      b[e] *= inv_vec ? inv_vec[c0 + 8 + e] : inv_scale;
    }
    reinterpret_cast<uint4*>(q)[i] = make_uint4(f8_pack4(a[0], a[1], a[2], a[3]), f8_pack4(a[4], a[5], a[6], a[7]),
                                                f8_pack4(b[0], b[1], b[2], b[3]), f8_pack4(b[4], b[5], b[6], b[7]));
  }
}

// global average pool of an int8 (FP8: e4m3) NHWC tensor -> bf16 [N][C] (dequantised with `scale`)
template <bool FP8>
__global__ __launch_bounds__(256) void gap_i8_kernel(const int8_t* __restrict__ X, bf16_t* __restrict__ Y, int N,
                                                     int HW, int C, float scale, const float* __restrict__ svec,
                                                     int u8) {
  const int cpr = C >> 3;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N * cpr; i += gridDim.x * blockDim.x) {
    const int chunk = i % cpr, n = i / cpr;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int8_t* base = X + (size_t)n * HW * C + chunk * 8;
    for (int s = 0; s < HW; ++s) {
      const uint2 v = *reinterpret_cast<const uint2*>(base + (size_t)s * C);
      if constexpr (FP8) {
        float f[8];
        f8_unpack4(v.x, f);
        f8_unpack4(v.y, f + 4);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] += (float)(int8_t)(v.x >> (8 * e));
          acc[4 + e] += (float)(int8_t)(v.y >> (8 * e));
        }
      }
    }
    const float zo = (!FP8 && u8) ? 128.f : 0.f;   // offset-coded input: mean(q) + 128
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = (acc[e] / (float)HW + zo) * (svec ? svec[chunk * 8 + e] : scale);
    *reinterpret_cast<uint4*>(Y + (size_t)n * C + chunk * 8) = pack8(acc);
  }
}

template <bool IS1x1, int BN, bool FP8>
static hipError_t launch_qc(const int8_t* X, const int8_t* W, void* Y, const float* cs, const float* bias,
                            const int8_t* resid, float rscale, const float* rvec, const ConvGeom& g, int relu,
                            int out_bf16, int qflags, hipStream_t st) {
  const int tiles = ((g.M + QC_BM - 1) / QC_BM) * ((g.K + BN - 1) / BN);
  const size_t main_b = (size_t)(g.ldb > QC_BK ? 2 : 1) * (QC_BM + BN) * QC_BK;
  const size_t epi_b = (size_t)QC_BM * (BN + 4) * sizeof(float);
  const size_t smem = main_b > epi_b ? main_b : epi_b;
  static bool attr = false;
  if (!attr) {
    const size_t mx = (size_t)2 * (QC_BM + BN) * QC_BK > epi_b ? (size_t)2 * (QC_BM + BN) * QC_BK : epi_b;
    hipFuncSetAttribute(reinterpret_cast<const void*>(&qconv_kernel<IS1x1, BN, FP8>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)mx);
    attr = true;
  }
  hipLaunchKernelGGL((qconv_kernel<IS1x1, BN, FP8>), dim3(tiles), dim3(QC_NT), smem, st, X, W, Y, cs, bias, resid, rscale,
                     rvec, g, relu, out_bf16, qflags);
  return hipGetLastError();
}

}  // namespace zoo

using namespace zoo;

// g: geometry in int8 elements (C, Ktot = R*S*C, ldb all multiples of 16); fp8: e4m3 operands
extern "C" hipError_t zoo_qconv(const void* X, const void* W, void* Y, const float* colscale, const float* bias,
                                const void* resid, float rscale, const float* rvec, const ConvGeom* g, int relu,
                                int out_bf16, int fp8, int qflags, hipStream_t st) {
  const int8_t* x = (const int8_t*)X;
  const int8_t* w = (const int8_t*)W;
  const int8_t* r = (const int8_t*)resid;
  const bool is1x1 = g->R == 1 && g->S == 1 && g->sh == 1 && g->sw == 1 && g->ph == 0 && g->pw == 0 &&
                     g->H == g->P && g->W == g->Q;
  const long tiles64 = (long)((g->M + QC_BM - 1) / QC_BM) * ((g->K + 63) / 64);
  const bool wide = g->K > 64 && tiles64 < 1536;   // few tiles: 128-wide n tiles fill the chip better
#define ZOO_QC(F8)                                                                                                 \
  do {                                                                                                             \
    if (is1x1)                                                                                                     \
      return wide ? launch_qc<true, 128, F8>(x, w, Y, colscale, bias, r, rscale, rvec, *g, relu, out_bf16, qflags, st)           \
                  : launch_qc<true, 64, F8>(x, w, Y, colscale, bias, r, rscale, rvec, *g, relu, out_bf16, qflags, st);           \
    return wide ? launch_qc<false, 128, F8>(x, w, Y, colscale, bias, r, rscale, rvec, *g, relu, out_bf16, qflags, st)            \
                : launch_qc<false, 64, F8>(x, w, Y, colscale, bias, r, rscale, rvec, *g, relu, out_bf16, qflags, st);            \
  } while (0)
  if (fp8) ZOO_QC(true);
  ZOO_QC(false);
#undef ZOO_QC
}

extern "C" hipError_t zoo_quantize_i8(const void* x, void* q, size_t n, float inv_scale, const float* inv_vec, int C,
                                       int u8, hipStream_t st) {
  const size_t n16 = n / 16;
  size_t blocks = (n16 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(quantize_i8_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, st, (const bf16_t*)x, (int8_t*)q,
                     n16, inv_scale, inv_vec, C, u8);
  return hipGetLastError();
}

extern "C" hipError_t zoo_quantize_f8(const void* x, void* q, size_t n, float inv_scale, const float* inv_vec, int C,
                                       hipStream_t st) {
  const size_t n16 = n / 16;
  size_t blocks = (n16 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(quantize_f8_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, st, (const bf16_t*)x, (int8_t*)q,
                     n16, inv_scale, inv_vec, C);
  return hipGetLastError();
}

extern "C" hipError_t zoo_gap_i8(const void* x, void* y, int N, int HW, int C, float scale, const float* svec, int fp8,
                                  int u8, hipStream_t st) {
  int blocks = (N * (C / 8) + 255) / 256;
  if (fp8)
    hipLaunchKernelGGL(gap_i8_kernel<true>, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, (const int8_t*)x,
                       (bf16_t*)y, N, HW, C, scale, svec, u8);
  else
    hipLaunchKernelGGL(gap_i8_kernel<false>, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, (const int8_t*)x,
                       (bf16_t*)y, N, HW, C, scale, svec, u8);
  return hipGetLastError();
}
