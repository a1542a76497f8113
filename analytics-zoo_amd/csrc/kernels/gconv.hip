// Grouped convolution (Caffe `group`, ResNeXt cardinality) in ONE launch per direction
// (gfx950 / MI355X).
//
// The implicit-GEMM kernels (igemm / igemm2 / pw) take dense convs; a grouped conv used to be
// lowered as one dense conv per group over a channel slice (slice + pad + conv + slice + cat per
// group, zoo/pipeline/api/net/native_lower.py before round 6). Here the group index is the grid's
// y dimension and each workgroup computes one 64 x 64 tile of its group's GEMM, addressing the
// group's channel slice of the NHWC activations and its row block of the packed weights in place:
//
//   forward  Y[m][g Kg + n]          = act(bias + sum_(r,s,c) X[im2col(m; r,s)][g Cg + c] W[g Kg + n][(r,s,c)])
//   dgrad    dX[m][g Cg + c]         = sum_(r,s,k) dY[p(m,r), q(m,s)][g Kg + k] W[g Kg + k][(r,s,c)]
//                                      (only taps whose strided position lands on an output pixel)
//   wgrad    dW[g Kg + k][(r,s,c)]  += sum_m dY[m][g Kg + k] X[im2col(m; r,s)][g Cg + c]
//                                      (pixels split over grid.z, fp32 atomics)
//
// Operands are gathered into LDS as [row][32-deep k] bf16 tiles (16-byte loads when a group's
// channel slice is a multiple of 8 wide, element loads otherwise, e.g. ResNeXt's 4-channel groups)
// and multiplied with v_mfma_f32_16x16x32_bf16: 4 waves x (32 x 32) sub-tiles. Reference parity:
// BigDL SpatialConvolution(nGroup) that the Caffe converter maps `group` to
// (Zs/models/caffe/LayerConverter.scala:41-46), SURVEY.md §2.16 HK3.
#include "common.h"
#include "geom.h"

namespace zoo {


constexpr int GC_BM = 64, GC_BN = 64, GC_BK = 32, GC_LD = GC_BK + 8;  // LDS row pitch in elements

template <int MODE>  // 0 forward, 1 data gradient, 2 weight gradient
__global__ __launch_bounds__(256) void gconv_kernel(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wt,
                                                    const bf16_t* __restrict__ Dy, void* __restrict__ out,
                                                    const float* __restrict__ bias, GConvArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t As[GC_BM * GC_LD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[GC_BN * GC_LD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int grp = blockIdx.y;
  const int PQ = a.P * a.Q, HW = a.H * a.W;
  // per-mode GEMM extents: rows (Mg) x cols (Ng), reduction [k0, k1)
  int Mg, Ng, kbeg, kend;
  if constexpr (MODE == 0) {
    Mg = a.N * PQ; Ng = a.Kg; kbeg = 0; kend = a.R * a.S * a.Cg;
  } else if constexpr (MODE == 1) {
    Mg = a.N * HW; Ng = a.Cg; kbeg = 0; kend = a.R * a.S * a.Kg;
  } else {
    Mg = a.Kg; Ng = a.R * a.S * a.Cg;
    kbeg = blockIdx.z * a.mper;
    kend = min(a.N * PQ, kbeg + a.mper);
  }
  const int tiles_n = (Ng + GC_BN - 1) / GC_BN;
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x - tm * tiles_n;
  const int m0 = tm * GC_BM, n0 = tn * GC_BN;
  if (m0 >= Mg || kbeg >= kend) return;

  // staging: thread -> tile row sr (0..63), 8 consecutive reduction indices at sk
  const int sr = tid >> 2, sk = (tid & 3) * 8;
  const bool vecA = MODE == 0 ? (a.Cg % 8 == 0) : MODE == 1 ? (a.Kg % 8 == 0) : false;
  const bool vecB = MODE == 0;   // packed weight rows: contiguous reduction index

  // A element (row, kk) for this mode
  auto a_elem = [&](int row, int kk) -> bf16_t {
    if (row >= Mg || kk >= kend) return 0;
    if constexpr (MODE == 0) {
      const int n = row / PQ, pq = row - n * PQ, p = pq / a.Q, q = pq - p * a.Q;
      const int rs = kk / a.Cg, c = kk - rs * a.Cg, r = rs / a.S, s = rs - r * a.S;
      const int ih = p * a.sh - a.ph + r * a.dh, iw = q * a.sw - a.pw + s * a.dw;
      if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return 0;
      return X[((size_t)(n * a.H + ih) * a.W + iw) * a.C + grp * a.Cg + c];
    } else if constexpr (MODE == 1) {
      const int n = row / HW, hw = row - n * HW, h = hw / a.W, x = hw - h * a.W;
      const int rs = kk / a.Kg, k = kk - rs * a.Kg, r = rs / a.S, s = rs - r * a.S;
      const int th = h + a.ph - r * a.dh, tw = x + a.pw - s * a.dw;
      if (th < 0 || tw < 0 || th % a.sh || tw % a.sw) return 0;
      const int p = th / a.sh, q = tw / a.sw;
      if (p >= a.P || q >= a.Q) return 0;
      return Dy[((size_t)(n * a.P + p) * a.Q + q) * a.K + grp * a.Kg + k];
    } else {
      return Dy[(size_t)kk * a.K + grp * a.Kg + row];   // row = output channel k, kk = pixel
    }
  };
  // B element (col, kk)
  auto b_elem = [&](int col, int kk) -> bf16_t {
    if (col >= Ng || kk >= kend) return 0;
    if constexpr (MODE == 0) {
      return Wt[(size_t)(grp * a.Kg + col) * a.ldb + kk];
    } else if constexpr (MODE == 1) {
      const int rs = kk / a.Kg, k = kk - rs * a.Kg;
      return Wt[(size_t)(grp * a.Kg + k) * a.ldb + rs * a.Cg + col];
    } else {
      const int n = kk / PQ, pq = kk - n * PQ, p = pq / a.Q, q = pq - p * a.Q;
      const int rs = col / a.Cg, c = col - rs * a.Cg, r = rs / a.S, s = rs - r * a.S;
      const int ih = p * a.sh - a.ph + r * a.dh, iw = q * a.sw - a.pw + s * a.dw;
      if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return 0;
      return X[((size_t)(n * a.H + ih) * a.W + iw) * a.C + grp * a.Cg + c];
    }
  };
  // 8 consecutive reduction indices of one row as a 16-byte piece
  auto a_piece = [&](int row, int kk0) -> uint4 {
    if (vecA && row < Mg && kk0 + 8 <= kend) {
      if constexpr (MODE == 0) {
        const int n = row / PQ, pq = row - n * PQ, p = pq / a.Q, q = pq - p * a.Q;
        const int rs = kk0 / a.Cg, c = kk0 - rs * a.Cg, r = rs / a.S, s = rs - r * a.S;
        const int ih = p * a.sh - a.ph + r * a.dh, iw = q * a.sw - a.pw + s * a.dw;
        if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return make_uint4(0u, 0u, 0u, 0u);
        return *reinterpret_cast<const uint4*>(X + ((size_t)(n * a.H + ih) * a.W + iw) * a.C + grp * a.Cg + c);
      } else if constexpr (MODE == 1) {
        const int n = row / HW, hw = row - n * HW, h = hw / a.W, x = hw - h * a.W;
        const int rs = kk0 / a.Kg, k = kk0 - rs * a.Kg, r = rs / a.S, s = rs - r * a.S;
        const int th = h + a.ph - r * a.dh, tw = x + a.pw - s * a.dw;
        if (th < 0 || tw < 0 || th % a.sh || tw % a.sw) return make_uint4(0u, 0u, 0u, 0u);
        const int p = th / a.sh, q = tw / a.sw;
        if (p >= a.P || q >= a.Q) return make_uint4(0u, 0u, 0u, 0u);
        return *reinterpret_cast<const uint4*>(Dy + ((size_t)(n * a.P + p) * a.Q + q) * a.K + grp * a.Kg + k);
      }
    }
    uint32_t v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = (uint32_t)a_elem(row, kk0 + 2 * e) | ((uint32_t)a_elem(row, kk0 + 2 * e + 1) << 16);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  auto b_piece = [&](int col, int kk0) -> uint4 {
    // packed weight rows are zero-padded to ldb: a whole piece below ldb is in bounds
    if (vecB && col < Ng && kk0 + 8 <= a.ldb) {
      if constexpr (MODE == 0) return *reinterpret_cast<const uint4*>(Wt + (size_t)(grp * a.Kg + col) * a.ldb + kk0);
    }
    uint32_t v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = (uint32_t)b_elem(col, kk0 + 2 * e) | ((uint32_t)b_elem(col, kk0 + 2 * e + 1) << 16);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = w >> 1, wn = w & 1, fr = lane & 15, fq = lane >> 4;

  uint4 pa = a_piece(m0 + sr, kbeg + sk), pb = b_piece(n0 + sr, kbeg + sk);
  for (int k0 = kbeg; k0 < kend; k0 += GC_BK) {
    __syncthreads();
    *reinterpret_cast<uint4*>(As + sr * GC_LD + sk) = pa;
    *reinterpret_cast<uint4*>(Bs + sr * GC_LD + sk) = pb;
    __syncthreads();
    if (k0 + GC_BK < kend) {   // next tile's loads in flight during the MFMAs
      pa = a_piece(m0 + sr, k0 + GC_BK + sk);
      pb = b_piece(n0 + sr, k0 + GC_BK + sk);
    }
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(As + (wm * 32 + i * 16 + fr) * GC_LD + 8 * fq);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 32 + j * 16 + fr) * GC_LD + 8 * fq);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  }

  // D[row][col]: row = 4 * fq + e of the 16-row block, col = fr
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * 32 + i * 16 + 4 * fq + e, col = n0 + wn * 32 + j * 16 + fr;
        if (row >= Mg || col >= Ng) continue;
        const float v = acc[i][j][e];
        if constexpr (MODE == 0) {
          const int ch = grp * a.Kg + col;
          const float o = apply_act(v + (bias ? bias[ch] : 0.f), a.act);
          reinterpret_cast<bf16_t*>(out)[(size_t)row * a.K + ch] = f2bf(o);
        } else if constexpr (MODE == 1) {
          reinterpret_cast<bf16_t*>(out)[(size_t)row * a.C + grp * a.Cg + col] = f2bf(v);
        } else {
          atomicAdd(reinterpret_cast<float*>(out) + (size_t)(grp * a.Kg + row) * a.ldb + col, v);
        }
      }
}

}  // namespace zoo

using namespace zoo;

// mode 0: out = Y bf16 [N, P, Q, K]; 1: out = dX bf16 [N, H, W, C]; 2: out = dW fp32 [K, ldb] (+=)
extern "C" hipError_t zoo_gconv(int mode, const void* X, const void* Wt, const void* Dy, void* out, const float* bias,
                                const GConvArgs* ap, hipStream_t st) {
  GConvArgs a = *ap;
  if (mode == 0) {
    const int tiles = ((a.N * a.P * a.Q + GC_BM - 1) / GC_BM) * ((a.Kg + GC_BN - 1) / GC_BN);
    hipLaunchKernelGGL(gconv_kernel<0>, dim3(tiles, a.groups), dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)Wt,
                       (const bf16_t*)Dy, out, bias, a);
  } else if (mode == 1) {
    const int tiles = ((a.N * a.H * a.W + GC_BM - 1) / GC_BM) * ((a.Cg + GC_BN - 1) / GC_BN);
    hipLaunchKernelGGL(gconv_kernel<1>, dim3(tiles, a.groups), dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)Wt,
                       (const bf16_t*)Dy, out, bias, a);
  } else {
    const int M = a.N * a.P * a.Q;
    const int tiles = ((a.Kg + GC_BM - 1) / GC_BM) * ((a.R * a.S * a.Cg + GC_BN - 1) / GC_BN);
    // pixel splits: ~1024 workgroups in flight in total, >= 256 pixels each
    int splits = (1024 + tiles * a.groups - 1) / (tiles * a.groups);
    const int maxs = (M + 255) / 256;
    if (splits > maxs) splits = maxs;
    if (splits < 1) splits = 1;
    a.mper = ((M + splits - 1) / splits + GC_BK - 1) / GC_BK * GC_BK;
    splits = (M + a.mper - 1) / a.mper;
    hipLaunchKernelGGL(gconv_kernel<2>, dim3(tiles, a.groups, splits), dim3(256), 0, st, (const bf16_t*)X,
                       (const bf16_t*)Wt, (const bf16_t*)Dy, out, bias, a);
  }
  return hipGetLastError();
}
