// Batched GEMM with arbitrary operand strides (HK2: AutoGrad.mm / batchDot, KNRM
// similarity, InternalMM with batch broadcast):
//
//   C[b][m][n] = sum_k A(b, m, k) * B(b, n, k)       fp32 accumulate, fp32 or bf16 out
//
// A(b, m, k) = A[b*sab + m*sam + k*sak], B(b, n, k) = B[b*sbb + n*sbn + k*sbk]; a batch
// stride of 0 broadcasts the operand. Either the k or the m/n dimension of each operand
// may be the contiguous one, so every transpose combination of torch.matmul / bmm (and
// both backward products) runs without a transposed copy: the register staging writes
// the tile into LDS k-contiguous ([row][k], padded rows) whichever way it was read.
//
// 64x64 output tile per workgroup of 4 waves (2x2, 32x32 each = 2x2 tiles of
// v_mfma_f32_16x16x32_bf16), 32-deep k steps, double-buffered LDS with the next tile's
// global loads issued before the current tile's MFMAs.
#include "common.h"

namespace zoo {

constexpr int BM_T = 64, BM_K = 32, BM_LD = BM_K + 8;  // padded LDS row (80 B): conflict-light b128 reads

struct BmmGeom {
  int B, M, N, K;
  long sab, sam, sak, sbb, sbn, sbk;
  long scb, scm;  // C strides (n contiguous)
};

// load 8 consecutive elements along the contiguous dim (vector when VEC), or 8 strided ones
template <bool VEC>
ZOO_DEV void ld8_bf(const bf16_t* base, long step, int valid, bf16_t* v) {
  if (VEC && valid == 8) {
    const uint4 q = *reinterpret_cast<const uint4*>(base);
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&q);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = e[i];
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = i < valid ? base[(long)i * step] : (bf16_t)0;
  }
}

// stage a [64 rows][32 k] tile: thread t loads 8 elements. K-contiguous operands: row
// t/4, k (t%4)*8..+7 (one 16-byte load). Row-contiguous operands: k t/8, rows (t%8)*8..+7,
// scattered into 8 LDS rows.
template <bool VEC>
ZOO_DEV void stage_tile(const bf16_t* P, long srow, long sk, int rows, int K, int r0, int k0, bool kcontig,
                        bf16_t* lds, bf16_t* reg) {
  const int t = threadIdx.x;
  if (kcontig) {
    const int r = r0 + (t >> 2), k = k0 + (t & 3) * 8;
    const int valid = (r < rows) ? max(0, min(8, K - k)) : 0;
    if (valid > 0) ld8_bf<VEC>(P + (long)r * srow + (long)k * sk, sk, valid, reg);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) reg[i] = 0;
    }
  } else {
    const int k = k0 + (t >> 3), r = r0 + (t & 7) * 8;
    const int valid = (k < K) ? max(0, min(8, rows - r)) : 0;
    if (valid > 0) ld8_bf<VEC>(P + (long)r * srow + (long)k * sk, srow, valid, reg);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) reg[i] = 0;
    }
  }
  (void)lds;
}

ZOO_DEV void store_tile(bool kcontig, bf16_t* lds, const bf16_t* reg) {
  const int t = threadIdx.x;
  if (kcontig) {
    *reinterpret_cast<uint4*>(lds + (t >> 2) * BM_LD + (t & 3) * 8) = *reinterpret_cast<const uint4*>(reg);
  } else {
    const int k = t >> 3, r = (t & 7) * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) lds[(r + i) * BM_LD + k] = reg[i];
  }
}

template <bool VEC, bool OUT_BF16>
__global__ __launch_bounds__(256) void bmm_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ Bm,
                                                  void* __restrict__ C, BmmGeom g) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][BM_T * BM_LD];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BM_T * BM_LD];
  const int b = blockIdx.z, m0 = blockIdx.y * BM_T, n0 = blockIdx.x * BM_T;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, wm = w >> 1, wn = w & 1;
  const bf16_t* Ab = A + (long)b * g.sab + (long)m0 * g.sam;
  const bf16_t* Bb = Bm + (long)b * g.sbb + (long)n0 * g.sbn;
  const int mrows = g.M - m0, nrows = g.N - n0;
  const bool akc = g.sak == 1, bkc = g.sbk == 1;
  bf16_t ra[8], rb[8];
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (g.K + BM_K - 1) / BM_K;
  stage_tile<VEC>(Ab, g.sam, g.sak, mrows, g.K, 0, 0, akc, As[0], ra);
  stage_tile<VEC>(Bb, g.sbn, g.sbk, nrows, g.K, 0, 0, bkc, Bs[0], rb);
  store_tile(akc, As[0], ra);
  store_tile(bkc, Bs[0], rb);
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      stage_tile<VEC>(Ab, g.sam, g.sak, mrows, g.K, 0, (kt + 1) * BM_K, akc, As[cur ^ 1], ra);
      stage_tile<VEC>(Bb, g.sbn, g.sbk, nrows, g.K, 0, (kt + 1) * BM_K, bkc, Bs[cur ^ 1], rb);
    }
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
      af[i] = *reinterpret_cast<const bf16x8*>(As[cur] + (wm * 32 + i * 16 + fr) * BM_LD + fk);
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bfr[j] = *reinterpret_cast<const bf16x8*>(Bs[cur] + (wn * 32 + j * 16 + fr) * BM_LD + fk);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    if (more) {
      store_tile(akc, As[cur ^ 1], ra);
      store_tile(bkc, Bs[cur ^ 1], rb);
    }
    __syncthreads();
  }
  // C/D map of 16x16x32: row = 4*(lane>>4) + r, col = lane & 15
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
      if (col >= g.N) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (row >= g.M) continue;
        const long off = (long)b * g.scb + (long)row * g.scm + col;
        if (OUT_BF16) reinterpret_cast<bf16_t*>(C)[off] = f2bf(acc[i][j][r]);
        else reinterpret_cast<float*>(C)[off] = acc[i][j][r];
      }
    }
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_bmm(const void* A, const void* Bm, void* C, const long* geom, int out_bf16, int vec,
                              hipStream_t st) {
  BmmGeom g;
  g.B = (int)geom[0]; g.M = (int)geom[1]; g.N = (int)geom[2]; g.K = (int)geom[3];
  g.sab = geom[4]; g.sam = geom[5]; g.sak = geom[6];
  g.sbb = geom[7]; g.sbn = geom[8]; g.sbk = geom[9];
  g.scb = geom[10]; g.scm = geom[11];
  const dim3 grid((g.N + BM_T - 1) / BM_T, (g.M + BM_T - 1) / BM_T, g.B);
#define ZOO_BMM(V_, O_) \
  hipLaunchKernelGGL((bmm_kernel<V_, O_>), grid, dim3(256), 0, st, (const bf16_t*)A, (const bf16_t*)Bm, C, g)
  if (vec) { if (out_bf16) ZOO_BMM(true, true); else ZOO_BMM(true, false); }
  else { if (out_bf16) ZOO_BMM(false, true); else ZOO_BMM(false, false); }
#undef ZOO_BMM
  return hipGetLastError();
}
