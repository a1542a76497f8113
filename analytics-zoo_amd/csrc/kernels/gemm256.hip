// Large-tile bf16 GEMM for gfx950:  Y[M, N] = epilogue( A[M, K] · B[N, K]^T )
//
// Used for the GEMM-shaped hot ops whose operands are plain K-contiguous
// matrices: Linear layers and 1x1 stride-1 convolutions (fwd: A = NHWC
// activations, B = weights [Cout][Cin]; dgrad: A = dY, B = transposed weights).
//
// Structure (cdna_hip_programming.md §5 "The 256² 8-phase template", re-derived):
//   * 256 x 256 output tile, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N);
//     each wave owns 128 x 64 outputs = 8 x 4 tiles of v_mfma_f32_16x16x32_bf16
//     (128 accumulator VGPRs).
//   * A K-tile is split into four 16 KiB "half-tiles": the two A halves hold the
//     rows each wave reads for its upper / lower 64-row quadrant, the two B halves
//     the columns for its left / right 32-column quadrant. Each half-tile is stored
//     as 16 fragment-shaped 1 KiB subtiles [16 rows][32 k], XOR-swizzled so the
//     16-lane groups of a ds_read_b128 hit 16 distinct 16-byte bank slots.
//   * Staging is global_load_lds (LDS-DMA, 16 B per lane, no VGPRs): the LDS image
//     is lane-linear and the swizzle lives in the per-lane SOURCE address. Rows
//     beyond M/N and k beyond K read a zero page.
//   * Each K-tile runs as 4 phases, one output quadrant (16 MFMAs) per phase.
//     One half-tile is staged per phase, 5-6 phases before it is read, into the
//     other LDS buffer or into the part of this buffer the earlier phases have
//     finished reading (>= 2 phases after its last read). The wait is a counted
//     `s_waitcnt vmcnt(8)` (4 younger half-tiles = 8 DMA instructions may stay in
//     flight) followed by one raw s_barrier per phase — never a full drain in the
//     main loop.
//   * Epilogue: accumulators -> LDS (per-wave 64x64 fp32 region, swizzled) -> row-
//     contiguous 16 B stores, with optional bias, residual, activation, BatchNorm
//     statistics (sum, sum^2) and the fused BN-backward reduction (BwdStats).
#include "common.h"
#include "geom.h"

namespace zoo {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gl_void;

constexpr int G_BM = 256, G_BN = 256, G_BK = 64, G_NT = 512;
constexpr int HALF_BYTES = 16384;

ZOO_DEV void wait_vm8() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }
ZOO_DEV void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
ZOO_DEV void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// byte offset of (row r in 0..15, 16-byte chunk c in 0..3) inside a 1 KiB subtile
ZOO_DEV int sub_off(int r, int c) { return r * 64 + (((c ^ (r >> 2)) & 3) << 4); }

__global__ __launch_bounds__(G_NT, 1) void gemm256_kernel(const bf16_t* __restrict__ A,
                                                          const bf16_t* __restrict__ B, bf16_t* __restrict__ Y,
                                                          float* __restrict__ Yf, const float* __restrict__ bias,
                                                          const bf16_t* __restrict__ resid, float* __restrict__ stats,
                                                          GemmGeom g, int act, BwdStats bs,
                                                          const bf16_t* __restrict__ zpage) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 2, wn = w & 3;

  const int ntn = (g.N + G_BN - 1) / G_BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * G_BM, n0 = (bid % ntn) * G_BN;
  const int nk = (g.K + G_BK - 1) / G_BK;

  // ---- per-thread DMA source rows (2 instructions per half-tile) ----
  const int r16 = lane >> 2;                          // row inside the subtile this lane fills
  const int kofs = (w & 1) * 32 + (((lane & 3) ^ (lane >> 4)) << 3);  // k inside the K-tile
  // A-half h, instr j: row = j*128 + h*64 + (w>>1)*16 + r16
  // B-half h, instr j: row = (j*2 + (w>>2))*64 + h*32 + ((w>>1)&1)*16 + r16
  int arow[2][2], brow[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      arow[h][j] = m0 + j * 128 + h * 64 + (w >> 1) * 16 + r16;
      brow[h][j] = n0 + (j * 2 + (w >> 2)) * 64 + h * 32 + ((w >> 1) & 1) * 16 + r16;
    }

  auto half_base = [&](int buf, int op, int h) -> char* {
    return smem + (((buf * 2 + op) * 2 + h) * HALF_BYTES);
  };

  // stage half-tile (op, h) of K-tile kt into its buffer
  auto stage = [&](int kt, int op, int h) {
    const int k = kt * G_BK + kofs;
    char* hb = half_base(kt & 1, op, h);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = op == 0 ? arow[h][j] : brow[h][j];
      const int lim = op == 0 ? g.M : g.N;
      const bool ok = row < lim && k < g.K;
      const bf16_t* src = op == 0 ? A + (size_t)row * g.lda + k : B + (size_t)row * g.ldb + k;
      src = ok ? src : zpage;
      char* dst = hb + (j * 8 + w) * 1024;
      __builtin_amdgcn_global_load_lds((gl_void*)src, (lds_void*)dst, 16, 0, 0);
    }
  };

  // fragment reads: lane (r = lane&15, c = lane>>4) of subtile st
  const int frag_off = sub_off(lane & 15, lane >> 4);
  auto read_frag = [&](int buf, int op, int h, int st) -> bf16x8 {
    return *reinterpret_cast<const bf16x8*>(half_base(buf, op, h) + st * 1024 + frag_off);
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];

  // prologue: the six half-tiles the steady state would have staged at phases -6..-1
  stage(0, 0, 0);
  stage(0, 1, 0);
  stage(0, 1, 1);
  stage(0, 0, 1);
  if (nk > 1) {
    stage(1, 0, 0);
    stage(1, 1, 0);
    wait_vm8();
  } else {
    wait_vm0();
  }
  __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // 1) fragment reads for this phase (retired by the previous phase's wait + barrier)
      if (p == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fa[i][kb] = read_frag(buf, 0, 0, (wm * 4 + i) * 2 + kb);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fb0[j][kb] = read_frag(buf, 1, 0, (wn * 2 + j) * 2 + kb);
      } else if (p == 1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fb1[j][kb] = read_frag(buf, 1, 1, (wn * 2 + j) * 2 + kb);
      } else if (p == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kb = 0; kb < 2; ++kb) fa[i][kb] = read_frag(buf, 0, 1, (wm * 4 + i) * 2 + kb);
      }
      // 2) stage one half-tile: P0 -> B1(kt+1), P1 -> A1(kt+1), P2 -> A0(kt+2), P3 -> B0(kt+2)
      const int skt = p < 2 ? kt + 1 : kt + 2;
      const bool valid = skt < nk;
      if (valid) stage(skt, p == 1 || p == 2 ? 0 : 1, p == 0 || p == 1 ? 1 : 0);
      // 3) retire the half-tile the NEXT phase reads, then sync the workgroup
      if (valid) wait_vm8(); else wait_vm0();
      __builtin_amdgcn_s_barrier();
      wait_lgkm0();
      // 4) 16 MFMAs on quadrant (qa, qb): P0 (0,0), P1 (0,1), P2 (1,1), P3 (1,0)
      const int qa = p >= 2 ? 1 : 0;
      const int qb = (p == 1 || p == 2) ? 1 : 0;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[qa][qb][i][j] = mfma16(fa[i][kb], qb ? fb1[j][kb] : fb0[j][kb], acc[qa][qb][i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  wait_vm0();
  __builtin_amdgcn_s_barrier();

  // ---- epilogue: two passes (row quadrants), each wave stages 64 x 64 fp32 ----
  float* Cs = reinterpret_cast<float*>(smem) + w * 64 * 64;
  const int fr = lane & 15, fq = lane >> 4;
  const int c8 = lane & 7;         // 8-column chunk of this lane
  const int rsub = lane >> 3;      // row offset 0..7
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  const int colg = n0 + wn * 64 + c8 * 8;
  const bool col_ok = colg < g.N;
  float bsv[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bsv[e] = (bias && col_ok) ? bias[colg + e] : 0.f;

#pragma unroll
  for (int qa = 0; qa < 2; ++qa) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int prow = i * 16 + fq * 4 + r;
            const int col = qb * 32 + j * 16 + fr;
            Cs[prow * 64 + ((((col >> 2) ^ (prow & 15)) << 2) | (col & 3))] = acc[qa][qb][i][j][r];
          }
    wait_lgkm0();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int prow = it * 8 + rsub;
      const int m = m0 + wm * 128 + qa * 64 + prow;
      if (m >= g.M || !col_ok) continue;
      const float4 lo = *reinterpret_cast<const float4*>(Cs + prow * 64 + (((2 * c8) ^ (prow & 15)) << 2));
      const float4 hi = *reinterpret_cast<const float4*>(Cs + prow * 64 + (((2 * c8 + 1) ^ (prow & 15)) << 2));
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const size_t off = (size_t)m * g.ldy + colg;
      if (resid) {
        float rv[8];
        unpack8(*reinterpret_cast<const uint4*>(resid + off), rv);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += rv[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e] + bsv[e], act);
      if (Yf) {
        *reinterpret_cast<float4*>(Yf + off) = make_float4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<float4*>(Yf + off + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
      if (bs.sums && bs.z) {
        float zz[8];
        unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.z) + off), zz);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = zz[e] > 0.f ? v[e] : 0.f;
      }
      if (Y) {
        const uint4 pk = pack8(v);
        *reinterpret_cast<uint4*>(Y + off) = pk;
        float q[8];
        unpack8(pk, q);
        if (stats) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { s1[e] += q[e]; s2[e] += q[e] * q[e]; }
        } else if (bs.sums) {
          float yy[8];
          unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off), yy);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += q[e];
            s2[e] += q[e] * (yy[e] - bs.mean[colg + e]) * bs.inv[colg + e];
          }
        }
      }
    }
  }

  float* const sacc = stats ? stats : bs.sums;
  if (sacc) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    }
    if (lane < 8 && col_ok) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(sacc + colg + e, s1[e]);
        atomicAdd(sacc + g.N + colg + e, s2[e]);
      }
    }
  }
}

}  // namespace zoo

using namespace zoo;

static const bf16_t* zero_page() {
  static bf16_t* z = nullptr;
  if (!z) {
    hipMalloc(&z, 4096);
    hipMemset(z, 0, 4096);
  }
  return z;
}

extern "C" hipError_t zoo_gemm256(const void* A, const void* B, void* Y, float* Yf, const float* bias,
                                  const void* resid, float* stats, const GemmGeom* gp, int act, const BwdStats* bsp,
                                  hipStream_t st) {
  const GemmGeom g = *gp;
  BwdStats bs = bsp ? *bsp : BwdStats{nullptr, nullptr, nullptr, nullptr, nullptr};
  const int tiles = ((g.M + G_BM - 1) / G_BM) * ((g.N + G_BN - 1) / G_BN);
  const size_t smem = 4 * 2 * HALF_BYTES;  // 2 buffers x (A, B) x 2 halves = 128 KiB
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm256_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                        (int)smem);
    attr = true;
  }
  const bf16_t* zp = zero_page();
  hipLaunchKernelGGL(gemm256_kernel, dim3(tiles), dim3(G_NT), smem, st, (const bf16_t*)A, (const bf16_t*)B,
                     (bf16_t*)Y, Yf, bias, (const bf16_t*)resid, stats, g, act, bs, zp);
  return hipGetLastError();
}
