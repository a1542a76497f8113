// Streaming pointwise (1x1, stride-1) convolution / GEMM for the memory-bound shapes of a
// ResNet training step (gfx950 / MI355X).
//
//   Y[m][n] = epilogue( sum_k A[m][k] * B[n][k] )      A: NHWC activations [M][K] (K = Cin),
//                                                       B: weights [N][ldb] (row n = output channel)
//
// Why a third GEMM kernel: the 1x1 convs whose output width is 64 / 128 channels (and the
// 64 / 128-deep ones with 256 / 512 outputs) do 26 GFLOP at b256 but move 0.1 - 0.6 GB, so they
// are bound by HBM, and the BN-fused epilogues are half of those bytes. The tiled kernels
// (igemm.hip / igemm2.hip) run one output tile per workgroup: every tile pays its operand
// latency, then its epilogue latency (the producer y loads of the fused BN backward), then
// atomics on the same 2K statistics addresses from every one of 6272 tiles -- a stage-1
// conv3 data gradient with the BN-backward epilogue took 283-316 us against ~110 us of bytes
// (profiles/r3/resnet50_b256_step_timeline_final_r3.md #353/#370).
//
// Structure (no LDS operand ring, no barrier in the main loop):
//   * persistent: every WAVE walks its own sequence of 16 / 32-pixel tiles; the grid is one
//     occupancy-full wave of workgroups. Output channels are split across workgroups in groups of
//     NP = 64 / 128 (N / NP = NSPLIT groups): workgroup b owns group g and LDS holds only that
//     group's NP x K weights (<= 64 KiB), loaded ONCE in MFMA fragment order (1 KiB per 16-row x
//     32-deep fragment, lane-linear: conflict-free ds_read_b128) as the MFMA A operand. The
//     NSPLIT workgroups that share a pixel range sit on one XCD (blocks b, b+8, ... share an XCD
//     under round-robin dispatch) and walk it in step, so the activations come from HBM once and
//     from that XCD's L2 the other NSPLIT - 1 times;
//   * the activations are the MFMA B operand and a 16x16x32 B fragment is exactly one 16-byte
//     global load per lane (pixel lane & 15, k-chunk lane >> 4): the tile goes straight from
//     HBM into VGPRs, and the NEXT tile's loads are issued before this tile's MFMAs (a 16 KiB
//     register double buffer per wave, 8 waves per CU: ~128 KiB in flight per CU);
//   * D = W . A^T puts one pixel on each lane and 4 consecutive output channels in its 4
//     accumulator registers; a wave-private LDS patch turns them into row-contiguous 16-byte
//     pieces for the epilogue (full-line NHWC loads / stores). Its global operands (producer y, residual gradient,
//     ReLU mask) are issued at the top of the tile, BEFORE the next tile's prefetch, so the
//     in-order vmcnt never makes the epilogue wait for the prefetch;
//   * BatchNorm statistics / BN-backward sums: per-lane registers for the whole kernel (a lane's
//     8-channel chunk is fixed), one shuffle reduction + LDS add at exit, one global atomic per
//     channel per WORKGROUP.
//
// Epilogues: EPI 1 = bf16 output + BN statistics of the stored values (the forward of every
// conv->BN unit); EPI 3 = EPI 1 for the ResNet stem as a 4x4 conv on the space-to-depth image
// (16 channels, 256-deep reduction): the activation fragments are gathered from the 4x4 window
// (two taps x 16 channels per 32-deep k-block: 64 contiguous bytes per pixel) instead of read as
// a row; EPI 2 = backward: residual-gradient add, producer ReLU mask (bnmask.h zmodes)
// and the producer's fused BN-backward sums (sum dy, sum dy * xhat).
// Prologue (PRO, EPI 2, K = 64 / 128): the activation operand is the unit's OWN BN backward,
// dy = A g + B y + Cc, formed in the operand registers from the masked gradient g and the unit's
// pre-BN output y as they arrive (per-channel A | B | Cc in LDS); channel group 0 also writes dy
// for the weight gradient (bnfold.hip: the separate BN-backward apply pass and the re-read of dy
// are gone).
// Reference parity: MKL-DNN 1x1 convolution primitives behind BigDL SpatialConvolution
// (Zs/pipeline/api/keras/layers/Convolution2D.scala:86-110), SURVEY.md §2.16 HK3 / HK5.
#include <stdlib.h>

#include "common.h"
#include "geom.h"

namespace zoo {

struct PwArgs {
  int M;          // rows (pixels)
  int N;          // output channels (row stride of Y / y / resid)
  int ldb;        // weight row stride (elements)
  int nsplit;     // channel groups of NP (N = nsplit * NP)
  int stat_mode;  // 0: atomics into stats[0..2N), >0: slotted (slot_ptr), kStatPartial: [grid][2N] rows
  int gH, gW, gP, gQ;   // EPI 3 (stem gather): input / output spatial size
};

constexpr int PW_NW = 8;  // waves per workgroup (2 per SIMD)

// NP = output channels per workgroup (64 / 128), TPM = pixels per wave tile (16 / 32), KT = K / 32
template <int NP, int TPM, int KT, int EPI, bool PRO>
__global__ __launch_bounds__(PW_NW * 64, 1) void pw_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                           bf16_t* __restrict__ Y, const bf16_t* __restrict__ resid,
                                                           float* __restrict__ stats, PwArgs p, BwdStats bs) {
  constexpr int K = KT * 32;
  constexpr int MJ = TPM / 16, NI = NP / 16;
  constexpr int NT = PW_NW * 64;
  // epilogue geometry: row-contiguous pieces of 8 channels; CPR lanes cover one NP-channel row
  constexpr int CPR = NP / 8, RPP = 64 / CPR, HP = 16 / RPP, PITCH = NP + 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wfr = smem;                                                // NI * KT fragments of 1 KiB
  float* ssum = reinterpret_cast<float*>(smem + NP * K * 2);       // [2][NP] statistics
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int N = p.N;
  float* patch = ssum + 2 * NP + w * 16 * PITCH;                   // wave-private fp32 16 x NP patch
  float* pco = ssum + 2 * NP + PW_NW * 16 * PITCH;                 // PRO: A | B | Cc, [3][K] (+ EPI 4: rA | - | rC)
  float* ssum3 = pco + (PRO ? (EPI == 4 ? 6 : 3) * K : 0);         // [NP] sums against y2 (EPI 2)
  // the y2 sums only in the short-reduction backward kernels (their registers have room; the
  // 256-deep prologue kernels run at 256 VGPRs): the host does not route y2 calls elsewhere
  constexpr bool Y2 = EPI == 2 && (KT <= 2 || (!PRO && KT <= 4));
  const bool y2on = Y2 && bs.y2 != nullptr;

  // ---- workgroup -> (channel group, pixel group); XCD-local channel groups ----
  const int b = blockIdx.x, G = gridDim.x;
  const int xcd = b & 7, li = b >> 3;
  const int g = li % p.nsplit;
  const int mg = (li / p.nsplit) * 8 + xcd;          // pixel group (set of 8 wave streams)
  const int MG = G / p.nsplit;                       // pixel groups (launcher: G % (8 * nsplit) == 0)
  const int n0 = g * NP;

  // ---- this group's weights -> LDS fragment image ----
  for (int idx = tid; idx < NP * KT * 4; idx += NT) {
    const int n = idx / (KT * 4), kc = idx - n * (KT * 4);
    const int kb = kc >> 2, q = kc & 3;
    const uint4 v = *reinterpret_cast<const uint4*>(B + (size_t)(n0 + n) * p.ldb + kc * 8);
    *reinterpret_cast<uint4*>(wfr + (((n >> 4) * KT + kb) * 64 + (n & 15) + 16 * q) * 16) = v;
  }
  for (int c = tid; c < 2 * NP; c += NT) ssum[c] = 0.f;
  if (y2on)
    for (int c = tid; c < NP; c += NT) ssum3[c] = 0.f;
  if constexpr (PRO)
    for (int c = tid; c < 3 * K; c += NT) pco[c] = bs.pro_coef[c];
  if constexpr (PRO && EPI == 4)
    if (bs.pro_rcoef)
      for (int c = tid; c < 3 * K; c += NT) pco[3 * K + c] = bs.pro_rcoef[c];
  __syncthreads();

  const bool bnsum = EPI == 2 && bs.sums != nullptr && !bs.zgelu;
  const bool want = EPI != 2 ? stats != nullptr : bnsum;
  const int ch = lane % CPR, lr = lane / CPR;
  const int c0 = n0 + ch * 8;                        // the lane's fixed 8-channel chunk
  // per-lane BN constants of that chunk (EPI 2)
  float cmu[8], civ[8], csc[8], csh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { cmu[e] = civ[e] = csc[e] = csh[e] = 0.f; }
  if (EPI == 2 && bnsum) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      cmu[e] = bs.mean[c0 + e];
      civ[e] = bs.inv[c0 + e];
      if (bs.zmode == 1) {
        csc[e] = bs.mgamma ? bs.mgamma[c0 + e] * civ[e] : civ[e];
        csh[e] = (bs.mbeta ? bs.mbeta[c0 + e] : 0.f) - cmu[e] * csc[e];
      }
    }
  }
  float s1[8], s2[8], s3[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; s3[e] = 0.f; }

  const int ntiles = (p.M + TPM - 1) / TPM;
  const int gw = mg * PW_NW + w, GW = MG * PW_NW;

  // A fragments of tile t: lane -> pixel row t*TPM + 16 j + fr, k-chunk kb*32 + 8 fq
  // (PRO: the unit's pre-BN output y at the same positions into yf)
  // PRO with EPI 1: the forward consumer-side BN apply -- one operand (X = y), no y fragments
  constexpr bool PRO_Y = PRO && EPI == 2;
  // EPI 4: the forward prologue of a residual unit reads the residual at the operand positions
  constexpr bool PRO_R = PRO && EPI == 4;
  constexpr int YJ = (PRO_Y || PRO_R) ? MJ : 1, YK = (PRO_Y || PRO_R) ? KT : 1;
  const bf16_t* const pro_y = reinterpret_cast<const bf16_t*>(bs.pro_y);
  bf16_t* const pro_dy = reinterpret_cast<bf16_t*>(bs.pro_dy);
  auto load_tile = [&](int t, bf16x8 (&af)[MJ][KT], bf16x8 (&yf)[YJ][YK]) {
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      int row = t * TPM + 16 * j + fr;
      row = row < p.M ? row : p.M - 1;  // rows past M compute garbage that is never stored
      if constexpr (EPI == 3) {
        // stem gather: k = (r * 4 + s) * 16 + c; k-block kb holds taps 2 kb, 2 kb + 1
        const int PQ = p.gP * p.gQ;
        const int n = row / PQ, rem = row - n * PQ, y = rem / p.gQ, x = rem - y * p.gQ;
        const bf16_t* base = A + (((size_t)n * p.gH + y) * p.gW + x) * 16 + 8 * (fq & 1);
#pragma unroll
        for (int kb = 0; kb < KT; ++kb) {
          const int tap = 2 * kb + (fq >> 1), r = tap >> 2, s = tap & 3;
          af[j][kb] = *reinterpret_cast<const bf16x8*>(base + ((size_t)r * p.gW + s) * 16);
        }
      } else {
        const bf16_t* src = A + (size_t)row * K + 8 * fq;
#pragma unroll
        for (int kb = 0; kb < KT; ++kb) af[j][kb] = *reinterpret_cast<const bf16x8*>(src + kb * 32);
      }
      if constexpr (PRO_Y) {
        const bf16_t* ys = pro_y + (size_t)row * K + 8 * fq;
#pragma unroll
        for (int kb = 0; kb < KT; ++kb) yf[j][kb] = *reinterpret_cast<const bf16x8*>(ys + kb * 32);
      }
      if constexpr (PRO_R) {
        const bf16_t* rs = reinterpret_cast<const bf16_t*>(bs.pro_res) + (size_t)row * K + 8 * fq;
#pragma unroll
        for (int kb = 0; kb < KT; ++kb) yf[j][kb] = *reinterpret_cast<const bf16x8*>(rs + kb * 32);
      }
    }
  };
  // PRO, EPI 1: z = relu(A y + Cc) in place of y (and, channel group 0, stored: the unit's output)
  auto prologue_fwd = [&](int t, bf16x8 (&af)[MJ][KT]) {
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int row = t * TPM + 16 * j + fr;
      const bool st = g == 0 && pro_dy != nullptr && row < p.M;
#pragma unroll
      for (int kb = 0; kb < KT; ++kb) {
        const int k0 = kb * 32 + 8 * fq;
        const uint4 xu = __builtin_bit_cast(uint4, af[j][kb]);
        const uint32_t xw4[4] = {xu.x, xu.y, xu.z, xu.w};
        uint32_t ow[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 a4 = *reinterpret_cast<const float4*>(pco + k0 + 4 * h);
          const float4 c4 = *reinterpret_cast<const float4*>(pco + 2 * K + k0 + 4 * h);
          const uint32_t x0 = xw4[2 * h], x1 = xw4[2 * h + 1];
          const float o0 = fmaxf(a4.x * __uint_as_float(x0 << 16) + c4.x, 0.f);
          const float o1 = fmaxf(a4.y * __uint_as_float(x0 & 0xffff0000u) + c4.y, 0.f);
          const float o2 = fmaxf(a4.z * __uint_as_float(x1 << 16) + c4.z, 0.f);
          const float o3 = fmaxf(a4.w * __uint_as_float(x1 & 0xffff0000u) + c4.w, 0.f);
          ow[2 * h] = pack2bf(o0, o1);
          ow[2 * h + 1] = pack2bf(o2, o3);
        }
        const uint4 pk = make_uint4(ow[0], ow[1], ow[2], ow[3]);
        af[j][kb] = __builtin_bit_cast(bf16x8, pk);
        if (st) *reinterpret_cast<uint4*>(pro_dy + (size_t)row * K + k0) = pk;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // PRO, EPI 4: z = relu(A y + Cc + R), R the residual (or rA r + rC with a shortcut BatchNorm); channel
  // group 0 stores z (the block output, the next residual) and its 1-bit ReLU mask
  auto prologue_fwd_res = [&](int t, bf16x8 (&af)[MJ][KT], const bf16x8 (&rf)[YJ][YK]) {
    asm volatile("" ::: "memory");
    const bool raff = bs.pro_rcoef != nullptr;
    uint8_t* const pmask = reinterpret_cast<uint8_t*>(bs.pro_mask);
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
      const int row = t * TPM + 16 * j + fr;
      const bool st = g == 0 && pro_dy != nullptr && row < p.M;
#pragma unroll
      for (int kb = 0; kb < KT; ++kb) {
        const int k0 = kb * 32 + 8 * fq;
        float yv[8], rv[8];
        unpack8(__builtin_bit_cast(uint4, af[j][kb]), yv);
        unpack8(__builtin_bit_cast(uint4, rf[j][kb]), rv);
        float o[8];
        unsigned bits = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 a4 = *reinterpret_cast<const float4*>(pco + k0 + 4 * h);
          const float4 c4 = *reinterpret_cast<const float4*>(pco + 2 * K + k0 + 4 * h);
          float r4[4] = {rv[4 * h], rv[4 * h + 1], rv[4 * h + 2], rv[4 * h + 3]};
          if (raff) {
            const float4 ra = *reinterpret_cast<const float4*>(pco + 3 * K + k0 + 4 * h);
            const float4 rc = *reinterpret_cast<const float4*>(pco + 5 * K + k0 + 4 * h);
            r4[0] = r4[0] * ra.x + rc.x;
            r4[1] = r4[1] * ra.y + rc.y;
            r4[2] = r4[2] * ra.z + rc.z;
            r4[3] = r4[3] * ra.w + rc.w;
          }
          const float v0 = a4.x * yv[4 * h] + c4.x + r4[0], v1 = a4.y * yv[4 * h + 1] + c4.y + r4[1];
          const float v2 = a4.z * yv[4 * h + 2] + c4.z + r4[2], v3 = a4.w * yv[4 * h + 3] + c4.w + r4[3];
          bits |= (v0 > 0.f ? 1u : 0u) << (4 * h);
          bits |= (v1 > 0.f ? 1u : 0u) << (4 * h + 1);
          bits |= (v2 > 0.f ? 1u : 0u) << (4 * h + 2);
          bits |= (v3 > 0.f ? 1u : 0u) << (4 * h + 3);
          o[4 * h] = fmaxf(v0, 0.f);
          o[4 * h + 1] = fmaxf(v1, 0.f);
          o[4 * h + 2] = fmaxf(v2, 0.f);
          o[4 * h + 3] = fmaxf(v3, 0.f);
        }
        const uint4 pk = pack8(o);
        af[j][kb] = __builtin_bit_cast(bf16x8, pk);
        if (st) {
          *reinterpret_cast<uint4*>(pro_dy + (size_t)row * K + k0) = pk;
          if (pmask) pmask[((size_t)row * K + k0) >> 3] = (uint8_t)bits;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  // PRO: dy = A g + B y + Cc in place of g (and, channel group 0, stored for the weight gradient)
  auto prologue = [&](int t, bf16x8 (&af)[MJ][KT], const bf16x8 (&yf)[YJ][YK]) {
    if constexpr (PRO && EPI == 1) {
      prologue_fwd(t, af);
    } else if constexpr (PRO_R) {
      prologue_fwd_res(t, af, yf);
    } else if constexpr (PRO) {
      // the coefficient reads are loop-invariant: hoisted out of the tile loop they would pin
      // 24 * KT registers for the whole kernel. The empty clobber keeps them per chunk.
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < MJ; ++j) {
        const int row = t * TPM + 16 * j + fr;
        const bool st = g == 0 && pro_dy != nullptr && row < p.M;
#pragma unroll
        for (int kb = 0; kb < KT; ++kb) {
          const int k0 = kb * 32 + 8 * fq;
          const uint4 gu = __builtin_bit_cast(uint4, af[j][kb]), yu = __builtin_bit_cast(uint4, yf[j][kb]);
          const uint32_t gw4[4] = {gu.x, gu.y, gu.z, gu.w}, yw4[4] = {yu.x, yu.y, yu.z, yu.w};
          uint32_t ow[4];
#pragma unroll
          for (int h = 0; h < 2; ++h) {   // 4 channels at a time: 12 coefficient registers live
            const float4 a4 = *reinterpret_cast<const float4*>(pco + k0 + 4 * h);
            const float4 b4 = *reinterpret_cast<const float4*>(pco + K + k0 + 4 * h);
            const float4 c4 = *reinterpret_cast<const float4*>(pco + 2 * K + k0 + 4 * h);
            const uint32_t g0 = gw4[2 * h], g1 = gw4[2 * h + 1], y0 = yw4[2 * h], y1 = yw4[2 * h + 1];
            const float o0 = a4.x * __uint_as_float(g0 << 16) + b4.x * __uint_as_float(y0 << 16) + c4.x;
            const float o1 = a4.y * __uint_as_float(g0 & 0xffff0000u) + b4.y * __uint_as_float(y0 & 0xffff0000u) + c4.y;
            const float o2 = a4.z * __uint_as_float(g1 << 16) + b4.z * __uint_as_float(y1 << 16) + c4.z;
            const float o3 = a4.w * __uint_as_float(g1 & 0xffff0000u) + b4.w * __uint_as_float(y1 & 0xffff0000u) + c4.w;
            ow[2 * h] = pack2bf(o0, o1);
            ow[2 * h + 1] = pack2bf(o2, o3);
          }
          const uint4 pk = make_uint4(ow[0], ow[1], ow[2], ow[3]);
          af[j][kb] = __builtin_bit_cast(bf16x8, pk);
          if (st) *reinterpret_cast<uint4*>(pro_dy + (size_t)row * K + k0) = pk;
          __builtin_amdgcn_sched_barrier(0);   // one chunk's coefficients live at a time
        }
      }
    }
  };
  auto wsync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  auto process = [&](int t, bf16x8 (&cur)[MJ][KT], bf16x8 (&nxt)[MJ][KT], bf16x8 (&ycur)[YJ][YK],
                     bf16x8 (&ynxt)[YJ][YK]) {
    // (1) epilogue operands of THIS tile first (in-order vmcnt: they must not queue behind the prefetch)
    uint4 ey[MJ][HP], er[MJ][HP], ey2[Y2 ? MJ : 1][Y2 ? HP : 1];
    unsigned em[MJ][HP];
    if constexpr (EPI == 2) {
#pragma unroll
      for (int j = 0; j < MJ; ++j)
#pragma unroll
        for (int h = 0; h < HP; ++h) {
          int m = t * TPM + 16 * j + lr + RPP * h;
          m = m < p.M ? m : p.M - 1;
          const size_t off = (size_t)m * N + c0;
          ey[j][h] = bnsum ? *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y) + off)
                           : make_uint4(0u, 0u, 0u, 0u);
          if constexpr (Y2)
            ey2[j][h] = y2on ? *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16_t*>(bs.y2) + off)
                             : make_uint4(0u, 0u, 0u, 0u);
          if (resid && bs.resid_half) {
            // half-resolution residual: even (h, w) only; the address stays in bounds for odd
            // positions (H, W even) and the value is dropped there, so the load is unconditional
            const int hw = p.gH * p.gW;
            const int n = m / hw, r = m - n * hw;
            const int yy = r / p.gW, xx = r - yy * p.gW;
            const size_t roff = ((size_t)(n * (p.gH >> 1) + (yy >> 1)) * (p.gW >> 1) + (xx >> 1)) * N + c0;
            const uint4 rv = *reinterpret_cast<const uint4*>(resid + roff);
            er[j][h] = ((yy | xx) & 1) ? make_uint4(0u, 0u, 0u, 0u) : rv;
          } else {
            er[j][h] = resid ? *reinterpret_cast<const uint4*>(resid + off) : make_uint4(0u, 0u, 0u, 0u);
          }
          em[j][h] = bs.zmode == 2 ? (unsigned)reinterpret_cast<const uint8_t*>(bs.z)[off >> 3] : 0u;
        }
    }
    // (2) prefetch the next tile of this wave
    // PRO: this tile's dy first (its g / y registers die before the next tile's are in flight)
    prologue(t, cur, ycur);
    if constexpr (PRO) __builtin_amdgcn_sched_barrier(0);
    const int tn = t + GW;
    if (tn < ntiles) load_tile(tn, nxt, ynxt);

    // (3) MFMAs: D[channel][pixel] = W . A^T; weight fragments double-buffered one k-block ahead,
    //     the scheduling fence per k-block keeps hipcc from hoisting every ds_read of the tile
    f32x4 acc[MJ][NI];
#pragma unroll
    for (int j = 0; j < MJ; ++j)
#pragma unroll
      for (int i = 0; i < NI; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 wf[2][NI];
    auto wload = [&](int kb, bf16x8 (&dst)[NI]) {
#pragma unroll
      for (int i = 0; i < NI; ++i) dst[i] = *reinterpret_cast<const bf16x8*>(wfr + ((i * KT + kb) * 64 + lane) * 16);
    };
    wload(0, wf[0]);
#pragma unroll
    for (int kb = 0; kb < KT; ++kb) {
      if (kb + 1 < KT) wload(kb + 1, wf[(kb + 1) & 1]);
#pragma unroll
      for (int j = 0; j < MJ; ++j)
#pragma unroll
        for (int i = 0; i < NI; ++i) acc[j][i] = mfma16(wf[kb & 1][i], cur[j][kb], acc[j][i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // (4) epilogue, one 16-pixel slice at a time through the wave's patch
#pragma unroll
    for (int j = 0; j < MJ; ++j) {
#pragma unroll
      for (int i = 0; i < NI; ++i) *reinterpret_cast<f32x4*>(patch + fr * PITCH + 16 * i + 4 * fq) = acc[j][i];
      wsync();
#pragma unroll
      for (int h = 0; h < HP; ++h) {
        const int row = lr + RPP * h;
        const int m = t * TPM + 16 * j + row;
        const bool ok = m < p.M;
        const float4 lo = *reinterpret_cast<const float4*>(patch + row * PITCH + ch * 8);
        const float4 hi = *reinterpret_cast<const float4*>(patch + row * PITCH + ch * 8 + 4);
        float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        float yy[8];
        if constexpr (EPI == 2) {
          if (resid) {
            float rv[8];
            unpack8(er[j][h], rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += rv[e];
          }
          unpack8(ey[j][h], yy);
          if (bs.zmode == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = yy[e] * csc[e] + csh[e] > 0.f ? v[e] : 0.f;
          } else if (bs.zmode == 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = (em[j][h] >> e) & 1u ? v[e] : 0.f;
          }
        }
        const uint4 pk = pack8(v);
        if (ok) *reinterpret_cast<uint4*>(Y + (size_t)m * N + c0) = pk;
        if (want && ok) {
          float q[8];
          unpack8(pk, q);
          if constexpr (EPI != 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              s1[e] += q[e];
              s2[e] += q[e] * q[e];
            }
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              s1[e] += q[e];
              s2[e] += q[e] * (yy[e] - cmu[e]) * civ[e];
            }
            if constexpr (Y2) {
              if (y2on) {
                float y2v[8];
                unpack8(ey2[j][h], y2v);
#pragma unroll
                for (int e = 0; e < 8; ++e) s3[e] += q[e] * y2v[e];
              }
            }
          }
        }
      }
      wsync();
    }
  };

  // the operand fragments are double-buffered (the next tile's load is in flight during this
  // tile's MFMAs); the prologue's y fragments are not: process() consumes them in the prologue
  // BEFORE it issues the next tile's loads into the same registers (KT * 4 VGPRs saved, which
  // is what lets the prologue run at K = 256)
  bf16x8 fa[MJ][KT], fb[MJ][KT];
  bf16x8 ya[YJ][YK];
  int t = gw;
  if (t < ntiles) load_tile(t, fa, ya);
  for (; t < ntiles; t += 2 * GW) {
    process(t, fa, fb, ya, ya);
    if (t + GW < ntiles) process(t + GW, fb, fa, ya, ya);
  }

  if (!want) return;
  // lanes sharing a channel chunk differ in the bits >= log2(CPR)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1) {
      s1[e] += __shfl_xor(s1[e], o, 64);
      s2[e] += __shfl_xor(s2[e], o, 64);
    }
    if (y2on) {
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1) s3[e] += __shfl_xor(s3[e], o, 64);
    }
    if (lane < CPR) {
      atomicAdd(ssum + ch * 8 + e, s1[e]);
      atomicAdd(ssum + NP + ch * 8 + e, s2[e]);
      if (y2on) atomicAdd(ssum3 + ch * 8 + e, s3[e]);
    }
  }
  __syncthreads();
  float* dst = EPI != 2 ? stats : bs.sums;
  if (p.stat_mode > 0) dst = slot_ptr(dst, 2 * N, p.stat_mode);
  for (int c = tid; c < NP; c += NT) {
    atomicAdd(dst + n0 + c, ssum[c]);
    atomicAdd(dst + N + n0 + c, ssum[NP + c]);
    if (y2on) atomicAdd(bs.sums2 + n0 + c, ssum3[c]);
  }
}

static int g_pw_mode = 1;  // 0 off, 1 on (zoo_pw_set: tests and A/B tools)

static int pw_mode() { return g_pw_mode; }

static int pw_ncu() {
  static int ncu = 0;
  if (ncu == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const int free_cus = ncu - g_reserved_cus;
  return free_cus >= 8 ? free_cus : 8;
}

// group weights + [2][NP] sums + one fp32 16 x (NP + 4) patch per wave (+ PRO: [3][K] coefficients,
// [6][K] with a residual's affine in EPI 4)
static size_t pw_smem(int NP, int K, bool pro, bool res = false) {
  return (size_t)NP * K * 2 + 2 * NP * 4 + (size_t)PW_NW * 16 * (NP + 4) * 4 +
         (pro ? (size_t)(res ? 6 : 3) * K * 4 : 0) + (size_t)NP * 4;   // + [NP] second-BN sums (y2)
}

template <int NP, int TPM, int KT, int EPI, bool PRO>
static hipError_t pw_launch(const ConvGeom& g, const bf16_t* X, const bf16_t* W, bf16_t* Y, const bf16_t* resid,
                            float* stats, const BwdStats& bs, hipStream_t st) {
  auto kfn = &pw_kernel<NP, TPM, KT, EPI, PRO>;
  const size_t smem = pw_smem(NP, KT * 32, PRO, EPI == 4);
  static int per_cu = 0;
  if (per_cu == 0) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, reinterpret_cast<const void*>(kfn), PW_NW * 64, smem) !=
            hipSuccess || nb < 1)
      nb = 1;
    per_cu = nb;
  }
  const int nsplit = g.K / NP;
  // pixel groups: one occupancy-full wave of workgroups, a multiple of 8 (XCD-local channel
  // groups), capped by the work (8 wave streams per group)
  int mgroups = pw_ncu() * per_cu / nsplit;
  mgroups = mgroups / 8 * 8;
  if (mgroups < 8) mgroups = 8;
  const int need = ((g.M + TPM - 1) / TPM + PW_NW - 1) / PW_NW;
  const int need8 = (need + 7) / 8 * 8;
  if (mgroups > need8) mgroups = need8;
  PwArgs a{g.M, g.K, g.ldb, nsplit, g.stat_slots, g.H, g.W, g.P, g.Q};
  hipLaunchKernelGGL(kfn, dim3(mgroups * nsplit), dim3(PW_NW * 64), smem, st, X, W, Y, resid, stats, a, bs);
  return hipGetLastError();
}

// (NP, K) -> TPM: 32 while the double-buffered activation fragments plus the accumulators stay
// within ~96 VGPRs, else 16 (no scratch spills at 2 waves / SIMD)
template <int EPI, bool PRO>
static hipError_t pw_dispatch(const ConvGeom& g, int NP, const bf16_t* X, const bf16_t* W, bf16_t* Y,
                              const bf16_t* resid, float* stats, const BwdStats& bs, hipStream_t st) {
  const int K = g.Ktot;
  // operand + y fragments of a double-buffered tile in registers: spill-free at K = 64, and at
  // K = 128 with 64-channel groups and 16-pixel tiles (198 VGPRs); K = 256 spills 108-308 bytes
  // per lane and ran 1.1-3.3x slower than apply + plain dgrad (profiles/r5/ab_bn_prologue_r5.md)
  if (PRO && K > 256) return hipErrorNotSupported;
  if constexpr (PRO) {
    if (K == 128) return NP == 64 ? pw_launch<64, 16, 4, EPI, PRO>(g, X, W, Y, resid, stats, bs, st)
                                  : pw_launch<128, 16, 4, EPI, PRO>(g, X, W, Y, resid, stats, bs, st);
    if (K == 256) return NP == 64 ? pw_launch<64, 16, 8, EPI, PRO>(g, X, W, Y, resid, stats, bs, st)
                                  : hipErrorNotSupported;
  }
#define PW_CASE(np, k, TPM)                                                                    \
  if constexpr (!PRO || (k) <= 64) {                                                           \
    if (NP == np && K == k) return pw_launch<np, TPM, k / 32, EPI, PRO>(g, X, W, Y, resid, stats, bs, st); \
  }
  PW_CASE(64, 64, 32)
  PW_CASE(64, 128, 32)
  PW_CASE(64, 256, 16)
  PW_CASE(64, 512, 16)
  PW_CASE(128, 64, EPI == 2 ? 16 : 32)
  PW_CASE(128, 128, 16)
  PW_CASE(128, 256, 16)
#undef PW_CASE
  return hipErrorNotSupported;
}

// channels per workgroup: 128 while its weights stay <= 64 KiB, else 64; 0 = not handled
static int pw_np(int N, int K) {
  if (K != 64 && K != 128 && K != 256 && K != 512) return 0;
  if (N % 128 == 0 && K <= 256) return 128;
  if (N % 64 == 0) return 64;
  return 0;
}

}  // namespace zoo

using namespace zoo;

extern "C" void zoo_pw_set(int mode) { g_pw_mode = mode; }

int zoo::g_reserved_cus = 0;
extern "C" void zoo_set_reserved_cus(int n) { zoo::g_reserved_cus = n > 0 ? n : 0; }

// 1x1 / stride 1 / unpadded, whole rows (A row stride == Ktot), no output remap, forward with
// BN statistics (EPI 1) or the backward epilogue (EPI 2, not the GELU form)
extern "C" int zoo_pw_eligible(const ConvGeom* g, int route, const BwdStats* bs) {
  if (pw_mode() <= 0) return 0;
  if (route != 1 && route != 2) return 0;
  // the backward epilogue handles the bit-mask (2) and recomputed (1) ReLU masks, or none
  if (route == 2 && bs && bs->zmode == 0 && bs->z) return 0;
  // deterministic / partial-buffer statistics: per-m-tile rows are the tiled kernels' contract
  if (g->stat_slots == kStatPartial) return 0;
  const bool is1x1 = g->R == 1 && g->S == 1 && g->sh == 1 && g->sw == 1 && g->ph == 0 && g->pw == 0 && g->lh == 1 &&
                     g->lw == 1 && g->H == g->P && g->W == g->Q && g->omap == 0;
  // forward with a 512-deep reduction: the tiled kernels are as fast or faster there
  // (tools/pw_bench.py --ab: 57 / 104 / 57 us vs 54 / 91 / 39 us on the three ResNet-50 shapes)
  static const int fwd_kmax = 256;
  if (route == 1 && g->Ktot > fwd_kmax) return 0;
  // the BN-backward prologue keeps operand and y fragments of a K <= 128 tile in registers
  if (bs && bs->pro_y && ((route != 2 && route != 1) || g->Ktot > 256)) return 0;
  // the forward consumer-side apply: plain forward epilogue, K <= 128 (register budget as above);
  // with a residual operand (EPI 4) up to K = 256 in 64-channel groups
  if (bs && bs->pro_fwd && (route != 1 || g->Ktot > (bs->pro_res ? 256 : 128) || bs->pro_y)) return 0;
  if (bs && bs->pro_res && (g->K % 64 != 0 || g->Ktot % 64 != 0)) return 0;
  // second-BN sums (BwdStats.y2): the short-reduction backward kernels only (pw_kernel Y2)
  if (bs && bs->y2 && (route != 2 || !bs->sums || g->Ktot > (bs->pro_y ? 64 : 128))) return 0;
  // a half-resolution residual (BwdStats::resid_half) needs the backward epilogue and even H, W
  if (bs && bs->resid_half && (route != 2 || (g->H & 1) || (g->W & 1))) return 0;
  return is1x1 && g->Ktot == g->C && g->M > 0 && pw_np(g->K, g->Ktot) > 0;
}

// the ResNet stem in space-to-depth form (4x4 stride-1 unpadded conv, 16 -> 64 channels) with BN
// statistics (EPI 3)
extern "C" int zoo_pw_stem_eligible(const ConvGeom* g, int route) {
  if (pw_mode() <= 0 || route != 1) return 0;
  if (g->stat_slots == kStatPartial) return 0;
  return g->R == 4 && g->S == 4 && g->C == 16 && g->K == 64 && g->sh == 1 && g->sw == 1 && g->ph == 0 &&
         g->pw == 0 && g->lh == 1 && g->lw == 1 && g->dh == 1 && g->dw == 1 && g->omap == 0 && g->Ktot == 256 &&
         g->ldb >= 256 && g->ldb % 8 == 0 && g->P == g->H - 3 && g->Q == g->W - 3 && g->M > 0;
}

extern "C" hipError_t zoo_pw_stem(const void* X, const void* W, void* Y, float* stats, const ConvGeom* g,
                                  hipStream_t st) {
  BwdStats bs{nullptr, nullptr, nullptr, nullptr, nullptr};
  return pw_launch<64, 16, 8, 3, false>(*g, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, nullptr, stats, bs, st);
}

extern "C" hipError_t zoo_pw(const void* X, const void* W, void* Y, const void* resid, float* stats,
                             const ConvGeom* g, int epi, const BwdStats* bsp, hipStream_t st) {
  BwdStats bs = bsp ? *bsp : BwdStats{nullptr, nullptr, nullptr, nullptr, nullptr};
  // the prologue at K = 128 runs 64-channel groups (register budget, see pw_dispatch)
  // prologue: 64-channel groups at K = 128 and K = 256 (256 VGPRs)
  const bool pro = bs.pro_y || bs.pro_fwd;
  const int NP = (pro && (g->Ktot == 128 || g->Ktot == 256) && g->K % 64 == 0) ? 64
                                                                                              : pw_np(g->K, g->Ktot);
  if (epi == 1 && bs.pro_fwd && bs.pro_res)
    return pw_dispatch<4, true>(*g, 64, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, nullptr, stats, bs, st);
  if (epi == 1 && bs.pro_fwd)
    return pw_dispatch<1, true>(*g, NP, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, nullptr, stats, bs, st);
  // the BN-backward prologue runs in the backward-epilogue kernel also for a plain dgrad (no
  // producer sums, no residual: a projection shortcut's dgrad, whose dx is handed to conv1)
  if (bs.pro_y)
    return pw_dispatch<2, true>(*g, NP, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, (const bf16_t*)resid, nullptr,
                                bs, st);
  if (epi == 1)
    return pw_dispatch<1, false>(*g, NP, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, nullptr, stats, bs, st);
  return pw_dispatch<2, false>(*g, NP, (const bf16_t*)X, (const bf16_t*)W, (bf16_t*)Y, (const bf16_t*)resid, nullptr,
                               bs, st);
}
