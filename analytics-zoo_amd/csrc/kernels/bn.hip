// BatchNorm for NHWC bf16 activations on gfx950 (training + inference), with
// the residual add and ReLU of ResNet bottlenecks fused into the same pass.
//
// Reference: BigDL BatchNormalization / SpatialBatchNormalization as wrapped by
// Zs/pipeline/api/keras/layers/BatchNormalization.scala:85-110.
//
// Forward (training):
//   stats  = (sum x, sum x^2) per channel — normally produced for free by the
//            producing conv's epilogue (igemm.hip); `bn_reduce` exists for the
//            unfused case;
//   apply  = y = relu?( x*scale + shift (+ residual) ), where every workgroup
//            derives scale/shift from the raw sums itself (no finalize launch),
//            and workgroup 0 updates the running statistics and saves
//            mean/invstd for the backward pass.
// Backward:
//   reduce = (sum dy, sum dy*xhat) with dy = dz * [z > 0] (ReLU mask recomputed
//            from the saved output z), one pass over [M][C];
//   apply  = dx = scale*(dy - mean(dy) - xhat*mean(dy*xhat)); optionally also
//            emits dy for the residual branch; workgroup 0 writes dgamma/dbeta.
// All passes move 8 bf16 per lane (16-byte vector loads, Guideline 13).
#include <stdlib.h>

#include "common.h"
#include "geom.h"

namespace zoo {

ZOO_DEV void load8f(const float* __restrict__ p, int chunk, float* v) {
  const float4 a = reinterpret_cast<const float4*>(p)[2 * chunk];
  const float4 b = reinterpret_cast<const float4*>(p)[2 * chunk + 1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// ---------------------------------------------------------------------------
// channel reduction over [M][C]; mode 0: (x, x^2); mode 1: (dy, dy*xhat)
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const bf16_t* __restrict__ A,    // x or dz
                                                        const bf16_t* __restrict__ Z,    // relu output (mode 1, may be null)
                                                        const bf16_t* __restrict__ Xin,  // conv output x (mode 1)
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        float* __restrict__ out,  // [2][C] (+ slots)
                                                        int M, int C, int rows_per_block, int nslot) {
  const int cpr = C >> 3;  // 8-channel chunks per row
  const int tid = threadIdx.x;
  // threads are laid out [row_lane][chunk]; if C/8 > 256 a thread walks several chunks
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const int lanes_per_row = cpr < 256 ? cpr : 256;
  const int row_step = 256 / lanes_per_row;
  const int my_row = tid / lanes_per_row;
  const int my_chunk0 = tid - my_row * lanes_per_row;
  // per-row-lane partials [row_step][2][C]: every (row lane, channel) slot has exactly one
  // writer, and the fold below adds the row lanes in a fixed order (no LDS float atomics,
  // so the block's sums are bit-reproducible)
  float* red = reinterpret_cast<float*>(smem);
  if (my_row < row_step) {
    for (int chunk = my_chunk0; chunk < cpr; chunk += lanes_per_row) {
      float s1[8], s2[8];
      float mu[8], is[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
      if (MODE == 1) {
        load8f(mean, chunk, mu);
        load8f(invstd, chunk, is);
      }
      // 4 rows per step, every load of the step issued before the first use: with one row per
      // step a thread had 2 loads in flight and the pass ran at ~3.5 TB/s (234 us for the 256-wide
      // stage-1 shortcut reduction, profiles/r6/ab4_prof_rn_step_r6.md row 345)
      constexpr int U = 4;
      const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);
      for (int rb = r0 + my_row; rb < r1; rb += U * row_step) {
        uint4 av[U], xv[U], zv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = rb + u * row_step;
          const bool ok = r < r1;
          const size_t off = (size_t)(ok ? r : rb) * C + chunk * 8;
          av[u] = ok ? *reinterpret_cast<const uint4*>(A + off) : zero4;
          if (MODE == 1) {
            xv[u] = ok ? *reinterpret_cast<const uint4*>(Xin + off) : zero4;
            zv[u] = (ok && Z) ? *reinterpret_cast<const uint4*>(Z + off) : zero4;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float a[8];
          unpack8(av[u], a);   // rows past r1 are zero: they add nothing
          if (MODE == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) { s1[e] += a[e]; s2[e] += a[e] * a[e]; }
          } else {
            float x[8];
            unpack8(xv[u], x);
            if (Z) {
              float z[8];
              unpack8(zv[u], z);
#pragma unroll
              for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              s1[e] += a[e];
              s2[e] += a[e] * (x[e] - mu[e]) * is[e];
            }
          }
        }
      }
      float* rr = red + (size_t)my_row * 2 * C;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        rr[chunk * 8 + e] = s1[e];
        rr[C + chunk * 8 + e] = s2[e];
      }
    }
  }
  __syncthreads();
  if (nslot == kStatPartial) {  // out = [gridDim.x][2C] partials, folded by stats_part_finalize
    float* const dst = out + (size_t)blockIdx.x * 2 * C;
    for (int i = tid; i < 2 * C; i += blockDim.x) {
      float a = 0.f;
      for (int r = 0; r < row_step; ++r) a += red[(size_t)r * 2 * C + i];
      dst[i] = a;
    }
    return;
  }
  float* const dst = nslot > 0 ? slot_ptr(out, 2 * C, nslot) : out;
  for (int i = tid; i < 2 * C; i += blockDim.x) {
    float a = 0.f;
    for (int r = 0; r < row_step; ++r) a += red[(size_t)r * 2 * C + i];
    atomicAdd(dst + i, a);
  }
}

// ---------------------------------------------------------------------------
// Apply passes: a thread owns one 8-channel chunk for a contiguous range of rows
// and keeps that chunk's per-channel coefficients in registers (no LDS: the
// previous LDS coefficient tables were read with 8-way bank conflicts).
// Blocks own contiguous row ranges; lanes of a wave cover consecutive chunks of
// consecutive rows, so every wave instruction moves whole contiguous rows.
// ---------------------------------------------------------------------------
struct RowSplit {
  int lpr, rstep, chunk0, rsub;
};

ZOO_DEV RowSplit row_split(int cpr) {
  RowSplit r;
  r.lpr = cpr < 256 ? cpr : 256;
  r.rstep = 256 / r.lpr;
  r.chunk0 = threadIdx.x % r.lpr;
  r.rsub = threadIdx.x / r.lpr;
  return r;
}

// training statistics of the BatchNorm applied to the residual input (downsample
// shortcut): the residual operand is then the raw shortcut conv output and is normalised
// with these in the same pass, so the shortcut's own apply pass and its output tensor go away
struct BnSide {
  const float* stats;  // null: the residual is added as is
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float* save_mean;
  float* save_invstd;
};

ZOO_DEV void bn_bookkeeping(const float* stats, float* running_mean, float* running_var, float* save_mean,
                            float* save_invstd, int M, int C, float eps, float momentum) {
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float mu = stats[c] * invM;
    const float var = fmaxf(stats[C + c] * invM - mu * mu, 0.f);
    save_mean[c] = mu;
    save_invstd[c] = rsqrtf(var + eps);
    if (running_mean) {
      const float unbiased = M > 1 ? var * (float)M / (float)(M - 1) : var;
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mu;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
    }
  }
}

ZOO_DEV void bn_coeffs(const float* stats, const float* gamma, const float* beta, int chunk, int C, float invM,
                       float eps, float* sc, float* sh) {
  float s1[8], s2[8], g8[8], b8[8];
  load8f(stats, chunk, s1);
  load8f(stats + C, chunk, s2);
  if (gamma) load8f(gamma, chunk, g8);
  if (beta) load8f(beta, chunk, b8);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float mu = s1[e] * invM;
    const float is = rsqrtf(fmaxf(s2[e] * invM - mu * mu, 0.f) + eps);
    sc[e] = gamma ? g8[e] * is : is;
    sh[e] = (beta ? b8[e] : 0.f) - mu * sc[e];
  }
}

// Consumer-side forward apply (conv_fwd pro_fwd): the saved statistics, running averages and the
// per-channel affine coef = [scale | 0 | shift] ([3][C]) of a conv -> BN -> ReLU unit whose
// apply pass is done by its 1x1 consumer's operand prologue (pw.hip) instead
__global__ __launch_bounds__(256) void bn_fwd_coef_kernel(const float* __restrict__ stats,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float* running_mean,
                                                          float* running_var, float* save_mean, float* save_invstd,
                                                          float* __restrict__ coef, int M, int C, float eps,
                                                          float momentum) {
  bn_bookkeeping(stats, running_mean, running_var, save_mean, save_invstd, M, C, eps, momentum);
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float mu = stats[c] * invM;
    const float is = rsqrtf(fmaxf(stats[C + c] * invM - mu * mu, 0.f) + eps);
    const float sc = gamma ? gamma[c] * is : is;
    coef[c] = sc;
    coef[C + c] = 0.f;
    coef[2 * C + c] = (beta ? beta[c] : 0.f) - mu * sc;
  }
}

// forward apply (training): stats -> scale/shift per thread
__global__ __launch_bounds__(256) void bn_fwd_apply_kernel(
    const bf16_t* __restrict__ X, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, const bf16_t* __restrict__ resid, bf16_t* __restrict__ Y,
    float* __restrict__ running_mean, float* __restrict__ running_var, float* __restrict__ save_mean,
    float* __restrict__ save_invstd, int M, int C, float eps, float momentum, int relu, int training,
    int rows_per_block, BnSide r2, uint8_t* __restrict__ mask) {
  const float invM = 1.f / (float)M;
  if (blockIdx.x == 0 && training) {  // bookkeeping: saved statistics + running averages
    bn_bookkeeping(stats, running_mean, running_var, save_mean, save_invstd, M, C, eps, momentum);
    if (r2.stats)
      bn_bookkeeping(r2.stats, r2.running_mean, r2.running_var, r2.save_mean, r2.save_invstd, M, C, eps, momentum);
  }
  const int cpr = C >> 3;
  const RowSplit rs = row_split(cpr);
  if (rs.rsub >= rs.rstep) return;
  // rows_per_block > 0: the block streams one contiguous row range; == 0: tiles of
  // 4*rstep rows are dealt round-robin over the grid (concurrent blocks touch
  // neighbouring memory)
  const int tile = 4 * rs.rstep;
  const bool inter = rows_per_block == 0;
  const int r0 = (inter ? blockIdx.x * tile : blockIdx.x * rows_per_block) + rs.rsub;
  const int r1 = inter ? M : min(M, blockIdx.x * rows_per_block + rows_per_block);
  const int rstride = inter ? gridDim.x * tile : tile;
  for (int chunk = rs.chunk0; chunk < cpr; chunk += rs.lpr) {
    float sc[8], sh[8];
    {
      // per-channel coefficients with 16-byte loads (all vectors are 8-channel aligned)
      float s1[8], s2[8], g8[8], b8[8];
      load8f(training ? stats : running_mean, chunk, s1);
      load8f(training ? stats + C : running_var, chunk, s2);
      if (gamma) load8f(gamma, chunk, g8);
      if (beta) load8f(beta, chunk, b8);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float mu, is;
        if (training) {
          mu = s1[e] * invM;
          is = rsqrtf(fmaxf(s2[e] * invM - mu * mu, 0.f) + eps);
        } else {
          mu = s1[e];
          is = rsqrtf(s2[e] + eps);
        }
        sc[e] = gamma ? g8[e] * is : is;
        sh[e] = (beta ? b8[e] : 0.f) - mu * sc[e];
      }
    }
    float sc2[8], sh2[8];
    if (r2.stats) {
      bn_coeffs(r2.stats, r2.gamma, r2.beta, chunk, C, invM, eps, sc2, sh2);
#pragma unroll
      for (int e = 0; e < 8; ++e) sh[e] += sh2[e];  // both shifts folded into one
    }
    // 4 rows per step: four independent 16-byte loads (x 2 with a residual) in flight per thread
    for (int rb = r0; rb < r1; rb += rstride) {
      uint4 xv[4], rv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + u * rs.rstep;
        const size_t off = (size_t)(r < r1 ? r : rb) * C + chunk * 8;
        xv[u] = *reinterpret_cast<const uint4*>(X + off);
        if (resid) rv[u] = *reinterpret_cast<const uint4*>(resid + off);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + u * rs.rstep;
        if (r >= r1) break;
        float v[8];
        unpack8(xv[u], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] * sc[e] + sh[e];
        if (resid) {
          float q[8];
          unpack8(rv[u], q);
          if (r2.stats) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += q[e] * sc2[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += q[e];
          }
        }
        if (mask) {  // ReLU bit mask for the consumer's fused BN-backward (BwdStats.zmode 2)
          unsigned b = 0;
#pragma unroll
          for (int e = 0; e < 8; ++e) b |= (v[e] > 0.f ? 1u : 0u) << e;
          mask[((size_t)r * C >> 3) + chunk] = (uint8_t)b;
        }
        if (relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        }
        *reinterpret_cast<uint4*>(Y + (size_t)r * C + chunk * 8) = pack8(v);
      }
    }
  }
}

// backward apply: dx = A_c*dy + B_c*x + D_c with
//   A = gamma*is, B = -A*is*mean(dy*xhat), D = A*(mu*is*mean(dy*xhat) - mean(dy))
// U rows per thread per step (2 or 4): U x (dz, x[, z]) 16-byte loads in flight per thread
template <int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dZ, const bf16_t* __restrict__ Z, const bf16_t* __restrict__ X,
    const float* __restrict__ save_mean, const float* __restrict__ save_invstd,
    const float* __restrict__ gamma, const float* __restrict__ sums,  // [2][C]: sum dy, sum dy*xhat
    bf16_t* __restrict__ dX, bf16_t* __restrict__ dResid, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int M, int C, int rows_per_block) {
  const float invM = 1.f / (float)M;
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      if (dgamma) dgamma[c] += sums[C + c];
      if (dbeta) dbeta[c] += sums[c];
    }
  }
  const int cpr = C >> 3;
  const RowSplit rs = row_split(cpr);
  if (rs.rsub >= rs.rstep) return;
  const int tile = U * rs.rstep;
  const bool inter = rows_per_block == 0;
  const int r0 = (inter ? blockIdx.x * tile : blockIdx.x * rows_per_block) + rs.rsub;
  const int r1 = inter ? M : min(M, blockIdx.x * rows_per_block + rows_per_block);
  const int rstride = inter ? gridDim.x * tile : tile;
  for (int chunk = rs.chunk0; chunk < cpr; chunk += rs.lpr) {
    float ka[8], kb[8], kd[8];
    float is8[8], mu8[8], g8[8], q1[8], q2[8];
    load8f(save_invstd, chunk, is8);
    load8f(save_mean, chunk, mu8);
    load8f(sums, chunk, q1);
    load8f(sums + C, chunk, q2);
    if (gamma) load8f(gamma, chunk, g8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float is = is8[e], mu = mu8[e];
      const float a = (gamma ? g8[e] : 1.f) * is;
      const float m1 = q1[e] * invM, m2 = q2[e] * invM;
      ka[e] = a;
      kb[e] = -a * is * m2;
      kd[e] = a * (mu * is * m2 - m1);
    }
    for (int rb = r0; rb < r1; rb += rstride) {
      uint4 dv[U], xv[U], zv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rb + u * rs.rstep;
        const size_t off = (size_t)(r < r1 ? r : rb) * C + chunk * 8;
        dv[u] = *reinterpret_cast<const uint4*>(dZ + off);
        xv[u] = *reinterpret_cast<const uint4*>(X + off);
        if (Z) zv[u] = *reinterpret_cast<const uint4*>(Z + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = rb + u * rs.rstep;
        if (r >= r1) break;
        const size_t off = (size_t)r * C + chunk * 8;
        float dy[8], x[8];
        unpack8(dv[u], dy);
        unpack8(xv[u], x);
        if (Z) {
          float z[8];
          unpack8(zv[u], z);
#pragma unroll
          for (int e = 0; e < 8; ++e) dy[e] = z[e] > 0.f ? dy[e] : 0.f;
        }
        if (dResid) *reinterpret_cast<uint4*>(dResid + off) = pack8(dy);
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = ka[e] * dy[e] + kb[e] * x[e] + kd[e];
        *reinterpret_cast<uint4*>(dX + off) = pack8(o);
      }
    }
  }
}

// fold the statistic slots: buf[i] = sum_k buf[n2*(1+k) + i]; a block owns 64
// columns, its 4 waves split the slots and meet in LDS
__global__ __launch_bounds__(256) void stats_finalize_kernel(float* __restrict__ buf, int n2, int nslot) {
  __shared__ float part[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  float s = 0.f;
  if (c < n2)
    for (int k = w; k < nslot; k += 4) s += buf[(size_t)n2 * (1 + k) + c];
  part[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < n2) buf[c] = (part[0][threadIdx.x] + part[1][threadIdx.x]) + (part[2][threadIdx.x] + part[3][threadIdx.x]);
}

// Backward of a conv epilogue's bias + ReLU: dy = dz * [z > 0] written out (bf16) and the
// bias gradient sum(dy) per channel accumulated, in ONE pass (replaces a compare, a multiply,
// a cast and a reduction launch). Z == null: no mask (bias only). Same row layout and
// per-row-lane LDS fold as bn_reduce_kernel; out = [C] fp32 (+= per block) or partials.
// Activation backward + column sums over a [M, C] row-major gradient (bias gradients of
// linear / 1x1-conv layers). Block = CT column threads (8 columns each, one coalesced
// CT*16-byte row segment) x RL = 256/CT row lanes; blockIdx = (row chunk, column group).
// Partial column sums are reduced through LDS, then one fp32 atomic (or, for the ordered
// deterministic fold, one partial row per row chunk) per column per block.
// ACT 0: dY = dZ (sums only); 1: dY = dZ * [Z > 0] (ReLU, Z = output);
// 2: dY = dZ * gelu'(Z) (erf GELU, Z = pre-activation). The sums are of the stored bf16 dY.
template <int ACT, int CT>
__global__ __launch_bounds__(256) void act_colsum_kernel(const bf16_t* __restrict__ dZ, const bf16_t* __restrict__ Z,
                                                         bf16_t* __restrict__ dY, float* __restrict__ out, int M,
                                                         int C, int rows_per_chunk, int col_groups, int partial) {
  constexpr int RL = 256 / CT;
  __shared__ float red[RL][CT * 8 + 4];
  const int cpr = C >> 3;
  const int chunk = blockIdx.x / col_groups, cg = blockIdx.x - chunk * col_groups;
  const int ct = threadIdx.x % CT, rl = threadIdx.x / CT;
  const int c = cg * CT + ct;
  const int r0 = chunk * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < cpr) {
#pragma unroll 4
    for (int r = r0 + rl; r < r1; r += RL) {
      const size_t off = (size_t)r * C + c * 8;
      float a[8];
      unpack8(*reinterpret_cast<const uint4*>(dZ + off), a);
      if (ACT != 0) {
        float z[8];
        unpack8(*reinterpret_cast<const uint4*>(Z + off), z);
        if (ACT == 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] *= gelu_grad_f(z[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) a[e] = z[e] > 0.f ? a[e] : 0.f;
        }
        const uint4 pk = pack8(a);
        *reinterpret_cast<uint4*>(dY + off) = pk;
        unpack8(pk, a);  // sum what is stored (bf16)
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += a[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rl][ct * 8 + e] = s[e];
  __syncthreads();
  if (!out) return;
  for (int i = threadIdx.x; i < CT * 8; i += 256) {
    const int col = cg * CT * 8 + i;
    if (col >= C) continue;
    float a = 0.f;
#pragma unroll
    for (int r = 0; r < RL; ++r) a += red[r][i];
    if (partial) out[(size_t)chunk * C + col] = a;
    else atomicAdd(out + col, a);
  }
}

// Deterministic fold of per-workgroup partials: out[c] += sum_p part[p][c], p in order.
// Level 1 (nparts > kPartGroup): block (column chunk, group g) sums the group's parts,
// 4 waves x 16 parts each then the waves in order, into lvl1[g][c]; level 2 sums the
// groups in order and adds into out.
constexpr int kPartGroup = 64;
__global__ __launch_bounds__(256) void stats_part_lvl1_kernel(const float* __restrict__ part,
                                                             float* __restrict__ lvl1, int n2, int nparts) {
  __shared__ float w4[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  const int p0 = blockIdx.y * kPartGroup + w * (kPartGroup / 4);
  const int p1 = min(nparts, p0 + kPartGroup / 4);
  float s = 0.f;
  if (c < n2)
    for (int p = p0; p < p1; ++p) s += part[(size_t)p * n2 + c];
  w4[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && c < n2)
    lvl1[(size_t)blockIdx.y * n2 + c] = ((w4[0][threadIdx.x] + w4[1][threadIdx.x]) + w4[2][threadIdx.x]) +
                                        w4[3][threadIdx.x];
}

__global__ __launch_bounds__(256) void stats_part_lvl2_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                             int n2, int nparts) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= n2) return;
  float s = 0.f;
  for (int p = 0; p < nparts; ++p) s += part[(size_t)p * n2 + c];
  out[c] += s;
}

// ---------------------------------------------------------------------------------------
// Stem fusion: BatchNorm -> ReLU -> max-pool in one pass over the RAW conv output (ResNet
// stem, reference SpatialBatchNormalization + ReLU + SpatialMaxPooling of
// Zs/models/image/imageclassification ResNet). relu(sc*x + sh) is monotone in x (increasing
// for sc >= 0, decreasing for sc < 0), so the pooled value is the affine image of the
// window max (or min) of the raw x: the [N,H,W,C] BN output is never written. Per pooled
// element the kernel keeps the raw winner (`best`, bf16 = exact) and its tap; a tap of
// kClipped marks a pooled value the ReLU clipped (no gradient flows back through it).
// Backward: (1) the BN reductions sum(dz), sum(dz*xhat) are taken in POOLED space (dz is
// non-zero only at winning taps: xhat there is (best - mu) * invstd), (2) one pass over the
// input gathers dz from the windows a pixel won and applies dx = A*dz + B*x + D. Together
// they replace bn_fwd_apply + maxpool_fwd and maxpool_bwd + bn_reduce + bn_bwd_apply.
// Row-per-block layout (power-of-two C/8 <= 256): each thread owns one fixed 8-channel
// chunk (threadIdx & (C/8-1)), so its per-channel coefficients load once.
constexpr uint8_t kClipped = 0xff;

// STEM: the ResNet geometry (3x3, stride 2, pad 1) as compile-time constants, so the
// window bounds and divisions fold (the runtime arguments are then ignored)
template <bool STEM>
__global__ __launch_bounds__(256) void bn_relu_maxpool_fwd_kernel(
    const bf16_t* __restrict__ X, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, bf16_t* __restrict__ Y, bf16_t* __restrict__ best_out,
    uint8_t* __restrict__ arg, float* __restrict__ running_mean, float* __restrict__ running_var,
    float* __restrict__ save_mean, float* __restrict__ save_invstd, int M, float eps, float momentum, int H, int W,
    int C, int P, int Q, int R_, int S_, int sh_r, int sw_r, int ph_r, int pw_r, int lg) {
  const int R = STEM ? 3 : R_, S = STEM ? 3 : S_, sh_ = STEM ? 2 : sh_r, sw_ = STEM ? 2 : sw_r;
  const int ph = STEM ? 1 : ph_r, pw = STEM ? 1 : pw_r;
  if (blockIdx.x == 0)
    bn_bookkeeping(stats, running_mean, running_var, save_mean, save_invstd, M, C, eps, momentum);
  const float invM = 1.f / (float)M;
  const int mask = (C >> 3) - 1;
  const int chunk = threadIdx.x & mask;
  float sc[8], sh[8], sg[8];
  bn_coeffs(stats, gamma, beta, chunk, C, invM, eps, sc, sh);
#pragma unroll
  for (int e = 0; e < 8; ++e) sg[e] = sc[e] >= 0.f ? 1.f : -1.f;
  const int row = blockIdx.x;  // n * P + p
  const int n = row / P, p = row - n * P;
  const int r_lo = max(0, ph - p * sh_), r_hi = min(R, H + ph - p * sh_);
  const bf16_t* xn = X + (size_t)n * H * W * C + (ptrdiff_t)(p * sh_ - ph) * W * C;
  const size_t ybase = (size_t)row * Q * C;
  for (int j = threadIdx.x; j < (Q << lg); j += 256) {
    const int q = j >> lg;
    const int s_lo = max(0, pw - q * sw_), s_hi = min(S, W + pw - q * sw_);
    float bt[8];  // best of sg * x
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { bt[e] = -INFINITY; bi[e] = 0; }
    const bf16_t* xq = xn + (ptrdiff_t)(q * sw_ - pw) * C + chunk * 8;
    if constexpr (STEM) {
      // 3x3 window fully unrolled: all nine 16-byte loads in flight at once (the runtime-bounded
      // loop below issued them one dependent iteration at a time); taps outside the image are
      // predicated off, never loaded
      uint4 raw[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const bool ok = r >= r_lo && r < r_hi && s >= s_lo && s < s_hi;
          raw[r * 3 + s] = ok ? *reinterpret_cast<const uint4*>(xq + (r * W + s) * C) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          if (!(r >= r_lo && r < r_hi && s >= s_lo && s < s_hi)) continue;
          float v[8];
          unpack8(raw[r * 3 + s], v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float t = sg[e] * v[e];
            if (t > bt[e]) { bt[e] = t; bi[e] = (uint8_t)(r * 3 + s); }
          }
        }
    } else {
      for (int r = r_lo; r < r_hi; ++r) {
        for (int s = s_lo; s < s_hi; ++s) {
          float v[8];
          unpack8(*reinterpret_cast<const uint4*>(xq + (r * W + s) * C), v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float t = sg[e] * v[e];
            if (t > bt[e]) { bt[e] = t; bi[e] = (uint8_t)(r * S + s); }
          }
        }
      }
    }
    float b[8], o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      b[e] = sg[e] * bt[e];
      const float z = b[e] * sc[e] + sh[e];
      o[e] = z > 0.f ? z : 0.f;
      if (!(z > 0.f)) bi[e] = kClipped;
    }
    const size_t off = ybase + (size_t)j * 8;
    *reinterpret_cast<uint4*>(Y + off) = pack8(o);
    *reinterpret_cast<uint4*>(best_out + off) = pack8(b);
    uint2 pk;
    pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(arg + off) = pk;
  }
}

// sums[c] += sum dz, sums[C + c] += sum dz * xhat over the pooled elements (grid-strided rows)
__global__ __launch_bounds__(256) void bn_relu_maxpool_bwd_reduce_kernel(
    const bf16_t* __restrict__ dY, const bf16_t* __restrict__ best, const uint8_t* __restrict__ arg,
    const float* __restrict__ save_mean, const float* __restrict__ save_invstd, float* __restrict__ sums, int rows,
    int Q, int C, int lg) {
  __shared__ float red[256][17];
  const int mask = (C >> 3) - 1;
  const int chunk = threadIdx.x & mask;
  float mu[8], is[8], s1[8], s2[8];
  load8f(save_mean, chunk, mu);
  load8f(save_invstd, chunk, is);
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  // two pooled pieces per step, their six loads issued before either is used (one piece per step
  // left three loads in flight per thread)
  const int nj = Q << lg;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const size_t base = (size_t)row * Q * C;
    for (int j0 = threadIdx.x; j0 < nj; j0 += 512) {
      uint2 ab[2];
      uint4 gv[2], bv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int j = j0 + 256 * u;
        const bool ok = j < nj;
        const size_t off = base + (size_t)(ok ? j : j0) * 8;
        ab[u] = ok ? *reinterpret_cast<const uint2*>(arg + off) : make_uint2(0xffffffffu, 0xffffffffu);
        gv[u] = *reinterpret_cast<const uint4*>(dY + off);
        bv[u] = *reinterpret_cast<const uint4*>(best + off);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        float g[8], b[8];
        unpack8(gv[u], g);
        unpack8(bv[u], b);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t t = ((e < 4 ? ab[u].x : ab[u].y) >> (8 * (e & 3))) & 0xff;
          const float d = t == kClipped ? 0.f : g[e];   // a piece past the row: all taps kClipped
          s1[e] += d;
          s2[e] += d * ((b[e] - mu[e]) * is[e]);
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[threadIdx.x][e] = s1[e]; red[threadIdx.x][8 + e] = s2[e]; }
  __syncthreads();
  const int lanes = 256 >> lg;  // threads sharing one chunk: tid = lane * (C/8) + chunk
  for (int i = threadIdx.x; i < 2 * C; i += 256) {
    const int which = i >= C, c = i - which * C, ch = c >> 3, e = c & 7;
    float a = 0.f;
    for (int l = 0; l < lanes; ++l) a += red[(l << lg) + ch][which * 8 + e];
    atomicAdd(sums + i, a);
  }
}

// dx = A*dz + B*x + D with dz gathered from the pooled windows this pixel won
template <bool STEM>
__global__ __launch_bounds__(256) void bn_relu_maxpool_bwd_apply_kernel(
    const bf16_t* __restrict__ dY, const uint8_t* __restrict__ arg, const bf16_t* __restrict__ X,
    const float* __restrict__ save_mean, const float* __restrict__ save_invstd, const float* __restrict__ gamma,
    const float* __restrict__ sums, bf16_t* __restrict__ dX, float* __restrict__ dgamma, float* __restrict__ dbeta,
    int M, int H, int W, int C, int P, int Q, int R_, int S_, int sh_r, int sw_r, int ph_r, int pw_r, int lg) {
  const int R = STEM ? 3 : R_, S = STEM ? 3 : S_, sh_ = STEM ? 2 : sh_r, sw_ = STEM ? 2 : sw_r;
  const int ph = STEM ? 1 : ph_r, pw = STEM ? 1 : pw_r;
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      if (dgamma) dgamma[c] += sums[C + c];
      if (dbeta) dbeta[c] += sums[c];
    }
  }
  const float invM = 1.f / (float)M;
  const int mask = (C >> 3) - 1;
  const int chunk = threadIdx.x & mask;
  float ka[8], kb[8], kd[8];
  {
    float is8[8], mu8[8], g8[8], q1[8], q2[8];
    load8f(save_invstd, chunk, is8);
    load8f(save_mean, chunk, mu8);
    load8f(sums, chunk, q1);
    load8f(sums + C, chunk, q2);
    if (gamma) load8f(gamma, chunk, g8);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float is = is8[e], mu = mu8[e];
      const float a = (gamma ? g8[e] : 1.f) * is;
      const float m1 = q1[e] * invM, m2 = q2[e] * invM;
      ka[e] = a;
      kb[e] = -a * is * m2;
      kd[e] = a * (mu * is * m2 - m1);
    }
  }
  const int row = blockIdx.x;  // n * H + h
  const int n = row / H, h = row - n * H;
  const int p_lo = max(0, (h + ph - R + sh_) / sh_);
  const int p_hi = min(P - 1, (h + ph) / sh_);
  const size_t nb = (size_t)n * P * Q * C + chunk * 8;
  const size_t xbase = (size_t)row * W * C;
  for (int j = threadIdx.x; j < (W << lg); j += 256) {
    const int w = j >> lg;
    const int q_lo = max(0, (w + pw - S + sw_) / sw_);
    const int q_hi = min(Q - 1, (w + pw) / sw_);
    float dz[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) dz[e] = 0.f;
    const size_t off = xbase + (size_t)j * 8;
    float x[8], o[8];
    if constexpr (STEM) {
      // stride 2, 3x3: a pixel lies in at most 2 x 2 windows (p_lo .. p_lo + 1, q_lo .. q_lo + 1);
      // all their dY / arg loads and the pixel's own x load are issued before any use
      uint4 gv[4];
      uint2 av[4];
      bool okv[4];
      uint32_t tapv[4];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int p = p_lo + a, q = q_lo + c, k = a * 2 + c;
          const int r = h - (p * 2 - 1), s = w - (q * 2 - 1);
          okv[k] = p <= p_hi && q <= q_hi && r >= 0 && r < 3 && s >= 0 && s < 3;
          tapv[k] = (uint32_t)(r * 3 + s);
          const size_t ofs = nb + (size_t)(p * Q + q) * C;
          av[k] = okv[k] ? *reinterpret_cast<const uint2*>(arg + ofs) : make_uint2(0xffffffffu, 0xffffffffu);
          gv[k] = okv[k] ? *reinterpret_cast<const uint4*>(dY + ofs) : make_uint4(0u, 0u, 0u, 0u);
        }
      unpack8(*reinterpret_cast<const uint4*>(X + off), x);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (!okv[k]) continue;
        float g[8];
        unpack8(gv[k], g);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (((av[k].x >> (8 * e)) & 0xff) == tapv[k]) dz[e] += g[e];
          if (((av[k].y >> (8 * e)) & 0xff) == tapv[k]) dz[4 + e] += g[4 + e];
        }
      }
    } else {
      for (int p = p_lo; p <= p_hi; ++p) {
        const int r = h - (p * sh_ - ph);
        if (r < 0 || r >= R) continue;
        for (int q = q_lo; q <= q_hi; ++q) {
          const int s = w - (q * sw_ - pw);
          if (s < 0 || s >= S) continue;
          const uint32_t tap = (uint32_t)(r * S + s);
          const size_t o2 = nb + (size_t)(p * Q + q) * C;
          const uint2 ab = *reinterpret_cast<const uint2*>(arg + o2);
          float g[8];
          unpack8(*reinterpret_cast<const uint4*>(dY + o2), g);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (((ab.x >> (8 * e)) & 0xff) == tap) dz[e] += g[e];
            if (((ab.y >> (8 * e)) & 0xff) == tap) dz[4 + e] += g[4 + e];
          }
        }
      }
      unpack8(*reinterpret_cast<const uint4*>(X + off), x);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = ka[e] * dz[e] + kb[e] * x[e] + kd[e];
    *reinterpret_cast<uint4*>(dX + off) = pack8(o);
  }
}

// contiguous row range per block: ~kApplyBlocks blocks, at least kMinRows rows per thread-row
static int apply_rows_per_block(int M, int C) {
  static const int target = 1024;
  static const int min_rows = 8;
  const int cpr = C / 8;
  const int rstep = 256 / (cpr < 256 ? cpr : 256);
  int rpb = (M + target - 1) / target;
  if (rpb < min_rows * rstep) rpb = min_rows * rstep;
  return rpb;
}


}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_bn_fwd_coef(const float* stats, const float* gamma, const float* beta, float* rmean,
                                      float* rvar, float* smean, float* sinv, float* coef, int M, int C, float eps,
                                      float momentum, hipStream_t st) {
  hipLaunchKernelGGL(bn_fwd_coef_kernel, dim3(1), dim3(256), 0, st, stats, gamma, beta, rmean, rvar, smean, sinv, coef,
                     M, C, eps, momentum);
  return hipGetLastError();
}

extern "C" hipError_t zoo_stats_finalize(float* buf, int n2, int nslot, hipStream_t st) {
  hipLaunchKernelGGL(stats_finalize_kernel, dim3((n2 + 63) / 64), dim3(256), 0, st, buf, n2, nslot);
  return hipGetLastError();
}

// scratch floats zoo_stats_part_finalize needs for `nparts` partial rows of n2 columns
extern "C" size_t zoo_stats_part_scratch(int n2, int nparts) {
  return nparts > kPartGroup ? (size_t)((nparts + kPartGroup - 1) / kPartGroup) * n2 : 0;
}

extern "C" hipError_t zoo_stats_part_finalize(float* out, const float* part, float* scratch, int n2, int nparts,
                                              hipStream_t st) {
  if (nparts > kPartGroup) {
    const int groups = (nparts + kPartGroup - 1) / kPartGroup;
    hipLaunchKernelGGL(stats_part_lvl1_kernel, dim3((n2 + 63) / 64, groups), dim3(256), 0, st, part, scratch, n2,
                       nparts);
    part = scratch;
    nparts = groups;
  }
  hipLaunchKernelGGL(stats_part_lvl2_kernel, dim3((n2 + 255) / 256), dim3(256), 0, st, part, out, n2, nparts);
  return hipGetLastError();
}

// grid of zoo_bn_reduce: ~1024 blocks owning contiguous row ranges, at least 16 rows per
// thread-row (small tensors such as bias gradients use few blocks)
static void bn_reduce_grid(int M, int C, int* blocks, int* rpb) {
  *blocks = 1024;
  *rpb = (M + *blocks - 1) / *blocks;
  const int cpr = C >> 3;
  const int row_step = 256 / (cpr < 256 ? cpr : 256);
  if (*rpb < 16 * row_step) *rpb = 16 * row_step;
  *blocks = (M + *rpb - 1) / *rpb;
}

extern "C" int zoo_bn_reduce_blocks(int M, int C) {
  int blocks, rpb;
  bn_reduce_grid(M, C, &blocks, &rpb);
  return blocks;
}

extern "C" hipError_t zoo_bn_reduce(const void* A, const void* Z, const void* X, const float* mean,
                                    const float* invstd, float* out, int M, int C, int mode, int nslot,
                                    hipStream_t st) {
  int blocks, rpb;
  bn_reduce_grid(M, C, &blocks, &rpb);
  const int cpr = C >> 3;
  const int row_step = 256 / (cpr < 256 ? cpr : 256);
  const size_t smem = (size_t)row_step * 2 * C * sizeof(float);
  if (mode == 0)
    hipLaunchKernelGGL(bn_reduce_kernel<0>, dim3(blocks), dim3(256), smem, st, (const bf16_t*)A,
                       (const bf16_t*)Z, (const bf16_t*)X, mean, invstd, out, M, C, rpb, nslot);
  else
    hipLaunchKernelGGL(bn_reduce_kernel<1>, dim3(blocks), dim3(256), smem, st, (const bf16_t*)A,
                       (const bf16_t*)Z, (const bf16_t*)X, mean, invstd, out, M, C, rpb, nslot);
  if (nslot > 0) return zoo_stats_finalize(out, 2 * C, nslot, st);
  return hipGetLastError();
}

// grid for the apply kernels: interleaved tiles (default) or contiguous ranges (ZOO_BN_INTERLEAVE=0)
static void apply_grid(int M, int C, int tile_units, int* blocks, int* rpb) {
  static const int inter = 1;
  // 512 blocks x 256 threads: 2 blocks per CU; tools/bn_bench.py sweep on the
  // ResNet-50 shapes (more blocks only repeat the coefficient prologue)
  static const int target = 512;
  if (inter) {
    const int cpr = C / 8;
    const int rstep = 256 / (cpr < 256 ? cpr : 256);
    const int tiles = (M + tile_units * rstep - 1) / (tile_units * rstep);
    *blocks = tiles < target ? (tiles > 0 ? tiles : 1) : target;
    *rpb = 0;
    return;
  }
  *rpb = apply_rows_per_block(M, C);
  *blocks = M > 0 ? (M + *rpb - 1) / *rpb : 1;
}

// r2 (7 pointers, nullable): BatchNorm of the residual (stats, gamma, beta, running mean,
// running var, save mean, save invstd); r2 == null or r2[0] == null: plain residual add
extern "C" hipError_t zoo_bn_fwd_apply(const void* X, const float* stats, const float* gamma,
                                       const float* beta, const void* resid, void* Y, float* rmean,
                                       float* rvar, float* smean, float* sinv, int M, int C, float eps,
                                       float momentum, int relu, int training, const void* const* r2,
                                       void* mask, hipStream_t st) {
  int rpb, blocks;
  apply_grid(M, C, 4, &blocks, &rpb);
  BnSide side{nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (r2 && r2[0] && training) {
    side.stats = (const float*)r2[0]; side.gamma = (const float*)r2[1]; side.beta = (const float*)r2[2];
    side.running_mean = (float*)r2[3]; side.running_var = (float*)r2[4];
    side.save_mean = (float*)r2[5]; side.save_invstd = (float*)r2[6];
  }
  hipLaunchKernelGGL(bn_fwd_apply_kernel, dim3(blocks), dim3(256), 0, st, (const bf16_t*)X,
                     stats, gamma, beta, (const bf16_t*)resid, (bf16_t*)Y, rmean, rvar, smean, sinv, M, C, eps,
                     momentum, relu, training, rpb, side, (uint8_t*)mask);
  return hipGetLastError();
}

extern "C" hipError_t zoo_bn_bwd_apply(const void* dZ, const void* Z, const void* X, const float* smean,
                                       const float* sinv, const float* gamma, const float* sums, void* dX,
                                       void* dResid, float* dgamma, float* dbeta, int M, int C,
                                       hipStream_t st) {
  // rows per step (ZOO_BN_BWD_ROWS=4: 8-12 loads in flight per thread): 2 and 4 measure the
  // same, 6-8.6 TB/s on the ResNet-50 shapes (tools/bn_bench.py, round 3)
  static const int rows = 2;
  int rpb, blocks;
  apply_grid(M, C, rows, &blocks, &rpb);
  if (rows == 2)
    hipLaunchKernelGGL(bn_bwd_apply_kernel<2>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)dZ,
                       (const bf16_t*)Z, (const bf16_t*)X, smean, sinv, gamma, sums, (bf16_t*)dX, (bf16_t*)dResid,
                       dgamma, dbeta, M, C, rpb);
  else
    hipLaunchKernelGGL(bn_bwd_apply_kernel<4>, dim3(blocks), dim3(256), 0, st, (const bf16_t*)dZ,
                       (const bf16_t*)Z, (const bf16_t*)X, smean, sinv, gamma, sums, (bf16_t*)dX, (bf16_t*)dResid,
                       dgamma, dbeta, M, C, rpb);
  return hipGetLastError();
}

// grid of act_colsum_kernel: column groups of CT threads, row chunks of >= 32 rows, ~1024 blocks
static void colsum_grid(int M, int C, int* ct, int* col_groups, int* chunks, int* rows_per_chunk) {
  const int cpr = C >> 3;
  *ct = (cpr % 64 == 0 || cpr > 256) ? 64 : 32;
  *col_groups = (cpr + *ct - 1) / *ct;
  // total blocks (ZOO_COLSUM_BLOCKS): every block ends in one fp32 atomic per column, so the
  // block count is also the number of adders per output address
  static const int target = 256;  // BERT b128: 17.37 -> 17.20 ms/step vs 1024
  int ch = target / *col_groups;
  const int max_ch = (M + 31) / 32;
  if (ch > max_ch) ch = max_ch;
  if (ch < 1) ch = 1;
  *rows_per_chunk = (M + ch - 1) / ch;
  *chunks = (M + *rows_per_chunk - 1) / *rows_per_chunk;
}

// number of partial rows the deterministic (partial) mode of zoo_act_bwd_reduce writes
extern "C" int zoo_act_bwd_reduce_parts(int M, int C) {
  int ct, cg, ch, rpc;
  colsum_grid(M, C, &ct, &cg, &ch, &rpc);
  return ch;
}

// dY = act'(dZ) (Z non-null: ReLU mask, or GELU derivative when gelu) and out[c] += sum_rows dY
// (out non-null; partial: out is [parts][C] partials for an ordered fold by the caller).
// Returns the number of partial rows.
extern "C" int zoo_act_bwd_reduce(const void* dZ, const void* Z, void* dY, float* out, int M, int C, int partial,
                                  int gelu, hipStream_t st) {
  int ct, cg, ch, rpc;
  colsum_grid(M, C, &ct, &cg, &ch, &rpc);
  const int act = Z ? (gelu ? 2 : 1) : 0;
#define ZOO_COLSUM(A_, CT_)                                                                                   \
  hipLaunchKernelGGL((act_colsum_kernel<A_, CT_>), dim3(ch * cg), dim3(256), 0, st, (const bf16_t*)dZ,       \
                     (const bf16_t*)Z, (bf16_t*)dY, out, M, C, rpc, cg, partial)
  if (ct == 64) {
    if (act == 2) ZOO_COLSUM(2, 64); else if (act == 1) ZOO_COLSUM(1, 64); else ZOO_COLSUM(0, 64);
  } else {
    if (act == 2) ZOO_COLSUM(2, 32); else if (act == 1) ZOO_COLSUM(1, 32); else ZOO_COLSUM(0, 32);
  }
#undef ZOO_COLSUM
  return ch;
}

// fused stem BN -> ReLU -> max-pool (see bn_relu_maxpool_fwd_kernel); C/8 must be a power of
// two <= 256, R*S < 255 (checked by the caller)
static int pool_row_lg(int C) {
  const int cpr = C >> 3;
  int lg = 0;
  while ((1 << lg) < cpr) ++lg;
  return lg;
}

extern "C" hipError_t zoo_bn_relu_maxpool_fwd(const void* X, const float* stats, const float* gamma,
                                              const float* beta, void* Y, void* best, void* arg, float* rmean,
                                              float* rvar, float* smean, float* sinv, float eps, float momentum,
                                              int N, int H, int W, int C, int P, int Q, int R, int S, int sh, int sw,
                                              int ph, int pw, hipStream_t st) {
  const bool stem = R == 3 && S == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1;
  hipLaunchKernelGGL(stem ? bn_relu_maxpool_fwd_kernel<true> : bn_relu_maxpool_fwd_kernel<false>, dim3(N * P),
                     dim3(256), 0, st, (const bf16_t*)X, stats, gamma, beta, (bf16_t*)Y, (bf16_t*)best,
                     (uint8_t*)arg, rmean, rvar, smean, sinv, N * H * W, eps, momentum, H, W, C, P, Q, R, S, sh, sw,
                     ph, pw, pool_row_lg(C));
  return hipGetLastError();
}

extern "C" hipError_t zoo_bn_relu_maxpool_bwd(const void* dY, const void* best, const void* arg, const void* X,
                                              const float* smean, const float* sinv, const float* gamma,
                                              float* sums, void* dX, float* dgamma, float* dbeta, int N, int H,
                                              int W, int C, int P, int Q, int R, int S, int sh, int sw, int ph,
                                              int pw, hipStream_t st) {
  const int lg = pool_row_lg(C);
  const int rows = N * P;
  hipLaunchKernelGGL(bn_relu_maxpool_bwd_reduce_kernel, dim3(rows < 512 ? rows : 512), dim3(256), 0, st,
                     (const bf16_t*)dY, (const bf16_t*)best, (const uint8_t*)arg, smean, sinv, sums, rows, Q, C, lg);
  const bool stem = R == 3 && S == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1;
  hipLaunchKernelGGL(stem ? bn_relu_maxpool_bwd_apply_kernel<true> : bn_relu_maxpool_bwd_apply_kernel<false>,
                     dim3(N * H), dim3(256), 0, st, (const bf16_t*)dY,
                     (const uint8_t*)arg, (const bf16_t*)X, smean, sinv, gamma, sums, (bf16_t*)dX, dgamma, dbeta,
                     N * H * W, H, W, C, P, Q, R, S, sh, sw, ph, pw, lg);
  return hipGetLastError();
}
