// Sparse / recommendation kernels on gfx950:
//   * embedding bag   out[b] = combine_{j in bag b} w_j * table[id_j]    (sum | mean | sqrtn)
//   * sparse linear   y[b]   = bias + sum_{j in row b} v_j * W[:, col_j]  (CSR input)
// with their backward passes accumulating fp32 into the (flat) parameter gradient.
//
// Reference: Zs/pipeline/api/keras/layers/SparseEmbedding.scala:76-88 (BigDL
// LookupTableSparse: combiner sum/mean/sqrtn, max-norm), SparseDense.scala:86-98 (BigDL
// SparseLinear) and the Wide&Deep wide/indicator columns (Zs/models/recommendation/
// WideAndDeep.scala:113-144).
//
// Layout: an embedding bag is one 64-lane wave; lanes cover the embedding row in 16-byte
// float4 chunks (64 x 4 = 256 floats per pass), so every gathered row is read as whole
// 1 KiB wave transactions. Bags come either from CSR offsets (sparse COO input) or from a
// dense padded id matrix [B][L] (ids < 0 or == pad are skipped), so neither layout needs a
// host-side conversion pass.
#include "common.h"

namespace zoo {

template <int VEC>
struct VecF;
template <>
struct VecF<4> {
  typedef float4 T;
  static ZOO_DEV void ld(const float* p, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  }
  static ZOO_DEV void st(float* p, const float* v) { *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]); }
};
template <>
struct VecF<1> {
  typedef float T;
  static ZOO_DEV void ld(const float* p, float* v) { v[0] = *p; }
  static ZOO_DEV void st(float* p, const float* v) { *p = v[0]; }
};

// max-norm renormalisation factor of one table row (wave-cooperative: every lane returns it)
template <int VEC>
ZOO_DEV float row_renorm(const float* row, int D, float max_norm, int lane) {
  float ss = 0.f;
  for (int c = lane * VEC; c < D; c += 64 * VEC) {
    float v[VEC];
    VecF<VEC>::ld(row + c, v);
#pragma unroll
    for (int e = 0; e < VEC; ++e) ss += v[e] * v[e];
  }
  ss = warp_sum(ss);
  const float n = sqrtf(ss);
  return n > max_norm ? max_norm / (n + 1e-7f) : 1.f;
}

// bag b's id range, clamped to [0, nnz) so a malformed offset vector cannot read out of bounds
ZOO_DEV void bag_range(const int64_t* offs, int L, int b, int64_t nnz, int64_t* j0, int64_t* j1) {
  int64_t a, e;
  if (offs) {
    a = offs[b];
    e = offs[b + 1];
  } else {
    a = (int64_t)b * L;
    e = a + L;
  }
  a = a < 0 ? 0 : (a > nnz ? nnz : a);
  e = e < a ? a : (e > nnz ? nnz : e);
  *j0 = a;
  *j1 = e;
}

// mode: 0 sum, 1 mean (divide by sum of weights), 2 sqrtn (divide by sqrt of sum of squared weights)
template <int VEC>
__global__ __launch_bounds__(256) void embedding_bag_fwd_kernel(const float* __restrict__ table,
                                                                const int64_t* __restrict__ ids,
                                                                const int64_t* __restrict__ offs, int L,
                                                                const float* __restrict__ wts, float* __restrict__ out,
                                                                float* __restrict__ bag_scale, int B, int D, int V,
                                                                int64_t nnz, int64_t pad, int mode, float max_norm) {
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (b >= B) return;
  int64_t j0, j1;
  bag_range(offs, L, b, nnz, &j0, &j1);
  // combiner denominator (wave-uniform)
  float ws = 0.f, ws2 = 0.f;
  for (int64_t j = j0; j < j1; ++j) {
    const int64_t id = ids[j];
    if (id < 0 || id >= V || id == pad) continue;
    const float w = wts ? wts[j] : 1.f;
    ws += w;
    ws2 += w * w;
  }
  float scale = 1.f;
  if (mode == 1) scale = 1.f / fmaxf(ws, 1e-12f);
  else if (mode == 2) scale = 1.f / sqrtf(fmaxf(ws2, 1e-12f));
  if (lane == 0 && bag_scale) bag_scale[b] = scale;
  for (int c = lane * VEC; c - lane * VEC < D; c += 64 * VEC) {
    float acc[VEC];
#pragma unroll
    for (int e = 0; e < VEC; ++e) acc[e] = 0.f;
    for (int64_t j = j0; j < j1; ++j) {
      const int64_t id = ids[j];
      if (id < 0 || id >= V || id == pad) continue;
      float w = wts ? wts[j] : 1.f;
      const float* row = table + (size_t)id * D;
      if (max_norm > 0.f) w *= row_renorm<VEC>(row, D, max_norm, lane);
      if (c < D) {
        float v[VEC];
        VecF<VEC>::ld(row + c, v);
#pragma unroll
        for (int e = 0; e < VEC; ++e) acc[e] += w * v[e];
      }
    }
    if (c < D) {
#pragma unroll
      for (int e = 0; e < VEC; ++e) acc[e] *= scale;
      VecF<VEC>::st(out + (size_t)b * D + c, acc);
    }
  }
}

// gtable[id_j] += w_j * renorm_j * scale_b * dout[b]   (the max-norm factor is treated as a
// constant, like an in-place renorm of the looked-up rows)
template <int VEC>
__global__ __launch_bounds__(256) void embedding_bag_bwd_kernel(const float* __restrict__ dout,
                                                                const float* __restrict__ table,
                                                                const int64_t* __restrict__ ids,
                                                                const int64_t* __restrict__ offs, int L,
                                                                const float* __restrict__ wts,
                                                                const float* __restrict__ bag_scale,
                                                                float* __restrict__ gtable, int B, int D, int V,
                                                                int64_t nnz, int64_t pad, float max_norm) {
  const int lane = threadIdx.x & 63;
  const int b = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  if (b >= B) return;
  int64_t j0, j1;
  bag_range(offs, L, b, nnz, &j0, &j1);
  const float scale = bag_scale[b];
  for (int c = lane * VEC; c - lane * VEC < D; c += 64 * VEC) {
    float g[VEC];
    if (c < D) {
      VecF<VEC>::ld(dout + (size_t)b * D + c, g);
#pragma unroll
      for (int e = 0; e < VEC; ++e) g[e] *= scale;
    }
    for (int64_t j = j0; j < j1; ++j) {
      const int64_t id = ids[j];
      if (id < 0 || id >= V || id == pad) continue;
      float w = wts ? wts[j] : 1.f;
      if (max_norm > 0.f) w *= row_renorm<VEC>(table + (size_t)id * D, D, max_norm, lane);
      if (c < D) {
        float* dst = gtable + (size_t)id * D + c;
#pragma unroll
        for (int e = 0; e < VEC; ++e) atomicAdd(dst + e, w * g[e]);
      }
    }
  }
}

// y[b][o] = bias[o] + sum_{j in [crow[b], crow[b+1])} val[j] * W[o][col[j]]   (one thread per (b, o))
__global__ __launch_bounds__(256) void sparse_linear_fwd_kernel(const int64_t* __restrict__ crow,
                                                                const int64_t* __restrict__ col,
                                                                const float* __restrict__ val,
                                                                const float* __restrict__ W,
                                                                const float* __restrict__ bias, float* __restrict__ y,
                                                                int B, int O, int IN, int64_t nnz) {
  const size_t total = (size_t)B * O;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(t / O), o = (int)(t - (size_t)b * O);
    float acc = bias ? bias[o] : 0.f;
    const float* wr = W + (size_t)o * IN;
    int64_t j0 = crow[b], j1 = crow[b + 1];
    j0 = j0 < 0 ? 0 : (j0 > nnz ? nnz : j0);
    j1 = j1 < j0 ? j0 : (j1 > nnz ? nnz : j1);
    for (int64_t j = j0; j < j1; ++j) {
      const int64_t c = col[j];
      if (c >= 0 && c < IN) acc += val[j] * wr[c];
    }
    y[t] = acc;
  }
}

// dW[o][col[j]] += val[j] * dy[row[j]][o]   (one thread per (nonzero, o); duplicates across
// rows collide, hence the atomics)
__global__ __launch_bounds__(256) void sparse_linear_bwd_w_kernel(const int64_t* __restrict__ row,
                                                                  const int64_t* __restrict__ col,
                                                                  const float* __restrict__ val,
                                                                  const float* __restrict__ dy,
                                                                  float* __restrict__ dW, int64_t nnz, int B, int O,
                                                                  int IN) {
  const size_t total = (size_t)nnz * O;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int64_t j = (int64_t)(t / O);
    const int o = (int)(t - (size_t)j * O);
    const int64_t c = col[j], r = row[j];
    if (c >= 0 && c < IN && r >= 0 && r < B) atomicAdd(dW + (size_t)o * IN + c, val[j] * dy[(size_t)r * O + o]);
  }
}

// db[o] += sum_b dy[b][o]: blocks own (64-column group, 1024-row chunk); 4 row lanes per
// column folded in LDS, one atomic per column per block
__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ dy, float* __restrict__ db, int B,
                                                      int O) {
  __shared__ float part[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int o = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * 1024, r1 = min(B, r0 + 1024);
  float s = 0.f;
  if (o < O)
    for (int r = r0 + rl; r < r1; r += 4) s += dy[(size_t)r * O + o];
  part[rl][cl] = s;
  __syncthreads();
  if (rl == 0 && o < O) atomicAdd(db + o, (part[0][cl] + part[1][cl]) + (part[2][cl] + part[3][cl]));
}

static bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

static int sgrid(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  return (int)(b ? b : 1);
}

}  // namespace zoo

using namespace zoo;

extern "C" hipError_t zoo_embedding_bag_fwd(const float* table, const int64_t* ids, const int64_t* offs, int L,
                                            const float* wts, float* out, float* bag_scale, int B, int D, int V,
                                            int64_t nnz, int64_t pad, int mode, float max_norm, hipStream_t st) {
  const dim3 grid((B + 3) / 4);
  if (D % 4 == 0 && al16(table) && al16(out))
    hipLaunchKernelGGL(embedding_bag_fwd_kernel<4>, grid, dim3(256), 0, st, table, ids, offs, L, wts, out, bag_scale,
                       B, D, V, nnz, pad, mode, max_norm);
  else
    hipLaunchKernelGGL(embedding_bag_fwd_kernel<1>, grid, dim3(256), 0, st, table, ids, offs, L, wts, out, bag_scale,
                       B, D, V, nnz, pad, mode, max_norm);
  return hipGetLastError();
}

extern "C" hipError_t zoo_embedding_bag_bwd(const float* dout, const float* table, const int64_t* ids,
                                            const int64_t* offs, int L, const float* wts, const float* bag_scale,
                                            float* gtable, int B, int D, int V, int64_t nnz, int64_t pad,
                                            float max_norm, hipStream_t st) {
  const dim3 grid((B + 3) / 4);
  if (D % 4 == 0 && al16(table) && al16(dout) && al16(gtable))
    hipLaunchKernelGGL(embedding_bag_bwd_kernel<4>, grid, dim3(256), 0, st, dout, table, ids, offs, L, wts,
                       bag_scale, gtable, B, D, V, nnz, pad, max_norm);
  else
    hipLaunchKernelGGL(embedding_bag_bwd_kernel<1>, grid, dim3(256), 0, st, dout, table, ids, offs, L, wts,
                       bag_scale, gtable, B, D, V, nnz, pad, max_norm);
  return hipGetLastError();
}

extern "C" hipError_t zoo_sparse_linear_fwd(const int64_t* crow, const int64_t* col, const float* val, const float* W,
                                            const float* bias, float* y, int B, int O, int IN, int64_t nnz,
                                            hipStream_t st) {
  hipLaunchKernelGGL(sparse_linear_fwd_kernel, dim3(sgrid((size_t)B * O)), dim3(256), 0, st, crow, col, val, W, bias,
                     y, B, O, IN, nnz);
  return hipGetLastError();
}

extern "C" hipError_t zoo_sparse_linear_bwd(const int64_t* row, const int64_t* col, const float* val, const float* dy,
                                            float* dW, float* db, int64_t nnz, int B, int O, int IN, hipStream_t st) {
  if (nnz > 0)
    hipLaunchKernelGGL(sparse_linear_bwd_w_kernel, dim3(sgrid((size_t)nnz * O)), dim3(256), 0, st, row, col, val, dy,
                       dW, nnz, B, O, IN);
  if (db)
    hipLaunchKernelGGL(col_sum_kernel, dim3((O + 63) / 64, (B + 1023) / 1024), dim3(256), 0, st, dy, db, B, O);
  return hipGetLastError();
}
