// Geometry structs shared by the HIP kernels and the host binding layer.
#pragma once

namespace zoo {

// Implicit-GEMM conv / GEMM geometry (igemm.hip).
// Per-channel statistics buffers in slotted form: [2C final][slots x 2C][counter]
constexpr int kStatSlots = 16;
constexpr int kStatPartial = -1;

struct ConvGeom {
  int N, H, W, C;        // input activation, NHWC
  int K;                 // output channels (GEMM N dimension)
  int R, S;              // filter
  int P, Q;              // output spatial (GEMM rows = N*P*Q)
  int sh, sw, ph, pw;    // stride / padding (in the possibly-dilated input space)
  int dh, dw;            // filter dilation
  int lh, lw;            // input dilation (1 = plain conv; >1 = transposed conv)
  int M;                 // N*P*Q
  int Ktot;              // R*S*C (logical reduction length)
  int ldb;               // leading dim of the weight matrix (>= Ktot, %8 == 0)
  // optional output-row remap (strided scatter into a larger NHWC tensor):
  // row (n,p,q) -> ((n*oH + oh0 + osh*p)*oW + ow0 + osw*q)*K
  int omap, oH, oW, osh, osw, oh0, ow0;
  // >0: per-channel statistics go through `stat_slots` contention-spreading slots
  // (see slotted_stats in common.h); 0: direct atomics into the [2*K] buffer;
  // kStatPartial: no atomics -- the stats pointer is a [tiles_m][2*K] partials buffer,
  // each workgroup STORES its column sums into row tm, and zoo_stats_part_finalize
  // folds the rows in a fixed order (deterministic, contention-free)
  int stat_slots;
  // experiment bits (igemm2 band tiles, ZOO_I2_DBG; 0 in production): 1 = no MFMA, 2 = no
  // epilogue stores, 4 = no B staging in the loop, 8 = no A fragment reads
  int dbg;
};

// Fused BatchNorm-backward statistics in a dgrad epilogue: the conv computing
// dL/dz of a conv->BN->ReLU unit writes dy = dz * [z > 0] instead of dz and
// accumulates sums[c] += dy, sums[K + c] += dy * (y - mean[c]) * inv[c].
struct BwdStats {
  const void* z;      // ReLU output of the producing unit (nullptr: no ReLU mask)
  const void* y;      // its pre-BN conv output
  const float* mean;
  const float* inv;
  float* sums;        // [2*K]
  // 1: z is a GELU pre-activation -- the output is scaled by GELU'(z) instead of masked, and
  // `sums` collects its plain column sums (the producing linear's bias gradient); y / mean /
  // inv are unused (the transformer FFN: GELU backward in the next linear's dgrad epilogue)
  int zgelu;
  // ReLU-mask source when zgelu == 0 (bnmask.h bnm_apply):
  //   0: z is the bf16 ReLU output, keep where z > 0 (nullptr: no mask);
  //   1: no z read -- the mask is recomputed from y (already read for the sums) with the
  //      producer's affine: y * gamma * inv + (beta - mean * gamma * inv) > 0, the expression its
  //      forward apply evaluated (units without a residual add);
  //   2: z is a bit mask written by the forward apply, bit (c % 8) of byte (m * K + c) / 8
  //      (units with a residual add, where y alone does not determine the sign)
  int zmode;
  const float* mgamma;  // zmode 1 (nullptr: gamma = 1 / beta = 0)
  const float* mbeta;
  int unbatched;        // 1: igemm.hip EPI 2 row loop without batched loads (A/B, ZOO_EPI2_BATCH=0)
  // BatchNorm-backward PROLOGUE (pw.hip EPI 2, bnfold.hip): the GEMM's A operand X is the
  // ReLU-masked gradient g of a conv -> BN unit; the kernel forms that unit's BN backward
  // dy = coef[k] g + coef[Kx + k] pro_y + coef[2 Kx + k] in registers (Kx = X channels) and, if
  // pro_dy is set, writes dy there for the weight gradient. nullptr: X is the operand itself.
  const void* pro_y;
  const float* pro_coef;
  void* pro_dy;
  // 1: `resid` is a half-resolution [N, H/2, W/2, K] gradient added at the even (h, w) output
  // positions only -- the compact data gradient of a 1x1 stride-2 projection shortcut, which
  // then never gets its zero-interleaved full-size tensor (pw.hip EPI 2 only)
  int resid_half;
  // 1: forward consumer-side BN apply (pw.hip EPI 1 prologue): X is a conv -> BN -> ReLU unit's
  // pre-BN output y; the GEMM runs on relu(coef[k] y + coef[2 Kx + k]) (pro_coef [3][Kx], the
  // middle row unused), written to pro_dy by channel group 0 -- that unit's output z
  int pro_fwd;
  // forward prologue of a RESIDUAL unit (pw.hip EPI 4, a ResNet block output consumed by the next
  // block's 1x1 conv1): z = relu(A y + Cc + R) with R = pro_res, or R = rA pro_res + rC when
  // pro_rcoef ([3][Kx], a projection shortcut's BatchNorm) is set; channel group 0 also writes
  // the 1-bit ReLU mask of z to pro_mask (BwdStats.zmode 2 layout) for the unit's BN backward
  const void* pro_res;
  const float* pro_rcoef;
  void* pro_mask;
  // igemm2.hip EPI 3 with an activation: the pre-activation (bias added) is also stored here as
  // bf16 -- the training forward of a GELU linear, whose backward needs it (nullptr: not stored)
  void* act_pre;
  // pw.hip EPI 2 (short reductions): sums2[c] += sum over rows of out[m][c] * y2[m][c] -- the
  // masked output gradient against a second pre-BN tensor (a fused projection shortcut's raw
  // output, whose BatchNorm sees the same gradient), so its backward needs no reduction pass
  const void* y2;
  float* sums2;
};

// One flipped (sub-)filter of a batched flip (igemm.hip flip_weights_batched_kernel):
// Wt[c][t][u][k] = W[k][r0 + sh*(Ra-1-t)][s0 + sw*(Sb-1-u)][c]; blocks [blk0, blk0+nblk).
struct FlipDesc {
  const void* W;   // bf16
  void* Wt;        // bf16
  int K, R, S, C, ldw, r0, s0, Ra, Sb, sh, sw, ldt, blk0, nblk;
};

// Epilogue class of an implicit-GEMM call (igemm.hip / igemm2.hip and the host binding agree on
// it): 1 = plain bf16 output (+ BN statistics), 2 = backward (residual-gradient add, ReLU mask,
// fused BN-backward sums, remap), 0 = general (bias / activation / fp32 output / ...)
inline int igemm_epi(bool y, bool yf, bool bias, bool resid, int act, bool omap, bool bsums, bool stats) {
  if (y && !yf && !bias && !resid && act == 0 && !omap && !bsums) return 1;
  if (y && !yf && !bias && act == 0 && !stats) return 2;
  // bf16 output with bias and / or ReLU / GELU only (transformer / MLP linears)
  if (y && !yf && !resid && !omap && !bsums && !stats && (act == 0 || act == 1 || act == 2)) return 3;
  return 0;
}

// Tile-routing class of an epilogue (igemm2.hip i2_choose): the GELU-backward form of EPI 2
// (BwdStats.zgelu) reads one tensor, not the BN-backward's two plus a reduction, and routes like
// the plain epilogues; everywhere else the routing class is the epilogue itself.
inline int igemm_route_epi(int epi, bool zgelu) { return (epi == 2 && zgelu) ? 4 : epi; }

// Plain GEMM geometry (gemm256.hip): Y[M, N] = A[M, K] . B[N, K]^T
struct GemmGeom {
  int M, N, K;
  int lda, ldb, ldy;   // leading dims (elements), all % 8 == 0
};

// Grouped convolution (gconv.hip): one launch per direction, group = grid y.
struct GConvArgs {
  int N, H, W, C;        // input NHWC; C = groups * Cg is also the pixel stride of X / dX
  int K;                 // output channels = groups * Kg, the pixel stride of Y / dY
  int groups, Cg, Kg;
  int R, S, P, Q;
  int sh, sw, ph, pw, dh, dw;
  int ldb;               // packed weight row stride (>= R*S*Cg, % 8 == 0), K rows
  int act;               // forward activation (Act)
  int mper;              // wgrad: output pixels per split (multiple of 32)
};

// Weight-gradient geometry (wgrad.hip).
struct WgradGeom {
  int N, H, W, C;      // input activation (NHWC)
  int K;               // output channels
  int R, S, P, Q;
  int sh, sw, ph, pw, dh, dw;
  int M;               // N*P*Q (reduction length)
  int Ktot;            // R*S*C (GEMM columns)
  int ldw;             // leading dim of dW (>= Ktot)
  int m_per_split;     // multiple of 64
};

// Recurrent cells (rnn.hip). Activation codes shared with zoo/ops/rnn.py.
enum RnnAct : int { RA_LINEAR = 0, RA_TANH = 1, RA_SIGMOID = 2, RA_HSIG = 3, RA_RELU = 4 };
// CELL_GRU: Keras / BigDL GRU (candidate over (r*h) . U_h); CELL_GRU_RA: the "reset-after" GRU of
// torch.nn.GRU / GRUCell (candidate tanh(xn + r * (U_n h + b_hn)))
enum RnnCell : int { CELL_RNN = 0, CELL_LSTM = 1, CELL_GRU = 2, CELL_GRU_RA = 3 };

struct RnnArgs {
  const float* xw;     // [B, T, G*H] input projections (bias included)
  const void* u;       // bf16: U [G*H, H] (forward) or U^T [H, G*H] (backward)
  const float* h0;     // [B, H] or null (zeros)
  const float* c0;     // [B, H] or null (LSTM)
  float* hseq;         // [B, T, H] (forward output; backward input)
  float* cseq;         // [B, T, H] LSTM cell states or null
  float* gates;        // [B, T, G*H] activated gates or null
  float* cT;           // [B, H] final LSTM cell state or null
  const float* dhseq;  // [B, T, H] or null (backward)
  const float* dcT;    // [B, H] or null (backward, LSTM)
  float* dgates;       // [B, T, G*H] (backward)
  float* dh0;          // [B, H] or null (backward)
  float* dc0;          // [B, H] or null (backward, LSTM)
  const float* bhn;    // [H] candidate recurrent bias b_hn (GRU_RA) or null
  float* dgn;          // [B, T, H] d(U_n h + b_hn) (backward, GRU_RA)
  int B, T, act, iact;
};


// JPEG batch geometry (image.hip jpeg_* kernels; host entropy decoder csrc/runtime/jpeg.cpp)
struct JpegGeom {
  int N, ncomp, w, h, hmax, vmax;
  int hs[3], vs[3], bw[3], bh[3], boff[3];   // sampling, padded block grid, block offset per component
  int total;                                 // blocks per image (all components)
};

// deep_input segments (wnd.hip): dense column blocks and embedding lookups of one row
constexpr int DI_MAX_SEG = 8;
struct DeepSeg {
  const float* src;   // dense: [B][ld] fp32; embedding: table [V][width] fp32
  float* gsrc;        // embedding: fp32 table gradient (null: no gradient)
  int col0, width, ld, id_col, V, emb;
};

struct DeepSegs {
  DeepSeg s[DI_MAX_SEG];
  int n;
};

}  // namespace zoo
