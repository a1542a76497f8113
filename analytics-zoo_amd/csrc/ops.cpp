// Python bindings for the zoo gfx950 kernel library (`zoo._C`).
//
// Every entry validates dtype / device / contiguity / shape on the host BEFORE
// launching, because the kernels index raw pointers with the geometry they are
// given (an out-of-bounds access on the GPU can take the whole node down).
// Kernels run on PyTorch's current HIP stream, so they order correctly with
// any other torch work and are capturable into hipGraphs.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include "kernels/geom.h"
#include "kernels/ncf.h"

using zoo::ConvGeom;
using zoo::WgradGeom;
using zoo::GConvArgs;
using zoo::BwdStats;
using zoo::GemmGeom;

extern "C" {
hipError_t zoo_jpeg_idct(const int16_t*, const int32_t*, uint8_t*, const zoo::JpegGeom*, hipStream_t);
hipError_t zoo_jpeg_color_resize(const uint8_t*, void*, const zoo::JpegGeom*, int, int, const float*, const float*,
                                 int, int, hipStream_t);
hipError_t zoo_prob_nll(const void*, int, const int64_t*, float*, float*, float*, int, int, float, int, int,
                        hipStream_t);
void zoo_optim_zero_grad(int);
void zoo_optim_device_hparams(const float*);
void zoo_set_seed_offset(const uint32_t*);
hipError_t zoo_prob_nll_mean(const void*, int, const int64_t*, float*, float*, int, int, float, int, int, hipStream_t);
hipError_t zoo_prob_nll_grad(const void*, int, const int64_t*, const float*, const float*, float*, int, int, float, int,
                             hipStream_t);
int zoo_ncf_tier(int, int, int, int, int, int, int);
int zoo_ncf_nwg(int, int, int, int, int, int, int);
hipError_t zoo_ncf(const zoo::NcfArgs*, float* const*, int, hipStream_t);
hipError_t zoo_igemm(const void*, const void*, void*, float*, const float*, const void*, float*, const ConvGeom*, int,
                     const zoo::BwdStats*, hipStream_t);
int zoo_igemm2_bm(const ConvGeom*, int);
int zoo_igemm2_tiles_m(const ConvGeom*, int);
void zoo_igemm2_band_set(int);
int zoo_c3_grid(const ConvGeom*, int, const zoo::BwdStats*);
void zoo_c3_set(int);
int zoo_c3_stamps(unsigned long long*, int);
void zoo_igemm2_set(int, int);
void zoo_igemm2_w192_set(int);
void zoo_convlstm_pers_set(int);
int zoo_pw_eligible(const ConvGeom*, int, const zoo::BwdStats*);
void zoo_pw_set(int);
void zoo_set_reserved_cus(int);
hipError_t zoo_wlrn(const void*, const void*, void*, float*, float*, int, int, int, int, int, float, float, int,
                    hipStream_t);
hipError_t zoo_resize_bilinear(const void*, void*, int, int, int, int, int, int, int, int, int, hipStream_t);
hipError_t zoo_upsample(const void*, void*, int, int, int, int, int, int, int, int, int, int, hipStream_t);
hipError_t zoo_lstm_step(const float*, const float*, int, const float*, float*, float*, float*, void*, int,
                         const float*, const void*, int, const float*, float*, void*, int, float*, int, int, int, int,
                         int, hipStream_t);
hipError_t zoo_lstm_gates(const float*, const float*, const float*, float*, float*, float*, const float*,
                          const float*, float*, float*, int, int, int, int, int, hipStream_t);
hipError_t zoo_roi_pool(const void*, const float*, void*, int*, const void*, float*, int, int, int, int, int, int,
                        int, float, int, int, hipStream_t);
hipError_t zoo_gemm256(const void*, const void*, void*, float*, const float*, const void*, float*, const GemmGeom*,
                       int, const zoo::BwdStats*, hipStream_t);
hipError_t zoo_flip_weights(const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                            hipStream_t);
hipError_t zoo_flip_weights_batched(const void*, int, int, hipStream_t);
hipError_t zoo_wgrad(const void*, const void*, float*, float*, const WgradGeom*, hipStream_t);
int zoo_wgrad_plan(WgradGeom*);
int zoo_wgrad_band(const WgradGeom*, const void*, const void*, float*, float*, hipStream_t);
hipError_t zoo_gconv(int, const void*, const void*, const void*, void*, const float*, const GConvArgs*, hipStream_t);
hipError_t zoo_bmm(const void*, const void*, void*, const long*, int, int, hipStream_t);
hipError_t zoo_row_reduce(const void*, float*, long, int, int, int, hipStream_t);
hipError_t zoo_ssd_match(const float*, const int*, const float*, int, int, int, float, float, float, int, int*,
                         float*, unsigned long long*, float*, long long*, hipStream_t);
hipError_t zoo_row_l2norm(const void*, const void*, const void*, void*, long, int, int, float, hipStream_t);
hipError_t zoo_deep_input(const float*, int, const zoo::DeepSegs*, void*, const void*, int, int, hipStream_t);
int zoo_wnd_head_blocks(int);
hipError_t zoo_wnd_head_fwd(const float*, const void*, int, const float*, float*, int, int, hipStream_t);
hipError_t zoo_wnd_head_bwd(const float*, const float*, float*, void*, int, float*, float*, int, int, hipStream_t);
hipError_t zoo_ssd_mine(const float*, const long long*, int, int, int, float, unsigned char*, hipStream_t);
hipError_t zoo_l2norm_scale_fwd(const void*, const float*, void*, float*, long, int, float, hipStream_t);
int zoo_l2norm_scale_bwd_blocks(long);
hipError_t zoo_l2norm_scale_bwd(const void*, const void*, const float*, const float*, void*, float*, float*, long, int,
                                float, hipStream_t);
hipError_t zoo_wgrad256(const void*, const void*, float*, float*, int, int, int, int, int, int, hipStream_t);
size_t zoo_wgrad256_part_floats(int, int, int);
void zoo_wgrad256_target(int);
void zoo_wgrad256_set_atomic(int);
hipError_t zoo_wgrad256_conv(const void*, const void*, float*, float*, int, int, int, int, int, int, int, int, int, int,
                             int, int, int, int, int, int, hipStream_t);
hipError_t zoo_stats_finalize(float*, int, int, hipStream_t);
size_t zoo_stats_part_scratch(int, int);
hipError_t zoo_stats_part_finalize(float*, const float*, float*, int, int, hipStream_t);
int zoo_bn_reduce_blocks(int, int);
int zoo_act_bwd_reduce(const void*, const void*, void*, float*, int, int, int, int, hipStream_t);
int zoo_act_bwd_reduce_parts(int, int);
hipError_t zoo_bn_reduce(const void*, const void*, const void*, const float*, const float*, float*, int, int, int, int,
                         hipStream_t);
hipError_t zoo_bn_fwd_apply(const void*, const float*, const float*, const float*, const void*, void*, float*, float*,
                            float*, float*, int, int, float, float, int, int, const void* const*, void*,
                            hipStream_t);
hipError_t zoo_bn_bwd_apply(const void*, const void*, const void*, const float*, const float*, const float*,
                            const float*, void*, void*, float*, float*, int, int, hipStream_t);
hipError_t zoo_maxpool_fwd(const void*, void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                           hipStream_t);
hipError_t zoo_bn_relu_maxpool_fwd(const void*, const float*, const float*, const float*, void*, void*, void*, float*,
                                   float*, float*, float*, float, float, int, int, int, int, int, int, int, int, int,
                                   int, int, int, hipStream_t);
hipError_t zoo_bn_relu_maxpool_bwd(const void*, const void*, const void*, const void*, const float*, const float*,
                                   const float*, float*, void*, float*, float*, int, int, int, int, int, int, int, int,
                                   int, int, int, int, hipStream_t);
hipError_t zoo_maxpool_bwd(const void*, const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int,
                           hipStream_t);
hipError_t zoo_gap_fwd(const void*, void*, int, int, int, hipStream_t);
hipError_t zoo_avgpool_fwd(const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                           hipStream_t);
hipError_t zoo_avgpool_bwd(const void*, void*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                           hipStream_t);
hipError_t zoo_dwconv_fwd(const void*, const void*, const float*, void*, const int*, int, hipStream_t);
hipError_t zoo_dwconv_dgrad(const void*, const void*, void*, const int*, hipStream_t);
hipError_t zoo_dwconv_wgrad(const void*, const void*, float*, float*, const int*, hipStream_t);
int zoo_dwconv_wgrad_blocks(const int*);
hipError_t zoo_softmax_rows(const void*, void*, int, int, int, int, hipStream_t);
hipError_t zoo_softmax_rows_bwd(const void*, const void*, void*, int, int, int, int, hipStream_t);
hipError_t zoo_lrn(const void*, const void*, void*, size_t, int, int, float, float, float, int, int, hipStream_t);
hipError_t zoo_gap_bwd(const void*, void*, int, int, int, hipStream_t);
hipError_t zoo_softmax_xent_mean(const void*, int, const int64_t*, float*, float*, void*, int, int, int, hipStream_t);
hipError_t zoo_xent_grad_scale(const void*, int, const float*, const float*, void*, size_t, hipStream_t);
hipError_t zoo_softmax_xent(const void*, int, const int64_t*, float*, float*, void*, int, int, float, int, int,
                            hipStream_t);
hipError_t zoo_sgd(float*, const float*, float*, void*, size_t, float, float, float, float, int, float, int,
                   hipStream_t);
hipError_t zoo_adam(float*, const float*, float*, float*, void*, size_t, float, float, float, float, float, float,
                    float, float, int, hipStream_t);
hipError_t zoo_adaptive(float*, const float*, float*, float*, void*, size_t, int, float, float, float, float, float,
                        float, float, hipStream_t);
hipError_t zoo_sumsq(const float*, size_t, float*, hipStream_t);
hipError_t zoo_clip(float*, size_t, float, float, const float*, float, hipStream_t);
hipError_t zoo_nchw_to_nhwc(const float*, void*, int, int, int, int, int, hipStream_t);
hipError_t zoo_dropout_add(const void*, const void*, void*, size_t, float, uint64_t, hipStream_t);
hipError_t zoo_nchw_to_s2d(const float*, void*, int, int, int, int, int, int, int, hipStream_t);
hipError_t zoo_nhwc_u8_to_s2d(const void*, void*, int, int, int, int, int, int, int, const float*, const float*,
                              hipStream_t);
hipError_t zoo_bnres_apply(const void*, const float*, const void*, const float*, void*, void*, size_t, int, hipStream_t);
hipError_t zoo_bnfold_coef(int, const float*, const float*, const float*, const float*, long long, float*, float*,
                           float*, hipStream_t);
hipError_t zoo_bnpro_apply(const void*, const void*, const float*, void*, size_t, int, int, hipStream_t);
hipError_t zoo_bn_fwd_coef(const float*, const float*, const float*, float*, float*, float*, float*, float*, int, int,
                           float, float, hipStream_t);
hipError_t zoo_convlstm_step(const void*, const void*, int, int, int, int, int, int, int, int, int, int, int, int, int,
                             const void*, int, const float*, float*, float*, float*, void*, int, const float*,
                             const float*, float*, int, float*, void*, int, int, float*, hipStream_t);
hipError_t zoo_bf16_to_f32(const void*, float*, size_t, int, hipStream_t);
hipError_t zoo_f32_to_bf16(const float*, void*, size_t, hipStream_t);
hipError_t zoo_sum_chunks_bf16(const void*, int, size_t, float*, void*, float, hipStream_t);
hipError_t zoo_add_bf16(const void*, const void*, void*, size_t, hipStream_t);
hipError_t zoo_layernorm_fwd(const void*, int, const float*, const float*, void*, float*, float*, int, int, float,
                             hipStream_t);
void zoo_layernorm_defer_fold(int);
int zoo_layernorm_bwd_v2_blocks(int, int, int);
hipError_t zoo_layernorm_fold(float*, int, int, float*, float*, hipStream_t);
hipError_t zoo_layernorm_bwd_drop(const void*, const void*, const float*, const float*, const float*, void*, void*,
                                  float*, float*, int, int, float*, const void*, float, uint64_t, hipStream_t);
hipError_t zoo_dropout_add_layernorm_fwd(const void*, const void*, const float*, const float*, void*, void*, float*,
                                         float*, int, int, float, float, uint64_t, hipStream_t);
hipError_t zoo_layernorm_bwd(const void*, const void*, int, const float*, const float*, const float*, void*, float*,
                             float*, int, int, float*, const void*, hipStream_t);
size_t zoo_layernorm_bwd_part_floats(int, int, int);
hipError_t zoo_embedding_fwd(const void*, int, const int64_t*, void*, int, int, int, int64_t, hipStream_t);
hipError_t zoo_resize_normalize(const void*, void*, int, int, int, int, int, int, const float*, const float*, int, int,
                                hipStream_t);
hipError_t zoo_embedding_bwd(const void*, int, const int64_t*, float*, int, int, int, int64_t, float, hipStream_t);
hipError_t zoo_absmax(const void*, int, size_t, float*, hipStream_t);
hipError_t zoo_im2col_q8(const void*, int, const float*, void*, int, int, int, int, int, int, int, int, int, int, int,
                         int, int, hipStream_t);
hipError_t zoo_qgemm(const void*, const void*, const float*, const float*, const float*, const void*, void*, int, int,
                     int, int, int, hipStream_t);
hipError_t zoo_attn_fwd(const void*, const void*, const void*, const float*, void*, float*, int, int, int, int, int,
                        float, int, const long*, float, uint64_t, hipStream_t);
hipError_t zoo_rnn(const zoo::RnnArgs*, int, int, int, hipStream_t);
hipError_t zoo_nms_mask(const float*, int, float, unsigned long long*, hipStream_t);
hipError_t zoo_embedding_bag_fwd(const float*, const int64_t*, const int64_t*, int, const float*, float*, float*, int,
                                 int, int, int64_t, int64_t, int, float, hipStream_t);
hipError_t zoo_embedding_bag_bwd(const float*, const float*, const int64_t*, const int64_t*, int, const float*,
                                 const float*, float*, int, int, int, int64_t, int64_t, float, hipStream_t);
hipError_t zoo_sparse_linear_fwd(const int64_t*, const int64_t*, const float*, const float*, const float*, float*, int,
                                 int, int, int64_t, hipStream_t);
hipError_t zoo_sparse_linear_bwd(const int64_t*, const int64_t*, const float*, const float*, float*, float*, int64_t,
                                 int, int, int, hipStream_t);
hipError_t zoo_qconv(const void*, const void*, void*, const float*, const float*, const void*, float, const float*,
                     const ConvGeom*, int, int, int, int, hipStream_t);
hipError_t zoo_quantize_i8(const void*, void*, size_t, float, const float*, int, int, hipStream_t);
hipError_t zoo_gap_i8(const void*, void*, int, int, int, float, const float*, int, int, hipStream_t);
hipError_t zoo_quantize_f8(const void*, void*, size_t, float, const float*, int, hipStream_t);
hipError_t zoo_act(const void*, const void*, void*, size_t, int, int, float, hipStream_t);
hipError_t zoo_dropout(const void*, void*, size_t, int, float, uint64_t, hipStream_t);
hipError_t zoo_loss(const void*, const void*, void*, float*, size_t, int, int, float, float, hipStream_t);
hipError_t zoo_auc_hist(const float*, const float*, float*, size_t, int, float, float, hipStream_t);
hipError_t zoo_box_decode(const float*, const float*, float*, int, int, float, float, int, hipStream_t);
hipError_t zoo_attn_bwd(const void*, const void*, const void*, const void*, const float*, const void*, const float*,
                        float*, void*, void*, void*, int, int, int, int, int, float, int, const long*, float, uint64_t,
                        hipStream_t);
}

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "zoo HIP kernel launch failed in ", what, ": ", hipGetErrorString(e));
}

// slotted per-channel statistics buffer: [2C final][kStatSlots x 2C][counter, padded to 4 floats]
int64_t stat_len(int64_t C) { return 2 * C * (zoo::kStatSlots + 1) + 4; }

// pooled output size (floor or ceil mode; a ceil-mode window must start inside the padded input)
int pool_out(int H, int R, int st, int pad, bool ceil_mode) {
  int o = ceil_mode ? (H + 2 * pad - R + st - 1) / st + 1 : (H + 2 * pad - R) / st + 1;
  if (ceil_mode && (o - 1) * st >= H + pad) --o;
  return o;
}

// Reduction modes.
//  * deterministic: every cross-workgroup float reduction of the conv/BN/loss path goes through
//    per-workgroup partials folded in a fixed order (no float atomics): identical inputs give
//    bit-identical outputs run to run. ZOO_DETERMINISTIC=1 or set_deterministic(True).
//  * stats_partial / wgrad_partial: the same partial-buffer reductions used for speed (no atomic
//    contention) -- on by default where they measured faster.
bool env_flag(const char* name, bool dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) != 0 : dflt;
}
bool g_deterministic = env_flag("ZOO_DETERMINISTIC", false);
// partial-row statistics / ordered weight-gradient folds: the deterministic mode's reductions
bool g_stats_partial = false;
bool g_wgrad_partial = false;
bool stats_partial() { return g_deterministic || g_stats_partial; }
bool wgrad_partial() { return g_deterministic || g_wgrad_partial; }

// out[0..n2) += ordered fold of part [nparts][n2]
void fold_partials(float* out, const torch::Tensor& part, int n2, int nparts) {
  const size_t scr = zoo_stats_part_scratch(n2, nparts);
  torch::Tensor s;
  if (scr) s = torch::empty({(int64_t)scr}, part.options());
  check_hip(zoo_stats_part_finalize(out, part.data_ptr<float>(), scr ? s.data_ptr<float>() : nullptr, n2, nparts,
                                    cur_stream()),
            "stats_part_finalize");
}

void req(const torch::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

template <typename T>
T* opt_ptr(const c10::optional<torch::Tensor>& t) {
  return t.has_value() && t->defined() ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

ConvGeom make_geom(const torch::Tensor& x, int K, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw,
                   int lh, int lw, int ldb) {
  ConvGeom g{};
  g.N = x.size(0); g.H = x.size(1); g.W = x.size(2); g.C = x.size(3);
  g.K = K; g.R = R; g.S = S;
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dw; g.lh = lh; g.lw = lw;
  const int Hd = (g.H - 1) * lh + 1, Wd = (g.W - 1) * lw + 1;  // extent of the (dilated) input
  g.P = (Hd + 2 * ph - dh * (R - 1) - 1) / sh + 1;
  g.Q = (Wd + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  g.M = g.N * g.P * g.Q;
  g.Ktot = R * S * g.C;
  g.ldb = ldb;
  return g;
}

static void check_al16(const void* p, const char* what);

// x: [N,H,W,C] bf16; w: [K, ldb] bf16 (logical [K][R][S][C] rows, zero padded to ldb)
void bn_reduce(torch::Tensor a, c10::optional<torch::Tensor> z, c10::optional<torch::Tensor> x,
               c10::optional<torch::Tensor> mean, c10::optional<torch::Tensor> invstd, torch::Tensor out, int mode);

torch::Tensor conv_fwd(torch::Tensor x, torch::Tensor w, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw,
                       int lh, int lw, c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> resid,
                       c10::optional<torch::Tensor> stats, int act, bool out_f32, bool out_bf16, int out_h,
                       int out_w, c10::optional<torch::Tensor> out, std::vector<int64_t> omap,
                       c10::optional<torch::Tensor> bz, c10::optional<torch::Tensor> by,
                       c10::optional<torch::Tensor> bmean, c10::optional<torch::Tensor> binv,
                       c10::optional<torch::Tensor> bsums, c10::optional<torch::Tensor> bgamma,
                       c10::optional<torch::Tensor> bbeta, c10::optional<torch::Tensor> pro_y,
                       c10::optional<torch::Tensor> pro_coef, c10::optional<torch::Tensor> pro_dy,
                       bool resid_half, bool pro_fwd, c10::optional<torch::Tensor> pro_rcoef,
                       c10::optional<torch::Tensor> pro_mask, c10::optional<torch::Tensor> act_pre,
                       c10::optional<torch::Tensor> by2, c10::optional<torch::Tensor> bsums2) {
  req(x, at::kBFloat16, "x");
  req(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2, "conv_fwd: x must be NHWC 4-D, w 2-D [K, ldb]");
  const int C = x.size(3), K = w.size(0), ldb = w.size(1);
  TORCH_CHECK(C == 4 || C % 8 == 0, "conv_fwd: input channels must be 4 or a multiple of 8, got ", C);
  TORCH_CHECK(K % 8 == 0, "conv_fwd: output channels must be a multiple of 8, got ", K);
  TORCH_CHECK(ldb % 8 == 0 && ldb >= R * S * C, "conv_fwd: bad weight leading dim ", ldb);
  TORCH_CHECK(R >= 1 && S >= 1 && sh >= 1 && sw >= 1 && dh >= 1 && dw >= 1 && lh >= 1 && lw >= 1 && ph >= 0 && pw >= 0,
              "conv_fwd: bad geometry");
  ConvGeom g = make_geom(x, K, R, S, sh, sw, ph, pw, dh, dw, lh, lw, ldb);
  // transposed convs (dgrad) may need one extra output row/col (asymmetric padding):
  // the loader zero-fills taps that fall outside the input, so a larger P/Q is safe.
  if (out_h > 0) { TORCH_CHECK(out_h <= g.P + sh, "conv_fwd: out_h"); g.P = out_h; }
  if (out_w > 0) { TORCH_CHECK(out_w <= g.Q + sw, "conv_fwd: out_w"); g.Q = out_w; }
  g.M = g.N * g.P * g.Q;
  g.omap = 0; g.oH = g.P; g.oW = g.Q; g.osh = 1; g.osw = 1; g.oh0 = 0; g.ow0 = 0;
  if (!omap.empty()) {
    // omap = {oH, oW, osh, osw, oh0, ow0}: write row (n,p,q) to (n, oh0+osh*p, ow0+osw*q) of [N,oH,oW,K]
    TORCH_CHECK(omap.size() == 6, "conv_fwd: omap needs 6 entries");
    g.omap = 1; g.oH = omap[0]; g.oW = omap[1]; g.osh = omap[2]; g.osw = omap[3]; g.oh0 = omap[4]; g.ow0 = omap[5];
    TORCH_CHECK(g.osh >= 1 && g.osw >= 1 && g.oh0 >= 0 && g.ow0 >= 0 &&
                g.oh0 + g.osh * (g.P - 1) < g.oH && g.ow0 + g.osw * (g.Q - 1) < g.oW,
                "conv_fwd: omap writes outside the output");
    TORCH_CHECK(out.has_value() && out->defined(), "conv_fwd: omap requires an explicit output tensor");
    TORCH_CHECK(!stats.has_value() || !stats->defined(), "conv_fwd: omap does not support stats");
  }
  TORCH_CHECK(g.P > 0 && g.Q > 0, "conv_fwd: empty output");
  TORCH_CHECK((int64_t)g.N * g.H * g.W * g.C < (1LL << 31) && (int64_t)g.M * K < (1LL << 31),
              "conv_fwd: tensor too large for 32-bit indexing");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == K, "bias size mismatch");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  torch::Tensor resid_full;   // fallback of a half-resolution residual (kernels other than pw.hip)
  if (resid.has_value() && resid->defined()) {
    req(*resid, at::kBFloat16, "resid");
    if (resid_half) {
      TORCH_CHECK(!g.omap && g.P % 2 == 0 && g.Q % 2 == 0 &&
                      resid->numel() == (int64_t)g.N * (g.P / 2) * (g.Q / 2) * K,
                  "conv_fwd: a half-resolution residual must be [N, P/2, Q/2, K] with P, Q even and no omap");
    } else {
      TORCH_CHECK(resid->numel() == (g.omap ? (int64_t)g.N * g.oH * g.oW * K : (int64_t)g.M * K),
                  "resid size mismatch");
    }
    rp = resid->data_ptr();
  } else {
    TORCH_CHECK(!resid_half, "conv_fwd: resid_half without a residual");
  }
  float* sp = nullptr;
  if (stats.has_value() && stats->defined()) {
    req(*stats, at::kFloat, "stats");
    TORCH_CHECK(stats->numel() == 2 * K || stats->numel() == stat_len(K),
                "stats must hold 2*K floats (or the slotted stat_len(K))");
    g.stat_slots = stats->numel() == 2 * K ? 0 : zoo::kStatSlots;
    TORCH_CHECK(out_bf16, "stats require the bf16 output");
    sp = stats->data_ptr<float>();
  }
  BwdStats bs{nullptr, nullptr, nullptr, nullptr, nullptr};
  bs.resid_half = resid_half ? 1 : 0;
  if (bsums.has_value() && bsums->defined()) {
    req(*bsums, at::kFloat, "bn sums");
    TORCH_CHECK(bsums->numel() == 2 * K || bsums->numel() == stat_len(K),
                "bn sums must be [2*K] (or the slotted stat_len(K))");
    g.stat_slots = bsums->numel() == 2 * K ? 0 : zoo::kStatSlots;
    const int64_t full = g.omap ? (int64_t)g.N * g.oH * g.oW * K : (int64_t)g.M * K;
    const bool gelu = !(by.has_value() && by->defined());
    if (gelu) {
      // GELU-backward mode: bz = the GELU pre-activation of this GEMM's output, sums = column
      // sums of the scaled output (bias gradient of the producing linear)
      TORCH_CHECK(bz.has_value() && bz->defined(), "gelu-backward epilogue needs the pre-activation (bz)");
      TORCH_CHECK(bp == nullptr && act == 0, "gelu-backward epilogue: no bias / activation");
      bs.zgelu = 1;
    } else {
      TORCH_CHECK(bmean.has_value() && binv.has_value(), "fused bn-backward needs y/mean/inv");
      req(*by, at::kBFloat16, "bn y");
      req(*bmean, at::kFloat, "bn mean");
      req(*binv, at::kFloat, "bn inv");
      TORCH_CHECK(bmean->numel() == K && binv->numel() == K, "bn mean/inv must be [K]");
      TORCH_CHECK(by->numel() == full, "bn y must match the output");
      bs.y = by->data_ptr();
      bs.mean = bmean->data_ptr<float>();
      bs.inv = binv->data_ptr<float>();
    }
    if (bz.has_value() && bz->defined() && !gelu && bz->scalar_type() == at::kByte) {
      // producer ReLU as a bit mask (bn_fwd_apply mask): 1 bit per output element
      TORCH_CHECK(bz->is_cuda() && bz->is_contiguous() && bz->numel() * 8 == full,
                  "bn z bit mask must be a contiguous uint8 [numel/8] tensor");
      bs.z = bz->data_ptr();
      bs.zmode = 2;
    } else if (bz.has_value() && bz->defined()) {
      req(*bz, at::kBFloat16, "bn z");
      TORCH_CHECK(bz->numel() == full, "bn z must match the output");
      bs.z = bz->data_ptr();
    } else if (!gelu && bgamma.has_value() && bgamma->defined()) {
      // producer ReLU recomputed from y with its affine (no residual add in that unit)
      req(*bgamma, at::kFloat, "bn gamma");
      TORCH_CHECK(bgamma->numel() == K, "bn gamma must be [K]");
      bs.mgamma = bgamma->data_ptr<float>();
      if (bbeta.has_value() && bbeta->defined()) {
        req(*bbeta, at::kFloat, "bn beta");
        TORCH_CHECK(bbeta->numel() == K, "bn beta must be [K]");
        bs.mbeta = bbeta->data_ptr<float>();
      }
      bs.zmode = 1;
    }
    TORCH_CHECK(!stats.has_value() || !stats->defined(), "stats and fused bn-backward are exclusive");
    TORCH_CHECK(out_bf16 && !out_f32, "fused bn-backward needs the bf16 output");
    bs.sums = bsums->data_ptr<float>();
    if (by2.has_value() && by2->defined()) {
      // a second BatchNorm on the same gradient (fused projection shortcut): sums2 += sum out * y2
      TORCH_CHECK(!gelu && bsums2.has_value() && bsums2->defined(), "bn y2 needs the BN-backward epilogue and sums2");
      req(*by2, at::kBFloat16, "bn y2");
      req(*bsums2, at::kFloat, "bn sums2");
      TORCH_CHECK(by2->numel() == full && bsums2->numel() >= K, "bn y2 must match the output, sums2 [K]");
      bs.y2 = by2->data_ptr();
      bs.sums2 = bsums2->data_ptr<float>();
    }
  }
  bs.unbatched = 0;
  // BN-backward prologue: x is a unit's masked output gradient g; the GEMM operand is that unit's
  // BN backward dy = A g + B pro_y + Cc (pw.hip forms it in registers and writes pro_dy); kernels
  // without the prologue get dy materialised first (into pro_dy when given)
  torch::Tensor xin = x;
  // forward prologue of a residual unit: pro_y is its residual operand (pw.hip EPI 4), not a BN input
  c10::optional<torch::Tensor> pro_res;
  if (pro_fwd && pro_y.has_value() && pro_y->defined()) {
    pro_res = pro_y;
    pro_y = c10::nullopt;
  }
  if (pro_y.has_value() && pro_y->defined()) {
    req(*pro_y, at::kBFloat16, "pro_y");
    TORCH_CHECK(pro_coef.has_value() && pro_coef->defined(), "conv_fwd: the BN-backward prologue needs pro_coef");
    req(*pro_coef, at::kFloat, "pro_coef");
    TORCH_CHECK(pro_y->numel() == x.numel() && pro_coef->numel() == 3 * (int64_t)C,
                "conv_fwd: pro_y must match x, pro_coef must be [3 * C]");
    if (pro_dy.has_value() && pro_dy->defined()) {
      req(*pro_dy, at::kBFloat16, "pro_dy");
      TORCH_CHECK(pro_dy->numel() == x.numel(), "conv_fwd: pro_dy must match x");
      check_al16(pro_dy->data_ptr(), "pro_dy");
    }
    check_al16(pro_y->data_ptr(), "pro_y");
    // the prologue kernel is the backward-epilogue one: it computes no forward statistics
    TORCH_CHECK(!(stats.has_value() && stats->defined()), "conv_fwd: the BN-backward prologue takes no stats");
    bs.pro_y = pro_y->data_ptr();
    bs.pro_coef = pro_coef->data_ptr<float>();
    bs.pro_dy = opt_ptr<void>(pro_dy);
  }
  // forward consumer-side BN apply: x is a conv -> BN -> ReLU unit's pre-BN output y; the GEMM runs
  // on z = relu(coef[c] y + coef[2C + c]), which pw.hip forms in registers and writes to pro_dy
  if (pro_fwd) {
    TORCH_CHECK(!(pro_y.has_value() && pro_y->defined()), "conv_fwd: pro_fwd and pro_y are exclusive");
    TORCH_CHECK(pro_coef.has_value() && pro_coef->defined() && pro_dy.has_value() && pro_dy->defined(),
                "conv_fwd: pro_fwd needs pro_coef and pro_dy");
    req(*pro_coef, at::kFloat, "pro_coef");
    req(*pro_dy, at::kBFloat16, "pro_dy");
    TORCH_CHECK(pro_coef->numel() == 3 * (int64_t)C && pro_dy->numel() == x.numel(),
                "conv_fwd: pro_coef must be [3 * C], pro_dy must match x");
    check_al16(pro_dy->data_ptr(), "pro_dy");
    bs.pro_fwd = 1;
    bs.pro_coef = pro_coef->data_ptr<float>();
    bs.pro_dy = pro_dy->data_ptr();
    if (pro_res.has_value()) {
      req(*pro_res, at::kBFloat16, "pro_res");
      TORCH_CHECK(pro_res->numel() == x.numel(), "conv_fwd: the prologue residual must match x");
      check_al16(pro_res->data_ptr(), "pro_res");
      bs.pro_res = pro_res->data_ptr();
      if (pro_rcoef.has_value() && pro_rcoef->defined()) {
        req(*pro_rcoef, at::kFloat, "pro_rcoef");
        TORCH_CHECK(pro_rcoef->numel() == 3 * (int64_t)C, "conv_fwd: pro_rcoef must be [3 * C]");
        bs.pro_rcoef = pro_rcoef->data_ptr<float>();
      }
      if (pro_mask.has_value() && pro_mask->defined()) {
        TORCH_CHECK(pro_mask->scalar_type() == at::kByte && pro_mask->numel() * 8 == x.numel(),
                    "conv_fwd: pro_mask must be uint8 [x.numel() / 8]");
        bs.pro_mask = pro_mask->data_ptr();
      }
    }
  }
  // partial-buffer statistics: the kernel stores per-m-tile column sums into `part`, then
  // they are folded in order into the caller's buffer (its first 2K floats)
  float* const stat_dst = sp ? sp : bs.sums;
  torch::Tensor part;
  // m-tile height of the kernel the dispatcher picks (igemm.hip: 128; igemm2.hip: 128 or 256)
  const int epi = zoo::igemm_epi(out_bf16, out_f32, bp != nullptr, rp != nullptr, act, g.omap != 0,
                                 bs.sums != nullptr, sp != nullptr);
  const int route = zoo::igemm_route_epi(epi, bs.zgelu != 0);
  // persistent 3x3 kernel (c3.hip): one statistics row per workgroup
  const int c3_grid = zoo_c3_grid(&g, epi, &bs);
  const int i2_tm = c3_grid > 0 ? 0 : zoo_igemm2_tiles_m(&g, route);
  const int tiles_m = c3_grid > 0 ? c3_grid : i2_tm > 0 ? i2_tm : (g.M + 127) / 128;
  // few m-tiles (<= 512 adders per address, e.g. every 14x14 / 7x7 ResNet layer at b256):
  // the atomics go straight into the final 2K floats, no slot fold launch needed
  static const int slot_min_tiles = 512;
  if (g.stat_slots == zoo::kStatSlots && tiles_m <= slot_min_tiles) g.stat_slots = 0;
  // the persistent 1x1 kernel (pw.hip) adds each workgroup's sums once (~256 adders per address):
  // straight into the final 2K floats, no slot fold
  if (g.stat_slots > 0 && !stats_partial() && (zoo_pw_eligible(&g, route, &bs) || c3_grid > 0)) g.stat_slots = 0;
  if (stat_dst && stats_partial()) {
    part = torch::empty({(int64_t)tiles_m, 2 * (int64_t)K}, x.options().dtype(at::kFloat));
    g.stat_slots = zoo::kStatPartial;
    if (sp) sp = part.data_ptr<float>();
    else bs.sums = part.data_ptr<float>();
  }
  // the y2 sums run in pw.hip's epilogue; any other kernel gets them from one reduction pass over
  // its output afterwards. Decided before the prologue fallbacks below, so a y2 request never
  // costs a call its prologue (y2 is dropped first)
  bool y2_pass = false;
  if (bs.y2) {
    const void* y2p = bs.y2;
    bs.y2 = nullptr;
    const bool base_ok = zoo_pw_eligible(&g, route, &bs);
    bs.y2 = y2p;
    y2_pass = !(base_ok && zoo_pw_eligible(&g, route, &bs));
    if (y2_pass) {
      bs.y2 = nullptr;
      bs.sums2 = nullptr;
    }
  }
  // the prologue runs only in pw.hip; any other kernel (including pw with the deterministic
  // partial statistics decided above) gets dy materialised first
  if (bs.pro_y) {
    if (!zoo_pw_eligible(&g, route, &bs)) {
      xin = (pro_dy.has_value() && pro_dy->defined()) ? *pro_dy : torch::empty_like(x);
      check_hip(zoo_bnpro_apply(x.data_ptr(), pro_y->data_ptr(), bs.pro_coef, xin.data_ptr(), x.numel(), C, 0,
                                cur_stream()),
                "bnpro_apply");
      bs.pro_y = nullptr;
      bs.pro_coef = nullptr;
      bs.pro_dy = nullptr;
    }
  }
  if (bs.pro_res && !zoo_pw_eligible(&g, route, &bs)) {
    // the EPI 4 prologue runs only in pw.hip (e.g. not with deterministic partial statistics or
    // a shape pw does not take): materialise z and the unit's mask, then convolve z
    check_hip(zoo_bnres_apply(x.data_ptr(), bs.pro_coef, bs.pro_res, bs.pro_rcoef, pro_dy->data_ptr(), bs.pro_mask,
                              x.numel(), C, cur_stream()),
              "bnres_apply");
    xin = *pro_dy;
    bs.pro_fwd = 0;
    bs.pro_coef = nullptr;
    bs.pro_dy = nullptr;
    bs.pro_res = nullptr;
    bs.pro_rcoef = nullptr;
    bs.pro_mask = nullptr;
  }
  if (bs.pro_fwd && !zoo_pw_eligible(&g, route, &bs)) {
    // no prologue outside pw.hip: materialise z = relu(A y + Cc) into pro_dy and convolve that
    check_hip(zoo_bnpro_apply(x.data_ptr(), x.data_ptr(), bs.pro_coef, pro_dy->data_ptr(), x.numel(), C, 1,
                              cur_stream()),
              "bnpro_apply relu");
    xin = *pro_dy;
    bs.pro_fwd = 0;
    bs.pro_coef = nullptr;
    bs.pro_dy = nullptr;
  }
  if (bs.resid_half && !zoo_pw_eligible(&g, route, &bs)) {
    // only pw.hip reads the half-resolution residual: zero-interleave it to full size
    resid_full = torch::zeros({g.N, g.P, g.Q, K}, x.options());
    resid_full.view({g.N, g.P / 2, 2, g.Q / 2, 2, K}).select(4, 0).select(2, 0).copy_(
        resid->view({g.N, g.P / 2, g.Q / 2, K}));
    rp = resid_full.data_ptr();
    bs.resid_half = 0;
  }
  if (act_pre.has_value() && act_pre->defined()) {
    // training forward of a GELU linear / conv: the output gelu(v) AND the pre-activation v (its
    // backward's operand). The large-tile kernel stores both from its EPI 3 epilogue; any other
    // kernel writes v and one pointwise pass applies GELU (the round-5 path)
    req(*act_pre, at::kBFloat16, "act_pre");
    TORCH_CHECK(act == 2 /* ACT_GELU */ && out_bf16 && !out_f32 && !sp && !(out.has_value() && out->defined()) &&
                    act_pre->is_contiguous() && act_pre->numel() == (int64_t)g.N * g.P * g.Q * K,
                "conv_fwd: act_pre takes a plain GELU conv with a bf16 output of the same size");
    check_al16(act_pre->data_ptr(), "act_pre");
    const int epi3 = zoo::igemm_epi(true, false, bp != nullptr, rp != nullptr, act, g.omap != 0, bs.sums != nullptr,
                                    false);
    if (epi3 == 3 && zoo_igemm2_tiles_m(&g, 3) > 0) {
      bs.act_pre = act_pre->data_ptr();
    } else {
      check_hip(zoo_igemm(xin.data_ptr(), w.data_ptr(), act_pre->data_ptr(), nullptr, bp, rp, nullptr, &g, 0, &bs,
                          cur_stream()),
                "igemm");
      auto ya = torch::empty({g.N, g.P, g.Q, K}, x.options());
      check_hip(zoo_act(act_pre->data_ptr(), nullptr, ya.data_ptr(), ya.numel(), false, 4, 0.f, cur_stream()), "act");
      return ya;
    }
  }
  torch::Tensor y, yf;
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(out_bf16 && !out_f32, "conv_fwd: explicit output must be bf16");
    req(*out, at::kBFloat16, "out");
    TORCH_CHECK(out->dim() == 4 && out->size(0) == g.N && out->size(1) == g.oH && out->size(2) == g.oW &&
                    out->size(3) == K, "conv_fwd: explicit output shape mismatch");
    y = *out;
  } else {
    if (out_bf16) y = torch::empty({g.N, g.P, g.Q, K}, x.options());
  }
  if (out_f32) yf = torch::empty({g.N, g.P, g.Q, K}, x.options().dtype(at::kFloat));
  check_hip(zoo_igemm(xin.data_ptr(), w.data_ptr(), out_bf16 ? y.data_ptr() : nullptr,
                      out_f32 ? yf.data_ptr<float>() : nullptr, bp, rp, sp, &g, act, &bs, cur_stream()),
            "igemm");
  if (g.stat_slots == zoo::kStatPartial) fold_partials(stat_dst, part, 2 * K, tiles_m);
  else if (g.stat_slots > 0)
    check_hip(zoo_stats_finalize(stat_dst, 2 * K, g.stat_slots, cur_stream()), "stats_finalize");
  if (y2_pass) {
    auto zero = torch::zeros({K}, x.options().dtype(at::kFloat));
    auto one = torch::ones({K}, x.options().dtype(at::kFloat));
    auto tmp = torch::zeros({2 * (int64_t)K}, x.options().dtype(at::kFloat));
    bn_reduce(y, c10::nullopt, *by2, zero, one, tmp, 1);   // tmp[K..2K) = sum y * y2
    bsums2->narrow(0, 0, K).add_(tmp.narrow(0, K, K));
  }
  return out_bf16 ? y : yf;
}

// w: [K, ldw] packed rows of [R][S][C]; returns [C, ceil8(Ra*Sb*K)] flipped sub-filter
// Wt[c][t][u][k] = W[k][r0 + sh*(Ra-1-t)][s0 + sw*(Sb-1-u)][c]
torch::Tensor flip_weights(torch::Tensor w, int K, int R, int S, int C, int r0, int s0, int Ra, int Sb, int sh,
                           int sw) {
  req(w, at::kBFloat16, "w");
  TORCH_CHECK(w.dim() == 2 && w.size(0) == K && w.size(1) >= R * S * C, "flip_weights: w must be [K, >=R*S*C]");
  TORCH_CHECK(Ra >= 1 && Sb >= 1 && r0 >= 0 && s0 >= 0 && sh >= 1 && sw >= 1 && r0 + sh * (Ra - 1) < R &&
                  s0 + sw * (Sb - 1) < S, "flip_weights: sub-filter outside the filter");
  const int ldt = (Ra * Sb * K + 7) / 8 * 8;
  auto wt = (ldt == Ra * Sb * K) ? torch::empty({C, ldt}, w.options()) : torch::zeros({C, ldt}, w.options());
  check_hip(zoo_flip_weights(w.data_ptr(), wt.data_ptr(), K, R, S, C, (int)w.size(1), r0, s0, Ra, Sb, sh, sw, ldt,
                             cur_stream()),
            "flip_weights");
  return wt;
}

// Batched flip into preallocated outputs. `table` is a device int64 tensor of n rows x 16:
// (W ptr, Wt ptr, K, R, S, C, ldw, r0, s0, Ra, Sb, sh, sw, ldt, blk0, nblk), written by
// zoo.ops._kern.FlipCache from tensors it keeps alive and validated there with the same
// checks as flip_weights (every row was first produced by flip_weights for that geometry).
void flip_weights_batched(torch::Tensor table, int n, int nblocks) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kInt && table.is_contiguous() &&
                  table.numel() == (int64_t)n * (int64_t)(sizeof(zoo::FlipDesc) / sizeof(int)),
              "flip_weights_batched: table must be a contiguous int32 [n, sizeof(FlipDesc)/4] device tensor");
  check_hip(zoo_flip_weights_batched(table.data_ptr(), n, nblocks, cur_stream()), "flip_weights_batched");
}

int flip_desc_ints() { return (int)(sizeof(zoo::FlipDesc) / sizeof(int)); }

// C[b] = A[b] (M x K) * B[b]^T where B is given as [Bt, N, K]: any strides (views from
// transpose / expand), at least one of each operand's two inner dims contiguous.
torch::Tensor bmm_nt(torch::Tensor a, torch::Tensor b, bool out_bf16) {
  TORCH_CHECK(a.is_cuda() && b.is_cuda(), "bmm: GPU tensors expected");
  TORCH_CHECK(a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16, "bmm: bf16 operands");
  TORCH_CHECK(a.dim() == 3 && b.dim() == 3, "bmm: [B, M, K] x [B, N, K] expected");
  TORCH_CHECK(a.size(0) == b.size(0) && a.size(2) == b.size(2), "bmm: batch / K mismatch");
  const int64_t B = a.size(0), M = a.size(1), K = a.size(2), N = b.size(1);
  TORCH_CHECK(B < 65536 && M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "bmm: size out of range");
  TORCH_CHECK((a.stride(2) == 1 || a.stride(1) == 1 || M == 1) && (b.stride(2) == 1 || b.stride(1) == 1 || N == 1),
              "bmm: one inner dim of each operand must be contiguous");
  auto c = torch::empty({B, M, N}, a.options().dtype(out_bf16 ? at::kBFloat16 : at::kFloat));
  if (c.numel() == 0) return c;
  if (K == 0) return c.zero_();
  auto al16 = [](const torch::Tensor& t) {
    const bool kc = t.stride(2) == 1;
    const int64_t other = kc ? t.stride(1) : t.stride(2);
    return reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 && other % 8 == 0 && t.stride(0) % 8 == 0;
  };
  const int vec = al16(a) && al16(b) ? 1 : 0;
  // a row-contiguous operand with stride(2) == 1 too (size-1 dims) counts as k-contiguous
  const long geom[12] = {(long)B, (long)M, (long)N, (long)K, (long)a.stride(0), (long)a.stride(1),
                         (long)a.stride(2), (long)b.stride(0), (long)b.stride(1), (long)b.stride(2),
                         (long)c.stride(0), (long)c.stride(1)};
  check_hip(zoo_bmm(a.data_ptr(), b.data_ptr(), c.data_ptr(), geom, out_bf16 ? 1 : 0, vec, cur_stream()), "bmm");
  return c;
}

// reduce over the last (contiguous) dim: op 0 sum, 1 mean, 2 max, 3 min, 4 sum of squares
torch::Tensor row_reduce(torch::Tensor x, int64_t op) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() >= 1, "row_reduce: contiguous GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "row_reduce: fp32 or bf16");
  TORCH_CHECK(op >= 0 && op <= 4, "row_reduce: op");
  const int64_t cols = x.size(-1);
  TORCH_CHECK(cols > 0 && cols < (1LL << 31), "row_reduce: last dim size");
  auto sizes = x.sizes().vec();
  sizes.pop_back();
  auto out = torch::empty(sizes, x.options().dtype(at::kFloat));
  const int64_t rows = x.numel() / cols;
  if (rows == 0) return out;
  check_hip(zoo_row_reduce(x.data_ptr(), out.data_ptr<float>(), rows, (int)cols, x.scalar_type() == at::kFloat,
                           (int)op, cur_stream()), "row_reduce");
  return out;
}

// L2-normalise rows of the last dim (dy/y given: the backward)
torch::Tensor row_l2norm(torch::Tensor x, c10::optional<torch::Tensor> dy, c10::optional<torch::Tensor> y,
                         double eps) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() >= 1, "row_l2norm: contiguous GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "row_l2norm: fp32 or bf16");
  const bool bwd = dy.has_value() && dy->defined();
  if (bwd) {
    TORCH_CHECK(y.has_value() && y->defined(), "row_l2norm backward needs y");
    TORCH_CHECK(dy->sizes() == x.sizes() && y->sizes() == x.sizes() && dy->is_contiguous() && y->is_contiguous() &&
                    dy->scalar_type() == x.scalar_type() && y->scalar_type() == x.scalar_type(),
                "row_l2norm: dy / y must match x");
  }
  auto out = torch::empty_like(x);
  const int64_t cols = x.size(-1);
  const int64_t rows = cols ? x.numel() / cols : 0;
  if (rows == 0) return out;
  check_hip(zoo_row_l2norm(x.data_ptr(), bwd ? dy->data_ptr() : nullptr, bwd ? y->data_ptr() : nullptr,
                           out.data_ptr(), rows, (int)cols, x.scalar_type() == at::kFloat, (float)eps, cur_stream()),
            "row_l2norm");
  return out;
}

// Wide&Deep deep-tower input row: segments k = dense fp32 [B, w] blocks (id_cols[k] < 0) or
// embedding lookups of fp32 tables [V, D] at the float id in column id_cols[k] of ids [B, E]
static zoo::DeepSegs deep_segs(const torch::Tensor& ids, const std::vector<torch::Tensor>& srcs,
                               const std::vector<int64_t>& id_cols, const std::vector<torch::Tensor>* grads, int* W) {
  TORCH_CHECK(srcs.size() == id_cols.size() && srcs.size() <= (size_t)zoo::DI_MAX_SEG && !srcs.empty(),
              "deep_input: 1..8 segments, one id column entry each");
  const int64_t B = ids.size(0);
  zoo::DeepSegs sg{};
  sg.n = (int)srcs.size();
  int col = 0;
  for (size_t k = 0; k < srcs.size(); ++k) {
    const auto& t = srcs[k];
    req(t, at::kFloat, "deep_input segment");
    TORCH_CHECK(t.dim() == 2, "deep_input: 2-D segments");
    zoo::DeepSeg& d = sg.s[k];
    d.src = t.data_ptr<float>();
    d.col0 = col;
    d.width = (int)t.size(1);
    d.emb = id_cols[k] >= 0;
    d.gsrc = nullptr;
    if (d.emb) {
      TORCH_CHECK(id_cols[k] < ids.size(1), "deep_input: id column out of range");
      d.id_col = (int)id_cols[k];
      d.V = (int)t.size(0);
      d.ld = d.width;
      if (grads && (*grads)[k].defined() && (*grads)[k].numel()) {
        const auto& g = (*grads)[k];
        req(g, at::kFloat, "deep_input table gradient");
        TORCH_CHECK(g.sizes() == t.sizes(), "deep_input: table gradient shape");
        d.gsrc = g.data_ptr<float>();
      }
    } else {
      TORCH_CHECK(t.size(0) == B, "deep_input: dense segment batch");
      d.id_col = 0;
      d.V = 0;
      d.ld = (int)t.size(1);
    }
    col += d.width;
  }
  *W = col;
  return sg;
}

torch::Tensor deep_input_fwd(torch::Tensor ids, std::vector<torch::Tensor> srcs, std::vector<int64_t> id_cols) {
  req(ids, at::kFloat, "ids");
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) < (1 << 30), "deep_input: ids [B, E]");
  int W = 0;
  const zoo::DeepSegs sg = deep_segs(ids, srcs, id_cols, nullptr, &W);
  auto out = torch::empty({ids.size(0), (int64_t)W}, ids.options().dtype(at::kBFloat16));
  if (ids.size(0) && W)
    check_hip(zoo_deep_input(ids.data_ptr<float>(), (int)ids.size(1), &sg, out.data_ptr(), nullptr, (int)ids.size(0), W,
                             cur_stream()),
              "deep_input_fwd");
  return out;
}

void deep_input_bwd(torch::Tensor dout, torch::Tensor ids, std::vector<torch::Tensor> srcs, std::vector<int64_t> id_cols,
                    std::vector<torch::Tensor> grads) {
  req(ids, at::kFloat, "ids");
  req(dout, at::kBFloat16, "dout");
  TORCH_CHECK(grads.size() == srcs.size(), "deep_input_bwd: one gradient entry per segment");
  int W = 0;
  const zoo::DeepSegs sg = deep_segs(ids, srcs, id_cols, &grads, &W);
  TORCH_CHECK(dout.dim() == 2 && dout.size(0) == ids.size(0) && dout.size(1) == W, "deep_input_bwd: dout [B, W]");
  if (ids.size(0) && W)
    check_hip(zoo_deep_input(ids.data_ptr<float>(), (int)ids.size(1), &sg, nullptr, dout.data_ptr(), (int)ids.size(0),
                             W, cur_stream()),
              "deep_input_bwd");
}

// Wide&Deep head: softmax(wide + bias + deep) (fp32 probabilities [B, C], C <= 32)
torch::Tensor wnd_head_fwd(c10::optional<torch::Tensor> wide, c10::optional<torch::Tensor> deep,
                           c10::optional<torch::Tensor> bias) {
  const torch::Tensor* ref = wide.has_value() ? &*wide : (deep.has_value() ? &*deep : nullptr);
  TORCH_CHECK(ref != nullptr, "wnd_head: wide or deep input required");
  const int64_t B = ref->size(0), C = ref->size(1);
  TORCH_CHECK(C >= 1 && C <= 32 && B < (1 << 30), "wnd_head: 1..32 classes");
  if (wide.has_value()) {
    req(*wide, at::kFloat, "wide");
    TORCH_CHECK(wide->dim() == 2 && wide->size(0) == B && wide->size(1) == C, "wnd_head: wide [B, C]");
  }
  bool dbf = false;
  if (deep.has_value()) {
    TORCH_CHECK(deep->is_cuda() && deep->is_contiguous() && deep->dim() == 2 && deep->size(0) == B && deep->size(1) == C,
                "wnd_head: deep [B, C] contiguous");
    TORCH_CHECK(deep->scalar_type() == at::kFloat || deep->scalar_type() == at::kBFloat16, "wnd_head: deep fp32/bf16");
    dbf = deep->scalar_type() == at::kBFloat16;
  }
  if (bias.has_value()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == C, "wnd_head: bias [C]");
  }
  auto prob = torch::empty({B, C}, ref->options().dtype(at::kFloat));
  if (B)
    check_hip(zoo_wnd_head_fwd(wide.has_value() ? wide->data_ptr<float>() : nullptr,
                               deep.has_value() ? deep->data_ptr() : nullptr, dbf,
                               bias.has_value() ? bias->data_ptr<float>() : nullptr, prob.data_ptr<float>(), (int)B,
                               (int)C, cur_stream()),
              "wnd_head_fwd");
  return prob;
}

// backward: returns (dwide fp32 | empty, ddeep in deep_dtype | empty); gbias (fp32 [C]) += column sums
std::vector<torch::Tensor> wnd_head_bwd(torch::Tensor prob, torch::Tensor g, bool need_wide, bool need_deep,
                                        bool deep_bf16, c10::optional<torch::Tensor> gbias) {
  req(prob, at::kFloat, "prob");
  req(g, at::kFloat, "grad");
  TORCH_CHECK(prob.dim() == 2 && g.sizes() == prob.sizes() && prob.size(1) <= 32, "wnd_head_bwd: [B, C <= 32]");
  const int64_t B = prob.size(0), C = prob.size(1);
  torch::Tensor dw, dd, part;
  if (need_wide) dw = torch::empty_like(prob);
  if (need_deep) dd = torch::empty({B, C}, prob.options().dtype(deep_bf16 ? at::kBFloat16 : at::kFloat));
  if (gbias.has_value()) {
    req(*gbias, at::kFloat, "gbias");
    TORCH_CHECK(gbias->numel() == C, "wnd_head_bwd: gbias [C]");
    part = torch::empty({(int64_t)zoo_wnd_head_blocks((int)B) * C}, prob.options());
  }
  if (B)
    check_hip(zoo_wnd_head_bwd(prob.data_ptr<float>(), g.data_ptr<float>(), need_wide ? dw.data_ptr<float>() : nullptr,
                               need_deep ? dd.data_ptr() : nullptr, deep_bf16,
                               gbias.has_value() ? gbias->data_ptr<float>() : nullptr,
                               gbias.has_value() ? part.data_ptr<float>() : nullptr, (int)B, (int)C, cur_stream()),
              "wnd_head_bwd");
  return {need_wide ? dw : torch::Tensor(), need_deep ? dd : torch::Tensor()};
}

// SSD hard negative mining: ce [B, P] fp32 (per-prior confidence loss), conf_t [B, P] int64 ->
// uint8 [B, P] mask of positives | the ceil(ratio * #pos) hardest negatives per image
torch::Tensor ssd_mine(torch::Tensor ce, torch::Tensor conf_t, int64_t bg_label, double ratio) {
  req(ce, at::kFloat, "ce");
  TORCH_CHECK(conf_t.is_cuda() && conf_t.scalar_type() == at::kLong && conf_t.is_contiguous(), "ssd_mine: conf_t int64");
  TORCH_CHECK(ce.dim() == 2 && conf_t.sizes() == ce.sizes(), "ssd_mine: ce / conf_t [B, P]");
  const int64_t B = ce.size(0), P = ce.size(1);
  TORCH_CHECK(B < (1 << 30) && P < (1 << 30), "ssd_mine: sizes");
  auto sel = torch::empty({B, P}, ce.options().dtype(at::kByte));
  if (B == 0 || P == 0) return sel;
  check_hip(zoo_ssd_mine(ce.data_ptr<float>(), reinterpret_cast<const long long*>(conf_t.data_ptr()), (int)B, (int)P,
                         (int)bg_label, (float)ratio, sel.data_ptr<uint8_t>(), cur_stream()),
            "ssd_mine");
  return sel;
}

// NormalizeScale over the last dim: y = x / (||x|| + eps) * w (bf16 x / y, fp32 w); returns (y, norm [R])
std::vector<torch::Tensor> l2norm_scale_fwd(torch::Tensor x, torch::Tensor w, double eps) {
  req(x, at::kBFloat16, "x");
  req(w, at::kFloat, "w");
  const int64_t C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && w.numel() == C, "l2norm_scale: C % 8 == 0, w [C]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "l2norm_scale: aligned x");
  const int64_t R = x.numel() / C;
  auto y = torch::empty_like(x);
  auto rn = torch::empty({R}, x.options().dtype(at::kFloat));
  if (R) check_hip(zoo_l2norm_scale_fwd(x.data_ptr(), w.data_ptr<float>(), y.data_ptr(), rn.data_ptr<float>(), R,
                                        (int)C, (float)eps, cur_stream()),
                   "l2norm_scale_fwd");
  return {y, rn};
}

// backward: (dx bf16, dw fp32 [C])
std::vector<torch::Tensor> l2norm_scale_bwd(torch::Tensor dy, torch::Tensor x, torch::Tensor w, torch::Tensor rn,
                                            double eps) {
  req(dy, at::kBFloat16, "dy");
  req(x, at::kBFloat16, "x");
  req(w, at::kFloat, "w");
  req(rn, at::kFloat, "norm");
  const int64_t C = x.size(-1), R = x.numel() / C;
  TORCH_CHECK(dy.sizes() == x.sizes() && C % 8 == 0 && w.numel() == C && rn.numel() == R && C <= 4096,
              "l2norm_scale_bwd: shapes");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0,
              "l2norm_scale_bwd: aligned");
  auto dx = torch::empty_like(x);
  auto dw = torch::zeros({C}, w.options());
  if (R == 0) return {dx, dw};
  auto part = torch::empty({(int64_t)zoo_l2norm_scale_bwd_blocks(R) * C}, w.options());
  check_hip(zoo_l2norm_scale_bwd(dy.data_ptr(), x.data_ptr(), w.data_ptr<float>(), rn.data_ptr<float>(), dx.data_ptr(),
                                 dw.data_ptr<float>(), part.data_ptr<float>(), R, (int)C, (float)eps, cur_stream()),
            "l2norm_scale_bwd");
  return {dx, dw};
}

// SSD matching: gt [B, G, 5] (label, x1, y1, x2, y2), count [B] int32, priors [P, 4]
// centre-size -> (loc_t [B, P, 4] fp32, conf_t [B, P] int64)
std::vector<torch::Tensor> ssd_match(torch::Tensor gt, torch::Tensor count, torch::Tensor priors, double overlap,
                                     double v0, double v1, int64_t bg_label) {
  req(gt, at::kFloat, "gt");
  req(priors, at::kFloat, "priors");
  TORCH_CHECK(count.is_cuda() && count.scalar_type() == at::kInt && count.is_contiguous(), "ssd_match: count int32");
  TORCH_CHECK(gt.dim() == 3 && gt.size(2) == 5 && priors.dim() == 2 && priors.size(1) == 4,
              "ssd_match: gt [B, G, 5], priors [P, 4]");
  TORCH_CHECK(count.numel() == gt.size(0), "ssd_match: count per image");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(priors.data_ptr()) % 16 == 0, "ssd_match: aligned priors");
  const int B = gt.size(0), G = gt.size(1), P = priors.size(0);
  TORCH_CHECK(B < 65536 && G < (1 << 20) && P < (1 << 30), "ssd_match: sizes");
  auto o = gt.options();
  auto loc_t = torch::empty({B, P, 4}, o);
  auto conf_t = torch::empty({B, P}, o.dtype(at::kLong));
  if (B == 0 || P == 0) return {loc_t, conf_t};
  auto best_gt = torch::empty({B, P}, o.dtype(at::kInt));
  auto best_iou = torch::empty({B, P}, o);
  auto gt_best = torch::empty({B, std::max(G, 1)}, o.dtype(at::kLong));
  check_hip(zoo_ssd_match(gt.data_ptr<float>(), count.data_ptr<int>(), priors.data_ptr<float>(), B, G, P,
                          (float)overlap, (float)v0, (float)v1, (int)bg_label, best_gt.data_ptr<int>(),
                          best_iou.data_ptr<float>(), reinterpret_cast<unsigned long long*>(gt_best.data_ptr()),
                          loc_t.data_ptr<float>(), reinterpret_cast<long long*>(conf_t.data_ptr()), cur_stream()),
            "ssd_match");
  return {loc_t, conf_t};
}

void linear_wgrad(torch::Tensor dy, torch::Tensor x, torch::Tensor dw);
static void check_al16(const void* p, const char* what);

// dW (fp32, [K, ldw]) += wgrad(x, dy)
void conv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, int R, int S, int sh, int sw, int ph, int pw,
                int dh, int dil_w) {
  req(x, at::kBFloat16, "x");
  req(dy, at::kBFloat16, "dy");
  req(dw, at::kFloat, "dw");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4, "conv_wgrad: NHWC inputs expected");
  WgradGeom g;
  g.N = x.size(0); g.H = x.size(1); g.W = x.size(2); g.C = x.size(3);
  g.K = dy.size(3); g.R = R; g.S = S; g.P = dy.size(1); g.Q = dy.size(2);
  g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw; g.dh = dh; g.dw = dil_w;
  TORCH_CHECK(dy.size(0) == g.N, "conv_wgrad: batch mismatch");
  TORCH_CHECK(g.C == 4 || g.C % 8 == 0, "conv_wgrad: C must be 4 or a multiple of 8");
  TORCH_CHECK(g.K % 8 == 0, "conv_wgrad: K must be a multiple of 8");
  const int P = (g.H + 2 * ph - dh * (R - 1) - 1) / sh + 1, Q = (g.W + 2 * pw - dil_w * (S - 1) - 1) / sw + 1;
  TORCH_CHECK(P == g.P && Q == g.Q, "conv_wgrad: dy spatial shape does not match the geometry");
  // conv weight gradients: the wgrad256 split target of conv calls (zoo_wgrad256_target), for the
  // duration of this call
  static const int conv_wg = 128;
  struct TargetGuard {
    explicit TargetGuard(int t) { zoo_wgrad256_target(t); }
    ~TargetGuard() { zoo_wgrad256_target(0); }
  } tguard(conv_wg);
  g.M = g.N * g.P * g.Q;
  g.Ktot = R * S * g.C;
  g.ldw = dw.size(-1);
  TORCH_CHECK(dw.dim() == 2 && dw.size(0) == g.K && g.ldw >= g.Ktot, "conv_wgrad: dw must be [K, >=R*S*C]");
  // the 64-output-channel stride-1 shapes of ResNet stage 1, the space-to-depth stem and (operands
  // swapped) the 1x1 64 -> 256 convs of stage 1: one workgroup per CU owns all of dW and walks
  // bands of output rows staged once in LDS
  // (wgrad.hip wgrad_band_kernel); deterministic ordered fold of the per-workgroup partials
  if (x.is_contiguous() && dy.is_contiguous() && dw.stride(1) == 1) {
    const int rows = zoo_wgrad_band(&g, nullptr, nullptr, nullptr, nullptr, nullptr);
    if (rows > 0) {
      check_al16(x.data_ptr(), "conv_wgrad x");
      check_al16(dy.data_ptr(), "conv_wgrad dy");
      auto part = torch::empty({(int64_t)rows, (int64_t)g.K * g.Ktot}, dw.options());
      zoo_wgrad_band(&g, x.data_ptr(), dy.data_ptr(), dw.data_ptr<float>(), part.data_ptr<float>(), cur_stream());
      check_hip(hipGetLastError(), "wgrad_band");
      return;
    }
  }
  // 1x1 stride-1 convs with >= 128 input and output channels (and up to 2^20 pixels) are plain
  // GEMMs where the 256x256-tile kernel (wgrad256.hip) beats the implicit-GEMM wgrad
  // (tools/wgrad_bench.py --resnet: 1.1-1.6x). At 802816 pixels (the stage-1 1x1 convs) the
  // 128-row tiles win in isolation, but inside the training step -- on the side stream beside
  // the data-gradient chain -- the 256-wide kernel wins: +0.3-0.45 % images/s over five same-box
  // pairs (profiles/r5/ab_wgrad256_mmax_r5.log), so the limit is 2^20 since round 5
  constexpr bool use256 = true;
  static const long long m_max = (1LL << 20);
  static const int c_min = 128;
  if (use256 && R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && g.K >= c_min && g.C >= c_min &&
      g.M <= m_max &&
      x.is_contiguous() && dy.is_contiguous() && dw.stride(1) == 1) {
    linear_wgrad(dy.view({(int64_t)g.M, g.K}), x.view({(int64_t)g.M, g.C}), dw);
    return;
  }
  // other convs with >= ZOO_WGRAD256_CONV_COUT output channels (3x3, strided 1x1): the same
  // 256x256-tile kernel with the im2col X operand gathered by its LDS-DMA (tools/wgrad_bench.py
  // --conv); narrower outputs waste most of its 256-row tile and stay on wgrad.hip
  static const int conv256_cout = 256;
  if (use256 && conv256_cout > 0 && g.K >= conv256_cout && g.C % 8 == 0 && x.is_contiguous() &&
      dy.is_contiguous() && dw.stride(1) == 1 && (int64_t)g.M * g.K < (1LL << 31) &&
      (int64_t)g.N * g.H * g.W * g.C < (1LL << 40)) {
    check_al16(x.data_ptr(), "conv_wgrad x");
    check_al16(dy.data_ptr(), "conv_wgrad dy");
    zoo_wgrad256_set_atomic(wgrad_partial() ? 0 : 1);   // atomics split-K unless deterministic
    const size_t pf = zoo_wgrad256_part_floats(g.M, g.K, g.Ktot);
    torch::Tensor part;
    if (pf) part = torch::empty({(int64_t)pf}, dw.options());
    check_hip(zoo_wgrad256_conv(dy.data_ptr(), x.data_ptr(), dw.data_ptr<float>(), pf ? part.data_ptr<float>() : nullptr,
                                g.N, g.H, g.W, g.C, g.K, R, S, g.P, g.Q, sh, sw, ph, pw, dh, dil_w, g.ldw, cur_stream()),
              "wgrad256_conv");
    return;
  }
  g.m_per_split = 0;
  // split-K reduction: fp32 atomics into dW, or per-split partials + an ordered fold. Atomics
  // run at ~1.3 TB/s of added bytes, plain stores + the fold's reads at ~5 TB/s: the partials
  // win once the split output is larger than ~ZOO_WGRAD_PARTIAL_MB (and are always used in
  // deterministic mode)
  static const double auto_mb = 16.0;
  torch::Tensor part;
  {
    WgradGeom gp = g;
    const int splits = zoo_wgrad_plan(&gp);
    const double mb = (double)splits * g.K * g.Ktot * 4 / 1e6;
    if (splits > 1 && (wgrad_partial() || (auto_mb > 0 && mb >= auto_mb))) {
      const int groups = (splits + 15) / 16;
      const int64_t extra = splits > 16 ? (int64_t)groups : 0;  // level-1 fold scratch
      part = torch::empty({(int64_t)splits + extra, (int64_t)g.K * g.Ktot}, dw.options());
    }
  }
  check_hip(zoo_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr<float>(), part.defined() ? part.data_ptr<float>() : nullptr,
                      &g, cur_stream()),
            "wgrad");
}

// dW (fp32 [N, >=K], row stride dw.stride(0)) += dy[M, N]^T x[M, K] on the 256x256-tile
// LDS-DMA + transposed-read kernel (wgrad256.hip); linear layers and 1x1 stride-1 convs
void linear_wgrad(torch::Tensor dy, torch::Tensor x, torch::Tensor dw) {
  TORCH_CHECK(dy.is_cuda() && x.is_cuda() && dw.is_cuda(), "linear_wgrad: GPU tensors expected");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && x.scalar_type() == at::kBFloat16, "linear_wgrad: bf16 dy / x");
  TORCH_CHECK(dw.scalar_type() == at::kFloat, "linear_wgrad: fp32 dw");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dw.dim() == 2, "linear_wgrad: 2-D tensors expected");
  TORCH_CHECK(dy.stride(1) == 1 && x.stride(1) == 1 && dw.stride(1) == 1, "linear_wgrad: rows must be contiguous");
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(x.size(0) == M, "linear_wgrad: dy / x row count differs");
  TORCH_CHECK(dw.size(0) == N && dw.size(1) >= K, "linear_wgrad: dw must be [N, >=K]");
  TORCH_CHECK(N % 8 == 0 && K % 8 == 0 && dy.stride(0) % 8 == 0 && x.stride(0) % 8 == 0,
              "linear_wgrad: N, K and leading dims must be multiples of 8");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0,
              "linear_wgrad: 16-byte aligned operands expected");
  TORCH_CHECK(M < (1LL << 31) && N < (1 << 30) && K < (1 << 30) && M * dy.stride(0) < (1LL << 40),
              "linear_wgrad: size out of range");
  if (M == 0 || N == 0 || K == 0) return;
  zoo_wgrad256_set_atomic(wgrad_partial() ? 0 : 1);     // atomics split-K unless deterministic
  const size_t pf = zoo_wgrad256_part_floats((int)M, (int)N, (int)K);
  torch::Tensor part;
  if (pf) part = torch::empty({(int64_t)pf}, dw.options());
  check_hip(zoo_wgrad256(dy.data_ptr(), x.data_ptr(), dw.data_ptr<float>(), pf ? part.data_ptr<float>() : nullptr,
                         (int)M, (int)N, (int)K, (int)dy.stride(0), (int)x.stride(0), (int)dw.stride(0), cur_stream()),
            "linear_wgrad");
}

static void check_al16(const void* p, const char* what) {
  TORCH_CHECK((reinterpret_cast<uintptr_t>(p) & 15) == 0, what, " must be 16-byte aligned");
}

void bn_reduce(torch::Tensor a, c10::optional<torch::Tensor> z, c10::optional<torch::Tensor> x,
               c10::optional<torch::Tensor> mean, c10::optional<torch::Tensor> invstd, torch::Tensor out, int mode) {
  req(a, at::kBFloat16, "a");
  req(out, at::kFloat, "out");
  const int C = a.size(-1);
  const int64_t M = a.numel() / C;
  TORCH_CHECK(C % 8 == 0, "bn_reduce: C must be a multiple of 8");
  TORCH_CHECK(out.numel() == 2 * C || out.numel() == stat_len(C), "bn_reduce: out must be [2*C] or stat_len(C)");
  int nslot = out.numel() == 2 * C ? 0 : zoo::kStatSlots;
  if (mode == 1) {
    TORCH_CHECK(x.has_value() && mean.has_value() && invstd.has_value(), "bn_reduce mode 1 needs x/mean/invstd");
    req(*x, at::kBFloat16, "x");
    TORCH_CHECK(x->numel() == a.numel(), "bn_reduce: x shape");
    if (z.has_value() && z->defined()) {
      req(*z, at::kBFloat16, "z");
      TORCH_CHECK(z->numel() == a.numel(), "bn_reduce: z shape");
    }
  }
  if (mode == 1) {
    check_al16(opt_ptr<float>(mean), "mean");
    check_al16(opt_ptr<float>(invstd), "invstd");
  }
  float* dst = out.data_ptr<float>();
  torch::Tensor part;
  int blocks = 0;
  if (stats_partial()) {
    blocks = zoo_bn_reduce_blocks((int)M, C);
    part = torch::empty({(int64_t)blocks, 2 * (int64_t)C}, out.options());
    dst = part.data_ptr<float>();
    nslot = zoo::kStatPartial;
  }
  check_hip(zoo_bn_reduce(a.data_ptr(), opt_ptr<void>(z), opt_ptr<void>(x), opt_ptr<float>(mean),
                          opt_ptr<float>(invstd), dst, (int)M, C, mode, nslot, cur_stream()),
            "bn_reduce");
  if (nslot == zoo::kStatPartial) fold_partials(out.data_ptr<float>(), part, 2 * C, blocks);
}

torch::Tensor bn_fwd_apply(torch::Tensor x, torch::Tensor stats, c10::optional<torch::Tensor> gamma,
                           c10::optional<torch::Tensor> beta, c10::optional<torch::Tensor> resid,
                           c10::optional<torch::Tensor> rmean, c10::optional<torch::Tensor> rvar,
                           torch::Tensor smean, torch::Tensor sinv, double eps, double momentum, bool relu,
                           bool training, std::vector<c10::optional<torch::Tensor>> resid_bn,
                           c10::optional<torch::Tensor> mask) {
  req(x, at::kBFloat16, "x");
  const int C = x.size(-1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0, "bn: C must be a multiple of 8");
  req(smean, at::kFloat, "save_mean");
  req(sinv, at::kFloat, "save_invstd");
  TORCH_CHECK(smean.numel() == C && sinv.numel() == C, "bn: save buffers must be [C]");
  if (training) {
    req(stats, at::kFloat, "stats");
    TORCH_CHECK(stats.numel() >= 2 * C, "bn: stats must hold [2*C]");
  } else {
    TORCH_CHECK(rmean.has_value() && rvar.has_value(), "bn eval needs running stats");
  }
  if (resid.has_value() && resid->defined()) {
    req(*resid, at::kBFloat16, "resid");
    TORCH_CHECK(resid->numel() == x.numel(), "bn: resid shape");
  }
  // the apply kernels read per-channel vectors with 16-byte loads
  check_al16(training ? stats.data_ptr<float>() : nullptr, "stats");
  check_al16(opt_ptr<float>(gamma), "gamma");
  check_al16(opt_ptr<float>(beta), "beta");
  check_al16(opt_ptr<float>(rmean), "running_mean");
  check_al16(opt_ptr<float>(rvar), "running_var");
  // resid_bn: [stats, gamma, beta, running_mean, running_var, save_mean, save_invstd] of the
  // BatchNorm applied to `resid` (the raw shortcut conv output) inside this pass; empty: none
  const void* r2[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (!resid_bn.empty()) {
    TORCH_CHECK(training && resid_bn.size() == 7, "bn: resid_bn needs 7 entries (training only)");
    TORCH_CHECK(resid.has_value() && resid->defined(), "bn: resid_bn without resid");
    const int64_t need[7] = {2 * (int64_t)C, C, C, C, C, C, C};
    for (int i = 0; i < 7; ++i) {
      auto& t = resid_bn[i];
      if (!t.has_value() || !t->defined()) {
        TORCH_CHECK(i == 1 || i == 2 || i == 3 || i == 4, "bn: resid_bn stats/save buffers are required");
        continue;
      }
      req(*t, at::kFloat, "resid_bn");
      TORCH_CHECK(t->is_contiguous() && t->numel() >= need[i], "bn: resid_bn buffer size");
      check_al16(t->data_ptr<float>(), "resid_bn");
      r2[i] = t->data_ptr();
    }
  }
  // mask: [M*C/8] uint8 ReLU bit mask of the pre-ReLU sign (BwdStats.zmode 2 consumers)
  void* mp = nullptr;
  if (mask.has_value() && mask->defined()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == M * C / 8, "bn: mask must be a contiguous uint8 [M*C/8] tensor");
    mp = mask->data_ptr();
  }
  auto y = torch::empty_like(x);
  check_hip(zoo_bn_fwd_apply(x.data_ptr(), training ? stats.data_ptr<float>() : nullptr, opt_ptr<float>(gamma),
                             opt_ptr<float>(beta), opt_ptr<void>(resid), y.data_ptr(), opt_ptr<float>(rmean),
                             opt_ptr<float>(rvar), smean.data_ptr<float>(), sinv.data_ptr<float>(), (int)M, C,
                             (float)eps, (float)momentum, relu, training, resid_bn.empty() ? nullptr : r2, mp,
                             cur_stream()),
            "bn_fwd_apply");
  return y;
}

std::vector<torch::Tensor> bn_bwd_apply(torch::Tensor dz, c10::optional<torch::Tensor> z, torch::Tensor x,
                                        torch::Tensor smean, torch::Tensor sinv, c10::optional<torch::Tensor> gamma,
                                        torch::Tensor sums, bool want_dresid, c10::optional<torch::Tensor> dgamma,
                                        c10::optional<torch::Tensor> dbeta) {
  req(dz, at::kBFloat16, "dz");
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(dz.numel() == x.numel(), "bn_bwd: shape mismatch");
  const int C = x.size(-1);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0, "bn_bwd: C must be a multiple of 8");
  req(sums, at::kFloat, "sums");
  TORCH_CHECK(sums.numel() >= 2 * C, "bn_bwd: sums must hold [2*C]");
  if (z.has_value() && z->defined()) {
    req(*z, at::kBFloat16, "z");
    TORCH_CHECK(z->numel() == x.numel(), "bn_bwd: z shape");
  }
  check_al16(sums.data_ptr<float>(), "sums");
  check_al16(smean.data_ptr<float>(), "save_mean");
  check_al16(sinv.data_ptr<float>(), "save_invstd");
  check_al16(opt_ptr<float>(gamma), "gamma");
  auto dx = torch::empty_like(x);
  torch::Tensor dr;
  if (want_dresid) dr = torch::empty_like(x);
  check_hip(zoo_bn_bwd_apply(dz.data_ptr(), opt_ptr<void>(z), x.data_ptr(), smean.data_ptr<float>(),
                             sinv.data_ptr<float>(), opt_ptr<float>(gamma), sums.data_ptr<float>(), dx.data_ptr(),
                             want_dresid ? dr.data_ptr() : nullptr, opt_ptr<float>(dgamma), opt_ptr<float>(dbeta),
                             (int)M, C, cur_stream()),
            "bn_bwd_apply");
  if (want_dresid) return {dx, dr};
  return {dx};
}

std::vector<torch::Tensor> maxpool_fwd(torch::Tensor x, int R, int S, int sh, int sw, int ph, int pw, bool save_arg,
                                       bool ceil_mode) {
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "maxpool: NHWC with C%8==0");
  TORCH_CHECK(R * S <= 256, "maxpool: window too large");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = pool_out(H, R, sh, ph, ceil_mode), Q = pool_out(W, S, sw, pw, ceil_mode);
  TORCH_CHECK(P > 0 && Q > 0, "maxpool: empty output");
  TORCH_CHECK((int64_t)N * H * W * C < (1LL << 31) && (int64_t)N * P * Q * C < (1LL << 31),
              "maxpool: tensor too large for 32-bit indexing");
  auto y = torch::empty({N, P, Q, C}, x.options());
  torch::Tensor arg;
  if (save_arg) arg = torch::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  check_hip(zoo_maxpool_fwd(x.data_ptr(), y.data_ptr(), save_arg ? arg.data_ptr() : nullptr, N, H, W, C, P, Q, R, S,
                            sh, sw, ph, pw, cur_stream()),
            "maxpool_fwd");
  if (save_arg) return {y, arg};
  return {y};
}

torch::Tensor maxpool_bwd(torch::Tensor dy, torch::Tensor arg, int H, int W, int R, int S, int sh, int sw, int ph,
                          int pw) {
  req(dy, at::kBFloat16, "dy");
  req(arg, at::kByte, "arg");
  TORCH_CHECK(dy.sizes() == arg.sizes(), "maxpool_bwd: arg shape");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  TORCH_CHECK((P == pool_out(H, R, sh, ph, false) || P == pool_out(H, R, sh, ph, true)) &&
                  (Q == pool_out(W, S, sw, pw, false) || Q == pool_out(W, S, sw, pw, true)),
              "maxpool_bwd: geometry");
  TORCH_CHECK((int64_t)N * H * W * C < (1LL << 31) && (int64_t)N * P * Q * C < (1LL << 31),
              "maxpool_bwd: tensor too large for 32-bit indexing");
  auto dx = torch::empty({N, H, W, C}, dy.options());
  check_hip(zoo_maxpool_bwd(dy.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, H, W, C, P, Q, R, S, sh, sw, ph, pw,
                            cur_stream()),
            "maxpool_bwd");
  return dx;
}


// Fused BatchNorm(training stats) -> ReLU -> max-pool over a raw conv output x [N,H,W,C]
// (ResNet stem). Returns {pooled, raw winner, tap}; see bn_relu_maxpool_fwd_kernel.
static void check_stem_pool(const torch::Tensor& x, int R, int S, int ph, int pw) {
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "bn_relu_maxpool: NHWC with C%8==0");
  const int cpr = x.size(3) / 8;
  TORCH_CHECK((cpr & (cpr - 1)) == 0 && cpr <= 256, "bn_relu_maxpool: C/8 must be a power of two <= 256");
  TORCH_CHECK(R * S < 255 && 2 * ph < R + 1 && 2 * pw < S + 1, "bn_relu_maxpool: window/padding");
  TORCH_CHECK(x.numel() < (1LL << 31), "bn_relu_maxpool: tensor too large for 32-bit indexing");
}

std::vector<torch::Tensor> bn_relu_maxpool_fwd(torch::Tensor x, torch::Tensor stats, torch::Tensor gamma,
                                               torch::Tensor beta, torch::Tensor rmean, torch::Tensor rvar,
                                               torch::Tensor smean, torch::Tensor sinv, double eps, double momentum,
                                               int R, int S, int sh, int sw, int ph, int pw) {
  check_stem_pool(x, R, S, ph, pw);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  for (auto* t : {&stats, &gamma, &beta, &rmean, &rvar, &smean, &sinv}) req(*t, at::kFloat, "bn vector");
  TORCH_CHECK(stats.numel() >= 2 * C && gamma.numel() == C && beta.numel() == C && rmean.numel() == C &&
                  rvar.numel() == C && smean.numel() == C && sinv.numel() == C, "bn_relu_maxpool: vector sizes");
  const int P = pool_out(H, R, sh, ph, false), Q = pool_out(W, S, sw, pw, false);
  TORCH_CHECK(P > 0 && Q > 0, "bn_relu_maxpool: empty output");
  auto y = torch::empty({N, P, Q, C}, x.options());
  auto best = torch::empty({N, P, Q, C}, x.options());
  auto arg = torch::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  check_hip(zoo_bn_relu_maxpool_fwd(x.data_ptr(), stats.data_ptr<float>(), gamma.data_ptr<float>(),
                                    beta.data_ptr<float>(), y.data_ptr(), best.data_ptr(), arg.data_ptr(),
                                    rmean.data_ptr<float>(), rvar.data_ptr<float>(), smean.data_ptr<float>(),
                                    sinv.data_ptr<float>(), (float)eps, (float)momentum, N, H, W, C, P, Q, R, S, sh,
                                    sw, ph, pw, cur_stream()),
            "bn_relu_maxpool_fwd");
  return {y, best, arg};
}

// backward of bn_relu_maxpool_fwd: sums (>= 2C fp32, zeroed by the caller) receive
// (sum dz, sum dz*xhat); dgamma/dbeta (optional) += them; returns dx [N,H,W,C]
torch::Tensor bn_relu_maxpool_bwd(torch::Tensor dy, torch::Tensor best, torch::Tensor arg, torch::Tensor x,
                                  torch::Tensor smean, torch::Tensor sinv, torch::Tensor gamma, torch::Tensor sums,
                                  c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta, int R,
                                  int S, int sh, int sw, int ph, int pw) {
  check_stem_pool(x, R, S, ph, pw);
  req(dy, at::kBFloat16, "dy");
  req(best, at::kBFloat16, "best");
  req(arg, at::kByte, "arg");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = pool_out(H, R, sh, ph, false), Q = pool_out(W, S, sw, pw, false);
  const std::vector<int64_t> pshape{N, P, Q, C};
  TORCH_CHECK(dy.sizes() == pshape && best.sizes() == pshape && arg.sizes() == pshape,
              "bn_relu_maxpool_bwd: pooled tensors must be [N,P,Q,C]");
  for (auto* t : {&smean, &sinv, &gamma, &sums}) req(*t, at::kFloat, "bn vector");
  TORCH_CHECK(smean.numel() == C && sinv.numel() == C && gamma.numel() == C && sums.numel() >= 2 * C,
              "bn_relu_maxpool_bwd: vector sizes");
  if (dgamma.has_value()) TORCH_CHECK(dgamma->numel() == C && dgamma->scalar_type() == at::kFloat, "dgamma");
  if (dbeta.has_value()) TORCH_CHECK(dbeta->numel() == C && dbeta->scalar_type() == at::kFloat, "dbeta");
  auto dx = torch::empty_like(x);
  check_hip(zoo_bn_relu_maxpool_bwd(dy.data_ptr(), best.data_ptr(), arg.data_ptr(), x.data_ptr(),
                                    smean.data_ptr<float>(), sinv.data_ptr<float>(), gamma.data_ptr<float>(),
                                    sums.data_ptr<float>(), dx.data_ptr(), opt_ptr<float>(dgamma),
                                    opt_ptr<float>(dbeta), N, H, W, C, P, Q, R, S, sh, sw, ph, pw, cur_stream()),
            "bn_relu_maxpool_bwd");
  return dx;
}

std::vector<int64_t> pool_shape(int H, int W, int R, int S, int sh, int sw, int ph, int pw, bool ceil_mode) {
  return {pool_out(H, R, sh, ph, ceil_mode), pool_out(W, S, sw, pw, ceil_mode)};
}

torch::Tensor avgpool_fwd(torch::Tensor x, int R, int S, int sh, int sw, int ph, int pw, bool ceil_mode,
                          bool count_include_pad) {
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "avgpool: NHWC with C%8==0");
  TORCH_CHECK(R >= 1 && S >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0 && ph * 2 <= R && pw * 2 <= S,
              "avgpool: bad geometry");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = pool_out(H, R, sh, ph, ceil_mode), Q = pool_out(W, S, sw, pw, ceil_mode);
  TORCH_CHECK(P > 0 && Q > 0, "avgpool: empty output");
  auto y = torch::empty({N, P, Q, C}, x.options());
  check_hip(zoo_avgpool_fwd(x.data_ptr(), y.data_ptr(), N, H, W, C, P, Q, R, S, sh, sw, ph, pw, count_include_pad,
                            cur_stream()),
            "avgpool_fwd");
  return y;
}

torch::Tensor avgpool_bwd(torch::Tensor dy, int H, int W, int R, int S, int sh, int sw, int ph, int pw,
                          bool count_include_pad) {
  req(dy, at::kBFloat16, "dy");
  TORCH_CHECK(dy.dim() == 4 && dy.size(3) % 8 == 0, "avgpool_bwd: NHWC with C%8==0");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  TORCH_CHECK((P - 1) * sh - ph < H && (Q - 1) * sw - pw < W, "avgpool_bwd: geometry");
  auto dx = torch::empty({N, H, W, C}, dy.options());
  check_hip(zoo_avgpool_bwd(dy.data_ptr(), dx.data_ptr(), N, H, W, C, P, Q, R, S, sh, sw, ph, pw, count_include_pad,
                            cur_stream()),
            "avgpool_bwd");
  return dx;
}

// grouped conv (gconv.hip): x [N,H,W,C] bf16 NHWC, w [K, ldb] bf16 packed per output channel over
// its group's (r, s, c) with C / groups channels, group g = output rows [g K/g, (g+1) K/g)
static GConvArgs gconv_args(int N, int H, int W, int C, int K, int groups, int R, int S, int sh, int sw, int ph,
                            int pw, int dh, int dw, int ldb, int act) {
  TORCH_CHECK(groups >= 1 && C % groups == 0 && K % groups == 0, "grouped conv: channels must split into groups");
  TORCH_CHECK(R >= 1 && S >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0 && dh >= 1 && dw >= 1,
              "grouped conv: bad geometry");
  GConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.K = K; a.groups = groups; a.Cg = C / groups; a.Kg = K / groups;
  a.R = R; a.S = S; a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw; a.dh = dh; a.dw = dw;
  a.P = (H + 2 * ph - dh * (R - 1) - 1) / sh + 1;
  a.Q = (W + 2 * pw - dw * (S - 1) - 1) / sw + 1;
  TORCH_CHECK(a.P > 0 && a.Q > 0, "grouped conv: empty output");
  TORCH_CHECK(ldb >= R * S * a.Cg && ldb % 8 == 0, "grouped conv: weight rows must be >= R*S*C/groups, %8 == 0");
  a.ldb = ldb; a.act = act;
  return a;
}

torch::Tensor gconv_fwd(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, int groups, int R,
                        int S, int sh, int sw, int ph, int pw, int dh, int dil_w, int act) {
  req(x, at::kBFloat16, "x");
  req(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2, "gconv_fwd: x NHWC, w [K, ldb]");
  const int K = w.size(0);
  auto a = gconv_args(x.size(0), x.size(1), x.size(2), x.size(3), K, groups, R, S, sh, sw, ph, pw, dh, dil_w,
                      w.size(1), act);
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == K, "gconv_fwd: bias size");
    bp = bias->data_ptr<float>();
  }
  if (a.Cg % 8 == 0) check_al16(x.data_ptr(), "gconv_fwd x");
  check_al16(w.data_ptr(), "gconv_fwd w");
  auto y = torch::empty({x.size(0), a.P, a.Q, K}, x.options());
  check_hip(zoo_gconv(0, x.data_ptr(), w.data_ptr(), nullptr, y.data_ptr(), bp, &a, cur_stream()), "gconv_fwd");
  return y;
}

torch::Tensor gconv_dgrad(torch::Tensor dy, torch::Tensor w, int groups, int H, int W, int C, int R, int S, int sh,
                          int sw, int ph, int pw, int dh, int dil_w) {
  req(dy, at::kBFloat16, "dy");
  req(w, at::kBFloat16, "w");
  const int K = w.size(0);
  auto a = gconv_args(dy.size(0), H, W, C, K, groups, R, S, sh, sw, ph, pw, dh, dil_w, w.size(1), 0);
  TORCH_CHECK(dy.dim() == 4 && dy.size(1) == a.P && dy.size(2) == a.Q && dy.size(3) == K, "gconv_dgrad: dy shape");
  if (a.Kg % 8 == 0) check_al16(dy.data_ptr(), "gconv_dgrad dy");
  auto dx = torch::empty({dy.size(0), H, W, C}, dy.options());
  check_hip(zoo_gconv(1, nullptr, w.data_ptr(), dy.data_ptr(), dx.data_ptr(), nullptr, &a, cur_stream()),
            "gconv_dgrad");
  return dx;
}

// dw (fp32 [K, ldb]) += grouped weight gradient
void gconv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, int groups, int R, int S, int sh, int sw,
                 int ph, int pw, int dh, int dil_w) {
  req(x, at::kBFloat16, "x");
  req(dy, at::kBFloat16, "dy");
  req(dw, at::kFloat, "dw");
  TORCH_CHECK(dw.dim() == 2, "gconv_wgrad: dw [K, ldb]");
  const int K = dw.size(0);
  auto a = gconv_args(x.size(0), x.size(1), x.size(2), x.size(3), K, groups, R, S, sh, sw, ph, pw, dh, dil_w,
                      dw.size(1), 0);
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == x.size(0) && dy.size(1) == a.P && dy.size(2) == a.Q && dy.size(3) == K,
              "gconv_wgrad: dy shape");
  check_hip(zoo_gconv(2, x.data_ptr(), nullptr, dy.data_ptr(), dw.data_ptr(), nullptr, &a, cur_stream()),
            "gconv_wgrad");
}

// depthwise conv: x [N,H,W,C] bf16, w [R*S, C] bf16 (tap-major)
std::vector<int> dw_geom(const torch::Tensor& x, int R, int S, int sh, int sw, int ph, int pw, int P, int Q) {
  return {(int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), P, Q, R, S, sh, sw, ph, pw};
}

torch::Tensor dwconv_fwd(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, int R, int S, int sh,
                         int sw, int ph, int pw, int act) {
  req(x, at::kBFloat16, "x");
  req(w, at::kBFloat16, "w");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "dwconv: NHWC with C%8==0");
  const int C = x.size(3);
  TORCH_CHECK(w.dim() == 2 && w.size(0) == R * S && w.size(1) == C, "dwconv: w must be [R*S, C]");
  TORCH_CHECK(R >= 1 && S >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0, "dwconv: bad geometry");
  const int P = (x.size(1) + 2 * ph - R) / sh + 1, Q = (x.size(2) + 2 * pw - S) / sw + 1;
  TORCH_CHECK(P > 0 && Q > 0, "dwconv: empty output");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == C, "dwconv: bias size");
    bp = bias->data_ptr<float>();
  }
  auto g = dw_geom(x, R, S, sh, sw, ph, pw, P, Q);
  auto y = torch::empty({x.size(0), P, Q, C}, x.options());
  check_hip(zoo_dwconv_fwd(x.data_ptr(), w.data_ptr(), bp, y.data_ptr(), g.data(), act, cur_stream()), "dwconv_fwd");
  return y;
}

torch::Tensor dwconv_dgrad(torch::Tensor dy, torch::Tensor w, int H, int W, int R, int S, int sh, int sw, int ph,
                           int pw) {
  req(dy, at::kBFloat16, "dy");
  req(w, at::kBFloat16, "w");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  TORCH_CHECK(C % 8 == 0 && w.size(0) == R * S && w.size(1) == C, "dwconv_dgrad: shapes");
  TORCH_CHECK(P == (H + 2 * ph - R) / sh + 1 && Q == (W + 2 * pw - S) / sw + 1, "dwconv_dgrad: geometry");
  auto dx = torch::empty({N, H, W, C}, dy.options());
  std::vector<int> g = {N, H, W, C, P, Q, R, S, sh, sw, ph, pw};
  check_hip(zoo_dwconv_dgrad(dy.data_ptr(), w.data_ptr(), dx.data_ptr(), g.data(), cur_stream()), "dwconv_dgrad");
  return dx;
}

// dw (fp32 [R*S, C]) += wgrad
void dwconv_wgrad(torch::Tensor x, torch::Tensor dy, torch::Tensor dw, int R, int S, int sh, int sw, int ph, int pw) {
  req(x, at::kBFloat16, "x");
  req(dy, at::kBFloat16, "dy");
  req(dw, at::kFloat, "dw");
  const int C = x.size(3);
  TORCH_CHECK(R * S <= 9, "dwconv_wgrad: at most 9 taps (3x3)");
  TORCH_CHECK(dw.numel() == (int64_t)R * S * C && dy.size(3) == C && dy.size(0) == x.size(0), "dwconv_wgrad: shapes");
  const int P = dy.size(1), Q = dy.size(2);
  TORCH_CHECK(P == (x.size(1) + 2 * ph - R) / sh + 1 && Q == (x.size(2) + 2 * pw - S) / sw + 1,
              "dwconv_wgrad: geometry");
  TORCH_CHECK((int64_t)R * S * C * 4 <= 160 * 1024, "dwconv_wgrad: R*S*C too large for the LDS fold");
  auto g = dw_geom(x, R, S, sh, sw, ph, pw, P, Q);
  auto partial = torch::empty({(int64_t)zoo_dwconv_wgrad_blocks(g.data()) * R * S * C}, dw.options());
  check_hip(zoo_dwconv_wgrad(x.data_ptr(), dy.data_ptr(), dw.data_ptr<float>(), partial.data_ptr<float>(), g.data(),
                             cur_stream()),
            "dwconv_wgrad");
}

// conv-epilogue backward: returns dy = dz * [z > 0] (z given) and/or db (fp32 [C]) = column sums
// gelu: z is the pre-activation and dy = dz * gelu'(z) (erf form)
std::vector<torch::Tensor> act_bwd_reduce(torch::Tensor dz, c10::optional<torch::Tensor> z, bool want_db,
                                          c10::optional<torch::Tensor> db_into, bool gelu) {
  req(dz, at::kBFloat16, "dz");
  const int C = dz.size(-1);
  const int64_t M = dz.numel() / C;
  TORCH_CHECK(C % 8 == 0, "act_bwd_reduce: C must be a multiple of 8");
  TORCH_CHECK(M < (1LL << 31), "act_bwd_reduce: too many rows");
  const bool mask = z.has_value() && z->defined();
  if (mask) {
    req(*z, at::kBFloat16, "z");
    TORCH_CHECK(z->numel() == dz.numel(), "act_bwd_reduce: z shape");
  }
  torch::Tensor dy = mask ? torch::empty_like(dz) : dz;
  torch::Tensor db;
  const bool part = g_deterministic;
  torch::Tensor partials;
  float* out = nullptr;
  if (want_db) {
    if (db_into.has_value() && db_into->defined()) {  // accumulate into an existing fp32 [C] (flat grad view)
      req(*db_into, at::kFloat, "db_into");
      TORCH_CHECK(db_into->numel() == C, "act_bwd_reduce: db_into size");
      db = *db_into;
    } else {
      db = torch::zeros({C}, dz.options().dtype(at::kFloat));
    }
    if (part) {
      partials = torch::empty({(int64_t)zoo_act_bwd_reduce_parts((int)M, C), (int64_t)C}, db.options());
      out = partials.data_ptr<float>();
    } else {
      out = db.data_ptr<float>();
    }
  }
  TORCH_CHECK(!gelu || mask, "act_bwd_reduce: gelu needs the pre-activation z");
  const int blocks = zoo_act_bwd_reduce(dz.data_ptr(), mask ? z->data_ptr() : nullptr, dy.data_ptr(), out, (int)M, C,
                                        part ? 1 : 0, gelu ? 1 : 0, cur_stream());
  check_hip(hipGetLastError(), "act_bwd_reduce");
  if (want_db && part) fold_partials(db.data_ptr<float>(), partials, C, blocks);
  if (want_db) return {dy, db};
  return {dy};
}

// row softmax / log-softmax over the last dim (fp32 or bf16)
torch::Tensor softmax_rows(torch::Tensor x, bool log_out) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "softmax: contiguous GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "softmax: fp32 or bf16");
  const int n = x.size(-1);
  const int64_t rows = n ? x.numel() / n : 0;
  TORCH_CHECK(rows < (1LL << 31), "softmax: too many rows");
  auto y = torch::empty_like(x);
  if (rows == 0) return y;
  check_hip(zoo_softmax_rows(x.data_ptr(), y.data_ptr(), (int)rows, n, log_out, x.scalar_type() == at::kFloat,
                             cur_stream()),
            "softmax_rows");
  return y;
}

torch::Tensor softmax_rows_bwd(torch::Tensor y, torch::Tensor dy, bool log_out) {
  TORCH_CHECK(y.is_cuda() && y.is_contiguous() && dy.is_contiguous() && dy.sizes() == y.sizes() &&
                  dy.scalar_type() == y.scalar_type(), "softmax_bwd: matching contiguous GPU tensors");
  const int n = y.size(-1);
  const int64_t rows = n ? y.numel() / n : 0;
  auto dx = torch::empty_like(y);
  if (rows == 0) return dx;
  check_hip(zoo_softmax_rows_bwd(y.data_ptr(), dy.data_ptr(), dx.data_ptr(), (int)rows, n, log_out,
                                 y.scalar_type() == at::kFloat, cur_stream()),
            "softmax_rows_bwd");
  return dx;
}

// cross-channel LRN over the last dim; backward when dy is given
torch::Tensor lrn(torch::Tensor x, c10::optional<torch::Tensor> dy, int size, double alpha, double beta, double k) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "lrn: contiguous GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "lrn: fp32 or bf16");
  TORCH_CHECK(size >= 1 && size <= 15, "lrn: window size 1..15");
  const int C = x.size(-1);
  const size_t rows = C ? x.numel() / C : 0;
  auto out = torch::empty_like(x);
  const bool bwd = dy.has_value() && dy->defined();
  if (bwd) TORCH_CHECK(dy->is_contiguous() && dy->sizes() == x.sizes() && dy->scalar_type() == x.scalar_type(),
                       "lrn: dy must match x");
  if (rows == 0) return out;
  check_hip(zoo_lrn(x.data_ptr(), bwd ? dy->data_ptr() : nullptr, out.data_ptr(), rows, C, size, (float)alpha,
                    (float)beta, (float)k, bwd, x.scalar_type() == at::kFloat, cur_stream()),
            "lrn");
  return out;
}

// ---- Keras layer kernels (keras_ops.hip) -------------------------------------------------
static void req_act(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), what, ": contiguous GPU tensor expected");
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, what, ": fp32 or bf16");
}

// WithinChannelLRN2D on NHWC: forward (dy absent) or backward (dx)
torch::Tensor within_lrn(torch::Tensor x, c10::optional<torch::Tensor> dy, int size, double alpha, double beta) {
  req_act(x, "within_lrn");
  TORCH_CHECK(x.dim() == 4, "within_lrn: NHWC input");
  TORCH_CHECK(size >= 1 && size <= 31, "within_lrn: window 1..31");
  const bool bwd = dy.has_value() && dy->defined();
  if (bwd) TORCH_CHECK(dy->sizes() == x.sizes() && dy->is_contiguous() && dy->scalar_type() == x.scalar_type(),
                       "within_lrn: dy must match x");
  auto out = torch::empty_like(x);
  if (x.numel() == 0) return out;
  TORCH_CHECK(x.numel() < (1LL << 40), "within_lrn: too large");
  torch::Tensor q, sc;
  if (bwd) {
    q = torch::empty(x.sizes(), x.options().dtype(at::kFloat));
    sc = torch::empty(x.sizes(), x.options().dtype(at::kFloat));
  }
  check_hip(zoo_wlrn(x.data_ptr(), bwd ? dy->data_ptr() : nullptr, out.data_ptr(), bwd ? q.data_ptr<float>() : nullptr,
                     bwd ? sc.data_ptr<float>() : nullptr, x.size(0), x.size(1), x.size(2), x.size(3), size,
                     (float)alpha, (float)beta, x.scalar_type() == at::kBFloat16, cur_stream()),
            "within_lrn");
  return out;
}

// bilinear resize on NHWC; align: 0 BigDL / TF-legacy, 1 align_corners, 2 half-pixel centres
torch::Tensor resize_bilinear(torch::Tensor x, int OH, int OW, int64_t align) {
  req_act(x, "resize_bilinear");
  TORCH_CHECK(x.dim() == 4 && OH > 0 && OW > 0 && x.size(1) > 0 && x.size(2) > 0, "resize_bilinear: NHWC, sizes");
  auto y = torch::empty({x.size(0), OH, OW, x.size(3)}, x.options());
  if (y.numel() == 0) return y;
  check_hip(zoo_resize_bilinear(x.data_ptr(), y.data_ptr(), x.size(0), x.size(1), x.size(2), x.size(3), OH, OW,
                                (int)align, 0, x.scalar_type() == at::kBFloat16, cur_stream()),
            "resize_bilinear");
  return y;
}

torch::Tensor resize_bilinear_bwd(torch::Tensor dy, int H, int W, int64_t align) {
  req_act(dy, "resize_bilinear_bwd");
  TORCH_CHECK(dy.dim() == 4 && H > 0 && W > 0, "resize_bilinear_bwd: NHWC dy");
  auto dx = torch::zeros({dy.size(0), H, W, dy.size(3)}, dy.options().dtype(at::kFloat));
  if (dy.numel() == 0) return dx.to(dy.scalar_type());
  check_hip(zoo_resize_bilinear(dy.data_ptr(), dx.data_ptr(), dy.size(0), H, W, dy.size(3), dy.size(1), dy.size(2),
                                (int)align, 1, dy.scalar_type() == at::kBFloat16, cur_stream()),
            "resize_bilinear_bwd");
  return dy.scalar_type() == at::kFloat ? dx : dx.to(dy.scalar_type());
}

// nearest upsampling of x [N, D, H, W, C] by (fd, fh, fw); backward sums the blocks
torch::Tensor upsample_nd(torch::Tensor x, int fd, int fh, int fw, bool backward) {
  req_act(x, "upsample");
  TORCH_CHECK(x.dim() == 5 && fd >= 1 && fh >= 1 && fw >= 1, "upsample: [N, D, H, W, C] and factors >= 1");
  torch::Tensor out;
  int D = x.size(1), H = x.size(2), W = x.size(3);
  if (!backward) {
    out = torch::empty({x.size(0), (int64_t)D * fd, (int64_t)H * fh, (int64_t)W * fw, x.size(4)}, x.options());
  } else {
    TORCH_CHECK(D % fd == 0 && H % fh == 0 && W % fw == 0, "upsample backward: dy dims must divide by the factors");
    D /= fd; H /= fh; W /= fw;
    out = torch::empty({x.size(0), D, H, W, x.size(4)}, x.options());
  }
  if (out.numel() == 0) return out;
  check_hip(zoo_upsample(x.data_ptr(), out.data_ptr(), x.size(0), D, H, W, x.size(4), fd, fh, fw, backward,
                         x.scalar_type() == at::kBFloat16, cur_stream()),
            "upsample");
  return out;
}

// ConvLSTM gate step: g = gx + gh ([M, 4F] fp32) -> (h, c, acts)
std::vector<torch::Tensor> lstm_gates_fwd(torch::Tensor gx, c10::optional<torch::Tensor> gh,
                                          c10::optional<torch::Tensor> cprev, int64_t iact, int64_t act) {
  req(gx, at::kFloat, "gx");
  TORCH_CHECK(gx.dim() == 2 && gx.size(1) % 4 == 0, "lstm_gates: gx [M, 4F]");
  const int64_t M = gx.size(0), F = gx.size(1) / 4;
  if (gh.has_value() && gh->defined()) {
    req(*gh, at::kFloat, "gh");
    TORCH_CHECK(gh->sizes() == gx.sizes(), "lstm_gates: gh must match gx");
  }
  if (cprev.has_value() && cprev->defined()) {
    req(*cprev, at::kFloat, "cprev");
    TORCH_CHECK(cprev->numel() == M * F, "lstm_gates: c_prev [M, F]");
  }
  TORCH_CHECK(iact >= 0 && iact <= 4 && act >= 0 && act <= 4, "lstm_gates: activation code");
  auto h = torch::empty({M, F}, gx.options());
  auto c = torch::empty({M, F}, gx.options());
  auto acts = torch::empty_like(gx);
  if (M * F == 0) return {h, c, acts};
  check_hip(zoo_lstm_gates(gx.data_ptr<float>(), gh.has_value() && gh->defined() ? gh->data_ptr<float>() : nullptr,
                           cprev.has_value() && cprev->defined() ? cprev->data_ptr<float>() : nullptr,
                           h.data_ptr<float>(), c.data_ptr<float>(), acts.data_ptr<float>(), nullptr, nullptr, nullptr,
                           nullptr, (int)M, (int)F, (int)iact, (int)act, 0, cur_stream()),
            "lstm_gates_fwd");
  return {h, c, acts};
}

std::vector<torch::Tensor> lstm_gates_bwd(c10::optional<torch::Tensor> dh, c10::optional<torch::Tensor> dcn,
                                          torch::Tensor acts, c10::optional<torch::Tensor> cprev, torch::Tensor c,
                                          int64_t iact, int64_t act) {
  req(acts, at::kFloat, "acts");
  req(c, at::kFloat, "c");
  const int64_t M = acts.size(0), F = acts.size(1) / 4;
  TORCH_CHECK(c.numel() == M * F, "lstm_gates_bwd: c [M, F]");
  auto opt = [&](const c10::optional<torch::Tensor>& t, const char* n) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    req(*t, at::kFloat, n);
    TORCH_CHECK(t->numel() == M * F, "lstm_gates_bwd: ", n, " [M, F]");
    return t->data_ptr<float>();
  };
  const float* pdh = opt(dh, "dh");
  const float* pdc = opt(dcn, "dc");
  const float* pcp = opt(cprev, "cprev");
  auto dg = torch::empty_like(acts);
  auto dcp = torch::empty_like(c);
  if (M * F == 0) return {dg, dcp};
  check_hip(zoo_lstm_gates(nullptr, nullptr, pcp, nullptr, c.data_ptr<float>(), acts.data_ptr<float>(), pdh, pdc,
                           dg.data_ptr<float>(), dcp.data_ptr<float>(), (int)M, (int)F, (int)iact, (int)act, 1,
                           cur_stream()),
            "lstm_gates_bwd");
  return {dg, dcp};
}

// Whole-sequence ConvLSTM step (keras_ops.hip lstm_step_*): every output is a caller-owned slot
// of the sequence buffers; gh / hb / dhr / dgb are NHWC rows with their own (padded) strides.
void lstm_step_fwd(torch::Tensor gx, c10::optional<torch::Tensor> gh, c10::optional<torch::Tensor> cprev,
                   torch::Tensor h, torch::Tensor c, torch::Tensor acts, torch::Tensor hb, int64_t iact, int64_t act) {
  req(gx, at::kFloat, "gx");
  TORCH_CHECK(gx.dim() == 2 && gx.size(1) % 4 == 0, "lstm_step: gx [M, 4F]");
  const int64_t M = gx.size(0), F = gx.size(1) / 4;
  req(h, at::kFloat, "h"); req(c, at::kFloat, "c"); req(acts, at::kFloat, "acts"); req(hb, at::kBFloat16, "hb");
  TORCH_CHECK(h.numel() == M * F && c.numel() == M * F && acts.numel() == M * 4 * F, "lstm_step: output sizes");
  TORCH_CHECK(hb.numel() % M == 0 && hb.numel() / M >= F, "lstm_step: hb [M, >=F]");
  const float* ghp = nullptr;
  int64_t ldgh = 4 * F;
  if (gh.has_value() && gh->defined()) {
    req(*gh, at::kFloat, "gh");
    TORCH_CHECK(gh->numel() % M == 0 && gh->numel() / M >= 4 * F, "lstm_step: gh [M, >=4F]");
    ghp = gh->data_ptr<float>();
    ldgh = gh->numel() / M;
  }
  const float* cp = nullptr;
  if (cprev.has_value() && cprev->defined()) {
    req(*cprev, at::kFloat, "cprev");
    TORCH_CHECK(cprev->numel() == M * F, "lstm_step: c_prev [M, F]");
    cp = cprev->data_ptr<float>();
  }
  TORCH_CHECK(iact >= 0 && iact <= 4 && act >= 0 && act <= 4, "lstm_step: activation code");
  if (M * F == 0) return;
  check_hip(zoo_lstm_step(gx.data_ptr<float>(), ghp, (int)ldgh, cp, h.data_ptr<float>(), c.data_ptr<float>(),
                          acts.data_ptr<float>(), hb.data_ptr(), (int)(hb.numel() / M), nullptr, nullptr, 0, nullptr,
                          nullptr, nullptr, 0, nullptr, (int)M, (int)F, (int)iact, (int)act, 0, cur_stream()),
            "lstm_step_fwd");
}

void lstm_step_bwd(c10::optional<torch::Tensor> dout, c10::optional<torch::Tensor> dhr, c10::optional<torch::Tensor> dcn,
                   torch::Tensor acts, c10::optional<torch::Tensor> cprev, torch::Tensor c, torch::Tensor dg,
                   torch::Tensor dgb, torch::Tensor dcp, int64_t iact, int64_t act) {
  req(acts, at::kFloat, "acts"); req(c, at::kFloat, "c"); req(dg, at::kFloat, "dg"); req(dcp, at::kFloat, "dcp");
  req(dgb, at::kBFloat16, "dgb");
  const int64_t M = acts.size(0), F = acts.size(1) / 4;
  TORCH_CHECK(acts.dim() == 2 && c.numel() == M * F && dg.numel() == M * 4 * F && dcp.numel() == M * F,
              "lstm_step_bwd: sizes");
  TORCH_CHECK(dgb.numel() % M == 0 && dgb.numel() / M >= 4 * F, "lstm_step_bwd: dgb [M, >=4F]");
  auto opt = [&](const c10::optional<torch::Tensor>& t, const char* n) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    req(*t, at::kFloat, n);
    TORCH_CHECK(t->numel() == M * F, "lstm_step_bwd: ", n, " [M, F]");
    return t->data_ptr<float>();
  };
  const float* pd = opt(dout, "dout");
  const float* pdc = opt(dcn, "dc");
  const float* pcp = opt(cprev, "cprev");
  const void* pr = nullptr;
  int64_t lddh = 0;
  if (dhr.has_value() && dhr->defined()) {
    req(*dhr, at::kBFloat16, "dhr");
    TORCH_CHECK(dhr->numel() % M == 0 && dhr->numel() / M >= F, "lstm_step_bwd: dhr [M, >=F]");
    pr = dhr->data_ptr();
    lddh = dhr->numel() / M;
  }
  if (M * F == 0) return;
  check_hip(zoo_lstm_step(nullptr, nullptr, 0, pcp, nullptr, c.data_ptr<float>(), acts.data_ptr<float>(), nullptr, 0,
                          pd, pr, (int)lddh, pdc, dg.data_ptr<float>(), dgb.data_ptr(), (int)(dgb.numel() / M),
                          dcp.data_ptr<float>(), (int)M, (int)F, (int)iact, (int)act, 1, cur_stream()),
            "lstm_step_bwd");
}

// One ConvLSTM2D step per launch (kernels/convlstm.hip), gate-interleaved layout (column 4j + g).
// x: the step's conv input [B][D][H][W][Cx] bf16 (ConvLSTM2D: [B][H][W][Cx], D = Q = 1; None: no
// recurrent term); wt: packed weights [rows][>= Q*R*S*Cx] -- forward the 4F gate rows, backward the
// flipped weight (rows = hidden channels).
static void convlstm_geom(const c10::optional<torch::Tensor>& x, const torch::Tensor& wt, int B, int D, int H, int W,
                          int Q, int R, int S, int rows_min, int* Cx) {
  req(wt, at::kBFloat16, "wt");
  TORCH_CHECK(wt.dim() == 2 && wt.size(0) >= rows_min && wt.size(0) <= 256 && wt.size(1) % 8 == 0,
              "convlstm: packed weight [rows <= 256][ldw % 8 == 0]");
  TORCH_CHECK(Q % 2 == 1 && R % 2 == 1 && S % 2 == 1 && D >= 1, "convlstm: odd (same-padded) kernels");
  *Cx = 0;
  if (x.has_value() && x->defined()) {
    req(*x, at::kBFloat16, "x");
    const int64_t C = x->size(-1);
    TORCH_CHECK(C % 8 == 0 && x->size(0) == B && x->numel() == (int64_t)B * D * H * W * C,
                "convlstm: x [B, (D,) H, W, Cx % 8 == 0]");
    *Cx = C;
    TORCH_CHECK(wt.size(1) >= (int64_t)Q * R * S * *Cx, "convlstm: weight row shorter than Q*R*S*Cx");
    check_al16(x->data_ptr(), "convlstm x");
    check_al16(wt.data_ptr(), "convlstm wt");
  }
}

void convlstm_fwd_step(c10::optional<torch::Tensor> x, torch::Tensor wt, int64_t B, int64_t D, int64_t H, int64_t W,
                       int64_t Q, int64_t R, int64_t S, torch::Tensor gx, c10::optional<torch::Tensor> cprev, torch::Tensor h,
                       torch::Tensor c, torch::Tensor acts, torch::Tensor hb, int64_t iact, int64_t act) {
  const int64_t M = B * D * H * W;
  req(gx, at::kFloat, "gx"); req(h, at::kFloat, "h"); req(c, at::kFloat, "c"); req(acts, at::kFloat, "acts");
  req(hb, at::kBFloat16, "hb");
  TORCH_CHECK(M > 0 && gx.numel() % (4 * M) == 0, "convlstm_fwd: gx [M, F, 4]");
  const int64_t F = gx.numel() / (4 * M);
  TORCH_CHECK(h.numel() == M * F && c.numel() == M * F && acts.numel() == 4 * M * F, "convlstm_fwd: outputs");
  TORCH_CHECK(hb.numel() % M == 0 && hb.numel() / M >= F, "convlstm_fwd: hb [M, >= F]");
  TORCH_CHECK(iact >= 0 && iact <= 4 && act >= 0 && act <= 4, "convlstm: activation code");
  int Cx;
  convlstm_geom(x, wt, B, D, H, W, Q, R, S, 4 * F, &Cx);
  const float* cp = nullptr;
  if (cprev.has_value() && cprev->defined()) {
    req(*cprev, at::kFloat, "cprev");
    TORCH_CHECK(cprev->numel() == M * F, "convlstm_fwd: c_prev [M, F]");
    cp = cprev->data_ptr<float>();
  }
  check_hip(zoo_convlstm_step(opt_ptr<void>(x), wt.data_ptr(), B, D, H, W, Cx, Q, R, S, wt.size(1), 4 * F, F, iact, act,
                              gx.data_ptr<float>(), 0, cp, h.data_ptr<float>(), c.data_ptr<float>(),
                              acts.data_ptr<float>(), hb.data_ptr(), hb.numel() / M, nullptr, nullptr, nullptr, 0,
                              nullptr, nullptr, 0, 0, nullptr, cur_stream()),
            "convlstm_fwd_step");
}

void convlstm_bwd_step(c10::optional<torch::Tensor> x, torch::Tensor wt, int64_t B, int64_t D, int64_t H, int64_t W,
                       int64_t Q, int64_t R, int64_t S, c10::optional<torch::Tensor> dout, torch::Tensor acts,
                       c10::optional<torch::Tensor> cprev, torch::Tensor cc, torch::Tensor dc, bool dc_in,
                       torch::Tensor dg, torch::Tensor dgb, int64_t iact, int64_t act) {
  const int64_t M = B * D * H * W;
  req(acts, at::kFloat, "acts"); req(cc, at::kFloat, "c"); req(dc, at::kFloat, "dc"); req(dg, at::kFloat, "dg");
  req(dgb, at::kBFloat16, "dgb");
  TORCH_CHECK(M > 0 && acts.numel() % (4 * M) == 0, "convlstm_bwd: acts [M, F, 4]");
  const int64_t F = acts.numel() / (4 * M);
  TORCH_CHECK(cc.numel() == M * F && dc.numel() == M * F && dg.numel() == 4 * M * F, "convlstm_bwd: sizes");
  TORCH_CHECK(dgb.numel() % M == 0 && dgb.numel() / M >= 4 * F && (dgb.numel() / M) % 4 == 0,
              "convlstm_bwd: dgb [M, >= 4F, % 4]");
  TORCH_CHECK(iact >= 0 && iact <= 4 && act >= 0 && act <= 4, "convlstm: activation code");
  int Cx;
  convlstm_geom(x, wt, B, D, H, W, Q, R, S, F, &Cx);
  auto opt = [&](const c10::optional<torch::Tensor>& t, const char* n) -> const float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    req(*t, at::kFloat, n);
    TORCH_CHECK(t->numel() == M * F, "convlstm_bwd: ", n, " [M, F]");
    return t->data_ptr<float>();
  };
  check_hip(zoo_convlstm_step(opt_ptr<void>(x), wt.data_ptr(), B, D, H, W, Cx, Q, R, S, wt.size(1), wt.size(0), F, iact,
                              act, nullptr, 0, opt(cprev, "cprev"), nullptr, nullptr, acts.data_ptr<float>(), nullptr, 0,
                              opt(dout, "dout"), cc.data_ptr<float>(), dc.data_ptr<float>(), dc_in ? 1 : 0,
                              dg.data_ptr<float>(), dgb.data_ptr(), dgb.numel() / M, 1, nullptr, cur_stream()),
            "convlstm_bwd_step");
}

// Whole ConvLSTM sequences: the step loop in C++ (T launches each way, no per-step Python view /
// binding overhead -- at T = 32 that overhead, not the kernels, bounded the step). Sequence buffers
// are time-major: gxs / acts / dgxs [T][M][F][4], hist [T+1][M][cph] (slot 0 zero), hseq / cseq
// [T][M][F], dgb [T][M][K8]; dout [T][M][F] (rseq) or [M][F] (last step only).
void convlstm_fwd_seq(torch::Tensor gxs, torch::Tensor wt, int64_t B, int64_t D, int64_t H, int64_t W, int64_t Q,
                      int64_t R, int64_t S, torch::Tensor hist, torch::Tensor hseq, torch::Tensor cseq,
                      torch::Tensor acts, int64_t iact, int64_t act) {
  TORCH_CHECK(gxs.is_cuda() && gxs.is_contiguous() &&
                  (gxs.scalar_type() == at::kFloat || gxs.scalar_type() == at::kBFloat16),
              "convlstm_fwd_seq: gxs contiguous fp32 / bf16");
  const bool gxb = gxs.scalar_type() == at::kBFloat16;
  req(hist, at::kBFloat16, "hist"); req(hseq, at::kFloat, "hseq");
  req(cseq, at::kFloat, "cseq"); req(acts, at::kFloat, "acts");
  const int64_t M = B * D * H * W, T = gxs.size(0);
  TORCH_CHECK(T > 0 && M > 0 && gxs.numel() % (4 * M * T) == 0, "convlstm_fwd_seq: gxs [T, M, F, 4]");
  const int64_t F = gxs.numel() / (4 * M * T);
  TORCH_CHECK(hseq.numel() == T * M * F && cseq.numel() == T * M * F && acts.numel() == 4 * T * M * F,
              "convlstm_fwd_seq: hseq / cseq / acts sizes");
  TORCH_CHECK(hist.size(0) == T + 1 && hist.numel() % ((T + 1) * M) == 0, "convlstm_fwd_seq: hist [T + 1, M, cph]");
  const int64_t cph = hist.numel() / ((T + 1) * M);
  TORCH_CHECK(cph % 8 == 0 && cph >= F, "convlstm_fwd_seq: hist channels");
  TORCH_CHECK(iact >= 0 && iact <= 4 && act >= 0 && act <= 4, "convlstm: activation code");
  auto x0 = hist[0].view({B, D * H, W, cph});
  int Cx;
  convlstm_geom(c10::optional<torch::Tensor>(x0), wt, B, D, H, W, Q, R, S, 4 * F, &Cx);
  const uint16_t* hp = reinterpret_cast<const uint16_t*>(hist.data_ptr());
  float* cs = cseq.data_ptr<float>();
  // K-split partial sums of the large steps (convlstm.hip persistent kernel), reused by every step
  auto part = torch::empty({M >= 32768 && T > 1 ? M * ((4 * F + 15) / 16 * 16) : 0}, hseq.options());
  float* pp = part.numel() ? part.data_ptr<float>() : nullptr;
  for (int64_t s = 0; s < T; ++s) {
    check_hip(zoo_convlstm_step(s > 0 ? hp + s * M * cph : nullptr, wt.data_ptr(), B, D, H, W, Cx, Q, R, S, wt.size(1),
                                4 * F, F, iact, act,
                                static_cast<const char*>(gxs.data_ptr()) + s * M * 4 * F * gxs.element_size(), gxb ? 1 : 0,
                                s > 0 ? cs + (s - 1) * M * F : nullptr, hseq.data_ptr<float>() + s * M * F,
                                cs + s * M * F, acts.data_ptr<float>() + s * M * 4 * F,
                                const_cast<uint16_t*>(hp) + (s + 1) * M * cph, cph, nullptr, nullptr, nullptr, 0,
                                nullptr, nullptr, 0, 0, pp, cur_stream()),
              "convlstm_fwd_seq");
  }
}

void convlstm_bwd_seq(torch::Tensor dout, bool rseq, torch::Tensor wt, int64_t B, int64_t D, int64_t H, int64_t W,
                      int64_t Q, int64_t R, int64_t S, torch::Tensor acts, torch::Tensor cseq, torch::Tensor dc,
                      c10::optional<torch::Tensor> dgxs_opt, torch::Tensor dgb, int64_t iact, int64_t act) {
  // dgxs None: the fp32 gate gradients are not written (the caller takes dgb, the bf16 copy)
  const bool dg32 = dgxs_opt.has_value() && dgxs_opt->defined();
  torch::Tensor dgxs = dg32 ? *dgxs_opt : acts;
  req(dout, at::kFloat, "dout"); req(acts, at::kFloat, "acts"); req(cseq, at::kFloat, "cseq");
  req(dc, at::kFloat, "dc"); req(dgxs, at::kFloat, "dgxs"); req(dgb, at::kBFloat16, "dgb");
  const int64_t M = B * D * H * W, T = acts.size(0);
  TORCH_CHECK(T > 0 && M > 0 && acts.numel() % (4 * M * T) == 0, "convlstm_bwd_seq: acts [T, M, F, 4]");
  const int64_t F = acts.numel() / (4 * M * T);
  TORCH_CHECK(cseq.numel() == T * M * F && dc.numel() == M * F && dgxs.numel() == 4 * T * M * F,
              "convlstm_bwd_seq: sizes");
  TORCH_CHECK(dout.numel() == (rseq ? T : 1) * M * F, "convlstm_bwd_seq: dout [T, M, F] or [M, F]");
  TORCH_CHECK(dgb.size(0) == T && dgb.numel() % (T * M) == 0, "convlstm_bwd_seq: dgb [T, M, K8]");
  const int64_t K8 = dgb.numel() / (T * M);
  TORCH_CHECK(K8 % 8 == 0 && K8 >= 4 * F, "convlstm_bwd_seq: dgb channels");
  TORCH_CHECK(iact >= 0 && iact <= 4 && act >= 0 && act <= 4, "convlstm: activation code");
  auto x0 = dgb[0].view({B, D * H, W, K8});
  int Cx;
  convlstm_geom(c10::optional<torch::Tensor>(x0), wt, B, D, H, W, Q, R, S, F, &Cx);
  uint16_t* gb = reinterpret_cast<uint16_t*>(dgb.data_ptr());
  const float* cs = cseq.data_ptr<float>();
  auto part = torch::empty({M >= 32768 && T > 1 ? M * ((wt.size(0) + 15) / 16 * 16) : 0}, cseq.options());
  float* pp = part.numel() ? part.data_ptr<float>() : nullptr;
  for (int64_t s = T - 1; s >= 0; --s) {
    const float* d = rseq ? dout.data_ptr<float>() + s * M * F : (s == T - 1 ? dout.data_ptr<float>() : nullptr);
    check_hip(zoo_convlstm_step(s < T - 1 ? gb + (s + 1) * M * K8 : nullptr, wt.data_ptr(), B, D, H, W, Cx, Q, R, S,
                                wt.size(1), wt.size(0), F, iact, act, nullptr, 0, s > 0 ? cs + (s - 1) * M * F : nullptr,
                                nullptr, nullptr, acts.data_ptr<float>() + s * M * 4 * F, nullptr, 0, d,
                                cs + s * M * F, dc.data_ptr<float>(), s < T - 1 ? 1 : 0,
                                dg32 ? dgxs.data_ptr<float>() + s * M * 4 * F : nullptr, gb + s * M * K8, K8, 1, pp,
                                cur_stream()),
              "convlstm_bwd_seq");
  }
}

// A stream restricted to `ncu` CUs spread evenly over the device (hipExtStreamCreateWithCUMask):
// the weight-gradient side stream, so its kernels never take CU slots a persistent compute-stream
// kernel is sized for (those size their grids to the remaining CUs, set_reserved_cus). Returns
// the hipStream_t as an integer (torch.cuda.ExternalStream); the stream lives for the process.
int64_t cu_mask_stream(int64_t ncu_side) {
  int dev = 0, n = 0;
  check_hip(hipGetDevice(&dev), "hipGetDevice");
  check_hip(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev), "cu count");
  TORCH_CHECK(ncu_side > 0 && ncu_side < n, "cu_mask_stream: 0 < ncu < ", n);
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int64_t i = 0; i < ncu_side; ++i) {
    const int cu = (int)(i * n / ncu_side);
    mask[cu / 32] |= 1u << (cu % 32);
  }
  hipStream_t s = nullptr;
  check_hip(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()), "hipExtStreamCreateWithCUMask");
  return reinterpret_cast<int64_t>(s);
}

// Max RoI pooling (Faster R-CNN): features NHWC, rois [R, 5] fp32 -> (out [R, PH, PW, C], argmax int32)
std::vector<torch::Tensor> roi_pool_fwd(torch::Tensor f, torch::Tensor rois, int PH, int PW, double scale) {
  req_act(f, "roi_pool");
  req(rois, at::kFloat, "rois");
  TORCH_CHECK(f.dim() == 4 && rois.dim() == 2 && rois.size(1) == 5, "roi_pool: f NHWC, rois [R, 5]");
  TORCH_CHECK(PH > 0 && PW > 0 && f.size(0) > 0, "roi_pool: pooled size / batch");
  const int R = rois.size(0), H = f.size(1), W = f.size(2), C = f.size(3);
  auto out = torch::empty({R, PH, PW, C}, f.options());
  auto arg = torch::empty({R, PH, PW, C}, f.options().dtype(at::kInt));
  if (out.numel() == 0) return {out, arg};
  TORCH_CHECK((int64_t)H * W < (1LL << 31) && out.numel() < (1LL << 40), "roi_pool: too large");
  check_hip(zoo_roi_pool(f.data_ptr(), rois.data_ptr<float>(), out.data_ptr(), arg.data_ptr<int>(), nullptr, nullptr,
                         f.size(0), R, H, W, C, PH, PW, (float)scale, 0, f.scalar_type() == at::kBFloat16,
                         cur_stream()),
            "roi_pool");
  return {out, arg};
}

torch::Tensor roi_pool_bwd(torch::Tensor dy, torch::Tensor argmax, torch::Tensor rois, int B, int H, int W) {
  req_act(dy, "roi_pool_bwd");
  req(rois, at::kFloat, "rois");
  TORCH_CHECK(argmax.is_cuda() && argmax.scalar_type() == at::kInt && argmax.sizes() == dy.sizes() &&
                  argmax.is_contiguous(), "roi_pool_bwd: argmax int32 like dy");
  TORCH_CHECK(dy.dim() == 4 && rois.size(0) == dy.size(0) && B > 0, "roi_pool_bwd: shapes");
  auto df = torch::zeros({B, H, W, dy.size(3)}, dy.options().dtype(at::kFloat));
  if (dy.numel() == 0) return df;
  check_hip(zoo_roi_pool(nullptr, rois.data_ptr<float>(), nullptr, argmax.data_ptr<int>(), dy.data_ptr(),
                         df.data_ptr<float>(), B, dy.size(0), H, W, dy.size(3), dy.size(1), dy.size(2), 1.f, 1,
                         dy.scalar_type() == at::kBFloat16, cur_stream()),
            "roi_pool_bwd");
  return df;
}

torch::Tensor gap_fwd(torch::Tensor x) {
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "gap: NHWC with C%8==0");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  auto y = torch::empty({N, C}, x.options());
  check_hip(zoo_gap_fwd(x.data_ptr(), y.data_ptr(), N, HW, C, cur_stream()), "gap_fwd");
  return y;
}

torch::Tensor gap_bwd(torch::Tensor dy, int H, int W) {
  req(dy, at::kBFloat16, "dy");
  TORCH_CHECK(dy.dim() == 2 && dy.size(1) % 8 == 0, "gap_bwd: [N,C] with C%8==0");
  const int N = dy.size(0), C = dy.size(1);
  auto dx = torch::empty({N, H, W, C}, dy.options());
  check_hip(zoo_gap_bwd(dy.data_ptr(), dx.data_ptr(), N, H * W, C, cur_stream()), "gap_bwd");
  return dx;
}

// returns (loss_sum[1], count[1], dlogits or empty)
std::vector<torch::Tensor> softmax_xent(torch::Tensor logits, torch::Tensor labels, bool want_grad, double grad_scale,
                                        int64_t ignore_index) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "softmax_xent: 2-D GPU logits");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16, "logits dtype");
  req(labels, at::kLong, "labels");
  TORCH_CHECK(labels.numel() == logits.size(0), "labels size");
  const int B = logits.size(0), NC = logits.size(1);
  const bool per_row = g_deterministic;
  auto loss = per_row ? torch::empty({2, B}, logits.options().dtype(at::kFloat))
                      : torch::zeros({2}, logits.options().dtype(at::kFloat));
  torch::Tensor dl;
  if (want_grad) dl = torch::empty_like(logits);
  const bool f32 = logits.scalar_type() == at::kFloat;
  check_hip(zoo_softmax_xent(logits.data_ptr(), f32, labels.data_ptr<int64_t>(), loss.data_ptr<float>(),
                             loss.data_ptr<float>() + (per_row ? B : 1), want_grad ? dl.data_ptr() : nullptr, B, NC,
                             (float)grad_scale, (int)ignore_index, per_row ? 1 : 0, cur_stream()),
            "softmax_xent");
  if (per_row) loss = loss.sum(1);
  if (want_grad) return {loss, dl};
  return {loss};
}

// {out [mean loss, count], unscaled dlogits}: two launches, deterministic (ordered fold)
std::vector<torch::Tensor> softmax_xent_mean(torch::Tensor logits, torch::Tensor labels, int64_t ignore_index) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous() && logits.dim() == 2, "softmax_xent_mean: 2-D GPU logits");
  TORCH_CHECK(logits.scalar_type() == at::kFloat || logits.scalar_type() == at::kBFloat16, "logits dtype");
  req(labels, at::kLong, "labels");
  TORCH_CHECK(labels.numel() == logits.size(0) && logits.size(0) > 0 && logits.size(0) < (1LL << 30),
              "softmax_xent_mean: labels size");
  const int B = logits.size(0), NC = logits.size(1);
  auto part = torch::empty({2 * B}, logits.options().dtype(at::kFloat));
  auto out = torch::empty({2}, logits.options().dtype(at::kFloat));
  auto dl = torch::empty_like(logits);
  check_hip(zoo_softmax_xent_mean(logits.data_ptr(), logits.scalar_type() == at::kFloat, labels.data_ptr<int64_t>(),
                                  part.data_ptr<float>(), out.data_ptr<float>(), dl.data_ptr(), B, NC,
                                  (int)ignore_index, cur_stream()),
            "softmax_xent_mean");
  return {out, dl};
}

// dl * (g / max(count, 1)) in dl's dtype (g, count: device scalars)
torch::Tensor xent_grad_scale(torch::Tensor dl, torch::Tensor g, torch::Tensor count) {
  TORCH_CHECK(dl.is_cuda() && dl.is_contiguous(), "xent_grad_scale: contiguous GPU dl");
  TORCH_CHECK(dl.scalar_type() == at::kFloat || dl.scalar_type() == at::kBFloat16, "xent_grad_scale: dtype");
  req(g, at::kFloat, "g");
  req(count, at::kFloat, "count");
  TORCH_CHECK(g.numel() >= 1 && count.numel() >= 1, "xent_grad_scale: scalar g / count");
  auto out = torch::empty_like(dl);
  if (dl.numel())
    check_hip(zoo_xent_grad_scale(dl.data_ptr(), dl.scalar_type() == at::kFloat, g.data_ptr<float>(),
                                  count.data_ptr<float>(), out.data_ptr(), (size_t)dl.numel(), cur_stream()),
              "xent_grad_scale");
  return out;
}

// NLL of probabilities [B, NC] against int64 labels: {loss_sum, count} (+ unscaled dprobs)
std::vector<torch::Tensor> prob_nll(torch::Tensor probs, torch::Tensor labels, bool want_grad, double eps,
                                    int64_t ignore_index) {
  TORCH_CHECK(probs.is_cuda() && probs.is_contiguous() && probs.dim() == 2, "prob_nll: 2-D GPU probabilities");
  TORCH_CHECK(probs.scalar_type() == at::kFloat || probs.scalar_type() == at::kBFloat16, "prob_nll: dtype");
  req(labels, at::kLong, "labels");
  TORCH_CHECK(labels.numel() == probs.size(0) && probs.size(0) < (1LL << 31), "prob_nll: labels size");
  const int B = probs.size(0), NC = probs.size(1);
  const bool per_row = g_deterministic;
  auto loss = per_row ? torch::empty({2, B}, probs.options().dtype(at::kFloat))
                      : torch::zeros({2}, probs.options().dtype(at::kFloat));
  torch::Tensor dp;
  if (want_grad) dp = torch::empty({B, NC}, probs.options().dtype(at::kFloat));
  if (B > 0)
    check_hip(zoo_prob_nll(probs.data_ptr(), probs.scalar_type() == at::kFloat, labels.data_ptr<int64_t>(),
                           loss.data_ptr<float>(), loss.data_ptr<float>() + (per_row ? B : 1),
                           want_grad ? dp.data_ptr<float>() : nullptr, B, NC, (float)eps, (int)ignore_index,
                           per_row ? 1 : 0, cur_stream()),
              "prob_nll");
  if (per_row) loss = loss.sum(1);
  if (want_grad) return {loss, dp};
  return {loss};
}

// [loss, count] of prob_nll in two native launches (block partials + an ordered fold): the loss
// is already the mean (size_average) or the sum, so the caller launches nothing else
torch::Tensor prob_nll_mean(torch::Tensor probs, torch::Tensor labels, double eps, int64_t ignore_index,
                            bool size_average) {
  TORCH_CHECK(probs.is_cuda() && probs.is_contiguous() && probs.dim() == 2, "prob_nll_mean: 2-D GPU probabilities");
  TORCH_CHECK(probs.scalar_type() == at::kFloat || probs.scalar_type() == at::kBFloat16, "prob_nll_mean: dtype");
  req(labels, at::kLong, "labels");
  TORCH_CHECK(labels.numel() == probs.size(0) && probs.size(0) < (1LL << 31), "prob_nll_mean: labels size");
  const int B = probs.size(0), NC = probs.size(1);
  auto part = torch::empty({256}, probs.options().dtype(at::kFloat));
  auto out = torch::empty({2}, probs.options().dtype(at::kFloat));
  check_hip(zoo_prob_nll_mean(probs.data_ptr(), probs.scalar_type() == at::kFloat, labels.data_ptr<int64_t>(),
                              part.data_ptr<float>(), out.data_ptr<float>(), B, NC, (float)eps, (int)ignore_index,
                              size_average ? 1 : 0, cur_stream()),
            "prob_nll_mean");
  return out;
}

// scaled gradient of prob_nll: dprobs = -g / (max(count, 1) * clamp(p[label])) at the label
torch::Tensor prob_nll_grad(torch::Tensor probs, torch::Tensor labels, torch::Tensor g, torch::Tensor count,
                            double eps, int64_t ignore_index) {
  TORCH_CHECK(probs.is_cuda() && probs.is_contiguous() && probs.dim() == 2, "prob_nll_grad: 2-D GPU probabilities");
  TORCH_CHECK(probs.scalar_type() == at::kFloat || probs.scalar_type() == at::kBFloat16, "prob_nll_grad: dtype");
  req(labels, at::kLong, "labels");
  req(g, at::kFloat, "g");
  req(count, at::kFloat, "count");
  TORCH_CHECK(g.numel() >= 1 && count.numel() >= 1, "prob_nll_grad: scalar g / count");
  TORCH_CHECK(labels.numel() == probs.size(0) && probs.size(0) < (1LL << 31), "prob_nll_grad: labels size");
  const int B = probs.size(0), NC = probs.size(1);
  auto dp = torch::empty({B, NC}, probs.options().dtype(at::kFloat));
  if (B > 0)
    check_hip(zoo_prob_nll_grad(probs.data_ptr(), probs.scalar_type() == at::kFloat, labels.data_ptr<int64_t>(),
                                g.data_ptr<float>(), count.data_ptr<float>(), dp.data_ptr<float>(), B, NC, (float)eps,
                                (int)ignore_index, cur_stream()),
              "prob_nll_grad");
  return dp;
}

void check_flat(const torch::Tensor& t, const char* n, int64_t numel) {
  req(t, at::kFloat, n);
  TORCH_CHECK(t.numel() == numel, n, " numel mismatch");
}

void sgd(torch::Tensor p, torch::Tensor g, c10::optional<torch::Tensor> mom, c10::optional<torch::Tensor> pbf,
         double lr, double momentum, double dampening, double wd, bool nesterov, double gscale, bool first_step) {
  req(p, at::kFloat, "p");
  check_flat(g, "g", p.numel());
  if (momentum != 0.0) {
    TORCH_CHECK(mom.has_value(), "sgd: momentum buffer required");
    check_flat(*mom, "mom", p.numel());
  }
  if (pbf.has_value() && pbf->defined()) {
    req(*pbf, at::kBFloat16, "pbf");
    TORCH_CHECK(pbf->numel() == p.numel(), "pbf numel");
  }
  check_hip(zoo_sgd(p.data_ptr<float>(), g.data_ptr<float>(), opt_ptr<float>(mom), opt_ptr<void>(pbf), p.numel(),
                    lr, momentum, dampening, wd, nesterov, gscale, first_step, cur_stream()),
            "sgd");
}

void adam(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, c10::optional<torch::Tensor> pbf,
          double lr, double b1, double b2, double eps, double wd, double bc1, double bc2, double gscale,
          bool decoupled) {
  req(p, at::kFloat, "p");
  check_flat(g, "g", p.numel());
  check_flat(m, "m", p.numel());
  check_flat(v, "v", p.numel());
  if (pbf.has_value() && pbf->defined()) {
    req(*pbf, at::kBFloat16, "pbf");
    TORCH_CHECK(pbf->numel() == p.numel(), "pbf numel");
  }
  check_hip(zoo_adam(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(),
                     opt_ptr<void>(pbf), p.numel(), lr, b1, b2, eps, wd, bc1, bc2, gscale, decoupled, cur_stream()),
            "adam");
}

void adaptive(torch::Tensor p, torch::Tensor g, torch::Tensor s1, c10::optional<torch::Tensor> s2,
              c10::optional<torch::Tensor> pbf, int kind, double lr, double rho, double rho2, double eps, double wd,
              double bc1, double gscale) {
  req(p, at::kFloat, "p");
  check_flat(g, "g", p.numel());
  check_flat(s1, "s1", p.numel());
  if (kind >= 2) {
    TORCH_CHECK(s2.has_value(), "adaptive: second state required");
    check_flat(*s2, "s2", p.numel());
  }
  if (pbf.has_value() && pbf->defined()) {
    req(*pbf, at::kBFloat16, "pbf");
    TORCH_CHECK(pbf->numel() == p.numel(), "pbf numel");
  }
  check_hip(zoo_adaptive(p.data_ptr<float>(), g.data_ptr<float>(), s1.data_ptr<float>(), opt_ptr<float>(s2),
                         opt_ptr<void>(pbf), p.numel(), kind, lr, rho, rho2, eps, wd, bc1, gscale, cur_stream()),
            "adaptive");
}

torch::Tensor sumsq(torch::Tensor g) {
  req(g, at::kFloat, "g");
  auto out = torch::zeros({1}, g.options());
  check_hip(zoo_sumsq(g.data_ptr<float>(), g.numel(), out.data_ptr<float>(), cur_stream()), "sumsq");
  return out;
}

void clip(torch::Tensor g, double lo, double hi, c10::optional<torch::Tensor> norm_sq, double max_norm) {
  req(g, at::kFloat, "g");
  check_hip(zoo_clip(g.data_ptr<float>(), g.numel(), lo, hi, opt_ptr<float>(norm_sq), max_norm, cur_stream()),
            "clip");
}

static bool xp_defined(const c10::optional<torch::Tensor>& x) { return x.has_value() && x->defined(); }

// out = x + dropout(a, p) (x optional), bf16, mask regenerated from `seed` (counter-based hash)
torch::Tensor dropout_add(torch::Tensor a, c10::optional<torch::Tensor> x, double p, int64_t seed) {
  req(a, at::kBFloat16, "a");
  TORCH_CHECK(a.numel() % 8 == 0, "dropout_add: numel must be a multiple of 8");
  if (x.has_value() && x->defined()) {
    req(*x, at::kBFloat16, "x");
    TORCH_CHECK(x->sizes() == a.sizes(), "dropout_add: shape mismatch");
  }
  TORCH_CHECK(a.is_contiguous() && (!xp_defined(x) || x->is_contiguous()), "dropout_add: contiguous inputs");
  check_al16(a.data_ptr(), "a");
  if (xp_defined(x)) check_al16(x->data_ptr(), "x");
  auto out = torch::empty_like(a);
  const void* xp = (x.has_value() && x->defined()) ? x->data_ptr() : nullptr;
  check_hip(zoo_dropout_add(a.data_ptr(), xp, out.data_ptr(), (size_t)a.numel(), (float)p, (uint64_t)seed,
                            cur_stream()),
            "dropout_add");
  return out;
}

// [N, C<=4, H, W] fp32 -> [N, Hs, Ws, 16] bf16 space-to-depth(2) of the input zero-padded by `pad`
torch::Tensor nchw_to_s2d(torch::Tensor x, int pad) {
  req(x, at::kFloat, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(1) <= 4, "nchw_to_s2d: [N, C<=4, H, W] input");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Hs = (H + 2 * pad + 1) / 2, Ws = (W + 2 * pad + 1) / 2;
  auto y = torch::empty({N, Hs, Ws, 16}, x.options().dtype(at::kBFloat16));
  if (y.numel() == 0) return y;
  check_hip(zoo_nchw_to_s2d(x.data_ptr<float>(), y.data_ptr(), N, C, H, W, pad, Hs, Ws, cur_stream()),
            "nchw_to_s2d");
  return y;
}

// uint8 NHWC images -> normalised s2d(2) NHWC bf16 (x * scale[c] + shift[c]), the stem's input
torch::Tensor nhwc_u8_to_s2d(torch::Tensor x, int pad, std::vector<double> scale, std::vector<double> shift) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kByte && x.is_contiguous(), "nhwc_u8_to_s2d: contiguous uint8 GPU");
  TORCH_CHECK(x.dim() == 4 && x.size(3) <= 4, "nhwc_u8_to_s2d: [N, H, W, C<=4] input");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK((int)scale.size() >= C && (int)shift.size() >= C, "nhwc_u8_to_s2d: one scale / shift per channel");
  float sc[4] = {0.f, 0.f, 0.f, 0.f}, sh[4] = {0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < C; ++c) { sc[c] = (float)scale[c]; sh[c] = (float)shift[c]; }
  const int Hs = (H + 2 * pad + 1) / 2, Ws = (W + 2 * pad + 1) / 2;
  auto y = torch::empty({N, Hs, Ws, 16}, x.options().dtype(at::kBFloat16));
  if (y.numel() == 0) return y;
  check_hip(zoo_nhwc_u8_to_s2d(x.data_ptr(), y.data_ptr(), N, C, H, W, pad, Hs, Ws, sc, sh, cur_stream()),
            "nhwc_u8_to_s2d");
  return y;
}

// BatchNorm-backward prologue (kernels/bnfold.hip, pw.hip PRO). Coefficients of a unit's BN
// backward dy = A g + B y + Cc from its final sums [0, 2K) (sum g, sum g * xhat) over M rows:
// returns coef [3K] = A | B | Cc; dgamma += S2, dbeta += S1 when given.
torch::Tensor bnfold_coef(torch::Tensor gamma, torch::Tensor mean, torch::Tensor inv, torch::Tensor sums, int64_t M,
                          c10::optional<torch::Tensor> dgamma, c10::optional<torch::Tensor> dbeta) {
  req(gamma, at::kFloat, "gamma");
  req(mean, at::kFloat, "mean");
  req(inv, at::kFloat, "inv");
  req(sums, at::kFloat, "sums");
  const int64_t K = gamma.numel();
  TORCH_CHECK(K > 0 && mean.numel() == K && inv.numel() == K && sums.numel() >= 2 * K && M > 0,
              "bnfold_coef: per-channel vectors of length K, sums >= 2K");
  for (auto* t : {&dgamma, &dbeta})
    if (t->has_value()) {
      req(**t, at::kFloat, "dgamma/dbeta");
      TORCH_CHECK((*t)->numel() == K, "bnfold_coef: dgamma / dbeta length");
    }
  auto coef = torch::empty({3 * K}, gamma.options());
  check_hip(zoo_bnfold_coef((int)K, gamma.data_ptr<float>(), mean.data_ptr<float>(), inv.data_ptr<float>(),
                            sums.data_ptr<float>(), (long long)M, coef.data_ptr<float>(), opt_ptr<float>(dgamma),
                            opt_ptr<float>(dbeta), cur_stream()),
            "bnfold_coef");
  return coef;
}

// dy = A g + B y + Cc materialised ([..., K] bf16, K % 8 == 0)
void bnpro_apply(torch::Tensor g, torch::Tensor y, torch::Tensor coef, torch::Tensor out) {
  req(g, at::kBFloat16, "g");
  req(y, at::kBFloat16, "y");
  req(coef, at::kFloat, "coef");
  req(out, at::kBFloat16, "out");
  const int64_t K = g.size(-1);
  TORCH_CHECK(K % 8 == 0 && y.numel() == g.numel() && out.numel() == g.numel() && coef.numel() == 3 * K,
              "bnpro_apply: g / y / out [..., K % 8 == 0], coef [3K]");
  check_hip(zoo_bnpro_apply(g.data_ptr(), y.data_ptr(), coef.data_ptr<float>(), out.data_ptr(), g.numel(), (int)K, 0,
                            cur_stream()),
            "bnpro_apply");
}

torch::Tensor nchw_to_nhwc(torch::Tensor x, int cpad) {
  req(x, at::kFloat, "x");
  TORCH_CHECK(x.dim() == 4, "nchw_to_nhwc: 4-D input");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(cpad >= C, "nchw_to_nhwc: cpad < C");
  auto y = torch::empty({N, H, W, cpad}, x.options().dtype(at::kBFloat16));
  check_hip(zoo_nchw_to_nhwc(x.data_ptr<float>(), y.data_ptr(), N, C, H, W, cpad, cur_stream()), "nchw_to_nhwc");
  return y;
}

void bf16_to_f32(torch::Tensor x, torch::Tensor y, bool accumulate) {
  req(x, at::kBFloat16, "x");
  req(y, at::kFloat, "y");
  TORCH_CHECK(x.numel() == y.numel(), "bf16_to_f32 numel");
  check_hip(zoo_bf16_to_f32(x.data_ptr(), y.data_ptr<float>(), x.numel(), accumulate, cur_stream()), "bf16_to_f32");
}

// out32 / out16 [cb] = scale * sum_c recv[c][:] with fp32 accumulation (recv bf16 [nchunks * cb])
void sum_chunks_bf16(torch::Tensor recv, int64_t nchunks, c10::optional<torch::Tensor> out32,
                     c10::optional<torch::Tensor> out16, double scale) {
  req(recv, at::kBFloat16, "recv");
  TORCH_CHECK(nchunks >= 1 && recv.numel() % nchunks == 0, "sum_chunks_bf16: recv not divisible into chunks");
  const int64_t cb = recv.numel() / nchunks;
  TORCH_CHECK(cb % 8 == 0, "sum_chunks_bf16: chunk must be a multiple of 8");
  check_al16(recv.data_ptr(), "recv");
  float* o32 = nullptr;
  void* o16 = nullptr;
  if (out32.has_value() && out32->defined()) {
    req(*out32, at::kFloat, "out32");
    TORCH_CHECK(out32->numel() == cb, "out32 size");
    check_al16(out32->data_ptr(), "out32");
    o32 = out32->data_ptr<float>();
  }
  if (out16.has_value() && out16->defined()) {
    req(*out16, at::kBFloat16, "out16");
    TORCH_CHECK(out16->numel() == cb, "out16 size");
    check_al16(out16->data_ptr(), "out16");
    o16 = out16->data_ptr();
  }
  TORCH_CHECK(o32 || o16, "sum_chunks_bf16: no output");
  check_hip(zoo_sum_chunks_bf16(recv.data_ptr(), (int)nchunks, (size_t)cb, o32, o16, (float)scale, cur_stream()),
            "sum_chunks_bf16");
}

void f32_to_bf16(torch::Tensor x, torch::Tensor y) {
  req(x, at::kFloat, "x");
  req(y, at::kBFloat16, "y");
  TORCH_CHECK(x.numel() == y.numel(), "f32_to_bf16 numel");
  check_hip(zoo_f32_to_bf16(x.data_ptr<float>(), y.data_ptr(), x.numel(), cur_stream()), "f32_to_bf16");
}

torch::Tensor add_bf16(torch::Tensor a, torch::Tensor b) {
  req(a, at::kBFloat16, "a");
  req(b, at::kBFloat16, "b");
  TORCH_CHECK(a.numel() == b.numel() && a.numel() % 8 == 0, "add_bf16: equal sizes, multiple of 8");
  auto y = torch::empty_like(a);
  check_hip(zoo_add_bf16(a.data_ptr(), b.data_ptr(), y.data_ptr(), a.numel(), cur_stream()), "add_bf16");
  return y;
}

bool is_f32(const torch::Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "expected float32 or bfloat16");
  return t.scalar_type() == at::kFloat;
}

std::vector<torch::Tensor> layernorm_fwd(torch::Tensor x, c10::optional<torch::Tensor> g,
                                         c10::optional<torch::Tensor> b, double eps) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "layernorm: contiguous GPU input");
  const bool f32 = is_f32(x);
  const int D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0, "layernorm: last dim must be a multiple of 8");
  if (g.has_value() && g->defined()) { req(*g, at::kFloat, "gamma"); TORCH_CHECK(g->numel() == D, "gamma size"); }
  if (b.has_value() && b->defined()) { req(*b, at::kFloat, "beta"); TORCH_CHECK(b->numel() == D, "beta size"); }
  auto y = torch::empty_like(x);
  auto mean = torch::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = torch::empty({rows}, x.options().dtype(at::kFloat));
  check_hip(zoo_layernorm_fwd(x.data_ptr(), f32, opt_ptr<float>(g), opt_ptr<float>(b), y.data_ptr(),
                              mean.data_ptr<float>(), rstd.data_ptr<float>(), (int)rows, D, (float)eps, cur_stream()),
            "layernorm_fwd");
  return {y, mean, rstd};
}

// y = LayerNorm(s), s = x + dropout(a, p, seed) (the Transformer residual): {y, s, mean, rstd}
std::vector<torch::Tensor> dropout_add_layernorm_fwd(torch::Tensor a, torch::Tensor x, torch::Tensor g, torch::Tensor b,
                                                     double eps, double p, int64_t seed) {
  req(a, at::kBFloat16, "a");
  req(x, at::kBFloat16, "x");
  req(g, at::kFloat, "gamma");
  req(b, at::kFloat, "beta");
  TORCH_CHECK(a.is_contiguous() && x.is_contiguous() && a.sizes() == x.sizes(), "dropout_add_layernorm: contiguous same-shape a / x");
  const int D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 2048 && g.numel() == D && b.numel() == D, "dropout_add_layernorm: D % 8 == 0, D <= 2048");
  TORCH_CHECK(rows < (1LL << 31), "dropout_add_layernorm: too many rows");
  auto y = torch::empty_like(x);
  auto s = torch::empty_like(x);
  auto mean = torch::empty({rows}, x.options().dtype(at::kFloat));
  auto rstd = torch::empty({rows}, x.options().dtype(at::kFloat));
  check_hip(zoo_dropout_add_layernorm_fwd(a.data_ptr(), x.data_ptr(), g.data_ptr<float>(), b.data_ptr<float>(),
                                          s.data_ptr(), y.data_ptr(), mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                          (int)rows, D, (float)eps, (float)p, (uint64_t)seed, cur_stream()),
            "dropout_add_layernorm_fwd");
  return {y, s, mean, rstd};
}

torch::Tensor layernorm_bwd(torch::Tensor dy, torch::Tensor x, c10::optional<torch::Tensor> g, torch::Tensor mean,
                            torch::Tensor rstd, c10::optional<torch::Tensor> dg, c10::optional<torch::Tensor> db,
                            c10::optional<torch::Tensor> dy2) {
  TORCH_CHECK(dy.is_cuda() && dy.is_contiguous() && x.is_contiguous(), "layernorm_bwd: contiguous GPU tensors");
  TORCH_CHECK(dy.scalar_type() == x.scalar_type() && dy.numel() == x.numel(), "layernorm_bwd: dy/x mismatch");
  const bool f32 = is_f32(x);
  const int D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && mean.numel() == rows && rstd.numel() == rows, "layernorm_bwd: shapes");
  if (dg.has_value() && dg->defined()) { req(*dg, at::kFloat, "dgamma"); TORCH_CHECK(dg->numel() == D, "dg"); }
  if (db.has_value() && db->defined()) { req(*db, at::kFloat, "dbeta"); TORCH_CHECK(db->numel() == D, "db"); }
  auto dx = torch::empty_like(x);
  torch::Tensor part;
  const size_t pf = zoo_layernorm_bwd_part_floats((int)rows, D, f32);
  if (pf && (opt_ptr<float>(dg) || opt_ptr<float>(db))) part = torch::empty({(int64_t)pf}, mean.options());
  // dy2: a second gradient of the output (the residual consumer's, GradAdd), summed inside the
  // kernel where it supports it, else added here first
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    TORCH_CHECK(dy2->is_cuda() && dy2->is_contiguous() && dy2->scalar_type() == dy.scalar_type() &&
                    dy2->numel() == dy.numel(), "layernorm_bwd: dy2 must match dy");
    d2 = dy2->data_ptr();
  }
  hipError_t e = zoo_layernorm_bwd(dy.data_ptr(), x.data_ptr(), f32, opt_ptr<float>(g), mean.data_ptr<float>(),
                                   rstd.data_ptr<float>(), dx.data_ptr(), opt_ptr<float>(dg), opt_ptr<float>(db),
                                   (int)rows, D, part.defined() ? part.data_ptr<float>() : nullptr, d2, cur_stream());
  if (e == hipErrorNotSupported && d2) {
    (void)hipGetLastError();
    auto dys = dy.add(*dy2);
    e = zoo_layernorm_bwd(dys.data_ptr(), x.data_ptr(), f32, opt_ptr<float>(g), mean.data_ptr<float>(),
                          rstd.data_ptr<float>(), dx.data_ptr(), opt_ptr<float>(dg), opt_ptr<float>(db), (int)rows,
                          D, part.defined() ? part.data_ptr<float>() : nullptr, nullptr, cur_stream());
  }
  check_hip(e, "layernorm_bwd");
  return dx;
}

// backward of dropout_add_layernorm_fwd: {dx, da} (da = keep * dx / (1 - p), the dropout
// branch's gradient, written by the same kernel where the bf16 v2 backward applies)
std::vector<torch::Tensor> layernorm_bwd_drop(torch::Tensor dy, torch::Tensor x, torch::Tensor g, torch::Tensor mean,
                                              torch::Tensor rstd, c10::optional<torch::Tensor> dg,
                                              c10::optional<torch::Tensor> db, c10::optional<torch::Tensor> dy2,
                                              double p, int64_t seed) {
  req(dy, at::kBFloat16, "dy");
  req(x, at::kBFloat16, "x");
  req(g, at::kFloat, "gamma");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.numel() == x.numel(), "layernorm_bwd_drop: dy / x");
  const int D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && mean.numel() == rows && rstd.numel() == rows && g.numel() == D, "layernorm_bwd_drop: shapes");
  if (dg.has_value() && dg->defined()) { req(*dg, at::kFloat, "dgamma"); TORCH_CHECK(dg->numel() == D, "dg"); }
  if (db.has_value() && db->defined()) { req(*db, at::kFloat, "dbeta"); TORCH_CHECK(db->numel() == D, "db"); }
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    TORCH_CHECK(dy2->is_contiguous() && dy2->scalar_type() == at::kBFloat16 && dy2->numel() == dy.numel(),
                "layernorm_bwd_drop: dy2 must match dy");
    d2 = dy2->data_ptr();
  }
  auto dx = torch::empty_like(x);
  auto da = torch::empty_like(x);
  torch::Tensor part;
  const size_t pf = zoo_layernorm_bwd_part_floats((int)rows, D, 0);
  if (pf && (opt_ptr<float>(dg) || opt_ptr<float>(db))) part = torch::empty({(int64_t)pf}, mean.options());
  hipError_t e = zoo_layernorm_bwd_drop(dy.data_ptr(), x.data_ptr(), g.data_ptr<float>(), mean.data_ptr<float>(),
                                        rstd.data_ptr<float>(), dx.data_ptr(), da.data_ptr(), opt_ptr<float>(dg),
                                        opt_ptr<float>(db), (int)rows, D, part.defined() ? part.data_ptr<float>() : nullptr,
                                        d2, (float)p, (uint64_t)seed, cur_stream());
  if (e == hipErrorNotSupported) {
    (void)hipGetLastError();
    dx = layernorm_bwd(dy, x, g, mean, rstd, dg, db, dy2);
    da = dropout_add(dx, c10::nullopt, p, seed);
    return {dx, da};
  }
  check_hip(e, "layernorm_bwd_drop");
  return {dx, da};
}

// LayerNorm backward with the dgamma / dbeta fold left to the caller (layernorm_fold, typically
// on the weight-gradient side stream): {dx, da (dropout branch, or empty), part}. bf16 v2 path
// only (raises otherwise: the caller uses layernorm_bwd / layernorm_bwd_drop).
std::vector<torch::Tensor> layernorm_bwd_split(torch::Tensor dy, torch::Tensor x, torch::Tensor g, torch::Tensor mean,
                                               torch::Tensor rstd, c10::optional<torch::Tensor> dy2, double p,
                                               int64_t seed, bool drop) {
  req(dy, at::kBFloat16, "dy");
  req(x, at::kBFloat16, "x");
  req(g, at::kFloat, "gamma");
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.numel() == x.numel(), "layernorm_bwd_split: dy / x");
  const int D = x.size(-1);
  const int64_t rows = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && mean.numel() == rows && rstd.numel() == rows && g.numel() == D, "layernorm_bwd_split: shapes");
  TORCH_CHECK(zoo_layernorm_bwd_v2_blocks((int)rows, D, 0) > 0 && (reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) == 0,
              "layernorm_bwd_split: needs the bf16 v2 backward");
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    TORCH_CHECK(dy2->is_contiguous() && dy2->scalar_type() == at::kBFloat16 && dy2->numel() == dy.numel(),
                "layernorm_bwd_split: dy2 must match dy");
    d2 = dy2->data_ptr();
  }
  auto dx = torch::empty_like(x);
  torch::Tensor da = drop ? torch::empty_like(x) : torch::empty({0}, x.options());
  auto part = torch::empty({(int64_t)zoo_layernorm_bwd_part_floats((int)rows, D, 0)}, mean.options());
  // dg / db pointers only switch the partial output on; nothing is folded into them here
  float* dummy = part.data_ptr<float>();
  zoo_layernorm_defer_fold(1);
  hipError_t e;
  if (drop)
    e = zoo_layernorm_bwd_drop(dy.data_ptr(), x.data_ptr(), g.data_ptr<float>(), mean.data_ptr<float>(),
                               rstd.data_ptr<float>(), dx.data_ptr(), da.data_ptr(), dummy, dummy, (int)rows, D,
                               part.data_ptr<float>(), d2, (float)p, (uint64_t)seed, cur_stream());
  else
    e = zoo_layernorm_bwd(dy.data_ptr(), x.data_ptr(), 0, g.data_ptr<float>(), mean.data_ptr<float>(),
                          rstd.data_ptr<float>(), dx.data_ptr(), dummy, dummy, (int)rows, D, part.data_ptr<float>(), d2,
                          cur_stream());
  zoo_layernorm_defer_fold(0);
  check_hip(e, "layernorm_bwd_split");
  return {dx, da, part};
}

void layernorm_fold(torch::Tensor part, int64_t rows, int64_t D, c10::optional<torch::Tensor> dg,
                    c10::optional<torch::Tensor> db) {
  req(part, at::kFloat, "part");
  if (dg.has_value() && dg->defined()) { req(*dg, at::kFloat, "dgamma"); TORCH_CHECK(dg->numel() == D, "dg"); }
  if (db.has_value() && db->defined()) { req(*db, at::kFloat, "dbeta"); TORCH_CHECK(db->numel() == D, "db"); }
  TORCH_CHECK((size_t)part.numel() >= zoo_layernorm_bwd_part_floats((int)rows, (int)D, 0), "layernorm_fold: part size");
  check_hip(zoo_layernorm_fold(part.data_ptr<float>(), (int)rows, (int)D, opt_ptr<float>(dg), opt_ptr<float>(db),
                               cur_stream()),
            "layernorm_fold");
}

torch::Tensor embedding_fwd(torch::Tensor table, torch::Tensor idx, int64_t pad) {
  TORCH_CHECK(table.is_cuda() && table.is_contiguous() && table.dim() == 2, "embedding: 2-D GPU table");
  req(idx, at::kLong, "indices");
  const bool f32 = is_f32(table);
  const int D = table.size(1), V = table.size(0);
  TORCH_CHECK((f32 ? D % 4 : D % 8) == 0, "embedding: row must be a multiple of 16 bytes");
  auto out_shape = idx.sizes().vec();
  out_shape.push_back(D);
  auto out = torch::empty(out_shape, table.options());
  check_hip(zoo_embedding_fwd(table.data_ptr(), f32, idx.data_ptr<int64_t>(), out.data_ptr(), (int)idx.numel(), D, V,
                              pad, cur_stream()),
            "embedding_fwd");
  return out;
}

void embedding_bwd(torch::Tensor dout, torch::Tensor idx, torch::Tensor gtable, int64_t pad, double scale) {
  TORCH_CHECK(dout.is_cuda() && dout.is_contiguous(), "embedding_bwd: contiguous GPU grad");
  req(idx, at::kLong, "indices");
  req(gtable, at::kFloat, "grad table");
  const bool f32 = is_f32(dout);
  const int D = gtable.size(1), V = gtable.size(0);
  TORCH_CHECK(dout.numel() == idx.numel() * (int64_t)D, "embedding_bwd: shape");
  check_hip(zoo_embedding_bwd(dout.data_ptr(), f32, idx.data_ptr<int64_t>(), gtable.data_ptr<float>(),
                              (int)idx.numel(), D, V, pad, (float)scale, cur_stream()),
            "embedding_bwd");
}


// ---- pointwise.hip: activations, dropout, elementwise objectives, AUC histogram, box decode ----
static bool pw_f32(const torch::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), what, " must be a contiguous GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, what, " must be fp32 or bf16");
  return t.scalar_type() == at::kFloat;
}

// dy empty: y = act(x); else dx = dy * act'(x)
torch::Tensor act_fwd_bwd(torch::Tensor x, c10::optional<torch::Tensor> dy, int64_t kind, double alpha) {
  const bool f32 = pw_f32(x, "x");
  TORCH_CHECK(kind >= 0 && kind <= 15, "act: unknown activation code");
  const void* dp = nullptr;
  if (dy.has_value() && dy->defined()) {
    TORCH_CHECK(pw_f32(*dy, "dy") == f32 && dy->numel() == x.numel(), "act: dy must match x");
    dp = dy->data_ptr();
  }
  auto out = torch::empty_like(x);
  if (x.numel() > 0)
    check_hip(zoo_act(x.data_ptr(), dp, out.data_ptr(), x.numel(), f32, (int)kind, (float)alpha, cur_stream()),
              "act");
  return out;
}

torch::Tensor dropout_fwd(torch::Tensor x, double p, int64_t seed) {
  const bool f32 = pw_f32(x, "x");
  TORCH_CHECK(p >= 0.0 && p <= 1.0, "dropout: p must be in [0, 1]");
  auto out = torch::empty_like(x);
  if (x.numel() > 0)
    check_hip(zoo_dropout(x.data_ptr(), out.data_ptr(), x.numel(), f32, (float)p, (uint64_t)seed, cur_stream()),
              "dropout");
  return out;
}

// -> (loss fp32 scalar, grad like pred); w = per-element weight (1/N for mean)
std::vector<torch::Tensor> loss_fwd(torch::Tensor pred, torch::Tensor target, int64_t kind, double beta, double w,
                                    bool want_grad) {
  const bool f32 = pw_f32(pred, "pred");
  TORCH_CHECK(pw_f32(target, "target") == f32 && target.numel() == pred.numel(), "loss: target must match pred");
  TORCH_CHECK(kind >= 0 && kind <= 10, "loss: unknown loss code");
  auto loss = torch::zeros({}, pred.options().dtype(at::kFloat));
  torch::Tensor grad;
  if (want_grad) grad = torch::empty_like(pred);
  if (pred.numel() > 0)
    check_hip(zoo_loss(pred.data_ptr(), target.data_ptr(), want_grad ? grad.data_ptr() : nullptr,
                       loss.data_ptr<float>(), pred.numel(), f32, (int)kind, (float)beta, (float)w, cur_stream()),
              "loss");
  if (want_grad) return {loss, grad};
  return {loss};
}

torch::Tensor auc_hist(torch::Tensor score, torch::Tensor label, int64_t nbins, double lo, double hi) {
  req(score, at::kFloat, "score");
  req(label, at::kFloat, "label");
  TORCH_CHECK(score.numel() == label.numel(), "auc_hist: score/label size");
  TORCH_CHECK(nbins >= 1 && nbins <= 16384, "auc_hist: 1 <= nbins <= 16384");
  auto hist = torch::zeros({2, nbins}, score.options());
  if (score.numel() > 0)
    check_hip(zoo_auc_hist(score.data_ptr<float>(), label.data_ptr<float>(), hist.data_ptr<float>(), score.numel(),
                           (int)nbins, (float)lo, (float)hi, cur_stream()),
              "auc_hist");
  return hist;
}

torch::Tensor box_decode(torch::Tensor loc, torch::Tensor priors, double v0, double v1, bool clip) {
  req(loc, at::kFloat, "loc");
  req(priors, at::kFloat, "priors");
  TORCH_CHECK(loc.dim() == 3 && loc.size(2) == 4 && priors.dim() == 2 && priors.size(1) == 4 &&
                  priors.size(0) == loc.size(1), "box_decode: loc [N,P,4], priors [P,4]");
  TORCH_CHECK(loc.numel() < (1LL << 31), "box_decode: too large");
  auto boxes = torch::empty_like(loc);
  if (loc.numel() > 0)
    check_hip(zoo_box_decode(loc.data_ptr<float>(), priors.data_ptr<float>(), boxes.data_ptr<float>(),
                             (int)loc.size(0), (int)loc.size(1), (float)v0, (float)v1, clip, cur_stream()),
              "box_decode");
  return boxes;
}

// ---- static-int8 implicit-GEMM conv (qconv.hip) ----
// x: int8 NHWC [N,H,W,C] (C % 16 == 0); w: int8 [K, ldb] rows of [R][S][C]; colscale/bias fp32 [K]
// (already divided by the output scale); resid: int8 [N,P,Q,K] scaled by rscale. Output int8
// (saturating round) or bf16 (out_bf16).
torch::Tensor qconv(torch::Tensor x, torch::Tensor w, int R, int S, int sh, int sw, int ph, int pw,
                    torch::Tensor colscale, c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> resid,
                    double rscale, bool relu, bool out_bf16, c10::optional<torch::Tensor> rvec, int64_t qflags) {
  // int8 or OCP fp8 e4m3 operands (the fp8 twin of the kernel); both operands the same format
  const bool fp8 = x.scalar_type() == at::kFloat8_e4m3fn;
  const auto qt = fp8 ? at::kFloat8_e4m3fn : at::kChar;
  req(x, qt, "x");
  req(w, qt, "w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 2, "qconv: x NHWC 4-D, w 2-D [K, ldb]");
  const int C = x.size(3), K = w.size(0), ldb = w.size(1);
  TORCH_CHECK(C % 16 == 0, "qconv: input channels must be a multiple of 16, got ", C);
  TORCH_CHECK(K % 8 == 0, "qconv: output channels must be a multiple of 8, got ", K);
  TORCH_CHECK(ldb % 16 == 0 && ldb >= R * S * C, "qconv: bad weight leading dim ", ldb);
  TORCH_CHECK(R >= 1 && S >= 1 && sh >= 1 && sw >= 1 && ph >= 0 && pw >= 0, "qconv: bad geometry");
  ConvGeom g = make_geom(x, K, R, S, sh, sw, ph, pw, 1, 1, 1, 1, ldb);
  TORCH_CHECK(g.P > 0 && g.Q > 0, "qconv: empty output");
  TORCH_CHECK((int64_t)g.N * g.H * g.W * g.C < (1LL << 31) && (int64_t)g.M * K < (1LL << 31),
              "qconv: tensor too large for 32-bit indexing");
  g.omap = 0; g.stat_slots = 0;
  req(colscale, at::kFloat, "colscale");
  TORCH_CHECK(colscale.numel() == K, "qconv: colscale must be [K]");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == K, "qconv: bias must be [K]");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  if (resid.has_value() && resid->defined()) {
    req(*resid, qt, "resid");
    TORCH_CHECK(resid->numel() == (int64_t)g.M * K, "qconv: resid must match the output");
    rp = resid->data_ptr();
  }
  const float* rv = nullptr;   // per-channel residual scale s_resid[c] / s_out[c] (overrides rscale)
  if (rvec.has_value() && rvec->defined()) {
    req(*rvec, at::kFloat, "rvec");
    TORCH_CHECK(rvec->numel() == K, "qconv: rvec must be [K]");
    rv = rvec->data_ptr<float>();
  }
  // qflags (int8 only): 1 input, 2 output, 4 residual offset-coded unsigned (qconv.hip QF_*)
  TORCH_CHECK(qflags >= 0 && qflags < 8 && (!fp8 || qflags == 0), "qconv: qflags are int8-only bits 0..2");
  TORCH_CHECK(!(qflags & 2) || (relu && !out_bf16), "qconv: an unsigned int8 output needs relu and an int8 output");
  auto y = torch::empty({g.N, g.P, g.Q, K}, x.options().dtype(out_bf16 ? at::kBFloat16 : qt));
  check_hip(zoo_qconv(x.data_ptr(), w.data_ptr(), y.data_ptr(), colscale.data_ptr<float>(), bp, rp, (float)rscale, rv,
                      &g, relu, out_bf16, fp8 ? 1 : 0, (int)qflags, cur_stream()),
            "qconv");
  return y;
}

// inv_vec (optional): one inverse scale per channel of the NHWC tensor (C = last dim, C % 16 == 0)
static const float* chan_vec(const c10::optional<torch::Tensor>& v, const torch::Tensor& x, const char* what) {
  if (!v.has_value() || !v->defined()) return nullptr;
  req(*v, at::kFloat, what);
  TORCH_CHECK(v->numel() == x.size(-1) && x.size(-1) % 16 == 0, what, ": one value per channel, C % 16 == 0");
  return v->data_ptr<float>();
}

torch::Tensor quantize_i8(torch::Tensor x, double inv_scale, c10::optional<torch::Tensor> inv_vec, bool u8) {
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(x.numel() % 16 == 0, "quantize_i8: numel must be a multiple of 16");
  const float* iv = chan_vec(inv_vec, x, "quantize_i8 inv_vec");
  auto q = torch::empty(x.sizes(), x.options().dtype(at::kChar));
  check_hip(zoo_quantize_i8(x.data_ptr(), q.data_ptr(), x.numel(), (float)inv_scale, iv, (int)x.size(-1), u8 ? 1 : 0,
                            cur_stream()),
            "quantize_i8");
  return q;
}

torch::Tensor quantize_f8(torch::Tensor x, double inv_scale, c10::optional<torch::Tensor> inv_vec) {
  req(x, at::kBFloat16, "x");
  TORCH_CHECK(x.numel() % 16 == 0, "quantize_f8: numel must be a multiple of 16");
  const float* iv = chan_vec(inv_vec, x, "quantize_f8 inv_vec");
  auto q = torch::empty(x.sizes(), x.options().dtype(at::kFloat8_e4m3fn));
  check_hip(zoo_quantize_f8(x.data_ptr(), q.data_ptr(), x.numel(), (float)inv_scale, iv, (int)x.size(-1), cur_stream()),
            "quantize_f8");
  return q;
}

torch::Tensor gap_i8(torch::Tensor x, double scale, c10::optional<torch::Tensor> svec, bool u8) {
  const bool fp8 = x.scalar_type() == at::kFloat8_e4m3fn;
  req(x, fp8 ? at::kFloat8_e4m3fn : at::kChar, "x");
  TORCH_CHECK(x.dim() == 4 && x.size(3) % 8 == 0, "gap_i8: NHWC with C % 8 == 0");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  const float* sv = nullptr;
  if (svec.has_value() && svec->defined()) {
    req(*svec, at::kFloat, "svec");
    TORCH_CHECK(svec->numel() == C, "gap_i8: svec must be [C]");
    sv = svec->data_ptr<float>();
  }
  auto y = torch::empty({N, C}, x.options().dtype(at::kBFloat16));
  TORCH_CHECK(!(fp8 && u8), "gap_i8: the unsigned code is int8-only");
  check_hip(zoo_gap_i8(x.data_ptr(), y.data_ptr(), N, HW, C, (float)scale, sv, fp8 ? 1 : 0, u8 ? 1 : 0, cur_stream()),
            "gap_i8");
  return y;
}

// ---- HK10: embedding bag / sparse linear (sparse.hip) ----
// Bags: offsets [B+1] (CSR over ids) or, when offsets is empty, a dense [B, L] id matrix.
// ids outside [0, V) or == pad are skipped in-kernel; offsets are clamped to [0, nnz).
std::vector<torch::Tensor> embedding_bag_fwd(torch::Tensor table, torch::Tensor ids, torch::Tensor offsets, int64_t L,
                                             c10::optional<torch::Tensor> wts, int64_t mode, double max_norm,
                                             int64_t pad) {
  req(table, at::kFloat, "table");
  req(ids, at::kLong, "ids");
  TORCH_CHECK(table.dim() == 2, "embedding_bag: 2-D table");
  TORCH_CHECK(mode >= 0 && mode <= 2, "embedding_bag: mode 0 sum / 1 mean / 2 sqrtn");
  const int64_t nnz = ids.numel();
  int64_t B;
  const int64_t* op = nullptr;
  if (offsets.numel() > 0) {
    req(offsets, at::kLong, "offsets");
    B = offsets.numel() - 1;
    op = offsets.data_ptr<int64_t>();
  } else {
    TORCH_CHECK(L > 0 && nnz % L == 0, "embedding_bag: dense ids need L > 0 dividing numel");
    B = nnz / L;
  }
  const float* wp = nullptr;
  if (wts.has_value() && wts->defined()) {
    req(*wts, at::kFloat, "per-id weights");
    TORCH_CHECK(wts->numel() == nnz, "embedding_bag: weights must match ids");
    wp = wts->data_ptr<float>();
  }
  const int D = table.size(1), V = table.size(0);
  TORCH_CHECK(B < (1LL << 31) && D > 0, "embedding_bag: shape");
  auto out = torch::empty({B, (int64_t)D}, table.options());
  auto scale = torch::empty({B}, table.options());
  if (B > 0)
    check_hip(zoo_embedding_bag_fwd(table.data_ptr<float>(), ids.data_ptr<int64_t>(), op, (int)L, wp,
                                    out.data_ptr<float>(), scale.data_ptr<float>(), (int)B, D, V, nnz, pad, (int)mode,
                                    (float)max_norm, cur_stream()),
              "embedding_bag_fwd");
  return {out, scale};
}

void embedding_bag_bwd(torch::Tensor dout, torch::Tensor table, torch::Tensor ids, torch::Tensor offsets, int64_t L,
                       c10::optional<torch::Tensor> wts, torch::Tensor scale, torch::Tensor gtable, double max_norm,
                       int64_t pad) {
  req(dout, at::kFloat, "dout");
  req(table, at::kFloat, "table");
  req(ids, at::kLong, "ids");
  req(scale, at::kFloat, "bag scale");
  req(gtable, at::kFloat, "grad table");
  TORCH_CHECK(gtable.sizes() == table.sizes(), "embedding_bag_bwd: grad table shape");
  const int64_t B = dout.size(0);
  const int D = table.size(1), V = table.size(0);
  TORCH_CHECK(dout.dim() == 2 && dout.size(1) == D && scale.numel() == B, "embedding_bag_bwd: shapes");
  const int64_t* op = nullptr;
  if (offsets.numel() > 0) {
    req(offsets, at::kLong, "offsets");
    TORCH_CHECK(offsets.numel() == B + 1, "embedding_bag_bwd: offsets");
    op = offsets.data_ptr<int64_t>();
  } else {
    TORCH_CHECK(ids.numel() == B * L, "embedding_bag_bwd: dense ids");
  }
  const float* wp = nullptr;
  if (wts.has_value() && wts->defined()) {
    req(*wts, at::kFloat, "per-id weights");
    TORCH_CHECK(wts->numel() == ids.numel(), "embedding_bag_bwd: weights");
    wp = wts->data_ptr<float>();
  }
  if (B > 0)
    check_hip(zoo_embedding_bag_bwd(dout.data_ptr<float>(), table.data_ptr<float>(), ids.data_ptr<int64_t>(), op,
                                    (int)L, wp, scale.data_ptr<float>(), gtable.data_ptr<float>(), (int)B, D, V,
                                    ids.numel(), pad, (float)max_norm, cur_stream()),
              "embedding_bag_bwd");
}

// y [B, O] = CSR(crow, col, val) [B, IN] . W[O, IN]^T + bias
torch::Tensor sparse_linear_fwd(torch::Tensor crow, torch::Tensor col, torch::Tensor val, torch::Tensor W,
                                c10::optional<torch::Tensor> bias) {
  req(crow, at::kLong, "crow");
  req(col, at::kLong, "col");
  req(val, at::kFloat, "values");
  req(W, at::kFloat, "weight");
  TORCH_CHECK(W.dim() == 2 && col.numel() == val.numel(), "sparse_linear: shapes");
  const int64_t B = crow.numel() - 1;
  const int O = W.size(0), IN = W.size(1);
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == O, "sparse_linear: bias");
    bp = bias->data_ptr<float>();
  }
  auto y = torch::empty({B, (int64_t)O}, W.options());
  if (B > 0 && O > 0)
    check_hip(zoo_sparse_linear_fwd(crow.data_ptr<int64_t>(), col.data_ptr<int64_t>(), val.data_ptr<float>(),
                                    W.data_ptr<float>(), bp, y.data_ptr<float>(), (int)B, O, IN, col.numel(),
                                    cur_stream()),
              "sparse_linear_fwd");
  return y;
}

// dW [O, IN] += sum_j val_j * dy[row_j] (x) e_{col_j};  db [O] += column sums of dy
void sparse_linear_bwd(torch::Tensor row, torch::Tensor col, torch::Tensor val, torch::Tensor dy, torch::Tensor dW,
                       c10::optional<torch::Tensor> db) {
  req(row, at::kLong, "row");
  req(col, at::kLong, "col");
  req(val, at::kFloat, "values");
  req(dy, at::kFloat, "dy");
  req(dW, at::kFloat, "dW");
  TORCH_CHECK(row.numel() == col.numel() && col.numel() == val.numel() && dy.dim() == 2 && dW.dim() == 2 &&
                  dW.size(0) == dy.size(1), "sparse_linear_bwd: shapes");
  float* dbp = nullptr;
  if (db.has_value() && db->defined()) {
    req(*db, at::kFloat, "db");
    TORCH_CHECK(db->numel() == dy.size(1), "sparse_linear_bwd: db");
    dbp = db->data_ptr<float>();
  }
  if (dy.size(0) > 0)
    check_hip(zoo_sparse_linear_bwd(row.data_ptr<int64_t>(), col.data_ptr<int64_t>(), val.data_ptr<float>(),
                                    dy.data_ptr<float>(), dW.data_ptr<float>(), dbp, col.numel(), (int)dy.size(0),
                                    (int)dy.size(1), (int)dW.size(1), cur_stream()),
              "sparse_linear_bwd");
}

// uint8 [N, Hi, Wi, C] (C in 1..4) -> resized + normalized image batch:
// layout 0 -> fp32 [N, C, Ho, Wo]; layout 1 -> bf16 [N, Ho, Wo, 4] (zero-padded channels)
torch::Tensor resize_normalize(torch::Tensor in, int64_t Ho, int64_t Wo, std::vector<double> mean,
                               std::vector<double> stdv, bool swap_rb, int64_t layout) {
  req(in, at::kByte, "image");
  TORCH_CHECK(in.dim() == 4, "image batch must be [N, H, W, C]");
  const int N = in.size(0), Hi = in.size(1), Wi = in.size(2), C = in.size(3);
  TORCH_CHECK(C >= 1 && C <= 4, "1..4 channels supported");
  TORCH_CHECK(Ho > 0 && Wo > 0 && Hi > 0 && Wi > 0, "bad image size");
  TORCH_CHECK(layout == 0 || layout == 1, "layout must be 0 (NCHW f32) or 1 (NHWC4 bf16)");
  float m[3] = {0.f, 0.f, 0.f}, sd[3] = {1.f, 1.f, 1.f};
  for (size_t i = 0; i < 3 && i < mean.size(); ++i) m[i] = (float)mean[i];
  for (size_t i = 0; i < 3 && i < stdv.size(); ++i) sd[i] = (float)stdv[i];
  if (mean.size() == 1) m[1] = m[2] = m[0];
  if (stdv.size() == 1) sd[1] = sd[2] = sd[0];
  for (int i = 0; i < 3; ++i) TORCH_CHECK(sd[i] != 0.f, "std must be non-zero");
  torch::Tensor out = layout == 0
      ? torch::empty({N, C, Ho, Wo}, in.options().dtype(at::kFloat))
      : torch::empty({N, Ho, Wo, 4}, in.options().dtype(at::kBFloat16));
  if (N == 0) return out;
  check_hip(zoo_resize_normalize(in.data_ptr(), out.data_ptr(), N, Hi, Wi, C, (int)Ho, (int)Wo, m, sd,
                                 swap_rb ? 1 : 0, (int)layout, cur_stream()),
            "resize_normalize");
  return out;
}



// GPU half of the JPEG decoder: geometry g = [N, ncomp, w, h, hmax, vmax, hs0..2, vs0..2, bw0..2, bh0..2,
// boff0..2, total] (zoo/feature/image/jpeg.py builds it from csrc/runtime/jpeg.cpp's batch output)
static zoo::JpegGeom jpeg_geom(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 22, "jpeg geometry: 22 ints");
  zoo::JpegGeom g;
  g.N = v[0]; g.ncomp = v[1]; g.w = v[2]; g.h = v[3]; g.hmax = v[4]; g.vmax = v[5];
  for (int c = 0; c < 3; ++c) {
    g.hs[c] = v[6 + c]; g.vs[c] = v[9 + c]; g.bw[c] = v[12 + c]; g.bh[c] = v[15 + c]; g.boff[c] = v[18 + c];
  }
  g.total = v[21];
  TORCH_CHECK(g.N > 0 && (g.ncomp == 1 || g.ncomp == 3) && g.w > 0 && g.h > 0 && g.hmax >= 1 && g.vmax >= 1,
              "jpeg geometry: header");
  long blocks = 0;
  for (int c = 0; c < g.ncomp; ++c) {
    TORCH_CHECK(g.hs[c] >= 1 && g.hs[c] <= g.hmax && g.vs[c] >= 1 && g.vs[c] <= g.vmax, "jpeg geometry: sampling");
    TORCH_CHECK(g.boff[c] == blocks, "jpeg geometry: component offsets");
    // the padded grid must cover the component (the kernels index it unchecked)
    TORCH_CHECK((long)g.bw[c] * 8 >= ((long)g.w * g.hs[c] + g.hmax - 1) / g.hmax &&
                    (long)g.bh[c] * 8 >= ((long)g.h * g.vs[c] + g.vmax - 1) / g.vmax,
                "jpeg geometry: block grid smaller than the component");
    blocks += (long)g.bw[c] * g.bh[c];
  }
  TORCH_CHECK(blocks == g.total, "jpeg geometry: total blocks");
  return g;
}

torch::Tensor jpeg_idct(torch::Tensor coef, torch::Tensor qt, std::vector<int64_t> geom) {
  const auto g = jpeg_geom(geom);
  req(coef, at::kShort, "jpeg coef");
  req(qt, at::kInt, "jpeg qt");
  TORCH_CHECK(coef.dim() == 3 && coef.size(0) == g.N && coef.size(1) == g.total && coef.size(2) == 64,
              "jpeg coef [N, total, 64]");
  TORCH_CHECK(qt.dim() == 3 && qt.size(0) == g.N && qt.size(1) == g.ncomp && qt.size(2) == 64, "jpeg qt [N, ncomp, 64]");
  auto planes = torch::empty({(int64_t)g.N, (int64_t)g.total * 64}, coef.options().dtype(at::kByte));
  check_hip(zoo_jpeg_idct(coef.data_ptr<int16_t>(), qt.data_ptr<int32_t>(), planes.data_ptr<uint8_t>(), &g,
                          cur_stream()),
            "jpeg_idct");
  return planes;
}

torch::Tensor jpeg_color_resize(torch::Tensor planes, std::vector<int64_t> geom, int64_t Ho, int64_t Wo,
                                std::vector<double> mean, std::vector<double> stdv, bool swap_rb, int64_t layout) {
  const auto g = jpeg_geom(geom);
  req(planes, at::kByte, "jpeg planes");
  TORCH_CHECK(planes.numel() == (int64_t)g.N * g.total * 64, "jpeg planes size");
  TORCH_CHECK(layout >= 0 && layout <= 2, "layout 0 (NCHW f32), 1 (NHWC4 bf16) or 2 (RGB uint8)");
  if (layout == 2) TORCH_CHECK(Ho == g.h && Wo == g.w, "layout 2 is the decoded image (no resize)");
  TORCH_CHECK(Ho > 0 && Wo > 0, "bad output size");
  float m[3] = {0.f, 0.f, 0.f}, sd[3] = {1.f, 1.f, 1.f};
  for (size_t i = 0; i < 3 && i < mean.size(); ++i) m[i] = (float)mean[i];
  for (size_t i = 0; i < 3 && i < stdv.size(); ++i) sd[i] = (float)stdv[i];
  if (mean.size() == 1) m[1] = m[2] = m[0];
  if (stdv.size() == 1) sd[1] = sd[2] = sd[0];
  for (int i = 0; i < 3; ++i) TORCH_CHECK(sd[i] != 0.f, "std must be non-zero");
  torch::Tensor out;
  if (layout == 0) out = torch::empty({(int64_t)g.N, 3, Ho, Wo}, planes.options().dtype(at::kFloat));
  else if (layout == 1) out = torch::empty({(int64_t)g.N, Ho, Wo, 4}, planes.options().dtype(at::kBFloat16));
  else out = torch::empty({(int64_t)g.N, Ho, Wo, 3}, planes.options());
  check_hip(zoo_jpeg_color_resize(planes.data_ptr<uint8_t>(), out.data_ptr(), &g, (int)Ho, (int)Wo, m, sd,
                                  swap_rb ? 1 : 0, (int)layout, cur_stream()),
            "jpeg_color_resize");
  return out;
}

// Y[M, N] = epilogue(A[M, K] . B[N, K]^T) on the 256x256 LDS-DMA kernel (gemm256.hip).
torch::Tensor gemm(torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> bias,
                   c10::optional<torch::Tensor> resid, c10::optional<torch::Tensor> stats, int64_t act, bool out_f32,
                   bool out_bf16, c10::optional<torch::Tensor> bz, c10::optional<torch::Tensor> by,
                   c10::optional<torch::Tensor> bmean, c10::optional<torch::Tensor> binv,
                   c10::optional<torch::Tensor> bsums) {
  req(a, at::kBFloat16, "a");
  req(b, at::kBFloat16, "b");
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm: 2-D operands");
  const int M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm: K mismatch");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0, "gemm: K and N must be multiples of 8");
  TORCH_CHECK(out_f32 || out_bf16, "gemm: no output requested");
  GemmGeom g{M, N, K, K, K, N};
  torch::Tensor y, yf;
  if (out_bf16) y = torch::empty({M, N}, a.options());
  if (out_f32) yf = torch::empty({M, N}, a.options().dtype(at::kFloat));
  if (bias.has_value() && bias->defined()) {
    req(*bias, at::kFloat, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm: bias shape");
  }
  if (resid.has_value() && resid->defined()) {
    req(*resid, at::kBFloat16, "resid");
    TORCH_CHECK(resid->numel() == (int64_t)M * N, "gemm: resid shape");
  }
  if (stats.has_value() && stats->defined()) {
    req(*stats, at::kFloat, "stats");
    TORCH_CHECK(stats->numel() == 2 * N && out_bf16, "gemm: stats must be [2*N] with bf16 output");
  }
  BwdStats bs{nullptr, nullptr, nullptr, nullptr, nullptr};
  if (bsums.has_value() && bsums->defined()) {
    req(*bsums, at::kFloat, "bsums");
    TORCH_CHECK(bsums->numel() == 2 * N && out_bf16, "gemm: bsums must be [2*N] with bf16 output");
    TORCH_CHECK(by.has_value() && bmean.has_value() && binv.has_value(), "gemm: bstats needs y/mean/inv");
    req(*by, at::kBFloat16, "by");
    TORCH_CHECK(by->numel() == (int64_t)M * N, "gemm: by shape");
    if (bz.has_value() && bz->defined()) {
      req(*bz, at::kBFloat16, "bz");
      TORCH_CHECK(bz->numel() == (int64_t)M * N, "gemm: bz shape");
    }
    bs = BwdStats{opt_ptr<void>(bz), by->data_ptr(), bmean->data_ptr<float>(), binv->data_ptr<float>(),
                  bsums->data_ptr<float>()};
  }
  if (M == 0) return out_bf16 ? y : yf;
  check_hip(zoo_gemm256(a.data_ptr(), b.data_ptr(), out_bf16 ? y.data_ptr() : nullptr,
                        out_f32 ? yf.data_ptr<float>() : nullptr, opt_ptr<float>(bias), opt_ptr<void>(resid),
                        opt_ptr<float>(stats), &g, (int)act, bs.sums ? &bs : nullptr, cur_stream()),
            "gemm256");
  return out_bf16 ? y : yf;
}


// ---- greedy NMS: boxes [N, 4] (x1, y1, x2, y2) fp32 already sorted by descending score ----
// The suppression bitmask is built on the GPU (detect.hip); the sequential greedy
// pass walks it on the host. Returns the kept row indices (int64, ascending = score order).
torch::Tensor nms_sorted(torch::Tensor boxes, double thresh, int64_t max_keep) {
  req(boxes, at::kFloat, "boxes");
  TORCH_CHECK(boxes.dim() == 2 && boxes.size(1) == 4, "nms: boxes must be [N, 4]");
  const int n = boxes.size(0);
  const int words = (n + 63) / 64;
  if (n == 0) return torch::empty({0}, boxes.options().dtype(at::kLong));
  auto mask = torch::empty({(int64_t)n * words}, boxes.options().dtype(at::kLong));
  check_hip(zoo_nms_mask(boxes.data_ptr<float>(), n, (float)thresh,
                         reinterpret_cast<unsigned long long*>(mask.data_ptr<int64_t>()), cur_stream()),
            "nms_mask");
  auto hm = mask.cpu();
  const unsigned long long* m = reinterpret_cast<const unsigned long long*>(hm.data_ptr<int64_t>());
  std::vector<unsigned long long> removed(words, 0ull);
  std::vector<int64_t> keep;
  keep.reserve(std::min<int64_t>(n, max_keep > 0 ? max_keep : n));
  for (int i = 0; i < n; ++i) {
    if (removed[i / 64] & (1ull << (i % 64))) continue;
    keep.push_back(i);
    if (max_keep > 0 && (int64_t)keep.size() >= max_keep) break;
    const unsigned long long* row = m + (size_t)i * words;
    for (int w = i / 64; w < words; ++w) removed[w] |= row[w];
  }
  auto out = torch::from_blob(keep.data(), {(int64_t)keep.size()}, torch::kLong).clone();
  return out.to(boxes.device());
}

// ---- fused attention: q [B,H,L,D], k/v [B,H,S,D] bf16, optional additive key mask [B,S] fp32 ----
void attn_check(const torch::Tensor& q, const torch::Tensor& k, const torch::Tensor& v,
                const c10::optional<torch::Tensor>& mask) {
  req(q, at::kBFloat16, "q");
  req(k, at::kBFloat16, "k");
  req(v, at::kBFloat16, "v");
  TORCH_CHECK(q.dim() == 4 && k.dim() == 4 && v.dim() == 4, "attention: q/k/v must be [B,H,T,D]");
  TORCH_CHECK(k.sizes() == v.sizes(), "attention: k and v shapes differ");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(1) == k.size(1) && q.size(3) == k.size(3),
              "attention: q/k batch, heads or head_dim differ");
  const int64_t D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "attention: head_dim must be 64 or 128");
  TORCH_CHECK(q.size(0) * q.size(1) < 65536, "attention: B*H must be < 65536");
  if (mask.has_value() && mask->defined()) {
    req(*mask, at::kFloat, "mask");
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == q.size(0) && mask->size(1) == k.size(2),
                "attention: mask must be [B, S]");
  }
}

std::vector<torch::Tensor> attn_fwd(torch::Tensor q, torch::Tensor k, torch::Tensor v,
                                    c10::optional<torch::Tensor> mask, bool causal, double pdrop, int64_t seed) {
  TORCH_CHECK(pdrop >= 0.0 && pdrop < 1.0, "attn_fwd: dropout p must be in [0, 1)");
  attn_check(q, k, v, mask);
  const int B = q.size(0), H = q.size(1), L = q.size(2), S = k.size(2), D = q.size(3);
  auto o = torch::empty_like(q);
  auto lse = torch::empty({B, H, L}, q.options().dtype(at::kFloat));
  if (q.numel() == 0) return {o, lse};
  check_hip(zoo_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), opt_ptr<float>(mask), o.data_ptr(),
                         lse.data_ptr<float>(), B, H, L, S, D, (float)(1.0 / std::sqrt((double)D)), causal,
                         nullptr, (float)pdrop, (uint64_t)seed, cur_stream()),
            "attn_fwd");
  return {o, lse};
}

// Forward attention on strided [B, H, T, D] views (D contiguous, 16-byte aligned rows), e.g. the
// q/k/v slices of one packed [B, T, 3, H, D] projection, so no per-head copies are made. With
// out_blhd the output is written as [B, L, H, D] (the layout the output projection reads).
std::vector<torch::Tensor> attn_fwd_strided(torch::Tensor q, torch::Tensor k, torch::Tensor v,
                                            c10::optional<torch::Tensor> mask, bool causal, bool out_blhd,
                                            double pdrop, int64_t seed) {
  TORCH_CHECK(pdrop >= 0.0 && pdrop < 1.0, "attn_fwd_strided: dropout p must be in [0, 1)");
  for (const torch::Tensor* t : {&q, &k, &v}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16, "attention: q/k/v must be bf16 GPU tensors");
    TORCH_CHECK(t->dim() == 4 && t->stride(3) == 1, "attention: head_dim must be the contiguous dim");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0 && t->stride(2) % 8 == 0 &&
                    t->stride(1) % 8 == 0 && t->stride(0) % 8 == 0,
                "attention: rows must be 16-byte aligned");
  }
  TORCH_CHECK(k.sizes() == v.sizes(), "attention: k and v shapes differ");
  TORCH_CHECK(q.size(0) == k.size(0) && q.size(1) == k.size(1) && q.size(3) == k.size(3),
              "attention: q/k batch, heads or head_dim differ");
  const int B = q.size(0), H = q.size(1), L = q.size(2), S = k.size(2), D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "attention: head_dim must be 64 or 128");
  TORCH_CHECK(B * H < 65536, "attention: B*H must be < 65536");
  if (mask.has_value() && mask->defined()) {
    req(*mask, at::kFloat, "mask");
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == B && mask->size(1) == S, "attention: mask must be [B, S]");
  }
  auto o = out_blhd ? torch::empty({B, L, H, D}, q.options()) : torch::empty({B, H, L, D}, q.options());
  auto lse = torch::empty({B, H, L}, q.options().dtype(at::kFloat));
  if (q.numel() == 0) return {o, lse};
  const long st[12] = {(long)q.stride(0), (long)q.stride(1), (long)q.stride(2), (long)k.stride(0),
                       (long)k.stride(1), (long)k.stride(2), (long)v.stride(0), (long)v.stride(1),
                       (long)v.stride(2), (long)o.stride(0), (long)(out_blhd ? o.stride(2) : o.stride(1)),
                       (long)(out_blhd ? o.stride(1) : o.stride(2))};
  check_hip(zoo_attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), opt_ptr<float>(mask), o.data_ptr(),
                         lse.data_ptr<float>(), B, H, L, S, D, (float)(1.0 / std::sqrt((double)D)), causal, st,
                         (float)pdrop, (uint64_t)seed, cur_stream()),
            "attn_fwd_strided");
  return {o, lse};
}

std::vector<torch::Tensor> attn_bwd(torch::Tensor dout, torch::Tensor q, torch::Tensor k, torch::Tensor v,
                                    c10::optional<torch::Tensor> mask, torch::Tensor o, torch::Tensor lse,
                                    bool causal, double pdrop, int64_t seed) {
  TORCH_CHECK(pdrop >= 0.0 && pdrop < 1.0, "attn_bwd: dropout p must be in [0, 1)");
  attn_check(q, k, v, mask);
  req(dout, at::kBFloat16, "dout");
  req(o, at::kBFloat16, "o");
  req(lse, at::kFloat, "lse");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes(), "attn_bwd: dout/o shape");
  const int B = q.size(0), H = q.size(1), L = q.size(2), S = k.size(2), D = q.size(3);
  TORCH_CHECK(lse.numel() == (int64_t)B * H * L, "attn_bwd: lse shape");
  auto dq = torch::empty_like(q);
  auto dk = torch::empty_like(k);
  auto dv = torch::empty_like(v);
  auto delta = torch::empty({B, H, L}, q.options().dtype(at::kFloat));
  if (q.numel() == 0 || k.numel() == 0) return {dq.zero_(), dk.zero_(), dv.zero_()};
  check_hip(zoo_attn_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), opt_ptr<float>(mask),
                         o.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(),
                         dv.data_ptr(), B, H, L, S, D, (float)(1.0 / std::sqrt((double)D)), causal, nullptr,
                         (float)pdrop, (uint64_t)seed, cur_stream()),
            "attn_bwd");
  return {dq, dk, dv};
}

// Backward on strided [B, H, T, D] views (the training counterpart of attn_fwd_strided): q/k/v
// are slices of the packed projection, dout/o any [B, H, L, D] views, and dq/dk/dv are written
// into caller-provided views (slices of the packed projection's gradient).
void attn_bwd_strided(torch::Tensor dout, torch::Tensor q, torch::Tensor k, torch::Tensor v,
                      c10::optional<torch::Tensor> mask, torch::Tensor o, torch::Tensor lse, torch::Tensor dq,
                      torch::Tensor dk, torch::Tensor dv, bool causal, double pdrop, int64_t seed) {
  TORCH_CHECK(pdrop >= 0.0 && pdrop < 1.0, "attn_bwd_strided: dropout p must be in [0, 1)");
  for (const torch::Tensor* t : {&dout, &q, &k, &v, &o, &dq, &dk, &dv}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16, "attn_bwd_strided: bf16 GPU tensors");
    TORCH_CHECK(t->dim() == 4 && t->stride(3) == 1, "attn_bwd_strided: head_dim must be the contiguous dim");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0 && t->stride(2) % 8 == 0 &&
                    t->stride(1) % 8 == 0 && t->stride(0) % 8 == 0,
                "attn_bwd_strided: rows must be 16-byte aligned");
  }
  const int B = q.size(0), H = q.size(1), L = q.size(2), S = k.size(2), D = q.size(3);
  TORCH_CHECK(D == 64 || D == 128, "attention: head_dim must be 64 or 128");
  TORCH_CHECK(B * H < 65536, "attention: B*H must be < 65536");
  TORCH_CHECK(k.sizes() == v.sizes() && dk.sizes() == k.sizes() && dv.sizes() == k.sizes(),
              "attn_bwd_strided: k/v/dk/dv shapes differ");
  TORCH_CHECK(dout.sizes() == q.sizes() && o.sizes() == q.sizes() && dq.sizes() == q.sizes(),
              "attn_bwd_strided: dout/o/dq shape");
  TORCH_CHECK(k.size(0) == B && k.size(1) == H && k.size(3) == D, "attn_bwd_strided: q/k batch, heads or dim");
  req(lse, at::kFloat, "lse");
  TORCH_CHECK(lse.is_contiguous() && lse.numel() == (int64_t)B * H * L, "attn_bwd_strided: lse shape");
  if (mask.has_value() && mask->defined()) {
    req(*mask, at::kFloat, "mask");
    TORCH_CHECK(mask->dim() == 2 && mask->size(0) == B && mask->size(1) == S, "attention: mask must be [B, S]");
  }
  if (q.numel() == 0 || k.numel() == 0) return;
  auto delta = torch::empty({B, H, L}, q.options().dtype(at::kFloat));
  long st[24];
  int n = 0;
  for (const torch::Tensor* t : {&q, &k, &v, &dout, &o, &dq, &dk, &dv})
    for (int d = 0; d < 3; ++d) st[n++] = (long)t->stride(d);
  check_hip(zoo_attn_bwd(dout.data_ptr(), q.data_ptr(), k.data_ptr(), v.data_ptr(), opt_ptr<float>(mask),
                         o.data_ptr(), lse.data_ptr<float>(), delta.data_ptr<float>(), dq.data_ptr(), dk.data_ptr(),
                         dv.data_ptr(), B, H, L, S, D, (float)(1.0 / std::sqrt((double)D)), causal, st,
                         (float)pdrop, (uint64_t)seed, cur_stream()),
            "attn_bwd_strided");
}


// ---- int8 quantized inference ----
torch::Tensor absmax(torch::Tensor x) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "absmax: contiguous GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "absmax: fp32 or bf16");
  auto out = torch::zeros({1}, x.options().dtype(at::kFloat));
  if (x.numel() == 0) return out;
  check_hip(zoo_absmax(x.data_ptr(), x.scalar_type() == at::kFloat, (size_t)x.numel(), out.data_ptr<float>(),
                       cur_stream()),
            "absmax");
  return out;
}

torch::Tensor im2col_q8(torch::Tensor x, torch::Tensor amax, int R, int S, int sh, int sw, int ph, int pw, int P,
                        int Q, int Kp) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.dim() == 4, "im2col_q8: contiguous NHWC GPU tensor");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "im2col_q8: fp32 or bf16");
  req(amax, at::kFloat, "amax");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(Kp % 16 == 0 && Kp >= R * S * C, "im2col_q8: Kp must be a multiple of 16 covering R*S*C");
  TORCH_CHECK(P > 0 && Q > 0 && R > 0 && S > 0 && sh > 0 && sw > 0, "im2col_q8: bad geometry");
  auto q = torch::empty({(int64_t)N * P * Q, Kp}, x.options().dtype(at::kChar));
  if (q.numel() == 0) return q;
  check_hip(zoo_im2col_q8(x.data_ptr(), x.scalar_type() == at::kFloat, amax.data_ptr<float>(), q.data_ptr(), N, H,
                          W, C, R, S, P, Q, sh, sw, ph, pw, Kp, cur_stream()),
            "im2col_q8");
  return q;
}

torch::Tensor qgemm(torch::Tensor a, torch::Tensor w, torch::Tensor amax, torch::Tensor wscale,
                    c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> resid, bool relu, bool out_f32) {
  req(a, at::kChar, "a");
  req(w, at::kChar, "w");
  req(amax, at::kFloat, "amax");
  req(wscale, at::kFloat, "wscale");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1), "qgemm: a [M,Kp], w [N,Kp]");
  const int M = a.size(0), N = w.size(0), Kp = a.size(1);
  TORCH_CHECK(Kp % 16 == 0, "qgemm: Kp must be a multiple of 16");
  TORCH_CHECK(wscale.numel() == N, "qgemm: wscale [N]");
  if (bias.has_value() && bias->defined()) { req(*bias, at::kFloat, "bias"); TORCH_CHECK(bias->numel() == N, "bias"); }
  if (resid.has_value() && resid->defined()) {
    req(*resid, at::kBFloat16, "resid");
    TORCH_CHECK(resid->numel() == (int64_t)M * N, "qgemm: resid [M,N]");
  }
  auto y = torch::empty({M, N}, a.options().dtype(out_f32 ? at::kFloat : at::kBFloat16));
  if (M == 0 || N == 0) return y;
  check_hip(zoo_qgemm(a.data_ptr(), w.data_ptr(), amax.data_ptr<float>(), wscale.data_ptr<float>(),
                      opt_ptr<float>(bias), opt_ptr<void>(resid), y.data_ptr(), M, N, Kp, relu, out_f32,
                      cur_stream()),
            "qgemm");
  return y;
}


// ---- persistent recurrent cells (rnn.hip): cell 0 SimpleRNN, 1 LSTM, 2 GRU ----
int rnn_gates(int64_t cell) {
  TORCH_CHECK(cell >= 0 && cell <= 3, "rnn: cell must be 0 (SimpleRNN), 1 (LSTM), 2 (GRU) or 3 (GRU reset-after)");
  return cell == 1 ? 4 : (cell >= 2 ? 3 : 1);
}

void rnn_check_state(const c10::optional<torch::Tensor>& s, int64_t B, int64_t H, const char* name) {
  if (s.has_value() && s->defined()) {
    req(*s, at::kFloat, name);
    TORCH_CHECK(s->dim() == 2 && s->size(0) == B && s->size(1) == H, "rnn: ", name, " must be [B, H]");
  }
}

void rnn_check_acts(int64_t act, int64_t iact) {
  TORCH_CHECK(act >= 0 && act <= 4 && iact >= 0 && iact <= 4, "rnn: unsupported activation code");
}

// xw [B, T, G*H] fp32 (bias included), u [G*H, H] bf16 -> {hseq [B,T,H], cT [B,H] (LSTM), cseq, gates}
std::vector<torch::Tensor> rnn_fwd(torch::Tensor xw, torch::Tensor u, c10::optional<torch::Tensor> h0,
                                   c10::optional<torch::Tensor> c0, int64_t cell, int64_t act, int64_t iact,
                                   bool save, c10::optional<torch::Tensor> bhn) {
  req(xw, at::kFloat, "xw");
  req(u, at::kBFloat16, "u");
  const int G = rnn_gates(cell);
  rnn_check_acts(act, iact);
  TORCH_CHECK(u.dim() == 2 && u.size(0) == G * u.size(1), "rnn_fwd: u must be [G*H, H]");
  const int64_t H = u.size(1);
  TORCH_CHECK(H == 32 || H == 64 || H == 128 || H == 256, "rnn_fwd: hidden size must be 32/64/128/256 (pad it)");
  TORCH_CHECK(xw.dim() == 3 && xw.size(2) == G * H, "rnn_fwd: xw must be [B, T, G*H]");
  const int64_t B = xw.size(0), T = xw.size(1);
  rnn_check_state(h0, B, H, "h0");
  rnn_check_state(c0, B, H, "c0");
  auto f32 = xw.options();
  auto hseq = torch::empty({B, T, H}, f32);
  torch::Tensor cT, cseq, gates;
  if (cell == 1) cT = torch::empty({B, H}, f32);
  if (save && (cell == 1 || cell == 3)) cseq = torch::empty({B, T, H}, f32);
  if (bhn.has_value() && bhn->defined()) {
    req(*bhn, at::kFloat, "bhn");
    TORCH_CHECK(cell == 3 && bhn->numel() == H, "rnn_fwd: bhn is the [H] candidate bias of the GRU_RA cell");
  }
  if (save && cell != 0) gates = torch::empty({B, T, G * H}, f32);
  zoo::RnnArgs a{};
  a.xw = xw.data_ptr<float>();
  a.u = u.data_ptr();
  a.h0 = opt_ptr<float>(h0);
  a.c0 = opt_ptr<float>(c0);
  a.hseq = hseq.data_ptr<float>();
  a.cseq = cseq.defined() ? cseq.data_ptr<float>() : nullptr;
  a.gates = gates.defined() ? gates.data_ptr<float>() : nullptr;
  a.cT = cT.defined() ? cT.data_ptr<float>() : nullptr;
  a.bhn = opt_ptr<float>(bhn);
  a.B = (int)B; a.T = (int)T; a.act = (int)act; a.iact = (int)iact;
  check_hip(zoo_rnn(&a, (int)cell, (int)H, 0, cur_stream()), "rnn_fwd");
  return {hseq, cT, cseq, gates};
}

// ut = U^T [H, G*H] bf16 -> {dgates [B,T,G*H] (= d xw), dh0 [B,H], dc0 [B,H] (LSTM)}
std::vector<torch::Tensor> rnn_bwd(c10::optional<torch::Tensor> dhseq, c10::optional<torch::Tensor> dcT,
                                   torch::Tensor ut, torch::Tensor hseq, c10::optional<torch::Tensor> cseq,
                                   c10::optional<torch::Tensor> gates, c10::optional<torch::Tensor> h0,
                                   c10::optional<torch::Tensor> c0, int64_t cell, int64_t act, int64_t iact) {
  req(ut, at::kBFloat16, "ut");
  req(hseq, at::kFloat, "hseq");
  const int G = rnn_gates(cell);
  rnn_check_acts(act, iact);
  TORCH_CHECK(ut.dim() == 2 && ut.size(1) == G * ut.size(0), "rnn_bwd: ut must be [H, G*H]");
  const int64_t H = ut.size(0);
  TORCH_CHECK(H == 32 || H == 64 || H == 128 || H == 256, "rnn_bwd: hidden size must be 32/64/128/256");
  TORCH_CHECK(hseq.dim() == 3 && hseq.size(2) == H, "rnn_bwd: hseq must be [B, T, H]");
  const int64_t B = hseq.size(0), T = hseq.size(1);
  if (dhseq.has_value() && dhseq->defined()) {
    req(*dhseq, at::kFloat, "dhseq");
    TORCH_CHECK(dhseq->sizes() == hseq.sizes(), "rnn_bwd: dhseq shape");
  }
  rnn_check_state(dcT, B, H, "dcT");
  rnn_check_state(h0, B, H, "h0");
  rnn_check_state(c0, B, H, "c0");
  if (cell == 1 || cell == 3) {
    TORCH_CHECK(cseq.has_value() && cseq->defined(), "rnn_bwd: LSTM / GRU_RA need the saved cseq");
    req(*cseq, at::kFloat, "cseq");
    TORCH_CHECK(cseq->sizes() == hseq.sizes(), "rnn_bwd: cseq shape");
  }
  if (cell != 0) {
    TORCH_CHECK(gates.has_value() && gates->defined(), "rnn_bwd: saved gates required");
    req(*gates, at::kFloat, "gates");
    TORCH_CHECK(gates->dim() == 3 && gates->size(0) == B && gates->size(1) == T && gates->size(2) == G * H,
                "rnn_bwd: gates shape");
  }
  auto f32 = hseq.options();
  auto dgates = torch::empty({B, T, G * H}, f32);
  auto dh0 = torch::empty({B, H}, f32);
  torch::Tensor dc0, dgn;
  if (cell == 1) dc0 = torch::empty({B, H}, f32);
  if (cell == 3) dgn = torch::empty({B, T, H}, f32);
  zoo::RnnArgs a{};
  a.u = ut.data_ptr();
  a.h0 = opt_ptr<float>(h0);
  a.c0 = opt_ptr<float>(c0);
  a.hseq = hseq.data_ptr<float>();
  a.cseq = opt_ptr<float>(cseq);
  a.gates = opt_ptr<float>(gates);
  a.dhseq = opt_ptr<float>(dhseq);
  a.dcT = opt_ptr<float>(dcT);
  a.dgates = dgates.data_ptr<float>();
  a.dh0 = dh0.data_ptr<float>();
  a.dc0 = dc0.defined() ? dc0.data_ptr<float>() : nullptr;
  a.dgn = dgn.defined() ? dgn.data_ptr<float>() : nullptr;
  a.B = (int)B; a.T = (int)T; a.act = (int)act; a.iact = (int)iact;
  check_hip(zoo_rnn(&a, (int)cell, (int)H, 1, cur_stream()), "rnn_bwd");
  return {dgates, dh0, dc0, dgn};
}

}  // namespace


// Fused NeuralCF forward / backward (kernels/ncf.hip).
//   t    = [tu, ti, tmu, tmi, w1, b1, w2, b2, w3, b3, wo, bo]   (empty tensor = absent)
//   dims = [eu, ei, em, h1, h2, h3, nc, id_off]
// forward (dprobs absent): returns probs [B, nc] fp32. backward: gradients are ADDED into
//   g = [gtu, gti, gtmu, gtmi, gw1, gb1, gw2, gb2, gw3, gb3, gwo, gbo] (fp32, empty = skip).
static bool has(const torch::Tensor& t) { return t.defined() && t.numel() > 0; }

static void ncf_req_w(const torch::Tensor& w, int64_t r, int64_t c, const char* what) {
  req(w, at::kFloat, what);
  TORCH_CHECK(w.numel() == r * c && (c == 1 || (w.dim() == 2 && w.size(0) == r && w.size(1) == c)), "ncf: ", what,
              " shape");
}

int64_t ncf_tier(std::vector<int64_t> d) {
  TORCH_CHECK(d.size() >= 7, "ncf_tier: dims");
  return zoo_ncf_tier(d[0], d[1], d[2], d[3], d[4], d[5], d[6]);
}

torch::Tensor ncf_fused(torch::Tensor ids, std::vector<torch::Tensor> t, std::vector<int64_t> dims,
                        c10::optional<torch::Tensor> dprobs, std::vector<torch::Tensor> g) {
  TORCH_CHECK(t.size() == 12 && dims.size() == 8, "ncf: 12 tensors, 8 dims");
  req(ids, at::kLong, "ncf ids");
  TORCH_CHECK(ids.dim() == 2 && ids.size(1) == 2 && ids.size(0) > 0 && ids.size(0) < (1LL << 31), "ncf: ids [B, 2]");
  const int eu = dims[0], ei = dims[1], em = dims[2], h1 = dims[3], h2 = dims[4], h3 = dims[5], nc = dims[6];
  TORCH_CHECK(zoo_ncf_tier(eu, ei, em, h1, h2, h3, nc) >= 0, "ncf: unsupported widths");
  const auto& tu = t[0];
  const auto& ti = t[1];
  TORCH_CHECK(tu.is_cuda() && (tu.scalar_type() == at::kBFloat16 || tu.scalar_type() == at::kFloat),
              "ncf: tables fp32 / bf16 on the GPU");
  const auto tdt = tu.scalar_type();
  const int align = tdt == at::kFloat ? 16 : 8;
  auto tab = [&](const torch::Tensor& x, int64_t rows, int e, const char* what) {
    req(x, tdt, what);
    TORCH_CHECK(x.dim() == 2 && x.size(1) == e && (rows < 0 || x.size(0) == rows) && x.size(0) < (1LL << 31),
                "ncf: ", what, " shape");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % align == 0, "ncf: ", what, " alignment");
  };
  tab(tu, -1, eu, "user table");
  tab(ti, -1, ei, "item table");
  if (em > 0) {
    tab(t[2], tu.size(0), em, "mf user table");
    tab(t[3], ti.size(0), em, "mf item table");
  }
  ncf_req_w(t[4], h1, eu + ei, "w1");
  ncf_req_w(t[6], h2, h1, "w2");
  ncf_req_w(t[8], h3, h2, "w3");
  ncf_req_w(t[10], nc, h3 + em, "wo");
  const int hb[4] = {h1, h2, h3, nc};
  for (int i = 0; i < 4; ++i)
    if (has(t[5 + 2 * i])) ncf_req_w(t[5 + 2 * i], hb[i], 1, "bias");
  zoo::NcfArgs a{};
  a.ids = ids.data_ptr<int64_t>();
  a.B = ids.size(0);
  a.id_off = dims[7];
  a.tu = tu.data_ptr();
  a.ti = ti.data_ptr();
  a.tmu = em > 0 ? t[2].data_ptr() : nullptr;
  a.tmi = em > 0 ? t[3].data_ptr() : nullptr;
  a.Vu = tu.size(0);
  a.Vi = ti.size(0);
  a.eu = eu; a.ei = ei; a.em = em; a.h1 = h1; a.h2 = h2; a.h3 = h3; a.nc = nc;
  auto fp = [&](int i) -> const float* { return has(t[i]) ? t[i].data_ptr<float>() : nullptr; };
  a.w1 = fp(4); a.b1 = fp(5); a.w2 = fp(6); a.b2 = fp(7); a.w3 = fp(8); a.b3 = fp(9); a.wo = fp(10); a.bo = fp(11);
  a.nwg = zoo_ncf_nwg(eu, ei, em, h1, h2, h3, nc);
  const int bf16 = tdt == at::kBFloat16;
  if (!dprobs.has_value() || !dprobs->defined()) {
    auto probs = torch::empty({a.B, nc}, ids.options().dtype(at::kFloat));
    a.probs = probs.data_ptr<float>();
    check_hip(zoo_ncf(&a, nullptr, bf16, cur_stream()), "ncf_fwd");
    return probs;
  }
  req(*dprobs, at::kFloat, "ncf dprobs");
  TORCH_CHECK(dprobs->dim() == 2 && dprobs->size(0) == a.B && dprobs->size(1) == nc, "ncf: dprobs [B, nc]");
  a.dprobs = dprobs->data_ptr<float>();
  TORCH_CHECK(g.size() == 12, "ncf: 12 gradient slots");
  auto gp = [&](int i, int64_t n) -> float* {
    if (!has(g[i])) return nullptr;
    req(g[i], at::kFloat, "ncf grad");
    TORCH_CHECK(g[i].numel() == n, "ncf: gradient ", i, " has ", g[i].numel(), " elements, expected ", n);
    return g[i].data_ptr<float>();
  };
  a.gtu = gp(0, tu.numel());
  a.gti = gp(1, ti.numel());
  a.gtmu = em > 0 ? gp(2, t[2].numel()) : nullptr;
  a.gtmi = em > 0 ? gp(3, t[3].numel()) : nullptr;
  float* dst[8] = {gp(4, (int64_t)h1 * (eu + ei)), gp(5, h1), gp(6, (int64_t)h2 * h1), gp(7, h2),
                   gp(8, (int64_t)h3 * h2), gp(9, h3), gp(10, (int64_t)nc * (h3 + em)), gp(11, nc)};
  const int grid = (a.B + 255) / 256;
  auto partial = torch::empty({grid, a.nwg}, ids.options().dtype(at::kFloat));
  a.partial = partial.data_ptr<float>();
  check_hip(zoo_ncf(&a, dst, bf16, cur_stream()), "ncf_bwd");
  return partial;
}

void register_comm(py::module& m);   // comm.cpp

PYBIND11_MODULE(_C, m) {
  register_comm(m);
  m.doc() = "zoo native gfx950 (MI355X) kernel library";
  m.def("resize_normalize", &resize_normalize);
  m.def("jpeg_idct", &jpeg_idct);
  m.def("jpeg_color_resize", &jpeg_color_resize);
  m.def("gemm", &gemm);
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("dh"), py::arg("dw"), py::arg("lh"), py::arg("lw"), py::arg("bias"), py::arg("resid"), py::arg("stats"), py::arg("act"), py::arg("out_f32"), py::arg("out_bf16"), py::arg("out_h"), py::arg("out_w"), py::arg("out"), py::arg("omap"), py::arg("bz"), py::arg("by"), py::arg("bmean"), py::arg("binv"), py::arg("bsums"),
        py::arg("bgamma") = py::none(), py::arg("bbeta") = py::none(), py::arg("pro_y") = py::none(),
        py::arg("pro_coef") = py::none(), py::arg("pro_dy") = py::none(), py::arg("resid_half") = false,
        py::arg("pro_fwd") = false, py::arg("pro_rcoef") = py::none(), py::arg("pro_mask") = py::none(),
        py::arg("act_pre") = py::none(), py::arg("by2") = py::none(), py::arg("bsums2") = py::none());
  m.def("bn_fwd_coef", [](torch::Tensor stats, torch::Tensor gamma, torch::Tensor beta, torch::Tensor rmean,
                          torch::Tensor rvar, torch::Tensor smean, torch::Tensor sinv, int64_t M, double eps,
                          double momentum) {
    const int C = gamma.numel();
    for (auto* t : {&stats, &gamma, &beta, &rmean, &rvar, &smean, &sinv}) req(*t, at::kFloat, "bn_fwd_coef vector");
    TORCH_CHECK(stats.numel() >= 2 * C && beta.numel() == C && rmean.numel() == C && rvar.numel() == C &&
                    smean.numel() == C && sinv.numel() == C && M > 0 && M < (1LL << 31),
                "bn_fwd_coef: sizes");
    auto coef = torch::empty({3 * (int64_t)C}, gamma.options());
    check_hip(zoo_bn_fwd_coef(stats.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                              rmean.data_ptr<float>(), rvar.data_ptr<float>(), smean.data_ptr<float>(),
                              sinv.data_ptr<float>(), coef.data_ptr<float>(), (int)M, C, (float)eps, (float)momentum,
                              cur_stream()),
              "bn_fwd_coef");
    return coef;
  }, "statistics -> saved mean / invstd, running averages and the [scale | 0 | shift] forward affine");
  m.def("flip_weights", &flip_weights);
  m.def("flip_weights_batched", &flip_weights_batched);
  m.def("flip_desc_ints", &flip_desc_ints);
  m.def("qconv", &qconv, py::arg("x"), py::arg("w"), py::arg("R"), py::arg("S"), py::arg("sh"), py::arg("sw"),
        py::arg("ph"), py::arg("pw"), py::arg("colscale"), py::arg("bias"), py::arg("resid"), py::arg("rscale"),
        py::arg("relu"), py::arg("out_bf16"), py::arg("rvec") = py::none(), py::arg("qflags") = 0);
  m.def("act_fwd_bwd", &act_fwd_bwd);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("loss_fwd", &loss_fwd);
  m.def("auc_hist", &auc_hist);
  m.def("box_decode", &box_decode);
  m.def("quantize_i8", &quantize_i8, py::arg("x"), py::arg("inv_scale"), py::arg("inv_vec") = py::none(),
        py::arg("u8") = false);
  m.def("gap_i8", &gap_i8, py::arg("x"), py::arg("scale"), py::arg("svec") = py::none(), py::arg("u8") = false);
  m.def("quantize_f8", &quantize_f8, py::arg("x"), py::arg("inv_scale"), py::arg("inv_vec") = py::none());
  m.def("embedding_bag_fwd", &embedding_bag_fwd);
  m.def("embedding_bag_bwd", &embedding_bag_bwd);
  m.def("sparse_linear_fwd", &sparse_linear_fwd);
  m.def("sparse_linear_bwd", &sparse_linear_bwd);
  m.def("conv_wgrad", &conv_wgrad);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("pool_shape", &pool_shape);
  m.def("gconv_fwd", &gconv_fwd);
  m.def("gconv_dgrad", &gconv_dgrad);
  m.def("gconv_wgrad", &gconv_wgrad);
  m.def("dwconv_fwd", &dwconv_fwd);
  m.def("dwconv_dgrad", &dwconv_dgrad);
  m.def("dwconv_wgrad", &dwconv_wgrad);
  m.def("softmax_rows", &softmax_rows);
  m.def("act_bwd_reduce", &act_bwd_reduce, py::arg("dz"), py::arg("z"), py::arg("want_db"), py::arg("db_into"),
        py::arg("gelu") = false);
  m.def("softmax_rows_bwd", &softmax_rows_bwd);
  m.def("lrn", &lrn);
  m.def("within_lrn", &within_lrn);
  m.def("roi_pool_fwd", &roi_pool_fwd);
  m.def("roi_pool_bwd", &roi_pool_bwd);
  m.def("ncf_fused", &ncf_fused);
  m.def("prob_nll", &prob_nll);
  m.def("prob_nll_grad", &prob_nll_grad);
  m.def("ncf_tier", &ncf_tier);
  m.def("resize_bilinear", &resize_bilinear);
  m.def("resize_bilinear_bwd", &resize_bilinear_bwd);
  m.def("upsample_nd", &upsample_nd);
  m.def("lstm_gates_fwd", &lstm_gates_fwd);
  m.def("lstm_gates_bwd", &lstm_gates_bwd);
  m.def("lstm_step_fwd", &lstm_step_fwd);
  m.def("lstm_step_bwd", &lstm_step_bwd);
  m.def("convlstm_fwd_step", &convlstm_fwd_step);
  m.def("convlstm_bwd_step", &convlstm_bwd_step);
  m.def("convlstm_fwd_seq", &convlstm_fwd_seq);
  m.def("cu_mask_stream", &cu_mask_stream);
  m.def("set_reserved_cus", [](int64_t n) { zoo_set_reserved_cus((int)n); });
  m.def("convlstm_bwd_seq", &convlstm_bwd_seq);
  m.def("pw_set", [](int mode) { zoo_pw_set(mode); },
        "streaming 1x1 conv kernel (pw.hip): 1 on, 0 off (igemm / igemm2), -1 back to ZOO_PW");
  m.def("convlstm_pers_set", [](int on) { zoo_convlstm_pers_set(on); },
        "persistent ConvLSTM step kernels for large steps: 1 K-split backward / forward below 64k pixels, row "
        "groups above (default), 2 row groups only, 0 off, +4 forward K-split at every size (A/B switch)");
  m.def("igemm2_w192_set", [](int mode) { zoo_igemm2_w192_set(mode); },
        "256x192 igemm2 tiles: 0 off (default), 1 forward-type epilogues, 2 also backward epilogues");
  m.def("igemm2_set", [](int mode, int tile) { zoo_igemm2_set(mode, tile); },
        "igemm2 A/B switch: mode 0 off / 1 on (-1 keep), tile 0 auto / I2Tile id (-1 keep)");
  m.def("c3_grid_for", [](int N, int H, int W) {
          ConvGeom g{};
          g.N = N; g.H = H; g.W = W; g.C = 64; g.K = 64; g.R = 3; g.S = 3; g.sh = 1; g.sw = 1; g.ph = 1; g.pw = 1;
          g.dh = 1; g.dw = 1; g.lh = 1; g.lw = 1; g.P = H; g.Q = W; g.M = N * H * W; g.Ktot = 576; g.ldb = 576;
          return zoo_c3_grid(&g, 1, nullptr);
        }, "workgroups the persistent 3x3 kernel would use for an N x H x W x 64 forward (0: not eligible)");
  m.def("c3_stamps", []() {
          std::vector<unsigned long long> v(4096 * 4 * 5);
          const int n = zoo_c3_stamps(v.data(), (int)v.size());
          v.resize(n > 0 ? n : 0);
          return v;
        }, "diagnostic build (ZOO_C3_STAMPS=1): per-workgroup, per-wave cycle sums of the band segments "
           "(row prefetch, MFMA taps, epilogue, wait+barrier, band count) of the last c3 launch");
  m.def("c3_set", [](int on) { zoo_c3_set(on); },
        "persistent 3x3 64-channel conv kernel (c3.hip): 1 on, 0 off, -1 back to ZOO_C3");
  m.def("igemm2_band_set", [](int on) { zoo_igemm2_band_set(on); },
        "igemm2 band tiles (stride-1 3x3 convs from an LDS halo patch): 1 on, 0 off, -1 keep");
  m.def("set_deterministic", [](bool on) { g_deterministic = on; });
  m.def("get_deterministic", []() { return g_deterministic; });
  m.def("set_reduce_modes", [](bool stats_part, bool wgrad_part) {
    g_stats_partial = stats_part;
    g_wgrad_partial = wgrad_part;
  });
  m.def("get_reduce_modes", []() { return std::make_tuple(g_stats_partial, g_wgrad_partial); });
  m.def("bn_reduce", &bn_reduce);
  m.def("stat_len", &stat_len);
  m.def("bn_fwd_apply", &bn_fwd_apply, py::arg("x"), py::arg("stats"), py::arg("gamma"), py::arg("beta"),
        py::arg("resid"), py::arg("rmean"), py::arg("rvar"), py::arg("smean"), py::arg("sinv"), py::arg("eps"),
        py::arg("momentum"), py::arg("relu"), py::arg("training"),
        py::arg("resid_bn") = std::vector<c10::optional<torch::Tensor>>(), py::arg("mask") = py::none());
  m.def("bn_bwd_apply", &bn_bwd_apply);
  m.def("bnfold_coef", &bnfold_coef);
  m.def("bnpro_apply", &bnpro_apply);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd);
  m.def("bn_relu_maxpool_bwd", &bn_relu_maxpool_bwd);
  m.def("gap_fwd", &gap_fwd);
  m.def("gap_bwd", &gap_bwd);
  m.def("softmax_xent", &softmax_xent);
  m.def("softmax_xent_mean", &softmax_xent_mean);
  m.def("xent_grad_scale", &xent_grad_scale);
  m.def("prob_nll_mean", &prob_nll_mean);
  m.def("optim_device_hparams", [](c10::optional<torch::Tensor> hp) {
          if (hp.has_value() && hp->defined()) {
            req(*hp, at::kFloat, "hp");
            TORCH_CHECK(hp->is_cuda() && hp->numel() >= 4 && hp->is_contiguous(), "optim_device_hparams: fp32 [4] GPU");
            zoo_optim_device_hparams(hp->data_ptr<float>());
          } else {
            zoo_optim_device_hparams(nullptr);
          }
        },
        "optimizer kernels read (lr, bc1, bc2, first_step) from this device buffer while set (None: off)");
  m.def("set_dropout_seed_offset", [](c10::optional<torch::Tensor> off) {
          if (off.has_value() && off->defined()) {
            TORCH_CHECK(off->is_cuda() && off->scalar_type() == at::kInt && off->numel() >= 1,
                        "set_dropout_seed_offset: int32 GPU tensor");
            zoo_set_seed_offset(reinterpret_cast<const uint32_t*>(off->data_ptr<int>()));
          } else {
            zoo_set_seed_offset(nullptr);
          }
        },
        "every dropout kernel xors this device word into its seed (hipGraph replays: fresh masks per step)");
  m.def("optim_zero_grad", [](bool on) { zoo_optim_zero_grad(on ? 1 : 0); },
        "sgd / adam / adaptive clear each gradient element after reading it (engine: no per-step grad fill)");
  m.def("sgd", &sgd);
  m.def("adam", &adam);
  m.def("adaptive", &adaptive);
  m.def("sumsq", &sumsq);
  m.def("clip", &clip);
  m.def("nchw_to_nhwc", &nchw_to_nhwc);
  m.def("bf16_to_f32", &bf16_to_f32);
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def("sum_chunks_bf16", &sum_chunks_bf16);
  m.def("add_bf16", &add_bf16);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("dropout_add_layernorm_fwd", &dropout_add_layernorm_fwd);
  m.def("layernorm_bwd_drop", &layernorm_bwd_drop);
  m.def("layernorm_bwd_split", &layernorm_bwd_split);
  m.def("layernorm_fold", &layernorm_fold);
  m.def("layernorm_bwd", &layernorm_bwd, py::arg("dy"), py::arg("x"), py::arg("g"), py::arg("mean"),
        py::arg("rstd"), py::arg("dg"), py::arg("db"), py::arg("dy2") = py::none());
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("linear_wgrad", &linear_wgrad);
  m.def("bmm_nt", &bmm_nt);
  m.def("ssd_match", &ssd_match);
  m.def("ssd_mine", &ssd_mine);
  m.def("deep_input_fwd", &deep_input_fwd);
  m.def("deep_input_bwd", &deep_input_bwd);
  m.def("wnd_head_fwd", &wnd_head_fwd);
  m.def("wnd_head_bwd", &wnd_head_bwd);
  m.def("l2norm_scale_fwd", &l2norm_scale_fwd);
  m.def("l2norm_scale_bwd", &l2norm_scale_bwd);
  m.def("row_reduce", &row_reduce);
  m.def("row_l2norm", &row_l2norm);
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("mask"), py::arg("causal"),
        py::arg("pdrop") = 0.0, py::arg("seed") = 0);
  m.def("nms_sorted", &nms_sorted);
  m.def("nchw_to_s2d", &nchw_to_s2d);
  m.def("nhwc_u8_to_s2d", &nhwc_u8_to_s2d);
  m.def("dropout_add", &dropout_add, py::arg("a"), py::arg("x") = py::none(), py::arg("p"), py::arg("seed"));
  m.def("attn_fwd_strided", &attn_fwd_strided, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("mask"),
        py::arg("causal"), py::arg("out_blhd"), py::arg("pdrop") = 0.0, py::arg("seed") = 0);
  m.def("absmax", &absmax);
  m.def("im2col_q8", &im2col_q8);
  m.def("qgemm", &qgemm);
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("mask"),
        py::arg("o"), py::arg("lse"), py::arg("causal"), py::arg("pdrop") = 0.0, py::arg("seed") = 0);
  m.def("attn_bwd_strided", &attn_bwd_strided);
  m.def("rnn_fwd", &rnn_fwd, py::arg("xw"), py::arg("u"), py::arg("h0"), py::arg("c0"), py::arg("cell"),
        py::arg("act"), py::arg("iact"), py::arg("save"), py::arg("bhn") = py::none());
  m.def("rnn_bwd", &rnn_bwd);
}
