"""Static-int8 ResNet inference on the int8 implicit-GEMM conv kernel (csrc/kernels/qconv.hip).

BigDL's ``quantize()`` (InferenceModelFactory.scala:33,47; ImageModel.scala:133-145) runs
calibrated int8 convolutions through MKL-DNN; this is the MI355X counterpart
(SURVEY.md §2.16 HK23):

* weights: BatchNorm folded in, symmetric int8 with one scale per output channel;
* activations: int8 NHWC between layers with one calibrated scale PER CHANNEL (absmax over a
  calibration batch run through the bf16 model, / 127). A per-tensor scale lets one outlier
  channel -- e.g. a BatchNorm with a near-zero running variance in a briefly trained model,
  whose folded bias is huge -- crush every other channel to a few int8 levels (r4: logit
  cosine -0.33 against bf16 on such a model). The input scales are folded into the next conv's
  weights before their per-output-channel quantization (w'[n, (r,s,c)] = w[n, (r,s,c)] * s_in[c]),
  the output scales go into the epilogue's per-channel colscale / bias, and the residual add
  takes a per-channel rscale vector -- the kernels' math is unchanged;
* every conv unit is ONE kernel: int8 x int8 on ``v_mfma_i32_16x16x64_i8`` (2x the bf16
  MFMA rate, half the bytes), epilogue ``acc * s_in*s_w[c]/s_out + b[c]/s_out
  (+ resid * s_r/s_out) -> ReLU -> saturating int8``;
* the stem (3-channel input) and the classifier stay bf16; the last block's int8 output
  is average-pooled and dequantised by one kernel.

``fmt="fp8"`` is the same network on OCP e4m3fn (per-channel weight scales amax / 448,
calibrated per-tensor activation scales amax / 448) through the fp8 twin of the kernel: one
``v_mfma_f32_16x16x128_f8f6f4`` per 128-byte k-step (the fp8 peak, 2x bf16), fp32 accumulation,
hardware e4m3 conversion in the epilogue (``Fp8ResNet``).

``qconv_ref`` is the float64 CPU model of the kernel (same rounding) used as the oracle.
"""
import torch
import torch.nn as nn

from zoo.ops._native import native


QMAX = {"int8": 127.0, "fp8": 448.0}
F8 = torch.float8_e4m3fn


def _fmt_of(t):
    return "fp8" if t.dtype == F8 else "int8"


def to_fp8(v):
    """float -> e4m3fn with the kernel's clamp to the finite range (round to nearest even)."""
    return v.float().clamp(-448.0, 448.0).to(F8)


def _fold_weight(unit):
    """ConvBN (eval) -> (BN-folded fp32 weight [K, R*S*C], folded bias [K])."""
    inv = torch.rsqrt(unit.running_var.float() + unit.eps)
    g = unit.gamma.detach().float() * inv
    w = unit.weight.detach().float()[:, :unit.k * unit.k * unit.cin] * g[:, None]
    b = unit.beta.detach().float() - unit.running_mean.float() * g
    return w, b


def _quant_rows(w, fmt="int8"):
    """fp32 [K, R*S*C] -> (int8 / e4m3 rows, per-row scale [K])."""
    s = w.abs().amax(dim=1).clamp_min(1e-12) / QMAX[fmt]
    if fmt == "fp8":
        q = to_fp8(w / s[:, None])
    else:
        q = torch.round(w / s[:, None]).clamp_(-127, 127).to(torch.int8)
    return q.contiguous(), s


def _q_weight(unit, fmt="int8"):
    """ConvBN (eval) -> (int8 / e4m3 [K, R*S*C], per-channel scale [K], folded bias [K])."""
    w, b = _fold_weight(unit)
    q, s = _quant_rows(w, fmt)
    return q, s, b


def _sat(v):
    return torch.clamp(torch.round(v), -127, 127)


def _sat_u8(v):
    """unsigned (offset-coded) int8: round, clamp to [0, 255], store minus 128 (qconv.hip QF_*)"""
    return torch.clamp(torch.round(v), 0, 255) - 128


QF_IN_U8, QF_OUT_U8, QF_RES_U8 = 1, 2, 4


def qconv_ref(xq, wq, R, S, stride, pad, colscale, bias, resid=None, rscale=0.0, relu=False, out_bf16=False,
              rvec=None, qflags=0):
    """float64 CPU model of qconv: xq int8 / e4m3 NHWC, wq [K, R*S*C] of the same format.
    ``qflags``: which of input / output / residual use the unsigned offset code."""
    import torch.nn.functional as F
    fmt = _fmt_of(xq)
    N, H, W, C = xq.shape
    K = wq.shape[0]
    w4 = wq[:, :R * S * C].double().reshape(K, R, S, C).permute(0, 3, 1, 2)
    xd = xq.double()
    if qflags & QF_IN_U8:   # the kernel pads with the code of 0 (-128) and the host folds 128 * sum(w)
        xd = F.pad(xd.permute(0, 3, 1, 2), (pad, pad, pad, pad), value=-128.0)
        acc = F.conv2d(xd, w4, stride=stride).permute(0, 2, 3, 1)
    else:
        acc = F.conv2d(xd.permute(0, 3, 1, 2), w4, stride=stride, padding=pad).permute(0, 2, 3, 1)
    v = acc * colscale.double() + (bias.double() if bias is not None else 0.0)
    if resid is not None:
        r = resid.double() + (128.0 if qflags & QF_RES_U8 else 0.0)
        v = v + r * (rvec.double() if rvec is not None else rscale)
    if relu:
        v = v.clamp_min(0)
    if out_bf16:
        return v.to(torch.bfloat16)
    if fmt == "fp8":
        return to_fp8(v)
    return (_sat_u8(v) if qflags & QF_OUT_U8 else _sat(v)).to(torch.int8)


def qconv(xq, wq, R, S, stride, pad, colscale, bias, resid=None, rscale=0.0, relu=False, out_bf16=False, rvec=None,
          qflags=0):
    """``rvec`` (optional [K]): per-channel residual scale, overrides ``rscale``."""
    if xq.is_cuda:
        return native().qconv(xq, wq, R, S, stride, stride, pad, pad, colscale, bias, resid, float(rscale),
                              bool(relu), bool(out_bf16), rvec, int(qflags))
    return qconv_ref(xq, wq, R, S, stride, pad, colscale, bias, resid, rscale, relu, out_bf16, rvec, qflags)


def quantize_act(x, scale, fmt="int8", u8=False):
    """bf16 NHWC -> int8 / e4m3 with ``scale`` a float (per tensor) or a [C] tensor (per channel);
    ``u8``: the unsigned offset code of a non-negative tensor (int8 only)."""
    vec = torch.is_tensor(scale)
    if x.is_cuda and x.dtype == torch.bfloat16 and x.numel() % 16 == 0 and (not vec or x.shape[-1] % 16 == 0):
        if fmt == "fp8":
            fn = native().quantize_f8
        else:
            def fn(t, inv, iv=None):
                return native().quantize_i8(t, inv, iv, bool(u8))
        if vec:
            return fn(x.contiguous(), 1.0, (1.0 / scale).float().contiguous())
        return fn(x.contiguous(), 1.0 / scale)
    s = scale.double().to(x.device) if vec else scale
    if fmt == "fp8":
        return to_fp8(x.double() / s)
    return (_sat_u8 if u8 else _sat)(x.double() / s).to(torch.int8)


def _dequant(xq, s, u8=False):
    """int8 / e4m3 NHWC -> fp32 with a per-tensor float or per-channel [C] scale."""
    v = xq.float() + 128.0 if u8 else xq.float()
    return v * (s.float().to(xq.device) if torch.is_tensor(s) else s)


class _QUnit:
    """One conv unit: quantized weights and the epilogue constants for given in/out scales
    (floats: per tensor; [C] tensors: per channel)."""

    def __init__(self, unit, device, fmt="int8"):
        self.w, self.b = (t.to(device) for t in _fold_weight(unit))
        self.fmt, self.cin = fmt, unit.cin
        self.k, self.stride, self.pad, self.relu = unit.k, unit.stride, unit.pad, unit.relu
        self.qflags = 0     # QF_* bits: input / output / residual in the unsigned offset code

    def bind(self, s_in, s_out):
        self.s_in, self.s_out = s_in, s_out
        if torch.is_tensor(s_in):
            # input scales folded into the weight columns (column (r, s, c) -> s_in[c]) before the
            # per-output-channel weight quantization: acc * sw[n] is then the real-valued output
            self.q, sw = _quant_rows(self.w * s_in.float().repeat(self.k * self.k)[None, :], self.fmt)
            self.colscale = (sw / s_out).float().contiguous()
        else:
            self.q, sw = _quant_rows(self.w, self.fmt)
            self.colscale = (sw * (s_in / s_out)).float().contiguous()
        self.bias = (self.b / s_out).float().contiguous()
        if self.qflags & QF_IN_U8:   # x = (q + 128) s: the MFMA sums q * w, the 128 * sum(w) term is constant
            self.bias = (self.bias + self.colscale * 128.0 * self.q.float().sum(1)).contiguous()

    def __call__(self, xq, resid=None, s_resid=None):
        rvec = None
        rscale = 0.0
        if resid is not None:
            r = s_resid / self.s_out
            if torch.is_tensor(r):
                rvec = r.float().contiguous()
            else:
                rscale = r
        qf = self.qflags if resid is not None else self.qflags & ~QF_RES_U8
        return qconv(xq, self.q, self.k, self.k, self.stride, self.pad, self.colscale, self.bias, resid,
                     rscale, self.relu, rvec=rvec, qflags=qf)


class Int8ResNet(nn.Module):
    """Calibrated static-int8 (``fmt="fp8"``: e4m3) inference twin of a
    ``zoo.models.image.resnet.ResNet``."""

    fmt = "int8"
    act_scales = "channel"
    act_clip = 0.0

    act_u8 = True

    def __init__(self, model, calib_x, fmt=None, act_scales=None, act_clip=None, bf16_blocks=(), max_block_err=None,
                 act_u8=None):
        """``act_scales``: "channel" (one activation scale per channel), "mse" (per channel, the
        clipping range minimising the calibration batch's squared quantization error) or "tensor"
        (one per tensor).
        ``act_clip``: fraction of each channel's calibration values allowed to saturate (0: absmax;
        e.g. 1e-4 keeps a few spatial outliers from stretching the channel's int8 grid).
        Mixed precision (TensorRT-style per-layer fallback): ``bf16_blocks`` -- indices of residual
        blocks that stay on the bf16 kernels; ``max_block_err`` -- additionally keep in bf16 every
        block whose calibrated local error (relative L2 of its quantized output against bf16, fed
        the same input; ``block_err``) exceeds this. Activations are dequantised / requantised at
        the boundaries.
        ``act_u8`` (int8 only, default on): the non-negative activations (block inputs / outputs and
        the ReLU outputs inside a block) use the unsigned offset code -- 255 levels over [0, amax]
        instead of 127 -- and only the projection shortcut's output stays signed."""
        super().__init__()
        if act_u8 is not None:
            self.act_u8 = bool(act_u8)
        self.bf16_blocks = set(int(i) for i in bf16_blocks)
        self.max_block_err = max_block_err
        if act_clip is not None:
            self.act_clip = float(act_clip)
        from zoo.models.image import resnet as R
        if fmt is not None:
            self.fmt = fmt
        if act_scales is not None:
            self.act_scales = act_scales
        if self.fmt not in QMAX:
            raise ValueError("quantized format must be one of %s" % sorted(QMAX))
        if self.act_scales not in ("channel", "tensor", "mse"):
            raise ValueError("act_scales must be 'channel', 'tensor' or 'mse'")
        model.eval()
        self.model = model
        dev = next(model.parameters()).device
        f = self.fmt
        self.blocks = []
        for stage in model.stages:
            for blk in stage:
                units = {"conv1": _QUnit(blk.conv1, dev, f), "conv2": _QUnit(blk.conv2, dev, f)}
                if isinstance(blk, R.Bottleneck):
                    units["conv3"] = _QUnit(blk.conv3, dev, f)
                if blk.down is not None:
                    units["down"] = _QUnit(blk.down, dev, f)
                self.blocks.append((blk, units))
        self.u8 = self.act_u8 and self.fmt == "int8"
        if self.u8:
            for _, u in self.blocks:
                # conv1 / conv2 / conv3 read and write unsigned tensors; the projection reads the
                # unsigned block input and writes a signed (BN-only) shortcut; conv3's residual is
                # the unsigned block input unless a projection produced it
                for k in ("conv1", "conv2", "conv3"):
                    if k in u:
                        u[k].qflags = QF_IN_U8 | QF_OUT_U8
                last = u["conv3"] if "conv3" in u else u["conv2"]
                if "down" in u:
                    u["down"].qflags = QF_IN_U8
                else:
                    last.qflags |= QF_RES_U8
        self.calibrate(calib_x)

    @torch.no_grad()
    def _stem(self, x):
        m = self.model
        from zoo import ops
        if m._stem_s2d_ok(x):
            xs = ops.native().nchw_to_s2d(x.float().contiguous(), 3)
            st = m.stem
            x = ops.conv_bn_act(xs, m._s2d_weight(), st.gamma, st.beta, st.running_mean, st.running_var,
                                kernel=(4, 4), stride=(1, 1), pad=(0, 0), eps=st.eps, momentum=st.momentum,
                                relu=True, training=False)
        else:
            x = m.stem(m.to_nhwc(x))
        return ops.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))

    @torch.no_grad()
    def calibrate(self, x):
        """Per-tensor absmax of every int8 tensor of the network on ``x`` (run in bf16)."""
        qmax0 = QMAX[self.fmt]
        clip = self.act_clip
        if self.act_scales == "channel":
            def amax(t, qmax=qmax0):
                a = t.float().abs().reshape(-1, t.shape[-1])
                if clip > 0:
                    k = max(1, int(a.shape[0] * clip))     # the k-th largest value per channel
                    a = a.topk(k, dim=0).values[-1]
                else:
                    a = a.amax(dim=0)
                return a.clamp_min(1e-6) / qmax
        elif self.act_scales == "mse":
            # per channel, the clipping range (a fraction of the absmax) that minimises the
            # calibration batch's squared quantization error: a heavy-tailed channel trades a few
            # saturated outliers for a finer grid under the bulk of its values
            def amax(t, qmax=qmax0):
                a = t.float().reshape(-1, t.shape[-1])
                m = a.abs().amax(dim=0).clamp_min(1e-6)
                best, best_err = m.clone(), None
                for r in (1.0, 0.9, 0.8, 0.7, 0.6, 0.5, 0.4, 0.3, 0.2):
                    sc = m * (r / qmax)
                    if self.fmt == "fp8":
                        dq = to_fp8((a / sc).clamp(-qmax, qmax)).float() * sc
                    else:
                        dq = (a / sc).round().clamp(-qmax if qmax < 200 else 0, qmax) * sc
                    err = (dq - a).square().sum(dim=0)
                    if best_err is None:
                        best_err = err
                        continue
                    win = err < best_err
                    best = torch.where(win, m * r, best)
                    best_err = torch.where(win, err, best_err)
                return best / qmax
        else:
            def amax(t, qmax=qmax0):
                return max(float(t.float().abs().max()), 1e-6) / qmax
        qu = 255.0 if self.u8 else qmax0      # range of a non-negative (unsigned-coded) tensor
        h = self._stem(x)
        self.s_in = amax(h, qu)
        s_x = self.s_in
        self.block_err = []
        for blk, u in self.blocks:
            sc = blk.down(h) if blk.down is not None else h
            s_sc = amax(sc) if blk.down is not None else s_x
            h1 = blk.conv1(h)
            s1 = amax(h1, qu)
            if "conv3" in u:
                h2 = blk.conv2(h1)
                s2 = amax(h2, qu)
                out = blk.conv3(h2, resid=sc)
            else:
                out = blk.conv2(h1, resid=sc)
            s_o = amax(out, qu)
            u["conv1"].bind(s_x, s1)
            if "conv3" in u:
                u["conv2"].bind(s1, s2)
                u["conv3"].bind(s2, s_o)
            else:
                u["conv2"].bind(s1, s_o)
            if "down" in u:
                u["down"].bind(s_x, s_sc)
            blk._q_scales = (s_x, s_sc, s_o)
            # the block's own quantization error: its quantized run on the bf16 input vs bf16
            oq = _dequant(self._run_block(u, quantize_act(h, s_x, self.fmt, self.u8), s_sc), s_o, self.u8)
            of = out.float()
            self.block_err.append(float((oq - of).norm() / of.norm().clamp_min(1e-12)))
            h, s_x = out, s_o
        self.s_out = s_x
        if self.max_block_err is not None:
            self.bf16_blocks |= {i for i, e in enumerate(self.block_err) if e > self.max_block_err}
        return self

    def _run_block(self, u, xq, s_sc):
        sc = u["down"](xq) if "down" in u else xq
        h1 = u["conv1"](xq)
        if "conv3" in u:
            return u["conv3"](u["conv2"](h1), resid=sc, s_resid=s_sc)
        return u["conv2"](h1, resid=sc, s_resid=s_sc)

    @torch.no_grad()
    def forward(self, x):
        h = self._stem(x)
        xq = None                     # quantized activation (None: h is the bf16 one)
        for i, (blk, u) in enumerate(self.blocks):
            s_x, s_sc, s_o = blk._q_scales
            if i in self.bf16_blocks:
                if xq is not None:
                    h, xq = _dequant(xq, s_x, self.u8).to(torch.bfloat16), None
                h = blk(h)
                continue
            if xq is None:
                xq = quantize_act(h, s_x, self.fmt, self.u8)
            xq = self._run_block(u, xq, s_sc)
        if xq is None:                # the last block ran in bf16
            from zoo import ops
            return self.model.fc(ops.global_avg_pool_nhwc(h))
        vec = torch.is_tensor(self.s_out)
        if xq.is_cuda:
            feat = native().gap_i8(xq.contiguous(), 1.0, self.s_out.float().contiguous(), self.u8) if vec else \
                native().gap_i8(xq.contiguous(), self.s_out, None, self.u8)
        else:
            s = self.s_out.double().to(xq.device) if vec else self.s_out
            feat = ((xq.double() + (128.0 if self.u8 else 0.0)) * s).mean((1, 2)).to(torch.bfloat16)
        return self.model.fc(feat)


class Fp8ResNet(Int8ResNet):
    """Calibrated static OCP-fp8 (e4m3fn) inference twin of a zoo ResNet."""

    fmt = "fp8"


def quantize_resnet(model, calib_x, fmt="int8", act_scales="channel"):
    """Static-int8 (or ``fmt="fp8"``) inference twin of ``model`` (a zoo ResNet), calibrated on
    ``calib_x`` with per-channel (default) or per-tensor activation scales."""
    return (Fp8ResNet if fmt == "fp8" else Int8ResNet)(model, calib_x, act_scales=act_scales)


__all__ = ["Int8ResNet", "Fp8ResNet", "quantize_resnet", "qconv", "qconv_ref", "quantize_act", "to_fp8"]
