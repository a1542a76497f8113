"""Native ops behind the remaining Keras layers (csrc/kernels/keras_ops.hip + the conv /
depthwise / pooling kernels), with fp32 PyTorch references for CPU tensors:

  within_channel_lrn   WithinChannelLRN2D    (SpatialWithinChannelLRN)
  resize_bilinear      ResizeBilinear        (BigDL nn.ResizeBilinear: TF-legacy sampling)
  upsample_nearest     UpSampling1D/2D/3D
  lstm_gates           ConvLSTM2D/3D gate step (fused activations + cell/hidden update)
  conv3d_ndhwc         Convolution3D         (depth taps stacked on channels: one implicit-GEMM conv2d)
  pool3d_ndhwc         MaxPooling3D / AveragePooling3D (separable: HxW then D, native 2-D pools)
  pool1d_nwc           MaxPooling1D / AveragePooling1D (native 2-D pool with H = 1)

Reference: Zs/pipeline/api/keras/layers/{WithinChannelLRN2D,ResizeBilinear,UpSampling*,
Convolution3D,MaxPooling3D,AveragePooling3D,ConvLSTM2D,ConvLSTM3D}.scala, InternalConvLSTM3D.scala.
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native

ACT_CODES = {None: 0, "linear": 0, "tanh": 1, "sigmoid": 2, "hard_sigmoid": 3, "relu": 4}


def _gpu_ok(x):
    return x.is_cuda and x.dtype in (torch.float32, torch.bfloat16) and x.numel() > 0


# ---------------------------------------------------------------------------- within-channel LRN
class _WLRNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, alpha, beta):
        ctx.save_for_backward(x)
        ctx.p = (size, alpha, beta)
        return native().within_lrn(x, None, size, alpha, beta)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        size, alpha, beta = ctx.p
        return native().within_lrn(x, dy.contiguous().to(x.dtype), size, alpha, beta), None, None, None


def within_channel_lrn_ref(x, size, alpha, beta):
    """x NHWC; y = x * (1 + alpha * mean_{size x size}(x^2))^-beta (zero padding, size^2 divisor)."""
    xc = x.float().permute(0, 3, 1, 2)
    lo = (size - 1) // 2
    sq = F.pad(xc * xc, (lo, size - 1 - lo, lo, size - 1 - lo))
    avg = F.avg_pool2d(sq, size, stride=1)
    return (xc * (1.0 + alpha * avg) ** (-beta)).permute(0, 2, 3, 1).to(x.dtype)


def within_channel_lrn(x, size=5, alpha=1.0, beta=0.75):
    if _gpu_ok(x) and x.dim() == 4:
        return _WLRNFn.apply(x.contiguous(), int(size), float(alpha), float(beta))
    return within_channel_lrn_ref(x, size, alpha, beta)


# ---------------------------------------------------------------------------- bilinear resize
class _ResizeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow, align):
        ctx.g = (x.shape[1], x.shape[2], align)
        return native().resize_bilinear(x, oh, ow, align)

    @staticmethod
    def backward(ctx, dy):
        H, W, align = ctx.g
        return native().resize_bilinear_bwd(dy.contiguous(), H, W, align), None, None, None


def _lerp_table(o, i, align, device):
    mode = int(align)
    scale = (i - 1) / (o - 1) if (mode == 1 and o > 1) else i / o
    s = torch.arange(o, device=device, dtype=torch.float64) * scale
    if mode == 2:
        s = (s + 0.5 * scale - 0.5).clamp_min(0)
    lo = s.floor().clamp(max=i - 1).long()
    hi = (lo + 1).clamp(max=i - 1)
    f = (s - lo.double()).clamp(0, 1).float()
    return lo, hi, f


def resize_bilinear_ref(x, oh, ow, align=False):
    """NHWC bilinear resize. ``align``: False / 0 BigDL / TF-legacy sampling (src = dst * scale),
    True / 1 align_corners, 2 half-pixel centres (PyTorch align_corners=False)."""
    xf = x.float()
    h0, h1, fh = _lerp_table(oh, x.shape[1], align, x.device)
    w0, w1, fw = _lerp_table(ow, x.shape[2], align, x.device)
    top = xf[:, h0]
    bot = xf[:, h1]
    fw_ = fw.view(1, 1, -1, 1)
    top = top[:, :, w0] + (top[:, :, w1] - top[:, :, w0]) * fw_
    bot = bot[:, :, w0] + (bot[:, :, w1] - bot[:, :, w0]) * fw_
    return (top + (bot - top) * fh.view(1, -1, 1, 1)).to(x.dtype)


def resize_bilinear(x, oh, ow, align=False):
    if _gpu_ok(x) and x.dim() == 4:
        return _ResizeFn.apply(x.contiguous(), int(oh), int(ow), int(align))
    return resize_bilinear_ref(x, oh, ow, align)


# ---------------------------------------------------------------------------- nearest upsampling
class _UpsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, fd, fh, fw):
        ctx.f = (fd, fh, fw)
        return native().upsample_nd(x, fd, fh, fw, False)

    @staticmethod
    def backward(ctx, dy):
        fd, fh, fw = ctx.f
        return native().upsample_nd(dy.contiguous(), fd, fh, fw, True), None, None, None


def upsample_nearest(x, factors):
    """x [N, *spatial (1..3 dims), C] channels-last; ``factors`` per spatial dim."""
    nsp = x.dim() - 2
    f = list(factors) + [1] * (3 - len(factors))
    if _gpu_ok(x) and 1 <= nsp <= 3:
        shp = list(x.shape)
        x5 = x.contiguous().reshape([shp[0]] + [1] * (3 - nsp) + shp[1:-1] + [shp[-1]])
        fd, fh, fw = ([1] * (3 - nsp) + list(factors))[:3]
        y = _UpsampleFn.apply(x5, fd, fh, fw)
        return y.reshape([shp[0]] + [s * k for s, k in zip(shp[1:-1], factors)] + [shp[-1]])
    y = x
    for i, k in enumerate(factors):
        y = y.repeat_interleave(int(k), dim=1 + i)
    return y


# ---------------------------------------------------------------------------- ConvLSTM gates
class _GatesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gx, gh, cprev, iact, act):
        h, c, acts = native().lstm_gates_fwd(gx, gh, cprev, iact, act)
        ctx.save_for_backward(acts, cprev if cprev is not None else None, c)
        ctx.p = (iact, act, gh is not None, cprev is not None)
        return h, c

    @staticmethod
    def backward(ctx, dh, dc):
        acts, cprev, c = ctx.saved_tensors
        iact, act, has_gh, has_c = ctx.p
        dh = None if dh is None else dh.contiguous().float()
        dc = None if dc is None else dc.contiguous().float()
        dg, dcp = native().lstm_gates_bwd(dh, dc, acts, cprev if has_c else None, c, iact, act)
        return dg, (dg if has_gh else None), (dcp if has_c else None), None, None


def _act_ref(x, code):
    if code == 1:
        return torch.tanh(x)
    if code == 2:
        return torch.sigmoid(x)
    if code == 3:
        return (0.2 * x + 0.5).clamp(0, 1)
    if code == 4:
        return torch.relu(x)
    return x


def lstm_gates(gx, gh, cprev, inner_activation="hard_sigmoid", activation="tanh"):
    """One ConvLSTM step over flattened rows: g = gx + gh [M, 4F] (i | f | candidate | o),
    c = f * c_prev + i * act(candidate), h = o * act(c). Returns (h, c), fp32 [M, F]."""
    iact, act = ACT_CODES[inner_activation], ACT_CODES[activation]
    if gx.is_cuda:
        gx = gx.float().contiguous()
        gh = None if gh is None else gh.float().contiguous()
        cprev = None if cprev is None else cprev.float().contiguous()
        return _GatesFn.apply(gx, gh, cprev, iact, act)
    g = gx.float() + (0 if gh is None else gh.float())
    Fh = g.shape[-1] // 4
    i, f = _act_ref(g[..., :Fh], iact), _act_ref(g[..., Fh:2 * Fh], iact)
    cc, o = _act_ref(g[..., 2 * Fh:3 * Fh], act), _act_ref(g[..., 3 * Fh:], iact)
    c = i * cc if cprev is None else f * cprev + i * cc
    return o * _act_ref(c, act), c


# ---------------------------------------------------------------------------- 3-D convolution
def conv3d_ndhwc(x, w5, bias=None, stride=(1, 1, 1), pad=(0, 0, 0)):
    """x [N, D, H, W, C]; w5 [K, KD, KH, KW, C] (channels-last filter). On the GPU: the KD
    depth-shifted input slices are stacked along channels ([N*Do, H, W, KD*C], channel kd*C + c)
    and convolved ONCE as a KH x KW conv2d with a KD*C-deep reduction, the depth taps summed in
    the GEMM's fp32 accumulators; the backward is that conv2d's native dgrad / wgrad through
    autograd (the stacking's gradient sums the slices back). Round 5 ran one conv2d per depth tap
    with fp32 outputs summed by elementwise adds: 3 output tensors of 4 bytes per element and
    their adds were a third of a ConvLSTM3D step (profiles/r6/ab7_convlstm3d_*_totals_r6.md)."""
    from zoo.ops.conv import conv2d_nhwc, pack_weight
    N, D, H, W, C = x.shape
    K, KD, KH, KW, _ = w5.shape
    sd, sh, sw = stride
    pd, ph, pw = pad
    if not x.is_cuda or C % 8 or K % 8:
        y = F.conv3d(x.float().permute(0, 4, 1, 2, 3), w5.float().permute(0, 4, 1, 2, 3),
                     None if bias is None else bias.float(), stride=stride, padding=pad)
        return y.permute(0, 2, 3, 4, 1).to(x.dtype)
    xp = F.pad(x, (0, 0, 0, 0, 0, 0, pd, pd)) if pd else x
    Do = (D + 2 * pd - KD) // sd + 1
    if KD == 1:
        xs = xp[:, 0:sd * (Do - 1) + 1:sd]
    else:
        xs = torch.cat([xp[:, kd:kd + sd * (Do - 1) + 1:sd] for kd in range(KD)], dim=-1)   # [N, Do, H, W, KD*C]
    wk = pack_weight(w5.permute(0, 2, 3, 1, 4).reshape(K, KH, KW, KD * C))
    y = conv2d_nhwc(xs.reshape(N * Do, H, W, KD * C), wk, bias, kernel=(KH, KW), stride=(sh, sw), pad=(ph, pw))
    return y.reshape(N, Do, y.shape[1], y.shape[2], K).to(x.dtype)


# ---------------------------------------------------------------------------- pooling
def pool1d_nwc(x, kind, length, stride, pad=(0, 0)):
    """x [N, L, C] -> native 2-D pooling on [N, 1, L, C] (window 1 x length)."""
    from zoo.ops.pool import avg_pool2d_nhwc, max_pool2d_nhwc
    if x.is_cuda and x.shape[-1] % 8 == 0 and pad == (0, 0):
        x4 = x.unsqueeze(1)
        f = max_pool2d_nhwc if kind == "max" else avg_pool2d_nhwc
        return f(x4, (1, length), (1, stride)).squeeze(1)
    xc = x.transpose(1, 2).float()
    if pad != (0, 0):
        xc = F.pad(xc, pad, value=float("-inf") if kind == "max" else 0.0)
    f = F.max_pool1d if kind == "max" else F.avg_pool1d
    return f(xc, length, stride).transpose(1, 2).to(x.dtype)


def pool3d_ndhwc(x, kind, size, stride):
    """x [N, D, H, W, C] -> (valid) 3-D max / average pooling as two native 2-D pools:
    H x W over [N*D, H, W, C], then D over [N, D, Ho*Wo, C] (both separable: a max of maxes /
    a mean of equal-size means)."""
    from zoo.ops.pool import avg_pool2d_nhwc, max_pool2d_nhwc
    N, D, H, W, C = x.shape
    kd, kh, kw = size
    sd, sh, sw = stride
    if not (x.is_cuda and C % 8 == 0):
        f = F.max_pool3d if kind == "max" else F.avg_pool3d
        y = f(x.float().permute(0, 4, 1, 2, 3), size, stride)
        return y.permute(0, 2, 3, 4, 1).to(x.dtype)
    f = max_pool2d_nhwc if kind == "max" else avg_pool2d_nhwc
    y = f(x.reshape(N * D, H, W, C), (kh, kw), (sh, sw))
    Ho, Wo = y.shape[1], y.shape[2]
    y = f(y.reshape(N, D, Ho * Wo, C), (kd, 1), (sd, 1))
    return y.reshape(N, y.shape[1], Ho, Wo, C)
