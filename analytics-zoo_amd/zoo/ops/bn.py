"""Fused Conv -> BatchNorm -> (+residual) -> (ReLU) for NHWC bf16 activations.

Forward (training), three kernels per conv-BN-act unit:
  1. implicit-GEMM conv whose epilogue also accumulates per-channel (sum, sum^2)
  2. BN apply with residual add + ReLU fused (each workgroup derives
     scale/shift from the raw sums; workgroup 0 updates running statistics)
Backward:
  3. one reduction pass (sum dy, sum dy*xhat) with the ReLU mask recomputed
     from the saved output
  4. BN backward apply (also emits the residual-branch gradient), then the conv
     dgrad / wgrad kernels.

This is the MI355X replacement for the MKL-DNN fused conv+BN+ReLU graphs the
reference used for ResNet-50 (SURVEY.md §2.13 row "MKL-DNN primitives",
§2.16 HK4/HK5; BigDL BatchNormalization behind
Zs/pipeline/api/keras/layers/BatchNormalization.scala:85-110).
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native
from zoo.ops.conv import bf16_weight, ceil8, conv2d_ref


def _notify(p):
    hook = getattr(p, "_zoo_grad_ready", None)
    if hook is not None:
        hook(p)


def _grad_target(p):
    g = getattr(p, "_zoo_grad", None)
    if g is not None:
        return g, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), False


class _ConvBNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, resid, running_mean, running_var, R, S, stride, pad, eps, momentum,
                relu, training):
        C_ = native()
        K = w.shape[0]
        wb = bf16_weight(w)
        stats = torch.zeros(2 * K, device=x.device, dtype=torch.float32) if training else None
        y = C_.conv_fwd(x, wb, R, S, stride[0], stride[1], pad[0], pad[1], 1, 1, 1, 1, None, None, stats, 0,
                        False, True, 0, 0)
        smean = torch.empty(K, device=x.device, dtype=torch.float32)
        sinv = torch.empty(K, device=x.device, dtype=torch.float32)
        z = C_.bn_fwd_apply(y, stats if training else torch.empty(0, device=x.device), gamma.detach(),
                            beta.detach(), resid, running_mean, running_var, smean, sinv, eps, momentum, relu,
                            training)
        ctx.save_for_backward(x, w, gamma, y, z if relu else None, smean, sinv)
        ctx.meta = (R, S, stride, pad, relu, resid is not None, x.shape)
        return z

    @staticmethod
    def backward(ctx, dz):
        C_ = native()
        x, w, gamma, y, z, smean, sinv = ctx.saved_tensors
        R, S, stride, pad, relu, has_resid, xshape = ctx.meta
        dz = dz.contiguous()
        if dz.dtype != torch.bfloat16:
            dz = dz.to(torch.bfloat16)
        K = w.shape[0]
        Cin = xshape[3]
        sums = torch.zeros(2 * K, device=dz.device, dtype=torch.float32)
        C_.bn_reduce(dz, z, y, smean, sinv, sums, 1)
        dgam, own_g = _grad_target(gamma)
        dbet, own_b = _grad_target(ctx.beta_ref) if hasattr(ctx, "beta_ref") else (None, False)
        outs = C_.bn_bwd_apply(dz, z, y, smean, sinv, gamma.detach(), sums, has_resid, dgam, dbet)
        dy = outs[0]
        dresid = outs[1] if has_resid else None
        dx = None
        if ctx.needs_input_grad[0]:
            wt = C_.flip_weights(bf16_weight(w)[:, : R * S * Cin].contiguous(), K, R, S, Cin)
            if wt.shape[1] % 8:
                wt = F.pad(wt, (0, ceil8(wt.shape[1]) - wt.shape[1]))
            dx = C_.conv_fwd(dy, wt, R, S, 1, 1, R - 1 - pad[0], S - 1 - pad[1], 1, 1, stride[0], stride[1], None,
                             None, None, 0, False, True, xshape[1], xshape[2])
        gw, own_w = _grad_target(w)
        C_.conv_wgrad(x, dy, gw, R, S, stride[0], stride[1], pad[0], pad[1], 1, 1)
        if own_w:
            _notify(w)
        if own_g:
            _notify(gamma)
        if own_b:
            _notify(ctx.beta_ref)
        return (dx, None if own_w else gw.to(w.dtype), None if own_g else dgam, None if own_b else dbet, dresid,
                None, None, None, None, None, None, None, None, None, None)


class _ConvBNActFnB(_ConvBNActFn):
    """Same as _ConvBNActFn but keeps a handle on beta for its gradient."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, resid, running_mean, running_var, R, S, stride, pad, eps, momentum,
                relu, training):
        ctx.beta_ref = beta
        return _ConvBNActFn.forward(ctx, x, w, gamma, beta, resid, running_mean, running_var, R, S, stride, pad,
                                    eps, momentum, relu, training)


def bn_ref(y, gamma, beta, running_mean, running_var, eps, momentum, training):
    """fp32 NHWC BatchNorm reference (updates running stats like BigDL/torch)."""
    C = y.shape[-1]
    yf = y.float().reshape(-1, C)
    if training:
        mean = yf.mean(0)
        var = yf.var(0, unbiased=False)
        if running_mean is not None:
            n = yf.shape[0]
            with torch.no_grad():
                running_mean.mul_(1 - momentum).add_(momentum * mean)
                running_var.mul_(1 - momentum).add_(momentum * var * n / max(n - 1, 1))
    else:
        mean, var = running_mean, running_var
    out = (yf - mean) / torch.sqrt(var + eps)
    if gamma is not None:
        out = out * gamma + beta
    return out.reshape(y.shape)


def conv_bn_act(x, w, gamma, beta, running_mean, running_var, kernel=(1, 1), stride=(1, 1), pad=(0, 0),
                eps=1e-5, momentum=0.1, relu=True, resid=None, training=True):
    """z = relu?(BN(conv(x)) + resid) for NHWC input with a packed weight."""
    R, S = kernel
    if x.is_cuda:
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        if resid is not None:
            resid = resid.to(torch.bfloat16).contiguous()
        return _ConvBNActFnB.apply(x.contiguous(), w, gamma, beta, resid, running_mean, running_var, R, S,
                                   tuple(stride), tuple(pad), float(eps), float(momentum), bool(relu),
                                   bool(training))
    y = conv2d_ref(x, w, (R, S, x.shape[3], tuple(stride), tuple(pad), (1, 1)))
    z = bn_ref(y, gamma, beta, running_mean, running_var, eps, momentum, training)
    if resid is not None:
        z = z + resid.float()
    if relu:
        z = torch.relu(z)
    return z.to(x.dtype) if x.dtype != torch.float32 else z


class _BNActFn(torch.autograd.Function):
    """Standalone NHWC BatchNorm (+residual, +ReLU) when there is no producing conv."""

    @staticmethod
    def forward(ctx, y, gamma, beta, resid, running_mean, running_var, eps, momentum, relu, training):
        C_ = native()
        K = y.shape[-1]
        stats = torch.zeros(2 * K, device=y.device, dtype=torch.float32)
        if training:
            C_.bn_reduce(y, None, None, None, None, stats, 0)
        smean = torch.empty(K, device=y.device, dtype=torch.float32)
        sinv = torch.empty(K, device=y.device, dtype=torch.float32)
        z = C_.bn_fwd_apply(y, stats, gamma.detach(), beta.detach(), resid, running_mean, running_var, smean,
                            sinv, eps, momentum, relu, training)
        ctx.save_for_backward(y, gamma, beta, z if relu else None, smean, sinv)
        ctx.has_resid = resid is not None
        return z

    @staticmethod
    def backward(ctx, dz):
        C_ = native()
        y, gamma, beta, z, smean, sinv = ctx.saved_tensors
        dz = dz.contiguous().to(torch.bfloat16)
        K = y.shape[-1]
        sums = torch.zeros(2 * K, device=dz.device, dtype=torch.float32)
        C_.bn_reduce(dz, z, y, smean, sinv, sums, 1)
        dgam, own_g = _grad_target(gamma)
        dbet, own_b = _grad_target(beta)
        outs = C_.bn_bwd_apply(dz, z, y, smean, sinv, gamma.detach(), sums, ctx.has_resid, dgam, dbet)
        if own_g:
            _notify(gamma)
        if own_b:
            _notify(beta)
        return (outs[0], None if own_g else dgam, None if own_b else dbet, outs[1] if ctx.has_resid else None,
                None, None, None, None, None, None)


def batch_norm_nhwc(y, gamma, beta, running_mean, running_var, eps=1e-5, momentum=0.1, relu=False, resid=None,
                    training=True):
    C = y.shape[-1]
    if y.is_cuda and C % 8 == 0:
        yb = y.to(torch.bfloat16).contiguous()
        r = None if resid is None else resid.to(torch.bfloat16).contiguous()
        out = _BNActFn.apply(yb, gamma, beta, r, running_mean, running_var, float(eps), float(momentum), bool(relu),
                             bool(training))
        return out if y.dtype == torch.bfloat16 else out.to(y.dtype)
    z = bn_ref(y, gamma, beta, running_mean, running_var, eps, momentum, training)
    if resid is not None:
        z = z + resid.float()
    if relu:
        z = torch.relu(z)
    return z.to(y.dtype)
