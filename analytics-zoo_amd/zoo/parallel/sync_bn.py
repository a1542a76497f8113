"""Synchronised BatchNorm across data-parallel ranks.

The reference shares BatchNorm statistics among the per-core model replicas of
one node (``BatchNormalization.setParallism``, Zs/examples/resnet/
TrainImageNet.scala:86-94, 145-153). Here the replicas are one process per GPU,
so the statistics are all-reduced over RCCL (xGMI): forward reduces the
per-channel (sum, sum of squares, count), backward the per-channel
(sum dy, sum dy*xhat). Each is ONE small all-reduce of 2C+1 floats per BN layer.

Enable for a process group with :func:`set_sync_bn` (``True`` = the default
world group). It applies to the Keras ``BatchNormalization`` layer and to the
fused conv+BN units of the ResNet models; it is off by default because each BN
layer then costs two latency-bound collectives per step.
"""
import torch
import torch.distributed as dist

_state = {"group": None, "on": False}


def set_sync_bn(group=True):
    """``group``: True (world), a ProcessGroup, or False/None to disable."""
    if group is False or group is None:
        _state.update(on=False, group=None)
    else:
        _state.update(on=True, group=None if group is True else group)


def sync_bn_active():
    return _state["on"] and dist.is_available() and dist.is_initialized() and \
        dist.get_world_size(_state["group"]) > 1


def sync_group():
    return _state["group"]


def all_reduce_stats(buf2c, m_local):
    """In place: all-reduce [sum | sumsq] (or [sum dy | sum dy*xhat]) over the
    sync group and rescale by m_local / m_global so kernels that divide by their
    LOCAL row count produce global means. Returns m_global."""
    g = sync_group()
    cnt = torch.tensor([float(m_local)], dtype=buf2c.dtype, device=buf2c.device)
    both = torch.cat([buf2c.reshape(-1), cnt])
    dist.all_reduce(both, group=g)
    m_global = both[-1]
    buf2c.copy_(both[:-1].reshape(buf2c.shape) * (float(m_local) / m_global))
    return m_global


class _SyncBNFn(torch.autograd.Function):
    """Channels-last SyncBN: x [..., C] -> y [..., C] (fp32 math)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, running_mean, running_var, eps, momentum):
        C = x.shape[-1]
        xf = x.reshape(-1, C).float()
        m = xf.shape[0]
        stats = torch.cat([xf.sum(0), (xf * xf).sum(0), torch.tensor([float(m)], device=x.device)])
        dist.all_reduce(stats, group=sync_group())
        n = stats[-1]
        mean = stats[:C] / n
        var = (stats[C:2 * C] / n - mean * mean).clamp_min(0.0)
        inv = torch.rsqrt(var + eps)
        if running_mean is not None:
            with torch.no_grad():
                running_mean.mul_(1 - momentum).add_(momentum * mean)
                running_var.mul_(1 - momentum).add_(momentum * var * n / torch.clamp(n - 1, min=1))
        xhat = (xf - mean) * inv
        y = xhat * gamma.float() + beta.float()
        ctx.save_for_backward(xhat, inv, gamma)
        ctx.n = n
        return y.reshape(x.shape).to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        xhat, inv, gamma = ctx.saved_tensors
        C = xhat.shape[-1]
        dyf = dy.reshape(-1, C).float()
        s1 = dyf.sum(0)
        s2 = (dyf * xhat).sum(0)
        dgamma, dbeta = s2.clone(), s1.clone()   # local: the DP gradient sync sums these
        both = torch.cat([s1, s2])
        dist.all_reduce(both, group=sync_group())
        n = ctx.n
        m1, m2 = both[:C] / n, both[C:] / n
        dx = gamma.float() * inv * (dyf - m1 - xhat * m2)
        return dx.reshape(dy.shape).to(dy.dtype), dgamma.to(gamma.dtype), dbeta.to(gamma.dtype), None, None, \
            None, None


def sync_batch_norm(x, gamma, beta, running_mean, running_var, eps=1e-5, momentum=0.1, channel_dim=-1):
    """Training-mode BatchNorm whose statistics span every rank of the sync group."""
    if channel_dim not in (-1, x.dim() - 1):
        xt = x.movedim(channel_dim, -1)
        return _SyncBNFn.apply(xt.contiguous(), gamma, beta, running_mean, running_var, float(eps),
                               float(momentum)).movedim(-1, channel_dim)
    return _SyncBNFn.apply(x.contiguous(), gamma, beta, running_mean, running_var, float(eps), float(momentum))
