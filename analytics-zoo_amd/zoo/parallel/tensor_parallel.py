"""Tensor (intra-layer) model parallelism over RCCL.

The reference has no tensor parallelism; the survey asks that the GEMM API allow
column/row-split Linear layers. These are the two Megatron-style halves, built
on the framework's linear op (MFMA / hipBLASLt) and torch.distributed
collectives, so a transformer MLP or attention block can be split over the GPUs
of one xGMI island:

  * :class:`ColumnParallelLinear` — weight rows (output features) split over the
    group; input replicated; output either kept sharded (feed a row-parallel
    layer) or all-gathered.
  * :class:`RowParallelLinear` — weight columns (input features) split; input
    sharded on its last dim; partial outputs summed with ONE all-reduce.

Column -> Row needs exactly one all-reduce per MLP in forward and one in
backward (the copy-to-region / reduce-from-region conjugate pair below).
"""
import torch
import torch.distributed as dist
import torch.nn as nn

from zoo import ops


def _world(group):
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _rank(group):
    return dist.get_rank(group) if _world(group) > 1 else 0


class _CopyToRegion(torch.autograd.Function):
    """identity forward, all-reduce of the gradient backward"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        if _world(ctx.group) > 1:
            dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromRegion(torch.autograd.Function):
    """all-reduce forward, identity backward"""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        if _world(group) > 1:
            dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromRegion(torch.autograd.Function):
    """all-gather along the last dim forward, take own slice backward"""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        w = _world(group)
        if w == 1:
            return x
        parts = [torch.empty_like(x) for _ in range(w)]
        dist.all_gather(parts, x.contiguous(), group=group)
        ctx.n = x.shape[-1]
        return torch.cat(parts, dim=-1)

    @staticmethod
    def backward(ctx, g):
        if _world(ctx.group) == 1:
            return g, None
        r = _rank(ctx.group)
        return g[..., r * ctx.n:(r + 1) * ctx.n].contiguous(), None


def _shard(n, world, rank):
    if n % world:
        raise ValueError("dimension %d is not divisible by the tensor-parallel size %d" % (n, world))
    per = n // world
    return slice(rank * per, (rank + 1) * per)


class ColumnParallelLinear(nn.Module):
    tensor_parallel = True  # TrainingEngine: data-parallel sync only over replicas of this shard

    def __init__(self, in_features, out_features, bias=True, gather_output=False, group=None, init_weight=None,
                 init_bias=None, activation=None):
        super().__init__()
        self.group, self.gather_output, self.activation = group, gather_output, activation
        w, r = _world(group), _rank(group)
        sl = _shard(out_features, w, r)
        full_w = init_weight if init_weight is not None else \
            torch.empty(out_features, in_features).normal_(0.0, 0.02)
        self.weight = nn.Parameter(full_w[sl].clone())
        self.bias = None
        if bias:
            full_b = init_bias if init_bias is not None else torch.zeros(out_features)
            self.bias = nn.Parameter(full_b[sl].clone())

    def forward(self, x):
        x = _CopyToRegion.apply(x, self.group)
        y = ops.linear(x, self.weight, self.bias, act=self.activation)
        return _GatherFromRegion.apply(y, self.group) if self.gather_output else y


class RowParallelLinear(nn.Module):
    tensor_parallel = True

    def __init__(self, in_features, out_features, bias=True, input_is_parallel=True, group=None, init_weight=None,
                 init_bias=None):
        super().__init__()
        self.group, self.input_is_parallel = group, input_is_parallel
        w, r = _world(group), _rank(group)
        self.sl = _shard(in_features, w, r)
        full_w = init_weight if init_weight is not None else \
            torch.empty(out_features, in_features).normal_(0.0, 0.02)
        self.weight = nn.Parameter(full_w[:, self.sl].clone())
        # the bias is added once, after the reduction
        self.bias = nn.Parameter((init_bias if init_bias is not None else torch.zeros(out_features)).clone()) \
            if bias else None

    def forward(self, x):
        if not self.input_is_parallel:
            x = x[..., self.sl]
        y = _ReduceFromRegion.apply(ops.linear(x, self.weight, None), self.group)
        return y + self.bias.to(y.dtype) if self.bias is not None else y


class ParallelMLP(nn.Module):
    """Transformer MLP split over the group: column-parallel fc1 (+activation) ->
    row-parallel fc2; one all-reduce forward, one backward."""

    def __init__(self, hidden, inter, activation="gelu", group=None, fc1=None, fc2=None):
        super().__init__()
        self.fc1 = ColumnParallelLinear(hidden, inter, group=group, activation=activation,
                                        init_weight=None if fc1 is None else fc1[0],
                                        init_bias=None if fc1 is None else fc1[1])
        self.fc2 = RowParallelLinear(inter, hidden, group=group, init_weight=None if fc2 is None else fc2[0],
                                     init_bias=None if fc2 is None else fc2[1])

    def forward(self, x):
        return self.fc2(self.fc1(x))
