"""Flat parameter / gradient storage (the MI355X analogue of BigDL's flat
parameter vector that AllReduceParameter shards, SURVEY.md §2.4 "DistriOptimizer
iteration", Topology.scala:1122-1128).

All trainable parameters of a model are re-homed into three contiguous buffers:

  master : fp32 weights (the optimizer's copy)
  grad   : fp32 gradients — the native backward kernels accumulate into it
           directly (conv wgrad atomics, BN dgamma/dbeta), so there is no
           per-parameter ``.grad`` allocation and no extra accumulation pass
  bf16   : the bf16 compute copy the forward kernels read; rewritten by the
           fused optimizer kernel in the same pass that updates ``master``

Parameters are laid out in REVERSE registration order, i.e. roughly the order
in which backward produces their gradients, so gradient buckets for the
all-reduce fill front-to-back and can be launched while backward continues.
Every parameter starts on a 64-element boundary (256-byte fp32 / 128-byte
bf16 alignment for vector loads).
"""
import torch

ALIGN = 64


def grad_slot(p):
    """The flat gradient view of ``p`` that native backward kernels write into (None when no
    engine owns p's gradient). Native ops call this right before they enqueue such a write, so
    a ``_zoo_grad_pre`` hook (the in-backward optimizer, GradSync._ibo_pre) can order the write
    after an update of the same slot that is already in flight on another stream."""
    g = getattr(p, "_zoo_grad", None)
    if g is not None:
        pre = getattr(p, "_zoo_grad_pre", None)
        if pre is not None:
            pre(p)
    return g


def _align(n, a=ALIGN):
    return (n + a - 1) // a * a


class FlatParams:
    def __init__(self, params, device=None, bf16_copy=True):
        seen = set()
        uniq = []
        for p in params:
            if id(p) in seen or not p.requires_grad:
                continue
            seen.add(id(p))
            uniq.append(p)
        self.params = list(reversed(uniq))
        dev = torch.device(device) if device is not None else (self.params[0].device if self.params else
                                                               torch.device("cpu"))
        self.device = dev
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _align(p.numel())
        self.numel = max(off, ALIGN)
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=dev)
        # True while every gradient slot is known to be 0 (fresh, or cleared by the optimizer
        # kernel that consumed it): the engine then skips its per-step fill of the buffer
        self.grad_clean = True
        self.bf16 = torch.zeros(self.numel, dtype=torch.bfloat16, device=dev) if bf16_copy else None
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.master[o:o + n].copy_(p.detach().reshape(-1).to(dev, torch.float32))
            p.data = self.master[o:o + n].view(p.shape)
            gview = self.grad[o:o + n].view(p.shape)
            p._zoo_grad = gview
            p.grad = gview
            if self.bf16 is not None:
                p._zoo_bf16 = self.bf16[o:o + n].view(p.shape)
        if self.bf16 is not None:
            from zoo.ops._kern import register_flat
            register_flat(self)
        self.refresh_bf16()

    # ------------------------------------------------------------------
    def refresh_bf16(self):
        if self.bf16 is not None:
            self.bf16.copy_(self.master)
            from zoo.ops._kern import bump_weights_epoch
            bump_weights_epoch()

    def zero_grad(self):
        self.grad.zero_()
        # keep .grad pointing at the flat views (torch may reset it to None)
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != p._zoo_grad.data_ptr():
                p.grad = p._zoo_grad

    def param_range(self, p):
        i = next(i for i, q in enumerate(self.params) if q is p)
        return self.offsets[i], self.offsets[i] + p.numel()

    def ranges(self):
        return [(o, o + p.numel()) for p, o in zip(self.params, self.offsets)]

    def state_dict(self):
        return {"master": self.master.detach().cpu()}

    def load_master(self, t):
        self.master.copy_(t.to(self.master.device))
        self.refresh_bf16()

    def detach(self):
        """Give parameters private storage again (undo the flat re-homing)."""
        for p in self.params:
            p.data = p.data.clone()
            for a in ("_zoo_grad", "_zoo_bf16", "_zoo_grad_pre"):
                if hasattr(p, a):
                    delattr(p, a)
            p.grad = None
