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

from zoo.ops._native import native, deterministic as _deterministic
from zoo.ops import _kern, workspace, wstream
from zoo.ops.conv import bf16_weight, ceil8, conv2d_ref, ref_relu, ref_storage
from zoo.parallel.sync_bn import all_reduce_stats, sync_batch_norm, sync_bn_active
from zoo.parallel.flat import grad_slot

# Per-channel statistics buffers are "slotted" ([2C final][STAT_SLOTS x 2C][counter]):
# producers spread their atomics over the slots and stats_finalize_kernel folds them
# (csrc/kernels/bn.hip). Must match zoo::kStatSlots.
STAT_SLOTS = 16

# How a consumer's fused BN-backward epilogue recovers this unit's ReLU mask (BwdStats.zmode,
# csrc/kernels/bnmask.h): 1 = recompute it from y (no residual) or read a 1-bit mask written by
# the forward apply (residual units); 0 = re-read the bf16 ReLU output z (A/B comparator).
_BN_MASK = True   # False: re-read the bf16 ReLU output z (test comparator)


# BatchNorm backward of a 1x1 / stride-1 conv -> BN unit as a PROLOGUE of its own dgrad
# (csrc/kernels/bnfold.hip, pw.hip PRO): when the consumer already produced the masked gradient g
# and its sums, dy = A g + B y + Cc is formed in the dgrad kernel's operand registers from g and
# the unit's y, and written once for the weight gradient -- no separate BN-backward pass and no
# re-read of dy (6 instead of 8 bytes per element). Shapes the prologue kernel does not take get
# dy materialised inside conv_fwd. ZOO_BN_FOLD=0 keeps bn_bwd_apply (A/B: profiles/r5/ab_bn_prologue_r5.md).
_BN_FOLD = [True]
# unit widths taken by the prologue (ZOO_BN_FOLD_K="64,128")
# the 1x1 stride-2 shortcut hands its data gradient to the block's conv1 in compact form
# (GradHandoff.half), added at the even positions by conv1's dgrad epilogue (pw.hip resid_half)
_HALF_RESID = True
# forward consumer-side BN apply for units of these widths (pw.hip prologue: K <= 128)
_FWD_PRO_K = (64, 128)
# ... and for RESIDUAL units (a ResNet block output consumed by the next block's 1x1 conv1, pw.hip EPI 4:
# the block's BN + residual + ReLU apply pass is gone, conv1 writes the block output and its mask)
_FWD_PRO_RES_K = (256,)
# 256: the stage-1 conv3 units (one 64-channel group): 12,804 / 12,822 -> 13,031 / 13,015 images/s with
# the band weight gradient (profiles/r6/ab1_r6.md)
_PRO_K = tuple(int(v) for v in __import__("os").environ.get("ZOO_BN_FOLD_K", "64,256").split(",") if v)
# wider units take the prologue only when their dgrad writes at most this many channels: one
# channel group in pw.hip, so the prologue (and its y / g reads) runs once, not Cin / 64 times
_PRO_NMAX = int(__import__("os").environ.get("ZOO_BN_FOLD_NMAX", "64"))


# projection shortcut (stride 1, stage 1 of ResNet-50): its BatchNorm backward as the shortcut
# dgrad's prologue instead of a bn_bwd_apply pass (oracle / A/B switch of round 6)
_SC_FOLD = True
# ... and its BN-backward sums taken in the consumer's epilogue (BNProducer.y2) instead of a
# bn_reduce pass over (dz, raw shortcut output)
_SC_SUMS = True


def _fold_ok(ctx, R, S, stride, pad, K, Cin, gamma):
    # K = 64 / 128: the widths whose prologue tile stays spill-free in registers (pw.hip PRO); wider
    # units and the deterministic mode (partial statistics: no pw) keep bn_bwd_apply
    return (_BN_FOLD[0] and R == 1 and S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0)
            and not getattr(ctx, "sync", False) and K in _PRO_K and Cin % 64 == 0 and (K <= 64 or Cin <= _PRO_NMAX)
            and gamma.dtype == torch.float32 and gamma.is_contiguous() and not _deterministic())


def stat_len(c):
    return 2 * int(c) * (STAT_SLOTS + 1) + 4


def _notify(p):
    hook = getattr(p, "_zoo_grad_ready", None)
    if hook is not None:
        hook(p)


def _grad_target(p):
    g = grad_slot(p)
    if g is not None:
        return g, True
    return torch.zeros(p.shape, dtype=torch.float32, device=p.device), False


class GradHandoff:
    """Carries the residual-branch gradient of a bottleneck's last conv to the
    block's FIRST conv, whose dgrad epilogue adds it (identity shortcut: both
    consume the block input). Replaces autograd's separate add kernel."""

    __slots__ = ("grad", "half")

    def __init__(self):
        self.grad = None
        self.half = False   # grad is the compact [N, H/2, W/2, C] gradient of a stride-2 1x1 shortcut


class BNProducer:
    """Handle attached to a conv->BN->ReLU unit's output. The single consumer
    conv of that output fuses this unit's BN-backward reduction (sum dy,
    sum dy*xhat) and ReLU mask into its dgrad epilogue (igemm BwdStats) and
    marks ``fused``; this unit's backward then skips its reduction pass."""

    # The producer's OUTPUT z is deliberately not held here: z -> grad_fn -> ctx ->
    # producer -> z would be a reference cycle that keeps every step's
    # activations alive until the cyclic GC runs. The consumer passes its own
    # saved input (which is z) to bstats() instead.
    # With ZOO_BN_MASK (default) the consumer never re-reads z for the mask: a unit without a
    # residual hands over its affine (gamma, beta) and the epilogue recomputes the sign from the
    # y it reads for the sums anyway; a residual unit hands over the 1-bit mask its forward
    # apply wrote (``mask``). 2 bytes per element less epilogue traffic either way.
    # Forward consumer-side apply (``fwd_pro``, set by the model when the single consumer is a 1x1
    # stride-1 conv): the unit skips its apply pass and leaves ``pending = (y, coef, z)`` -- z an
    # unwritten tensor -- and the consumer's conv forms z = relu(A y + Cc) in its operand prologue
    # (pw.hip), writing z as it goes. 2 bytes per element of the z re-read saved, and a launch.
    # ``y2``: a fused projection shortcut's raw output. Its BatchNorm receives the same gradient as
    # this unit's, so the consumer's epilogue also sums grad * y2 per channel into ``sums2`` and the
    # shortcut's BN backward needs no reduction pass of its own (pw.hip BwdStats.y2).
    __slots__ = ("relu", "y", "mean", "inv", "sums", "fused", "gamma", "beta", "mask", "fwd_pro", "pending",
                 "y2", "sums2")

    def __init__(self, relu, y, mean, inv):
        self.relu, self.y, self.mean, self.inv = relu, y, mean, inv
        self.sums = None
        self.fused = False
        self.gamma = self.beta = self.mask = None
        self.fwd_pro = False
        self.pending = None
        self.y2 = self.sums2 = None

    def bstats(self, z, y2_ok=True):
        """``y2_ok``: the consumer's dgrad runs on pw.hip with room for the second sums (a 1x1
        stride-1 dgrad with a <= 64-deep reduction when it has its own BN prologue, <= 128 without);
        otherwise the shortcut keeps its own reduction pass (cheaper than the generic fallback)."""
        self.sums = workspace.zeros(stat_len(self.y.shape[-1]), self.y.device)
        self.fused = True
        if not self.relu:
            t = (None, self.y, self.mean, self.inv, self.sums)
        elif self.mask is not None:
            t = (self.mask, self.y, self.mean, self.inv, self.sums)
        elif self.gamma is not None:
            t = (None, self.y, self.mean, self.inv, self.sums, self.gamma, self.beta)
        else:
            t = (z, self.y, self.mean, self.inv, self.sums)
        if self.y2 is not None and y2_ok:
            self.sums2 = torch.zeros(self.y.shape[-1], dtype=torch.float32, device=self.y.device)
            t = t + (None, None)[len(t) - 5:] + (self.y2, self.sums2)
        return t

    def release(self):
        self.y = self.mean = self.inv = self.sums = None
        self.gamma = self.beta = self.mask = None
        self.y2 = self.sums2 = None
        self.fused = False


def _sync_bwd(ctx, sums, K, m_local, dgam, dbet):
    """SyncBN backward: dgamma/dbeta take the LOCAL sums (the DP gradient sync
    combines ranks), then (sum dy, sum dy*xhat) are all-reduced for dx."""
    if not getattr(ctx, "sync", False):
        return dgam, dbet
    if dgam is not None:
        dgam.add_(sums[K:2 * K])
    if dbet is not None:
        dbet.add_(sums[:K])
    all_reduce_stats(sums[:2 * K], m_local)
    return None, None


class _ConvBNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, gamma, beta, resid, running_mean, running_var, R, S, stride, pad, eps, momentum,
                relu, training, handoff_out=None, handoff_in=None, producer_in=None, producer_out=None,
                dx_out=None, resid_bn=None, gamma2=None, beta2=None):
        C_ = native()
        K = w.shape[0]
        ctx.resid_bn = resid_bn if (resid_bn is not None and training) else None
        ctx.handoff_out, ctx.handoff_in, ctx.dx_out = handoff_out, handoff_in, dx_out
        ctx.producer_in = producer_in
        wb = bf16_weight(w)
        stats = workspace.zeros(stat_len(K), x.device) if training else None
        pend = producer_in.pending if producer_in is not None else None
        if pend is not None:
            # this conv applies the producer's BN (+ residual) + ReLU in its operand prologue and
            # writes x (= z, and the producer's ReLU mask for a residual unit)
            producer_in.pending = None
            y = _kern.conv_fwd(pend[0], wb, R, S, stride, pad, stats=stats, pro_fwd=(pend[1], x) + tuple(pend[2:]))
        else:
            y = _kern.conv_fwd(x, wb, R, S, stride, pad, stats=stats)
        ctx.sync = bool(training) and sync_bn_active()
        if ctx.sync:  # SyncBN (P5): global statistics over the data-parallel group
            all_reduce_stats(stats[:2 * K], y.numel() // K)
        smean = torch.empty(K, device=x.device, dtype=torch.float32)
        sinv = torch.empty(K, device=x.device, dtype=torch.float32)
        rb = ctx.resid_bn
        side = []
        if rb is not None:
            # `resid` is the raw shortcut conv output: its BatchNorm runs inside this apply pass
            rb.smean = torch.empty(K, device=x.device, dtype=torch.float32)
            rb.sinv = torch.empty(K, device=x.device, dtype=torch.float32)
            side = [rb.stats, gamma2.detach(), beta2.detach(), rb.running_mean, rb.running_var, rb.smean, rb.sinv]
            ctx.gamma2, ctx.beta2 = gamma2, beta2
        if training:
            _kern.bump_stats_epoch()
        mask = None
        po = producer_out if (training and relu and _BN_MASK) else None
        if po is not None and resid is not None:
            mask = torch.empty(y.numel() // 8, device=x.device, dtype=torch.uint8)
        if (po is not None and po.fwd_pro and resid is None and rb is None and not ctx.sync and K in _FWD_PRO_K
                and gamma.dtype == torch.float32 and beta.dtype == torch.float32):
            # consumer-side apply: statistics bookkeeping + affine here, z formed by the consumer
            coef = C_.bn_fwd_coef(stats, gamma.detach().contiguous(), beta.detach().contiguous(), running_mean,
                                  running_var, smean, sinv, y.numel() // K, eps, momentum)
            z = torch.empty_like(y)
            po.pending = (y, coef)
        elif (po is not None and po.fwd_pro and mask is not None and not ctx.sync and K in _FWD_PRO_RES_K
              and not _deterministic() and resid.dtype == torch.bfloat16 and resid.is_contiguous()
              and resid.shape == y.shape and gamma.dtype == torch.float32 and beta.dtype == torch.float32
              and (rb is None or (gamma2.dtype == torch.float32 and beta2.dtype == torch.float32))):
            # residual unit, consumer-side: the next block's conv1 forms z = relu(A y + Cc + R) and the
            # mask; here only the statistics bookkeeping (both BatchNorms) and the affine coefficients
            M_ = y.numel() // K
            coef = C_.bn_fwd_coef(stats, gamma.detach().contiguous(), beta.detach().contiguous(), running_mean,
                                  running_var, smean, sinv, M_, eps, momentum)
            rcoef = None
            if rb is not None:
                rcoef = C_.bn_fwd_coef(rb.stats, gamma2.detach().contiguous(), beta2.detach().contiguous(),
                                       rb.running_mean, rb.running_var, rb.smean, rb.sinv, M_, eps, momentum)
            z = torch.empty_like(y)
            po.pending = (y, coef, resid, rcoef, mask)
        else:
            z = C_.bn_fwd_apply(y, stats if training else torch.empty(0, device=x.device), gamma.detach(),
                                beta.detach(), resid, running_mean, running_var, smean, sinv, eps, momentum, relu,
                                training, side, mask)
        if po is not None:
            po.mask = mask
            if resid is None:
                po.gamma, po.beta = gamma.detach(), beta.detach()
            # the fused shortcut BatchNorm's sums come from the consumer's epilogue (not under SyncBN:
            # there the two BNs all-reduce their own sums)
            po.y2 = resid if (_SC_SUMS and rb is not None and not ctx.sync and not _deterministic()) else None
        if rb is not None:
            ctx.yres = resid        # shortcut conv output: its BN backward needs it
        ctx.save_for_backward(x, w, gamma, y, z if relu else None, smean, sinv)
        ctx.meta = (R, S, stride, pad, relu, resid is not None, x.shape)
        ctx.producer_out = producer_out
        if producer_out is not None:
            producer_out.relu, producer_out.y, producer_out.mean, producer_out.inv = bool(relu), y, smean, sinv
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
        dgam, own_g = _grad_target(gamma)
        dbet, own_b = _grad_target(ctx.beta_ref) if hasattr(ctx, "beta_ref") else (None, False)
        po = ctx.producer_out
        fold = None
        if po is not None and po.fused:
            # dz arrived already ReLU-masked with its (dy, dy*xhat) sums from the consumer's epilogue
            sums = po.sums
            if _fold_ok(ctx, R, S, stride, pad, K, Cin, gamma):
                # the BN backward runs as the dgrad's prologue (see _BN_FOLD); dy is its by-product
                coef = C_.bnfold_coef(gamma.detach(), smean, sinv, sums, y.numel() // K, dgam, dbet)
                dy = torch.empty_like(dz)
                fold = (y, coef, dy)
            else:
                dg, db = _sync_bwd(ctx, sums, K, y.numel() // K, dgam, dbet)
                outs = C_.bn_bwd_apply(dz, None, y, smean, sinv, gamma.detach(), sums, False, dg, db)
                dy = outs[0]
            dresid = dz if has_resid else None
            sc_sums = (sums, po.sums2) if po.sums2 is not None else None
            po.release()
        else:
            sc_sums = None
            sums = workspace.zeros(stat_len(K), dz.device)
            C_.bn_reduce(dz, z, y, smean, sinv, sums, 1)
            dg, db = _sync_bwd(ctx, sums, K, y.numel() // K, dgam, dbet)
            outs = C_.bn_bwd_apply(dz, z, y, smean, sinv, gamma.detach(), sums, has_resid, dg, db)
            dy = outs[0]
            dresid = outs[1] if has_resid else None
        if dresid is not None and ctx.handoff_out is not None:
            ctx.handoff_out.grad = dresid   # consumed by the block's first conv (fused add)
            dresid = None
        dgam2 = dbet2 = None
        if ctx.resid_bn is not None and dresid is not None:
            dresid, dgam2, dbet2 = _shortcut_bn_bwd(ctx, dresid, K, sc_sums)
        dx = None
        if ctx.needs_input_grad[0]:
            add, half = None, False
            if ctx.handoff_in is not None:
                add, half = ctx.handoff_in.grad, ctx.handoff_in.half
                ctx.handoff_in.grad, ctx.handoff_in.half = None, False
                if add is None:
                    raise RuntimeError("GradHandoff: residual gradient missing (backward order violated)")
            if half and tuple(stride) != (1, 1):   # only a stride-1 dgrad epilogue reads the compact form
                full = torch.zeros(xshape[0], xshape[1], xshape[2], Cin, dtype=add.dtype, device=add.device)
                full[:, ::2, ::2] = add
                add, half = full, False
            pin = ctx.producer_in
            y2_ok = (R, S) == (1, 1) and tuple(stride) == (1, 1) and K <= (64 if fold is not None else 128)
            bst = pin.bstats(x, y2_ok) if (pin is not None and pin.y is not None) else None
            # a handed-off gradient is a temporary owned by this unit now: accumulate into it in place
            dx = _kern.conv_dgrad(dz if fold is not None else dy, bf16_weight(w), K, R, S, Cin, xshape[1],
                                  xshape[2], stride, pad, resid=add, bstats=bst, resid_inplace=add is not None,
                                  pro=fold, resid_half=half)
            if ctx.dx_out is not None:
                # another consumer of x adds this gradient in its own dgrad epilogue
                ctx.dx_out.grad = dx
                dx = None
        elif fold is not None:
            C_.bnpro_apply(dz, fold[0], fold[1], dy)   # no data gradient: dy for the wgrad alone
        gw, own_w = _grad_target(w)
        with wstream.wgrad(dy.device, x, dy, on=own_w):
            C_.conv_wgrad(x, dy, gw, R, S, stride[0], stride[1], pad[0], pad[1], 1, 1)
            if own_w:
                _notify(w)
        if own_g:
            _notify(gamma)
        if own_b:
            _notify(ctx.beta_ref)
        return (dx, None if own_w else gw.to(w.dtype), None if own_g else dgam, None if own_b else dbet, dresid,
                None, None, None, None, None, None, None, None, None, None, None, None, None, None, None,
                None, dgam2, dbet2)


class _ConvBNActFnB(_ConvBNActFn):
    """Same as _ConvBNActFn but keeps a handle on beta for its gradient."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, resid, running_mean, running_var, R, S, stride, pad, eps, momentum,
                relu, training, handoff_out=None, handoff_in=None, producer_in=None, producer_out=None,
                dx_out=None, resid_bn=None, gamma2=None, beta2=None):
        ctx.beta_ref = beta
        return _ConvBNActFn.forward(ctx, x, w, gamma, beta, resid, running_mean, running_var, R, S, stride, pad,
                                    eps, momentum, relu, training, handoff_out, handoff_in, producer_in,
                                    producer_out, dx_out, resid_bn, gamma2, beta2)


class ShortcutBN:
    """The BatchNorm of a projection shortcut whose apply is fused into the block's last
    unit: ``conv_stats`` fills ``stats`` (the shortcut conv's epilogue statistics), the last
    unit's BN apply normalises the raw shortcut output with them in the same pass
    (bn_fwd_apply resid_bn) and its backward runs this BatchNorm's backward, handing the
    shortcut conv the gradient of its raw output. The shortcut's own apply pass and its
    normalised output tensor are never materialised."""
    __slots__ = ("stats", "running_mean", "running_var", "smean", "sinv", "sync", "m_local", "conv_geo", "fold")

    def __init__(self, running_mean, running_var):
        self.running_mean, self.running_var = running_mean, running_var
        self.stats = self.smean = self.sinv = None
        self.sync, self.m_local = False, 0
        self.conv_geo = None   # (R, S, stride, pad, Cin) of the shortcut conv (set by its forward)
        self.fold = None       # (y_raw, coef, dy_out): BN backward handed to the shortcut dgrad's prologue


def _shortcut_bn_bwd(ctx, dres, K, pre=None):
    """BatchNorm backward of the fused shortcut: (sum dz, sum dz*xhat) over the raw
    shortcut output, then dx = A dz + B x + D. Returns (d_raw, dgamma2, dbeta2).
    ``pre = (main sums, sum dz * y_raw)`` from the consumer's epilogue (BNProducer.y2): the
    shortcut's sums follow without a pass, sum dz*xhat = inv (sum dz*y - mean sum dz)."""
    C_ = native()
    rb, yres = ctx.resid_bn, ctx.yres
    gamma2, beta2 = ctx.gamma2, ctx.beta2
    sums = workspace.zeros(stat_len(K), dres.device)
    if pre is not None:
        s1 = pre[0][:K]
        sums[:K].copy_(s1)
        sums[K:2 * K].copy_(rb.sinv * (pre[1] - rb.smean * s1))
    else:
        C_.bn_reduce(dres, None, yres, rb.smean, rb.sinv, sums, 1)
    dgam, own_g = _grad_target(gamma2)
    dbet, own_b = _grad_target(beta2)
    dg, db = dgam, dbet
    if rb.sync:
        if dgam is not None:
            dgam.add_(sums[K:2 * K])
        if dbet is not None:
            dbet.add_(sums[:K])
        all_reduce_stats(sums[:2 * K], rb.m_local)
        dg = db = None
    geo = rb.conv_geo
    if (_SC_FOLD and geo is not None and not rb.sync and gamma2.dtype == torch.float32 and gamma2.is_contiguous()
            and _fold_ok(ctx, geo[0], geo[1], geo[2], geo[3], K, geo[4], gamma2)):
        # the shortcut conv's dgrad forms d_raw = A dz + B y_raw + Cc in its operand prologue and
        # writes it for its weight gradient (pw.hip PRO, as the block's own 1x1 units): the
        # shortcut's bn_bwd_apply pass is gone (ResNet stage 1 block 1: 64 -> 256, 281 us at b256,
        # profiles/r6/ab4_prof_rn_step_r6.md row 347). The returned gradient is dz; the shortcut's
        # backward (_ConvStatsFn) finds the fold on the holder.
        coef = C_.bnfold_coef(gamma2.detach(), rb.smean, rb.sinv, sums, yres.numel() // K, dg, db)
        rb.fold = (yres, coef, torch.empty_like(dres))
        out = dres
    else:
        out = C_.bn_bwd_apply(dres, None, yres, rb.smean, rb.sinv, gamma2.detach(), sums, False, dg, db)[0]
    if own_g:
        _notify(gamma2)
    if own_b:
        _notify(beta2)
    ctx.yres = ctx.resid_bn = None
    return out, (None if own_g else dgam), (None if own_b else dbet)


class _ConvStatsFn(torch.autograd.Function):
    """Projection-shortcut conv with BatchNorm statistics only (its BN is applied by the
    block's last unit, see ShortcutBN). Backward: dgrad (adding the gradient handed off by
    the block's first conv, GradHandoff) + wgrad of the raw-output gradient."""

    @staticmethod
    def forward(ctx, x, w, R, S, stride, pad, holder, handoff_in, dx_out=None):
        K = w.shape[0]
        stats = workspace.zeros(stat_len(K), x.device)
        y = _kern.conv_fwd(x, bf16_weight(w), R, S, stride, pad, stats=stats)
        holder.sync = sync_bn_active()
        holder.m_local = y.numel() // K
        if holder.sync:
            all_reduce_stats(stats[:2 * K], holder.m_local)
        holder.stats = stats
        holder.conv_geo = (R, S, tuple(stride), tuple(pad), x.shape[3])
        holder.fold = None
        ctx.save_for_backward(x, w)
        ctx.meta = (R, S, stride, pad, x.shape)
        ctx.handoff_in = handoff_in
        ctx.dx_out = dx_out
        ctx.holder = holder
        return y

    @staticmethod
    def backward(ctx, dy):
        C_ = native()
        x, w = ctx.saved_tensors
        R, S, stride, pad, xshape = ctx.meta
        dy = dy.contiguous()
        if dy.dtype != torch.bfloat16:
            dy = dy.to(torch.bfloat16)
        K = w.shape[0]
        dx = None
        fold, ctx.holder.fold = ctx.holder.fold, None
        if ctx.needs_input_grad[0]:
            add = None
            if ctx.handoff_in is not None:
                add = ctx.handoff_in.grad
                ctx.handoff_in.grad = None
                if add is None:
                    raise RuntimeError("GradHandoff: residual gradient missing (backward order violated)")
            if fold is not None:
                # dy is the block output's dz: the shortcut BN backward runs in this dgrad's prologue
                dx = _kern.conv_dgrad(dy, bf16_weight(w), K, R, S, xshape[3], xshape[1], xshape[2], stride, pad,
                                      resid=add, resid_inplace=add is not None, pro=fold)
                dy = fold[2]
            elif (_HALF_RESID and add is None and ctx.dx_out is not None and (R, S) == (1, 1) and stride == (2, 2)
                    and pad == (0, 0) and xshape[1] % 2 == 0 and xshape[2] % 2 == 0):
                # 1x1 stride 2: the gradient is zero at every odd position -- hand the block's conv1
                # the compact [N, H/2, W/2, C] values, its dgrad epilogue adds them at the even ones
                ctx.dx_out.grad = _kern.conv_dgrad_s2_compact(dy, bf16_weight(w), K, xshape[3])
                ctx.dx_out.half = True
                dx = None
            else:
                dx = _kern.conv_dgrad(dy, bf16_weight(w), K, R, S, xshape[3], xshape[1], xshape[2], stride, pad,
                                      resid=add, resid_inplace=add is not None)
            if dx is not None and ctx.dx_out is not None:
                # the other consumer of x (the block's conv1) adds it in its dgrad epilogue
                ctx.dx_out.grad = dx
                dx = None
        elif fold is not None:
            C_.bnpro_apply(dy, fold[0], fold[1], fold[2])   # no data gradient: d_raw for the wgrad alone
            dy = fold[2]
        gw, own_w = _grad_target(w)
        with wstream.wgrad(dy.device, x, dy, on=own_w):
            C_.conv_wgrad(x, dy, gw, R, S, stride[0], stride[1], pad[0], pad[1], 1, 1)
            if own_w:
                _notify(w)
        return dx, None if own_w else gw.to(w.dtype), None, None, None, None, None, None, None


def conv_stats(x, w, running_mean, running_var, kernel=(1, 1), stride=(1, 1), pad=(0, 0), grad_add=None,
               dx_handoff=None):
    """Training-mode projection shortcut (GPU): (raw conv output, ShortcutBN) -- the BN is
    applied by the consumer unit (``conv_bn_act(..., resid=raw, resid_bn=holder, ...)``).
    ``grad_add`` / ``dx_handoff``: see :func:`conv_bn_act`."""
    holder = ShortcutBN(running_mean, running_var)
    xb = (x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)).contiguous()
    y = _ConvStatsFn.apply(xb, w, kernel[0], kernel[1], tuple(stride), tuple(pad), holder, grad_add, dx_handoff)
    return y, holder


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


def _folded(w, gamma, beta, running_mean, running_var, eps, cols=None):
    """Inference-time BatchNorm folding: W' = W * gamma/sqrt(var+eps) (per output row),
    b' = beta - mean * gamma/sqrt(var+eps). Cached on the weight parameter and rebuilt
    when any of the five tensors changes (in-place updates bump ``_version``)."""
    # the engine's fused optimizer writes weights, and the native BN kernels write running
    # statistics, through raw pointers (no ``_version`` bump): the two epochs cover those writers
    key = tuple((t.data_ptr(), t._version) for t in (w, gamma, beta, running_mean, running_var)) + (
        float(eps), _kern.weights_epoch(), _kern.stats_epoch())
    c = getattr(w, "_zoo_bn_fold", None)
    if c is not None and c[0] == key:
        return c[1], c[2]
    with torch.no_grad():
        scale = gamma.float() * torch.rsqrt(running_var.float() + eps)
        bias = (beta.float() - running_mean.float() * scale).contiguous()
        shape = (-1,) + (1,) * (w.dim() - 1) if cols is None else (1, -1)
        wf = (w.float() * scale.reshape(shape)).to(torch.bfloat16).contiguous()
    try:
        w._zoo_bn_fold = (key, wf, bias)
    except (AttributeError, RuntimeError):
        pass
    return wf, bias


def conv_bn_act_eval(x, w, gamma, beta, running_mean, running_var, kernel, stride, pad, eps, relu, resid=None):
    """Eval-mode conv -> BN(running stats) -> (+resid) -> ReLU as ONE implicit-GEMM
    launch: BN folded into the weights and a bias, residual add and ReLU in the epilogue
    (no statistics, no separate apply pass)."""
    wf, bf = _folded(w, gamma, beta, running_mean, running_var, eps)
    r = None if resid is None else resid.to(torch.bfloat16).contiguous()
    return _kern.conv_fwd(x.to(torch.bfloat16).contiguous(), wf, kernel[0], kernel[1], stride, pad, bias=bf,
                          resid=r, act=1 if relu else 0)


def conv_bn_act(x, w, gamma, beta, running_mean, running_var, kernel=(1, 1), stride=(1, 1), pad=(0, 0),
                eps=1e-5, momentum=0.1, relu=True, resid=None, training=True, resid_handoff=None, grad_add=None,
                producer_in=None, producer_out=None, dx_handoff=None, resid_bn=None):
    """z = relu?(BN(conv(x)) + resid) for NHWC input with a packed weight.

    ``resid_handoff``/``grad_add``: a shared :class:`GradHandoff` that routes the
    residual gradient of the unit with ``resid`` into the dgrad epilogue of the
    unit that consumes the same input first (GPU only).
    ``producer_in``: the :class:`BNProducer` of the unit that produced ``x``,
    when this unit is its ONLY consumer (fuses that unit's BN-backward
    reduction into this unit's dgrad). ``producer_out``: a fresh BNProducer
    to be filled for this unit's own output. ``dx_handoff``: this unit's input
    gradient is handed to the unit whose ``grad_add`` is the same GradHandoff
    (which must run its backward later) instead of being returned — two
    consumers of one tensor then need no separate gradient-add pass.
    ``resid_bn``: ``(ShortcutBN, gamma2, beta2)`` -- ``resid`` is a raw shortcut conv output
    (``conv_stats``) whose BatchNorm is applied in this unit's apply pass (GPU training)."""
    R, S = kernel
    if x.is_cuda and not training and not (torch.is_grad_enabled() and (x.requires_grad or w.requires_grad)):
        return conv_bn_act_eval(x, w, gamma, beta, running_mean, running_var, kernel, tuple(stride), tuple(pad),
                                eps, relu, resid)
    if x.is_cuda:
        if x.dtype != torch.bfloat16:
            x = x.to(torch.bfloat16)
        if resid is not None:
            resid = resid.to(torch.bfloat16).contiguous()
        holder, g2, b2 = resid_bn if resid_bn is not None else (None, None, None)
        if holder is not None and not training:
            raise ValueError("conv_bn_act: resid_bn (fused shortcut BatchNorm) is a training-mode path")
        return _ConvBNActFnB.apply(x.contiguous(), w, gamma, beta, resid, running_mean, running_var, R, S,
                                   tuple(stride), tuple(pad), float(eps), float(momentum), bool(relu),
                                   bool(training), resid_handoff, grad_add, producer_in, producer_out, dx_handoff,
                                   holder, g2, b2)
    if resid_bn is not None:
        raise ValueError("conv_bn_act: resid_bn (fused shortcut BatchNorm) needs the GPU path")
    y = ref_storage(conv2d_ref(x, w, (R, S, x.shape[3], tuple(stride), tuple(pad), (1, 1))))
    if training and sync_bn_active():
        z = sync_batch_norm(y.float(), gamma, beta, running_mean, running_var, eps, momentum)
    else:
        z = bn_ref(y, gamma, beta, running_mean, running_var, eps, momentum, training)
    if resid is not None:
        z = z + resid.float()
    if relu:
        z = ref_relu(z)
    return z.to(x.dtype) if x.dtype != torch.float32 else z


class _BNActFn(torch.autograd.Function):
    """Standalone NHWC BatchNorm (+residual, +ReLU) when there is no producing conv."""

    @staticmethod
    def forward(ctx, y, gamma, beta, resid, running_mean, running_var, eps, momentum, relu, training):
        C_ = native()
        K = y.shape[-1]
        stats = workspace.zeros(stat_len(K), y.device) if training else torch.empty(0, device=y.device)
        ctx.sync = bool(training) and sync_bn_active()
        if training:
            C_.bn_reduce(y, None, None, None, None, stats, 0)
            if ctx.sync:
                all_reduce_stats(stats[:2 * K], y.numel() // K)
        smean = torch.empty(K, device=y.device, dtype=torch.float32)
        sinv = torch.empty(K, device=y.device, dtype=torch.float32)
        if training:
            _kern.bump_stats_epoch()
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
        sums = workspace.zeros(stat_len(K), dz.device)
        C_.bn_reduce(dz, z, y, smean, sinv, sums, 1)
        dgam, own_g = _grad_target(gamma)
        dbet, own_b = _grad_target(beta)
        dg, db = _sync_bwd(ctx, sums, K, y.numel() // K, dgam, dbet)
        outs = C_.bn_bwd_apply(dz, z, y, smean, sinv, gamma.detach(), sums, ctx.has_resid, dg, db)
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
    if training and sync_bn_active():
        z = sync_batch_norm(y.float(), gamma, beta, running_mean, running_var, eps, momentum)
    else:
        z = bn_ref(y, gamma, beta, running_mean, running_var, eps, momentum, training)
    if resid is not None:
        z = z + resid.float()
    if relu:
        z = ref_relu(z)
    return z.to(y.dtype)


class _BNReluMaxPoolFn(torch.autograd.Function):
    """Training-mode BatchNorm -> ReLU -> max-pool over a RAW conv output whose statistics
    the conv epilogue produced (``conv_stats``): one pass forward, two backward, and the
    [N,H,W,C] BN output is never materialised (csrc/kernels/bn.hip, stem fusion)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, holder, eps, momentum, R, S, sh, sw, ph, pw):
        K = y.shape[-1]
        smean = torch.empty(K, device=y.device, dtype=torch.float32)
        sinv = torch.empty(K, device=y.device, dtype=torch.float32)
        _kern.bump_stats_epoch()
        out, best, arg = native().bn_relu_maxpool_fwd(y, holder.stats, gamma.detach().float().contiguous(),
                                                      beta.detach().float().contiguous(), holder.running_mean,
                                                      holder.running_var, smean, sinv, eps, momentum,
                                                      R, S, sh, sw, ph, pw)
        holder.stats = None
        ctx.save_for_backward(y, gamma, beta, best, arg, smean, sinv)
        ctx.geom = (R, S, sh, sw, ph, pw)
        ctx.mark_non_differentiable(best, arg)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, gamma, beta, best, arg, smean, sinv = ctx.saved_tensors
        dout = dout.contiguous()
        if dout.dtype != torch.bfloat16:
            dout = dout.to(torch.bfloat16)
        K = y.shape[-1]
        sums = workspace.zeros(stat_len(K), dout.device)
        dgam, own_g = _grad_target(gamma)
        dbet, own_b = _grad_target(beta)
        dx = native().bn_relu_maxpool_bwd(dout, best, arg, y, smean, sinv, gamma.detach().float().contiguous(),
                                          sums, dgam, dbet, *ctx.geom)
        if own_g:
            _notify(gamma)
        if own_b:
            _notify(beta)
        return (dx, None if own_g else dgam, None if own_b else dbet) + (None,) * 9


def stem_pool_fusable(y, kernel, pad):
    """Whether ``bn_relu_maxpool`` applies: GPU, power-of-two C/8 <= 256, no SyncBN, and not
    the deterministic mode (its pooled-space reduction uses fp32 atomics)."""
    from zoo.ops._native import deterministic
    cpr = y.shape[-1] // 8
    return (y.is_cuda and y.shape[-1] % 8 == 0 and 0 < cpr <= 256 and (cpr & (cpr - 1)) == 0
            and kernel[0] * kernel[1] < 255 and not sync_bn_active() and not deterministic())


def bn_relu_maxpool(y, holder, gamma, beta, eps=1e-5, momentum=0.1, kernel=(3, 3), stride=(2, 2), pad=(1, 1)):
    """relu(BN(y)) -> max_pool for a raw conv output ``y`` with its ``conv_stats`` holder
    (training, GPU). Equals ``max_pool2d_nhwc(batch_norm_nhwc(y, ..., relu=True), ...)``."""
    return _BNReluMaxPoolFn.apply(y, gamma, beta, holder, float(eps), float(momentum), kernel[0], kernel[1],
                                  stride[0], stride[1], pad[0], pad[1])
