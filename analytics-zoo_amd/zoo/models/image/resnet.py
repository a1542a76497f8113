"""ResNet (v1.5, NHWC, bf16) built on the zoo gfx950 kernels.

The reference trains ResNet-50 through BigDL's MKL-DNN graph
(Zs/examples/resnet/TrainImageNet.scala, `nn.mkldnn.ResNet.graph`) and serves
it through ImageClassifier configs (Zs/models/image/imageclassification/
ImageClassificationConfig.scala:56-190). Here every conv is fused with its
BatchNorm (+ residual + ReLU) into the conv_bn_act op (implicit-GEMM conv with
BN statistics in the epilogue, then one apply pass), activations stay NHWC
bf16 end-to-end, and weights are stored in the packed [K, ceil8(R*S*C)]
layout the MFMA kernels read directly.
"""
import math

import os

import torch
import torch.nn as nn

from zoo import ops
from zoo.ops.bn import BNProducer, GradHandoff, bn_relu_maxpool, conv_stats, stem_pool_fusable


class ConvBN(nn.Module):
    """conv(KxK) -> BatchNorm -> (+residual) -> (ReLU), NHWC."""

    def __init__(self, cin, cout, k, stride=1, pad=0, relu=True, zero_gamma=False, eps=1e-5, momentum=0.1):
        super().__init__()
        self.cin, self.cout, self.k, self.stride, self.pad, self.relu = cin, cout, k, stride, pad, relu
        self.eps, self.momentum = eps, momentum
        w4 = torch.empty(cout, k, k, cin)
        fan_out = cout * k * k
        nn.init.normal_(w4, 0.0, math.sqrt(2.0 / fan_out))
        self.weight = nn.Parameter(ops.pack_weight(w4))
        self.gamma = nn.Parameter(torch.zeros(cout) if zero_gamma else torch.ones(cout))
        self.beta = nn.Parameter(torch.zeros(cout))
        self.register_buffer("running_mean", torch.zeros(cout))
        self.register_buffer("running_var", torch.ones(cout))

    def forward(self, x, resid=None, resid_handoff=None, grad_add=None, producer_in=None, producer_out=None,
                dx_handoff=None, resid_bn=None):
        return ops.conv_bn_act(x, self.weight, self.gamma, self.beta, self.running_mean, self.running_var,
                               kernel=(self.k, self.k), stride=(self.stride, self.stride),
                               pad=(self.pad, self.pad), eps=self.eps, momentum=self.momentum, relu=self.relu,
                               resid=resid, training=self.training, resid_handoff=resid_handoff, grad_add=grad_add,
                               producer_in=producer_in, producer_out=producer_out, dx_handoff=dx_handoff,
                               resid_bn=resid_bn)

    def forward_stats(self, x, grad_add=None, dx_handoff=None):
        """Training-mode projection shortcut: raw conv output + its BN (ShortcutBN), to be
        applied inside the consuming unit's BN pass. Returns (raw, resid_bn argument)."""
        y, holder = conv_stats(x, self.weight, self.running_mean, self.running_var, kernel=(self.k, self.k),
                               stride=(self.stride, self.stride), pad=(self.pad, self.pad), grad_add=grad_add,
                               dx_handoff=dx_handoff)
        return y, (holder, self.gamma, self.beta)


# cross-unit BN-backward fusion (BNProducer); the switch exists for A/B numerics tests
FUSE_BN_BACKWARD = True
# projection-shortcut BatchNorm applied inside the block's last BN pass (ShortcutBN)
FUSE_SHORTCUT_BN = True
# ResNet stem BatchNorm + ReLU fused into the max-pool pass (bn_relu_maxpool)
FUSE_STEM_POOL = True
# 7x7/2 stem computed as a 4x4/1 conv on a space-to-depth(2) input (GPU)
S2D_STEM = True
# projection blocks: the shortcut's dgrad runs first and hands its dx to conv1's dgrad, which then
# also fuses the previous block's BN-backward reduction (stage transitions)
SHORTCUT_FIRST = True
# bottlenecks: conv2's BN + ReLU applied by conv3 (1x1) in its operand prologue, conv2's apply pass
# skipped (BNProducer.fwd_pro, pw.hip forward prologue). Off: -0.3 % with the 64- and 128-wide
# units, +-0 with the 64-wide ones alone (profiles/r5/ab_fwd_consumer_apply_r5.md); on the
# round-6 kernels -0.3 % again (profiles/r6/ab18_downfp*_r6.log)
FWD_PRO = False
# block outputs: the block's last BN + residual + ReLU applied by the NEXT block's 1x1 conv1 in its
# operand prologue (which writes the block output and its ReLU mask); the block's apply pass over
# the full-width tensor is skipped (zoo.ops.bn _FWD_PRO_RES_K: the 256-wide stage-1 outputs)
FWD_PRO_RES = True
# ... also at the stage-1 -> stage-2 transition (the next block has a projection shortcut, stride
# on conv2). Off: that conv1 writes 128 channels, i.e. two 64-channel workgroup groups, so the
# prologue's y + residual reads and BN math run twice; it measured -0.2 % against the 267 us
# apply pass it removes (13,149 vs 13,173 img/s over 3 same-box pairs, profiles/r6/ab18_*_r6.log)
FWD_PRO_RES_DOWN = False


def _bp():
    return BNProducer(False, None, None, None) if FUSE_BN_BACKWARD else None


def _fusing(x):
    """Cross-unit backward fusion applies to GPU training with autograd on."""
    return x.is_cuda and torch.is_grad_enabled()


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, zero_init_residual=False):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = ConvBN(cin, width, 1)
        self.conv2 = ConvBN(width, width, 3, stride=stride, pad=1)
        self.conv3 = ConvBN(width, cout, 1, relu=True, zero_gamma=zero_init_residual)
        self.down = ConvBN(cin, cout, 1, stride=stride, relu=False) if (stride != 1 or cin != cout) else None

    def consumes_block_output_1x1(self):
        """The block's input is formed by its own 1x1 stride-1 conv1: with an identity shortcut conv1
        is its only reader; with a projection shortcut (SHORTCUT_FIRST order) conv1 runs first, its
        prologue writes the input, and the shortcut conv reads it after. Either way the previous
        block's output apply can move into conv1's prologue."""
        if not (self.conv1.k == 1 and self.conv1.stride == 1):
            return False
        return self.down is None or (FWD_PRO_RES_DOWN and SHORTCUT_FIRST)

    def forward(self, x, prod=None, out_pro=False):
        """``prod``: BNProducer of ``x`` (the previous block's last unit). ``out_pro``: the next
        block's conv1 applies this block's output BN + residual + ReLU. Returns
        (out, BNProducer of out) when fusing, else out."""
        if not (self.training and _fusing(x)):
            sc = self.down(x) if self.down is not None else x
            return self.conv3(self.conv2(self.conv1(x)), resid=sc)
        p1, p2, p3 = _bp(), _bp(), _bp()
        if p2 is not None and FWD_PRO and self.conv3.k == 1 and self.conv3.stride == 1:
            p2.fwd_pro = True
        if p3 is not None and out_pro:
            p3.fwd_pro = True
        if self.down is None:
            # identity shortcut: conv3's residual gradient is added in conv1's dgrad epilogue, which makes
            # conv1 the sole consumer of x -> it also fuses the previous block's BN-backward reduction
            ho = GradHandoff()
            h = self.conv1(x, grad_add=ho, producer_in=prod, producer_out=p1)
            h = self.conv2(h, producer_in=p1, producer_out=p2)
            return self.conv3(h, resid=x, resid_handoff=ho, producer_in=p2, producer_out=p3), p3
        dh = GradHandoff()
        fuse_sc = FUSE_SHORTCUT_BN and self.down.eps == self.conv3.eps and self.down.momentum == self.conv3.momentum
        if SHORTCUT_FIRST and self.conv1.stride == 1 and self.conv1.k == 1:
            # x feeds both `down` and conv1. `down` is created after conv1, so its backward runs first
            # and hands its (possibly strided, zero-filled) dx to conv1, whose stride-1 dgrad covers
            # every position: its epilogue adds it AND fuses the previous block's BN-backward
            # reduction (producer_in) -- no separate reduction pass over x at stage transitions
            h = self.conv1(x, grad_add=dh, producer_in=prod, producer_out=p1)
            if fuse_sc:
                sc, rbn = self.down.forward_stats(x, dx_handoff=dh)
            else:
                sc, rbn = self.down(x, dx_handoff=dh), None
        else:
            # conv1 (created later, so its backward runs first) hands its dx to down's dgrad
            # epilogue, which adds it -- no separate gradient-add pass over x
            if fuse_sc:
                # the shortcut's BatchNorm is applied inside conv3's BN pass (no shortcut apply pass)
                sc, rbn = self.down.forward_stats(x, grad_add=dh)
            else:
                sc, rbn = self.down(x, grad_add=dh), None
            h = self.conv1(x, producer_out=p1, dx_handoff=dh)
        h = self.conv2(h, producer_in=p1, producer_out=p2)
        return self.conv3(h, resid=sc, producer_in=p2, producer_out=p3, resid_bn=rbn), p3


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, width, stride=1, zero_init_residual=False):
        super().__init__()
        self.conv1 = ConvBN(cin, width, 3, stride=stride, pad=1)
        self.conv2 = ConvBN(width, width, 3, pad=1, relu=True, zero_gamma=zero_init_residual)
        self.down = ConvBN(cin, width, 1, stride=stride, relu=False) if (stride != 1 or cin != width) else None

    def forward(self, x, prod=None):
        if not (self.training and _fusing(x)):
            sc = self.down(x) if self.down is not None else x
            return self.conv2(self.conv1(x), resid=sc)
        p1, p2 = _bp(), _bp()
        if self.down is None:
            ho = GradHandoff()
            h = self.conv1(x, grad_add=ho, producer_in=prod, producer_out=p1)
            return self.conv2(h, resid=x, resid_handoff=ho, producer_in=p1, producer_out=p2), p2
        dh = GradHandoff()
        if FUSE_SHORTCUT_BN and self.down.eps == self.conv2.eps and self.down.momentum == self.conv2.momentum:
            sc, rbn = self.down.forward_stats(x, grad_add=dh)
        else:
            sc, rbn = self.down(x, grad_add=dh), None
        h = self.conv1(x, producer_out=p1, dx_handoff=dh)
        return self.conv2(h, resid=sc, producer_in=p1, producer_out=p2, resid_bn=rbn), p2


class Dense(nn.Module):
    """Final classifier on the MFMA GEMM (fp32 logits). The class dimension is
    padded to a multiple of 8 (16-byte rows for the kernel); padded rows stay
    exactly zero (their logits are sliced off, so their gradient is zero)."""

    def __init__(self, cin, cout):
        super().__init__()
        self.cout = cout
        cpad = ops.ceil8(cout)
        w = torch.zeros(cpad, cin)
        nn.init.normal_(w[:cout], 0.0, 0.01)
        self.weight = nn.Parameter(w)
        self.bias = nn.Parameter(torch.zeros(cpad))

    def forward(self, x):
        if x.is_cuda:
            y = ops.conv2d_nhwc(x.reshape(x.shape[0], 1, 1, x.shape[1]), self.weight, self.bias, out_f32=True)
            y = y.reshape(x.shape[0], -1)
        else:
            y = torch.nn.functional.linear(x.float(), self.weight, self.bias)
        return y if self.cout == y.shape[1] else y[:, : self.cout].contiguous()


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, width=64, in_channels=3, zero_init_residual=False):
        """``zero_init_residual``: the last BN gamma of every residual block starts at 0 (each block
        is the identity at init; the standard large-batch ImageNet recipe)."""
        super().__init__()
        self.in_channels = in_channels
        self.cin_pad = 4 if in_channels <= 4 else ops.ceil8(in_channels)
        self.stem = ConvBN(self.cin_pad, width, 7, stride=2, pad=3)
        cin = width
        stages = []
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            blocks = []
            for j in range(n):
                blocks.append(block(cin, w, stride=(2 if (j == 0 and i > 0) else 1),
                                    zero_init_residual=zero_init_residual))
                cin = w * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.Sequential(*stages)
        self.fc = Dense(cin, num_classes)
        self.num_classes = num_classes
        # uint8 NHWC image batches (the input pipeline's wire format) are normalised on the device,
        # fused into the stem's space-to-depth pass: x / 255 - mean) / std per channel (ImageNet)
        self.input_mean, self.input_std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)

    def to_nhwc(self, x):
        """NCHW fp32 images -> NHWC bf16 with channels zero-padded for 16-byte loads."""
        if x.dim() == 4 and x.shape[1] == self.in_channels:
            if x.is_cuda:
                return ops.native().nchw_to_nhwc(x.float().contiguous(), self.cin_pad)
            x = x.permute(0, 2, 3, 1)
        pad = self.cin_pad - x.shape[-1]
        if pad:
            x = torch.nn.functional.pad(x, (0, pad))
        return x.contiguous()

    def _stem_s2d_ok(self, x):
        return x.is_cuda and type(self.stem) is ConvBN and x.dim() == 4 and x.shape[1] == self.in_channels and \
            self.cin_pad == 4 and \
            self.stem.k == 7 and self.stem.stride == 2 and self.stem.pad == 3 and S2D_STEM

    def _s2d_weight(self):
        """7x7x4 stem weight -> the equivalent 4x4x16 space-to-depth weight (differentiable:
        the gradient flows back to the 7x7 parameter). Tap (r, s) = (2R+dy, 2S+dx); r = s = 7
        are the zero pad row/column."""
        K = self.stem.cout
        w7 = self.stem.weight[:, :7 * 7 * 4].reshape(K, 7, 7, 4)
        w8 = torch.nn.functional.pad(w7, (0, 0, 0, 1, 0, 1))                 # [K, 8, 8, 4]
        return w8.reshape(K, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(K, 256).contiguous()

    def _stem_bn(self, y, holder):
        """Unfused fallback of the stem-pool fusion: BN+ReLU of the raw stem output (its
        statistics were already taken by the conv and are recomputed by batch_norm_nhwc)."""
        st = self.stem
        holder.stats = None
        return ops.batch_norm_nhwc(y, st.gamma, st.beta, st.running_mean, st.running_var, st.eps, st.momentum,
                                   relu=True, training=True)

    def _u8_scale_shift(self, c):
        mean = list(self.input_mean) + [0.0] * (c - len(self.input_mean))
        std = list(self.input_std) + [1.0] * (c - len(self.input_std))
        return [1.0 / (255.0 * s) for s in std[:c]], [-m / s for m, s in zip(mean[:c], std[:c])]

    def _from_u8(self, x):
        """uint8 NHWC [N, H, W, C] -> normalised fp32 NCHW (reference / non-fused path)."""
        sc, sh = self._u8_scale_shift(x.shape[-1])
        y = x.float() * torch.tensor(sc, device=x.device) + torch.tensor(sh, device=x.device)
        return y.permute(0, 3, 1, 2).contiguous()

    def forward(self, x):
        if x.dtype == torch.uint8 and x.dim() == 4 and x.shape[-1] == self.in_channels:
            if self._stem_s2d_ok(x.permute(0, 3, 1, 2)):
                # normalisation fused into the space-to-depth pass (no fp32 NCHW copy on the device)
                sc, sh = self._u8_scale_shift(self.in_channels)
                xs = ops.native().nhwc_u8_to_s2d(x.contiguous(), 3, sc, sh)
                return self._forward_s2d(xs)
            x = self._from_u8(x)
        if self._stem_s2d_ok(x):
            # stem as a 4x4 stride-1 conv on the space-to-depth(2) image: 16 input channels
            # take the vector implicit-GEMM path; the NCHW->NHWC pass becomes the s2d pass
            return self._forward_s2d(ops.native().nchw_to_s2d(x.float().contiguous(), 3))
        x = self.to_nhwc(x)
        x = self.stem(x)
        x = ops.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))
        return self._forward_stages(x)

    def _forward_s2d(self, xs):
        st = self.stem
        if st.training and FUSE_STEM_POOL and torch.is_grad_enabled():
            # stem BN + ReLU applied inside the max-pool pass (bn_relu_maxpool): the conv
            # emits statistics only and the 112x112 BN output is never written
            y, holder = conv_stats(xs, self._s2d_weight(), st.running_mean, st.running_var, kernel=(4, 4))
            if stem_pool_fusable(y, (3, 3), (1, 1)):
                x = bn_relu_maxpool(y, holder, st.gamma, st.beta, st.eps, st.momentum)
            else:
                x = ops.max_pool2d_nhwc(self._stem_bn(y, holder), (3, 3), (2, 2), (1, 1))
        else:
            x = ops.conv_bn_act(xs, self._s2d_weight(), st.gamma, st.beta, st.running_mean, st.running_var,
                                kernel=(4, 4), stride=(1, 1), pad=(0, 0), eps=st.eps, momentum=st.momentum,
                                relu=True, training=st.training)
            x = ops.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))
        return self._forward_stages(x)

    def _forward_stages(self, x):
        if self.training and _fusing(x):
            prod = None
            blocks = [blk for stage in self.stages for blk in stage]
            for i, blk in enumerate(blocks):
                nxt = blocks[i + 1] if i + 1 < len(blocks) else None
                if FWD_PRO_RES and isinstance(blk, Bottleneck) and isinstance(nxt, Bottleneck) and \
                        nxt.consumes_block_output_1x1():
                    x, prod = blk(x, prod, out_pro=True)
                else:
                    x, prod = blk(x, prod)
        else:
            x = self.stages(x)
        x = ops.global_avg_pool_nhwc(x)
        return self.fc(x)


def resnet50(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet18(num_classes=1000, **kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet34(num_classes=1000, **kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet101(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes=num_classes, **kw)
