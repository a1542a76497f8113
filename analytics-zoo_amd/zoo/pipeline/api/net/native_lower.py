"""Lowering of imported / wrapped PyTorch-style models onto the native MI355X kernels.

The Net loaders (BigDL ``.model`` graphs, Caffe prototxt/caffemodel, Torch7 ``.t7``), the ONNX
importer and ``TorchNet.from_pytorch`` produce ordinary ``torch.nn`` modules in the source
layout (NCHW). Executed as-is on the GPU they run on the vendor libraries (MIOpen convolutions /
pooling / batch norm, hipBLASLt GEMMs). This pass swaps the CLASS of every supported module, in place, for a
native twin (a subclass of the torch class): parameters, buffers, ``state_dict`` keys and
``isinstance`` stay those of the original model (savers, optimizers and checkpoints see the same
tensors), only ``forward`` computes on the zoo kernels:

* ``nn.Conv2d`` (+ a following eval-mode ``BatchNorm2d`` folded in, + ReLU / tanh / sigmoid
  fused into the epilogue) -> ``ops.conv2d_nhwc`` (igemm / igemm2 / pw implicit-GEMM MFMA);
* ``nn.Linear`` -> ``ops.linear`` (MFMA GEMM, bias + activation epilogue);
* max / average / global pooling -> the NHWC pooling kernels;
* ``BatchNorm2d`` alone -> the native NHWC batch norm (training and inference);
* ReLU / Tanh / Sigmoid / ELU / ... -> the native activation kernel; LRN -> the native LRN;
* ``nn.LSTM`` / ``nn.GRU`` (single direction or bidirectional, any layer count) and
  ``nn.GRUCell`` -> the persistent recurrent kernel (``ops.rnn.recurrent``; torch's reset-after
  GRU is its CELL_GRU_RA cell);
* grouped / depthwise ``nn.Conv2d`` (Caffe ``group``, MobileNet) -> per-group implicit GEMMs /
  the depthwise kernel; ``nn.ConvTranspose2d`` (Caffe ``Deconvolution``) -> the conv
  data-gradient kernels.

Layout: a native module takes NCHW and returns NCHW whose memory is channels-last (a
``permute`` view of the NHWC kernel output), so the next native module's NCHW -> NHWC permute is
free and a chain of lowered layers runs NHWC end to end; only the graph input and the
consumers that need a dense NCHW tensor (e.g. ``Flatten``) pay a copy. Channel counts that are
not 8-aligned are zero-padded inside each module (weights and activations).

Reference: the MKL-DNN execution of loaded models in the reference -- ``Net.loadBigDL`` /
``Net.loadCaffe`` (zoo/src/main/scala/com/intel/analytics/zoo/pipeline/api/Net.scala:157,184),
the ONNX importer mapping nodes onto Zoo Keras layers
(pyzoo/zoo/pipeline/api/onnx/mapper/conv.py:18,68) and Cluster Serving's model loading
(zoo/src/main/scala/com/intel/analytics/zoo/serving/utils/ClusterServingHelper.scala:274-295);
mirrors ``zoo/pipeline/inference/openvino.py``'s native IR executor.
"""
import copy
import weakref

import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.ops import _kern
from zoo.ops import pointwise as P
from zoo.ops import pool as PO
from zoo.pipeline.api.net import graph_net as G

_ACTS = {nn.ReLU: "relu", nn.Tanh: "tanh", nn.Sigmoid: "sigmoid", nn.ELU: "elu", nn.SELU: "selu",
         nn.Softplus: "softplus", nn.Softsign: "softsign", nn.ReLU6: "relu6", nn.SiLU: "swish",
         nn.LogSigmoid: "log_sigmoid", nn.Tanhshrink: "tanh_shrink", nn.GELU: "gelu"}
_FUSABLE = ("relu", "tanh", "sigmoid")      # conv epilogue activations


def _cin_pad(c):
    return c if c % 8 == 0 else (4 if c <= 4 else ops.ceil8(c))


def to_nhwc(x, cpad=None):
    """NCHW (any memory format) -> contiguous NHWC bf16 with channels zero-padded to ``cpad``
    (free when ``x`` is the channels-last view a native module returned)."""
    y = x.permute(0, 2, 3, 1)
    if cpad is not None and cpad != y.shape[-1]:
        y = F.pad(y, (0, cpad - y.shape[-1]))
    if y.dtype != torch.bfloat16:
        y = y.to(torch.bfloat16)
    return y.contiguous()


def from_nhwc(y, c, dtype):
    """NHWC (maybe channel-padded) -> NCHW view with channels-last memory, in ``dtype``."""
    if y.shape[-1] != c:
        y = y[..., :c]
    if y.dtype != dtype:
        y = y.to(dtype)
    return y.permute(0, 3, 1, 2)


def _act_name(m):
    for cls, name in _ACTS.items():
        if type(m) is cls:
            return name
    if isinstance(m, nn.LeakyReLU):
        return "leaky_relu"
    fn = getattr(m, "fname", None)             # graph_net.Fn wrappers of the BigDL / Caffe loaders
    if isinstance(fn, str):
        return {"ReLU": "relu", "Tanh": "tanh", "Sigmoid": "sigmoid", "ELU": "elu", "SoftPlus": "softplus",
                "SoftSign": "softsign", "ReLU6": "relu6"}.get(fn)
    return None


def _native_ok(x):
    return torch.is_tensor(x) and x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16,
                                                                            torch.float16)


# ---------------------------------------------------------------------------------------------
# native twins: subclasses of the torch modules. Lowering swaps a module's CLASS in place, so
# the module keeps its parameters, buffers, state_dict keys and isinstance() identity (weight
# savers, optimizers, checkpoints and user code see an unchanged model); only forward changes.
# A module absorbed into a fused neighbour (eval BatchNorm / activation after a conv) gets
# ``_zoo_absorbed`` and passes its input through.
# ---------------------------------------------------------------------------------------------
class _Twin:
    _zoo_absorbed = False


class ZConv2d(_Twin, nn.Conv2d):
    """nn.Conv2d (zero padding) [+ folded eval BatchNorm2d] [+ fused activation] on the native
    kernels: dense convs on the implicit-GEMM kernels (igemm / igemm2 / pw); depthwise convs
    (groups = in_channels, any channel multiplier, <= 3x3 taps) on the depthwise kernel
    (dwconv.hip); other grouped convs (Caffe ``group``, e.g. AlexNet's group 2; ResNeXt) as ONE
    grouped implicit-GEMM launch per direction with the group index in the grid (gconv.hip)."""
    _zoo_bn = None
    _zoo_act = None
    _zoo_cache = None

    def _group_mode(self):
        g, C, K = self.groups, self.in_channels, self.out_channels
        if g == 1:
            return "dense"
        R, S = self.kernel_size
        if g == C and K % C == 0 and R * S <= 9 and tuple(self.dilation) == (1, 1):
            return "depthwise"
        if C % g == 0 and K % g == 0:
            return "grouped"
        return None

    def _native_supported(self, x):
        return (_native_ok(x) and self.padding_mode == "zeros" and isinstance(self.padding, tuple) and
                len(self.kernel_size) == 2 and self._group_mode() is not None)

    def _folded_wb(self, training_bn):
        """(fp32 weight [K, C/groups, R, S], bias [K]) with an eval BatchNorm folded in."""
        bn = self._zoo_bn
        w = self.weight.float()
        K = w.shape[0]
        b = self.bias.float() if self.bias is not None else torch.zeros(K, device=w.device)
        if bn is not None and not training_bn:
            s = torch.rsqrt(bn.running_var.float() + bn.eps)
            if bn.weight is not None:
                s = s * bn.weight.float()
            b = (b - bn.running_mean.float()) * s + (bn.bias.float() if bn.bias is not None else 0.0)
            w = w * s[:, None, None, None]
        return w, b

    @staticmethod
    def _pack(w, b):
        """[K, C, R, S] fp32 -> (packed [Kp, ceil8(R*S*Cp)], bias [Kp]) in the implicit-GEMM layout."""
        K, C, R, S = w.shape
        cp, kp = _cin_pad(C), ops.ceil8(K)
        w2 = F.pad(w.permute(0, 2, 3, 1), (0, cp - C, 0, 0, 0, 0, 0, kp - K)).reshape(kp, R * S * cp)
        ld = ops.ceil8(R * S * cp)
        if ld != R * S * cp:
            w2 = F.pad(w2, (0, ld - R * S * cp))
        return w2, F.pad(b, (0, kp - K))

    def _packed(self, training_bn):
        """Native operands for this conv's group mode, cached by parameter versions when no
        gradient is needed: dense -> (packed weight, bias); grouped -> (weight [K, ceil8(R*S*C/g)], bias);
        depthwise -> (tap-major weight [R*S, Kp], bias [Kp])."""
        bn = self._zoo_bn
        need_grad = torch.is_grad_enabled() and (self.weight.requires_grad or
                                                 (self.bias is not None and self.bias.requires_grad))
        key = None
        if not need_grad:
            # the engine's fused optimizer (weights) and the native BN forward (running statistics)
            # write through raw pointers without bumping ``_version``: their epochs are in the key
            key = (self.weight._version, self.weight.data_ptr(), None if self.bias is None else self.bias._version,
                   training_bn, None if bn is None else (bn.running_mean._version, bn.running_var._version,
                                                         None if bn.weight is None else bn.weight._version,
                                                         None if bn.bias is None else bn.bias._version,
                                                         bn.running_mean.data_ptr()),
                   _kern.weights_epoch(), _kern.stats_epoch())
            if self._zoo_cache is not None and self._zoo_cache[0] == key:
                return self._zoo_cache[1]
        w, b = self._folded_wb(training_bn)
        mode = self._group_mode()
        K, Cg, R, S = w.shape
        if mode == "dense":
            out = self._pack(w, b)
        elif mode == "grouped":
            # [K, ceil8(R*S*Cg)]: each output channel's filter over its own group's channels
            w2 = w.permute(0, 2, 3, 1).reshape(K, R * S * Cg)
            ld = ops.ceil8(R * S * Cg)
            out = (F.pad(w2, (0, ld - R * S * Cg)) if ld != R * S * Cg else w2, b)
        else:   # depthwise: output channel o reads input channel o // multiplier
            kp = ops.ceil8(K)
            out = (F.pad(w.reshape(K, R * S).t(), (0, kp - K)), F.pad(b, (0, kp - K)))
        if key is not None:
            out = (out[0].detach().contiguous(), out[1].detach().contiguous())
            self._zoo_cache = (key, out)
        return out

    def forward(self, x):
        bn, act = self._zoo_bn, self._zoo_act
        if not self._native_supported(x):
            y = nn.Conv2d.forward(self, x)
            if bn is not None:
                y = F.batch_norm(y, bn.running_mean, bn.running_var, bn.weight, bn.bias, bn.training,
                                 bn.momentum if bn.momentum is not None else 0.1, bn.eps)
            return P.act_ref(y, act) if act else y
        training_bn = bn is not None and bn.training
        K, C = self.out_channels, self.in_channels
        mode = self._group_mode()
        fused = act if (act in _FUSABLE and not training_bn) else None
        geo = dict(kernel=tuple(self.kernel_size), stride=tuple(self.stride), pad=tuple(self.padding))
        if mode == "dense":
            w2, b = self._packed(training_bn)
            y = ops.conv2d_nhwc(to_nhwc(x, _cin_pad(C)), w2, b, dil=tuple(self.dilation), act=fused, **geo)
        elif mode == "grouped":
            # one launch per direction, group index in the grid (csrc/kernels/gconv.hip)
            from zoo.ops.conv import grouped_conv2d_nhwc
            w2, b = self._packed(training_bn)
            y = grouped_conv2d_nhwc(to_nhwc(x), w2, b, groups=self.groups, dil=tuple(self.dilation), act=fused,
                                    **geo)
        else:
            from zoo.ops.nn import depthwise_conv2d_nhwc
            wdw, b = self._packed(training_bn)
            xn = to_nhwc(x)
            if K != C:
                xn = xn.repeat_interleave(K // C, dim=3)
            if ops.ceil8(K) != K:
                xn = F.pad(xn, (0, ops.ceil8(K) - K))
            dfuse = fused if fused == "relu" else None
            y = depthwise_conv2d_nhwc(xn, wdw, b, act=dfuse, **geo)
            if fused is not None and dfuse is None:
                y = P.activation(y, fused)
        if training_bn:
            y = _bn_nhwc(y, bn, K)
        if act and fused is None:
            y = P.activation(y, act)
        return from_nhwc(y, K, x.dtype)


class ZConvTranspose2d(_Twin, nn.ConvTranspose2d):
    """nn.ConvTranspose2d (Caffe ``Deconvolution``, groups 1, no dilation) on the conv data-gradient
    kernels: the transposed conv IS the dgrad of the conv whose weight it holds
    (ops.conv.conv_transpose2d_nhwc); backward is a forward conv plus a weight gradient."""

    def _native_supported(self, x):
        return (_native_ok(x) and self.groups == 1 and tuple(self.dilation) == (1, 1) and
                self.padding_mode == "zeros" and len(self.kernel_size) == 2)

    def forward(self, x, output_size=None):
        if not self._native_supported(x):
            return nn.ConvTranspose2d.forward(self, x, output_size)
        from zoo.ops.conv import conv_transpose2d_nhwc
        R, S = self.kernel_size
        sh, sw = self.stride
        ph, pw = self.padding
        opad = self._output_padding(x, output_size, list(self.stride), list(self.padding), list(self.kernel_size),
                                    2, list(self.dilation))
        H, W = x.shape[-2:]
        oh = (H - 1) * sh - 2 * ph + R + opad[0]
        ow = (W - 1) * sw - 2 * pw + S + opad[1]
        Cin, Cout = self.in_channels, self.out_channels
        cp, kp = ops.ceil8(Cin), ops.ceil8(Cout)
        wd = F.pad(self.weight.float(), (0, 0, 0, 0, 0, kp - Cout, 0, cp - Cin))     # [cp, kp, R, S]
        wf = wd.permute(0, 2, 3, 1).reshape(cp, R * S * kp)
        if ops.ceil8(R * S * kp) != R * S * kp:
            wf = F.pad(wf, (0, ops.ceil8(R * S * kp) - R * S * kp))
        y = conv_transpose2d_nhwc(to_nhwc(x, cp), wf, (R, S), (sh, sw), (ph, pw), (oh, ow), kp)[..., :Cout]
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return from_nhwc(y, Cout, x.dtype)


def _bn_nhwc(y, bn, C):
    """BatchNorm over an NHWC tensor with C real channels (y may carry zero padding). Channel
    counts that are not 8-aligned run padded: the affine and the running statistics are padded
    with identity values and the updated statistics are copied back."""
    mom = bn.momentum if bn.momentum is not None else 0.1
    dev = y.device
    g = bn.weight if bn.weight is not None else torch.ones(C, device=dev)
    b = bn.bias if bn.bias is not None else torch.zeros(C, device=dev)
    training = bn.training or not bn.track_running_stats
    rm = bn.running_mean if bn.running_mean is not None else torch.zeros(C, device=dev)
    rv = bn.running_var if bn.running_var is not None else torch.ones(C, device=dev)
    Cp = ops.ceil8(C)
    if Cp == C:
        if y.shape[-1] != C:
            y = y[..., :C].contiguous()
        return ops.batch_norm_nhwc(y, g, b, rm, rv, bn.eps, mom, training=training)
    if y.shape[-1] != Cp:
        y = F.pad(y[..., :C], (0, Cp - C)) if y.shape[-1] > C else F.pad(y, (0, Cp - C))
    pad = lambda t, v: torch.cat([t.float(), torch.full((Cp - C,), v, device=dev)])  # noqa: E731
    rmp, rvp = pad(rm.detach(), 0.0), pad(rv.detach(), 1.0)
    out = ops.batch_norm_nhwc(y.contiguous(), pad(g, 1.0), pad(b, 0.0), rmp, rvp, bn.eps, mom, training=training)
    if training and bn.track_running_stats:
        with torch.no_grad():
            bn.running_mean.copy_(rmp[:C])
            bn.running_var.copy_(rvp[:C])
    return out[..., :C]


class ZBatchNorm2d(_Twin, nn.BatchNorm2d):
    def forward(self, x):
        if self._zoo_absorbed:
            return x
        if not _native_ok(x):
            return nn.BatchNorm2d.forward(self, x)
        C = x.shape[1]
        return from_nhwc(_bn_nhwc(to_nhwc(x), self, C), C, x.dtype)


class ZLinear(_Twin, nn.Linear):
    _zoo_act = None

    def forward(self, x):
        act = self._zoo_act
        if not (torch.is_tensor(x) and x.is_cuda):
            y = nn.Linear.forward(self, x)
            return P.act_ref(y, act) if act else y
        fuse = act in (None, "relu", "gelu")
        y = ops.linear(x if x.is_contiguous() else x.contiguous(), self.weight, self.bias, act=act if fuse else None)
        return y if fuse else P.activation(y, act)


def _pool_native(x, kind, k, s, p, ceil_mode=False, count_include_pad=True, global_pool=False):
    """NCHW pooling on the NHWC kernels (channels padded to 8); None when unsupported."""
    if not _native_ok(x):
        return None
    C = x.shape[1]
    if global_pool:
        k = s = tuple(x.shape[-2:])
        p = (0, 0)
    if kind == "max" and (2 * p[0] > k[0] or 2 * p[1] > k[1]):
        return None
    xn = to_nhwc(x, ops.ceil8(C))
    if kind == "max":
        y = ops.max_pool2d_nhwc(xn, k, s, p, ceil_mode=ceil_mode)
    elif global_pool:
        y = ops.global_avg_pool_nhwc(xn).reshape(xn.shape[0], 1, 1, -1)
    else:
        if 2 * p[0] > k[0] or 2 * p[1] > k[1]:
            return None
        y = PO.avg_pool2d_nhwc(xn, k, s, p, ceil_mode=ceil_mode, count_include_pad=count_include_pad)
    return from_nhwc(y, C, x.dtype)


class ZMaxPool2d(_Twin, nn.MaxPool2d):
    def forward(self, x):
        y = None
        if not self.return_indices and self.dilation in (1, (1, 1)):
            y = _pool_native(x, "max", _pair(self.kernel_size), _pair(self.stride or self.kernel_size),
                             _pair(self.padding), self.ceil_mode)
        return nn.MaxPool2d.forward(self, x) if y is None else y


class ZAvgPool2d(_Twin, nn.AvgPool2d):
    def forward(self, x):
        y = None
        if self.divisor_override is None:
            y = _pool_native(x, "avg", _pair(self.kernel_size), _pair(self.stride or self.kernel_size),
                             _pair(self.padding), self.ceil_mode, self.count_include_pad)
        return nn.AvgPool2d.forward(self, x) if y is None else y


class ZAdaptiveAvgPool2d(_Twin, nn.AdaptiveAvgPool2d):
    def forward(self, x):
        y = _pool_native(x, "avg", None, None, None, global_pool=True) if _pair(self.output_size) == (1, 1) else None
        return nn.AdaptiveAvgPool2d.forward(self, x) if y is None else y


class ZPool2d(_Twin, G.Pool2d):
    """graph_net.Pool2d (BigDL SpatialMax/AveragePooling, Caffe Pooling)."""

    def forward(self, x):
        y = _pool_native(x, self.kind, _pair(self.kernel) if self.kernel is not None else None,
                         _pair(self.stride) if self.stride is not None else None, _pair(self.pad), self.ceil_mode,
                         self.count_include_pad, self.global_pool)
        return G.Pool2d.forward(self, x) if y is None else y


def _lrn_native(x, size, alpha, beta, k):
    if not _native_ok(x):
        return None
    C = x.shape[1]
    return from_nhwc(ops.lrn_channels_last(to_nhwc(x), size, alpha, beta, k), C, x.dtype)


class ZLocalResponseNorm(_Twin, nn.LocalResponseNorm):
    def forward(self, x):
        y = _lrn_native(x, self.size, self.alpha, self.beta, self.k)
        return nn.LocalResponseNorm.forward(self, x) if y is None else y


class ZLRN(_Twin, G.LRN):
    def forward(self, x):
        y = _lrn_native(x, self.size, self.alpha, self.beta, self.k)
        return G.LRN.forward(self, x) if y is None else y


def _act_native(x, name, alpha=None):
    if not (torch.is_tensor(x) and x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)):
        return None
    if x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last):
        # a channels-last view (a native producer's output): run on its NHWC memory, stay channels-last
        return P.activation(x.permute(0, 2, 3, 1), name, alpha).permute(0, 3, 1, 2)
    return P.activation(x, name, alpha)


def _act_forward(base, name_of):
    def forward(self, x):
        if self._zoo_absorbed:
            return x
        y = _act_native(x, *name_of(self))
        return base.forward(self, x) if y is None else y
    return forward


class ZReLU(_Twin, nn.ReLU):
    forward = _act_forward(nn.ReLU, lambda m: ("relu",))


class ZTanh(_Twin, nn.Tanh):
    forward = _act_forward(nn.Tanh, lambda m: ("tanh",))


class ZSigmoid(_Twin, nn.Sigmoid):
    forward = _act_forward(nn.Sigmoid, lambda m: ("sigmoid",))


class ZELU(_Twin, nn.ELU):
    forward = _act_forward(nn.ELU, lambda m: ("elu", m.alpha))


class ZLeakyReLU(_Twin, nn.LeakyReLU):
    forward = _act_forward(nn.LeakyReLU, lambda m: ("leaky_relu", m.negative_slope))


class ZReLU6(_Twin, nn.ReLU6):
    forward = _act_forward(nn.ReLU6, lambda m: ("relu6",))


class ZGELU(_Twin, nn.GELU):
    forward = _act_forward(nn.GELU, lambda m: ("gelu" if m.approximate == "none" else "gelu_tanh",))


class ZSoftplus(_Twin, nn.Softplus):
    def forward(self, x):
        y = _act_native(x, "softplus") if self.beta == 1 and self.threshold == 20 else None
        return nn.Softplus.forward(self, x) if y is None else y


class ZFn(_Twin, G.Fn):
    """graph_net.Fn activation wrappers (BigDL Tanh / ReLU / Sigmoid ... nodes)."""
    forward = _act_forward(G.Fn, lambda m: (_act_name(m),))


class ZLSTM(_Twin, nn.LSTM):
    """nn.LSTM on the persistent recurrent kernel (rnn.hip): every layer / direction is one input
    GEMM + one kernel launch for the whole sequence. nn.LSTM's call signature and outputs
    (``(output, (h_n, c_n))``); sigmoid gates, tanh cell."""

    def _native_supported(self, x):
        from zoo.ops import rnn as R
        return (torch.is_tensor(x) and x.is_cuda and x.dim() == 3 and self.proj_size == 0 and
                R.padded_hidden(self.hidden_size) is not None and (self.dropout == 0 or not self.training))

    def forward(self, x, hx=None):
        if not self._native_supported(x):
            return nn.LSTM.forward(self, x, hx)
        from zoo.ops import rnn as R
        xs = x if self.batch_first else x.transpose(0, 1)
        B = xs.shape[0]
        D = 2 if self.bidirectional else 1
        h0, c0 = hx if hx is not None else (None, None)
        hs, cs = [], []
        inp = xs.float()
        for layer in range(self.num_layers):
            outs = []
            for d in range(D):
                sfx = "_l%d%s" % (layer, "_reverse" if d else "")
                W, U = getattr(self, "weight_ih" + sfx), getattr(self, "weight_hh" + sfx)
                b = (getattr(self, "bias_ih" + sfx) + getattr(self, "bias_hh" + sfx)) if self.bias else \
                    torch.zeros(W.shape[0], device=x.device)
                i = layer * D + d
                hseq, hT, cT = R.recurrent(inp, W, b, U, "lstm", "tanh", "sigmoid",
                                           None if h0 is None else h0[i].float(),
                                           None if c0 is None else c0[i].float(), go_backwards=bool(d))
                outs.append((hseq.flip(1) if d else hseq).float())
                hs.append(hT.float())
                cs.append(cT.float())
            inp = outs[0] if D == 1 else torch.cat(outs, -1)
        out = inp if self.batch_first else inp.transpose(0, 1)
        hn = torch.stack(hs, 0)
        cn = torch.stack(cs, 0)
        return out.to(x.dtype), (hn.to(x.dtype), cn.to(x.dtype))


def _zrn(t, H):
    """torch GRU gate blocks (r, z, n) -> the kernel's order (z, r, n)."""
    return torch.cat([t[H:2 * H], t[:H], t[2 * H:]], 0)


def _gru_operands(W, U, b_ih, b_hh, H):
    """(W [3H, D], U [3H, H], xw bias [3H], b_hn [H]) of a torch GRU layer / cell in the
    reset-after kernel's gate order: the input projection carries b_ih (+ b_hh for z and r); the
    candidate's recurrent bias b_hn is applied inside the reset gate (rnn.hip CELL_GRU_RA)."""
    Wz, Uz = _zrn(W, H), _zrn(U, H)
    if b_ih is None:
        return Wz, Uz, torch.zeros(3 * H, device=W.device), None
    b = _zrn(b_ih, H) + torch.cat([b_hh[H:2 * H], b_hh[:H], torch.zeros(H, device=W.device, dtype=b_hh.dtype)])
    return Wz, Uz, b, b_hh[2 * H:]


def gru_cell_native(x, h, W, U, b_ih, b_hh, act="tanh"):
    """One torch.nn.GRUCell step (reset-after; candidate activation ``act``) on the native
    kernels: the input projection on the MFMA GEMM, the recurrent GEMM + gate math in one
    persistent-kernel launch (T = 1). None when the shape is unsupported."""
    from zoo.ops import rnn as R
    H = U.shape[1]
    if not (torch.is_tensor(x) and x.is_cuda and x.dim() == 2 and R.padded_hidden(H) is not None):
        return None
    Wz, Uz, b, bhn = _gru_operands(W, U, b_ih, b_hh, H)
    _, hT, _ = R.recurrent(x.float().unsqueeze(1), Wz, b, Uz, "gru_ra", act, "sigmoid",
                           None if h is None else h.float(), bhn=bhn)
    return hT


class ZGRU(_Twin, nn.GRU):
    """nn.GRU (any layer count, bidirectional) on the persistent recurrent kernel's reset-after GRU
    cell (rnn.hip CELL_GRU_RA): one input GEMM + one launch per layer and direction for the whole
    sequence, forward and backward. nn.GRU's signature and outputs ``(output, h_n)``."""

    def _native_supported(self, x):
        from zoo.ops import rnn as R
        return (torch.is_tensor(x) and x.is_cuda and x.dim() == 3 and
                R.padded_hidden(self.hidden_size) is not None and (self.dropout == 0 or not self.training))

    def forward(self, x, hx=None):
        if not self._native_supported(x):
            return nn.GRU.forward(self, x, hx)
        from zoo.ops import rnn as R
        xs = x if self.batch_first else x.transpose(0, 1)
        D = 2 if self.bidirectional else 1
        H = self.hidden_size
        hs = []
        inp = xs.float()
        for layer in range(self.num_layers):
            outs = []
            for d in range(D):
                sfx = "_l%d%s" % (layer, "_reverse" if d else "")
                W, U = getattr(self, "weight_ih" + sfx), getattr(self, "weight_hh" + sfx)
                bi = getattr(self, "bias_ih" + sfx) if self.bias else None
                bh = getattr(self, "bias_hh" + sfx) if self.bias else None
                Wz, Uz, b, bhn = _gru_operands(W, U, bi, bh, H)
                i = layer * D + d
                hseq, hT, _ = R.recurrent(inp, Wz, b, Uz, "gru_ra", "tanh", "sigmoid",
                                          None if hx is None else hx[i].float(), go_backwards=bool(d), bhn=bhn)
                outs.append((hseq.flip(1) if d else hseq).float())
                hs.append(hT.float())
            inp = outs[0] if D == 1 else torch.cat(outs, -1)
        out = inp if self.batch_first else inp.transpose(0, 1)
        return out.to(x.dtype), torch.stack(hs, 0).to(x.dtype)


class ZGRUCell(_Twin, nn.GRUCell):
    """nn.GRUCell on the native GEMM + one recurrent-kernel step (``gru_cell_native``)."""

    def forward(self, x, hx=None):
        if torch.is_tensor(x) and x.dim() == 2:
            y = gru_cell_native(x, hx, self.weight_ih, self.weight_hh, self.bias_ih, self.bias_hh)
            if y is not None:
                return y.to(x.dtype)
        return nn.GRUCell.forward(self, x, hx)


# exact torch class -> twin class (subclasses of the torch classes are left alone: they may
# override forward)
_TWINS = {nn.Conv2d: ZConv2d, nn.ConvTranspose2d: ZConvTranspose2d, nn.Linear: ZLinear, nn.BatchNorm2d: ZBatchNorm2d, nn.MaxPool2d: ZMaxPool2d,
          nn.AvgPool2d: ZAvgPool2d, nn.AdaptiveAvgPool2d: ZAdaptiveAvgPool2d, nn.LocalResponseNorm: ZLocalResponseNorm,
          nn.ReLU: ZReLU, nn.Tanh: ZTanh, nn.Sigmoid: ZSigmoid, nn.ELU: ZELU, nn.LeakyReLU: ZLeakyReLU,
          nn.ReLU6: ZReLU6, nn.GELU: ZGELU, nn.Softplus: ZSoftplus, nn.LSTM: ZLSTM, nn.GRU: ZGRU,
          nn.GRUCell: ZGRUCell,
          G.Pool2d: ZPool2d, G.LRN: ZLRN}


def _pair(v):
    return tuple(v) if isinstance(v, (list, tuple)) else (v, v)


def is_native(m):
    return isinstance(m, _Twin)


def to_twin(m):
    """Swap ``m``'s class for its native twin in place (no-op when it has none); returns m."""
    cls = _TWINS.get(type(m))
    if cls is None and type(m) is G.Fn and _act_name(m) is not None:
        cls = ZFn
    if cls is not None:
        m.__class__ = cls
    return m


def _fuse(conv, bn=None, act_mod=None):
    """conv [-> eval BatchNorm] [-> activation] as ONE native conv: the conv carries the BN and the
    activation, the absorbed modules pass their input through."""
    to_twin(conv)
    # a plain attribute, not a registered submodule: the BN stays where it is in the module tree
    # and the state dict keeps its original keys (the lowering is a class swap only)
    object.__setattr__(conv, "_zoo_bn", bn)
    conv._zoo_cache = None
    if bn is not None:
        to_twin(bn)
        bn._zoo_absorbed = True
    if act_mod is not None:
        conv._zoo_act = _act_name(act_mod)
        to_twin(act_mod)
        act_mod._zoo_absorbed = True


def _fusable_conv(m):
    return type(m) is nn.Conv2d


def _lower_sequence(mods, training):
    i = 0
    while i < len(mods):
        m = mods[i]
        if _fusable_conv(m):
            j, bn, act = i + 1, None, None
            if j < len(mods) and type(mods[j]) is nn.BatchNorm2d and not training and \
                    mods[j].num_features == m.out_channels:
                bn, j = mods[j], j + 1
            if j < len(mods) and _act_name(mods[j]) in _FUSABLE and type(mods[j]) in _TWINS:
                act, j = mods[j], j + 1
            _fuse(m, bn, act)
            i = j
            continue
        if type(m) is nn.Linear:
            to_twin(m)
            if i + 1 < len(mods) and type(mods[i + 1]) in (nn.ReLU, nn.GELU) and \
                    (type(mods[i + 1]) is not nn.GELU or mods[i + 1].approximate == "none"):
                m._zoo_act = _act_name(mods[i + 1])
                to_twin(mods[i + 1])
                mods[i + 1]._zoo_absorbed = True
                i += 2
                continue
        lower_module(m, training)
        i += 1


def lower_module(module, training=False, inplace=True):
    """Swap every supported submodule of ``module`` (and ``module`` itself) for its native twin,
    in place (``inplace=False`` works on a deep copy); ``nn.Sequential`` runs additionally fuse
    conv [-> BatchNorm (inference only)] [-> ReLU / tanh / sigmoid] and linear -> ReLU / GELU.
    Parameters, buffers and state_dict keys are unchanged."""
    if not inplace:
        module = copy.deepcopy(module)
    if isinstance(module, nn.Sequential):
        _lower_sequence(list(module), training)
        return module
    to_twin(module)
    for child in module.children():
        lower_module(child, training)
    return module


def lower_graph(graph, training=False):
    """Lower a GraphNet in place: every node op gets its native twin; in inference
    (``training=False``) a conv node feeding only a BatchNorm node (feeding only an activation
    node) becomes one fused native conv and the absorbed nodes pass through."""
    consumers = {}
    for n in graph.node_names:
        for i in graph.node_inputs[n]:
            consumers.setdefault(i, []).append(n)
    outputs = set(graph.outputs)

    def sole(n):
        c = consumers.get(n, [])
        return c[0] if len(c) == 1 and n not in outputs else None

    done = set()
    for n in graph.node_names:
        if n in done:
            continue
        op = graph.node(n).op
        if _fusable_conv(op):
            bn = act = None
            nxt = sole(n)
            if nxt is not None and not training and type(graph.node(nxt).op) is nn.BatchNorm2d and \
                    graph.node(nxt).op.num_features == op.out_channels:
                bn = graph.node(nxt).op
                done.add(nxt)
                nxt = sole(nxt)
            if nxt is not None and _act_name(graph.node(nxt).op) in _FUSABLE and \
                    (type(graph.node(nxt).op) in _TWINS or type(graph.node(nxt).op) is G.Fn):
                act = graph.node(nxt).op
                done.add(nxt)
            _fuse(op, bn, act)
            continue
        lower_module(op, training)
    graph._native = True
    return graph


# ---------------------------------------------------------------------------------------------
# functional forms (the ONNX importer's node ops)
# ---------------------------------------------------------------------------------------------
_PACK_CACHE = {}


def _packed_cached(w, b):
    """Packed native weight / padded bias of an NCHW conv weight (ONNX initialisers: cached by
    tensor identity and version, recomputed only after an update)."""
    key = (id(w), None if b is None else id(b))
    ver = (w._version, w.data_ptr(), None if b is None else b._version, _kern.weights_epoch())
    hit = _PACK_CACHE.get(key)
    need_grad = torch.is_grad_enabled() and (w.requires_grad or (b is not None and b.requires_grad))
    # ids are reused after garbage collection: the entry also holds weak references to its tensors
    if hit is not None and hit[0] == ver and not need_grad and hit[3]() is w and \
            (b is None or (hit[4] is not None and hit[4]() is b)):
        return hit[1], hit[2]
    K, C, R, S = w.shape
    cp, kp = _cin_pad(C), ops.ceil8(K)
    w2 = F.pad(w.float().permute(0, 2, 3, 1), (0, cp - C, 0, 0, 0, 0, 0, kp - K)).reshape(kp, R * S * cp)
    ld = ops.ceil8(R * S * cp)
    if ld != R * S * cp:
        w2 = F.pad(w2, (0, ld - R * S * cp))
    bb = F.pad(b.float() if b is not None else torch.zeros(K, device=w.device), (0, kp - K))
    if not need_grad:
        _PACK_CACHE[key] = (ver, w2.detach().contiguous(), bb.detach().contiguous(), weakref.ref(w),
                            None if b is None else weakref.ref(b))
        if len(_PACK_CACHE) > 4096:
            _PACK_CACHE.clear()
    return w2, bb


def conv2d_nchw(x, w, b=None, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups=1, act=None):
    """F.conv2d semantics (NCHW in / out) on the native kernels; None when unsupported."""
    if not (_native_ok(x) and groups == 1 and w.dim() == 4):
        return None
    K, C, R, S = w.shape
    w2, bb = _packed_cached(w, b)
    y = ops.conv2d_nhwc(to_nhwc(x, _cin_pad(C)), w2, bb, kernel=(R, S), stride=tuple(stride), pad=tuple(pad),
                        dil=tuple(dil), act=act if act in _FUSABLE else None)
    return from_nhwc(y, K, x.dtype)


def pool2d_nchw(x, kind, kernel, stride, pad=(0, 0), ceil_mode=False, count_include_pad=True):
    """max / avg pooling (NCHW in / out) on the native kernels; None when unsupported."""
    if not _native_ok(x):
        return None
    if kind == "max" and (2 * pad[0] > kernel[0] or 2 * pad[1] > kernel[1]):
        return None
    return _pool_native(x, kind, tuple(kernel), tuple(stride), tuple(pad), ceil_mode, count_include_pad)


def global_avg_pool_nchw(x):
    if not _native_ok(x):
        return None
    return _pool_native(x, "avg", None, None, None, global_pool=True)


def batch_norm_nchw_eval(x, mean, var, gamma, beta, eps):
    """Inference BatchNorm as a native per-channel affine (NHWC BN kernel, running statistics)."""
    if not _native_ok(x):
        return None
    C = x.shape[1]
    bn = nn.BatchNorm2d(C, eps=eps).to(x.device).eval()
    with torch.no_grad():
        bn.running_mean.copy_(mean.float())
        bn.running_var.copy_(var.float())
        bn.weight.copy_(gamma.float())
        bn.bias.copy_(beta.float())
    return from_nhwc(_bn_nhwc(to_nhwc(x), bn, C), C, x.dtype)


def activation(x, name, alpha=None):
    """Native elementwise activation for CUDA tensors (layout preserved)."""
    return _act_native(x, name, alpha)


__all__ = ["lower_module", "lower_graph", "to_twin", "is_native", "ZConv2d", "ZLinear", "ZBatchNorm2d", "ZMaxPool2d",
           "ZAvgPool2d", "ZLSTM", "to_nhwc", "from_nhwc", "conv2d_nchw", "pool2d_nchw"]
