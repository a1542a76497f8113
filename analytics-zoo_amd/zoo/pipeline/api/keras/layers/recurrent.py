"""Recurrent layers: SimpleRNN, LSTM, GRU, ConvLSTM2D, ConvLSTM3D
(Py/pipeline/api/keras/layers/recurrent.py, convolutional_recurrent.py;
Zs LSTM.scala:71-80, GRU, SimpleRNN, InternalRecurrent.scala:80-140).

The input projection of ALL timesteps is one GEMM on the native MFMA kernel
(``zoo.ops.linear`` over [batch*steps, input_dim]). On the GPU the whole
recurrence (forward and BPTT) is then ONE persistent HIP kernel launch
(``zoo.ops.rnn``, csrc/kernels/rnn.hip) for hidden sizes up to 256; the
per-step path below (one [batch, hidden] x [hidden, gates*hidden] GEMM per step
plus the gate math) is the CPU reference and the fallback for wider layers.
Gate order follows Keras 1: LSTM (i, f, c, o), GRU (z, r, h).
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from zoo import ops
from zoo.ops.layers import lstm_gates
from zoo.ops import rnn as rnn_ops
from zoo.pipeline.api.keras.base import Layer, apply_activation, init_tensor
from zoo.parallel.flat import grad_slot


class _RNNBase(Layer):
    n_gates = 1

    def __init__(self, output_dim, activation="tanh", inner_activation="hard_sigmoid", return_sequences=False,
                 go_backwards=False, W_regularizer=None, U_regularizer=None, b_regularizer=None, input_shape=None,
                 init="glorot_uniform", inner_init="orthogonal", return_state=False, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.output_dim = int(output_dim)
        self.return_state = return_state
        self.activation, self.inner_activation = activation, inner_activation
        self.return_sequences, self.go_backwards = return_sequences, go_backwards
        self.init, self.inner_init = init, inner_init
        self.add_regularizer(W_regularizer, "W")
        self.add_regularizer(U_regularizer, "U")
        self.add_regularizer(b_regularizer, "b")

    def build(self, input_shape):
        d, h, g = input_shape[-1], self.output_dim, self.n_gates
        self.W = nn.Parameter(init_tensor(torch.empty(g * h, d), self.init, fan_in=d, fan_out=h))
        U = torch.empty(g * h, h)
        for i in range(g):
            if self.inner_init == "orthogonal":
                nn.init.orthogonal_(U[i * h:(i + 1) * h])
            else:
                init_tensor(U[i * h:(i + 1) * h], self.inner_init)
        self.U = nn.Parameter(U)
        b = torch.zeros(g * h)
        if isinstance(self, LSTM):
            b[h:2 * h] = 1.0  # forget-gate bias (Keras unit_forget_bias)
        self.b = nn.Parameter(b)

    def build_shapes(self, input_shape):
        return input_shape[0] if isinstance(input_shape, list) else input_shape

    def _ensure_built(self, input_shape):
        super()._ensure_built(self.build_shapes(input_shape))

    def compute_output_shape(self, input_shape):
        input_shape = self.build_shapes(input_shape)
        out = (None, input_shape[1], self.output_dim) if self.return_sequences else (None, self.output_dim)
        if self.return_state:
            return [out] + [(None, self.output_dim)] * self._n_state
        return out

    _n_state = 1
    _cell = None  # zoo.ops.rnn cell name of the fused GPU path

    def _fused_ok(self, x):
        acts = (self.activation,) if self._cell == "rnn" else (self.activation, self.inner_activation)
        return self._cell is not None and rnn_ops.supported(x, self.output_dim, *acts)

    def _call_fused(self, x, init):
        h0 = init[0] if init else None
        c0 = init[1] if (init and len(init) > 1) else None
        hseq, hT, cT = rnn_ops.recurrent(x, self.W, self.b, self.U, self._cell, self.activation,
                                         self.inner_activation if self._cell != "rnn" else None, h0=h0, c0=c0,
                                         go_backwards=self.go_backwards)
        dt = x.dtype if x.is_floating_point() else hseq.dtype
        out = (hseq if self.return_sequences else hT).to(dt)
        if self.return_state:
            return [out, hT.to(dt)] + ([cT.to(dt)] if cT is not None else [])
        return out

    def _step(self, xt, state):
        raise NotImplementedError

    def _init_state(self, x):
        h = x.new_zeros(x.shape[0], self.output_dim)
        return (h,)

    def call(self, x):
        init = None
        if isinstance(x, (list, tuple)):  # [sequence, initial states...] (Seq2seq decoder / bridge)
            x, init = x[0], tuple(x[1:])
        if self._fused_ok(x):
            return self._call_fused(x, init)
        B, T, D = x.shape
        xw = ops.linear(x.reshape(B * T, D), self.W, self.b).reshape(B, T, -1)
        state = self._init_state(x) if not init else tuple(t.to(xw.dtype) for t in init)
        outs = []
        steps = range(T - 1, -1, -1) if self.go_backwards else range(T)
        for t in steps:
            state = self._step(xw[:, t], state)
            if self.return_sequences:
                outs.append(state[0])
        out = torch.stack(outs, dim=1) if self.return_sequences else state[0]
        if self.return_state:
            return [out] + list(state)
        return out


class SimpleRNN(_RNNBase):
    n_gates = 1
    _cell = "rnn"

    def __init__(self, output_dim, activation="tanh", return_sequences=False, go_backwards=False,
                 W_regularizer=None, U_regularizer=None, b_regularizer=None, input_shape=None, **kwargs):
        super().__init__(output_dim, activation, None, return_sequences, go_backwards, W_regularizer, U_regularizer,
                         b_regularizer, input_shape, **kwargs)

    def _step(self, xt, state):
        (h,) = state
        return (apply_activation(xt + ops.linear(h, self.U), self.activation),)


class LSTM(_RNNBase):
    n_gates = 4
    _n_state = 2
    _cell = "lstm"

    def _init_state(self, x):
        z = x.new_zeros(x.shape[0], self.output_dim)
        return (z, z.clone())

    def _step(self, xt, state):
        h, c = state
        H = self.output_dim
        g = xt + ops.linear(h, self.U)
        i = apply_activation(g[:, :H], self.inner_activation)
        f = apply_activation(g[:, H:2 * H], self.inner_activation)
        cc = apply_activation(g[:, 2 * H:3 * H], self.activation)
        o = apply_activation(g[:, 3 * H:], self.inner_activation)
        c = f * c + i * cc
        h = o * apply_activation(c, self.activation)
        return (h, c)


class GRU(_RNNBase):
    n_gates = 3
    _cell = "gru"

    def _step(self, xt, state):
        (h,) = state
        H = self.output_dim
        uh = ops.linear(h, self.U[: 2 * H])
        z = apply_activation(xt[:, :H] + uh[:, :H], self.inner_activation)
        r = apply_activation(xt[:, H:2 * H] + uh[:, H:], self.inner_activation)
        hh = apply_activation(xt[:, 2 * H:] + ops.linear(r * h, self.U[2 * H:]), self.activation)
        return (z * h + (1 - z) * hh,)


# whole-sequence ConvLSTM2D path (_ConvLSTMSeqFn); ZOO_CONVLSTM_SEQ=0 keeps the per-step
# autograd loop (A/B and fallback)
_CONVLSTM_SEQ = True
# one launch per step (_ConvLSTMFusedFn, csrc/kernels/convlstm.hip) for up to 64 filters;
# ZOO_CONVLSTM_FUSED=0 keeps the conv + step-kernel sequence path (A/B)
_CONVLSTM_FUSED = True


def _gate_perm(f, device):
    """Row order of the gate-interleaved layout: row 4j + g takes torch row g*f + j (gate g of
    hidden channel j), so one MFMA accumulator lane holds all four gates of a channel."""
    return (torch.arange(4, device=device)[None, :] * f + torch.arange(f, device=device)[:, None]).reshape(-1)


def _gate_interleave(w, f):
    """``w[_gate_perm(f)]`` as a reshape / transpose (no index kernels: the fancy index's backward
    sorted the indices, a dozen small launches per call)."""
    return w.reshape((4, f) + tuple(w.shape[1:])).transpose(0, 1).reshape(tuple(w.shape))


class _ConvLSTMFusedFn(torch.autograd.Function):
    """Whole ConvLSTM2D sequence, ONE launch per step each way, issued by a C++ loop
    (convlstm_fwd_seq / convlstm_bwd_seq; csrc/kernels/convlstm.hip): the
    recurrent conv is an MFMA implicit GEMM whose epilogue runs the LSTM cell (forward) or the
    cell backward on the recurrent data gradient (backward). Gate tensors are gate-interleaved
    ([M][F][4], weights permuted by _gate_perm). The recurrent weight gradient is ONE conv_wgrad
    over all steps at the end (the per-step bf16 gate gradients are kept, [T][B,H,W,K8]).
    Reference: InternalConvLSTM2D.scala (Zs/pipeline/api/keras/layers)."""

    @staticmethod
    def forward(ctx, gxs, wh, B, Ho, Wo, f, cph, R, S, iact, act, return_sequences):
        C_ = ops.native()
        from zoo.ops.conv import bf16_weight
        T, M, K = gxs.shape
        dev = gxs.device
        whb = bf16_weight(wh)
        hist = torch.zeros(T + 1, B, Ho, Wo, cph, dtype=torch.bfloat16, device=dev)
        hseq = torch.empty(T, M, f, dtype=torch.float32, device=dev)
        cseq = torch.empty_like(hseq)
        acts = torch.empty(T, M, K, dtype=torch.float32, device=dev)
        C_.convlstm_fwd_seq(gxs, whb, B, 1, Ho, Wo, 1, R, S, hist, hseq, cseq, acts, iact, act)
        ctx.save_for_backward(wh, hist, cseq, acts)
        ctx.geo = (B, Ho, Wo, f, cph, R, S, iact, act, return_sequences)
        return hseq if return_sequences else hseq[T - 1].clone()

    @staticmethod
    def backward(ctx, dout):
        C_ = ops.native()
        from zoo.ops import _kern
        from zoo.ops.conv import bf16_weight
        wh, hist, cseq, acts = ctx.saved_tensors
        B, Ho, Wo, f, cph, R, S, iact, act, rseq = ctx.geo
        T, M, K = acts.shape
        dev = acts.device
        K8 = wh.shape[0]
        whf = _kern.flip_weights(bf16_weight(wh), K8, R, S, cph)
        dgxs = torch.empty(T, M, K, dtype=torch.float32, device=dev)
        dgb = torch.zeros(T, B, Ho, Wo, K8, dtype=torch.bfloat16, device=dev)
        dc = torch.empty(M, f, dtype=torch.float32, device=dev)
        dout = dout.contiguous().float()
        C_.convlstm_bwd_seq(dout, bool(rseq), whf, B, 1, Ho, Wo, 1, R, S, acts, cseq, dc, dgxs, dgb, iact, act)
        dw = None
        if ctx.needs_input_grad[1]:
            gbuf = grad_slot(wh)
            dwh = gbuf if gbuf is not None else torch.zeros(wh.shape, dtype=torch.float32, device=dev)
            if T > 1:
                # every step's recurrent weight gradient in one conv: (T-1)*B images
                C_.conv_wgrad(hist[1:T].reshape((T - 1) * B, Ho, Wo, cph), dgb[1:T].reshape((T - 1) * B, Ho, Wo, K8),
                              dwh, R, S, 1, 1, R // 2, S // 2, 1, 1)
            if gbuf is not None:
                hook = getattr(wh, "_zoo_grad_ready", None)
                if hook is not None:
                    hook(wh)
            else:
                dw = dwh.to(wh.dtype)
        return dgxs, dw, None, None, None, None, None, None, None, None, None, None


class _ConvLSTMSeqFn(torch.autograd.Function):
    """Whole ConvLSTM2D sequence on the native kernels with no per-step Python tensor glue:
    per step ONE recurrent implicit-GEMM conv (fp32 gate pre-activations) and ONE fused step
    kernel (gates, cell, hidden; h_t also written as bf16 into the padded NHWC history slot the
    next step's conv reads). Backward through time per step: one fused step-backward kernel
    (gate gradients fp32 for the input conv + bf16 for the recurrent convs, dc_prev), one
    recurrent dgrad (weights flipped once per sequence) and one wgrad accumulating dWh in fp32.
    Reference: InternalConvLSTM2D.scala (Zs/pipeline/api/keras/layers)."""

    @staticmethod
    def forward(ctx, gxs, wh, B, Ho, Wo, f, cph, R, S, iact, act, return_sequences):
        C_ = ops.native()
        from zoo.ops import _kern
        from zoo.ops.conv import bf16_weight
        T, M, K = gxs.shape
        dev = gxs.device
        pad = (R // 2, S // 2)
        whb = bf16_weight(wh)
        hist = torch.zeros(T + 1, B, Ho, Wo, cph, dtype=torch.bfloat16, device=dev)
        hseq = torch.empty(T, M, f, dtype=torch.float32, device=dev)
        cseq = torch.empty_like(hseq)
        acts = torch.empty(T, M, K, dtype=torch.float32, device=dev)
        for s in range(T):
            gh = None
            if s > 0:
                gh = _kern.conv_fwd(hist[s], whb, R, S, (1, 1), pad, out_f32=True, out_bf16=False)
            C_.lstm_step_fwd(gxs[s], gh, cseq[s - 1] if s > 0 else None, hseq[s], cseq[s], acts[s], hist[s + 1],
                             iact, act)
        ctx.save_for_backward(wh, hist, cseq, acts)
        ctx.geo = (B, Ho, Wo, f, cph, R, S, iact, act, return_sequences)
        return hseq if return_sequences else hseq[T - 1].clone()

    @staticmethod
    def backward(ctx, dout):
        C_ = ops.native()
        from zoo.ops import _kern
        from zoo.ops.conv import bf16_weight
        wh, hist, cseq, acts = ctx.saved_tensors
        B, Ho, Wo, f, cph, R, S, iact, act, rseq = ctx.geo
        T, M, K = acts.shape
        dev = acts.device
        pad = (R // 2, S // 2)
        K8 = wh.shape[0]
        whb = bf16_weight(wh)
        whf = _kern.flip_weights(whb, K8, R, S, cph)          # once per sequence
        dgxs = torch.empty(T, M, K, dtype=torch.float32, device=dev)
        dgb = torch.zeros(B, Ho, Wo, K8, dtype=torch.bfloat16, device=dev)
        dc = torch.empty(M, f, dtype=torch.float32, device=dev)
        dc_next = None
        dhr = None
        gbuf = grad_slot(wh)
        dwh = gbuf if (gbuf is not None and ctx.needs_input_grad[1]) else \
            torch.zeros(wh.shape, dtype=torch.float32, device=dev)
        dout = dout.contiguous().float()
        for s in range(T - 1, -1, -1):
            d = dout[s] if rseq else (dout if s == T - 1 else None)
            C_.lstm_step_bwd(d, dhr, dc_next, acts[s], cseq[s - 1] if s > 0 else None, cseq[s], dgxs[s], dgb, dc,
                             iact, act)
            dc_next = dc.clone() if s > 0 else None
            if s > 0:
                if ctx.needs_input_grad[1]:
                    C_.conv_wgrad(hist[s], dgb, dwh, R, S, 1, 1, pad[0], pad[1], 1, 1)
                dhr = _kern.conv_fwd(dgb, whf, R, S, (1, 1), (R - 1 - pad[0], S - 1 - pad[1]))
        if gbuf is not None and ctx.needs_input_grad[1]:
            hook = getattr(wh, "_zoo_grad_ready", None)
            if hook is not None:
                hook(wh)
            dw = None
        else:
            dw = dwh.to(wh.dtype) if ctx.needs_input_grad[1] else None
        return dgxs, dw, None, None, None, None, None, None, None, None, None, None


class ConvLSTM2D(Layer):
    """Convolutional LSTM over (batch, time, channels, rows, cols) ('th')."""

    def __init__(self, nb_filter, nb_row, nb_col, activation="tanh", inner_activation="hard_sigmoid",
                 dim_ordering="th", border_mode="same", subsample=(1, 1), W_regularizer=None, U_regularizer=None,
                 b_regularizer=None, return_sequences=False, go_backwards=False, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.k = int(nb_filter), (nb_row, nb_col)
        self.activation, self.inner_activation = activation, inner_activation
        self.return_sequences, self.go_backwards = return_sequences, go_backwards
        self.subsample = tuple(subsample) if isinstance(subsample, (tuple, list)) else (subsample, subsample)

    def build(self, input_shape):
        c = input_shape[2]
        f = self.nb_filter
        self.Wx = nn.Parameter(init_tensor(torch.empty(4 * f, c, *self.k), "glorot_uniform"))
        self.Wh = nn.Parameter(init_tensor(torch.empty(4 * f, f, *self.k), "glorot_uniform"))
        self.b = nn.Parameter(torch.zeros(4 * f))

    def compute_output_shape(self, s):
        h = (s[3] + self.subsample[0] - 1) // self.subsample[0]
        w = (s[4] + self.subsample[1] - 1) // self.subsample[1]
        if self.return_sequences:
            return (None, s[1], self.nb_filter, h, w)
        return (None, self.nb_filter, h, w)

    def _packed(self, w):
        """[4f, c, kh, kw] torch-layout weight -> the native kernels' packed [K8, ldb] weight
        (differentiable: the conv's weight gradient flows back to the parameter)."""
        K, C, R, S = w.shape
        cp = C if C % 8 == 0 else (4 if C <= 4 else ops.ceil8(C))
        w4 = F.pad(w.permute(0, 2, 3, 1), (0, cp - C, 0, 0, 0, 0, 0, ops.ceil8(K) - K))
        return ops.pack_weight(w4), cp

    def _call_native(self, x):
        """GPU path: input and recurrent convolutions on the implicit-GEMM MFMA kernel in
        NHWC (bf16), gate math on the same tensors."""
        B, T, C, H, W = x.shape
        f = self.nb_filter
        K = 4 * f
        R, S = self.k
        pad = (R // 2, S // 2)
        fused = _CONVLSTM_SEQ and _CONVLSTM_FUSED and f <= 64 and K % 8 == 0
        Wx, Wh, b = self.Wx, self.Wh, self.b
        if fused:   # gate-interleaved rows (the permutation's gradient flows back to the parameters)
            Wx, Wh, b = _gate_interleave(Wx, f), _gate_interleave(Wh, f), _gate_interleave(b, f)
        wx, cpx = self._packed(Wx)
        wh, cph = self._packed(Wh)
        bias = F.pad(b, (0, ops.ceil8(K) - K)).float()
        seq = _CONVLSTM_SEQ and K % 8 == 0 and ops.ceil8(K) == wh.shape[0]
        if seq:
            # time-major in processing order already at the (small) input: the input conv then
            # writes the [T, M, K] gate inputs the sequence kernels read, no gate-tensor permute
            xt = x.transpose(0, 1)
            if self.go_backwards:
                xt = xt.flip(0)
            xn = xt.reshape(T * B, C, H, W).permute(0, 2, 3, 1)
        else:
            xn = x.reshape(B * T, C, H, W).permute(0, 2, 3, 1)
        if cpx != C:
            xn = F.pad(xn, (0, cpx - C))
        xs = ops.conv2d_nhwc(xn, wx, bias, kernel=(R, S), stride=self.subsample, pad=pad, out_f32=True)[..., :K]
        Ho, Wo = xs.shape[1], xs.shape[2]
        from zoo.ops.layers import ACT_CODES
        if seq:
            # whole-sequence path: time-major gate inputs in processing order, one autograd node
            M = B * Ho * Wo
            gxs = xs.reshape(T, M, K)
            fn = _ConvLSTMFusedFn if fused else _ConvLSTMSeqFn
            hs = fn.apply(gxs.contiguous(), wh, B, Ho, Wo, f, cph, R, S,
                                      ACT_CODES[self.inner_activation], ACT_CODES[self.activation],
                                      bool(self.return_sequences))
            if self.return_sequences:
                return hs.reshape(T, B, Ho, Wo, f).permute(1, 0, 4, 2, 3)
            return hs.reshape(B, Ho, Wo, f).permute(0, 3, 1, 2)
        xs = xs.reshape(B, T, Ho * Wo, K)
        M = B * Ho * Wo
        h = c = None
        outs = []
        for t in (range(T - 1, -1, -1) if self.go_backwards else range(T)):
            gh = None
            if h is not None:   # h_0 = 0: no recurrent conv on the first step
                hn = h.reshape(B, Ho, Wo, f)
                hp = F.pad(hn, (0, cph - f)) if cph != f else hn
                gh = ops.conv2d_nhwc(hp, wh, None, kernel=(R, S), stride=(1, 1), pad=pad,
                                     out_f32=True)[..., :K].reshape(M, K)
            # gate activations, cell and hidden update in ONE native pass (keras_ops.hip)
            h, c = lstm_gates(xs[:, t].reshape(M, K), gh, c, self.inner_activation, self.activation)
            outs.append(h.reshape(B, Ho, Wo, f).permute(0, 3, 1, 2))
        return torch.stack(outs, 1) if self.return_sequences else outs[-1]

    def call(self, x):
        from zoo.ops.layers import ACT_CODES
        if x.is_cuda and (self.k[0] % 2 == 1 and self.k[1] % 2 == 1) and \
                self.activation in ACT_CODES and self.inner_activation in ACT_CODES:
            return self._call_native(x)
        B, T = x.shape[:2]
        pad = (self.k[0] // 2, self.k[1] // 2)
        xs = F.conv2d(x.reshape(B * T, *x.shape[2:]), self.Wx.to(x.dtype), self.b.to(x.dtype), self.subsample, pad)
        xs = xs.reshape(B, T, *xs.shape[1:])
        f = self.nb_filter
        h = x.new_zeros(B, f, xs.shape[3], xs.shape[4])
        c = h.clone()
        outs = []
        for t in (range(T - 1, -1, -1) if self.go_backwards else range(T)):
            g = xs[:, t] + F.conv2d(h, self.Wh.to(h.dtype), None, 1, pad)
            i = apply_activation(g[:, :f], self.inner_activation)
            fg = apply_activation(g[:, f:2 * f], self.inner_activation)
            cc = apply_activation(g[:, 2 * f:3 * f], self.activation)
            o = apply_activation(g[:, 3 * f:], self.inner_activation)
            c = fg * c + i * cc
            h = o * apply_activation(c, self.activation)
            outs.append(h)
        return torch.stack(outs, 1) if self.return_sequences else h


class _ConvLSTM3DFusedFn(torch.autograd.Function):
    """Whole ConvLSTM3D sequence, one launch per step each way: the convlstm.hip step kernels
    with a depth axis (no per-step pad / permute / conv3d glue). ``whp``: the recurrent weight
    [4f, f, k, k, k] in gate-interleaved row order; packed (and flipped for the backward) here
    once per call. Recurrent weight gradient: one conv_wgrad over all steps, the depth taps stacked
    on channels.
    ``gxs``: the input convolution's bf16 output [T, M, 4f] as is (the step kernel widens it; no
    fp32 copy of the gate tensor), and its gradient is the step kernels' bf16 gate gradients (the
    operand the recurrent data / weight gradients read anyway; no fp32 gate-gradient tensor).
    Reference: InternalConvLSTM3D.scala (Zs/pipeline/api/keras/layers)."""

    @staticmethod
    def forward(ctx, gxs, whp, B, D, H, W, f, k, return_sequences):
        C_ = ops.native()
        T, M, K = gxs.shape
        dev = gxs.device
        cph, K8 = ops.ceil8(f), ops.ceil8(K)
        w5 = F.pad(whp.detach().permute(0, 2, 3, 4, 1), (0, cph - f, 0, 0, 0, 0, 0, 0, 0, K8 - K))
        wpk = ops.pack_weight(w5.reshape(K8, k, k * k, cph)).to(torch.bfloat16)   # [K8][k^3 * cph]
        hist = torch.zeros(T + 1, B, D, H, W, cph, dtype=torch.bfloat16, device=dev)
        hseq = torch.empty(T, M, f, dtype=torch.float32, device=dev)
        cseq = torch.empty_like(hseq)
        acts = torch.empty(T, M, K, dtype=torch.float32, device=dev)
        C_.convlstm_fwd_seq(gxs, wpk, B, D, H, W, k, k, k, hist, hseq, cseq, acts, 2, 1)
        ctx.save_for_backward(whp, hist, cseq, acts)
        ctx.geo = (B, D, H, W, f, k, return_sequences)
        return hseq if return_sequences else hseq[T - 1].clone()

    @staticmethod
    def backward(ctx, dout):
        C_ = ops.native()
        whp, hist, cseq, acts = ctx.saved_tensors
        B, D, H, W, f, k, rseq = ctx.geo
        T, M, K = acts.shape
        dev = acts.device
        cph, K8 = ops.ceil8(f), ops.ceil8(K)
        # flipped weight for the recurrent data gradient: [cph][k^3 * K8], taps reversed
        w5 = F.pad(whp.detach().permute(0, 2, 3, 4, 1), (0, cph - f, 0, 0, 0, 0, 0, 0, 0, K8 - K))
        wfl = w5.flip(1, 2, 3).permute(4, 1, 2, 3, 0).reshape(cph, k, k * k, K8)
        wfl = ops.pack_weight(wfl).to(torch.bfloat16)
        # every step kernel writes all K = 4f gate channels: zero-filled only for K8 > K padding
        dgb = (torch.empty if K8 == K else torch.zeros)(T, B, D, H, W, K8, dtype=torch.bfloat16, device=dev)
        dc = torch.empty(M, f, dtype=torch.float32, device=dev)
        dout = dout.contiguous().float()
        C_.convlstm_bwd_seq(dout, bool(rseq), wfl, B, D, H, W, k, k, k, acts, cseq, dc, None, dgb, 2, 1)
        dgxs = dgb.view(T, M, K8)[..., :K]
        dw = None
        if ctx.needs_input_grad[1]:
            dw5 = torch.zeros(K8, k, k, k, cph, dtype=torch.float32, device=dev)
            if T > 1:
                p = k // 2
                hp = F.pad(hist[1:T], (0, 0, 0, 0, 0, 0, p, p))          # depth-padded inputs of steps 1..T-1
                gy = dgb[1:T].reshape((T - 1) * B * D, H, W, K8)
                # the depth taps stacked on channels (channel kd * cph + c, as conv3d_ndhwc): ONE
                # k x k weight gradient with a k * cph-deep input instead of one per depth tap
                xk = torch.cat([hp[:, :, kd:kd + D] for kd in range(k)], dim=-1).reshape((T - 1) * B * D, H, W, k * cph)
                part = torch.zeros(K8, k * k * k * cph, dtype=torch.float32, device=dev)
                C_.conv_wgrad(xk, gy, part, k, k, 1, 1, p, p, 1, 1)
                dw5 = part.view(K8, k, k, k, cph).permute(0, 3, 1, 2, 4)   # [K8][kh][kw][kd][c] -> [K8][kd][kh][kw][c]
            dw = dw5[:K, ..., :f].permute(0, 4, 1, 2, 3).to(whp.dtype)
        return dgxs, dw, None, None, None, None, None, None, None


class ConvLSTM3D(Layer):
    """Convolutional LSTM over (batch, time, channels, d1, d2, d3)."""

    def __init__(self, nb_filter, nb_kernel, dim_ordering="th", border_mode="same", subsample=(1, 1, 1),
                 W_regularizer=None, U_regularizer=None, b_regularizer=None, return_sequences=False,
                 go_backwards=False, input_shape=None, **kwargs):
        super().__init__(input_shape=input_shape, **kwargs)
        self.nb_filter, self.k = int(nb_filter), int(nb_kernel)
        self.return_sequences, self.go_backwards = return_sequences, go_backwards

    def build(self, input_shape):
        c, f, k = input_shape[2], self.nb_filter, self.k
        self.Wx = nn.Parameter(init_tensor(torch.empty(4 * f, c, k, k, k), "glorot_uniform"))
        self.Wh = nn.Parameter(init_tensor(torch.empty(4 * f, f, k, k, k), "glorot_uniform"))
        self.b = nn.Parameter(torch.zeros(4 * f))

    def compute_output_shape(self, s):
        if self.return_sequences:
            return (None, s[1], self.nb_filter) + tuple(s[3:])
        return (None, self.nb_filter) + tuple(s[3:])

    def _call_native(self, x):
        """GPU path (InternalConvLSTM3D.scala): the input convolution for all timesteps in one
        3-D conv (implicit-GEMM launches), then the whole sequence on the one-launch-per-step
        kernels (_ConvLSTM3DFusedFn); beyond 64 filters (or with ZOO_CONVLSTM_FUSED=0) per step one
        recurrent 3-D conv and one fused gate / cell / hidden pass."""
        from zoo.ops.layers import conv3d_ndhwc
        B, T, C = x.shape[:3]
        sp = tuple(x.shape[3:])
        f, k = self.nb_filter, self.k
        K = 4 * f
        p = k // 2
        cp, fp, kp = (-C) % 8, (-f) % 8, (-K) % 8
        # gate-interleaved one-launch-per-step path (convlstm.hip) up to 64 filters
        il = _CONVLSTM_SEQ and _CONVLSTM_FUSED and f <= 64 and K % 8 == 0
        if il:   # time-major in processing order at the input (see ConvLSTM2D)
            xt = x.transpose(0, 1)
            if self.go_backwards:
                xt = xt.flip(0)
        else:
            xt = x
        # [N, C, *sp] -> channels-last bf16 [N, *sp, C + cp] in ONE strided copy (reshape of the
        # transposed input, pad and cast were three full passes over it)
        xn = torch.empty((T * B,) + sp + (C + cp,), dtype=torch.bfloat16, device=x.device)
        xv = xn.view((xt.shape[0], xt.shape[1]) + sp + (C + cp,))
        if cp:
            xv[..., C:].zero_()
        xv[..., :C].copy_(xt.permute(0, 1, 3, 4, 5, 2))
        Wx, Whp, b = self.Wx, self.Wh, self.b
        if il:
            Wx, Whp, b = _gate_interleave(Wx, f), _gate_interleave(Whp, f), _gate_interleave(b, f)
        wx = F.pad(Wx.permute(0, 2, 3, 4, 1), (0, cp, 0, 0, 0, 0, 0, 0, 0, kp))
        wh = F.pad(Whp.permute(0, 2, 3, 4, 1), (0, fp, 0, 0, 0, 0, 0, 0, 0, kp))
        bias = F.pad(b, (0, kp))
        xs = conv3d_ndhwc(xn, wx, bias, stride=(1, 1, 1), pad=(p, p, p))
        xs = xs[..., :K] if il else xs.float()[..., :K]
        osp = tuple(xs.shape[1:4])
        P = osp[0] * osp[1] * osp[2]
        M = B * P
        if il:
            # whole sequence, one launch per step: time-major gate inputs in processing order
            gxs = xs.reshape(T, M, K)
            hs = _ConvLSTM3DFusedFn.apply(gxs.contiguous(), Whp, B, osp[0], osp[1], osp[2], f, k,
                                          bool(self.return_sequences))
            if self.return_sequences:
                return hs.reshape(T, B, *osp, f).permute(1, 0, 5, 2, 3, 4).to(x.dtype)
            return hs.reshape(B, *osp, f).permute(0, 4, 1, 2, 3).to(x.dtype)
        xs = xs.reshape(B, T, P, K)
        h = c = None
        outs = []
        for t in (range(T - 1, -1, -1) if self.go_backwards else range(T)):
            gh = None
            if h is not None:
                hn = F.pad(h.reshape(B, *osp, f), (0, fp)).to(torch.bfloat16)
                gh = conv3d_ndhwc(hn, wh, None, stride=(1, 1, 1), pad=(p, p, p)).float()[..., :K].reshape(M, K)
            h, c = lstm_gates(xs[:, t].reshape(M, K), gh, c, "sigmoid", "tanh")
            outs.append(h.reshape(B, *osp, f).permute(0, 4, 1, 2, 3))
        return torch.stack(outs, 1).to(x.dtype) if self.return_sequences else outs[-1].to(x.dtype)

    def call(self, x):
        if x.is_cuda and self.k % 2 == 1:
            return self._call_native(x)
        B, T = x.shape[:2]
        p = self.k // 2
        xs = F.conv3d(x.reshape(B * T, *x.shape[2:]), self.Wx.to(x.dtype), self.b.to(x.dtype), 1, p)
        xs = xs.reshape(B, T, *xs.shape[1:])
        f = self.nb_filter
        h = x.new_zeros(B, f, *xs.shape[3:])
        c = h.clone()
        outs = []
        for t in (range(T - 1, -1, -1) if self.go_backwards else range(T)):
            g = xs[:, t] + F.conv3d(h, self.Wh.to(h.dtype), None, 1, p)
            i, fg = torch.sigmoid(g[:, :f]), torch.sigmoid(g[:, f:2 * f])
            cc, o = torch.tanh(g[:, 2 * f:3 * f]), torch.sigmoid(g[:, 3 * f:])
            c = fg * c + i * cc
            h = o * torch.tanh(c)
            outs.append(h)
        return torch.stack(outs, 1) if self.return_sequences else h
