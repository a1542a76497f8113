"""Recurrent cells (SimpleRNN / LSTM / GRU) on the persistent HIP kernels
(csrc/kernels/rnn.hip).

Reference: Zs/pipeline/api/keras/layers/{LSTM,GRU,SimpleRNN}.scala and the
unrolled time loop of InternalRecurrent.scala:80-140. Here:

* the input projection of every time step is ONE MFMA GEMM (``ops.linear``
  over [B*T, D]) producing ``xw`` [B, T, G*H] with the bias folded in;
* the recurrence is ONE kernel launch for the whole sequence (forward) and
  one for BPTT (backward); it returns d(xw), from which autograd of
  ``ops.linear`` produces dW, db and dx;
* dU = sum_t dgates_t^T . h_{t-1} is one plain library GEMM over [B*T].

Hidden sizes are padded to 32/64/128/256 by zero-padding each gate block of
W, b and U (padded units stay exactly zero and never feed real units, so the
result is identical); larger layers use the per-step path in
``keras/layers/recurrent.py``.
"""
import torch
import torch.nn.functional as F

from zoo.ops._native import native

ACT_CODES = {None: 0, "linear": 0, "tanh": 1, "sigmoid": 2, "hard_sigmoid": 3, "relu": 4}
# "gru": Keras / BigDL GRU (candidate over (r * h) . U_h); "gru_ra": torch.nn.GRU / GRUCell
# (reset applied after the recurrent GEMM: n = tanh(xn + r * (U_n h + b_hn)))
CELL_CODES = {"rnn": 0, "lstm": 1, "gru": 2, "gru_ra": 3}
N_GATES = {0: 1, 1: 4, 2: 3, 3: 3}
_SIZES = (32, 64, 128, 256)


def padded_hidden(h):
    for s in _SIZES:
        if h <= s:
            return s
    return None


def supported(x, hidden, *acts):
    return (x.is_cuda and x.dim() == 3 and padded_hidden(hidden) is not None
            and all(isinstance(a, str) or a is None for a in acts) and all(a in ACT_CODES for a in acts))


class _RnnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xw, U, h0, c0, cell, act, iact, bhn=None):
        ub = U.detach().to(torch.bfloat16).contiguous()
        # gates / cell states are only kept when a backward pass can follow
        save = any(ctx.needs_input_grad[:4]) or (bhn is not None and ctx.needs_input_grad[7])
        bh = None if bhn is None else bhn.detach().float().contiguous()
        hseq, cT, cseq, gates = native().rnn_fwd(xw, ub, h0, c0, cell, act, iact, save, bh)
        if save:
            ctx.save_for_backward(U, h0, c0, hseq, cseq, gates, bh)
        ctx.cfg = (cell, act, iact)
        if cT is None:
            cT = hseq.new_zeros(0)
        return hseq, cT

    @staticmethod
    def backward(ctx, dhseq, dcT):
        U, h0, c0, hseq, cseq, gates, bh = ctx.saved_tensors
        cell, act, iact = ctx.cfg
        G = N_GATES[cell]
        Hp = U.shape[1]
        B, T = hseq.shape[:2]
        ut = U.detach().t().contiguous().to(torch.bfloat16)
        dh = None if dhseq is None else dhseq.float().contiguous()
        dc = dcT.float().contiguous() if (cell == 1 and dcT is not None and dcT.numel()) else None
        dgates, dh0, dc0, dgn = native().rnn_bwd(dh, dc, ut, hseq, cseq, gates, h0, c0, cell, act, iact)
        dU = dbhn = None
        if ctx.needs_input_grad[1]:
            first = h0.unsqueeze(1) if h0 is not None else hseq.new_zeros(B, 1, Hp)
            hprev = torch.cat([first, hseq[:, :-1]], 1).reshape(-1, Hp)
            dg = dgates.reshape(-1, G * Hp)
            if cell == 3:
                # reset-after GRU: every gate's recurrent input is h_{t-1}; the candidate's
                # recurrent gradient is d(U_n h + b_hn) (dgn), not d(xn). dU on the native
                # weight-gradient GEMM (wgrad256.hip)
                dgu = torch.cat([dg[:, :2 * Hp], dgn.reshape(-1, Hp)], 1).to(torch.bfloat16).contiguous()
                dU = torch.zeros(3 * Hp, Hp, device=dg.device, dtype=torch.float32)
                native().linear_wgrad(dgu, hprev.to(torch.bfloat16).contiguous(), dU)
            elif cell == 2:  # GRU: the candidate's recurrent input is r * h_{t-1}
                r = gates.reshape(-1, 3 * Hp)[:, Hp:2 * Hp]
                dU = torch.cat([dg[:, :2 * Hp].t() @ hprev, dg[:, 2 * Hp:].t() @ (r * hprev)], 0)
            else:
                dU = dg.t() @ hprev
            dU = dU.to(U.dtype)
        if cell == 3 and bh is not None and ctx.needs_input_grad[7]:
            dbhn = dgn.reshape(-1, Hp).sum(0)
        return (dgates, dU, dh0 if ctx.needs_input_grad[2] else None,
                dc0 if (cell == 1 and ctx.needs_input_grad[3]) else None, None, None, None, dbhn)


def _pad_gates(t, G, H, Hp, cols=False):
    """Zero-pad each of the G gate blocks (rows) of t from H to Hp; with
    ``cols`` the hidden (column) dim of U is padded as well."""
    if Hp == H:
        return t
    if t.dim() == 1:
        return F.pad(t.view(G, H), (0, Hp - H)).reshape(G * Hp)
    D = t.shape[1]
    v = t.view(G, H, D)
    v = F.pad(v, (0, Hp - H if cols else 0, 0, Hp - H))
    return v.reshape(G * Hp, v.shape[-1])


def _pad_state(s, H, Hp):
    if s is None:
        return None
    s = s.float()
    if Hp != H:
        s = F.pad(s, (0, Hp - H))
    return s.contiguous()


def recurrent(x, W, b, U, cell, act="tanh", inner_act="hard_sigmoid", h0=None, c0=None, go_backwards=False,
              linear=None, bhn=None):
    """Run a whole recurrent layer on the GPU.

    x [B, T, D]; W [G*H, D]; b [G*H]; U [G*H, H] (Keras gate order; "gru_ra": z, r, n with
    ``bhn`` [H] the candidate's recurrent bias).
    Returns (hseq [B, T, H], h_T [B, H], c_T [B, H] or None), in processing
    order (``go_backwards`` processes the sequence back to front)."""
    from zoo.ops.conv import linear as _linear
    linear = linear or _linear
    code = CELL_CODES[cell]
    G = N_GATES[code]
    B, T, D = x.shape
    H = U.shape[1]
    Hp = padded_hidden(H)
    Wp, bp, Up = _pad_gates(W, G, H, Hp), _pad_gates(b, G, H, Hp), _pad_gates(U, G, H, Hp, cols=True)
    xs = x.flip(1) if go_backwards else x
    xw = linear(xs.reshape(B * T, D), Wp, bp).reshape(B, T, G * Hp).float().contiguous()
    bh = None
    if code == 3 and bhn is not None:
        bh = bhn.float() if Hp == H else F.pad(bhn.float(), (0, Hp - H))
    hseq, cT = _RnnFn.apply(xw, Up, _pad_state(h0, H, Hp), _pad_state(c0, H, Hp) if code == 1 else None, code,
                            ACT_CODES[act], ACT_CODES[inner_act], bh)
    if Hp != H:
        hseq = hseq[..., :H]
        if code == 1:
            cT = cT[:, :H]
    return hseq, hseq[:, -1], (cT if code == 1 else None)
