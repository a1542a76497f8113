"""Persistent recurrent-cell kernels (csrc/kernels/rnn.hip) vs a plain fp32
PyTorch time loop of the same Keras-1 cells (LSTM.scala / GRU.scala /
SimpleRNN.scala semantics: gate order i,f,c,o and z,r,h)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def _act(x, name):
    if name == "tanh":
        return torch.tanh(x)
    if name == "sigmoid":
        return torch.sigmoid(x)
    if name == "hard_sigmoid":
        return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)
    if name == "relu":
        return torch.relu(x)
    return x


def _reference(x, W, b, U, cell, act, iact, h0, c0):
    B, T, _ = x.shape
    H = U.shape[1]
    xw = x @ W.t() + b
    h = h0 if h0 is not None else x.new_zeros(B, H)
    c = c0 if c0 is not None else x.new_zeros(B, H)
    outs = []
    for t in range(T):
        g = xw[:, t]
        if cell == "rnn":
            h = _act(g + h @ U.t(), act)
        elif cell == "lstm":
            g = g + h @ U.t()
            i, f = _act(g[:, :H], iact), _act(g[:, H:2 * H], iact)
            cc, o = _act(g[:, 2 * H:3 * H], act), _act(g[:, 3 * H:], iact)
            c = f * c + i * cc
            h = o * _act(c, act)
        else:
            uh = h @ U[:2 * H].t()
            z = _act(g[:, :H] + uh[:, :H], iact)
            r = _act(g[:, H:2 * H] + uh[:, H:], iact)
            hh = _act(g[:, 2 * H:] + (r * h) @ U[2 * H:].t(), act)
            h = z * h + (1 - z) * hh
        outs.append(h)
    return torch.stack(outs, 1), c


CASES = [("lstm", 20, "tanh", "hard_sigmoid"), ("lstm", 64, "tanh", "sigmoid"), ("lstm", 128, "tanh", "hard_sigmoid"),
         ("lstm", 200, "tanh", "sigmoid"), ("gru", 48, "tanh", "hard_sigmoid"), ("gru", 128, "tanh", "sigmoid"),
         ("gru", 256, "tanh", "hard_sigmoid"), ("rnn", 32, "tanh", None), ("rnn", 100, "relu", None),
         ("rnn", 256, "tanh", None)]


@pytest.mark.parametrize("cell,H,act,iact", CASES)
def test_rnn_kernel_matches_fp32_loop(gpu, cell, H, act, iact):
    from zoo.ops import rnn as R
    torch.manual_seed(0)
    G = {"rnn": 1, "lstm": 4, "gru": 3}[cell]
    B, T, D = 37, 9, 24
    x = torch.randn(B, T, D, device=gpu)
    W = (torch.randn(G * H, D, device=gpu) / D ** 0.5)
    b = torch.randn(G * H, device=gpu) * 0.1
    U = (torch.randn(G * H, H, device=gpu) / H ** 0.5)
    h0 = torch.randn(B, H, device=gpu) * 0.5
    c0 = torch.randn(B, H, device=gpu) * 0.5 if cell == "lstm" else None
    leaves = [t.requires_grad_(True) for t in (x, W, b, U, h0)] + ([c0.requires_grad_(True)] if c0 is not None else [])
    hseq, hT, cT = R.recurrent(x, W, b, U, cell, act, iact, h0=h0, c0=c0)
    refs = [t.detach().clone().requires_grad_(True) for t in leaves]
    rh, rc = _reference(*refs[:4], cell, act, iact, refs[4], refs[5] if c0 is not None else None)
    assert hseq.shape == (B, T, H)
    assert nrel(hseq, rh) < 2e-2, nrel(hseq, rh)
    assert torch.equal(hT, hseq[:, -1])
    gh = torch.randn_like(rh)
    loss = (hseq * gh).sum()
    rloss = (rh * gh).sum()
    if cell == "lstm":
        gc = torch.randn_like(rc)
        assert nrel(cT, rc) < 2e-2
        loss = loss + (cT * gc).sum()
        rloss = rloss + (rc * gc).sum()
    loss.backward()
    rloss.backward()
    # relu recurrences amplify bf16 rounding through activation-mask flips
    tol = 1e-1 if act == "relu" else 4e-2
    for name, a, r in zip(["x", "W", "b", "U", "h0", "c0"], leaves, refs):
        err = nrel(a.grad, r.grad)
        assert err < tol, (name, err)


def test_rnn_go_backwards_and_no_grad(gpu):
    from zoo.ops import rnn as R
    B, T, D, H = 16, 5, 8, 32
    x = torch.randn(B, T, D, device=gpu)
    W, b, U = torch.randn(4 * H, D, device=gpu) * 0.3, torch.zeros(4 * H, device=gpu), torch.randn(4 * H, H, device=gpu) * 0.2
    with torch.no_grad():
        hs, _, _ = R.recurrent(x, W, b, U, "lstm", go_backwards=True)
        rh, _ = _reference(x.flip(1), W, b, U, "lstm", "tanh", "hard_sigmoid", None, None)
    assert nrel(hs, rh) < 2e-2


@pytest.mark.parametrize("name", ["LSTM", "GRU", "SimpleRNN"])
def test_keras_recurrent_layer_uses_fused_kernel(gpu, name):
    """The Keras layer on the GPU takes the fused path and matches its own CPU loop."""
    from zoo.pipeline.api.keras import layers as L
    from zoo.pipeline.api.keras.models import Sequential
    torch.manual_seed(0)
    m = Sequential()
    m.add(getattr(L, name)(48, return_sequences=True, input_shape=(7, 16)))
    x = torch.randn(20, 7, 16)
    y_cpu = m(x)
    m = m.to(gpu)
    layer = m.layers[0] if hasattr(m, "layers") else None
    y_gpu = m(x.to(gpu))
    assert nrel(y_gpu.cpu(), y_cpu) < 2e-2
    if layer is not None:
        assert layer._fused_ok(x.to(gpu))
