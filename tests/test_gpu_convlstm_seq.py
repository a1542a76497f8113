"""Whole-sequence ConvLSTM2D (recurrent.py _ConvLSTMSeqFn: recurrent conv + fused step kernel
per step, fused BPTT) against the fp32 PyTorch reference of the same layer (F.conv2d, the
layer's own CPU path): output, input gradient and both weight gradients, with and without
return_sequences / go_backwards. Reference: InternalConvLSTM2D.scala."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-12))


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("rseq,back", [(True, False), (False, False), (True, True)])
def test_convlstm2d_sequence_path_matches_fp32(gpu, rseq, back, fused, monkeypatch):
    """fused: one launch per step (_ConvLSTMFusedFn, convlstm.hip, gate-interleaved weights);
    otherwise the recurrent conv + step kernel sequence (_ConvLSTMSeqFn)."""
    from zoo.pipeline.api.keras.layers import recurrent as R
    monkeypatch.setattr(R, "_CONVLSTM_FUSED", fused)
    used = []
    orig_f, orig_s = R._ConvLSTMFusedFn.apply, R._ConvLSTMSeqFn.apply
    monkeypatch.setattr(R._ConvLSTMFusedFn, "apply", lambda *a: (used.append("fused"), orig_f(*a))[1])
    monkeypatch.setattr(R._ConvLSTMSeqFn, "apply", lambda *a: (used.append("seq"), orig_s(*a))[1])
    torch.manual_seed(0)
    T, B, C, H, W, f = 6, 2, 8, 10, 12, 16
    layer = R.ConvLSTM2D(f, 3, 3, return_sequences=rseq, go_backwards=back, input_shape=(T, C, H, W))
    layer._ensure_built((None, T, C, H, W))
    ref = copy.deepcopy(layer)
    x = torch.randn(B, T, C, H, W)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    layer = layer.to(gpu)
    assert R._CONVLSTM_SEQ
    xg = x.to(gpu).requires_grad_(True)
    y = layer(xg)
    assert y.shape == yr.shape
    (y.float() * g.to(gpu)).sum().backward()
    assert rel(y, yr) < 3e-2
    assert rel(xg.grad, xr.grad) < 5e-2
    assert rel(layer.Wh.grad, ref.Wh.grad) < 5e-2
    assert rel(layer.Wx.grad, ref.Wx.grad) < 5e-2
    assert rel(layer.b.grad, ref.b.grad) < 5e-2
    assert used == ["fused" if fused else "seq"], used


def test_convlstm2d_fused_odd_filters_and_wide_channels(gpu, monkeypatch):
    """The fused step at F = 6 (24 gate rows: a partial MFMA row block; 8-channel padded history)
    with a 5x3 kernel, against the fp32 reference."""
    from zoo.pipeline.api.keras.layers import recurrent as R
    monkeypatch.setattr(R, "_CONVLSTM_FUSED", True)
    torch.manual_seed(1)
    T, B, C, H, W, f = 4, 3, 5, 7, 9, 6
    layer = R.ConvLSTM2D(f, 5, 3, return_sequences=True, input_shape=(T, C, H, W))
    layer._ensure_built((None, T, C, H, W))
    ref = copy.deepcopy(layer)
    x = torch.randn(B, T, C, H, W)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    g = torch.randn_like(yr)
    (yr * g).sum().backward()
    layer = layer.to(gpu)
    xg = x.to(gpu).requires_grad_(True)
    y = layer(xg)
    (y.float() * g.to(gpu)).sum().backward()
    assert rel(y, yr) < 3e-2
    assert rel(xg.grad, xr.grad) < 5e-2
    assert rel(layer.Wh.grad, ref.Wh.grad) < 5e-2
    assert rel(layer.Wx.grad, ref.Wx.grad) < 5e-2


@pytest.mark.parametrize("B,sp,f,pers", [(2, (32, 32, 32), 32, 0), (2, (32, 32, 32), 32, 1),
                                         (2, (32, 32, 32), 32, 2), (1, (41, 40, 40), 32, 1),
                                         (1, (41, 40, 40), 32, 2), (1, (41, 40, 40), 24, 1),
                                         (1, (32, 32, 32), 32, 1), (2, (32, 32, 32), 32, 5),
                                         (2, (32, 32, 32), 32, 10)])
def test_convlstm3d_large_volume_two_blocks_per_wave(gpu, monkeypatch, B, sp, f, pers):
    """ConvLSTM3D over >= 65536 pixels per step against the per-step loop of the same layer on the
    GPU (recurrent 3-D conv + gate kernel per step): output, input and recurrent-weight gradients.
    pers 0: the one-tile-per-workgroup step kernels with two 16-pixel blocks per wave (MJ = 2);
    pers 1: the persistent K-split kernels (all rows, the reduction in two launches whose weights fit
    LDS, fp32 partial sums between them); pers 2: the persistent row-group kernel (2 row groups whose
    weights fit LDS). 41 x 40 x 40 leaves a partial last tile, 24 filters partial row blocks;
    1 x 32^3 = 32768 pixels is the K-split path's lower bound (there the forward is K-split too; at
    64k+ pixels it runs the row-group kernel unless pers 5 = 1 | 4 forces the forward K-split; the
    row-group forward has the channel-blocked epilogue unless pers 10 = 2 | 8)."""
    from zoo.ops._kern import native
    from zoo.pipeline.api.keras.layers import recurrent as R
    torch.manual_seed(4)
    T, C = 3, 8
    layer = R.ConvLSTM3D(f, 3, return_sequences=True, input_shape=(T, C) + sp)
    layer._ensure_built((None, T, C) + sp)
    layer = layer.to(gpu)
    x = torch.randn((B, T, C) + sp, device=gpu)
    outs = []
    native().convlstm_pers_set(pers)
    try:
        for fused in (False, True):
            monkeypatch.setattr(R, "_CONVLSTM_FUSED", fused)
            xg = x.clone().requires_grad_(True)
            layer.zero_grad(set_to_none=True)
            y = layer(xg)
            y.float().square().mean().backward()
            outs.append((y.detach().float(), xg.grad.detach(), layer.Wh.grad.detach().clone()))
    finally:
        native().convlstm_pers_set(1)
    (y0, dx0, dw0), (y1, dx1, dw1) = outs
    assert rel(y1, y0) < 5e-3
    assert rel(dx1, dx0) < 3e-2
    assert rel(dw1, dw0) < 1e-2
