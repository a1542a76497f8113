"""Native pointwise kernels (csrc/kernels/pointwise.hip) vs their PyTorch fp32 definitions:
activations fwd+bwd, dropout statistics and mask replay, one-pass objectives (loss and
gradient), threshold AUC, SSD box decoding; plus the Keras layers that route to them."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("name", ["relu", "relu6", "elu", "selu", "gelu", "gelu_tanh", "sigmoid", "hard_sigmoid",
                                  "tanh", "softplus", "softsign", "swish", "log_sigmoid", "tanh_shrink",
                                  "exponential", "leaky_relu"])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_activation_fwd_bwd(gpu, name, dt):
    from zoo.ops.pointwise import act_ref, activation
    torch.manual_seed(0)
    x = (torch.randn(3, 1000, device=gpu) * 3).to(dt)
    xr = x.float().clone().requires_grad_(True)
    alpha = 0.01 if name == "leaky_relu" else 1.0
    ref = act_ref(xr, name, alpha)
    xn = x.clone().requires_grad_(True)
    out = activation(xn, name)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert rel(out, ref) < tol
    g = torch.randn_like(ref)
    ref.backward(g)
    out.backward(g.to(dt))
    assert rel(xn.grad, xr.grad) < (1e-4 if dt == torch.float32 else 2e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_dropout_statistics_and_backward_mask(gpu, dt):
    from zoo.ops.pointwise import dropout
    x = torch.ones(1 << 20, device=gpu, dtype=dt, requires_grad=True)
    y = dropout(x, 0.3, True)
    kept = (y != 0).float().mean().item()
    assert abs(kept - 0.7) < 0.005
    assert torch.allclose(y[y != 0].float(), torch.full_like(y[y != 0].float(), 1 / 0.7), rtol=1e-2)
    y.sum().backward()
    assert torch.equal((x.grad != 0), (y != 0))          # the backward regenerates the same mask
    assert torch.equal(dropout(x, 0.3, False), x)


@pytest.mark.parametrize("kind", ["mse", "mae", "smooth_l1", "bce", "bce_logits", "hinge", "squared_hinge",
                                  "poisson", "mape", "msle", "kld"])
def test_elementwise_loss_and_grad(gpu, kind):
    from zoo.ops.pointwise import elementwise_loss
    torch.manual_seed(1)
    n = (64, 37)
    if kind in ("bce", "poisson", "msle", "kld"):
        p = torch.rand(n, device=gpu) * 0.9 + 0.05
        t = torch.rand(n, device=gpu)
    elif kind in ("hinge", "squared_hinge"):
        p = torch.randn(n, device=gpu)
        t = torch.randint(0, 2, n, device=gpu).float() * 2 - 1
    else:
        p = torch.randn(n, device=gpu)
        t = torch.randn(n, device=gpu) + 0.5
    pr = p.clone().requires_grad_(True)
    w = 1.0 / p.numel() if kind != "kld" else 1.0 / p.shape[0]
    ref = {"mse": lambda: F.mse_loss(pr, t), "mae": lambda: F.l1_loss(pr, t),
           "smooth_l1": lambda: F.smooth_l1_loss(pr, t, beta=1.0), "bce": lambda: F.binary_cross_entropy(pr, t),
           "bce_logits": lambda: F.binary_cross_entropy_with_logits(pr, t),
           "hinge": lambda: torch.clamp(1 - t * pr, min=0).mean(),
           "squared_hinge": lambda: (torch.clamp(1 - t * pr, min=0) ** 2).mean(),
           "poisson": lambda: (pr - t * torch.log(pr + 1e-7)).mean(),
           "mape": lambda: 100 * ((pr - t).abs() / t.abs().clamp_min(1e-7)).mean(),
           "msle": lambda: ((torch.log(pr.clamp_min(1e-7) + 1) - torch.log(t.clamp_min(1e-7) + 1)) ** 2).mean(),
           "kld": lambda: (t.clamp(1e-7, 1) * torch.log(t.clamp(1e-7, 1) / pr.clamp(1e-7, 1))).sum(-1).mean()}[kind]()
    pn = p.clone().requires_grad_(True)
    out = elementwise_loss(pn, t, kind, w)
    assert abs(out.item() - ref.item()) <= 1e-4 * max(1.0, abs(ref.item()))
    ref.backward()
    (out * 2.0).backward()
    assert rel(pn.grad, 2.0 * pr.grad) < 1e-4


def test_auc_and_keras_auc_metric(gpu):
    from zoo.ops.pointwise import auc
    from sklearn.metrics import roc_auc_score
    torch.manual_seed(2)
    lab = (torch.rand(20000, device=gpu) > 0.6).float()
    score = (torch.rand(20000, device=gpu) * 0.7 + lab * 0.3).clamp(0, 1)
    a = auc(score, lab, nbins=2000)
    ref = roc_auc_score(lab.cpu().numpy(), score.cpu().numpy())
    assert abs(a - ref) < 2e-3
    from zoo.pipeline.api.keras.metrics import AUC
    m = AUC(200)
    acc_g = [0.0] * m.n_acc
    m.update(acc_g, score, lab)
    acc_c = [0.0] * m.n_acc
    m.update(acc_c, score.cpu(), lab.cpu())
    assert abs(m.result(acc_g) - m.result(acc_c)) < 1e-3


def test_box_decode_matches_reference(gpu):
    from zoo.ops.pointwise import box_decode
    torch.manual_seed(3)
    pri = torch.rand(500, 4, device=gpu) * 0.5 + 0.1
    loc = torch.randn(2, 500, 4, device=gpu) * 0.5
    out = box_decode(loc, pri)
    ref = box_decode(loc.cpu(), pri.cpu())
    assert torch.allclose(out.cpu(), ref, atol=1e-5)


def test_keras_layers_route_to_native(gpu):
    from zoo.pipeline.api.keras.layers import Activation, Dropout
    from zoo.pipeline.api.keras.objectives import MeanSquaredError
    x = torch.randn(8, 16, device=gpu, requires_grad=True)
    a = Activation("gelu")
    a._ensure_built((None, 16))
    y = a(x)
    assert torch.allclose(y, F.gelu(x), atol=1e-5)
    d = Dropout(0.5)
    d._ensure_built((None, 16))
    d.train()
    z = d(y)
    assert ((z == 0).float().mean() - 0.5).abs() < 0.2
    loss = MeanSquaredError()(z, torch.zeros_like(z))
    loss.backward()
    assert x.grad is not None and torch.isfinite(x.grad).all()
