"""Round-3 GPU regressions.

* eval-mode BatchNorm folding must follow the weights and running statistics that the
  engine's fused optimizer and the native BN kernels rewrite through raw pointers
  (the fold cache keyed only on ``_version`` froze validation at the first
  evaluation's weights).
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def test_eval_bn_fold_tracks_training(gpu):
    from zoo.models.image.resnet import resnet18
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine

    torch.manual_seed(0)
    model = resnet18(num_classes=10)
    cpu_twin = copy.deepcopy(model)
    eng = TrainingEngine(model, softmax_cross_entropy, SGD(learningrate=0.05, momentum=0.9))
    x = torch.randn(16, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (16,), device=gpu)
    for _ in range(2):
        eng.train_step(x, y)
    o1 = eng.predict([x])[0]
    for _ in range(3):
        eng.train_step(x, y)
    o2 = eng.predict([x])[0]
    torch.cuda.synchronize()
    assert (o2 - o1).abs().max().item() > 1e-3, "evaluation did not see the new weights / statistics"
    # unfused fp32 reference of the same (trained) state on the CPU path
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    cpu_twin.load_state_dict(sd)
    cpu_twin.eval()
    with torch.no_grad():
        ref = cpu_twin(x.cpu())
    assert _rel(o2.cpu(), ref) < 5e-2
