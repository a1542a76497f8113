"""NNEstimator on the GPU learns (VERDICT r5 "do this" #3): ResNet-50 trained through
NNEstimator.fit -> FeatureSet -> pinned uint8 NHWC batches -> copy stream -> the stem's fused
uint8 normalisation (the bench.py --input featureset path, NNEstimator.scala:382-470) on a
LEARNABLE synthetic task: the label is the quadrant of the image that carries a bright square.
The mean loss of the last 10 iterations must be at least 30 % below the first 10."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _task(n, size, rng):
    imgs = rng.integers(0, 96, size=(n, size, size, 3), dtype=np.uint8)
    labels = rng.integers(0, 4, size=n)
    h = size // 2
    for i, lab in enumerate(labels):
        r0, c0 = (lab // 2) * h, (lab % 2) * h
        imgs[i, r0 + h // 4:r0 + 3 * h // 4, c0 + h // 4:c0 + 3 * h // 4, :] = 230
    return imgs, labels


def test_nnestimator_resnet50_learns_through_featureset(gpu):
    import pandas as pd
    from zoo.common.nncontext import init_nncontext
    from zoo.common.triggers import MaxIteration
    from zoo.feature.common import Lambda
    from zoo.models.image.resnet import resnet50
    from zoo.ops import softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.nnframes.nn_classifier import NNEstimator
    init_nncontext("nnestimator-learn")
    torch.manual_seed(0)
    rng = np.random.default_rng(7)
    iters, bs = 50, 32
    imgs, labels = _task(iters * bs, 64, rng)
    df = pd.DataFrame({"features": list(imgs), "label": labels})
    model = resnet50(num_classes=4, zero_init_residual=True)
    est = NNEstimator(model, softmax_cross_entropy, Lambda(lambda v: v), Lambda(lambda v: np.int64(v)))
    est.setBatchSize(bs).setOptimMethod(SGD(learningrate=0.05, momentum=0.9)).setEndWhen(MaxIteration(iters))
    losses = []

    def track(eng, state):
        # the device loss of this iteration (a log_every flush has already moved it to the host)
        losses.append(eng._pending_loss[-1][1] if eng._pending_loss else torch.tensor(state["Loss"]))
    est._train_callbacks = (track,)
    est.fit(df)
    vals = [float(v.float().item()) for v in losses]
    assert len(vals) == iters
    first, last = np.mean(vals[:10]), np.mean(vals[-10:])
    assert last <= 0.7 * first, (first, last, vals)
    # the model really consumed the uint8 NHWC wire format on the device
    assert est.engine.device.type == "cuda"
