"""hipGraph-captured training over several input shapes (one graph per shape, interleaved with
eager warm-up steps of the next shape) against eager training: the per-step workspace memset
must cover what every captured graph dirtied (BN statistics accumulators)."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(model, shapes, hip_graph, gpu):
    from zoo.ops import native, softmax_cross_entropy
    from zoo.pipeline.api.keras.optimizers import SGD
    from zoo.pipeline.engine import TrainingEngine
    eng = TrainingEngine(model, softmax_cross_entropy, SGD(learningrate=0.02, momentum=0.9), hip_graph=hip_graph)
    g = torch.Generator(device=gpu)
    g.manual_seed(7)
    data = {s: (torch.randn(8, 3, s, s, device=gpu, generator=g), torch.randint(0, 10, (8,), device=gpu, generator=g))
            for s in sorted(set(shapes))}
    native().set_deterministic(True)
    try:
        losses = [float(eng.train_step(*data[s]).float().item()) for s in shapes]
    finally:
        native().set_deterministic(False)
    return losses, eng


def test_graph_three_shapes_match_eager(gpu):
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import resnet18
    init_nncontext("graph-shapes")
    torch.manual_seed(0)
    m = resnet18(num_classes=10)
    shapes = [64, 64, 64, 64, 32, 32, 32, 96, 96, 96, 96, 32, 64, 96, 32, 96, 64]
    eager, _ = _run(copy.deepcopy(m), shapes, False, gpu)
    graph, eng = _run(copy.deepcopy(m), shapes, True, gpu)
    assert eng.hip_graph and len(eng._graphs) == 3
    for i, (a, b) in enumerate(zip(eager, graph)):
        assert abs(a - b) < 2e-3 * max(1.0, abs(a)), (i, eager, graph)
