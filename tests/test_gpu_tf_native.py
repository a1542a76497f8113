"""Native bf16 execution of TF graph Conv2D / MatMul (tf_graph.py, TFNet.use_native_kernels)
against the fp32 PyTorch execution of the same nodes (synthetic graphs: no fixtures)."""
import pytest
import torch


@pytest.mark.gpu
def test_tf_conv2d_native_matches_fp32(gpu):
    from zoo.pipeline.api.net.tf_graph import Node, TFGraph, _conv2d
    g = TFGraph([], {})
    g.native_bf16 = True
    torch.manual_seed(0)
    x = torch.randn(2, 9, 9, 3)
    w = torch.randn(3, 3, 3, 16) * 0.2
    for pad, st in (("SAME", 1), ("SAME", 2), ("VALID", 2)):
        n = Node("c", "Conv2D", [], [], {"strides": [1, st, st, 1], "padding": pad, "data_format": "NHWC"})
        ref = _conv2d(n, x, w)
        out = _conv2d(n, x.to(gpu), w.to(gpu), g=g).float().cpu()
        assert out.shape == ref.shape
        assert (out - ref).abs().max().item() < 5e-2 * ref.abs().max().item()
    assert g.native_calls == 3


@pytest.mark.gpu
def test_tf_graph_matmul_native_matches_fp32(gpu):
    from zoo.pipeline.api.net.tf_graph import Node, TFGraph
    torch.manual_seed(1)
    w = torch.randn(64, 32) * 0.1
    nodes = [Node("x", "Placeholder", [], [], {}), Node("w", "Const", [], [], {}),
             Node("mm", "MatMul", ["x", "w"], [], {"transpose_a": False, "transpose_b": False})]
    x = torch.randn(16, 64)
    ref = TFGraph(nodes, {}).run({"x:0": x, "w:0": w}, ["mm:0"])[0]
    g = TFGraph(nodes, {})
    g.native_bf16 = True
    out = g.run({"x:0": x.to(gpu), "w:0": w.to(gpu)}, ["mm:0"])[0].float().cpu()
    assert g.native_calls == 1
    assert (out - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
