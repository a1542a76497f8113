#!/usr/bin/env python3
"""Which framework-level ops launch the non-native ("glue") GPU kernels of a training step:
torch.profiler with CUDA activity over a few engine steps, aten ops ranked by the device time of
the kernels they launch, with input shapes; zoo:: kernels (hand-written HIP) are reported as one
line. Models: wnd (Wide&Deep ml-20m shape), ssd (SSD-300 VGG), ncf, resnet (bench.py ResNet-50 b256), bert (BERT-base b128 s128).

  python tools/glue_report.py --model wnd [--steps 3]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def _engine(name):
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.optimizers import SGD, Adam
    from zoo.pipeline.engine import TrainingEngine
    ctx = init_nncontext("glue")
    if name == "wnd":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import wnd_bench
        from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
        model, xs, y = wnd_bench.build(8192, ctx.device)
        eng = TrainingEngine(model, ClassNLLCriterion(log_prob_as_input=False, zero_based_label=False), Adam(lr=1e-3))
        return eng, xs, y
    if name == "ncf":
        from zoo.models.recommendation.neuralcf import NeuralCF
        from zoo.pipeline.api.keras.objectives import SparseCategoricalCrossEntropy
        m = NeuralCF(138493, 26744, 5, 20, 20, (40, 20, 10), True, 20)
        x = torch.stack([torch.randint(1, 138494, (65536,)), torch.randint(1, 26745, (65536,))], 1).to(ctx.device)
        y = torch.randint(0, 5, (65536,), device=ctx.device)
        return TrainingEngine(m, SparseCategoricalCrossEntropy(), Adam(lr=1e-3)), x, y
    if name == "ssd":
        from zoo.models.image.objectdetection.ssd import SSD, MultiBoxLoss
        m = SSD(21)
        crit = MultiBoxLoss(21)
        pri = m.priors

        def loss_fn(out, targets):
            return crit(out[0], out[1], pri.to(out[0].device), targets)
        x = torch.randn(16, 3, 300, 300, device=ctx.device)
        g = torch.Generator().manual_seed(0)
        gt = []
        for _ in range(16):
            xy = torch.rand(3, 2, generator=g) * 0.6
            wh = torch.rand(3, 2, generator=g) * 0.3 + 0.05
            lab = torch.randint(1, 21, (3, 1), generator=g).float()
            gt.append(torch.cat([lab, xy, xy + wh], 1).to(ctx.device))
        return TrainingEngine(m, loss_fn, SGD(learningrate=1e-3, momentum=0.9)), x, gt
    if name == "bert":
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from bert_train import _Classifier
        from zoo.ops import softmax_cross_entropy
        from zoo.pipeline.api.keras.layers import BERT
        from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
        bert = BERT(vocab=30522, hidden_size=768, n_block=12, n_head=12, max_position_len=512,
                    intermediate_size=3072, output_all_block=False)
        B, L = 128, 128
        dev = ctx.device
        xs = [torch.randint(0, 30522, (B, L), device=dev), torch.zeros(B, L, dtype=torch.long, device=dev),
              torch.arange(L, device=dev).repeat(B, 1), torch.ones(B, L, device=dev)]
        y = torch.randint(0, 2, (B,), device=dev)
        return TrainingEngine(_Classifier(bert), softmax_cross_entropy, AdamWeightDecay(lr=2e-5)), xs, y
    if name == "resnet":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
        import bench
        eng, (x, y), _, _ = bench.build_resnet50(ctx, 256)
        return eng, x, y
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="wnd", choices=["wnd", "ssd", "ncf", "resnet", "bert"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--rows", type=int, default=30)
    a = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile
    eng, x, y = _engine(a.model)
    for _ in range(3):
        eng.train_step(x, y)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as p:
        for _ in range(a.steps):
            eng.train_step(x, y)
        torch.cuda.synchronize()
    kern = [e for e in p.events() if e.device_type.name == "CUDA"]
    tot = sum(e.device_time for e in kern) or 1.0
    zoo_t = sum(e.device_time for e in kern if "zoo::" in e.name)
    print("device time per step %.3f ms, zoo:: share %.1f%%" % (tot / a.steps / 1e3, 100.0 * zoo_t / tot))
    rows = []
    for ev in p.key_averages(group_by_input_shape=True):
        if "zoo::" in ev.key or ev.key.startswith("_") or ev.self_device_time_total <= 0:
            continue            # hand-written kernels and the autograd Functions wrapping them
        rows.append((ev.self_device_time_total / a.steps, ev.count / a.steps, ev.key, str(ev.input_shapes)[:90]))
    rows.sort(reverse=True)
    print("| us/step | calls/step | op | input shapes |")
    print("|---|---|---|---|")
    for t, c, k, s in rows[:a.rows]:
        print("| %.1f | %.1f | `%s` | %s |" % (t, c, k, s))


if __name__ == "__main__":
    main()
