#!/usr/bin/env python3
"""Wide&Deep training throughput on one GPU, ml-20m-shape synthetic data
(reference: Zs/models/recommendation/WideAndDeep.scala:113-144 and the pyzoo
wide_n_deep example's column setup, scaled to ml-20m: 138,493 users x 26,744 items).

The wide part is a SparseEmbedding sum-bag over the hashed base+cross columns
(native embedding-bag kernel, csrc/kernels/sparse.hip), the deep part indicator
columns + user/item embeddings + an MLP. One step = forward, NLL loss, backward,
fused Adam over the flat parameter buffer.

  python tools/wnd_bench.py [--batch 8192] [--steps 30] [--warmup 5] [--hip-graph]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402


def build(batch, device, hidden=(1024, 512, 256), seed=0):
    from zoo.models.recommendation.wide_and_deep import ColumnFeatureInfo, WideAndDeep
    users, items = 138493, 26744
    ci = ColumnFeatureInfo(wide_base_cols=["occupation", "gender"], wide_base_dims=[21, 3],
                           wide_cross_cols=["age-gender", "user-genre"], wide_cross_dims=[100, 100000],
                           indicator_cols=["genres", "gender"], indicator_dims=[20, 3],
                           embed_cols=["userId", "itemId"], embed_in_dims=[users, items], embed_out_dims=[64, 64],
                           continuous_cols=["age"])
    torch.manual_seed(seed)
    model = WideAndDeep(5, ci, hidden_layers=hidden)
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    offs = torch.tensor([0, 21, 24, 124], device=device)
    hi = torch.tensor([21, 3, 100, 100000], device=device)
    wide = (torch.rand(batch, 4, device=device, generator=g) * hi).long() + offs
    ind = torch.zeros(batch, 23, device=device)
    ind[torch.arange(batch, device=device), torch.randint(0, 20, (batch,), device=device, generator=g)] = 1
    ind[torch.arange(batch, device=device), 20 + torch.randint(0, 3, (batch,), device=device, generator=g)] = 1
    emb = torch.stack([torch.randint(1, users + 1, (batch,), device=device, generator=g),
                       torch.randint(1, items + 1, (batch,), device=device, generator=g)], 1).float()
    cont = torch.rand(batch, 1, device=device, generator=g)
    y = torch.randint(1, 6, (batch,), device=device, generator=g)
    return model, [wide.float(), ind, emb, cont], y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--hip-graph", action="store_true")
    a = ap.parse_args()
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.objectives import ClassNLLCriterion
    from zoo.pipeline.api.keras.optimizers import Adam
    from zoo.pipeline.engine import TrainingEngine
    ctx = init_nncontext("wnd_bench")
    model, xs, y = build(a.batch, ctx.device)
    eng = TrainingEngine(model, ClassNLLCriterion(log_prob_as_input=False, zero_based_label=False), Adam(lr=1e-3),
                         hip_graph=a.hip_graph)
    first = None
    for _ in range(a.warmup):
        l0 = eng.train_step(xs, y)
        first = l0 if first is None else first
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = eng.train_step(xs, y)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"model": "WideAndDeep(ml-20m shape)", "batch": a.batch, "steps": a.steps,
                      "ms_per_step": round(dt / a.steps * 1e3, 3), "records_per_sec": round(a.batch * a.steps / dt, 1),
                      "hip_graph": a.hip_graph, "first_loss": round(float(first), 4),
                      "final_loss": round(float(loss), 4)}), flush=True)


if __name__ == "__main__":
    main()
