#!/usr/bin/env python3
"""BERT-base fine-tuning step throughput (random init, sequence classification head,
AdamWeightDecay, bf16 compute with fp32 master weights, dropout on), for profiling:
  python analytics-zoo_amd/tools/bert_train.py [--batch 32] [--seq 128] [--iters 20]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402


class _Classifier(nn.Module):
    def __init__(self, bert, n_cls=2):
        super().__init__()
        self.bert = bert
        self.fc = nn.Linear(768, n_cls)

    def forward(self, xs):
        return self.fc(self.bert(xs)[1].float())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--graph", action="store_true",
                    help="capture forward + backward + in-backward optimizer as one hipGraph per step")
    ap.add_argument("--i2-tile", type=int, default=0,
                    help="force one igemm2 tile for every linear (igemm2.hip I2Tile; 0 = per-shape choice)")
    ap.add_argument("--i2-192", type=int, default=-1,
                    help="256x192 igemm2 tiles: 0 off, 1 forward-type epilogues, 2 all (-1: default)")
    a = ap.parse_args()
    from zoo.common.nncontext import init_nncontext
    from zoo.pipeline.api.keras.layers import BERT
    from zoo.pipeline.api.keras.optimizers import AdamWeightDecay
    from zoo.pipeline.engine import TrainingEngine
    from zoo.ops import softmax_cross_entropy
    init_nncontext("bert-train")
    if a.i2_tile or a.i2_192 >= 0:
        from zoo.ops import native
        native().igemm2_set(-1, a.i2_tile)
        native().igemm2_w192_set(a.i2_192)
    dev = torch.device("cuda")
    bert = BERT(vocab=30522, hidden_size=768, n_block=12, n_head=12, max_position_len=512, intermediate_size=3072,
                output_all_block=False)
    eng = TrainingEngine(_Classifier(bert), softmax_cross_entropy, AdamWeightDecay(lr=2e-5), hip_graph=a.graph)
    B, L = a.batch, a.seq
    xs = [torch.randint(0, 30522, (B, L), device=dev), torch.zeros(B, L, dtype=torch.long, device=dev),
          torch.arange(L, device=dev).repeat(B, 1), torch.ones(B, L, device=dev)]
    y = torch.randint(0, 2, (B,), device=dev)
    for _ in range(3):
        eng.train_step(xs, y)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(a.iters):
        h0 = time.perf_counter()
        loss = eng.train_step(xs, y)
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    replay_ms = None
    if eng._graphs:
        # host cost of the bare hipGraph launch (no staging, no optimizer tail)
        g = next(iter(eng._graphs.values()))[0]
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        replay_ms = (time.perf_counter() - h0) / 5 * 1e3
        torch.cuda.synchronize()
    # issue_ms_per_step: the host time of one step issued onto an IDLE device (synchronised
    # before each probe step), i.e. pure issue cost with no blocking on a full queue or a ring slot.
    # ms_per_step well above it means the step is device-bound; close to it means host-bound.
    issue = []
    for _ in range(5):
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        eng.train_step(xs, y)
        issue.append(time.perf_counter() - h0)
    torch.cuda.synchronize()
    issue_ms = sorted(issue)[len(issue) // 2] * 1e3
    # host_ms_per_step: time the Python / launch side spends in train_step inside the pipelined loop
    # (issue time PLUS any time blocked on the device); kept for comparison with earlier logs
    print('{"bench": "bert-base-finetune-train", "batch": %d, "seq": %d, "ms_per_step": %.3f, "seq_per_s": %.1f, '
          '"tokens_per_s": %.0f, "loss": %.4f, "host_ms_per_step": %.3f, "hip_graph": %s, "graphs": %d, "graph_replay_host_ms": %s, '
          '"issue_ms_per_step": %.3f}'
          % (B, L, dt * 1e3, B / dt, B * L / dt, float(loss), host / a.iters * 1e3, "true" if eng.hip_graph else "false",
             len(eng._graphs), "null" if replay_ms is None else "%.3f" % replay_ms, issue_ms))


if __name__ == "__main__":
    main()
