"""Embedding scatter-add backward: zoo native kernel vs torch index_add_ (fp32 grad table).
Shapes: BERT-base word / position / token-type tables (16384 tokens x 768) and the NCF
ml-20m user / item tables (65536 ids)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    from zoo.ops import native
    dev = torch.device("cuda:0")
    cases = [("bert_word", 16384, 768, 30522, "rand"), ("bert_pos", 16384, 768, 512, "pos"),
             ("bert_type", 16384, 768, 2, "rand"), ("ncf_user", 65536, 64, 138493, "rand"),
             ("ncf_item", 65536, 64, 26744, "rand")]
    for name, n, D, V, pat in cases:
        ids = (torch.arange(n, device=dev) % 128) if pat == "pos" else torch.randint(0, V, (n,), device=dev)
        dout = torch.randn(n, D, device=dev)
        g = torch.zeros(V, D, device=dev)
        us = timeit(lambda: native().embedding_bwd(dout, ids, g, -1, 1.0))
        ut = timeit(lambda: g.index_add_(0, ids, dout))
        print(json.dumps({"case": name, "n": n, "D": D, "V": V, "zoo_us": round(us, 1), "torch_index_add_us": round(ut, 1)}))


if __name__ == "__main__":
    main()
