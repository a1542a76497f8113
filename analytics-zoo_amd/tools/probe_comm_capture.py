#!/usr/bin/env python3
"""Probe: can the C++ RCCL comm layer's collectives be captured into a hipGraph on a one-rank
communicator? Prints one line per collective: captured+replayed OK or the failure."""
import faulthandler
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
faulthandler.enable()
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    from zoo.common.nncontext import init_nncontext
    from zoo.parallel.comm import NativeComm
    init_nncontext("probe")
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    c = NativeComm(None)
    s = torch.cuda.Stream()
    a = torch.arange(4096, device="cuda", dtype=torch.float32)
    b = torch.empty_like(a)
    ops = {"all_reduce": lambda: c.all_reduce(a),
           "all_gather": lambda: c.all_gather(b, a),
           "all_to_all": lambda: c.all_to_all(b, a),
           "reduce_scatter": lambda: c.reduce_scatter(b, a)}
    for name, fn in ops.items():
        if which not in ("all", name):
            continue
        print("capturing", name, flush=True)
        with torch.cuda.stream(s):
            fn()                      # eager once
        s.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        g.replay()
        torch.cuda.synchronize()
        print(name, "captured and replayed ok", flush=True)
    c.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
