#!/usr/bin/env python3
"""Cluster Serving quick start (docs/ClusterServingGuide, pyzoo/zoo/serving): start the
native queue server, a serving worker for a model, enqueue images / tensors with the
client's InputQueue, and read the top-N results with OutputQueue -- all in one process
here; in production ``cluster-serving queue`` / ``cluster-serving start`` run them as
separate processes, one worker per GPU."""
import argparse
import os
import sys
import tempfile
import threading

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--images", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--resnet", action="store_true", help="serve ResNet-50 (default: a tiny conv net)")
    a = ap.parse_args(argv)
    import torch
    from zoo.common.nncontext import init_nncontext
    from zoo.serving import ClusterServing, InputQueue, OutputQueue
    from zoo.serving.resp import RespServer
    init_nncontext("serving_quick_start")
    srv = RespServer("127.0.0.1", 0)
    try:
        with tempfile.TemporaryDirectory() as d:
            cfg = os.path.join(d, "config.yaml")
            size = 224 if a.resnet else 32
            with open(cfg, "w") as f:
                f.write("data:\n  src: 127.0.0.1:%d\n  image_shape: 3,%d,%d\n  filter: topN(3)\n"
                        "params:\n  batch_size: %d\n" % (srv.port, size, size, a.batch))
            if a.resnet:
                from zoo.models.image.resnet import resnet50
                model = resnet50()
            else:
                torch.manual_seed(0)
                model = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.AdaptiveAvgPool2d(1),
                                            torch.nn.Flatten(), torch.nn.Linear(8, 10), torch.nn.Softmax(-1))
            serving = ClusterServing(cfg, model=model)
            worker = threading.Thread(target=serving.run, kwargs={"max_records": a.images, "idle_timeout": 20})
            worker.start()
            inq, outq = InputQueue(cfg), OutputQueue(cfg)
            rng = np.random.default_rng(0)
            for i in range(a.images):
                inq.enqueue_image("img-%d" % i, rng.integers(0, 255, (48, 64, 3)).astype(np.uint8))
            worker.join()
            res = outq.dequeue()
            for k in sorted(res):
                print(k, res[k])
            return res
    finally:
        srv.shutdown()


if __name__ == "__main__":
    main()
