#!/usr/bin/env python3
"""Synchronous parameter server with actors (pyzoo/zoo/examples/ray/parameter_server/
sync_parameter_server.py) on the framework's RayContext (a local process-pool emulation of
Ray: remote functions, actors, get/put/wait): workers compute gradients of a linear model
on their data shard, the parameter-server actor averages and applies them."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import _common  # noqa: E402,F401
import numpy as np  # noqa: E402


class ParameterServer:
    def __init__(self, dim, lr):
        self.w = np.zeros(dim, np.float64)
        self.lr = lr

    def apply_gradients(self, *grads):
        self.w -= self.lr * np.mean(grads, axis=0)
        return self.w

    def get_weights(self):
        return self.w


class Worker:
    def __init__(self, seed, dim, n):
        rng = np.random.default_rng(seed)
        self.x = rng.standard_normal((n, dim))
        true_w = np.arange(1, dim + 1, dtype=np.float64)
        self.y = self.x @ true_w

    def compute_gradient(self, w):
        err = self.x @ w - self.y
        return self.x.T @ err / len(self.y)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--workers", type=int, default=2)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--dim", type=int, default=4)
    a = ap.parse_args(argv)
    from zoo.ray import RayContext, get, remote
    ctx = RayContext(sc=None, object_store_memory="100m", num_ray_nodes=1, ray_node_cpu_cores=a.workers)
    ctx.init()
    try:
        ps = remote(ParameterServer).remote(a.dim, 0.1)
        workers = [remote(Worker).remote(i, a.dim, 200) for i in range(a.workers)]
        w = get(ps.get_weights.remote())
        for _ in range(a.iters):
            grads = get([wk.compute_gradient.remote(w) for wk in workers])
            w = get(ps.apply_gradients.remote(*grads))
        print("learned weights:", np.round(w, 3))
        return w
    finally:
        ctx.stop()


if __name__ == "__main__":
    main()
