"""Tensor parallelism: a column->row parallel MLP over two
gloo ranks equals the unsplit MLP — outputs, input gradients and (re-assembled)
weight gradients."""
import multiprocessing as mp
import os
import socket

import numpy as np
import torch
import torch.nn.functional as F


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params():
    g = torch.Generator().manual_seed(5)
    return (torch.randn(16, 8, generator=g) * 0.3, torch.randn(16, generator=g) * 0.1,
            torch.randn(8, 16, generator=g) * 0.3, torch.randn(8, generator=g) * 0.1,
            torch.randn(6, 8, generator=g), torch.randn(6, 8, generator=g))


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import zoo.common.nncontext as nc
    nc._CTX = None
    ctx = nc.init_nncontext(backend="gloo")
    from zoo.parallel.tensor_parallel import ColumnParallelLinear, ParallelMLP
    w1, b1, w2, b2, x, dy = _params()
    mlp = ParallelMLP(8, 16, activation="relu", fc1=(w1, b1), fc2=(w2, b2))
    xr = x.clone().requires_grad_(True)
    y = mlp(xr)
    y.backward(dy)
    col = ColumnParallelLinear(8, 16, gather_output=True, init_weight=w1, init_bias=b1)
    yc = col(x)
    q.put((rank, {"y": y.detach().numpy(), "dx": xr.grad.numpy(), "dw1": mlp.fc1.weight.grad.numpy(),
                  "dw2": mlp.fc2.weight.grad.numpy(), "db2": mlp.fc2.bias.grad.numpy(), "yc": yc.detach().numpy()}))
    ctx.stop()


def test_parallel_mlp_two_ranks_matches_dense():
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    w1, b1, w2, b2, x, dy = _params()
    w1r, w2r = w1.clone().requires_grad_(True), w2.clone().requires_grad_(True)
    b2r = b2.clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y = F.linear(F.relu(F.linear(xr, w1r, b1)), w2r, b2r)
    y.backward(dy)
    for r in (0, 1):
        np.testing.assert_allclose(res[r]["y"], y.detach().numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(res[r]["dx"], xr.grad.numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(res[r]["db2"], b2r.grad.numpy(), rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(res[r]["yc"], F.linear(x, w1, b1).numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(np.concatenate([res[0]["dw1"], res[1]["dw1"]], 0), w1r.grad.numpy(), rtol=1e-5,
                               atol=1e-5)
    np.testing.assert_allclose(np.concatenate([res[0]["dw2"], res[1]["dw2"]], 1), w2r.grad.numpy(), rtol=1e-5,
                               atol=1e-5)
