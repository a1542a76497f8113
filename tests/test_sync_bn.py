"""SyncBN: BatchNorm statistics shared across data-parallel
ranks. Two gloo ranks each holding half a batch must reproduce single-process
BatchNorm over the whole batch — outputs, input gradients, gamma/beta gradients
(after the DP sum) and running statistics — for the Keras layer (NCHW and
channels-last) and for the fused conv+BN unit of the ResNet models."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest
import torch

from zoo.parallel.sync_bn import set_sync_bn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _collect(q, procs, n, timeout):
    """Results from n workers; fail fast (instead of waiting out the timeout) if one dies."""
    import queue
    import time
    out, t0 = {}, time.time()
    while len(out) < n:
        try:
            r, v = q.get(timeout=1.0)
            out[r] = v
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            assert not dead, "worker died with exit code %s" % dead
            assert time.time() - t0 < timeout, "workers timed out"
    return out


def _data():
    g = torch.Generator().manual_seed(7)
    return (torch.randn(8, 6, 5, 5, generator=g) * 2 + 1, torch.randn(8, 6, 5, 5, generator=g),
            torch.randn(8, 5, 5, 4, generator=g), torch.randn(8, 5, 5, 8, generator=g))


def _run(x, dy, xc, dyc, world_rank=None):
    """Keras BN (th), Keras BN (tf ordering), conv+BN unit; returns outputs/grads."""
    from zoo.pipeline.api.keras.layers import BatchNormalization
    from zoo import ops
    torch.manual_seed(0)
    out = {}
    bn = BatchNormalization(dim_ordering="th", momentum=0.1)
    bn.build((None, 6, 5, 5))
    bn.train()
    xr = x.clone().requires_grad_(True)
    y = bn.call(xr)
    y.backward(dy)
    out.update(y=y.detach(), dx=xr.grad, dg=bn.gamma.grad, db=bn.beta.grad, rm=bn.running_mean.clone(),
               rv=bn.running_var.clone())
    # fused conv -> BN -> ReLU unit (CPU reference path of conv_bn_act)
    w4 = torch.randn(8, 3, 3, 4, generator=torch.Generator().manual_seed(3)) * 0.2
    w = torch.nn.Parameter(ops.pack_weight(w4))
    gam = torch.nn.Parameter(torch.ones(8) * 1.5)
    bet = torch.nn.Parameter(torch.ones(8) * 0.1)
    rm, rv = torch.zeros(8), torch.ones(8)
    xcr = xc.clone().requires_grad_(True)
    z = ops.conv_bn_act(xcr, w, gam, bet, rm, rv, kernel=(3, 3), pad=(1, 1), relu=True, training=True)
    z.backward(dyc)
    out.update(z=z.detach(), dxc=xcr.grad, dw=w.grad, dgam=gam.grad, dbet=bet.grad, rm2=rm, rv2=rv)
    return out


def _worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import zoo.common.nncontext as nc
    nc._CTX = None
    ctx = nc.init_nncontext(backend="gloo")
    set_sync_bn(True)
    x, dy, xc, dyc = _data()
    h = 4
    sl = slice(rank * h, rank * h + h)
    # the loss of each rank is its half of the global loss: dy as is (sum loss)
    out = _run(x[sl], dy[sl], xc[sl], dyc[sl])
    # DP gradient sync sums parameter gradients over ranks
    import torch.distributed as dist
    for k in ("dg", "db", "dw", "dgam", "dbet"):
        dist.all_reduce(out[k])
    q.put((rank, {k: v.numpy().copy() for k, v in out.items()}))
    set_sync_bn(False)
    ctx.stop()


def test_sync_bn_two_ranks_match_full_batch():
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 2, 240)
    for p in procs:
        p.join(timeout=60)
    x, dy, xc, dyc = _data()
    ref = _run(x, dy, xc, dyc)
    for k in ("y", "dx", "z", "dxc"):
        got = np.concatenate([res[0][k], res[1][k]])
        np.testing.assert_allclose(got, ref[k].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
    for k in ("dg", "db", "rm", "rv", "dw", "dgam", "dbet", "rm2", "rv2"):
        np.testing.assert_allclose(res[0][k], ref[k].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)
        np.testing.assert_allclose(res[1][k], ref[k].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)


# ---- native GPU path (fused conv+BN kernels), 2 processes sharing cuda:0 over gloo ----
def _gpu_unit(xc, dyc):
    from zoo import ops
    dev = torch.device("cuda")
    w4 = torch.randn(16, 3, 3, 16, generator=torch.Generator().manual_seed(3)) * 0.1
    w = torch.nn.Parameter(ops.pack_weight(w4).to(dev))
    gam = torch.nn.Parameter(torch.full((16,), 1.5, device=dev))
    bet = torch.nn.Parameter(torch.full((16,), 0.1, device=dev))
    rm, rv = torch.zeros(16, device=dev), torch.ones(16, device=dev)
    xr = xc.to(dev, torch.bfloat16).requires_grad_(True)
    z = ops.conv_bn_act(xr, w, gam, bet, rm, rv, kernel=(3, 3), pad=(1, 1), relu=True, training=True)
    z.backward(dyc.to(dev, torch.bfloat16))
    return {"z": z.detach().float().cpu(), "dx": xr.grad.float().cpu(), "dgam": gam.grad.cpu(),
            "dbet": bet.grad.cpu(), "rm": rm.cpu(), "rv": rv.cpu()}


def _gpu_data():
    g = torch.Generator().manual_seed(11)
    return torch.randn(8, 12, 12, 16, generator=g) * 2 + 0.5, torch.randn(8, 12, 12, 16, generator=g)


def _gpu_worker(rank, world, port, q):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    import torch.distributed as dist
    import zoo.common.nncontext as nc
    nc._CTX = None
    ctx = nc.init_nncontext(backend="gloo")
    set_sync_bn(True)
    xc, dyc = _gpu_data()
    sl = slice(rank * 4, rank * 4 + 4)
    out = _gpu_unit(xc[sl], dyc[sl])
    for k in ("dgam", "dbet"):
        dist.all_reduce(out[k])
    q.put((rank, {k: v.numpy().copy() for k, v in out.items()}))
    set_sync_bn(False)
    ctx.stop()



@pytest.mark.gpu
def test_sync_bn_native_gpu_path_two_ranks(gpu):
    ctx_mp = mp.get_context("spawn")
    q = ctx_mp.Queue()
    port = _free_port()
    procs = [ctx_mp.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 2, 100)
    for p in procs:
        p.join(timeout=60)
    xc, dyc = _gpu_data()
    ref = _gpu_unit(xc, dyc)
    for k in ("z", "dx"):
        got = np.concatenate([res[0][k], res[1][k]])
        r = ref[k].numpy()
        assert np.abs(got - r).max() <= 3e-2 * np.abs(r).max(), k
    for k in ("dgam", "dbet", "rm", "rv"):
        r = ref[k].numpy()
        assert np.abs(res[0][k] - r).max() <= 2e-2 * max(np.abs(r).max(), 1.0), k
