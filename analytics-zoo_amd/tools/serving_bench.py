#!/usr/bin/env python3
"""Serving benchmark (BASELINE.json config "Cluster Serving batched inference:
ResNet-50 + BERT-base, throughput + p50 latency").

  serving_bench.py model [--iters N]   InferenceModel (hipGraph replica) throughput and
                                       p50/p99 latency per batch size: ResNet-50 bf16,
                                       ResNet-50 int8, BERT-base (seq 128)
  serving_bench.py e2e [--images N]    end-to-end Cluster Serving: JPEG images through the
                                       RESP (Redis-protocol) queue -> batching worker ->
                                       GPU resize/normalize -> ResNet-50 -> top-N results
  serving_bench.py openloop            open-loop load: client processes send at FIXED offered
                                       rates (independent of responses) for --duration s each;
                                       per rate: achieved throughput, p50 / p99 service latency
                                       (send -> result written), unfinished records
  serving_bench.py suite               BASELINE config 5 in one command: ResNet-50 (JPEG records)
                                       and BERT-base (token-id tensor records), one serving worker
                                       per GPU (run it unchanged under torch.distributed.run
                                       --nproc-per-node N), the C++ open-loop load generator of
                                       csrc/runtime/serving.cpp at fractions of the measured
                                       capacity; rank 0 prints whole-node JSON per offered load

Random-init weights, synthetic inputs. Prints one JSON line per measurement.
"""
import argparse
import io
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def _pct(v, q):
    return float(np.percentile(np.asarray(v), q))


def bench_model(name, im, make_input, batches, iters):
    for bs in batches:
        x = make_input(bs)
        for _ in range(3):
            im.predict(x)
        lat = []
        t0 = time.perf_counter()
        for _ in range(iters):
            t = time.perf_counter()
            im.predict(x)
            lat.append((time.perf_counter() - t) * 1e3)
        el = time.perf_counter() - t0
        print(json.dumps({"bench": "serving-model", "model": name, "batch": bs, "throughput": round(bs * iters / el, 1),
                          "unit": "records/sec", "p50_ms": round(_pct(lat, 50), 3), "p99_ms": round(_pct(lat, 99), 3),
                          "n_gpus": 1, "data": "synthetic"}), flush=True)


def run_models(a):
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import resnet50
    from zoo.pipeline.api.keras.layers import BERT
    from zoo.pipeline.inference import InferenceModel
    init_nncontext("serving-bench")
    torch.manual_seed(0)
    rn = resnet50()
    im = InferenceModel(1).load_module(rn)
    bench_model("ResNet-50 bf16", im, lambda b: torch.randn(b, 3, 224, 224), [1, 8, 32, 128, 256], a.iters)
    im8 = InferenceModel(1).load_module(resnet50(), blas=False)
    bench_model("ResNet-50 int8", im8, lambda b: torch.randn(b, 3, 224, 224), [1, 32, 256], a.iters)
    L = 128
    bert = BERT(vocab=30522, hidden_size=768, n_block=12, n_head=12, max_position_len=512, intermediate_size=3072,
                output_all_block=False)

    class Head(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

        def forward(self, xs):
            return self.m(xs)[1]  # pooled output [B, 768]

    imb = InferenceModel(1).load_module(Head(bert))

    def bert_in(b):
        tok = torch.randint(0, 30522, (b, L))
        return [tok, torch.zeros(b, L, dtype=torch.long), torch.arange(L).repeat(b, 1), torch.ones(b, L)]
    bench_model("BERT-base seq128", imb, bert_in, [1, 8, 32, 128], a.iters)


def _producer_proc(cfg, p, n, images, jpgs, ready=None, go=None):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from zoo.serving import InputQueue
    q = InputQueue(cfg)
    if ready is not None:  # imports + connection done: the timed run starts when all are ready
        ready.put(p)
        go.wait()
    for i in range(p, images, n):
        _send(q, "im%d" % i, jpgs[i % len(jpgs)])


def _send(q, uri, payload):
    """JPEG bytes -> image record; a numpy array (BERT token ids) -> tensor record"""
    if isinstance(payload, np.ndarray):
        q.enqueue_tensor(uri, payload)
    else:
        q.enqueue_encoded(uri, payload)


class _BertTokens(torch.nn.Module):
    """Serving head for BERT-base: a [B, L] float tensor of token ids (the Cluster Serving
    tensor record format) -> pooled [B, 768] output; segment 0, positions 0..L-1, full mask."""

    def __init__(self, L=128):
        super().__init__()
        from zoo.pipeline.api.keras.layers import BERT
        self.L = L
        self.m = BERT(vocab=30522, hidden_size=768, n_block=12, n_head=12, max_position_len=512,
                      intermediate_size=3072, output_all_block=False)

    def forward(self, x):
        tok = x.long()
        b = tok.shape[0]
        pos = torch.arange(self.L, device=tok.device).repeat(b, 1)
        return self.m([tok, torch.zeros_like(tok), pos, torch.ones(b, self.L, device=tok.device)])[1]


def _jpegs(kind, seed, n=16):
    """16 distinct 256x256 JPEGs. ``noise``: uniform random pixels (the entropy decoder's worst
    case, ~60 KB each); ``natural``: photo-like content -- low-frequency colour fields, soft
    blobs and edges plus sensor-level noise, quality 90 (~2 bits / pixel, the range of ImageNet
    JPEGs)."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    out = []
    yy, xx = np.mgrid[0:256, 0:256].astype(np.float32) / 256.0
    for _ in range(n):
        if kind == "noise":
            img = rng.integers(0, 255, (256, 256, 3), dtype=np.uint8)
            q = 75
        else:
            img = np.zeros((256, 256, 3), np.float32)
            for c in range(3):
                for _ in range(4):
                    fx, fy, ph = rng.uniform(0.5, 4.0), rng.uniform(0.5, 4.0), rng.uniform(0, 6.28)
                    img[..., c] += rng.uniform(10, 40) * np.sin(6.28 * (fx * xx + fy * yy) + ph)
                img[..., c] += rng.uniform(60, 190)
            for _ in range(6):
                cx, cy, r = rng.uniform(0, 1), rng.uniform(0, 1), rng.uniform(0.03, 0.2)
                blob = np.exp(-((xx - cx) ** 2 + (yy - cy) ** 2) / (2 * r * r))
                img += blob[..., None] * rng.uniform(-80, 80, 3)
            for _ in range(3):                                   # hard edges (object boundaries)
                a_, b_, c_ = rng.uniform(-1, 1, 3)
                img += ((a_ * xx + b_ * yy + c_) > 0)[..., None] * rng.uniform(-40, 40, 3)
            img += rng.normal(0, 3.0, img.shape)
            img = np.clip(img, 0, 255).astype(np.uint8)
            q = 90
        buf = io.BytesIO()
        Image.fromarray(img).save(buf, format="JPEG", quality=q)
        out.append(buf.getvalue())
    return out


def run_e2e(a):
    from PIL import Image
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import resnet50
    from zoo.serving import ClusterServing, InputQueue, OutputQueue
    from zoo.serving.resp import RespServer
    import tempfile
    init_nncontext("serving-e2e")
    srv = RespServer("127.0.0.1", 0).start()
    jpgs = _jpegs(a.images_kind, 0)
    try:
        with tempfile.TemporaryDirectory() as d:
            cfg = os.path.join(d, "config.yaml")
            open(cfg, "w").write("data:\n  src: 127.0.0.1:%d\n  image_shape: 3,224,224\n  filter: topN(5)\n"
                                 "params:\n  batch_size: %d\n" % (srv.port, a.batch))
            bert = a.model == "bert"
            if bert:  # token-id tensor records instead of JPEGs
                jpgs = [rng.integers(0, 30522, 128).astype(np.float32) for _ in range(16)]
            s = ClusterServing(cfg, model=_BertTokens() if bert else resnet50(), device="cuda")
            model_name = "BERT-base seq128 bf16" if bert else "ResNet-50 bf16"
            data_name = "synthetic token ids [128]" if bert else "synthetic 256x256 JPEG"
            inq, outq = InputQueue(cfg), OutputQueue(cfg)
            # warm-up (graph capture for the batch shape)
            for i in range(a.batch):
                _send(inq, "warm%d" % i, jpgs[i % len(jpgs)])
            s.run(max_records=a.batch, idle_timeout=30)
            outq.dequeue()
            s.records = 0
            sent = {}

            if a.drain:  # worker-only throughput: the queue is filled before the worker starts
                for i in range(a.images):
                    _send(inq, "im%d" % i, jpgs[i % len(jpgs)])
                s.records = 0
                td = time.perf_counter()
                s.run(max_records=a.images, idle_timeout=30)
                el = time.perf_counter() - td
                got = outq.dequeue()
                print(json.dumps({"bench": "cluster-serving-drain", "model": model_name, "batch": a.batch,
                                  "images": len(got), "throughput": round(len(got) / el, 1), "unit": "records/sec",
                                  "n_gpus": 1, "data": data_name}), flush=True)
                return

            if a.client_procs:  # producers in separate processes (spawned: no GPU state in them)
                import multiprocessing as mp
                ctxmp = mp.get_context("spawn")
                ready, go = ctxmp.Queue(), ctxmp.Event()
                procs = [ctxmp.Process(target=_producer_proc,
                                       args=(cfg, p, a.client_procs, a.images, jpgs, ready, go))
                         for p in range(a.client_procs)]
                for pr in procs:
                    pr.start()
                for _ in procs:
                    ready.get(timeout=240)
                t0 = time.perf_counter()
                go.set()
                sent_q = None
                ths = []
                for i in range(a.images):
                    sent["im%d" % i] = t0   # latency measured from the run start (send times live in the children)
            else:
                ths = None

            def producer(p):
                q = inq if p == 0 else InputQueue(cfg)   # one connection per producer thread
                for i in range(p, a.images, a.producers):
                    sent["im%d" % i] = time.perf_counter()
                    _send(q, "im%d" % i, jpgs[i % len(jpgs)])
            if ths is None:
                ths = [threading.Thread(target=producer, args=(p,)) for p in range(a.producers)]
                t0 = time.perf_counter()
                for th in ths:
                    th.start()
            done = {}
            worker = threading.Thread(target=s.run, kwargs={"max_records": a.images, "idle_timeout": 30})
            worker.start()
            while len(done) < a.images and time.perf_counter() - t0 < 300:
                for k in outq.dequeue():
                    done.setdefault(k, time.perf_counter())
                time.sleep(0.002)
            worker.join()
            for th in ths:
                th.join()
            if a.client_procs:
                for pr in procs:
                    pr.join()
            el = time.perf_counter() - t0
            lat = [(done[k] - sent[k]) * 1e3 for k in done if k in sent]
            # the model alone at the same batch (same InferenceModel replica, input already on the GPU)
            xm = (torch.randint(0, 30522, (a.batch, 128), device="cuda").float() if bert
                  else torch.randn(a.batch, 3, 224, 224, device="cuda"))
            for _ in range(3):
                s.im.predict(xm)
            tm = time.perf_counter()
            for _ in range(20):
                s.im.predict(xm)
            model_tp = 20 * a.batch / (time.perf_counter() - tm)
            from zoo.serving.resp import NativeRespServer
            print(json.dumps({"bench": "cluster-serving-e2e", "model": model_name, "batch": a.batch,
                              "images": len(done), "throughput": round(len(done) / el, 1), "unit": "records/sec",
                              "p50_ms": round(_pct(lat, 50), 2), "p99_ms": round(_pct(lat, 99), 2),
                              "model_only_throughput": round(model_tp, 1),
                              "e2e_over_model": round(len(done) / el / model_tp, 3),
                              "producers": ("%d processes" % a.client_procs) if a.client_procs else a.producers,
                              "queue": "native" if isinstance(srv, NativeRespServer) else "python",
                              "n_gpus": 1, "data": data_name}), flush=True)
    finally:
        srv.shutdown()
        srv.server_close()


def _openloop_client(cfg, rate, t_start, duration, prefix, payloads, out_q):
    """Send at ``rate`` records/s from ``t_start`` (wall clock) for ``duration`` s, on a fixed
    schedule regardless of responses; report [(uri, send_wall_time)]."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from zoo.serving import InputQueue
    q = InputQueue(cfg)
    sent = []
    n = int(rate * duration)
    while time.time() < t_start:
        time.sleep(0.001)
    for i in range(n):
        due = t_start + i / rate
        now = time.time()
        if due > now:
            time.sleep(due - now)
        uri = "%s-%d" % (prefix, i)
        ts = time.time()
        _send(q, uri, payloads[i % len(payloads)])
        sent.append((uri, ts))
    out_q.put(sent)


def run_openloop(a):
    import multiprocessing as mp
    import tempfile
    from PIL import Image
    from zoo.common.nncontext import init_nncontext
    from zoo.models.image.resnet import resnet50
    from zoo.serving import ClusterServing, InputQueue
    from zoo.serving.resp import RespServer
    init_nncontext("serving-openloop")
    srv = RespServer("127.0.0.1", 0).start()
    jpgs = _jpegs(a.images_kind, 0)
    done = {}
    try:
        with tempfile.TemporaryDirectory() as d:
            cfg = os.path.join(d, "config.yaml")
            open(cfg, "w").write("data:\n  src: 127.0.0.1:%d\n  image_shape: 3,224,224\n  filter: topN(5)\n"
                                 "params:\n  batch_size: %d\n" % (srv.port, a.batch))
            s = ClusterServing(cfg, model=resnet50(), device="cuda")

            def hook(uris, t):
                for u in uris:
                    done[u] = t
            s.finish_hook = hook
            inq = InputQueue(cfg)
            # warm-up: every bucket shape captured, then the worker keeps running
            for i in range(4 * a.batch):
                _send(inq, "warm%d" % i, jpgs[i % len(jpgs)])
            worker = threading.Thread(target=s.run, kwargs={"idle_timeout": None}, daemon=True)
            worker.start()
            t = time.time()
            while sum(1 for k in done if k.startswith("warm")) < 4 * a.batch and time.time() - t < 120:
                time.sleep(0.01)
            for bsz in (8, 16, 32, 64, 128, 256, 512):   # capture the remaining buckets
                if bsz > a.batch:
                    break
                x = torch.zeros(bsz, 3, 224, 224, device="cuda")
                s.im.predict(x)
            # capacity: a pre-filled queue drained by the worker
            n_cap = 20 * a.batch
            t0 = time.time()
            for i in range(n_cap):
                _send(inq, "cap%d" % i, jpgs[i % len(jpgs)])
            while sum(1 for k in done if k.startswith("cap")) < n_cap and time.time() - t0 < 120:
                time.sleep(0.005)
            cap_done = [done[k] for k in done if k.startswith("cap")]
            capacity = len(cap_done) / max(1e-9, max(cap_done) - t0) if cap_done else 0.0
            print(json.dumps({"bench": "cluster-serving-capacity", "batch": a.batch, "records": len(cap_done),
                              "closed_loop_throughput": round(capacity, 1), "note": "includes enqueue from one "
                              "client thread"}), flush=True)
            rates = [float(r) for r in a.rates.split(",")] if a.rates else \
                [round(f * capacity) for f in (0.1, 0.25, 0.5, 0.7, 0.85, 1.0, 1.2)]
            ctx = mp.get_context("spawn")
            for ri, rate in enumerate(rates):
                if rate <= 0:
                    continue
                nproc = max(1, int(np.ceil(rate / a.client_rate)))
                outq = ctx.Queue()
                t_start = time.time() + 3.0
                procs = [ctx.Process(target=_openloop_client,
                                     args=(cfg, rate / nproc, t_start, a.duration, "r%dp%d" % (ri, p), jpgs, outq))
                         for p in range(nproc)]
                for p in procs:
                    p.start()
                sent = []
                for _ in procs:
                    sent += outq.get(timeout=a.duration + 240)
                for p in procs:
                    p.join()
                grace = time.time() + 10.0
                while time.time() < grace and any(u not in done for u, _ in sent[-200:]):
                    time.sleep(0.01)
                warm = t_start + 1.0
                win = [(u, ts) for u, ts in sent if ts >= warm]
                lat = [(done[u] - ts) * 1e3 for u, ts in win if u in done]
                fin = [done[u] for u, _ in sent if u in done and warm <= done[u] <= t_start + a.duration]
                achieved = len(fin) / max(1e-9, a.duration - 1.0)
                offered = len(sent) / a.duration
                print(json.dumps({"bench": "cluster-serving-openloop", "model": "ResNet-50 bf16",
                                  "batch_cap": a.batch, "offered_rate": round(offered, 1),
                                  "achieved_throughput": round(achieved, 1), "unit": "records/sec",
                                  "p50_ms": round(_pct(lat, 50), 2) if lat else None,
                                  "p99_ms": round(_pct(lat, 99), 2) if lat else None,
                                  "unfinished": sum(1 for u, _ in sent if u not in done),
                                  "client_procs": nproc, "duration_s": a.duration, "n_gpus": 1,
                                  "decode": "gpu-jpeg" if os.environ.get("ZOO_SERVING_GPU_JPEG", "1") != "0"
                                  else "cpu", "data": "synthetic 256x256 JPEG (%s)" % a.images_kind}), flush=True)
                time.sleep(1.0)
            s.stop()
    finally:
        srv.shutdown()
        srv.server_close()


def run_dist(a):
    """One serving worker per GPU, launched unchanged by torch.distributed.run on 1..8 GPUs:
    every rank owns an in-process native queue, pre-fills it with --images JPEG records and
    drains it through its own worker (C++ Huffman decode threads + GPU IDCT / resize + ResNet-50
    + topN); ranks start together (barrier) and rank 0 prints the whole-node throughput."""
    import tempfile
    import torch.distributed as dist
    from PIL import Image
    from zoo.models.image.resnet import resnet50
    from zoo.serving import ClusterServing, InputQueue
    from zoo.serving.resp import RespServer
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")
    # each rank gets its share of the node's CPU threads for the entropy decoder
    os.environ.setdefault("ZOO_SERVING_JPEG_THREADS", str(max(2, (os.cpu_count() or 16) // max(1, world) // 2)))
    from zoo.common.nncontext import init_nncontext
    init_nncontext("serving-dist")
    srv = RespServer("127.0.0.1", 0).start()
    jpgs = _jpegs(a.images_kind, rank)
    try:
        with tempfile.TemporaryDirectory() as d:
            cfg = os.path.join(d, "config.yaml")
            open(cfg, "w").write("data:\n  src: 127.0.0.1:%d\n  image_shape: 3,224,224\n  filter: topN(5)\n"
                                 "params:\n  batch_size: %d\n" % (srv.port, a.batch))
            s = ClusterServing(cfg, model=resnet50(), device="cuda:%d" % local)
            inq = InputQueue(cfg)
            for i in range(2 * a.batch):
                _send(inq, "warm%d" % i, jpgs[i % len(jpgs)])
            s.run(max_records=2 * a.batch, idle_timeout=60)
            s.records = 0
            for i in range(a.images):
                _send(inq, "im%d" % i, jpgs[i % len(jpgs)])
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            s.run(max_records=a.images, idle_timeout=60)
            el = time.perf_counter() - t0
            tp = torch.tensor([s.records / el, el], dtype=torch.float64)
            if world > 1:
                allv = [torch.zeros_like(tp) for _ in range(world)]
                dist.all_gather(allv, tp)
            else:
                allv = [tp]
            if rank == 0:
                total = sum(float(v[0]) for v in allv)
                print(json.dumps({"bench": "cluster-serving-dist-drain", "model": "ResNet-50 bf16", "batch": a.batch,
                                  "images_per_gpu": a.images, "throughput": round(total, 1), "unit": "records/sec",
                                  "per_gpu": [round(float(v[0]), 1) for v in allv], "n_gpus": world,
                                  "decode": "gpu-jpeg" if os.environ.get("ZOO_SERVING_GPU_JPEG", "1") != "0"
                                  else "cpu", "data": "synthetic 256x256 JPEG (%s)" % a.images_kind}), flush=True)
    finally:
        srv.shutdown()
        srv.server_close()
        if world > 1:
            dist.destroy_process_group()


class _GcWatch:
    """Python GC pauses (gc.callbacks) -- a collector pass on the serving thread stalls every
    batch behind it, which shows in the latency tail."""

    def __init__(self):
        import gc
        self.t0, self.pauses = None, []
        gc.callbacks.append(self._cb)

    def _cb(self, phase, info):
        if phase == "start":
            self.t0 = time.perf_counter()
        elif self.t0 is not None:
            self.pauses.append((info.get("generation", -1), (time.perf_counter() - self.t0) * 1e3))
            self.t0 = None

    def take(self):
        p, self.pauses = self.pauses, []
        return {"n": len(p), "gen2": sum(1 for g, _ in p if g == 2),
                "max_ms": round(max((d for _, d in p), default=0.0), 2),
                "total_ms": round(sum(d for _, d in p), 1)}


def _slowest(trace, frac=0.01):
    """Stage breakdown (mean ms) of the slowest ``frac`` of the batches by read-to-written time,
    next to the median batch: which stage the tail stalls in."""
    if not trace:
        return None
    tr = sorted(trace, key=lambda r: r["total"])
    k = max(1, int(round(len(tr) * frac)))
    keys = [c for c in tr[0] if c != "n"]

    def mean(rows):
        return {c: round(sum(r[c] for r in rows) / len(rows), 2) for c in keys + ["n"]}
    return {"batches": len(tr), "slowest": k, "slowest_mean_ms": mean(tr[-k:]),
            "median_batch_ms": mean([tr[len(tr) // 2]]), "max_total_ms": round(tr[-1]["total"], 2)}


def _suite_model(name, a, rank, world, local, gather):
    """One model through the suite on this rank: capacity (drain), model-only, open-loop loads."""
    import base64
    import tempfile
    from zoo.models.image.resnet import resnet50
    from zoo.serving import ClusterServing, InputQueue
    from zoo.serving.resp import RespServer
    bert = name == "bert"
    srv = RespServer("127.0.0.1", 0).start()
    out = []
    try:
        with tempfile.TemporaryDirectory() as d:
            cfg = os.path.join(d, "config.yaml")
            shape = "3,224,224" if not bert else "128"
            open(cfg, "w").write("data:\n  src: 127.0.0.1:%d\n  image_shape: %s\n  filter: topN(5)\n"
                                 "params:\n  batch_size: %d\n" % (srv.port, shape, a.batch))
            model = _BertTokens() if bert else resnet50()
            s = ClusterServing(cfg, model=model, device="cuda:%d" % local)
            inq = InputQueue(cfg)
            if bert:
                rng = np.random.default_rng(rank)
                toks = [rng.integers(0, 30522, (128,)).astype(np.float32) for _ in range(16)]
                raw = toks
                payloads = [base64.b64encode(t.tobytes()).decode() for t in toks]
                kind, pshape = "tensor", "128"
            else:
                raw = _jpegs(a.images_kind, rank)
                payloads = [base64.b64encode(j).decode() for j in raw]
                kind, pshape = "image", ""
            # warm-up: every batch bucket captured
            for i in range(4 * a.batch):
                _send(inq, "warm%d" % i, raw[i % len(raw)])
            s.run(max_records=4 * a.batch, idle_timeout=120)
            for bsz in (8, 16, 32, 64, 128, 256, 512):
                if bsz > a.batch:
                    break
                x = (torch.randint(0, 30522, (bsz, 128), device="cuda:%d" % local).float() if bert
                     else torch.zeros(bsz, 3, 224, 224, device="cuda:%d" % local))
                s.im.predict(x)
                # the look-ahead path's pinned output ring is per output shape: allocate it now, not
                # in the first open-loop batch of that size (a pinned allocation stalls for ms)
                for _ in range(3):
                    s.im.predict_async(x).result()
            # capacity: a pre-filled queue drained by the worker (the worker alone)
            n_cap = a.images
            for i in range(n_cap):
                _send(inq, "cap%d" % i, raw[i % len(raw)])
            s.records = 0
            for k in s.stage_time:
                s.stage_time[k] = 0 if k == "batches" else 0.0
            gather(None)
            t0 = time.perf_counter()
            s.run(max_records=n_cap, idle_timeout=60)
            cap = s.records / (time.perf_counter() - t0)
            nbat = max(1, s.stage_time["batches"])
            stages = {k: round(v * 1e3 / nbat, 3) for k, v in s.stage_time.items() if k != "batches"}
            # the ceiling: the same InferenceModel replica at the serving batch, input already on
            # the GPU, driven exactly the way the worker drives it -- back-to-back predict_async
            # graph replays with one batch of look-ahead (batch i+1 enqueued before batch i's
            # D2H result is read) -- over 200 batches. (Rounds <= 5 divided by 10 synchronous
            # predict calls, each with its own host sync: a low ceiling; still reported.)
            xm = (torch.randint(0, 30522, (a.batch, 128), device="cuda:%d" % local).float() if bert
                  else torch.randn(a.batch, 3, 224, 224, device="cuda:%d" % local))
            for _ in range(5):
                s.im.predict_async(xm).result()
            torch.cuda.synchronize()
            nb_model = 200
            tm = time.perf_counter()
            prev = None
            for _ in range(nb_model):
                h = s.im.predict_async(xm)
                if prev is not None:
                    prev.result()
                prev = h
            prev.result()
            model_tp = nb_model * a.batch / (time.perf_counter() - tm)
            tm = time.perf_counter()
            for _ in range(10):
                s.im.predict(xm)
            torch.cuda.synchronize()
            model_sync_tp = 10 * a.batch / (time.perf_counter() - tm)
            caps = gather([cap, model_tp, model_sync_tp])
            node_cap = sum(c[0] for c in caps)
            node_model = sum(c[1] for c in caps)
            node_model_sync = sum(c[2] for c in caps)
            model_name = "BERT-base seq128 bf16" if bert else "ResNet-50 bf16"
            if rank == 0:
                print(json.dumps({"bench": "cluster-serving-capacity", "model": model_name, "batch_cap": a.batch,
                                  "n_gpus": world, "drain_throughput": round(node_cap, 1),
                                  "model_only_throughput": round(node_model, 1),
                                  "model_only_def": "200 back-to-back predict_async replays, one batch look-ahead",
                                  "model_only_sync_throughput": round(node_model_sync, 1),
                                  "drain_over_model": round(node_cap / max(node_model, 1e-9), 3),
                                  "rank0_host_ms_per_batch": stages, "batches": nbat,
                                  "overlap": os.environ.get("ZOO_SERVING_ASYNC", "1") != "0",
                                  "unit": "records/sec"}), flush=True)
            # open loop: the C++ load generator on this rank's store, the worker in a thread
            srv.store.track(True)
            worker = threading.Thread(target=s.run, kwargs={"idle_timeout": None}, daemon=True)
            worker.start()
            fracs = [float(f) for f in a.fractions.split(",")]
            gcw = _GcWatch()
            for fi, f in enumerate(fracs):
                rate = f * cap
                gather(None)
                gcw.take()
                s.batch_trace = []
                st = srv.store.loadgen("image_stream", kind, payloads, pshape, rate, a.duration, a.lg_threads,
                                       "r%d-%d-%s" % (rank, fi, name), 1.0, 15.0, bool(a.tcp))
                allst = gather([st["offered_rate"], st["achieved_throughput"], st["p50_ms"], st["p99_ms"],
                                st["unfinished"], st["p90_ms"]])
                if rank == 0:
                    rec = {"bench": "cluster-serving-suite", "model": model_name, "n_gpus": world,
                           "load_fraction_of_capacity": f,
                           "offered_rate": round(sum(v[0] for v in allst), 1),
                           "achieved_throughput": round(sum(v[1] for v in allst), 1), "unit": "records/sec",
                           "p50_ms": round(max(v[2] for v in allst), 2), "p90_ms": round(max(v[5] for v in allst), 2),
                           "p99_ms": round(max(v[3] for v in allst), 2),
                           "unfinished": int(sum(v[4] for v in allst)),
                           "achieved_over_model": round(sum(v[1] for v in allst) / max(node_model, 1e-9), 3),
                           "rank0_gc": gcw.take(),
                           "rank0_slowest_batches": _slowest(s.batch_trace),
                           "latency_note": "send -> result written; worst rank's percentile",
                           "client": "C++ open-loop generator, %d threads per GPU, %s" % (
                               a.lg_threads, "RESP over TCP" if a.tcp else "in-process XADD"),
                           "batch_cap": a.batch, "duration_s": a.duration,
                           "data": ("synthetic token ids [128]" if bert else
                                    "synthetic 256x256 JPEG (%s)" % a.images_kind)}
                    out.append(rec)
                    print(json.dumps(rec), flush=True)
                time.sleep(0.5)
            s.stop()
            worker.join(timeout=30)
    finally:
        srv.shutdown()
        srv.server_close()
    return out


def run_suite(a):
    """ResNet-50 and BERT-base serving, one worker per GPU (torch.distributed.run ranks)."""
    import torch.distributed as dist
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")
    os.environ.setdefault("ZOO_SERVING_JPEG_THREADS", str(max(2, min(16, (os.cpu_count() or 16) // max(1, world) // 2))))
    from zoo.common.nncontext import init_nncontext
    init_nncontext("serving-suite")

    def gather(vals):
        """barrier (vals None) or all-gather of a small float list"""
        if world == 1:
            return [vals] if vals is not None else None
        if vals is None:
            dist.barrier()
            return None
        t = torch.tensor([float(v) for v in vals], dtype=torch.float64)
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        return [v.tolist() for v in allv]

    results = []
    try:
        for name in a.models.split(","):
            results += _suite_model(name, a, rank, world, local, gather)
    finally:
        if world > 1:
            dist.destroy_process_group()
    if rank == 0 and a.out:
        with open(a.out, "w") as f:
            json.dump(results, f, indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["model", "e2e", "openloop", "dist", "suite"])
    ap.add_argument("--models", default="resnet50,bert", help="suite: models to serve")
    ap.add_argument("--fractions", default="0.25,0.5,0.7,0.85,1.0,1.2",
                    help="suite: offered loads as fractions of the measured drain capacity")
    ap.add_argument("--lg-threads", type=int, default=4, help="suite: C++ load-generator threads per GPU")
    ap.add_argument("--tcp", action="store_true", help="suite: load generator over RESP/TCP (else in-process)")
    ap.add_argument("--out", default="", help="suite: also write the records to this JSON file")
    ap.add_argument("--rates", default="", help="openloop: comma-separated offered rates (default: fractions "
                    "of the measured capacity)")
    ap.add_argument("--duration", type=float, default=8.0, help="openloop: seconds per offered rate")
    ap.add_argument("--client-rate", type=float, default=1500.0, help="openloop: records/s per client process")
    ap.add_argument("--images-kind", default="natural", choices=["natural", "noise"],
                    help="synthetic JPEG content: photo-like (default) or uniform noise (decoder worst case)")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--images", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--producers", type=int, default=4)
    ap.add_argument("--client-procs", type=int, default=0, help="producers in N separate processes")
    ap.add_argument("--drain", action="store_true", help="prefill the queue, time the worker alone")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert"],
                    help="e2e: ResNet-50 on JPEG records or BERT-base on token-id tensor records")
    a = ap.parse_args()
    {"model": run_models, "e2e": run_e2e, "openloop": run_openloop, "dist": run_dist, "suite": run_suite}[a.mode](a)


if __name__ == "__main__":
    main()
