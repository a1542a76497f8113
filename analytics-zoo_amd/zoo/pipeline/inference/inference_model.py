"""InferenceModel — thread-safe, replica-pooled predictor.

Reference: Zs/pipeline/inference/InferenceModel.scala:30-830 (a
LinkedBlockingQueue of ``concurrentNum`` weight-sharing model copies;
``retrieveModel`` 784-805 takes one — blocking, or cloning a new one when
auto-scaling — and ``predict`` offers it back), FloatModel.scala:31-89,
InferenceModelFactory.scala:23-204, Python Py/pipeline/inference/inference_model.py:24-223.

MI355X design: a replica is NOT a copy of the weights. All replicas share
one bf16/fp32 parameter set resident in HBM; a replica owns a HIP stream,
pinned host staging buffers and, per input shape, a captured hipGraph
(``torch.cuda.CUDAGraph`` is hipGraph on ROCm) of the whole forward pass —
so a request is: H2D copy into the graph's static input, one graph launch,
D2H copy, all on the replica's stream. ``concurrent_num`` replicas let that
many host threads keep requests in flight on separate streams
(SURVEY.md §2.14 P10). Without a GPU the same pool runs eagerly on CPU.
"""
import logging
import queue
import threading
import time
import weakref

import numpy as np
import torch

log = logging.getLogger("zoo.inference")


def _tensor(t):
    t = t if torch.is_tensor(t) else torch.as_tensor(np.asarray(t))
    return t.float() if t.dtype == torch.float64 else t


def _as_tensors(inputs):
    if isinstance(inputs, (list, tuple)):
        return [_tensor(t) for t in inputs], True
    return [_tensor(inputs)], False


class _Replica:
    def __init__(self, owner, idx):
        self.owner = owner
        self.idx = idx
        dev = owner.device
        self.stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        # a private memory pool: graphs of different replicas replay concurrently,
        # so their static buffers must never alias
        self.pool = torch.cuda.graph_pool_handle() if dev.type == "cuda" else None
        self.graphs = {}
        self.host_rings, self.host_idx, self.slot_events = {}, {}, {}
        self.slot_owner = {}   # (key, slot) -> weakref of the _Pending whose result lives in the slot

    RING = 3

    def _forward(self, xs):
        m = self.owner.model
        return m(xs[0]) if len(xs) == 1 else m(xs)

    def _graph_for(self, xs):
        key = tuple((tuple(t.shape), t.dtype) for t in xs)
        g = self.graphs.get(key)
        if g is not None:
            return g
        dev = self.owner.device
        # one capture at a time per process; thread-local capture mode lets the
        # other replicas keep replaying / copying on their own streams meanwhile
        with self.owner._capture_lock:
            static_in = [torch.zeros(t.shape, dtype=t.dtype, device=dev) for t in xs]
            for s, t in zip(static_in, xs):
                s.copy_(t)
            # warm up on the side stream (lazy allocations, kernel attributes), then capture
            with torch.cuda.stream(self.stream):
                for _ in range(2):
                    self._forward(static_in)
            self.stream.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=self.stream, pool=self.pool, capture_error_mode="thread_local"):
                static_out = self._forward(static_in)
        g = (graph, static_in, static_out)
        self.graphs[key] = g
        return g

    @torch.no_grad()
    def run(self, xs):
        dev = self.owner.device
        if dev.type != "cuda":
            return self._forward([t.to(dev) for t in xs])
        # inputs may have been produced on the caller's stream (e.g. GPU preprocessing): order them first
        self.stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self.stream):
            g = None
            if self.owner.use_graph:
                try:
                    g = self._graph_for(xs)
                except RuntimeError as e:  # model does host syncs inside forward: serve it eagerly
                    log.warning("hipGraph capture failed (%s); serving this model without graphs", e)
                    self.owner.use_graph = False
                    self.graphs.clear()
            if g is not None:
                graph, sin, sout = g
                for s, t in zip(sin, xs):
                    s.copy_(t, non_blocking=True)
                graph.replay()
                out = sout
            else:
                out = self._forward([t.to(dev, non_blocking=True) for t in xs])
            if isinstance(out, (list, tuple)):
                res = [o.float().cpu() for o in out]
            else:
                res = out.float().cpu()
        self.stream.synchronize()
        return res

    @torch.no_grad()
    def run_async(self, xs, multi):
        """Enqueue the forward on this replica's stream and copy the outputs into a pinned host
        ring slot; the caller overlaps its host work (post-processing the previous batch,
        preparing the next) with the GPU and collects the result later (_Pending.result)."""
        dev = self.owner.device
        if dev.type != "cuda":
            out = self._forward([t.to(dev) for t in xs])
            outs = list(out) if isinstance(out, (list, tuple)) else [out]
            return _Pending(None, [o.float() for o in outs], multi, xs[0].shape[0])
        cur = torch.cuda.current_stream(dev)
        self.stream.wait_stream(cur)
        for t in xs:   # the caller may free / reuse its inputs right away: keep them alive on our stream
            if t.is_cuda:
                t.record_stream(self.stream)
        with torch.cuda.stream(self.stream):
            g = None
            if self.owner.use_graph:
                try:
                    g = self._graph_for(xs)
                except RuntimeError as e:
                    log.warning("hipGraph capture failed (%s); serving this model without graphs", e)
                    self.owner.use_graph = False
                    self.graphs.clear()
            if g is not None:
                graph, sin, sout = g
                for s, t in zip(sin, xs):
                    s.copy_(t, non_blocking=True)
                graph.replay()
                out = sout
            else:
                out = self._forward([t.to(dev, non_blocking=True) for t in xs])
            outs = list(out) if isinstance(out, (list, tuple)) else [out]
            key = tuple((tuple(o.shape), o.dtype) for o in outs)
            ring = self.host_rings.get(key)
            if ring is None:
                ring = self.host_rings[key] = [[torch.empty(o.shape, dtype=torch.float32, pin_memory=True)
                                                for o in outs] for _ in range(self.RING)]
                self.host_idx[key] = 0
            i = self.host_idx[key]
            self.host_idx[key] = i + 1
            si = i % self.RING
            prev = self.slot_owner.get((key, si))
            prev = prev() if prev is not None else None
            if prev is not None and not prev.consumed:
                # more than RING handles outstanding: the slot's last result has not been read yet,
                # so this batch gets fresh pinned buffers (the unread handle keeps the old ones)
                ring[si] = [torch.empty(o.shape, dtype=torch.float32, pin_memory=True) for o in outs]
            else:
                ev = self.slot_events.get((key, si))
                if ev is not None:   # the slot's previous D2H copy must be complete before it is rewritten
                    ev.synchronize()
            slot = ring[si]
            for h, o in zip(slot, outs):
                h.copy_(o if o.dtype == torch.float32 else o.float(), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.slot_events[(key, si)] = ev
        pend = _Pending(ev, slot, multi, xs[0].shape[0])
        self.slot_owner[(key, si)] = weakref.ref(pend)
        return pend


class _Pending:
    """An enqueued prediction: result() waits for its D2H copy and returns the host output."""

    def __init__(self, event, host, multi, n):
        self.event, self.host, self.multi, self.n = event, host, multi, n
        self.consumed = False

    def done(self):
        return self.event is None or self.event.query()

    def result(self):
        if self.event is not None:
            self.event.synchronize()
        h = [t[:self.n].numpy().copy() for t in self.host]   # the pinned slot is reused RING batches later
        self.consumed = True
        return h if self.multi else h[0]


class InferenceModel:
    """Load once, predict from many threads."""

    def __init__(self, supported_concurrent_num=1, auto_scaling=False, device=None, use_graph=None,
                 dtype=None, max_batch=None):
        from zoo.common.nncontext import get_nncontext
        if supported_concurrent_num < 1:
            raise ValueError("concurrentNum should > 0")
        self.concurrent_num = int(supported_concurrent_num)
        self.auto_scaling = bool(auto_scaling)
        self.device = torch.device(device) if device is not None else get_nncontext().device
        self.use_graph = (self.device.type == "cuda") if use_graph is None else bool(use_graph)
        self.dtype = dtype
        self.max_batch = max_batch
        self.model = None
        self._queue = None
        self._lock = threading.Lock()
        self._capture_lock = threading.Lock()
        self._n_replicas = 0
        self.summary = None
        self._records = 0
        self._t0 = None

    # ------------------------------------------------------------------ loading
    def _install(self, model, quantize=False, calib_data=None, qdtype="int8"):
        model = model.to(self.device)
        if self.dtype is not None:
            model = model.to(self.dtype)
        model.eval()
        if quantize:  # blas=false in the reference loaders -> BigDL quantize() (int8)
            from zoo.ops.quant import quantize as _q
            model = _q(model, calib_data, dtype=qdtype)
        for p in model.parameters():
            p.requires_grad_(False)
        self.model = model
        self._queue = queue.Queue(maxsize=max(self.concurrent_num, 1) if not self.auto_scaling else 0)
        self._n_replicas = 0
        if not self.auto_scaling:
            for _ in range(self.concurrent_num):
                self._queue.put(self._new_replica())
        return self

    def _new_replica(self):
        with self._lock:
            r = _Replica(self, self._n_replicas)
            self._n_replicas += 1
        return r

    def load_module(self, module, blas=True, calib_data=None, qdtype="int8"):
        """Serve an in-memory torch.nn.Module (the PyTorch loader, doLoadPyTorch).
        ``blas=False`` quantizes to int8 as the reference loaders do; with ``calib_data`` a
        zoo ResNet gets the calibrated static-int8 kernels (zoo.ops.qresnet), or with
        ``qdtype="fp8"`` the OCP-fp8 ones."""
        return self._install(module, quantize=not blas, calib_data=calib_data, qdtype=qdtype)

    def load(self, model_path, weight_path=None, blas=True):
        """Zoo Keras/ZooModel file (doLoad, InferenceModel.scala:97-110)."""
        from zoo.pipeline.api.keras.serialization import load_model
        return self._install(load_model(model_path), quantize=not blas)

    def load_bigdl(self, model_path, weight_path=None, blas=True):
        """BigDL protobuf ``.model`` (doLoadBigDL, InferenceModel.scala:81-95)."""
        from zoo.pipeline.api.net import Net
        return self._install(Net.load_bigdl(model_path, weight_path), quantize=not blas)

    def load_caffe(self, model_path, weight_path, blas=True):
        """Caffe prototxt + caffemodel (doLoadCaffe, InferenceModel.scala:112-124)."""
        from zoo.pipeline.api.net import Net
        return self._install(Net.load_caffe(model_path, weight_path), quantize=not blas)

    def quantize(self, calib_data=None, dtype="int8"):
        """Re-install the loaded model as its int8 version (InferenceModelFactory.scala:33,47);
        ``calib_data`` selects the calibrated static path where the model supports it, and
        ``dtype="fp8"`` its e4m3 variant on the fp8 matrix cores."""
        if self.model is None:
            raise RuntimeError("load a model first")
        return self._install(self.model, quantize=True, calib_data=calib_data, qdtype=dtype)

    def load_onnx(self, model_path):
        from zoo.pipeline.api.onnx import load_onnx
        return self._install(load_onnx(model_path))

    def load_torch(self, model_path):
        """TorchScript file (doLoadPyTorch, InferenceModel.scala:246-266)."""
        return self._install(torch.jit.load(model_path, map_location="cpu"))

    def load_openvino(self, model_path, weight_path=None, batch_size=0):
        """OpenVINO IR xml + bin (doLoadOpenVINO, InferenceModel.scala; OpenVINOModel.scala):
        the IR is decoded and executed by this framework (zoo.pipeline.inference.openvino),
        convolutions / matmuls on the native kernels."""
        from zoo.pipeline.inference.openvino import load_openvino
        return self._install(load_openvino(model_path, weight_path, batch_size))

    def load_tensorflow(self, model_path, model_type="frozenModel", inputs=None, outputs=None, **kw):
        """TF frozen graph / export folder / SavedModel (doLoadTensorflow,
        InferenceModel.scala:126-244) executed by TFNet on this device."""
        from zoo.tfpark.tfnet import TFNet
        sig = kw.get("signature")
        tag = kw.get("tag") or "serve"
        return self._install(TFNet(model_path, inputs, outputs, tag=tag, signature=sig))

    load_tf = load_tensorflow

    # ------------------------------------------------------------------ predict
    def _take(self):
        if self.model is None:
            raise RuntimeError("no model loaded")
        if self.auto_scaling:
            try:
                return self._queue.get_nowait()
            except queue.Empty:
                return self._new_replica()
        return self._queue.get()

    def _give(self, r):
        try:
            self._queue.put_nowait(r)
        except queue.Full:
            pass

    def predict(self, inputs):
        """ndarray / tensor / list of them (multi-input) -> ndarray (or list)."""
        xs, _ = _as_tensors(inputs)
        n = xs[0].shape[0]
        mb = self.max_batch or n
        r = self._take()
        try:
            outs = []
            for s in range(0, n, max(mb, 1)):
                outs.append(r.run([t[s:s + mb] for t in xs]))
        finally:
            self._give(r)
        self._account(n)
        if isinstance(outs[0], list):
            return [torch.cat([o[i] for o in outs]).numpy() for i in range(len(outs[0]))]
        return torch.cat(outs).numpy()

    def predict_async(self, inputs):
        """Enqueue one batch (no max_batch split) and return a handle: ``.result()`` -> ndarray
        (or list). Host work done between the two calls overlaps the model on the GPU; up to
        _Replica.RING results of one replica may be outstanding."""
        xs, multi = _as_tensors(inputs)
        r = self._take()
        try:
            p = r.run_async(xs, multi)
        finally:
            self._give(r)
        self._account(xs[0].shape[0])
        return p

    def do_predict(self, inputs):
        return self.predict(inputs)

    def predict_classes(self, inputs, zero_based_label=True):
        c = np.argmax(self.predict(inputs), axis=-1)
        return c if zero_based_label else c + 1

    # ------------------------------------------------------------------ summary
    def set_inference_summary(self, summary):
        """InferenceSummary.scala:24-46: throughput scalars to TensorBoard."""
        self.summary = summary
        return self

    def _account(self, n):
        if self.summary is None:
            return
        now = time.time()
        if self._t0 is None:
            self._t0 = now
        self._records += n
        dt = now - self._t0
        if dt > 0:
            self.summary.add_scalar("Throughput", self._records / dt, self._records)

    def __repr__(self):
        return "InferenceModel(auto_scaling=%s, concurrent_num=%d, device=%s, graph=%s)" % (
            self.auto_scaling, self.concurrent_num, self.device, self.use_graph)
