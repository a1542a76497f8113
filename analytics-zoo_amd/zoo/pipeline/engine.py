"""The training / evaluation engine (MI355X replacement of Zoo's
InternalDistriOptimizer + BigDL DistriOptimizer, SURVEY.md §2.4 E1-E3, E5;
call stack §3.2).

One process per GPU. Per iteration:
  1. ``flat.grad`` zeroed (one memset over the flat fp32 gradient buffer -- or none: the native
     optimizer kernels clear each gradient slot after reading it, FlatParams.grad_clean)
  2. forward on the native kernels (bf16 activations, bf16 weight copies)
  3. loss (+ fused loss gradient) and backward; conv/BN backward kernels
     accumulate straight into the flat gradient buffer and each finished
     parameter triggers its RCCL bucket on the comm stream (overlap)
  4. optional clipping (constant / global L2 with one all-reduce), then ONE
     fused optimizer launch over the flat master buffer, which also rewrites
     the bf16 compute copy (or the ZeRO-1 sharded variant)
No host synchronisation happens inside the iteration; loss values stay on the
device until a trigger (logging / validation / checkpoint) needs them.

Failure handling mirrors Topology.scala:1180-1262: any exception inside the
loop (other than ValueError, the analogue of IllegalArgumentException) is
retried up to ``failure_retry_times`` within ``failure_retry_interval_s`` by
reloading the latest checkpoint, if one is configured. ``ZOO_FAULT_INJECT_STEP``
injects a failure at a chosen iteration to exercise that path.
"""
import glob
import logging
import math
import os
import random
import time

import torch

from zoo.common.triggers import EveryEpoch, MaxEpoch, Trigger
from zoo.parallel.ddp import GradSync
from zoo.parallel.flat import FlatParams
from zoo.ops import _kern, workspace, wstream
from zoo.ops.devscalar import seed_offset_used

log = logging.getLogger("zoo.engine")


class InjectedFault(RuntimeError):
    pass


class CommFailure(RuntimeError):
    """A collective failed (RCCL/gloo error or timeout). The process group cannot be
    trusted any more: the engine exits non-zero so the launcher (torchrun
    ``--max-restarts``) restarts every rank, which then auto-resume from the latest
    checkpoint (``ZooConfig.auto_resume``)."""


class CoordinatedFailure(RuntimeError):
    """Every rank agreed that some rank failed locally: all of them reload the
    latest checkpoint together (Topology.scala:1229-1262 retry, made collective)."""


def _tp_groups(model):
    """Process group of the tensor-parallel layers in ``model`` (None if none)."""
    groups = {id(m.group): m.group for m in model.modules() if getattr(m, "tensor_parallel", False)}
    if not groups:
        return None, False
    if len(groups) > 1:
        raise ValueError("TrainingEngine: tensor-parallel layers must share one process group")
    return next(iter(groups.values())), True


def data_parallel_group(model):
    """The data-parallel group for a model with tensor-parallel layers: the ranks
    holding the SAME shard (same TP rank), TP groups being contiguous rank blocks.
    Without TP layers: None (the world)."""
    import torch.distributed as dist
    tpg, has_tp = _tp_groups(model)
    if not has_tp or not (dist.is_available() and dist.is_initialized()):
        return None
    world = dist.get_world_size()
    tp = dist.get_world_size(tpg)
    if world % tp:
        raise ValueError("world size %d is not a multiple of the tensor-parallel size %d" % (world, tp))
    mine = None
    for t in range(tp):  # every rank creates every group, in the same order
        g = dist.new_group(list(range(t, world, tp)))
        if dist.get_rank() % tp == t:
            mine = g
    return mine


class _Phases:
    """roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm: visible with
    ``rocprofv3 --marker-trace``) and optional device-side phase timings with
    HIP events. Both are off unless configured, and neither
    synchronises inside a step: event pairs are resolved at the next report."""

    def __init__(self, roctx, timing, device):
        self.roctx = roctx and device.type == "cuda"
        self.timing = timing and device.type == "cuda"
        self.pending = []
        self.totals = {}
        self.counts = {}

    def range(self, name):
        return _PhaseRange(self, name)

    def resolve(self):
        keep = []
        for name, a, b in self.pending:
            if b.query():
                self.totals[name] = self.totals.get(name, 0.0) + a.elapsed_time(b)
                self.counts[name] = self.counts.get(name, 0) + 1
            else:
                keep.append((name, a, b))
        self.pending = keep
        return {k: self.totals[k] / max(self.counts[k], 1) for k in self.totals}


class _PhaseRange:
    __slots__ = ("ph", "name", "ev")

    def __init__(self, ph, name):
        self.ph, self.name, self.ev = ph, name, None

    def __enter__(self):
        if self.ph.roctx:
            torch.cuda.nvtx.range_push("zoo." + self.name)
        if self.ph.timing:
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record()
        return self

    def __exit__(self, *exc):
        if self.ph.timing:
            end = torch.cuda.Event(enable_timing=True)
            end.record()
            self.ph.pending.append((self.name, self.ev, end))
        if self.ph.roctx:
            torch.cuda.nvtx.range_pop()


def _checkpoint_iteration(path):
    """Iteration a ``model[.<n>]`` checkpoint file records: its numeric suffix, else the
    ``zoo_neval`` attribute of the file (overwrite-mode checkpoints), else -1."""
    base = os.path.basename(path)
    suf = base[len("model"):].lstrip(".")
    if suf.isdigit():
        return int(suf)
    try:
        from zoo.utils.bigdl_model import is_bigdl_model_file, read_attr
        if is_bigdl_model_file(path):
            return int(read_attr(path, "zoo_neval", -1))
    except (OSError, ValueError, TypeError):
        pass
    return -1


def _tensors(b):
    if isinstance(b, torch.Tensor):
        return [b] if b.is_cuda else []
    if isinstance(b, (list, tuple)):
        return [t for v in b for t in _tensors(v)]
    if isinstance(b, dict):
        return [t for v in b.values() for t in _tensors(v)]
    return []


def _move(batch, device, non_blocking=True):
    if isinstance(batch, torch.Tensor):
        return batch.to(device, non_blocking=non_blocking)
    if isinstance(batch, (list, tuple)):
        return type(batch)(_move(b, device, non_blocking) for b in batch)
    if isinstance(batch, dict):
        return {k: _move(v, device, non_blocking) for k, v in batch.items()}
    return batch


class TrainingEngine:
    def __init__(self, model, criterion, optim_method, device=None, ctx=None, clip=None, sharded=None,
                 bucket_mb=None, model_forward=None, hip_graph=None, dp_group=None):
        from zoo.common.nncontext import get_nncontext
        self.ctx = ctx or get_nncontext()
        cfg = self.ctx.config
        self.device = torch.device(device) if device is not None else self.ctx.device
        self.model = model.to(self.device)
        self.criterion = criterion
        self.optim = optim_method
        self.flat = FlatParams(list(self.model.parameters()), device=self.device,
                               bf16_copy=self.device.type == "cuda")
        self.dp_group = dp_group if dp_group is not None else data_parallel_group(self.model)
        self.sync = GradSync(self.flat, group=self.dp_group, bucket_mb=bucket_mb or cfg.bucket_mb,
                             mode="sharded" if (cfg.sharded_optimizer if sharded is None else sharded)
                             else "allreduce", overlap=cfg.overlap_comm, compress=cfg.grad_compression or None,
                             force_comm=cfg.force_comm, comm=cfg.comm, rccl_channels=cfg.rccl_channels)
        self.sync.broadcast_parameters()
        # gradient writes outside train_step (a user's own backward) mark the flat gradient dirty
        self.sync.engine_managed = True
        self._local_failure = None
        self.clip = clip
        self.forward_fn = model_forward or (lambda m, x: m(x))
        self.state = {"epoch": 1, "neval": 1, "Loss": float("nan"), "score": None, "records": 0}
        self._pending_loss = []
        self.train_summary = None
        self.val_summary = None
        self.checkpoint_path = None
        self.checkpoint_trigger = None
        self.checkpoint_overwrite = True
        self.fault_step = cfg.fault_inject_step
        self._fault_fired = False
        # hipGraph capture of forward+backward (launch-bound models, e.g. NCF):
        # the graph replays every kernel of the step with one launch; the
        # gradient all-reduce and the optimizer stay eager after the replay
        self.phases = _Phases(cfg.roctx, cfg.phase_timing, self.device)
        self.debug_sync = cfg.debug_sync
        self.hip_graph = (cfg.hip_graph if hip_graph is None else bool(hip_graph)) and self.device.type == "cuda"
        self._graphs = {}
        self._graph_warm = {}
        # single-rank jobs: each bucket's optimizer update runs on the weight-gradient side
        # stream as soon as its gradients are final, overlapping the rest of the backward
        # (GradSync.enable_ibo). Not with gradient clipping (a global norm). Under hipGraph
        # capture the updates are captured too: the optimizer kernels then read the learning rate
        # and bias corrections from a device buffer staged before every replay
        # (OptimMethod.enable_device_hparams), so the graph follows the schedule.
        # Captured steps keep the optimizer at the end of the step unless ZOO_OPTIM_IN_BWD_GRAPH=1:
        # NCF (one small bucket, the step launch-bound) replays 0.234 ms/step with the updates
        # inside the graph against 0.228 without (profiles/r5/bench_ncf_r5.log)
        ibo_graph_ok = not self.hip_graph or os.environ.get("ZOO_OPTIM_IN_BWD_GRAPH", "0") != "0"
        self.ibo = bool(os.environ.get("ZOO_OPTIM_IN_BWD", "1") != "0" and clip is None and ibo_graph_ok and
                        wstream.on() and getattr(optim_method, "supports_ranges", lambda: False)() and
                        self.sync.enable_ibo(optim_method))
        if self.ibo and self.hip_graph and hasattr(optim_method, "enable_device_hparams"):
            optim_method.enable_device_hparams(self.device)
        # hipGraph with collectives over the native comm layer (ZooConfig.comm = "native"): the WHOLE
        # data-parallel step -- forward, backward, the bucket collectives (RCCL on the comm stream,
        # captured with the graph) and the optimizer update (device-scalar lr / bias corrections) --
        # is ONE replay (BigDL's per-iteration AllReduceParameter sync in
        # Topology.scala:1128-1206). The row-sparse protocol reads a host flag per step, so models
        # with row-sparse tables keep the eager path; ZOO_GRAPH_FULL_STEP=0 keeps comm + update eager.
        s_ = self.sync
        self.full_graph = bool(
            self.hip_graph and s_.comm and s_.ncomm is not None and not self.ibo and clip is None
            and s_.mode == "allreduce" and getattr(optim_method, "supports_ranges", lambda: False)()
            and hasattr(optim_method, "enable_device_hparams")
            and not any(b.sparse for b in s_.buckets)
            and os.environ.get("ZOO_GRAPH_FULL_STEP", "1") != "0")
        self._full_optim = optim_method if self.full_graph else None
        self._replayed_full = False
        if self.full_graph:
            optim_method.enable_device_hparams(self.device)
        # dropout under hipGraph: a device seed offset, restaged every step, is xored into the
        # seeds the captured kernels replay (fresh masks per step)
        self._seed_stager = None
        if self.hip_graph:
            from zoo.ops.devscalar import dropout_seed_stager
            self._seed_stager = dropout_seed_stager(self.device)
            self._seed_rng = random.Random(torch.initial_seed() + 977)

    # ------------------------------------------------------------------
    def _maybe_inject_fault(self):
        cfg = self.ctx.config
        if self.fault_step >= 0 and self.state["neval"] == self.fault_step and not self._fault_fired and \
                (cfg.fault_inject_rank < 0 or cfg.fault_inject_rank == self.ctx.rank):
            self._fault_fired = True
            raise InjectedFault("injected fault at iteration %d" % self.fault_step)

    def train_step(self, inputs, target):
        """One synchronous-DP iteration. Returns the (device) loss tensor.

        Multi-rank failure protocol: an exception in this rank's forward/backward
        does not leave the other ranks blocked in a collective. The rank turns into
        a "zombie" that keeps taking part in every collective with a zero gradient
        until the next agreement point (:meth:`flush_loss`, checkpoints), where all
        ranks learn of the failure together and reload the latest checkpoint.
        A failing collective raises :class:`CommFailure` (restart by the launcher)."""
        multi = self.sync.comm and self.sync.world > 1
        if self.sync.ibo_optim is not None and (self.sync.ibo_optim is not self.optim or self.clip is not None or
                                                (self.hip_graph and getattr(self.optim, "_dev_hp", None) is None)):
            self.sync.ibo_optim = None   # optimizer / clipping / graph mode changed: plain end-of-step update
            self.ibo = False
            # graphs captured with the in-backward updates inside would keep replaying them
            # (unclipped, and doubled by the end-of-step update): recapture without
            if any(g[4] for g in self._graphs.values()):
                torch.cuda.synchronize(self.device)
                self._graphs.clear()
                self._graph_warm.clear()
        if self.full_graph and (self.clip is not None or self.optim is not self._full_optim):
            # clipping / a new optimizer: the captured update no longer applies -- recapture the
            # step without it (comm + update eager after the replay)
            self.full_graph = False
            torch.cuda.synchronize(self.device)
            self._graphs.clear()
            self._graph_warm.clear()
        if getattr(self.optim, "_dev_hp", None) is not None:
            self.optim.stage_device_hparams()
        if self._seed_stager is not None and (not self._graphs or seed_offset_used(self.device)):
            # this step's dropout seed offset -- only while a captured graph reads it (a model
            # without dropout skips the per-step pinned copy: NCF's step is 0.23 ms)
            self._seed_stager.stage([self._seed_rng.getrandbits(31)])
        self.model.train()
        ph = self.phases
        loss = None
        if self._local_failure is None:
            try:
                self._maybe_inject_fault()
                with ph.range("fwd_bwd"):
                    if self.hip_graph and torch.is_tensor(target):
                        loss = self._graph_fwd_bwd(inputs, target)
                    else:
                        loss = self._fwd_bwd(inputs, target)
            except (ValueError, KeyboardInterrupt):
                raise
            except Exception as e:  # noqa: BLE001
                if not multi:
                    raise
                log.warning("rank %d: step failed (%s); continuing with zero gradients until the ranks agree",
                            self.ctx.rank, e)
                self._local_failure = e
        if loss is None:  # zombie step: contribute nothing, stay in lock-step
            # buckets launched before the failure may still be read by in-flight collectives
            self.sync.wait_comm()
            self.flat.grad.zero_()
            self.flat.grad_clean = False
            loss = torch.zeros((), device=self.device)
        with ph.range("comm_optim"):
            if self._replayed_full:
                # collectives and update ran inside the replay: host-side bookkeeping only
                self._replayed_full = False
                self.optim.finish_step(self.flat.bf16 is not None)
                self.sync.reset()
                self.state["neval"] += 1
                return loss
            try:
                self.sync.step(self.optim, self.clip)
            except Exception as e:  # noqa: BLE001
                if multi and not isinstance(e, (ValueError, KeyboardInterrupt)):
                    raise CommFailure("gradient synchronisation failed on rank %d: %s" % (self.ctx.rank, e)) from e
                raise
        self.state["neval"] += 1
        if self.debug_sync:  # debug mode: surface asynchronous HIP errors / divergence at the failing step
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            if not torch.isfinite(loss).all():
                raise FloatingPointError("non-finite loss at iteration %d" % (self.state["neval"] - 1))
        return loss

    def phase_times(self):
        """Mean device milliseconds per phase so far (needs ``phase_timing``)."""
        return self.phases.resolve()

    def _fwd_bwd(self, inputs, target):
        if not getattr(self.flat, "grad_clean", False):
            self.flat.grad.zero_()
        self.flat.grad_clean = False
        workspace.begin_step(self.device)
        self.sync.in_step = True
        try:
            _kern.prefetch_flips(self.device)   # the dgrad filters of the updated weights, beside the forward
            out = self.forward_fn(self.model, inputs)
            loss = self.criterion(out, target)
            # weight gradients overlap the data-gradient chain on a side stream, joined back
            # before anything reads the gradients (zoo.ops.wstream)
            with wstream.enabled(self.device):
                loss.backward()
        finally:
            self.sync.in_step = False
            workspace.end_step()
        return loss.detach()

    def _graph_fwd_bwd(self, inputs, target):
        """Replay a captured forward+backward for this input signature. Two eager
        warm-up steps per signature settle lazy allocations (workspace high-water
        mark, kernel attributes) before the capture."""
        xs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        if not all(torch.is_tensor(t) for t in xs):
            return self._fwd_bwd(inputs, target)
        key = tuple((tuple(t.shape), t.dtype) for t in xs + [target])
        g = self._graphs.get(key)
        if g is None:
            n = self._graph_warm.get(key, 0)
            if n < 2:
                self._graph_warm[key] = n + 1
                return self._fwd_bwd(inputs, target)
            try:
                g = self._capture(key, xs, target, isinstance(inputs, (list, tuple)))
            except RuntimeError as e:  # a host sync inside the step: stay eager for this model
                log.warning("hipGraph capture failed (%s); training eagerly", e)
                self.hip_graph = False
                torch.cuda.synchronize(self.device)
                return self._fwd_bwd(inputs, target)
        graph, sx, sy, sloss, ibo_done, full = g
        if not getattr(self.flat, "grad_clean", False):
            self.flat.grad.zero_()      # the captured step may rely on the optimizer's clearing
        self.flat.grad_clean = False
        for s_, t in zip(sx, xs):
            s_.copy_(t, non_blocking=True)
        sy.copy_(target, non_blocking=True)
        graph.replay()
        if full:   # the captured update cleared every gradient slot
            self.flat.grad_clean = True
            self._replayed_full = True
        # the buckets whose in-backward update is part of the graph: step() updates the rest
        self.sync._ibo_done = set(ibo_done)
        return sloss.clone()

    def _capture(self, key, xs, target, as_list):
        sx = [t.detach().clone() for t in xs]
        sy = target.detach().clone()
        overlap = self.sync.overlap
        self.sync.overlap = False  # no collectives inside the capture: finish() launches them after replay
        _kern.begin_capture()
        torch.cuda.synchronize(self.device)
        graph = torch.cuda.CUDAGraph()
        full = self.full_graph
        try:
            with torch.cuda.graph(graph):
                sloss = self._fwd_bwd(sx if as_list else sx[0], sy)
                if full:
                    # the bucket collectives (native comm, comm stream forked from the capture
                    # stream) and the update, which reads its hyper-parameters from device memory
                    flat = self.flat
                    self.sync.finish()
                    self.optim.step_range(flat.master, flat.grad, flat.bf16, 1.0 / self.sync.world, 0,
                                          flat.master.numel(), zero_grad=True)
        finally:
            self.sync.overlap = overlap
        ibo_done = set(self.sync._ibo_done)   # in-backward updates captured into the graph
        self.sync.reset()
        g = (graph, sx, sy, sloss, ibo_done, full)
        self._graphs[key] = g
        log.info("captured %s as a hipGraph for inputs %s",
                 "forward+backward+collectives+update" if full else "forward+backward", key)
        return g

    # ------------------------------------------------------------------
    def fit(self, data, end_trigger=None, validation=None, val_methods=None, val_trigger=None,
            batch_size=None, log_every=None, callbacks=()):
        """Train over an iterable of (x, y) minibatches until ``end_trigger``.

        ``data`` is anything with ``data(train=True)`` (a FeatureSet) or a
        re-iterable of batches (one pass = one epoch).
        """
        end_trigger = end_trigger or MaxEpoch(1)
        val_trigger = val_trigger or EveryEpoch()
        log_every = log_every or self.ctx.config.log_every
        cfg = self.ctx.config
        retries = []
        if cfg.auto_resume and self.latest_checkpoint() is not None and self.state["neval"] == 1:
            log.info("auto-resume from %s", self.latest_checkpoint())
            self.load_checkpoint(self.latest_checkpoint())
        multi = self.sync.comm and self.sync.world > 1
        while True:
            try:
                self._fit_loop(data, end_trigger, validation, val_methods, val_trigger, log_every, callbacks)
                self.flush_loss()  # final agreement point
                break
            except (ValueError, KeyboardInterrupt, CommFailure):
                raise
            except Exception as e:  # noqa: BLE001 - mirrors Topology.scala:1229 catch Throwable
                if multi and not isinstance(e, CoordinatedFailure):
                    raise  # a local failure outside train_step: no safe way to keep the ranks in step
                now = time.time()
                retries = [t for t in retries if now - t < cfg.failure_retry_interval_s] + [now]
                ck = self.latest_checkpoint()
                if ck is None or len(retries) > cfg.failure_retry_times:
                    raise
                log.warning("training failed (%s); retry %d/%d from checkpoint %s", e, len(retries),
                            cfg.failure_retry_times, ck)
                self._local_failure = None
                self._pending_loss = []
                self.load_checkpoint(ck)
        self.sync.sync_master()
        return self

    def _iter_epoch(self, data):
        if hasattr(data, "data"):
            return data.data(train=True, epoch=self.state["epoch"])
        return iter(data)

    def _device_batches(self, it):
        """(x, y) on the device, one batch ahead: host batch i+1's copy is issued on a dedicated
        copy stream BEFORE step i is issued, so the DMA overlaps step i's kernels; the compute
        stream waits on the copy's event only when it reaches the batch (FeatureSet /
        SampleToMiniBatch prefetch, NNEstimator.scala:382-470 -- here over PCIe from pinned host
        batches). ``ZOO_COPY_STREAM=0``: copies on the compute stream right before the step."""
        dev = self.device
        if dev.type != "cuda" or os.environ.get("ZOO_COPY_STREAM", "1") == "0":
            for batch in it:
                yield _move(batch[0], dev), _move(batch[1], dev)
            return
        if getattr(self, "_copy_stream", None) is None:
            self._copy_stream = torch.cuda.Stream(dev)
        cs = self._copy_stream

        def issue(batch):
            with torch.cuda.stream(cs):
                x, y = _move(batch[0], dev), _move(batch[1], dev)
                ev = torch.cuda.Event()
                ev.record(cs)
            return x, y, ev

        def handoff(item):
            x, y, ev = item
            cur = torch.cuda.current_stream(dev)
            cur.wait_event(ev)
            for t in _tensors(x) + _tensors(y):
                t.record_stream(cur)   # allocated on the copy stream, consumed on the compute stream
            return x, y

        ahead = None
        for batch in it:
            nxt = issue(batch)
            if ahead is not None:
                yield handoff(ahead)
            ahead = nxt
        if ahead is not None:
            yield handoff(ahead)

    def _fit_loop(self, data, end_trigger, validation, val_methods, val_trigger, log_every, callbacks):
        state = self.state
        while not end_trigger(state):
            t_epoch = time.time()
            recs = 0
            t_last = time.time()
            n_since = 0
            for x, y in self._device_batches(self._iter_epoch(data)):
                loss = self.train_step(x, y)
                bs = (x[0] if isinstance(x, (list, tuple)) else x).shape[0] * self.sync.world
                recs += bs
                n_since += bs
                state["records"] += bs
                self._pending_loss.append((state["neval"] - 1, loss))
                if (state["neval"] - 1) % log_every == 0:
                    lval = self.flush_loss()
                    dt = time.time() - t_last
                    thr = n_since / dt if dt > 0 else 0.0
                    state["Throughput"] = thr
                    log.info("Epoch %d iter %d loss %.5f throughput %.1f records/s lr %.6g", state["epoch"],
                             state["neval"] - 1, lval, thr, self.optim.current_lr())
                    if self.train_summary is not None:
                        self.train_summary.add_scalar("Throughput", thr, state["neval"] - 1)
                        self.train_summary.add_scalar("LearningRate", self.optim.current_lr(), state["neval"] - 1)
                        for name, ms in self.phase_times().items():
                            self.train_summary.add_scalar("StepTime/%s_ms" % name, ms, state["neval"] - 1)
                    t_last, n_since = time.time(), 0
                for cb in callbacks:
                    cb(self, state)
                if end_trigger.iteration_based and end_trigger(state):
                    break
                if self.checkpoint_trigger is not None and self.checkpoint_trigger.iteration_based and \
                        self.checkpoint_trigger(state):
                    self.save_checkpoint()
            self.flush_loss()
            log.info("Epoch %d finished: %d records in %.2fs", state["epoch"], recs, time.time() - t_epoch)
            state["epoch"] += 1
            self.optim.update_epoch(state["epoch"])
            state["epoch_end"] = True
            if validation is not None and val_methods and val_trigger(state):
                res = self.evaluate(validation, val_methods)
                state["score"] = res[0][1] if res else None
                self.optim.state["score"] = state["score"]
                if self.val_summary is not None:
                    for name, v in res:
                        self.val_summary.add_scalar(name, v, state["neval"] - 1)
            if self.checkpoint_trigger is not None and self.checkpoint_trigger(state):
                self.save_checkpoint()
            state["epoch_end"] = False

    def flush_loss(self):
        """Bring the device-side per-iteration losses to the host (one sync),
        average over ranks (one all-reduce) and log them to TensorBoard."""
        multi = self.sync.comm and self.sync.world > 1
        if not self._pending_loss and not multi:
            return self.state["Loss"]
        its = [i for i, _ in self._pending_loss]
        vals = torch.stack([l.float().reshape(()) for _, l in self._pending_loss]) if self._pending_loss \
            else torch.zeros(0)
        # the failure flag rides in the same all-reduce as the losses (no extra collective)
        red = self.sync.all_reduce_scalars(vals.detach().cpu().tolist() + [1.0 if self._local_failure else 0.0])
        self._pending_loss = []
        if red[-1] > 0:
            cause = self._local_failure
            raise CoordinatedFailure("%d rank(s) failed before iteration %d%s" % (
                int(red[-1]), self.state["neval"] - 1, (": %s" % cause) if cause else ""))
        red = red[:-1] / self.sync.world
        if not its:
            return self.state["Loss"]
        if self.train_summary is not None:
            for it, v in zip(its, red.tolist()):
                self.train_summary.add_scalar("Loss", v, it)
        self.state["Loss"] = float(red[-1])
        self.optim.state["Loss"] = self.state["Loss"]
        return self.state["Loss"]

    # ------------------------------------------------------------------
    @torch.no_grad()
    def predict(self, data, batch_size=None):
        self.model.eval()
        outs = []
        for batch in (data.data(train=False) if hasattr(data, "data") else data):
            x = batch[0] if isinstance(batch, (list, tuple)) else batch
            out = self.forward_fn(self.model, _move(x, self.device))
            outs.append(out.float() if isinstance(out, torch.Tensor) else out)
        return outs

    @torch.no_grad()
    def evaluate(self, data, val_methods):
        """Distributed validation: per-rank partial results, ONE all-reduce of a
        small vector (Topology.scala:1459-1519, CC6)."""
        self.model.eval()
        accs = [m.new_accumulator() for m in val_methods]
        for batch in (data.data(train=False) if hasattr(data, "data") else data):
            x, y = _move(batch[0], self.device), _move(batch[1], self.device)
            out = self.forward_fn(self.model, x)
            for m, a in zip(val_methods, accs):
                m.update(a, out, y, self.criterion)
        flat = []
        for a in accs:
            flat.extend(a)
        red = self.sync.all_reduce_scalars(flat).tolist()
        res = []
        i = 0
        for m, a in zip(val_methods, accs):
            n = len(a)
            res.append((m.name, m.result(red[i:i + n])))
            i += n
        self.model.train()
        return res

    # ------------------------------------------------------------------
    # checkpoint / resume: model.<neval> + optimMethod-<name>.<neval>
    def set_checkpoint(self, path, trigger=None, overwrite=True):
        self.checkpoint_path = path
        self.checkpoint_trigger = trigger or EveryEpoch()
        self.checkpoint_overwrite = overwrite
        os.makedirs(path, exist_ok=True)

    def _sharded(self):
        return self.sync.mode == "sharded" and self.sync.comm

    def save_checkpoint(self):
        """``model<suffix>`` (rank 0) + ``optimMethod-<name><suffix>``; with the ZeRO-1
        sharded optimizer every rank writes its own state shard as
        ``optimMethod-<name><suffix>.rank<r>``. Collective: every rank calls it."""
        if self.checkpoint_path is None:
            return
        multi = self.sync.comm and self.sync.world > 1
        if multi:
            self.flush_loss()  # agreement point: never checkpoint a state a failed rank diverged from
        self.sync.sync_master()
        from zoo.utils.bigdl_model import save_optim_method
        it = self.state["neval"] - 1
        suffix = "" if self.checkpoint_overwrite else ".%d" % it
        name = type(self.optim).__name__
        opath = os.path.join(self.checkpoint_path, "optimMethod-%s%s" % (name, suffix))
        # OptimMethod state as a BigDL-protobuf record (zoo.utils.bigdl_model.save_optim_method)
        if self._sharded():
            save_optim_method(self.optim.state_dict(), "%s.rank%d" % (opath, self.sync.rank), True)
        if self.ctx.rank == 0:
            if not self._sharded():
                save_optim_method(self.optim.state_dict(), opath, True)
            # the model file goes last: latest_checkpoint() only sees complete checkpoints. It is a
            # BigDL/Zoo ``.model`` protobuf (Net.load / KerasNet.loadModel read it), with the engine
            # counters as top-level attributes
            import json as _json
            from zoo.utils.bigdl_model import save_bigdl_model
            eng = {k: v for k, v in self.state.items() if isinstance(v, (int, float, str, bool, type(None)))}
            save_bigdl_model(self.model, os.path.join(self.checkpoint_path, "model" + suffix), True,
                             extra_attr={"zoo_engine_state": _json.dumps(eng), "zoo_neval": int(it),
                                         "zoo_world": int(self.sync.world), "zoo_sharded": bool(self._sharded())})
        if multi:
            self.ctx.barrier()

    def save_flat_checkpoint(self, path):
        """Fast native snapshot: the flat fp32 master buffer and the
        optimizer state buffers as one safetensors file per rank (ZeRO-1 ranks each
        hold their shard's state), plus the engine counters in the metadata."""
        from safetensors.torch import save_file
        import json as _json
        t = {"master": self.flat.master.detach().cpu().contiguous()}
        for i, b in enumerate(self.optim._buffers or []):
            t["optim_state_%d" % i] = b.detach().cpu().contiguous()
        meta = {"engine_state": _json.dumps({k: v for k, v in self.state.items()
                                             if isinstance(v, (int, float, str, type(None)))}),
                "optim_state": _json.dumps({k: v for k, v in self.optim.state.items()
                                            if isinstance(v, (int, float, str))}),
                "rank": str(self.ctx.rank), "world": str(self.sync.world)}
        p = path if self.sync.world == 1 else "%s.rank%d" % (path, self.ctx.rank)
        os.makedirs(os.path.dirname(os.path.abspath(p)), exist_ok=True)
        save_file(t, p, metadata=meta)
        return p

    def load_flat_checkpoint(self, path):
        from safetensors import safe_open
        import json as _json
        p = path if self.sync.world == 1 else "%s.rank%d" % (path, self.ctx.rank)
        with safe_open(p, framework="pt", device="cpu") as f:
            meta = f.metadata() or {}
            self.flat.master.copy_(f.get_tensor("master").to(self.flat.master.device))
            keys = sorted(k for k in f.keys() if k.startswith("optim_state_"))
            if keys:
                bufs = [f.get_tensor(k).to(self.device) for k in keys]
                self.optim._buffers = bufs
                self.optim._key = (bufs[0].numel(), str(self.device))
        self.flat.refresh_bf16()
        self.flat.grad_clean = False
        self.state.update(_json.loads(meta.get("engine_state", "{}")))
        self.optim.state.update(_json.loads(meta.get("optim_state", "{}")))
        self.sync.reset()
        return self

    def latest_checkpoint(self):
        """The newest complete ``model[.<neval>]`` snapshot, by the iteration it records (the
        ``.<n>`` suffix, else its ``zoo_neval`` attribute) -- never by file mtime, which a copied
        or restored checkpoint directory does not preserve."""
        if self.checkpoint_path is None:
            return None
        cands = [c for c in glob.glob(os.path.join(self.checkpoint_path, "model*"))
                 if not os.path.basename(c).startswith("model.tmp") and not c.endswith(".part")]
        if not cands:
            return None
        return max(cands, key=_checkpoint_iteration)

    def load_checkpoint(self, model_file):
        """Collective in multi-rank runs (every rank loads, then one broadcast)."""
        import json as _json
        from zoo.utils.bigdl_model import is_bigdl_model_file, load_bigdl_model, load_optim_method, read_attr
        from zoo.utils.checkpoint import load_object

        def load_opt(p):  # BigDL OptimMethod record (round 3+) or a round-2 torch file
            return load_optim_method(p) if is_bigdl_model_file(p) else load_object(p)
        if is_bigdl_model_file(model_file):
            load_bigdl_model(model_file, model=self.model)
            d = {"engine_state": _json.loads(read_attr(model_file, "zoo_engine_state", "{}") or "{}"),
                 "world": read_attr(model_file, "zoo_world", self.sync.world),
                 "sharded": bool(read_attr(model_file, "zoo_sharded", False))}
        else:  # round-1 torch-file checkpoints
            d = load_object(model_file)
            self.model.load_state_dict(d["model"])
        self.flat.refresh_bf16()
        self.state.update(d.get("engine_state", {}))
        suffix = os.path.basename(model_file)[len("model"):]
        name = type(self.optim).__name__
        opath = os.path.join(os.path.dirname(model_file), "optimMethod-%s%s" % (name, suffix))
        if "sharded" in d and bool(d["sharded"]) != bool(self._sharded()):
            # a ZeRO-1 checkpoint holds only per-rank state shards, a replicated one a single file:
            # the optimizer state cannot be carried across that change
            log.warning("checkpoint %s was written %s but this engine runs %s: optimizer state not restored "
                        "(history reset)", model_file, "sharded" if d["sharded"] else "replicated",
                        "sharded" if self._sharded() else "replicated")
            self.optim.clear_history()
        elif self._sharded():
            if d.get("world", self.sync.world) != self.sync.world:
                log.warning("checkpoint written by %s ranks, running on %d: optimizer state shards reset",
                            d.get("world"), self.sync.world)
                self.optim.clear_history()
            elif os.path.exists("%s.rank%d" % (opath, self.sync.rank)):
                self.optim.load_state_dict(load_opt("%s.rank%d" % (opath, self.sync.rank)))
                self.optim.to(self.device)
        elif os.path.exists(opath):
            self.optim.load_state_dict(load_opt(opath))
            self.optim.to(self.device)
        self.sync.broadcast_parameters()
        self.flat.grad_clean = False
        self.sync.reset()
