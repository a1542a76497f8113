"""Data-parallel gradient synchronisation over RCCL (xGMI) — one process per GPU.

This replaces BigDL's Spark-BlockManager ``AllReduceParameter`` (SURVEY.md
§2.4 "DistriOptimizer iteration", §2.17 CC1-CC4; Topology.scala:1128-1206,
docs/docs/wp-bigdl.md:140-160):

* Gradients live in ONE flat fp32 buffer (:class:`FlatParams`) laid out in
  backward order and cut into contiguous buckets (``bucket_mb``, 16 MB by
  default: big enough for full per-link bandwidth on xGMI, small enough that
  the last bucket -- launched when backward ends -- is a short exposed tail).
* A bucket is launched on a dedicated comm stream (waiting on an event of the
  compute stream) as soon as EVERY gradient contribution of its parameters has
  been enqueued. The number of contributions per parameter is learned in the
  first (calibration) step, in which nothing launches early: a weight used
  twice (shared Keras layers, siamese KNRM/TextMatcher, tied embeddings)
  triggers its bucket only after its second contribution. A later step that
  adds MORE contributions than calibrated raises instead of reducing a partial
  gradient.
* ``mode="allreduce"``: every rank ends with the summed gradient.
  - fp32: one ``all_reduce`` per bucket.
  - ``compress="bf16"``: the bucket is packed to bf16 into a persistent buffer
    and exchanged with ONE ``all_to_all`` (xGMI is a full point-to-point mesh:
    every rank sends chunk r straight to rank r over its own link); the owner
    sums the chunks with fp32 accumulation (``sum_chunks_bf16`` kernel: one
    bf16 rounding per input, not one per ring hop), and an ``all_gather``
    returns the bf16 sums, unpacked into the fp32 flat gradient.
* ``mode="sharded"`` (ZeRO-1, BigDL's exact algorithm: each rank owns 1/N of
  the parameters and optimizer state): the per-bucket reduce-scatter runs
  OVERLAPPED with backward (fp32 ``reduce_scatter_tensor``, or the bf16
  all-to-all + fp32 accumulate above), each rank runs the fused optimizer on
  its contiguous shard (the concatenation of its chunk of every bucket), and
  the updated fp32 master shards are all-gathered per bucket back into the
  flat buffer (layers read some fp32 parameters directly, so every rank must
  hold identical fp32 values), followed by one cast pass for the bf16 copy.

* Row-sparse embedding tables (``mark_row_sparse``; NCF / Wide&Deep lookups,
  SURVEY.md §2.17 note, NeuralCF.scala:45-53) get buckets of their own that do
  not all-reduce the dense table gradient: the ranks all-gather the ids they
  looked up this step, and only the rows of the union are all-reduced (a table
  of 138k users with 8k lookups per rank moves ~|union| x dim floats instead of
  the whole table). The rows nobody touched are zero on every rank, so the
  result equals the dense all-reduce (the table must get gradient only through
  lookups: no dense regulariser on it).

All persistent comm buffers are allocated once (chunk = ceil(bucket/N) rounded
to 64 elements). ``force_comm`` runs the whole bucket / comm-stream / event
path on a world-size-1 process group (RCCL with one rank), so the overlapped
code is exercised on a single GPU (``ZOO_FORCE_COMM=1``).

Gradient averaging (1/N) is folded into the optimizer kernel's ``gscale``.
On CPU (gloo) the same code runs synchronously; that is what the
multi-process CPU tests exercise.
"""
import threading

import torch
import torch.distributed as dist

from zoo.parallel.flat import FlatParams

CHUNK_ALIGN = 64
# step counter for the row-sparse id records (bumped by GradSync.reset): an embedding lookup
# in a new step starts a new record list; a hipGraph replay runs no Python forward, so the
# captured id tensors (rewritten by every replay) stay recorded
_TOUCH_STEP = [0]


def mark_row_sparse(*params):
    """Sync these embedding tables' gradients row-sparsely (see module doc)."""
    for p in params:
        p._zoo_row_sparse = True
        p._zoo_touched = []
        p._zoo_touch_step = -1


def mark_row_sparse_embeddings(module):
    """Mark the table of every Keras ``Embedding`` layer inside ``module``."""
    from zoo.pipeline.api.keras.layers.embeddings import Embedding
    n = 0
    for m in module.modules():
        if isinstance(m, Embedding) and getattr(m, "embeddings", None) is not None:
            mark_row_sparse(m.embeddings)
            n += 1
    return n


def record_lookup(table, idx):
    """Called by the embedding ops: remember the ids looked up in ``table`` this step."""
    if not getattr(table, "_zoo_row_sparse", False):
        return
    if getattr(table, "_zoo_touch_step", -1) != _TOUCH_STEP[0]:
        table._zoo_touched = []
        table._zoo_touch_step = _TOUCH_STEP[0]
    table._zoo_touched.append(idx.detach().reshape(-1))


class _Bucket:
    __slots__ = ("idx", "lo", "hi", "params", "pending", "launched", "cb", "so", "pack", "recv", "gath",
                 "works", "post", "sparse")

    def __init__(self, idx, lo, hi):
        self.idx, self.lo, self.hi = idx, lo, hi
        self.params = []
        self.pending = 0
        self.launched = False
        self.cb = 0          # per-rank chunk (elements)
        self.so = 0          # offset of this bucket's chunk in the rank's shard
        self.pack = self.recv = self.gath = None
        self.works = []
        self.post = None
        self.sparse = []     # [(param, lo, hi)] when every parameter of the bucket is row-sparse


class GradSync:
    def __init__(self, flat: FlatParams, group=None, bucket_mb=16.0, mode="allreduce", overlap=True,
                 compress=None, force_comm=False):
        """``group``: the data-parallel process group (default: the world). With
        tensor parallelism it holds the ranks that share a tensor-parallel rank,
        so TP-sharded weights are only averaged over true replicas."""
        self.flat = flat
        self.compress = compress if compress in ("bf16",) else None
        self.group = group
        initialized = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if initialized else 1
        self.rank = dist.get_rank(group) if initialized else 0
        self.comm = initialized and (self.world > 1 or force_comm)
        self.backend = dist.get_backend(group) if initialized else None
        self.mode = mode if self.comm else "allreduce"
        self.is_cuda = flat.grad.is_cuda
        self.overlap = bool(overlap) and self.comm and self.is_cuda
        self.comm_stream = torch.cuda.Stream(device=flat.grad.device) if (self.is_cuda and self.comm) else None
        self._lock = threading.Lock()
        self.src = dist.get_global_rank(group, 0) if (initialized and group is not None) else 0
        # -- buckets over contiguous parameter ranges ---------------------------
        cap = max(int(bucket_mb * 1024 * 1024 / 4), 1)
        self.buckets = []
        self.param_bucket = {}
        cur = None
        prev_sparse = False
        for p, (lo, hi) in zip(flat.params, flat.ranges()):
            sp = bool(getattr(p, "_zoo_row_sparse", False)) and p.dim() == 2
            if cur is None or ((hi - cur.lo) > cap and cur.params) or sp or prev_sparse:
                cur = _Bucket(len(self.buckets), lo, hi)
                self.buckets.append(cur)
            cur.hi = hi
            cur.params.append(id(p))
            if sp:
                cur.sparse.append((p, lo, hi))
            self.param_bucket[id(p)] = cur
            prev_sparse = sp
        if self.buckets:
            self.buckets[-1].hi = flat.numel  # include the alignment tail
            self.buckets[0].lo = 0
            for a, b in zip(self.buckets, self.buckets[1:]):
                b.lo = a.hi
        so = 0
        for b in self.buckets:
            n = b.hi - b.lo
            b.cb = max((n + self.world - 1) // self.world, 1)
            b.cb = (b.cb + CHUNK_ALIGN - 1) // CHUNK_ALIGN * CHUNK_ALIGN
            b.so = so
            so += b.cb
        self.shard_size = so
        self._bufs = False
        self.shard_master = self.shard_grad = None
        # contribution counting (calibration) -----------------------------------
        self._counts = {}
        self._expected = None
        self._install_hooks()
        self.reset()

    # ------------------------------------------------------------------
    # persistent buffers
    def _wire_dtype(self):
        return torch.bfloat16 if self.compress else torch.float32

    def _ensure_buffers(self):
        if self._bufs or not self.comm:
            return
        dev = self.flat.grad.device
        need_pack = self.compress is not None or self.mode == "sharded"
        if need_pack:
            tot = sum(b.cb for b in self.buckets) * self.world
            pack = torch.zeros(tot, dtype=self._wire_dtype(), device=dev)
            recv = torch.empty(tot, dtype=torch.bfloat16, device=dev) if self.compress else None
            off = 0
            for b in self.buckets:
                n = b.cb * self.world
                b.pack = pack[off:off + n]
                if recv is not None:
                    b.recv = recv[off:off + n]
                off += n
        if self.mode == "allreduce" and self.compress:
            # bf16 sums of this rank's chunk, all-gathered into b.gath
            self._mine16 = torch.empty(self.shard_size, dtype=torch.bfloat16, device=dev)
            gath = torch.empty(sum(b.cb for b in self.buckets) * self.world, dtype=torch.bfloat16, device=dev)
            off = 0
            for b in self.buckets:
                n = b.cb * self.world
                b.gath = gath[off:off + n]
                off += n
        if self.mode == "sharded":
            self.shard_grad = torch.zeros(self.shard_size, dtype=torch.float32, device=dev)
            self.shard_master = torch.zeros(self.shard_size, dtype=torch.float32, device=dev)
            gath = torch.empty(sum(b.cb for b in self.buckets) * self.world, dtype=torch.float32, device=dev)
            off = 0
            for b in self.buckets:
                n = b.cb * self.world
                b.gath = gath[off:off + n]
                off += n
            self.load_shard_from_master()
        self._bufs = True

    def _chunk(self, b):
        """Global [lo, hi) of this rank's chunk of bucket b (may be empty)."""
        lo = b.lo + self.rank * b.cb
        return lo, max(lo, min(lo + b.cb, b.hi))

    def load_shard_from_master(self):
        """Copy this rank's owned fp32 masters out of the full flat buffer."""
        if self.shard_master is None:
            return
        self.shard_master.zero_()
        for b in self.buckets:
            lo, hi = self._chunk(b)
            if hi > lo:
                self.shard_master[b.so:b.so + hi - lo].copy_(self.flat.master[lo:hi])

    def shard_range(self, glo, ghi):
        """Map a global flat range onto this rank's shard: (slo, shi) or None.
        Between two buckets' chunks the shard is contiguous (padding slots of a
        short last chunk included, which hold zero gradient and weight)."""
        first = last = None
        for b in self.buckets:
            lo, hi = self._chunk(b)
            a, z = max(lo, glo), min(hi, ghi)
            if a < z:
                s0, s1 = b.so + a - lo, b.so + z - lo
                first = s0 if first is None else first
                last = s1
        return None if first is None else (first, last)

    # ------------------------------------------------------------------
    # readiness tracking
    def _install_hooks(self):
        for p in self.flat.params:
            p._zoo_grad_ready = self._ready
            old = getattr(p, "_zoo_sync_hook", None)
            if old is not None:  # a previous engine over the same model: its hook must not fire
                old.remove()
            if hasattr(p, "register_post_accumulate_grad_hook"):
                p._zoo_sync_hook = p.register_post_accumulate_grad_hook(self._ready)

    def reset(self):
        self._counts = {}
        _TOUCH_STEP[0] += 1
        for b in self.buckets:
            if self._expected is None or b.sparse:
                b.pending = -1  # calibration step / row-sparse bucket: launched by finish()
            else:
                b.pending = sum(1 for pid in b.params if self._expected.get(pid, 0) > 0)
            b.launched = False
            b.works = []
            b.post = None

    def _ready(self, p):
        if not self.comm:
            return
        with self._lock:
            pid = id(p)
            c = self._counts.get(pid, 0) + 1
            self._counts[pid] = c
            if not self.overlap or self._expected is None:
                return
            b = self.param_bucket.get(pid)
            if b is None:
                return
            exp = self._expected.get(pid, 0)
            if c > exp:
                if b.launched:
                    raise RuntimeError(
                        "GradSync: parameter %s got %d gradient contributions this step but %d in the "
                        "calibration step, after its bucket was launched; dynamic graphs need "
                        "overlap_comm=False (ZOO_OVERLAP_COMM=0)" % (tuple(p.shape), c, exp))
                b.pending = -1  # never launch this bucket early again this step
                return
            if c == exp and b.pending > 0:
                b.pending -= 1
                if b.pending == 0:
                    self._launch(b)

    # ------------------------------------------------------------------
    # collectives
    def _launch(self, b):
        self._ensure_buffers()
        b.launched = True
        if self.comm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.grad.device))
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                self._issue(b)
        else:
            self._issue(b)

    def _a2a(self, out, inp):
        if self.backend == "gloo":  # gloo has no all-to-all: gather every pack, keep our chunk of each
            parts = [torch.empty_like(inp) for _ in range(self.world)]
            dist.all_gather(parts, inp, group=self.group)
            cb = inp.numel() // self.world
            for w, t in enumerate(parts):
                out[w * cb:(w + 1) * cb].copy_(t[self.rank * cb:(self.rank + 1) * cb])
            return
        dist.all_to_all_single(out, inp, group=self.group)

    def _gather(self, out, mine):
        if self.backend == "gloo":
            parts = list(out.chunk(self.world))
            dist.all_gather(parts, mine, group=self.group)
            return
        dist.all_gather_into_tensor(out, mine, group=self.group)

    def _rs_fp32(self, out, inp):
        if self.backend == "gloo":
            dist.all_reduce(inp, group=self.group)
            out.copy_(inp[self.rank * out.numel():(self.rank + 1) * out.numel()])
            return
        dist.reduce_scatter_tensor(out, inp, group=self.group)

    def _sum_chunks(self, recv, out32=None, out16=None):
        if recv.is_cuda:
            from zoo.ops._native import native
            native().sum_chunks_bf16(recv, self.world, out32, out16, 1.0)
            return
        s = recv.view(self.world, -1).float().sum(0)
        if out32 is not None:
            out32.copy_(s)
        if out16 is not None:
            out16.copy_(s)

    def _row_sparse_allreduce(self, p, lo, hi):
        """Sum table p's gradient over the ranks through the union of looked-up rows
        (False: no lookup was recorded, the caller reduces the dense range)."""
        touched = getattr(p, "_zoo_touched", None)
        if not touched:
            return False
        V, D = p.shape
        g = self.flat.grad[lo:lo + V * D].view(V, D)
        dev = g.device
        ids = torch.cat([t.to(dev).long() for t in touched])
        u = torch.unique(ids[(ids >= 0) & (ids < V)])
        cnt = torch.tensor([u.numel()], device=dev, dtype=torch.long)
        cnts = [torch.empty_like(cnt) for _ in range(self.world)]
        dist.all_gather(cnts, cnt, group=self.group)
        m = int(max(int(c.item()) for c in cnts))
        if m == 0:
            return True
        pad = torch.full((m,), V, device=dev, dtype=torch.long)
        pad[:u.numel()] = u
        allids = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(allids, pad, group=self.group)
        union = torch.unique(torch.cat(allids))
        union = union[union < V]
        rows = g.index_select(0, union)
        dist.all_reduce(rows, group=self.group)
        g.index_copy_(0, union, rows)
        self.sparse_rows = getattr(self, "sparse_rows", 0) + int(union.numel())
        return True

    def _issue(self, b):
        """Enqueue bucket b's reduction on the current (comm) stream. Every step
        after a collective that consumes its result waits on the device only."""
        g = self.flat.grad[b.lo:b.hi]
        n = b.hi - b.lo
        if self.mode == "allreduce" and not self.compress:
            if b.sparse and all(self._row_sparse_allreduce(p, lo, hi) for p, lo, hi in b.sparse):
                return
            dist.all_reduce(g, group=self.group)
            return
        lo, hi = self._chunk(b)
        if self.compress:
            b.pack[:n].copy_(g)                     # fp32 -> bf16 pack (padding stays 0)
            self._a2a(b.recv, b.pack)
            if self.mode == "sharded":
                self._sum_chunks(b.recv, out32=self.shard_grad[b.so:b.so + b.cb])
            else:
                mine = self._mine16[b.so:b.so + b.cb]
                self._sum_chunks(b.recv, out16=mine)
                self._gather(b.gath, mine)
                g.copy_(b.gath[:n])                 # bf16 sums -> fp32 flat gradient
            return
        # sharded, fp32 wire
        b.pack[:n].copy_(g)
        self._rs_fp32(self.shard_grad[b.so:b.so + b.cb], b.pack)

    # ------------------------------------------------------------------
    def broadcast_parameters(self, src=None):
        """CC5: model weights from the group's first rank (or global rank ``src``)
        to every rank of the data-parallel group (RCCL broadcast)."""
        if self.comm and self.world > 1:
            dist.broadcast(self.flat.master, self.src if src is None else src, group=self.group)
        self.flat.refresh_bf16()
        if self.shard_master is not None:
            self.load_shard_from_master()

    def finish(self):
        """Called after backward: launch what is left, make the compute stream
        wait for every bucket's collectives."""
        if not self.comm:
            return
        if self._expected is None:  # end of the calibration step
            self._expected = dict(self._counts)
        for b in self.buckets:
            if not b.launched:
                self._launch(b)
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(self.comm_stream)

    def step(self, optim, clip=None):
        """finish comm, (clip), run the optimizer."""
        flat = self.flat
        gscale = 1.0 / self.world
        if self.mode == "sharded" and self.comm:
            self.finish()
            self._sharded_step(optim, gscale, clip)
        else:
            self.finish()
            if clip is not None:
                clip(flat.grad, gscale, self)
            optim.step(flat.master, flat.grad, flat.bf16, gscale)
        self.reset()

    def _sharded_step(self, optim, gscale, clip):
        flat = self.flat
        if clip is not None:
            clip(self.shard_grad, gscale, self)
        if getattr(optim, "parts", None) is not None:   # MultiOptimMethod: per-part shard ranges
            optim.step_ranges([(self.shard_range(lo, hi), o) for _, o, lo, hi in optim.parts],
                              self.shard_master, self.shard_grad, None, gscale)
        else:
            optim.step(self.shard_master, self.shard_grad, None, gscale)
        # all-gather the updated fp32 master shards straight back into the full flat buffer
        # (per bucket, on the comm stream), then ONE cast pass refreshes the bf16 compute copy.
        # The fp32 masters are gathered (not only 16-bit weights) because layers read fp32
        # parameters directly (BN gamma/beta, biases, embeddings): every rank must see the
        # same values, bit for bit.
        stream = self.comm_stream
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(flat.master.device))
            with torch.cuda.stream(stream):
                self._gather_masters()
            torch.cuda.current_stream(flat.master.device).wait_stream(stream)
        else:
            self._gather_masters()
        flat.refresh_bf16()

    def _gather_masters(self):
        flat = self.flat
        for b in self.buckets:
            self._gather(b.gath, self.shard_master[b.so:b.so + b.cb])
            flat.master[b.lo:b.hi].copy_(b.gath[:b.hi - b.lo])

    def sync_master(self):
        """Kept for API compatibility: the fp32 masters are gathered every step."""
        return

    def all_reduce_scalars(self, values):
        """CC4/CC6: batch small metric/loss reductions into ONE all-reduce."""
        t = torch.as_tensor(values, dtype=torch.float64, device=self.flat.grad.device)
        if self.comm and self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def agree(self, flag):
        """Cross-rank failure agreement: 1 if ANY rank passes a true flag."""
        if not (self.comm and self.world > 1):
            return int(bool(flag))
        t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float32,
                         device=self.flat.grad.device if self.backend != "gloo" else "cpu")
        dist.all_reduce(t, group=self.group)
        return int(t.item() > 0)


def global_norm_clip(max_norm):
    """L2-norm gradient clipping across ranks (Estimator.scala:137-150, CC4)."""
    from zoo.ops._native import native

    def _clip(g, gscale, sync):
        if g.is_cuda:
            ss = native().sumsq(g)
        else:
            ss = (g.float() ** 2).sum().reshape(1)
        if sync.comm and sync.world > 1 and sync.mode == "sharded":
            dist.all_reduce(ss, group=sync.group)
        # gradients are summed over ranks; the optimizer applies gscale later
        scale_sq = gscale * gscale
        ss = ss * scale_sq
        if g.is_cuda:
            native().clip(g, -3.4e38, 3.4e38, ss, float(max_norm))
        else:
            nrm = ss.sqrt().item()
            if nrm > max_norm:
                g.mul_(max_norm / (nrm + 1e-6))
    return _clip


def constant_clip(lo, hi):
    from zoo.ops._native import native

    def _clip(g, gscale, sync):
        # bounds apply to the averaged gradient: scale them to the summed buffer
        s = 1.0 / gscale
        if g.is_cuda:
            native().clip(g, lo * s, hi * s, None, 0.0)
        else:
            g.clamp_(lo * s, hi * s)
    return _clip
