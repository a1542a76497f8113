"""Data-parallel gradient synchronisation over RCCL (xGMI) — one process per GPU.

This replaces BigDL's Spark-BlockManager ``AllReduceParameter`` (SURVEY.md
§2.4 "DistriOptimizer iteration", §2.17 CC1-CC4; Topology.scala:1128-1206,
docs/docs/wp-bigdl.md:140-160):

* Gradients live in ONE flat fp32 buffer (:class:`FlatParams`) laid out in
  backward order and cut into contiguous buckets (``bucket_mb``, 32 MB by
  default: big enough for full per-link bandwidth on xGMI, small enough that
  the last bucket -- launched when backward ends -- is a short exposed tail).
* The wire format defaults to bf16 on the GPU (``compress="auto"``; BigDL ships
  16-bit gradient chunks, wp-bigdl.md:140-160), fp32 on gloo/CPU.
* A bucket is launched on a dedicated comm stream (waiting on an event of the
  compute stream) as soon as EVERY gradient contribution of its parameters has
  been enqueued. The number of contributions per parameter is learned in the
  first (calibration) step, in which nothing launches early: a weight used
  twice (shared Keras layers, siamese KNRM/TextMatcher, tied embeddings)
  triggers its bucket only after its second contribution. A later step that
  adds MORE contributions than calibrated raises instead of reducing a partial
  gradient (collectives cannot be recalled). The single-rank in-backward
  optimizer (``enable_ibo``) never raises: it calibrates over two steps, updates
  in-backward only buckets whose counts agreed in both, and moves a bucket that
  later breaks its count to the end-of-step update for the rest of the run.
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

Ordering (every rank must issue the same collectives in the same order): the calibration
step records the order in which buckets BECOME ready (the sequence number of each parameter's
last contribution); later steps launch early in that order, and ``finish()`` launches whatever
is left -- including all buckets of a zombie rank that failed part-way through backward -- in
that same recorded order, so a zombie's collective sequence matches the healthy ranks'.

Row-sparse sync (fp32 wire, or the 16-bit wire of the dense buckets for the union rows): each rank scatters a per-row "touched" mask (uint8, V bytes; int32 at >= 256
ranks), the masks are summed (one all-reduce), the union rows are compacted on the device into a
fixed-capacity index buffer (capacity min(V, world * ids-per-step), agreed in the calibration
step) and ONE fixed-size all-reduce moves just those rows. A rank without lookups contributes a
zero mask, so every rank always issues the same collectives. A rank that looks up more ids than
agreed raises a flag carried in the same mask all-reduce; every rank reads the summed flag and
falls back to the dense all-reduce together for that step. Tables whose capacity reaches V/2 are
always reduced densely (the mask + rows would move more than the dense table).

ZeRO-1 weight all-gather: the updated shards go out as bf16 (half of BigDL's fp32 bytes are
not needed for the bf16 compute copy); the 1-D parameters that layers read in fp32 (BatchNorm
gamma/beta, biases) are reassembled exactly with one small fp32 all-reduce, and the fp32 view
of every other parameter is the bf16 value on EVERY rank (identical across ranks; the exact
fp32 masters live in the owners' shards and are gathered in full only for checkpoints,
``sync_master``).

All persistent comm buffers are allocated once (chunk = ceil(bucket/N) rounded
to 64 elements). ``force_comm`` runs the whole bucket / comm-stream / event
path on a world-size-1 process group (RCCL with one rank), so the overlapped
code is exercised on a single GPU (``ZOO_FORCE_COMM=1``).

Gradient averaging (1/N) is folded into the optimizer kernel's ``gscale``.
On CPU (gloo) the same code runs synchronously; that is what the
multi-process CPU tests exercise.
"""
import logging
import threading

import torch
import torch.distributed as dist

from zoo.parallel.flat import FlatParams
from zoo.ops import wstream

CHUNK_ALIGN = 64
log = logging.getLogger("zoo")
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
                 "works", "post", "sparse", "gath16", "ev0", "ev1", "ibo_off", "carry", "carry_late")

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
        self.gath16 = None   # ZeRO-1 bf16 weight all-gather target
        self.carry = None    # in-backward optimizer: a late gradient contribution for the next update
        self.carry_late = False
        self.ev0 = self.ev1 = None  # comm-stream events around the bucket's collectives (stats)
        self.ibo_off = False        # in-backward update switched off (counts not stable)


class GradSync:
    def __init__(self, flat: FlatParams, group=None, bucket_mb=16.0, mode="allreduce", overlap=True,
                 compress=None, force_comm=False, comm="torch", rccl_channels=0):
        """``group``: the data-parallel process group (default: the world). With
        tensor parallelism it holds the ranks that share a tensor-parallel rank,
        so TP-sharded weights are only averaged over true replicas."""
        self.flat = flat
        self.group = group
        initialized = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if initialized else 1
        self.rank = dist.get_rank(group) if initialized else 0
        self.comm = initialized and (self.world > 1 or force_comm)
        self.backend = dist.get_backend(group) if initialized else None
        if compress == "auto":   # BigDL's 16-bit gradient chunks on the GPU path, exact fp32 on gloo/CPU
            compress = "bf16" if (self.comm and flat.grad.is_cuda) else None
        self.compress = compress if compress in ("bf16",) else None
        self.mode = mode if self.comm else "allreduce"
        self.is_cuda = flat.grad.is_cuda
        self.overlap = bool(overlap) and self.comm and self.is_cuda
        self.comm_stream = torch.cuda.Stream(device=flat.grad.device) if (self.is_cuda and self.comm) else None
        # bucket collectives through the C++ comm layer (zoo/parallel/comm.py) instead of the
        # ProcessGroup: same stream, same order, no per-call work objects
        self.ncomm = None
        if comm == "native" and self.comm and self.is_cuda:
            from zoo.parallel.comm import NativeComm, native_comm_ok
            if native_comm_ok(group):
                with torch.cuda.device(flat.grad.device):
                    self.ncomm = NativeComm(group, rccl_channels)
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
        self._seq = 0
        self._last_seq = {}
        self.order = None          # bucket launch order learned in the calibration step
        self.launch_log = []       # bucket indices in the order this step launched them
        # row-sparse capacity (rows) per table, agreed in the calibration step
        self._sparse_cap = {}
        # ZeRO-1: flat ranges of the 1-D (fp32-read) parameters, gathered exactly in fp32
        self._small_idx = None
        self._small_buf = None
        # comm statistics (bench.py at N > 1): exposed wait + per-bucket collective time
        self.collect_stats = False
        self.stats = {"steps": 0, "exposed_ms": 0.0, "bucket_ms": {}, "bucket_bytes": {}}
        self._wait_ev = None
        # in-backward optimizer (world 1, see enable_ibo): each bucket's update is issued on the
        # weight-gradient side stream as soon as its last gradient contribution is in
        self.ibo_optim = None
        self.ibo_steps = 0
        self._ibo_done = set()
        self._ibo_cleared = True
        self._ibo_calib1 = None     # contribution counts of the first calibration step
        self._ibo_hooks = []
        # set by the TrainingEngine: gradients written while no engine step runs (a user's own
        # loss.backward(), another driver) invalidate FlatParams.grad_clean and are not counted
        self.engine_managed = False
        self.in_step = False
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
            tot = sum(b.cb for b in self.buckets) * self.world
            gath = torch.empty(tot, dtype=torch.float32, device=dev)      # checkpoint-time fp32 gather
            gath16 = torch.empty(tot, dtype=torch.bfloat16, device=dev)   # per-step bf16 weight gather
            self._shard16 = torch.empty(self.shard_size, dtype=torch.bfloat16, device=dev)
            off = 0
            for b in self.buckets:
                n = b.cb * self.world
                b.gath = gath[off:off + n]
                b.gath16 = gath16[off:off + n]
                off += n
            # parameters the layers read in fp32 travel exactly: every parameter that no native
            # kernel read through its bf16 compute copy (``_zoo_bf16_read``, set by the conv / linear
            # / embedding / NCF ops in the calibration forward) -- BN gamma/beta, biases, fp32
            # embedding tables (compute_dtype=None), fp32 torch layers of the Keras/AutoML fallbacks
            idx = []
            for p, (lo, hi) in zip(self.flat.params, self.flat.ranges()):
                if p.dim() <= 1 or not getattr(p, "_zoo_bf16_read", False):
                    idx.append(torch.arange(lo, hi, dtype=torch.long))
            if idx and self.flat.bf16 is not None:
                self._small_idx = torch.cat(idx).to(dev)
                self._small_buf = torch.zeros(self._small_idx.numel(), dtype=torch.float32, device=dev)
                own = torch.zeros(self.flat.numel, dtype=torch.bool)
                for b in self.buckets:
                    lo, hi = self._chunk(b)
                    own[lo:hi] = True
                self._small_own = own[self._small_idx.cpu()].to(dev)
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

    def enable_ibo(self, optim):
        """In-backward optimizer for a single-rank job: the update of bucket b runs on the
        weight-gradient side stream (zoo.ops.wstream) once every parameter of b has received
        the gradient contributions counted in the calibration step, overlapping the backward of
        the remaining layers (a layer's weights are never read again in a backward after their
        last gradient contribution). ``optim`` must support element ranges (supports_ranges)."""
        if self.comm or not self.is_cuda:
            return False
        self.ibo_optim = optim
        for h in self._ibo_hooks:
            h.remove()
        self._ibo_hooks = []
        for p in self.flat.params:
            # native ops announce a gradient write before they enqueue it (flat.grad_slot);
            # autograd-accumulated parameters through a tensor hook, which runs BEFORE the
            # accumulation kernel is issued
            p._zoo_grad_pre = self._ibo_pre
            self._ibo_hooks.append(p.register_hook(lambda g, p=p: self._ibo_pre(p)))
        return True

    def _ibo_pre(self, p):
        """A gradient write into p's slot is about to be enqueued on the current stream. If
        p's bucket was already updated in-backward this step, that write must not overlap the
        side-stream update that reads and clears the slot: order it after the update."""
        if self.ibo_optim is None or not self.in_step:
            return
        b = self.param_bucket.get(id(p))
        if b is not None and b.launched:
            dev = self.flat.grad.device
            cur = torch.cuda.current_stream(dev)
            side = wstream.side_for(dev)
            if cur != side:
                cur.wait_stream(side)

    def reset(self):
        self._counts = {}
        self._ibo_done = set()
        _TOUCH_STEP[0] += 1
        for b in self.buckets:
            if self._expected is None or b.sparse or b.ibo_off:
                # calibration step / row-sparse bucket / in-backward update switched off for the
                # bucket: launched (updated) by finish() / step()
                b.pending = -1
            else:
                b.pending = sum(1 for pid in b.params if self._expected.get(pid, 0) > 0)
            b.launched = False
            b.works = []
            b.post = None
        self.launch_log = []

    def _ready(self, p):
        if self.engine_managed and not self.in_step:
            # a gradient written outside an engine step: the slots are no longer known clear
            self.flat.grad_clean = False
            return
        if not self.comm:
            if self.ibo_optim is not None:
                self._ibo_ready(p)
            return
        with self._lock:
            pid = id(p)
            c = self._counts.get(pid, 0) + 1
            self._counts[pid] = c
            self._seq += 1
            self._last_seq[pid] = self._seq
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
        self.launch_log.append(b.idx)
        if self.comm_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.flat.grad.device))
            side = wstream.pending(self.flat.grad.device)
            with torch.cuda.stream(self.comm_stream):
                self.comm_stream.wait_event(ev)
                if side is not None:   # weight gradients still running on the side stream
                    self.comm_stream.wait_stream(side)
                if self.collect_stats:
                    b.ev0 = torch.cuda.Event(enable_timing=True)
                    b.ev1 = torch.cuda.Event(enable_timing=True)
                    b.ev0.record(self.comm_stream)
                self._issue(b)
                if self.collect_stats:
                    b.ev1.record(self.comm_stream)
        else:
            self._issue(b)

    def _a2a(self, out, inp):
        if self.ncomm is not None:
            self.ncomm.all_to_all(out, inp)
            return
        if self.backend == "gloo":  # gloo has no all-to-all: gather every pack, keep our chunk of each
            parts = [torch.empty_like(inp) for _ in range(self.world)]
            dist.all_gather(parts, inp, group=self.group)
            cb = inp.numel() // self.world
            for w, t in enumerate(parts):
                out[w * cb:(w + 1) * cb].copy_(t[self.rank * cb:(self.rank + 1) * cb])
            return
        dist.all_to_all_single(out, inp, group=self.group)

    def _gather(self, out, mine):
        if self.ncomm is not None:
            self.ncomm.all_gather(out, mine)
            return
        if self.backend == "gloo":
            parts = list(out.chunk(self.world))
            dist.all_gather(parts, mine, group=self.group)
            return
        dist.all_gather_into_tensor(out, mine, group=self.group)

    def _rs_fp32(self, out, inp):
        if self.ncomm is not None:
            self.ncomm.reduce_scatter(out, inp)
            return
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

    def _touched_ids(self, p):
        touched = getattr(p, "_zoo_touched", None) or []
        if getattr(p, "_zoo_touch_step", -1) != _TOUCH_STEP[0]:
            touched = []
        return touched

    def _sparse_capacity(self, p, n_local):
        """(rows the fixed-size union buffer holds, agreed ids-per-rank), agreed once (calibration)
        with a MAX all-reduce of the per-rank id counts: capacity min(V, world * ids-per-step).
        Capacity ``None`` = the union can cover half the table or more: the row-sparse protocol
        (a V-sized mask all-reduce plus the rows) would move MORE than the dense all-reduce, so
        the table is reduced densely (e.g. NCF ml-20m at b65536 x 8 ranks: capacity >= V)."""
        key = id(p)
        cap = self._sparse_cap.get(key)
        if cap is None:
            dev = self.flat.grad.device if self.backend != "gloo" else torch.device("cpu")
            t = torch.tensor([n_local], dtype=torch.long, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
            n_max = int(t.item())
            rows = min(p.shape[0], max(n_max, 1) * self.world)
            cap = (rows if 2 * rows < p.shape[0] else None, n_max)
            self._sparse_cap[key] = cap
        return cap

    def _rows16_allreduce(self, rows):
        """Sum a [cap, D] fp32 row block over the ranks on the 16-bit wire: the dense buckets'
        protocol (bf16 pack, all-to-all, fp32 sum of this rank's chunk, all-gather of the bf16
        sums), so the row-sparse path moves half the bytes of its fp32 form."""
        n = rows.numel()
        cb = (n + self.world - 1) // self.world
        cb = (cb + CHUNK_ALIGN - 1) // CHUNK_ALIGN * CHUNK_ALIGN
        pack = torch.zeros(cb * self.world, dtype=torch.bfloat16, device=rows.device)
        pack[:n].copy_(rows.reshape(-1))
        recv = torch.empty_like(pack)
        self._a2a(recv, pack)
        mine = torch.empty(cb, dtype=torch.bfloat16, device=rows.device)
        self._sum_chunks(recv, out16=mine)
        gath = torch.empty_like(pack)
        self._gather(gath, mine)
        return gath[:n].view_as(rows).float()

    def _row_sparse_allreduce(self, p, lo, hi):
        """Sum table p's gradient over the ranks through the union of looked-up rows: a summed
        uint8 touched mask, device-side compaction into a fixed-capacity row list, one fixed-size
        all-reduce of those rows. One small host read per step (the summed overflow flag, which
        picks the dense fallback identically on every rank), and the same collectives on every
        rank whatever it looked up (an idle rank sends a zero mask). Runs on the fp32 wire only:
        with the bf16 wire (``compress``, the GPU default) the bucket takes the dense path."""
        V, D = p.shape
        g = self.flat.grad[lo:lo + V * D].view(V, D)
        dev = g.device
        touched = self._touched_ids(p)
        n_local = int(sum(t.numel() for t in touched))
        cap, n_max = self._sparse_capacity(p, n_local)
        if cap is None:                       # dense wins (decided identically on every rank)
            dist.all_reduce(g, group=self.group)
            return False
        # uint8 sums wrap at 256 ranks; gloo has no uint8 sum
        mdt = torch.uint8 if (self.backend != "gloo" and self.world < 256) else torch.int32
        mask = torch.zeros(V + 1, dtype=mdt, device=dev)
        if touched:
            ids = torch.cat([t.to(dev).long() for t in touched])
            ids = ids[(ids >= 0) & (ids < V)] if not ids.is_cuda else ids.clamp(0, V - 1)
            mask[:V].index_fill_(0, ids, 1)
        # slot V: this rank looked up more ids than agreed (variable-length ids, a larger batch than
        # the calibration batch) -> the union could overflow the capacity. The flag travels in the
        # mask all-reduce, so every rank sees the same sum and takes the same branch below.
        if n_local > n_max:
            mask[V] = 1
        dist.all_reduce(mask, group=self.group)
        if bool(mask[V].item()):   # one small host read per step: the price of a collective decision
            dist.all_reduce(g, group=self.group)  # every rank: dense fallback for this step
            return False
        mask = mask[:V]
        on = mask > 0
        pos = torch.cumsum(on.to(torch.int32), 0) - 1
        slot = torch.where(on, pos.long(), torch.full_like(pos, cap, dtype=torch.long))
        slot = slot.clamp(max=cap)
        buf = torch.full((cap + 1,), V, dtype=torch.long, device=dev)
        buf.scatter_(0, slot, torch.arange(V, device=dev))
        rows_idx = buf[:cap]
        first = rows_idx[:1].clamp(max=V - 1)
        rows_idx = torch.where(rows_idx < V, rows_idx, first)   # padding slots repeat the first row
        rows = g.index_select(0, rows_idx)
        if self.compress:
            rows = self._rows16_allreduce(rows)
        else:
            dist.all_reduce(rows, group=self.group)
        g.index_copy_(0, rows_idx, rows)
        self.sparse_rows = getattr(self, "sparse_rows", 0) + cap
        return True

    def _issue(self, b):
        """Enqueue bucket b's reduction on the current (comm) stream. Every step
        after a collective that consumes its result waits on the device only."""
        g = self.flat.grad[b.lo:b.hi]
        n = b.hi - b.lo
        if self.mode == "allreduce" and b.sparse:
            # always the sparse protocol (fp32 or 16-bit wire): identical collectives on every rank
            for p, plo, phi in b.sparse:
                self._row_sparse_allreduce(p, plo, phi)
            return
        if self.mode == "allreduce" and not self.compress:
            if self.ncomm is not None:
                self.ncomm.all_reduce(g)
            else:
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

    def _ibo_ready(self, p):
        pid = id(p)
        c = self._counts.get(pid, 0) + 1
        self._counts[pid] = c
        if self._expected is None:
            return   # calibration steps: counting only
        b = self.param_bucket.get(pid)
        if b is None:
            return
        exp = self._expected.get(pid, 0)
        if c > exp:
            # checked before the pending test: a launched bucket has pending 0
            if not b.ibo_off:
                self._ibo_disable(b, p, c, exp)
            return
        if b.pending <= 0:
            return
        if c == exp:
            b.pending -= 1
            if b.pending == 0:
                self._ibo_launch(b)

    def _ibo_disable(self, b, p, c, exp):
        """p got more gradient contributions than calibrated: bucket b is updated at the end of
        every later step. Not yet updated this step -> the end-of-step update sees the whole
        gradient. Already updated -> the late contribution was ordered behind the update
        (_ibo_pre) and lands in the cleared slot; the end of the step saves it (``b.carry``) and
        the bucket's next update adds it in: nothing is lost or applied twice, the late part of
        this one step arrives one update later."""
        b.ibo_off = True
        if b.launched:
            self._ibo_cleared = False
            b.carry_late = True
            log.warning("in-backward optimizer: parameter %s got %d gradient contributions, %d calibrated, "
                        "after its bucket was updated; this step's late contribution is applied with the "
                        "next update and the bucket is updated at the end of each step from now on "
                        "(ZOO_OPTIM_IN_BWD=0 turns the in-backward update off)", tuple(p.shape), c, exp)
        else:
            b.pending = -1
            log.warning("in-backward optimizer: parameter %s got %d gradient contributions, %d calibrated; "
                        "its bucket is updated at the end of each step from now on", tuple(p.shape), c, exp)

    def _ibo_launch(self, b):
        from zoo.ops import wstream
        flat, dev = self.flat, self.flat.grad.device
        side = wstream.side_for(dev) if wstream.active(dev) else None
        if side is None:
            return   # outside the engine's backward scope: step() updates it
        side.wait_stream(torch.cuda.current_stream(dev))   # BN / bias gradients written on the compute stream
        with torch.cuda.stream(side):
            cl = self.ibo_optim.step_range(flat.master, flat.grad, flat.bf16, 1.0, b.lo, b.hi, zero_grad=True)
        self._ibo_cleared = self._ibo_cleared and bool(cl)
        wstream.mark_used(dev)
        b.launched = True
        self._ibo_done.add(b.idx)

    def _ibo_step(self):
        """End of an in-backward-optimizer step: update the buckets not launched during the
        backward (calibration step, extra contributions, no gradient), then bump the counters."""
        flat = self.flat
        if self._expected is None:
            # two calibration steps: a bucket whose parameters' contribution counts differ
            # between them (a layer used a variable number of times) is never updated in-backward
            if self._ibo_calib1 is None:
                self._ibo_calib1 = dict(self._counts)
            else:
                self._expected = dict(self._counts)
                for b in self.buckets:
                    if any(self._ibo_calib1.get(pid, 0) != self._expected.get(pid, 0) for pid in b.params):
                        b.ibo_off = True
        cleared = True
        for b in self.buckets:
            if b.idx not in self._ibo_done:
                carry = getattr(b, "carry", None)
                if carry is not None:   # a late contribution of the previous step (_ibo_disable)
                    flat.grad[b.lo:b.hi].add_(carry)
                    b.carry = None
                cleared &= bool(self.ibo_optim.step_range(flat.master, flat.grad, flat.bf16, 1.0, b.lo, b.hi,
                                                          zero_grad=True))
            elif getattr(b, "carry_late", False):
                # updated in-backward before the late contribution arrived: the slot holds only
                # that contribution; keep it for this bucket's next (end-of-step) update
                b.carry = flat.grad[b.lo:b.hi].clone()
                b.carry_late = False
        flat.grad_clean = cleared and self._ibo_cleared
        self._ibo_cleared = True
        self.ibo_optim.finish_step(flat.bf16 is not None)
        self.ibo_steps += 1

    def finish(self):
        """Called after backward: launch what is left, make the compute stream
        wait for every bucket's collectives."""
        if not self.comm:
            return
        calib = self._expected is None
        order = self.order if self.order is not None else range(len(self.buckets))
        for i in order:
            b = self.buckets[i]
            if not b.launched:
                self._launch(b)
        if calib:  # end of the calibration step: learn counts and the readiness order
            self._expected = dict(self._counts)
            self.order = self._readiness_order()
        if self.comm_stream is not None:
            cur = torch.cuda.current_stream(self.flat.grad.device)
            if self.collect_stats:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(cur)
                cur.wait_stream(self.comm_stream)
                e1.record(cur)
                self._wait_ev = (e0, e1)
            else:
                cur.wait_stream(self.comm_stream)

    def _readiness_order(self):
        """Bucket launch order of every later step: buckets that launch early, by the sequence
        number of their last gradient contribution; then the ones only finish() launches
        (row-sparse, no contributions) by index -- exactly what a healthy rank does."""
        early, late = [], []
        for b in self.buckets:
            seqs = [self._last_seq.get(pid, 0) for pid in b.params if self._expected.get(pid, 0) > 0]
            if b.sparse or not seqs:
                late.append(b.idx)
            else:
                early.append((max(seqs), b.idx))
        return [i for _, i in sorted(early)] + late

    def wait_comm(self):
        """Make the current stream wait for everything issued on the comm stream (a zombie
        rank calls this before zeroing gradients that in-flight collectives may still read)."""
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.flat.grad.device).wait_stream(self.comm_stream)

    def collect_comm_stats(self):
        """Fold this step's events into ``self.stats`` (synchronises on the events)."""
        if not self.collect_stats or self.comm_stream is None:
            return
        if self._wait_ev is not None:
            e0, e1 = self._wait_ev
            e1.synchronize()
            self.stats["exposed_ms"] += e0.elapsed_time(e1)
            self._wait_ev = None
        for b in self.buckets:
            if b.ev0 is not None and b.ev1 is not None:
                b.ev1.synchronize()
                self.stats["bucket_ms"][b.idx] = self.stats["bucket_ms"].get(b.idx, 0.0) + b.ev0.elapsed_time(b.ev1)
                self.stats["bucket_bytes"][b.idx] = (b.hi - b.lo) * (2 if self.compress else 4)
                b.ev0 = b.ev1 = None
        self.stats["steps"] += 1

    def comm_summary(self):
        """exposed comm ms/step and per-bucket algorithm / bus bandwidth (GB/s)."""
        st = self.stats
        n = max(st["steps"], 1)
        out = {"exposed_comm_ms_per_step": round(st["exposed_ms"] / n, 3), "buckets": []}
        k = 2.0 * (self.world - 1) / self.world if self.world > 1 else 0.0
        for i in sorted(st["bucket_ms"]):
            ms = st["bucket_ms"][i] / n
            by = st["bucket_bytes"].get(i, 0)
            alg = by / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
            out["buckets"].append({"bucket": i, "bytes": by, "MB": round(by / 1e6, 3), "ms": round(ms, 3),
                                   "algbw_GBs": round(alg, 1), "busbw_GBs": round(alg * k, 1)})
        return out

    def step(self, optim, clip=None):
        """finish comm, (clip), run the optimizer."""
        flat = self.flat
        gscale = 1.0 / self.world
        if self.ibo_optim is not None and optim is self.ibo_optim and clip is None:
            self._ibo_step()
            self.reset()
            return
        if self.mode == "sharded" and self.comm:
            self.finish()
            self._sharded_step(optim, gscale, clip)
        else:
            self.finish()
            if clip is not None:
                clip(flat.grad, gscale, self)
            if getattr(optim, "_native_zero_grad", False) and flat.grad.is_cuda:
                # the optimizer kernel clears each gradient slot after reading it
                flat.grad_clean = bool(optim.step(flat.master, flat.grad, flat.bf16, gscale, zero_grad=True))
            else:
                optim.step(flat.master, flat.grad, flat.bf16, gscale)
        if self.collect_stats:
            self.collect_comm_stats()
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
        # all-gather the updated shards. The bf16 compute copy is gathered directly (2 bytes per
        # parameter on the wire instead of BigDL's fp32 4); the 1-D fp32-read parameters get
        # their exact fp32 values from one small all-reduce; every other fp32 master view
        # becomes the (rank-identical) bf16 value. Without a bf16 compute copy (CPU) the fp32
        # masters are gathered as before.
        stream = self.comm_stream
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(flat.master.device))
            with torch.cuda.stream(stream):
                self._gather_weights()
            torch.cuda.current_stream(flat.master.device).wait_stream(stream)
        else:
            self._gather_weights()
        from zoo.ops._kern import bump_weights_epoch
        bump_weights_epoch()

    def _gather_weights(self):
        flat = self.flat
        if flat.bf16 is None or not flat.master.is_cuda:
            # CPU (gloo) / no compute copy: the layers read the fp32 masters -> gather them exactly
            self._gather_masters()
            flat.refresh_bf16()
            return
        self._shard16.copy_(self.shard_master)
        for b in self.buckets:
            self._gather(b.gath16, self._shard16[b.so:b.so + b.cb])
            flat.bf16[b.lo:b.hi].copy_(b.gath16[:b.hi - b.lo])
        flat.master.copy_(flat.bf16)
        if self._small_idx is not None:
            # exact fp32 for the 1-D parameters: owners contribute their values, others zero
            mine = self._exact_master(self._small_idx)
            self._small_buf.copy_(torch.where(self._small_own, mine, torch.zeros_like(mine)))
            dist.all_reduce(self._small_buf, group=self.group)
            flat.master.index_copy_(0, self._small_idx, self._small_buf)

    def _exact_master(self, gidx):
        """Exact fp32 values of global flat positions ``gidx`` that this rank owns (zeros
        elsewhere) from the shard (positions map through the bucket chunks)."""
        if not hasattr(self, "_g2s"):
            g2s = torch.full((self.flat.numel,), -1, dtype=torch.long)
            for b in self.buckets:
                lo, hi = self._chunk(b)
                if hi > lo:
                    g2s[lo:hi] = torch.arange(b.so, b.so + hi - lo)
            self._g2s_small = g2s[gidx.cpu()].to(gidx.device)
            self._g2s = True
        sidx = self._g2s_small
        return torch.where(sidx >= 0, self.shard_master[sidx.clamp(min=0)], torch.zeros((), device=sidx.device))

    def _gather_masters(self):
        flat = self.flat
        for b in self.buckets:
            self._gather(b.gath, self.shard_master[b.so:b.so + b.cb])
            flat.master[b.lo:b.hi].copy_(b.gath[:b.hi - b.lo])

    def sync_master(self):
        """Exact fp32 masters on every rank (checkpoints): ZeRO-1 steps only gather the bf16
        weights plus the exact 1-D parameters, so gather the full fp32 shards here."""
        if self.mode != "sharded" or not self.comm or self.shard_master is None:
            return
        stream = self.comm_stream
        if stream is not None:
            stream.wait_stream(torch.cuda.current_stream(self.flat.master.device))
            with torch.cuda.stream(stream):
                self._gather_masters()
            torch.cuda.current_stream(self.flat.master.device).wait_stream(stream)
        else:
            self._gather_masters()

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
