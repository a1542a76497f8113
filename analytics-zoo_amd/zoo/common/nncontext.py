"""Runtime bring-up: ``init_nncontext`` and the typed engine configuration.

Reference: Py/common/nncontext.py:104-124 (init_nncontext -> SparkContext +
BigDL Engine.init) and Zs/common/NNContext.scala:133-246. On MI355X the
"context" is one process per GPU:

  * device from ``LOCAL_RANK`` (``torch.cuda.set_device``)
  * ``torch.distributed`` process group over RCCL ("nccl" backend on ROCm) when
    ``WORLD_SIZE > 1`` (gloo on CPU-only hosts, used by the CPU test suite)
  * the native kernel library is loaded eagerly so a missing build fails here
  * a typed :class:`ZooConfig` assembled from defaults < env (``ZOO_*`` and the
    honoured legacy ``bigdl.failure.*`` / ``OMP_NUM_THREADS`` names) < kwargs
    

``init_nncontext`` returns a :class:`ZooContext`; it never starts Spark. Spark
integration (NNFrames) is optional and only used when pyspark is importable.
"""
import dataclasses
import datetime
import logging
import os
import socket

import torch

log = logging.getLogger("zoo")


@dataclasses.dataclass
class ZooConfig:
    # engine
    dtype: str = "bf16"
    # gradient bucket size (MB of fp32 gradient): xGMI is 7 point-to-point links per GPU, and a
    # collective only reaches per-link bandwidth with multi-MB per-peer messages -- 32 MB (16 MB
    # on a bf16 wire, 2 MB per peer at N=8) amortises RCCL's per-call latency while the last
    # bucket (the earliest layers, exposed after backward) stays a short tail. Engines size
    # buckets per model (bench.py: NCF = one bucket)
    bucket_mb: float = 32.0
    overlap_comm: bool = True
    # 16-bit gradient transfer, BigDL's default (docs/docs/wp-bigdl.md:140-160: gradients always
    # travel as 16-bit chunks): "auto" = bf16 wire with fp32 accumulation whenever GPU
    # collectives run (world > 1, or force_comm), fp32 on CPU/gloo; "" / "none" = fp32 wire
    grad_compression: str = "auto"      # ZOO_GRAD_COMPRESSION
    sharded_optimizer: bool = False
    hip_graph: bool = False
    # failure handling (bigdl.failure.retryTimes / retryTimeInterval, Topology.scala:1181-1182)
    failure_retry_times: int = 5
    failure_retry_interval_s: float = 120.0
    fault_inject_step: int = -1          # ZOO_FAULT_INJECT_STEP: raise at this iteration (tests the retry path)
    fault_inject_rank: int = -1          # ZOO_FAULT_INJECT_RANK: only this rank raises (-1: every rank)
    auto_resume: bool = False            # ZOO_AUTO_RESUME: fit() resumes from the latest checkpoint (launcher restarts)
    force_comm: bool = False             # ZOO_FORCE_COMM: run the collective path on a world-size-1 process group
    # gradient-bucket collectives: "torch" = torch.distributed ProcessGroup calls; "native" = the
    # C++ comm layer (csrc/comm.cpp: RCCL communicator of our own on GradSync's comm stream)
    comm: str = "torch"                  # ZOO_COMM
    # RCCL channels (CTAs) of the native communicator; 0 = RCCL's own choice. The 8 MI355X of a
    # node are fully connected by 7 xGMI links each: one ring per link needs >= 7 channels
    rccl_channels: int = 0               # ZOO_RCCL_CHANNELS
    # data
    num_workers: int = 4
    pin_memory: bool = True
    # logging / tracing
    log_every: int = 50
    roctx: bool = False                  # ZOO_ROCTX: roctx ranges around engine phases (rocprofv3 --marker-trace)
    phase_timing: bool = False           # ZOO_PHASE_TIMING: per-phase device timings (fwd+bwd / comm / optim)
    debug_sync: bool = False             # ZOO_DEBUG_SYNC: synchronise + check for non-finite loss every step
    deterministic: bool = False          # ZOO_DETERMINISTIC: ordered (atomic-free) reductions, bit-reproducible
    seed: int = 1
    backend: str = ""                    # "", "nccl" (RCCL), "gloo"
    timeout_s: float = 1800.0

    _ENV = {
        "dtype": "ZOO_DTYPE", "bucket_mb": "ZOO_BUCKET_MB", "overlap_comm": "ZOO_OVERLAP_COMM",
        "sharded_optimizer": "ZOO_SHARDED_OPTIM", "hip_graph": "ZOO_HIP_GRAPH",
        "grad_compression": "ZOO_GRAD_COMPRESSION",
        "failure_retry_times": "ZOO_FAILURE_RETRY_TIMES", "failure_retry_interval_s": "ZOO_FAILURE_RETRY_INTERVAL",
        "fault_inject_step": "ZOO_FAULT_INJECT_STEP", "num_workers": "ZOO_NUM_WORKERS",
        "fault_inject_rank": "ZOO_FAULT_INJECT_RANK", "auto_resume": "ZOO_AUTO_RESUME",
        "force_comm": "ZOO_FORCE_COMM", "comm": "ZOO_COMM", "rccl_channels": "ZOO_RCCL_CHANNELS",
        "pin_memory": "ZOO_PIN_MEMORY", "log_every": "ZOO_LOG_EVERY", "roctx": "ZOO_ROCTX", "seed": "ZOO_SEED",
        "phase_timing": "ZOO_PHASE_TIMING", "debug_sync": "ZOO_DEBUG_SYNC", "deterministic": "ZOO_DETERMINISTIC",
        "backend": "ZOO_DIST_BACKEND", "timeout_s": "ZOO_DIST_TIMEOUT",
    }
    _LEGACY = {"failure_retry_times": "bigdl.failure.retryTimes",
               "failure_retry_interval_s": "bigdl.failure.retryTimeInterval"}

    @classmethod
    def from_sources(cls, conf=None, **kw):
        c = cls()
        sources = {}
        for f in dataclasses.fields(cls):
            for key in (cls._LEGACY.get(f.name), cls._ENV.get(f.name)):
                if key and key in os.environ:
                    sources[f.name] = os.environ[key]
        if isinstance(conf, dict):
            for k, v in conf.items():
                name = k
                for f, legacy in cls._LEGACY.items():
                    if k == legacy:
                        name = f
                sources[name] = v
        sources.update(kw)
        for k, v in sources.items():
            if not hasattr(c, k):
                continue
            cur = getattr(c, k)
            if isinstance(cur, bool):
                v = v if isinstance(v, bool) else str(v).lower() in ("1", "true", "yes", "on")
            elif isinstance(cur, int):
                v = int(v)
            elif isinstance(cur, float):
                v = float(v)
            setattr(c, k, v)
        return c


class ZooContext:
    """Handle returned by :func:`init_nncontext` (replaces the SparkContext)."""

    def __init__(self, config, device, rank, world_size, local_rank, group=None, app_name="zoo"):
        self.config = config
        self.device = device
        self.rank = rank
        self.world_size = world_size
        self.local_rank = local_rank
        self.group = group
        self.app_name = app_name
        self.start_time = datetime.datetime.now()

    # spark-like helpers used by the reference APIs
    @property
    def defaultParallelism(self):  # noqa: N802 (reference name)
        return self.world_size

    @property
    def node_number(self):
        return int(os.environ.get("ZOO_NUM_NODES", os.environ.get("NNODES", "1")))

    @property
    def core_number(self):
        return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))

    @property
    def is_distributed(self):
        return self.world_size > 1

    def barrier(self):
        if self.world_size > 1:
            import torch.distributed as dist
            dist.barrier(group=self.group)

    def stop(self):
        global _CTX
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
        _CTX = None

    def __repr__(self):
        return "ZooContext(rank=%d/%d, device=%s, backend=%s)" % (self.rank, self.world_size, self.device,
                                                                  self.config.backend or "none")


_CTX = None


def _env_int(*names, default=0):
    for n in names:
        if n in os.environ:
            return int(os.environ[n])
    return default


def init_nncontext(conf=None, redirect_spark_log=True, app_name=None, **kw):
    """Create (or return) the process-wide :class:`ZooContext`.

    ``conf`` may be an app-name string (as in the reference) or a dict of
    config keys; keyword arguments override everything.
    """
    global _CTX
    if _CTX is not None:
        return _CTX
    if isinstance(conf, str):
        app_name, conf = conf, None
    cfg = ZooConfig.from_sources(conf, **kw)
    rank = _env_int("RANK", default=0)
    world = _env_int("WORLD_SIZE", default=1)
    local_rank = _env_int("LOCAL_RANK", default=rank)
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % max(ndev, 1))
        device = torch.device("cuda", local_rank % max(ndev, 1))
        from zoo.ops._native import native
        native()  # fail early and loudly if the kernel library is missing
        if cfg.deterministic:
            native().set_deterministic(True)
    else:
        device = torch.device("cpu")
    group = None
    if world == 1 and cfg.force_comm:
        # one-rank process group (RCCL on a GPU): exercises the bucketed / overlapped collective
        # path of the data-parallel engine on a single device; an in-memory store needs no network
        import torch.distributed as dist
        if not dist.is_initialized():
            backend = cfg.backend or ("nccl" if use_gpu else "gloo")
            dist.init_process_group(backend=backend, store=dist.HashStore(), rank=0, world_size=1,
                                    device_id=device if use_gpu else None)
            cfg.backend = backend
        else:
            cfg.backend = dist.get_backend()
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            backend = cfg.backend or ("nccl" if use_gpu else "gloo")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29500")
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=cfg.timeout_s),
                                    device_id=device if use_gpu else None)
            cfg.backend = backend
        else:
            cfg.backend = dist.get_backend()
    torch.manual_seed(cfg.seed + rank)
    if "OMP_NUM_THREADS" in os.environ:
        try:
            torch.set_num_threads(int(os.environ["OMP_NUM_THREADS"]))
        except ValueError:
            pass
    logging.basicConfig(level=logging.INFO if rank == 0 else logging.WARNING,
                        format="%(asctime)s zoo[%(process)d] %(levelname)s %(message)s")
    _CTX = ZooContext(cfg, device, rank, world, local_rank, group, app_name or "zoo")
    log.info("init_nncontext: %r on %s", _CTX, socket.gethostname())
    return _CTX


def get_nncontext():
    return _CTX if _CTX is not None else init_nncontext()


def init_spark_on_local(cores=2, conf=None, python_location=None, spark_log_level="WARN",
                        redirect_spark_log=True):
    """Reference launcher (Py/common/nncontext.py:23). Local mode == one process."""
    os.environ.setdefault("OMP_NUM_THREADS", str(cores))
    return init_nncontext(conf)


def init_spark_on_yarn(hadoop_conf=None, conda_name=None, num_executors=2, executor_cores=4,
                       executor_memory="2g", driver_memory="1g", driver_cores=4, extra_executor_memory_for_ray=None,
                       extra_python_lib=None, penv_archive=None, additional_archive=None, hadoop_user_name="root",
                       spark_yarn_archive=None, spark_log_level="WARN", redirect_spark_log=True, jars=None,
                       conf=None, **kwargs):
    """Reference launcher (Py/common/nncontext.py:43-170). There is no YARN/JVM tier on an
    MI355X node: an application's executors are the ranks of a torch.distributed job (one
    process per GPU). Inside a launched job (``WORLD_SIZE`` set by
    ``zoo.common.launcher`` / torchrun) this joins it; otherwise it starts the local
    single-process context. The requested executor shape is recorded on the context
    (``ctx.executor_request``) so scripts can hand it to ``zoo.common.launcher.launch``
    (``num_executors`` -> ranks, ``executor_cores`` -> OMP threads per rank)."""
    if "WORLD_SIZE" not in os.environ:
        log.warning("init_spark_on_yarn: no YARN here; running in-process. Start %d ranks with "
                    "`python -m zoo.common.launcher --nproc-per-node %d <script>` for a distributed job",
                    num_executors, num_executors)
    os.environ.setdefault("OMP_NUM_THREADS", str(int(executor_cores)))
    ctx = init_nncontext(conf)
    ctx.executor_request = {"num_executors": int(num_executors), "executor_cores": int(executor_cores),
                            "executor_memory": executor_memory, "driver_memory": driver_memory,
                            "conda_name": conda_name, "hadoop_conf": hadoop_conf}
    return ctx


def init_spark_standalone(num_executors=1, executor_cores=2, conf=None, **kwargs):
    """Standalone-cluster launcher of later reference versions: same mapping as
    :func:`init_spark_on_yarn`."""
    return init_spark_on_yarn(num_executors=num_executors, executor_cores=executor_cores, conf=conf)
