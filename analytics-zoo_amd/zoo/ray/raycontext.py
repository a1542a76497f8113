"""RayContext: a local task/actor runtime with the reference's entry points
(Py/ray/raycontext.py:190-340 RayContext(sc, redis_port, password,
object_store_memory, verbose, env, extra_params).init()/stop()/get()).

The reference boots a Ray cluster inside Spark executors with barrier
mapPartitions. Ray is not part of this stack; the
rebuild keeps the programming model -- remote functions, stateful actors,
``get``/``wait``/``put`` futures -- on plain processes of one node:

  * tasks run on a spawn-started process pool of ``num_ray_nodes *
    ray_node_cpu_cores`` workers (callables shipped with cloudpickle);
  * every actor is one dedicated spawn-started process that executes its
    method calls in order (Ray's actor semantics), answered through a pipe;
  * ``stop()`` ends exactly the processes this context started.

Multi-GPU work inside actors uses torch.distributed (RCCL) like the rest of
the framework; see zoo.ray.mxnet.MXNetTrainer.
"""
import concurrent.futures as cf
import itertools
import logging
import multiprocessing as mp
import os
import threading

import cloudpickle

from zoo.ray.utils import resource_to_bytes

log = logging.getLogger("zoo.ray")


class ObjectRef:
    """Handle to a (future) value; resolved with :func:`get`."""

    _ids = itertools.count()

    def __init__(self, future):
        self._future = future
        self.id = next(ObjectRef._ids)

    def ready(self):
        return self._future.done()

    def result(self, timeout=None):
        return self._future.result(timeout)

    def __repr__(self):
        return "ObjectRef(%d%s)" % (self.id, ", ready" if self.ready() else "")


def _run_pickled(payload):
    fn, args, kwargs = cloudpickle.loads(payload)
    return fn(*args, **kwargs)


def _actor_main(conn, payload, env):
    if env:
        os.environ.update({k: str(v) for k, v in env.items()})
    try:
        cls, args, kwargs = cloudpickle.loads(payload)
        inst = cls(*args, **kwargs)
        conn.send_bytes(cloudpickle.dumps((True, None)))
    except BaseException as e:  # noqa: BLE001 - reported to the caller
        conn.send_bytes(cloudpickle.dumps((False, e)))
        return
    while True:
        try:
            msg = conn.recv_bytes()
        except EOFError:
            return
        name, a, kw = cloudpickle.loads(msg)
        if name is None:
            conn.send_bytes(cloudpickle.dumps((True, None)))
            return
        try:
            res = (True, getattr(inst, name)(*a, **kw))
        except BaseException as e:  # noqa: BLE001
            res = (False, e)
        try:
            conn.send_bytes(cloudpickle.dumps(res))
        except Exception as e:  # noqa: BLE001 - unpicklable result
            conn.send_bytes(cloudpickle.dumps((False, RuntimeError("actor result not serialisable: %s" % e))))


class ActorHandle:
    def __init__(self, cls, args, kwargs, env=None):
        ctx = mp.get_context("spawn")
        self._conn, child = ctx.Pipe()
        self._proc = ctx.Process(target=_actor_main, args=(child, cloudpickle.dumps((cls, args, kwargs)), env),
                                 daemon=True)
        self._proc.start()
        child.close()
        self._lock = threading.Lock()
        self._pending = []  # FIFO of futures; replies arrive in call order
        self._closed = False
        self._ready = cf.Future()
        self._pending.append(self._ready)
        self._reader = threading.Thread(target=self._read_loop, daemon=True)
        self._reader.start()
        self.__class_name = cls.__name__
        RayContext._register_actor(self)

    def _read_loop(self):
        while True:
            try:
                ok, val = cloudpickle.loads(self._conn.recv_bytes())
            except (EOFError, OSError):
                with self._lock:
                    pend, self._pending = self._pending, []
                for f in pend:
                    if not f.done():
                        f.set_exception(RuntimeError("actor process exited"))
                return
            with self._lock:
                f = self._pending.pop(0)
            if ok:
                f.set_result(val)
            else:
                f.set_exception(val)

    def _call(self, name, args, kwargs):
        f = cf.Future()
        with self._lock:
            if self._closed:
                raise RuntimeError("actor %s has been terminated" % self.__class_name)
            self._pending.append(f)
            self._conn.send_bytes(cloudpickle.dumps((name, args, kwargs)))
        return ObjectRef(f)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return _ActorMethod(self, name)

    def _terminate(self, timeout=10.0):
        if self._closed:
            return
        try:
            self._call(None, (), {}).result(timeout)
        except Exception:  # noqa: BLE001
            pass
        self._closed = True
        self._proc.join(timeout)
        if self._proc.is_alive():
            self._proc.terminate()
            self._proc.join(timeout)


class _ActorMethod:
    def __init__(self, handle, name):
        self._h, self._name = handle, name

    def remote(self, *args, **kwargs):
        return self._h._call(self._name, args, kwargs)


class ActorClass:
    def __init__(self, cls, options):
        self._cls, self._options = cls, dict(options)

    def options(self, **kw):
        o = dict(self._options)
        o.update(kw)
        return ActorClass(self._cls, o)

    def remote(self, *args, **kwargs):
        RayContext.get(initialize=True)
        return ActorHandle(self._cls, args, kwargs, env=self._options.get("env"))


class RemoteFunction:
    def __init__(self, fn, options):
        self._fn, self._options = fn, dict(options)

    def options(self, **kw):
        o = dict(self._options)
        o.update(kw)
        return RemoteFunction(self._fn, o)

    def remote(self, *args, **kwargs):
        ctx = RayContext.get(initialize=True)
        return ObjectRef(ctx._pool.submit(_run_pickled, cloudpickle.dumps((self._fn, args, kwargs))))

    def __call__(self, *a, **kw):
        raise TypeError("remote functions are called with .remote(...)")


def remote(*args, **kwargs):
    """``@remote`` / ``@remote(num_cpus=.., num_gpus=.., resources=..)`` on a function or class."""
    def wrap(obj):
        return ActorClass(obj, kwargs) if isinstance(obj, type) else RemoteFunction(obj, kwargs)
    if len(args) == 1 and not kwargs and callable(args[0]):
        return wrap(args[0])
    return wrap


def get(refs, timeout=None):
    if isinstance(refs, (list, tuple)):
        return [r.result(timeout) if isinstance(r, ObjectRef) else r for r in refs]
    return refs.result(timeout) if isinstance(refs, ObjectRef) else refs


def wait(refs, num_returns=1, timeout=None):
    futs = {r._future: r for r in refs}
    done, _ = cf.wait(list(futs), timeout=timeout, return_when=cf.ALL_COMPLETED
                      if num_returns >= len(refs) else cf.FIRST_COMPLETED)
    ready = [futs[f] for f in futs if f in done][:num_returns]
    return ready, [r for r in refs if r not in ready]


def put(value):
    f = cf.Future()
    f.set_result(value)
    return ObjectRef(f)


class RayContext:
    _active = None
    _actors = []

    def __init__(self, sc=None, redis_port=None, password="123456", object_store_memory=None, verbose=False,
                 env=None, extra_params=None, num_ray_nodes=None, ray_node_cpu_cores=None):
        self.sc = sc
        self.redis_port = redis_port
        self.redis_password = password
        self.object_store_memory = resource_to_bytes(object_store_memory)
        self.verbose = verbose
        self.env = env or {}
        self.extra_params = extra_params or {}
        self.num_ray_nodes = int(num_ray_nodes or 1)
        cores = ray_node_cpu_cores or getattr(sc, "defaultParallelism", None) or min(os.cpu_count() or 1, 8)
        self.ray_node_cpu_cores = int(cores)
        self.stopped = True
        self.initialized = False
        self._pool = None
        self.address_info = None

    # ---- lifecycle -------------------------------------------------------
    def init(self, driver_cores=0):
        if self.initialized and not self.stopped:
            return self.address_info
        os.environ.update({k: str(v) for k, v in self.env.items()})
        n = max(1, self.num_ray_nodes * self.ray_node_cpu_cores)
        self._pool = cf.ProcessPoolExecutor(max_workers=n, mp_context=mp.get_context("spawn"))
        self.initialized, self.stopped = True, False
        RayContext._active = self
        self.address_info = {"node_ip_address": "127.0.0.1", "num_workers": n, "pid": os.getpid()}
        log.info("RayContext started: %d task workers on one node", n)
        return self.address_info

    def stop(self):
        if self.stopped:
            return
        for a in list(RayContext._actors):
            a._terminate()
        RayContext._actors = []
        if self._pool is not None:
            self._pool.shutdown(wait=True, cancel_futures=True)
            self._pool = None
        self.stopped = True
        if RayContext._active is self:
            RayContext._active = None

    def purge(self):
        self.stop()

    @classmethod
    def get(cls, initialize=True):
        if cls._active is None:
            if not initialize:
                raise RuntimeError("No active RayContext. Please create and init a RayContext first")
            cls(None).init()
        return cls._active

    @classmethod
    def _register_actor(cls, handle):
        cls._actors.append(handle)

    @staticmethod
    def kill(actor):
        actor._terminate()
        if actor in RayContext._actors:
            RayContext._actors.remove(actor)
