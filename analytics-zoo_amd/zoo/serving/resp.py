"""A small Redis-protocol (RESP2) queue server and client.

Cluster Serving in the reference is a Spark Streaming job reading a Redis
stream (``image_stream``) and writing ``result:<uri>`` hashes
(Zs/serving/ClusterServing.scala:106-116, 278-283; Py/serving/client.py).
Redis is not part of this image, so the framework ships the subset of Redis
it needs — streams with consumer groups, hashes, keys, INFO memory and
back-pressure — speaking the real wire protocol. A stock ``redis-py`` client
(or ``redis-cli``) can talk to it, and the serving worker works unchanged
against a real Redis server when one is available.

Supported commands: PING, ECHO, XADD, XLEN, XRANGE, XGROUP CREATE/DESTROY,
XREADGROUP, XACK, XDEL, XTRIM MAXLEN, HSET/HMSET, HGET, HGETALL, KEYS, DEL,
EXISTS, INFO, CONFIG GET/SET maxmemory, DBSIZE, FLUSHALL, SHUTDOWN.

``RespServer`` is the native C++ store + multi-threaded TCP server
(``zoo._runtime.NativeStore``, csrc/runtime/serving.cpp) whenever the runtime is
built; the pure-Python ``PyRespServer`` below is the fallback and the executable
specification the native one is tested against. A worker in the same process as
a native server gets a :class:`LocalClient` from :func:`connect` (``local=True``):
no socket, no RESP codec, and the batch fast paths ``read_batch``/``finish``.
"""
import fnmatch
import socket
import socketserver
import threading
import time


class RespError(Exception):
    pass


# ---- codec ------------------------------------------------------------------------------
def encode(v):
    if v is None:
        return b"$-1\r\n"
    if isinstance(v, RespError):
        return b"-" + str(v).encode() + b"\r\n"
    if isinstance(v, bool):
        return b":%d\r\n" % int(v)
    if isinstance(v, int):
        return b":%d\r\n" % v
    if isinstance(v, str) and v.startswith("+"):
        return v.encode() + b"\r\n"
    if isinstance(v, (bytes, str)):
        b = v if isinstance(v, bytes) else v.encode()
        return b"$%d\r\n%s\r\n" % (len(b), b)
    if isinstance(v, (list, tuple)):
        return b"*%d\r\n" % len(v) + b"".join(encode(x) for x in v)
    raise TypeError(type(v))


class _Reader:
    def __init__(self, sock):
        self.sock = sock
        self.buf = bytearray()

    def _fill(self):
        chunk = self.sock.recv(1 << 16)
        if not chunk:
            raise ConnectionError("connection closed")
        self.buf += chunk

    def line(self):
        while True:
            i = self.buf.find(b"\r\n")
            if i >= 0:
                out = bytes(self.buf[:i])
                del self.buf[:i + 2]
                return out
            self._fill()

    def exact(self, n):
        while len(self.buf) < n + 2:
            self._fill()
        out = bytes(self.buf[:n])
        del self.buf[:n + 2]
        return out

    def read(self):
        ln = self.line()
        t, rest = ln[:1], ln[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            raise RespError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self.exact(n)
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self.read() for _ in range(n)]
        # inline command (telnet / redis-cli without RESP)
        return ln.split()


# ---- store ------------------------------------------------------------------------------
class _Stream:
    def __init__(self):
        self.entries = []          # [(id_str, {field: value})], ids increasing
        self.last = (0, 0)
        self.groups = {}           # name -> {"last": (ms, seq), "pending": {id: consumer}}


def _parse_id(s):
    s = s.decode() if isinstance(s, bytes) else s
    a, _, b = s.partition("-")
    return int(a), int(b or 0)


class Store:
    def __init__(self, maxmemory=4 << 30):
        self.data = {}
        self.lock = threading.Condition()
        self.maxmemory = int(maxmemory)
        self.used = 0

    @staticmethod
    def _size(fields):
        return sum(len(k) + len(v) for k, v in fields.items()) + 64

    # command dispatch
    def execute(self, args):
        if not args:
            return RespError("ERR empty command")
        cmd = (args[0].decode() if isinstance(args[0], bytes) else args[0]).upper()
        fn = getattr(self, "c_" + cmd.lower(), None)
        if fn is None:
            return RespError("ERR unknown command '%s'" % cmd)
        try:
            with self.lock:
                return fn(*args[1:])
        except RespError as e:
            return e
        except (IndexError, ValueError, KeyError) as e:
            return RespError("ERR %s" % e)

    def c_ping(self, *a):
        return a[0] if a else "+PONG"

    def c_echo(self, x):
        return x

    def c_dbsize(self):
        return len(self.data)

    def c_flushall(self, *a):
        self.data.clear()
        self.used = 0
        return "+OK"

    def c_info(self, *a):
        txt = "# Memory\r\nused_memory:%d\r\nmaxmemory:%d\r\n# Keyspace\r\ndb0:keys=%d\r\n" % (
            self.used, self.maxmemory, len(self.data))
        return txt.encode()

    def c_config(self, sub, *a):
        sub = sub.decode().lower()
        if sub == "set" and a[0].decode().lower() == "maxmemory":
            v = a[1].decode().lower()
            mult = {"k": 1 << 10, "m": 1 << 20, "g": 1 << 30}.get(v[-1:], 1)
            self.maxmemory = int(float(v[:-1] if v[-1:] in "kmg" else v) * mult)
            return "+OK"
        if sub == "get":
            return [b"maxmemory", str(self.maxmemory).encode()]
        return "+OK"

    def _stream(self, key, create=False):
        s = self.data.get(key)
        if s is None:
            if not create:
                return None
            s = self.data[key] = _Stream()
        if not isinstance(s, _Stream):
            raise RespError("WRONGTYPE Operation against a key holding the wrong kind of value")
        return s

    def c_xadd(self, key, *a):
        a = list(a)
        maxlen = None
        if a and a[0].upper() == b"MAXLEN":
            a.pop(0)
            if a[0] in (b"~", b"="):
                a.pop(0)
            maxlen = int(a.pop(0))
        rid = a.pop(0)
        fields = {a[i]: a[i + 1] for i in range(0, len(a), 2)}
        size = self._size(fields)
        if self.used + size > self.maxmemory:
            return RespError("OOM command not allowed when used memory > 'maxmemory'.")
        s = self._stream(key, True)
        if rid == b"*":
            ms = int(time.time() * 1000)
            nid = (ms, s.last[1] + 1) if ms <= s.last[0] else (ms, 0)
            if ms < s.last[0]:
                nid = (s.last[0], s.last[1] + 1)
        else:
            nid = _parse_id(rid)
            if nid <= s.last:
                return RespError("ERR The ID specified in XADD is equal or smaller than the target stream top item")
        s.last = nid
        sid = ("%d-%d" % nid).encode()
        s.entries.append((nid, sid, fields, size))
        self.used += size
        if maxlen is not None:
            self._trim(s, maxlen)
        self.lock.notify_all()
        return sid

    def _trim(self, s, maxlen):
        n = 0
        while len(s.entries) > maxlen:
            self.used -= s.entries.pop(0)[3]
            n += 1
        return n

    def c_xtrim(self, key, kind, *a):
        a = [x for x in a if x not in (b"~", b"=")]
        s = self._stream(key)
        return 0 if s is None else self._trim(s, int(a[0]))

    def c_xlen(self, key):
        s = self._stream(key)
        return 0 if s is None else len(s.entries)

    def c_xrange(self, key, start, end, *a):
        s = self._stream(key)
        if s is None:
            return []
        lo = (0, 0) if start == b"-" else _parse_id(start)
        hi = (1 << 62, 0) if end == b"+" else _parse_id(end)
        out = [[sid, [x for kv in f.items() for x in kv]] for nid, sid, f, _ in s.entries if lo <= nid <= hi]
        if a and a[0].upper() == b"COUNT":
            out = out[:int(a[1])]
        return out

    def c_xgroup(self, sub, *a):
        sub = sub.decode().upper()
        if sub == "CREATE":
            key, name, start = a[0], a[1], a[2]
            mk = len(a) > 3 and a[3].upper() == b"MKSTREAM"
            s = self._stream(key, create=True) if mk or True else self._stream(key)
            if name in s.groups:
                return RespError("BUSYGROUP Consumer Group name already exists")
            s.groups[name] = {"last": s.last if start == b"$" else _parse_id(start if start != b"0" else b"0-0"),
                              "pending": {}}
            return "+OK"
        if sub == "DESTROY":
            s = self._stream(a[0])
            return int(s is not None and s.groups.pop(a[1], None) is not None)
        return RespError("ERR unsupported XGROUP subcommand")

    def c_xreadgroup(self, *a):
        a = list(a)
        if a.pop(0).upper() != b"GROUP":
            raise RespError("ERR syntax error")
        group, consumer = a.pop(0), a.pop(0)
        count, block = None, None
        while a and a[0].upper() in (b"COUNT", b"BLOCK", b"NOACK"):
            opt = a.pop(0).upper()
            if opt == b"COUNT":
                count = int(a.pop(0))
            elif opt == b"BLOCK":
                block = int(a.pop(0))
        if a.pop(0).upper() != b"STREAMS":
            raise RespError("ERR syntax error")
        half = len(a) // 2
        keys, ids = a[:half], a[half:]
        deadline = None if block is None else time.time() + block / 1000.0
        while True:
            res = []
            for key, rid in zip(keys, ids):
                s = self._stream(key)
                if s is None or group not in s.groups:
                    raise RespError("NOGROUP No such key or consumer group")
                g = s.groups[group]
                if rid != b">":
                    continue
                got = [(nid, sid, f) for nid, sid, f, _ in s.entries if nid > g["last"]]
                if count:
                    got = got[:count]
                if got:
                    g["last"] = got[-1][0]
                    for _, sid, _ in got:
                        g["pending"][sid] = consumer
                    res.append([key, [[sid, [x for kv in f.items() for x in kv]] for _, sid, f in got]])
            if res or deadline is None:
                return res or None
            remaining = deadline - time.time() if block else 0.05
            if block and remaining <= 0:
                return None
            self.lock.wait(timeout=min(remaining, 0.05) if block else 0.05)

    def c_xack(self, key, group, *ids):
        s = self._stream(key)
        if s is None or group not in s.groups:
            return 0
        return sum(1 for i in ids if s.groups[group]["pending"].pop(i, None) is not None)

    def c_xdel(self, key, *ids):
        s = self._stream(key)
        if s is None:
            return 0
        keep, n = [], 0
        ids = set(ids)
        for e in s.entries:
            if e[1] in ids:
                self.used -= e[3]
                n += 1
            else:
                keep.append(e)
        s.entries = keep
        return n

    def _hash(self, key, create=False):
        h = self.data.get(key)
        if h is None and create:
            h = self.data[key] = {}
        if h is not None and not isinstance(h, dict):
            raise RespError("WRONGTYPE Operation against a key holding the wrong kind of value")
        return h

    def c_hset(self, key, *a):
        h = self._hash(key, True)
        n = 0
        for i in range(0, len(a), 2):
            n += a[i] not in h
            self.used += len(a[i]) + len(a[i + 1])
            h[a[i]] = a[i + 1]
        self.lock.notify_all()
        return n

    def c_hmset(self, key, *a):
        self.c_hset(key, *a)
        return "+OK"

    def c_hget(self, key, field):
        h = self._hash(key)
        return None if h is None else h.get(field)

    def c_hgetall(self, key):
        h = self._hash(key)
        return [] if h is None else [x for kv in h.items() for x in kv]

    def c_keys(self, pattern):
        pat = pattern.decode()
        return [k for k in list(self.data) if fnmatch.fnmatchcase(k.decode(), pat)]

    def c_exists(self, *keys):
        return sum(1 for k in keys if k in self.data)

    def c_del(self, *keys):
        n = 0
        for k in keys:
            v = self.data.pop(k, None)
            if v is not None:
                n += 1
                if isinstance(v, dict):
                    self.used -= sum(len(a) + len(b) for a, b in v.items())
                else:
                    self.used -= sum(e[3] for e in v.entries)
        return n

    def c_shutdown(self, *a):
        raise SystemExit


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        r = _Reader(self.request)
        store = self.server.store
        while True:
            try:
                args = r.read()
            except (ConnectionError, OSError):
                return
            if isinstance(args, list) and args and isinstance(args[0], bytes) and args[0].upper() == b"SHUTDOWN":
                self.request.sendall(encode("+OK"))
                threading.Thread(target=self.server.shutdown, daemon=True).start()
                return
            out = store.execute(args if isinstance(args, list) else [args])
            try:
                self.request.sendall(encode(out))
            except OSError:
                return


class PyRespServer(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, host="127.0.0.1", port=6379, maxmemory=4 << 30):
        super().__init__((host, port), _Handler)
        self.store = Store(maxmemory)

    @property
    def port(self):
        return self.server_address[1]

    def start(self):
        t = threading.Thread(target=self.serve_forever, daemon=True)
        t.start()
        return self


_LOCAL = {}   # port -> NativeStore of native servers running in this process


def _native_runtime():
    try:
        from zoo import _runtime
        return _runtime if hasattr(_runtime, "NativeStore") else None
    except ImportError:
        return None


class NativeRespServer:
    """The C++ queue server; binds at construction (``port`` 0 = ephemeral)."""

    def __init__(self, host="127.0.0.1", port=6379, maxmemory=4 << 30):
        rt = _native_runtime()
        self.store = rt.NativeStore(int(maxmemory))
        self._port = self.store.serve(host, int(port))
        _LOCAL[self._port] = self.store

    @property
    def port(self):
        return self._port

    def start(self):
        return self

    def serve_forever(self):
        while self.store.running():
            time.sleep(0.2)

    def shutdown(self):
        _LOCAL.pop(self._port, None)
        self.store.stop()

    def server_close(self):
        pass


def RespServer(host="127.0.0.1", port=6379, maxmemory=4 << 30):  # noqa: N802 - class-like factory
    """Native C++ queue server when the runtime is built, else the Python one."""
    if _native_runtime() is not None:
        return NativeRespServer(host, port, maxmemory)
    return PyRespServer(host, port, maxmemory)


# ---- client ------------------------------------------------------------------------------
class RespClient:
    """The redis-py (StrictRedis) subset used by serving; bytes in, bytes out."""

    def __init__(self, host="127.0.0.1", port=6379, db=0, timeout=30.0):
        self.sock = socket.create_connection((host, int(port)), timeout=timeout)
        self.reader = _Reader(self.sock)
        self.lock = threading.Lock()

    def execute_command(self, *args):
        parts = [a if isinstance(a, bytes) else str(a).encode() for a in args]
        with self.lock:
            self.sock.sendall(encode(parts))
            return self.reader.read()

    def ping(self):
        return self.execute_command("PING") in ("PONG", b"PONG")

    def xadd(self, name, fields, id="*", maxlen=None):  # noqa: A002
        args = ["XADD", name] + (["MAXLEN", "~", maxlen] if maxlen else []) + [id]
        for k, v in fields.items():
            args += [k, v]
        return self.execute_command(*args)

    def xlen(self, name):
        return self.execute_command("XLEN", name)

    def xgroup_create(self, name, groupname, id="$", mkstream=True):  # noqa: A002
        return self.execute_command("XGROUP", "CREATE", name, groupname, id, *(["MKSTREAM"] if mkstream else []))

    def xreadgroup(self, groupname, consumername, streams, count=None, block=None):
        args = ["XREADGROUP", "GROUP", groupname, consumername]
        if count:
            args += ["COUNT", count]
        if block is not None:
            args += ["BLOCK", block]
        args += ["STREAMS"] + list(streams.keys()) + list(streams.values())
        res = self.execute_command(*args)
        if not res:
            return []
        return [[k, [(sid, dict(zip(kv[::2], kv[1::2]))) for sid, kv in msgs]] for k, msgs in res]

    def xack(self, name, groupname, *ids):
        return self.execute_command("XACK", name, groupname, *ids) if ids else 0

    def xdel(self, name, *ids):
        return self.execute_command("XDEL", name, *ids) if ids else 0

    def xtrim(self, name, maxlen):
        return self.execute_command("XTRIM", name, "MAXLEN", maxlen)

    def hset(self, name, key=None, value=None, mapping=None):
        args = []
        if key is not None:
            args += [key, value]
        for k, v in (mapping or {}).items():
            args += [k, v]
        return self.execute_command("HSET", name, *args)

    def hget(self, name, key):
        return self.execute_command("HGET", name, key)

    def hgetall(self, name):
        r = self.execute_command("HGETALL", name) or []
        return dict(zip(r[::2], r[1::2]))

    def keys(self, pattern="*"):
        return self.execute_command("KEYS", pattern)

    def delete(self, *names):
        return self.execute_command("DEL", *names) if names else 0

    def exists(self, *names):
        return self.execute_command("EXISTS", *names)

    def info(self, section=None):
        txt = self.execute_command("INFO", *([section] if section else []))
        out = {}
        for line in (txt.decode() if isinstance(txt, bytes) else txt).splitlines():
            if ":" in line and not line.startswith("#"):
                k, v = line.split(":", 1)
                out[k] = int(v) if v.isdigit() else v
        return out

    def config_set(self, name, value):
        return self.execute_command("CONFIG", "SET", name, value)

    def flushall(self):
        return self.execute_command("FLUSHALL")

    def shutdown(self):
        try:
            self.execute_command("SHUTDOWN")
        except (ConnectionError, OSError):
            pass

    def close(self):
        self.sock.close()


class LocalClient(RespClient):
    """RespClient over an in-process NativeStore: commands skip the socket and the
    codec, and the serving worker gets the batch fast paths."""

    def __init__(self, store):  # noqa: D107 - no socket
        self.store = store
        self.sock = None
        self.lock = threading.Lock()

    def execute_command(self, *args):
        parts = [a if isinstance(a, bytes) else str(a).encode() for a in args]
        try:
            return self.store.execute(parts)
        except RuntimeError as e:
            raise RespError(str(e)) from None

    def read_batch(self, stream, group, consumer, count, block_ms):
        """[(id, uri, kind, decoded payload bytes, shape)]; blocks without the GIL."""
        return self.store.read_batch(stream, group, consumer, int(count), int(block_ms))

    def finish(self, stream, group, ids, results, field="value"):
        """HSET every (key, value) result, then XACK + XDEL ``ids``, under one lock."""
        self.store.finish(stream, group, list(ids), list(results), field)

    def shutdown(self):
        self.store.stop()

    def close(self):
        pass


def connect(host="127.0.0.1", port=6379, local=False):
    """``local``: an in-process native server on that port is used directly
    (:class:`LocalClient`); otherwise a real redis-py client when installed, else
    the built-in RESP client."""
    if local and host in ("127.0.0.1", "localhost") and int(port) in _LOCAL:
        return LocalClient(_LOCAL[int(port)])
    try:
        import redis  # noqa: F401
        return redis.StrictRedis(host=host, port=int(port), db=0)
    except ImportError:
        return RespClient(host, port)
