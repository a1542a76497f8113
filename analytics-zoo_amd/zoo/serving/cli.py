"""cluster-serving-{init,start,stop,restart,shutdown} (scripts/cluster-serving/*).

  python -m zoo.serving.cli init                # write config.yaml here
  python -m zoo.serving.cli start [--config config.yaml] [--workers N]
  python -m zoo.serving.cli stop | restart | shutdown

``start`` launches the RESP queue server (when ``data.src`` is local and no
server answers there) and one serving worker per GPU, each pinned with
HIP_VISIBLE_DEVICES. A ``running`` flag file keeps workers alive; ``stop``
removes it, ``shutdown`` also stops the queue server. PIDs go to
``serving.pids``.
"""
import argparse
import os
import shutil
import signal
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
TEMPLATE = os.path.join(HERE, "..", "..", "..", "scripts", "cluster-serving", "config.yaml")


def _pids(path="serving.pids"):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [int(x) for x in f.read().split()]


def cmd_init(a):
    if os.path.exists("config.yaml"):
        print("config.yaml exists")
        return 0
    shutil.copy(os.path.abspath(TEMPLATE), "config.yaml")
    print("wrote config.yaml")
    return 0


def _queue_alive(host, port):
    from zoo.serving.resp import RespClient
    try:
        c = RespClient(host, port, timeout=1.0)
        ok = c.ping()
        c.close()
        return ok
    except OSError:
        return False


def cmd_start(a):
    import yaml
    from zoo.serving.server import load_config
    cfg = load_config(a.config)
    with open(a.config) as f:
        raw = yaml.safe_load(f) or {}
    workers = a.workers or int(((raw.get("params") or {}).get("workers")) or 1)
    pids = []
    env = dict(os.environ)
    env["PYTHONPATH"] = os.path.abspath(os.path.join(HERE, "..", "..")) + os.pathsep + env.get("PYTHONPATH", "")
    if cfg["host"] in ("127.0.0.1", "localhost") and not _queue_alive(cfg["host"], cfg["port"]):
        p = subprocess.Popen([sys.executable, "-m", "zoo.serving.cli", "queue", "--port", str(cfg["port"]),
                              "--maxmem", str(cfg["maxmem"])], env=env)
        pids.append(p.pid)
        for _ in range(100):
            if _queue_alive(cfg["host"], cfg["port"]):
                break
            time.sleep(0.1)
    open("running", "w").close()
    for w in range(workers):
        e = dict(env)
        e["HIP_VISIBLE_DEVICES"] = str(w)
        p = subprocess.Popen([sys.executable, "-m", "zoo.serving.cli", "worker", "--config", a.config], env=e)
        pids.append(p.pid)
    with open("serving.pids", "w") as f:
        f.write(" ".join(str(p) for p in pids))
    print("started %d worker(s)" % workers)
    return 0


def cmd_stop(a):
    if os.path.exists("running"):
        os.remove("running")
    print("stop requested (workers exit after their current batch)")
    return 0


def cmd_shutdown(a):
    cmd_stop(a)
    from zoo.serving.resp import RespClient
    from zoo.serving.server import load_config
    try:
        cfg = load_config(a.config)
        c = RespClient(cfg["host"], cfg["port"], timeout=2.0)
        c.shutdown()
    except (OSError, FileNotFoundError):
        pass
    for pid in _pids():
        try:
            os.kill(pid, signal.SIGTERM)
        except OSError:
            pass
    if os.path.exists("serving.pids"):
        os.remove("serving.pids")
    return 0


def cmd_restart(a):
    cmd_shutdown(a)
    time.sleep(1.0)
    return cmd_start(a)


def cmd_queue(a):
    from zoo.serving.resp import RespServer
    mult = {"k": 1 << 10, "m": 1 << 20, "g": 1 << 30}
    mm = str(a.maxmem).lower()
    maxmem = int(float(mm[:-1]) * mult[mm[-1]]) if mm[-1:] in mult else int(mm)
    srv = RespServer("127.0.0.1", a.port, maxmem)
    print("queue server on 127.0.0.1:%d" % srv.port, flush=True)
    srv.serve_forever()
    return 0


def cmd_worker(a):
    from zoo.serving.server import ClusterServing
    s = ClusterServing(a.config)
    s.run(running_flag="running")
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="cluster-serving")
    ap.add_argument("command", choices=["init", "start", "stop", "restart", "shutdown", "queue", "worker"])
    ap.add_argument("--config", default="config.yaml")
    ap.add_argument("--workers", type=int, default=0)
    ap.add_argument("--port", type=int, default=6379)
    ap.add_argument("--maxmem", default="4g")
    a = ap.parse_args(argv)
    return {"init": cmd_init, "start": cmd_start, "stop": cmd_stop, "restart": cmd_restart,
            "shutdown": cmd_shutdown, "queue": cmd_queue, "worker": cmd_worker}[a.command](a)


if __name__ == "__main__":
    sys.exit(main())
