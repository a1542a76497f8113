"""Process bookkeeping for the actor runtime (Py/ray/process.py:27-152).

``session_execute`` runs a shell command in its own session (process group) and
records the pgid; ``ProcessMonitor`` keeps the ProcessInfos of everything the
context started and tears exactly those process groups down on stop / exit /
SIGTERM (the reference's JVMGuard + shutdown hooks)."""
import atexit
import os
import signal
import subprocess

from zoo.ray.utils import gen_shutdown_per_node


class ProcessInfo:
    def __init__(self, out, err, errorcode, pgid, tag="default", pids=None, node_ip=None):
        self.out, self.err, self.errorcode = str(out).strip(), str(err).strip(), errorcode
        self.pgid, self.tag, self.pids, self.node_ip = pgid, tag, pids or [], node_ip

    def __str__(self):
        return "node_ip: {} tag: {}, pgid: {}, pids: {}, returncode: {}, \nerr: {}, \nout: {}".format(
            self.node_ip, self.tag, self.pgid, self.pids, self.errorcode, self.err, self.out)


def pids_from_gpid(gpid):
    """All live pids of one process group (read from /proc, no pattern matching)."""
    pids = []
    for d in os.listdir("/proc"):
        if not d.isdigit():
            continue
        try:
            if os.getpgid(int(d)) == gpid:
                pids.append(int(d))
        except (ProcessLookupError, PermissionError):
            continue
    return pids


def session_execute(command, env=None, tag=None, fail_fast=False, timeout=120):
    pro = subprocess.Popen(command, shell=True, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           start_new_session=True)
    pgid = os.getpgid(pro.pid)
    try:
        out, err = pro.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(pgid, signal.SIGKILL)
        out, err = pro.communicate()
    out, err = out.decode("utf-8", "replace"), err.decode("utf-8", "replace")
    if pro.returncode != 0 and fail_fast:
        raise RuntimeError(err)
    return ProcessInfo(out=out, err=err, errorcode=pro.returncode, pgid=pgid, pids=pids_from_gpid(pgid), tag=tag)


class ProcessMonitor:
    def __init__(self, process_infos, sc=None, ray_rdd=None, raycontext=None, verbose=False):
        self.process_infos = list(process_infos)
        self.raycontext = raycontext
        self.verbose = verbose
        self.pgids = [p.pgid for p in self.process_infos]
        for p in self.process_infos:
            if p.errorcode != 0:
                raise RuntimeError("service %s failed to start:\n%s" % (p.tag, p))
        ProcessMonitor.register_shutdown_hook(extra_close_fn=self.clean_fn)

    def print_ray_remote_err_out(self):
        for p in self.process_infos:
            print(p)

    def clean_fn(self):
        if self.raycontext is not None and not getattr(self.raycontext, "stopped", True):
            self.raycontext.stop()
        gen_shutdown_per_node(self.pgids)()

    @staticmethod
    def register_shutdown_hook(pgid=None, extra_close_fn=None):
        def _shutdown():
            if pgid:
                gen_shutdown_per_node(pgid)()
            if extra_close_fn is not None:
                extra_close_fn()

        def _signal_shutdown(_signo, _frame):
            _shutdown()
            raise SystemExit(0)

        atexit.register(_shutdown)
        try:
            signal.signal(signal.SIGTERM, _signal_shutdown)
        except ValueError:  # not the main thread
            pass
