"""Job launcher: the counterpart of the reference's cluster launchers
(``init_spark_on_local`` / ``init_spark_on_yarn``, Py/common/nncontext.py:23-170, and the
spark-submit scripts under scripts/). A Spark application with N executors becomes a
torch.distributed job with one process per GPU: ``launch`` starts
``python -m torch.distributed.run`` (rendezvous on ``master_addr``), each rank calls
``init_nncontext()`` and joins the RCCL process group.

  python -m zoo.common.launcher --nproc-per-node 8 train.py --epochs 3
"""
import argparse
import os
import shlex
import subprocess
import sys


def gpu_count():
    """GPUs visible to this process (counting devices does not initialise the GPU)."""
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


def build_command(script, script_args=(), nnodes=1, nproc_per_node=None, node_rank=0, master_addr="127.0.0.1",
                  master_port=29500, python=None, module=False):
    nproc = int(nproc_per_node or max(gpu_count(), 1))
    cmd = [python or sys.executable, "-m", "torch.distributed.run", "--nnodes", str(int(nnodes)),
           "--nproc-per-node", str(nproc), "--node-rank", str(int(node_rank)), "--master-addr", str(master_addr),
           "--master-port", str(int(master_port))]
    if module:
        cmd.append("-m")
    return cmd + [script] + [str(a) for a in script_args]


def launch_env(base=None, omp_threads=None, nproc=1):
    """Environment for the ranks: dmabuf IPC for RCCL, per-rank CPU threads."""
    env = dict(base if base is not None else os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if omp_threads is None:
        omp_threads = max(1, (os.cpu_count() or 1) // max(nproc, 1))
    env.setdefault("OMP_NUM_THREADS", str(int(omp_threads)))
    return env


def launch(script, script_args=(), nnodes=1, nproc_per_node=None, node_rank=0, master_addr="127.0.0.1",
           master_port=29500, env=None, module=False, dry_run=False):
    """Run ``script`` as a distributed job; returns the exit code (or the command when
    ``dry_run``)."""
    cmd = build_command(script, script_args, nnodes, nproc_per_node, node_rank, master_addr, master_port,
                        module=module)
    if dry_run:
        return cmd
    nproc = int(cmd[cmd.index("--nproc-per-node") + 1])
    return subprocess.run(cmd, env=launch_env(env, nproc=nproc)).returncode


def main(argv=None):
    ap = argparse.ArgumentParser(description="launch a zoo job, one process per GPU")
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--nproc-per-node", type=int, default=None)
    ap.add_argument("--node-rank", type=int, default=0)
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=29500)
    ap.add_argument("-m", dest="module", action="store_true", help="run the target as a module")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    r = launch(a.script, a.args, a.nnodes, a.nproc_per_node, a.node_rank, a.master_addr, a.master_port,
               module=a.module, dry_run=a.dry_run)
    if a.dry_run:
        print(" ".join(shlex.quote(c) for c in r))
        return 0
    return r


if __name__ == "__main__":
    sys.exit(main())
