"""R4/R5: the job launcher (torch.distributed.run, one process per GPU), the
init_spark_on_yarn mapping and the ROCm environment preparation."""
import os
import subprocess
import sys


def test_build_command_and_dry_run():
    from zoo.common.launcher import build_command, main
    cmd = build_command("train.py", ["--epochs", 3], nnodes=2, nproc_per_node=8, node_rank=1,
                        master_addr="127.0.0.1", master_port=1234)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8" and cmd[cmd.index("--node-rank") + 1] == "1"
    assert cmd[-3:] == ["train.py", "--epochs", "3"]
    assert main(["--dry-run", "--nproc-per-node", "2", "x.py", "a"]) == 0


def test_launch_runs_two_ranks_with_gloo(tmp_path):
    from zoo.common.launcher import launch
    script = tmp_path / "job.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text(
        "import os, sys\n"
        "sys.path.insert(0, %r)\n"
        "import torch, torch.distributed as dist\n"
        "import zoo.common.nncontext as nc\n"
        "ctx = nc.init_nncontext(backend='gloo')\n"
        "t = torch.tensor([float(ctx.rank + 1)])\n"
        "dist.all_reduce(t)\n"
        "open(os.path.join(%r, 'r%%d' %% ctx.rank), 'w').write('%%d %%s %%s' %% (ctx.world_size, t.item(), "
        "os.environ['HSA_ENABLE_IPC_MODE_LEGACY']))\n"
        "ctx.stop()\n" % (os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                       "analytics-zoo_amd"), str(out)))
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    rc = launch(str(script), nproc_per_node=2, master_port=port, env=env)
    assert rc == 0
    assert sorted(os.listdir(out)) == ["r0", "r1"]
    assert open(out / "r0").read() == "2 3.0 0"


def test_init_spark_on_yarn_maps_to_context(monkeypatch):
    import zoo.common.nncontext as nc
    monkeypatch.setattr(nc, "_CTX", None)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    ctx = nc.init_spark_on_yarn(hadoop_conf="/etc/hadoop", num_executors=4, executor_cores=2)
    try:
        assert ctx.executor_request["num_executors"] == 4 and ctx.world_size == 1
    finally:
        nc._CTX = None


def test_engine_prepare_env_and_info(monkeypatch):
    from zoo.util import engine
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    env = engine.prepare_env(local_world_size=4)
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert int(env["OMP_NUM_THREADS"]) == max(1, (os.cpu_count() or 1) // 4)
    info = engine.get_env_info()
    assert info["python"] and "gpus" in info and "native_kernels" in info
