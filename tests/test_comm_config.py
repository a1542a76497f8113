"""The comm-layer switches of ZooConfig (C++ RCCL communicator, channel count) come from the
environment like every other job setting; without an RCCL group GradSync keeps the local path."""
import torch

from zoo.common.nncontext import ZooConfig


def test_comm_switches_from_env(monkeypatch):
    monkeypatch.setenv("ZOO_COMM", "native")
    monkeypatch.setenv("ZOO_RCCL_CHANNELS", "14")
    c = ZooConfig.from_sources()
    assert c.comm == "native" and c.rccl_channels == 14
    monkeypatch.delenv("ZOO_COMM")
    monkeypatch.delenv("ZOO_RCCL_CHANNELS")
    c = ZooConfig.from_sources()
    assert c.comm == "torch" and c.rccl_channels == 0


def test_native_comm_request_without_rccl_group_stays_local():
    from zoo.parallel.ddp import GradSync
    from zoo.parallel.flat import FlatParams
    m = torch.nn.Linear(8, 4)
    flat = FlatParams(list(m.parameters()))
    s = GradSync(flat, comm="native", rccl_channels=8)
    assert s.ncomm is None and not s.comm
