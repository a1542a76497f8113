"""Per-step scratch (zoo.ops.workspace): the begin-of-step memset covers the high-water mark of
every step so far, so slots a replayed hipGraph dirtied (the replay never runs the Python
bookkeeping) are clear for the next eager step; a replaced buffer stays alive for captured graphs."""
import torch

from zoo.ops import workspace


def _reset():
    workspace._state.update({"buf": None, "off": 0, "active": False, "need": 1 << 16, "hw": 0, "retired": []})


def test_memset_covers_high_water_of_all_steps():
    _reset()
    dev = torch.device("cpu")
    workspace.begin_step(dev)
    big = workspace.zeros(5000, dev)       # a large step (e.g. the shape a graph was captured for)
    big.fill_(1.0)
    workspace.end_step()
    workspace.begin_step(dev)
    small = workspace.zeros(100, dev)      # a smaller eager step
    small.fill_(2.0)
    workspace.end_step()
    # a replay of the large graph dirties its slots again without running begin/end_step
    workspace._state["buf"][:5000].fill_(3.0)
    workspace.begin_step(dev)
    assert workspace.high_water() >= 5000
    assert float(workspace._state["buf"][:5000].abs().max()) == 0.0
    a = workspace.zeros(4000, dev)
    assert float(a.abs().max()) == 0.0
    workspace.end_step()
    _reset()


def test_grown_buffer_keeps_old_one_alive():
    _reset()
    dev = torch.device("cpu")
    workspace.begin_step(dev)
    first = workspace._state["buf"]
    t = workspace.zeros((1 << 16) + 10, dev)    # does not fit: fallback allocation, buffer grows next step
    assert t.numel() == (1 << 16) + 10 and t.data_ptr() != first.data_ptr()
    workspace.end_step()
    workspace.begin_step(dev)
    assert workspace._state["buf"].numel() > first.numel()
    assert any(r is first for r in workspace._state["retired"])
    workspace.end_step()
    _reset()
