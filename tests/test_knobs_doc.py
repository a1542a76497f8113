"""KNOBS.md names only switches the sources actually read, every ``ZOO_*`` variable the sources read
is either a ZooConfig field or listed in KNOBS.md, and the list stays short (A/B
leftovers are deleted with their code paths instead of accumulating as untested switches)."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "analytics-zoo_amd"


def _sources():
    for pat in ("csrc/**/*.hip", "csrc/**/*.cpp", "zoo/**/*.py"):
        for f in PKG.glob(pat):
            yield f, f.read_text(errors="ignore")


def _doc_names():
    return set(re.findall(r"`(ZOO_[A-Z0-9_]+)`", (ROOT / "KNOBS.md").read_text()))


def test_every_documented_switch_is_read_by_the_code():
    names = _doc_names()
    assert len(names) >= 10
    text = "\n".join(t for _, t in _sources())
    missing = sorted(n for n in names if '"%s"' % n not in text)
    assert not missing, missing


def test_every_switch_the_code_reads_is_config_or_documented():
    cfg = set(re.findall(r'"(ZOO_[A-Z0-9_]+)"', (PKG / "zoo/common/nncontext.py").read_text()))
    doc = _doc_names()
    read = {}
    for f, t in _sources():
        for n in re.findall(r'(?:getenv|environ\.get|env_flag)\(\s*"(ZOO_[A-Z0-9_]+)"', t):
            read.setdefault(n, f.relative_to(PKG).as_posix())
    stray = sorted("%s (%s)" % (n, f) for n, f in read.items() if n not in cfg and n not in doc)
    assert not stray, stray


def test_knob_list_is_short():
    rows = [ln for ln in (ROOT / "KNOBS.md").read_text().splitlines()
            if ln.startswith("| `ZOO_")]
    assert len(rows) <= 25, len(rows)
