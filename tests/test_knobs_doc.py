"""KNOBS.md names only switches the sources actually read, so the table cannot drift into
describing removed paths."""
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _sources():
    pkg = ROOT / "analytics-zoo_amd"
    for pat in ("csrc/**/*.hip", "csrc/**/*.cpp", "zoo/**/*.py"):
        for f in pkg.glob(pat):
            yield f.read_text(errors="ignore")


def test_every_documented_switch_is_read_by_the_code():
    doc = (ROOT / "KNOBS.md").read_text()
    names = set(re.findall(r"`(ZOO_[A-Z0-9_]+)`", doc))
    assert len(names) >= 10
    text = "\n".join(_sources())
    missing = sorted(n for n in names if '"%s"' % n not in text)
    assert not missing, missing
