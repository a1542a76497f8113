"""Ray helper utilities (Py/ray/utils.py:22-85): list coercion, resource strings,
per-process-group shutdown, local-mode detection."""
import os
import re
import signal


def to_list(value):
    if isinstance(value, (list, tuple)):
        return list(value)
    return [value]


def resource_to_bytes(resource_str):
    """'50b' / '100k' / '250m' / '30g' -> bytes (decimal units, as the reference)."""
    if not resource_str:
        return resource_str
    s = str(resource_str).lower()
    if re.match(r"^[0-9]+\.[0-9]+", s):
        raise ValueError("Fractional values are not supported. Input was: {}".format(resource_str))
    m = re.match(r"^([0-9]+)([a-z]+)?$", s)
    if not m:
        raise ValueError("Size must be specified as bytes(b), kilobytes(k), megabytes(m), gigabytes(g). "
                         "E.g. 50b, 100k, 250m, 30g")
    mult = {"b": 1, "k": 1000, "m": 1000 ** 2, "g": 1000 ** 3}
    if m.group(2) not in mult:
        raise ValueError("Not supported type: {}".format(resource_str))
    return int(m.group(1)) * mult[m.group(2)]


def gen_shutdown_per_node(pgids, node_ips=None):
    """Return a callable that SIGTERMs exactly the given process groups (never by pattern)."""
    pgids = to_list(pgids)

    def _shutdown_per_node(_it=None):
        for pgid in pgids:
            try:
                os.killpg(pgid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
        return iter(())

    return _shutdown_per_node


def is_local(sc=None):
    """True when running single-node (the rebuild has no Spark master)."""
    if sc is None:
        return int(os.environ.get("ZOO_NUM_NODES", "1")) <= 1
    master = sc.getConf().get("spark.master") if hasattr(sc, "getConf") else "local"
    return master == "local" or str(master).startswith("local[")
