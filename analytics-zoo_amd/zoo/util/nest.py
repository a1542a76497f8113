"""Nested-structure helpers (Py/util/nest.py): flatten lists/tuples/dicts (dicts
in sorted-key order) and rebuild a structure from a flat sequence."""


def is_sequence(s):
    return isinstance(s, (dict, list, tuple))


def _children(s):
    return [s[k] for k in sorted(s)] if isinstance(s, dict) else list(s)


def flatten(seq):
    if not is_sequence(seq):
        return [seq]
    out = []
    for c in _children(seq):
        out.extend(flatten(c))
    return out


def _rebuild(like, values):
    if isinstance(like, dict):
        by_key = dict(zip(sorted(like), values))
        return type(like)((k, by_key[k]) for k in like)
    if isinstance(like, tuple) and hasattr(like, "_fields"):  # namedtuple
        return type(like)(*values)
    return type(like)(values)


def _pack(structure, flat, i):
    vals = []
    for c in _children(structure):
        if is_sequence(c):
            i, v = _pack(c, flat, i)
            vals.append(v)
        else:
            vals.append(flat[i])
            i += 1
    return i, _rebuild(structure, vals)


def pack_sequence_as(structure, flat_sequence):
    if not is_sequence(structure):
        if len(flat_sequence) != 1:
            raise ValueError("structure is a scalar but %d values given" % len(flat_sequence))
        return flat_sequence[0]
    n = len(flatten(structure))
    if n != len(flat_sequence):
        raise ValueError("structure has %d leaves, %d values given" % (n, len(flat_sequence)))
    return _pack(structure, list(flat_sequence), 0)[1]
