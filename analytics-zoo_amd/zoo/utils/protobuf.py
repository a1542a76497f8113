"""Minimal protobuf codec: wire-format decode/encode and a text-format
(prototxt) parser. Nothing in a decoded file is executed — messages become
plain dicts/lists/bytes/numpy arrays — which is what makes it safe to read
the reference's serialized fixtures (BigDL ``.model``, Caffe ``.caffemodel``
/ ``.prototxt``, ONNX) with it.

The hot scan (field splitting) uses the C++ ``zoo._runtime.pb_fields`` when
built; ``pb_fields_py`` is the identical pure-Python fallback.
"""
import re
import struct

import numpy as np

try:  # native wire scanner (csrc/runtime/runtime.cpp)
    from zoo import _runtime as _R
    _native_fields = _R.pb_fields
except Exception:  # pragma: no cover - build-less environments
    _native_fields = None


def _varint(b, i):
    r = s = 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        if c < 0x80:
            return r, i
        s += 7


def pb_fields_py(b):
    """[(field, wire_type, value)] — value: int (varint / fixed) or bytes."""
    out, i, n = [], 0, len(b)
    while i < n:
        k, i = _varint(b, i)
        f, w = k >> 3, k & 7
        if w == 0:
            v, i = _varint(b, i)
        elif w == 1:
            v = int.from_bytes(b[i:i + 8], "little")
            i += 8
        elif w == 2:
            ln, i = _varint(b, i)
            v = bytes(b[i:i + ln])
            i += ln
        elif w == 5:
            v = int.from_bytes(b[i:i + 4], "little")
            i += 4
        else:
            raise ValueError("protobuf: unsupported wire type %d" % w)
        out.append((f, w, v))
    return out


def fields(b):
    if _native_fields is not None:
        return _native_fields(bytes(b))
    return pb_fields_py(b)


def group(b):
    """bytes -> {field: [values...]} preserving order within a field."""
    d = {}
    for f, w, v in fields(b):
        d.setdefault(f, []).append((w, v))
    return d


# ---- scalar helpers ------------------------------------------------------------
def as_str(v):
    return v.decode("utf-8", "replace") if isinstance(v, (bytes, bytearray)) else str(v)


def as_int32(v):
    v &= 0xFFFFFFFFFFFFFFFF
    if v >= 1 << 63:
        v -= 1 << 64
    return int(v)


def as_float32(w, v):
    if w == 5:
        return struct.unpack("<f", int(v).to_bytes(4, "little"))[0]
    if w == 1:
        return struct.unpack("<d", int(v).to_bytes(8, "little"))[0]
    return float(v)


def as_float64(w, v):
    return as_float32(w, v)


def packed_varints(entries):
    """repeated int field: packed (wire 2) and/or unpacked (wire 0) entries."""
    out = []
    for w, v in entries:
        if w == 2:
            i = 0
            while i < len(v):
                x, i = _varint(v, i)
                out.append(as_int32(x))
        else:
            out.append(as_int32(v))
    return out


def packed_floats(entries):
    parts = []
    for w, v in entries:
        if w == 2:
            parts.append(np.frombuffer(v, dtype="<f4"))
        else:
            parts.append(np.array([as_float32(w, v)], dtype=np.float32))
    return np.concatenate(parts) if parts else np.zeros(0, np.float32)


def packed_doubles(entries):
    parts = []
    for w, v in entries:
        if w == 2:
            parts.append(np.frombuffer(v, dtype="<f8"))
        else:
            parts.append(np.array([as_float64(w, v)]))
    return np.concatenate(parts) if parts else np.zeros(0, np.float64)


# ---- encoder ---------------------------------------------------------------------
def enc_varint(x):
    x &= 0xFFFFFFFFFFFFFFFF
    out = bytearray()
    while True:
        c = x & 0x7F
        x >>= 7
        if x:
            out.append(c | 0x80)
        else:
            out.append(c)
            return bytes(out)


def enc_key(field, wire):
    return enc_varint((field << 3) | wire)


def enc_int(field, v):
    return enc_key(field, 0) + enc_varint(int(v))


def enc_bytes(field, b):
    if isinstance(b, str):
        b = b.encode()
    return enc_key(field, 2) + enc_varint(len(b)) + b


def enc_float(field, v):
    return enc_key(field, 5) + struct.pack("<f", float(v))


def enc_packed_ints(field, vals):
    body = b"".join(enc_varint(int(v)) for v in vals)
    return enc_bytes(field, body)


def enc_packed_floats(field, arr):
    return enc_bytes(field, np.asarray(arr, dtype="<f4").tobytes())


def enc_packed_doubles(field, arr):
    return enc_bytes(field, np.asarray(arr, dtype="<f8").tobytes())


# ---- text format (prototxt) ---------------------------------------------------------
_TOK = re.compile(r'\s*(?:(#[^\n]*)|("(?:[^"\\]|\\.)*"|\'(?:[^\'\\]|\\.)*\')|([{}:\[\],;<>])|([^\s{}:\[\],;<>"\']+))')


def _tokens(text):
    pos = 0
    n = len(text)
    while pos < n:
        m = _TOK.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                return
            raise ValueError("prototxt: cannot parse near %r" % text[pos:pos + 30])
        pos = m.end()
        if m.group(1):
            continue
        tok = m.group(2) or m.group(3) or m.group(4)
        if tok is not None:
            yield tok


def _scalar(tok):
    if tok[0] in "\"'":
        return bytes(tok[1:-1], "utf-8").decode("unicode_escape")
    low = tok.lower()
    if low in ("true", "false"):
        return low == "true"
    try:
        return int(tok, 0) if re.fullmatch(r"[-+]?(0x[0-9a-fA-F]+|\d+)", tok) else float(tok)
    except ValueError:
        return tok  # enum identifier


def parse_text(text):
    """prototxt -> {name: [values]} (every field repeated; messages are dicts)."""
    toks = list(_tokens(text))
    pos = 0

    def msg(end):
        nonlocal pos
        d = {}
        while pos < len(toks) and toks[pos] != end:
            name = toks[pos]
            pos += 1
            if toks[pos] == ":":
                pos += 1
            if toks[pos] in ("{", "<"):
                close = "}" if toks[pos] == "{" else ">"
                pos += 1
                val = msg(close)
                pos += 1
                d.setdefault(name, []).append(val)
            elif toks[pos] == "[":
                pos += 1
                while toks[pos] != "]":
                    if toks[pos] != ",":
                        d.setdefault(name, []).append(_scalar(toks[pos]))
                    pos += 1
                pos += 1
            else:
                d.setdefault(name, []).append(_scalar(toks[pos]))
                pos += 1
            if pos < len(toks) and toks[pos] in (",", ";"):
                pos += 1
        return d

    return msg(None)
