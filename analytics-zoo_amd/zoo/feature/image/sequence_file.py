"""Hadoop SequenceFile codec for the image datasets BigDL writes with
``ImageNetSeqFileGenerator`` and the reference reads with ``ImageSet.readSequenceFiles``
(Zs/feature/image/ImageSet.scala:335-352; BigDL SeqFileFolder):

* file: ``SEQ`` + version (6) + key / value class names (Text) + compression flags
  (+ codec class) + metadata (int32 count of Text pairs) + 16-byte sync marker;
* record: int32 record length, int32 key length, key bytes, value bytes; a record
  length of -1 escapes a sync marker. Record-compressed values (DefaultCodec = zlib)
  are inflated; block-compressed files are rejected.
* BigDL's image records: key = Text ``"<label>\\n<name>"``, value = Text holding
  int32 width, int32 height (big-endian) and the 3*w*h BGR pixel bytes.
"""
import os
import struct
import zlib

_SYNC_ESCAPE = -1
_TEXT = b"org.apache.hadoop.io.Text"


def _read_vint(buf, pos):
    """Hadoop WritableUtils.readVLong -> (value, new position)."""
    first = struct.unpack_from(">b", buf, pos)[0]
    pos += 1
    if first >= -112:
        return first, pos
    neg = first < -120
    n = (-119 - first) if neg else (-111 - first)   # total bytes including the first
    v = 0
    for _ in range(n - 1):
        v = (v << 8) | buf[pos]
        pos += 1
    return (~v if neg else v), pos


def _write_vint(v):
    if -112 <= v <= 127:
        return struct.pack(">b", v)
    length = -112
    if v < 0:
        v = ~v
        length = -120
    tmp = v
    while tmp:
        tmp >>= 8
        length -= 1
    out = struct.pack(">b", length)
    n = (-(length + 120)) if length < -120 else (-(length + 112))
    for i in range(n - 1, -1, -1):
        out += bytes([(v >> (8 * i)) & 0xFF])
    return out


def _read_text(buf, pos):
    n, pos = _read_vint(buf, pos)
    return bytes(buf[pos:pos + n]), pos + n


def _text(b):
    return _write_vint(len(b)) + b


def read_sequence_file(path):
    """Yield (key, value) payloads (the Text contents, without their length prefixes)."""
    with open(path, "rb") as f:
        buf = f.read()
    if buf[:3] != b"SEQ":
        raise ValueError("%s is not a Hadoop SequenceFile" % path)
    version = buf[3]
    pos = 4
    key_cls, pos = _read_text(buf, pos)
    val_cls, pos = _read_text(buf, pos)
    compressed = block = False
    codec = None
    if version > 2:
        compressed, block = bool(buf[pos]), bool(buf[pos + 1])
        pos += 2
        if compressed and version >= 5:
            codec, pos = _read_text(buf, pos)
    if version >= 6:
        (nmeta,) = struct.unpack_from(">i", buf, pos)
        pos += 4
        for _ in range(nmeta):
            _, pos = _read_text(buf, pos)
            _, pos = _read_text(buf, pos)
    if block:
        raise NotImplementedError("block-compressed SequenceFiles are not supported (%s)" % path)
    if compressed and codec not in (None, b"org.apache.hadoop.io.compress.DefaultCodec"):
        raise NotImplementedError("SequenceFile codec %r is not supported" % codec)
    sync = buf[pos:pos + 16]
    pos += 16
    n = len(buf)
    while pos + 4 <= n:
        (rlen,) = struct.unpack_from(">i", buf, pos)
        pos += 4
        if rlen == _SYNC_ESCAPE:
            if buf[pos:pos + 16] != sync:
                raise ValueError("corrupt SequenceFile %s: bad sync marker" % path)
            pos += 16
            continue
        (klen,) = struct.unpack_from(">i", buf, pos)
        pos += 4
        kraw = buf[pos:pos + klen]
        vraw = buf[pos + klen:pos + rlen]
        pos += rlen
        key = _read_text(kraw, 0)[0] if key_cls == _TEXT else bytes(kraw)
        if compressed:
            vraw = zlib.decompress(vraw)
        val = _read_text(vraw, 0)[0] if val_cls == _TEXT else bytes(vraw)
        yield key, val


def write_sequence_file(path, records, sync_every=2000, compress=False):
    """Write (key bytes, value bytes) pairs as a version-6 Text/Text SequenceFile."""
    sync = os.urandom(16)
    out = bytearray(b"SEQ" + bytes([6]) + _text(_TEXT) + _text(_TEXT))
    out += bytes([1 if compress else 0, 0])
    if compress:
        out += _text(b"org.apache.hadoop.io.compress.DefaultCodec")
    out += struct.pack(">i", 0) + sync
    last = len(out)
    for k, v in records:
        kb, vb = _text(bytes(k)), _text(bytes(v))
        if compress:
            vb = zlib.compress(vb)
        if len(out) - last >= sync_every:
            out += struct.pack(">i", _SYNC_ESCAPE) + sync
            last = len(out)
        out += struct.pack(">ii", len(kb) + len(vb), len(kb)) + kb + vb
    with open(path, "wb") as f:
        f.write(bytes(out))


def encode_image_record(label, name, bgr):
    """BigDL image record: key ``"<label>\\n<name>"``, value = width, height, BGR bytes."""
    h, w = bgr.shape[:2]
    return ("%s\n%s" % (label, name)).encode(), struct.pack(">ii", w, h) + bgr.astype("uint8").tobytes()


def decode_image_record(key, value):
    """-> (label float, name, [H, W, 3] uint8 BGR array)."""
    import numpy as np
    parts = key.decode().split("\n")
    w, h = struct.unpack_from(">ii", value, 0)
    img = np.frombuffer(value, np.uint8, count=3 * w * h, offset=8).reshape(h, w, 3)
    return float(parts[0]), (parts[1] if len(parts) > 1 else ""), img
