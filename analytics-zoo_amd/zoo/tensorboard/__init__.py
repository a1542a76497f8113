"""TensorBoard event files (Zs/tensorboard/*: EventWriter, FileWriter,
RecordWriter with TFRecord framing + masked CRC32C, Summary, FileReader).

Events are hand-encoded ``tensorflow.Event`` protobufs (wall_time, step,
summary{value{tag, simple_value}}) framed by the native C++ TFRecord writer
(zoo._runtime.tfrecord_frame); a background thread flushes them like the
reference's EventWriter. ``read_scalar`` parses the files back (FileReader).
"""
import glob
import os
import queue
import socket
import struct
import threading
import time


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num, wt, payload):
    key = _varint((num << 3) | wt)
    if wt == 2:
        return key + _varint(len(payload)) + payload
    return key + payload


def _frame(data):
    try:
        import zoo._runtime as R
        return R.tfrecord_frame(data)
    except ImportError:  # pure-python fallback (CRC32C)
        def crc(b):
            c = 0xFFFFFFFF
            for x in b:
                c ^= x
                for _ in range(8):
                    c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
            return c ^ 0xFFFFFFFF

        def mask(c):
            return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF
        ln = struct.pack("<Q", len(data))
        return ln + struct.pack("<I", mask(crc(ln))) + data + struct.pack("<I", mask(crc(data)))


def scalar_event(tag, value, step, wall_time=None):
    val = _field(1, 2, tag.encode()) + _field(2, 5, struct.pack("<f", float(value)))
    summary = _field(1, 2, val)
    ev = _field(1, 1, struct.pack("<d", wall_time or time.time())) + _field(2, 0, _varint(int(step))) + \
        _field(5, 2, summary)
    return ev


def histogram_event(tag, values, step, wall_time=None):
    import numpy as np
    v = np.asarray(values, dtype=np.float64).reshape(-1)
    edges = np.linspace(v.min(), v.max() if v.max() > v.min() else v.min() + 1, 31)
    counts, _ = np.histogram(v, bins=edges)
    h = _field(1, 1, struct.pack("<d", v.min())) + _field(2, 1, struct.pack("<d", v.max())) + \
        _field(3, 1, struct.pack("<d", float(v.size))) + _field(4, 1, struct.pack("<d", float(v.sum()))) + \
        _field(5, 1, struct.pack("<d", float((v * v).sum()))) + \
        _field(6, 2, b"".join(struct.pack("<d", e) for e in edges[1:])) + \
        _field(7, 2, b"".join(struct.pack("<d", float(c)) for c in counts))
    val = _field(1, 2, tag.encode()) + _field(5, 2, h)
    return _field(1, 1, struct.pack("<d", wall_time or time.time())) + _field(2, 0, _varint(int(step))) + \
        _field(5, 2, _field(1, 2, val))


class FileWriter:
    """Async event-file writer (FileWriter.scala + EventWriter.scala)."""

    def __init__(self, log_dir, flush_secs=1.0):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "events.out.tfevents.%d.%s" % (int(time.time()), socket.gethostname()))
        self.q = queue.Queue()
        self.flush_secs = flush_secs
        self._f = open(self.path, "ab")
        ver = _field(1, 1, struct.pack("<d", time.time())) + _field(3, 2, b"brain.Event:2")
        self._f.write(_frame(ver))
        self._stop = False
        self._t = threading.Thread(target=self._run, daemon=True)
        self._t.start()

    def _run(self):
        while not self._stop or not self.q.empty():
            try:
                ev = self.q.get(timeout=self.flush_secs)
                self._f.write(_frame(ev))
                while not self.q.empty():
                    self._f.write(_frame(self.q.get_nowait()))
                self._f.flush()
            except queue.Empty:
                continue

    def add_event(self, ev):
        self.q.put(ev)

    def add_scalar(self, tag, value, step):
        self.add_event(scalar_event(tag, value, step))

    def add_histogram(self, tag, values, step):
        self.add_event(histogram_event(tag, values, step))

    def flush(self):
        while not self.q.empty():
            time.sleep(0.01)
        self._f.flush()

    def close(self):
        self._stop = True
        self._t.join(timeout=5)
        self._f.close()


def read_records(path):
    with open(path, "rb") as f:
        data = f.read()
    off = 0
    while off + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, off)
        off += 12
        yield data[off:off + n]
        off += n + 4


def _pb(data):
    try:
        import zoo._runtime as R
        return R.pb_fields(data)
    except ImportError:
        from zoo.utils.bigdl_proto import pb_fields_py
        return pb_fields_py(data)


def read_scalar(log_dir, tag):
    """[(step, value, wall_time)] for ``tag`` over every event file in log_dir (FileReader.readScalar)."""
    out = []
    for p in sorted(glob.glob(os.path.join(log_dir, "events.out.tfevents.*"))):
        for rec in read_records(p):
            wall, step, summ = 0.0, 0, None
            for f, wt, v in _pb(rec):
                if f == 1 and wt == 1:
                    wall = struct.unpack("<d", struct.pack("<Q", v))[0]
                elif f == 2:
                    step = v
                elif f == 5:
                    summ = v
            if summ is None:
                continue
            for f, wt, val in _pb(summ):
                if f != 1:
                    continue
                t, sv = None, None
                for f2, wt2, v2 in _pb(val):
                    if f2 == 1:
                        t = v2.decode()
                    elif f2 == 2 and wt2 == 5:
                        sv = struct.unpack("<f", struct.pack("<I", v2))[0]
                if t == tag and sv is not None:
                    out.append((step, sv, wall))
    return out


class _Summary:
    folder = "train"

    def __init__(self, log_dir, app_name):
        self.dir = os.path.join(log_dir, app_name, self.folder)
        self.writer = FileWriter(self.dir)

    def add_scalar(self, tag, value, step):
        self.writer.add_scalar(tag, value, step)

    def add_histogram(self, tag, values, step):
        self.writer.add_histogram(tag, values, step)

    def read_scalar(self, tag):
        self.writer.flush()
        return read_scalar(self.dir, tag)

    def close(self):
        self.writer.close()


class TrainSummary(_Summary):
    folder = "train"


class ValidationSummary(_Summary):
    folder = "validation"
