"""Minimal HDF5 reader / writer (standard library + numpy), enough for Keras weight
files: the reference's ``Net.load_keras(json, hdf5)`` and ``saveToKeras2`` go through
h5py/Keras (Py/pipeline/api/net/net_load.py:127-138), neither of which exists here.

Reader: superblock v0/v1 and v2/v3; object headers v1 and v2 (with continuation
blocks); old-style groups (symbol table -> v1 B-tree -> SNOD + local heap) and
new-style compact groups (link messages); datasets with compact, contiguous or chunked
(v1 B-tree, deflate / shuffle filters) layout; attributes v1-v3; fixed-point, float and
fixed-length string types (variable-length strings from the global heap too).

Writer: superblock v0 with old-style groups, contiguous datasets and attributes --
files the HDF5 library (and h5py) read back.
"""
import struct
import zlib

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
_SIG = b"\x89HDF\r\n\x1a\n"


class _Datatype:
    __slots__ = ("cls", "size", "dtype", "strpad", "vlen")

    def __init__(self, cls, size, dtype=None, strpad=0, vlen=False):
        self.cls, self.size, self.dtype, self.strpad, self.vlen = cls, size, dtype, strpad, vlen


class Dataset:
    def __init__(self, f, name, hdr):
        self.file, self.name, self._hdr = f, name, hdr
        self.attrs = hdr["attrs"]
        self.shape = hdr["shape"]
        self.dtype = hdr["dtype"].dtype

    def __getitem__(self, item):
        return self.read()[item]

    def read(self):
        return self.file._read_data(self._hdr)

    def __array__(self, dtype=None):
        a = self.read()
        return a if dtype is None else a.astype(dtype)


class Group:
    def __init__(self, f, name, hdr):
        self.file, self.name, self._hdr = f, name, hdr
        self.attrs = hdr["attrs"]
        self._links = hdr["links"]

    def keys(self):
        return list(self._links.keys())

    def __contains__(self, k):
        try:
            self[k]
            return True
        except KeyError:
            return False

    def __iter__(self):
        return iter(self.keys())

    def __getitem__(self, path):
        node = self
        for part in [p for p in str(path).split("/") if p]:
            if not isinstance(node, Group) or part not in node._links:
                raise KeyError(path)
            node = node.file._object(node._links[part], node.name.rstrip("/") + "/" + part)
        return node

    def items(self):
        return [(k, self[k]) for k in self.keys()]


class File(Group):
    """Read-only HDF5 file: ``File(path)["group/dataset"].read()``, ``.attrs``."""

    def __init__(self, path):
        with open(path, "rb") as fh:
            self.buf = fh.read()
        b = self.buf
        base = b.find(_SIG)
        if base < 0:
            raise ValueError("%s is not an HDF5 file" % path)
        self._base = base
        ver = b[base + 8]
        if ver in (0, 1):
            self.so, self.sl = b[base + 13], b[base + 14]
            self.leaf_k, = struct.unpack_from("<H", b, base + 16)
            p = base + 24 + (4 if ver == 1 else 0)
            p += 4 * self.so  # base, free-space, eof, driver addresses
            root = self._u(p + self.so, self.so)   # root symbol-table entry: name offset, header address
        elif ver in (2, 3):
            self.so, self.sl = b[base + 9], b[base + 10]
            p = base + 12
            root = self._u(p + 3 * self.so, self.so)
        else:
            raise NotImplementedError("HDF5 superblock version %d" % ver)
        self._cache = {}
        super().__init__(self, "/", self._header(root))

    # -- primitives
    def _u(self, pos, n):
        return int.from_bytes(self.buf[pos:pos + n], "little")

    def _addr(self, a):
        return a + self._base

    def _object(self, addr, name):
        hdr = self._cache.get(addr)
        if hdr is None:
            hdr = self._cache[addr] = self._header(addr)
        return Group(self, name, hdr) if hdr["kind"] == "group" else Dataset(self, name, hdr)

    # -- object headers
    def _messages(self, addr):
        b = self.buf
        a = self._addr(addr)
        msgs = []
        if b[a:a + 4] == b"OHDR":
            flags = b[a + 5]
            p = a + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            csz = 1 << (flags & 3)
            size = self._u(p, csz)
            p += csz
            tracked = bool(flags & 0x04)
            blocks = [(p, p + size)]
            while blocks:
                s, e = blocks.pop(0)
                q = s
                while q + 4 <= e:
                    mtype = b[q]
                    msize = struct.unpack_from("<H", b, q + 1)[0]
                    q += 4 + (2 if tracked else 0)
                    data = b[q:q + msize]
                    q += msize
                    if mtype == 0x10:
                        ca, cl = self._u_bytes(data, 0, self.so), self._u_bytes(data, self.so, self.sl)
                        cs = self._addr(ca)
                        blocks.append((cs + 4, cs + cl - 4))   # "OCHK" + messages + checksum
                    elif mtype != 0:
                        msgs.append((mtype, data))
            return msgs
        # version 1
        nmsg = struct.unpack_from("<H", b, a + 2)[0]
        hsize = struct.unpack_from("<I", b, a + 8)[0]
        blocks = [(a + 16, a + 16 + hsize)]
        count = 0
        while blocks and count < nmsg:
            s, e = blocks.pop(0)
            q = s
            while q + 8 <= e and count < nmsg:
                mtype, msize = struct.unpack_from("<HH", b, q)
                data = b[q + 8:q + 8 + msize]
                q += 8 + msize
                count += 1
                if mtype == 0x10:
                    ca, cl = self._u(q - msize, self.so), self._u(q - msize + self.so, self.sl)
                    blocks.append((self._addr(ca), self._addr(ca) + cl))
                else:
                    msgs.append((mtype, data))
        return msgs

    def _header(self, addr):
        info = {"attrs": {}, "links": {}, "kind": "group", "shape": None, "dtype": None, "layout": None,
                "filters": []}
        symtab = None
        for mtype, d in self._messages(addr):
            if mtype == 0x0001:
                info["shape"] = self._dataspace(d)
                info["kind"] = "dataset"
            elif mtype == 0x0003:
                info["dtype"] = self._datatype(d)[0]
            elif mtype == 0x0008:
                info["layout"] = d
            elif mtype == 0x000B:
                info["filters"] = self._filters(d)
            elif mtype == 0x000C:
                k, v = self._attribute(d)
                info["attrs"][k] = v
            elif mtype == 0x0011:
                symtab = (self._u_bytes(d, 0, self.so), self._u_bytes(d, self.so, self.so))
            elif mtype == 0x0006:
                name, target = self._link(d)
                if target is not None:
                    info["links"][name] = target
        if symtab is not None:
            info["links"].update(self._group_links(*symtab))
        if info["layout"] is None:
            info["kind"] = "group"
        return info

    @staticmethod
    def _u_bytes(d, off, n):
        return int.from_bytes(d[off:off + n], "little")

    def _dataspace(self, d):
        ver, rank, flags = d[0], d[1], d[2]
        p = 8 if ver == 1 else 4
        if ver == 2 and d[3] == 0:
            return ()
        return tuple(self._u_bytes(d, p + i * self.sl, self.sl) for i in range(rank))

    def _datatype(self, d):
        cls, ver = d[0] & 0x0F, d[0] >> 4
        bits = d[1] | (d[2] << 8) | (d[3] << 16)
        size = struct.unpack_from("<I", d, 4)[0]
        end = "<" if not bits & 1 else ">"
        if cls == 0:
            signed = bool(bits & 0x08)
            dt = np.dtype("%s%s%d" % (end, "i" if signed else "u", size))
            return _Datatype(0, size, dt), 8 + 4
        if cls == 1:
            return _Datatype(1, size, np.dtype("%sf%d" % (end, size))), 8 + 12
        if cls == 3:
            return _Datatype(3, size, np.dtype("S%d" % size), strpad=bits & 0x0F), 8
        if cls == 9:
            base, blen = self._datatype(d[8:])
            is_str = (bits & 0x0F) == 1
            return _Datatype(9, size, np.dtype(object), vlen=is_str), 8 + blen
        raise NotImplementedError("HDF5 datatype class %d" % cls)

    def _filters(self, d):
        ver, n = d[0], d[1]
        p = 8 if ver == 1 else 2
        out = []
        for _ in range(n):
            fid, = struct.unpack_from("<H", d, p)
            if ver == 1 or fid >= 256:
                nlen, flags, ncv = struct.unpack_from("<HHH", d, p + 2)
                p += 8
                if nlen:
                    p += (nlen + 7) // 8 * 8 if ver == 1 else nlen
            else:
                flags, ncv = struct.unpack_from("<HH", d, p + 2)
                p += 6
            cvals = struct.unpack_from("<%dI" % ncv, d, p)
            p += 4 * ncv + (4 if ver == 1 and ncv % 2 else 0)
            out.append((fid, cvals))
        return out

    def _attribute(self, d):
        ver = d[0]
        nsz, tsz, ssz = struct.unpack_from("<HHH", d, 2)
        p = 8 + (1 if ver == 3 else 0)
        pad = (lambda n: (n + 7) // 8 * 8) if ver == 1 else (lambda n: n)
        name = d[p:p + nsz].split(b"\0")[0].decode("utf-8")
        p += pad(nsz)
        dt, _ = self._datatype(d[p:p + tsz])
        p += pad(tsz)
        shape = self._dataspace(d[p:p + ssz])
        p += pad(ssz)
        return name, self._decode(d[p:], dt, shape)

    def _decode(self, raw, dt, shape):
        n = int(np.prod(shape)) if shape else 1
        if dt.cls == 9:
            vals = []
            for i in range(n):
                p = i * (4 + self.so + 4)
                ln = struct.unpack_from("<I", raw, p)[0]
                col, idx = self._u_bytes(raw, p + 4, self.so), struct.unpack_from("<I", raw, p + 4 + self.so)[0]
                s = self._global_heap(col, idx)[:ln] if dt.vlen else self._global_heap(col, idx)
                vals.append(s.decode("utf-8") if dt.vlen else s)
            arr = np.array(vals, dtype=object)
        else:
            arr = np.frombuffer(bytes(raw[:n * dt.size]), dtype=dt.dtype, count=n).copy()
        return arr.reshape(shape) if shape else arr[0]

    def _global_heap(self, col, idx):
        b = self.buf
        a = self._addr(col)
        size = self._u(a + 8, self.sl)
        p, end = a + 8 + self.sl, a + size
        while p < end:
            hid = struct.unpack_from("<H", b, p)[0]
            osz = self._u(p + 8, self.sl)
            if hid == idx:
                return bytes(b[p + 8 + self.sl:p + 8 + self.sl + osz])
            if hid == 0:
                break
            p += 8 + self.sl + (osz + 7) // 8 * 8
        raise KeyError("global heap object %d" % idx)

    def _link(self, d):
        flags = d[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = d[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        lsz = 1 << (flags & 3)
        nlen = self._u_bytes(d, p, lsz)
        p += lsz
        name = d[p:p + nlen].decode("utf-8")
        p += nlen
        return name, (self._u_bytes(d, p, self.so) if ltype == 0 else None)

    def _group_links(self, btree, heap):
        b = self.buf
        h = self._addr(heap)
        if b[h:h + 4] != b"HEAP":
            raise ValueError("bad local heap")
        data = self._addr(self._u(h + 8 + 2 * self.sl, self.so))
        links = {}

        def walk(node):
            n = self._addr(node)
            if b[n:n + 4] != b"TREE":
                raise ValueError("bad B-tree node")
            level = b[n + 5]
            used = struct.unpack_from("<H", b, n + 6)[0]
            p = n + 8 + 2 * self.so + self.sl   # first key
            for _ in range(used):
                child = self._u(p, self.so)
                p += self.so + self.sl
                if level > 0:
                    walk(child)
                else:
                    s = self._addr(child)
                    if b[s:s + 4] != b"SNOD":
                        raise ValueError("bad symbol table node")
                    nsym = struct.unpack_from("<H", b, s + 6)[0]
                    q = s + 8
                    for _ in range(nsym):
                        noff, oaddr = self._u(q, self.so), self._u(q + self.so, self.so)
                        end = b.index(b"\0", data + noff)
                        links[b[data + noff:end].decode("utf-8")] = oaddr
                        q += 2 * self.so + 24
        walk(btree)
        return links

    # -- dataset data
    def _read_data(self, hdr):
        d, dt, shape = hdr["layout"], hdr["dtype"], hdr["shape"]
        n = int(np.prod(shape)) if shape else 1
        ver = d[0]
        if ver == 3:
            cls = d[1]
            if cls == 0:
                size = struct.unpack_from("<H", d, 2)[0]
                return self._decode(d[4:4 + size], dt, shape)
            if cls == 1:
                addr = self._u_bytes(d, 2, self.so)
                if addr == UNDEF:
                    return np.zeros(shape, dt.dtype)
                a = self._addr(addr)
                return self._decode(self.buf[a:a + n * dt.size], dt, shape)
            if cls == 2:
                rank = d[2] - 1
                addr = self._u_bytes(d, 3, self.so)
                cdims = struct.unpack_from("<%dI" % rank, d, 3 + self.so)
                return self._read_chunked(addr, cdims, dt, shape, hdr["filters"])
            raise NotImplementedError("HDF5 layout class %d" % cls)
        if ver in (1, 2):
            rank, cls = d[1], d[2]
            p = 8
            if cls == 0:
                dims = struct.unpack_from("<%dI" % rank, d, p)
                p += 4 * rank
                size = struct.unpack_from("<I", d, p)[0]
                return self._decode(d[p + 4:p + 4 + size], dt, shape)
            addr = self._u_bytes(d, p, self.so)
            p += self.so
            dims = struct.unpack_from("<%dI" % rank, d, p)
            if cls == 1:
                a = self._addr(addr)
                return self._decode(self.buf[a:a + n * dt.size], dt, shape)
            return self._read_chunked(addr, dims[:-1], dt, shape, hdr["filters"])
        raise NotImplementedError("HDF5 layout message version %d" % ver)

    def _read_chunked(self, btree, cdims, dt, shape, filters):
        b = self.buf
        out = np.zeros(shape, dt.dtype)
        rank = len(shape)
        csize = int(np.prod(cdims)) * dt.size

        def unfilter(raw, mask):
            for i, (fid, cv) in reversed(list(enumerate(filters))):
                if mask & (1 << i):
                    continue
                if fid == 1:
                    raw = zlib.decompress(raw)
                elif fid == 2:
                    es = cv[0] if cv else dt.size
                    a = np.frombuffer(raw, np.uint8).reshape(es, -1)
                    raw = a.T.tobytes()
                elif fid == 3:   # fletcher32: drop the trailing checksum
                    raw = raw[:-4]
                else:
                    raise NotImplementedError("HDF5 filter %d" % fid)
            return raw

        def walk(node):
            n = self._addr(node)
            if b[n:n + 4] != b"TREE":
                raise ValueError("bad chunk B-tree")
            level = b[n + 5]
            used = struct.unpack_from("<H", b, n + 6)[0]
            ksz = 8 + 8 * (rank + 1)
            p = n + 8 + 2 * self.so
            for _ in range(used):
                nbytes, mask = struct.unpack_from("<II", b, p)
                offs = struct.unpack_from("<%dQ" % rank, b, p + 8)
                child = self._u(p + ksz, self.so)
                p += ksz + self.so
                if level > 0:
                    walk(child)
                    continue
                a = self._addr(child)
                raw = unfilter(bytes(b[a:a + nbytes]), mask)[:csize]
                chunk = np.frombuffer(raw, dt.dtype, count=int(np.prod(cdims))).reshape(cdims)
                sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, shape))
                out[sl] = chunk[tuple(slice(0, x.stop - x.start) for x in sl)]
        walk(btree)
        return out


def open_file(path):
    return File(path)


# ---------------------------------------------------------------------------
# writer (superblock v0, old-style groups, contiguous datasets)
# ---------------------------------------------------------------------------
class _WNode:
    def __init__(self, kind):
        self.kind, self.children, self.attrs, self.data = kind, {}, {}, None


class Writer:
    """``w = Writer(); w.create_dataset("a/b", arr); w.attrs("a")["k"] = v; w.save(path)``"""

    def __init__(self):
        self.root = _WNode("group")

    def _node(self, path, create_kind="group"):
        node = self.root
        parts = [p for p in str(path).split("/") if p]
        for i, p in enumerate(parts):
            if p not in node.children:
                node.children[p] = _WNode(create_kind if i == len(parts) - 1 else "group")
            node = node.children[p]
        return node

    def create_group(self, path):
        return self._node(path, "group")

    def create_dataset(self, path, data):
        n = self._node(path, "dataset")
        n.kind, n.data = "dataset", np.ascontiguousarray(data)
        return n

    def attrs(self, path="/"):
        return self._node(path).attrs if path not in ("", "/") else self.root.attrs

    # -- encoding helpers
    @staticmethod
    def _dtype_msg(arr):
        dt = arr.dtype
        if dt.kind == "f":
            # IEEE little-endian: bit offset 0, precision, exponent location/size, mantissa location/size, bias
            if dt.itemsize == 4:
                props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            elif dt.itemsize == 8:
                props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            else:
                props = struct.pack("<HHBBBBI", 0, 16, 10, 5, 0, 10, 15)
            # class bit field: byte 0 = LE, pad 0, mantissa normalisation 2 (implied msb); byte 1 = sign location
            b0 = 0x20
            b1 = dt.itemsize * 8 - 1
            return bytes([0x11, b0, b1, 0]) + struct.pack("<I", dt.itemsize) + props
        if dt.kind in "iu":
            b0 = 0x08 if dt.kind == "i" else 0
            return bytes([0x10, b0, 0, 0]) + struct.pack("<I", dt.itemsize) + struct.pack("<HH", 0, dt.itemsize * 8)
        if dt.kind == "S":
            return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", dt.itemsize)   # null-padded ASCII
        raise NotImplementedError("HDF5 writer: dtype %s" % dt)

    @staticmethod
    def _space_msg(shape):
        out = bytes([1, len(shape), 0, 0]) + b"\0" * 4
        for d in shape:
            out += struct.pack("<Q", d)
        return out

    @staticmethod
    def _pad8(b):
        return b + b"\0" * ((-len(b)) % 8)

    @staticmethod
    def _as_array(v):
        if isinstance(v, str):
            v = v.encode("utf-8")
        if isinstance(v, bytes):
            return np.array(v, dtype="S%d" % max(len(v), 1))
        a = np.asarray(v)
        if a.dtype.kind == "U":
            a = np.char.encode(a, "utf-8")
        if a.dtype.kind == "O":
            a = np.array([x.encode("utf-8") if isinstance(x, str) else bytes(x) for x in a.ravel()]).reshape(a.shape)
        if a.dtype.kind == "S" and a.dtype.itemsize == 0:
            a = a.astype("S1")
        if a.dtype == np.bool_:
            a = a.astype(np.uint8)
        return a

    def _attr_msg(self, name, value):
        a = self._as_array(value)
        nm = name.encode("utf-8") + b"\0"
        dt = self._dtype_msg(a)
        sp = self._space_msg(a.shape) if a.shape else bytes([1, 0, 0, 0]) + b"\0" * 4
        head = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(sp))
        return head + self._pad8(nm) + self._pad8(dt) + self._pad8(sp) + a.tobytes()

    def save(self, path):
        out = bytearray()
        so = 8

        def alloc(n, align=8):
            while len(out) % align:
                out.append(0)
            p = len(out)
            out.extend(b"\0" * n)
            return p

        def put(pos, data):
            out[pos:pos + len(data)] = data

        def header(msgs):
            body = b""
            for t, d in msgs:
                d = self._pad8(d)
                body += struct.pack("<HHB3x", t, len(d), 0) + d
            # v1 object header (16-byte prefix incl. alignment)
            hdr = struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4
            pos = alloc(len(hdr) + len(body))
            put(pos, hdr + body)
            return pos

        leaf_k = max(4, (max(self._max_children(self.root), 1) + 1) // 2)
        internal_k = 16
        root_symtab = []

        def write(node, is_root=False):
            msgs = []
            if node.kind == "dataset":
                a = node.data
                if a.dtype == np.bool_:
                    a = a.astype(np.uint8)
                raw = a.tobytes()
                dpos = alloc(max(len(raw), 1)) if raw else UNDEF
                if raw:
                    put(dpos, raw)
                msgs.append((0x0001, self._space_msg(a.shape)))
                msgs.append((0x0003, self._dtype_msg(a)))
                msgs.append((0x0005, bytes([2, 2, 2, 0])))   # fill value v2: allocate late, write never, undefined
                msgs.append((0x0008, bytes([3, 1]) + struct.pack("<QQ", dpos, len(raw))))
            else:
                names = sorted(node.children)
                addrs = {k: write(node.children[k]) for k in names}
                # local heap with the link names (offset 0 = empty string)
                heap_data = bytearray(b"\0" * 8)
                offs = {}
                for k in names:
                    offs[k] = len(heap_data)
                    heap_data += k.encode("utf-8") + b"\0"
                    while len(heap_data) % 8:
                        heap_data.append(0)
                heap_data += b"\0" * 16
                hd = alloc(len(heap_data))
                put(hd, bytes(heap_data))
                hp = alloc(32)
                put(hp, b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap_data), UNDEF, hd))
                # one SNOD with every entry (leaf K in the superblock is set large enough)
                snod = b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names))
                for k in names:
                    snod += struct.pack("<QQII", offs[k], addrs[k], 0, 0) + b"\0" * 16
                sp = alloc(8 + 2 * leaf_k * 40)     # readers size the node by the superblock's leaf K
                put(sp, snod)
                tree = b"TREE" + bytes([0, 0]) + struct.pack("<HQQ", 1 if names else 0, UNDEF, UNDEF)
                tree += struct.pack("<Q", 0) + struct.pack("<Q", sp) + struct.pack("<Q", offs[names[-1]] if names
                                                                                     else 0)
                tp = alloc(8 + 2 * so + (2 * internal_k + 1) * 8 + 2 * internal_k * so)
                put(tp, tree)
                msgs.append((0x0011, struct.pack("<QQ", tp, hp)))
                if is_root:
                    root_symtab.extend([tp, hp])
            for k, v in node.attrs.items():
                msgs.append((0x000C, self._attr_msg(k, v)))
            return header(msgs)

        # superblock v0 placeholder (size 96 with the root symbol-table entry)
        sb = alloc(96)
        root_hdr = write(self.root, is_root=True)
        sbd = _SIG + bytes([0, 0, 0, 0, 0, so, 8, 0]) + struct.pack("<HHI", leaf_k, internal_k, 0)
        sbd += struct.pack("<QQQQ", 0, UNDEF, len(out), UNDEF)
        sbd += struct.pack("<QQII", 0, root_hdr, 1, 0) + struct.pack("<QQ", *root_symtab)
        put(sb, sbd)
        with open(path, "wb") as f:
            f.write(bytes(out))

    def _max_children(self, node):
        m = len(node.children)
        for c in node.children.values():
            if c.kind == "group":
                m = max(m, self._max_children(c))
        return m


__all__ = ["File", "Group", "Dataset", "Writer", "open_file"]
