"""Self-contained HDF5 reader / writer for the dataset files the library uses
(no libhdf5 / h5py needed).

Reference: ``utility/io/hdf5_io.hpp:10-262`` (``ReadHDF5`` of dense and
sparse matrices), ``ml/io.hpp:18-526`` (``write_hdf5`` / ``read_hdf5`` with
datasets ``X``/``Y`` or ``dimensions``/``indptr``/``indices``/``values``),
``ml/skylark_convert2hdf5.cpp``.

Reader coverage (the subset produced by libhdf5 with default/"earliest"
file-format settings and by h5py): superblock versions 0-3; object headers
v1 and v2 (``OHDR``, with continuation blocks); groups stored as symbol
tables (v1 B-tree + local heap) or as link messages (compact v2 groups);
datasets with contiguous, compact or chunked layout (v1 B-tree chunk index),
filters deflate (zlib), shuffle and fletcher32; little/big-endian integer
and IEEE float element types.  Writer: superblock v0, one root group
(symbol table), contiguous little-endian datasets — readable by libhdf5.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF


class H5Error(Exception):
    pass


# ===================================================================== reader
class _Reader:
    def __init__(self, data: bytes):
        self.d = data
        if data[:8] != b"\x89HDF\r\n\x1a\n":
            raise H5Error("not an HDF5 file (bad signature)")
        ver = data[8]
        if ver in (0, 1):
            self.so, self.sl = data[13], data[14]
            p = 24 if ver == 0 else 28
            self.base = self.off(p)
            p += 4 * self.so                     # base, free-space, EOF, driver
            # root group symbol table entry
            self.root = self.off(p + self.so)    # object header address
            self.root_scratch = data[p + 2 * self.so + 8: p + 2 * self.so + 24]
            self.root_cache = struct.unpack_from("<I", data, p + 2 * self.so)[0]
        elif ver in (2, 3):
            self.so, self.sl = data[9], data[10]
            p = 12
            self.base = self.off(p)
            self.root = self.off(p + 3 * self.so)   # base, ext, EOF, root object header
            self.root_cache = 0
        else:
            raise H5Error(f"unsupported superblock version {ver}")

    # ---------------------------------------------------------- primitives
    def off(self, p):
        return int.from_bytes(self.d[p:p + self.so], "little")

    def length(self, p):
        return int.from_bytes(self.d[p:p + self.sl], "little")

    # ------------------------------------------------------ object headers
    def messages(self, addr):
        """[(type, data bytes)] of the object header at addr (v1 or v2)."""
        d = self.d
        out = []
        if d[addr:addr + 4] == b"OHDR":
            ver = d[addr + 4]
            if ver != 2:
                raise H5Error("unsupported object header version")
            flags = d[addr + 5]
            p = addr + 6
            if flags & 0x20:
                p += 16                                  # times
            if flags & 0x10:
                p += 4                                   # attribute phase change
            csize = 1 << (flags & 3)
            size = int.from_bytes(d[p:p + csize], "little")
            p += csize
            blocks = [(p, size)]
            while blocks:
                bp, bs = blocks.pop(0)
                end = bp + bs
                q = bp
                while q + 4 <= end:
                    mtype = d[q]
                    msize = struct.unpack_from("<H", d, q + 1)[0]
                    mflags = d[q + 3]
                    q += 4
                    if flags & 0x04:
                        q += 2                           # creation order
                    body = d[q:q + msize]
                    q += msize
                    if mtype == 0x10:                    # continuation
                        caddr = self.off_b(body, 0)
                        clen = int.from_bytes(body[self.so:self.so + self.sl], "little")
                        blocks.append((caddr + 4, clen - 4 - 4))   # "OCHK" ... checksum
                    elif mtype != 0:
                        out.append((mtype, body, mflags))
            return out
        ver = d[addr]
        if ver != 1:
            raise H5Error(f"unsupported object header version {ver}")
        nmsg = struct.unpack_from("<H", d, addr + 2)[0]
        hsize = struct.unpack_from("<I", d, addr + 8)[0]
        blocks = [(addr + 16, hsize)]
        count = 0
        while blocks and count < nmsg:
            bp, bs = blocks.pop(0)
            q, end = bp, bp + bs
            while q + 8 <= end and count < nmsg:
                mtype, msize, mflags = struct.unpack_from("<HHB", d, q)
                body = d[q + 8:q + 8 + msize]
                q += 8 + msize
                count += 1
                if mtype == 0x10:
                    caddr = self.off_b(body, 0)
                    clen = int.from_bytes(body[self.so:self.so + self.sl], "little")
                    blocks.append((caddr, clen))
                elif mtype != 0:
                    out.append((mtype, body, mflags))
        return out

    def off_b(self, b, p):
        return int.from_bytes(b[p:p + self.so], "little")

    # ------------------------------------------------------------- groups
    def group_links(self, addr, scratch=None, cache=0):
        """{name: object header address} of a group."""
        links = {}
        if cache == 1 and scratch is not None:
            btree, heap = self.off_b(scratch, 0), self.off_b(scratch, self.so)
            self._symtab(btree, heap, links)
            return links
        for mtype, body, _ in self.messages(addr):
            if mtype == 0x11:                                   # symbol table
                self._symtab(self.off_b(body, 0), self.off_b(body, self.so), links)
            elif mtype == 0x06:                                 # link message
                name, target = self._link(body)
                if target is not None:
                    links[name] = target
            elif mtype == 0x02:                                 # link info (dense storage)
                fheap = self.off_b(body, 2 + (8 if body[1] & 1 else 0))
                if fheap != UNDEF:
                    raise H5Error("dense (fractal-heap) groups are not supported")
        return links

    def _link(self, b):
        flags = b[1]
        p = 2
        ltype = 0
        if flags & 0x08:
            ltype = b[p]
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        lsize = 1 << (flags & 3)
        nlen = int.from_bytes(b[p:p + lsize], "little")
        p += lsize
        name = b[p:p + nlen].decode()
        p += nlen
        if ltype != 0:
            return name, None                                   # soft / external link
        return name, self.off_b(b, p)

    def _symtab(self, btree, heap, links):
        d = self.d
        if d[heap:heap + 4] != b"HEAP":
            raise H5Error("bad local heap")
        hdata = self.off(heap + 8 + 2 * self.sl)

        def name_at(o):
            e = d.find(b"\x00", hdata + o)
            if e < 0:
                raise H5Error("unterminated link name in the local heap")
            return d[hdata + o:e].decode()

        def walk(node):
            if d[node:node + 4] != b"TREE":
                raise H5Error("bad group B-tree node")
            level = d[node + 5]
            used = struct.unpack_from("<H", d, node + 6)[0]
            p = node + 8 + 2 * self.so
            for _ in range(used):
                p += self.sl                                    # key
                child = self.off(p)
                p += self.so
                if level > 0:
                    walk(child)
                else:
                    if d[child:child + 4] != b"SNOD":
                        raise H5Error("bad symbol node")
                    nsym = struct.unpack_from("<H", d, child + 6)[0]
                    q = child + 8
                    for _ in range(nsym):
                        nm = name_at(self.off(q))
                        links[nm] = self.off(q + self.so)
                        q += 2 * self.so + 24

        walk(btree)

    # ----------------------------------------------------------- datasets
    def dataset(self, addr):
        shape = dtype = layout = None
        filters = []
        for mtype, body, _ in self.messages(addr):
            if mtype == 0x01:
                shape = self._dataspace(body)
            elif mtype == 0x03:
                dtype = self._datatype(body)
            elif mtype == 0x08:
                layout = body
            elif mtype == 0x0B:
                filters = self._filters(body)
        if shape is None or dtype is None or layout is None:
            raise H5Error("object is not a dataset")
        return shape, dtype, layout, filters

    def _dataspace(self, b):
        ver, rank = b[0], b[1]
        p = 8 if ver == 1 else 4
        return tuple(int.from_bytes(b[p + i * self.sl:p + (i + 1) * self.sl], "little") for i in range(rank))

    def _datatype(self, b):
        cls = b[0] & 0x0F
        bits = b[1]
        size = struct.unpack_from("<I", b, 4)[0]
        order = ">" if bits & 1 else "<"
        if cls == 0:
            signed = bool(bits & 0x08)
            return np.dtype(f"{order}{'i' if signed else 'u'}{size}")
        if cls == 1:
            return np.dtype(f"{order}f{size}")
        raise H5Error(f"unsupported datatype class {cls}")

    def _filters(self, b):
        ver, n = b[0], b[1]
        p = 8 if ver == 1 else 2
        out = []
        for _ in range(n):
            fid = struct.unpack_from("<H", b, p)[0]
            p += 2
            nlen = 0
            if ver == 1 or fid >= 256:
                nlen = struct.unpack_from("<H", b, p)[0]
                p += 2
            flags, ncv = struct.unpack_from("<HH", b, p)
            p += 4
            if ver == 1:
                p += (nlen + 7) & ~7
            else:
                p += nlen
            cv = struct.unpack_from(f"<{ncv}I", b, p) if ncv else ()
            p += 4 * ncv
            if ver == 1 and ncv % 2:
                p += 4
            out.append((fid, cv))
        return out

    def read_dataset(self, addr) -> np.ndarray:
        shape, dt, lay, filters = self.dataset(addr)
        n = int(np.prod(shape)) if shape else 1
        ver = lay[0]
        if ver == 3 or ver == 4:
            cls = lay[1]
            if cls == 0:
                size = struct.unpack_from("<H", lay, 2)[0]
                raw = lay[4:4 + size]
                return np.frombuffer(raw, dt, n).reshape(shape).copy()
            if cls == 1:
                a = self.off_b(lay, 2)
                if a == UNDEF:
                    return np.zeros(shape, dt)
                return np.frombuffer(self.d, dt, n, a).reshape(shape).copy()
            if cls == 2:
                if ver != 3:
                    raise H5Error("only v1-B-tree chunk indexes are supported")
                rank = lay[2]
                btree = self.off_b(lay, 3)
                cdims = struct.unpack_from(f"<{rank}I", lay, 3 + self.so)
                return self._read_chunked(btree, shape, cdims[:-1], dt, filters)
            raise H5Error(f"unsupported layout class {cls}")
        # layout message versions 1 / 2
        rank = lay[1]
        cls = lay[2]
        p = 8
        if cls == 0:
            raise H5Error("compact layout v1/2 unsupported")
        a = self.off_b(lay, p)
        p += self.so
        dims = struct.unpack_from(f"<{rank}I", lay, p)
        if cls == 1:
            return np.frombuffer(self.d, dt, n, a).reshape(shape).copy()
        return self._read_chunked(a, shape, dims[:-1] if len(dims) > len(shape) else dims, dt, filters)

    def _read_chunked(self, btree, shape, cdims, dt, filters):
        out = np.zeros(shape, dt)
        rank = len(shape)
        if btree == UNDEF:
            return out
        d = self.d
        esz = dt.itemsize

        def decode(raw, mask):
            for i, (fid, cv) in reversed(list(enumerate(filters))):
                if mask & (1 << i):
                    continue
                if fid == 1:
                    raw = zlib.decompress(raw)
                elif fid == 2:
                    a = np.frombuffer(raw, np.uint8)
                    raw = a.reshape(esz, -1).T.tobytes()
                elif fid == 3:
                    raw = raw[:-4]
                else:
                    raise H5Error(f"unsupported filter {fid}")
            return raw

        def walk(node):
            if d[node:node + 4] != b"TREE":
                raise H5Error("bad chunk B-tree node")
            level = d[node + 5]
            used = struct.unpack_from("<H", d, node + 6)[0]
            p = node + 8 + 2 * self.so
            ksz = 8 + 8 * (rank + 1)
            for _ in range(used):
                csize, mask = struct.unpack_from("<II", d, p)
                offs = struct.unpack_from(f"<{rank}Q", d, p + 8)
                child = self.off(p + ksz)
                p += ksz + self.so
                if level > 0:
                    walk(child)
                    continue
                raw = decode(d[child:child + csize], mask)
                chunk = np.frombuffer(raw, dt, int(np.prod(cdims))).reshape(cdims)
                sl_out = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, shape))
                sl_in = tuple(slice(0, s.stop - s.start) for s in sl_out)
                out[sl_out] = chunk[sl_in]

        walk(btree)
        return out


class H5File:
    """Read-only view of an HDF5 file: ``f.keys()``, ``f["name"]`` -> ndarray,
    nested paths ``"group/name"``."""

    def __init__(self, path):
        # memory-mapped: a rank that reads a hyperslab touches only its pages
        import mmap
        self._fh = open(path, "rb")
        try:
            self._mm = mmap.mmap(self._fh.fileno(), 0, access=mmap.ACCESS_READ)
        except ValueError:            # empty file
            self._mm = b""
        self._r = _Reader(self._mm)
        r = self._r
        self._root = r.group_links(r.root, r.root_scratch if r.root_cache == 1 else None, r.root_cache)

    def keys(self):
        return list(self._root.keys())

    def __contains__(self, name):
        try:
            self._resolve(name)
            return True
        except KeyError:
            return False

    def _resolve(self, name):
        links = self._root
        parts = [p for p in name.split("/") if p]
        for i, part in enumerate(parts):
            if part not in links:
                raise KeyError(name)
            addr = links[part]
            if i == len(parts) - 1:
                return addr
            links = self._r.group_links(addr)
        raise KeyError(name)

    def __getitem__(self, name) -> np.ndarray:
        return self._r.read_dataset(self._resolve(name))

    def shape(self, name):
        return self._r.dataset(self._resolve(name))[0]

    def read_slice(self, name, axis: int, s0: int, s1: int) -> np.ndarray:
        """``f[name]`` restricted to [s0, s1) along ``axis``.  Contiguous
        datasets are sliced from a zero-copy view of the mapping (only the
        slab's pages are read); chunked / compact ones are read whole."""
        r = self._r
        addr = self._resolve(name)
        shape, dt, lay, _ = r.dataset(addr)
        a = None
        if lay[0] in (3, 4) and lay[1] == 1:
            a = r.off_b(lay, 2)
        elif lay[0] in (1, 2) and lay[2] == 1:
            a = r.off_b(lay, 8)
        if a is None or a == UNDEF:
            full = r.read_dataset(addr)
        else:
            n = int(np.prod(shape)) if shape else 1
            full = np.frombuffer(r.d, dt, n, a).reshape(shape)
        sl = [slice(None)] * len(shape)
        sl[axis] = slice(s0, s1)
        out = np.array(full[tuple(sl)], copy=True, order="C")   # never a view of the mapping
        del full
        return out

    def close(self):
        self._r = None
        if hasattr(self._mm, "close"):
            try:
                self._mm.close()
            except BufferError:   # a caller still holds a view: the GC unmaps later
                pass
        self._fh.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
        return False


# ===================================================================== writer
def write_h5(path, datasets: dict):
    """Write ``{name: ndarray}`` as contiguous little-endian datasets in the
    root group (superblock v0, symbol-table group)."""
    so = sl = 8
    names = list(datasets)
    arrays = [np.ascontiguousarray(np.asarray(datasets[n])) for n in names]
    for a in arrays:
        if a.dtype.kind not in "fiu":
            raise H5Error(f"unsupported dtype {a.dtype}")
    arrays = [a.astype(a.dtype.newbyteorder("<")) for a in arrays]
    out = bytearray()

    def align8():
        while len(out) % 8:
            out.append(0)

    # layout: superblock (96) | root object header | local heap (+data) | B-tree | SNOD | dataset headers | data
    SB = 96
    heap_names = b"\x00" * 8                          # offset 0: empty name
    name_off = []
    for n in names:
        name_off.append(len(heap_names))
        nb = n.encode() + b"\x00"
        nb += b"\x00" * ((8 - len(nb) % 8) % 8)
        heap_names += nb
    root_oh = SB
    root_oh_size = 16 + 8 + 16 + 8                     # header + symbol table message (16) + null msg pad
    heap = root_oh + 16 + 8 + 16
    heap_hdr = 32
    heap_data = heap + heap_hdr
    btree = heap_data + len(heap_names)
    btree_size = 8 + 2 * so + (2 * 16 + 1) * sl + 2 * 16 * so     # leaf K=4 -> room for 2K entries
    btree_size = 8 + 2 * so + sl + 1 * (so + sl)                    # we write one child
    # allocate generously for the fixed-size node libhdf5 expects (2K children, 2K+1 keys)
    K = 4
    btree_full = 8 + 2 * so + (2 * K + 1) * sl + 2 * K * so
    snod = btree + btree_full
    nent = max(2 * K, len(names))
    snod_size = 8 + nent * (2 * so + 24)
    ds_hdr = []
    p = snod + snod_size
    p = (p + 7) & ~7
    for a in arrays:
        ds_hdr.append(p)
        p += _ds_header_size(a, so, sl)
        p = (p + 7) & ~7
    data_addr = []
    for a in arrays:
        data_addr.append(p)
        p += a.nbytes
        p = (p + 7) & ~7
    eof = p

    # superblock v0
    out += b"\x89HDF\r\n\x1a\n" + bytes([0, 0, 0, 0, 0, so, sl, 0]) + struct.pack("<HHI", K, 16, 0)
    out += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
    # root symbol table entry: cache type 1 with B-tree + heap in scratch
    out += struct.pack("<QQII", 0, root_oh, 1, 0) + struct.pack("<QQ", btree, heap)
    assert len(out) == SB
    # root object header v1: one symbol table message
    out += struct.pack("<BBHII", 1, 0, 1, 1, 24) + b"\x00" * 4
    out += struct.pack("<HHB3x", 0x11, 16, 0) + struct.pack("<QQ", btree, heap)
    assert len(out) == heap
    # local heap
    out += b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap_names), UNDEF, heap_data)
    out += heap_names
    assert len(out) == btree
    # group B-tree (leaf, one child: the SNOD)
    node = bytearray(b"TREE" + bytes([0, 0]) + struct.pack("<H", 1) + struct.pack("<QQ", UNDEF, UNDEF))
    last_name = name_off[max(range(len(names)), key=lambda i: names[i])] if names else 0
    node += struct.pack("<Q", 0) + struct.pack("<Q", snod) + struct.pack("<Q", last_name)
    node += b"\x00" * (btree_full - len(node))
    out += node
    assert len(out) == snod
    sn = bytearray(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names)))
    order = sorted(range(len(names)), key=lambda i: names[i])       # symbol nodes are name-sorted
    for i in order:
        sn += struct.pack("<QQII", name_off[i], ds_hdr[i], 0, 0) + b"\x00" * 16
    sn += b"\x00" * (snod_size - len(sn))
    out += sn
    for a, h, da in zip(arrays, ds_hdr, data_addr):
        align8()
        while len(out) < h:
            out.append(0)
        out += _ds_header(a, da, so, sl)
    for a, da in zip(arrays, data_addr):
        while len(out) < da:
            out.append(0)
        out += a.tobytes()
    align8()
    with open(path, "wb") as fh:
        fh.write(bytes(out))


def _dt_message(a):
    if a.dtype.kind == "f":
        bits = 0x20 | (0x0F if a.dtype.itemsize == 8 else 0x00)   # LE, IEEE, mantissa norm implied
        body = bytes([0x11, 0x20, 0x3F if a.dtype.itemsize == 8 else 0x1F, 0]) + struct.pack("<I", a.dtype.itemsize)
        if a.dtype.itemsize == 8:
            body += struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        else:
            body += struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        del bits
    else:
        signed = a.dtype.kind == "i"
        body = bytes([0x10, 0x08 if signed else 0x00, 0, 0]) + struct.pack("<I", a.dtype.itemsize)
        body += struct.pack("<HH", 0, 8 * a.dtype.itemsize)
    return body


def _messages_for(a, data_addr, so, sl):
    rank = a.ndim
    ds = bytes([1, rank, 0, 0]) + b"\x00" * 4 + b"".join(struct.pack("<Q", s) for s in a.shape)
    dt = _dt_message(a)
    lay = bytes([3, 1]) + struct.pack("<QQ", data_addr, a.nbytes)
    fill = bytes([2, 2, 2, 0])                         # fill value message v2: never written, undefined
    return [(0x01, ds), (0x03, dt), (0x05, fill), (0x08, lay)]


def _pad8(b):
    return b + b"\x00" * ((8 - len(b) % 8) % 8)


def _ds_header_size(a, so, sl):
    msgs = _messages_for(a, 0, so, sl)
    return 16 + sum(8 + len(_pad8(b)) for _, b in msgs)


def _ds_header(a, data_addr, so, sl):
    msgs = _messages_for(a, data_addr, so, sl)
    body = b"".join(struct.pack("<HHB3x", t, len(_pad8(b)), 1 if t == 0x03 else 0) + _pad8(b) for t, b in msgs)
    return struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\x00" * 4 + body


__all__ = ["H5File", "write_h5", "H5Error"]
