"""Minimal reader for MATLAB v7.3 MAT-files (HDF5) -- enough for the
reference's datasets that scipy.io cannot read (datasets_paper/Misc/
CollegeMsg.mat, Drugs.mat, as_735.mat).  h5py is not
available in this image, so this parses the HDF5 structures MATLAB writes
directly:

  * superblock version 0 (with the 512-byte MAT user block), 8-byte offsets
  * version-1 object headers (+ continuation blocks)
  * groups as symbol tables (v1 B-tree "TREE" -> "SNOD" nodes + local "HEAP")
  * datasets: dataspace, datatype (fixed-point / IEEE float / string /
    reference), layout (compact, contiguous, chunked via a v1 B-tree),
    filter pipeline (deflate, shuffle)
  * attributes (MATLAB_class, MATLAB_sparse, ...)

``loadmat(path)`` returns a dict of top-level variables; MATLAB structs
become dicts, sparse matrices scipy CSC matrices, numeric arrays numpy
arrays (MATLAB's column-major dims restored), char arrays str.  Nothing is
executed from the file; unsupported features raise ``NotImplementedError``.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

_SIG = b"\x89HDF\r\n\x1a\n"


class _File:
    def __init__(self, path):
        with open(path, "rb") as f:
            self.b = f.read()
        self.base = None
        for off in (0, 512, 1024, 2048, 4096):
            if self.b[off:off + 8] == _SIG:
                self.base = off
                break
        if self.base is None:
            raise ValueError(f"{path}: not an HDF5 file")
        sb = self.base
        ver = self.b[sb + 8]
        if ver not in (0, 1):
            raise NotImplementedError(f"HDF5 superblock version {ver}")
        self.so, self.sl = self.b[sb + 13], self.b[sb + 14]
        if (self.so, self.sl) != (8, 8):
            raise NotImplementedError("HDF5 offsets/lengths other than 8 bytes")
        p = sb + 24 + (4 if ver == 1 else 0)
        base_addr = self.u64(p)
        self.addr0 = base_addr  # addresses are relative to the base address
        root_entry = p + 32
        self.root = self.u64(root_entry + 8)

    # raw readers -----------------------------------------------------------
    def u8(self, p):
        return self.b[p]

    def u16(self, p):
        return struct.unpack_from("<H", self.b, p)[0]

    def u32(self, p):
        return struct.unpack_from("<I", self.b, p)[0]

    def u64(self, p):
        return struct.unpack_from("<Q", self.b, p)[0]

    def at(self, addr):
        return self.addr0 + addr

    # object headers -----------------------------------------------------------
    def messages(self, addr):
        """(type, data bytes) of every message of the v1 object header at addr."""
        p = self.at(addr)
        if self.b[p] != 1:
            raise NotImplementedError(f"object header version {self.b[p]}")
        nmsg = self.u16(p + 2)
        hsize = self.u32(p + 8)
        blocks = [(p + 16, hsize)]
        out = []
        while blocks and len(out) < nmsg:
            q, size = blocks.pop(0)
            end = q + size
            while q + 8 <= end and len(out) < nmsg:
                mtype, msize = self.u16(q), self.u16(q + 2)
                data = self.b[q + 8:q + 8 + msize]
                out.append((mtype, data))
                if mtype == 0x0010:  # continuation
                    caddr, clen = struct.unpack_from("<QQ", data, 0)
                    blocks.append((self.at(caddr), clen))
                q += 8 + msize
        return out

    def global_object(self, coll, idx):
        """Object idx of the global heap collection at coll (vlen data)."""
        p = self.at(coll)
        if self.b[p:p + 4] != b"GCOL":
            raise ValueError("bad global heap collection")
        end = p + self.u64(p + 8)
        q = p + 16
        while q + 16 <= end:
            oid, size = self.u16(q), self.u64(q + 8)
            if oid == 0:
                break
            if oid == idx:
                return self.b[q + 16:q + 16 + size]
            q += 16 + (size + 7) // 8 * 8
        raise ValueError(f"global heap object {idx} not found")

    # groups ----------------------------------------------------------------
    def heap_name(self, heap_addr, off):
        p = self.at(heap_addr)
        if self.b[p:p + 4] != b"HEAP":
            raise ValueError("bad local heap")
        data = self.at(self.u64(p + 24))
        q = data + off
        e = self.b.index(b"\0", q)
        return self.b[q:e].decode("latin-1")

    def group_links(self, btree_addr, heap_addr):
        """name -> object header address of a symbol-table group."""
        out = {}

        def walk(addr):
            p = self.at(addr)
            sig = self.b[p:p + 4]
            if sig == b"TREE":
                level = self.b[p + 5]
                used = self.u16(p + 6)
                q = p + 24 + 8  # skip key 0
                for _ in range(used):
                    child = self.u64(q)
                    walk(child)
                    q += 16
                return
            if sig == b"SNOD":
                nsym = self.u16(p + 6)
                q = p + 8
                for _ in range(nsym):
                    name_off, obj = struct.unpack_from("<QQ", self.b, q)
                    out[self.heap_name(heap_addr, name_off)] = obj
                    q += 40
                return
            raise ValueError(f"unexpected node {sig!r}")

        walk(btree_addr)
        return out


# message decoders --------------------------------------------------------------
def _dataspace(d):
    ver = d[0]
    rank = d[1]
    if ver == 1:
        dims = struct.unpack_from("<" + "Q" * rank, d, 8)
    elif ver == 2:
        dims = struct.unpack_from("<" + "Q" * rank, d, 4)
    else:
        raise NotImplementedError(f"dataspace version {ver}")
    return tuple(dims)


def _datatype(d):
    cls = d[0] & 0x0F
    bits = d[1] | (d[2] << 8) | (d[3] << 16)
    size = struct.unpack_from("<I", d, 4)[0]
    if cls == 0:  # fixed point
        signed = bool(bits & 0x08)
        big = bool(bits & 0x01)
        return np.dtype(("<" if not big else ">") + ("i" if signed else "u") + str(size)), "int"
    if cls == 1:  # floating point
        big = bool(bits & 0x01)
        return np.dtype(("<" if not big else ">") + "f" + str(size)), "float"
    if cls == 3:
        return np.dtype("S" + str(size)), "string"
    if cls == 7:
        return np.dtype("<u8"), "reference"
    if cls == 9:  # variable length: (u32 length, u64 collection, u32 index)
        return np.dtype([("len", "<u4"), ("addr", "<u8"), ("idx", "<u4")]), "vlen"
    raise NotImplementedError(f"HDF5 datatype class {cls}")


def _layout(d):
    ver = d[0]
    if ver == 3:
        cls = d[1]
        if cls == 0:
            n = struct.unpack_from("<H", d, 2)[0]
            return ("compact", d[4:4 + n])
        if cls == 1:
            addr, size = struct.unpack_from("<QQ", d, 2)
            return ("contiguous", addr, size)
        if cls == 2:
            rank = d[2]
            addr = struct.unpack_from("<Q", d, 3)[0]
            dims = struct.unpack_from("<" + "I" * rank, d, 11)
            return ("chunked", addr, dims)
    if ver in (1, 2):
        rank, cls = d[1], d[2]
        p = 8
        if cls == 0:
            dims = struct.unpack_from("<" + "I" * rank, d, p)
            p += 4 * rank
            n = struct.unpack_from("<I", d, p)[0]
            return ("compact", d[p + 4:p + 4 + n])
        addr = struct.unpack_from("<Q", d, p)[0]
        p += 8
        dims = struct.unpack_from("<" + "I" * rank, d, p)
        if cls == 1:
            return ("contiguous", addr, None)
        return ("chunked", addr, dims)
    raise NotImplementedError(f"layout version {ver}")


def _filters(d):
    ver, nf = d[0], d[1]
    p = 8 if ver == 1 else 2
    out = []
    for _ in range(nf):
        fid = struct.unpack_from("<H", d, p)[0]
        if ver == 1 or fid >= 256:
            nlen = struct.unpack_from("<H", d, p + 2)[0]
            ncd = struct.unpack_from("<H", d, p + 6)[0]
            p += 8
            if ver == 1:
                p += (nlen + 7) // 8 * 8
            else:
                p += nlen
        else:
            ncd = struct.unpack_from("<H", d, p + 4)[0]
            p += 6
        cd = struct.unpack_from("<" + "I" * ncd, d, p) if ncd else ()
        p += 4 * ncd
        if ver == 1 and ncd % 2:
            p += 4
        out.append((fid, cd))
    return out


def _attribute(f, d):
    ver = d[0]
    if ver != 1:
        raise NotImplementedError(f"attribute message version {ver}")
    nlen, tlen, slen = struct.unpack_from("<HHH", d, 2)
    p = 8
    name = d[p:p + nlen].split(b"\0")[0].decode("latin-1")
    p += (nlen + 7) // 8 * 8
    dt, kind = _datatype(d[p:p + tlen])
    p += (tlen + 7) // 8 * 8
    dims = _dataspace(d[p:p + slen]) if slen else ()
    p += (slen + 7) // 8 * 8
    count = int(np.prod(dims)) if dims else 1
    raw = d[p:p + count * dt.itemsize]
    val = np.frombuffer(raw, dtype=dt, count=count)
    if kind == "string":
        return name, b"".join(val.tolist()).split(b"\0")[0].decode("latin-1")
    if kind == "vlen":  # MATLAB_fields: one char sequence per struct field
        return name, [f.global_object(int(v["addr"]), int(v["idx"])).decode("latin-1")
                      for v in val]
    return name, (val[0] if count == 1 else val.copy())


class _Node:
    def __init__(self, f, addr):
        self.f, self.addr = f, addr
        self.attrs = {}
        self.links = None
        self.space = self.dtype = self.kind = self.layout = None
        self.filters = []
        for mtype, d in f.messages(addr):
            if mtype == 0x0001:
                self.space = _dataspace(d)
            elif mtype == 0x0003:
                self.dtype, self.kind = _datatype(d)
            elif mtype == 0x0008:
                self.layout = _layout(d)
            elif mtype == 0x000B:
                self.filters = _filters(d)
            elif mtype == 0x000C:
                k, v = _attribute(f, d)
                self.attrs[k] = v
            elif mtype == 0x0011:
                bt, heap = struct.unpack_from("<QQ", d, 0)
                self.links = f.group_links(bt, heap)

    @property
    def is_group(self):
        return self.links is not None

    def read(self):
        f = self.f
        dims = self.space or ()
        count = int(np.prod(dims)) if dims else 0
        dt = self.dtype
        lay = self.layout
        if lay is None or count == 0:
            return np.zeros(dims, dtype=dt)
        if lay[0] == "compact":
            raw = lay[1]
        elif lay[0] == "contiguous":
            if lay[1] == 0xFFFFFFFFFFFFFFFF:
                return np.zeros(dims, dtype=dt)
            raw = f.b[f.at(lay[1]):f.at(lay[1]) + count * dt.itemsize]
        else:
            raw = self._read_chunked(count)
        arr = np.frombuffer(raw, dtype=dt, count=count).reshape(dims)
        return arr

    def _read_chunked(self, count):
        f = self.f
        _, bt, cdims = self.layout
        rank = len(cdims) - 1
        shape = self.space
        itemsize = self.dtype.itemsize
        out = np.zeros(int(np.prod(shape)) * itemsize, dtype=np.uint8).reshape(tuple(shape) + (itemsize,))
        chunk = tuple(cdims[:rank])

        def walk(addr):
            p = f.at(addr)
            if f.b[p:p + 4] != b"TREE" or f.b[p + 4] != 1:
                raise ValueError("bad chunk B-tree")
            level = f.b[p + 5]
            used = f.u16(p + 6)
            q = p + 24
            keysz = 8 + 8 * (rank + 1)
            for _ in range(used):
                csize, mask = struct.unpack_from("<II", f.b, q)
                offs = struct.unpack_from("<" + "Q" * rank, f.b, q + 8)
                child = f.u64(q + keysz)
                if level > 0:
                    walk(child)
                else:
                    data = f.b[f.at(child):f.at(child) + csize]
                    for i, (fid, cd) in enumerate(reversed(self.filters)):
                        if mask & (1 << (len(self.filters) - 1 - i)):
                            continue
                        if fid == 1:
                            data = zlib.decompress(data)
                        elif fid == 2:  # shuffle
                            a = np.frombuffer(data, dtype=np.uint8)
                            data = a.reshape(itemsize, -1).T.tobytes()
                        else:
                            raise NotImplementedError(f"HDF5 filter {fid}")
                    blk = np.frombuffer(data, dtype=np.uint8).reshape(chunk + (itemsize,))
                    sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, chunk, shape))
                    sub = tuple(slice(0, s.stop - s.start) for s in sl)
                    out[sl] = blk[sub]
                q += keysz + 8

        walk(bt)
        return out.tobytes()


def _matlab(f, node, refs):
    """MATLAB value of a node (MATLAB_class attribute conventions)."""
    cls = node.attrs.get("MATLAB_class")
    if node.is_group:
        if "MATLAB_sparse" in node.attrs:
            import scipy.sparse as sp
            m = int(node.attrs["MATLAB_sparse"])
            ch = {k: _Node(f, a) for k, a in node.links.items()}
            jc = ch["jc"].read().astype(np.int64).ravel()
            n = len(jc) - 1
            ir = ch["ir"].read().astype(np.int64).ravel() if "ir" in ch else np.zeros(0, np.int64)
            if "data" in ch:
                data = ch["data"].read().ravel()
                if cls == "logical":
                    data = data.astype(bool)
                data = data.astype(np.float64) if data.dtype != bool else data
            else:
                data = np.ones(len(ir))
            return sp.csc_matrix((data, ir, jc), shape=(m, n))
        return {k: _matlab(f, _Node(f, a), refs) for k, a in node.links.items() if not k.startswith("#")}
    arr = node.read()
    if node.attrs.get("MATLAB_empty"):
        return np.zeros((0, 0))
    if cls == "char":
        return "".join(chr(c) for c in arr.T.ravel())
    if cls == "cell" and node.kind == "reference":
        return [_matlab(f, _Node(f, int(r)), refs) for r in arr.T.ravel()]
    if arr.ndim >= 2:
        arr = arr.T  # HDF5 stores MATLAB's column-major arrays transposed
    return arr


def loadmat(path, variables=None):
    """Top-level variables of a MATLAB v7.3 MAT-file as Python objects."""
    f = _File(path)
    root = _Node(f, f.root)
    out = {}
    for k, a in root.links.items():
        if k.startswith("#") or (variables and k not in variables):
            continue
        out[k] = _matlab(f, _Node(f, a), None)
    return out


def load_sparse(path, field_path=("Problem", "A")):
    """The sparse matrix at the given struct path (default Problem.A, the
    layout of the reference's datasets_paper files)."""
    v = loadmat(path, variables=[field_path[0]])[field_path[0]]
    for k in field_path[1:]:
        v = v[k]
    return v
