"""Classic netCDF (CDF-1/2/5) files, the PnetCDF "64BIT_DATA" format of the reference.

Reference: the notebook writer ``to_nc`` (mnist_to_netcdf.ipynb cell 2 lines 83-104: dims
``Y=28, X=28, idx=N``; vars ``images(idx,Y,X)`` and ``labels(idx)`` NC_UBYTE) and the reader
``MNISTNetCDF`` (mnist_pnetcdf_cpu_mp.py:18-49) over pncpy/libpnetcdf/MPI-IO.  This module
has no MPI dependency: :class:`NcFile` parses the header once and reads hyperslabs with
``pread`` (native ``_io.NcFile``) — either one sample (the reference's per-sample independent
``get_var``) or a whole rank shard at once into pinned memory.  A pure-Python implementation
is kept for environments without the native library and as a cross-check in tests.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..ops.native import load_io

NC_TYPES = {1: "i1", 2: "S1", 3: ">i2", 4: ">i4", 5: ">f4", 6: ">f8", 7: "u1", 8: ">u2", 9: ">u4",
            10: ">i8", 11: ">u8"}
NC_SIZES = {1: 1, 2: 1, 3: 2, 4: 4, 5: 4, 6: 8, 7: 1, 8: 2, 9: 4, 10: 8, 11: 8}
NP_TO_NC = {("u", 1): 7, ("i", 1): 1, ("i", 2): 3, ("u", 2): 8, ("i", 4): 4, ("u", 4): 9, ("f", 4): 5,
            ("f", 8): 6, ("i", 8): 10, ("u", 8): 11}


class _PyNcFile:
    """Pure-Python CDF-1/2/5 header parser + reader (fallback / cross-check)."""

    def __init__(self, path: str):
        self.path = path
        with open(path, "rb") as f:
            head = f.read(1 << 20)
        if head[:3] != b"CDF" or head[3] not in (1, 2, 5):
            raise ValueError(f"{path}: not a classic netCDF file")
        self.version = head[3]
        p = 4
        v5 = self.version == 5

        def nonneg():
            nonlocal p
            if v5:
                (v,) = struct.unpack_from(">Q", head, p); p += 8
            else:
                (v,) = struct.unpack_from(">I", head, p); p += 4
            return v

        def u32():
            nonlocal p
            (v,) = struct.unpack_from(">I", head, p); p += 4
            return v

        def name():
            nonlocal p
            n = nonneg()
            s = head[p:p + n].decode()
            p += (n + 3) & ~3
            return s

        def atts():
            nonlocal p
            tag, n = u32(), nonneg()
            out = {}
            if tag == 0 and n == 0:
                return out
            for _ in range(n):
                k = name()
                t = u32()
                ne = nonneg()
                nb = ne * NC_SIZES[t]
                out[k] = np.frombuffer(head[p:p + nb], dtype=NC_TYPES[t]).copy()
                p += (nb + 3) & ~3
            return out

        self.numrecs = nonneg()
        tag, n = u32(), nonneg()
        self._dims: List[Tuple[str, int]] = []
        if not (tag == 0 and n == 0):
            for _ in range(n):
                self._dims.append((name(), nonneg()))
        self.gatts = atts()
        tag, n = u32(), nonneg()
        self._vars: Dict[str, dict] = {}
        for _ in range(0 if (tag == 0 and n == 0) else n):
            vn = name()
            nd = nonneg()
            dimids = [nonneg() for _ in range(nd)]
            va = atts()
            t = u32()
            vsize = nonneg()
            if self.version == 1:
                begin = u32()
            else:
                (begin,) = struct.unpack_from(">Q", head, p); p += 8
            self._vars[vn] = dict(type=t, vsize=vsize, begin=begin, dimids=dimids, atts=va,
                                  shape=[self._dims[i][1] for i in dimids],
                                  dims=[self._dims[i][0] for i in dimids])

    def dims(self):
        return list(self._dims)

    def variables(self):
        return list(self._vars)

    def shape(self, n):
        return list(self._vars[n]["shape"])

    def begin(self, n):
        return self._vars[n]["begin"]

    def var_info(self, n):
        v = self._vars[n]
        return {k: v[k] for k in ("type", "vsize", "begin", "shape", "dims")}

    def read_rows(self, n, start=0, count=-1, threads=1):
        v = self._vars[n]
        shp = v["shape"]
        rows = shp[0] - start if count < 0 else count
        rb = NC_SIZES[v["type"]] * int(np.prod(shp[1:], dtype=np.int64))
        with open(self.path, "rb") as f:
            f.seek(v["begin"] + start * rb)
            raw = f.read(rows * rb)
        a = np.frombuffer(raw, dtype=NC_TYPES[v["type"]]).reshape([rows] + shp[1:])
        return a.astype(a.dtype.newbyteorder("=")) if a.dtype.byteorder == ">" else a.copy()

    def read_row(self, n, index):
        return self.read_rows(n, index, 1)


def open_nc(path: str, native: bool = True):
    io = load_io() if native else None
    return io.NcFile(path) if io is not None else _PyNcFile(path)


def _py_write(path: str, dims: Sequence[Tuple[str, int]], variables, align: int = 512) -> None:
    h = bytearray(b"CDF\x05")
    h += struct.pack(">Q", 0)

    def put_name(s: str):
        b = s.encode()
        h.extend(struct.pack(">Q", len(b)) + b + b"\0" * ((4 - len(b) % 4) % 4))

    if dims:
        h += struct.pack(">IQ", 0x0A, len(dims))
        for n, ln in dims:
            put_name(n)
            h += struct.pack(">Q", ln)
    else:
        h += struct.pack(">IQ", 0, 0)
    h += struct.pack(">IQ", 0, 0)
    patches = []
    h += struct.pack(">IQ", 0x0B, len(variables)) if variables else struct.pack(">IQ", 0, 0)
    for vn, dimids, arr in variables:
        arr = np.ascontiguousarray(arr)
        t = NP_TO_NC[(arr.dtype.kind, arr.dtype.itemsize)]
        put_name(vn)
        h += struct.pack(">Q", len(dimids))
        for d in dimids:
            h += struct.pack(">Q", d)
        h += struct.pack(">IQ", 0, 0)
        h += struct.pack(">I", t)
        vsize = (arr.nbytes + 3) & ~3
        h += struct.pack(">Q", vsize)
        patches.append((len(h), vsize, arr))
        h += struct.pack(">Q", 0)
    off = (len(h) + align - 1) // align * align
    begins = []
    for pos, vsize, _ in patches:
        h[pos:pos + 8] = struct.pack(">Q", off)
        begins.append(off)
        off += (vsize + align - 1) // align * align
    with open(path, "wb") as f:
        f.write(h)
        for b, (_, vsize, arr) in zip(begins, patches):
            f.write(b"\0" * (b - f.tell()))
            be = arr.astype(arr.dtype.newbyteorder(">")) if arr.dtype.itemsize > 1 else arr
            f.write(be.tobytes())
            f.write(b"\0" * (vsize - arr.nbytes))


def write_cdf5(path: str, dims: Sequence[Tuple[str, int]], variables, align: int = 512, native: bool = True) -> None:
    """variables: [(name, [dimids], ndarray)] — non-record variables, no attributes."""
    io = load_io() if native else None
    if io is not None:
        io.cdf5_write(path, [(n, int(l)) for n, l in dims],
                      [(n, [int(d) for d in ids], np.ascontiguousarray(a)) for n, ids, a in variables], align)
    else:
        _py_write(path, dims, variables, align)


def write_mnist_nc(path: str, images: np.ndarray, labels: np.ndarray, native: bool = True) -> None:
    """The notebook's to_nc(): dims Y, X, idx; images(idx,Y,X), labels(idx), NC_UBYTE, CDF-5."""
    images = np.ascontiguousarray(images, dtype=np.uint8).reshape(-1, 28, 28)
    labels = np.ascontiguousarray(labels, dtype=np.uint8).reshape(-1)
    if os.path.exists(path):
        os.remove(path)
    write_cdf5(path, [("Y", 28), ("X", 28), ("idx", images.shape[0])],
               [("images", [2, 0, 1], images), ("labels", [2], labels)], native=native)


def read_mnist_nc(path: str, limit: Optional[int] = None, rank: int = 0, world: int = 1, native: bool = True):
    """Bulk read (images [n,28,28] uint8, labels [n] uint8).  With world>1 each rank reads only
    its contiguous shard (the per-rank hyperslab of the reference's independent I/O)."""
    f = open_nc(path, native)
    n = f.shape("images")[0]
    if limit is not None:
        n = min(n, int(limit))
    s = n * rank // world
    e = n * (rank + 1) // world
    return f.read_rows("images", s, e - s), f.read_rows("labels", s, e - s)
