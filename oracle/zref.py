"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of ``oracle/libzref.so`` (built from ``oracle/zref.c`` by
``oracle/Makefile``).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product
path (``zarr_amd``) never does.  See ``zref.c`` for what is restated and
which reference file:line each function follows.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import List, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libzref.so")
_lib = None

OK, EOF, INVALID_DATA, INVALID_INPUT, UNSUPPORTED, TOO_SMALL = 0, 1, 2, 3, 4, 5
RAW, BZIP2, GZIP, LZ4, XZ = 0, 1, 2, 3, 4


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        u8p = ctypes.c_void_p
        L.zref_decode.argtypes = [ctypes.c_int] * 4 + [ctypes.c_uint32, u8p, ctypes.c_uint64, u8p,
                                                       ctypes.c_uint64]
        L.zref_decode.restype = ctypes.c_int
        L.zref_encode.argtypes = [ctypes.c_int] * 5 + [u8p, ctypes.c_uint64, ctypes.c_uint64, u8p,
                                                       ctypes.c_uint64,
                                                       ctypes.POINTER(ctypes.c_uint64)]
        L.zref_encode.restype = ctypes.c_int
        L.zref_decode_batch.argtypes = [ctypes.c_int] * 4 + [
            ctypes.c_uint32, u8p, u8p, u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_int]
        L.zref_decode_batch.restype = ctypes.c_int
        L.zref_encode_batch.argtypes = [ctypes.c_int] * 5 + [
            u8p, ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, ctypes.c_uint32, u8p, ctypes.c_int]
        L.zref_encode_batch.restype = ctypes.c_int
        L.zref_lz4_frame_custom.argtypes = [ctypes.c_int] * 6 + [
            ctypes.c_uint64, u8p, ctypes.c_uint64, u8p, ctypes.c_uint64,
            ctypes.POINTER(ctypes.c_uint64)]
        L.zref_lz4_frame_custom.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(b) -> int:
    if isinstance(b, np.ndarray):
        return b.ctypes.data
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value


def decode(codec: int, src: bytes, dlen: int, elem_size: int = 1, big_endian: bool = False,
           is_bool: bool = False, flags: int = 0) -> Tuple[int, bytes]:
    """DefaultChunkReader::read_chunk (chunk.rs:270-286) -> (status, N bytes)."""
    out = np.zeros(max(dlen, 1), np.uint8)
    s = np.frombuffer(src, np.uint8) if len(src) else np.zeros(1, np.uint8)
    st = lib().zref_decode(codec, elem_size, int(big_endian), int(is_bool), flags, s.ctypes.data,
                           len(src), out.ctypes.data, dlen)
    return st, out[:dlen].tobytes()


def encode(codec: int, param: int, elems: np.ndarray, chunk_num_elements: int = None,
           elem_size: int = None, big_endian: bool = False, is_bool: bool = False,
           cap: int = None) -> Tuple[int, bytes]:
    """DefaultChunkWriter::write_chunk (chunk.rs:306-323) -> (status, stream)."""
    elems = np.ascontiguousarray(elems)
    es = elem_size or elems.dtype.itemsize
    n = elems.size
    cnum = n if chunk_num_elements is None else chunk_num_elements
    nb = n * es
    cap = cap if cap is not None else nb + nb // 8 + 65536
    out = np.zeros(cap, np.uint8)
    ol = ctypes.c_uint64(0)
    src = elems.view(np.uint8) if nb else np.zeros(1, np.uint8)
    st = lib().zref_encode(codec, param, es, int(big_endian), int(is_bool), src.ctypes.data, n,
                           cnum, out.ctypes.data, cap, ctypes.byref(ol))
    return st, out[: ol.value].tobytes()


def decode_batch(codec: int, srcs: Sequence[np.ndarray], dlen: int, elem_size=1, big_endian=False,
                 is_bool=False, threads=1, flags=0, dsts: List[np.ndarray] = None):
    """One chunk per task on a pthread pool (cpu_baseline)."""
    n = len(srcs)
    if dsts is None:
        dsts = [np.empty(dlen, np.uint8) for _ in range(n)]
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in srcs])
    sl = (ctypes.c_uint64 * n)(*[s.size for s in srcs])
    dp = (ctypes.c_void_p * n)(*[d.ctypes.data for d in dsts])
    st = np.zeros(n, np.int32)
    lib().zref_decode_batch(codec, elem_size, int(big_endian), int(is_bool), flags,
                            ctypes.addressof(sp), ctypes.addressof(sl), ctypes.addressof(dp), dlen,
                            n, st.ctypes.data, threads)
    return st, dsts


def encode_batch(codec: int, param: int, srcs: Sequence[np.ndarray], elem_size=1,
                 big_endian=False, is_bool=False, threads=1, cap=None):
    n = len(srcs)
    n_el = srcs[0].size
    nb = n_el * elem_size
    cap = cap or nb + nb // 8 + 65536
    outs = [np.empty(cap, np.uint8) for _ in range(n)]
    sp = (ctypes.c_void_p * n)(*[s.ctypes.data for s in srcs])
    op = (ctypes.c_void_p * n)(*[o.ctypes.data for o in outs])
    ol = np.zeros(n, np.uint64)
    st = np.zeros(n, np.int32)
    lib().zref_encode_batch(codec, param, elem_size, int(big_endian), int(is_bool),
                            ctypes.addressof(sp), n_el, ctypes.addressof(op), cap,
                            ol.ctypes.data, n, st.ctypes.data, threads)
    return st, [o[: int(k)] for o, k in zip(outs, ol)]


def lz4_frame_custom(data: bytes, block_size_id=4, linked=False, content_checksum=True,
                     block_checksum=False, content_size=False, auto_flush=False,
                     feed=0) -> bytes:
    """LZ4F frames with non-reference preferences (fixture generation)."""
    src = np.frombuffer(data, np.uint8) if data else np.zeros(1, np.uint8)
    cap = len(data) + len(data) // 4 + 65536
    out = np.zeros(cap, np.uint8)
    ol = ctypes.c_uint64(0)
    st = lib().zref_lz4_frame_custom(block_size_id, int(linked), int(content_checksum),
                                     int(block_checksum), int(content_size), int(auto_flush), feed,
                                     src.ctypes.data, len(data), out.ctypes.data, cap,
                                     ctypes.byref(ol))
    assert st == OK, st
    return out[: ol.value].tobytes()
