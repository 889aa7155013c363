"""Several GPUs in one process: chunk i is decoded or encoded
on ``devices[i % len(devices)]``, one host thread and one ``zcg_ctx`` per
device, no collective (chunks are independent: each read_chunk builds a fresh
decoder, chunk.rs:282,297).  Wraps the ``zcg_multi_*`` entry points."""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

from . import _native
from .chunk import ZarrIOError, abi_array, check_array_type
from .metadata import ArrayMetadata


class MultiDeviceCodec:
    def __init__(self, devices: Sequence[int]):
        self.lib = _native.load_library()
        self.devices = list(devices)
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        self.handle = self.lib.zcg_multi_create(ctypes.addressof(arr), len(self.devices))
        if not self.handle:
            raise _native.NativeUnavailable(f"zcg_multi_create({self.devices}) failed")

    def close(self):
        if self.handle:
            self.lib.zcg_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, r, what):
        if r != _native.OK:
            msg = (self.lib.zcg_multi_last_error(self.handle) or b"").decode()
            raise ZarrIOError(_native.STATUS_NAMES.get(r, str(r)), f"{what}: {msg}")

    def read_chunks_host(self, meta: ArrayMetadata, buffers: Sequence[bytes], t):
        """n read_chunk calls over host buffers -> (status, element arrays)."""
        check_array_type(t, meta)
        n = len(buffers)
        N = meta.get_chunk_num_elements()
        outs = [np.zeros(N, np.dtype(t).newbyteorder("=")) for _ in range(n)]
        keep = [ctypes.create_string_buffer(bytes(b), max(len(b), 1)) for b in buffers]
        srcs = (ctypes.c_void_p * max(n, 1))(*[ctypes.addressof(k) for k in keep])
        lens = (ctypes.c_uint64 * max(n, 1))(*[len(b) for b in buffers])
        dsts = (ctypes.c_void_p * max(n, 1))(*[o.ctypes.data for o in outs])
        st = np.zeros(max(n, 1), np.int32)
        arr = abi_array(meta)
        self._check(self.lib.zcg_multi_read_chunks_host(self.handle, ctypes.byref(arr), n, ctypes.addressof(srcs),
                                                        ctypes.addressof(lens), ctypes.addressof(dsts),
                                                        st.ctypes.data), "multi_read_chunks_host")
        return st[:n], outs

    def store_read(self, meta: ArrayMetadata, paths: Sequence[str], t, io_threads: int = 16):
        check_array_type(t, meta)
        n = len(paths)
        N = meta.get_chunk_num_elements()
        buf = np.empty(max(n * N, 1), np.dtype(t).newbyteorder("="))
        outs = [buf[i * N:(i + 1) * N] for i in range(n)]
        enc = [os.fsencode(p) for p in paths]
        cp = (ctypes.c_char_p * max(n, 1))(*enc)
        dsts = (ctypes.c_void_p * max(n, 1))(*[o.ctypes.data for o in outs])
        st = np.zeros(max(n, 1), np.int32)
        arr = abi_array(meta)
        self._check(self.lib.zcg_multi_store_read_chunks(self.handle, ctypes.byref(arr), n, ctypes.addressof(cp),
                                                         ctypes.addressof(dsts), st.ctypes.data, io_threads),
                    "multi_store_read_chunks")
        return outs, st[:n]

    def store_write(self, meta: ArrayMetadata, paths: Sequence[str], datas, io_threads: int = 16):
        n = len(paths)
        N = meta.get_chunk_num_elements()
        datas = [np.ascontiguousarray(d) for d in datas]
        for d in datas:
            check_array_type(d.dtype, meta)
            if d.size != N:
                raise ZarrIOError("InvalidData", "Wrong number of elements")
        if meta.effective_type().kind == "bool":
            datas = [d.astype(np.uint8) for d in datas]
        enc = [os.fsencode(p) for p in paths]
        cp = (ctypes.c_char_p * max(n, 1))(*enc)
        ep = (ctypes.c_void_p * max(n, 1))(*[d.ctypes.data for d in datas])
        st = np.zeros(max(n, 1), np.int32)
        arr = abi_array(meta)
        self._check(self.lib.zcg_multi_store_write_chunks(self.handle, ctypes.byref(arr), n, ctypes.addressof(cp),
                                                          ctypes.addressof(ep), st.ctypes.data, io_threads),
                    "multi_store_write_chunks")
        return st[:n]
