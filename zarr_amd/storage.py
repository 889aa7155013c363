"""Minimal FilesystemHierarchy — the caller of the chunk path on both ends
of the north_star e2e path (files -> decode -> files).

Mirrors only what the chunk path needs from ``src/storage.rs`` and
``src/store/filesystem.rs``: the entry point ``zarr.json`` (lib.rs:165-182),
array metadata keys ``/meta/root/<path>.array.json`` (lib.rs:194-201),
chunk keys ``/data/root/<path>/c<i>/<j>/…`` (``get_chunk_key``,
storage.rs:109-127), ``read_chunk`` with a missing chunk -> ``None``
(storage.rs:206-235), ``read_chunk_into`` (237-267), ``write_chunk``
(456-470) and ``delete_chunk``.  Chunk files go through the native store
path (zcg_store.cpp): shared flock on read, exclusive flock + truncate on
write (filesystem.rs:201-210,260-280), read into pinned staging on a host
thread pool and pipelined with the GPU.  Groups/attributes/listing are out
of scope.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _native
from .chunk import DefaultChunk, SliceDataChunk, ZarrIOError, abi_array, check_array_type
from .metadata import ArrayMetadata

ENTRY_POINT_KEY = "zarr.json"
DATA_ROOT_PATH = "/data/root"
META_ROOT_PATH = "/meta/root"
ZARR_FORMAT = "https://purl.org/zarr/spec/protocol/core/3.0"


def canonicalize_path(path: str) -> str:
    """lib.rs:187-189."""
    return path.strip("/")


def get_chunk_key(base_path: str, array_meta: ArrayMetadata, grid_position: Sequence[int]) -> str:
    """storage.rs:109-127."""
    canon = canonicalize_path(base_path)
    key = f"{DATA_ROOT_PATH}/c" if not canon else f"{DATA_ROOT_PATH}/{canon}/c"
    return key + array_meta.separator.join(str(int(c)) for c in grid_position)


class FilesystemHierarchy:
    def __init__(self, base_path: str, entry: dict):
        self.base_path = os.path.abspath(base_path)
        self.entry = entry

    @staticmethod
    def open(base_path: str) -> "FilesystemHierarchy":
        with open(os.path.join(base_path, ENTRY_POINT_KEY)) as f:
            entry = json.load(f)
        if not str(entry.get("zarr_format", "")).endswith("/3.0"):
            raise ZarrIOError("Other", "TODO: Incompatible version")
        return FilesystemHierarchy(base_path, entry)

    @staticmethod
    def open_or_create(base_path: str) -> "FilesystemHierarchy":
        p = os.path.join(base_path, ENTRY_POINT_KEY)
        if os.path.exists(p):
            return FilesystemHierarchy.open(base_path)
        os.makedirs(base_path, exist_ok=True)
        entry = {"zarr_format": ZARR_FORMAT, "metadata_encoding": ZARR_FORMAT,
                 "metadata_key_suffix": ".json", "extensions": []}
        with open(p, "w") as f:
            json.dump(entry, f)
        return FilesystemHierarchy(base_path, entry)

    # ---- keys -----------------------------------------------------------------
    def _path(self, key: str) -> str:
        """FilesystemHierarchy::get_path (filesystem.rs:151-190) through the
        C ABI (zcg_store_path): the key relative to the root, refused with
        NotFound when its net nesting is negative.  Like the reference this
        checks only the NET nesting, so '../x' and 'a/../../b' resolve outside
        the root (a reference flaw kept for parity)."""
        st, p = _native.store_path(self.base_path, key)
        if st == _native.NOT_FOUND:
            raise ZarrIOError("NotFound", "Path name is outside this Zarr filesystem")
        if st != _native.OK:
            raise ZarrIOError(_native.STATUS_NAMES.get(st, "Other"), f"zcg_store_path: status {st}")
        return p

    def array_metadata_key(self, path_name: str) -> str:
        suffix = self.entry.get("metadata_key_suffix", ".json").lstrip(".")
        return f"{META_ROOT_PATH}/{canonicalize_path(path_name)}.array.{suffix}"

    # ---- arrays -----------------------------------------------------------------
    def create_array(self, path_name: str, array_meta: ArrayMetadata) -> None:
        p = self._path(self.array_metadata_key(path_name))
        if os.path.exists(p):
            raise ZarrIOError("AlreadyExists", "array already exists")
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(array_meta.to_json())

    def get_array_metadata(self, path_name: str) -> ArrayMetadata:
        p = self._path(self.array_metadata_key(path_name))
        if not os.path.isfile(p):
            raise ZarrIOError("NotFound", path_name)
        with open(p) as f:
            return ArrayMetadata.from_json(f.read())

    def chunk_path(self, path_name: str, array_meta: ArrayMetadata, grid_position) -> str:
        return self._path(get_chunk_key(path_name, array_meta, grid_position))

    # ---- chunks (the path) ---------------------------------------------------------
    def read_chunk(self, path_name: str, array_meta: ArrayMetadata, grid_position, t,
                   device: int = 0) -> Optional[SliceDataChunk]:
        """storage.rs:206-235: get() under a shared flock; None if absent."""
        return self.read_chunks(path_name, array_meta, [grid_position], t, device=device, io_threads=1)[0]

    def read_chunk_into(self, path_name: str, array_meta: ArrayMetadata, grid_position,
                        chunk: SliceDataChunk, t, device: int = 0) -> Optional[bool]:
        """storage.rs:237-267: None if absent, else the chunk reinitialised
        (ReinitDataChunk::reinitialize, chunk.rs:91-94) with the decoded data."""
        got = self.read_chunk(path_name, array_meta, grid_position, t, device=device)
        if got is None:
            return None
        chunk.grid_position = list(grid_position)
        new = got.get_data()
        old = chunk.data
        if isinstance(old, np.ndarray) and old.shape == new.shape and old.dtype == new.dtype \
                and old.flags.writeable:
            np.copyto(old, new)  # the caller's buffer is filled in place (read_chunk_into)
        else:
            chunk.data = new
        return True

    def read_chunks(self, path_name: str, array_meta: ArrayMetadata, grid_positions, t,
                    device: int = 0, io_threads: int = 16) -> List[Optional[SliceDataChunk]]:
        """Batched read_chunk through the native store path
        (zcg_store_read_chunks): files read under a shared flock into pinned
        staging by `io_threads` host threads, pipelined with H2D, the batch
        decode and D2H on two streams.  A missing chunk is None."""
        for g in grid_positions:
            assert array_meta.in_bounds(g)  # storage.rs:217 (a panic there)
        paths = [self.chunk_path(path_name, array_meta, g) for g in grid_positions]
        arrs, status = store_read(array_meta, paths, t, device=device, io_threads=io_threads)
        out: List[Optional[SliceDataChunk]] = []
        for g, a, st in zip(grid_positions, arrs, status):
            if st == _native.ABSENT:
                out.append(None)
                continue
            if st != _native.OK:
                raise ZarrIOError(_native.STATUS_NAMES.get(int(st), str(st)), f"chunk {list(g)}")
            out.append(SliceDataChunk(list(g), a))
        return out

    def write_chunks(self, path_name: str, array_meta: ArrayMetadata, chunks: Sequence[SliceDataChunk],
                     device: int = 0, io_threads: int = 16) -> None:
        """Batched write_chunk (zcg_store_write_chunks): GPU encode, then each
        file written under an exclusive flock, truncated after locking
        (filesystem.rs:260-280)."""
        paths = [self.chunk_path(path_name, array_meta, c.get_grid_position()) for c in chunks]
        status = store_write(array_meta, paths, [c.get_data() for c in chunks], device=device,
                             io_threads=io_threads)
        for c, st in zip(chunks, status):
            if st != _native.OK:
                raise ZarrIOError(_native.STATUS_NAMES.get(int(st), str(st)), f"chunk {c.get_grid_position()}")

    def write_chunk(self, path_name: str, array_meta: ArrayMetadata, chunk: SliceDataChunk,
                    device: int = 0) -> None:
        """storage.rs:456-470 + DefaultChunk::write_chunk (chunk.rs:306-323),
        stored by set() under an exclusive flock (filesystem.rs:260-280)."""
        data = np.asarray(chunk.get_data())
        check_array_type(data.dtype, array_meta)
        if data.size != array_meta.get_chunk_num_elements():  # chunk.rs:309-318
            raise ZarrIOError("InvalidData",
                              f"Can not write chunk with too few elements. Expected "
                              f"{array_meta.get_chunk_num_elements()} given {data.size}")
        self.write_chunks(path_name, array_meta, [chunk], device=device, io_threads=1)

    def delete_chunk(self, path_name: str, array_meta: ArrayMetadata, grid_position) -> bool:
        p = self.chunk_path(path_name, array_meta, grid_position)
        if os.path.isfile(p):
            os.remove(p)
        return True

    def exists_chunk(self, path_name: str, array_meta: ArrayMetadata, grid_position) -> bool:
        return os.path.isfile(self.chunk_path(path_name, array_meta, grid_position))


def _cstrs(paths):
    enc = [os.fsencode(p) for p in paths]
    arr = (ctypes.c_char_p * max(len(enc), 1))(*enc)
    return arr, enc


# batches at least this large land in page-locked host memory, which the
# store fills by direct D2H copies (no staging copy, no first-touch faults)
PINNED_MIN_BYTES = 64 << 20


def _host_buffer(nbytes: int, pinned: bool) -> np.ndarray:
    if pinned:
        try:
            import torch
            return torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True).numpy()
        except Exception:
            pass
    return np.empty(max(nbytes, 1), np.uint8)


def store_read(array_meta: ArrayMetadata, paths: Sequence[str], t, device: int = 0, io_threads: int = 16,
               pinned=None):
    """zcg_store_read_chunks: (list of element arrays, status array).  The
    arrays are views of one host allocation, page-locked for large batches."""
    check_array_type(t, array_meta)
    ctx = _native.context(device)
    n = len(paths)
    dt = np.dtype(t).newbyteorder("=")
    N = array_meta.get_chunk_num_elements()
    nbytes = n * N * dt.itemsize
    if pinned is None:
        pinned = nbytes >= PINNED_MIN_BYTES
    buf = _host_buffer(nbytes, pinned)[:max(nbytes, dt.itemsize)].view(dt)
    arrs = [buf[i * N:(i + 1) * N] for i in range(n)]
    dp = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    cp, keep = _cstrs(paths)
    st = np.zeros(max(n, 1), np.int32)
    arr = abi_array(array_meta)
    r = ctx.lib.zcg_store_read_chunks(ctx.handle, ctypes.byref(arr), n, ctypes.addressof(cp),
                                      ctypes.addressof(dp), st.ctypes.data, io_threads)
    if r != _native.OK:
        raise ZarrIOError(_native.STATUS_NAMES.get(r, str(r)), f"store_read_chunks: {ctx.last_error()}")
    return arrs, st[:n]


def store_write(array_meta: ArrayMetadata, paths: Sequence[str], datas, device: int = 0, io_threads: int = 16):
    """zcg_store_write_chunks: status array.  Each element array must hold
    exactly get_chunk_num_elements() elements (chunk.rs:309-318)."""
    ctx = _native.context(device)
    n = len(paths)
    N = array_meta.get_chunk_num_elements()
    t = array_meta.effective_type()
    datas = [np.ascontiguousarray(d) for d in datas]
    for d in datas:
        check_array_type(d.dtype, array_meta)
        if d.size != N:
            raise ZarrIOError("InvalidData", "Wrong number of elements")
    if t.kind == "bool":
        datas = [d.astype(np.uint8) for d in datas]
    ep = (ctypes.c_void_p * max(n, 1))(*[d.ctypes.data for d in datas])
    cp, keep = _cstrs(paths)
    st = np.zeros(max(n, 1), np.int32)
    arr = abi_array(array_meta)
    r = ctx.lib.zcg_store_write_chunks(ctx.handle, ctypes.byref(arr), n, ctypes.addressof(cp),
                                       ctypes.addressof(ep), st.ctypes.data, io_threads)
    if r != _native.OK:
        raise ZarrIOError(_native.STATUS_NAMES.get(r, str(r)), f"store_write_chunks: {ctx.last_error()}")
    return st[:n]


def store_read_device(array_meta: ArrayMetadata, paths: Sequence[str], d_ptrs: Sequence[int], device: int = 0,
                      io_threads: int = 16):
    """zcg_store_read_chunks_device: chunk files (shared flock, reader pool,
    pinned staging) decoded straight into the device slots `d_ptrs`
    (N*elem_size bytes each); returns the status array."""
    ctx = _native.context(device)
    n = len(paths)
    dp = (ctypes.c_void_p * max(n, 1))(*[int(p) for p in d_ptrs])
    cp, keep = _cstrs(paths)
    st = np.zeros(max(n, 1), np.int32)
    arr = abi_array(array_meta)
    r = ctx.lib.zcg_store_read_chunks_device(ctx.handle, ctypes.byref(arr), n, ctypes.addressof(cp),
                                             ctypes.addressof(dp), st.ctypes.data, io_threads)
    if r != _native.OK:
        raise ZarrIOError(_native.STATUS_NAMES.get(r, str(r)), f"store_read_chunks_device: {ctx.last_error()}")
    return st[:n]


def store_write_device(array_meta: ArrayMetadata, paths: Sequence[str], d_ptrs: Sequence[int], device: int = 0,
                       io_threads: int = 16):
    """zcg_store_write_chunks_device: the device element slots `d_ptrs`
    encoded on the GPU and written as set() does (exclusive flock, truncate
    after the lock); returns the status array."""
    ctx = _native.context(device)
    n = len(paths)
    dp = (ctypes.c_void_p * max(n, 1))(*[int(p) for p in d_ptrs])
    cp, keep = _cstrs(paths)
    st = np.zeros(max(n, 1), np.int32)
    arr = abi_array(array_meta)
    r = ctx.lib.zcg_store_write_chunks_device(ctx.handle, ctypes.byref(arr), n, ctypes.addressof(cp),
                                              ctypes.addressof(dp), st.ctypes.data, io_threads)
    if r != _native.OK:
        raise ZarrIOError(_native.STATUS_NAMES.get(r, str(r)), f"store_write_chunks_device: {ctx.last_error()}")
    return st[:n]


def chunk_key_native(base_path: str, separator: str, grid_position: Sequence[int]) -> str:
    """zcg_chunk_key (the C-ABI restatement of get_chunk_key, storage.rs:109-127)."""
    L = _native.load_library()
    g = (ctypes.c_uint64 * max(len(grid_position), 1))(*[int(x) for x in grid_position])
    need = L.zcg_chunk_key(base_path.encode(), separator.encode(), ctypes.addressof(g), len(grid_position), None, 0)
    out = ctypes.create_string_buffer(int(need) + 1)
    L.zcg_chunk_key(base_path.encode(), separator.encode(), ctypes.addressof(g), len(grid_position), out, need + 1)
    return out.value.decode()
