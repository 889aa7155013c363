"""Region assembly on the device — ``ZarrNdarrayReader`` (src/ndarray.rs).

``read_ndarray`` / ``read_ndarray_into`` (ndarray.rs:153-268) read every
chunk that ``bounded_coord_iter`` (ndarray.rs:410-432) visits from the
FilesystemHierarchy, decode them in one batch on the GPU (the chunk-codec hot
path), and scatter them into the bounding box with ``zcg_read_region`` — the
decoded chunks never leave HBM.  ``BoundingBox`` mirrors ndarray.rs:42-149.
"""
from __future__ import annotations

import ctypes
import itertools
import os
from typing import List, Sequence

import numpy as np

from . import _native
from .batch import BatchCodec
from .chunk import ZarrIOError, _raise_status, check_array_type
from .metadata import ArrayMetadata


class BoundingBox:
    """ndarray.rs:42-149 (offset/shape per dimension, u64)."""

    def __init__(self, offset: Sequence[int], shape: Sequence[int]):
        assert len(offset) == len(shape)
        self.offset = [int(o) for o in offset]
        self.shape = [int(s) for s in shape]

    def intersect(self, other: "BoundingBox") -> None:
        """ndarray.rs:71-85 (saturating)."""
        for d in range(len(self.offset)):
            new_o = max(other.offset[d], self.offset[d])
            self.shape[d] = max(0, min(self.shape[d] + self.offset[d], other.offset[d] + other.shape[d]) - new_o)
            self.offset[d] = new_o

    def union(self, other: "BoundingBox") -> None:
        """ndarray.rs:95-109."""
        for d in range(len(self.offset)):
            new_o = min(other.offset[d], self.offset[d])
            self.shape[d] = max(self.shape[d] + self.offset[d], other.offset[d] + other.shape[d]) - new_o
            self.offset[d] = new_o

    def end(self) -> List[int]:
        return [o + s for o, s in zip(self.offset, self.shape)]

    def is_empty(self) -> bool:
        return 0 in self.shape

    def __eq__(self, other) -> bool:
        return isinstance(other, BoundingBox) and self.offset == other.offset and self.shape == other.shape

    def __repr__(self) -> str:
        return f"BoundingBox(offset={self.offset}, shape={self.shape})"


def effective_fill_value(meta: ArrayMetadata, t) -> int:
    """lib.rs:448-454: the metadata fill_value as T, else T::default()."""
    v = meta.fill_value
    a = np.array(0 if v is None else v, dtype=np.dtype(t).newbyteorder("="))
    return int.from_bytes(a.tobytes().ljust(8, b"\0"), "little")


def _region(meta: ArrayMetadata, bbox: BoundingBox, es: int, fill: bool, fill_value: int,
            out_strides: Sequence[int]) -> _native.Region:
    nd = meta.get_ndim()
    if nd > _native.MAX_DIMS:
        raise _native.NativeUnavailable(f"region assembly supports up to {_native.MAX_DIMS} dimensions")
    r = _native.Region()
    r.ndim = nd
    r.elem_size = es
    r.chunk_order = 1 if meta.chunk_memory_layout == "F" else 0
    r.fill_missing = 1 if fill else 0
    for d in range(nd):
        r.array_shape[d] = meta.shape[d]
        r.chunk_shape[d] = meta.chunk_shape[d]
        r.bbox_offset[d] = bbox.offset[d]
        r.bbox_shape[d] = bbox.shape[d]
        r.out_strides[d] = int(out_strides[d])
    r.fill_value = fill_value
    return r


def region_grid(meta: ArrayMetadata, bbox: BoundingBox):
    """bounded_coord_iter's grid range (ndarray.rs:410-432) -> (lo, n)."""
    L = _native.load_library()
    nd = meta.get_ndim()
    r = _region(meta, bbox, 1, False, 0, [0] * nd)
    lo = (ctypes.c_uint64 * _native.MAX_DIMS)()
    n = (ctypes.c_uint64 * _native.MAX_DIMS)()
    L.zcg_region_grid(ctypes.byref(r), ctypes.addressof(lo), ctypes.addressof(n))
    return [int(lo[d]) for d in range(nd)], [int(n[d]) for d in range(nd)]


def _strides(shape: Sequence[int], order: str) -> List[int]:
    st, acc = [0] * len(shape), 1
    dims = range(len(shape)) if order == "F" else reversed(range(len(shape)))
    for d in dims:
        st[d] = acc
        acc *= max(int(shape[d]), 1)
    return st


def assemble_region(meta: ArrayMetadata, bbox: BoundingBox, es: int, table, out, out_strides,
                    fill: bool, fill_value: int, device: int = 0, stream=None) -> None:
    """Device-level call: `table` = device int64 tensor of chunk pointers
    (C order over region_grid's range, 0 = absent), `out` = device tensor
    whose data_ptr() is element (0, ..., 0) of the output view."""
    import torch
    ctx = _native.context(device)
    r = _region(meta, bbox, es, fill, fill_value, out_strides)
    s = stream if stream is not None else torch.cuda.current_stream(device)
    h = s.cuda_stream if hasattr(s, "cuda_stream") else int(s)
    st = ctx.lib.zcg_read_region(ctx.handle, ctypes.byref(r), table.data_ptr() if table is not None else None,
                                 out.data_ptr(), h)
    _raise_status(st, ctx, "read_region")


def scatter_region(meta: ArrayMetadata, bbox: BoundingBox, es: int, table, box, box_strides, device: int = 0,
                   stream=None) -> None:
    """Device-level inverse of assemble_region (zcg_write_region): the box
    (`box` = device tensor whose data_ptr() is element (0, ..., 0) of a view
    with `box_strides`) is written into the chunk slots of `table`."""
    import torch
    ctx = _native.context(device)
    r = _region(meta, bbox, es, False, 0, box_strides)
    s = stream if stream is not None else torch.cuda.current_stream(device)
    h = s.cuda_stream if hasattr(s, "cuda_stream") else int(s)
    st = ctx.lib.zcg_write_region(ctx.handle, ctypes.byref(r), table.data_ptr() if table is not None else None,
                                  box.data_ptr(), h)
    _raise_status(st, ctx, "write_region")


# write_ndarray works through the touched chunks in sub-batches of at most this
# many bytes of decoded slots plus encode capacity (device memory bound)
WRITE_BATCH_BYTES = 1 << 30


def _decode_visited(hier, path_name: str, meta: ArrayMetadata, bbox: BoundingBox, device: int):
    """Read + batch-decode the chunks bounded_coord_iter visits, through the
    store's get() semantics (shared flock, filesystem.rs:201-210) straight
    into device slots (zcg_store_read_chunks_device); returns (table tensor,
    keep-alive objects).  An absent chunk is skipped (ndarray.rs:229-231)."""
    import torch
    from .storage import store_read_device
    lo, n = region_grid(meta, bbox)
    coords = list(itertools.product(*[range(l, l + k) for l, k in zip(lo, n)]))  # C order
    for c in coords:
        assert meta.in_bounds(c)  # storage.rs:217 (read_chunk panics out of bounds)
    dev = torch.device("cuda", device)
    table = np.zeros(max(len(coords), 1), np.int64)
    keep = []
    if coords:
        es = meta.effective_type().size_of()
        D = meta.get_chunk_num_elements() * es
        slots = torch.empty(max(len(coords) * D, 1), dtype=torch.uint8, device=dev)
        ptrs = [slots.data_ptr() + i * D for i in range(len(coords))]
        st = store_read_device(meta, [hier.chunk_path(path_name, meta, c) for c in coords], ptrs, device)
        for i, c in enumerate(coords):
            if st[i] == _native.ABSENT:
                continue  # read_chunk -> Ok(None)
            if st[i] != _native.OK:
                raise ZarrIOError(_native.STATUS_NAMES.get(int(st[i]), str(st[i])), f"chunk {list(c)}")
            table[i] = ptrs[i]
        keep.append(slots)
    return torch.from_numpy(table).to(dev), keep


def read_ndarray(hier, path_name: str, meta: ArrayMetadata, bbox: BoundingBox, t, device: int = 0,
                 as_tensor: bool = False):
    """ZarrNdarrayReader::read_ndarray (ndarray.rs:153-174): an array of the
    box's shape in the chunk memory order, fill value where no chunk is."""
    import torch
    check_array_type(t, meta)
    if len(bbox.offset) != meta.get_ndim():
        raise ZarrIOError("InvalidData", "Wrong number of dimensions")
    dt = np.dtype(t).newbyteorder("=")
    es = dt.itemsize
    order = "F" if meta.chunk_memory_layout == "F" else "C"
    st = _strides(bbox.shape, order)
    total = int(np.prod(bbox.shape)) if bbox.shape else 1
    out = torch.empty(max(total * es, 1), dtype=torch.uint8, device=torch.device("cuda", device))
    table, keep = _decode_visited(hier, path_name, meta, bbox, device)
    assemble_region(meta, bbox, es, table, out, st, True, effective_fill_value(meta, dt), device)
    torch.cuda.synchronize(device)
    if as_tensor:
        return out[: total * es], st
    host = out[: total * es].cpu().numpy()
    return np.ndarray(tuple(bbox.shape), dtype=dt, buffer=host, strides=tuple(s * es for s in st)).copy(order=order)


def read_ndarray_into(hier, path_name: str, meta: ArrayMetadata, bbox: BoundingBox, arr: np.ndarray, t,
                      device: int = 0) -> None:
    """ZarrNdarrayReader::read_ndarray_into (ndarray.rs:176-268): elements
    that no present chunk covers keep their values; `arr` may be any
    writable view of the box's shape."""
    import torch
    check_array_type(t, meta)
    if len(bbox.offset) != meta.get_ndim() or meta.get_ndim() != arr.ndim:
        raise ZarrIOError("InvalidData", "Wrong number of dimensions")
    if list(arr.shape) != list(bbox.shape):
        raise ZarrIOError("InvalidData", "Bounding box and array have different shape")
    dt = np.dtype(t).newbyteorder("=")
    es = dt.itemsize
    staged = np.ascontiguousarray(arr, dtype=dt)
    st = _strides(bbox.shape, "C")
    dev = torch.device("cuda", device)
    out = torch.from_numpy(staged.reshape(-1).view(np.uint8).copy() if staged.size else np.zeros(1, np.uint8)).to(dev)
    table, keep = _decode_visited(hier, path_name, meta, bbox, device)
    assemble_region(meta, bbox, es, table, out, st, False, 0, device)
    torch.cuda.synchronize(device)
    if staged.size:
        np.copyto(arr, out.cpu().numpy().view(dt).reshape(staged.shape))


def write_ndarray(hier, path_name: str, meta: ArrayMetadata, offset: Sequence[int], array: np.ndarray,
                  device: int = 0) -> None:
    """ZarrNdarrayWriter::write_ndarray (ndarray.rs:276-385) on the GPU: the
    chunks the box touches are read and decoded when only partly covered
    (absent ones start as fill value), the box is scattered into them by
    zcg_write_region, and all of them are encoded in one batch and written
    through the store's set() semantics (filesystem.rs:260-280)."""
    import torch
    if array.ndim != meta.get_ndim():
        raise ZarrIOError("InvalidData", "Wrong number of dimensions")
    dt = array.dtype.newbyteorder("=")
    check_array_type(dt, meta)
    es = dt.itemsize
    bbox = BoundingBox(offset, list(array.shape))
    lo, n = region_grid(meta, bbox)
    coords = list(itertools.product(*[range(l, l + k) for l, k in zip(lo, n)]))  # C order
    if not coords or bbox.is_empty():
        return
    cs = meta.get_chunk_shape()
    N = meta.get_chunk_num_elements()
    D = N * es
    dev = torch.device("cuda", device)
    codec = BatchCodec(device)
    cap = codec.encode_bound(meta, D)
    box = torch.from_numpy(np.ascontiguousarray(array, dtype=dt).reshape(-1).view(np.uint8).copy()).to(dev)
    ctx = _native.context(device)
    r = _region(meta, bbox, es, False, 0, _strides(bbox.shape, "C"))
    h = torch.cuda.current_stream(device).cuda_stream
    per = max(1, WRITE_BATCH_BYTES // max(D + cap, 1))
    for b0 in range(0, len(coords), per):
        _write_sub_batch(hier, path_name, meta, bbox, coords, b0, min(len(coords), b0 + per), dt, D, N, cap,
                         box, ctx, r, h, codec, dev)


def _write_sub_batch(hier, path_name, meta, bbox, coords, b0, b1, dt, D, N, cap, box, ctx, r, h, codec, dev):
    """write_ndarray for coords[b0:b1]: read/decode the partly covered chunks
    into their slots (store get(): shared flock), scatter the box into all of
    them, encode and write every chunk file through the store's set()
    (zcg_store_write_chunks_device: exclusive flock, then truncate)."""
    import torch
    from .storage import store_read_device, store_write_device
    cs = meta.get_chunk_shape()
    m = b1 - b0
    slots = torch.empty(m * D, dtype=torch.uint8, device=dev)
    ptrs = [slots.data_ptr() + i * D for i in range(m)]
    paths = [hier.chunk_path(path_name, meta, coords[b0 + i]) for i in range(m)]
    partial = []
    for i in range(m):
        c = coords[b0 + i]
        assert meta.in_bounds(c)  # storage.rs:217
        nom = BoundingBox([ci * s for ci, s in zip(c, cs)], cs)
        wb = BoundingBox(nom.offset, nom.shape)
        wb.intersect(bbox)
        if wb != nom:
            partial.append(i)  # fully overwritten chunks are not read (ndarray.rs:328-337)
    absent = []
    if partial:
        st = store_read_device(meta, [paths[i] for i in partial], [ptrs[i] for i in partial], ctx.device)
        for k, i in enumerate(partial):
            if st[k] == _native.ABSENT:
                absent.append(i)  # starts as fill value (ndarray.rs:357-368)
            elif st[k] != _native.OK:
                raise ZarrIOError(_native.STATUS_NAMES.get(int(st[k]), str(st[k])), f"chunk {list(coords[b0 + i])}")
    if absent:
        fill = np.full(N, 0 if meta.fill_value is None else meta.fill_value, dtype=dt)
        ft = torch.from_numpy(fill.view(np.uint8)).to(dev)
        for i in absent:
            slots[i * D:(i + 1) * D].copy_(ft)
    # the region call covers the whole grid range: chunks outside this
    # sub-batch get NULL slots and are skipped
    table_h = np.zeros(len(coords), np.int64)
    table_h[b0:b1] = ptrs
    table = torch.from_numpy(table_h).to(dev)
    _raise_status(ctx.lib.zcg_write_region(ctx.handle, ctypes.byref(r), table.data_ptr(), box.data_ptr(), h),
                  ctx, "write_region")
    torch.cuda.synchronize(dev)  # the store's streams read the slots next
    st = store_write_device(meta, paths, ptrs, ctx.device)
    bad = np.nonzero(st != 0)[0]
    if len(bad):
        i = int(bad[0])
        raise ZarrIOError(_native.STATUS_NAMES.get(int(st[i]), str(st[i])), f"chunk {list(coords[b0 + i])}")
