"""Chunk containers and ``DefaultChunk`` — host-side mirror of the reference's
``src/chunk.rs``, computing on the GPU through the C ABI.

* ``SliceDataChunk`` / ``VecDataChunk``  (chunk.rs:64-101)
* ``DefaultChunk.read_chunk``            (chunk.rs:270-286)
* ``DefaultChunk.read_chunk_into``       (chunk.rs:288-301)
* ``DefaultChunk.write_chunk``           (chunk.rs:306-323)
* ``check_array_type``                   (chunk.rs:253-266)

Errors are :class:`ZarrIOError` carrying the reference's ``io::ErrorKind``
name in ``.kind`` (``UnexpectedEof``, ``InvalidData``, ``InvalidInput`` …).
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Any, List, Sequence

import numpy as np

from . import _native
from .compression import to_abi_fields
from .data_type import DataType, NATIVE_ENDIAN, zarr_type
from .metadata import ArrayMetadata


class ZarrIOError(OSError):
    """``std::io::Error`` of the reference: ``kind`` is the ErrorKind name."""

    def __init__(self, kind: str, msg: str = ""):
        super().__init__(f"{kind}: {msg}" if msg else kind)
        self.kind = kind


def _raise_status(st: int, ctx: _native.Context = None, what: str = ""):
    if st == _native.OK:
        return
    kind = _native.STATUS_NAMES.get(st, f"Status{st}")
    msg = what
    if st == _native.RUNTIME and ctx is not None:
        msg = f"{what}: {ctx.last_error()}"
    if st == _native.UNSUPPORTED:
        raise _native.NativeUnavailable(f"{what}: no GPU implementation ({ctx.last_error() if ctx else ''})")
    raise ZarrIOError(kind, msg)


@dataclasses.dataclass
class SliceDataChunk:
    """``SliceDataChunk<T, C>`` (chunk.rs:64-84): grid position + element data."""

    grid_position: List[int]
    data: Any  # numpy array (or anything np.asarray accepts) of the element type

    def get_grid_position(self) -> List[int]:
        return list(self.grid_position)

    def get_data(self) -> np.ndarray:
        return np.asarray(self.data)

    def get_num_elements(self) -> int:
        return int(np.asarray(self.data).size)

    def into_data(self):
        return self.data


VecDataChunk = SliceDataChunk  # chunk.rs:86-88 — read chunks are returned as this


def abi_dtype(dt: DataType) -> _native.DType:
    es = dt.size_of()
    be = 1 if (dt.effective_endian().value == ">" and es > 1 and dt.kind != "bool") else 0
    return _native.DType(es, be, 1 if dt.kind == "bool" else 0, 0)


def abi_array(meta: ArrayMetadata, flags: int = 0) -> _native.Array:
    dt = meta.effective_type()
    f = to_abi_fields(meta.compressor)
    comp = _native.Compression(f["codec"], f["gzip_level"], f["lz4_block_size"],
                               f["bzip2_block_size"], f["xz_preset"], flags)
    return _native.Array(comp, abi_dtype(dt), meta.get_chunk_num_elements())


def check_array_type(t, meta: ArrayMetadata) -> None:
    """chunk.rs:253-266 — element type must match modulo endianness."""
    if not meta.effective_type().eq_modulo_endian(zarr_type(t)):
        raise ZarrIOError("InvalidInput", "Attempt to create data chunk for wrong type.")


class DefaultChunk:
    """``DefaultChunkReader`` / ``DefaultChunkWriter`` (chunk.rs:268-335)."""

    @staticmethod
    def read_chunk(buffer, array_meta: ArrayMetadata, grid_position: Sequence[int], t,
                   device: int = 0, flags: int = 0) -> SliceDataChunk:
        check_array_type(t, array_meta)
        nel = array_meta.get_chunk_num_elements()
        out = np.zeros(nel, dtype=np.dtype(t))  # create_data_chunk zero-fills (data_type.rs:463-468)
        DefaultChunk._decode_into(buffer, array_meta, out, device, flags)
        return SliceDataChunk(list(grid_position), out)

    @staticmethod
    def read_chunk_into(buffer, array_meta: ArrayMetadata, grid_position: Sequence[int],
                        chunk: SliceDataChunk, t, device: int = 0, flags: int = 0) -> None:
        check_array_type(t, array_meta)
        nel = array_meta.get_chunk_num_elements()
        # ReinitDataChunk::reinitialize (chunk.rs:91-94): resize to N elements
        data = np.asarray(chunk.data)
        if data.dtype != np.dtype(t) or data.size != nel or not data.flags.c_contiguous:
            data = np.zeros(nel, dtype=np.dtype(t))
        chunk.grid_position = list(grid_position)
        chunk.data = data
        DefaultChunk._decode_into(buffer, array_meta, data, device, flags)

    @staticmethod
    def _decode_into(buffer, meta, out: np.ndarray, device: int, flags: int) -> None:
        ctx = _native.context(device)
        # the stream is passed in place (zcg_read_chunk only reads it): no copy
        # for bytes / bytearray / contiguous memoryviews
        try:
            src = np.frombuffer(buffer, dtype=np.uint8)
        except (TypeError, ValueError, BufferError):
            src = np.frombuffer(bytes(buffer), dtype=np.uint8)
        if src.size == 0:
            src = np.zeros(1, np.uint8)[:0]
        arr = abi_array(meta, flags)
        st = ctx.lib.zcg_read_chunk(ctx.handle, ctypes.byref(arr), src.ctypes.data, src.size,
                                    out.ctypes.data if out.size else None)
        _raise_status(st, ctx, "read_chunk")

    @staticmethod
    def write_chunk(array_meta: ArrayMetadata, chunk: SliceDataChunk, t=None,
                    device: int = 0) -> bytes:
        data = np.ascontiguousarray(np.asarray(chunk.get_data()))
        t = data.dtype if t is None else np.dtype(t)
        check_array_type(t, array_meta)
        if data.size != array_meta.get_chunk_num_elements():  # chunk.rs:309-318
            raise ZarrIOError(
                "InvalidData",
                f"Can not write chunk with too few elements. Expected "
                f"{array_meta.get_chunk_num_elements()} given {data.size}")
        ctx = _native.context(device)
        arr = abi_array(array_meta)
        data = data.astype(np.dtype(t).newbyteorder("="), copy=False)
        nb = data.size * data.dtype.itemsize
        cap = int(ctx.lib.zcg_encode_bound(ctypes.byref(arr.compression), nb)) + 64
        out = np.empty(cap, np.uint8)
        olen = ctypes.c_uint64(0)
        src = data.view(np.uint8) if nb else np.zeros(1, np.uint8)
        st = ctx.lib.zcg_write_chunk(ctx.handle, ctypes.byref(arr), src.ctypes.data, data.size,
                                     out.ctypes.data, cap, ctypes.byref(olen))
        _raise_status(st, ctx, "write_chunk")
        return out[: olen.value].tobytes()


def read_chunks_host(array_meta: ArrayMetadata, buffers: Sequence[bytes], t, device: int = 0,
                     flags: int = 0):
    """Batched read_chunk over host buffers (e2e path: pinned H2D, one
    decode launch, D2H).  Returns (status array, list of element arrays)."""
    check_array_type(t, array_meta)
    ctx = _native.context(device)
    n = len(buffers)
    nel = array_meta.get_chunk_num_elements()
    outs = [np.zeros(nel, dtype=np.dtype(t)) for _ in range(n)]
    keep = [ctypes.create_string_buffer(bytes(b), max(len(b), 1)) for b in buffers]
    srcs = (ctypes.c_void_p * n)(*[ctypes.addressof(k) for k in keep])
    lens = (ctypes.c_uint64 * n)(*[len(b) for b in buffers])
    dsts = (ctypes.c_void_p * n)(*[o.ctypes.data if o.size else None for o in outs])
    status = np.zeros(n, np.int32)
    arr = abi_array(array_meta, flags)
    r = ctx.lib.zcg_read_chunks_host(ctx.handle, ctypes.byref(arr), n, ctypes.addressof(srcs),
                                     ctypes.addressof(lens), ctypes.addressof(dsts),
                                     status.ctypes.data)
    _raise_status(r, ctx, "read_chunks_host")
    return status, outs
