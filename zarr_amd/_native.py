"""ctypes binding of ``libzchunk_gpu.so`` (C ABI: ``include/zchunk_gpu.h``).

The product path has no CPU fallback: if the HIP library is missing or no
GPU is visible, every compute call raises :class:`NativeUnavailable`.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZCG_LIB: an alternative build of the same library (A/B kernel experiments)
LIB_PATH = os.environ.get("ZCG_LIB") or os.path.join(_HERE, "libzchunk_gpu.so")

OK, UNEXPECTED_EOF, INVALID_DATA, INVALID_INPUT, UNSUPPORTED, OUTPUT_TOO_SMALL = 0, 1, 2, 3, 4, 5
ABSENT, IO = 6, 7  # store: no chunk file (read_chunk -> None); filesystem error
NOT_FOUND = 8  # store: key outside the hierarchy (filesystem.rs:180-186)
RUNTIME = 100

FLAG_SKIP_LZ4_BLOCK_CHECKSUM = 0x4
FLAG_SERIAL_INFLATE = 0x100
FLAG_DEBUG_COUNTERS = 0x200
FLAG_INFLATE_BLOCK_PAR = 0x2000
FLAG_INFLATE_WAVE = 0x4000
FLAG_DEBUG_INFLATE_LONG_SEG = 0x10000

STATUS_NAMES = {OK: "Ok", UNEXPECTED_EOF: "UnexpectedEof", INVALID_DATA: "InvalidData",
                INVALID_INPUT: "InvalidInput", UNSUPPORTED: "Unsupported",
                OUTPUT_TOO_SMALL: "OutputTooSmall", ABSENT: "NotFound", IO: "Other", NOT_FOUND: "NotFound",
                RUNTIME: "Runtime"}

EXPORTED_SYMBOLS = (
    "zcg_abi_version", "zcg_build_config", "zcg_create", "zcg_destroy", "zcg_last_error",
    "zcg_effective_gzip_level", "zcg_effective_lz4_block_size", "zcg_codec_on_gpu",
    "zcg_decode_batch", "zcg_encode_batch", "zcg_encode_bound", "zcg_workspace_bytes",
    "zcg_read_chunk", "zcg_write_chunk", "zcg_read_chunks_host",
    "zcg_region_grid", "zcg_read_region", "zcg_write_region",
    "zcg_store_read_chunks", "zcg_store_write_chunks",
    "zcg_multi_create", "zcg_multi_destroy", "zcg_multi_last_error", "zcg_multi_device_count",
    "zcg_multi_read_chunks_host", "zcg_multi_store_read_chunks", "zcg_multi_store_write_chunks",
    "zcg_array_meta_from_json", "zcg_chunk_key", "zcg_store_path",
    "zcg_store_read_chunks_device", "zcg_store_write_chunks_device",
)


class NativeUnavailable(RuntimeError):
    pass


class Compression(ctypes.Structure):
    _fields_ = [("codec", ctypes.c_int32), ("gzip_level", ctypes.c_int32),
                ("lz4_block_size", ctypes.c_int32), ("bzip2_block_size", ctypes.c_int32),
                ("xz_preset", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class DType(ctypes.Structure):
    _fields_ = [("elem_size", ctypes.c_uint8), ("big_endian", ctypes.c_uint8),
                ("is_bool", ctypes.c_uint8), ("reserved", ctypes.c_uint8)]


class Array(ctypes.Structure):
    _fields_ = [("compression", Compression), ("dtype", DType),
                ("chunk_num_elements", ctypes.c_uint64)]


class Chunk(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("src_len", ctypes.c_uint64),
                ("dst", ctypes.c_void_p), ("dst_cap", ctypes.c_uint64)]


MAX_DIMS = 8


class Region(ctypes.Structure):
    _fields_ = [("ndim", ctypes.c_uint32), ("elem_size", ctypes.c_uint32),
                ("chunk_order", ctypes.c_uint32), ("fill_missing", ctypes.c_uint32),
                ("array_shape", ctypes.c_uint64 * MAX_DIMS), ("chunk_shape", ctypes.c_uint64 * MAX_DIMS),
                ("bbox_offset", ctypes.c_uint64 * MAX_DIMS), ("bbox_shape", ctypes.c_uint64 * MAX_DIMS),
                ("out_strides", ctypes.c_int64 * MAX_DIMS), ("fill_value", ctypes.c_uint64)]


class ArrayMeta(ctypes.Structure):
    _fields_ = [("array", Array), ("ndim", ctypes.c_uint32), ("chunk_ndim", ctypes.c_uint32),
                ("chunk_order", ctypes.c_uint32), ("dtype_kind", ctypes.c_uint32),
                ("extended_type", ctypes.c_uint32), ("has_fill_value", ctypes.c_uint32),
                ("fill_value_status", ctypes.c_int32), ("reserved", ctypes.c_uint32),
                ("fill_value", ctypes.c_uint64), ("shape", ctypes.c_uint64 * MAX_DIMS),
                ("chunk_shape", ctypes.c_uint64 * MAX_DIMS), ("separator", ctypes.c_char * 8)]


assert ctypes.sizeof(Region) == 16 + 5 * 8 * MAX_DIMS + 8
assert ctypes.sizeof(Compression) == 24 and ctypes.sizeof(Array) == 40
assert ctypes.sizeof(Chunk) == 32

_lib = None
_lock = threading.Lock()


def load_library(path: str = LIB_PATH):
    """Load the HIP library (without touching the GPU)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise NativeUnavailable(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        try:  # share torch's HIP runtime when torch is present (one libamdhip64 per process)
            import torch  # noqa: F401
        except Exception:
            pass
        L = ctypes.CDLL(path)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32
        L.zcg_abi_version.restype = ctypes.c_int
        L.zcg_build_config.restype = ctypes.c_char_p
        L.zcg_create.argtypes = [ctypes.c_int]
        L.zcg_create.restype = vp
        L.zcg_destroy.argtypes = [vp]
        L.zcg_last_error.argtypes = [vp]
        L.zcg_last_error.restype = ctypes.c_char_p
        L.zcg_effective_gzip_level.argtypes = [i32]
        L.zcg_effective_gzip_level.restype = i32
        L.zcg_effective_lz4_block_size.argtypes = [i32]
        L.zcg_effective_lz4_block_size.restype = i32
        L.zcg_codec_on_gpu.argtypes = [i32, ctypes.c_int]
        L.zcg_codec_on_gpu.restype = ctypes.c_int
        L.zcg_decode_batch.argtypes = [vp, ctypes.POINTER(Array), vp, u32, vp, vp]
        L.zcg_decode_batch.restype = ctypes.c_int
        L.zcg_encode_batch.argtypes = [vp, ctypes.POINTER(Array), vp, u32, vp, vp, vp]
        L.zcg_encode_batch.restype = ctypes.c_int
        L.zcg_encode_bound.argtypes = [ctypes.POINTER(Compression), u64]
        L.zcg_encode_bound.restype = u64
        L.zcg_workspace_bytes.argtypes = [ctypes.POINTER(Array), u32, ctypes.c_int]
        L.zcg_workspace_bytes.restype = u64
        L.zcg_read_chunk.argtypes = [vp, ctypes.POINTER(Array), vp, u64, vp]
        L.zcg_read_chunk.restype = ctypes.c_int
        L.zcg_write_chunk.argtypes = [vp, ctypes.POINTER(Array), vp, u64, vp, u64,
                                      ctypes.POINTER(u64)]
        L.zcg_write_chunk.restype = ctypes.c_int
        L.zcg_read_chunks_host.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, vp]
        L.zcg_read_chunks_host.restype = ctypes.c_int
        L.zcg_region_grid.argtypes = [ctypes.POINTER(Region), ctypes.c_void_p, ctypes.c_void_p]
        L.zcg_region_grid.restype = ctypes.c_uint64
        L.zcg_read_region.argtypes = [ctypes.c_void_p, ctypes.POINTER(Region), ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.zcg_read_region.restype = ctypes.c_int
        L.zcg_write_region.argtypes = [ctypes.c_void_p, ctypes.POINTER(Region), ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p]
        L.zcg_write_region.restype = ctypes.c_int
        L.zcg_store_read_chunks.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, u32]
        L.zcg_store_read_chunks.restype = ctypes.c_int
        L.zcg_store_write_chunks.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, u32]
        L.zcg_store_write_chunks.restype = ctypes.c_int
        L.zcg_multi_create.argtypes = [vp, u32]
        L.zcg_multi_create.restype = vp
        L.zcg_multi_destroy.argtypes = [vp]
        L.zcg_multi_last_error.argtypes = [vp]
        L.zcg_multi_last_error.restype = ctypes.c_char_p
        L.zcg_multi_device_count.argtypes = [vp]
        L.zcg_multi_device_count.restype = u32
        L.zcg_multi_read_chunks_host.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, vp]
        L.zcg_multi_read_chunks_host.restype = ctypes.c_int
        L.zcg_multi_store_read_chunks.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, u32]
        L.zcg_multi_store_read_chunks.restype = ctypes.c_int
        L.zcg_multi_store_write_chunks.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, u32]
        L.zcg_multi_store_write_chunks.restype = ctypes.c_int
        L.zcg_array_meta_from_json.argtypes = [ctypes.c_char_p, u64, ctypes.POINTER(ArrayMeta), vp, u64]
        L.zcg_array_meta_from_json.restype = ctypes.c_int
        L.zcg_chunk_key.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, u32, vp, u64]
        L.zcg_chunk_key.restype = u64
        L.zcg_store_path.argtypes = [ctypes.c_char_p, ctypes.c_char_p, vp, u64, ctypes.POINTER(u64)]
        L.zcg_store_path.restype = ctypes.c_int
        L.zcg_store_read_chunks_device.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, u32]
        L.zcg_store_read_chunks_device.restype = ctypes.c_int
        L.zcg_store_write_chunks_device.argtypes = [vp, ctypes.POINTER(Array), u32, vp, vp, vp, u32]
        L.zcg_store_write_chunks_device.restype = ctypes.c_int
        _lib = L
        return L


class Context:
    """One ``zcg_ctx`` (one GPU)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        self.device = device
        self.handle = self.lib.zcg_create(device)
        if not self.handle:
            raise NativeUnavailable(f"zcg_create({device}) failed: no HIP device visible")

    def last_error(self) -> str:
        return (self.lib.zcg_last_error(self.handle) or b"").decode()

    def close(self):
        if self.handle:
            self.lib.zcg_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_contexts = {}


def context(device: int = 0) -> Context:
    with _lock:
        ctx = _contexts.get(device)
    if ctx is None:
        ctx = Context(device)
        with _lock:
            _contexts[device] = ctx
    return ctx


def store_path(root: str, key: str) -> "tuple[int, str]":
    """zcg_store_path (host code, no GPU): (status, path)."""
    L = load_library()
    n = ctypes.c_uint64(0)
    st = L.zcg_store_path(root.encode(), key.encode(), None, 0, ctypes.byref(n))
    if st != OK:
        return st, ""
    out = ctypes.create_string_buffer(n.value + 1)
    st = L.zcg_store_path(root.encode(), key.encode(), ctypes.addressof(out), n.value + 1, ctypes.byref(n))
    return st, out.value.decode()


def array_meta_from_json(text) -> "tuple[int, ArrayMeta, str]":
    """zcg_array_meta_from_json (host code, no GPU): (status, ArrayMeta, message)."""
    L = load_library()
    b = text.encode() if isinstance(text, str) else bytes(text)
    m = ArrayMeta()
    err = ctypes.create_string_buffer(256)
    st = L.zcg_array_meta_from_json(b, len(b), ctypes.byref(m), ctypes.addressof(err), 256)
    return st, m, err.value.decode(errors="replace")
