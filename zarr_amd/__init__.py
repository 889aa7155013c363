"""zarr_amd — MI355X-native Zarr chunk-codec path.

Drop-in for the chunk encode/decode path of sci-rs/zarr v0.0.1
(``src/chunk.rs`` + ``src/compression``): every ``CompressionType`` chunk is
decoded/encoded by hand-written gfx950 HIP kernels behind the C ABI in
``include/zchunk_gpu.h``.  The Python layer mirrors the reference's types so
callers (and the parity tests) read like the reference's own.
"""
from .compression import GZIP_CODEC_ID, Bzip2, CompressionType, Gzip, Lz4, Raw, Xz
from .data_type import (DataType, Endian, ExtendedDataType, MetadataError, NATIVE_ENDIAN,
                        REFLECTED_TYPES, effective_type, zarr_type)
from .metadata import ArrayMetadata, u64_ceil_div
from .chunk import (DefaultChunk, SliceDataChunk, VecDataChunk, ZarrIOError, check_array_type,
                    read_chunks_host)
from .storage import FilesystemHierarchy, get_chunk_key
from ._native import NativeUnavailable

__all__ = [
    "ArrayMetadata", "Bzip2", "CompressionType", "DataType", "DefaultChunk", "Endian",
    "ExtendedDataType", "FilesystemHierarchy", "GZIP_CODEC_ID", "Gzip", "Lz4", "MetadataError",
    "NATIVE_ENDIAN", "NativeUnavailable", "REFLECTED_TYPES", "Raw", "SliceDataChunk",
    "VecDataChunk", "Xz", "ZarrIOError", "check_array_type", "effective_type", "get_chunk_key",
    "read_chunks_host", "u64_ceil_div", "zarr_type",
]
