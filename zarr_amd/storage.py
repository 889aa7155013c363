"""Minimal FilesystemHierarchy — the caller of the chunk path on both ends
of the north_star e2e path (files -> decode -> files).

Mirrors only what the chunk path needs from ``src/storage.rs`` and
``src/store/filesystem.rs``: the entry point ``zarr.json`` (lib.rs:165-182),
array metadata keys ``/meta/root/<path>.array.json`` (lib.rs:194-201),
chunk keys ``/data/root/<path>/c<i>/<j>/…`` (``get_chunk_key``,
storage.rs:109-127), ``read_chunk`` with a missing chunk -> ``None``
(storage.rs:206-235), ``read_chunk_into`` (237-267), ``write_chunk``
(456-470) and ``delete_chunk``.  Groups/attributes/listing and the flock
concurrency protocol are out of scope.
"""
from __future__ import annotations

import json
import os
from typing import List, Optional, Sequence

from .chunk import DefaultChunk, SliceDataChunk, ZarrIOError, read_chunks_host
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
        parts = [p for p in key.split("/") if p not in ("", ".")]
        if ".." in parts:
            raise ZarrIOError("NotFound", "key escapes the hierarchy root")
        return os.path.join(self.base_path, *parts)

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
        assert array_meta.in_bounds(grid_position)  # storage.rs:217 (a panic there)
        p = self.chunk_path(path_name, array_meta, grid_position)
        if not os.path.isfile(p):
            return None
        with open(p, "rb") as f:
            buf = f.read()
        return DefaultChunk.read_chunk(buf, array_meta, grid_position, t, device=device)

    def read_chunk_into(self, path_name: str, array_meta: ArrayMetadata, grid_position,
                        chunk: SliceDataChunk, t, device: int = 0) -> Optional[bool]:
        assert array_meta.in_bounds(grid_position)
        p = self.chunk_path(path_name, array_meta, grid_position)
        if not os.path.isfile(p):
            return None
        with open(p, "rb") as f:
            buf = f.read()
        DefaultChunk.read_chunk_into(buf, array_meta, grid_position, chunk, t, device=device)
        return True

    def read_chunks(self, path_name: str, array_meta: ArrayMetadata, grid_positions, t,
                    device: int = 0) -> List[Optional[SliceDataChunk]]:
        """Batched read_chunk: all present chunks are decoded in one launch."""
        bufs, idx = [], []
        out: List[Optional[SliceDataChunk]] = [None] * len(grid_positions)
        for i, g in enumerate(grid_positions):
            assert array_meta.in_bounds(g)
            p = self.chunk_path(path_name, array_meta, g)
            if os.path.isfile(p):
                with open(p, "rb") as f:
                    bufs.append(f.read())
                idx.append(i)
        if bufs:
            status, arrs = read_chunks_host(array_meta, bufs, t, device=device)
            for k, i in enumerate(idx):
                if status[k] != 0:
                    from ._native import STATUS_NAMES
                    raise ZarrIOError(STATUS_NAMES.get(int(status[k]), str(status[k])),
                                      f"chunk {list(grid_positions[i])}")
                out[i] = SliceDataChunk(list(grid_positions[i]), arrs[k])
        return out

    def write_chunk(self, path_name: str, array_meta: ArrayMetadata, chunk: SliceDataChunk,
                    device: int = 0) -> None:
        data = DefaultChunk.write_chunk(array_meta, chunk, device=device)
        p = self.chunk_path(path_name, array_meta, chunk.get_grid_position())
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "wb") as f:  # set(): truncate + write (filesystem.rs:260-280)
            f.write(data)

    def delete_chunk(self, path_name: str, array_meta: ArrayMetadata, grid_position) -> bool:
        p = self.chunk_path(path_name, array_meta, grid_position)
        if os.path.isfile(p):
            os.remove(p)
        return True

    def exists_chunk(self, path_name: str, array_meta: ArrayMetadata, grid_position) -> bool:
        return os.path.isfile(self.chunk_path(path_name, array_meta, grid_position))
