"""ArrayMetadata — host-side mirror of the reference's ``src/lib.rs:382-527``.

Chunk sizing and the codec/dtype carrier of the chunk path.  Chunk memory
order (C/F) does not affect the codec; it is carried for
the JSON round trip only.
"""
from __future__ import annotations

import dataclasses
import json
from typing import Any, Dict, List, Optional, Sequence

from . import compression as _c
from .data_type import (DataType, ExtensibleDataType, effective_type, extensible_to_json,
                        parse_extensible)


def u64_ceil_div(a: int, b: int) -> int:
    """lib.rs:340-342 — kept verbatim, including its over-count when
    ``a % b == b - 1``."""
    return (a + 1) // b + (1 if a % b != 0 else 0)


@dataclasses.dataclass
class ArrayMetadata:
    shape: List[int]
    chunk_shape: List[int]
    data_type: ExtensibleDataType
    compressor: Any = dataclasses.field(default_factory=_c.Raw)
    chunk_memory_layout: str = "F"  # ArrayMetadata::new defaults to F (lib.rs:424)
    separator: str = "/"
    fill_value: Any = None
    extensions: List[Any] = dataclasses.field(default_factory=list)
    attributes: Dict[str, Any] = dataclasses.field(default_factory=dict)
    grid_type: str = "regular"

    @staticmethod
    def new(shape: Sequence[int], chunk_shape: Sequence[int], data_type, compressor=None):
        """lib.rs:405-430."""
        if len(shape) != len(chunk_shape):
            raise ValueError("Number of array dimensions must match number of chunk size dimensions.")
        if isinstance(data_type, str):
            data_type = DataType.parse(data_type)
        return ArrayMetadata(list(shape), list(chunk_shape), data_type,
                             compressor if compressor is not None else _c.Raw())

    # ---- lib.rs:432-527 ----------------------------------------------------
    def get_shape(self) -> List[int]:
        return self.shape

    def get_chunk_shape(self) -> List[int]:
        return self.chunk_shape

    def get_ndim(self) -> int:
        return len(self.shape)

    def get_num_elements(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n

    def get_chunk_num_elements(self) -> int:
        """lib.rs:474-480 (the reference casts to u32 at chunk.rs:280)."""
        n = 1
        for d in self.chunk_shape:
            n *= d
        return n

    def get_grid_extent(self) -> List[int]:
        return [u64_ceil_div(d, b) for d, b in zip(self.shape, self.chunk_shape)]

    def get_num_chunks(self) -> int:
        n = 1
        for d in self.get_grid_extent():
            n *= d
        return n

    def in_bounds(self, grid_position: Sequence[int]) -> bool:
        return len(self.shape) == len(grid_position) and all(
            c < b for b, c in zip(self.get_grid_extent(), grid_position))

    def effective_type(self) -> DataType:
        return effective_type(self.data_type)

    # ---- JSON (serde field names of lib.rs:382-402) -----------------------
    def to_json_dict(self) -> Dict[str, Any]:
        d: Dict[str, Any] = {
            "shape": list(self.shape),
            "data_type": extensible_to_json(self.data_type),
            "chunk_grid": {"type": self.grid_type, "chunk_shape": list(self.chunk_shape),
                           "separator": self.separator},
            "chunk_memory_layout": self.chunk_memory_layout,
            "fill_value": self.fill_value,
            "extensions": self.extensions,
            "attributes": self.attributes,
        }
        if not _c.CompressionType.is_default(self.compressor):
            d["compressor"] = _c.CompressionType.to_json(self.compressor)
        return d

    def to_json(self) -> str:
        return json.dumps(self.to_json_dict())

    @staticmethod
    def from_json(s) -> "ArrayMetadata":
        d = json.loads(s) if isinstance(s, (str, bytes)) else s
        grid = d["chunk_grid"]
        return ArrayMetadata(
            shape=[int(x) for x in d["shape"]],
            chunk_shape=[int(x) for x in grid["chunk_shape"]],
            data_type=parse_extensible(d["data_type"]),
            compressor=_c.CompressionType.from_json(d.get("compressor")),
            chunk_memory_layout=d.get("chunk_memory_layout", "C"),
            separator=grid.get("separator", "/"),
            fill_value=d.get("fill_value"),
            extensions=d.get("extensions", []),
            attributes=d.get("attributes", {}),
            grid_type=grid.get("type", "regular"),
        )

    @staticmethod
    def parse_order(o: Optional[str]) -> str:
        return o or "C"
