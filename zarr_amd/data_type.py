"""Zarr v3.0-dev data types — host-side mirror of the reference's
``src/data_type.rs``.

Only what the chunk-codec path needs is mirrored: parsing of the JSON type
string (data_type.rs:125-251), ``ExtensibleDataType.effective_type``
(data_type.rs:282-310), ``size_of`` / ``endian`` / ``eq_modulo_endian``
(data_type.rs:417-444) and the ``ReflectedType`` mapping of element types
(data_type.rs:458-496), expressed with numpy dtypes instead of Rust types.
"""
from __future__ import annotations

import dataclasses
import enum
import sys
from typing import Optional, Union

import numpy as np


class Endian(enum.Enum):
    """data_type.rs:18-60 (serial chars '<' and '>')."""

    Big = ">"
    Little = "<"


NATIVE_ENDIAN = Endian.Little if sys.byteorder == "little" else Endian.Big


class MetadataError(ValueError):
    pass


@dataclasses.dataclass(frozen=True)
class DataType:
    """``enum DataType {Bool, Int, UInt, Float, Raw}`` (data_type.rs:116-123).

    ``kind`` is one of "bool", "int", "uint", "float", "raw"; ``size`` is the
    element size in bytes (Raw: size in BITS as in the reference's ``rN``).
    """

    kind: str
    size: int = 1
    endian: Endian = NATIVE_ENDIAN

    # ---- JSON string form (data_type.rs:125-251) --------------------------
    @staticmethod
    def parse(s: str) -> "DataType":
        if s == "bool":
            return DataType("bool", 1, NATIVE_ENDIAN)
        # "i1"/"u1" parse as Little (data_type.rs:182-189)
        if s == "i1":
            return DataType("int", 1, Endian.Little)
        if s == "u1":
            return DataType("uint", 1, Endian.Little)
        if s.startswith("r"):
            try:
                bits = int(s[1:])
            except ValueError as e:
                raise MetadataError(f"invalid data type {s!r}") from e
            if bits % 8 != 0:
                raise MetadataError(f"invalid data type {s!r}")
            return DataType("raw", bits, NATIVE_ENDIAN)
        if len(s) == 3:
            e, k, n = s[0], s[1], s[2]
            if e not in "<>":
                raise MetadataError(f"invalid data type {s!r}")
            endian = Endian(e)
            kinds = {"i": "int", "u": "uint", "f": "float"}
            if k not in kinds:
                raise MetadataError(f"invalid data type {s!r}")
            if k == "f":
                if n not in "248":
                    raise MetadataError(f"invalid data type {s!r}")
            elif n not in "1248":
                raise MetadataError(f"invalid data type {s!r}")
            return DataType(kinds[k], int(n), endian)
        raise MetadataError(f"invalid data type {s!r}")

    def to_json(self) -> str:
        if self.kind == "bool":
            return "bool"
        if self.kind == "raw":
            return f"r{self.size}"
        k = {"int": "i", "uint": "u", "float": "f"}[self.kind]
        if self.size == 1 and self.kind in ("int", "uint"):
            return f"{k}1"
        return f"{self.endian.value}{k}{self.size}"

    # ---- reflection (data_type.rs:417-444) --------------------------------
    def size_of(self) -> int:
        if self.kind == "raw":
            return self.size // 8
        return self.size

    def effective_endian(self) -> Endian:
        """``DataType::endian`` — single-byte types and bool are native."""
        if self.kind in ("int", "uint", "float"):
            return self.endian
        return NATIVE_ENDIAN

    def eq_modulo_endian(self, other: "DataType") -> bool:
        return self.kind == other.kind and self.size == other.size

    def numpy_dtype(self) -> np.dtype:
        """Host-native element type (``ReflectedType``, data_type.rs:471-482)."""
        if self.kind == "bool":
            return np.dtype(np.bool_)
        if self.kind == "raw":
            raise MetadataError("Raw data types have no ReadableDataChunk impl")
        code = {"int": "i", "uint": "u", "float": "f"}[self.kind]
        return np.dtype(f"{code}{self.size}")


@dataclasses.dataclass(frozen=True)
class ExtendedDataType:
    """``ExtensibleDataType::Extended`` (data_type.rs:282-300)."""

    extension: str
    type_string: str
    fallback: Optional[DataType] = None


ExtensibleDataType = Union[DataType, ExtendedDataType]


def effective_type(d: ExtensibleDataType) -> DataType:
    """data_type.rs:302-310.  The reference panics (``todo!()``) on an
    extended type without fallback; here that is a MetadataError."""
    if isinstance(d, DataType):
        return d
    if d.fallback is not None:
        return d.fallback
    raise MetadataError("extended data type without fallback is not supported")


def parse_extensible(v) -> ExtensibleDataType:
    if isinstance(v, str):
        return DataType.parse(v)
    if isinstance(v, dict):
        fb = v.get("fallback")
        return ExtendedDataType(v["extension"], v["type"], DataType.parse(fb) if fb else None)
    raise MetadataError(f"invalid data type {v!r}")


def extensible_to_json(d: ExtensibleDataType):
    if isinstance(d, DataType):
        return d.to_json()
    out = {"extension": d.extension, "type": d.type_string}
    if d.fallback is not None:
        out["fallback"] = d.fallback.to_json()
    return out


# ReflectedType::ZARR_TYPE for each element type (data_type.rs:471-482).
_REFLECTED = {
    np.dtype(np.bool_): DataType("bool", 1, NATIVE_ENDIAN),
    np.dtype(np.uint8): DataType("uint", 1, NATIVE_ENDIAN),
    np.dtype(np.uint16): DataType("uint", 2, NATIVE_ENDIAN),
    np.dtype(np.uint32): DataType("uint", 4, NATIVE_ENDIAN),
    np.dtype(np.uint64): DataType("uint", 8, NATIVE_ENDIAN),
    np.dtype(np.int8): DataType("int", 1, NATIVE_ENDIAN),
    np.dtype(np.int16): DataType("int", 2, NATIVE_ENDIAN),
    np.dtype(np.int32): DataType("int", 4, NATIVE_ENDIAN),
    np.dtype(np.int64): DataType("int", 8, NATIVE_ENDIAN),
    np.dtype(np.float16): DataType("float", 2, NATIVE_ENDIAN),
    np.dtype(np.float32): DataType("float", 4, NATIVE_ENDIAN),
    np.dtype(np.float64): DataType("float", 8, NATIVE_ENDIAN),
}


def zarr_type(t) -> DataType:
    """``T::ZARR_TYPE`` for a numpy element type."""
    return _REFLECTED[np.dtype(t)]


REFLECTED_TYPES = tuple(_REFLECTED.keys())
