"""CompressionType — host-side mirror of ``src/compression/mod.rs``.

The reference's codec plugin surface is ``trait Compression { decoder;
encoder }`` (mod.rs:30-34) selected through the closed enum
``CompressionType`` (mod.rs:40-51).  Here each variant carries its
configuration and maps onto the C ABI's ``zcg_compression``; the actual
decode/encode is done by the HIP kernels behind ``include/zchunk_gpu.h``.
"""
from __future__ import annotations

import dataclasses
from typing import Any, Dict, Optional

GZIP_CODEC_ID = "https://purl.org/zarr/spec/codec/gzip/1.0"  # mod.rs:45

# Numbering of include/zchunk_gpu.h (enum zcg_codec).
CODEC_RAW, CODEC_BZIP2, CODEC_GZIP, CODEC_LZ4, CODEC_XZ = 0, 1, 2, 3, 4


@dataclasses.dataclass(frozen=True)
class Raw:
    """raw.rs:13-24 — identity."""

    codec_id = CODEC_RAW
    name = "Raw"

    def configuration(self) -> Optional[Dict[str, Any]]:
        return None


@dataclasses.dataclass(frozen=True)
class Bzip2:
    """bzip.rs:16-46 — ``blockSize`` (default 9) is the libbz2 level."""

    block_size: int = 9
    codec_id = CODEC_BZIP2
    name = "Bzip2"

    def configuration(self):
        return {"blockSize": self.block_size}


@dataclasses.dataclass(frozen=True)
class Gzip:
    """gzip.rs:16-57 — ``level`` defaults to -1 (Java's default)."""

    level: int = -1
    codec_id = CODEC_GZIP
    name = "Gzip"

    def effective_level(self) -> int:
        """gzip.rs:28-34: outside [0, 9] -> flate2's default 6."""
        return 6 if self.level < 0 or self.level > 9 else self.level

    def configuration(self):
        return {"level": self.level}


@dataclasses.dataclass(frozen=True)
class Lz4:
    """lz.rs:45-93 — ``blockSize`` default 65 536."""

    block_size: int = 65536
    codec_id = CODEC_LZ4
    name = "Lz4"

    def effective_block_size(self) -> int:
        """lz.rs:55-65: smallest of 64K/256K/1M/4M that is >= blockSize."""
        for b in (65536, 262144, 1048576):
            if self.block_size <= b:
                return b
        return 4194304

    def configuration(self):
        return {"blockSize": self.block_size}


@dataclasses.dataclass(frozen=True)
class Xz:
    """xz.rs:15-43 — ``preset`` default 6."""

    preset: int = 6
    codec_id = CODEC_XZ
    name = "Xz"

    def configuration(self):
        return {"preset": self.preset}


_BY_JSON = {"raw": Raw, "bzip2": Bzip2, GZIP_CODEC_ID: Gzip, "lz4": Lz4, "xz": Xz}
_JSON_KEY = {Raw: "raw", Bzip2: "bzip2", Gzip: GZIP_CODEC_ID, Lz4: "lz4", Xz: "xz"}
_CFG_FIELD = {Bzip2: ("blockSize", "block_size"), Gzip: ("level", "level"),
              Lz4: ("blockSize", "block_size"), Xz: ("preset", "preset")}


class CompressionType:
    """Namespace mirroring the reference enum's constructors and traits."""

    Raw = Raw
    Bzip2 = Bzip2
    Gzip = Gzip
    Lz4 = Lz4
    Xz = Xz

    @staticmethod
    def default():
        """mod.rs:66-70: Raw."""
        return Raw()

    @staticmethod
    def from_str(s: str):
        """``FromStr`` (mod.rs:134-156): case-insensitive variant names."""
        m = {"raw": Raw, "bzip2": Bzip2, "gzip": Gzip, "xz": Xz, "lz4": Lz4}
        k = s.lower()
        if k not in m:
            raise ValueError(f"InvalidInput: unknown compression {s!r}")
        return m[k]()

    @staticmethod
    def display(c) -> str:
        """``Display`` (mod.rs:110-132)."""
        return c.name

    @staticmethod
    def from_json(v: Optional[Dict[str, Any]]):
        """serde ``tag = "codec", content = "configuration"`` (mod.rs:36-51);
        absent compressor -> Raw (lib.rs:398-401, ``#[serde(default)]``)."""
        if v is None:
            return Raw()
        cls = _BY_JSON.get(v.get("codec"))
        if cls is None:
            raise ValueError(f"unknown codec {v.get('codec')!r}")
        if cls is Raw:
            return Raw()
        cfg = v.get("configuration") or {}
        key, field = _CFG_FIELD[cls]
        if key in cfg:
            return cls(**{field: int(cfg[key])})
        return cls()

    @staticmethod
    def to_json(c) -> Dict[str, Any]:
        out: Dict[str, Any] = {"codec": _JSON_KEY[type(c)]}
        cfg = c.configuration()
        if cfg is not None:
            out["configuration"] = cfg
        return out

    @staticmethod
    def is_default(c) -> bool:
        return isinstance(c, Raw)


def to_abi_fields(c) -> Dict[str, int]:
    """Fields of ``zcg_compression`` for this variant."""
    f = {"codec": c.codec_id, "gzip_level": -1, "lz4_block_size": 65536,
         "bzip2_block_size": 9, "xz_preset": 6}
    if isinstance(c, Gzip):
        f["gzip_level"] = c.level
    elif isinstance(c, Lz4):
        f["lz4_block_size"] = c.block_size
    elif isinstance(c, Bzip2):
        f["bzip2_block_size"] = c.block_size
    elif isinstance(c, Xz):
        f["xz_preset"] = c.preset
    return f


def codec_param(c) -> int:
    """The single integer parameter the oracle's encoders take."""
    if isinstance(c, Gzip):
        return c.level
    if isinstance(c, Lz4):
        return c.block_size
    if isinstance(c, Bzip2):
        return c.block_size
    if isinstance(c, Xz):
        return c.preset
    return 0
