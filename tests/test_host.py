"""Host-side mirror of the reference's metadata / codec / dtype types (CPU)."""
import json

import numpy as np
import pytest

from golden_util import zarrita_meta_json
from zarr_amd import (ArrayMetadata, Bzip2, CompressionType, DataType, Endian, Gzip, Lz4, Raw, Xz,
                      ZarrIOError, check_array_type, get_chunk_key, u64_ceil_div, zarr_type)
from zarr_amd.data_type import ExtendedDataType, MetadataError, effective_type, parse_extensible


def test_array_metadata_deserialization():
    """tests.rs:14-95."""
    js = {
        "shape": [10000, 1000], "data_type": "<f8",
        "chunk_grid": {"type": "regular", "chunk_shape": [1000, 100], "separator": "/"},
        "chunk_memory_layout": "C",
        "compressor": {"codec": "https://purl.org/zarr/spec/codec/gzip/1.0",
                       "configuration": {"level": 1}},
        "fill_value": "NaN", "extensions": [],
        "attributes": {"foo": 42, "bar": "apples", "baz": [1, 2, 3, 4]},
    }
    m = ArrayMetadata.from_json(json.dumps(js))
    assert m.shape == [10000, 1000] and m.chunk_shape == [1000, 100]
    assert m.data_type == DataType("float", 8, Endian.Little)
    assert m.compressor == Gzip(1)
    assert m.fill_value == "NaN" and m.attributes["foo"] == 42
    del js["compressor"]
    assert ArrayMetadata.from_json(json.dumps(js)).compressor == Raw()


def test_zarrita_metadata():
    m = ArrayMetadata.from_json(zarrita_meta_json())
    assert m.shape == [4, 5, 6] and m.chunk_shape == [2, 3, 4]
    assert m.compressor == Gzip(1) and m.data_type.to_json() == "<i2"
    # u64_ceil_div over-counts dim 1 (5 % 3 == 3 - 1), as the reference does
    assert m.get_grid_extent() == [2, 3, 2] and m.get_chunk_num_elements() == 24


@pytest.mark.parametrize("s,expect", [
    ("<f8", DataType("float", 8, Endian.Little)), (">u4", DataType("uint", 4, Endian.Big)),
    ("r24", DataType("raw", 24)), ("bool", DataType("bool", 1)),
    ("i1", DataType("int", 1, Endian.Little)), ("u1", DataType("uint", 1, Endian.Little)),
])
def test_data_type_parse(s, expect):
    """data_type.rs doctests (lines 103-114) and the i1/u1 rule (182-189)."""
    d = DataType.parse(s)
    assert d.kind == expect.kind and d.size == expect.size
    if d.kind in ("int", "uint", "float"):
        assert d.endian == expect.endian
    assert DataType.parse(d.to_json()) == d


@pytest.mark.parametrize("bad", ["<f1", "x", "r7", "<q4", "?i2"])
def test_data_type_parse_errors(bad):
    with pytest.raises(MetadataError):
        DataType.parse(bad)


def test_size_of_reflection():
    """data_type.rs:498-524."""
    for t, n in [(np.bool_, 1), (np.uint8, 1), (np.uint16, 2), (np.uint32, 4), (np.uint64, 8),
                 (np.int8, 1), (np.int16, 2), (np.int32, 4), (np.int64, 8), (np.float16, 2),
                 (np.float32, 4), (np.float64, 8)]:
        assert zarr_type(t).size_of() == n
    assert DataType("raw", 24).size_of() == 3


def test_effective_type():
    e = parse_extensible({"extension": "x", "type": "<M8[ns]", "fallback": "<i8"})
    assert effective_type(e) == DataType("int", 8, Endian.Little)
    with pytest.raises(MetadataError):
        effective_type(ExtendedDataType("x", "y", None))


def test_endianness_rule():
    """Single-byte types and bool use native endianness (data_type.rs:425-432)."""
    assert DataType.parse(">i2").effective_endian() == Endian.Big
    assert DataType.parse("bool").effective_endian() == Endian.Little


def test_compression_from_str_display():
    """mod.rs:110-156."""
    for s, cls in [("raw", Raw), ("GZIP", Gzip), ("Lz4", Lz4), ("bzip2", Bzip2), ("xz", Xz)]:
        c = CompressionType.from_str(s)
        assert isinstance(c, cls)
        assert CompressionType.display(c) == cls.name
    with pytest.raises(ValueError):
        CompressionType.from_str("zstd")
    assert CompressionType.default() == Raw()


def test_compression_json_roundtrip():
    for c in [Raw(), Gzip(1), Gzip(), Lz4(123), Bzip2(3), Xz(9)]:
        assert CompressionType.from_json(CompressionType.to_json(c)) == c
    assert CompressionType.from_json({"codec": "lz4"}) == Lz4(65536)
    assert CompressionType.from_json({"codec": "https://purl.org/zarr/spec/codec/gzip/1.0"}) == Gzip(-1)


def test_effective_params():
    """gzip.rs:28-34 and lz.rs:55-65."""
    assert Gzip(-1).effective_level() == 6 and Gzip(10).effective_level() == 6
    assert Gzip(0).effective_level() == 0 and Gzip(9).effective_level() == 9
    assert Lz4(1).effective_block_size() == 65536
    assert Lz4(65537).effective_block_size() == 262144
    assert Lz4(1048576).effective_block_size() == 1048576
    assert Lz4(1048577).effective_block_size() == 4194304


def test_grid_quirks():
    """lib.rs doctests: get_num_chunks == 60, in_bounds; u64_ceil_div quirk."""
    m = ArrayMetadata.new([50, 40, 30], [11, 10, 10], "i1")
    assert m.get_num_chunks() == 60
    assert m.in_bounds([4, 3, 2]) and not m.in_bounds([5, 3, 2])
    assert u64_ceil_div(10, 5) == 2 and u64_ceil_div(11, 5) == 3 and u64_ceil_div(3, 5) == 1
    assert u64_ceil_div(14, 5) == 4  # over-count when a % b == b - 1 (kept)
    assert ArrayMetadata.new([1], [1], "i1").chunk_memory_layout == "F"


def test_chunk_keys():
    """storage.rs:86-108 doctests."""
    m = ArrayMetadata.new([50, 40, 30], [11, 10, 10], "i1")
    assert get_chunk_key("/foo/baz", m, [0, 0, 0]) == "/data/root/foo/baz/c0/0/0"
    assert get_chunk_key("/foo/baz", m, [1, 2, 3]) == "/data/root/foo/baz/c1/2/3"
    m0 = ArrayMetadata.new([], [], "i1")
    assert get_chunk_key("/foo/baz", m0, []) == "/data/root/foo/baz/c"


def test_check_array_type():
    """chunk.rs:253-266: mismatch -> InvalidInput; endianness ignored."""
    m = ArrayMetadata.new([10], [5], ">i2")
    check_array_type(np.int16, m)
    with pytest.raises(ZarrIOError) as e:
        check_array_type(np.int32, m)
    assert e.value.kind == "InvalidInput"


def test_metadata_json_roundtrip():
    m = ArrayMetadata.new([100, 200, 300], [44, 33, 22], "<i2", Lz4(65536))
    m2 = ArrayMetadata.from_json(m.to_json())
    assert m2.shape == m.shape and m2.chunk_shape == m.chunk_shape
    assert m2.compressor == m.compressor and m2.data_type == m.data_type
    assert "compressor" not in json.loads(ArrayMetadata.new([1], [1], "i1").to_json())
