"""The C++ array-metadata parser behind the ABI (zcg_array_meta_from_json,
SURVEY §8(f) rank 4) against the host mirror (zarr_amd.metadata, itself
pinned to the reference's serde rules: lib.rs:382-402, data_type.rs:125-251,
compression/mod.rs:36-51).  Pure host code: runs without a GPU."""
import ctypes
import json
import os
import struct

import numpy as np
import pytest

from golden_util import GOLDEN
from zarr_amd import ArrayMetadata, _native
from zarr_amd.compression import Bzip2, CompressionType, Gzip, Lz4, Raw, Xz

CODEC_ID = {"Raw": 0, "Bzip2": 1, "Gzip": 2, "Lz4": 3, "Xz": 4}

DTYPES = ["bool", "i1", "u1", "<i1", ">u1", "<i2", ">i2", "<u2", ">u2", "<i4", ">i4", "<u4", ">u4",
          "<i8", ">i8", "<u8", ">u8", "<f2", ">f2", "<f4", ">f4", "<f8", ">f8"]


def native(doc):
    st, m, err = _native.array_meta_from_json(doc if isinstance(doc, str) else json.dumps(doc))
    return st, m, err


def check_same(meta: ArrayMetadata, m):
    assert m.ndim == len(meta.shape) and list(m.shape)[:m.ndim] == meta.shape
    assert list(m.chunk_shape)[:m.chunk_ndim] == meta.chunk_shape
    assert m.chunk_order == (1 if meta.chunk_memory_layout == "F" else 0)
    assert m.separator.decode() == meta.separator
    t = meta.effective_type()
    assert m.array.dtype.elem_size == t.size_of()
    assert m.array.dtype.is_bool == (1 if t.kind == "bool" else 0)
    assert m.array.dtype.big_endian == (1 if (t.size_of() > 1 and t.effective_endian().value == ">") else 0)
    assert m.array.chunk_num_elements == meta.get_chunk_num_elements()
    c = meta.compressor
    assert m.array.compression.codec == CODEC_ID[type(c).__name__]
    if isinstance(c, Gzip):
        assert m.array.compression.gzip_level == c.level
    if isinstance(c, Lz4):
        assert m.array.compression.lz4_block_size == c.block_size
    if isinstance(c, Bzip2):
        assert m.array.compression.bzip2_block_size == c.block_size
    if isinstance(c, Xz):
        assert m.array.compression.xz_preset == c.preset


def test_zarrita_array_document():
    text = open(os.path.join(GOLDEN, "zarrita", "meta", "root", "seq", "i2.array.json")).read()
    st, m, err = native(text)
    assert st == _native.OK, err
    check_same(ArrayMetadata.from_json(text), m)
    assert m.array.compression.codec == 2 and m.array.compression.gzip_level == 1
    assert m.has_fill_value == 0 and m.fill_value == 0


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("comp", [Raw(), Gzip(-1), Gzip(9), Lz4(65536), Lz4(1 << 20), Bzip2(9), Bzip2(1), Xz(6),
                                  Xz(0)], ids=lambda c: CompressionType.display(c))
def test_roundtrip_with_host_mirror(dt, comp):
    meta = ArrayMetadata.new([100, 200, 300], [44, 33, 22], dt, comp)
    meta.chunk_memory_layout = "C" if len(dt) % 2 else "F"
    st, m, err = native(meta.to_json())
    assert st == _native.OK, err
    check_same(ArrayMetadata.from_json(meta.to_json()), m)


def _doc(**over):
    d = {"shape": [10, 20], "data_type": "<i4",
         "chunk_grid": {"type": "regular", "chunk_shape": [5, 4], "separator": "/"},
         "chunk_memory_layout": "C", "fill_value": None, "extensions": [], "attributes": {}}
    d.update(over)
    return {k: v for k, v in d.items() if v is not ...}


def test_codec_defaults_and_configuration():
    # configuration keys absent -> the codecs' serde defaults
    for codec, field, want in (("https://purl.org/zarr/spec/codec/gzip/1.0", "gzip_level", -1),
                               ("lz4", "lz4_block_size", 65536), ("bzip2", "bzip2_block_size", 9),
                               ("xz", "xz_preset", 6)):
        st, m, err = native(_doc(compressor={"codec": codec, "configuration": {}}))
        assert st == _native.OK, err
        assert getattr(m.array.compression, field) == want
    st, m, _ = native(_doc(compressor={"codec": "lz4", "configuration": {"blockSize": 262144}}))
    assert st == _native.OK and m.array.compression.lz4_block_size == 262144
    st, m, _ = native(_doc())  # absent compressor -> Raw (#[serde(default)])
    assert st == _native.OK and m.array.compression.codec == 0
    st, _, _ = native(_doc(compressor={"codec": "zstd"}))
    assert st == _native.INVALID_DATA
    st, _, _ = native(_doc(compressor={"codec": "xz", "configuration": {"preset": "six"}}))
    assert st == _native.INVALID_DATA


@pytest.mark.parametrize("codec,key", [("https://purl.org/zarr/spec/codec/gzip/1.0", "level"),
                                       ("lz4", "blockSize"), ("xz", "preset")])
def test_codec_configuration_outside_i32(codec, key):
    # the reference's configuration fields are i32: serde rejects values outside it
    for v in (2 ** 31, -(2 ** 31) - 1, 2 ** 40):
        st, _, _ = native(_doc(compressor={"codec": codec, "configuration": {key: v}}))
        assert st == _native.INVALID_DATA, (codec, v)
    st, _, _ = native(_doc(compressor={"codec": codec, "configuration": {key: 2 ** 31 - 1}}))
    assert st == _native.OK


def test_chunk_shape_product_overflow():
    st, _, err = native(_doc(chunk_grid={"type": "regular", "chunk_shape": [2 ** 32 - 1] * 3, "separator": "/"}))
    assert st == _native.INVALID_DATA and "overflow" in err
    st, m, _ = native(_doc(chunk_grid={"type": "regular", "chunk_shape": [2 ** 32 - 1, 2 ** 32 - 1],
                                       "separator": "/"}))
    assert st == _native.OK and m.array.chunk_num_elements == (2 ** 32 - 1) ** 2


def test_extended_types_and_extensions():
    ext = {"extension": "https://example.org/dt/complex", "type": "complex128", "fallback": ">u8"}
    st, m, err = native(_doc(data_type=ext))
    assert st == _native.OK, err
    assert m.extended_type == 1 and m.array.dtype.elem_size == 8 and m.array.dtype.big_endian == 1
    st, _, err = native(_doc(data_type={"extension": "x", "type": "y"}))
    assert st == _native.UNSUPPORTED  # effective_type: todo!() in the reference
    st, _, _ = native(_doc(extensions=[{"extension": "http://e/foo", "must_understand": False}]))
    assert st == _native.OK
    st, _, err = native(_doc(extensions=[{"extension": "http://e/foo", "must_understand": True}]))
    assert st == _native.UNSUPPORTED and "must be understood" in err  # storage.rs:172-176


@pytest.mark.parametrize("bad", ["|i2", "<i3", "<f1"])
def test_reference_panics_are_unsupported(bad):
    st, _, _ = native(_doc(data_type=bad))  # expect("TODO") / unwrap() in DataTypeVisitor
    assert st == _native.UNSUPPORTED


@pytest.mark.parametrize("bad", ["<c8", "int32", "r12", "rx", ""])
def test_invalid_data_types(bad):
    st, _, _ = native(_doc(data_type=bad))
    assert st == _native.INVALID_DATA


def test_raw_types_parse():
    st, m, _ = native(_doc(data_type="r24"))
    assert st == _native.OK and m.dtype_kind == _native_kind("raw") and m.array.dtype.elem_size == 3


def _native_kind(k):
    return {"bool": 0, "int": 1, "uint": 2, "float": 3, "raw": 4}[k]


@pytest.mark.parametrize("missing", ["shape", "data_type", "chunk_grid", "chunk_memory_layout", "extensions",
                                     "attributes"])
def test_required_fields(missing):
    d = _doc()
    del d[missing]
    st, _, err = native(d)
    assert st == _native.INVALID_DATA and missing in err
    d = _doc()
    del d["fill_value"]  # Option<Value>: absent is None
    assert native(d)[0] == _native.OK


@pytest.mark.parametrize("text", ["", "{", "[]", '{"shape": [1,]}', '{"a": 1} x', "nul",
                                  '{"shape": [01]}'])
def test_malformed_json(text):
    assert native(text)[0] == _native.INVALID_DATA


@pytest.mark.parametrize("dt,val,want", [
    ("<i4", 5, 5), ("<i4", -1, 0xFFFFFFFF), ("<i2", -32768, 0x8000), ("<u1", 255, 255),
    ("<i8", -9223372036854775808, 1 << 63), ("<u8", 18446744073709551615, (1 << 64) - 1),
    ("<f4", 1.5, struct.unpack("<I", struct.pack("<f", 1.5))[0]),
    ("<f8", -2.25, struct.unpack("<Q", struct.pack("<d", -2.25))[0]),
    ("<f2", 0.333, int(np.array(0.333, np.float16).view(np.uint16))),
    ("bool", True, 1), ("<f4", 3, struct.unpack("<I", struct.pack("<f", 3.0))[0])])
def test_fill_values(dt, val, want):
    st, m, err = native(_doc(data_type=dt, fill_value=val))
    assert st == _native.OK, err
    assert m.has_fill_value == 1 and m.fill_value_status == 0 and m.fill_value == want


@pytest.mark.parametrize("dt,val", [("<u1", 256), ("<i1", -129), ("<u4", -1), ("<i4", 1.5), ("bool", 1),
                                    ("<f4", "NaN"), ("<i2", [1])])
def test_fill_values_that_do_not_convert(dt, val):
    # the document parses (Option<Value>); get_effective_fill_value fails later
    st, m, _ = native(_doc(data_type=dt, fill_value=val))
    assert st == _native.OK and m.has_fill_value == 0 and m.fill_value_status != 0


def test_unicode_and_escapes():
    d = _doc(attributes={"name": "café 😀 \"q\" \\ /"}, chunk_grid={
        "type": "regular", "chunk_shape": [5, 4], "separator": "."})
    st, m, err = native(json.dumps(d))
    assert st == _native.OK, err
    assert m.separator == b"."


def test_chunk_key_matches_get_chunk_key():
    """zcg_chunk_key is storage.rs:109-127 (with canonicalize_path, lib.rs:187-189),
    including the reference's doctest (storage.rs:86-108)."""
    from zarr_amd.storage import chunk_key_native, get_chunk_key
    assert chunk_key_native("/foo/baz", "/", []) == "/data/root/foo/baz/c"
    assert chunk_key_native("foo/baz", "/", [1, 2, 3]) == "/data/root/foo/baz/c1/2/3"
    assert chunk_key_native("", ".", [0, 10]) == "/data/root/c0.10"
    assert chunk_key_native("///", "/", [7]) == "/data/root/c7"
    for path in ("/seq/i2", "a/b/", "//x//", "", "/"):
        for sep in ("/", ".", "--"):
            for grid in ([], [0], [3, 4], [2 ** 40, 0, 5, 1]):
                meta = ArrayMetadata.new([1] * max(len(grid), 1), [1] * max(len(grid), 1), "<i2", Raw())
                meta.separator = sep
                assert chunk_key_native(path, sep, grid) == get_chunk_key(path, meta, grid), (path, sep, grid)


def test_store_path_net_nesting_rule(tmp_path):
    """zcg_store_path is FilesystemHierarchy::get_path (filesystem.rs:151-190):
    leading '/'s dropped, '.' and empty components dropped, '..' kept, and
    NotFound only when the NET nesting is negative (not a prefix check)."""
    root = str(tmp_path)
    ok = {
        "/data/root/c0/0": root + "/data/root/c0/0",
        "a/../b": root + "/a/../b",          # net 1: accepted, '..' left to the OS
        "/./c0/0": root + "/c0/0",
        "//a//b/": root + "/a/b",
        "../a/b": root + "/../a/b",          # net 1: the reference accepts it too
        "a/../../b": root + "/a/../../b",    # net 0: accepted (prefix escape the rule allows)
        "": root,
        "/": root,
        ".": root,
    }
    for key, want in ok.items():
        st, p = _native.store_path(root, key)
        assert st == _native.OK and p == want, (key, st, p)
    # "../x" nets 0: the reference accepts it (its check is the net count only)
    st, p = _native.store_path(root, "../x")
    assert st == _native.OK and p == root + "/../x"
    for key in ("..", "/../", "../../x", "a/../../x/..", "./../", "a/b/../../.."):
        st, p = _native.store_path(root, key)
        assert st == _native.NOT_FOUND, (key, st, p)
    # an empty root: PathBuf::from("").join(rel) is the relative path itself
    for key, want in {"a/b": "a/b", "/c0/0": "c0/0", "": "", "./x": "x"}.items():
        st, p = _native.store_path("", key)
        assert st == _native.OK and p == want, (key, st, p)
    # the Python store goes through the same rule
    from zarr_amd.storage import FilesystemHierarchy
    from zarr_amd.chunk import ZarrIOError
    h = FilesystemHierarchy.open_or_create(root)
    assert h._path("a/../b") == root + "/a/../b"
    with pytest.raises(ZarrIOError) as e:
        h._path("/../../x")
    assert e.value.kind == "NotFound"
    # a too-small buffer reports the length
    L = _native.load_library()
    n = ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(4)
    assert L.zcg_store_path(root.encode(), b"abc", ctypes.addressof(buf), 4, ctypes.byref(n)) == \
        _native.OUTPUT_TOO_SMALL
    assert n.value == len(root) + 4
