"""GPU encoders (write_chunk, chunk.rs:306-323).

The reference pins encoded bytes only for the doc-spec vectors
(tests.rs:147-159); everything larger is "parity unpinned" in the reference's
own tests (zarrita_compat.rs:101-102).  LZ4 frames are
nevertheless compared byte for byte with the oracle's liblz4 LZ4F frames
(the library lz4-rs wraps, fed as lz4-rs feeds it): the GPU block compressor
restates liblz4's, so write_chunk's bytes are the reference's.  For every
codec the GPU stream must also (a) decode with the oracle to exactly the
serialised input, (b) carry the crate's container conventions (lz4: lz.rs:81-92
FLG 0x64, BD from the effective block size, header checksum, independent
blocks, content checksum = XXH32 of the content), and (c) decode with our own
GPU decoder.
"""
import os
import struct

import numpy as np
import pytest

from golden_util import doc_spec
from zarr_amd import ArrayMetadata, DefaultChunk, Lz4, SliceDataChunk, ZarrIOError

pytestmark = pytest.mark.gpu

zref = pytest.importorskip("zref")


def xxh32(b: bytes) -> int:
    import xxhash
    return xxhash.xxh32_intdigest(b)


def serialised(data: np.ndarray, dt: str) -> bytes:
    """write_data's byte stream (chunk.rs:118-140): array byte order, bool 0/1."""
    if dt == "bool":
        return data.astype(np.uint8).tobytes()
    return data.astype(np.dtype(dt)).tobytes()


def encode_batch(meta, arrays, cap_extra=0):
    """zcg_encode_batch over device buffers; returns (status, [bytes])."""
    import torch
    from zarr_amd.batch import BatchCodec, make_encode_batch
    codec = BatchCodec(0)
    D = arrays[0].nbytes
    n = len(arrays)
    host = np.concatenate([a.view(np.uint8).reshape(-1) for a in arrays]) if D else np.zeros(1, np.uint8)
    elems = torch.from_numpy(host).to("cuda:0")
    cap = codec.encode_bound(meta, D) + cap_extra
    desc, dst, out_len, status = make_encode_batch(elems, n, cap, "cuda:0") if D else (None,) * 4
    if not D:  # zero-byte chunks: descriptors by hand
        desc, dst, out_len, status = make_encode_batch(torch.zeros(n, dtype=torch.uint8, device="cuda:0"),
                                                       n, cap, "cuda:0")
        d = desc.cpu().numpy().view(np.uint64).reshape(n, 4).copy()
        d[:, 1] = 0
        desc = torch.from_numpy(d.view(np.int64)).to("cuda:0")
    codec.encode(meta, desc, n, out_len, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    ol = out_len.cpu().numpy()
    buf = dst.cpu().numpy().reshape(n, cap)
    return st, [buf[i, : ol[i]].tobytes() for i in range(n)]


def check_lz4_frame(stream: bytes, content: bytes, block_size: int):
    # byte-identical to lz4-rs's frame (liblz4 LZ4F, level 0, independent blocks)
    st, ref = zref.encode(zref.LZ4, block_size, np.frombuffer(content, np.uint8))
    assert st == zref.OK
    if stream != ref:
        k = next((i for i in range(min(len(stream), len(ref))) if stream[i] != ref[i]), min(len(stream), len(ref)))
        raise AssertionError(f"lz4 frame differs from liblz4's at byte {k} (len {len(stream)} vs {len(ref)})")
    assert stream[:4] == b"\x04\x22\x4d\x18"
    flg, bd = stream[4], stream[5]
    assert flg == 0x64  # version 01 | independent blocks | content checksum
    eff = 65536 if block_size <= 65536 else 262144 if block_size <= 262144 else \
        1048576 if block_size <= 1048576 else 4194304
    assert bd == {65536: 0x40, 262144: 0x50, 1048576: 0x60, 4194304: 0x70}[eff]
    assert stream[6] == (xxh32(bytes([flg, bd])) >> 8) & 0xFF
    pos, total = 7, 0
    while True:
        (w,) = struct.unpack_from("<I", stream, pos)
        pos += 4
        if w == 0:
            break
        size = w & 0x7FFFFFFF
        raw = w >> 31
        blk = min(eff, len(content) - total)
        assert size <= (blk if raw else blk - 1)
        if raw:
            assert stream[pos:pos + size] == content[total:total + size]
        total += blk
        pos += size
    assert total == len(content)
    assert struct.unpack_from("<I", stream, pos)[0] == xxh32(content)
    assert pos + 4 == len(stream)


def test_lz4_encode_doc_spec_exact():
    """tests.rs:147-159 + lz.rs:101-115: byte-identical to the reference vector."""
    d = doc_spec()
    meta = ArrayMetadata.new([5, 6, 7], [1, 2, 3], ">i2", Lz4(65536))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0, 0, 0], np.array(d["expected_values"], np.int16)))
    assert out.hex() == d["encode_expected"]["lz4"]


def _data(kind, nbytes, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "zeros":
        return np.zeros(nbytes, np.uint8)
    if kind == "uniform":
        return rng.integers(0, 256, nbytes, dtype=np.uint8)
    if kind == "randwalk":
        return np.cumsum(rng.integers(-3, 4, nbytes // 2 + 1)).astype("<i2").view(np.uint8)[:nbytes]
    if kind == "text":
        return np.frombuffer((b"the quick brown fox jumps over the lazy dog %d\n" * (nbytes // 40 + 2)
                              )[:nbytes], np.uint8).copy()
    if kind == "ramp":
        return (np.arange(nbytes // 2 + 1) % 4096).astype("<i2").view(np.uint8)[:nbytes]
    if kind == "mixed":  # compressible and incompressible blocks alternate
        a = rng.integers(0, 256, nbytes, dtype=np.uint8)
        for s in range(0, nbytes, 131072):
            a[s:s + 65536] = 7
        return a
    raise ValueError(kind)


@pytest.mark.parametrize("block", [65536, 262144, 1048576, 4194304])
@pytest.mark.parametrize("kind", ["zeros", "uniform", "randwalk", "text", "ramp", "mixed"])
def test_lz4_encode_roundtrip(kind, block):
    D = 1 << 20
    arrays = [_data(kind, D, seed=s) for s in range(3)]
    meta = ArrayMetadata.new([D * 3], [D], "u1", Lz4(block))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        content = a.tobytes()
        check_lz4_frame(s, content, block)
        rst, dec = zref.decode(zref.LZ4, s, D, 1, False, False)
        assert rst == zref.OK and dec == content
        back = DefaultChunk.read_chunk(s, meta, [0], np.uint8).get_data()
        assert back.tobytes() == content
    if kind in ("zeros", "text", "ramp"):
        assert max(len(s) for s in outs) < D // 4  # it does compress


@pytest.mark.parametrize("nbytes", [1, 5, 12, 13, 14, 100, 4095, 65535, 65536, 65537, 65536 + 13,
                                    131072 + 100, 300001])
def test_lz4_encode_edge_sizes(nbytes):
    arrays = [_data("text", nbytes, 1), _data("uniform", nbytes, 2), _data("zeros", nbytes)]
    meta = ArrayMetadata.new([nbytes * 3], [nbytes], "u1", Lz4(65536))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        content = a.tobytes()
        check_lz4_frame(s, content, 65536)
        rst, dec = zref.decode(zref.LZ4, s, nbytes, 1, False, False)
        assert rst == zref.OK and dec == content


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", "<f8", ">u8", "bool", "i1"])
def test_lz4_encode_dtypes(dt):
    """write_data serialises in the array's byte order, bool as 0/1
    (chunk.rs:118-140,192-206); the GPU encoder applies that transform."""
    rng = np.random.default_rng(4)
    n = 200003
    if dt == "bool":
        data = rng.integers(0, 2, n).astype(bool)
    else:
        data = (np.cumsum(rng.integers(-3, 4, n)) % 100).astype(np.dtype(dt).newbyteorder("="))
    meta = ArrayMetadata.new([n], [n], dt, Lz4(65536))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0], data))
    content = serialised(data, dt)
    check_lz4_frame(out, content, 65536)
    rst, dec = zref.decode(zref.LZ4, out, len(content), 1, False, False)
    assert rst == zref.OK and dec == content
    back = DefaultChunk.read_chunk(out, meta, [0], data.dtype).get_data()
    assert np.array_equal(back, data)


def test_lz4_encode_errors():
    meta = ArrayMetadata.new([100], [50], "<i4", Lz4(65536))
    with pytest.raises(ZarrIOError) as e:  # chunk.rs:309-318
        DefaultChunk.write_chunk(meta, SliceDataChunk([0], np.arange(49, dtype=np.int32)))
    assert e.value.kind == "InvalidData"
    # a destination below zcg_encode_bound is refused per chunk
    D = 65536
    meta = ArrayMetadata.new([D], [D], "u1", Lz4(65536))
    st, _ = encode_batch(meta, [_data("uniform", D)], cap_extra=-64)
    assert st[0] == 5  # ZCG_ERR_OUTPUT_TOO_SMALL


# ---- gzip (gzip.rs:50-56 -> flate2 GzEncoder, zlib raw deflate) ----------------------
import zlib  # noqa: E402

from zarr_amd import Gzip  # noqa: E402


def zlib_raw(content: bytes, level: int) -> bytes:
    """flate2's deflate body: zlib raw deflate, windowBits -15, memLevel 8, default strategy."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(content) + c.flush()


def check_gzip_member(stream: bytes, content: bytes, level: int, exact=None):
    eff = 6 if (level < 0 or level > 9) else level
    xfl = 2 if eff >= 9 else (4 if eff <= 1 else 0)
    assert stream[:10] == bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, xfl, 255])
    crc, isize = struct.unpack_from("<II", stream, len(stream) - 8)
    assert crc == zlib.crc32(content) and isize == len(content) & 0xFFFFFFFF
    d = zlib.decompressobj(-15)
    assert d.decompress(stream[10:-8]) == content and d.eof and not d.unused_data
    if exact if exact is not None else eff >= 1:
        # levels 1-9: byte-identical to zlib (gzip.rs:54-56 -> flate2 -> zlib deflate_fast / deflate_slow)
        ref = zlib_raw(content, eff)
        body = stream[10:-8]
        if body != ref:
            k = next((i for i in range(min(len(body), len(ref))) if body[i] != ref[i]), min(len(body), len(ref)))
            raise AssertionError(f"gzip level {eff}: deflate body differs from zlib's at byte {k} "
                                 f"(len {len(body)} vs {len(ref)})")


def test_gzip_encode_doc_spec_exact():
    """tests.rs:147-159 + gzip.rs:66-80: byte-identical to the reference vector."""
    d = doc_spec()
    meta = ArrayMetadata.new([5, 6, 7], [1, 2, 3], ">i2", Gzip(-1))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0, 0, 0], np.array(d["expected_values"], np.int16)))
    assert out.hex() == d["encode_expected"]["gzip"]


@pytest.mark.parametrize("level", [0, 1, 4, 6, 9, -1])
@pytest.mark.parametrize("kind", ["zeros", "uniform", "randwalk", "text", "ramp", "mixed"])
def test_gzip_encode_roundtrip(kind, level):
    D = 1 << 20
    arrays = [_data(kind, D, seed=s) for s in range(2)]
    meta = ArrayMetadata.new([D * 2], [D], "u1", Gzip(level))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        content = a.tobytes()
        check_gzip_member(s, content, level)
        rst, dec = zref.decode(zref.GZIP, s, D, 1, False, False)
        assert rst == zref.OK and dec == content
        back = DefaultChunk.read_chunk(s, meta, [0], np.uint8).get_data()
        assert back.tobytes() == content
        if level != 0 and kind in ("zeros", "text", "ramp", "randwalk"):
            # compresses within a bounded factor of zlib at the same level
            ref_len = len(zlib.compress(content, 6 if level < 0 else level))
            bound = 2.5 if kind == "ramp" else 1.5  # ramp: exact 8 KiB period; zlib hash chains vs our 1-slot buckets
            assert len(s) <= bound * ref_len + 48 * (D // 16384), (len(s), ref_len)  # + per-block header/sync


@pytest.mark.parametrize("nbytes", [1, 2, 3, 4, 5, 100, 16383, 16384, 16385, 32768 + 5, 300001])
def test_gzip_encode_edge_sizes(nbytes):
    arrays = [_data("text", nbytes, 1), _data("uniform", nbytes, 2), _data("zeros", nbytes)]
    meta = ArrayMetadata.new([nbytes * 3], [nbytes], "u1", Gzip(6))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_gzip_member(s, a.tobytes(), 6)


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", "<f8", ">u8", "bool", "i1"])
def test_gzip_encode_dtypes(dt):
    rng = np.random.default_rng(5)
    n = 150001
    if dt == "bool":
        data = rng.integers(0, 2, n).astype(bool)
    else:
        data = (np.cumsum(rng.integers(-3, 4, n)) % 100).astype(np.dtype(dt).newbyteorder("="))
    meta = ArrayMetadata.new([n], [n], dt, Gzip(6))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0], data))
    content = serialised(data, dt)
    check_gzip_member(out, content, 6)
    back = DefaultChunk.read_chunk(out, meta, [0], data.dtype).get_data()
    assert np.array_equal(back, data)


def test_gzip_encode_quant_ratio():
    """C5 data ('quant' f32): report and bound the ratio against zlib-6."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import quant_chunk
    arrays = [quant_chunk(i).view(np.uint8) for i in range(4)]
    meta = ArrayMetadata.new([1 << 22], [1 << 20], "u1", Gzip(6))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    ours = sum(len(s) for s in outs)
    ref = sum(len(zlib.compress(a.tobytes(), 6)) for a in arrays)
    for a, s in zip(arrays, outs):
        check_gzip_member(s, a.tobytes(), 6)
    assert ours <= 1.4 * ref, (ours, ref)


@pytest.mark.parametrize("level", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_gzip_encode_matches_zlib_levels(level):
    """write_chunk bytes = flate2/zlib's at every level (1-3 deflate_fast, 4-9 deflate_slow), on a mixed
    batch: the five DATASETS kinds, the C5 'quant' f32 chunk, and sizes that
    end blocks / windows at their edges."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import quant_chunk
    D = 1 << 19
    arrays = [_data(k, D, seed=3) for k in ("zeros", "uniform", "randwalk", "text", "ramp", "mixed")]
    arrays.append(quant_chunk(7).view(np.uint8)[:D].copy())
    meta = ArrayMetadata.new([D * len(arrays)], [D], "u1", Gzip(level))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_gzip_member(s, a.tobytes(), level, exact=True)


@pytest.mark.parametrize("level", [1, 6])
@pytest.mark.parametrize("nbytes", [1, 2, 3, 258, 259, 16383, 32506, 32768, 65274, 65275, 65536, 98304 + 7])
def test_gzip_encode_matches_zlib_edges(nbytes, level):
    """Window-slide and block-flush edges: zlib's bytes exactly (deflate_fast
    at level 1, deflate_slow at level 6)."""
    arrays = [_data("text", nbytes, 4), _data("uniform", nbytes, 5), _data("zeros", nbytes), _data("ramp", nbytes)]
    meta = ArrayMetadata.new([nbytes * 4], [nbytes], "u1", Gzip(level))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_gzip_member(s, a.tobytes(), level, exact=True)


# ---- Xz (xz.rs:34-43: xz2 XzEncoder = lzma_easy_encoder(preset, CRC64)) ----
def check_xz_stream(stream: bytes, content: bytes, preset: int):
    """xz2's container conventions + liblzma (Python lzma = the reference's
    decoder library) reproduces the content with every check verified."""
    import lzma
    assert stream[:12] == bytes.fromhex("fd377a585a000004e6d6b446")  # CRC64 stream
    assert stream[-2:] == b"YZ" and stream[-4:-2] == b"\x00\x04"
    if content:
        lg = [18, 20, 21, 22, 22, 23, 23, 24, 25, 26][6 if preset < 0 or preset > 9 else preset]
        assert stream[12:20] == bytes([0x02, 0x00, 0x21, 0x01, 2 * (lg - 12), 0, 0, 0])
    d = lzma.LZMADecompressor(format=lzma.FORMAT_XZ)
    assert d.decompress(stream) == content and d.eof and not d.unused_data


@pytest.mark.parametrize("preset", [0, 6, 9])
@pytest.mark.parametrize("kind", ["zeros", "uniform", "randwalk", "text", "ramp", "mixed"])
def test_xz_encode_roundtrip(kind, preset):
    from zarr_amd.compression import Xz
    D = 1 << 20
    arrays = [_data(kind, D, seed=s) for s in range(2)]
    meta = ArrayMetadata.new([D * 2], [D], "u1", Xz(preset))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        content = a.tobytes()
        check_xz_stream(s, content, preset)
        rst, dec = zref.decode(zref.XZ, s, D, 1, False, False)
        assert rst == zref.OK and dec == content
        back = DefaultChunk.read_chunk(s, meta, [0], np.uint8).get_data()
        assert back.tobytes() == content


@pytest.mark.parametrize("nbytes", [1, 2, 3, 5, 100, 65536, 65537, 300001])
def test_xz_encode_edge_sizes(nbytes):
    from zarr_amd.compression import Xz
    arrays = [_data("text", nbytes, 1), _data("uniform", nbytes, 2), _data("zeros", nbytes)]
    meta = ArrayMetadata.new([nbytes * 3], [nbytes], "u1", Xz(6))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_xz_stream(s, a.tobytes(), 6)


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", ">u8", "bool", "i1"])
def test_xz_encode_dtypes(dt):
    from zarr_amd.compression import Xz
    rng = np.random.default_rng(6)
    n = 150001
    if dt == "bool":
        data = rng.integers(0, 2, n).astype(bool)
    else:
        data = (np.cumsum(rng.integers(-3, 4, n)) % 100).astype(np.dtype(dt).newbyteorder("="))
    meta = ArrayMetadata.new([n], [n], dt, Xz(6))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0], data))
    check_xz_stream(out, serialised(data, dt), 6)
    back = DefaultChunk.read_chunk(out, meta, [0], data.dtype).get_data()
    assert np.array_equal(back, data)


def test_xz_encode_doc_spec_exact():
    """tests.rs:147-159 + xz.rs:52-75,84-90: byte-identical to the reference
    vector (one LZMA2 uncompressed chunk `01 00 0b` + the 12 bytes)."""
    from zarr_amd.compression import Xz
    d = doc_spec()
    meta = ArrayMetadata.new([5, 6, 7], [1, 2, 3], ">i2", Xz(6))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0, 0, 0], np.array(d["expected_values"], np.int16)))
    assert out.hex() == d["encode_expected"]["xz"]
    st, dec = zref.decode(zref.XZ, out, 12, 2, True)
    assert st == zref.OK and np.frombuffer(dec, "<i2").tolist() == d["expected_values"]


@pytest.mark.parametrize("nbytes", [1, 7, 12, 40, 1000])
def test_xz_encode_small_matches_liblzma(nbytes):
    """Inputs too small to compress: liblzma emits one uncompressed LZMA2
    chunk, so the whole .xz stream is determined; the GPU stream must be the
    same bytes (lzma_easy_encoder(6, CRC64) = Python lzma preset 6)."""
    import lzma
    from zarr_amd.compression import Xz
    rng = np.random.default_rng(nbytes)
    a = rng.integers(0, 256, nbytes, dtype=np.uint8)
    meta = ArrayMetadata.new([nbytes], [nbytes], "u1", Xz(6))
    st, outs = encode_batch(meta, [a])
    assert st[0] == 0
    ref = lzma.compress(a.tobytes(), format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6)
    assert outs[0].hex() == ref.hex()


def test_xz_encode_incompressible_no_expansion():
    """Uniform bytes: every LZMA2 chunk falls back to an uncompressed one, as
    liblzma's do, so the stream is no longer than liblzma's (plus chunk-header
    slack), and mixed data (compressible / incompressible 64 KiB runs) round
    trips through uncompressed chunks followed by state-reset LZMA chunks."""
    import lzma
    from zarr_amd.compression import Xz
    D = 1 << 20
    arrays = [_data("uniform", D, 11), _data("mixed", D, 12)]
    meta = ArrayMetadata.new([2 * D], [D], "u1", Xz(6))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_xz_stream(s, a.tobytes(), 6)
    ref = lzma.compress(arrays[0].tobytes(), format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6)
    assert len(outs[0]) <= len(ref) + 64, (len(outs[0]), len(ref))
    assert len(outs[0]) < D + D // 1000


@pytest.mark.parametrize("preset", [4, 6, 9])
@pytest.mark.parametrize("kind", ["text", "randwalk", "mixed", "zeros", "uniform", "quant"])
def test_xz_opt_matches_restatement(kind, preset):
    """Presets 4-9 (liblzma's optimal-parse presets) take the optimal-parse
    coder: its streams equal the serial restatement's byte for byte
    (tests/hostcore/xz_opt_ref.cpp) across 256 KiB segments, LZMA2 chunk
    limits and stored chunks, and decode with liblzma."""
    from test_hostcore import xz_opt_ref
    from zarr_amd.compression import Xz
    if kind == "quant":
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import quant_chunk
        arrays = [quant_chunk(i).view(np.uint8) for i in range(2)]
    else:
        arrays = [_data(kind, 600001, seed=s) for s in range(2)]
    D = arrays[0].nbytes
    meta = ArrayMetadata.new([D * 2], [D], "u1", Xz(preset))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    lg = [18, 20, 21, 22, 22, 23, 23, 24, 25, 26][preset]
    for a, s in zip(arrays, outs):
        ref = xz_opt_ref(a.tobytes(), lg)
        if s != ref:
            k = next((i for i in range(min(len(s), len(ref))) if s[i] != ref[i]), min(len(s), len(ref)))
            raise AssertionError(f"xz stream differs from the restatement at byte {k} (len {len(s)} vs {len(ref)})")
        check_xz_stream(s, a.tobytes(), preset)


def test_xz_encode_quant_ratio():
    """C2 "quant" chunks at preset 6: >= 97 % of liblzma preset 6's ratio
    (>= 6.66 against liblzma's 6.87)."""
    import lzma
    import sys
    from zarr_amd.compression import Xz
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import quant_chunk
    arrays = [quant_chunk(i) for i in range(4)]
    meta = ArrayMetadata.new([256 * 4, 256, 4], [256, 256, 4], "<f4", Xz(6))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    tot = sum(a.nbytes for a in arrays)
    ours = sum(len(s) for s in outs)
    ref = sum(len(lzma.compress(a.tobytes(), format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6))
              for a in arrays)
    for a, s in zip(arrays, outs):
        check_xz_stream(s, a.tobytes(), 6)
    assert tot / ours >= 6.66 and tot / ours >= 0.97 * tot / ref, (tot / ours, tot / ref)


# ---- Bzip2 (bzip.rs:36-45: bzip2-rs BzEncoder = libbz2 BZ2_bzCompressInit(block_size)) ----
def check_bz2_stream(stream: bytes, content: bytes, level: int):
    """A single bzip2 stream for this level that libbz2 (Python bz2 = the
    reference decoder's library) decodes to the content, every block and the
    stream CRC verified, every block within the level's 100 000*L limit."""
    import bz2
    assert stream[:4] == b"BZh" + bytes([0x30 + level])
    d = bz2.BZ2Decompressor()
    assert d.decompress(stream) == content and d.eof and not d.unused_data


@pytest.mark.parametrize("level", [1, 9])
@pytest.mark.parametrize("kind", ["zeros", "uniform", "randwalk", "text", "ramp", "mixed"])
def test_bzip2_encode_roundtrip(kind, level):
    from zarr_amd.compression import Bzip2
    D = 1 << 20
    arrays = [_data(kind, D, seed=s) for s in range(2)]
    meta = ArrayMetadata.new([D * 2], [D], "u1", Bzip2(level))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        content = a.tobytes()
        check_bz2_stream(s, content, level)
        rst, dec = zref.decode(zref.BZIP2, s, D, 1, False, False)
        assert rst == zref.OK and dec == content
        back = DefaultChunk.read_chunk(s, meta, [0], np.uint8).get_data()
        assert back.tobytes() == content


def test_bzip2_encode_many_blocks():
    """More than 256 blocks in one sort sub-batch (level 1: ~11 blocks per
    1 MiB chunk, 28 chunks): the first rotation sort keys then hold 2 prefix
    bytes under 9+ block-index bits instead of 3 (zcg_bz2_enc.hip
    bze_init_keys)."""
    from zarr_amd.compression import Bzip2
    D = 1 << 20
    kinds = ["randwalk", "text", "mixed", "uniform"]
    arrays = [_data(kinds[i % 4], D, seed=i) for i in range(28)]
    meta = ArrayMetadata.new([D * 28], [D], "u1", Bzip2(1))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_bz2_stream(s, a.tobytes(), 1)


@pytest.mark.parametrize("nbytes", [1, 2, 3, 4, 5, 6, 255, 256, 259, 1000, 99981, 100000, 300001])
def test_bzip2_encode_edge_sizes(nbytes):
    from zarr_amd.compression import Bzip2
    arrays = [_data("text", nbytes, 1), _data("uniform", nbytes, 2), _data("zeros", nbytes),
              np.full(nbytes, 0xFB, np.uint8)]
    meta = ArrayMetadata.new([nbytes * 4], [nbytes], "u1", Bzip2(1))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    for a, s in zip(arrays, outs):
        check_bz2_stream(s, a.tobytes(), 1)


def test_bzip2_encode_runs():
    """RLE1 pieces of every length around 4 and 255 (libbz2 ADD_CHAR_TO_BLOCK),
    runs that straddle the level-1 block limit."""
    from zarr_amd.compression import Bzip2
    rng = np.random.default_rng(3)
    parts = []
    for ln in list(range(1, 12)) + [250, 251, 252, 253, 254, 255, 256, 257, 258, 259, 260, 509, 510, 511, 5000]:
        parts.append(np.full(ln, rng.integers(0, 256), np.uint8))
    base = np.concatenate(parts)
    a = np.resize(base, 400000)
    b = np.concatenate([np.full(99978, 1, np.uint8), np.full(300, 2, np.uint8), np.arange(100, dtype=np.uint8)])
    b = np.resize(b, 400000)
    meta = ArrayMetadata.new([800000], [400000], "u1", Bzip2(1))
    st, outs = encode_batch(meta, [a, b])
    assert (st == 0).all()
    for x, s in zip([a, b], outs):
        check_bz2_stream(s, x.tobytes(), 1)


def test_bzip2_encode_empty():
    from zarr_amd.compression import Bzip2
    meta = ArrayMetadata.new([0], [0], "u1", Bzip2(9))
    st, outs = encode_batch(meta, [np.zeros(0, np.uint8)] * 2)
    assert (st == 0).all()
    import bz2
    for s in outs:
        assert s == bz2.compress(b"", 9)  # "BZh9" + end-of-stream record, CRC 0


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", ">u8", "bool", "i1"])
def test_bzip2_encode_dtypes(dt):
    from zarr_amd.compression import Bzip2
    rng = np.random.default_rng(6)
    n = 150001
    if dt == "bool":
        data = rng.integers(0, 2, n).astype(bool)
    else:
        data = (np.cumsum(rng.integers(-3, 4, n)) % 100).astype(np.dtype(dt).newbyteorder("="))
    meta = ArrayMetadata.new([n], [n], dt, Bzip2(9))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0], data))
    check_bz2_stream(out, serialised(data, dt), 9)
    back = DefaultChunk.read_chunk(out, meta, [0], data.dtype).get_data()
    assert np.array_equal(back, data)


def test_bzip2_encode_doc_spec_decodes():
    """bzip.rs:83-84: the reference's own doc-spec bzip2 encode vector is not
    libbz2's output either, so the GPU stream must decode to the doc-spec
    values through the reference decoder library."""
    from zarr_amd.compression import Bzip2
    d = doc_spec()
    meta = ArrayMetadata.new([5, 6, 7], [1, 2, 3], ">i2", Bzip2(9))
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0, 0, 0], np.array(d["expected_values"], np.int16)))
    st, dec = zref.decode(zref.BZIP2, out, 12, 2, True)
    assert st == zref.OK and np.frombuffer(dec, "<i2").tolist() == d["expected_values"]


def test_bzip2_encode_quant_ratio():
    """C2-shaped f32 chunks: same Huffman machinery as libbz2, so the ratio
    must be close to libbz2 level 9's on the same data."""
    import bz2
    from test_gpu_parity import quant_f32
    from zarr_amd.compression import Bzip2
    arrays = [quant_f32(s) for s in range(4)]
    D = arrays[0].nbytes
    meta = ArrayMetadata.new([256 * 4, 256, 4], [256, 256, 4], "<f4", Bzip2(9))
    st, outs = encode_batch(meta, arrays)
    assert (st == 0).all()
    ours = sum(len(s) for s in outs)
    ref = sum(len(bz2.compress(a.tobytes(), 9)) for a in arrays)
    for a, s in zip(arrays, outs):
        check_bz2_stream(s, a.tobytes(), 9)
    assert ours <= ref * 1.05, (ours, ref)


def test_bzip2_encode_bad_level():
    from zarr_amd.compression import Bzip2
    meta = ArrayMetadata.new([100], [100], "u1", Bzip2(0))
    with pytest.raises(ZarrIOError) as e:
        DefaultChunk.write_chunk(meta, SliceDataChunk([0], np.zeros(100, np.uint8)))
    assert e.value.kind == "InvalidInput"


# ---- descriptor edge cases and the encoders' internal sub-batch splits ----------
def _codec(name, level=None):
    from zarr_amd.compression import Bzip2, Raw, Xz
    return {"raw": lambda: Raw(), "gzip": lambda: Gzip(6), "lz4": lambda: Lz4(65536),
            "xz": lambda: Xz(6), "bzip2": lambda: Bzip2(9)}[name]()


@pytest.mark.parametrize("codec", ["raw", "gzip", "lz4", "xz", "bzip2"])
def test_encode_short_src_is_invalid_data(codec):
    """A chunk whose src holds fewer than N*size bytes is write_chunk's
    element-count error (chunk.rs:309-318): INVALID_DATA for that chunk only,
    no out-of-bounds read, and the other chunks of the batch still encode."""
    import torch
    from zarr_amd.batch import BatchCodec, make_encode_batch
    D = 200000
    arrays = [_data("text", D, 1), _data("randwalk", D, 2), _data("uniform", D, 3)]
    meta = ArrayMetadata.new([3 * D], [D], "u1", _codec(codec))
    bc = BatchCodec(0)
    elems = torch.from_numpy(np.concatenate(arrays)).to("cuda:0")
    cap = bc.encode_bound(meta, D)
    desc, dst, out_len, status = make_encode_batch(elems, 3, cap, "cuda:0")
    d = desc.cpu().numpy().view(np.uint64).reshape(3, 4).copy()
    d[1, 1] = 3  # src_len < D (shorter than one match-finder key)
    desc = torch.from_numpy(d.view(np.int64)).to("cuda:0")
    bc.encode(meta, desc, 3, out_len, status)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert st.tolist() == [0, 2, 0]
    ol = out_len.cpu().numpy()
    buf = dst.cpu().numpy().reshape(3, cap)
    cid = {"raw": zref.RAW, "gzip": zref.GZIP, "lz4": zref.LZ4, "xz": zref.XZ, "bzip2": zref.BZIP2}[codec]
    for i in (0, 2):
        rst, dec = zref.decode(cid, buf[i, :ol[i]].tobytes(), D, 1, False, False)
        assert rst == zref.OK and dec == arrays[i].tobytes()


@pytest.mark.parametrize("codec", ["lz4", "gzip", "xz"])
def test_encode_sub_batch_splits_roundtrip(codec):
    """1 100 distinct 1 MiB chunks: more than one 128 MiB match-finder
    sub-batch and more than one 1 GiB coder launch (the m / sm splits of
    lz_layout / df_layout / xe_layout).  Every stream must decode with the
    reference libraries to its own chunk."""
    import torch
    from zarr_amd.batch import BatchCodec, make_encode_batch
    D, n = 1 << 20, 1100
    rng = np.random.default_rng(21)
    base = np.cumsum(rng.integers(-3, 4, (64 << 20) // 2 + D)).astype("<i2").view(np.uint8)
    offs = [(i * 40009) & ~1 for i in range(n)]  # distinct, overlapping windows of one walk
    meta = ArrayMetadata.new([n * D], [D], "u1", _codec(codec))
    bc = BatchCodec(0)
    elems = torch.empty(n * D, dtype=torch.uint8, device="cuda:0")
    for i, o in enumerate(offs):
        elems[i * D:(i + 1) * D].copy_(torch.from_numpy(base[o:o + D]))
    cap = bc.encode_bound(meta, D)
    desc, dst, out_len, status = make_encode_batch(elems, n, cap, "cuda:0")
    bc.encode(meta, desc, n, out_len, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    ol = out_len.cpu().numpy()
    del elems
    host = dst.view(n, cap).cpu().numpy()
    del dst
    cid = {"gzip": zref.GZIP, "lz4": zref.LZ4, "xz": zref.XZ}[codec]
    srcs = [np.ascontiguousarray(host[i, :ol[i]]) for i in range(n)]
    st, outs = zref.decode_batch(cid, srcs, D, threads=16)
    assert (st == 0).all()
    bad = [i for i in range(n) if not np.array_equal(outs[i], base[offs[i]:offs[i] + D])]
    assert not bad, bad[:10]


def test_lz4_encode_block_count_limit():
    """More than 4096 LZ4 blocks per chunk is refused up front with
    ZCG_ERR_UNSUPPORTED and a message; nothing is launched (the chunk table
    below points at 1-byte buffers and is never read)."""
    import ctypes
    import torch
    from zarr_amd import _native
    from zarr_amd.chunk import abi_array
    ctx = _native.context(0)
    meta = ArrayMetadata.new([(4097 << 16)], [(4097 << 16)], "u1", Lz4(65536))
    dummy = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    st = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    ol = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    arr = abi_array(meta)
    r = ctx.lib.zcg_encode_batch(ctx.handle, ctypes.byref(arr), ctypes.c_void_p(dummy.data_ptr()), 1,
                                 ctypes.c_void_p(ol.data_ptr()), ctypes.c_void_p(st.data_ptr()), None)
    assert r == _native.UNSUPPORTED and "4096" in ctx.last_error()


@pytest.mark.gpu
def test_gzip_encode_huge_chunk_is_per_chunk_unsupported():
    """A gzip chunk of >= 2 GiB (the zlib-exact coder's u32 positions) is
    refused per chunk: the launch succeeds, every chunk's status is
    ZCG_ERR_UNSUPPORTED and its length 0 (before round 6 the
    whole batch failed with an invalid-value launch error).  The chunk table
    points at a zeroed dummy and is never read."""
    import ctypes
    import torch
    from zarr_amd import _native
    from zarr_amd.chunk import abi_array
    ctx = _native.context(0)
    D = 1 << 31
    meta = ArrayMetadata.new([D], [D], "u1", Gzip(6))
    dummy = torch.zeros(128, dtype=torch.uint8, device="cuda:0")
    st = torch.full((2,), 77, dtype=torch.int32, device="cuda:0")
    ol = torch.full((2,), 5, dtype=torch.int64, device="cuda:0")
    arr = abi_array(meta)
    r = ctx.lib.zcg_encode_batch(ctx.handle, ctypes.byref(arr), ctypes.c_void_p(dummy.data_ptr()), 2,
                                 ctypes.c_void_p(ol.data_ptr()), ctypes.c_void_p(st.data_ptr()), None)
    torch.cuda.synchronize()
    assert r == _native.OK, ctx.last_error()
    assert st.cpu().tolist() == [_native.UNSUPPORTED] * 2
    assert ol.cpu().tolist() == [0, 0]
