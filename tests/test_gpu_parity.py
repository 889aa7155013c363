"""GPU parity: the HIP path (through the C ABI) vs the oracle, bit-exact.

Mirrors the reference's tests (src/tests.rs:132-219, tests/zarrita_compat.rs,
tests/integration_test.rs) plus stream variants the reference decoder
accepts.  Every expected output comes from the oracle (oracle/zref.c over the
reference's own C codec libraries) or from the committed golden fixtures.
"""
import os
import struct
import zlib

import numpy as np
import pytest

import zref
from golden_util import (CODEC_IDS, DEFAULT_PARAM, doc_spec, dtype_info, reencoded,
                         zarrita_chunks, zarrita_meta_json)
from zarr_amd import (ArrayMetadata, DefaultChunk, Gzip, Lz4, NativeUnavailable, Raw, SliceDataChunk,
                      ZarrIOError, read_chunks_host)
from zarr_amd.compression import Bzip2, Xz

pytestmark = pytest.mark.gpu

GPU_DECODE = ["raw", "gzip", "lz4", "xz", "bzip2"]
COMP = {"raw": lambda p: Raw(), "gzip": lambda p: Gzip(p), "lz4": lambda p: Lz4(p),
        "bzip2": lambda p: Bzip2(p), "xz": lambda p: Xz(p)}
NPT = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def meta_for(codec, dt, n, param=None):
    p = DEFAULT_PARAM[codec] if param is None else param
    return ArrayMetadata.new([n], [n], dt, COMP[codec](p))


def gpu_decode(codec, stream, dt, n, param=None, flags=0):
    """read_chunk on the GPU; returns (kind or 'Ok', host-native bytes)."""
    es, be, isb, npdt = dtype_info(dt)
    meta = meta_for(codec, dt, n, param)
    try:
        ch = DefaultChunk.read_chunk(stream, meta, [0], npdt, flags=flags)
    except ZarrIOError as e:
        return e.kind, b""
    return "Ok", ch.get_data().tobytes()


# a one-chunk gzip read runs the 256-lane kernel by default (small batch);
# every gzip check also forces the one-wave-per-chunk kernel (the C2 kernel)
FLAG_INFLATE_WAVE = 0x4000


KIND = {zref.OK: "Ok", zref.EOF: "UnexpectedEof", zref.INVALID_DATA: "InvalidData"}


def check(codec, stream, dt, n, param=None):
    es, be, isb, _ = dtype_info(dt)
    st, ref = zref.decode(CODEC_IDS[codec], stream, n * es, es, be, isb)
    for flags in ((0, FLAG_INFLATE_WAVE) if codec == "gzip" else (0,)):
        kind, out = gpu_decode(codec, stream, dt, n, param, flags)
        assert kind == KIND[st], (kind, st, flags)
        if st == zref.OK:
            assert out == ref, flags


def test_native_library_is_loaded():
    from zarr_amd import _native
    _native.context(0)
    maps = open("/proc/self/maps").read()
    assert "libzchunk_gpu.so" in maps
    hips = {l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}
    assert len(hips) == 1, hips  # one HIP runtime in the process


# ---- reference golden vectors ---------------------------------------------------
@pytest.mark.parametrize("codec", GPU_DECODE)
def test_read_doc_spec_chunk(codec):
    """tests.rs:132-145 on the GPU."""
    d = doc_spec()
    meta = ArrayMetadata.new([5, 6, 7], [1, 2, 3], ">i2", COMP[codec](DEFAULT_PARAM[codec]))
    ch = DefaultChunk.read_chunk(bytes.fromhex(d["chunks"][codec]["hex"]), meta, [0, 0, 0], np.int16)
    assert ch.get_grid_position() == [0, 0, 0]
    assert ch.get_data().tolist() == d["expected_values"]


def test_write_doc_spec_chunk_raw():
    d = doc_spec()
    meta = ArrayMetadata.new([5, 6, 7], [1, 2, 3], ">i2", Raw())
    out = DefaultChunk.write_chunk(meta, SliceDataChunk([0, 0, 0], np.array(d["expected_values"], np.int16)))
    assert out.hex() == d["encode_expected"]["raw"]


def test_zarrita_golden_replay():
    """zarrita_compat.rs:30-46: all 8 chunks, batched and one at a time."""
    meta = ArrayMetadata.from_json(zarrita_meta_json())
    chunks = zarrita_chunks()
    for g, stream, expected in chunks:
        for flags in (0, FLAG_INFLATE_WAVE):
            ch = DefaultChunk.read_chunk(stream, meta, list(g), np.int16, flags=flags)
            assert np.array_equal(ch.get_data(), expected), (g, flags)
    status, outs = read_chunks_host(meta, [c[1] for c in chunks], np.int16)
    assert (status == 0).all()
    for (g, _, expected), o in zip(chunks, outs):
        assert np.array_equal(o, expected)


@pytest.mark.parametrize("codec", GPU_DECODE)
def test_reencoded_fixtures(codec):
    """All 21 dtype/endianness variants: transform (swap / bool) parity."""
    for e in reencoded():
        if e["codec"] != codec:
            continue
        es, be, isb, npdt = dtype_info(e["dtype"])
        kind, out = gpu_decode(codec, bytes.fromhex(e["stream"]), e["dtype"], e["num_elements"])
        assert kind == "Ok", e["dtype"]
        assert out.hex() == e["decoded"], e["dtype"]


@pytest.mark.parametrize("codec", GPU_DECODE)
def test_chunk_compression_rw_decode(codec):
    """tests.rs:161-189 (decode half; encode by the oracle)."""
    data = np.arange(125, dtype="<i4")
    st, enc = zref.encode(CODEC_IDS[codec], DEFAULT_PARAM[codec], data)
    meta = ArrayMetadata.new([10, 10, 10], [5, 5, 5], "<i4", COMP[codec](DEFAULT_PARAM[codec]))
    assert DefaultChunk.read_chunk(enc, meta, [0, 0, 0], np.int32).get_data().tolist() == list(range(125))


@pytest.mark.parametrize("codec", GPU_DECODE)
def test_varlength_chunk_rw(codec):
    """tests.rs:191-219: short streams -> UnexpectedEof; short writes -> InvalidData."""
    meta = ArrayMetadata.new([10, 10, 10], [5, 5, 5], "<i4", COMP[codec](DEFAULT_PARAM[codec]))
    st, enc = zref.encode(CODEC_IDS[codec], DEFAULT_PARAM[codec], np.arange(100, dtype="<i4"))
    with pytest.raises(ZarrIOError) as e:
        DefaultChunk.read_chunk(enc, meta, [0, 0, 0], np.int32)
    assert e.value.kind == "UnexpectedEof"
    with pytest.raises(ZarrIOError) as e:
        DefaultChunk.read_chunk(b"", meta, [0, 0, 0], np.int32)
    assert e.value.kind == "UnexpectedEof"
    if codec == "raw":
        with pytest.raises(ZarrIOError) as e:
            DefaultChunk.write_chunk(meta, SliceDataChunk([0, 0, 0], np.arange(100, dtype=np.int32)))
        assert e.value.kind == "InvalidData"


def test_unsupported_codecs_fail_loudly():
    """No CPU fallback in the product path: a codec without a GPU kernel raises."""
    from zarr_amd import _native
    L = _native.load_library()
    for codec in ("bzip2", "xz"):
        if L.zcg_codec_on_gpu(CODEC_IDS[codec], 0):
            continue
        st, enc = zref.encode(CODEC_IDS[codec], DEFAULT_PARAM[codec], np.arange(10, dtype="<i2"))
        meta = ArrayMetadata.new([10], [10], "<i2", COMP[codec](DEFAULT_PARAM[codec]))
        with pytest.raises(NativeUnavailable):
            DefaultChunk.read_chunk(enc, meta, [0], np.int16)


# ---- larger streams: every deflate/LZ4 structure the reference decoder accepts --
def rw(n, seed=0):
    return np.cumsum(np.random.default_rng(seed).integers(-3, 4, n)).astype("<i2")


def quant_f32(seed=0):
    i = np.arange(256)[:, None, None]
    j = np.arange(256)[None, :, None]
    k = np.arange(4)[None, None, :]
    phi = seed * 7
    v = np.round(64 * (100 * np.sin(0.05 * (i + phi)) * np.cos(0.03 * j) + k)) / 64
    return v.astype("<f4").reshape(-1)


def gzip_wrap(raw_deflate: bytes, payload: bytes, flags=0, extra=b"", name=b"", comment=b"",
              hcrc=False):
    h = bytearray([0x1f, 0x8b, 8, flags | (2 if hcrc else 0), 0, 0, 0, 0, 0, 255])
    if flags & 4:
        h += struct.pack("<H", len(extra)) + extra
    if flags & 8:
        h += name + b"\0"
    if flags & 16:
        h += comment + b"\0"
    if hcrc:
        h += struct.pack("<H", zlib.crc32(bytes(h)) & 0xFFFF)
    tr = struct.pack("<II", zlib.crc32(payload), len(payload) & 0xFFFFFFFF)
    return bytes(h) + raw_deflate + tr


def deflate(payload, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8, wbits=-15):
    c = zlib.compressobj(level, zlib.DEFLATED, wbits, mem, strategy)
    return c.compress(payload) + c.flush()


DATASETS = {
    "randwalk_i2": lambda: rw(524288).tobytes(),
    "quant_f4": lambda: quant_f32(3).tobytes(),
    "uniform_u1": lambda: np.random.default_rng(5).integers(0, 256, 1 << 20, dtype=np.uint8).tobytes(),
    "zeros": lambda: bytes(1 << 20),
    "text_like": lambda: (b"the quick brown fox jumps over the lazy dog %d\n" * 30000)[: 1 << 20],
}


@pytest.mark.parametrize("data", list(DATASETS))
@pytest.mark.parametrize("variant", ["l1", "l6", "l9", "l0_stored", "huffman_only", "rle",
                                     "fixed", "flags_hdr"])
def test_gzip_large(data, variant):
    payload = DATASETS[data]()
    if variant == "l1":
        s = gzip_wrap(deflate(payload, 1), payload)
    elif variant == "l6":
        st, s = zref.encode(zref.GZIP, 6, np.frombuffer(payload, np.uint8))
    elif variant == "l9":
        s = gzip_wrap(deflate(payload, 9), payload)
    elif variant == "l0_stored":
        s = gzip_wrap(deflate(payload, 0), payload)
    elif variant == "huffman_only":
        s = gzip_wrap(deflate(payload, 6, zlib.Z_HUFFMAN_ONLY), payload)
    elif variant == "rle":
        s = gzip_wrap(deflate(payload, 6, zlib.Z_RLE), payload)
    elif variant == "fixed":
        s = gzip_wrap(deflate(payload[:200000], 6, zlib.Z_FIXED), payload[:200000])
        payload = payload[:200000]
    else:
        s = gzip_wrap(deflate(payload, 6), payload, flags=4 | 8 | 16, extra=b"xy" * 5,
                      name=b"chunk.bin", comment=b"hello", hcrc=True)
    check("gzip", s, "u1", len(payload))


@pytest.mark.parametrize("data", ["zeros", "text_like", "quant_f4", "randwalk_i2"])
def test_inflate_wave_near_batches(data):
    """The wave kernel resolves near bytes in batches of 64 whose markers are
    cleared per batch (no tag that could wrap): long near runs
    (zeros: 258-byte dist-1 matches), short-period repeats (text) and the C2
    data decode to the input."""
    payload = DATASETS[data]()
    st, s = zref.encode(zref.GZIP, 6, np.frombuffer(payload, np.uint8))
    assert st == 0
    assert gpu_decode("gzip", s, "u1", len(payload), flags=FLAG_INFLATE_WAVE) == ("Ok", payload)


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", ">u8", "bool"])
def test_gzip_transform_large(dt):
    es, be, isb, npdt = dtype_info(dt)
    n = 262144 // es
    raw = np.random.default_rng(9).integers(0, 4, n * es, dtype=np.uint8)
    st, s = zref.encode(zref.GZIP, 6, raw, elem_size=1)
    check("gzip", s, dt, n)


def test_gzip_errors():
    payload = rw(100000).tobytes()
    s = bytearray(gzip_wrap(deflate(payload, 6), payload))
    check("gzip", bytes(s[: len(s) // 2]), "u1", len(payload))  # truncated -> EOF
    check("gzip", bytes(s[:5]), "u1", len(payload))
    bad = bytearray(s)
    bad[0] = 0x1e
    check("gzip", bytes(bad), "u1", len(payload))  # bad magic
    bad = bytearray(s)
    bad[10] |= 0x06  # BTYPE = 3 (reserved)
    check("gzip", bytes(bad), "u1", len(payload))
    for i in range(20):  # random corruption: classification must match the oracle
        bad = bytearray(s)
        pos = 12 + (i * 7919) % (len(s) - 30)
        bad[pos] ^= 0x5A
        check("gzip", bytes(bad), "u1", len(payload))
    check("gzip", bytes(s), "u1", len(payload) + 10)  # stream shorter than N -> EOF


LZ4_VARIANTS = {
    "reference": {},
    "linked": dict(linked=True),
    "block_checksum": dict(block_checksum=True),
    "content_size": dict(content_size=True),
    "bd256k": dict(block_size_id=5),
    "bd4m": dict(block_size_id=7),
    "small_blocks": dict(auto_flush=True, feed=10000),
    "no_content_checksum": dict(content_checksum=False),
}


@pytest.mark.parametrize("data", list(DATASETS))
@pytest.mark.parametrize("variant", list(LZ4_VARIANTS))
def test_lz4_large(data, variant):
    payload = DATASETS[data]()
    if variant == "reference":
        st, s = zref.encode(zref.LZ4, 65536, np.frombuffer(payload, np.uint8))
    else:
        s = zref.lz4_frame_custom(payload, **LZ4_VARIANTS[variant])
    check("lz4", s, "u1", len(payload))
    check("lz4", s, "u1", len(payload) - 1000)  # truncating read_exact
    check("lz4", s, "<i2", len(payload) // 2)


def test_lz4_skip_block_checksum_flag():
    """ZCG_FLAG_SKIP_LZ4_BLOCK_CHECKSUM: a frame with block checksums whose
    checksum words are corrupt is InvalidData by default (LZ4F verifies them,
    as the oracle does) and decodes to the intact payload with the flag, on
    both block decoders."""
    import torch
    from zarr_amd._native import FLAG_SKIP_LZ4_BLOCK_CHECKSUM
    from zarr_amd.batch import BatchCodec, PackedStreams
    payload = rw(300000).tobytes()
    s = zref.lz4_frame_custom(payload, block_checksum=True)
    # walk the blocks (7-byte header: magic, FLG, BD, HC) and corrupt every checksum word
    bad = bytearray(s)
    pos, nblk = 7, 0
    while True:
        bs = struct.unpack_from("<I", bad, pos)[0]
        if bs == 0:
            break
        n = bs & 0x7FFFFFFF
        bad[pos + 4 + n] ^= 0x5A
        pos += 4 + n + 4
        nblk += 1
    assert nblk >= 4
    st_ref, _ = zref.decode_batch(zref.LZ4, [np.frombuffer(bytes(bad), np.uint8)], len(payload))
    assert st_ref[0] == zref.INVALID_DATA
    for lz4_sel in (0, 0x800, 0x1000):
        for flags, want in ((0, zref.INVALID_DATA), (FLAG_SKIP_LZ4_BLOCK_CHECKSUM, zref.OK)):
            packed = PackedStreams([bytes(bad)] * 3, len(payload), "cuda:0")
            BatchCodec(0).decode(meta_for("lz4", "u1", len(payload)), packed, flags=flags | lz4_sel)
            torch.cuda.synchronize()
            st = packed.status.cpu().numpy()
            assert (st == want).all(), (lz4_sel, flags, st)
            if want == zref.OK:
                out = packed.dst.cpu().numpy().reshape(3, len(payload))
                assert all(out[i].tobytes() == payload for i in range(3))


def test_lz4_errors():
    payload = rw(300000).tobytes()
    st, s = zref.encode(zref.LZ4, 65536, np.frombuffer(payload, np.uint8))
    check("lz4", s[: len(s) // 2], "u1", len(payload))
    check("lz4", s[:6], "u1", len(payload))
    check("lz4", s, "u1", len(payload) + 2)
    for i in range(20):
        bad = bytearray(s)
        pos = 11 + (i * 7919) % (len(s) - 20)
        bad[pos] ^= 0x5A
        check("lz4", bytes(bad), "u1", len(payload))
    bad = bytearray(s)
    bad[6] ^= 1  # header checksum
    check("lz4", bytes(bad), "u1", len(payload))


@pytest.mark.parametrize("lz4_flags", [0, 0x1000, 0x800], ids=["default", "lane_per_block", "wave_per_block"])
def test_lz4_corruption_sweep(lz4_flags):
    """Byte corruptions and truncations of LZ4 frames everywhere (block
    headers, tokens, length bytes, offsets, literals, end mark, checksums),
    batched, each classified and decoded like LZ4F_decompress (oracle); both
    block decoders (small batches pick one wave per block by default)."""
    rng = np.random.default_rng(31)
    payloads = [rw(100000, seed=3).tobytes(), DATASETS["text_like"]()[:150000],
                np.random.default_rng(8).integers(0, 4, 120000, dtype=np.uint8).tobytes()]
    for k, payload in enumerate(payloads):
        if k == 1:
            s = zref.lz4_frame_custom(payload, block_checksum=True)
        else:
            st, s = zref.encode(zref.LZ4, 65536, np.frombuffer(payload, np.uint8))
        for D in (len(payload), len(payload) // 2 + 3):
            streams = [s[:int(t)] for t in rng.integers(0, len(s), 48)]
            for _ in range(464):
                b = bytearray(s)
                p = int(rng.integers(0, len(b)))
                b[p] ^= int(rng.integers(1, 256))
                if rng.random() < 0.2:
                    q = int(rng.integers(0, len(b)))
                    b[q] = int(rng.integers(0, 256))
                streams.append(bytes(b))
            check_many("lz4", streams, "u1", D, flags=lz4_flags)


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f8", "bool", "u1"])
def test_raw_large_and_unaligned(dt):
    es, be, isb, npdt = dtype_info(dt)
    n = 300001
    raw = np.random.default_rng(2).integers(0, 3, n * es, dtype=np.uint8).tobytes()
    check("raw", raw, dt, n)
    check("raw", b"\x00" + raw, dt, n)  # (host copy shifts alignment in staging)
    check("raw", raw[:-1], dt, n)


# ---- device batch API -------------------------------------------------------------
@pytest.mark.parametrize("codec", ["gzip", "lz4", "raw", "xz", "bzip2"])
def test_batch_api_device_resident(codec):
    import torch
    from zarr_amd.batch import BatchCodec, PackedStreams
    n_unique, D = 24, 262144
    vals = [rw(D // 2, seed=s) for s in range(n_unique)]
    streams = []
    for v in vals:
        st, e = zref.encode(CODEC_IDS[codec], DEFAULT_PARAM[codec], v)
        streams.append(e)
    meta = ArrayMetadata.new([D // 2 * 100], [D // 2], "<i2", COMP[codec](DEFAULT_PARAM[codec]))
    packed = PackedStreams(streams, D, "cuda:0", slot_copies=3)
    codec_ = BatchCodec(0)
    codec_.decode(meta, packed)
    torch.cuda.synchronize()
    assert (packed.status.cpu().numpy() == 0).all()
    out = packed.dst.cpu().numpy().reshape(packed.n, D)
    for i in range(packed.n):
        assert out[i].tobytes() == vals[i % n_unique].tobytes(), i


def test_gzip_lookahead_after_n_bytes():
    """zlib validates the symbols after byte N that lie in flate2's current
    32 KiB input window: corruptions there must classify like the oracle."""
    payload = rw(150000).tobytes()
    s = gzip_wrap(deflate(payload, 6), payload)
    rng = np.random.default_rng(11)
    for D in (40000, 100001, 149999):
        # find roughly where byte D is produced: scan corruptions in a band
        for pos in rng.integers(12, len(s) - 8, 40):
            bad = bytearray(s)
            bad[int(pos)] ^= int(rng.integers(1, 256))
            check("gzip", bytes(bad), "u1", D)
    fixed = gzip_wrap(deflate(payload[:20000], 6, zlib.Z_FIXED), payload[:20000])
    for pos in range(len(fixed) - 40, len(fixed) - 8):
        for x in (0x01, 0x80, 0xFF):
            bad = bytearray(fixed)
            bad[pos] ^= x
            check("gzip", bytes(bad), "u1", 20000)


def test_lz4_next_header_after_n_bytes():
    """LZ4F reads the block header that follows a block ending exactly at N."""
    payload = rw(65536 * 3).tobytes()
    st, s = zref.encode(zref.LZ4, 65536, np.frombuffer(payload, np.uint8))
    hdr = 7
    pos, blocks = hdr, []
    while True:
        bs = struct.unpack_from("<I", s, pos)[0]
        blocks.append(pos)
        if bs == 0:
            break
        pos += 4 + (bs & 0x7FFFFFFF)
    for k in range(1, len(blocks)):
        for val in (0x7FFFFFFF, 0x00010001, 0x80010000, 0):
            bad = bytearray(s)
            struct.pack_into("<I", bad, blocks[k], val)
            check("lz4", bytes(bad), "u1", 65536 * k)


@pytest.mark.parametrize("data", list(DATASETS))
def test_inflate_parallel_vs_serial_kernel(data):
    """The speculative inflate kernels (one wave per chunk, the default; the
    256-lane round kernel, FLAG_INFLATE_BLOCK_PAR) and the wave-serial one
    must agree bit for bit (and with the oracle) on every deflate structure;
    the debug-counter flag must not change the output."""
    from zarr_amd._native import FLAG_DEBUG_COUNTERS, FLAG_INFLATE_BLOCK_PAR, FLAG_SERIAL_INFLATE
    payload = DATASETS[data]()
    streams = [gzip_wrap(deflate(payload, lvl, strat), payload)
               for lvl, strat in ((1, 0), (6, 0), (9, 0), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_RLE))]
    for s in streams:
        for D in (len(payload), len(payload) // 3 + 1):
            meta = meta_for("gzip", "u1", D)
            a = DefaultChunk.read_chunk(s, meta, [0], np.uint8).get_data()
            b = DefaultChunk.read_chunk(s, meta, [0], np.uint8, flags=FLAG_SERIAL_INFLATE).get_data()
            c = DefaultChunk.read_chunk(s, meta, [0], np.uint8, flags=FLAG_INFLATE_BLOCK_PAR).get_data()
            w = DefaultChunk.read_chunk(s, meta, [0], np.uint8, flags=FLAG_INFLATE_WAVE).get_data()
            assert np.array_equal(a, b) and np.array_equal(a, c) and np.array_equal(a, w)
            assert a.tobytes() == payload[:D]
    s = streams[1]
    meta = meta_for("gzip", "u1", len(payload))
    for f in (FLAG_DEBUG_COUNTERS | FLAG_INFLATE_WAVE, FLAG_DEBUG_COUNTERS | FLAG_INFLATE_BLOCK_PAR):
        assert DefaultChunk.read_chunk(s, meta, [0], np.uint8, flags=f).get_data().tobytes() == payload


@pytest.mark.parametrize("codec", ["gzip", "lz4", "raw", "xz", "bzip2"])
def test_decode_never_writes_past_n(codec):
    """read_exact stops at byte N even inside a long match: the bytes after
    N*elem_size in the caller's buffer stay untouched (chunk.rs:112-113)."""
    import torch
    from zarr_amd._native import FLAG_INFLATE_BLOCK_PAR, FLAG_SERIAL_INFLATE
    from zarr_amd.batch import BatchCodec, PackedStreams
    payloads = [bytes(300000), (b"abcdefgh" * 40000), rw(150000).tobytes()]
    streams = [zref.encode(CODEC_IDS[codec], DEFAULT_PARAM[codec], np.frombuffer(p, np.uint8))[1]
               for p in payloads]
    guard = 4096
    for D in (1, 777, 16385, 65537, 99999, 200003):
        flag_sets = (0, FLAG_SERIAL_INFLATE, FLAG_INFLATE_BLOCK_PAR, FLAG_INFLATE_WAVE) if codec == "gzip" else (0,)
        for flags in flag_sets:
            dst = torch.full((len(streams) * (D + guard),), 0xAB, dtype=torch.uint8, device="cuda:0")
            packed = PackedStreams(streams, D + guard, "cuda:0", dst=dst)
            BatchCodec(0).decode(meta_for(codec, "u1", D), packed, flags=flags)
            torch.cuda.synchronize()
            assert (packed.status.cpu().numpy() == 0).all()
            out = dst.cpu().numpy().reshape(len(streams), D + guard)
            for i, p in enumerate(payloads):
                assert out[i, :D].tobytes() == p[:D], (D, i)
                assert (out[i, D:] == 0xAB).all(), (D, i, flags)


def check_many(codec, streams, dt, n, flags=0, param=None):
    """Batch decode of many streams; each result must classify and decode like
    the oracle (one launch, so sweeps of corruptions stay fast)."""
    import torch
    from zarr_amd.batch import BatchCodec, PackedStreams
    es, be, isb, _ = dtype_info(dt)
    st_ref, out_ref = zref.decode_batch(CODEC_IDS[codec], [np.frombuffer(s, np.uint8) for s in streams],
                                        n * es, elem_size=es, big_endian=be, is_bool=isb)
    packed = PackedStreams(streams, n * es, "cuda:0")
    BatchCodec(0).decode(meta_for(codec, dt, n, param), packed, flags=flags)
    torch.cuda.synchronize()
    st = packed.status.cpu().numpy()
    out = packed.dst.cpu().numpy().reshape(len(streams), n * es)
    for i in range(len(streams)):
        assert KIND[int(st[i])] == KIND[int(st_ref[i])], (i, int(st[i]), int(st_ref[i]))
        if st_ref[i] == zref.OK:
            assert out[i].tobytes() == out_ref[i].tobytes(), i


def test_gzip_dynamic_header_corruption():
    """Every byte of three dynamic block headers (the first, and two after
    full flushes) flipped several ways: the wave-parallel header decoder (and
    the 256-lane kernel's block-parallel one) must classify and decode exactly
    like zlib."""
    from zarr_amd._native import FLAG_INFLATE_BLOCK_PAR, FLAG_SERIAL_INFLATE
    parts = [rw(20000, seed=s).tobytes() for s in range(3)]
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    raw, offs = b"", []
    for p in parts:
        offs.append(len(raw))
        raw += c.compress(p) + c.flush(zlib.Z_FULL_FLUSH)
    raw += c.flush()
    payload = b"".join(parts)
    s = gzip_wrap(raw, payload)
    hdr = len(s) - len(raw) - 8
    variants = [s]
    for off in offs:
        for k in range(90):
            for x in (0x01, 0x08, 0x40, 0xFF):
                bad = bytearray(s)
                bad[hdr + off + k] ^= x
                variants.append(bytes(bad))
    for flags in (0, FLAG_SERIAL_INFLATE, FLAG_INFLATE_BLOCK_PAR, FLAG_INFLATE_WAVE):
        check_many("gzip", variants, "u1", len(payload), flags)


def test_inflate_wave_capped_chain_keeps_block_positions():
    """Round-6 regression: when the first round's chain runs past a block's
    EOB and its last member's list is capped, the segment size is halved for
    the next round; the EOB's bit position (the next header) must still come
    from this round's segment starts.  All-literal 16 383-symbol blocks with
    the long-segment test hook (116 %) hit exactly that path; before the fix
    the next header was read at the halved-segment position (InvalidData)."""
    payload = DATASETS["randwalk_i2"]()
    s = gzip_wrap(deflate(payload, 6, zlib.Z_HUFFMAN_ONLY), payload)
    st, ref = zref.decode(zref.GZIP, s, len(payload), 1, 0, 0)
    assert st == zref.OK and ref == payload
    for flags in (FLAG_INFLATE_WAVE | 0x10000, FLAG_INFLATE_WAVE):
        kind, out = gpu_decode("gzip", s, "u1", len(payload), None, flags)
        assert kind == "Ok", (kind, flags)
        assert out == payload, flags
