"""GPU parity of the Xz decoder (zcg_xz.hip) against the oracle.

The reference decodes Xz with xz2's read::XzDecoder (src/compression/xz.rs:
34-43) = liblzma 5.2's stream decoder; the oracle runs that same liblzma
with the same 32 KiB input windows.  Streams come from the oracle encoder
(xz2 XzEncoder = lzma_easy_encoder(preset, CRC64), xz.rs:34-43) and from
Python's lzma (the same liblzma) for structures xz2 never writes but
liblzma decodes: other checks, lc/lp/pb, multiple LZMA2 chunks, stored
(uncompressed) chunks.  The same decode core is fuzzed on the CPU in
tests/test_hostcore.py; here the GPU kernel runs the corruption sweeps in
batches.
"""
import lzma

import numpy as np
import pytest

import zref
from test_gpu_parity import DATASETS, check, check_many, rw

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("data", list(DATASETS))
@pytest.mark.parametrize("preset", [0, 6, 9])
def test_xz_large(data, preset):
    payload = DATASETS[data]()
    st, s = zref.encode(zref.XZ, preset, np.frombuffer(payload, np.uint8))
    assert st == zref.OK
    for D in (len(payload), len(payload) // 3 + 7):
        check("xz", s, "u1", D, param=preset)


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", ">u8", "bool", "i1"])
def test_xz_transform(dt):
    from golden_util import dtype_info
    es = dtype_info(dt)[0]
    n = 70001
    raw = rw(n * es // 2 + 1).tobytes()[: n * es]
    st, s = zref.encode(zref.XZ, 6, np.frombuffer(raw, np.uint8))
    check("xz", s, dt, n)


@pytest.mark.parametrize("check_id", [lzma.CHECK_NONE, lzma.CHECK_CRC32, lzma.CHECK_CRC64, lzma.CHECK_SHA256])
@pytest.mark.parametrize("lclppb", [(3, 0, 2), (0, 4, 0), (4, 0, 4), (1, 3, 1), (2, 2, 3)])
def test_xz_liblzma_variants(check_id, lclppb):
    lc, lp, pb = lclppb
    payload = rw(200000, seed=lc * 7 + lp).tobytes()
    filt = [{"id": lzma.FILTER_LZMA2, "preset": 6, "lc": lc, "lp": lp, "pb": pb}]
    s = lzma.compress(payload, format=lzma.FORMAT_XZ, check=check_id, filters=filt)
    for D in (len(payload), 123457):
        check("xz", s, "u1", D)


def test_xz_uncompressed_chunks_and_many_lzma_chunks():
    rng = np.random.default_rng(3)
    noise = rng.integers(0, 256, 300000, dtype=np.uint8).tobytes()   # stored LZMA2 chunks
    mixed = noise[:100000] + bytes(200000) + noise[100000:200000]
    for payload in (noise, mixed):
        s = lzma.compress(payload, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6)
        for D in (len(payload), 65536, 65537, 250001):
            check("xz", s, "u1", D)


def test_xz_corruption_sweep():
    """Truncations and byte corruptions everywhere, including after byte N
    (liblzma validates what its current input window holds)."""
    rng = np.random.default_rng(17)
    for k, payload in enumerate([rw(30000, seed=1).tobytes(), bytes(50000),
                                 rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()]):
        s = lzma.compress(payload, format=lzma.FORMAT_XZ, check=(lzma.CHECK_CRC64, lzma.CHECK_CRC32)[k % 2],
                          preset=6)
        for D in (len(payload), len(payload) // 2):
            streams = [s[:int(t)] for t in rng.integers(0, len(s), 64)]
            for _ in range(448):
                b = bytearray(s)
                if rng.random() < 0.3:
                    p = len(b) - 1 - int(rng.integers(0, min(len(b), 64)))
                else:
                    p = int(rng.integers(0, len(b)))
                b[p] ^= int(rng.integers(1, 256))
                streams.append(bytes(b))
            check_many("xz", streams, "u1", D)


@pytest.mark.parametrize("dist", [1, 2, 4, 7, 64, 256])
def test_xz_delta_filter(dist):
    """delta + LZMA2 chains (liblzma's delta decoder after LZMA2, history zero
    at the block start): whole and partial reads, CRC32/CRC64/no check, and a
    corruption sweep, against the oracle's liblzma."""
    rng = np.random.default_rng(dist)
    for k, payload in enumerate([rw(200001, seed=dist).tobytes(),
                                 (np.arange(150000) * 3 % 256).astype(np.uint8).tobytes(),
                                 rng.integers(0, 256, 30000, dtype=np.uint8).tobytes(), b"\x05"]):
        s = lzma.compress(payload, format=lzma.FORMAT_XZ,
                          check=(lzma.CHECK_CRC64, lzma.CHECK_CRC32, lzma.CHECK_NONE)[k % 3],
                          filters=[{"id": lzma.FILTER_DELTA, "dist": dist}, {"id": lzma.FILTER_LZMA2, "preset": 6}])
        for D in sorted({len(payload), max(1, len(payload) // 3), len(payload) + 5}):
            check("xz", s, "u1", D)
    payload = rw(40000, seed=3).tobytes()
    s = lzma.compress(payload, format=lzma.FORMAT_XZ, filters=[{"id": lzma.FILTER_DELTA, "dist": dist},
                                                               {"id": lzma.FILTER_LZMA2}])
    streams = [s[:int(t)] for t in rng.integers(0, len(s), 32)]
    for _ in range(96):
        b = bytearray(s)
        b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
        streams.append(bytes(b))
    check_many("xz", streams, "u1", len(payload))


def test_xz_delta_filter_dtypes():
    """A delta filter over multi-byte elements ('>' byte order applied after
    the filter)."""
    for dt, dist in ((">i2", 2), ("<f4", 4), (">u8", 8)):
        v = (np.cumsum(np.random.default_rng(4).integers(-3, 4, 50000)) % 1000).astype(dt)
        s = lzma.compress(v.tobytes(), format=lzma.FORMAT_XZ,
                          filters=[{"id": lzma.FILTER_DELTA, "dist": dist}, {"id": lzma.FILTER_LZMA2}])
        check("xz", s, dt, v.nbytes)


@pytest.mark.parametrize("name", ["X86", "ARM", "ARMTHUMB", "POWERPC", "SPARC", "IA64"])
def test_xz_bcj_filters(name):
    """BCJ + LZMA2 chains (liblzma simple/*.c) against the oracle's liblzma:
    whole reads, reads past the end, reads that stop inside the block (the
    simple coder's look-past decode), start offsets, and a corruption sweep."""
    from test_hostcore import bcj_payload
    fid = getattr(lzma, "FILTER_" + name)
    rng = np.random.default_rng(len(name) + 7)
    for n in (5, 4097, 200001):
        for so in (0, 1024):
            raw = bcj_payload(rng, n, fid)
            f0 = {"id": fid} if so == 0 else {"id": fid, "start_offset": so}
            s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=[f0, {"id": lzma.FILTER_LZMA2}])
            for D in sorted({n, n + 5, *range(max(1, n // 3), max(1, n // 3) + 6)}):
                check("xz", s, "u1", D)
    raw = bcj_payload(rng, 40000, fid)
    s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=[{"id": fid}, {"id": lzma.FILTER_LZMA2}])
    streams = [s[:int(t)] for t in rng.integers(0, len(s), 24)]
    for _ in range(72):
        b = bytearray(s)
        b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
        streams.append(bytes(b))
    check_many("xz", streams, "u1", len(raw))


@pytest.mark.parametrize("chain", [("DELTA", "X86"), ("X86", "DELTA"), ("ARM", "DELTA", "SPARC"), ("ARMTHUMB", "IA64")])
def test_xz_filter_chains(chain):
    """Two or three delta / BCJ filters before LZMA2, against the oracle."""
    from test_hostcore import bcj_payload, host_xz
    rng = np.random.default_rng(len(chain) * 5 + len(chain[-1]))
    filters = [{"id": lzma.FILTER_DELTA, "dist": 4} if c == "DELTA" else {"id": getattr(lzma, "FILTER_" + c)}
               for c in chain] + [{"id": lzma.FILTER_LZMA2}]
    bcj = [c for c in chain if c != "DELTA"]
    for n in (4097, 200001):
        raw = bcj_payload(rng, n, getattr(lzma, "FILTER_" + bcj[0]))
        s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=filters)
        part = [D for D in range(n // 3, n // 3 + 6) if host_xz(s, D)[0] != 4]
        for D in sorted({n, n + 5, *part}):
            check("xz", s, "u1", D)


def test_xz_sha256_check_parity():
    """Check ID 10: liblzma verifies the SHA-256 of each block; whole and
    partial reads, a corrupted digest byte, corrupted data, two blocks."""
    rng = np.random.default_rng(11)
    payload = rw(150000, seed=2).tobytes()
    s = lzma.compress(payload, format=lzma.FORMAT_XZ, check=lzma.CHECK_SHA256, preset=6)
    streams, Ds = [s], [len(payload), 70001]
    isz = (int.from_bytes(s[-8:-4], "little") + 1) * 4  # backward size: the index
    dend = len(s) - 12 - isz                            # the block's digest ends here
    for k in (0, 5, 31):
        b = bytearray(s)
        b[dend - 32 + k] ^= 0x10
        streams.append(bytes(b))
    for _ in range(6):
        b = bytearray(s)
        b[int(rng.integers(24, dend - 32))] ^= 1 << int(rng.integers(0, 8))
        streams.append(bytes(b))
    small = lzma.compress(payload[:333], format=lzma.FORMAT_XZ, check=lzma.CHECK_SHA256)
    streams.append(small)
    Ds.append(333)
    for st_ in streams:
        for D in Ds:
            check("xz", st_, "u1", D)


def test_xz_lzma1_block_is_invalid_like_liblzma():
    """An LZMA1 block (filter 0x4000000000000001 as the last filter, raw LZMA1
    data with its end marker) in an .xz container: liblzma 5.2 answers
    LZMA_DATA_ERROR, so the reference's read_chunk is InvalidData, and so is ours."""
    import struct
    import zlib

    def vli(x):
        out = b""
        while True:
            b, x = x & 0x7F, x >> 7
            out += bytes([b | (0x80 if x else 0)])
            if not x:
                return out

    def crc(b):
        return struct.pack("<I", zlib.crc32(b) & 0xFFFFFFFF)

    payload = rw(20000, seed=3).tobytes()
    for lc, lp, pb, ds in [(3, 0, 2, 1 << 16), (0, 0, 0, 4096), (1, 3, 1, 1 << 20)]:
        raw = lzma.compress(payload, format=lzma.FORMAT_RAW,
                            filters=[{"id": lzma.FILTER_LZMA1, "lc": lc, "lp": lp, "pb": pb, "dict_size": ds}])
        hb = bytes([0]) + vli(0x4000000000000001) + vli(5) + bytes([(pb * 5 + lp) * 9 + lc]) + struct.pack("<I", ds)
        hsize = (len(hb) + 5 + 3) // 4 * 4
        hdr = bytes([hsize // 4 - 1]) + hb
        hdr += b"\0" * (hsize - 4 - len(hdr))
        hdr += crc(hdr)
        body = hdr + raw + b"\0" * ((4 - len(raw) % 4) % 4) + crc(payload)
        idx = b"\0" + vli(1) + vli(len(hdr) + len(raw) + 4) + vli(len(payload))
        idx += b"\0" * ((4 - len(idx) % 4) % 4)
        idx += crc(idx)
        ft = struct.pack("<I", len(idx) // 4 - 1) + bytes([0, 1])
        s = b"\xfd7zXZ\0\x00\x01" + crc(b"\x00\x01") + body + idx + crc(ft) + ft + b"YZ"
        for D in (len(payload), 100, 1):
            assert zref.decode(zref.XZ, s, D)[0] == zref.INVALID_DATA
            check("xz", s, "u1", D)


@pytest.mark.parametrize("name", ["X86", "ARMTHUMB", "IA64", "SPARC"])
def test_xz_bcj_look_past_parity(name):
    """A read that stops inside a BCJ block: liblzma's simple coder decodes
    past the caller's end to release the bytes its loop held back.  Every
    stop offset over a range, and truncations / corruptions of the stream
    around the compressed position of the stop (EOF when the input cannot
    supply the look-past bytes, InvalidData when they are corrupt), with and
    without an outer delta stage, one batch per case list, against the oracle."""
    from test_hostcore import _min_input, bcj_payload
    fid = getattr(lzma, "FILTER_" + name)
    rng = np.random.default_rng(len(name) + 200)
    raw = bcj_payload(rng, 30001, fid)
    for chain in ([{"id": fid}], [{"id": lzma.FILTER_DELTA, "dist": 3}, {"id": fid}]):
        s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=chain + [{"id": lzma.FILTER_LZMA2}])
        for D in range(10000, 10024):
            check("xz", s, "u1", D)
        for D in (12345, 20002):
            lo = _min_input(s, D)
            cases = [s[:t] for t in range(lo - 24, min(len(s), lo + 24))]
            for p in range(lo - 24, min(len(s), lo + 12)):
                b = bytearray(s)
                b[p] ^= 0x55
                cases.append(bytes(b))
            check_many("xz", cases, "u1", D)


def test_xz_bcj_unmodelled_look_past_fails_loudly():
    """The look-past decode is modelled for one BCJ stage fed by LZMA2 (outer
    delta stages allowed).  A partial read of an x86-over-delta block whose
    last bytes could start a cut-off instruction raises instead of returning
    bytes that might differ."""
    from test_hostcore import bcj_payload, host_xz
    from zarr_amd import ArrayMetadata, DefaultChunk, NativeUnavailable
    from zarr_amd.compression import Xz
    payload = bcj_payload(np.random.default_rng(5), 5000, lzma.FILTER_X86)
    s = lzma.compress(payload, format=lzma.FORMAT_XZ,
                      filters=[{"id": lzma.FILTER_X86}, {"id": lzma.FILTER_DELTA, "dist": 1}, {"id": lzma.FILTER_LZMA2}])
    D = next(d for d in range(1000, 5000) if host_xz(s, d)[0] == 4)
    assert zref.decode(zref.XZ, s, D)[0] == zref.OK
    meta = ArrayMetadata.new([D], [D], "u1", Xz(6))
    with pytest.raises(NativeUnavailable):
        DefaultChunk.read_chunk(s, meta, [0], np.uint8)