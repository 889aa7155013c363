"""CPU fuzzing of the device decode cores (zarr_amd/csrc/*_core.h, compiled
for the host by tests/hostcore) against the oracle.  The GPU kernels run the
same core source; this is where the long corruption sweeps run, because a
host decode costs microseconds.  TEST INFRASTRUCTURE ONLY."""
import ctypes
import lzma
import os
import subprocess

import numpy as np
import pytest

import zref

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hostcore")
_H = None


def host():
    global _H
    if _H is None:
        subprocess.run(["make", "-s", "-C", HERE], check=True)
        _H = ctypes.CDLL(os.path.join(HERE, "libzcg_host.so"))
        _H.zh_xz_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        _H.zh_xz_decode.restype = ctypes.c_int
        _H.zh_bz2_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64]
        _H.zh_bz2_decode.restype = ctypes.c_int
    return _H


def host_xz(s: bytes, D: int):
    out = np.zeros(max(D, 1), np.uint8)
    a = np.frombuffer(s, np.uint8) if s else np.zeros(1, np.uint8)
    st = host().zh_xz_decode(a.ctypes.data, len(s), out.ctypes.data, D)
    return st, out[:D].tobytes()


def same(s, D):
    r1 = zref.decode(zref.XZ, s, D)
    r2 = host_xz(s, D)
    assert r1[0] == r2[0], (r1[0], r2[0], D, len(s))
    if r1[0] == zref.OK:
        assert r1[1] == r2[1]


def _data(rng, k, n):
    if k == 0:
        return rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    if k == 1:
        return np.cumsum(rng.integers(-3, 4, n // 2 + 1)).astype("<i2").tobytes()[:n]
    if k == 2:
        return bytes(n)
    return (np.arange(n) % 251).astype(np.uint8).tobytes()


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_xz_core_fuzz_vs_liblzma(seed):
    rng = np.random.default_rng(seed)
    checks = [lzma.CHECK_CRC64, lzma.CHECK_CRC32, lzma.CHECK_NONE]
    for _ in range(120):
        k = int(rng.integers(0, 4))
        n = int(rng.choice([1, 7, 300, 4000, 40000, 120000]))
        raw = _data(rng, k, n)
        lc = int(rng.integers(0, 5))
        lp = int(rng.integers(0, 5 - lc))
        filt = [{"id": lzma.FILTER_LZMA2, "preset": int(rng.integers(0, 10)), "lc": lc, "lp": lp,
                 "pb": int(rng.integers(0, 5))}]
        s = lzma.compress(raw, format=lzma.FORMAT_XZ, check=checks[int(rng.integers(0, 3))], filters=filt)
        Ds = [len(raw), max(1, len(raw) // 3), len(raw) + 1]
        for D in Ds:
            same(s, D)
        for t in rng.integers(0, len(s), 4):
            same(s[:int(t)], len(raw))
        for _ in range(20):
            b = bytearray(s)
            if rng.random() < 0.3:
                p = len(b) - 1 - int(rng.integers(0, min(len(b), 48)))
            else:
                p = int(rng.integers(0, len(b)))
            b[p] ^= 1 << int(rng.integers(0, 8)) if rng.random() < 0.5 else int(rng.integers(1, 256))
            same(bytes(b), Ds[int(rng.integers(0, 3))])


@pytest.mark.parametrize("dist", [1, 2, 3, 4, 8, 100, 256])
def test_xz_core_delta_filter_vs_liblzma(dist):
    """delta + LZMA2 chains: the core's block-end delta decode (and the one at
    an early stop) against liblzma, whole / partial / overlong reads, and
    corruptions."""
    rng = np.random.default_rng(dist)
    for k in range(4):
        raw = _data(rng, k, int(rng.choice([1, 5, 300, 40000, 120000])))
        s = lzma.compress(raw, format=lzma.FORMAT_XZ, check=[lzma.CHECK_CRC64, lzma.CHECK_CRC32][k % 2],
                          filters=[{"id": lzma.FILTER_DELTA, "dist": dist}, {"id": lzma.FILTER_LZMA2, "preset": 6}])
        for D in (len(raw), max(1, len(raw) // 3), len(raw) + 1):
            same(s, D)
        for t in rng.integers(0, len(s), 4):
            same(s[:int(t)], len(raw))
        for _ in range(20):
            b = bytearray(s)
            b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
            same(bytes(b), len(raw))


def bcj_payload(rng, n, fid):
    """Random bytes with the filter's instruction patterns planted densely
    (x86 E8/E9 + 0x00/0xFF high byte, ARM BL, Thumb BL pairs, PowerPC bl,
    SPARC call), so conversions and their skip rules are exercised."""
    b = rng.integers(0, 256, max(n, 16), dtype=np.uint8)
    for _ in range(max(n, 16) // 12):
        i = int(rng.integers(0, len(b) - 8))
        if fid == lzma.FILTER_X86:
            b[i] = 0xE8 if rng.random() < 0.5 else 0xE9
            b[i + 4] = 0 if rng.random() < 0.5 else 0xFF
        elif fid == lzma.FILTER_ARM:
            b[(i & ~3) + 3] = 0xEB
        elif fid == lzma.FILTER_ARMTHUMB:
            i &= ~1
            b[i + 1] = 0xF0 | (int(b[i + 1]) & 7)
            b[i + 3] = 0xF8 | (int(b[i + 3]) & 7)
        elif fid == lzma.FILTER_POWERPC:
            i &= ~3
            b[i] = 0x48 | (int(b[i]) & 3)
            b[i + 3] = (int(b[i + 3]) & 0xFC) | 1
        elif fid == lzma.FILTER_IA64:  # template 0x10 (slot 2 a branch slot), opcode 5, bits 9-11 zero
            i &= ~15
            if i + 16 <= len(b):
                b[i] = (int(b[i]) & 0xE0) | 0x10
                b[i + 15] = (int(b[i + 15]) & 0x0F) | 0x50
                b[i + 12] = int(b[i + 12]) & 0xF8
        elif fid == lzma.FILTER_SPARC:
            i &= ~3
            b[i] = 0x40 if rng.random() < 0.5 else 0x7F
            b[i + 1] = (int(b[i + 1]) & 0x3F) | (0 if b[i] == 0x40 else 0xC0)
    return b.tobytes()[:n]


BCJ_FILTERS = ["X86", "ARM", "ARMTHUMB", "POWERPC", "SPARC", "IA64"]


@pytest.mark.parametrize("name", BCJ_FILTERS)
def test_xz_core_bcj_filters_vs_liblzma(name):
    """BCJ + LZMA2 chains (liblzma simple/*.c): the core's block-end BCJ decode
    against liblzma for whole reads, reads that stop inside the block (the
    simple coder's look-past decode, exact), start offsets, and corruptions."""
    fid = getattr(lzma, "FILTER_" + name)
    rng = np.random.default_rng(len(name))
    for n in (1, 3, 4, 5, 7, 100, 4097, 70001):
        for so in (0, 16 if name == "IA64" else 4, 1024):
            raw = bcj_payload(rng, n, fid)
            f0 = {"id": fid} if so == 0 else {"id": fid, "start_offset": so}
            s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=[f0, {"id": lzma.FILTER_LZMA2}])
            st, out = host_xz(s, n)
            assert st == 0 and out == raw
            for D in sorted({max(1, n // 3), max(1, n // 3) + 1, max(1, n - 2), n + 1}):
                r1 = zref.decode(zref.XZ, s, D)
                r2 = host_xz(s, D)
                assert r1[0] == r2[0], (n, so, D, r1[0], r2[0])
                if r1[0] == zref.OK:
                    assert r1[1] == r2[1], (n, so, D)
    raw = bcj_payload(rng, 30000, fid)
    s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=[{"id": fid}, {"id": lzma.FILTER_LZMA2}])
    for _ in range(30):
        b = bytearray(s)
        b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
        r1, r2 = zref.decode(zref.XZ, bytes(b), len(raw)), host_xz(bytes(b), len(raw))
        assert r1[0] == r2[0]
        if r1[0] == zref.OK:
            assert r1[1] == r2[1]


def _min_input(s, D):
    """The shortest prefix of s from which liblzma's read_exact of D succeeds."""
    lo, hi = 0, len(s)
    while lo < hi:
        m = (lo + hi) // 2
        if zref.decode(zref.XZ, s[:m], D)[0] == zref.OK:
            hi = m
        else:
            lo = m + 1
    return lo


@pytest.mark.parametrize("name", BCJ_FILTERS)
def test_xz_core_bcj_look_past_vs_liblzma(name):
    """A read that stops inside a BCJ block: liblzma's simple coder holds back
    the bytes its loop has not processed and decodes up to 2 x unfiltered_max
    bytes past the end to release them (EOF if the input cannot supply them,
    InvalidData if that data is corrupt).  Every stop offset over a range,
    and truncations / corruptions of the stream around the compressed
    position of the stop, against liblzma; outer delta stages too."""
    fid = getattr(lzma, "FILTER_" + name)
    rng = np.random.default_rng(len(name) + 100)
    raw = bcj_payload(rng, 30001, fid)
    for chain in ([{"id": fid}], [{"id": lzma.FILTER_DELTA, "dist": 3}, {"id": fid}]):
        s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=chain + [{"id": lzma.FILTER_LZMA2}])
        for D in range(10000, 10040):
            r1, r2 = zref.decode(zref.XZ, s, D), host_xz(s, D)
            assert r1[0] == r2[0] == zref.OK and r1[1] == r2[1], (D, r1[0], r2[0])
        kinds = set()
        for D in (12345, 20002):
            lo = _min_input(s, D)
            cases = [s[:t] for t in range(lo - 24, min(len(s), lo + 24))]
            for p in range(lo - 24, min(len(s), lo + 12)):
                b = bytearray(s)
                b[p] ^= 0x55
                cases.append(bytes(b))
            for c in cases:
                r1, r2 = zref.decode(zref.XZ, c, D), host_xz(c, D)
                kinds.add(r1[0])
                assert r1[0] == r2[0], (D, len(c), r1[0], r2[0])
                if r1[0] == zref.OK:
                    assert r1[1] == r2[1]
        assert zref.OK in kinds and zref.EOF in kinds


@pytest.mark.parametrize("chain", [("DELTA", "X86"), ("X86", "DELTA"), ("ARM", "DELTA", "SPARC"),
                                   ("DELTA", "DELTA"), ("ARMTHUMB", "IA64")])
def test_xz_core_filter_chains_vs_liblzma(chain):
    """Chains of two or three delta / BCJ filters before LZMA2 (decoded in
    reverse chain order, each over the previous one's output) against
    liblzma, whole and partial reads.  A partial read may be UNSUPPORTED
    only where the look-past decode is not modelled: a second BCJ stage, or
    a delta stage under the BCJ."""
    rng = np.random.default_rng(len(chain) * 7 + len(chain[0]))
    filters = [{"id": lzma.FILTER_DELTA, "dist": 4} if c == "DELTA" else {"id": getattr(lzma, "FILTER_" + c)}
               for c in chain] + [{"id": lzma.FILTER_LZMA2}]
    bcj = [c for c in chain if c != "DELTA"]
    for n in (3, 4097, 70001):
        raw = bcj_payload(rng, n, getattr(lzma, "FILTER_" + bcj[0])) if bcj else rng.bytes(n)
        s = lzma.compress(raw, format=lzma.FORMAT_XZ, filters=filters)
        st, out = host_xz(s, n)
        assert st == 0 and out == raw
        for D in (max(1, n // 3), n + 1):
            r1, r2 = zref.decode(zref.XZ, s, D), host_xz(s, D)
            if r2[0] == 4 and r1[0] == zref.OK:
                assert D < n and (len(bcj) > 1 or chain[-1] == "DELTA")
                continue
            assert r1[0] == r2[0] and (r1[0] != zref.OK or r1[1] == r2[1]), (n, D)


def test_xz_core_reference_vectors():
    """doc-spec vector (xz.rs:52-75) and the oracle's xz2-style encodes."""
    from golden_util import doc_spec
    d = doc_spec()
    s = bytes.fromhex(d["chunks"]["xz"]["hex"])
    st, out = host_xz(s, 12)
    assert st == 0
    assert np.frombuffer(out, ">i2").tolist() == d["expected_values"]
    for preset in range(10):
        v = np.cumsum(np.random.default_rng(preset).integers(-3, 4, 50000)).astype("<i2")
        st, enc = zref.encode(zref.XZ, preset, v)
        assert st == 0
        same(enc, v.nbytes)


def host_bz2(s: bytes, D: int):
    out = np.zeros(max(D, 1), np.uint8)
    a = np.frombuffer(s, np.uint8) if s else np.zeros(1, np.uint8)
    st = host().zh_bz2_decode(a.ctypes.data, len(s), out.ctypes.data, D)
    return st, out[:D].tobytes()


def same_bz2(s, D):
    r1 = zref.decode(zref.BZIP2, s, D)
    r2 = host_bz2(s, D)
    assert r1[0] == r2[0], (r1[0], r2[0], D, len(s))
    if r1[0] == zref.OK:
        assert r1[1] == r2[1]


@pytest.mark.parametrize("seed", [1, 2])
def test_bzip2_core_fuzz_vs_libbz2(seed):
    """Block parsing, selectors, code lengths, libbz2's limit/base/perm
    Huffman decoding, RUNA/RUNB + MTF, origPtr checks, the tPos walk,
    unRLE_obuf_to_output_FAST, block/combined CRCs, randomised blocks and
    the 32 KiB-window post-N behaviour, against libbz2 1.0.8."""
    import bz2
    rng = np.random.default_rng(seed)
    for _ in range(80):
        k = int(rng.integers(0, 5))
        n = int(rng.choice([1, 7, 300, 4000, 40000, 250000]))
        raw = (_data(rng, k, n) if k < 4 else
               bytes(rng.integers(0, 3, n, dtype=np.uint8).repeat(7)[:n]))
        s = bz2.compress(raw, int(rng.integers(1, 10)))
        Ds = [len(raw), max(1, len(raw) // 3), len(raw) + 1]
        for D in Ds:
            same_bz2(s, D)
        for t in rng.integers(0, len(s), 4):
            same_bz2(s[:int(t)], len(raw))
        for _ in range(12):
            b = bytearray(s)
            if rng.random() < 0.3:
                p = len(b) - 1 - int(rng.integers(0, min(len(b), 24)))
            else:
                p = int(rng.integers(0, len(b)))
            b[p] ^= 1 << int(rng.integers(0, 8)) if rng.random() < 0.5 else int(rng.integers(1, 256))
            same_bz2(bytes(b), Ds[int(rng.integers(0, 3))])


def test_bzip2_core_reference_vector():
    """doc-spec vector (bzip.rs:55-72)."""
    from golden_util import doc_spec
    d = doc_spec()
    st, out = host_bz2(bytes.fromhex(d["chunks"]["bzip2"]["hex"]), 12)
    assert st == 0
    assert np.frombuffer(out, ">i2").tolist() == d["expected_values"]


# ---- LZ4 block compressor: serial restatement vs liblz4 (byte-exact) -------
_LZ4 = None


def liblz4():
    global _LZ4
    if _LZ4 is None:
        import ctypes.util
        _LZ4 = ctypes.CDLL(ctypes.util.find_library("lz4") or "liblz4.so.1")
        _LZ4.LZ4_compress_fast.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int]
        _LZ4.LZ4_compress_fast.restype = ctypes.c_int
    return _LZ4


def lz4_pair(block: bytes):
    """(liblz4, restatement) of one block at LZ4F's capacity srcSize - 1."""
    n = len(block)
    a = np.frombuffer(block, np.uint8) if n else np.zeros(1, np.uint8)
    cap = max(n - 1, 0)
    o1 = np.zeros(n + 64, np.uint8)
    o2 = np.zeros(n + 64, np.uint8)
    r1 = liblz4().LZ4_compress_fast(a.ctypes.data, o1.ctypes.data, n, cap, 1)
    h = host()
    h.zref_lz4_fast_block.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    r2 = h.zref_lz4_fast_block(a.ctypes.data, n, o2.ctypes.data, cap)
    return (r1, o1[:max(r1, 0)].tobytes()), (r2, o2[:max(r2, 0)].tobytes())


def lz4_blocks_corpus(seed):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(4):
        for n in (0, 1, 12, 13, 14, 100, 4095, 4096, 65535, 65536):
            out.append(_data(rng, k, n))
    # C4-shaped blocks (random walk i16), the C2 "quant" f32 field, sparse
    # repeats, near-incompressible blocks around the stored/compressed boundary
    for _ in range(12):
        out.append(np.cumsum(rng.integers(-3, 4, 32768)).astype("<i2").tobytes())
    i = np.arange(16384)
    out.append((np.round(64 * (100 * np.sin(0.05 * (i + seed)) + i % 7)) / 64).astype("<f4").tobytes())
    for frac in (0.0, 0.002, 0.01, 0.03):
        b = rng.integers(0, 256, 65536, dtype=np.uint8)
        m = rng.random(65536) < frac
        b[m] = 0
        out.append(b.tobytes())
    b = bytearray(rng.integers(0, 256, 65536, dtype=np.uint8).tobytes())
    for _ in range(40):  # copies of earlier pieces at random offsets
        L = int(rng.integers(4, 300)); s = int(rng.integers(0, 65536 - L)); d = int(rng.integers(0, 65536 - L))
        b[d:d + L] = b[s:s + L]
    out.append(bytes(b))
    # byU32 blocks (lz4 blockSize 256K / 1M): distances past 65 535 are skipped
    for n in (65546, 65547, 70000, 262144):
        out.append(np.cumsum(rng.integers(-3, 4, n // 2)).astype("<i2").tobytes())
    b = rng.integers(0, 256, 200000, dtype=np.uint8)
    b[100000:150000] = b[0:50000]  # repeats 100 000 back: out of range
    b[150000:160000] = b[120000:130000]
    out.append(b.tobytes())
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_lz4_fast_block_restatement_matches_liblz4(seed):
    for blk in lz4_blocks_corpus(seed):
        (r1, o1), (r2, o2) = lz4_pair(blk)
        assert r1 == r2 and o1 == o2, (len(blk), r1, r2)


def xz_opt_ref(content: bytes, dict_lg: int = 23) -> bytes:
    """tests/hostcore/xz_opt_ref.cpp: the GPU optimal-parse xz coder restated."""
    h = host()
    h.zref_xz_opt_encode.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_char_p,
                                     ctypes.c_uint64]
    h.zref_xz_opt_encode.restype = ctypes.c_uint64
    cap = len(content) + len(content) // 16 + 4096
    out = ctypes.create_string_buffer(cap)
    k = h.zref_xz_opt_encode(content, len(content), dict_lg, out, cap)
    assert k > 0
    return out.raw[:k]


@pytest.mark.parametrize("kind", ["text", "uniform", "zeros", "randwalk", "small"])
def test_xz_opt_restatement_decodes_with_liblzma(kind):
    """The restated optimal-parse coder's streams decode with liblzma (the
    reference's decoder) across segment and LZMA2-chunk boundaries, stored
    (incompressible) chunks and state resets."""
    rng = np.random.default_rng(3)
    n = 600001
    if kind == "text":
        b = (b"the quick brown fox jumps over the lazy dog %d\n" * 20000)[:n]
    elif kind == "uniform":
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
    elif kind == "zeros":
        b = bytes(n)
    elif kind == "randwalk":
        b = np.cumsum(rng.integers(-3, 4, n // 2)).astype("<i2").tobytes()
    else:
        b = bytes(range(7))
    s = xz_opt_ref(b)
    assert lzma.decompress(s, format=lzma.FORMAT_XZ) == b
    if kind == "uniform":
        assert len(s) < n + n // 1000


def test_xz_opt_restatement_quant_ratio():
    """SURVEY §8(d) C2 "quant" chunks: the optimal parse reaches >= 97 % of
    liblzma preset 6's ratio (round-3 greedy coder: 87 %)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import quant_chunk
    tot = ours = ref = 0
    for i in range(2):
        v = quant_chunk(i).tobytes()
        s = xz_opt_ref(v)
        assert lzma.decompress(s, format=lzma.FORMAT_XZ) == v
        tot += len(v)
        ours += len(s)
        ref += len(lzma.compress(v, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6))
    assert tot / ours >= 0.97 * tot / ref, (tot / ours, tot / ref)


# ---- gzip encode: the zlib deflate_slow restatement (zcg_zlib_core.h) ------------
import zlib  # noqa: E402


def host_deflate(b: bytes, level: int) -> bytes:
    h = host()
    h.zz_host_deflate.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64]
    h.zz_host_deflate.restype = ctypes.c_int64
    cap = len(b) + len(b) // 8 + 1024
    out = ctypes.create_string_buffer(cap)
    n = h.zz_host_deflate(b, len(b), level, out, cap)
    assert n >= 0
    return out.raw[:n]


def zlib_raw(b: bytes, level: int) -> bytes:
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(b) + c.flush()


@pytest.mark.parametrize("level", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_zlib_core_matches_zlib(level):
    """The GPU gzip encoder's core driven serially: deflate_fast (levels 1-3:
    the greedy parse building its chains as it goes) and deflate_slow (4-9:
    match search per position, lazy parse), then trees: byte-identical to the
    system zlib 1.2.11 (the library flate2 wraps, gzip.rs:54-56) on mixed
    inputs, incl. window-slide and block-flush edges."""
    rng = np.random.default_rng(level)
    cases = [b"", b"a", b"abcabcabcabc", bytes(70000), rng.integers(0, 256, 20000, dtype=np.uint8).tobytes(),
             rng.integers(0, 4, 100000, dtype=np.uint8).tobytes(),
             (b"the quick brown fox jumps over the lazy dog " * 2000)[:65275],
             np.cumsum(rng.integers(-3, 4, 70000)).astype("<i2").tobytes(),
             (np.arange(60000) % 4096).astype("<i2").tobytes()]
    for b in cases:
        assert host_deflate(b, level) == zlib_raw(b, level), (level, len(b))


def test_zlib_core_matches_zlib_quant():
    """C5's 'quant' f32 chunk (1 MiB) at levels 1 and 6: zlib's bytes."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import quant_chunk
    b = quant_chunk(2).tobytes()
    for level in (1, 6):
        assert host_deflate(b, level) == zlib_raw(b, level)


def test_xz_sha256_core_matches_liblzma():
    """Check ID 10 (SHA-256) in the device core, host build: whole and partial
    reads, every byte of the digest corrupted, random corruptions."""
    rng = np.random.default_rng(23)
    for n in (0, 1, 55, 56, 63, 64, 65, 119, 120, 5000, 70000):
        payload = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
        s = lzma.compress(payload, format=lzma.FORMAT_XZ, check=lzma.CHECK_SHA256, preset=1)
        same(s, n)
        if n:
            same(s, n // 2 + 1)
        isz = (int.from_bytes(s[-8:-4], "little") + 1) * 4
        dend = len(s) - 12 - isz
        for k in range(32):
            b = bytearray(s)
            b[dend - 32 + k] ^= 1 << (k % 8)
            same(bytes(b), n)
        for _ in range(20):
            b = bytearray(s)
            b[int(rng.integers(0, len(s)))] ^= 1 << int(rng.integers(0, 8))
            same(bytes(b), n)
