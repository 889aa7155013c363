"""GPU parity of the Bzip2 decoder (zcg_bz2.hip) against the oracle.

The reference decodes Bzip2 with bzip2-rs read::BzDecoder (src/compression/
bzip.rs:35-46) = libbz2 1.0.x; the oracle runs that libbz2 with the same
32 KiB input windows.  Streams come from the oracle encoder (BzEncoder,
blockSize 1..9) and Python's bz2 (the same libbz2).  The serial stage shared
with the kernel is fuzzed on the CPU in tests/test_hostcore.py; here the
parallel inverse BWT / RLE1 / CRC stages run on real blocks, and the
corruption sweeps run in batches.
"""
import bz2

import numpy as np
import pytest

import zref
from test_gpu_parity import DATASETS, check, check_many, rw

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("data", list(DATASETS))
@pytest.mark.parametrize("level", [1, 9])
def test_bzip2_large(data, level):
    payload = DATASETS[data]()
    st, s = zref.encode(zref.BZIP2, level, np.frombuffer(payload, np.uint8))
    assert st == zref.OK
    for D in (len(payload), len(payload) // 3 + 7, 100000 * level):
        if D <= len(payload):
            check("bzip2", s, "u1", D, param=level)


@pytest.mark.parametrize("meta_level", [1, 4])
def test_bzip2_blocks_larger_than_metadata_level(meta_level):
    """The stage-B kept-byte region is sized from the array's level; a stream
    written at level 9 under level-1/4 metadata keeps fewer bytes per walk
    and must decode the same (the reference ignores the level on read)."""
    payload = b"".join(rw(450000, seed=s).tobytes() for s in range(2)) + bytes(300000)
    s = bz2.compress(payload, 9)
    for D in (len(payload), 900001, 123457):
        check("bzip2", s, "u1", D, param=meta_level)
    check_many("bzip2", [s, bz2.compress(payload[:500000], 9)], "u1", 500000, param=meta_level)


@pytest.mark.parametrize("dt", ["<i2", ">i2", ">f4", ">u8", "bool", "i1"])
def test_bzip2_transform(dt):
    from golden_util import dtype_info
    es = dtype_info(dt)[0]
    n = 70001
    raw = rw(n * es // 2 + 1).tobytes()[: n * es]
    st, s = zref.encode(zref.BZIP2, 9, np.frombuffer(raw, np.uint8))
    check("bzip2", s, dt, n)


def test_bzip2_runs_and_rle1_edges():
    """Long RUNA/RUNB runs, RLE1 count bytes of 0..255, runs across blocks."""
    rng = np.random.default_rng(4)
    parts = [bytes([7]) * 4, bytes([9]) * 259, bytes(100000), bytes([1, 1, 1, 1, 2]) * 1000,
             rng.integers(0, 256, 5000, dtype=np.uint8).tobytes(), bytes([3]) * 1000000]
    payload = b"".join(parts)
    for level in (1, 5, 9):
        s = bz2.compress(payload, level)
        for D in (len(payload), 100000 * level, 100000 * level + 1, 777777):
            check("bzip2", s, "u1", min(D, len(payload)))


def test_bzip2_corruption_sweep():
    rng = np.random.default_rng(23)
    for k, payload in enumerate([rw(30000, seed=1).tobytes(), bytes(50000),
                                 rng.integers(0, 256, 40000, dtype=np.uint8).tobytes()]):
        s = bz2.compress(payload, (9, 1, 5)[k])
        for D in (len(payload), len(payload) // 2):
            streams = [s[:int(t)] for t in rng.integers(0, len(s), 48)]
            for _ in range(208):
                b = bytearray(s)
                if rng.random() < 0.3:
                    p = len(b) - 1 - int(rng.integers(0, min(len(b), 32)))
                else:
                    p = int(rng.integers(0, len(b)))
                b[p] ^= int(rng.integers(1, 256))
                streams.append(bytes(b))
            check_many("bzip2", streams, "u1", D)


def test_bzip2_two_streams_one_context():
    """Batches enqueued on two HIP streams of one context must not share the
    decoder's scratch (zcg_ctx keeps a workspace per stream)."""
    import torch
    from zarr_amd import ArrayMetadata
    from zarr_amd.batch import BatchCodec, PackedStreams
    from zarr_amd.compression import Bzip2
    D = 300000
    vals = [rw(D // 2, seed=s).tobytes() for s in range(6)]
    streams = [bz2.compress(v, 9) for v in vals]
    meta = ArrayMetadata.new([D * 6], [D], "u1", Bzip2(9))
    codec = BatchCodec(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    p1 = PackedStreams(streams[:3], D, "cuda:0", slot_copies=8)
    p2 = PackedStreams(streams[3:], D, "cuda:0", slot_copies=8)
    for _ in range(2):
        codec.decode(meta, p1, stream=s1)
        codec.decode(meta, p2, stream=s2)
    torch.cuda.synchronize()
    for p, base in ((p1, 0), (p2, 3)):
        assert (p.status.cpu().numpy() == 0).all()
        out = p.dst.cpu().numpy().reshape(p.n, D)
        for i in range(p.n):
            assert out[i].tobytes() == vals[base + i % 3]


def test_bzip2_mixed_batch():
    """A 640-chunk batch of valid, truncated and corrupted streams (several
    rounds' worth of pending / finished chunks side by side) vs the oracle."""
    rng = np.random.default_rng(31)
    payloads = [rw(60000, seed=s).tobytes() for s in range(4)] + [bytes(120000)]
    base = [bz2.compress(p, 1 + 4 * (i % 3)) for i, p in enumerate(payloads)]
    streams = []
    for i in range(640):
        s = base[i % len(base)]
        u = rng.random()
        if u < 0.15:
            s = s[:int(rng.integers(0, len(s)))]
        elif u < 0.35:
            b = bytearray(s)
            b[int(rng.integers(0, len(b)))] ^= int(rng.integers(1, 256))
            s = bytes(b)
        streams.append(s)
    for D in (120000, 60000):
        check_many("bzip2", streams, "u1", D)
