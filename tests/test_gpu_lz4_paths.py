"""ZCG_FLAG_LZ4_{WAVE,LANE}_PER_BLOCK: the two LZ4 block decoders (one lane per
block, picked for large batches; one wave per block, picked for small ones)
and the default pick must give the same bytes and statuses on valid,
truncated and corrupted frames (lz.rs:81-83 -> LZ4F_decompress), and all must
match the oracle."""
import os
import sys

import numpy as np
import pytest

from zarr_amd import ArrayMetadata, Lz4
from zarr_amd.batch import BatchCodec, PackedStreams

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import zref  # noqa: E402  (oracle: checker only)

pytestmark = pytest.mark.gpu

FLAG_WAVE = 0x800
FLAG_LANE = 0x1000


def _decode(streams, D, flags, dt="u1"):
    import torch
    meta = ArrayMetadata.new([D * len(streams)], [D], dt, Lz4(65536))
    packed = PackedStreams(streams, D, "cuda:0")
    BatchCodec(0).decode(meta, packed, flags=flags)
    torch.cuda.synchronize()
    return packed.status.cpu().numpy(), packed.dst.view(len(streams), -1).cpu().numpy()


def _payloads():
    rng = np.random.default_rng(44)
    walk = np.cumsum(rng.integers(-3, 4, 524288)).astype("<i2").tobytes()       # C4 shape
    far = np.empty(1 << 20, np.uint8)                                             # offsets 128 B .. 64 KiB
    base = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    far[:70000] = base[:70000]
    p = 70000
    while p < len(far):
        d, ln = int(rng.integers(100, 65535)), int(rng.integers(4, 90))
        ln = min(ln, len(far) - p)
        far[p:p + ln] = far[p - d:p - d + ln]
        if p + ln + 3 <= len(far):
            far[p + ln:p + ln + 3] = rng.integers(0, 256, 3, dtype=np.uint8)
        p += ln + 3
    runs = np.repeat(rng.integers(0, 4, 20000, dtype=np.uint8), rng.integers(1, 200, 20000))[: 1 << 20]
    runs = np.pad(runs, (0, (1 << 20) - len(runs)))
    return [walk, far.tobytes(), runs.tobytes(), rng.integers(0, 256, 1 << 20, dtype=np.uint8).tobytes()]


def test_lane_and_wave_decoders_agree():
    D = 1 << 20
    pays = _payloads()
    streams = [zref.encode(zref.LZ4, 65536, np.frombuffer(p, np.uint8))[1] for p in pays]
    rng = np.random.default_rng(5)
    extra = [streams[0][: len(streams[0]) // 3]]
    for _ in range(60):
        b = bytearray(streams[int(rng.integers(0, 3))])
        b[int(rng.integers(7, len(b)))] ^= int(rng.integers(1, 256))
        extra.append(bytes(b))
    allst = streams + extra
    s0, o0 = _decode(allst, D, FLAG_LANE)
    s1, o1 = _decode(allst, D, FLAG_WAVE)
    s2, o2 = _decode(allst, D, 0)
    assert s0.tolist() == s1.tolist() == s2.tolist()
    for i, p in enumerate(pays):
        assert s0[i] == 0 and bytes(o0[i]) == p and bytes(o1[i]) == p and bytes(o2[i]) == p
    for i, st in enumerate(allst):
        ost, ref = zref.decode(zref.LZ4, st, D, 1)
        assert ost == s0[i], i
        if ost == 0:
            assert bytes(o0[i]) == ref and bytes(o1[i]) == ref and bytes(o2[i]) == ref


FRAMES = {"reference": {}, "linked": dict(linked=True), "block_checksum": dict(block_checksum=True),
          "content_size": dict(content_size=True), "bd256k": dict(block_size_id=5),
          "bd4m": dict(block_size_id=7), "small_blocks": dict(auto_flush=True, feed=10000)}


@pytest.mark.parametrize("flags", [0, FLAG_LANE], ids=["default", "lane"])
@pytest.mark.parametrize("frame", list(FRAMES))
def test_decoder_frame_variants(frame, flags):
    """Every frame layout the reference decoder accepts, through the default
    and the lane decoder, at full length and truncating read_exact lengths."""
    pays = _payloads()
    streams = []
    for p in pays:
        if frame == "reference":
            streams.append(zref.encode(zref.LZ4, 65536, np.frombuffer(p, np.uint8))[1])
        else:
            streams.append(zref.lz4_frame_custom(p, **FRAMES[frame]))
    for D in (1 << 20, (1 << 20) - 1000, 65536 * 3, 65536 * 3 + 7):
        st, out = _decode(streams, D, flags)
        for i, s in enumerate(streams):
            ost, ref = zref.decode(zref.LZ4, s, D, 1)
            assert ost == st[i], (frame, D, i)
            if ost == 0:
                assert bytes(out[i]) == ref, (frame, D, i)


def test_side_by_side_batch_agrees():
    """8 192 chunks = 131 072 blocks: the default runs the lane and the wave
    decoders side by side on two streams (lanes for the first 55 % of the
    chunks); statuses and bytes must equal the lane decoder's alone, valid and
    corrupted frames alike."""
    import torch
    D = 1 << 20
    pays = _payloads()
    streams = [zref.encode(zref.LZ4, 65536, np.frombuffer(p, np.uint8))[1] for p in pays]
    rng = np.random.default_rng(9)
    while len(streams) < 64:
        b = bytearray(streams[int(rng.integers(0, 4))])
        b[int(rng.integers(7, len(b)))] ^= int(rng.integers(1, 256))
        streams.append(bytes(b))
    n = 8192
    meta = ArrayMetadata.new([D * n], [D], "u1", Lz4(65536))
    packed = PackedStreams(streams, D, "cuda:0", slot_copies=n // 64)
    assert packed.n == n
    codec = BatchCodec(0)
    codec.decode(meta, packed, flags=FLAG_LANE)
    torch.cuda.synchronize()
    st_lane, out_lane = packed.status.clone(), packed.dst.clone()
    packed.dst.zero_()
    codec.decode(meta, packed, flags=0)
    torch.cuda.synchronize()
    assert torch.equal(packed.status, st_lane)
    ok = (st_lane == 0).view(-1, 1)
    for c0 in range(0, n, 1024):  # (in slices: the products are 1 GiB each)
        assert torch.equal(packed.dst.view(n, -1)[c0:c0 + 1024] * ok[c0:c0 + 1024],
                           out_lane.view(n, -1)[c0:c0 + 1024] * ok[c0:c0 + 1024])
    del out_lane
    for i in range(4):  # the valid payloads, wherever their copies landed
        rows = [g for g in range(n) if g % 64 == i][:8]
        for g in rows:
            assert bytes(packed.dst.view(n, -1)[g].cpu().numpy()) == pays[i]
