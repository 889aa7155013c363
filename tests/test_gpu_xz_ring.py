"""ZCG_FLAG_XZ_RING_32K: the xz decoder with 32 KiB of LDS history must give
the same bytes and statuses as the default 4 KiB history (xz.rs:34-43 ->
liblzma), on long-distance data, all check types and truncated streams."""
import lzma

import numpy as np
import pytest

from zarr_amd import ArrayMetadata
from zarr_amd.batch import BatchCodec, PackedStreams
from zarr_amd.compression import Xz

pytestmark = pytest.mark.gpu

FLAG_RING_32K = 0x400


def _data(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "far":  # repeats 4-60 KiB back: matches beyond both histories
        base = rng.integers(0, 256, 65536, dtype=np.uint8)
        out = np.empty(n, np.uint8)
        p = 0
        while p < n:
            d = int(rng.integers(4096, 61440))
            ln = min(int(rng.integers(8, 300)), n - p)
            src = base if p < d else out[p - d:p - d + ln]
            out[p:p + ln] = src[:ln] if p >= d else base[:ln]
            p += ln
        return out
    return (np.cumsum(rng.integers(-2, 3, n)) % 97).astype(np.uint8)


def _decode(streams, D, flags):
    import torch
    meta = ArrayMetadata.new([D * len(streams)], [D], "u1", Xz(6))
    packed = PackedStreams(streams, D, "cuda:0")
    BatchCodec(0).decode(meta, packed, flags=flags)
    torch.cuda.synchronize()
    return packed.status.cpu().numpy(), packed.dst.view(len(streams), -1).cpu().numpy()


@pytest.mark.parametrize("kind", ["far", "walk"])
@pytest.mark.parametrize("check", [lzma.CHECK_CRC64, lzma.CHECK_CRC32, lzma.CHECK_NONE])
def test_ring_32k_matches_default(kind, check):
    D = 1 << 20
    datas = [_data(kind, D, s) for s in range(4)]
    streams = [lzma.compress(d.tobytes(), format=lzma.FORMAT_XZ, check=check, preset=6) for d in datas]
    streams.append(streams[0][: len(streams[0]) // 2])  # truncated -> UnexpectedEof
    s0, o0 = _decode(streams, D, 0)
    s1, o1 = _decode(streams, D, FLAG_RING_32K)
    assert s0.tolist() == s1.tolist()
    assert s0[:4].tolist() == [0, 0, 0, 0] and s0[4] == 1
    for i in range(4):
        assert np.array_equal(o0[i], datas[i]) and np.array_equal(o1[i], datas[i])
