#!/usr/bin/env python3
"""xz decode of the bench batch with the 4 KiB and the 32 KiB LDS history
(ZCG_FLAG_XZ_RING_32K): time per batch and bit-exactness against the default.
usage: xz_ring.py N [4k|32k|both]"""
import lzma, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import quant_chunk
from zarr_amd import ArrayMetadata
from zarr_amd.compression import Xz
from zarr_amd.batch import BatchCodec, PackedStreams
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
which = sys.argv[2] if len(sys.argv) > 2 else "both"
streams = [lzma.compress(quant_chunk(i).tobytes(), format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6)
           for i in range(8)]
meta = ArrayMetadata.new([256, 256, 4], [256, 256, 4], "<f4", Xz(6))
packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // 8)
codec = BatchCodec(0)
import numpy as np
want = [np.frombuffer(lzma.decompress(x), np.uint8) for x in streams]
res = {}
for name, fl in (("4k", 0), ("32k", 0x400)):
    if which not in (name, "both"):
        continue
    codec.decode(meta, packed, flags=fl)
    torch.cuda.synchronize()
    t0 = time.time()
    codec.decode(meta, packed, flags=fl)
    torch.cuda.synchronize()
    res[name + "_ms"] = round((time.time() - t0) * 1e3, 2)
    assert int((packed.status != 0).sum()) == 0, name
    out = packed.dst.view(packed.n, -1).cpu().numpy()
    for i in range(0, packed.n, max(1, packed.n // 64)):
        assert np.array_equal(out[i], want[i % 8]), (name, i)
    res[name + "_exact"] = True
print(res)
