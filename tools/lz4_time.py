#!/usr/bin/env python3
"""HIP-event time of the LZ4 decode of n C4-shaped chunks (liblz4 streams
with lz4-rs settings), with no parity gate: for diagnostic builds whose
output is knowingly wrong (variants/*.so via ZCG_LIB).  Usage:
lz4_time.py n [flags]"""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import lz4rs_frame, randwalk_chunk
from zarr_amd import ArrayMetadata, Lz4
from zarr_amd.batch import BatchCodec, PackedStreams
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
flags = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0
streams = [lz4rs_frame(randwalk_chunk(i).tobytes()) for i in range(64)]
meta = ArrayMetadata.new([128, 64, 64], [128, 64, 64], "<i2", Lz4(65536))
packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // 64)
codec = BatchCodec(0)
codec.decode(meta, packed, flags=flags)
torch.cuda.synchronize()
ts = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); codec.decode(meta, packed, flags=flags); b.record(); torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ms = float(np.median(ts))
print(json.dumps({"lib": os.path.basename(os.environ.get("ZCG_LIB", "intree")), "n": packed.n, "ms": round(ms, 3),
                  "gibs": round(packed.n / 1024 / (ms * 1e-3), 1)}))
