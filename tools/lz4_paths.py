#!/usr/bin/env python3
"""LZ4 decode of n C4-shaped chunks (liblz4 streams with lz4-rs settings)
through each block decoder: HIP-event time (median of 3) and a parity check
of every chunk against its input.  Usage: lz4_paths.py n1 n2 ..."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import lz4rs_frame, randwalk_chunk
from zarr_amd import ArrayMetadata, Lz4
from zarr_amd.batch import BatchCodec, PackedStreams
pool = 64
vals = [randwalk_chunk(i) for i in range(pool)]
streams = [lz4rs_frame(v.tobytes()) for v in vals]
meta = ArrayMetadata.new([128, 64, 64], [128, 64, 64], "<i2", Lz4(65536))
ref = torch.from_numpy(np.stack([v.view(np.uint8) for v in vals])).to("cuda:0")
codec = BatchCodec(0)
paths = os.environ.get("LZ4_PATHS", "default,lane,wave").split(",")
for n in [int(x) for x in sys.argv[1:]] or [8192]:
    packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // pool)
    for tag, fl in [(t, {"default": 0, "lane": 0x1000, "wave": 0x800}[t]) for t in paths]:
        packed.dst.zero_()
        codec.decode(meta, packed, flags=fl)
        torch.cuda.synchronize()
        ok = int((packed.status.cpu().numpy() == 0).sum())
        out = packed.dst.view(packed.n, 1 << 20)
        bad = 0
        for c0 in range(0, packed.n, 512):
            idx = torch.arange(c0, min(c0 + 512, packed.n), device="cuda:0") % pool
            bad += int((out[c0:c0 + 512] != ref[idx]).any(dim=1).sum().item())
        ts = []
        for _ in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); codec.decode(meta, packed, flags=fl); b.record(); torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = float(np.median(ts))
        print(json.dumps({"n": packed.n, "path": tag, "ms": round(ms, 3), "gibs": round(packed.n / 1024 / (ms * 1e-3), 1),
                          "status_ok": ok, "bad_chunks": bad}), flush=True)
    del packed
    torch.cuda.empty_cache()
