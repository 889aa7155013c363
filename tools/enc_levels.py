#!/usr/bin/env python3
"""Gzip write_chunk across levels on the GPU (zlib-exact coder): C5-shaped
batch (n 'quant' f32 1 MiB chunks), HIP-event time of the encode call, the
ratio, and 4 sampled streams compared with zlib's bytes (flate2 framing).
  usage: enc_levels.py [n] [levels, comma-separated]"""
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import gzip_flate2, quant_chunk  # noqa: E402
from zarr_amd import ArrayMetadata, Gzip  # noqa: E402
from zarr_amd.batch import BatchCodec, make_encode_batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
levels = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,3,6,9").split(",")]
pool = 64
vals = [quant_chunk(i) for i in range(pool)]
D = vals[0].nbytes
host = np.concatenate([vals[i % pool].view(np.uint8) for i in range(n)])
dev = torch.device("cuda:0")
elems = torch.from_numpy(host).to(dev)
bc = BatchCodec(0)
for level in levels:
    meta = ArrayMetadata.new([256 * 64, 256 * 64, 4], [256, 256, 4], "<f4", Gzip(level))
    cap = bc.encode_bound(meta, D)
    desc, dst, out_len, status = make_encode_batch(elems, n, cap, dev)
    s = torch.cuda.current_stream(dev)
    bc.encode(meta, desc, n, out_len, status, stream=s)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        bc.encode(meta, desc, n, out_len, status, stream=s)
        b.record(s)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ol = out_len.cpu().numpy()
    same = 0
    for i in sorted({0, 1, n // 2, n - 1}):
        got = dst[i * cap:i * cap + int(ol[i])].cpu().numpy().tobytes()
        same += int(got == gzip_flate2(vals[i % pool].tobytes(), level))
        assert zlib.decompress(got, 31) == vals[i % pool].tobytes()
    ms = float(np.median(ts))
    print(json.dumps({"level": level, "n": n, "ms": round(ms, 3), "gibs_input": round(n * D / 2**30 / (ms * 1e-3), 3),
                      "ratio": round(n * D / float(ol.sum()), 3), "bytes_equal_zlib_sample": f"{same}/4"}), flush=True)
    del desc, dst, out_len, status
