#!/usr/bin/env python3
"""Xz encode (preset 6, the optimal-parse coder) of n C2 quant chunks: HIP-event
time (median of 3), ratio, liblzma decode of a sample, and — with a library
built with -DXO_PROF=1 (tools/build_variants.sh) — the coder's phase counters.
Usage: ZCG_LIB=... python tools/xz_stats.py [n]"""
import ctypes
import json
import lzma
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from bench import quant_chunk  # noqa: E402
from zarr_amd import ArrayMetadata, _native  # noqa: E402
from zarr_amd.batch import BatchCodec, make_encode_batch  # noqa: E402
from zarr_amd.compression import Xz  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
pool = 64
vals = [quant_chunk(i) for i in range(pool)]
D = vals[0].nbytes
meta = ArrayMetadata.new([256 * n, 256, 4], [256, 256, 4], "<f4", Xz(6))
host = np.concatenate([vals[i % pool].view(np.uint8) for i in range(n)])
elems = torch.from_numpy(host).to("cuda:0")
codec = BatchCodec(0)
cap = codec.encode_bound(meta, D)
desc, dst, out_len, status = make_encode_batch(elems, n, cap, "cuda:0")
lib = _native.load_library()
prof = getattr(lib, "zcg__debug_xz_opt_counters", None)
buf = (ctypes.c_ulonglong * 16)()
if prof:
    prof(buf, 1)
codec.encode(meta, desc, n, out_len, status)
torch.cuda.synchronize()
cnt = list(buf)
if prof:
    prof(buf, 1)
    cnt = list(buf)
st = status.cpu().numpy()
ol = out_len.cpu().numpy()
ratio = n * D / float(ol.sum())
sample = dst.view(n, cap)[:4].cpu().numpy()
ok = all(lzma.decompress(sample[i, :ol[i]].tobytes(), format=lzma.FORMAT_XZ) == vals[i % pool].tobytes()
         for i in range(min(4, n)))
ts = []
for _ in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    codec.encode(meta, desc, n, out_len, status)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
ms = float(np.median(ts))
res = {"n": n, "ms": round(ms, 2), "gibs": round(n * D / 2**30 / (ms * 1e-3), 3), "ratio": round(ratio, 4),
       "status_ok": int((st == 0).sum()), "sample_decodes": ok}
if prof and cnt[5]:
    seg = int(os.environ.get("XO_SEG_KB", "256")) << 10
    segs = n * ((D + seg - 1) // seg)
    res["prof"] = {"plan_share": round(cnt[0] / cnt[5], 3), "code_share": round(cnt[1] / cnt[5], 3),
                   "cycles_per_node_plan": round(cnt[0] / max(1, cnt[2]), 1),
                   "cycles_per_symbol_code": round(cnt[1] / max(1, cnt[3]), 1),
                   "nodes": cnt[2], "symbols": cnt[3], "windows": cnt[4],
                   "kcycles_per_segment": round(cnt[5] / segs / 1e3, 1),
                   "segment_ms": round(cnt[6] / segs / 1e5, 2),
                   "effective_ghz": round(cnt[5] / max(1, cnt[6]) / 10, 3)}
    if cnt[15]:
        t0 = (~cnt[14]) & (2**64 - 1)
        res["prof"].update({"max_wave_ms": round(cnt[7] / 1e5, 2), "start_spread_ms": round((cnt[13] - t0) / 1e5, 2),
                            "span_ms": round((cnt[15] - t0) / 1e5, 2)})
    if cnt[8]:
        names = ["next_node_and_issue", "reps", "lit_flags", "arc_setup", "arc_price_relax"]
        res["prof"]["node_cycles"] = {k: round(cnt[8 + q] / max(1, cnt[2]), 1) for q, k in enumerate(names)}
print(json.dumps(res), flush=True)
