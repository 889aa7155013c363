#!/usr/bin/env python3
"""Run one gzip bench-shaped batch with the inflate debug counters on."""
import ctypes, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import quant_chunk, gzip_flate2
from zarr_amd import ArrayMetadata, Gzip
from zarr_amd.batch import BatchCodec, PackedStreams
from zarr_amd import _native
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
streams = [gzip_flate2(quant_chunk(i).tobytes(), 6) for i in range(8)]
meta = ArrayMetadata.new([256, 256, 4], [256, 256, 4], "<f4", Gzip(6))
packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // 8)
codec = BatchCodec(0)
L = _native.load_library()
fn = L.zcg__debug_inflate_counters
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = np.zeros(32, np.uint64)
codec.decode(meta, packed)
torch.cuda.synchronize()
fn(out.ctypes.data, 1)
t0 = time.time()
codec.decode(meta, packed, flags=0x200)
torch.cuda.synchronize()
t1 = time.time()
fn(out.ctypes.data, 1)
names = ["rounds", "chain_lanes", "end_cap", "end_eob", "end_bad", "skips", "mrr_iters", "cuts",
         "blocks", "bytes", "tokens", "end_round", "pass2_tokens", "p2h_32_48", "p2h_48up", "p2_max",
         "cyc_hdr", "cyc_stage", "cyc_pass1", "cyc_pass2", "cyc_chain", "cyc_place", "cyc_lit",
         "cyc_mrr", "cyc_commit", "cyc_total", "hdr_pre", "hdr_walk", "hdr_post", "p2h_0_8", "p2h_8_16", "p2h_16_32"]
d = {k: int(v) for k, v in zip(names, out)}
d["n_chunks"] = packed.n
d["per_chunk"] = {k: round(v / packed.n, 2) for k, v in d.items() if k != "n_chunks"}
d["cycles_per_round"] = {k: round(d[k] / max(1, d["rounds"])) for k in names if k.startswith("cyc_")}
d["hdr_cycles_per_block"] = {k: round(d[k] / max(1, d["blocks"])) for k in ("hdr_pre", "hdr_walk", "hdr_post", "cyc_hdr")}
d["avg_chain"] = round(d["chain_lanes"] / max(1, d["rounds"]), 2)
d["mrr_per_round"] = round(d["mrr_iters"] / max(1, d["rounds"]), 2)
d["bytes_per_round"] = round(d["bytes"] / max(1, d["rounds"]), 1)
best = 1e9
for _ in range(3):
    t2 = time.time(); codec.decode(meta, packed); torch.cuda.synchronize(); t3 = time.time()
    best = min(best, t3 - t2)
t2, t3 = 0.0, best
d["ms_debug"] = round((t1 - t0) * 1e3, 2)
d["ms_nodebug"] = round((t3 - t2) * 1e3, 2)
d["status_ok"] = bool((packed.status.cpu().numpy() == 0).all())
print(json.dumps(d, indent=1))
