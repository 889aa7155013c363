#!/usr/bin/env python3
"""C2-shaped gzip batch through the one-wave-per-chunk inflate kernel: parity
of every chunk against its input, HIP-event time of the default kernel vs the
256-lane round kernel (ZCG_FLAG_INFLATE_BLOCK_PAR), and the wave kernel's
debug counters (ZCG_FLAG_DEBUG_COUNTERS).  Usage: iw_stats.py [n_chunks]"""
import ctypes, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import quant_chunk, gzip_flate2
from zarr_amd import ArrayMetadata, Gzip
from zarr_amd.batch import BatchCodec, PackedStreams
from zarr_amd import _native

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
pool = 64
vals = [quant_chunk(i) for i in range(pool)]
streams = [gzip_flate2(v.tobytes(), 6) for v in vals]
meta = ArrayMetadata.new([256, 256, 4], [256, 256, 4], "<f4", Gzip(6))
packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // pool)
codec = BatchCodec(0)
ref = torch.from_numpy(np.stack([v.view(np.uint8) for v in vals])).to("cuda:0")
res = {"n": packed.n}


def check(tag):
    st = packed.status.cpu().numpy()
    out = packed.dst.view(packed.n, 1 << 20)
    bad = 0
    for c0 in range(0, packed.n, 256):
        idx = torch.arange(c0, min(c0 + 256, packed.n), device="cuda:0") % pool
        bad += int((out[c0:c0 + 256] != ref[idx]).any(dim=1).sum().item())
    res[tag + "_status_ok"] = int((st == 0).sum())
    res[tag + "_bad_chunks"] = bad


def timed(flags, reps=5):
    codec.decode(meta, packed, flags=flags)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        codec.decode(meta, packed, flags=flags)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return round(min(ts), 3), round(float(np.median(ts)), 3)


for tag, fl in (("wave", _native.FLAG_INFLATE_WAVE), ("blockpar", _native.FLAG_INFLATE_BLOCK_PAR)):
    packed.dst.zero_()
    mn, med = timed(fl)
    check(tag)
    res[tag + "_ms_min"], res[tag + "_ms_med"] = mn, med
    res[tag + "_gibs"] = round(packed.n / 1024 / (med * 1e-3), 2)

L = _native.load_library()
fn = L.zcg__debug_inflate_wave_counters
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = np.zeros(32, np.uint64)
fn(out.ctypes.data, 1)
codec.decode(meta, packed, flags=_native.FLAG_DEBUG_COUNTERS | _native.FLAG_INFLATE_WAVE)
torch.cuda.synchronize()
fn(out.ctypes.data, 1)
names = {0: "rounds", 1: "blocks", 2: "stages", 3: "groups", 4: "p1_lane_it", 5: "p2_lane_it", 6: "chain",
         7: "spare", 8: "caps", 9: "rounds_no_eob", 10: "cyc_hdr", 11: "cyc_p1", 12: "cyc_p2",
         13: "cyc_chain", 14: "cyc_classify", 15: "cyc_far", 16: "cyc_near", 17: "cyc_place", 18: "cyc_commit",
         19: "cyc_total", 20: "far_iters", 21: "near_batches", 22: "near_passes", 23: "near_straddle_batches", 24: "cyc_hdr_tables", 25: "cyc_refetch", 26: "cyc_eob", 27: "cyc_hdr_walk"}
d = {v: int(out[k]) for k, v in names.items()}
res["per_chunk"] = {k: round(v / packed.n, 1) for k, v in d.items()}
cyc = {k: v for k, v in d.items() if k.startswith("cyc_") and k not in ("cyc_total", "cyc_hdr_tables", "cyc_hdr_walk")}
tot = max(1, sum(cyc.values()))
res["cycle_share"] = {k: round(v / tot, 3) for k, v in cyc.items()}
res["kcyc_per_chunk_total"] = round(d["cyc_total"] / packed.n / 1e3, 1)
print(json.dumps(res, indent=1))
