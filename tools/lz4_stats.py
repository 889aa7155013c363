#!/usr/bin/env python3
"""LZ4 block-decoder phase counters (ZCG_FLAG_DEBUG_COUNTERS; needs a -DLZ_DBG=1 build) on C4-shaped
chunks: liblz4 streams with lz4-rs settings, n chunks (GPU box)."""
import ctypes, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import lz4rs_frame, randwalk_chunk
from zarr_amd import ArrayMetadata, Lz4, _native
from zarr_amd.batch import BatchCodec, PackedStreams
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sel = int(sys.argv[2], 0) if len(sys.argv) > 2 else 0  # decoder flags (0x800 wave, 0x1000 lane)
streams = [lz4rs_frame(randwalk_chunk(i).tobytes()) for i in range(64)]
meta = ArrayMetadata.new([128, 64, 64], [128, 64, 64], "<i2", Lz4(65536))
packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // 64)
codec = BatchCodec(0)
L = _native.load_library()
fn = L.zcg__debug_lz4_counters
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = np.zeros(16, np.uint64)
codec.decode(meta, packed, flags=sel); torch.cuda.synchronize()
fn(out.ctypes.data, 1)
t0 = time.time(); codec.decode(meta, packed, flags=0x200 | sel); torch.cuda.synchronize(); t1 = time.time()
fn(out.ctypes.data, 1)
names = ["steps", "heavy_steps", "bytes", "cyc_parse", "cyc_chain", "cyc_entries", "cyc_finish", "cyc_total"]
d = {k: int(v) for k, v in zip(names, out)}
st = d["steps"]
d["per_step"] = {k: round(d[k] / st, 1) for k in names if k.startswith("cyc_")}
d["bytes_per_step"] = round(d["bytes"] / st, 1)
d["heavy_frac"] = round(d["heavy_steps"] / st, 4)
best = 1e9
for _ in range(3):
    t2 = time.time(); codec.decode(meta, packed, flags=sel); torch.cuda.synchronize(); best = min(best, time.time() - t2)
d["ms_debug"] = round((t1 - t0) * 1e3, 2); d["ms_nodebug"] = round(best * 1e3, 2)
d["status_ok"] = bool((packed.status.cpu().numpy() == 0).all())
print(json.dumps(d, indent=1))
