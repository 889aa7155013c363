#!/usr/bin/env python3
"""One bench-shaped bzip2 decode batch with the stage timers read back
(g_bz_dbg: cycles summed over blocks, stamped by thread 0 of each workgroup)."""
import bz2, ctypes, json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import quant_chunk
from zarr_amd import ArrayMetadata
from zarr_amd.compression import Bzip2
from zarr_amd.batch import BatchCodec, PackedStreams
from zarr_amd import _native
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
streams = [bz2.compress(quant_chunk(i).tobytes(), 9) for i in range(8)]
meta = ArrayMetadata.new([256, 256, 4], [256, 256, 4], "<f4", Bzip2(9))
packed = PackedStreams(streams, 1 << 20, "cuda:0", slot_copies=n // 8)
codec = BatchCodec(0)
fn = _native.load_library().zcg__debug_bz2_counters
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
out = np.zeros(8, np.uint64)
codec.decode(meta, packed)
torch.cuda.synchronize()
fn(out.ctypes.data, 1)
t0 = time.time()
st = codec.decode(meta, packed)
torch.cuda.synchronize()
ms = (time.time() - t0) * 1e3
fn(out.ctypes.data, 1)
names = ["stage_a", "sort", "walk1", "rank", "walk2", "rle_out_crc"]
blocks = max(1, int(out[6]))
print(json.dumps({"n_chunks": n, "ms": round(ms, 2), "blocks": blocks,
                  "kcycles_per_block": {k: round(int(v) / blocks / 1e3, 1) for k, v in zip(names, out)}}, indent=1))
