#!/usr/bin/env python3
"""The bench's C2 gzip batch (4 096 chunks from the 64-chunk pool, one HBM
slot each, bench.py decode_leg layout) decoded by the one-wave-per-chunk
kernel 3 times (1 warm + 2; argv[1]: chunks, default 4 096), for rocprofv3 --pmc passes over timing-only
ablation builds (tools/iw_ablate.py): unlike bench.py it does not stop on a
wrong chunk, it only reports how many differ.  ZCG_LIB picks the build."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import host_encode, quant_chunk
from zarr_amd import ArrayMetadata, Gzip
from zarr_amd.batch import BatchCodec
from zarr_amd import _native

n, pool, D = (int(sys.argv[1]) if len(sys.argv) > 1 else 4096), 64, 1 << 20
vals = [quant_chunk(i) for i in range(pool)]
streams = host_encode("gzip", vals, 16)
meta = ArrayMetadata.new([256 * 64, 256 * 64, 4], [256, 256, 4], "<f4", Gzip(6))
dev = torch.device("cuda:0")
order = np.arange(n) % pool
lens = np.array([len(s) for s in streams], np.int64)
slot = int((lens.max() + 255) // 256 * 256)
hp = np.zeros((pool, slot), np.uint8)
for u, s in enumerate(streams):
    hp[u, :len(s)] = np.frombuffer(s, np.uint8)
src = torch.from_numpy(hp).to(dev).index_select(0, torch.from_numpy(order).to(dev))
dst = torch.empty(n * D, dtype=torch.uint8, device=dev)
desc = np.stack([src.data_ptr() + np.arange(n, dtype=np.uint64) * slot, lens[order].astype(np.uint64),
                 dst.data_ptr() + np.arange(n, dtype=np.uint64) * D, np.full(n, D, np.uint64)], 1)


class _P:
    pass


packed = _P()
packed.n = n
packed.desc = torch.from_numpy(np.ascontiguousarray(desc).view(np.int64)).to(dev)
packed.status = torch.full((n,), -1, dtype=torch.int32, device=dev)
bc = BatchCodec(0)
ms = []
for i in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    bc.decode(meta, packed, flags=_native.FLAG_INFLATE_WAVE)
    b.record()
    torch.cuda.synchronize()
    ms.append(a.elapsed_time(b))
ref = torch.from_numpy(np.stack([v.view(np.uint8) for v in vals])).to(dev)
out = dst.view(n, D)
bad = sum(int((out[c0:c0 + 256] != ref[torch.arange(c0, c0 + 256, device=dev) % pool]).any(dim=1).sum().item())
          for c0 in range(0, n, 256))
print(json.dumps({"n": n, "lib": os.environ.get("ZCG_LIB", "in-tree"), "ms": [round(x, 3) for x in ms],
                  "status_ok": int((packed.status == 0).sum().item()), "bad_chunks": bad,
                  "compressed_bytes": int(lens[order].sum())}))
