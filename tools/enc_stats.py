#!/usr/bin/env python3
"""Time the GPU encoders per data distribution (kernel time via HIP events),
with the CPU reference library's ratio on the same data for comparison.
    python tools/enc_stats.py [n_chunks] [lz4|gzip|xz|bzip2]"""
import os, sys, json, zlib, bz2, lzma, hashlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from bench import randwalk_chunk, quant_chunk
from zarr_amd import ArrayMetadata, Lz4, Gzip
from zarr_amd.compression import Bzip2, Xz
from zarr_amd.batch import BatchCodec, make_encode_batch
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
codec = sys.argv[2] if len(sys.argv) > 2 else "lz4"
D = 1 << 20
gens = {"zeros": lambda i: np.zeros(D, np.uint8), "uniform": lambda i: np.random.default_rng(i).integers(0, 256, D, dtype=np.uint8),
        "randwalk": lambda i: randwalk_chunk(i).view(np.uint8), "quant": lambda i: quant_chunk(i).view(np.uint8)}
bc = BatchCodec(0)
meta = ArrayMetadata.new([D * n], [D], "u1", {"lz4": Lz4(65536), "gzip": Gzip(6), "xz": Xz(6),
                                             "bzip2": Bzip2(9)}[codec])
for name, g in gens.items():
    pool = [g(i) for i in range(16)]
    elems = torch.from_numpy(np.concatenate([pool[i % 16] for i in range(n)])).cuda()
    cap = bc.encode_bound(meta, D)
    desc, dst, ol, st = make_encode_batch(elems, n, cap, "cuda:0")
    bc.encode(meta, desc, n, ol, st); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3): bc.encode(meta, desc, n, ol, st)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    ref = None
    if codec == "gzip":
        ref = round(4 * D / sum(len(zlib.compress(pool[i].tobytes(), 6)) for i in range(4)), 3)
    elif codec == "bzip2":
        ref = round(4 * D / sum(len(bz2.compress(pool[i].tobytes(), 9)) for i in range(4)), 3)
    elif codec == "xz":
        ref = round(4 * D / sum(len(lzma.compress(pool[i].tobytes(), preset=6)) for i in range(4)), 3)
    olc = ol.cpu().numpy()
    dcpu = dst.view(n, -1)[:, :int(olc.max())].cpu().numpy() if n else None
    h = hashlib.sha1()
    for i in range(n): h.update(dcpu[i, :int(olc[i])].tobytes())
    print(json.dumps({"codec": codec, "data": name, "sha1": h.hexdigest()[:16], "ms": round(ms, 2), "GiBps": round(n * D / ms / 1e-3 / 2**30, 2),
                      "ratio": round(n * D / float(ol.sum().item()), 3), "ref_ratio": ref,
                      "ok": bool((st == 0).all().item())}), flush=True)
