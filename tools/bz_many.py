#!/usr/bin/env python3
"""Bzip2 encode of batches with many blocks per sort sub-batch: which chunks
fail to decode with libbz2 (Python bz2).  Usage: bz_many.py"""
import bz2
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_encode import _data, encode_batch  # noqa: E402
from zarr_amd import ArrayMetadata  # noqa: E402
from zarr_amd.compression import Bzip2  # noqa: E402

D = 1 << 20
kinds = ["randwalk", "text", "mixed", "uniform"]
for name, n, level, kk in (("u28", 28, 1, ["uniform"]), ("mix12", 12, 1, kinds), ("mix24", 24, 1, kinds),
                           ("mix28", 28, 1, kinds), ("rw28", 28, 1, ["randwalk"]), ("mix28_l9", 28, 9, kinds)):
    arrays = [_data(kk[i % len(kk)], D, seed=i) for i in range(n)]
    meta = ArrayMetadata.new([D * n], [D], "u1", Bzip2(level))
    st, outs = encode_batch(meta, arrays)
    bad = []
    for i, (a, s) in enumerate(zip(arrays, outs)):
        try:
            ok = bz2.decompress(s) == a.tobytes()
        except Exception:
            ok = False
        if not ok:
            bad.append(i)
    print(json.dumps({"case": name, "status_ok": int((st == 0).sum()), "bad": bad}), flush=True)
