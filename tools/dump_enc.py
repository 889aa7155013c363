#!/usr/bin/env python3
"""Debug helper: GPU-encode one chunk and save input + stream under gpurun_out/."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch
from test_gpu_encode import _data, encode_batch
from zarr_amd import ArrayMetadata, Gzip
kind, level = sys.argv[1], int(sys.argv[2])
D = 1 << 20
a = _data(kind, D, 0)
meta = ArrayMetadata.new([D], [D], "u1", Gzip(level))
st, outs = encode_batch(meta, [a])
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
open(os.path.join(ROOT, "gpurun_out", f"enc_{kind}_{level}.gz"), "wb").write(outs[0])
print(st, len(outs[0]))
