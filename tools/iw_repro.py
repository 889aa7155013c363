#!/usr/bin/env python3
"""Decode one test_gzip_large stream with the wave kernel (flag 0x4000) and
print the status; with a ZIW_TRACE build (variants/<name>.so via ZCG_LIB)
the kernel printfs its rounds / chains / failures.  Debug tooling only.
    python tools/iw_repro.py [variant] [data]   (default huffman_only randwalk_i2)"""
import os, sys, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import test_gpu_parity as T
variant = sys.argv[1] if len(sys.argv) > 1 else "huffman_only"
data = sys.argv[2] if len(sys.argv) > 2 else "randwalk_i2"
payload = T.DATASETS[data]()
if variant == "huffman_only":
    s = T.gzip_wrap(T.deflate(payload, 6, zlib.Z_HUFFMAN_ONLY), payload)
elif variant == "l1":
    s = T.gzip_wrap(T.deflate(payload, 1), payload)
else:
    s = T.gzip_wrap(T.deflate(payload, 6), payload)
kind, out = T.gpu_decode("gzip", s, "u1", len(payload), None, T.FLAG_INFLATE_WAVE)
print("RESULT", kind, out == payload if kind == "Ok" else None, "stream bytes", len(s), flush=True)
