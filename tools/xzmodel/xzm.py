#!/usr/bin/env python3
"""DEV TOOLING ONLY: ratio of xz parse strategies on the C2 xz pool (CPU).

Builds tools/xzmodel/libxzm.so (xzm.cpp), encodes a few pool chunks with
  mode 0 (the GPU coder's greedy/lazy rep0 parse) and mode 1 (optimal parse)
and compares the ratio with the system liblzma preset 6 (the reference's
encoder).  Every stream is checked by liblzma's decoder.
  usage: python tools/xzmodel/xzm.py [chunks] [mode:depth:nice:window ...]"""
import ctypes
import lzma
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from bench import quant_chunk  # noqa: E402


def lib():
    so = os.path.join(HERE, "libxzm.so")
    src = os.path.join(HERE, "xzm.cpp")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", so, src], check=True)
    L = ctypes.CDLL(so)
    L.xzm_encode.restype = ctypes.c_uint64
    L.xzm_group.argtypes = [ctypes.c_uint32]
    L.xzm_lclp.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    L.xzm_set.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32]
    L.xzm_encode.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32,
                             ctypes.c_uint32, ctypes.c_uint32]
    return L


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    specs = sys.argv[2:] or ["0:16:64:0", "1:16:64:4096", "1:48:273:4096"]
    L = lib()
    vals = [quant_chunk(i).tobytes() for i in range(n)]
    ref = sum(len(lzma.compress(v, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6)) for v in vals)
    tot = sum(len(v) for v in vals)
    print(f"liblzma preset 6: ratio {tot / ref:.3f}")
    for sp in specs:
        f = [int(x) for x in sp.split(":")]
        mode, depth, nice, window = f[:4]
        L.xzm_group(f[12] if len(f) > 12 else 64)
        L.xzm_lclp(f[9] if len(f) > 9 else 3, f[10] if len(f) > 10 else 0, f[11] if len(f) > 11 else 0)
        L.xzm_set(f[4] if len(f) > 4 else 1, f[5] if len(f) > 5 else 0, f[6] if len(f) > 6 else 0, f[7] if len(f) > 7 else 0, f[8] if len(f) > 8 else 0)
        clen = 0
        t0 = time.time()
        for v in vals:
            out = ctypes.create_string_buffer(len(v) + len(v) // 8 + 4096)
            k = L.xzm_encode(v, len(v), out, mode, depth, nice, window)
            s = out.raw[:k]
            assert lzma.decompress(s, format=lzma.FORMAT_XZ) == v, sp
            clen += k
        print(f"mode {mode} depth {depth} nice {nice} window {window}: ratio {tot / clen:.3f} "
              f"({(time.time() - t0) / n:.2f} s/chunk)")


if __name__ == "__main__":
    main()
