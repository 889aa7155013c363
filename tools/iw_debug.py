#!/usr/bin/env python3
"""Differential check of the gzip decoders on corrupted streams: the default
one-wave-per-chunk kernel vs the 256-lane round kernel vs the oracle; prints
every disagreement (stream, corruption, statuses, first differing byte)."""
import os, sys, zlib
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch
import zref
from zarr_amd import ArrayMetadata, Gzip, _native
from zarr_amd.batch import BatchCodec, PackedStreams


def rw(n, seed=0):
    rng = np.random.default_rng(seed)
    return np.cumsum(rng.integers(-3, 4, n)).astype("<i2")


def gzip_wrap(raw, payload):
    return bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, 0, 255]) + raw + zlib.crc32(payload).to_bytes(4, "little") + \
        (len(payload) & 0xFFFFFFFF).to_bytes(4, "little")


def deflate(p, lvl, strat=0):
    c = zlib.compressobj(lvl, zlib.DEFLATED, -15, 8, strat)
    return c.compress(p) + c.flush()


def run(streams, D, flags):
    packed = PackedStreams(streams, D, "cuda:0", dst=torch.zeros(len(streams) * D, dtype=torch.uint8, device="cuda:0"))
    BatchCodec(0).decode(ArrayMetadata.new([D], [D], "u1", Gzip(6)), packed, flags=flags)
    torch.cuda.synchronize()
    return packed.status.cpu().numpy(), packed.dst.cpu().numpy().reshape(len(streams), D)


payload = rw(150000).tobytes()
s = gzip_wrap(deflate(payload, 6), payload)
rng = np.random.default_rng(11)
nbad = 0
for D in (40000, 100001, 149999):
    variants, info = [], []
    for pos in rng.integers(12, len(s) - 8, 40):
        bad = bytearray(s)
        x = int(rng.integers(1, 256))
        bad[int(pos)] ^= x
        variants.append(bytes(bad)); info.append((int(pos), x))
    st_ref, out_ref = zref.decode_batch(zref.GZIP,
                                        [np.frombuffer(v, np.uint8) for v in variants], D)
    sw, ow = run(variants, D, 0)
    sb, ob = run(variants, D, _native.FLAG_INFLATE_BLOCK_PAR)
    for i in range(len(variants)):
        okw = (sw[i] == 0) == (st_ref[i] == 0) and (sw[i] != 0 or (ow[i] == out_ref[i]).all())
        if not okw or sw[i] != sb[i]:
            nbad += 1
            dw = np.nonzero(ow[i] != ob[i])[0]
            print(f"D={D} pos={info[i][0]} xor={info[i][1]:#x} ref={int(st_ref[i])} wave={int(sw[i])} "
                  f"blockpar={int(sb[i])} first_diff_wave_vs_blockpar={int(dw[0]) if len(dw) else -1}")
print("mismatches", nbad)
