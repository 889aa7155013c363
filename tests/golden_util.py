"""Helpers shared by the CPU and GPU parity tests: golden fixture loading."""
import glob
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")

CODEC_IDS = {"raw": 0, "bzip2": 1, "gzip": 2, "lz4": 3, "xz": 4}
DEFAULT_PARAM = {"raw": 0, "gzip": -1, "lz4": 65536, "bzip2": 9, "xz": 6}


def doc_spec():
    with open(os.path.join(GOLDEN, "doc_spec.json")) as f:
        return json.load(f)


def reencoded():
    with open(os.path.join(GOLDEN, "reencoded.json")) as f:
        return json.load(f)["entries"]


def dtype_info(dt: str):
    """(elem_size, big_endian, is_bool, numpy dtype) of a zarr dtype string."""
    if dt == "bool":
        return 1, False, True, np.dtype(np.bool_)
    if dt in ("u1", "i1"):
        return 1, False, False, np.dtype(dt)
    es = int(dt[2])
    return es, dt[0] == ">", False, np.dtype("<" + dt[1:])


def zarrita_chunks():
    """[(grid position, stream bytes, expected i2 values in C order)] for the
    8 zarrita chunks: arange(120) as 4x5x6, chunk 2x3x4, overhang zero-padded
    (zarrita_compat.rs:16-46)."""
    full = np.arange(120, dtype="<i2").reshape(4, 5, 6)
    out = []
    for path in sorted(glob.glob(os.path.join(GOLDEN, "zarrita/data/root/seq/i2/c*/*/*"))):
        parts = path.split(os.sep)
        g = (int(parts[-3][1:]), int(parts[-2]), int(parts[-1]))
        block = np.zeros((2, 3, 4), "<i2")
        sub = full[g[0] * 2:(g[0] + 1) * 2, g[1] * 3:(g[1] + 1) * 3, g[2] * 4:(g[2] + 1) * 4]
        block[:sub.shape[0], :sub.shape[1], :sub.shape[2]] = sub
        with open(path, "rb") as f:
            out.append((g, f.read(), block.reshape(-1)))
    return out


def zarrita_meta_json():
    with open(os.path.join(GOLDEN, "zarrita/meta/root/seq/i2.array.json")) as f:
        return f.read()
