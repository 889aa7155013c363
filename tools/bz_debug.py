"""Debug driver (GPU box): small bzip2 streams through the GPU decoder with
CRC verdicts off (ZCG_FLAG_DEBUG_COUNTERS), first differing byte vs input."""
import bz2
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from zarr_amd import ArrayMetadata, DefaultChunk, ZarrIOError  # noqa: E402
from zarr_amd.compression import Bzip2  # noqa: E402

rng = np.random.default_rng(0)
cases = {
    "abc": b"abcabcabcabcabcabc" * 10,
    "small_rand": rng.integers(0, 4, 200, dtype=np.uint8).tobytes(),
    "zeros": bytes(1000),
    "rw": np.cumsum(rng.integers(-3, 4, 5000)).astype("<i2").tobytes(),
    "big_rw": np.cumsum(rng.integers(-3, 4, 300000)).astype("<i2").tobytes(),
}
for name, raw in cases.items():
    s = bz2.compress(raw, 1)
    meta = ArrayMetadata.new([len(raw)], [len(raw)], "u1", Bzip2(1))
    for flags in (0, 0x200):
        try:
            out = DefaultChunk.read_chunk(s, meta, [0], np.uint8, flags=flags).get_data().tobytes()
            diff = next((i for i in range(len(raw)) if out[i] != raw[i]), None)
            print(name, "flags", flags, "OK", "first diff", diff, "len", len(raw), flush=True)
            if diff is not None:
                print("  got", list(out[diff:diff + 16]), "want", list(raw[diff:diff + 16]))
        except ZarrIOError as e:
            print(name, "flags", flags, "ERR", e.kind, flush=True)
