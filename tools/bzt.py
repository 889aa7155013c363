import bz2, numpy as np, sys
sys.path.insert(0, '.')
from zarr_amd import ArrayMetadata, DefaultChunk, ZarrIOError
from zarr_amd.compression import Bzip2
rng = np.random.default_rng(0)
raw = rng.integers(0, 4, 200, dtype=np.uint8).tobytes()
s = bz2.compress(raw, 1)
open('gpurun_out/bzt.bin', 'wb').write(s)
meta = ArrayMetadata.new([len(raw)], [len(raw)], "u1", Bzip2(1))
try:
    DefaultChunk.read_chunk(s, meta, [0], np.uint8, flags=0x200)
except ZarrIOError as e:
    print("ERR", e.kind)
