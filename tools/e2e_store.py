#!/usr/bin/env python3
"""File -> device -> file rate of the FilesystemHierarchy path (SURVEY §8(d)
e2e, §8(f) rank 1): write_chunks (host elements -> H2D -> zcg_encode_batch
-> D2H -> one file per chunk under an exclusive flock) and read_chunks (files
under a shared flock -> pinned staging by a reader pool -> H2D ->
zcg_decode_batch -> D2H), through the native store (zcg_store_*).  Prints one
JSON line per direction.  The files live in --dir (default $TMPDIR); the read
pass follows the write pass, so it reads from the page cache.

    python tools/e2e_store.py --codec gzip --chunks 1024 [--threads 8]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import workload  # noqa: E402
from zarr_amd import ArrayMetadata  # noqa: E402
from zarr_amd.chunk import SliceDataChunk  # noqa: E402
from zarr_amd.storage import FilesystemHierarchy  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="gzip", choices=["gzip", "lz4", "raw", "xz", "bzip2"])
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--pool", type=int, default=32)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default=os.path.join(os.environ.get("TMPDIR", "/tmp"), "zcg_e2e_store"))
    args = ap.parse_args()
    meta0, gen, desc = workload(args.codec)
    cs = meta0.chunk_shape
    meta = ArrayMetadata.new([cs[0] * args.chunks] + cs[1:], cs, meta0.data_type, meta0.compressor)
    vals = [gen(i) for i in range(args.pool)]
    D = vals[0].nbytes
    shutil.rmtree(args.dir, ignore_errors=True)
    h = FilesystemHierarchy.open_or_create(args.dir)
    h.create_array("a", meta)
    coords = [[i] + [0] * (len(cs) - 1) for i in range(args.chunks)]
    chunks = [SliceDataChunk(c, vals[i % args.pool]) for i, c in enumerate(coords)]
    h.write_chunks("a", meta, chunks[:8], io_threads=args.threads)  # warm: context, workspace
    t0 = time.time()
    h.write_chunks("a", meta, chunks, io_threads=args.threads)
    tw = time.time() - t0
    comp = sum(os.path.getsize(h.chunk_path("a", meta, c)) for c in coords)
    h.read_chunks("a", meta, coords[:8], vals[0].dtype, io_threads=args.threads)
    trs = []
    for _ in range(args.reps):  # the first read also pays the pinned destination's allocation
        got = None
        t0 = time.time()
        got = h.read_chunks("a", meta, coords, vals[0].dtype, io_threads=args.threads)
        trs.append(time.time() - t0)
    tr = min(trs)
    for i in range(0, args.chunks, max(1, args.chunks // 32)):
        assert np.array_equal(got[i].get_data(), vals[i % args.pool]), i
    fs = os.statvfs(args.dir)
    common = {"codec": args.codec, "workload": desc, "chunks": args.chunks, "chunk_bytes": D,
              "compressed_bytes": comp, "ratio": round(args.chunks * D / comp, 3), "io_threads": args.threads,
              "dir_fs_bytes": fs.f_blocks * fs.f_frsize}
    print(json.dumps(dict(common, direction="write_chunks (elements -> files)",
                          gib_s=round(args.chunks * D / tw / GIB, 3), seconds=round(tw, 3))))
    print(json.dumps(dict(common, direction="read_chunks (files -> elements, page cache)",
                          gib_s=round(args.chunks * D / tr / GIB, 3), seconds=round(tr, 3),
                          first_read_gib_s=round(args.chunks * D / trs[0] / GIB, 3))))
    shutil.rmtree(args.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
