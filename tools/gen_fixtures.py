#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run once in the build container (it reads /root/reference, which does not
exist on the GPU box); the outputs are small data files.  Sources:

1. doc_spec.json — the reference's own golden byte arrays for the Zarr
   doc-spec chunk ([1..6] as ``>i2``, shape 5x6x7, chunk 1x2x3,
   tests.rs:120-145): raw.rs:33-45, gzip.rs:66-80, lz.rs:101-115,
   bzip.rs:55-72, xz.rs:52-75.  Also the expected ENCODE bytes
   (tests.rs:147-159): raw, gzip with byte 9 patched to 255 (gzip.rs:90-101),
   lz4, xz; bzip2 encode is #[ignore]d by the reference (bzip.rs:82-90).
2. zarrita/ — the 8 gzip-1 chunk files + array metadata of
   tests/data/zarrita.zr3 (zarrita_compat.rs:30-46), copied byte for byte.
3. reencoded.json — one 2x3x4 chunk of every ReflectedType in both byte
   orders, encoded by the ORACLE (same C codec libraries as the reference's
   -sys crates) with each codec's default parameters, with the decoded bytes
   the oracle produces (tests/integration_test.rs:60-128 re-created with a
   fixed seed instead of the reference's unseeded thread_rng).
"""
import json
import os
import re
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import zref  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden")


def rust_byte_array(path, const_name):
    """Extract ``const NAME: [u8; K] = [ ... ];`` bytes from a reference file."""
    src = open(os.path.join(REF, path)).read()
    m = re.search(const_name + r":\s*\[u8;\s*(\d+)\]\s*=\s*\[(.*?)\];", src, re.S)
    body = m.group(2)
    body = "\n".join(l.split("//")[0] for l in body.splitlines())
    vals = [int(x, 16) for x in re.findall(r"0x[0-9a-fA-F]{2}", body)]
    assert len(vals) == int(m.group(1)), (path, len(vals))
    return bytes(vals)


def main():
    os.makedirs(OUT, exist_ok=True)
    # ---- 1. doc-spec -------------------------------------------------------
    vecs = {
        "raw": ("src/compression/raw.rs", "TEST_CHUNK_I16_RAW"),
        "gzip": ("src/compression/gzip.rs", "TEST_CHUNK_I16_GZIP"),
        "lz4": ("src/compression/lz.rs", "TEST_CHUNK_I16_LZ4"),
        "bzip2": ("src/compression/bzip.rs", "TEST_CHUNK_I16_BZIP2"),
        "xz": ("src/compression/xz.rs", "TEST_CHUNK_I16_XZ"),
    }
    doc = {"array": {"shape": [5, 6, 7], "chunk_shape": [1, 2, 3], "data_type": ">i2"},
           "expected_values": [1, 2, 3, 4, 5, 6], "chunks": {}, "encode_expected": {}}
    for name, (path, const) in vecs.items():
        b = rust_byte_array(path, const)
        doc["chunks"][name] = {"hex": b.hex(), "source": f"{path} {const}"}
    enc = {k: bytes.fromhex(doc["chunks"][k]["hex"]) for k in ("raw", "lz4", "xz")}
    g = bytearray(bytes.fromhex(doc["chunks"]["gzip"]["hex"]))
    g[9] = 255  # gzip.rs:90-101: flate2 writes OS=255 where Java wrote 0
    enc["gzip"] = bytes(g)
    for k, v in enc.items():
        doc["encode_expected"][k] = v.hex()
    with open(os.path.join(OUT, "doc_spec.json"), "w") as f:
        json.dump(doc, f, indent=1)

    # ---- 2. zarrita --------------------------------------------------------
    zdir = os.path.join(OUT, "zarrita")
    if os.path.exists(zdir):
        shutil.rmtree(zdir)
    src_root = os.path.join(REF, "tests/data/zarrita.zr3")
    shutil.copytree(src_root, zdir)

    # ---- 3. oracle re-encodings -------------------------------------------
    rng = np.random.default_rng(20201222)
    dtypes = ["bool", "u1", "i1", "<u2", ">u2", "<u4", ">u4", "<u8", ">u8", "<i2", ">i2", "<i4",
              ">i4", "<i8", ">i8", "<f2", ">f2", "<f4", ">f4", "<f8", ">f8"]
    codecs = [("raw", zref.RAW, 0), ("gzip", zref.GZIP, -1), ("lz4", zref.LZ4, 65536),
              ("bzip2", zref.BZIP2, 9), ("xz", zref.XZ, 6)]
    n = 24  # zarrita chunk 2x3x4
    entries = []
    for dt in dtypes:
        if dt == "bool":
            vals = rng.integers(0, 2, n).astype(np.bool_)
            es, be, isb = 1, False, True
        else:
            npdt = np.dtype(dt.replace(">", "<").replace("u1", "u1"))
            es = npdt.itemsize
            be = dt.startswith(">")
            isb = False
            raw = rng.integers(0, 256, n * es, dtype=np.uint8)
            vals = raw.view(npdt.newbyteorder("<") if es > 1 else npdt)
        for cname, cid, param in codecs:
            st, stream = zref.encode(cid, param, vals, elem_size=es, big_endian=be, is_bool=isb)
            assert st == zref.OK
            st2, dec = zref.decode(cid, stream, n * es, es, be, isb)
            assert st2 == zref.OK
            assert dec == np.ascontiguousarray(vals).view(np.uint8).tobytes()
            entries.append({"dtype": dt, "codec": cname, "param": param, "num_elements": n,
                            "stream": stream.hex(), "decoded": dec.hex()})
    with open(os.path.join(OUT, "reencoded.json"), "w") as f:
        json.dump({"note": "oracle (zref) encodings, decoded bytes host-native", "entries": entries},
                  f, indent=0)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
