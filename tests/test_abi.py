"""The C-ABI library loads and exports every symbol include/*.h declares.

No compute call is made here (CPU container); the GPU tests exercise them.
"""
import ctypes
import glob
import os
import re

from zarr_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        syms |= set(re.findall(r"\b(zcg_[a-z0-9_]+)\s*\(", src))
    return syms


def test_header_declares_the_api():
    syms = declared_symbols()
    assert "zcg_decode_batch" in syms and "zcg_encode_batch" in syms
    assert syms == set(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_native.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_abi_version_and_pure_helpers():
    L = _native.load_library()
    assert L.zcg_abi_version() == 1
    assert L.zcg_effective_gzip_level(-1) == 6 and L.zcg_effective_gzip_level(3) == 3
    assert L.zcg_effective_lz4_block_size(70000) == 262144
    assert L.zcg_codec_on_gpu(0, 0) == 1


def test_struct_layout_matches_header():
    """sizeof checks mirrored from include/zchunk_gpu.h (compiled with gcc)."""
    import subprocess
    import tempfile
    src = r'''
#include <stdio.h>
#include "zchunk_gpu.h"
#include <stddef.h>
int main(){printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(zcg_compression), sizeof(zcg_dtype),
 sizeof(zcg_array), sizeof(zcg_chunk), offsetof(zcg_array, chunk_num_elements), sizeof(zcg_region),
 offsetof(zcg_region, out_strides), offsetof(zcg_region, fill_value));return 0;}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    assert [int(x) for x in out] == [ctypes.sizeof(_native.Compression), ctypes.sizeof(_native.DType),
                                     ctypes.sizeof(_native.Array), ctypes.sizeof(_native.Chunk),
                                     _native.Array.chunk_num_elements.offset, ctypes.sizeof(_native.Region),
                                     _native.Region.out_strides.offset, _native.Region.fill_value.offset]
