"""The C-ABI library loads and exports every symbol include/*.h declares.

No compute call is made here (CPU container); the GPU tests exercise them.
"""
import ctypes
import glob
import os
import re

import pytest

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


# The product build's tuning constants (A/B builds under tools/ pass -D
# overrides; the shipped library must not be one of them).
DEFAULT_BUILD_CONFIG = ("inflate_wave:S=2048,TCAP=768,WPE=4,EST_PCT=108,MARKW=32,G=4,DBG=0;"
                        "inflate_par:PF=16,FU=16,WPE=3;deflate:CHAIN6=32,SUB=128;raw:VPT=1;region:U=4;"
                        "lz4_dec:CORUN=55/131072/196608,LPW=64/64/262144;xz_opt:SEG_KB=256,WPE=4,PROF=0;bz2:KMUL=4,GSAFE=1")


def test_library_built_with_default_knobs():
    L = _native.load_library()
    assert L.zcg_build_config().decode() == DEFAULT_BUILD_CONFIG


def test_product_sources_hold_no_diagnostic_modes():
    """Timing-diagnostic modes that produce wrong output live in tools/, not in
    the product kernels."""
    srcs = glob.glob(os.path.join(ROOT, "zarr_amd", "csrc", "*.hip")) + \
        glob.glob(os.path.join(ROOT, "zarr_amd", "csrc", "*.h"))
    for p in srcs:
        txt = open(p).read()
        assert "DIAG" not in txt, p


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


C_ABI_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c_abi")


def test_c_caller_compiles_against_header():
    """A plain-C program (gcc, no HIP headers) builds against
    include/zchunk_gpu.h and links to the in-tree library."""
    import subprocess
    r = subprocess.run(["make", "-s", "-B", "-C", C_ABI_DIR], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.isfile(os.path.join(C_ABI_DIR, "doc_spec_c"))
    assert os.path.isfile(os.path.join(C_ABI_DIR, "zarrita_c"))


@pytest.mark.gpu
def test_c_caller_doc_spec_roundtrip():
    """The C caller decodes and re-encodes the reference's doc-spec chunk of
    every CompressionType through zcg_read_chunk / zcg_write_chunk."""
    import subprocess
    exe = os.path.join(C_ABI_DIR, "doc_spec_c")
    assert os.path.isfile(exe), "build tests/c_abi first (__graft_entry__.build)"
    r = subprocess.run([exe, "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "doc_spec_c: ok" in r.stdout, (r.stdout, r.stderr)


@pytest.mark.gpu
def test_c_caller_reads_zarrita_hierarchy():
    """A plain-C caller opens the reference's zarrita store with no Python in
    the loop: zcg_array_meta_from_json on meta/root/seq/i2.array.json, the 8
    chunk keys from zcg_chunk_key, zcg_store_read_chunks (shared flock, GPU
    decode), compared with arange(120) (tests/zarrita_compat.rs:16-46)."""
    import subprocess
    exe = os.path.join(C_ABI_DIR, "zarrita_c")
    assert os.path.isfile(exe), "build tests/c_abi first (__graft_entry__.build)"
    store = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "zarrita")
    r = subprocess.run([exe, store, "0"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "zarrita_c: ok (8 chunks" in r.stdout, (r.stdout, r.stderr)
