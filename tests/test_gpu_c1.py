"""C1 (BASELINE.json configs[0]): the reference README's roundtrip
(README.md:18-43, run there as a doctest via lib.rs:6-7) through
FilesystemHierarchy, with the chunk codec on the GPU.

i16 array 100x200x300, chunk 44x33x22, CompressionType::default() (Raw),
chunk [0,0,0] of zeros written under /test/array/group and read back.
"""
import json
import os

import numpy as np
import pytest

from zarr_amd import ArrayMetadata
from zarr_amd.chunk import SliceDataChunk
from zarr_amd.compression import Bzip2, CompressionType, Gzip, Lz4, Raw, Xz
from zarr_amd.data_type import zarr_type
from zarr_amd.storage import FilesystemHierarchy

pytestmark = pytest.mark.gpu


def _roundtrip(root, compression, chunk_data=None):
    n = FilesystemHierarchy.open_or_create(root)
    array_meta = ArrayMetadata.new([100, 200, 300], [44, 33, 22], zarr_type(np.int16), compression)
    if chunk_data is None:
        chunk_data = np.zeros(array_meta.get_chunk_num_elements(), np.int16)  # vec![0i16; N]
    chunk_in = SliceDataChunk([0, 0, 0], chunk_data)
    path_name = "/test/array/group"
    n.create_array(path_name, array_meta)
    n.write_chunk(path_name, array_meta, chunk_in)
    chunk_out = n.read_chunk(path_name, array_meta, [0, 0, 0], np.int16)
    assert chunk_out is not None, "Chunk is empty"
    assert np.array_equal(chunk_out.get_data(), chunk_data)
    return n, array_meta, path_name


def test_readme_roundtrip(tmp_path):
    root = str(tmp_path / "tmp.zr3")
    n, meta, path = _roundtrip(root, CompressionType.default())
    assert isinstance(meta.compressor, Raw) and meta.get_chunk_num_elements() == 44 * 33 * 22
    # the store layout the reference writes: zarr.json, the array document,
    # and the chunk under data/root/<path>/c0/0/0 (storage.rs:109-127)
    chunk_file = os.path.join(root, "data", "root", "test", "array", "group", "c0", "0", "0")
    assert os.path.isfile(chunk_file) and os.path.getsize(chunk_file) == 44 * 33 * 22 * 2
    assert open(chunk_file, "rb").read() == bytes(44 * 33 * 22 * 2)
    doc = json.load(open(os.path.join(root, "meta", "root", "test", "array", "group.array.json")))
    assert doc["shape"] == [100, 200, 300] and doc["data_type"] == "<i2"
    assert "compressor" not in doc  # Raw is omitted when default (lib.rs:398-401)
    # reopen and read through the stored metadata; absent chunks are None
    n2 = FilesystemHierarchy.open(root)
    meta2 = n2.get_array_metadata(path)
    assert meta2.get_chunk_shape() == [44, 33, 22]
    out = n2.read_chunk(path, meta2, [0, 0, 0], np.int16)
    assert out.get_data().tobytes() == bytes(44 * 33 * 22 * 2)
    assert n2.read_chunk(path, meta2, [1, 2, 3], np.int16) is None


@pytest.mark.parametrize("comp", [Raw(), Gzip(-1), Lz4(65536), Bzip2(9), Xz(6)],
                         ids=["raw", "gzip", "lz4", "bzip2", "xz"])
def test_readme_roundtrip_data_every_codec(tmp_path, comp):
    """The same roundtrip with non-zero data and every CompressionType."""
    rng = np.random.default_rng(44)
    data = np.cumsum(rng.integers(-3, 4, 44 * 33 * 22)).astype(np.int16)
    _roundtrip(str(tmp_path / "tmp.zr3"), comp, data)
