"""Region assembly on the GPU (read_ndarray / read_ndarray_into,
ndarray.rs:153-268) against the numpy oracle (oracle/region_ref.py) and the
reference's own ndarray tests (tests/ndarray.rs)."""
import itertools
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import region_ref  # noqa: E402  (oracle: checker only)

from test_region_host import ref_test_chunks  # noqa: E402
from zarr_amd import ArrayMetadata, FilesystemHierarchy, Gzip, Lz4, Raw, SliceDataChunk  # noqa: E402
from zarr_amd.compression import Bzip2, Xz  # noqa: E402
from zarr_amd.region import BoundingBox, read_ndarray, read_ndarray_into  # noqa: E402

pytestmark = pytest.mark.gpu


def test_reference_read_ndarray(tmp_path):
    """tests/ndarray.rs:14-100 through the filesystem, GPU decode + region."""
    shape, cs, chunks = ref_test_chunks()
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new(shape, cs, "<i4")
    h.create_array("test/array/group", meta)
    for c, d in chunks.items():
        h.write_chunk("test/array/group", meta, SliceDataChunk(list(c), d))
    a = read_ndarray(h, "test/array/group", meta, BoundingBox([0, 5, 4, 3], [3, 35, 15, 7]), np.int32)
    assert a.flags.f_contiguous
    x = np.arange(35)[:, None, None]
    y = np.arange(15)[None, :, None]
    z = np.arange(7)[None, None, :]
    assert (a[0] == 1005 + x + 0 * y + 0 * z).all()
    assert (a[1] == 2004 + y + 0 * x + 0 * z).all()
    assert (a[2] == 3003 + z + 0 * x + 0 * y).all()


def test_reference_read_ndarray_oob(tmp_path):
    """tests/ndarray.rs:102-133."""
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([100, 200], [50, 100], "<i4")
    h.create_array("test/array/group", meta)
    d = np.zeros(5000, np.int32)
    d[0] = 1
    h.write_chunk("test/array/group", meta, SliceDataChunk([1, 1], d))
    a = read_ndarray(h, "test/array/group", meta, BoundingBox([45, 175], [50, 50]), np.int32)
    assert a.shape == (50, 50) and (a == 0).all()


def test_reference_write_read_ndarray(tmp_path):
    """tests/ndarray.rs:135-176: whole chunks written from a random array,
    read back with read_ndarray (F) and read_ndarray_into a C-order array."""
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    cs = [3, 4, 2, 1]
    meta = ArrayMetadata.new([3, 300, 200, 100], cs, "<i4", Gzip(6))
    h.create_array("test/array/group", meta)
    rng = np.random.default_rng(11)
    arr = rng.integers(-2**31, 2**31 - 1, (3, 36, 16, 7), dtype=np.int32)
    off = [0, 4, 4, 3]  # chunk-aligned so every chunk is written whole
    for c in itertools.product(*[range(o // s, (o + n) // s) for o, n, s in zip(off, arr.shape, cs)]):
        sl = tuple(slice(ci * s - o, ci * s - o + s) for ci, s, o in zip(c, cs, off))
        h.write_chunk("test/array/group", meta, SliceDataChunk(list(c), arr[sl].reshape(-1, order="F")))
    bbox = BoundingBox(off, list(arr.shape))
    a = read_ndarray(h, "test/array/group", meta, bbox, np.int32)
    assert np.array_equal(a, arr)
    a_c = np.zeros(arr.shape, np.int32)
    read_ndarray_into(h, "test/array/group", meta, bbox, a_c, np.int32)
    assert np.array_equal(a_c, arr)


CODECS = [Raw(), Gzip(1), Lz4(65536), Bzip2(1), Xz(0)]


@pytest.mark.parametrize("seed", range(12))
def test_region_random_vs_oracle(tmp_path, seed):
    """Random shapes/chunks/orders/dtypes/boxes (partly outside the array),
    missing chunks, overhanging edge chunks, fill values."""
    rng = np.random.default_rng(100 + seed)
    nd = int(rng.integers(1, 5))
    dt = ["<i2", "<u1", "<f8", "<i4", "bool", ">u2", ">f4"][seed % 7]
    npdt = np.dtype("bool") if dt == "bool" else np.dtype(dt).newbyteorder("=")
    for attempt in range(50):
        shape = [int(rng.integers(1, 30 if nd < 3 else 12)) for _ in range(nd)]
        cs = [int(rng.integers(1, 9)) for _ in range(nd)]
        off = [int(rng.integers(0, s + 3)) for s in shape]
        shp = [int(rng.integers(0, 25 if nd < 3 else 10)) for _ in range(nd)]
        meta = ArrayMetadata.new(shape, cs, dt, CODECS[seed % len(CODECS)])
        coords = region_ref.bounded_coord_iter(shape, cs, off, shp)
        if all(meta.in_bounds(c) for c in coords):
            break
    meta.chunk_memory_layout = "F" if seed % 2 else "C"
    if seed % 3 == 0 and dt != "bool":
        meta.fill_value = 7
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    h.create_array("a", meta)
    n_el = int(np.prod(cs))
    chunks = {}
    grid = [(s + c - 1) // c for s, c in zip(shape, cs)]
    for c in itertools.product(*[range(g) for g in grid]):
        if rng.random() < 0.25:
            continue  # absent chunk -> fill / untouched
        if dt == "bool":
            d = rng.integers(0, 2, n_el).astype(bool)
        elif npdt.kind == "f":
            d = rng.standard_normal(n_el).astype(npdt)
        else:
            d = rng.integers(0, 200, n_el).astype(npdt)
        chunks[c] = d
        h.write_chunk("a", meta, SliceDataChunk(list(c), d))
    fill = 7 if meta.fill_value is not None else 0
    bbox = BoundingBox(off, shp)
    want = region_ref.read_ndarray(shape, cs, meta.chunk_memory_layout, off, shp, chunks.get, npdt, fill)
    got = read_ndarray(h, "a", meta, bbox, npdt)
    assert got.shape == tuple(shp) and np.array_equal(got, want)
    # read_ndarray_into keeps what no chunk covers, on a strided view
    base = np.full([s * 2 for s in shp] or [1], 3 if dt != "bool" else True, dtype=npdt)
    view = base[tuple(slice(None, None, 2) for _ in shp)]
    exp = view.copy()
    region_ref.read_ndarray_into(shape, cs, meta.chunk_memory_layout, off, shp, chunks.get, exp)
    read_ndarray_into(h, "a", meta, bbox, view, npdt)
    assert np.array_equal(view, exp)


def test_region_device_large_unaligned():
    """Device-level assembly of a big box straddling chunk boundaries at an
    odd offset (vector path + run path), against numpy on the host."""
    import torch
    from zarr_amd.region import assemble_region
    meta = ArrayMetadata.new([1000, 600, 40], [100, 64, 8], "<i2")
    meta.chunk_memory_layout = "C"
    off, shp = [37, 5, 3], [900, 590, 33]
    lo = [o // c for o, c in zip(off, meta.chunk_shape)]
    hi = [(o + s + c - 1) // c for o, s, c in zip(off, shp, meta.chunk_shape)]
    coords = list(itertools.product(*[range(a, b) for a, b in zip(lo, hi)]))
    rng = np.random.default_rng(1)
    full = rng.integers(-30000, 30000, [g * c for g, c in zip(hi, meta.chunk_shape)], dtype=np.int16)
    N = int(np.prod(meta.chunk_shape))
    dev = torch.device("cuda", 0)
    slots = torch.empty(len(coords) * N, dtype=torch.int16, device=dev)
    host = np.empty((len(coords), N), np.int16)
    for i, c in enumerate(coords):
        sl = tuple(slice(ci * s, ci * s + s) for ci, s in zip(c, meta.chunk_shape))
        host[i] = full[sl].reshape(-1)
    slots.copy_(torch.from_numpy(host.reshape(-1)))
    table = torch.tensor([slots.data_ptr() + i * N * 2 for i in range(len(coords))], dtype=torch.int64, device=dev)
    out = torch.empty(int(np.prod(shp)), dtype=torch.int16, device=dev)
    st = [shp[1] * shp[2], shp[2], 1]
    assemble_region(meta, BoundingBox(off, shp), 2, table, out, st, True, 0)
    torch.cuda.synchronize()
    want = full[tuple(slice(o, o + s) for o, s in zip(off, shp))]
    assert np.array_equal(out.cpu().numpy().reshape(shp), want)


@pytest.mark.parametrize("es,order,ostride_c", [(2, "F", False), (8, "F", False), (1, "C", False),
                                                 (4, "F", True)])
def test_region_device_long_rows(es, order, ostride_c):
    """Row-per-wave path (long fast dimension): unaligned offsets, chunk
    boundaries inside 16-byte pieces, absent chunks with fill, and a
    non-unit output stride along the fast dimension."""
    import torch
    from zarr_amd.region import assemble_region, region_grid, _strides
    dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[es]
    meta = ArrayMetadata.new([700, 50, 9], [301, 7, 4], {1: "u1", 2: "<i2", 4: "<i4", 8: "<i8"}[es])
    meta.chunk_memory_layout = order
    if order == "C":
        meta = ArrayMetadata.new([9, 50, 700], [4, 7, 301], "u1")
        meta.chunk_memory_layout = "C"
        off, shp = [1, 3, 13], [8, 40, 680]
    else:
        off, shp = [13, 3, 1], [680, 40, 8]
    bbox = BoundingBox(off, shp)
    lo, n = region_grid(meta, bbox)
    coords = list(itertools.product(*[range(a, a + k) for a, k in zip(lo, n)]))
    cs = meta.chunk_shape
    N = int(np.prod(cs))
    rng = np.random.default_rng(es)
    full = rng.integers(0, 120, [(l + k) * c for l, k, c in zip(lo, n, cs)]).astype(dt)
    dev = torch.device("cuda", 0)
    host = np.empty((len(coords), N), dt)
    absent = set(i for i in range(len(coords)) if rng.random() < 0.2)
    for i, c in enumerate(coords):
        sl = tuple(slice(ci * s, ci * s + s) for ci, s in zip(c, cs))
        host[i] = full[sl].reshape(-1, order=order)
        if i in absent:
            full[sl] = 99
    slots = torch.from_numpy(host.reshape(-1).view(np.uint8).copy()).to(dev)
    table = torch.tensor([0 if i in absent else slots.data_ptr() + i * N * es for i in range(len(coords))],
                         dtype=torch.int64, device=dev)
    st = _strides(shp, "C" if ostride_c else order)
    out = torch.zeros(int(np.prod(shp)) * es, dtype=torch.uint8, device=dev)
    assemble_region(meta, bbox, es, table, out, st, True, 99)
    torch.cuda.synchronize()
    got = np.ndarray(tuple(shp), dtype=dt, buffer=out.cpu().numpy(), strides=tuple(s * es for s in st))
    want = full[tuple(slice(o, o + s) for o, s in zip(off, shp))]
    assert np.array_equal(got, want)


def test_reference_write_ndarray_unaligned(tmp_path):
    """tests/ndarray.rs:135-176 through write_ndarray itself: a random box at
    an unaligned offset (partial chunks are read-modified-written), read back
    with read_ndarray (F) and read_ndarray_into (C)."""
    from zarr_amd.region import write_ndarray
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([3, 300, 200, 100], [3, 4, 2, 1], "<i4", Gzip(6))
    h.create_array("test/array/group", meta)
    rng = np.random.default_rng(12)
    arr = rng.integers(-2**31, 2**31 - 1, (3, 35, 15, 7), dtype=np.int32)
    off = [0, 5, 4, 3]
    write_ndarray(h, "test/array/group", meta, off, arr)
    bbox = BoundingBox(off, list(arr.shape))
    assert np.array_equal(read_ndarray(h, "test/array/group", meta, bbox, np.int32), arr)
    a_c = np.zeros(arr.shape, np.int32)
    read_ndarray_into(h, "test/array/group", meta, bbox, a_c, np.int32)
    assert np.array_equal(a_c, arr)


@pytest.mark.parametrize("seed", range(10))
def test_write_ndarray_random_vs_oracle(tmp_path, seed):
    """Random stores (some chunks present, some absent), random boxes (partly
    outside the array), both memory orders, fill values, several codecs:
    every chunk of the store afterwards equals the oracle's."""
    from zarr_amd.region import write_ndarray
    rng = np.random.default_rng(300 + seed)
    nd = int(rng.integers(1, 4))
    dt = ["<i2", "<u1", "<f8", "<i4", ">u2"][seed % 5]
    npdt = np.dtype(dt).newbyteorder("=")
    for _ in range(50):
        shape = [int(rng.integers(1, 40 if nd < 3 else 14)) for _ in range(nd)]
        cs = [int(rng.integers(1, 9)) for _ in range(nd)]
        off = [int(rng.integers(0, s + 2)) for s in shape]
        shp = [int(rng.integers(1, 20 if nd < 3 else 9)) for _ in range(nd)]
        meta = ArrayMetadata.new(shape, cs, dt, CODECS[seed % len(CODECS)])
        coords = region_ref.bounded_coord_iter(shape, cs, off, shp)
        if coords and all(meta.in_bounds(c) for c in coords):
            break
    meta.chunk_memory_layout = "F" if seed % 2 else "C"
    if seed % 3 == 0:
        meta.fill_value = 5
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    h.create_array("a", meta)
    n_el = int(np.prod(cs))
    chunks = {}
    grid = [(s + c - 1) // c for s, c in zip(shape, cs)]
    for c in itertools.product(*[range(g) for g in grid]):
        if rng.random() < 0.4:
            continue
        d = (rng.standard_normal(n_el) * 50).astype(npdt) if npdt.kind == "f" else \
            rng.integers(0, 200, n_el).astype(npdt)
        chunks[c] = d
        h.write_chunk("a", meta, SliceDataChunk(list(c), d))
    box = (rng.standard_normal(shp) * 50).astype(npdt) if npdt.kind == "f" else \
        rng.integers(0, 250, shp).astype(npdt)
    region_ref.write_ndarray(shape, cs, meta.chunk_memory_layout, off, box, chunks,
                             5 if meta.fill_value is not None else 0)
    write_ndarray(h, "a", meta, off, box)
    for c, want in chunks.items():
        got = h.read_chunk("a", meta, list(c), npdt)
        assert got is not None, c
        assert np.array_equal(got.get_data(), np.asarray(want, npdt)), c


@pytest.mark.parametrize("es,order,istride_c,unaligned", [(1, "F", False, True), (2, "F", False, True),
                                                          (4, "F", True, False), (8, "F", False, True),
                                                          (2, "C", True, True)])
def test_write_region_device_long_rows(es, order, istride_c, unaligned):
    """zcg_write_region's row-per-wave path (box rows of >= 32*16/es elements
    along the fast dimension): rows that start at unaligned offsets inside a
    chunk, absent (NULL) chunks that must stay untouched, and a strided input
    view; compared with region_ref.write_ndarray's element placement."""
    import torch
    from zarr_amd.region import region_grid, scatter_region, _strides
    dt = {1: np.uint8, 2: np.int16, 4: np.int32, 8: np.int64}[es]
    ts = {1: "u1", 2: "<i2", 4: "<i4", 8: "<i8"}[es]
    if order == "C":
        meta = ArrayMetadata.new([9, 50, 900], [4, 7, 301], ts)
        off, shp = ([1, 3, 13] if unaligned else [0, 0, 0]), [8, 40, 880]
    else:
        meta = ArrayMetadata.new([900, 50, 9], [301, 7, 4], ts)
        off, shp = ([13, 3, 1] if unaligned else [0, 0, 0]), [880, 40, 8]
    meta.chunk_memory_layout = order
    bbox = BoundingBox(off, shp)
    lo, n = region_grid(meta, bbox)
    coords = list(itertools.product(*[range(a, a + k) for a, k in zip(lo, n)]))
    cs = meta.chunk_shape
    N = int(np.prod(cs))
    rng = np.random.default_rng(40 + es)
    chunks = {c: rng.integers(0, 100, N).astype(dt) for c in coords}
    absent = set(c for c in coords if rng.random() < 0.2)
    box = rng.integers(0, 100, shp).astype(dt)
    # expected: the oracle's write_ndarray placement on the present chunks
    want = {c: v.copy() for c, v in chunks.items() if c not in absent}
    region_ref.write_ndarray(meta.shape, cs, order, off, box, want, 0)
    dev = torch.device("cuda", 0)
    host = np.stack([chunks[c] for c in coords]).reshape(-1)
    slots = torch.from_numpy(host.view(np.uint8).copy()).to(dev)
    table = torch.tensor([0 if c in absent else slots.data_ptr() + i * N * es for i, c in enumerate(coords)],
                         dtype=torch.int64, device=dev)
    st = _strides(shp, "C" if istride_c else order)
    flat = np.empty(int(np.prod(shp)), dt)
    view = np.ndarray(tuple(shp), dtype=dt, buffer=flat, strides=tuple(s * es for s in st))
    view[...] = box
    boxd = torch.from_numpy(flat.view(np.uint8).copy()).to(dev)
    scatter_region(meta, bbox, es, table, boxd, st)
    torch.cuda.synchronize()
    got = slots.cpu().numpy().view(dt).reshape(len(coords), N)
    for i, c in enumerate(coords):
        exp = chunks[c] if c in absent else want[c]
        assert np.array_equal(got[i], exp), c


def test_write_ndarray_sub_batches(tmp_path, monkeypatch):
    """write_ndarray split into several sub-batches (a small byte budget):
    chunks outside a sub-batch are NULL in that region call, and every chunk
    still ends up equal to the oracle's."""
    import zarr_amd.region as R
    from zarr_amd.region import write_ndarray
    monkeypatch.setattr(R, "WRITE_BATCH_BYTES", 3 * 1024)
    rng = np.random.default_rng(77)
    shape, cs = [30, 20, 10], [4, 3, 5]
    meta = ArrayMetadata.new(shape, cs, "<i4", Gzip(1))
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    h.create_array("a", meta)
    chunks = {}
    n_el = int(np.prod(cs))
    for c in itertools.product(*[range((s + k - 1) // k) for s, k in zip(shape, cs)]):
        if rng.random() < 0.5:
            d = rng.integers(0, 1000, n_el).astype(np.int32)
            chunks[c] = d
            h.write_chunk("a", meta, SliceDataChunk(list(c), d))
    off, shp = [3, 2, 1], [21, 15, 8]
    box = rng.integers(0, 1000, shp).astype(np.int32)
    region_ref.write_ndarray(shape, cs, meta.chunk_memory_layout, off, box, chunks, 0)
    write_ndarray(h, "a", meta, off, box)
    for c, want in chunks.items():
        got = h.read_chunk("a", meta, list(c), np.int32)
        assert got is not None and np.array_equal(got.get_data(), want), c
