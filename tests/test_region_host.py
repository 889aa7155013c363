"""Region assembly host side (no GPU): the numpy oracle of read_ndarray
(oracle/region_ref.py) against the reference's own ndarray tests
(tests/ndarray.rs), BoundingBox against its doc tests, and the C ABI's
zcg_region_grid against bounded_coord_iter."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import region_ref  # noqa: E402  (oracle: checker only)

from zarr_amd import ArrayMetadata  # noqa: E402
from zarr_amd.region import BoundingBox, region_grid  # noqa: E402


def ref_test_chunks():
    """tests/ndarray.rs:19-58: i32 [3,300,200,100], chunks [3,4,2,1], F order."""
    cs = [3, 4, 2, 1]
    chunks = {}
    for k in range(10):
        z = cs[3] * k
        for j in range(10):
            y = cs[2] * j
            for i in range(10):
                x = cs[1] * i
                data = []
                for zo in range(cs[3]):
                    for yo in range(cs[2]):
                        for xo in range(cs[1]):
                            data += [1000 + x + xo, 2000 + y + yo, 3000 + z + zo]
                chunks[(0, i, j, k)] = np.array(data, np.int32)
    return [3, 300, 200, 100], cs, chunks


def test_oracle_reference_read_ndarray():
    """tests/ndarray.rs:14-100 expected values."""
    shape, cs, chunks = ref_test_chunks()
    a = region_ref.read_ndarray(shape, cs, "F", [0, 5, 4, 3], [3, 35, 15, 7], chunks.get, np.int32)
    x = np.arange(35)[:, None, None]
    y = np.arange(15)[None, :, None]
    z = np.arange(7)[None, None, :]
    assert (a[0] == 1005 + x + 0 * y + 0 * z).all()
    assert (a[1] == 2004 + y + 0 * x + 0 * z).all()
    assert (a[2] == 3003 + z + 0 * x + 0 * y).all()


def test_oracle_reference_read_ndarray_oob():
    """tests/ndarray.rs:102-133."""
    d = np.zeros(5000, np.int32)
    d[0] = 1
    chunks = {(1, 1): d}
    a = region_ref.read_ndarray([100, 200], [50, 100], "F", [45, 175], [50, 50], chunks.get, np.int32)
    assert (a == 0).all()


def test_bounding_box_doc_tests():
    """ndarray.rs:64-70 (intersect) and 88-94 (union)."""
    a = BoundingBox([0, 0], [5, 8])
    a.intersect(BoundingBox([3, 3], [5, 3]))
    assert a == BoundingBox([3, 3], [2, 3])
    a = BoundingBox([0, 0], [5, 8])
    a.union(BoundingBox([3, 3], [5, 3]))
    assert a == BoundingBox([0, 0], [8, 8])


def test_region_grid_matches_bounded_coord_iter():
    rng = np.random.default_rng(5)
    for _ in range(300):
        nd = int(rng.integers(1, 5))
        shape = [int(rng.integers(0, 40)) for _ in range(nd)]
        cs = [int(rng.integers(1, 9)) for _ in range(nd)]
        off = [int(rng.integers(0, 50)) for _ in range(nd)]
        shp = [int(rng.integers(0, 30)) for _ in range(nd)]
        meta = ArrayMetadata.new(shape, cs, "<i2")
        lo, n = region_grid(meta, BoundingBox(off, shp))
        import itertools
        coords = list(itertools.product(*[range(l, l + k) for l, k in zip(lo, n)]))
        assert coords == region_ref.bounded_coord_iter(shape, cs, off, shp)
