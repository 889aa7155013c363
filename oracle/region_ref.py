"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of ZarrNdarrayReader::read_ndarray / read_ndarray_into
(sci-rs/zarr src/ndarray.rs) in numpy, the checker for the device region
assembly (zarr_amd/region.py -> zcg_read_region).  Only tests/ import it.

  bounded_coord_iter   ndarray.rs:410-432  (array bounds ∩ bbox, floor/ceil)
  get_chunk_bounds     ndarray.rs:434-446  (nominal bounds, edge overhang kept)
  as_ndarray           ndarray.rs:453-476  (chunk data in the memory order)
  read_ndarray         ndarray.rs:153-174  (Array::from_elem(fill) + read_into)
  read_ndarray_into    ndarray.rs:195-268  (assign read_bb per present chunk)

`get_chunk(coord) -> np.ndarray | None` stands in for read_chunk: the
decoded chunk elements (flat, chunk_num_elements) or None when absent.
"""
from __future__ import annotations

import itertools

import numpy as np


def intersect(off_a, shp_a, off_b, shp_b):
    """BoundingBox::intersect (ndarray.rs:71-85), saturating."""
    off, shp = [], []
    for oa, sa, ob, sb in zip(off_a, shp_a, off_b, shp_b):
        new_o = max(ob, oa)
        shp.append(max(0, min(sa + oa, ob + sb) - new_o))
        off.append(new_o)
    return off, shp


def bounded_coord_iter(shape, chunk_shape, bbox_off, bbox_shape):
    """ndarray.rs:410-432: C-order (last index fastest, CoordIterator) coords."""
    off, shp = intersect([0] * len(shape), list(shape), bbox_off, bbox_shape)
    floor = [o // cs for o, cs in zip(off, chunk_shape)]
    ceil = [(o + s + cs - 1) // cs for o, s, cs in zip(off, shp, chunk_shape)]
    return list(itertools.product(*[range(f, c) for f, c in zip(floor, ceil)]))


def read_ndarray_into(shape, chunk_shape, order, bbox_off, bbox_shape, get_chunk, arr):
    for coord in bounded_coord_iter(shape, chunk_shape, bbox_off, bbox_shape):
        data = get_chunk(coord)
        if data is None:
            continue
        c_off = [c * cs for c, cs in zip(coord, chunk_shape)]
        r_off, r_shp = intersect(bbox_off, bbox_shape, c_off, chunk_shape)
        if 0 in r_shp:
            continue
        chunk = np.asarray(data).reshape(tuple(chunk_shape), order=order)
        a_sl = tuple(slice(o - b, o - b + s) for o, b, s in zip(r_off, bbox_off, r_shp))
        c_sl = tuple(slice(o - c, o - c + s) for o, c, s in zip(r_off, c_off, r_shp))
        arr[a_sl] = chunk[c_sl]


def read_ndarray(shape, chunk_shape, order, bbox_off, bbox_shape, get_chunk, dtype, fill=0):
    arr = np.full(tuple(bbox_shape), fill, dtype=dtype, order=order)
    read_ndarray_into(shape, chunk_shape, order, bbox_off, bbox_shape, get_chunk, arr)
    return arr


def write_ndarray(shape, chunk_shape, order, offset, array, chunks, fill=0):
    """ZarrNdarrayWriter::write_ndarray (ndarray.rs:276-385) on a dict
    coord -> flat chunk elements (the store): fully covered chunks are
    replaced, partly covered ones are read (or start as fill) and overlaid."""
    bshape = list(array.shape)
    for coord in bounded_coord_iter(shape, chunk_shape, offset, bshape):
        nom = [c * cs for c, cs in zip(coord, chunk_shape)]
        w_off, w_shp = intersect(nom, chunk_shape, offset, bshape)
        a_sl = tuple(slice(o - b, o - b + s) for o, b, s in zip(w_off, offset, w_shp))
        if w_off == nom and w_shp == list(chunk_shape):
            data = np.asarray(array[a_sl]).flatten(order=order)
        else:
            ex = chunks.get(coord)
            ch = (np.asarray(ex).reshape(tuple(chunk_shape), order=order).copy() if ex is not None
                  else np.full(tuple(chunk_shape), fill, dtype=array.dtype))
            c_sl = tuple(slice(o - n, o - n + s) for o, n, s in zip(w_off, nom, w_shp))
            ch[c_sl] = array[a_sl]
            data = ch.flatten(order=order)
        chunks[coord] = data
