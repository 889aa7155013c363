"""The FilesystemHierarchy end of the path through the native store
(zcg_store_read_chunks / zcg_store_write_chunks) and the
in-process multi-GPU entry (zcg_multi_*).

Reference semantics: get() = open + shared flock + read, a missing file is
Ok(None) (filesystem.rs:201-210, storage.rs:226-234); set() = create_dir_all
+ open + exclusive flock + truncate after the lock + write (filesystem.rs:260-280)."""
import fcntl
import os
import threading
import time

import numpy as np
import pytest

from zarr_amd import ArrayMetadata, _native
from zarr_amd.chunk import SliceDataChunk, ZarrIOError
from zarr_amd.compression import Bzip2, Gzip, Lz4, Raw, Xz
from zarr_amd.multi import MultiDeviceCodec
from zarr_amd.storage import FilesystemHierarchy, store_read

pytestmark = pytest.mark.gpu

zref = pytest.importorskip("zref")

CODECS = [Raw(), Gzip(6), Lz4(65536), Bzip2(9), Xz(6)]


def _walk(n, seed, dt=np.int16):
    rng = np.random.default_rng(seed)
    return (np.cumsum(rng.integers(-3, 4, n)) % 1000).astype(dt)


@pytest.mark.parametrize("comp", CODECS, ids=["raw", "gzip", "lz4", "bzip2", "xz"])
@pytest.mark.parametrize("dt", ["<i2", ">f4", "bool"])
def test_store_roundtrip_with_absent_chunks(tmp_path, comp, dt):
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([40, 30, 20], [8, 7, 6], dt, comp)
    h.create_array("a/b", meta)
    npdt = np.dtype(dt).newbyteorder("=")
    grid = meta.get_grid_extent()
    coords = [[i, j, k] for i in range(grid[0]) for j in range(grid[1]) for k in range(grid[2])]
    written = {}
    N = meta.get_chunk_num_elements()
    chunks = []
    for n, c in enumerate(coords):
        if n % 3 == 1:
            continue
        d = (_walk(N, n).astype(npdt) if dt != "bool" else (_walk(N, n) % 2).astype(bool))
        written[tuple(c)] = d
        chunks.append(SliceDataChunk(c, d))
    h.write_chunks("a/b", meta, chunks)
    got = h.read_chunks("a/b", meta, coords, npdt)
    for c, g in zip(coords, got):
        if tuple(c) in written:
            assert g is not None and np.array_equal(g.get_data(), written[tuple(c)]), c
        else:
            assert g is None, c
    # the files decode with the reference libraries (oracle) as well
    c0 = next(iter(written))
    raw = open(h.chunk_path("a/b", meta, list(c0)), "rb").read()
    cid = {"Raw": zref.RAW, "Gzip": zref.GZIP, "Lz4": zref.LZ4, "Bzip2": zref.BZIP2, "Xz": zref.XZ}[type(comp).__name__]
    es = meta.effective_type().size_of()
    st, dec = zref.decode(cid, raw, N * es, es, dt.startswith(">"), dt == "bool")
    assert st == zref.OK and dec == written[c0].astype(npdt).tobytes()


def test_store_many_sub_batches_and_errors(tmp_path):
    """300 x 1 MiB chunks (two 256 MiB pipeline sub-batches), a truncated file,
    a directory where a chunk file would be, a missing chunk."""
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([300 * 524288], [524288], "<i2", Lz4(65536))
    h.create_array("big", meta)
    datas = [_walk(524288, 1000 + i) for i in range(300)]
    h.write_chunks("big", meta, [SliceDataChunk([i], d) for i, d in enumerate(datas)])
    p7 = h.chunk_path("big", meta, [7])
    b = open(p7, "rb").read()
    open(p7, "wb").write(b[: len(b) // 2])  # truncated frame
    os.remove(h.chunk_path("big", meta, [8]))
    os.remove(h.chunk_path("big", meta, [9]))
    os.makedirs(h.chunk_path("big", meta, [9]))
    os.remove(h.chunk_path("big", meta, [299]))
    paths = [h.chunk_path("big", meta, [i]) for i in range(300)]
    arrs, st = store_read(meta, paths, np.int16)
    assert st[7] == _native.UNEXPECTED_EOF
    assert st[8] == _native.ABSENT and st[9] == _native.ABSENT and st[299] == _native.ABSENT
    for i in range(300):
        if i not in (7, 8, 9, 299):
            assert st[i] == 0 and np.array_equal(arrs[i], datas[i]), i
    with pytest.raises(ZarrIOError):
        h.read_chunks("big", meta, [[6], [7]], np.int16)


def test_write_truncates_after_lock(tmp_path):
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([1 << 20], [1 << 18], "<u1", Gzip(6))
    h.create_array("t", meta)
    rng = np.random.default_rng(3)
    h.write_chunk("t", meta, SliceDataChunk([0], rng.integers(0, 256, 1 << 18, dtype=np.uint8)))
    big = os.path.getsize(h.chunk_path("t", meta, [0]))
    h.write_chunk("t", meta, SliceDataChunk([0], np.zeros(1 << 18, np.uint8)))
    small = os.path.getsize(h.chunk_path("t", meta, [0]))
    assert small < big // 10  # set_len(0) then write: no stale tail
    assert np.array_equal(h.read_chunk("t", meta, [0], np.uint8).get_data(), np.zeros(1 << 18, np.uint8))


def test_read_waits_for_exclusive_lock_and_write_for_shared(tmp_path):
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([4096], [4096], "<i2", Raw())
    h.create_array("l", meta)
    d = _walk(4096, 5)
    h.write_chunk("l", meta, SliceDataChunk([0], d))
    p = h.chunk_path("l", meta, [0])
    res = {}
    with open(p, "rb+") as f:
        fcntl.flock(f, fcntl.LOCK_EX)  # a writer holds the chunk
        t = threading.Thread(target=lambda: res.setdefault("r", h.read_chunk("l", meta, [0], np.int16)))
        t.start()
        time.sleep(0.5)
        assert t.is_alive(), "read_chunk did not wait for the exclusive lock"
        fcntl.flock(f, fcntl.LOCK_UN)
    t.join(60)
    assert np.array_equal(res["r"].get_data(), d)
    d2 = _walk(4096, 6)
    with open(p, "rb") as f:
        fcntl.flock(f, fcntl.LOCK_SH)  # a reader holds the chunk
        t = threading.Thread(target=lambda: h.write_chunk("l", meta, SliceDataChunk([0], d2)))
        t.start()
        time.sleep(0.5)
        assert t.is_alive(), "write_chunk did not wait for the shared lock"
        assert np.array_equal(np.frombuffer(open(p, "rb").read(), "<i2"), d)  # not truncated yet
        fcntl.flock(f, fcntl.LOCK_UN)
    t.join(60)
    assert np.array_equal(h.read_chunk("l", meta, [0], np.int16).get_data(), d2)


def test_multi_device_round_robin(tmp_path):
    """zcg_multi over two contexts (device 0 twice on a one-GPU box): chunk i
    goes to context i mod 2; statuses and data merge back in order."""
    mc = MultiDeviceCodec([0, 0])
    meta = ArrayMetadata.new([64 * 9], [64 * 9], "<i4", Gzip(6))
    N = meta.get_chunk_num_elements()
    datas = [_walk(N, 50 + i, np.int32) for i in range(41)]
    streams = [zref.encode(zref.GZIP, 6, d)[1] for d in datas]
    streams[5] = streams[5][:20]  # truncated: UnexpectedEof for that chunk only
    st, outs = mc.read_chunks_host(meta, streams, np.int32)
    assert st[5] == _native.UNEXPECTED_EOF
    for i in range(41):
        if i != 5:
            assert st[i] == 0 and np.array_equal(outs[i], datas[i]), i
    paths = [str(tmp_path / "m" / f"c{i}") for i in range(41)]
    wst = mc.store_write(meta, paths, datas)
    assert (wst == 0).all()
    os.remove(paths[40])
    outs, rst = mc.store_read(meta, paths, np.int32)
    assert rst[40] == _native.ABSENT
    for i in range(40):
        assert rst[i] == 0 and np.array_equal(outs[i], datas[i]), i
    mc.close()


# ---- device-resident ends and the region path on the store's semantics --------------
def test_store_read_device_into_slots(tmp_path):
    """zcg_store_read_chunks_device: files decoded straight into device slots;
    absent chunks leave their slot untouched; pinned host destinations take
    the direct D2H path and agree."""
    import torch
    from zarr_amd.storage import store_read_device, store_write_device
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([20 * 4096], [4096], ">i4", Gzip(6))
    h.create_array("d", meta)
    datas = [_walk(4096, 70 + i, np.int32) for i in range(20)]
    h.write_chunks("d", meta, [SliceDataChunk([i], d) for i, d in enumerate(datas) if i != 3])
    paths = [h.chunk_path("d", meta, [i]) for i in range(20)]
    D = 4096 * 4
    slots = torch.full((20 * D,), 0xAB, dtype=torch.uint8, device="cuda:0")
    st = store_read_device(meta, paths, [slots.data_ptr() + i * D for i in range(20)])
    out = slots.cpu().numpy().reshape(20, D)
    assert st[3] == _native.ABSENT and (out[3] == 0xAB).all()
    for i in range(20):
        if i != 3:
            assert st[i] == 0 and np.array_equal(out[i].view(np.int32), datas[i]), i
    arrs, st2 = store_read(meta, paths, np.int32, pinned=True)
    assert st2[3] == _native.ABSENT
    for i in range(20):
        if i != 3:
            assert st2[i] == 0 and np.array_equal(arrs[i], datas[i]), i
    # the write direction from device slots: files decode with the reference library
    wpaths = [str(tmp_path / "w" / f"c{i}") for i in range(20)]
    wst = store_write_device(meta, wpaths, [slots.data_ptr() + i * D for i in range(20)])
    assert (wst == 0).all()
    for i in (0, 7, 19):
        s = open(wpaths[i], "rb").read()
        rs, dec = zref.decode(zref.GZIP, s, D, 4, True, False)
        assert rs == zref.OK and np.frombuffer(dec, "<i4").tolist() == datas[i].tolist()


def test_store_read_under_low_descriptor_limit(tmp_path):
    """More chunk files than RLIMIT_NOFILE: the reader pool holds at most one
    descriptor per thread (no EMFILE -> 'Other' for small chunks)."""
    import resource
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([1500 * 2048], [2048], "<i2", Lz4(65536))
    h.create_array("s", meta)
    datas = [_walk(2048, 9000 + i) for i in range(1500)]
    h.write_chunks("s", meta, [SliceDataChunk([i], d) for i, d in enumerate(datas)])
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    resource.setrlimit(resource.RLIMIT_NOFILE, (256, hard))
    try:
        got = h.read_chunks("s", meta, [[i] for i in range(1500)], np.int16)
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))
    for i in range(1500):
        assert np.array_equal(got[i].get_data(), datas[i]), i


def test_write_ndarray_takes_the_store_locks(tmp_path):
    """write_ndarray writes through set(): it waits for a reader's shared lock
    and does not truncate the chunk before it holds the exclusive lock
    (filesystem.rs:268-275); read_ndarray waits for a writer's exclusive lock
    (get(), filesystem.rs:201-210)."""
    from zarr_amd.region import BoundingBox, read_ndarray, write_ndarray
    h = FilesystemHierarchy.open_or_create(str(tmp_path))
    meta = ArrayMetadata.new([64, 48], [16, 16], "<i2", Gzip(6))
    h.create_array("r", meta)
    base = (np.arange(64 * 48) % 3000).astype(np.int16).reshape(64, 48)
    write_ndarray(h, "r", meta, [0, 0], base)
    p = h.chunk_path("r", meta, [1, 1])
    before = open(p, "rb").read()
    patch = np.full((20, 20), -7, np.int16)
    res = {}
    with open(p, "rb") as f:
        fcntl.flock(f, fcntl.LOCK_SH)  # a reader holds chunk (1, 1)
        t = threading.Thread(target=lambda: res.setdefault("w", write_ndarray(h, "r", meta, [10, 10], patch)))
        t.start()
        time.sleep(1.0)
        assert t.is_alive(), "write_ndarray did not wait for the shared lock"
        assert open(p, "rb").read() == before  # not truncated before the lock
        fcntl.flock(f, fcntl.LOCK_UN)
    t.join(120)
    assert not t.is_alive()
    want = base.copy()
    want[10:30, 10:30] = -7
    with open(p, "rb+") as f:
        fcntl.flock(f, fcntl.LOCK_EX)  # a writer holds chunk (1, 1)
        t = threading.Thread(target=lambda: res.setdefault(
            "r", read_ndarray(h, "r", meta, BoundingBox([0, 0], [64, 48]), np.int16)))
        t.start()
        time.sleep(1.0)
        assert t.is_alive(), "read_ndarray did not wait for the exclusive lock"
        fcntl.flock(f, fcntl.LOCK_UN)
    t.join(120)
    assert np.array_equal(res["r"], want)
