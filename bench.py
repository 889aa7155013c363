#!/usr/bin/env python3
"""Benchmark of the MI355X Zarr chunk-codec path (driver contract).

Headline workload (BASELINE.json configs[1], "C2"): gzip level-6 chunks of
f32 256x256x4 (1 MiB decoded), batch of 4096 device-resident chunks per GPU,
decoded by one zcg_decode_batch call per step.  A step = one decode of the
whole batch.  Inputs are synthetic ("quant" distribution of SURVEY §8(d),
seeded), encoded on the host with the system zlib 1.2.11 (the library the
reference's flate2 `zlib` backend wraps) using flate2's header convention.
A pool of distinct chunks is replicated into distinct HBM slots (compressed
AND decoded buffers each have their own address) up to the batch size.

The same JSON line carries "per_codec" legs for the other CompressionTypes:
  * lz4 = C4 (configs[3]): i16 random-walk 1 MiB chunks, a FIXED job of
    65 536 chunks split round-robin over the ranks (strong scaling), streams
    made on the host by liblz4's LZ4F streaming API with lz4-rs's settings
    (lz.rs:85-92: level 0, independent 64 KiB blocks, content checksum);
  * raw, xz (liblzma preset 6, CRC64), bzip2 (libbz2 level 9) decode;
  * encode legs (C5 = gzip level 6 f32) with device time and CPU baselines;
  * region assembly (read_ndarray's scatter).
`--codec lz4|raw|xz|bzip2` makes one of them the headline instead.

N>1: one process per GPU (torch.distributed, RCCL only for the barrier and
the max-over-ranks time).  Chunks are independent, so each rank decodes its
own chunks with no data-path collective: weak scaling for the headline
(4 096 chunks per GPU), strong scaling with `--global-batch G` (G chunks
split round-robin, chunk g -> rank g mod N; C4's leg always runs this way).
value = decoded bytes of ALL ranks / max rank time.

roofline: algorithmic bytes per launch = sum(C + D) over the batch (C =
compressed stream bytes read once, D = decoded bytes written once) / the
decode launch's average duration measured with HIP events on the stream the
kernel runs on.  traffic: memory-side bytes per launch from rocprofv3 --pmc
passes over the same bench leg (tools/pmc_traffic.sh ->
profiles/<round>_pmc_traffic.json): reads = the L2's sized read requests
(every miss is one 128 B request, profiles/r05_pmc_calibration.json), writes =
WRITE_SIZE; Infinity-Cache hits are included, so it bounds HBM bytes above.
cpu_baseline: the oracle (the reference's C codec libraries via
oracle/zref.c) on host threads over a bounded sample, rank 0, N=1 only, at
T = every CPU this process may run on and at T = 1.
"""
import argparse
import ctypes
import ctypes.util
import json
import os
import struct
import sys
import time
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "decoded chunk GiB/s (device-resident) per CompressionType at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
GIB = float(1 << 30)
# The kernels one zcg_decode_batch call launches (kernel_ms and roofline.traffic
# cover the whole sequence: HIP events around the call, PMC summed per call).
KERNEL = {"gzip": "zcg::inflate_wave_kernel", "lz4": "zcg::lz4_{frames,lanes,finish}_kernel",
          "raw": "zcg::raw_kernel", "xz": "zcg::xz_decode_kernel<{7990,14134}u, 4096u>",
          "bzip2": "zcg::bz2_{init,stage_a,stage_bc,decode}_kernel"}
# per-codec leg shapes: pool of distinct chunks, chunks per rank (weak) or per job (strong)
LEG = {"gzip": {"pool": 64, "batch": 4096, "strong": False},
       "lz4": {"pool": 512, "batch": 65536, "strong": True},   # C4: fixed 65 536-chunk job
       "raw": {"pool": 64, "batch": 1024, "strong": False},
       "xz": {"pool": 64, "batch": 2048, "strong": False},
       "bzip2": {"pool": 64, "batch": 4096, "strong": False}}
# encode legs: chunks per rank, timed steps
ENCODE_LEG = {"gzip": (512, 2), "lz4": (1024, 3), "xz": (1024, 2), "bzip2": (512, 2)}
# committed PMC traffic passes, newest first: a leg takes the first file that
# measured it at the bench's own batch (kernels change between rounds)
TRAFFIC_FILES = [os.path.join(ROOT, "profiles", f) for f in ("r06_pmc_traffic.json", "r05_pmc_traffic.json", "r04_pmc_traffic.json", "r03_pmc_traffic.json",
                                                              "r02_pmc_traffic.json")]


# ---------------------------------------------------------------- inputs ----
def quant_chunk(idx: int) -> np.ndarray:
    """SURVEY §8(d) C2 "quant": v = round(64*(100*sin(0.05*(i+phi))*cos(0.03*j)+k))/64."""
    i = np.arange(256, dtype=np.float64)[:, None, None]
    j = np.arange(256, dtype=np.float64)[None, :, None]
    k = np.arange(4, dtype=np.float64)[None, None, :]
    phi = idx * 7
    v = np.round(64 * (100 * np.sin(0.05 * (i + phi)) * np.cos(0.03 * j) + k)) / 64
    return v.astype("<f4").reshape(-1)


def randwalk_chunk(idx: int, n: int = 524288) -> np.ndarray:
    """cumsum(rng.integers(-3,4)) with default_rng(1+idx)."""
    rng = np.random.default_rng(1 + idx)
    return np.cumsum(rng.integers(-3, 4, n)).astype("<i2")


def gzip_flate2(payload: bytes, level: int = 6) -> bytes:
    """flate2 GzEncoder framing (gzip.rs:53-56): mtime 0, XFL 0 at level 6, OS 255."""
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
    body = c.compress(payload) + c.flush()
    xfl = 2 if level >= 9 else (4 if level <= 1 else 0)
    hdr = bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, xfl, 255])
    return hdr + body + struct.pack("<II", zlib.crc32(payload), len(payload) & 0xFFFFFFFF)


class _LZ4FFrameInfo(ctypes.Structure):  # lz4frame.h (liblz4 1.9.x)
    _fields_ = [("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int),
                ("contentChecksumFlag", ctypes.c_int), ("frameType", ctypes.c_int),
                ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
                ("blockChecksumFlag", ctypes.c_int)]


class _LZ4FPrefs(ctypes.Structure):
    _fields_ = [("frameInfo", _LZ4FFrameInfo), ("compressionLevel", ctypes.c_int),
                ("autoFlush", ctypes.c_uint), ("favorDecSpeed", ctypes.c_uint),
                ("reserved", ctypes.c_uint * 3)]


_LZ4 = None


def _liblz4():
    global _LZ4
    if _LZ4 is None:
        L = ctypes.CDLL(ctypes.util.find_library("lz4") or "liblz4.so.1")
        sz, vp = ctypes.c_size_t, ctypes.c_void_p
        L.LZ4F_isError.argtypes, L.LZ4F_isError.restype = [sz], ctypes.c_uint
        L.LZ4F_createCompressionContext.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        L.LZ4F_freeCompressionContext.argtypes = [vp]
        L.LZ4F_compressBegin.argtypes = [vp, vp, sz, ctypes.POINTER(_LZ4FPrefs)]
        L.LZ4F_compressBound.argtypes = [sz, ctypes.POINTER(_LZ4FPrefs)]
        L.LZ4F_compressUpdate.argtypes = [vp, vp, sz, vp, sz, vp]
        L.LZ4F_compressEnd.argtypes = [vp, vp, sz, vp]
        L.LZ4F_createDecompressionContext.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
        L.LZ4F_freeDecompressionContext.argtypes = [vp]
        L.LZ4F_decompress.argtypes = [vp, vp, ctypes.POINTER(sz), vp, ctypes.POINTER(sz), vp]
        for f in ("LZ4F_compressBegin", "LZ4F_compressBound", "LZ4F_compressUpdate", "LZ4F_compressEnd",
                  "LZ4F_createCompressionContext", "LZ4F_freeCompressionContext", "LZ4F_decompress",
                  "LZ4F_createDecompressionContext", "LZ4F_freeDecompressionContext"):
            getattr(L, f).restype = sz
        _LZ4 = L
    return _LZ4


def lz4rs_frame(payload: bytes, block: int = 65536) -> bytes:
    """Input synthesis with the system liblz4 (the library lz4-rs wraps),
    configured as lz4-rs's EncoderBuilder in lz.rs:85-92: level 0, BlockMode
    Independent, content checksum on, block size 64 KiB; fed through the
    streaming API one block-size piece per LZ4F_compressUpdate."""
    L = _liblz4()
    p = _LZ4FPrefs()
    p.frameInfo.blockSizeID = {65536: 4, 262144: 5, 1048576: 6, 4194304: 7}[block]
    p.frameInfo.blockMode = 1
    p.frameInfo.contentChecksumFlag = 1
    ctx = ctypes.c_void_p()
    assert not L.LZ4F_isError(L.LZ4F_createCompressionContext(ctypes.byref(ctx), 100))
    cap = L.LZ4F_compressBound(block, ctypes.byref(p)) + 64
    buf = ctypes.create_string_buffer(cap)
    src = ctypes.create_string_buffer(payload, len(payload))
    out = []
    try:
        r = L.LZ4F_compressBegin(ctx, buf, cap, ctypes.byref(p))
        assert not L.LZ4F_isError(r)
        out.append(buf.raw[:r])
        for off in range(0, len(payload), block):
            k = min(block, len(payload) - off)
            r = L.LZ4F_compressUpdate(ctx, buf, cap, ctypes.addressof(src) + off, k, None)
            assert not L.LZ4F_isError(r)
            out.append(buf.raw[:r])
        r = L.LZ4F_compressEnd(ctx, buf, cap, None)
        assert not L.LZ4F_isError(r)
        out.append(buf.raw[:r])
    finally:
        L.LZ4F_freeCompressionContext(ctx)
    return b"".join(out)


def lz4f_decompress(stream: bytes, n: int) -> bytes:
    """The system liblz4's LZ4F_decompress (an independent check of GPU-encoded frames)."""
    L = _liblz4()
    ctx = ctypes.c_void_p()
    assert not L.LZ4F_isError(L.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100))
    dst = ctypes.create_string_buffer(max(n, 1))
    src = ctypes.create_string_buffer(stream, len(stream))
    try:
        ds, ss = ctypes.c_size_t(n), ctypes.c_size_t(len(stream))
        r = L.LZ4F_decompress(ctx, dst, ctypes.byref(ds), src, ctypes.byref(ss), None)
        assert not L.LZ4F_isError(r) and r == 0, "LZ4F_decompress failed"
        return dst.raw[:ds.value]
    finally:
        L.LZ4F_freeDecompressionContext(ctx)


def workload(codec: str):
    """(meta, value generator, description) of each codec's bench shape."""
    from zarr_amd import ArrayMetadata, Gzip, Lz4, Raw
    from zarr_amd.compression import Bzip2, Xz
    if codec == "bzip2":  # bzip.rs default blockSize 9 on the C2 data shape
        meta = ArrayMetadata.new([256 * 64, 256 * 64, 4], [256, 256, 4], "<f4", Bzip2(9))
        return meta, quant_chunk, "bzip2 level 9 f32 256x256x4 (1 MiB) chunks, decode"
    if codec == "xz":  # xz2 default preset 6 on the C2 data shape
        meta = ArrayMetadata.new([256 * 64, 256 * 64, 4], [256, 256, 4], "<f4", Xz(6))
        return meta, quant_chunk, "xz preset 6 f32 256x256x4 (1 MiB) chunks, decode"
    if codec == "gzip":
        meta = ArrayMetadata.new([256 * 64, 256 * 64, 4], [256, 256, 4], "<f4", Gzip(6))
        return meta, quant_chunk, "C2: gzip f32 256x256x4 (1 MiB) chunks, decode"
    if codec == "lz4":
        meta = ArrayMetadata.new([128 * 64, 64 * 64, 64], [128, 64, 64], "<i2", Lz4(65536))
        return meta, randwalk_chunk, "C4: lz4 i16 128x64x64 (1 MiB) chunks, decode"
    meta = ArrayMetadata.new([128 * 64, 64 * 64, 64], [128, 64, 64], "<i2", Raw())
    return meta, randwalk_chunk, "raw i16 128x64x64 (1 MiB) chunks, decode"


def host_encode(codec, vals, threads):
    """Compressed pool made by the reference's own C libraries (system builds)."""
    from concurrent.futures import ThreadPoolExecutor
    if codec == "gzip":
        f = lambda a: gzip_flate2(a.tobytes(), 6)  # noqa: E731  (zlib releases the GIL)
    elif codec == "lz4":
        f = lambda a: lz4rs_frame(a.tobytes(), 65536)  # noqa: E731
    elif codec == "bzip2":
        import bz2
        f = lambda a: bz2.compress(a.tobytes(), 9)  # noqa: E731  BzEncoder(Compression::new(9))
    elif codec == "xz":
        import lzma  # xz2 XzEncoder = lzma_easy_encoder(preset 6, CRC64)
        f = lambda a: lzma.compress(a.tobytes(), format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64,  # noqa: E731
                                    preset=6)
    else:
        return [v.tobytes() for v in vals]
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(f, vals))


def host_decode_check(codec, stream: bytes, n: int) -> bytes:
    """Decode one GPU-encoded stream with the system library the reference wraps."""
    if codec == "gzip":
        return zlib.decompress(stream, 31)
    if codec == "lz4":
        return lz4f_decompress(stream, n)
    if codec == "bzip2":
        import bz2
        return bz2.decompress(stream)
    if codec == "xz":
        import lzma
        return lzma.decompress(stream, format=lzma.FORMAT_XZ)
    return stream


# ------------------------------------------------------ partition + timing ----
def chunk_ids(rank: int, world: int, batch: int, strong: bool):
    """This rank's global chunk ids (chunk g -> GPU g mod N):
    strong = a fixed job of `batch` chunks split over the ranks; weak =
    `batch` chunks per rank."""
    from zarr_amd.shard import round_robin_ids, split_round_robin
    return split_round_robin(batch, rank, world) if strong else round_robin_ids(rank, world, batch)


def timed_region(step, steps: int, world: int, sync, device=None):
    """The contract's timed region: barrier + sync on both sides of exactly
    `steps` steps; returns (local wall seconds, max over ranks)."""
    from zarr_amd.shard import max_over_ranks
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    wall = time.perf_counter() - t0
    return wall, (max_over_ranks(wall, device) if world > 1 else wall)


def timed_launches(step, steps, world, stream, dev):
    """timed_region over `steps` launches, each bracketed by HIP events on
    the launch stream: (wall, max over ranks, mean device ms per launch)."""
    import torch
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    it = iter(evs)

    def one():
        a, b = next(it)
        a.record(stream)
        step()
        b.record(stream)

    wall, t_max = timed_region(one, steps, world, torch.cuda.synchronize, dev)
    return wall, t_max, sum(a.elapsed_time(b) for a, b in evs) / steps


def pmc_traffic(leg, n):
    """HBM bytes per launch (decode) or per encode call of bench leg `leg` at
    batch n, from the committed rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes
    over this same leg (tools/pmc_traffic.sh -> tools/pmc_traffic.py).  None
    unless the pass was taken at this batch (no scaling between batches)."""
    f = traffic_file(leg)
    if f is None:
        return None
    e = json.load(open(f))["legs"][leg]
    return int(e["traffic_bytes"]) if int(e["batch_per_gpu"]) == int(n) else None


def traffic_file(leg):
    """The newest committed traffic file that measured `leg`."""
    for f in TRAFFIC_FILES:
        try:
            if leg in json.load(open(f))["legs"]:
                return f
        except (OSError, KeyError, ValueError):
            continue
    return None


# ------------------------------------------------------------------ legs ----
def decode_leg(codec, batch, strong, steps, warmup, pool, rank, world, dev, threads):
    """Decode this rank's chunks (device-resident), `steps` timed launches.
    Returns (result dict, vals, streams)."""
    import torch
    from zarr_amd.batch import BatchCodec
    meta, gen, desc_txt = workload(codec)
    vals = [gen(i) for i in range(pool)]
    streams = host_encode(codec, vals, threads)
    D = vals[0].nbytes
    ids = chunk_ids(rank, world, batch, strong)
    n = len(ids)
    order = np.array([g % pool for g in ids], np.int64)  # chunk g's content = pool entry g mod pool
    lens = np.array([len(s) for s in streams], np.int64)
    slot = int((lens.max() + 255) // 256 * 256)
    host_pool = np.zeros((pool, slot), np.uint8)
    for u, s in enumerate(streams):
        host_pool[u, :len(s)] = np.frombuffer(s, np.uint8)
    pool_dev = torch.from_numpy(host_pool).to(dev)
    src = pool_dev.index_select(0, torch.from_numpy(order).to(dev))  # [n, slot]: every chunk its own slot
    del pool_dev
    dst = torch.empty(n * D, dtype=torch.uint8, device=dev)
    desc = np.stack([src.data_ptr() + np.arange(n, dtype=np.uint64) * slot, lens[order].astype(np.uint64),
                     dst.data_ptr() + np.arange(n, dtype=np.uint64) * D, np.full(n, D, np.uint64)], 1)
    desc_dev = torch.from_numpy(np.ascontiguousarray(desc).view(np.int64)).to(dev)
    status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    comp_bytes = int(lens[order].sum())
    algo_bytes = comp_bytes + n * D  # C + D per launch
    bc = BatchCodec(dev.index or 0)
    stream = torch.cuda.current_stream(dev)

    class _P:  # PackedStreams-shaped view for BatchCodec.decode
        pass
    packed = _P()
    packed.n, packed.desc, packed.status = n, desc_dev, status

    def step():
        bc.decode(meta, packed, stream=stream)

    for _ in range(max(warmup, 1)):  # the parity gate needs one decoded batch
        step()
    torch.cuda.synchronize()
    # parity gate on the bench data: every chunk bit-exact against its input
    st = status.cpu().numpy()
    assert (st == 0).all(), f"{codec}: decode status != Ok for {int((st != 0).sum())} chunks"
    ref = torch.from_numpy(np.stack([v.view(np.uint8) for v in vals])).to(dev)
    out = dst.view(n, D)
    bad = 0
    ord_dev = torch.from_numpy(order).to(dev)
    for c0 in range(0, n, 256):  # slices keep the gate's temporaries small
        bad += int((out[c0:c0 + 256] != ref[ord_dev[c0:c0 + 256]]).any(dim=1).sum().item())
    assert bad == 0, f"{codec}: {bad} chunks differ from their input"
    del ref, out
    _, t_max, kern_ms = timed_launches(step, steps, world, stream, dev)
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    total_n = batch if strong else world * n
    res = {
        "workload": desc_txt, "value": round(total_n * D * steps / t_max / GIB, 3), "unit": "GiB/s",
        "ms_per_step": round(t_max / steps * 1e3, 3), "batch_per_gpu": n, "job_chunks": total_n,
        "scaling": "strong" if strong else "weak", "chunk_bytes": D,
        "compressed_bytes_per_gpu": comp_bytes, "ratio": round(n * D / comp_bytes, 3),
        "input_streams": "system zlib/liblz4/libbz2/liblzma with the reference crates' settings",
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": pmc_traffic(codec, n),
                     "traffic_source": os.path.relpath(traffic_file(codec) or TRAFFIC_FILES[-1], ROOT) +
                                       " (sized read requests + WRITE_SIZE per launch, same leg and batch; "
                                       "multipliers profiles/r05_pmc_calibration.json)",
                     "kernel": KERNEL[codec], "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": algo_bytes},
    }
    del src, dst, packed, desc_dev, status
    torch.cuda.empty_cache()
    return res, vals, streams


def encode_leg(codec, n, steps, warmup, pool, rank, world, dev, cpu_seconds=0.0, threads_all=1):
    """GPU encode throughput (input GiB/s) of `n` chunks per rank, device
    time from HIP events, a sample of streams decoded by the system library,
    and (rank 0, N=1) the oracle's CPU encode of the same chunks."""
    import torch
    from zarr_amd.batch import BatchCodec, make_encode_batch
    meta, gen, desc_txt = workload(codec)
    vals = [gen(i) for i in range(pool)]
    D = vals[0].nbytes
    ids = chunk_ids(rank, world, n, False)
    host = np.concatenate([vals[g % pool].view(np.uint8) for g in ids])
    elems = torch.from_numpy(host).to(dev)
    del host
    bc = BatchCodec(dev.index or 0)
    cap = bc.encode_bound(meta, D)
    desc, dst, out_len, status = make_encode_batch(elems, n, cap, dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(max(warmup, 1)):
        bc.encode(meta, desc, n, out_len, status, stream=stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    ol = out_len.cpu().numpy()
    out_bytes = int(ol.sum())
    # decodability: a sample of the streams through the reference's library,
    # and whether the bytes equal the reference library's own stream
    same = 0
    sample = sorted({0, 1, n // 2, n - 1})
    for i in sample:
        s = dst[i * cap:i * cap + int(ol[i])].cpu().numpy().tobytes()
        assert host_decode_check(codec, s, D) == vals[ids[i] % pool].tobytes(), f"{codec} encode: chunk {i}"
        same += int(s == host_encode(codec, [vals[ids[i] % pool]], 1)[0])
    _, t_max, dev_ms = timed_launches(lambda: bc.encode(meta, desc, n, out_len, status, stream=stream),
                                      steps, world, stream, dev)
    achieved = (n * D + out_bytes) / (dev_ms * 1e-3) / 1e9
    sub = vals[:8]
    ref_ratio = round(len(sub) * D / sum(len(s) for s in host_encode(codec, sub, 8)), 3)
    res = {"workload": desc_txt.replace("decode", "encode"), "direction": "encode",
           "ref_ratio": ref_ratio, "ref_ratio_source": "the reference's library on 8 pool chunks",
           "value": round(world * n * D * steps / t_max / GIB, 3), "unit": "GiB/s (input)",
           "ms_per_step": round(t_max / steps * 1e3, 3), "device_ms": round(dev_ms, 3),
           "batch_per_gpu": n, "ratio": round(n * D / out_bytes, 3), "decoded_sample_ok": True,
           "bytes_equal_reference_sample": f"{same}/{len(sample)}",
           "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                        "traffic": pmc_traffic(f"{codec}_encode", n),
                        "traffic_source": os.path.relpath(traffic_file(f"{codec}_encode") or TRAFFIC_FILES[-1], ROOT) +
                                          " (all encode kernels per call, same leg and batch)",
                        "algorithmic_bytes_per_launch": n * D + out_bytes}}
    del elems, dst, desc, out_len, status
    torch.cuda.empty_cache()
    if cpu_seconds > 0 and rank == 0 and world == 1:
        res["cpu_baseline"] = cpu_encode_leg(codec, vals, cpu_seconds, threads_all)
    return res


def region_leg(steps, dev):
    """Region assembly (read_ndarray's scatter, ndarray.rs:195-268) of 1 024
    decoded f32 256x256x4 chunks (1 GiB, F order) already in HBM into a box
    at an unaligned offset; roofline bytes = box bytes read + written."""
    import torch
    from zarr_amd import ArrayMetadata
    from zarr_amd.region import BoundingBox, assemble_region, region_grid, _strides
    meta = ArrayMetadata.new([256 * 32, 256 * 32, 4], [256, 256, 4], "<f4")
    off, shp = [100, 37, 0], [256 * 32 - 200, 256 * 32 - 100, 4]
    bbox = BoundingBox(off, shp)
    lo, n = region_grid(meta, bbox)
    N = 256 * 256 * 4
    nch = n[0] * n[1] * n[2]
    g = torch.Generator(device=dev).manual_seed(3)
    slots = torch.randint(-2**31, 2**31 - 1, (nch * N,), dtype=torch.int32, device=dev, generator=g)
    table = torch.tensor([slots.data_ptr() + i * N * 4 for i in range(nch)], dtype=torch.int64, device=dev)
    total = shp[0] * shp[1] * shp[2]
    out = torch.empty(total, dtype=torch.int32, device=dev)
    st = _strides(shp, "F")
    stream = torch.cuda.current_stream(dev)
    assemble_region(meta, bbox, 4, table, out, st, True, 0, dev.index or 0, stream)
    torch.cuda.synchronize()
    # gate: 4096 random elements against the index math of ndarray.rs:234-258
    rng = np.random.default_rng(0)
    idx = [rng.integers(0, s, 4096) for s in shp]
    gpos = [i + o for i, o in zip(idx, off)]
    c = [p // cs for p, cs in zip(gpos, meta.chunk_shape)]
    w = [p % cs for p, cs in zip(gpos, meta.chunk_shape)]
    ci = (c[0] - lo[0]) * n[1] * n[2] + (c[1] - lo[1]) * n[2] + (c[2] - lo[2])
    src = torch.from_numpy(ci * N + w[0] + 256 * (w[1] + 256 * w[2])).to(dev)
    dst = torch.from_numpy(idx[0] + shp[0] * (idx[1] + shp[1] * idx[2])).to(dev)
    assert bool((out[dst] == slots[src]).all()), "region: assembled elements differ"
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(steps):
        assemble_region(meta, bbox, 4, table, out, st, True, 0, dev.index or 0, stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    byts = 2 * total * 4
    achieved = byts / (ms * 1e-3) / 1e9
    del slots, out
    torch.cuda.empty_cache()
    return {"workload": "read_ndarray region assembly: 1024 decoded f32 256x256x4 chunks (F order) -> "
                        f"box {shp} at offset {off}", "value": round(total * 4 / (ms * 1e-3) / GIB, 2),
            "unit": "GiB/s (box)", "ms_per_step": round(ms, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel": "zcg::region_rows_kernel",
                         "algorithmic_bytes_per_launch": byts}}


# ------------------------------------------------------------ CPU baseline ----
CPU_LIB = {"gzip": "zlib 1.2.11 inflate + flate2 header rules",
           "lz4": "liblz4 1.9.3 LZ4F (lz4-rs feeding)", "raw": "memcpy",
           "xz": "liblzma 5.2.5 stream decoder (xz2 feeding)",
           "bzip2": "libbz2 1.0.8 (bzip2-rs feeding)"}
CPU_ENC_LIB = {"gzip": "zlib 1.2.11 deflate level 6 + flate2 GzEncoder framing",
               "lz4": "liblz4 1.9.3 LZ4F streaming (lz4-rs settings)",
               "xz": "liblzma 5.2.5 easy encoder preset 6 CRC64", "bzip2": "libbz2 1.0.8 level 9"}


def host_cpu_info():
    """What the CPU baseline ran on: model, CPUs this process may use, the
    machine's count and the cgroup CPU quota (the GPU box shares its host)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    usable = aff if quota is None else max(1, min(aff, int(-(-quota // 1))))
    return {"cpu_model": model, "usable_cpus": usable, "affinity_cpus": aff, "os_cpu_count": os.cpu_count(),
            "cgroup_cpu_quota": quota}


def _oracle():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import zref  # oracle: CPU baseline leg only
    return zref


def _cpu_decode_rate(codec, streams, D, seconds, threads):
    zref = _oracle()
    cid = {"gzip": zref.GZIP, "lz4": zref.LZ4, "raw": zref.RAW, "xz": zref.XZ, "bzip2": zref.BZIP2}[codec]
    es = {"gzip": 4, "lz4": 2, "raw": 2, "xz": 4, "bzip2": 4}[codec]
    srcs = [np.frombuffer(s, np.uint8) for s in streams]
    dsts = [np.empty(D, np.uint8) for _ in srcs]
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < seconds:
        st, _ = zref.decode_batch(cid, srcs, D, elem_size=es, threads=threads, dsts=dsts)
        assert (st == 0).all()
        done += len(srcs)
    el = time.perf_counter() - t0
    cbytes = sum(len(s) for s in streams) * (done // max(len(srcs), 1))
    return done * D / el / GIB, done, el, (cbytes + done * D) / el / 1e9


def cpu_leg(codec, streams, D, seconds, threads_all):
    """The oracle (reference C codec libraries, oracle/zref.c) decoding the
    same pool on host threads: T = the CPUs this process may use (affinity
    capped by the cgroup quota) for `seconds`, T = 1 for a third of that —
    cpu_baseline only.  value = decoded GiB/s; value_cd_gbs = (C + D) GB/s,
    the roofline's algorithmic bytes."""
    v, done, el, cd = _cpu_decode_rate(codec, streams, D, seconds, threads_all)
    v1, done1, el1, cd1 = _cpu_decode_rate(codec, streams[:8], D, max(1.0, seconds / 3), 1)
    info = host_cpu_info()
    return {"value": round(v, 4), "unit": "GiB/s", "cores": threads_all, "kind": "port",
            "value_cd_gbs": round(cd, 3), "value_t1": round(v1, 4), **info,
            "sample": f"{done} decodes of the {len(streams)}-chunk pool (1 MiB each) by {CPU_LIB[codec]} "
                      f"(oracle/zref.c), {threads_all} threads, {el:.1f} s; T=1: {done1} decodes, {el1:.1f} s"}


def compact_leg(r):
    """A per_codec leg as it goes on the bench line (the full record stays in
    DESIGN.md): value, time, batch, ratio, roofline fraction, PMC traffic as a
    multiple of the algorithmic bytes, kernel ms, CPU baseline [T=usable, T=1,
    usable CPUs]."""
    rf = r.get("roofline", {})
    out = {"value": r["value"], "unit": r["unit"], "ms": r.get("ms_per_step"),
           "batch": r.get("batch_per_gpu"), "ratio": r.get("ratio"), "frac": rf.get("frac"),
           "kernel_ms": rf.get("kernel_ms", r.get("device_ms"))}
    tr, ab = rf.get("traffic"), rf.get("algorithmic_bytes_per_launch")
    if tr and ab:
        out["traffic_x"] = round(tr / ab, 2)
    if "ref_ratio" in r:
        out["ref_ratio"] = r["ref_ratio"]
    if "bytes_equal_reference_sample" in r:
        out["same_bytes"] = r["bytes_equal_reference_sample"]
    cb = r.get("cpu_baseline")
    if cb:
        out["cpu"] = [cb["value"], cb["value_t1"], cb["cores"]]
    return out


def cpu_encode_leg(codec, vals, seconds, threads_all):
    """The oracle's write_chunk restatement (the reference's encoder library)
    on host threads: T = all usable CPUs and T = 1."""
    zref = _oracle()
    cid, param = {"gzip": (zref.GZIP, 6), "lz4": (zref.LZ4, 65536), "xz": (zref.XZ, 6),
                  "bzip2": (zref.BZIP2, 9)}[codec]
    es = vals[0].dtype.itemsize
    srcs = [np.ascontiguousarray(v).view(np.uint8) for v in vals]
    D = vals[0].nbytes

    def rate(sub, secs, threads):
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < secs:
            st, _ = zref.encode_batch(cid, param, [s.view(vals[0].dtype) for s in sub], elem_size=es,
                                      threads=threads)
            assert (st == 0).all()
            done += len(sub)
        el = time.perf_counter() - t0
        return done * D / el / GIB, done, el
    v, done, el = rate(srcs, seconds, threads_all)
    v1, done1, el1 = rate(srcs[:2], max(1.0, seconds / 3), 1)
    return {"value": round(v, 4), "unit": "GiB/s (input)", "cores": threads_all, "kind": "port",
            "value_t1": round(v1, 4), **host_cpu_info(),
            "sample": f"{done} encodes of the {len(srcs)}-chunk pool (1 MiB each) by {CPU_ENC_LIB[codec]} "
                      f"(oracle/zref.c), {threads_all} threads, {el:.1f} s; T=1: {done1} encodes, {el1:.1f} s"}


# ------------------------------------------------------------------ main ----
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--codec", default="gzip", choices=["gzip", "lz4", "raw", "xz", "bzip2"])
    ap.add_argument("--batch", type=int, default=None, help="chunks per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="chunks of the whole job, split round-robin over the GPUs (strong scaling)")
    ap.add_argument("--pool", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the per_codec legs")
    ap.add_argument("--legs", default="lz4,raw,xz,bzip2,gzip,encode,region",
                    help="per_codec legs to run (comma list)")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    threads_all = host_cpu_info()["usable_cpus"]
    pool_threads = max(1, min(16, threads_all))  # input synthesis only
    cfg = dict(LEG[args.codec])
    if args.global_batch:
        cfg["batch"], cfg["strong"] = args.global_batch, True
    elif args.batch:
        cfg["batch"], cfg["strong"] = args.batch, False
    pool = args.pool or cfg["pool"]
    main_res, vals, streams = decode_leg(args.codec, cfg["batch"], cfg["strong"], args.steps, args.warmup, pool,
                                         rank, world, dev, pool_threads)
    D = vals[0].nbytes
    result = {
        "metric": METRIC, "value": main_res["value"], "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": main_res["ms_per_step"],
        "higher_is_better": True, "scaling": main_res["scaling"], "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (SURVEY §8(d) distributions, seeded; streams made by the reference's C codec "
                "libraries; a pool of distinct chunks replicated into distinct HBM slots; every chunk "
                "gated bit-exact before timing)",
        "config": {"workload": main_res["workload"], "codec": args.codec,
                   "batch_per_gpu": main_res["batch_per_gpu"], "job_chunks": main_res["job_chunks"],
                   "chunk_bytes": D, "compressed_bytes_per_gpu": main_res["compressed_bytes_per_gpu"],
                   "ratio": main_res["ratio"], "parallelism": f"chunks round-robin x{world}"},
        "roofline": main_res["roofline"],
    }
    del vals
    if not args.no_extra:
        legs = [x for x in args.legs.split(",") if x]
        per = {}
        for c in ("lz4", "raw", "xz", "bzip2", "gzip"):
            if c == args.codec or c not in legs:
                continue
            lc = LEG[c]
            r, _, s_c = decode_leg(c, lc["batch"], lc["strong"],
                                   2 if c in ("xz", "bzip2", "lz4") else max(3, args.steps // 2), 1,
                                   lc["pool"], rank, world, dev, pool_threads)
            if rank == 0 and world == 1 and not args.no_cpu_baseline and c != "raw":
                r["cpu_baseline"] = cpu_leg(c, s_c, r["chunk_bytes"], 3.0, threads_all)
            per[c] = compact_leg(r)
            del s_c
        cs = 0.0 if args.no_cpu_baseline else 3.0
        for c, (nb, st) in ENCODE_LEG.items():  # gzip = C5
            if "encode" in legs or f"{c}_encode" in legs:
                per[f"{c}_encode"] = compact_leg(encode_leg(c, nb, st, 1, 64, rank, world, dev, cs,
                                                            threads_all))
        if "region" in legs:
            per["region"] = compact_leg(region_leg(max(3, args.steps), dev))
        result["per_codec"] = per

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_leg(args.codec, streams, D, args.cpu_seconds, threads_all)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
