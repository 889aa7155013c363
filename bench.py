#!/usr/bin/env python3
"""Benchmark of the MI355X Zarr chunk-codec path (driver contract).

Headline workload (BASELINE.json configs[1], "C2"): gzip level-6 chunks of
f32 256x256x4 (1 MiB decoded), batch of 4096 device-resident chunks per GPU,
decoded by one zcg_decode_batch call per step.  A step = one decode of the
whole batch.  Inputs are synthetic ("quant" distribution of SURVEY §8(d),
seeded), encoded on the host with the standard-library zlib (same zlib
1.2.11 as the reference's flate2 backend) using flate2's header convention.
A pool of distinct chunks is replicated into distinct HBM slots (compressed
AND decoded buffers each have their own address) up to the batch size.

The same JSON line carries "per_codec" legs for the other CompressionTypes
on the GPU (metric = decoded GiB/s per CompressionType): LZ4 decode on the C4
shape (i16 random-walk 1 MiB chunks, inputs made by the GPU LZ4 encoder and
gated bit-exact), Raw decode, and LZ4 encode.  `--codec lz4|raw` makes one of
them the headline instead.

N>1: one process per GPU (torch.distributed, RCCL only for the barrier and
the max-over-ranks time).  Chunks are independent, so each rank decodes its
own batch (round-robin partition, no data-path collective): "scaling":
"weak".  value = decoded bytes of ALL ranks / max rank time.

roofline: algorithmic bytes per launch = sum(C + D) over the batch (C =
compressed stream bytes read once, D = decoded bytes written once) / the
decode kernel's average launch time measured with HIP events on the stream
the kernel runs on.  cpu_baseline: the oracle (reference C codec libraries
via oracle/zref.c) on host threads over a bounded sample, rank 0, N=1 only.
"""
import argparse
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
KERNEL = {"gzip": "zcg::inflate_par_kernel", "lz4": "zcg::lz4_decode_kernel", "raw": "zcg::raw_kernel",
          "xz": "zcg::xz_decode_kernel<7990u>", "bzip2": "zcg::bz2_decode_kernel"}


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


class _Batch:  # PackedStreams-shaped holder for BatchCodec.decode
    pass


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


def gpu_encode_pool(meta, vals, dev):
    """Pool streams made by the GPU encoder (zcg_encode_batch)."""
    import torch
    from zarr_amd.batch import BatchCodec, make_encode_batch
    bc = BatchCodec(dev.index or 0)
    D = vals[0].nbytes
    elems = torch.from_numpy(np.concatenate([v.view(np.uint8) for v in vals])).to(dev)
    cap = bc.encode_bound(meta, D)
    desc, dst, out_len, status = make_encode_batch(elems, len(vals), cap, dev)
    bc.encode(meta, desc, len(vals), out_len, status)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all(), "GPU encode failed"
    ol = out_len.cpu().numpy()
    buf = dst.cpu().numpy().reshape(len(vals), cap)
    return [buf[i, :ol[i]].tobytes() for i in range(len(vals))]


def build_pool(codec, meta, gen, pool, threads, dev):
    from concurrent.futures import ThreadPoolExecutor
    vals = [gen(i) for i in range(pool)]
    if codec == "gzip":
        with ThreadPoolExecutor(threads) as ex:  # zlib releases the GIL
            streams = list(ex.map(lambda a: gzip_flate2(a.tobytes(), 6), vals))
    elif codec == "lz4":
        streams = gpu_encode_pool(meta, vals, dev)
    elif codec == "bzip2":
        import bz2
        with ThreadPoolExecutor(threads) as ex:  # BzEncoder(Compression::new(9))
            streams = list(ex.map(lambda a: bz2.compress(a.tobytes(), 9), vals))
    elif codec == "xz":
        import lzma
        with ThreadPoolExecutor(threads) as ex:  # xz2 XzEncoder = easy encoder, preset 6, CRC64
            streams = list(ex.map(lambda a: lzma.compress(a.tobytes(), format=lzma.FORMAT_XZ,
                                                          check=lzma.CHECK_CRC64, preset=6), vals))
    else:
        streams = [v.tobytes() for v in vals]
    return vals, streams


def sync_max(t_local, world, dev):
    """Slowest rank's time (zarr_amd.shard.max_over_ranks; RCCL on GPU ranks)."""
    from zarr_amd.shard import max_over_ranks
    return max_over_ranks(t_local, dev) if world > 1 else t_local


def barrier(world):
    import torch
    if world > 1:
        torch.distributed.barrier()


TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")


def pmc_traffic(kernel, n):
    """HBM bytes per launch of `kernel` at batch n, from the committed
    rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE passes over this same bench leg
    (tools/pmc_traffic.sh -> tools/pmc_traffic.py), scaled to n chunks."""
    try:
        e = json.load(open(TRAFFIC_FILE))["kernels"][kernel]
    except (OSError, KeyError, ValueError):
        return None
    return int(e["traffic_bytes"] * n / e["batch_per_gpu"])


def decode_leg(codec, n, steps, warmup, pool, rank, world, dev, threads):
    """Decode `n` device-resident chunks per rank, `steps` timed launches.
    Returns (result dict, vals, streams)."""
    import torch
    from zarr_amd.batch import BatchCodec
    meta, gen, desc_txt = workload(codec)
    vals, streams = build_pool(codec, meta, gen, pool, threads, dev)
    D = vals[0].nbytes
    ALIGN = 256
    slot = [(len(s) + ALIGN - 1) // ALIGN * ALIGN for s in streams]
    from zarr_amd.shard import round_robin_ids
    # chunk g of the job goes to GPU g mod world; its content
    # is pool entry g mod pool
    order = [g % pool for g in round_robin_ids(rank, world, n)]
    offs = np.zeros(n + 1, np.int64)
    for i, u in enumerate(order):
        offs[i + 1] = offs[i] + slot[u]
    src = torch.empty(int(offs[-1]), dtype=torch.uint8, device=dev)
    pool_dev = [torch.from_numpy(np.frombuffer(s, np.uint8).copy()).to(dev) for s in streams]
    for i, u in enumerate(order):
        src[offs[i]:offs[i] + len(streams[u])].copy_(pool_dev[u])
    dst = torch.empty(n * D, dtype=torch.uint8, device=dev)
    desc = np.zeros((n, 4), np.uint64)
    for i, u in enumerate(order):
        desc[i] = (src.data_ptr() + int(offs[i]), len(streams[u]), dst.data_ptr() + i * D, D)
    packed = _Batch()
    packed.n = n
    packed.desc = torch.from_numpy(desc.view(np.int64)).to(dev)
    packed.status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    comp_bytes = int(sum(len(streams[u]) for u in order))
    algo_bytes = comp_bytes + n * D  # C + D per launch
    bc = BatchCodec(dev.index or 0)
    stream = torch.cuda.current_stream(dev)

    def step():
        bc.decode(meta, packed, stream=stream)

    for _ in range(max(warmup, 1)):  # the parity gate needs one decoded batch
        step()
    torch.cuda.synchronize()
    # parity gate on the bench data: every chunk bit-exact
    st = packed.status.cpu().numpy()
    assert (st == 0).all(), f"{codec}: decode status != Ok for {int((st != 0).sum())} chunks"
    ref = torch.stack([torch.from_numpy(v.view(np.uint8).copy()) for v in vals]).to(dev)
    out = dst.view(n, D)
    bad = 0
    for c0 in range(0, n, 256):  # slices keep the gate's temporaries small
        idx = torch.tensor(order[c0:c0 + 256], device=dev)
        bad += int((out[c0:c0 + 256] != ref[idx]).any(dim=1).sum().item())
    assert bad == 0, f"{codec}: {bad} chunks differ from their input"
    del ref, pool_dev
    # timed region
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    barrier(world)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / steps  # one launch per step
    t_max = sync_max(wall, world, dev)
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    res = {
        "workload": desc_txt, "value": round(world * n * D * steps / t_max / GIB, 3), "unit": "GiB/s",
        "ms_per_step": round(t_max / steps * 1e3, 3), "batch_per_gpu": n, "chunk_bytes": D,
        "compressed_bytes_per_gpu": comp_bytes, "ratio": round(n * D / comp_bytes, 3),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                     "traffic": pmc_traffic(KERNEL[codec], n),
                     "traffic_source": "profiles/r01_pmc_traffic.json (2*FETCH_SIZE + WRITE_SIZE per launch)",
                     "kernel": KERNEL[codec], "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": algo_bytes},
    }
    del src, dst, packed
    torch.cuda.empty_cache()
    return res, vals, streams


def encode_leg(codec, n, steps, warmup, pool, rank, world, dev):
    """GPU encode throughput (input GiB/s) of `n` chunks per rank."""
    import torch
    from zarr_amd.batch import BatchCodec, make_encode_batch
    meta, gen, desc_txt = workload(codec)
    vals = [gen(i) for i in range(pool)]
    D = vals[0].nbytes
    from zarr_amd.shard import round_robin_ids
    host = np.concatenate([vals[g % pool].view(np.uint8) for g in round_robin_ids(rank, world, n)])
    elems = torch.from_numpy(host).to(dev)
    bc = BatchCodec(dev.index or 0)
    cap = bc.encode_bound(meta, D)
    desc, dst, out_len, status = make_encode_batch(elems, n, cap, dev)
    stream = torch.cuda.current_stream(dev)
    for _ in range(max(warmup, 1)):
        bc.encode(meta, desc, n, out_len, status, stream=stream)
    torch.cuda.synchronize()
    assert (status.cpu().numpy() == 0).all()
    out_bytes = int(out_len.sum().item())
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        bc.encode(meta, desc, n, out_len, status, stream=stream)
    torch.cuda.synchronize()
    barrier(world)
    t_max = sync_max(time.perf_counter() - t0, world, dev)
    achieved = (n * D + out_bytes) / (t_max / steps) / 1e9
    ref_ratio = None
    if codec == "gzip":  # C5: ratio of the CPU reference library (zlib level 6) on the same pool
        ref_ratio = round(len(vals) * D / sum(len(gzip_flate2(v.tobytes(), 6)) for v in vals), 3)
    elif codec == "bzip2":  # libbz2 level 9 (bzip2-rs BzEncoder) on 8 pool chunks
        import bz2
        sub = vals[:8]
        ref_ratio = round(len(sub) * D / sum(len(bz2.compress(v.tobytes(), 9)) for v in sub), 3)
    elif codec == "xz":  # liblzma preset 6 (xz2's XzEncoder) on 8 pool chunks
        import lzma
        sub = vals[:8]
        ref_ratio = round(len(sub) * D / sum(len(lzma.compress(v.tobytes(), format=lzma.FORMAT_XZ,
                                                               check=lzma.CHECK_CRC64, preset=6))
                                             for v in sub), 3)
    res = {"workload": desc_txt.replace("decode", "encode"), "direction": "encode",
           "ref_ratio": ref_ratio,
           "value": round(world * n * D * steps / t_max / GIB, 3), "unit": "GiB/s (input)",
           "batch_per_gpu": n, "ratio": round(n * D / out_bytes, 3),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5)}}
    del elems, dst
    torch.cuda.empty_cache()
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
    return {"workload": "read_ndarray region assembly: 1024 decoded f32 256x256x4 chunks (F order) -> "
                        f"box {shp} at offset {off}", "value": round(total * 4 / (ms * 1e-3) / GIB, 2),
            "unit": "GiB/s (box)", "ms_per_step": round(ms, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel": "zcg::region_rows_kernel",
                         "algorithmic_bytes_per_launch": byts}}


CPU_LIB = {"gzip": "zlib 1.2.11 inflate + flate2 header rules",
           "lz4": "liblz4 1.9.3 LZ4F (lz4-rs feeding)", "raw": "memcpy",
           "xz": "liblzma 5.2.5 stream decoder (xz2 feeding)",
           "bzip2": "libbz2 1.0.8 (bzip2-rs feeding)"}


def cpu_leg(codec, streams, D, seconds, threads):
    """The oracle (reference C codec libraries, oracle/zref.c) decoding the
    same pool on host threads for about `seconds` — cpu_baseline only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import zref  # oracle: CPU baseline leg only
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
    return {"value": round(done * D / el / GIB, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{done} decodes of the {len(srcs)}-chunk pool (1 MiB each) by {CPU_LIB[codec]} "
                      f"(oracle/zref.c), {threads} threads, {el:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--codec", default="gzip", choices=["gzip", "lz4", "raw", "xz", "bzip2"])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--pool", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the per_codec legs")
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

    host_threads = max(1, min(16, os.cpu_count() or 1))
    main_res, vals, streams = decode_leg(args.codec, args.batch, args.steps, args.warmup, args.pool,
                                         rank, world, dev, host_threads)
    D = vals[0].nbytes
    result = {
        "metric": METRIC, "value": main_res["value"], "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": main_res["ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (SURVEY §8(d) distributions, seeded; a pool of distinct chunks "
                "replicated into distinct HBM slots; every chunk gated bit-exact before timing)",
        "config": {"workload": main_res["workload"], "codec": args.codec,
                   "batch_per_gpu": main_res["batch_per_gpu"], "chunk_bytes": D,
                   "compressed_bytes_per_gpu": main_res["compressed_bytes_per_gpu"],
                   "ratio": main_res["ratio"], "parallelism": f"chunks round-robin x{world}"},
        "roofline": main_res["roofline"],
    }

    if not args.no_extra:
        per = {}
        for c in ("gzip", "lz4", "raw", "xz", "bzip2"):
            if c == args.codec:
                continue
            n_c = {"lz4": 16384, "xz": 2048, "bzip2": 2048}.get(c, 1024)
            r, _, s_c = decode_leg(c, n_c, 2 if c in ("xz", "bzip2") else max(3, args.steps // 2), 1,
                                   args.pool, rank, world, dev, host_threads)
            if rank == 0 and world == 1 and not args.no_cpu_baseline and c != "raw":
                r["cpu_baseline"] = cpu_leg(c, s_c, r["chunk_bytes"], 3.0, host_threads)
            per[c] = r
        per["lz4_encode"] = encode_leg("lz4", 1024, 3, 1, args.pool, rank, world, dev)
        per["gzip_encode"] = encode_leg("gzip", 512, 2, 1, args.pool, rank, world, dev)  # C5 shape
        per["xz_encode"] = encode_leg("xz", 1024, 2, 1, args.pool, rank, world, dev)
        per["bzip2_encode"] = encode_leg("bzip2", 512, 2, 1, args.pool, rank, world, dev)
        per["region"] = region_leg(max(3, args.steps), dev)
        result["per_codec"] = per

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_leg(args.codec, streams, D, args.cpu_seconds, host_threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
