#!/usr/bin/env python3
"""Benchmark of the MI355X Zarr chunk-codec path (driver contract).

Default workload (BASELINE.json configs[1], "C2"): gzip level-6 chunks of
f32 256x256x4 (1 MiB decoded), batch of 4096 device-resident chunks per GPU,
decoded by one zcg_decode_batch call per step.  A step = one decode of the
whole batch.  Inputs are synthetic ("quant" distribution of SURVEY §8(d),
seeded), encoded on the host with the standard-library zlib (same zlib
1.2.11 as the reference's flate2 backend) using flate2's header convention.
A pool of distinct chunks is replicated into distinct HBM slots (compressed
AND decoded buffers each have their own address) up to the batch size.

N>1: one process per GPU (torch.distributed, RCCL backend only for the
barrier and the max-over-ranks time).  Chunks are independent, so each rank
decodes its own batch (round-robin partition, no data-path collective):
"scaling": "weak".  value = decoded bytes of ALL ranks / max rank time.

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


def build_pool(codec: str, pool: int, threads: int):
    from concurrent.futures import ThreadPoolExecutor
    if codec == "gzip":
        gen = quant_chunk
        enc = lambda a: gzip_flate2(a.tobytes(), 6)  # noqa: E731
    else:
        raise SystemExit(f"codec {codec}: host-side input generation not available")
    vals = [gen(i) for i in range(pool)]
    with ThreadPoolExecutor(threads) as ex:  # zlib releases the GIL
        streams = list(ex.map(enc, vals))
    return vals, streams


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--codec", default="gzip", choices=["gzip"])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--pool", type=int, default=64)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
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

    from zarr_amd import ArrayMetadata, Gzip
    from zarr_amd.batch import BatchCodec

    host_threads = max(1, min(16, os.cpu_count() or 1))
    vals, streams = build_pool(args.codec, args.pool, host_threads)
    D = vals[0].nbytes
    n = args.batch
    meta = ArrayMetadata.new([256 * 64, 256 * 64, 4], [256, 256, 4], "<f4", Gzip(6))

    # ---- device-resident inputs: distinct HBM slots for every chunk ----------
    ALIGN = 256
    slot = [(len(s) + ALIGN - 1) // ALIGN * ALIGN for s in streams]
    order = [(rank * n + i) % args.pool for i in range(n)]  # round-robin pool mapping
    offs = np.zeros(n + 1, np.int64)
    for i, u in enumerate(order):
        offs[i + 1] = offs[i] + slot[u]
    pool_host = [np.frombuffer(s, np.uint8) for s in streams]
    src = torch.empty(int(offs[-1]), dtype=torch.uint8, device=dev)
    pool_dev = [torch.from_numpy(p.copy()).to(dev) for p in pool_host]
    for i, u in enumerate(order):
        src[offs[i]:offs[i] + len(streams[u])].copy_(pool_dev[u])
    dst = torch.empty(n * D, dtype=torch.uint8, device=dev)
    desc = np.zeros((n, 4), np.uint64)
    for i, u in enumerate(order):
        desc[i] = (src.data_ptr() + int(offs[i]), len(streams[u]), dst.data_ptr() + i * D, D)

    class P:  # minimal PackedStreams-compatible holder
        pass
    packed = P()
    packed.n = n
    packed.desc = torch.from_numpy(desc.view(np.int64)).to(dev)
    packed.status = torch.full((n,), -1, dtype=torch.int32, device=dev)
    comp_bytes = int(sum(len(streams[u]) for u in order))
    algo_bytes = comp_bytes + n * D  # C + D per launch

    codec = BatchCodec(local)
    stream = torch.cuda.current_stream(dev)

    def step():
        codec.decode(meta, packed, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- parity gate on the bench data: every chunk bit-exact --------------------
    st = packed.status.cpu().numpy()
    assert (st == 0).all(), f"decode status != Ok for {int((st != 0).sum())} chunks"
    ref = torch.stack([torch.from_numpy(v.view(np.uint8).copy()) for v in vals]).to(dev)
    out = dst.view(n, D)
    idx = torch.tensor(order, device=dev)
    bad = (out != ref[idx]).any(dim=1).sum().item()
    assert bad == 0, f"{bad} chunks differ from their input"
    del ref

    # ---- timed region --------------------------------------------------------------
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # one launch per step
    t_local = wall
    if world > 1:
        t = torch.tensor([t_local], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        t_max = float(t.item())
    else:
        t_max = t_local
    ms_per_step = t_max / args.steps * 1e3
    total_decoded = world * n * D * args.steps
    value = total_decoded / t_max / GIB

    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
    result = {
        "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (SURVEY §8(d) 'quant' f32, zlib-6, flate2 header; 64-chunk pool "
                "replicated into distinct HBM slots)",
        "config": {"workload": "C2: gzip f32 256x256x4 (1 MiB) chunks, decode", "codec": args.codec,
                   "batch_per_gpu": n, "chunk_bytes": D, "compressed_bytes_per_gpu": comp_bytes,
                   "ratio": round(n * D / comp_bytes, 3), "parallelism": f"chunks round-robin x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "kernel": "zcg::inflate_par_kernel", "kernel_ms": round(kern_ms, 4),
                     "algorithmic_bytes_per_launch": algo_bytes},
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import zref  # oracle: CPU baseline leg only
        srcs = [np.frombuffer(s, np.uint8) for s in streams]
        dsts = [np.empty(D, np.uint8) for _ in srcs]
        t0 = time.perf_counter()
        done = 0
        while time.perf_counter() - t0 < args.cpu_seconds:
            st, _ = zref.decode_batch(zref.GZIP, srcs, D, elem_size=4, threads=host_threads, dsts=dsts)
            assert (st == 0).all()
            done += len(srcs)
        el = time.perf_counter() - t0
        result["cpu_baseline"] = {
            "value": round(done * D / el / GIB, 4), "unit": "GiB/s", "cores": host_threads,
            "kind": "port",
            "sample": f"{done} decodes of the {len(srcs)}-chunk pool (1 MiB each) by zlib 1.2.11 "
                      f"inflate + flate2 header rules (oracle/zref.c), {host_threads} threads, "
                      f"{el:.1f} s"}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
