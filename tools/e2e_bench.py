#!/usr/bin/env python3
"""End-to-end (host-resident) decode rate, SURVEY §8(d) 'e2e'.

Compressed chunks start in pinned host memory and decoded chunks end in
pinned host memory: H2D of each sub-batch's streams, zcg_decode_batch, D2H
of its decoded elements, software-pipelined over several HIP streams so the
copy engines and the decode kernel overlap.  Prints one JSON line with the
e2e GiB/s next to the device-resident rate measured in the same process.

    python tools/e2e_bench.py [--codec gzip] [--chunks 1024] [--sub 128] [--streams 3]
    python tools/e2e_bench.py --encode ...   # write_chunk direction (C5)

--encode: elements start in pinned host memory; H2D, zcg_encode_batch, D2H
of the per-chunk lengths, then D2H of exactly each chunk's compressed bytes
into one packed pinned host buffer (the lengths of sub-batch b are waited for
while sub-batch b+1 is already enqueued).  Every stream is checked by the
oracle-independent reference library (zlib/lz4/bz2/lzma via Python) on a
sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (device memory, streams, pinned host buffers)

from bench import host_encode, workload  # noqa: E402
from zarr_amd.batch import BatchCodec  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="gzip", choices=["gzip", "lz4", "raw", "xz", "bzip2"])
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--sub", type=int, default=128)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--encode", action="store_true")
    args = ap.parse_args()
    if args.encode:
        return encode_e2e(args)
    dev = torch.device("cuda:0")
    meta, gen, _ = workload(args.codec)
    vals = [gen(i) for i in range(32)]
    streams = host_encode(args.codec, vals, 16)
    uniq = [v.tobytes() for v in vals]
    D = len(uniq[0])
    n, sub = args.chunks, args.sub
    assert n % sub == 0
    slot = max(len(s) for s in streams)
    slot = (slot + 255) // 256 * 256
    # pinned host: compressed slots (one per chunk) and decoded output
    h_src = torch.empty(n * slot, dtype=torch.uint8).pin_memory()
    h_dst = torch.empty(n * D, dtype=torch.uint8).pin_memory()
    hs = h_src.numpy()
    lens = np.zeros(n, np.uint64)
    for i in range(n):
        s = streams[i % len(streams)]
        hs[i * slot:i * slot + len(s)] = np.frombuffer(s, np.uint8)
        lens[i] = len(s)
    codec = BatchCodec(0)
    ns = args.streams
    strm = [torch.cuda.Stream(device=dev) for _ in range(ns)]
    # per-stream device buffers for one sub-batch
    d_src = [torch.empty(sub * slot, dtype=torch.uint8, device=dev) for _ in range(ns)]
    d_dst = [torch.empty(sub * D, dtype=torch.uint8, device=dev) for _ in range(ns)]
    d_stat = [torch.empty(sub, dtype=torch.int32, device=dev) for _ in range(ns)]
    descs = []
    for k in range(ns):
        d = np.zeros((sub, 4), np.uint64)
        for j in range(sub):
            d[j] = (d_src[k].data_ptr() + j * slot, 0, d_dst[k].data_ptr() + j * D, D)
        descs.append(d)
    d_desc = [[None] * (n // sub) for _ in range(ns)]
    for b in range(n // sub):
        k = b % ns
        d = descs[k].copy()
        d[:, 1] = lens[b * sub:(b + 1) * sub]
        d_desc[k][b] = torch.from_numpy(d.view(np.int64)).to(dev)
    stat_host = torch.empty(n, dtype=torch.int32).pin_memory()

    class _P:  # PackedStreams-shaped view for BatchCodec.decode
        pass

    def run():
        for b in range(n // sub):
            k = b % ns
            s = strm[k]
            with torch.cuda.stream(s):
                d_src[k].copy_(h_src[b * sub * slot:(b + 1) * sub * slot], non_blocking=True)
                p = _P()
                p.desc, p.n, p.status = d_desc[k][b], sub, d_stat[k]
                codec.decode(meta, p, stream=s)
                h_dst[b * sub * D:(b + 1) * sub * D].copy_(d_dst[k], non_blocking=True)
                stat_host[b * sub:(b + 1) * sub].copy_(d_stat[k], non_blocking=True)
        torch.cuda.synchronize()

    run()  # warm-up + parity of the pipeline
    assert (stat_host.numpy() == 0).all()
    hd = h_dst.numpy()
    for i in range(0, n, max(1, n // 16)):
        assert hd[i * D:(i + 1) * D].tobytes() == uniq[i % len(uniq)], i
    best = 1e9
    for _ in range(args.reps):
        t0 = time.perf_counter()
        run()
        best = min(best, time.perf_counter() - t0)
    # device-resident reference point: one sub-batch stream's decode alone, repeated
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = strm[0]
    p = _P()
    p.desc, p.n, p.status = d_desc[0][0], sub, d_stat[0]
    with torch.cuda.stream(s):
        codec.decode(meta, p, stream=s)
        ev0.record(s)
        for _ in range(4):
            codec.decode(meta, p, stream=s)
        ev1.record(s)
    torch.cuda.synchronize()
    dev_s = ev0.elapsed_time(ev1) / 4 * 1e-3
    out = {
        "what": f"e2e {args.codec} decode, pinned host -> H2D -> decode -> D2H -> pinned host",
        "chunks": n, "sub_batch": sub, "streams": ns, "chunk_bytes": D,
        "compressed_bytes": int(lens.sum()),
        "e2e_GiBps": round(n * D / best / GIB, 3),
        "e2e_ms": round(best * 1e3, 2),
        "device_only_GiBps_sub_batch": round(sub * D / dev_s / GIB, 3),
        "h2d_plus_d2h_bytes": int(lens.sum()) + n * D,
    }
    print(json.dumps(out))


def encode_e2e(args):
    from zarr_amd.batch import make_encode_batch  # noqa: F401  (descriptor layout)
    dev = torch.device("cuda:0")
    meta, gen, _ = workload(args.codec)
    vals = [gen(i) for i in range(32)]
    D = vals[0].nbytes
    n, sub, ns = args.chunks, args.sub, args.streams
    assert n % sub == 0
    codec = BatchCodec(0)
    cap = codec.encode_bound(meta, D)
    h_src = torch.empty(n * D, dtype=torch.uint8).pin_memory()
    hs = h_src.numpy()
    for i in range(n):
        hs[i * D:(i + 1) * D] = vals[i % len(vals)].view(np.uint8)
    h_out = torch.empty(n * cap, dtype=torch.uint8).pin_memory()  # packed results (worst case)
    h_len = torch.empty(n, dtype=torch.int64).pin_memory()
    h_st = torch.empty(n, dtype=torch.int32).pin_memory()
    strm = [torch.cuda.Stream(device=dev) for _ in range(ns)]
    d_src = [torch.empty(sub * D, dtype=torch.uint8, device=dev) for _ in range(ns)]
    d_dst = [torch.empty(sub * cap, dtype=torch.uint8, device=dev) for _ in range(ns)]
    d_len = [torch.zeros(sub, dtype=torch.int64, device=dev) for _ in range(ns)]
    d_st = [torch.zeros(sub, dtype=torch.int32, device=dev) for _ in range(ns)]
    d_desc = []
    for k in range(ns):
        d = np.zeros((sub, 4), np.uint64)
        for j in range(sub):
            d[j] = (d_src[k].data_ptr() + j * D, D, d_dst[k].data_ptr() + j * cap, cap)
        d_desc.append(torch.from_numpy(d.view(np.int64)).to(dev))
    offs = np.zeros(n + 1, np.int64)

    def run():
        evs = []
        pos = 0

        def drain(b, ev):
            nonlocal pos
            ev.synchronize()
            k = b % ns
            with torch.cuda.stream(strm[k]):
                for j in range(sub):
                    i = b * sub + j
                    ln = int(h_len[i])
                    offs[i] = pos
                    h_out[pos:pos + ln].copy_(d_dst[k][j * cap:j * cap + ln], non_blocking=True)
                    pos += ln
            offs[n] = pos

        for b in range(n // sub):
            k = b % ns
            s = strm[k]
            if b >= ns:  # the stream's buffers are reused: drain its previous sub-batch first
                drain(*evs[b - ns])
            with torch.cuda.stream(s):
                d_src[k].copy_(h_src[b * sub * D:(b + 1) * sub * D], non_blocking=True)
                codec.encode(meta, d_desc[k], sub, d_len[k], d_st[k], stream=s)
                h_len[b * sub:(b + 1) * sub].copy_(d_len[k], non_blocking=True)
                h_st[b * sub:(b + 1) * sub].copy_(d_st[k], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s)
            evs.append((b, ev))
        for b in range(max(0, n // sub - ns), n // sub):
            drain(*evs[b])
        torch.cuda.synchronize()
        return pos

    total = run()
    assert (h_st.numpy() == 0).all()
    import bz2
    import lzma
    import zlib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import zref  # oracle: checker only
    cid = {"gzip": zref.GZIP, "lz4": zref.LZ4, "raw": zref.RAW, "xz": zref.XZ, "bzip2": zref.BZIP2}[args.codec]
    ho = h_out.numpy()
    for i in range(0, n, max(1, n // 8)):
        stream = ho[offs[i]:offs[i] + int(h_len[i])].tobytes()
        st, dec = zref.decode(cid, stream, D, 1, False, False)
        assert st == zref.OK and dec == vals[i % len(vals)].tobytes(), i
    best = 1e9
    for _ in range(args.reps):
        t0 = time.perf_counter()
        run()
        best = min(best, time.perf_counter() - t0)
    print(json.dumps({
        "what": f"e2e {args.codec} encode (write_chunk), pinned host -> H2D -> encode -> D2H lengths + "
                "exact compressed bytes -> packed pinned host",
        "chunks": n, "sub_batch": sub, "streams": ns, "chunk_bytes": D, "compressed_bytes": int(total),
        "ratio": round(n * D / total, 3), "e2e_GiBps_input": round(n * D / best / GIB, 3),
        "e2e_ms": round(best * 1e3, 2)}))


if __name__ == "__main__":
    main()
