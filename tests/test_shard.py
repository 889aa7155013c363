"""The N>1 path of bench.py on the CPU: round-robin chunk partition and the
max-over-ranks timing collective, run as world_size-2 gloo process groups
(chunks are independent, no data-path collective)."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from zarr_amd.shard import aggregate_rate, max_over_ranks, round_robin_ids, split_round_robin


def test_round_robin_partition_is_disjoint_and_complete():
    world, n = 8, 1000
    ids = [round_robin_ids(r, world, n) for r in range(world)]
    flat = sorted(x for l in ids for x in l)
    assert flat == list(range(world * n))
    for r in range(world):
        assert all(g % world == r for g in ids[r])
    parts = [split_round_robin(65536, r, 8) for r in range(8)]
    assert sorted(x for p in parts for x in p) == list(range(65536))
    assert all(len(p) == 8192 for p in parts)
    with pytest.raises(ValueError):
        round_robin_ids(2, 2, 1)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ids = round_robin_ids(rank, world, 16)
        t = 0.5 + rank  # rank 1 is the slow one
        mx = max_over_ranks(t)
        rate = aggregate_rate(1 << 20, t)
        dist.barrier()
        q.put((rank, ids, mx, rate))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_max_over_ranks_and_aggregate():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1] == list(range(0, 32, 2)) and res[1][1] == list(range(1, 32, 2))
    for _, _, mx, rate in res:
        assert mx == 1.5                      # max over ranks
        assert rate == 2 * (1 << 20) / 1.5   # all ranks' bytes / slowest rank


def _bench_worker(rank, world, port, q):
    """bench.py's own N>1 code: chunk_ids (strong and weak) and timed_region
    (barrier + sync on both sides, max over ranks) on a gloo group."""
    import sys
    import time
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        strong = bench.chunk_ids(rank, world, 65536, True)
        weak = bench.chunk_ids(rank, world, 4096, False)
        calls = []
        synced = []
        wall, t_max = bench.timed_region(lambda: (calls.append(1), time.sleep(0.05 * (rank + 1))),
                                         3, world, lambda: synced.append(1))
        q.put((rank, strong[:4], len(strong), weak[:4], len(weak), len(calls), len(synced), wall, t_max))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bench_partition_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, ns0, w0, nw0, c0, y0, wall0, m0), (r1, s1, ns1, w1, nw1, c1, y1, wall1, m1) = res
    assert s0 == [0, 2, 4, 6] and s1 == [1, 3, 5, 7] and ns0 == ns1 == 32768  # C4 strong split
    assert w0 == [0, 2, 4, 6] and w1 == [1, 3, 5, 7] and nw0 == nw1 == 4096   # weak: 4096 per rank
    assert c0 == c1 == 3 and y0 == y1 == 2            # exactly K steps, sync on both sides
    assert m0 == m1 == max(wall0, wall1) and wall1 >= 0.15  # every rank reports the slowest rank's time
