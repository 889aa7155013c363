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
