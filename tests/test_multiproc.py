"""The N>1 path of bench.py on CPU: two ranks over gloo (127.0.0.1) run the
harness's cross-rank aggregation (max time, summed work) and get disjoint
image shards.  The data path itself has no collective."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    bench.torch = torch
    B = 1024
    seeds = set(range(bench.shard_seed0(rank, B), bench.shard_seed0(rank, B) + B))
    elapsed = 1.0 + rank  # rank 1 is slower
    t, n = bench.aggregate(dist, elapsed, 100 * B * (rank + 1), "cpu")
    dist.barrier()
    q.put((rank, t, n, min(seeds), max(seeds)))
    dist.destroy_process_group()


def test_two_rank_aggregation_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, n, lo, hi in res:
        assert t == 2.0                       # max over ranks
        assert n == 100 * 1024 * 3            # summed work of both ranks
    assert res[0][4] < res[1][3]              # disjoint shards
