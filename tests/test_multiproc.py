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


def test_bench_spawns_one_rank_per_gpu_stub():
    """`bench.py --gpus 2` without torchrun starts two rank processes itself
    (gloo harness, no GPU in --stub mode, a fixed wait per solve): n_gpus is
    the number of ranks that ran, C5's 8192 images are split 4096 + 4096, and
    value counts the image-iterations of both ranks."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub",
                          "--steps", "3", "--warmup", "1", "--no-cpu", "--config", "c5",
                          "--maxit", "10"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    assert r["config"]["images_per_gpu"] == 4096 and r["config"]["images_total"] == 8192
    # 2 ranks x 4096 images x 10 iterations per step; >= 10 ms wait per step
    assert r["value"] <= 2 * 4096 * 10 / 0.010 * 1.001
    assert r["value"] == pytest.approx(3 * 2 * 4096 * 10 / (r["ms_per_step"] * 3 / 1e3), rel=1e-9)


def test_shard_bounds_cover_the_job():
    import bench
    for world in (1, 2, 3, 8):
        parts = [bench.shard_bounds(8192, world, r) for r in range(world)]
        assert parts[0][0] == 0 and parts[-1][1] == 8192
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))


@pytest.mark.parametrize("fail_rank", [0, 1])
def test_bench_fails_fast_when_a_rank_dies(fail_rank):
    """One rank exits 1 before the gloo rendezvous: the launcher stops the
    other rank (which would otherwise wait in the rendezvous until its
    timeout) and returns non-zero within seconds."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--stub",
                          "--stub-fail-rank", str(fail_rank), "--steps", "3", "--warmup", "1",
                          "--no-cpu", "--config", "c3", "--maxit", "10"], capture_output=True,
                         text=True, timeout=120, env=env)
    el = time.time() - t0
    assert out.returncode != 0
    assert el < 30, el
    assert f"rank {fail_rank} exited with 1" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_kernel_bytes_model_c3():
    """bench.py's algorithmic byte model on C3's shape with the
    device's per-iteration counters of a 100-iteration solve: the per-kernel
    formulas, the setup's 140 B/px + 12 S + 3 TF per image, and the total the
    roofline divides by (1.65 TB with the setups, 1.636 TB without)."""
    import numpy as np
    import bench
    B, it, N = 1024, 100, 256 * 256
    cnt = np.zeros((B, 8))
    cnt[:, 2] = 1.407578125 * it          # line-search passes (BENCH_r05 counters)
    cnt[:, 6] = 1.698193359375 * it       # projection full passes
    cnt[:, 7] = 0.15436440110206603 * it * N  # list entries read
    b = bench.kernel_bytes(256, 256, 270, 136, cnt, np.full(B, it), beta=True, series=True,
                           compact=True, bmap=False, fused_at_col=True)
    S, TF = 16.0 * 256 * 136, 16.0 * 270 * 136
    assert b["k_setup"] == B * (140.0 * N + 12 * S + 3 * TF)
    assert b["k_col"] == B * it * (2 * S + TF)
    iters_bytes = sum(v for k, v in b.items() if k != "k_setup")
    assert abs(iters_bytes / 1.6356e12 - 1) < 2e-3   # the round-5 driver line's bytes
    assert abs(b["k_setup"] / iters_bytes - 0.011) < 0.002
