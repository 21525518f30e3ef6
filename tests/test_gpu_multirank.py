"""The real multi-rank bench path on a GPU.

`bench.py --gpus 2` without torchrun starts two rank processes itself; here
both ranks run on device 0 (BSGP_RANK_DEVICE, applied before any GPU call of
a rank), so the one-GPU box rehearses exactly what the driver's 8-GPU node
runs: per-rank shards solved through the C ABI, gloo for the harness's two
scalars, max wall over ranks, summed image-iterations.  The parent process
never touches the GPU (launch_ranks spawns, it does not exec)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ, BSGP_RANK_DEVICE="0", BSGP_DIST_TIMEOUT_S="120")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args],
                         capture_output=True, text=True, timeout=timeout, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # rank 0 prints, rank 1 does not
    return json.loads(lines[0])


@pytest.mark.gpu
def test_bench_two_ranks_weak_c3_on_one_gpu():
    """C3 at 64 images per rank, MAXIT 5 (stop rule 1: every image runs 5
    iterations), one workgroup per image as C3 runs (the persistent solver;
    two ranks' spinning teams on one device are not what a node runs): n_gpus
    2, images_total = 2 x per-rank, the summed image-iterations of both
    ranks' real solves, value = that / max wall."""
    B, M = 64, 5
    r = _run(["--gpus", "2", "--steps", "2", "--warmup", "1", "--maxit", str(M), "--batch", str(B),
              "--team", "1", "--no-cpu", "--no-e2e", "--no-profile"])
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    c = r["config"]
    assert c["images_per_gpu"] == B and c["images_total"] == 2 * B
    assert c["iterations_per_step"] == 2 * B * M          # both ranks solved, gloo summed
    assert "stub" not in r["data"] and c["team"] == 1     # device counters were read
    assert r["value"] == pytest.approx(2 * 2 * B * M / (r["ms_per_step"] * 2 / 1e3), rel=1e-9)


@pytest.mark.gpu
def test_bench_two_ranks_strong_c5_split_on_one_gpu():
    """C5 (8192 images in total) split 4096 + 4096 over two ranks on one
    device, MAXIT 2: the strong-scaling shard bounds with real solves."""
    r = _run(["--gpus", "2", "--config", "c5", "--steps", "1", "--warmup", "1", "--maxit", "2",
              "--no-cpu", "--no-e2e", "--no-profile"])
    assert r["n_gpus"] == 2 and r["scaling"] == "strong"
    c = r["config"]
    assert c["images_per_gpu"] == 4096 and c["images_total"] == 8192
    assert c["iterations_per_step"] == 8192 * 2
