"""bench.py --gpus N starts N ranks itself (one process per GPU under
torch.distributed.run on 127.0.0.1, before anything touches the GPU), so the
driver's `bench.py --gpus N` measures N GPUs.  Checked on the CPU through the
launcher self-test, whose ranks join a gloo group and report the world size."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


import pytest


@pytest.mark.parametrize("n", [2, 8])
def test_bench_gpus_n_launches_n_ranks(n):
    """--gpus N (2, and the driver's 8) starts N ranks that join, reduce and
    report; every rank takes a disjoint core share (rank_cpu_plan on two
    synthetic NUMA nodes) and sizes the shared rANS pool to it, so a rank runs
    at most lanes + stream_part coder threads (GOP lane threads + pool
    workers), however many coders its lanes create."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--launcher-selftest"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_joined"] == n and d["rank_sum"] == n * (n - 1) // 2 and d["requested"] == n
    # one shard record per rank, in rank order (the N > 1 bench line's "ranks")
    assert [r["rank"] for r in d["ranks"]] == list(range(n)), d["ranks"]
    for r in d["ranks"]:
        assert r["frames"] > 0 and r["elapsed_s"] > 0 and r["fps"] > 0 and r["precision_fallbacks"] == 0, r
    shares = [set(p["share"]) for p in d["plans"]]
    ncpu = len(os.sched_getaffinity(0))
    if ncpu >= n:
        for i in range(n):
            for j in range(i + 1, n):
                assert not shares[i] & shares[j], (i, j, d["plans"])
    for p in d["plans"]:
        assert p["set_rc"] == 0 and 1 <= p["coder_workers"] <= 8 - 1, p
        assert p["coders"] == 2 * 3
        # (lane threads are the bench's own; the selftest counts the pool)
        assert p["coder_workers"] <= max(1, len(p["share"]) - 3) or p["coder_workers"] == 1, p
