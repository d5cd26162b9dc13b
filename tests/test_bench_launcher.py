"""bench.py --gpus N starts N ranks itself (one process per GPU under
torch.distributed.run on 127.0.0.1, before anything touches the GPU), so the
driver's `bench.py --gpus N` measures N GPUs.  Checked on the CPU through the
launcher self-test, whose ranks join a gloo group and report the world size."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_launches_two_ranks():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launcher-selftest"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks_joined"] == 2 and d["rank_sum"] == 1 and d["requested"] == 2
