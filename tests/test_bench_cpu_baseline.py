"""bench.py's worker-per-core CPU baseline (the reference's deployment,
DCVC-DC/test_video.py:276-290): a spawn pool of single-thread oracle
workers, run here on a tiny frame so the record's shape and arithmetic are
checked without the minutes a full-size frame takes.  No GPU is touched."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_baseline_workers_record():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--cpu-baseline-workers", "2",
                          "--height", "64", "--width", "96", "--gop", "4"],
                         capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["cores"] == 2 and rec["kind"] == "port" and rec["workload"] == ["dc", 64, 96, False]
    assert len(rec["ms_I"]) == 2 and len(rec["ms_P"]) == 2
    t_i = sum(rec["ms_I"]) / 2e3
    t_p = sum(rec["ms_P"]) / 2e3
    assert abs(rec["value"] - 2 * 4 / (t_i + 3 * t_p)) < 1e-3 * rec["value"]
