"""Two codecs on one GPU at once: two processes (the reference's several
workers per GPU, DCVC-DC/test_video.py:289-290), each coding its own 1080p
sequence and checking, frame by frame, that its decoder reproduces every
value its encoder computed (scripts/corun_debug.py: per-call bit checksums of
the priors, motion compensation and every quadtree step).  Before the kernels
were built without packed-f32 instructions (scripts/check_isa.sh), this failed
within a few frames; a single codec never did."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("precision", ["split", "fast"])
def test_two_codec_processes_share_the_gpu(precision):
    """split: the bench precision (its kernels co-run at the default 3 GOP
    lanes); fast: the bf16 kernels the failure was first seen with."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(REPO, "scripts", "corun_debug.py"), "--frames", "12",
           "--precision", precision]
    env = dict(os.environ)
    procs = [subprocess.Popen(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for _ in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out))
    for rc, out in outs:
        tail = "\n".join(out.splitlines()[-15:])
        assert rc == 0, tail
        assert "encoder and decoder agree" in out, tail
