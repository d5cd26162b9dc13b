"""Host-side profile of the P-frame loop (cProfile + coder timers):
python scripts/profile_host.py [frames]  -> gpurun_out/host_profile.txt"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from dcvc_amd import hip as K  # noqa: E402
from dcvc_amd import entropy  # noqa: E402
from dcvc_amd.dc import DMC, IntraNoAR  # noqa: E402
from dcvc_amd.layers import Precision  # noqa: E402
from dcvc_amd.synth import moving_pattern  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda", 0)
isd, psd = bench.make_weights(None, 0, dev)
prec = Precision.fast(latent_compute=K.BF16)
inet = IntraNoAR(precision=prec, stream_part=8, device=dev).load_state_dict(isd)
pnet = DMC(precision=prec, stream_part=8, device=dev).load_state_dict(psd)
inet.update(force=True)
pnet.update(force=True)
h, w = 1080, 1920
frames = [torch.from_numpy(moving_pattern(h, w, t)).to(dev) for t in range(n + 3)]
x = K.empty(1088, 1920, 3, K.F32, dev)
timers = {"enc": 0.0, "dec": 0.0, "flush": 0.0}
for name, attr in (("enc", "encode"), ("dec", "decode"), ("flush", "flush")):
    orig = getattr(entropy.EntropyCoder, attr)

    def wrap(self, *a, _o=orig, _n=name, **k):
        t = time.perf_counter()
        r = _o(self, *a, **k)
        timers[_n] += time.perf_counter() - t
        return r
    setattr(entropy.EntropyCoder, attr, wrap)

K.frame_to_nhwc(frames[0], h, w, x)
r = inet.encode_decode(x, False, 0, "/dev/shm/p0.bin", pic_width=w, pic_height=h)
dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None, "ref_y": None, "ref_mv_y": None}
for i in range(1, 3):
    K.frame_to_nhwc(frames[i], h, w, x)
    dpb = pnet.encode_decode(x, dpb, False, 0, "/dev/shm/p.bin", pic_width=w, pic_height=h, frame_idx=i % 4)["dpb"]
torch.cuda.synchronize()
for k in timers:
    timers[k] = 0.0
pr = cProfile.Profile()
t0 = time.time()
encs, decs = [], []
pr.enable()
for i in range(3, 3 + n):
    K.frame_to_nhwc(frames[i], h, w, x)
    r = pnet.encode_decode(x, dpb, False, 0, "/dev/shm/p.bin", pic_width=w, pic_height=h, frame_idx=i % 4)
    dpb = r["dpb"]
    encs.append(r["encoding_time"])
    decs.append(r["decoding_time"])
torch.cuda.synchronize()
pr.disable()
el = time.time() - t0
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(35)
os.makedirs("gpurun_out", exist_ok=True)
with open("gpurun_out/host_profile.txt", "w") as f:
    f.write(f"frames {n} wall {el:.3f}s per frame {el / n * 1e3:.1f} ms\n")
    f.write(f"encoding_time avg {1e3 * sum(encs) / n:.1f} ms decoding_time avg {1e3 * sum(decs) / n:.1f} ms\n")
    f.write("coder host time per frame (ms): " + str({k: round(v / n * 1e3, 2) for k, v in timers.items()}) + "\n")
    f.write(s.getvalue())
print(open("gpurun_out/host_profile.txt").read()[:3000])
