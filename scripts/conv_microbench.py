"""Time individual conv / fused-block shapes of the DC P-frame on the GPU.

    python scripts/conv_microbench.py [--reps 20] [--libs libdcvc_hip.so,libX.so]

Each shape runs `reps` times between two HIP events on the launch stream;
prints us/launch, TFLOP/s (algorithmic 2*MAC) and GB/s (input + weights +
output once).  --libs times the same shapes against alternative builds in
dcvc_amd/lib (one subprocess per library).
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (k, stride, cin, cout, H, W) at the DC 1080p P-frame (input resolution)
SHAPES = [
    (3, 1, 48, 48, 1088, 1920),
    (3, 1, 96, 48, 1088, 1920),
    (3, 1, 128, 64, 544, 960),
    (3, 1, 64, 64, 544, 960),
    (3, 1, 96, 96, 272, 480),
    (3, 1, 128, 192, 544, 960),
    (3, 1, 128, 128, 68, 120),
    (3, 2, 48, 64, 1088, 1920),
    (7, 1, 32, 64, 1088, 1920),
    (7, 1, 64, 32, 1088, 1920),
    (7, 1, 8, 32, 1088, 1920),
    (7, 1, 32, 16, 1088, 1920),
    (1, 1, 384, 384, 68, 120),
    (1, 1, 48, 48, 1088, 1920),
    (1, 1, 64, 64, 1088, 1920),
    (1, 1, 64, 32, 1088, 1920),
    (3, 1, 480, 384, 68, 120),
    (3, 1, 384, 288, 68, 120),
    (3, 1, 288, 288, 68, 120),
    (3, 1, 192, 192, 68, 120),
]


def run(reps, shapes, fixed=False, options=""):
    import torch
    from dcvc_amd import hip as K
    for kv in filter(None, options.split(",")):
        k, v = kv.split("=")
        K.set_option(k, int(v))
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    out = []
    for k, s, cin, cout, H, W in shapes:
        w = torch.randn(cout, cin, k, k) / (cin * k * k) ** 0.5
        cw = K.ConvW(w, torch.randn(cout) * 0.1, stride=s, compute=K.BF16, device=dev)
        x = K.from_nchw(torch.randn(1, cin, H, W, device=dev), K.BF16)
        y = K.conv(cw, x)
        st = torch.cuda.current_stream()
        for _ in range(3):
            K.conv(cw, x, y)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        # size the run to >= ~50 ms so the clock has ramped
        e0.record(st)
        K.conv(cw, x, y)
        e1.record(st)
        torch.cuda.synchronize()
        if not fixed:
            reps = max(reps, int(0.05 / max(e0.elapsed_time(e1) * 1e-3, 1e-6)))
        e0.record(st)
        for _ in range(reps):
            K.conv(cw, x, y)
        e1.record(st)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps * 1e-3
        Ho, Wo = cw.out_hw(H, W)
        fl = 2 * Ho * Wo * cout * cin * k * k
        nb = 2 * (H * W * cin + Ho * Wo * cout) + cw.w.numel() * 2
        out.append({"shape": f"k{k}s{s} {cin}->{cout} {H}x{W}", "us": round(t * 1e6, 1),
                    "tflops": round(fl / t / 1e12, 1), "gbs": round(nb / t / 1e9, 1)})
    # streaming copy of a 1088x1920x48 bf16 image (HBM reference point)
    a = torch.randn(1088 * 1920 * 48, device=dev).to(torch.bfloat16)
    b = torch.empty_like(a)
    for _ in range(5):
        b.copy_(a)
    e0.record(st)
    for _ in range(50):
        b.copy_(a)
    e1.record(st)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 50 * 1e-3
    out.append({"shape": "torch copy 200MB", "us": round(t * 1e6, 1), "tflops": 0.0,
                "gbs": round(2 * a.numel() * 2 / t / 1e9, 1)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--libs", default="")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--option", default="", help="NAME=V,... dcvc_set_option switches")
    ap.add_argument("--only", type=int, default=-1, help="run only SHAPES[i] (profiling)")
    ap.add_argument("--fixed", action="store_true", help="exactly --reps launches (profiling)")
    a = ap.parse_args()
    if a.child or not a.libs:
        shapes = SHAPES if a.only < 0 else [SHAPES[a.only]]
        print(json.dumps(run(a.reps, shapes, a.fixed, a.option)), flush=True)
        return
    res = {}
    # --libs entries: LIB or LIB:NAME=V+NAME=V (option switches for that run)
    for spec in a.libs.split(","):
        lib, _, opts = spec.partition(":")
        env = dict(os.environ, DCVC_HIP_LIB=lib)
        r = subprocess.run([sys.executable, __file__, "--child", "--reps", str(a.reps),
                            "--option", opts.replace("+", ",")], env=env,
                           capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            print(spec, "failed rc", r.returncode, r.stderr[-2000:])
            return r.returncode
        res[spec] = json.loads(r.stdout.strip().splitlines()[-1])
    libs = list(res)
    print("%-32s" % "shape" + "".join("%26s" % l[:24] for l in libs))
    for i, row in enumerate(res[libs[0]]):
        print("%-32s" % row["shape"] + "".join(
            "%10.1fus %5.0fTF %5.0fGB" % (res[l][i]["us"], res[l][i]["tflops"], res[l][i]["gbs"])
            for l in libs))


if __name__ == "__main__":
    sys.exit(main() or 0)
