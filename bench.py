"""DCVC-DC encode+decode throughput on MI355X (BASELINE.json metric, config C3:
DCVC-DC RGB 1920x1080, padded to 1088, IP=32, write mode = real bitstreams).
``--model hem`` runs config C2 instead (DCVC-HEM 1920x1080, zero-padded to
1088, IP=32, the loop of DCVC-HEM/test_video.py:108-160).

One step = one frame through ``encode_decode(..., output_path=...)``: the
I-frame codec when frame_idx % gop == 0, else the P-frame codec, exactly the
loop of DCVC-DC/test_video.py:108-167.  Frames are synthetic (moving sinusoid
pattern + noise, uint8, resident in HBM before timing); weights are seeded
random in the reference's architecture (no checkpoints offline).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Multi-GPU: one process per GPU (torchrun), each rank codes its own sequence
(seed 1 + rank; the reference shards (sequence, rate) jobs the same way,
test_video.py:396-436), weights are created on rank 0 and broadcast once over
RCCL; no collective touches the per-frame path.  value = frames of all ranks
/ max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 / f16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
# split-fp16 convs (sconv.hip) issue 3 f16 MFMAs per fp32 product: their
# algorithmic (fp32) flops are priced against a third of the f16 peak
PEAK_F16X3_TFLOPS = PEAK_BF16_TFLOPS / 3
PEAK_HBM_GBS = 8000.0
# precisions held to the strict parity bar (tests/parity.py) carry the metric
# with its qualifier; the bf16 modes are labelled as not held to it
STRICT_PRECISIONS = ("split", "parity")


# the strict teacher-forced GPU test that holds each workload's arithmetic to
# the bar at full size (tests/test_gpu_parity_strict.py), by (model, yuv420)
STRICT_TESTS = {("dc", False): ("tests/test_gpu_parity_strict.py::test_strict_parity_c3_1080p",
                                 "I + P frames at 1920x1080"),
                ("hem", False): ("tests/test_gpu_parity_strict.py::test_strict_parity_hem_c2_1080p",
                                 "I + P frames at 1920x1080"),
                ("dc", True): ("tests/test_gpu_parity_strict.py::test_strict_parity_c4_yuv420",
                               "I + P frames at 3840x2160 and at 1920x1080")}


def parity_evidence(args, parity):
    """What backs the line's parity qualifier: its own parity_check (when it
    ran), else the strict GPU test of this workload in this precision, else
    nothing ('unpinned')."""
    if args.precision not in STRICT_PRECISIONS:
        return "none: precision not held to the strict bar"
    if parity is not None:
        return "parity_check passed" if parity.get("passed") else "parity_check FAILED"
    t = STRICT_TESTS.get((args.model, bool(args.yuv420)))
    return (f"strict GPU test {t[0]} ({args.precision} precision; {t[1]}), not this run's frames" if t
            else "unpinned")


def metric_name(args, parity=None):
    """BASELINE.json's metric, its "bpp bit-exact" qualifier only when the
    line's evidence backs it (parity_evidence)."""
    res = f"{args.width}x{args.height}"
    base = f"encode+decode fps @{res} per GPU"
    if args.precision not in STRICT_PRECISIONS:
        return f"{base}; {args.precision} precision, NOT held to the bit-exact bar (see parity_check)"
    ev = parity_evidence(args, parity)
    if ev == "parity_check FAILED":
        return f"{base}; parity check FAILED against the oracle (see parity_check)"
    if ev == "unpinned":
        return f"{base}; parity unpinned"
    if parity is None:
        # no check of this run's frames: say which test holds the arithmetic
        t = STRICT_TESTS[(args.model, bool(args.yuv420))]
        return f"{base}; bpp bit-exact + PSNR \u0394<1e-4 dB vs ref (strict GPU test, {t[1]}; not this run's frames)"
    return f"{base}; bpp bit-exact + PSNR \u0394<1e-4 dB vs ref"


def peak_of(family, key):
    """MFMA peak of one launch's compute type: f16x3 (split) convs, fp32
    (f32 MFMA) convs and GEMMs, everything else bf16."""
    if family in ("sconv_kernel", "xconv3_kernel") or " f16x3" in key:
        return PEAK_F16X3_TFLOPS
    if family.startswith("gemm1x1f") or " f32 " in key:
        return PEAK_F32_TFLOPS
    return PEAK_BF16_TFLOPS


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", choices=["dc", "hem"], default="dc",
                    help="dc = DCVC-DC (config C3, the 30 fps target); hem = DCVC-HEM (config C2)")
    ap.add_argument("--rate", type=int, default=0,
                    help="HEM rate point: index into the checkpoint's q_scale ladders (test_video.py:274-300)")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--height", type=int, default=None, help="default 1080 (2160 with --yuv420)")
    ap.add_argument("--width", type=int, default=None, help="default 1920 (3840 with --yuv420)")
    ap.add_argument("--yuv420", action="store_true",
                    help="config C4: DCVC-DC YUV420 source coded as YCbCr 4:4:4 (dist_in_yuv420), 3840x2160")
    ap.add_argument("--gop", type=int, default=32)
    ap.add_argument("--q_index", type=int, default=0)
    ap.add_argument("--precision", choices=["split", "parity", "fast", "fast-bf16-tail"], default="split",
                    help="split = fp32 storage, every conv on split-fp16 MFMA (held to the strict parity bar, the "
                         "default); parity = fp32 MFMA end to end; fast = bf16 feature convs + fp32 entropy tail "
                         "and fast-bf16-tail = bf16 throughout (labelled lines, not held to the bar)")
    ap.add_argument("--no-parity-check", action="store_true",
                    help="skip the teacher-forced I + P parity check against the oracle (rank 0, N = 1)")
    ap.add_argument("--stream_part", type=int, default=8,
                    help="rANS stream parts (the reference's --stream_part_i/p); parts code in parallel threads")
    ap.add_argument("--lanes", type=int, default=3,
                    help="GOP lanes per GPU: independent GOPs coded concurrently by host threads on their own HIP "
                         "streams (the reference's several workers per GPU, test_video.py:289-290), so one lane's "
                         "host rANS work overlaps another's kernels")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the cpu_baseline oracle run (capped at the cores this process may use)")
    ap.add_argument("--cpu-baseline-workers", type=int, default=0,
                    help="only measure the oracle in the reference's worker-per-core mode with this many "
                         "single-thread workers (no GPU); prints the record profiles/cpu_baseline_workers.json holds")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--launcher-selftest", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--profile-out", default="", help="per-shape kernel timing JSON of one P-frame")
    a = ap.parse_args()
    if a.yuv420 and a.model != "dc":
        ap.error("--yuv420 is the DCVC-DC YUV path (config C4)")
    if a.cpu_baseline_workers and a.model != "dc":
        ap.error("--cpu-baseline-workers measures the DCVC-DC oracle")
    if a.height is None:
        a.height = 2160 if a.yuv420 else 1080
    if a.width is None:
        a.width = 3840 if a.yuv420 else 1920
    return a


HEM_GAIN = 1.6   # tests/golden/make_golden_hem.py: latents beyond 0/+-1 without blow-up


def spec(model="dc"):
    with open(os.path.join(HERE, "dcvc_amd", "data", f"{model}_param_spec.json")) as f:
        d = json.load(f)
    return [(n, tuple(s)) for n, s in d["intra"]], [(n, tuple(s)) for n, s in d["inter"]]


def make_weights(dist, rank, device, model="dc"):
    """Rank 0 builds the state dicts; one RCCL broadcast of the flat blob."""
    from dcvc_amd.weights import synthetic_state_dict
    i_spec, p_spec = spec(model)
    names = [("i", n, s) for n, s in i_spec] + [("p", n, s) for n, s in p_spec]
    total = sum(int(np.prod(s)) for _, _, s in names)
    if rank == 0:
        if model == "hem":
            isd = synthetic_state_dict(i_spec, seed=0, gain=HEM_GAIN)
            psd = synthetic_state_dict(p_spec, seed=1, gain=HEM_GAIN)
        else:
            isd, psd = synthetic_state_dict(i_spec, seed=0), synthetic_state_dict(p_spec, seed=1)
        flat = torch.cat([(isd if k == "i" else psd)[n].reshape(-1) for k, n, _ in names]).to(device)
    else:
        flat = torch.empty(total, dtype=torch.float32, device=device)
    if dist is not None:
        dist.broadcast(flat, 0)
    flat = flat.cpu()
    isd, psd, o = {}, {}, 0
    for k, n, s in names:
        m = int(np.prod(s))
        (isd if k == "i" else psd)[n] = flat[o:o + m].reshape(s)
        o += m
    return isd, psd


def max_over_ranks(dist, elapsed, device):
    """The job's wall time: the slowest rank's (contract: MAX over ranks)."""
    if dist is None:
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def rank_records(dist, rank, world, frames, own, fallbacks=0):
    """Every rank's own shard: frames coded, its own timed wall time (before
    the closing barrier) and rate, so a multi-GPU line shows each shard and the
    slowest rank's distance from the mean (rank order)."""
    rec = {"rank": rank, "frames": frames, "elapsed_s": round(own, 4), "fps": round(frames / own, 4),
           "precision_fallbacks": fallbacks}
    if dist is None or world == 1:
        return [rec]
    allr = [None] * world
    dist.all_gather_object(allr, rec)
    return sorted(allr, key=lambda r: r["rank"])


def shard_seed(rank):
    """Sequence of rank r: its own synthetic sequence (weak scaling)."""
    return 1 + rank


def host_info():
    """nproc, the cores this process may run on, the physical cores of the
    node (distinct (physical id, core id) pairs) and the CPU model."""
    model = "unknown"
    cores, phys, core = set(), None, None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name") and model == "unknown":
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                elif not line.strip():
                    if core is not None:
                        cores.add((phys, core))
                    phys, core = None, None
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return {"nproc": os.cpu_count() or 1, "usable": usable, "physical_cores": len(cores) or None, "cpu": model}


def oracle_ip_times(isd, psd, args, threads, capture=None):
    """(t_I, t_P) seconds of the oracle (PyTorch fp32 CPU restatement, pinned
    to the reference) on one full-size I-frame and one full-size P-frame
    (1088x1920 for C3), each compress + rANS encode + rANS decode +
    decompress in write mode, on `threads` torch threads.  capture (a dict)
    receives what the parity check needs: per frame the padded input, the
    coder calls, the rounding taps, the stream bits and the reconstruction."""
    from oracle import dc_oracle as O
    from oracle import rans_oracle as R
    from dcvc_amd.synth import moving_pattern, moving_pattern_yuv420, to_float
    torch.set_num_threads(threads)
    h, w = args.height, args.width
    Hp, Wp = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    inet = O.IntraOracle(isd, R.pmf_to_quantized_cdf)
    pnet = O.DMCOracle(psd, R.pmf_to_quantized_cdf)
    tabs = {"i_y": (inet.y_cdf, inet.y_sizes, inet.y_offsets), "i_z": inet.z_tab,
            "p_y": (pnet.y_cdf, pnet.y_sizes, pnet.y_offsets), "p_z": pnet.z_tab, "p_mvz": pnet.mvz_tab}

    nbytes = []

    def code(calls, pre):
        cc = [(s.clamp(-30000, 30000).to(torch.int16).numpy(), i.to(torch.int16).numpy(), tabs[pre + k])
              for k, s, i in calls]
        enc = R.DCStream(args.stream_part)   # the product's part count, so the stream bytes compare
        st = enc.encode(cc)
        nbytes.append(len(st))
        dec = enc.decode(st)
        pos = [0]

        def decoder(kind, idx):
            n = idx.numel()
            v = dec[pos[0]:pos[0] + n]
            pos[0] += n
            return v
        return decoder

    def frame(t):
        if args.yuv420:
            from oracle.harness_oracle import yuv_u8_to_input
            y, uv = moving_pattern_yuv420(h, w, t, seed=1)
            return torch.from_numpy(yuv_u8_to_input(y, uv, Hp, Wp)).permute(2, 0, 1).unsqueeze(0).contiguous()
        x = torch.from_numpy(to_float(moving_pattern(h, w, t, seed=1))).unsqueeze(0)
        return torch.nn.functional.pad(x, (0, Wp - w, 0, Hp - h), mode="replicate")

    frames = [frame(t) for t in range(2)]
    taps = [{}, {}] if capture is not None else [None, None]
    with torch.no_grad():
        t0 = time.time()
        calls_i = inet.compress(frames[0], False, args.q_index, tap=taps[0])
        xh = inet.decompress(code(calls_i, "i_"), h, w, False, args.q_index)
        t_i = time.time() - t0
        dpb = {"ref_frame": xh, "ref_feature": None, "ref_mv_feature": None, "ref_y": None, "ref_mv_y": None}
        t0 = time.time()
        calls_p = pnet.compress(frames[1], dpb, False, args.q_index, 1, tap=taps[1])
        dpb_p = pnet.decompress(dpb, code(calls_p, "p_"), h, w, False, args.q_index, 1)
        t_p = time.time() - t0
    if capture is not None:
        capture.update(onets=(inet, pnet), tabs=tabs,
                       frames=frames, calls=[calls_i, calls_p], taps=taps,
                       bits=[(nbytes[0] + 13) * 8, (nbytes[1] + 6) * 8], dpb_i=dpb,
                       recon=[xh, dpb_p["ref_frame"] if isinstance(dpb_p, dict) else dpb_p], h=h, w=w)
    return t_i, t_p


def cpu_baseline(isd, psd, args, capture=None):
    """The oracle timed on this host in one process on `threads` cores: one
    full-size I-frame and one full-size P-frame; fps = the GOP average
    gop / (t_I + (gop - 1) t_P).  No area scaling.  The reference's own
    worker-per-core mode is measured separately (``--cpu-baseline-workers``)
    and attached as ``workers`` when its committed record exists."""
    info = host_info()
    threads = max(1, min(args.cpu_threads, info["usable"]))
    h, w = args.height, args.width
    Hp, Wp = (h + 15) // 16 * 16, (w + 15) // 16 * 16
    t_i, t_p = oracle_ip_times(isd, psd, args, threads, capture)
    gop = args.gop
    fps = gop / (t_i + (gop - 1) * t_p)
    return {"value": fps, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle write-mode encode+decode of one full-size I-frame ({t_i:.1f} s) and one full-size "
                      f"P-frame ({t_p:.1f} s) at {Hp}x{Wp}, {threads} torch threads in one process; fps = GOP "
                      f"{gop} average; host nproc {info['nproc']}, usable {info['usable']}, CPU {info['cpu']}",
            "ms_I": round(t_i * 1e3, 1), "ms_P": round(t_p * 1e3, 1),
            **({"workers": _workers_record(args)} if _workers_record(args) else {})}


WORKERS_RECORD = os.path.join(HERE, "profiles", "cpu_baseline_workers.json")


def _workers_record(args):
    """The committed worker-per-core measurement of this workload, if any."""
    try:
        with open(WORKERS_RECORD) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    if rec.get("workload") != [args.model, args.height, args.width, bool(args.yuv420)]:
        return None
    # the record's rate per worker core and, for scale, that rate times this
    # node's physical cores (linear scaling assumed: an upper bound, the
    # workers share memory bandwidth)
    rec["source"] = "profiles/cpu_baseline_workers.json (committed record, not re-measured in this run)"
    rec["per_core_fps"] = rec["value"] / rec["cores"]
    pc = host_info()["physical_cores"]
    if pc:
        rec["node_physical_cores"] = pc
        rec["node_total_fps_est"] = rec["per_core_fps"] * pc
    return rec


def _worker(job):
    isd, psd, args = job
    return oracle_ip_times(isd, psd, args, 1)


def cpu_baseline_workers(args):
    """The reference's own CPU deployment, DCVC-DC/test_video.py:276-290: a
    pool of `workers` processes with torch.set_num_threads(1) each, every
    worker coding its own sequence; here each worker codes one full-size
    I-frame and one full-size P-frame.  fps = workers x gop / (t_I + (gop - 1)
    t_P) with each worker's own times (mean), i.e. all workers' frames over
    the wall time of a GOP.  Runs without touching the GPU (a separate
    invocation: ``python bench.py --cpu-baseline-workers N``)."""
    import multiprocessing as mp
    info = host_info()
    n = args.cpu_baseline_workers
    isd, psd = make_weights(None, 0, torch.device("cpu"), args.model)
    t0 = time.time()
    with mp.get_context("spawn").Pool(n) as pool:
        times = pool.map(_worker, [(isd, psd, args)] * n)
    wall = time.time() - t0
    t_i = float(np.mean([t[0] for t in times]))
    t_p = float(np.mean([t[1] for t in times]))
    fps = n * args.gop / (t_i + (args.gop - 1) * t_p)
    rec = {"value": fps, "unit": "frames/s", "cores": n, "kind": "port",
           "workload": [args.model, args.height, args.width, bool(args.yuv420)],
           "sample": f"{n} worker processes x 1 torch thread (DCVC-DC/test_video.py:276-290), each coding one "
                     f"full-size I-frame (mean {t_i:.1f} s) and one full-size P-frame (mean {t_p:.1f} s) in write "
                     f"mode; fps = workers x GOP {args.gop} / (t_I + {args.gop - 1} t_P); wall {wall:.0f} s; host "
                     f"nproc {info['nproc']}, usable {info['usable']}, CPU {info['cpu']}",
           "ms_I": [round(t[0] * 1e3, 1) for t in times], "ms_P": [round(t[1] * 1e3, 1) for t in times]}
    print(json.dumps(rec), flush=True)


def parity_check(cap, inet, pnet, args):
    """The bench precision's own parity on the cpu_baseline frames: the
    product codes the oracle's I-frame input and then the P-frame from the
    ORACLE's decoded picture buffer (teacher forcing, as the strict tests do),
    and every coder call is compared with the oracle's under tests/parity.py's
    bar.  Reports differing symbols / indexes, bits and PSNR deltas; a frame
    with a flipped symbol is coded again by the oracle with the product's
    symbols replayed at its ties (tests/parity.py's replay), and every element
    of that replay is checked too."""
    import tempfile
    from oracle import dc_oracle as O
    from oracle import rans_oracle as R
    from tests.parity import (IDX_TIE_EPS, PSNR_DB, REC_MAXABS, SYM_TIE_EPS, TIE_EPS, compare_forced, compare_frame,
                              idx_allowed, rec_maxabs)

    def psnr(a, x):
        mse = torch.mean((a.float().cpu()[..., :cap["h"], :cap["w"]].clamp(0, 1) - x[..., :cap["h"], :cap["w"]]) ** 2)
        return float(-10 * torch.log10(mse))
    out = []
    with tempfile.TemporaryDirectory() as td:
        for t in range(2):
            xp = cap["frames"][t]
            net = inet if t == 0 else pnet
            net.entropy_coder.trace = []
            path = os.path.join(td, f"{t}.bin")
            if t == 0:
                r = inet.encode_decode(xp.cuda(), False, args.q_index, path, pic_width=cap["w"], pic_height=cap["h"])
                rec = r["x_hat"]
            else:
                dpb = {k: (v.cuda() if v is not None else None) for k, v in cap["dpb_i"].items()}
                r = pnet.encode_decode(xp.cuda(), dpb, False, args.q_index, path, pic_width=cap["w"],
                                       pic_height=cap["h"], frame_idx=1)
                rec = r["dpb"]["ref_frame"]
            torch.cuda.synchronize()
            tr = net.entropy_coder.trace
            net.entropy_coder.trace = None
            enc = [(sy, ix) for k, sy, ix in tr if k == "enc"]
            st = compare_frame(enc, cap["calls"][t], cap["taps"][t])
            ff = st["first_flip"]
            hw = (slice(None), slice(None), slice(0, cap["h"]), slice(0, cap["w"]))
            row = {"frame": "IP"[t], "symbols": st["symbols"], "sym_diff": st["sym_diff"],
                   "idx_diff": st["idx_diff"], "unexplained": len(st["unexplained"]),
                   "idx_ties": st["idx_diff_compared"], "idx_ties_allowed": idx_allowed(st["idx_compared"]),
                   "first_flip_tie_dist": max(ff["tie_dist"]) if ff else None,
                   "bits": int(r["bit"]), "bits_oracle": int(cap["bits"][t]),
                   "dpsnr_db": psnr(rec, xp) - psnr(cap["recon"][t], xp),
                   "rec_maxabs": rec_maxabs(rec[hw].float().cpu().clamp(0, 1), cap["recon"][t][hw].clamp(0, 1))}
            if st["sym_diff"]:
                # the cascade, element by element: the oracle replays the
                # product's symbols at its ties (tests/parity.py)
                oi, op = cap["onets"]
                fr = O.Forcer([sy for sy, _ in enc], TIE_EPS)
                tap = {}
                with torch.no_grad():
                    if t == 0:
                        calls_f, rec_f = oi.compress(xp, False, args.q_index, tap=tap, recon=True, force=fr)
                    else:
                        calls_f, d_f = op.compress(xp, cap["dpb_i"], False, args.q_index, 1, tap=tap, recon=True,
                                                   force=fr)
                        rec_f = d_f["ref_frame"]
                pre = "i_" if t == 0 else "p_"
                cc = [(sy.clamp(-30000, 30000).to(torch.int16).numpy(), ix.to(torch.int16).numpy(),
                       cap["tabs"][pre + k]) for k, sy, ix in calls_f]
                bits_f = (len(R.DCStream(args.stream_part).encode(cc)) + (13 if t == 0 else 6)) * 8
                sf = compare_forced(enc, calls_f, tap, fr.forced)
                row["replay"] = {"forced": sf["forced"], "sym_diff": sf["sym_diff"], "idx_diff": sf["idx_diff"],
                                 "unexplained": len(sf["unexplained"]), "bits_replay": int(bits_f),
                                 "dpsnr_db": psnr(rec, xp) - psnr(rec_f, xp),
                                 "rec_maxabs": rec_maxabs(rec[hw].float().cpu().clamp(0, 1), rec_f[hw].clamp(0, 1))}
            out.append(row)

    def frame_ok(r):
        if r["unexplained"] or r["idx_ties"] > r["idx_ties_allowed"]:
            return False
        if "replay" not in r:
            return r["sym_diff"] > 0 or (abs(r["dpsnr_db"]) < PSNR_DB and r["rec_maxabs"] <= REC_MAXABS)
        f = r["replay"]
        return (f["unexplained"] == 0 and abs(f["dpsnr_db"]) < PSNR_DB
                and (f["sym_diff"] > 0 or f["rec_maxabs"] <= REC_MAXABS))
    ok = all(frame_ok(r) for r in out)
    return {"teacher_forced": out, "passed": ok,
            "bar": f"tests/parity.py: every differing symbol a rounding tie (< {SYM_TIE_EPS:g} from the half-integer), "
                   f"every differing index a tie (< {IDX_TIE_EPS:g} from the integer) and at most "
                   "max(8, 1e-4 x compared) of them per frame; after a flipped symbol the oracle replays the product's "
                   "symbols at its ties and every element of the rest of the frame is checked the same way; identical "
                   f"calls give identical bits, dPSNR < {PSNR_DB:g} dB and decoded pixels within {REC_MAXABS:g} "
                   "(against the replay when a symbol flipped)"}


def launch_ranks(args):
    """`bench.py --gpus N` outside a launcher: start N ranks of this script
    under torch.distributed.run on 127.0.0.1, one per GPU (the reference fans
    its jobs out to one worker per GPU, DCVC-DC/test_video.py:282-290), and
    return their exit code.  Runs before anything touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def parse_cpulist(text):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def gpu_cpulists(n):
    """The host CPUs local to each of the first n visible GPUs (their PCI
    device's NUMA node, from sysfs), or None where sysfs does not say."""
    out = []
    for i in range(n):
        try:
            p = torch.cuda.get_device_properties(i)
            bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            with open(f"/sys/bus/pci/devices/{bus}/local_cpulist") as f:
                out.append(parse_cpulist(f.read()))
        except (OSError, AttributeError, ValueError, RuntimeError):
            out.append(None)
    return out


def rank_cpu_plan(local, local_world, lists, allowed):
    """The host cores of local rank `local` (one process per GPU, local_world
    of them on this node): the cores local to its GPU that this process may
    use, split evenly between the ranks whose GPUs share that NUMA node, so
    no two ranks' coder threads and GOP lanes run on one core.  `lists`:
    gpu_cpulists(local_world); `allowed`: the process's affinity.  Falls back
    to an even split of `allowed` when sysfs gives no NUMA placement."""
    allowed = sorted(allowed)
    mine = lists[local] if local < len(lists) else None
    if mine:
        pool = [c for c in mine if c in set(allowed)]
        peers = [r for r in range(local_world) if r < len(lists) and lists[r] and set(lists[r]) == set(mine)]
    else:
        pool, peers = allowed, list(range(local_world))
    if not pool:
        pool, peers = allowed, list(range(local_world))
    k = peers.index(local) if local in peers else 0
    n = len(peers) or 1
    per = max(1, len(pool) // n)
    share = pool[k * per:(k + 1) * per] if len(pool) >= n else pool
    return share or allowed


def pin_rank(local, local_world, lanes, parts):
    """Pin this rank to its share of the host (rank_cpu_plan) and size the
    rANS worker pool to it: parts - 1 workers at most (a frame's stream parts
    are coded by the workers plus the lane's own thread), at most the share
    less the lanes' threads.  Returns the plan for the bench line."""
    from dcvc_amd._native import rans_lib
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        allowed = list(range(os.cpu_count() or 1))
    lists = gpu_cpulists(local_world)
    share = rank_cpu_plan(local, local_world, lists, allowed)
    try:
        os.sched_setaffinity(0, share)
    except (AttributeError, OSError):
        pass
    workers = max(1, min(parts - 1, len(share) - lanes))
    rc = rans_lib().dcvc_rans_set_threads(workers)
    return {"cores": len(share), "cpus": f"{share[0]}-{share[-1]}" if share else "",
            "numa_local": lists[local] is not None if local < len(lists) else False,
            "coder_workers": workers if rc == 0 else rans_lib().dcvc_rans_threads(), "lane_threads": lanes}


def launcher_selftest(args):
    """--launcher-selftest: the rank plumbing of the N-GPU bench without a GPU
    (gloo): every rank joins, contributes its rank, and rank 0 prints one JSON
    line with the world size it saw (tests/test_bench_launcher.py)."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.tensor([1.0, float(rank)])
    dist.all_reduce(t)
    dist.barrier()
    elapsed = max_over_ranks(dist, 0.001 * (rank + 1), "cpu")
    # the host plan each rank would take on a node whose GPUs sit on two NUMA
    # nodes of the allowed cores (sysfs is not read here: no GPU)
    local = int(os.environ.get("LOCAL_RANK", rank))
    allowed = sorted(os.sched_getaffinity(0))
    half = len(allowed) // 2
    lists = [allowed[:half] if r < world // 2 else allowed[half:] for r in range(world)]
    share = rank_cpu_plan(local, world, lists, allowed)
    from dcvc_amd._native import rans_lib
    L = rans_lib()
    workers = max(1, min(args.stream_part - 1, len(share) - args.lanes))
    set_rc = L.dcvc_rans_set_threads(workers)
    from dcvc_amd import rans as P
    coders = [(P.RansEncoder(True, args.stream_part), P.RansDecoder(args.stream_part))
              for _ in range(2 * args.lanes)]
    nthreads = len(os.listdir("/proc/self/task"))
    plans = [None] * world
    dist.all_gather_object(plans, {"rank": rank, "share": share, "coder_workers": L.dcvc_rans_threads(),
                                   "set_rc": set_rc, "coders": len(coders), "threads": nthreads})
    ranks = rank_records(dist, rank, world, args.lanes * args.steps, 0.001 * (rank + 1))
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_joined": int(t[0]), "rank_sum": int(t[1]),
                          "max_elapsed": elapsed, "requested": args.gpus, "plans": plans, "ranks": ranks}),
              flush=True)
    dist.destroy_process_group()


def hem_q(sd_i, sd_p, rate):
    """(i q_scale, mv_y q_scale, y q_scale) of rate point `rate` from the
    checkpoints' ladders, as DCVC-HEM/test_video.py:274-300 picks them."""
    return (float(sd_i["q_scale"].reshape(-1)[rate]), float(sd_p["mv_y_q_scale"].reshape(-1)[rate]),
            float(sd_p["y_q_scale"].reshape(-1)[rate]))


def cpu_baseline_hem(isd, psd, args):
    """HEM oracle on the same sample as cpu_baseline: one full-size I-frame and
    one full-size P-frame (zero-padded to a multiple of 64), write mode with
    per-call rANS encode + decode, GOP average, no area scaling."""
    from oracle import hem_oracle as O
    from oracle import rans_oracle as R
    from dcvc_amd.synth import moving_pattern, to_float
    info = host_info()
    threads = max(1, min(args.cpu_threads, info["usable"]))
    torch.set_num_threads(threads)
    h, w = args.height, args.width
    Hp, Wp = (h + 63) // 64 * 64, (w + 63) // 64 * 64
    inet = O.IntraOracle(isd, R.pmf_to_quantized_cdf)
    pnet = O.DMCOracle(psd, R.pmf_to_quantized_cdf)
    tabs = {"i_y": inet.tab_y[:3], "i_z": inet.tab_z[:3], "p_y": pnet.tab_y[:3], "p_z": pnet.tab_z[:3],
            "p_mvz": pnet.tab_mvz[:3]}
    qi, qmv, qy = (round(q * 100) / 100 for q in hem_q(isd, psd, args.rate))

    def coder(calls):
        pos = [0]

        def decoder(kind, idx):
            sym = calls[pos[0]][1]
            pos[0] += 1
            st = R.hem_encode(sym.to(torch.int32).numpy(), idx.numpy(), *tabs[kind])
            return torch.from_numpy(R.hem_decode(st, idx.numpy(), *tabs[kind]).astype(np.int64))
        return decoder

    def frame(t):
        x = torch.from_numpy(to_float(moving_pattern(h, w, t, seed=1))).unsqueeze(0)
        return torch.nn.functional.pad(x, (0, Wp - w, 0, Hp - h))

    frames = [frame(t) for t in range(2)]
    with torch.no_grad():
        t0 = time.time()
        xh = inet.decompress(coder(inet.compress(frames[0], qi)), Hp, Wp, qi)
        t_i = time.time() - t0
        dpb = {"ref_frame": xh, "ref_feature": None, "ref_y": None, "ref_mv_y": None}
        t0 = time.time()
        pnet.decompress(dpb, coder(pnet.compress(frames[1], dpb, qmv, qy)), Hp, Wp, qmv, qy)
        t_p = time.time() - t0
    gop = args.gop
    fps = gop / (t_i + (gop - 1) * t_p)
    return {"value": fps, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"HEM oracle write-mode encode+decode of one full-size I-frame ({t_i:.1f} s) and one "
                      f"full-size P-frame ({t_p:.1f} s) at {Hp}x{Wp}, {threads} torch threads in one process; "
                      f"fps = GOP {gop} average; host nproc {info['nproc']}, usable {info['usable']}, "
                      f"CPU {info['cpu']}",
            "ms_I": round(t_i * 1e3, 1), "ms_P": round(t_p * 1e3, 1),
            **({"workers": _workers_record(args)} if _workers_record(args) else {})}


def workload_key(argv):
    """(model, yuv420, height, width) of a bench.py command line."""
    toks = argv.split() if isinstance(argv, str) else list(argv)

    def opt(name, default):
        return toks[toks.index(name) + 1] if name in toks else default
    yuv = "--yuv420" in toks
    return (opt("--model", "dc"), yuv, int(opt("--height", 2160 if yuv else 1080)),
            int(opt("--width", 3840 if yuv else 1920)))


def pmc_traffic(kname, workload):
    """HBM bytes per launch of `kname` (instantiation@grid) from the committed
    rocprofv3 PMC summary (profiles/*_pmc.json, written by
    scripts/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE passes,
    FETCH_SIZE doubled per the gfx950 calibration) of the same workload
    (model, source format, frame size); None when no summary has this kernel
    on this workload."""
    import glob
    for path in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                              "profiles", "*_pmc.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if workload_key(d.get("command", "")) != workload:
            continue
        for e in d.get("kernels", []):
            if e.get("kernel") == kname and e.get("hbm_bytes_per_launch"):
                return {"hbm_bytes_per_launch": e["hbm_bytes_per_launch"], "source": os.path.basename(path),
                        "rocprof_avg_launch_us": e.get("avg_us")}
    return None


def pmc_layer_traffic(kname, layer, nbytes):
    """HBM bytes per launch of one layer shape from a committed per-layer PMC
    record (profiles/*_pmc_layers.json, scripts/pmc_layer.sh: the split conv
    microbenchmark of that shape under separate FETCH_SIZE / WRITE_SIZE
    passes), for a dominant kernel whose whole-frame PMC average mixes layer
    shapes; matched by instantiation@grid, layer key and algorithmic bytes
    (within 1 %, which tells a residual from none)."""
    import glob
    for path in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                              "profiles", "*_pmc_layers.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        recs = [e for e in d.get("layers", []) if e.get("kernel") == kname and e.get("layer") == layer]
        for e in recs:
            if abs(e.get("algorithmic_bytes_no_weights", 0) - nbytes) <= 0.01 * nbytes:
                return {"hbm_bytes_per_launch": e["hbm_bytes_per_launch"], "source": os.path.basename(path),
                        "rocprof_avg_launch_us": e.get("avg_us")}
        # the layer key's launches mix calls with and without a residual: the
        # traffic of that mix is linear in the mix, as the algorithmic bytes are
        plain = [e for e in recs if not e.get("residual")]
        resid = [e for e in recs if e.get("residual")]
        if plain and resid:
            b0, b1 = plain[0]["algorithmic_bytes_no_weights"], resid[0]["algorithmic_bytes_no_weights"]
            if b0 < nbytes < b1:
                f = (nbytes - b0) / (b1 - b0)
                t = plain[0]["hbm_bytes_per_launch"] * (1 - f) + resid[0]["hbm_bytes_per_launch"] * f
                return {"hbm_bytes_per_launch": int(t), "source": os.path.basename(path),
                        "rocprof_avg_launch_us": None, "mix_residual_fraction": round(f, 3)}
    return None


def heartbeat(period=60.0):
    """A line on stderr every `period` seconds while the bench runs (long CPU
    baseline samples would otherwise look like a hung process to a watchdog
    that expects output); the JSON result stays the only stdout line."""
    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f"bench: running, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.launcher_selftest:
        return launcher_selftest(args)
    heartbeat()
    if args.cpu_baseline_workers:
        return cpu_baseline_workers(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    host_plan = pin_rank(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)), args.lanes, args.stream_part)

    from dcvc_amd import hip as K
    from dcvc_amd.layers import Precision
    from dcvc_amd.harness import FrameStage, psnr_rgb, psnr_yuv
    from dcvc_amd.synth import moving_pattern, moving_pattern_yuv420

    for kv in filter(None, os.environ.get("DCVC_OPTS", "").split(",")):
        k, v = kv.split("=")
        K.set_option(k, int(v))
    hem = args.model == "hem"
    isd, psd = make_weights(dist, rank, device, args.model)
    prec = {"split": Precision.split(), "fast": Precision.fast(), "parity": Precision.parity(),
            "fast-bf16-tail": Precision.fast(latent_compute=K.BF16)}[args.precision]
    if hem:
        from dcvc_amd.hem import DMC, IntraNoAR
        qi, qmv, qy = hem_q(isd, psd, args.rate)
    else:
        from dcvc_amd.dc import DMC, IntraNoAR

    h, w = args.height, args.width
    align = 64 if hem else 16     # HEM test_video.py:113-119 pads to 64, DC to 16
    # frame schedule: W warmup frames, then K timed frames starting at the next
    # GOP boundary, so the timed window opens with an I-frame (an I-frame resets
    # the DPB, test_video.py:140-150) and holds the IP=gop mix of the metric
    start = -(-args.warmup // args.gop) * args.gop
    warm_idx = list(range(args.warmup))
    timed_idx = list(range(start, start + args.steps))
    extra = start + args.steps if (start + args.steps) % args.gop else start + args.steps + 1
    sched = warm_idx + timed_idx + [extra]
    nframes = len(sched)
    out_root = f"/dev/shm/dcvc_bench_{os.getpid()}"

    class Lane:
        """One GOP lane: its own codec instances, HIP stream, frame staging
        and output folder.  Lane l codes GOP l of this rank's sequence (an
        I-frame resets the DPB, so GOPs are independent, test_video.py:
        140-150).  With several lanes each runs on its own host thread and
        HIP stream, so one lane's host rANS work overlaps another's kernels."""

        def __init__(self, l):
            self.l = l
            if hem:
                self.inet = IntraNoAR(precision=prec, device=device).load_state_dict(isd)
                self.pnet = DMC(precision=prec, device=device).load_state_dict(psd)
            else:
                self.inet = IntraNoAR(precision=prec, stream_part=args.stream_part, device=device).load_state_dict(isd)
                self.pnet = DMC(precision=prec, stream_part=args.stream_part, device=device).load_state_dict(psd)
            self.inet.update(force=True)
            self.pnet.update(force=True)
            self.stream = torch.cuda.Stream(device) if args.lanes > 1 else torch.cuda.current_stream(device)
            # run_test's frame handling (dcvc_amd.harness.FrameStage): uint8
            # source resident in HBM, converted to the padded NHWC input
            # inside the step; the distortion (in-place clamp + squared-error
            # sums) is part of the step
            self.stage = FrameStage(h, w, align, args.yuv420, zero_pad=hem, frame_num=nframes + 2, device=device)
            t0 = l * args.gop
            self.slot = {t: n for n, t in enumerate(sched)}
            if args.yuv420:
                self.frames = {t: tuple(torch.from_numpy(a).to(device)
                                        for a in moving_pattern_yuv420(h, w, t0 + t, seed=shard_seed(rank)))
                               for t in sched}
            else:
                self.frames = {t: torch.from_numpy(moving_pattern(h, w, t0 + t, seed=shard_seed(rank))).to(device)
                               for t in sched}
            self.out_dir = os.path.join(out_root, str(l))
            os.makedirs(self.out_dir, exist_ok=True)
            self.dpb = None
            self.bits, self.kinds, self.per = {}, {}, []

        def step(self, i):
            # uint8 source -> padded NHWC: replicate (DC test_video.py:130) / zeros (HEM)
            x = self.stage.load(self.frames[i])
            path = os.path.join(self.out_dir, f"{i}.bin")
            inet, pnet = self.inet, self.pnet
            if hem:
                if i % args.gop == 0:
                    r = inet.encode_decode(x, qi, path, pic_width=w, pic_height=h)
                    self.dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_y": None, "ref_mv_y": None}
                    self.kinds[i] = "I"
                else:
                    r = pnet.encode_decode(x, self.dpb, path, pic_width=w, pic_height=h,
                                           mv_y_q_scale=qmv, y_q_scale=qy)
                    self.dpb = r["dpb"]
                    self.kinds[i] = "P"
            elif i % args.gop == 0:
                r = inet.encode_decode(x, False, args.q_index, path, pic_width=w, pic_height=h)
                self.dpb = {"ref_frame": r["x_hat"], "ref_feature": None, "ref_mv_feature": None,
                            "ref_y": None, "ref_mv_y": None}
                self.kinds[i] = "I"
            else:
                r = pnet.encode_decode(x, self.dpb, False, args.q_index, path, pic_width=w, pic_height=h,
                                       frame_idx=i % 4)
                self.dpb = r["dpb"]
                self.kinds[i] = "P"
            self.bits[i] = r["bit"]
            self.stage.distortion(self.dpb["ref_frame"], self.frames[i], self.slot[i])

        def run(self, idx, timed):
            with torch.cuda.device(device), torch.cuda.stream(self.stream):
                for i in idx:
                    ts = time.time()
                    self.step(i)
                    if timed:
                        self.per.append(time.time() - ts)
                self.stream.synchronize()

    lanes = [Lane(l) for l in range(args.lanes)]
    H, W = lanes[0].stage.H, lanes[0].stage.W
    torch.cuda.synchronize(device)   # setup work on the default stream is done before lanes start

    def run_all(idx, timed):
        if len(lanes) == 1:
            lanes[0].run(idx, timed)
            return
        import threading
        errs = []

        def go(ln):
            try:
                ln.run(idx, timed)
            except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
                errs.append(e)
        th = [threading.Thread(target=go, args=(ln,)) for ln in lanes]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]

    run_all(warm_idx, False)
    torch.cuda.synchronize(device)
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    run_all(timed_idx, True)
    torch.cuda.synchronize(device)
    own = time.time() - t0
    if dist is not None:
        dist.barrier()
    elapsed = max_over_ranks(dist, time.time() - t0, device)
    # frames re-coded on the fp32 twin after the split range guard tripped
    # (layers.split_guarded): such a frame is timed on the fp32 kernels, so
    # the line counts them, and the metric is flagged when any occurred
    fallbacks = sum(getattr(net, "fallbacks", 0) for ln in lanes for net in (ln.inet, ln.pnet))
    ranks = rank_records(dist, rank, world, args.lanes * args.steps, own, fallbacks)

    def step(i):   # one more frame on lane 0 (the roofline P-frame below)
        lanes[0].run([i], False)

    # ---- roofline of the dominant kernel, from per-launch HIP events recorded
    # on the stream the kernels run on, over one extra P-frame.  "Dominant" =
    # the (kernel instantiation, layer shape) with the most time per P-frame;
    # its bound is the larger of its MFMA time and its HBM time at peak.
    roof = None
    if not args.no_roofline and rank == 0:
        K.PROFILE = []
        step(extra)
        torch.cuda.synchronize(device)
        fam, shapes = {}, {}
        for f, e0, e1, fl, nb, key in K.PROFILE:
            dt = e0.elapsed_time(e1) * 1e-3
            for tab, k in ((fam, f), (shapes, f + " " + key if "|" not in key else key)):
                d = tab.setdefault(k, [0.0, 0, 0, 0])
                d[0] += dt
                d[1] += fl
                d[2] += nb
                d[3] += 1
        K.PROFILE = None
        rows = sorted(shapes.items(), key=lambda kv: -kv[1][0])
        if args.profile_out:
            with open(args.profile_out, "w") as f:
                json.dump([{"op": k, "ms": round(v[0] * 1e3, 4), "n": v[3],
                            "tflops": round(v[1] / max(v[0], 1e-12) / 1e12, 2),
                            "gbs": round(v[2] / max(v[0], 1e-12) / 1e9, 1)} for k, v in rows], f, indent=0)
        key, (tsec, fl, nb, n) = rows[0]
        peak_f = peak_of(key.split("<")[0].split(" ")[0], key)
        t_mfma, t_hbm = fl / (peak_f * 1e12), nb / (PEAK_HBM_GBS * 1e9)
        if t_mfma >= t_hbm:
            ach = fl / tsec / 1e12
            roof = {"bound": "mfma", "achieved": round(ach, 3), "peak": peak_f, "unit": "TFLOP/s",
                    "frac": round(ach / peak_f, 5)}
        else:
            ach = nb / tsec / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": round(ach / PEAK_HBM_GBS, 5)}
        kname, _, shape = key.partition(" | ")
        tr = pmc_traffic(kname, (args.model, args.yuv420, h, w))
        roof["traffic"] = tr["hbm_bytes_per_launch"] if tr else None
        if tr:
            roof["traffic_source"] = tr["source"]
            roof["rocprof_avg_launch_us"] = tr["rocprof_avg_launch_us"]
            # the PMC summary is keyed by instantiation@grid; a persistent
            # kernel keeps its grid across layer shapes, so its per-launch
            # average can mix layers.  Report traffic only when the rocprof
            # average launch time agrees with this layer's (within 25 %).
            ev = tsec / n * 1e6
            if tr["rocprof_avg_launch_us"] and abs(tr["rocprof_avg_launch_us"] - ev) > 0.25 * ev:
                roof["traffic"] = None
                roof["traffic_note"] = ("PMC summary of this instantiation@grid averages several layer shapes "
                                        f"(rocprof {tr['rocprof_avg_launch_us']} us vs {ev:.1f} us for this layer)")
                lt = pmc_layer_traffic(kname, shape, nb / n)
                if lt:
                    roof["traffic"] = lt["hbm_bytes_per_launch"]
                    roof["traffic_source"] = lt["source"]
                    roof["traffic_note"] += ("; traffic from the per-layer PMC records of this shape (microbenchmark"
                                             + (f", {lt['mix_residual_fraction']} of the launches with a residual"
                                                if "mix_residual_fraction" in lt else "") + ")")
        roof["kernel"] = kname
        roof["layer"] = shape
        roof["launches_per_P_frame"] = n
        roof["avg_launch_us"] = round(tsec / n * 1e6, 2)
        roof["algorithmic_per_launch"] = {"flop": fl // n, "bytes": nb // n}
        roof["families_ms_per_P_frame"] = {k: round(v[0] * 1e3, 3) for k, v in fam.items()}
        # whole-frame layer roofline: sum over launches of max(F/P, B/BW)
        t_all = sum(v[0] for v in shapes.values())
        t_roof = sum(max(v[1] / (peak_of(k.split("<")[0].split(" ")[0], k) * 1e12), v[2] / (PEAK_HBM_GBS * 1e9))
                     for k, v in shapes.items())
        roof["P_frame_kernels"] = {"gpu_ms": round(t_all * 1e3, 3), "roofline_ms": round(t_roof * 1e3, 3),
                                   "frac": round(t_roof / max(t_all, 1e-12), 4),
                                   "tflop": round(sum(v[1] for v in shapes.values()) / 1e12, 3),
                                   "gbytes": round(sum(v[2] for v in shapes.values()) / 1e9, 2)}

    if rank == 0:
        kinds = [ln.kinds[i] for ln in lanes for i in timed_idx]
        per = [p for ln in lanes for p in ln.per]
        n_i = kinds.count("I")
        ti = [p for p, k in zip(per, kinds) if k == "I"]
        tp = [p for p, k in zip(per, kinds) if k == "P"]
        cpu, parity = None, None
        if not args.no_cpu_baseline and world == 1:
            cap = {} if (not hem and not args.yuv420 and not args.no_parity_check) else None
            cpu = cpu_baseline_hem(isd, psd, args) if hem else cpu_baseline(isd, psd, args, cap)
            if cap:
                with torch.cuda.device(device), torch.cuda.stream(lanes[0].stream):
                    parity = parity_check(cap, lanes[0].inet, lanes[0].pnet, args)
        timed_bits = [ln.bits[i] for ln in lanes for i in timed_idx]
        sse = np.concatenate([ln.stage.sums()[[ln.slot[i] for i in timed_idx]] for ln in lanes])
        if args.yuv420:
            per = [psnr_yuv(e, h, w) for e in sse]
            psnr = {"psnr": round(float(np.mean([p[3] for p in per])), 4),
                    "psnr_yuv": [round(float(np.mean([p[c] for p in per])), 4) for c in range(3)]}
        else:
            psnr = {"psnr": round(float(np.mean([psnr_rgb(e, h, w) for e in sse])), 4)}
        line = {
            "metric": metric_name(args, parity),
            "parity_evidence": parity_evidence(args, parity),
            "value": round(world * args.lanes * args.steps / elapsed, 4),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": {"split": "f32 (convs on split-fp16 f16x3 MFMA, fp32 accumulation)", "parity": "f32",
                      "fast": "bf16 features, fp32 entropy params",
                      "fast-bf16-tail": "bf16 (entropy-parameter tail in bf16 too)"}[args.precision],
            "data": "synthetic (moving sinusoid + noise frames, seeded random weights)",
            "host_plan": host_plan,
            "config": {"workload": (f"C2 DCVC-HEM RGB {w}x{h} (zero pad {W}x{H}) IP={args.gop} write mode"
                                    if hem else
                                    f"C4 DCVC-DC YUV420 {w}x{h} (pad {W}x{H}) IP={args.gop} write mode" if args.yuv420
                                    else f"C3 DCVC-DC RGB {w}x{h} (pad {W}x{H}) IP={args.gop} write mode"),
                       "gop": args.gop, "precision": args.precision,
                       **({"rate": args.rate, "q_scales": [round(qi, 4), round(qmv, 4), round(qy, 4)]} if hem
                          else {"q_index": args.q_index, "stream_part": args.stream_part}), "parallelism": f"sequence-sharded x{world}, {args.lanes} GOP lane(s) per GPU",
                       "lanes": args.lanes, "frames_timed": world * args.lanes * args.steps,
                       "I_frames_timed": n_i,
                       "ms_I": round(1e3 * float(np.mean(ti)), 2) if ti else None,
                       "ms_P": round(1e3 * float(np.mean(tp)), 2) if tp else None,
                       "timed_frames": [timed_idx[0], timed_idx[-1]],
                       # steady-state GOP mix from the per-frame latencies: lanes x
                       # gop / (t_I + (gop - 1) t_P), every lane count
                       **({"fps_gop_avg": round(args.lanes * args.gop / (float(np.mean(ti))
                                                                        + (args.gop - 1) * float(np.mean(tp))), 3),
                           "fps_gop_avg_note": (f"value times {n_i} I-frame(s) in {len(kinds)} frames (1 in "
                                                f"{len(kinds) / max(n_i, 1):.0f}); the sequence has 1 in {args.gop}: "
                                                "fps_gop_avg is lanes x gop / (ms_I + (gop - 1) ms_P), the rate at "
                                                "the sequence's own I-frame share")}
                          if ti and tp else {}),
                       "step": f"one frame on each of {args.lanes} lane(s)",
                       "bpp": round(float(np.mean(timed_bits)) / (h * w), 5), **psnr,
                       **({"bits_per_lane": [int(sum(ln.bits[i] for i in timed_idx)) for ln in lanes]}
                          if args.lanes > 1 else {})},
            "precision_fallbacks": sum(r["precision_fallbacks"] for r in ranks),
            **({"ranks": ranks, "rank_fps_spread": {
                "min": min(r["fps"] for r in ranks), "mean": round(float(np.mean([r["fps"] for r in ranks])), 4),
                "max": max(r["fps"] for r in ranks)}} if world > 1 else {}),
            "roofline": roof,
            "cpu_baseline": cpu,
            "parity_check": parity,
        }
        if line["precision_fallbacks"]:
            line["metric"] += (f" [{line['precision_fallbacks']} frame(s) re-coded on the fp32 twin after the split "
                               "range guard tripped: not all timed frames ran in split precision]")
        print(json.dumps(line), flush=True)
    import shutil
    shutil.rmtree(out_root, ignore_errors=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
