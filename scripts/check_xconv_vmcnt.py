"""Build-time check of xconv3_kernel's exact vmcnt waits (make runs it).

xconv.hip waits for a stage's weight LDS-DMA with vmcnt(N), N = the count of
vector-memory instructions issued after that DMA, computed at compile time
from the schedule the kernel template assumes (XG::after_dma / wait_for).
That is only right if hipcc emits exactly those instructions in that order.
Round 5's ring race came from a load the template counted and hipcc deleted
as dead: the waits then passed with the DMA still in flight (DESIGN.md
section 9.0).  This script compares, for every instantiation in the built
library, the template's schedule (dcvc_internal_xconv_schedule, host-side:
no GPU) with the instructions in the code object:

  * the vector-memory instructions between consecutive stage barriers of the
    tile loop, in program order, must be exactly the template's (D weight
    LDS-DMA, L image / residual load, S output store): a deleted, merged,
    added (a spill's scratch access) or reordered one fails;
  * the vmcnt of the wait in front of each stage barrier must be the
    template's (a smaller one is stricter, reported, not fatal).

The same script checks wconv.hip's object (its DMA wave's loop against
dcvc_internal_wconv_schedule) and sffn.hip's (the streamed kernels: on every
control-flow path to a barrier, the slice DMA it waits for is followed by at
least vmcnt(N) vector-memory instructions; check_sffn_kernel).

    python scripts/check_xconv_vmcnt.py dcvc_amd/lib/libdcvc_hip.so build/hip/xconv.o
    python scripts/check_xconv_vmcnt.py LIB disasm.s      (an llvm-objdump -d listing)
"""
import ctypes
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MANGLED = re.compile(r"xconv3_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)E")
WMANGLED = re.compile(r"wconv3_kernelILi(\d+)ELi(\d+)ELi(\d+)E")


def schedules(lib_path, sym="dcvc_internal_xconv_schedule", nprm=6):
    """{(cin, bn, rw, nw, nres, ks): [(ops, wait)] per stage} of every
    instantiation the library registered (wconv.hip's: {(cin, bn, nres): ..},
    its producer waves' schedule)."""
    lib = ctypes.CDLL(os.path.abspath(lib_path))
    f = getattr(lib, sym)
    f.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
    f.restype = ctypes.c_int
    out = {}
    i = 0
    while True:
        prm = (ctypes.c_int * nprm)()
        buf = ctypes.create_string_buffer(1 << 16)
        if f(i, prm, buf, len(buf)) != 0:
            break
        lines = buf.value.decode().strip().split("\n")
        stages = []
        for ln in lines[1:]:
            ops, w = ln.split()
            stages.append(("" if ops == "-" else ops, int(w)))
        out[tuple(prm)] = stages
        i += 1
    return out


def disassemble(obj):
    """llvm-objdump -d listing of the gfx950 code object inside a host object
    (its .hip_fatbin), or the listing itself for a .s path."""
    if obj.endswith(".s"):
        return open(obj).read()
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "x.fat"), os.path.join(td, "x.co")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                       check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True,
                              text=True).stdout


def kernels(listing, tag="xconv3_kernel"):
    """{mangled name: [(address, mnemonic, operands, branch target or None)]}
    of the xconv3_kernel (or tag) functions."""
    out, cur, base = {}, None, 0
    for ln in listing.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:", ln)
        if m:
            cur = m.group(2) if tag in m.group(2) else None
            base = int(m.group(1), 16)
            if cur:
                out[cur] = []
            continue
        if cur is None:
            continue
        m = re.match(r"\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$", ln)
        if not m:
            continue
        mn, ops, addr, rest = m.group(1), m.group(2), int(m.group(3), 16), m.group(4)
        t = re.search(r"<[^>+]*\+0x([0-9a-f]+)>", rest)
        tgt = base + int(t.group(1), 16) if t and mn.startswith("s_") and "branch" in mn else None
        out[cur].append((addr, mn, ops, tgt))
    return out


def kind(mn, ops):
    if mn.startswith("scratch_") or mn.startswith("buffer_wbl2") or mn.startswith("buffer_inv"):
        return "X"
    if mn.startswith("buffer_load") or mn.startswith("global_load"):
        return "D" if re.search(r"\blds\b", ops) else "L"
    if mn.startswith("buffer_store") or mn.startswith("global_store"):
        return "S"
    if mn.startswith("buffer_") or mn.startswith("global_") or mn.startswith("flat_"):
        return "X"
    return None


def vmcnt_of(ops):
    m = re.search(r"vmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


def check_kernel(name, ins, sched, dma_loop=False):
    """Errors and notes for one instantiation.

    The tile loop is the address range from the target of its back-edges to
    the last of them (hipcc may rotate it, so that its last stage barrier
    sits at the top).  Its barriers cut it into as many intervals, taken
    cyclically (the interval that contains the loop's entry runs from the last
    barrier around to the first); the template's intervals end at its barrier
    stages, so the two lists must agree under one rotation."""
    errs, notes = [], []
    bar_stages = [s for s, (_, w) in enumerate(sched) if w >= 0]
    nb = len(bar_stages)
    back = [(a, t) for a, mn, _, t in ins if t is not None and t < a]
    if not back:
        return [f"{name}: no loop back-edge"], notes
    if dma_loop:
        # wconv3_kernel: the producer waves' tile loop is the one that issues
        # the weight LDS-DMAs (the consumer loop, after it, issues none)
        cand = [(a, t) for a, t in back
                if any(kind(mn, o) == "D" for x, mn, o, _ in ins if t <= x <= a)]
        if not cand:
            return [f"{name}: no loop issues a weight LDS-DMA"], notes
        end, top = max(cand, key=lambda e: e[0] - e[1])
        outside = ""
    else:
        # (the last back-edge is the tile loop's; small loops before it, such
        # as the prologue's bias copy, lie outside its range)
        end, top = max(back)
        outside = "".join(c for c in (kind(mn, ops) for a, mn, ops, _ in ins if a > end) if c and c != "S")
    body = [(a, mn, ops) for a, mn, ops, _ in ins if top <= a <= end]
    bars = [i for i, (_, mn, _) in enumerate(body) if mn == "s_barrier"]
    if len(bars) != nb:
        return [f"{name}: {len(bars)} barriers in the tile loop, the schedule has {nb} stage barriers"], notes
    if outside:
        errs.append(f"{name}: vector-memory instructions {outside} after the tile loop")
    # the loop's intervals, cyclic: cyc[i] ends at body barrier i
    cyc = []
    for i in range(nb):
        seg = body[bars[i - 1] + 1:bars[i]] if i else body[bars[-1] + 1:] + body[:bars[0]]
        ops = "".join(c for c in (kind(mn, o) for _, mn, o in seg) if c)
        w = None
        for _, mn, o in reversed(seg):
            if mn == "s_waitcnt" and vmcnt_of(o) is not None:
                w = vmcnt_of(o)
                break
            if kind(mn, o):
                break
        cyc.append((ops, w))
    want = []
    for k, s in enumerate(bar_stages):
        prev = bar_stages[k - 1] if k else bar_stages[-1] - len(sched)
        ops = "".join(sched[x % len(sched)][0] for x in range(prev + 1, s + 1))
        want.append((ops.replace("I", "L").replace("R", "L"), sched[s][1], f"{prev + 1 if k else 0}..{s}"))
    best = None
    for r in range(nb):
        bad, nts = [], []
        for i in range(nb):
            ops, w = cyc[i]
            wops, ww, rng = want[(i + r) % nb]
            if ops != wops:
                bad.append(f"stages {rng}: vector-memory instructions {ops or '-'}, the vmcnt schedule assumes "
                           f"{wops or '-'}")
            if w is None:
                bad.append(f"stages {rng}: no vmcnt wait before the barrier (the schedule's: vmcnt({ww}))")
            elif w > ww:
                bad.append(f"stages {rng}: vmcnt({w}) before the barrier, the schedule needs vmcnt({ww})")
            elif w < ww:
                nts.append(f"stages {rng}: vmcnt({w}), stricter than the schedule's vmcnt({ww})")
        if best is None or len(bad) < len(best[0]):
            best = (bad, nts)
        if not bad:
            break
    errs += [f"{name}: {b}" for b in best[0]]
    notes += [f"{name}: {n}" for n in best[1]]
    return errs, notes


def main(argv):
    if len(argv) != 3:
        print(__doc__)
        return 2
    listing = disassemble(argv[2])
    if "wconv3_kernel" in listing:
        return main_wconv(argv[1], listing)
    if "sffn_kernel" in listing:
        return main_sffn(listing)
    sched = schedules(argv[1])
    ks = kernels(listing)
    if not ks:
        print("check_xconv_vmcnt: no xconv3_kernel in", argv[2], file=sys.stderr)
        return 1
    errs, notes, seen = [], [], 0
    for name, ins in sorted(ks.items()):
        m = MANGLED.search(name)
        if not m:
            errs.append(f"{name}: cannot read the template parameters")
            continue
        cin, bn, rw, nw, nres, _shuf, k = (int(v) for v in m.groups())
        key = (cin, bn, rw, nw, nres, k)
        if key not in sched:
            errs.append(f"{name}: no schedule registered for {key}")
            continue
        e, n = check_kernel(f"xconv3_kernel<{cin},{bn},{rw},{nw},{nres},{_shuf},{k}>", ins, sched[key])
        errs += e
        notes += n
        seen += 1
    for n in notes:
        print("check_xconv_vmcnt: note:", n)
    for e in errs:
        print("check_xconv_vmcnt:", e, file=sys.stderr)
    if errs:
        return 1
    print(f"check_xconv_vmcnt: {seen} xconv3_kernel instantiations match their vmcnt schedules")
    return 0


def main_wconv(lib, listing):
    """wconv.hip's object: the producer loop of every wconv3_kernel."""
    sched = schedules(lib, "dcvc_internal_wconv_schedule", 3)
    errs, notes, seen = [], [], 0
    for name, ins in sorted(kernels(listing, "wconv3_kernel").items()):
        m = WMANGLED.search(name)
        key = tuple(int(v) for v in m.groups()) if m else None
        if key not in sched:
            errs.append(f"{name}: no schedule registered for {key}")
            continue
        e, n = check_kernel("wconv3_kernel<%d,%d,%d>" % key, ins, sched[key], dma_loop=True)
        errs += e
        notes += n
        seen += 1
    for n in notes:
        print("check_xconv_vmcnt: note:", n)
    for e in errs:
        print("check_xconv_vmcnt:", e, file=sys.stderr)
    if errs or not seen:
        return 1
    print(f"check_xconv_vmcnt: {seen} wconv3_kernel instantiations match their vmcnt schedules")
    return 0


SMANGLED = re.compile(r"sffn_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E")


def sffn_ndw(c, nw):
    """LDS-DMA instructions per wave per streamed slice (sffn.hip FG::NDW)."""
    kc1, c16 = (c + 31) // 32, (c + 15) // 16 * 16
    slice_halves = 2 * kc1 * 32 * 32 + 2 * c16 * 32
    return slice_halves * 2 // 1024 // nw


def successors(ins):
    """Control-flow successors (indexes) of every instruction."""
    at = {a: i for i, (a, _, _, _) in enumerate(ins)}
    out = []
    for i, (a, mn, _, t) in enumerate(ins):
        nxt = [i + 1] if i + 1 < len(ins) else []
        if mn == "s_branch":
            out.append([at[t]] if t in at else [])
        elif mn.startswith("s_cbranch"):
            out.append(([at[t]] if t in at else []) + nxt)
        elif mn == "s_endpgm" or mn.startswith("s_setpc"):
            out.append([])
        else:
            out.append(nxt)
    return out


def check_sffn_kernel(name, ins, ndw):
    """Errors for one streamed sffn_kernel.  Barrier B_s waits for slice s's
    LDS-DMA, issued two barriers earlier (each barrier issues the DMA of the
    slice two ahead): walking back from B_s's vmcnt(N) wait along any path,
    the first NDW DMA instructions met are slice s + 1's and the next one is
    the youngest of slice s's, so at least N vector-memory instructions must
    lie between it and the wait (then vmcnt(N) covers it).  The walk is over
    the control-flow graph, so the runtime-selected waits of B_1 / B_2 (the
    next tile's input prefetch counted or not) are each checked on their own
    paths, and a prefetch that hipcc hoisted above a DMA shows up."""
    succ = successors(ins)
    pred = [[] for _ in ins]
    for i, ss in enumerate(succ):
        for j in ss:
            pred[j].append(i)
    errs, nbar = [], 0
    for b, (addr, mn, _, _) in enumerate(ins):
        if mn != "s_barrier":
            continue
        nbar += 1
        # (index, N or None while looking for the wait, vm ops since the wait, D ops since the wait)
        best = {}
        stack = [(p, None, 0, 0) for p in pred[b]]
        worst = None
        while stack:
            i, n, nops, nd = stack.pop()
            key = (i, n, nd)
            if key in best and best[key] <= nops:
                continue
            best[key] = nops
            a, m, o, _ = ins[i]
            k = kind(m, o)
            if n is None:
                if m == "s_waitcnt" and vmcnt_of(o) is not None:
                    n = vmcnt_of(o)
                elif m == "s_barrier":
                    errs.append(f"{name}: barrier at {addr:#x}: a path from the barrier at {a:#x} has no vmcnt wait")
                    continue
            elif k:
                if k == "D" and nd == ndw:
                    if worst is None or nops - n < worst[0]:
                        worst = (nops - n, nops, n, a)
                    continue
                nops += 1
                nd += k == "D"
            stack += [(p, n, nops, nd) for p in pred[i]]
        if worst is not None and worst[0] < 0:
            errs.append(f"{name}: barrier at {addr:#x}: vmcnt({worst[2]}), but only {worst[1]} vector-memory "
                        f"instructions follow the DMA it waits for (at {worst[3]:#x}) on some path")
    if nbar == 0:
        errs.append(f"{name}: no barrier")
    return errs, nbar


def main_sffn(listing):
    """sffn.hip's object: every streamed (NBUF > 0) sffn_kernel."""
    errs, seen = [], 0
    for name, ins in sorted(kernels(listing, "sffn_kernel").items()):
        m = SMANGLED.search(name)
        if not m:
            errs.append(f"{name}: cannot read the template parameters")
            continue
        c, nw, np_, nbuf = (int(v) for v in m.groups())
        if nbuf == 0:
            continue   # every slice resident: vmcnt(0) before the one barrier
        e, nb = check_sffn_kernel(f"sffn_kernel<{c},{nw},{np_},{nbuf}>", ins, sffn_ndw(c, nw))
        errs += e
        seen += 1
    for e in errs:
        print("check_xconv_vmcnt:", e, file=sys.stderr)
    if errs or not seen:
        return 1
    print(f"check_xconv_vmcnt: {seen} streamed sffn_kernel instantiations wait for each slice's DMA")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
