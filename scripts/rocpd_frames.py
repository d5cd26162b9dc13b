"""Per-frame kernel summary from a rocprofv3 rocpd database (box diagnostic).

Frames are delimited by frame_kernel launches (one per coded frame).

    python scripts/rocpd_frames.py <results.db> [frame_index] [top]
"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    fi = int(sys.argv[2]) if len(sys.argv) > 2 else -2
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if "frame_kernel" in r[0]] + [len(rows)]
    a, b = idx[fi - 1], idx[fi]
    seg = rows[a:b]
    busy = sum(r[2] - r[1] for r in seg) / 1e6
    span = (seg[-1][2] - seg[0][1]) / 1e6
    gaps = [(seg[i + 1][1] - seg[i][2]) / 1e6 for i in range(len(seg) - 1)]
    print(f"launches {len(seg)}  busy {busy:.2f} ms  span {span:.2f} ms  gaps {sum(gaps):.2f} ms "
          f"(>0.5 ms: {sum(g for g in gaps if g > 0.5):.2f})")
    agg = collections.defaultdict(lambda: [0.0, 0])
    for r in seg:
        n = r[0].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:90]
        agg[n][0] += (r[2] - r[1]) / 1e6
        agg[n][1] += 1
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{v[0]:8.3f} {v[1]:4d}  {k}")


if __name__ == "__main__":
    main()
