#!/usr/bin/env python3
"""Kernel timeline of a rocprofv3 --kernel-trace CSV: per kernel name the
count and mean duration, and the idle time between consecutive kernels
(start of one minus end of the previous) over the last N kernels — the
launch gaps a hipGraph or fewer launches would remove.

    python3 tools/trace_gaps.py DIR [--last N] [--span-ms MS] [--by-grid]

--span-ms keeps the kernels that start in the trace's last MS milliseconds
(a solve at the end of the run); --by-grid splits a kernel name by its grid
size (the levels of a GAMG hierarchy launch the same kernels).
"""
import argparse
import csv
from collections import defaultdict
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=1000)
    ap.add_argument("--span-ms", type=float, default=0.0)
    ap.add_argument("--by-grid", action="store_true")
    a = ap.parse_args()
    rows = []
    for f in Path(a.dir).rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("aijhip::", "")
                name = name.split("(")[0][-90:]
                if a.by_grid:
                    name = f"{name} [grid {r['Grid_Size_X']}]"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    if a.span_ms > 0:
        rows = [q for q in rows if q[0] >= rows[-1][1] - a.span_ms * 1e6]
    else:
        rows = rows[-a.last:]
    busy = sum(e - s for s, e, _ in rows)
    span = rows[-1][1] - rows[0][0]
    gaps = defaultdict(list)
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        gaps[n1].append(s1 - e0)
    per = defaultdict(list)
    for s, e, n in rows:
        per[n].append(e - s)
    print(f"{len(rows)} kernels, span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us ({busy / span:.3f})")
    for n, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        g = gaps.get(n, [0])
        print(f"{len(d):6d} x {sum(d) / len(d) / 1e3:9.2f} us  gap before {sum(g) / len(g) / 1e3:7.2f} us  {n}")


if __name__ == "__main__":
    main()
