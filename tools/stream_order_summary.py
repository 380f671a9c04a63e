#!/usr/bin/env python3
"""Kernel durations, gaps and hardware queues of the skewed stand-in's
MatMult under tools/ab_opts.py --dummy-streams K (does
the stream-order swing move the kernels or the gaps between them, and on
which queue?). Reads the rocprofv3 kernel traces tools/runs/stream_order.sh
writes; one JSON line per trace: per kernel family the launches, mean
duration and queue ids, and the mean gap from the previous kernel's end to
each family's start.

    python3 tools/stream_order_summary.py gpurun_out/r06/so
"""
import csv
import json
import statistics
import sys
from pathlib import Path


def family(name):
    for k in ("k_spmv_stream", "k_long_partial", "k_long_finish", "k_spmv_template", "k_spmv_pattern"):
        if k in name:
            if k == "k_spmv_stream":
                return "row_blocks_wide" if ", 65," in name else "row_blocks"
            return k
    return None


def main():
    for d in sorted(Path(sys.argv[1]).glob("trace_*")):
        rows = list(csv.DictReader(open(next(d.rglob("*kernel_trace.csv")))))
        ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), family(r["Kernel_Name"]), r["Queue_Id"])
                     for r in rows if family(r["Kernel_Name"])), key=lambda k: k[0])
        ks = ks[len(ks) // 5:]  # past the build and the first rounds
        out = {}
        prev_end = None
        for s, e, f, q in ks:
            o = out.setdefault(f, {"n": 0, "dur": [], "gap": [], "queues": set()})
            o["n"] += 1
            o["dur"].append((e - s) / 1e3)
            o["queues"].add(q)
            if prev_end is not None:
                o["gap"].append((s - prev_end) / 1e3)
            prev_end = e if prev_end is None else max(prev_end, e)
        print(json.dumps({"trace": d.name, **{f: {"launches": o["n"], "us_mean": round(statistics.mean(o["dur"]), 2),
                                                  "gap_us_mean": round(statistics.mean(o["gap"]), 2) if o["gap"] else None,
                                                  "queues": sorted(o["queues"])} for f, o in out.items()}}))


if __name__ == "__main__":
    main()
