#!/usr/bin/env python3
"""Per-kernel averages (kernel trace) and read bytes (FETCH_SIZE, the gfx950
2x correction of MI355X_MICROARCH.md) of the row-template launches in the
records tools/runs/tmpl_ab.sh writes: one line per setting and epilogue.

    python3 tools/tmpl_summary.py gpurun_out/r06/v
"""
import collections
import csv
import glob
import sys
from pathlib import Path


def op_name(k):
    for op in ("OpMult<false>", "OpMult<true>", "OpMgPost<true>", "OpMgPost<false>", "OpMgResid<true>",
               "OpMgResid<false>", "OpDinvMult"):
        if op in k:
            return op
    return "?"


def main():
    d = Path(sys.argv[1])
    for tr in sorted(d.glob("trace_*")):
        if not tr.is_dir():
            continue
        name = tr.name[len("trace_"):]
        us = {}
        for r in csv.DictReader(open(next(tr.rglob("*kernel_stats.csv")))):
            if "k_spmv_template" in r["Name"] or "k_spmv_pattern" in r["Name"]:
                us[op_name(r["Name"])] = (int(r["Calls"]), round(float(r["AverageNs"]) / 1e3, 1))
        rd = collections.defaultdict(list)
        f = d / f"fetch_{name}"
        if f.exists():
            for r in csv.DictReader(open(next(f.rglob("*counter_collection.csv")))):
                if "k_spmv_template" in r["Kernel_Name"] or "k_spmv_pattern" in r["Kernel_Name"]:
                    rd[op_name(r["Kernel_Name"])].append(2 * float(r["Counter_Value"]) * 1024)
        log = (d / f"trace_{name}.log").read_text().splitlines() if (d / f"trace_{name}.log").exists() else []
        solve = [x for x in log if x.startswith("gamg: set-up")]
        print(name, solve[-1] if solve else "")
        for op, (calls, avg) in sorted(us.items()):
            v = sorted(rd.get(op, []))
            print(f"   {op:18s} calls {calls:4d}  avg {avg:7.1f} us  read {v[len(v) // 2] / 1e9 if v else float('nan'):.3f} GB")


if __name__ == "__main__":
    main()
