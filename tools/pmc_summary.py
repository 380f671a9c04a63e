#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh) per kernel.

Per kernel: mean of each counter over its dispatches, plus derived HBM
traffic per launch with the gfx950 correction of MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KiB) reads 1/2 of a wide coalesced stream's bytes, so
read_bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KiB) is exact for streaming
stores: write_bytes = WRITE_SIZE * 1024. Also the effective clock
GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH 'DVFS give-back').
"""
from __future__ import annotations

import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def load_counters(d: Path):
    out = defaultdict(lambda: defaultdict(list))
    for f in d.rglob("*counter_collection.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "")
                out[short(k)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return out


def load_durations(d: Path):
    dur = defaultdict(list)
    for f in d.rglob("*kernel_trace.csv"):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                dur[short(row["Kernel_Name"])].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return dur


def main():
    root = Path(sys.argv[1])
    counters = defaultdict(dict)
    for sub in root.iterdir():
        if sub.is_dir():
            for k, cs in load_counters(sub).items():
                for c, v in cs.items():
                    counters[k][c] = sum(v) / len(v)
    durs = load_durations(root / "trace") if (root / "trace").exists() else {}
    res = {}
    for k, cs in counters.items():
        if "spmv" not in k and "long" not in k:
            continue
        r = dict(cs)
        if k in durs and durs[k]:
            t = sum(durs[k]) / len(durs[k])
            r["duration_ns_mean"] = t
            if "GRBM_GUI_ACTIVE" in cs:
                r["eff_clock_GHz"] = cs["GRBM_GUI_ACTIVE"] / 8 / t
        if "FETCH_SIZE" in cs:
            r["read_bytes_corrected"] = 2 * cs["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in cs:
            r["write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            r["hbm_traffic_bytes"] = r["read_bytes_corrected"] + r["write_bytes"]
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs:
            tot = cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]
            r["l2_hit_rate"] = cs["TCC_HIT_sum"] / tot if tot else None
        if cs.get("SQ_WAVE_CYCLES"):
            if "SQ_WAIT_ANY" in cs:
                r["sq_wait_frac"] = cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"]
            if "SQ_ACTIVE_INST_ANY" in cs:
                r["sq_active_inst_frac"] = cs["SQ_ACTIVE_INST_ANY"] / cs["SQ_WAVE_CYCLES"]
        if cs.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in cs:
            r["lds_bank_conflict_frac"] = cs["SQ_LDS_BANK_CONFLICT"] / cs["SQ_LDS_IDX_ACTIVE"]
        if "TCC_EA0_RDREQ_sum" in cs:
            r["ea_rd_bytes_64B"] = cs["TCC_EA0_RDREQ_sum"] * 64
        res[k] = r
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
