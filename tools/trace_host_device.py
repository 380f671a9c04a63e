#!/usr/bin/env python3
"""Host enqueue time vs device busy time per CG iteration from a rocprofv3
kernel + HIP API trace of tools/graph_probe.py.

Each solve is the window from its k_init launch call to the end of its
k_final_x kernel. Host time = the summed duration of the process's HIP API
calls in the window that enqueue work (polls and waits — hipEventQuery,
hipStreamSynchronize, hipEventSynchronize — excluded); device time = the
union of the kernel intervals in the window. Both divided by the solve's
iterations (--its). One JSON line per solve.

    python tools/trace_host_device.py DIR --its 160
"""
import argparse
import csv
import json
from pathlib import Path

WAITS = {"hipEventQuery", "hipStreamSynchronize", "hipEventSynchronize", "hipDeviceSynchronize",
         "hipStreamQuery"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--its", type=int, required=True)
    a = ap.parse_args()
    d = Path(a.dir)
    api = list(csv.DictReader(open(next(d.rglob("*hip_api_trace.csv")))))
    ker = list(csv.DictReader(open(next(d.rglob("*kernel_trace.csv")))))
    by_corr = {r["Correlation_Id"]: r for r in api}
    inits = [k for k in ker if "k_init" in k["Kernel_Name"] and "gamg" not in k["Kernel_Name"]]
    finals = [k for k in ker if "k_final_x" in k["Kernel_Name"]]
    inits.sort(key=lambda k: int(k["Start_Timestamp"]))
    finals.sort(key=lambda k: int(k["Start_Timestamp"]))
    for n, (ki, kf) in enumerate(zip(inits, finals)):
        call = by_corr.get(ki["Correlation_Id"])
        t0 = int(call["Start_Timestamp"]) if call else int(ki["Start_Timestamp"])
        t1 = int(kf["End_Timestamp"])
        host = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in api
                   if t0 <= int(r["Start_Timestamp"]) < t1 and r["Function"] not in WAITS
                   and not r["Function"].startswith("__hip"))
        graphs = sum(1 for r in api if t0 <= int(r["Start_Timestamp"]) < t1 and r["Function"] == "hipGraphLaunch")
        iv = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"])) for k in ker
                    if t0 <= int(k["Start_Timestamp"]) < t1)
        busy, cur0, cur1 = 0, None, None
        for s, e in iv:
            if cur1 is None or s > cur1:
                if cur1 is not None:
                    busy += cur1 - cur0
                cur0, cur1 = s, e
            else:
                cur1 = max(cur1, e)
        if cur1 is not None:
            busy += cur1 - cur0
        print(json.dumps({"solve": n, "graph_launches": graphs, "window_us": round((t1 - t0) / 1e3, 1),
                          "host_api_us_per_iter": round(host / 1e3 / a.its, 2),
                          "device_busy_us_per_iter": round(busy / 1e3 / a.its, 2),
                          "kernels": len(iv)}))


if __name__ == "__main__":
    main()
