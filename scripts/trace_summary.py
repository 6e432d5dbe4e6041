#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run of bench.py: per-kernel average
over the LAST `steps` dispatches (bench.py's timed region; earlier dispatches
are the parity run, warmup and clock-settle steps) next to the all-dispatch
average.  usage: trace_summary.py <run_kernel_trace.csv> <steps>"""
import csv, json, sys
from collections import defaultdict

path, steps = sys.argv[1], int(sys.argv[2])
rows = defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    short = ("crc_batch_kernel" if "crc_batch_kernel" in name else "plan_kernel" if "plan_kernel" in name else
             "rocprim_scan" if "trampoline_kernel" in name else
             "rocprim_scan_init" if "init_lookback" in name else name.split("(")[0][-48:])
    rows[short].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
out = {}
for k, v in rows.items():
    v.sort()
    d_all = [x[1] for x in v]
    d_last = d_all[-steps:]
    out[k] = {"dispatches": len(v), "avg_us_all": round(sum(d_all) / len(d_all) / 1e3, 2),
              "avg_us_timed": round(sum(d_last) / len(d_last) / 1e3, 2),
              "min_us_timed": round(min(d_last) / 1e3, 2), "max_us_timed": round(max(d_last) / 1e3, 2)}
print(json.dumps(out, indent=1))
