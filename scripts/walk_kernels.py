#!/usr/bin/env python3
"""Per-kernel median durations of the f3 walk from a rocprofv3 kernel trace
of scripts/walk_probe.py, grouped by chunk size (the search kernel's grid =
one workgroup of 256 threads per chunk)."""
import collections, csv, json, sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
seq = []
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]
    seq.append((n, int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"])))
seq.sort(key=lambda x: x[1])
cur, d = None, collections.defaultdict(list)
for name, s, e, g in seq:
    if name == "walk_search_kernel":
        cur = g // 256
    if cur and (name.startswith("walk") or name in ("crc_batch_kernel_v3", "plan_kernel", "verify_kernel")):
        d[(cur, name)].append((e - s) / 1e3)
out = collections.defaultdict(dict)
for (nch, name), v in sorted(d.items()):
    out[f"{nch}_chunks"][name] = {"calls": len(v), "median_us": round(float(np.median(v)), 1)}
print(json.dumps(out, indent=1))
