#!/usr/bin/env python3
"""Per-kernel effective clock from scripts/clock_pmc.sh: GRBM_GUI_ACTIVE / 8
(XCDs) / dispatch duration, averaged over the dispatches of each kernel."""
import csv, json, sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
pmc = defaultdict(dict)
for f in root.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        pmc[r["Dispatch_Id"]][r["Counter_Name"]] = pmc[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        pmc[r["Dispatch_Id"]]["name"] = r["Kernel_Name"]
dur = {}
for f in root.rglob("*kernel_trace.csv"):
    for r in csv.DictReader(open(f)):
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9
agg = defaultdict(list)
for d, v in pmc.items():
    if d in dur and "GRBM_GUI_ACTIVE" in v and dur[d] > 1e-4:
        short = v["name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][-70:]
        agg[short].append((v["GRBM_GUI_ACTIVE"] / 8 / dur[d] / 1e9, dur[d] * 1e3))
print(json.dumps({k: {"dispatches": len(x), "ghz_mean": round(sum(a for a, _ in x) / len(x), 3),
                      "ms_mean": round(sum(b for _, b in x) / len(x), 4)} for k, x in agg.items()}, indent=1))
