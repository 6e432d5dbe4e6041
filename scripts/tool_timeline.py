#!/usr/bin/env python3
"""f1 ingest timeline: the integrity-check tool on 8 and 32 copies of a
256 MiB datafile (65,000 x 4 KiB values, as bench.py's e2e leg) per engine,
wall time and the tool's ZDBCRC_TOOL_TRACE lines (process-relative times)."""
import json, os, subprocess, sys, tempfile, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import numpy as np, zdbcrc

n = 65000
vals = zdbcrc.synth_fill(n * 4096, 0xC1)
vo = np.arange(n, dtype=np.uint64) * 4096
vl = np.full(n, 4096, np.uint32)
crcs = np.array([zdbcrc.crc32(vals[i * 4096:(i + 1) * 4096]) for i in range(n)], np.uint32)
keys = [b"k%d" % i for i in range(n)]
body, _, _ = zdbcrc.encode_batch(keys, vals, vo, vl, crcs, file_offset=28)
tool = str(ROOT / "0-db_amd/bin/zdb-integrity-check")
with tempfile.TemporaryDirectory() as td:
    with open(f"{td}/d0", "wb") as f:
        f.write(zdbcrc.encode_header(0) + body)
    files = []
    for i in range(8):
        d = f"{td}/ns{i}"
        os.mkdir(d)
        os.link(f"{td}/d0", f"{d}/d0")
        os.symlink("d0", f"{d}/zdb-data-0")
        files.append(f"{d}/zdb-data-0")
    fb = 28 + len(body)
    for nf in (8, 32):
        fl = (files * 4)[:nf]
        for eng in sys.argv[1:] or ["hip", "auto", "cpu"]:
          for pin in (("1", "0") if eng == "hip" else ("1",)):
            walls, runs = [], []
            for rep in range(5):
                t0 = time.perf_counter()
                p = subprocess.run([tool, f"--engine={eng}", "--jobs=8"] + fl, stdout=subprocess.DEVNULL,
                                   stderr=subprocess.PIPE, env=dict(os.environ, ZDBCRC_TOOL_TRACE="1",
                                                                    ZDBCRC_TOOL_PIN=pin), timeout=300)
                walls.append(time.perf_counter() - t0)
                assert p.returncode == 0, p.stderr[-400:]
                su = [ln for ln in p.stderr.decode().splitlines() if ln.startswith("[trace] GPU start-up")]
                if su:  # process-relative: GPU up, reports done; the rest of the wall time is process exit
                    import re
                    up = float(re.search(r"up at ([\d.]+) ms", su[0]).group(1))
                    done = float(re.search(r"reports done at ([\d.]+) ms", su[0]).group(1))
                    runs.append({"wall_ms": round(walls[-1] * 1e3, 1), "gpu_up_ms": up, "reports_done_ms": done,
                                 "after_reports_ms": round(walls[-1] * 1e3 - done, 1)})
            tr = [ln for ln in p.stderr.decode().splitlines() if ln.startswith("[trace]")]
            print(json.dumps({"files": nf, "engine": eng, "pin": pin, "wall_s": [round(w, 4) for w in walls],
                              "gibs_best": round(nf * fb / min(walls) / 2**30, 2), "runs": runs,
                              "trace_last_run": [ln.replace(td, "") for ln in tr if "payloads" not in ln]}), flush=True)
