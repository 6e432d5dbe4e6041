#!/usr/bin/env python3
"""Per-launch kernel time over a long back-to-back run (C3 batch): does the
kernel speed drift with sustained load (clock ramp / power limit)?
Prints windows of 50 launches: median / min / max ms."""
import ctypes as C, json, subprocess, sys, time
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "0-db_amd")]
# the diagnostic build: A/B variants and zdbcrc_debug_* hooks (not in libzdbcrc.so)
import os as _os
_os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
import torch, zdbcrc

kt = zdbcrc._lib.zdbcrc_debug_kernel_times
kt.restype = C.c_long
kt.argtypes = [C.c_void_p, C.c_size_t]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
gap_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
lens = zdbcrc.zipf_lengths(4 << 30, 0xC3C3C3).astype(np.int64)
offs = np.zeros(len(lens), np.int64); offs[1:] = np.cumsum(lens[:-1])
arena = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
zdbcrc.synth_fill_device(arena, 7)
do, dl = torch.from_numpy(offs).cuda(), torch.from_numpy(lens.astype(np.int32)).cuda()
out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
times = np.zeros(N, np.float32)
zdbcrc.set_timing(True)
t0 = time.time()
for i in range(N):
    zdbcrc.batch_device(arena, do, dl, out)
    if gap_ms:
        torch.cuda.synchronize(); time.sleep(gap_ms / 1e3)
    if i % 100 == 99:
        torch.cuda.synchronize()
torch.cuda.synchronize()
wall = time.time() - t0
zdbcrc.set_timing(False)
k = kt(times.ctypes.data, N)
for w in range(0, k, 50):
    t = times[w:w + 50]
    print(json.dumps({"launch": w, "median_ms": round(float(np.median(t)), 4), "min_ms": round(float(t.min()), 4),
                      "max_ms": round(float(t.max()), 4)}))
print(json.dumps({"launches": int(k), "wall_s": round(wall, 2), "gap_ms": gap_ms,
                  "overall_median_ms": round(float(np.median(times[:k])), 4)}))
