#!/usr/bin/env python3
"""LDS lookup microbenchmark (zdbcrc_debug_lds_bench): wave-instructions of
ds_read per CU-cycle for 5-bit table lookups with 1 or 2 VALU ops of index
extraction, b32 vs b64, at 24 waves/CU.  Clock assumed 2.3 GHz (report ns too)."""
import ctypes as C, json, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "0-db_amd")]
# the diagnostic build: A/B variants and zdbcrc_debug_* hooks (not in libzdbcrc.so)
import os as _os
_os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
import torch, zdbcrc
f = zdbcrc._lib.zdbcrc_debug_lds_bench
f.restype = C.c_float
f.argtypes = [C.c_int, C.c_uint32, C.c_void_p, C.c_int, C.c_void_p]
sink = torch.zeros(16, dtype=torch.int32, device="cuda")
cus = torch.cuda.get_device_properties(0).multi_processor_count
st = torch.cuda.current_stream().cuda_stream
iters = 4000
for _ in range(20):
    f(0, iters, sink.data_ptr(), cus, st)
for mode in (0, 1, 2, 3, 0):
    ts = [f(mode, iters, sink.data_ptr(), cus, st) for _ in range(7)][2:]
    ms = float(np.median(ts))
    instr_per_cu = 24 * iters * 16
    ns = ms * 1e6 / instr_per_cu
    print(json.dumps({"mode": ["b32_v1", "b32_v2", "b64_v1", "b64_v2"][mode], "ms": round(ms, 4),
                      "ns_per_lds_instr_per_cu": round(ns, 4), "cycles_at_2.3GHz": round(ns * 2.3, 3)}), flush=True)
