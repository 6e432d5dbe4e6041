#!/usr/bin/env python3
"""f3 search filter throughput without the search loop (diagnostic library):
every wave scans its own slice of the C4 image with scan_block -- full
filter (0), loads only (1), two-pass filter (2), full filter + a barrier per
block (3), full filter in 4 KiB blocks (4) -- at full occupancy; GB/s."""
import ctypes as C, json, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import torch, zdbcrc, bench

lib = C.CDLL(os.environ["ZDBCRC_LIB"])
lib.zdbcrc_debug_search_rate.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint64, C.c_uint32]
lib.zdbcrc_debug_search_rate.restype = C.c_float
lay = bench.c4_layout(0)
img, d_poff, d_len, expected, crcs = bench.c4_build_device(lay, bench.C4_SEED)
L = img.numel() - 64
for grid in (1536, 3072):
    per_wave = (L - 8192) // (grid * 4) // 8192 * 8192
    for mode in (1, 0, 5, 2, 3, 4, 1, 0, 5):
        ms = [lib.zdbcrc_debug_search_rate(img.data_ptr(), L, mode, per_wave, grid) for _ in range(3)]
        b = per_wave * grid * 4
        print(json.dumps({"grid": grid, "mode": mode, "ms": round(min(ms), 3), "GBs": round(b / min(ms) / 1e6, 1)}),
              flush=True)
