#!/usr/bin/env python3
"""Per-wave start/end spread of the checksum kernel (diagnostic STAMP variant):
is the kernel's end set by a tail of slow waves?"""
import ctypes as C, json, sys, time
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "0-db_amd")]
# the diagnostic build: A/B variants and zdbcrc_debug_* hooks (not in libzdbcrc.so)
import os as _os
_os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
import torch, zdbcrc
sv = zdbcrc._lib.zdbcrc_debug_set_variant; sv.restype = C.c_char_p; sv.argtypes = [C.c_int]
rd = zdbcrc._lib.zdbcrc_debug_read_stamps; rd.restype = C.c_int; rd.argtypes = [C.c_void_p, C.c_size_t]
vname = sys.argv[2] if len(sys.argv) > 2 else "v3_wg768_prio_nt_stamp"
idx = [i for i in range(64) if sv(i) and sv(i).decode() == vname][0]
sv(idx)
for label in sys.argv[1].split(","):
    wl, size = label, 4 << 30
    if "@" in wl:
        wl, mib = wl.split("@")
        size = int(mib) << 20
    if wl == "zipf":
        lens = zdbcrc.zipf_lengths(size, 0xC3C3C3).astype(np.int64)
    elif wl == "fixed4k":
        lens = np.full(size >> 12, 4096, np.int64)
    else:
        lens = np.array([size - 16], np.int64)
    offs = np.zeros(len(lens), np.int64); offs[1:] = np.cumsum(lens[:-1])
    arena = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    zdbcrc.synth_fill_device(arena, 1)
    do, dl = torch.from_numpy(offs).cuda(), torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    t_end = time.time() + 1.0  # ~1 s of back-to-back work first: clocks settle
    while time.time() < t_end:
        for _ in range(8):
            zdbcrc.batch_device(arena, do, dl, out)
        torch.cuda.synchronize()
    # back-to-back launches (steady clocks); the stamps are the last launch's
    zdbcrc.kernel_stats(); zdbcrc.set_timing(True)
    for _ in range(8):
        zdbcrc.batch_device(arena, do, dl, out)
    torch.cuda.synchronize(); zdbcrc.set_timing(False)
    kms, nl = zdbcrc.kernel_stats()
    kms /= nl
    print(json.dumps({"workload": label, "variant": vname, "kernel_ms_event": round(kms, 4)}))
    waves = 256 * 2 * 12
    st = np.zeros(waves * 4, np.uint64)
    assert rd(st.ctypes.data, waves) == 0
    st = st.reshape(-1, 4).astype(np.int64)
    gw = np.arange(waves)[st[:, 1] > 0]
    st = st[st[:, 1] > 0]
    hw, xcc = st[:, 2], st[:, 3] & 0xF
    cu = (hw >> 8) & 0xF; sh = (hw >> 12) & 1; se = (hw >> 13) & 0x7; simd = (hw >> 4) & 3
    cukey = xcc * 1000 + se * 100 + sh * 16 + cu
    t0 = st[:, 0].min()
    s_, e_ = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0  # memrealtime = 100 MHz -> us
    dur = e_ - s_
    block = gw // 12
    per_cu = {}
    for k, e in zip(cukey, e_):
        per_cu.setdefault(int(k), []).append(e)
    cu_mean = np.array([np.mean(v) for v in per_cu.values()])
    cu_spread = np.array([np.max(v) - np.min(v) for v in per_cu.values()])
    per_x = {int(x): round(float(np.mean(e_[xcc == x])), 1) for x in np.unique(xcc)}
    wgs = {}
    for b, e in zip(block, e_):
        wgs.setdefault(int(b), []).append(e)
    wg_spread = np.array([np.max(v) - np.min(v) for v in wgs.values()])
    wg_mean = {b: np.mean(v) for b, v in wgs.items()}
    # the two workgroups sharing a CU: difference of their mean end times
    cu_wgs = {}
    for b, k in zip(block, cukey):
        cu_wgs.setdefault(int(k), set()).add(int(b))
    pair_gap = np.array([abs(wg_mean[min(v)] - wg_mean[max(v)]) for v in cu_wgs.values() if len(v) == 2])
    print(json.dumps({"within_wg_spread_us_p50_max": [round(float(np.median(wg_spread)), 1), round(float(wg_spread.max()), 1)],
                      "wg_pair_mean_gap_us_p50_max": [round(float(np.median(pair_gap)), 1) if len(pair_gap) else None,
                                                      round(float(pair_gap.max()), 1) if len(pair_gap) else None]}))
    per_simd_rank = {}
    print(json.dumps({"cus": len(per_cu), "waves_per_cu": round(len(st) / max(len(per_cu), 1), 1),
                      "cu_mean_end_us_min_p50_max": [round(float(x), 1) for x in (cu_mean.min(), np.median(cu_mean), cu_mean.max())],
                      "within_cu_spread_us_p50_max": [round(float(np.median(cu_spread)), 1), round(float(cu_spread.max()), 1)],
                      "xcd_mean_end_us": per_x}))
    print(json.dumps({"workload": label, "waves": len(st), "start_us_p50_max": [round(float(np.median(s_)), 1), round(float(s_.max()), 1)],
                      "end_us_p10_p50_p90_max": [round(float(np.percentile(e_, q)), 1) for q in (10, 50, 90, 100)],
                      "dur_us_min_p50_max": [round(float(dur.min()), 1), round(float(np.median(dur)), 1), round(float(dur.max()), 1)]}))
    del arena
    slow = np.argsort(dur)[-8:][::-1]
    print(json.dumps({"workload": label, "slowest_waves": [[int(gw[i]), round(float(s_[i]), 1), round(float(dur[i]), 1)]
                                                             for i in slow]}))
