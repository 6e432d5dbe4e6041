#!/usr/bin/env python3
"""Per-wave start/end spread of the checksum kernel (diagnostic STAMP variant):
is the kernel's end set by a tail of slow waves?"""
import ctypes as C, json, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "0-db_amd")]
import torch, zdbcrc
sv = zdbcrc._lib.zdbcrc_debug_set_variant; sv.restype = C.c_char_p; sv.argtypes = [C.c_int]
rd = zdbcrc._lib.zdbcrc_debug_read_stamps; rd.restype = C.c_int; rd.argtypes = [C.c_void_p, C.c_size_t]
idx = [i for i in range(20) if sv(i) and sv(i).decode() == "v3_wg768_stamp"][0]
sv(idx)
for wl in sys.argv[1].split(","):
    if wl == "zipf":
        lens = zdbcrc.zipf_lengths(4 << 30, 0xC3C3C3).astype(np.int64)
    elif wl == "fixed4k":
        lens = np.full(1 << 20, 4096, np.int64)
    else:
        lens = np.array([(4 << 30) - 16], np.int64)
    offs = np.zeros(len(lens), np.int64); offs[1:] = np.cumsum(lens[:-1])
    arena = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device="cuda")
    zdbcrc.synth_fill_device(arena, 1)
    do, dl = torch.from_numpy(offs).cuda(), torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    for _ in range(4):
        zdbcrc.batch_device(arena, do, dl, out)
    torch.cuda.synchronize()
    waves = 256 * 2 * 12
    st = np.zeros(waves * 2, np.uint64)
    assert rd(st.ctypes.data, waves) == 0
    st = st.reshape(-1, 2).astype(np.int64)
    st = st[st[:, 1] > 0]
    t0 = st[:, 0].min()
    s_, e_ = (st[:, 0] - t0) / 100.0, (st[:, 1] - t0) / 100.0  # memrealtime = 100 MHz -> us
    dur = e_ - s_
    print(json.dumps({"workload": wl, "waves": len(st), "start_us_p50_max": [round(float(np.median(s_)), 1), round(float(s_.max()), 1)],
                      "end_us_p10_p50_p90_max": [round(float(np.percentile(e_, q)), 1) for q in (10, 50, 90, 100)],
                      "dur_us_min_p50_max": [round(float(dur.min()), 1), round(float(np.median(dur)), 1), round(float(dur.max()), 1)]}))
    del arena
