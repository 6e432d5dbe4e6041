#!/usr/bin/env python3
"""Where the f3 walk's time goes (diagnostic library): per-chunk
s_memrealtime stamps (100 MHz) of the fused search + chain kernel on the C4
shard of rank 0 -- launch skew, search time, chain time, window loads --
per chunk size and chain window (args: chunk_bytes:wb ...)."""
import ctypes as C, json, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import numpy as np, torch, zdbcrc, bench

lib = C.CDLL(os.environ["ZDBCRC_LIB"])
lib.zdbcrc_debug_set_chain_wb.argtypes = [C.c_int]
lib.zdbcrc_debug_walk_stamps.argtypes = [C.c_void_p, C.c_uint64]
lib.zdbcrc_debug_walk_stamps.restype = C.c_uint64
lay = bench.c4_layout(0)
n = len(lay["lens"])
img, d_poff, d_len, expected, crcs = bench.c4_build_device(lay, bench.C4_SEED)
st = zdbcrc.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 1024)
cases = sys.argv[1:] or ["8388608:0", "8388608:2048", "4194304:2048", "16777216:2048"]
buf = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")


def pct(a, qs=(50, 90, 99, 100)):
    return {f"p{q}": round(float(np.percentile(a, q)), 1) for q in qs}


for case in cases:
    cb, wb = (int(x) for x in case.split(":"))
    assert lib.zdbcrc_debug_set_chain_wb(wb) == 0
    assert st.scan(cb) == n
    for _ in range(3):
        st.walk(cb)
    torch.cuda.synchronize()
    lib.zdbcrc_debug_walk_stamps(buf.data_ptr(), buf.numel() // 4)
    st.walk(cb)
    torch.cuda.synchronize()
    used = lib.zdbcrc_debug_walk_stamps(None, 0)
    s = buf[: 4 * used].view(-1, 4).cpu().numpy().astype(np.int64)
    if os.environ.get("WALK_STAMPS_DUMP"):
        np.save(Path(os.environ["WALK_STAMPS_DUMP"]) / f"stamps_{cb}_{wb}.npy", s)
    t0, t1, t2, loads = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
    base = t0.min()
    us = lambda x: x / 100.0  # 100 MHz ticks -> us
    search, chain = us(t1 - t0), us(t2 - t1)
    crit = int(np.argmax(t2))
    per_load = chain[loads > 0] / loads[loads > 0]
    print(json.dumps({
        "chunk_bytes": cb, "chain_wb": wb, "chunks": int(used), "kernel_span_us": round(us(t2.max() - base), 1),
        "launch_skew_us": pct(us(t0 - base)), "search_us": pct(search), "chain_us": pct(chain),
        "loads": pct(loads), "us_per_load": pct(per_load),
        "critical": {"chunk": crit, "start_us": round(us(t0[crit] - base), 1), "search_us": round(search[crit], 1),
                     "chain_us": round(chain[crit], 1), "loads": int(loads[crit])},
        "search_done_by_us": round(us(t1.max() - base), 1)}), flush=True)
