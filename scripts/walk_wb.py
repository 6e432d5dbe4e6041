#!/usr/bin/env python3
"""A/B of the f3 chain window (diagnostic library: zdbcrc_debug_set_chain_wb)
on the C4 shard of rank 0: walk alone and full scan per window size,
interleaved rounds in one process; records and exits must not change."""
import ctypes as C, json, os, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import torch, zdbcrc, bench

lib = C.CDLL(os.environ["ZDBCRC_LIB"])
lib.zdbcrc_debug_set_chain_wb.argtypes = [C.c_int]
lay = bench.c4_layout(0)
n = len(lay["lens"])
img, d_poff, d_len, expected, crcs = bench.c4_build_device(lay, bench.C4_SEED)
st = zdbcrc.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 1024)
wbs = [int(x) for x in sys.argv[1:]] or [0, 1024, 2048, 4096, 8192]
ref = None
res = {w: {"walk": [], "scan": []} for w in wbs}
for rnd in range(4):
    for w in wbs:
        assert lib.zdbcrc_debug_set_chain_wb(w) == 0
        assert st.scan() == n
        desc = torch.stack([st.payload_off[:n], st.payload_len[:n].to(torch.int64)]).cpu() if rnd == 0 else None
        if desc is not None:
            if ref is None:
                ref = desc
            assert torch.equal(desc, ref), w
        for _ in range(3):
            st.walk()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            st.walk()
        e1.record()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            st.scan()
        torch.cuda.synchronize()
        res[w]["walk"].append(e0.elapsed_time(e1) / 10)
        res[w]["scan"].append((time.perf_counter() - t0) / 10 * 1e3)
        assert int(st.rewalks[-1].item()) == 0 and int(st.mismatch_count.item()) == 0
for w in wbs:
    wk, sc = sorted(res[w]["walk"]), sorted(res[w]["scan"])
    print(json.dumps({"chain_wb": w, "walk_ms_median": round(wk[len(wk) // 2], 4), "walk_ms_min": round(wk[0], 4),
                      "scan_ms_median": round(sc[len(sc) // 2], 4), "same_records": True}), flush=True)
