#!/usr/bin/env python3
"""f3 walk timing on the C4 shard of rank 0 (64 x 256 MiB datafiles in HBM):
walk alone and the full scan per chunk size (HIP events via torch on the
current stream, which is the stream the library launches on)."""
import json, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import torch, zdbcrc, bench

lay = bench.c4_layout(0)
n = len(lay["lens"])
img, d_poff, d_len, expected, crcs = bench.c4_build_device(lay, bench.C4_SEED)
st = zdbcrc.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 1024)
chunks = [int(x) for x in sys.argv[1:]] or [1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20]
res = {}
for c in chunks:
    assert st.scan(c) == n
    for _ in range(3):
        st.walk(c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        st.walk(c)
    e1.record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        st.scan(c)
    torch.cuda.synchronize()
    res[c] = {"walk_ms": e0.elapsed_time(e1) / 10, "scan_ms": (time.perf_counter() - t0) / 10 * 1e3,
              "rewalks": int(st.rewalks[-1].item()), "mismatches": int(st.mismatch_count.item())}
    print(json.dumps({c: res[c]}), flush=True)
