#!/usr/bin/env python3
"""f3 walk on a store of small values (C2u-like: 4 KiB payloads behind 26-byte
headers+keys, 16 x 256 MiB datafiles): walk and scan time per chunk size --
the chain of a chunk has one dependent hop per record, so a chunk size made
for C4's Zipf mix (8 MiB, ~170 records) is ~2,000 hops here."""
import json, sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import numpy as np, torch, zdbcrc, bench

val = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
files, cap = 16, bench.C4_FILE_CAP
per = (cap - bench.FILE_HDR) // (bench.ENTRY_HDR + bench.C4_KEY + val)
n = per * files
lens = np.full(n, val, np.int64)
ent = bench.ENTRY_HDR + bench.C4_KEY + lens
file_of = np.repeat(np.arange(files), per)
rel = bench.FILE_HDR + (np.arange(n) % per) * (bench.ENTRY_HDR + bench.C4_KEY + val)
fsize = np.full(files, bench.FILE_HDR + per * (bench.ENTRY_HDR + bench.C4_KEY + val), np.int64)
file_off = np.concatenate([[0], np.cumsum(fsize[:-1])])
prev = np.where(np.arange(n) % per == 0, 0, rel - (bench.ENTRY_HDR + bench.C4_KEY + val))
entry_off = file_off[file_of] + rel
lay = {"lens": lens, "entry_off": entry_off, "payload_off": entry_off + bench.ENTRY_HDR + bench.C4_KEY, "prev": prev,
       "file_of": file_of, "file_off": file_off, "file_size": fsize, "total": int(file_off[-1] + fsize[-1])}
img, d_poff, d_len, expected, crcs = bench.c4_build_device(lay, bench.C4_SEED)
st = zdbcrc.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 1024)
chunks = [int(x) for x in sys.argv[2:]] or [8 << 20, 2 << 20, 1 << 20, 512 << 10, 256 << 10, 128 << 10, 0]
for c in chunks:
    assert st.scan(c) == n
    assert int(st.mismatch_count.item()) == 0
    for _ in range(2):
        st.walk(c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        st.walk(c)
    e1.record()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        st.scan(c)
    torch.cuda.synchronize()
    print(json.dumps({"value_bytes": val, "records": n, "chunk_bytes": c, "walk_ms": round(e0.elapsed_time(e1) / 5, 3),
                      "scan_ms": round((time.perf_counter() - t0) / 5 * 1e3, 3),
                      "rewalks": int(st.rewalks[-1].item())}), flush=True)
