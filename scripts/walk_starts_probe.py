#!/usr/bin/env python3
"""Debug probe: chunks whose speculative start (search) differs from the
true start, for the search variant in ZDBCRC_SEARCH_VARIANT (diag library)."""
import ctypes as C, json, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd/lib/libzdbcrc_diag.so"))
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import numpy as np, torch, zdbcrc, bench

lib = zdbcrc._lib
lib.zdbcrc_debug_walk_starts.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64]
lay = bench.c4_layout(0)
n = len(lay["lens"])
img, _, _, _, _ = bench.c4_build_device(lay, bench.C4_SEED)
st = zdbcrc.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 1024)
chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
st.walk(chunk)
torch.cuda.synchronize()
cpf = -(-int(lay["file_size"].max()) // chunk)
nch = cpf * len(lay["file_off"])
s0 = np.zeros(nch, np.uint64)
t0 = np.zeros(nch, np.uint64)
assert lib.zdbcrc_debug_walk_starts(s0.ctypes.data, t0.ctypes.data, nch) == 0
NONE = np.uint64(2**64 - 1)
bad = [w for w in range(nch) if t0[w] != NONE and s0[w] != t0[w]]
out = []
for w in bad[:20]:
    c0 = (w % cpf) * chunk
    s, t = int(s0[w]), int(t0[w])
    out.append({"chunk": w, "c0": c0, "spec": None if s0[w] == NONE else s - c0, "true": t - c0,
                "true_mod_16K": (t - c0) % 16384, "true_mod_1K": (t - c0) % 1024})
print(json.dumps({"variant": os.environ.get("ZDBCRC_SEARCH_VARIANT"), "chunks": nch, "bad": len(bad),
                  "rewalks": int(st.rewalks[-1].item()), "first": out}, indent=1))
