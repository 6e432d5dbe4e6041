#!/usr/bin/env python3
"""Debug probe: the failing 2^28+1-piece record under the segment-dump
variant of the default kernel (diagnostic library): every wave's segment
(pa, pb, value) against the value its bytes should contribute."""
import ctypes as C, json, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
os.environ["ZDBCRC_LIB"] = str(ROOT / "0-db_amd/lib/libzdbcrc_diag.so")
sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
import numpy as np, torch, zdbcrc

lib = zdbcrc._lib
lib.zdbcrc_debug_set_variant.restype = C.c_char_p
lib.zdbcrc_debug_set_variant.argtypes = [C.c_int]
lib.zdbcrc_debug_read_stamps.argtypes = [C.c_void_p, C.c_size_t]
print(lib.zdbcrc_debug_set_variant(int(sys.argv[1]) if len(sys.argv) > 1 else 29), flush=True)
SEED = 0x5A0DB5EED + 9
total = (1 << 32) + 4096
host = zdbcrc.synth_fill(total, SEED)
arena = torch.from_numpy(host).cuda()
OFF = int(sys.argv[2]) if len(sys.argv) > 2 else 100
L = (1 << 32) - 1
o = torch.tensor([OFF], dtype=torch.int64, device="cuda")
l = torch.tensor([np.uint32(L).view(np.int32)], dtype=torch.int32, device="cuda")
out = torch.zeros(1, dtype=torch.int32, device="cuda")
zdbcrc.batch_device(arena, o, l, out)
torch.cuda.synchronize()
got = int(out.cpu().numpy().view(np.uint32)[0])
waves = 6144
st = np.zeros(waves * 4, np.uint64)
assert lib.zdbcrc_debug_read_stamps(st.ctypes.data, waves) == 0
st = st.reshape(waves, 4)
A = OFF
Aend = OFF + L
P0 = A & ~15
want_total = zdbcrc.crc32(host[A:Aend])
acc, bad = 0, []
for gw in range(waves):
    pa, pb, x, rn = (int(v) for v in st[gw])
    if pb == 0 and x == 0:
        continue
    lo = max(A, P0 + 16 * pa)
    hi = min(Aend, P0 + 16 * pb)
    e = zdbcrc._shift(zdbcrc.crc32(host[lo:hi]), Aend - hi)
    acc ^= x
    if e != x:
        bad.append({"wave": gw, "pa": pa, "pb": pb, "np": rn >> 32, "x": f"{x:08x}", "expected": f"{e:08x}"})
print(json.dumps({"got": f"{got:08x}", "want": f"{want_total:08x}", "xor_of_dumped": f"{acc:08x}",
                  "bad_segments": bad[:4] + bad[-4:], "n_bad": len(bad)}, indent=1), flush=True)
np.save(str(ROOT / "gpurun_out" / "segdump_raw.npy"), st)
