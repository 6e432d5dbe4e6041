#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in ONE process (rule 24): for each
round, every variant runs STEPS batches of the same device-resident dataset;
reports median/min kernel ms per variant and checks each variant's output
against variant 0 bit for bit."""
import ctypes as C, json, os, sys, time
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "0-db_amd")]
# the diagnostic build: A/B variants and zdbcrc_debug_* hooks (not in libzdbcrc.so)
import os as _os
_os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
import torch, zdbcrc
sys.path.insert(0, str(ROOT))
import bench

set_variant_raw = zdbcrc._lib.zdbcrc_debug_set_variant
set_variant_raw.restype = C.c_char_p
set_variant_raw.argtypes = [C.c_int]
set_split = zdbcrc._lib.zdbcrc_debug_set_split
set_split.argtypes = [C.c_uint32]
_small_stats = zdbcrc._lib.zdbcrc_debug_small_kernel_stats
_small_stats.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_uint64)]


def small_kernel_stats():
    ms, k = C.c_double(0), C.c_uint64(0)
    _small_stats(C.byref(ms), C.byref(k))
    return ms.value, k.value
set_variant = set_variant_raw
names = []
i = 0
while True:
    n = set_variant(i)
    if not n:
        break
    names.append(n.decode()); i += 1
probe = zdbcrc._lib.zdbcrc_debug_stream_read
probe.restype = C.c_float
probe.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_int, C.c_void_p]
sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for mib in [int(x) for x in os.environ.get("PROBE_MIB", "4096").split(",") if x]:
    buf = torch.empty(mib << 20, dtype=torch.uint8, device="cuda"); buf.fill_(7)
    for spec in [x for x in os.environ.get("PROBE_BLOCKS", "2048,8192,16384,-4,-8,-16").split(",") if x and x != "none"]:
        # "<blocks>@<misalign>": the same probe over a base address misaligned by that many bytes
        blocks, mis = (int(x) for x in spec.split("@")) if "@" in spec else (int(spec), 0)
        ts = [probe(buf.data_ptr() + mis, buf.numel() - 64, sink.data_ptr(), blocks, st) for _ in range(6)][1:]
        print(json.dumps({"probe": "stream_read_%dMiB" % mib, "blocks": blocks, "misalign": mis,
                          "median_ms": round(float(np.median(ts)), 4),
                          "tbs": round(buf.numel() / (np.median(ts) / 1e3) / 1e12, 3)}), flush=True)
    del buf
# a variant spec is "<index>" or "<index>s<bytes>": the kernel variant, and
# unbounded batches split at that many bytes (small records to the packed
# kernel; the time reported is then both kernels' sum)
specs = sys.argv[2].split(",") if len(sys.argv) > 2 else [str(i) for i in range(len(names))]
sel = list(range(len(specs)))
vidx = [int(x.split("s")[0]) for x in specs]
vsplit = [int(x.split("s")[1]) if "s" in x else 0 for x in specs]
vname = [names[vidx[i]] + (f"+split{vsplit[i]}" if vsplit[i] else "") for i in sel]


def set_spec(i):
    set_variant_raw(vidx[i])
    set_split(vsplit[i])
work = sys.argv[1] if len(sys.argv) > 1 else "zipf"
ROUNDS, STEPS = 5, 5
for wl in [w for w in work.split(",") if w and w != "none"]:
    align = 1
    size = 4 << 30
    label = wl
    if "@" in wl:  # e.g. single@128: the same workload scaled to 128 MiB (cache-resident probe)
        wl, mib = wl.split("@")
        size = int(mib) << 20
    if wl in ("zipf", "fixed4k", "c2u"):  # bench.py's workloads, rank-0 datasets
        offs, lens, seed, _ = bench.make_dataset(wl, size, 0)
    elif wl == "zipf16":
        lens = zdbcrc.zipf_lengths(size, 0xC3C3C3).astype(np.int64)
        seed = 0x5A0DB5EED + 3
        align = 16 if wl == "zipf16" else 1
    elif wl in ("zipf_small", "zipf_large"):
        # C3's records split by size (<= 4 KiB / larger), each class tiled
        # until the batch holds `size` bytes: per-record vs per-byte cost
        base = zdbcrc.zipf_lengths(4 << 30, 0xC3C3C3).astype(np.int64)
        base = base[base <= 4096] if wl == "zipf_small" else base[base > 4096]
        reps = max(1, -(-size // int(base.sum())))
        lens = np.tile(base, reps)
        lens = lens[:int(np.searchsorted(np.cumsum(lens), size))]
        seed = 0x5A0DB5EED + 3
    elif wl.startswith("zipf_le"):  # C3's records up to N bytes, tiled to `size`
        base = zdbcrc.zipf_lengths(4 << 30, 0xC3C3C3).astype(np.int64)
        base = base[base <= int(wl[7:])]
        reps = max(1, -(-size // int(base.sum())))
        lens = np.tile(base, reps)
        lens = lens[:int(np.searchsorted(np.cumsum(lens), size))]
        seed = 0x5A0DB5EED + 3
    elif wl.startswith("fixed") and wl[5:].isdigit():  # fixed N-byte records, packed back to back
        lens = np.full(size // int(wl[5:]), int(wl[5:]), np.int64); seed = 0x5A0DB5EED
    elif wl == "single":
        lens = np.array([size - 16], np.int64); seed = 0x5A0DB5EED
    elif wl == "fixed64k":
        lens = np.full(1 << 16, 65536, np.int64); seed = 0x5A0DB5EED
    else:
        lens = np.full(size >> 12, 4096, np.int64); seed = 0x5A0DB5EED
    if wl not in ("zipf", "fixed4k", "c2u"):
        padded = (lens + align - 1) // align * align
        offs = np.zeros(len(lens), np.int64); offs[1:] = np.cumsum(padded[:-1])
    total = int(offs[-1] + lens[-1])
    arena = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    zdbcrc.synth_fill_device(arena, seed)
    do, dl = torch.from_numpy(offs).cuda(), torch.from_numpy(lens.astype(np.int32)).cuda()
    outs = {v: torch.empty(len(lens), dtype=torch.int32, device="cuda") for v in sel}
    times = {v: [] for v in sel}
    walls = {v: [] for v in sel}
    # clock settle: ~1 s of untimed launches before the first timed round
    set_spec(sel[0])
    t_end = time.time() + float(os.environ.get("SETTLE_S", "1.0"))
    while time.time() < t_end:
        for _ in range(20):
            zdbcrc.batch_device(arena, do, dl, outs[sel[0]])
        torch.cuda.synchronize()
    for r in range(ROUNDS):
        for v in sel:
            set_spec(v)
            zdbcrc.batch_device(arena, do, dl, outs[v])
            torch.cuda.synchronize(); zdbcrc.kernel_stats(); small_kernel_stats(); zdbcrc.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(STEPS):
                zdbcrc.batch_device(arena, do, dl, outs[v])
            torch.cuda.synchronize(); t1 = time.perf_counter(); zdbcrc.set_timing(False)
            ms, k = zdbcrc.kernel_stats()
            ms2, k2 = small_kernel_stats()
            times[v].append(ms / k + (ms2 / k2 if k2 else 0.0))
            walls[v].append((t1 - t0) / STEPS * 1e3)
    ref = outs[sel[0]].cpu()
    payload = int(lens.sum())
    for v in sel:
        t = np.array(times[v])
        same = bool(torch.equal(outs[v].cpu(), ref))
        print(json.dumps({"workload": label, "variant": vname[v], "median_ms": round(float(np.median(t)), 4),
                          "step_ms_median": round(float(np.median(walls[v])), 4),
                          "min_ms": round(float(t.min()), 4),
                          "gibs_median": round(payload / (np.median(t) / 1e3) / 2**30, 1),
                          "frac_spec": round((payload + 16 * len(lens)) / (np.median(t) / 1e3) / 8e12, 4),
                          "same_as_first": same}), flush=True)
    del arena
