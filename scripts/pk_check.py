#!/usr/bin/env python3
"""Packed small-record kernel variants (diagnostic library, by index) against
the oracle on crafted batches: every length 0..300, 4 KiB values at every
alignment, records in the first 16 bytes of 4 KiB pages (the shifted
first-piece path), a wrong max-length hint (1 MiB records), records past
4 GiB offsets are covered by the product tests.  Prints one JSON line per
(variant, case); exits 1 on any mismatch."""
import ctypes as C, json, os, sys
from pathlib import Path
import numpy as np
ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "0-db_amd"), str(ROOT / "oracle")]
os.environ.setdefault("ZDBCRC_LIB", str(ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"))
import torch, zdbcrc, oracle

set_variant = zdbcrc._lib.zdbcrc_debug_set_variant
set_variant.restype = C.c_char_p
set_variant.argtypes = [C.c_int]
orc = oracle.Oracle()


def cases():
    rng = np.random.default_rng(5)
    out = {}
    lens = np.arange(0, 301)
    offs = np.cumsum(np.concatenate([[1], lens[:-1] + 3]))
    out["every_len_0_300"] = (offs, lens, int(offs[-1] + lens[-1]) + 64)
    lens = np.full(64 * 16, 4096)
    offs = np.array([4096 * 4 * i + (i % 64) for i in range(len(lens))])  # every alignment
    out["4k_every_alignment"] = (offs, lens, int(offs[-1]) + 4096 + 64)
    # page starts: record at page + (0..15) with lengths that put piece 0 below the page
    offs, lens = [], []
    for p in range(64):
        for a in range(16):
            for L in (1, 2, 3, 5, 17, 100, 4095, 4093):
                offs.append(4096 * (p * 4 + 1) + a)
                lens.append(L)
    offs = np.array(offs); lens = np.array(lens)
    out["page_start_records"] = (offs, lens, int(offs.max() + lens.max()) + 64)
    # arena-start records (piece 0 would start below the allocation)
    offs = np.array([0, 1, 2, 3, 5, 9, 15, 0, 3])
    lens = np.array([100, 1, 2, 3, 7, 13, 1, 4096, 4093])
    out["arena_start"] = (offs, lens, 8192)
    lens = rng.integers(0, 4097, 200_000)
    offs = np.zeros(len(lens), np.int64); offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 5, len(lens) - 1))
    out["random_0_4k"] = (offs, lens, int(offs[-1] + lens[-1]) + 64)
    lens = np.concatenate([rng.integers(0, 300, 5000), [1 << 20, 3 << 20], rng.integers(0, 4097, 5000)])
    offs = np.zeros(len(lens), np.int64); offs[1:] = np.cumsum(lens[:-1] + 1)
    out["wrong_hint_big_records"] = (offs, lens, int(offs[-1] + lens[-1]) + 64)
    return out


bad = 0
cs = cases()
variants = [int(x) for x in sys.argv[1].split(",")]
for name, (offs, lens, size) in cs.items():
    host = oracle.splitmix_bytes(size, 77)
    want = orc.batch(host, offs.astype(np.uint64), lens.astype(np.uint32))
    arena = torch.from_numpy(host).cuda()
    do = torch.from_numpy(offs.astype(np.int64)).cuda()
    dl = torch.from_numpy(lens.astype(np.int32)).cuda()
    for v in variants:
        vn = set_variant(v).decode()
        out = torch.full((len(lens),), -1, dtype=torch.int32, device="cuda")
        for rep in range(2):
            zdbcrc.batch_device(arena, do, dl, out)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        nbad = int((got != want).sum())
        bad += nbad
        first = np.flatnonzero(got != want)[:5].tolist()
        print(json.dumps({"case": name, "variant": vn, "records": len(lens), "mismatches": nbad,
                          "first_bad": first, "first_bad_len": [int(lens[i]) for i in first],
                          "first_bad_off": [int(offs[i]) for i in first]}), flush=True)
sys.exit(1 if bad else 0)
