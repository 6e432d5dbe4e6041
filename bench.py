#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC32 (0-db zdb_crc32) on MI355X.

One step = one zdb_crc32_batch_device call (plan scan + kernel) over the
whole per-GPU batch, inputs already resident in HBM.  Default workload is
BASELINE.json configs[2] / SURVEY §8(d) C3: Zipf-mixed records 64 B..1 MiB,
packed back to back at arbitrary byte alignment, ~4 GiB per GPU.  Each rank
checksums its own batch (different seed): weak scaling, no collective on the
data path (torch.distributed is used only for the barrier and the max/sum of
the timing).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload zipf|fixed4k|c2u]
  N > 1: either launched by torch.distributed.run (WORLD_SIZE must equal N),
  or started plainly, in which case bench.py starts the N rank processes
  itself (one per GPU) before touching any GPU.  Every rank checks its own
  shard against the reference's digest of it (tests/golden/digests.json).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
for p in (ROOT / "0-db_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))

METRIC = "GiB/s device-resident batched CRC32, mixed 4KiB–1MiB records, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
C2_SEED = 0x5A0DB5EED
C3_SEED = 0x5A0DB5EED + 3
C3_LEN_SEED = 0xC3C3C3
C4_SEED = 0x5A0DB5EED + 4
C4_LEN_SEED = 0xC4C4C4
C4_FILES = 64
C4_FILE_CAP = 256 << 20  # bytes per datafile (64 x 256 MiB per GPU)
C4_KEY = 8               # key bytes per entry
C4_TIMESTAMP = 1700000000
ENTRY_HDR = 18           # data_entry_header_t (libzdb/data.h:56-65)
FILE_HDR = 28            # data_header_t (libzdb/data.h:38-45)
GIB = float(1 << 30)


def log(msg: str):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def make_dataset(workload: str, target: int, rank: int):
    """Host descriptors for this rank's batch (rank 0 = the golden dataset)."""
    import zdbcrc
    if workload == "zipf":
        lens = zdbcrc.zipf_lengths(target, C3_LEN_SEED + rank).astype(np.int64)
        offs = np.zeros(len(lens), np.int64)
        offs[1:] = np.cumsum(lens[:-1])
        seed = C3_SEED + rank
        desc = "C3: Zipf-mixed 64 B..1 MiB records, packed at any byte alignment"
    elif workload == "fixed4k":
        n = target // 4096
        lens = np.full(n, 4096, np.int64)
        offs = np.arange(n, dtype=np.int64) * 4096
        seed = C2_SEED + rank
        desc = "C2: fixed 4 KiB records, 4 KiB-aligned"
    elif workload == "c2u":
        # the C2 payloads laid out as a datafile image (18 B
        # entry header + 8 B key before each), so every payload is misaligned
        n = target // 4096
        lens = np.full(n, 4096, np.int64)
        offs = FILE_HDR + np.arange(n, dtype=np.int64) * (ENTRY_HDR + C4_KEY + 4096) + ENTRY_HDR + C4_KEY
        seed = C2_SEED + rank
        desc = "C2u: fixed 4 KiB payloads inside a datafile image (26 B header+key each), misaligned"
    else:
        raise SystemExit(f"unknown workload {workload}")
    return offs, lens, seed, desc


def c4_layout(rank: int, files: int = C4_FILES, file_cap: int = C4_FILE_CAP) -> dict:
    """SURVEY §8(d) C4 shard of one GPU: reference-valid datafiles (format of
    libzdb/data.h, version 3) holding C3-distributed payloads with 8-byte
    keys, packed into `files` datafiles of at most `file_cap` bytes, placed
    back to back in one arena.  Entry e's header sits at entry_off[e], its
    key right after, its payload at payload_off[e]; `previous` is the
    file-relative offset of the entry before it (0 for the first), as
    data_insert writes it (data.c:594-633)."""
    import zdbcrc
    target = files * file_cap
    lens = zdbcrc.zipf_lengths(target, C4_LEN_SEED + rank).astype(np.int64)
    ent = ENTRY_HDR + C4_KEY + lens
    file_of = np.zeros(len(lens), np.int64)
    rel = np.zeros(len(lens), np.int64)  # file-relative entry offset
    f, pos, n = 0, FILE_HDR, 0
    for e in range(len(lens)):
        if pos + ent[e] > file_cap:
            f += 1
            pos = FILE_HDR
            if f == files:
                break
        file_of[e], rel[e] = f, pos
        pos += ent[e]
        n = e + 1
    lens, ent, file_of, rel = lens[:n], ent[:n], file_of[:n], rel[:n]
    nfiles = int(file_of[-1]) + 1
    fsize = np.full(nfiles, FILE_HDR, np.int64)
    np.add.at(fsize, file_of, ent)
    file_off = np.zeros(nfiles, np.int64)
    file_off[1:] = np.cumsum(fsize[:-1])
    prev = np.zeros(n, np.int64)
    same = np.zeros(n, bool)
    same[1:] = file_of[1:] == file_of[:-1]
    prev[1:][same[1:]] = rel[:-1][same[1:]]
    entry_off = file_off[file_of] + rel
    return {"lens": lens, "entry_off": entry_off, "payload_off": entry_off + ENTRY_HDR + C4_KEY,
            "prev": prev, "file_of": file_of, "file_off": file_off, "file_size": fsize,
            "total": int(file_off[-1] + fsize[-1])}


def c4_entry_headers(layout: dict, crcs: np.ndarray) -> np.ndarray:
    """(n, 26) bytes: data_entry_header_t (packed, little endian) + 8-byte key
    (the entry index), with the payload crcs in `integrity`."""
    n = len(layout["lens"])
    dt = np.dtype([("idlength", "u1"), ("datalength", "<u4"), ("previous", "<u4"), ("integrity", "<u4"),
                   ("flags", "u1"), ("timestamp", "<u4"), ("key", "<u8")])
    assert dt.itemsize == ENTRY_HDR + C4_KEY
    h = np.zeros(n, dt)
    h["idlength"] = C4_KEY
    h["datalength"] = layout["lens"]
    h["previous"] = layout["prev"]
    h["integrity"] = crcs
    h["timestamp"] = C4_TIMESTAMP
    h["key"] = np.arange(n, dtype=np.uint64)
    return h.view(np.uint8).reshape(n, ENTRY_HDR + C4_KEY)


def c4_file_headers(layout: dict) -> np.ndarray:
    import zdbcrc
    return np.stack([np.frombuffer(zdbcrc.encode_header(f), np.uint8)
                     for f in range(len(layout["file_off"]))])


def c4_image_host(layout: dict, seed: int, crcs: np.ndarray, files: int | None = None) -> np.ndarray:
    """Host image of the first `files` datafiles of a C4 shard (tests, golden
    checks): synthetic bytes at every arena position, then the headers."""
    import zdbcrc
    nf = len(layout["file_off"]) if files is None else files
    end = int(layout["file_off"][nf - 1] + layout["file_size"][nf - 1])
    img = zdbcrc.synth_fill(end, seed)
    sel = layout["file_of"] < nf
    hdr = c4_entry_headers(layout, crcs)[sel]
    idx = layout["entry_off"][sel][:, None] + np.arange(ENTRY_HDR + C4_KEY)
    img[idx] = hdr
    fidx = layout["file_off"][:nf, None] + np.arange(FILE_HDR)
    img[fidx] = c4_file_headers(layout)[:nf]
    return img


def c4_build_device(lay: dict, seed: int):
    """The C4 images in HBM: synthetic bytes at every position, then the file
    and entry headers (integrity = the payload crc from an untimed checksum
    pass).  Returns (image, payload offsets, lengths, expected crcs read back
    out of the image headers, host crcs)."""
    import torch
    import zdbcrc
    n = len(lay["lens"])
    img = torch.empty(lay["total"] + 64, dtype=torch.uint8, device="cuda")
    zdbcrc.synth_fill_device(img, seed)
    d_poff = torch.from_numpy(lay["payload_off"]).cuda()
    d_len = torch.from_numpy(lay["lens"].astype(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    zdbcrc.batch_device(img, d_poff, d_len, out)
    crcs = out.cpu().numpy().view(np.uint32).copy()
    hdr = torch.from_numpy(c4_entry_headers(lay, crcs).reshape(-1)).cuda()
    idx = torch.from_numpy((lay["entry_off"][:, None] + np.arange(ENTRY_HDR + C4_KEY)).reshape(-1)).cuda()
    img[idx] = hdr
    fidx = torch.from_numpy((lay["file_off"][:, None] + np.arange(FILE_HDR)).reshape(-1)).cuda()
    img[fidx] = torch.from_numpy(c4_file_headers(lay).reshape(-1)).cuda()
    del hdr, idx, fidx
    ioff = torch.from_numpy(lay["entry_off"] + 9).cuda()  # `integrity` at byte 9 of the entry header
    b = [img[ioff + i].to(torch.int64) for i in range(4)]
    expected = (b[0] | (b[1] << 8) | (b[2] << 16) | (b[3] << 24)).to(torch.int32)
    return img, d_poff, d_len, expected, crcs


def c4_leg(rank: int, world: int, steps: int, warmup: int, settle_s: float, barrier) -> dict:
    """the integrity scan of this rank's 64 reference-valid
    datafiles (~16 GiB), device-resident, from the images alone: one step =
    zdb_datafile_scan_device = the GPU record-boundary discovery (f3: chunked
    speculative walk + exact stitch), then plan + checksum + compare with the
    `integrity` field of every entry header over the record count the walk
    left in device memory, and one synchronisation at the end.  The image is built in HBM (synthetic bytes, then the
    headers, whose crcs come from an untimed checksum pass and are checked
    against the reference's digest of this shard).  Reported beside it: the
    walk alone and the verify with descriptors known in advance (round 1's
    C4 figure)."""
    import torch
    import zdbcrc
    lay = c4_layout(rank)
    n = len(lay["lens"])
    img, d_poff, d_len, expected, crcs = c4_build_device(lay, C4_SEED + rank)
    parity = parity_of(digest(crcs), shard_digest_ref("C4", rank, 4.0), f"C4 shard {rank}")
    store = zdbcrc.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 1024)
    n_walk = store.scan()
    walk_ok = n_walk == n and bool(torch.equal(store.entry_off[:n].cpu(), torch.from_numpy(lay["entry_off"])))
    scan_ok = walk_ok and bool(torch.equal(store.computed[:n], store.expected[:n]))
    if not walk_ok:
        parity += f"; DEVICE WALK MISMATCH ({n_walk} records vs {n})"

    def timed(fn, k):
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        t_settle = time.perf_counter() + settle_s
        while time.perf_counter() < t_settle:
            fn()
            torch.cuda.synchronize()
        barrier()
        zdbcrc.kernel_stats()
        zdbcrc.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        barrier()
        zdbcrc.set_timing(False)
        km, kl = zdbcrc.kernel_stats()
        return t1 - t0, km / max(kl, 1)

    scan_s, kern_ms = timed(store.scan, steps)
    mismatches = int(store.mismatch_count.item())
    walk_s, _ = timed(store.walk, steps)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    mism = torch.zeros(1024, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    verify_s, _ = timed(lambda: zdbcrc.verify_device(img, d_poff, d_len, expected, out, mism, cnt), steps)
    payload = int(lay["lens"].sum())
    elapsed, all_payload = combine_ranks(scan_s, payload, world)
    kern_s = kern_ms / 1e3
    alg = payload + 20 * n  # integrity scan: + 4 B expected crc read
    res = {"desc": f"C4: integrity scan of {len(lay['file_off'])} reference-valid datafiles per GPU "
                   f"({lay['total']} B images, {n} records, C3 payload sizes, 8 B keys), device-resident, "
                   "from the images alone (GPU walk + checksum + compare per step)",
           "records_per_gpu": n, "payload_bytes_per_gpu": payload, "n_gpus": world,
           "gibs": round(all_payload * steps / elapsed / GIB, 2),
           "ms_per_step": round(elapsed / steps * 1e3, 4),
           "walk_ms": round(walk_s / steps * 1e3, 4),
           "verify_known_descriptors_ms": round(verify_s / steps * 1e3, 4),
           "kernel_ms": round(kern_ms, 4),
           "roofline_frac": round(alg / kern_s / 1e9 / HBM_PEAK_GBS, 4),
           "rewalked_chunks": int(store.rewalks[-1].item()),
           "mismatches": mismatches, "scan_clean": scan_ok, "parity_by_rank": gather_ranks(parity, world)}
    del img, out, expected, store
    torch.cuda.empty_cache()
    return res


def digest(crcs: np.ndarray) -> dict:
    import zdbcrc  # the scalar drop-in engine (CPU) hashes the crc array
    return {"count": int(len(crcs)), "xor": f"{int(np.bitwise_xor.reduce(crcs)):08x}",
            "crc_of_crcs": f"{zdbcrc.crc32(crcs.astype('<u4').tobytes()):08x}"}


def cpu_baseline(offs, lens, seed, seconds: float) -> dict | None:
    """The reference CPU path (oracle/_ref: libzdb/crc32.c compiled from the
    reference sources), or the oracle port if _ref is absent, timed on this
    host on the same records (host copy of rank 0's batch)."""
    import oracle
    import zdbcrc
    threads = cpu_threads()
    total = int(offs[-1] + lens[-1])
    arena = zdbcrc.synth_fill(total + 16, seed)
    o = offs.astype(np.uint64)
    l = lens.astype(np.uint32)
    if oracle.Reference.available():
        ref, kind = oracle.Reference(), "reference"
        run = lambda th: ref.batch(arena, o, l, threads=th)
    else:
        orc, kind = oracle.Oracle(), "port"
        threads = 1
        run = lambda th: orc.batch(arena, o, l)
    # multi-threaded passes over the full batch, then one single-thread pass
    passes, t0 = 0, time.perf_counter()
    while True:
        run(threads)
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    mt = passes * total / (time.perf_counter() - t0) / GIB
    # SURVEY §8(d) also asks for the host's whole CPU count: every CPU of the
    # affinity mask (on the GPU box many of them belong to other jobs' shares,
    # so this is an upper bound that the job share above does not claim)
    full = len(os.sched_getaffinity(0))
    full_res = None
    if kind == "reference" and full > threads:
        fp, t0 = 0, time.perf_counter()
        while True:
            run(full)
            fp += 1
            if time.perf_counter() - t0 >= seconds:
                break
        full_res = {"value": round(fp * total / (time.perf_counter() - t0) / GIB, 3), "unit": "GiB/s",
                    "cores": full, "passes": fp}
    n1 = int(np.searchsorted(np.cumsum(lens), 1 << 30)) + 1  # ~1 GiB prefix
    t0 = time.perf_counter()
    if kind == "reference":
        ref.batch(arena, o[:n1], l[:n1], threads=1)
    else:
        orc.batch(arena, o[:n1], l[:n1])
    b1 = int(lens[:n1].sum())
    st = b1 / (time.perf_counter() - t0) / GIB
    return {"value": round(mt, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"full rank-0 batch ({len(lens)} records, {total} B) x {passes} passes on {threads} "
                      f"threads ({seconds:.0f}+ s wall); single-thread {st:.2f} GiB/s on a "
                      f"{b1 >> 20} MiB prefix",
            "single_thread_gibs": round(st, 3), "cpu_model": cpu_model(),
            "affinity_cpus": full, "all_affinity_cpus": full_res,
            "threads_rule": "value: one thread per CPU of this job's share, min(sched_getaffinity, "
                            "OMP_NUM_THREADS); all_affinity_cpus: one thread per CPU of the affinity mask"}


def cpu_threads() -> int:
    """the CPUs this job may use: its affinity mask, capped by OMP_NUM_THREADS
    where the launcher sets it (the GPU box gives a one-GPU job 16 of its
    256 CPUs and says so there)"""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline_shapes(seconds: float) -> dict:
    """the reference CPU path on the other BASELINE shapes (C2: 1 Mi x 4 KiB;
    C4: a 4 GiB prefix of rank 0's C4 shard -- C3 payload sizes inside
    datafiles), same thread rule, bounded samples"""
    import oracle
    import zdbcrc
    if not oracle.Reference.available():
        return {}
    ref, th, out = oracle.Reference(), cpu_threads(), {}
    shapes = {}
    o2, l2, s2, _ = make_dataset("fixed4k", 4 << 30, 0)
    shapes["C2"] = (o2, l2, s2)
    lay = c4_layout(0)
    k = int(np.searchsorted(lay["payload_off"] + lay["lens"], 4 << 30))
    shapes["C4_prefix"] = (lay["payload_off"][:k], lay["lens"][:k], C4_SEED)
    for name, (o, l, seed) in shapes.items():
        total = int(o[-1] + l[-1])
        arena = zdbcrc.synth_fill(total + 16, seed)
        ou, lu = o.astype(np.uint64), l.astype(np.uint32)
        passes, t0 = 0, time.perf_counter()
        while True:
            ref.batch(arena, ou, lu, threads=th)
            passes += 1
            if time.perf_counter() - t0 >= seconds:
                break
        out[name] = {"gibs": round(passes * int(l.sum()) / (time.perf_counter() - t0) / GIB, 3),
                     "records": len(l), "payload_bytes": int(l.sum()), "passes": passes, "threads": th}
        del arena
    return out


def e2e_legs(offs, lens, seed) -> dict:
    """Host-memory paths, reported beside the
    device-resident number: the SET path's 256 KiB value through the
    host-buffer entry (zero-copy from pinned memory, results through the
    mailbox), the zipf batch
    from pinned host memory (PCIe-inclusive rate), and the integrity-check
    tool on a 256 MiB datafile (65,000 x 4 KiB, as SURVEY §6) against the
    reference tool and the scalar engine."""
    import subprocess
    import tempfile
    import oracle
    import zdbcrc
    res = {}
    V = 256 * 1024
    pin = zdbcrc.PinnedBuffer(64 * V)
    pin.array[:] = zdbcrc.synth_fill(64 * V, 0xC5)
    one = pin.array[:V]
    want = zdbcrc.crc32(one)
    for _ in range(5):
        assert zdbcrc.batch_host(one, [0], [V])[0] == want
    set_path = {}
    for b in (1, 8, 64):
        offs_b = np.arange(b, dtype=np.uint64) * V
        lens_b = np.full(b, V, np.uint32)
        ts = []
        for _ in range(50 if b < 64 else 20):
            t0 = time.perf_counter()
            zdbcrc.batch_host(pin.array[:b * V], offs_b, lens_b)
            ts.append(time.perf_counter() - t0)
        med = float(np.median(ts))
        set_path[f"batch{b}"] = {"us_per_call": round(med * 1e6, 1), "gibs": round(b * V / med / GIB, 2)}
    ts = []
    for _ in range(200):
        t0 = time.perf_counter()
        zdbcrc.crc32(one)
        ts.append(time.perf_counter() - t0)
    set_path["cpu_scalar_engine_us"] = round(float(np.median(ts)) * 1e6, 1)
    if oracle.Reference.available():
        ref = oracle.Reference()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            ref.crc32(one)
            ts.append(time.perf_counter() - t0)
        set_path["cpu_reference_us"] = round(float(np.median(ts)) * 1e6, 1)
    res["set_path_256KiB"] = set_path
    pin.free()

    # f2: pipelined SETs through the two-phase batch harness (zdb-set-pipeline):
    # values checksummed in one call per receive buffer, GPU (in place, pinned)
    # vs the scalar engine; crc_s is phase 1 alone
    import subprocess
    sys.path.insert(0, str(ROOT / "tests"))
    from test_set_pipeline import resp_set
    vals = zdbcrc.synth_fill(64 * V, 0xF2)
    pipeline = {}
    for nset in (8, 64, 240):
        # 6 receive-buffer batches of nset SETs; the first batch of a process
        # pays one-time costs (plan buffers, first mapping of the pinned
        # buffer), so the per-SET figures are over batches 2..6
        reqs = [resp_set(b"k%05d" % (i % 64), vals[((i * 7) % 64) * V:((i * 7) % 64 + 1) * V].tobytes())
                for i in range(6 * nset)]
        stream = b"".join(reqs)
        row = {}
        for eng in ("hip", "auto", "cpu"):
            with tempfile.TemporaryDirectory() as td:
                # stdin is a file: one read fills the receive buffer, so a batch
                # is --batch SETs (a pipe would hand over 64 KiB per read)
                with open(f"{td}/stream", "wb") as f:
                    f.write(stream)
                with open(f"{td}/stream", "rb") as f:
                    p = subprocess.run([str(ROOT / "0-db_amd/bin/zdb-set-pipeline"), f"--engine={eng}", "--stats",
                                        f"--batch={nset}", f"{td}/d"], stdin=f, capture_output=True, timeout=300)
                assert p.returncode == 0, p.stderr[-500:]
                st = json.loads(p.stderr.decode().strip().splitlines()[-1])
            w = max(st["sets_after_first_batch"], 1)
            row[eng] = {"crc_us_per_set": round(st["crc_s_after_first_batch"] / w * 1e6, 2),
                        "apply_us_per_set": round(st["apply_s"] / st["sets"] * 1e6, 2),
                        "crc_gibs": round(w * V / max(st["crc_s_after_first_batch"], 1e-9) / GIB, 2),
                        "batches": st["batches"], "gpu_batches": st["gpu_batches"], "unchanged": st["unchanged"]}
        pipeline[f"{nset}x256KiB"] = row
    res["set_pipeline"] = pipeline

    # zipf batch from pinned host memory: PCIe-inclusive
    total = int(offs[-1] + lens[-1])
    hp = zdbcrc.PinnedBuffer(total + 16)
    hp.array[:total + 16] = zdbcrc.synth_fill(total + 16, seed)
    o, l = offs.astype(np.uint64), lens.astype(np.uint32)
    zdbcrc.batch_host(hp.array, o, l)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        zdbcrc.batch_host(hp.array, o, l)
        ts.append(time.perf_counter() - t0)
    res["zipf_from_pinned_host"] = {"gibs": round(int(lens.sum()) / min(ts) / GIB, 1),
                                    "s": round(min(ts), 4)}
    hp.free()

    # integrity-check on a 256 MiB datafile written through the SET batch path
    n = 65000
    vals = zdbcrc.synth_fill(n * 4096, 0xC1)
    vo = np.arange(n, dtype=np.uint64) * 4096
    vl = np.full(n, 4096, np.uint32)
    crcs = zdbcrc.batch_host(vals, vo, vl)  # SET-path batch checksum on the GPU
    keys = [b"k%d" % i for i in range(n)]
    body, _, _ = zdbcrc.encode_batch(keys, vals, vo, vl, crcs, file_offset=28)
    with tempfile.TemporaryDirectory() as td:
        with open(f"{td}/d0", "wb") as f:
            f.write(zdbcrc.encode_header(0) + body)
        os.symlink("d0", f"{td}/zdb-data-0")
        tools = {"gpu_tool": [str(ROOT / "0-db_amd/bin/zdb-integrity-check"), "--engine=hip", f"{td}/zdb-data-0"],
                 "auto_engine_tool": [str(ROOT / "0-db_amd/bin/zdb-integrity-check"), "--engine=auto",
                                      f"{td}/zdb-data-0"],
                 "scalar_engine_tool": [str(ROOT / "0-db_amd/bin/zdb-integrity-check"), "--engine=cpu",
                                        f"{td}/zdb-data-0"]}
        if oracle.REF_INTEGRITY.exists():
            tools["reference_tool"] = [str(oracle.REF_INTEGRITY), f"{td}/zdb-data-0"]
        ic = {"file_bytes": 28 + len(body), "records": n}
        for name, cmd in tools.items():
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=120)
                ts.append(time.perf_counter() - t0)
                assert p.returncode == 0, (name, p.stderr[-500:])
            ic[name + "_s"] = round(min(ts), 4)
        res["integrity_check_256MiB"] = ic

        # store-wide scan: 8 datafiles in one tool run, worker
        # threads sharing the GPU, against the reference tool run once per file
        files = []
        for i in range(8):
            d = f"{td}/ns{i}"
            os.mkdir(d)
            os.link(f"{td}/d0", f"{d}/d0")
            os.symlink("d0", f"{d}/zdb-data-0")
            files.append(f"{d}/zdb-data-0")
        tool = str(ROOT / "0-db_amd/bin/zdb-integrity-check")
        scan = {"files": len(files), "file_bytes": 28 + len(body)}
        # 32 files (8 GiB): the GPU engine's fixed cost (HIP start-up and exit) spread over more
        # bytes; `auto` still takes the scalar engine here (J x AUTO_CPU_GIBS >= AUTO_PCIE_GIBS for 8 workers)
        files32 = files * 4
        runs = {"gpu_tool_jobs8": ([[tool, "--engine=hip", "--jobs=8"] + files], 8),
                "auto_engine_tool_jobs8": ([[tool, "--engine=auto", "--jobs=8"] + files], 8),
                "scalar_engine_tool_jobs8": ([[tool, "--engine=cpu", "--jobs=8"] + files], 8),
                "gpu_tool_jobs8_32files": ([[tool, "--engine=hip", "--jobs=8"] + files32], 32),
                "auto_engine_tool_jobs8_32files": ([[tool, "--engine=auto", "--jobs=8"] + files32], 32),
                "scalar_engine_tool_jobs8_32files": ([[tool, "--engine=cpu", "--jobs=8"] + files32], 32)}
        if oracle.REF_INTEGRITY.exists():
            runs["reference_tool_per_file"] = ([[str(oracle.REF_INTEGRITY), f] for f in files], 8)
        for name, (cmds, nf) in runs.items():
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                for cmd in cmds:
                    p = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=300)
                    assert p.returncode == 0, (name, p.stderr[-500:])
                ts.append(time.perf_counter() - t0)
            scan[name + "_s"] = round(min(ts), 4)
            scan[name + "_gibs"] = round(nf * (28 + len(body)) / min(ts) / GIB, 2)
        # where the time goes in one GPU-engine run (ZDBCRC_TOOL_TRACE)
        p = subprocess.run([tool, "--engine=hip", "--jobs=8"] + files, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           env=dict(os.environ, ZDBCRC_TOOL_TRACE="1"), timeout=300)
        scan["gpu_tool_trace"] = [ln for ln in p.stderr.decode().splitlines() if ln.startswith("[trace]")][:8]
        res["integrity_scan_8x256MiB"] = scan
    return res


def combine_ranks(elapsed_s: float, payload: int, world: int) -> tuple[float, float]:
    """Whole-job aggregation: the slowest rank's time and the bytes of all
    ranks (the only cross-rank traffic; the data path has no collective).
    Works on any initialised backend (nccl on the GPU box, gloo in tests)."""
    if world == 1:
        return elapsed_s, float(payload)
    import torch
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    b = torch.tensor([float(payload)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), float(b.item())


def pmc_traffic(workload: str) -> tuple:
    """(HBM bytes per launch, where that number was measured): the PMC pass
    cannot run inside this process (rocprofv3 wraps the whole program), so
    the figure is the committed FETCH_SIZE pass of the same kernel
    (profiles/pmc_traffic.json), labelled with its source"""
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None, None
    try:
        d = json.loads(p.read_text()).get(workload, {})
        return d.get("hbm_bytes_per_launch"), d.get("source")
    except Exception:
        return None, None


def shard_digest_ref(kind: str, rank: int, gib: float) -> dict | None:
    """The reference's digest of this rank's shard (tests/golden/digests.json,
    computed by oracle/_ref in the build container: make_golden.py)."""
    gold = ROOT / "tests" / "golden" / "digests.json"
    if not gold.exists():
        return None
    d = json.loads(gold.read_text())
    key = {("C3", 4.0): "C3_ranks", ("C3", 1 / 64): "C3_16MiB_ranks", ("C4", 4.0): "C4_ranks"}.get((kind, gib))
    ranks = d.get(key, []) if key else []
    if rank < len(ranks):
        return ranks[rank]
    if rank == 0 and kind in d and gib == 4.0:  # round-1 layout: rank 0 only
        return d[kind]
    return None


def workload_parity(workload: str, out, rank: int, gib: float) -> str:
    """the full-size output of one workload (the device `out` tensor of the
    last step) against the reference's digest of it: C3 per rank, C2 and
    C2u for rank 0's 4 GiB batch (tests/golden/digests.json)"""
    got = digest(out.cpu().numpy().view(np.uint32))
    if workload == "zipf":
        return parity_of(got, shard_digest_ref("C3", rank, gib), f"C3 shard {rank}")
    key = {"fixed4k": "C2", "c2u": "C2u"}[workload]
    if rank == 0 and gib == 4.0:
        return parity_of(got, json.loads((ROOT / "tests/golden/digests.json").read_text()).get(key), key)
    return "unchecked (no reference digest for this shard)"


def parity_of(got: dict, ref: dict | None, what: str) -> str:
    if ref is None:
        return "unchecked (no reference digest for this shard)"
    ok = all(got[k] == ref[k] for k in ("count", "xor", "crc_of_crcs"))
    return f"bit-exact vs reference digest {what}" if ok else f"MISMATCH {got} vs {ref}"


def summarize_parity(parities: list) -> str:
    if len(parities) == 1:
        return parities[0]
    bad = [i for i, p in enumerate(parities) if not p.startswith("bit-exact")]
    if not bad:
        return f"bit-exact vs reference digests on all {len(parities)} shards"
    return f"NOT bit-exact (or unchecked) on ranks {bad}: see parity_by_rank"


def gather_ranks(obj, world: int) -> list:
    """every rank's small result object on every rank (parity strings)"""
    if world == 1:
        return [obj]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def read_ceiling(arena, nbytes: int, achieved_gbs: float):
    """the achievable HBM read ceiling on THIS box, measured right
    after the timed steps over the same 4 GiB arena -- read-only streaming
    probes of the checksum kernel's access shape (each wave its own contiguous
    slice, 1 KiB per load instruction, nontemporal loads; U = 4 or 8 loads in
    flight per lane).  The probes live in the diagnostic library
    (libzdbcrc_diag.so, never in the product library); None if it is absent."""
    import ctypes
    import torch
    lib_path = ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"
    if not lib_path.exists():
        return None
    lib = ctypes.CDLL(str(lib_path))
    probe = lib.zdbcrc_debug_stream_read
    probe.restype = ctypes.c_float
    probe.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    sink = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    nb = nbytes // 16 * 16
    best = None
    runs = {}
    for code, name in ((-104, "slices_nt_u4_wg1024"), (-204, "slices_nt_u4_wg768"), (-108, "slices_nt_u8_wg1024")):
        ts = [probe(arena.data_ptr(), nb, sink.data_ptr(), code, st) for _ in range(7)][2:]
        if min(ts) <= 0:
            return None
        tbs = nb / (float(np.median(ts)) / 1e3) / 1e12
        runs[name] = round(tbs, 3)
        if best is None or tbs > best[1]:
            best = (name, tbs)
    del sink
    return {"probe": best[0], "tbs": round(best[1], 3), "frac_of_spec": round(best[1] * 1e3 / HBM_PEAK_GBS, 4),
            "probes_tbs": runs, "bytes": nb,
            "kernel_frac_of_ceiling": round(achieved_gbs / (best[1] * 1e3), 4)}


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` outside torch.distributed.run: start N rank
    processes (one per GPU) before this process touches any GPU, with the
    environment torchrun would give them, and return the worst exit code.
    Only rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    return rc


def cpu_rank(args, rank: int, world: int) -> None:
    """--device cpu: the multi-rank plumbing on the CPU (gloo), for the
    world-size-2 test -- each rank checksums its own C3 shard with the scalar
    drop-in engine and checks it against the reference digest of that shard;
    the timing and aggregation are the GPU path's (combine_ranks)."""
    import torch.distributed as dist
    import zdbcrc
    result_out = sys.stdout  # one JSON line on stdout (see main)
    if world > 1:
        sys.stdout.flush()
        result_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        dist.init_process_group("gloo")
    target = int(args.gib * (1 << 30))
    offs, lens, seed, desc = make_dataset(args.workload, target, rank)
    arena = zdbcrc.synth_fill(int(offs[-1] + lens[-1]), seed)
    crcs = np.array([zdbcrc.crc32(arena[o:o + l]) for o, l in zip(offs, lens)], dtype=np.uint32)
    parity = parity_of(digest(crcs), shard_digest_ref("C3", rank, args.gib), f"C3 shard {rank}")
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for o, l in zip(offs, lens):
            zdbcrc.crc32(arena[o:o + l])
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    payload = int(lens.sum())
    elapsed, all_payload = combine_ranks(t1 - t0, payload, world)
    parities = gather_ranks(parity, world)
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(all_payload * args.steps / elapsed / GIB, 4), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic", "device": "cpu (plumbing test: scalar engine)",
            "config": {"workload": desc, "records_per_gpu": len(lens), "payload_bytes_per_gpu": payload,
                       "parallelism": f"{world} independent shards, no data-path collective"},
            "parity": summarize_parity(parities), "parity_by_rank": parities}), file=result_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="zipf", choices=["zipf", "fixed4k", "c2u"])
    ap.add_argument("--gib", type=float, default=4.0, help="batch size per GPU (GiB)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 integrity-scan leg")
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="untimed steps after the warmup until this many seconds have passed")
    ap.add_argument("--rehearsal", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share devices over gloo; the line says so)")
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"],
                    help="cpu: multi-rank plumbing test on gloo with the scalar engine (tests only)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {args.gpus}: refusing to measure "
                 "a different number of GPUs than asked for")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device == "cpu":
        cpu_rank(args, rank, world)
        return

    import torch
    import torch.distributed as dist
    import zdbcrc

    # one rank per GPU (the driver's N-GPU runs: RCCL for the barrier and the
    # max-over-ranks time; the path itself exchanges nothing).  More ranks than
    # GPUs -- a rehearsal of the N-rank plumbing on a one-GPU box -- share the
    # devices round-robin and use gloo, which allows that.
    ndev = torch.cuda.device_count()
    shared = world > ndev
    if shared and not args.rehearsal:
        # a --gpus N line from fewer than N devices would read as an N-GPU
        # weak-scaling result; only an explicit rehearsal may share devices
        sys.exit(f"bench.py: {world} ranks but {ndev} visible GPU(s): refusing to report a {world}-GPU result "
                 "(pass --rehearsal to run the N-rank plumbing on shared devices; the line is then marked)")
    local = local % max(ndev, 1)
    torch.cuda.set_device(local)
    # stdout carries exactly one JSON line: the communication libraries print
    # their connection chatter on fd 1 (gloo: "Rank 0 is connected to 1 peer
    # ranks"), so fd 1 goes to stderr and the result line to the original stdout
    result_out = sys.stdout
    if world > 1:
        sys.stdout.flush()
        result_out = os.fdopen(os.dup(1), "w")
        os.dup2(2, 1)
        if world <= ndev:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            log(f"rank {rank}: {world} ranks on {ndev} GPU(s): gloo, device {local} shared")
            dist.init_process_group("gloo")

    def barrier():
        if world > 1:
            dist.barrier()

    target = int(args.gib * (1 << 30))
    offs, lens, seed, desc = make_dataset(args.workload, target, rank)
    n = len(lens)
    total = int(offs[-1] + lens[-1])
    payload = int(lens.sum())
    log(f"rank {rank}/{world}: {desc}: {n} records, {payload} payload bytes")

    arena = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    zdbcrc.synth_fill_device(arena, seed)
    d_offs = torch.from_numpy(offs).cuda()
    d_lens = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")

    ml = 4096 if args.workload in ("fixed4k", "c2u") else None  # fixed 4 KiB values: the caller knows the bound

    def step():
        zdbcrc.batch_device(arena, d_offs, d_lens, out, max_length=ml)

    # parity at full size: every rank's shard against the reference's digest of it
    step()
    torch.cuda.synchronize()
    parity = workload_parity(args.workload, out, rank, args.gib)
    log(f"rank {rank} parity: {parity}")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # untimed settle: keep stepping until the clocks have ramped (a cold GPU
    # runs the first ~0.5 s of work up to 25 % slower; reported as settle_steps)
    settle = 0
    t_settle = time.perf_counter() + args.settle_s
    while time.perf_counter() < t_settle:
        for _ in range(4):
            step()
        settle += 4
        torch.cuda.synchronize()
    barrier()
    zdbcrc.kernel_stats()  # drop anything recorded so far
    zdbcrc.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    zdbcrc.set_timing(False)
    kern_ms, launches = zdbcrc.kernel_stats()

    elapsed, all_payload = combine_ranks(t1 - t0, payload, world)
    value = all_payload * args.steps / elapsed / GIB
    ms_per_step = elapsed / args.steps * 1e3

    avg_kernel_s = kern_ms / max(launches, 1) / 1e3
    alg_bytes = payload + 16 * n  # len + 8 B offset + 4 B length + 4 B crc
    achieved = alg_bytes / avg_kernel_s / 1e9
    traffic, traffic_src = pmc_traffic(args.workload)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": f"rocprofv3 --pmc FETCH_SIZE pass (separate run): {traffic_src}" if traffic else None,
                "kernel": "crc_batch_kernel", "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                "alg_bytes_per_launch": alg_bytes}

    extra = {}
    if rank == 0 and world == 1 and not args.no_extra:
        extra["read_ceiling"] = read_ceiling(arena, total, achieved)
    if not args.no_extra and not args.no_c4:
        del arena
        torch.cuda.empty_cache()
        log("C4 leg: integrity scan of 64 datafiles per GPU")
        extra["c4"] = c4_leg(rank, world, args.steps, args.warmup, args.settle_s / 2, barrier)
        arena = None
    if rank == 0 and world == 1 and not args.no_extra:
        for other in [w for w in ("zipf", "fixed4k", "c2u") if w != args.workload]:
            o2, l2, s2, d2 = make_dataset(other, target, 0)
            arena = None
            a2 = torch.empty(int(o2[-1] + l2[-1]) + 64, dtype=torch.uint8, device="cuda")
            zdbcrc.synth_fill_device(a2, s2)
            do2, dl2 = torch.from_numpy(o2).cuda(), torch.from_numpy(l2.astype(np.int32)).cuda()
            out2 = torch.empty(len(l2), dtype=torch.int32, device="cuda")
            # C2 / C2u: fixed 4 KiB values -- the caller knows the bound
            # (zdb_crc32_batch_device_sized picks the packed kernel, rows of 16 lanes)
            ml = 4096 if other in ("fixed4k", "c2u") else None
            t_settle = time.perf_counter() + args.settle_s / 2
            while time.perf_counter() < t_settle:
                for _ in range(4):
                    zdbcrc.batch_device(a2, do2, dl2, out2, max_length=ml)
                torch.cuda.synchronize()
            zdbcrc.kernel_stats()
            zdbcrc.set_timing(True)
            ta = time.perf_counter()
            for _ in range(args.steps):
                zdbcrc.batch_device(a2, do2, dl2, out2, max_length=ml)
            torch.cuda.synchronize()
            tb = time.perf_counter()
            zdbcrc.set_timing(False)
            km, kl = zdbcrc.kernel_stats()
            pb = int(l2.sum())
            # the output of the last timed step, at full size, against the reference
            p2 = workload_parity(other, out2, 0, args.gib)
            log(f"{other} parity: {p2}")
            t2, t2_src = pmc_traffic(other)
            extra[other] = {"desc": d2, "records": len(l2), "gibs": round(pb * args.steps / (tb - ta) / GIB, 2),
                            "shape": "packed kernel, rows of 16 lanes (max_length 4096)" if ml else "default",
                            "parity": p2, "kernel_ms": round(km / max(kl, 1), 4),
                            "roofline_frac": round((pb + 16 * len(l2)) / (km / max(kl, 1) / 1e3) / 1e9
                                                   / HBM_PEAK_GBS, 4),
                            "traffic": t2, "traffic_source": t2_src}
            del a2, do2, dl2, out2
            torch.cuda.empty_cache()

    if rank == 0 and world == 1 and not args.no_extra:
        log("end-to-end legs (host memory)")
        extra["e2e"] = e2e_legs(offs, lens, seed)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU baseline")
        cpu = cpu_baseline(offs, lens, seed, args.cpu_seconds)
        if not args.no_extra:
            extra["cpu_baseline_shapes"] = cpu_baseline_shapes(args.cpu_seconds / 2)

    parities = gather_ranks(parity, world)
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "physical_gpus": ndev, "shared_devices": shared,
            "steps": args.steps, "warmup": args.warmup, "settle_steps": settle,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes; SURVEY §8(d) Zipf sizes), resident in HBM",
            "config": {"workload": desc, "records_per_gpu": n, "payload_bytes_per_gpu": payload,
                       "parallelism": f"{world} independent shards, no data-path collective"},
            "parity": summarize_parity(parities), "parity_by_rank": parities, "roofline": roofline, "cpu_baseline": cpu, "extra": extra,
        }
        print(json.dumps(line), file=result_out, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
