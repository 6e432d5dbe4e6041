#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC32 (0-db zdb_crc32) on MI355X.

One step = one zdb_crc32_batch_device call (plan scan + kernel) over the
whole per-GPU batch, inputs already resident in HBM.  Default workload is
BASELINE.json configs[2] / SURVEY §8(d) C3: Zipf-mixed records 64 B..1 MiB,
packed back to back at arbitrary byte alignment, ~4 GiB per GPU.  Each rank
checksums its own batch (different seed): weak scaling, no collective on the
data path (torch.distributed is used only for the barrier and the max/sum of
the timing).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload zipf|fixed4k]
  (N > 1: launched by torch.distributed.run, one rank per GPU)

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
    else:
        raise SystemExit(f"unknown workload {workload}")
    return offs, lens, seed, desc


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
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1))
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
            "single_thread_gibs": round(st, 3)}


def e2e_legs(offs, lens, seed) -> dict:
    """Host-memory paths, reported beside the
    device-resident number: the SET path's 256 KiB value through the
    host-buffer entry (pinned staging, H2D + kernel + D2H), the zipf batch
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
        tools = {"gpu_tool": [str(ROOT / "0-db_amd/bin/zdb-integrity-check"), f"{td}/zdb-data-0"],
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


def pmc_traffic(workload: str):
    p = ROOT / "profiles" / "pmc_traffic.json"
    if not p.exists():
        return None
    try:
        d = json.loads(p.read_text())
        return d.get(workload, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="zipf", choices=["zipf", "fixed4k"])
    ap.add_argument("--gib", type=float, default=4.0, help="batch size per GPU (GiB)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    ap.add_argument("--settle-s", type=float, default=1.0,
                    help="untimed steps after the warmup until this many seconds have passed")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist
    import zdbcrc

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

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

    def step():
        zdbcrc.batch_device(arena, d_offs, d_lens, out)

    # parity at full size: rank 0's batch is the golden dataset
    step()
    torch.cuda.synchronize()
    parity = "unchecked"
    gold = ROOT / "tests" / "golden" / "digests.json"
    if rank == 0 and gold.exists():
        key = "C3" if args.workload == "zipf" else "C2"
        ref = json.loads(gold.read_text()).get(key)
        got = digest(out.cpu().numpy().view(np.uint32))
        if ref and abs(args.gib - 4.0) < 1e-9:
            ok = all(got[k] == ref[k] for k in ("count", "xor", "crc_of_crcs"))
            parity = f"bit-exact vs reference digest {key}" if ok else f"MISMATCH {got} vs {ref}"
            log(f"parity: {parity}")

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
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(args.workload),
                "kernel": "crc_batch_kernel", "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                "alg_bytes_per_launch": alg_bytes}

    extra = {}
    if rank == 0 and world == 1 and not args.no_extra:
        other = "fixed4k" if args.workload == "zipf" else "zipf"
        o2, l2, s2, d2 = make_dataset(other, target, 0)
        del arena
        a2 = torch.empty(int(o2[-1] + l2[-1]) + 64, dtype=torch.uint8, device="cuda")
        zdbcrc.synth_fill_device(a2, s2)
        do2, dl2 = torch.from_numpy(o2).cuda(), torch.from_numpy(l2.astype(np.int32)).cuda()
        out2 = torch.empty(len(l2), dtype=torch.int32, device="cuda")
        t_settle = time.perf_counter() + args.settle_s / 2
        while time.perf_counter() < t_settle:
            for _ in range(4):
                zdbcrc.batch_device(a2, do2, dl2, out2)
            torch.cuda.synchronize()
        zdbcrc.kernel_stats()
        zdbcrc.set_timing(True)
        ta = time.perf_counter()
        for _ in range(args.steps):
            zdbcrc.batch_device(a2, do2, dl2, out2)
        torch.cuda.synchronize()
        tb = time.perf_counter()
        zdbcrc.set_timing(False)
        km, kl = zdbcrc.kernel_stats()
        pb = int(l2.sum())
        extra[other] = {"desc": d2, "records": len(l2), "gibs": round(pb * args.steps / (tb - ta) / GIB, 2),
                        "kernel_ms": round(km / max(kl, 1), 4),
                        "roofline_frac": round((pb + 16 * len(l2)) / (km / max(kl, 1) / 1e3) / 1e9
                                               / HBM_PEAK_GBS, 4)}
        del a2

    if rank == 0 and world == 1 and not args.no_extra:
        log("end-to-end legs (host memory)")
        extra["e2e"] = e2e_legs(offs, lens, seed)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU baseline")
        cpu = cpu_baseline(offs, lens, seed, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "settle_steps": settle,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 bytes; SURVEY §8(d) Zipf sizes), resident in HBM",
            "config": {"workload": desc, "records_per_gpu": n, "payload_bytes_per_gpu": payload,
                       "parallelism": f"{world} independent shards, no data-path collective"},
            "parity": parity, "roofline": roofline, "cpu_baseline": cpu, "extra": extra,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
