"""World-size-2 `gloo` test (CPU) of bench.py's multi-rank plumbing: every
rank owns a distinct shard (rank 0 is the golden dataset), the job's time is
the slowest rank's, its bytes are the sum over ranks, and the per-shard
checksums need no exchange (the scalar drop-in engine stands in for the GPU
here; the GPU path is covered by tests/test_gpu.py)."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "0-db_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import zdbcrc
    offs, lens, seed, _ = bench.make_dataset("zipf", 4 << 20, rank)
    total = int(offs[-1] + lens[-1])
    arena = zdbcrc.synth_fill(total, seed)
    crcs = [zdbcrc.crc32(arena[o:o + l]) for o, l in zip(offs[:50], lens[:50])]
    elapsed = 1.0 + rank  # rank 1 is "slower"
    t, b = bench.combine_ranks(elapsed, int(lens.sum()), world)
    q.put((rank, seed, int(lens.sum()), len(lens), crcs[:3], t, b))
    dist.destroy_process_group()


def test_two_rank_shards_and_aggregation():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, s0, b0, n0, c0, t0, tot0), (r1, s1, b1, n1, c1, t1, tot1) = res
    assert s0 != s1 and c0 != c1                   # distinct shards
    assert t0 == t1 == 2.0                         # max over ranks
    assert tot0 == tot1 == float(b0 + b1)          # whole-job bytes
    import bench
    assert s0 == bench.C3_SEED                     # rank 0 == golden C3 recipe


def test_bench_spawns_its_own_ranks():
    """`python bench.py --gpus 2` started plainly (no torchrun) launches two
    rank processes itself; both check their own shard against the
    reference's digest of it, and rank 0 reports the whole job (n_gpus 2)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--device", "cpu",
                        "--gib", str(1 / 64), "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]  # only rank 0 prints, and only its JSON line (gloo chatter -> stderr)
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["parity_by_rank"] == ["bit-exact vs reference digest C3 shard 0",
                                   "bit-exact vs reference digest C3 shard 1"]
    assert d["parity"] == "bit-exact vs reference digests on all 2 shards"


def test_bench_refuses_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--device", "cpu"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode != 0 and "WORLD_SIZE=1" in p.stderr
