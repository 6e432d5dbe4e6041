"""f2 / a9: the SET path with two-phase batching (0-db_amd/bin/zdb-set-pipeline)
against the REFERENCE daemon: oracle/_ref/zdbd/zdb is zdbd compiled from the
reference sources (oracle/Makefile `zdbd`), run on a unix socket in user-key
mode; both get the same pipelined RESP stream -- new keys, overwrites,
re-SETs of identical values (the "$-1" path, commands_set.c:111-116),
empty values, an empty key, an over-long key, datafile rotation
(--datasize) -- and must give byte-identical replies and datafiles
(timestamps aside).  The harness's own datafiles then pass the reference
integrity-check.  CPU engine here; tests/test_gpu.py repeats it with the GPU
engine."""
from __future__ import annotations

import json
import os
import signal
import socket
import subprocess
import threading
import time
from pathlib import Path

import numpy as np
import pytest

import oracle
import zdbcrc
from conftest import ROOT

ZDBD = Path(oracle.__file__).resolve().parent / "_ref" / "zdbd" / "zdb"
HARNESS = ROOT / "0-db_amd" / "bin" / "zdb-set-pipeline"


def resp_set(key: bytes, value: bytes) -> bytes:
    return b"*3\r\n$3\r\nSET\r\n$%d\r\n%s\r\n$%d\r\n%s\r\n" % (len(key), key, len(value), value)


def build_stream(seed: int, n: int = 400):
    """pipelined SETs: sizes 0 B .. 96 KiB, ~1/4 overwrites, ~1/8 identical
    re-SETs, one empty key and one 300-byte key"""
    rng = np.random.default_rng(seed)
    keys = [b"key-%d" % i for i in range(n // 2)]
    last = {}
    out, nreq = [], 0
    for i in range(n):
        k = keys[int(rng.integers(len(keys)))]
        r = rng.random()
        if k in last and r < 0.125:
            v = last[k]  # identical payload: "$-1"
        else:
            size = int(rng.choice([0, 1, 17, 64, 500, 4096, 20000, 98304]))
            v = oracle.splitmix_bytes(size, seed * 1000 + i).tobytes()
        last[k] = v
        out.append(resp_set(k, v))
        nreq += 1
        if i == n // 3:
            out.append(resp_set(b"", b"orphan"))
            out.append(resp_set(b"x" * 300, b"too long a key"))
            nreq += 2
    return b"".join(out), nreq


def build_stream_large(seed: int, n: int = 24):
    """pipelined SETs of large values up to the maximum payload
    (ZDB_DATA_MAX_PAYLOAD, libzdb/data.h:6 = 8 MiB): overwrites, identical
    re-SETs and small values in between"""
    rng = np.random.default_rng(seed)
    keys = [b"big-%d" % i for i in range(n // 3)]
    last = {}
    out = []
    for i in range(n):
        k = keys[int(rng.integers(len(keys)))]
        if k in last and rng.random() < 0.2:
            v = last[k]
        else:
            size = int(rng.choice([0, 100, 1 << 20, (3 << 20) + 7, 8 << 20]))
            v = oracle.splitmix_bytes(size, seed * 1000 + i).tobytes()
        last[k] = v
        out.append(resp_set(k, v))
    return b"".join(out), n


def read_replies(data: bytes, count: int):
    """split RESP replies ($-1, $n + bulk, -error); None if incomplete"""
    out, p = [], 0
    while len(out) < count:
        e = data.find(b"\r\n", p)
        if e < 0:
            return None
        line = data[p:e]
        if line.startswith(b"$") and line != b"$-1":
            n = int(line[1:])
            if len(data) < e + 2 + n + 2:
                return None
            out.append(data[p:e + 2 + n + 2])
            p = e + 2 + n + 2
        else:
            out.append(data[p:e + 2])
            p = e + 2
    return out


def run_reference_zdbd(stream: bytes, nreq: int, tmp: Path, datasize: int):
    d, i, sock = tmp / "zdata", tmp / "zindex", tmp / "zdb.sock"
    proc = subprocess.Popen([str(ZDBD), "--data", str(d), "--index", str(i), "--socket", str(sock),
                             "--mode", "user", "--datasize", str(datasize)],
                            stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    try:
        t_end = time.time() + 20
        while not sock.exists():
            assert proc.poll() is None and time.time() < t_end, "reference zdbd did not start"
            time.sleep(0.02)
        c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        c.connect(str(sock))
        sender = threading.Thread(target=c.sendall, args=(stream,))
        sender.start()
        buf = b""
        t_end = time.time() + 60
        while True:
            reps = read_replies(buf, nreq)
            if reps is not None:
                break
            assert time.time() < t_end, "reference zdbd replies timed out"
            chunk = c.recv(1 << 20)
            assert chunk, "reference zdbd closed the connection"
            buf += chunk
        sender.join()
        c.close()
    finally:
        proc.send_signal(signal.SIGINT)
        try:
            proc.wait(timeout=10)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
    files = {p.name: p.read_bytes() for p in sorted((d / "default").glob("d*"))}
    return reps, files


def run_harness(stream: bytes, tmp: Path, datasize: int, engine: str = "cpu", batch: int = 64,
                from_file: bool = False):
    """from_file: the stream is stdin as a regular file, so one read takes all
    of it and batches are bounded by --batch alone (a pipe hands over 64 KiB
    at a time)"""
    out = tmp / f"harness_{engine}_{batch}"
    args = [str(HARNESS), f"--engine={engine}", f"--datasize={datasize}", f"--batch={batch}", "--stats", str(out)]
    if from_file:
        src = tmp / f"stream_{engine}_{batch}"
        src.write_bytes(stream)
        with open(src, "rb") as f:
            p = subprocess.run(args, stdin=f, capture_output=True, timeout=120)
    else:
        p = subprocess.run(args, input=stream, capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    files = {q.name: q.read_bytes() for q in sorted(out.glob("d*"))}
    return p.stdout, files, p.stderr.decode()


def without_clock(img: bytes) -> bytes:
    """zero the wall-clock fields: data_header_t created/opened and every
    entry's timestamp"""
    b = bytearray(img)
    b[8:24] = bytes(16)
    recs, _ = zdbcrc.datafile_walk(img)
    for h in recs["header_offset"]:
        b[int(h) + 14:int(h) + 18] = bytes(4)
    return bytes(b)


needs_ref = pytest.mark.skipif(not ZDBD.exists(), reason="make -C oracle zdbd (needs /root/reference)")


@needs_ref
@pytest.mark.parametrize("datasize,batch", [(256 << 20, 64), (600_000, 7), (600_000, 4096)])
def test_set_pipeline_matches_reference_daemon(tmp_path, datasize, batch):
    stream, nreq = build_stream(3 + datasize % 7)
    reps, ref_files = run_reference_zdbd(stream, nreq, tmp_path, datasize)
    out, files, _ = run_harness(stream, tmp_path, datasize, "cpu", batch)
    assert out == b"".join(reps)
    assert sorted(files) == sorted(ref_files)
    if datasize < (1 << 20):
        assert len(files) > 2  # rotation happened
    for name in files:
        assert without_clock(files[name]) == without_clock(ref_files[name]), name
    assert b"$-1\r\n" in out and b"-Key too large\r\n" in out and b"-Invalid argument, key needed\r\n" in out


@needs_ref
def test_set_pipeline_large_values_match_reference_daemon(tmp_path):
    """values up to the 8 MiB maximum, with datafile rotation between them"""
    stream, nreq = build_stream_large(5)
    reps, ref_files = run_reference_zdbd(stream, nreq, tmp_path, 20 << 20)
    out, files, _ = run_harness(stream, tmp_path, 20 << 20, "cpu", 16)
    assert out == b"".join(reps)
    assert sorted(files) == sorted(ref_files) and len(files) > 1
    for name in files:
        assert without_clock(files[name]) == without_clock(ref_files[name]), name


@needs_ref
def test_set_pipeline_datafiles_pass_reference_tool(tmp_path):
    stream, _ = build_stream(11)
    _, files, _ = run_harness(stream, tmp_path, 600_000, "cpu", 32)
    for name, img in files.items():
        d = tmp_path / f"chk_{name}"
        d.mkdir()
        (d / "d0").write_bytes(img)
        os.symlink("d0", d / "zdb-data-0")
        p = subprocess.run([str(oracle.REF_INTEGRITY), str(d / "zdb-data-0")], capture_output=True, timeout=60)
        assert p.returncode == 0 and b"integrity check failed" not in p.stderr, name


def test_set_pipeline_rejects_other_commands(tmp_path):
    stream = resp_set(b"a", b"b") + b"*2\r\n$3\r\nGET\r\n$1\r\na\r\n"
    p = subprocess.run([str(HARNESS), "--engine=cpu", str(tmp_path / "d")], input=stream, capture_output=True,
                       timeout=60)
    assert p.returncode == 2 and p.stdout == b"$1\r\na\r\n"


@needs_ref
def test_set_pipeline_auto_engine_without_gpu(tmp_path):
    """--engine=auto with no usable GPU (this container): the scalar engine
    alone, same replies and datafiles as the reference daemon"""
    stream, nreq = build_stream(17)
    reps, ref_files = run_reference_zdbd(stream, nreq, tmp_path, 600_000)
    out, files, stats = run_harness(stream, tmp_path, 600_000, "auto", 64, from_file=True)
    assert out == b"".join(reps)
    assert sorted(files) == sorted(ref_files)
    for name in files:
        assert without_clock(files[name]) == without_clock(ref_files[name]), name
    st = json.loads(stats.strip().splitlines()[-1])
    assert st["engine"] in ("cpu", "auto")  # "cpu": no usable GPU, the scalar engine alone
    if st["engine"] == "cpu":
        assert st["gpu_batches"] == 0
