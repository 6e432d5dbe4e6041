"""GPU parity tests: the HIP path (through the C ABI) against the oracle and
the reference-generated golden fixtures.  Bit-exact everywhere (integer
work).  Run on an MI355X with `pytest -m gpu`."""
from __future__ import annotations

import os
import sys
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, ROOT, kat_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible to torch (tests marked gpu must run on the MI355X box)")
    import zdbcrc
    return zdbcrc


def gpu_batch(zdbcrc, arena: np.ndarray, offs, lens, pad: int = 64) -> np.ndarray:
    a = torch.zeros(len(arena) + pad, dtype=torch.uint8, device="cuda")
    if len(arena):
        a[: len(arena)] = torch.from_numpy(np.ascontiguousarray(arena)).cuda()
    o = torch.from_numpy(np.asarray(offs, dtype=np.int64)).cuda()
    l = torch.from_numpy(np.asarray(lens, dtype=np.int64).astype(np.int32)).cuda()
    out = torch.full((len(o),), -1, dtype=torch.int32, device="cuda")
    zdbcrc.batch_device(a, o, l, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_engine_binds(dev):
    gpu_batch(dev, np.zeros(16, np.uint8), [0], [16])
    assert dev.batch_engine() == "hip-gfx950"
    assert dev.gpu_initialized()


def test_known_answers(dev, kats):
    blobs = [kat_bytes(e) for e in kats]
    offs, pos = [], 0
    for b in blobs:
        offs.append(pos)
        pos += len(b) + 5  # odd gaps: every record at a different alignment
    arena = np.zeros(pos, np.uint8)
    for o, b in zip(offs, blobs):
        arena[o:o + len(b)] = np.frombuffer(b, np.uint8)
    got = gpu_batch(dev, arena, offs, [len(b) for b in blobs])
    for e, g in zip(kats, got):
        assert g == int(e["crc"], 16), e["name"]


def test_vectors_every_alignment(dev, vectors):
    """1546 reference vectors (0..4160 B and up to 1 MiB), each placed at all
    16 start alignments in one batch."""
    lens, seeds, crcs = vectors
    offs, blobs, pos = [], [], 0
    for n, s in zip(lens, seeds):
        data = oracle.splitmix_bytes(int(n), int(s))
        for mis in range(16):
            pos = (pos + 15) // 16 * 16 + mis
            offs.append(pos)
            blobs.append(data)
            pos += int(n)
    arena = np.zeros(pos + 16, np.uint8)
    for o, b in zip(offs, blobs):
        arena[o:o + len(b)] = b
    got = gpu_batch(dev, arena, offs, [len(b) for b in blobs])
    np.testing.assert_array_equal(got, np.repeat(crcs, 16))


@pytest.mark.parametrize("seed,nrec,maxlen", [(1, 3000, 200), (2, 2000, 5000), (3, 400, 70_000),
                                              (4, 40, 3_000_000), (5, 1, 8 << 20)])
def test_random_batches(dev, oracle_c, seed, nrec, maxlen):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen + 1, nrec)
    span = int(lens.sum()) // 2 + maxlen + 1
    arena = oracle.splitmix_bytes(span, seed)
    offs = np.array([rng.integers(0, span - l + 1) for l in lens])  # overlapping records
    np.testing.assert_array_equal(gpu_batch(dev, arena, offs, lens), oracle_c.batch(arena, offs, lens))


def test_record_relative_grid(dev, oracle_c):
    """1 KiB-multiple records at misaligned addresses (the 4 KiB value after a
    26-byte datafile header) take the record-relative piece grid and
    byte-misaligned loads; mixed with records of nearby lengths that keep the
    aligned grid, cut across many waves."""
    rng = np.random.default_rng(31)
    base = [1024, 2048, 4096, 8192, 65536, 1 << 20]
    lens = np.concatenate([rng.choice(base, 3000), rng.choice([4080, 4095, 4097, 4112, 1008, 16], 600)])
    rng.shuffle(lens)
    gaps = rng.integers(0, 40, len(lens))
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1] + gaps[:-1])
    offs += 26
    arena = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 16, 31)
    np.testing.assert_array_equal(gpu_batch(dev, arena, offs, lens), oracle_c.batch(arena, offs, lens))


def test_overlapping_and_empty(dev, oracle_c):
    arena = oracle.splitmix_bytes(100_000, 77)
    offs = [0, 0, 1, 0, 50_000, 99_999, 12_345, 12_345]
    lens = [100_000, 0, 99_999, 1, 0, 1, 65_536, 65_537]
    np.testing.assert_array_equal(gpu_batch(dev, arena, offs, lens), oracle_c.batch(arena, offs, lens))


def test_split_heavy_geometry(dev, oracle_c):
    """One huge record among thousands of tiny ones: forces slices of the unit
    space to cut records (atomic XOR recombination) and tiny-record walks."""
    rng = np.random.default_rng(9)
    lens = np.concatenate([rng.integers(1, 64, 20_000), [7 << 20], rng.integers(1, 300, 5000)])
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1])
    arena = oracle.splitmix_bytes(int(lens.sum()), 10)
    np.testing.assert_array_equal(gpu_batch(dev, arena, offs, lens), oracle_c.batch(arena, offs, lens))


def test_device_arena_unaligned_base(dev, oracle_c):
    arena = oracle.splitmix_bytes(300_000, 12)
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 20_000, 200)
    offs = np.array([rng.integers(0, 300_000 - l - 8) for l in lens])
    a = torch.zeros(300_064, dtype=torch.uint8, device="cuda")
    a[3:300_003] = torch.from_numpy(arena).cuda()
    view = a[3:]  # data_ptr() = base + 3
    o = torch.from_numpy(offs.astype(np.int64)).cuda()
    l = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.zeros(len(offs), dtype=torch.int32, device="cuda")
    dev.batch_device(view, o, l, out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), oracle_c.batch(arena, offs, lens))


def test_verify_reports_mismatches(dev, oracle_c):
    arena = oracle.splitmix_bytes(200_000, 13)
    rng = np.random.default_rng(13)
    lens = rng.integers(1, 3000, 500)
    offs = np.array([rng.integers(0, 200_000 - l) for l in lens])
    exp = oracle_c.batch(arena, offs, lens)
    bad = [3, 77, 499]
    exp_t = exp.copy()
    exp_t[bad] ^= 1
    a = torch.from_numpy(arena).cuda()
    o = torch.from_numpy(offs.astype(np.int64)).cuda()
    l = torch.from_numpy(lens.astype(np.int32)).cuda()
    e = torch.from_numpy(exp_t.view(np.int32)).cuda()
    out = torch.zeros(500, dtype=torch.int32, device="cuda")
    mism = torch.zeros(16, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    dev.verify_device(a, o, l, e, out, mism, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 3
    assert sorted(mism[:3].cpu().tolist()) == bad
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)


def test_verify_more_mismatches_than_room(dev, oracle_c):
    """more mismatching records (300) than the mismatch list holds (16): the
    count is the full count, the list holds 16 distinct mismatching indices,
    and nothing is written past it"""
    arena = oracle.splitmix_bytes(400_000, 21)
    rng = np.random.default_rng(21)
    lens = rng.integers(0, 3000, 5000)
    offs = np.array([rng.integers(0, 400_000 - l) for l in lens])
    exp = oracle_c.batch(arena, offs, lens)
    bad = np.sort(rng.choice(5000, 300, replace=False))
    exp_t = exp.copy()
    exp_t[bad] ^= 0x80000000
    a = torch.from_numpy(arena).cuda()
    o = torch.from_numpy(offs.astype(np.int64)).cuda()
    l = torch.from_numpy(lens.astype(np.int32)).cuda()
    e = torch.from_numpy(exp_t.view(np.int32)).cuda()
    out = torch.zeros(5000, dtype=torch.int32, device="cuda")
    guard = torch.full((32,), -7, dtype=torch.int32, device="cuda")
    mism = guard[:16]
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    dev.verify_device(a, o, l, e, out, mism, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 300
    listed = guard[:16].cpu().numpy()
    assert len(set(listed.tolist())) == 16 and set(listed.tolist()) <= set(bad.tolist())
    assert (guard[16:].cpu().numpy() == -7).all()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)


def test_host_buffer_api(dev, oracle_c):
    arena = oracle.splitmix_bytes(1 << 20, 14)
    rng = np.random.default_rng(14)
    lens = rng.integers(0, 100_000, 64)
    offs = np.array([rng.integers(0, (1 << 20) - l) for l in lens])
    np.testing.assert_array_equal(dev.batch_host(arena, offs, lens), oracle_c.batch(arena, offs, lens))


def test_set_path_256k_value(dev, oracle_c):
    """C5: one 256 KiB value through the host-buffer entry (pinned staging)."""
    buf = dev.PinnedBuffer(256 * 1024)
    buf.array[:] = oracle.splitmix_bytes(256 * 1024, 15)
    got = dev.batch_host(buf.array, [0], [256 * 1024])
    assert got[0] == oracle_c.crc32(buf.array)
    buf.free()


def test_synth_device_matches_host(dev):
    t = torch.empty(1 << 20 | 5, dtype=torch.uint8, device="cuda")
    dev.synth_fill_device(t, 0xFEED)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(t.cpu().numpy(), oracle.splitmix_bytes(t.numel(), 0xFEED))


def _digest(ref_crc, crcs: np.ndarray):
    return {"count": len(crcs), "xor": f"{int(np.bitwise_xor.reduce(crcs)):08x}",
            "crc_of_crcs": f"{ref_crc(crcs.astype('<u4').tobytes()):08x}"}


def test_full_size_c2_digest(dev, oracle_c, digests):
    """C2 at BASELINE size (1 Mi x 4 KiB = 4 GiB), bit-exact vs the digest of
    the reference's own crcs."""
    d = digests["C2"]
    n = d["records"]
    arena = torch.empty(n * 4096, dtype=torch.uint8, device="cuda")
    dev.synth_fill_device(arena, d["seed"])
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * 4096
    lens = torch.full((n,), 4096, dtype=torch.int32, device="cuda")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    dev.batch_device(arena, offs, lens, out)
    torch.cuda.synchronize()
    got = _digest(oracle_c.crc32, out.cpu().numpy().view(np.uint32))
    assert got == {k: d[k] for k in ("count", "xor", "crc_of_crcs")}
    del arena


@pytest.mark.parametrize("workload", ["fixed4k", "c2u"])
@pytest.mark.parametrize("max_length", [None, 4096])
def test_full_size_small_record_digests(dev, oracle_c, digests, workload, max_length):
    """C2 (4 KiB-aligned) and C2u (4 KiB payloads behind 26-byte datafile
    headers, byte-misaligned: SURVEY §8(d)) at full size, 1 Mi records each,
    in BOTH kernels the library carries for them -- the main kernel and the
    packed kernel (rows of 16 lanes) that zdb_crc32_batch_device_sized picks
    for max_length <= 4096, i.e. the shape bench.py times for these workloads --
    bit-exact vs the reference's digest (make_golden.py --only-c2u)."""
    sys.path.insert(0, str(ROOT))
    import bench
    d = digests["C2" if workload == "fixed4k" else "C2u"]
    offs, lens, seed, _ = bench.make_dataset(workload, 4 << 30, 0)
    assert seed == d["seed"] and len(lens) == d["count"]
    total = int(offs[-1] + lens[-1])
    arena = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    dev.synth_fill_device(arena[:total], seed)
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    dev.batch_device(arena, torch.from_numpy(offs).cuda(), torch.from_numpy(lens.astype(np.int32)).cuda(), out,
                     max_length=max_length)
    torch.cuda.synchronize()
    got = _digest(oracle_c.crc32, out.cpu().numpy().view(np.uint32))
    assert got == {k: d[k] for k in ("count", "xor", "crc_of_crcs")}
    del arena


@pytest.mark.parametrize("bound", [512, 2048, 4096])
def test_packed_shapes_at_scale(dev, oracle_c, bound):
    """each packed shape (rows of 4 / 8 / 16 lanes) on 512 MiB of C3's own
    record sizes up to its bound (Zipf, tiled; records at every alignment):
    equal to the default kernel on every record, and to the oracle on a
    sample of 20,000 records spread over the batch"""
    base = dev.zipf_lengths(4 << 30, 0xC3C3C3).astype(np.int64)
    base = base[base <= bound]
    size = 512 << 20
    lens = np.tile(base, -(-size // int(base.sum())))
    lens = lens[:int(np.searchsorted(np.cumsum(lens), size))]
    rng = np.random.default_rng(bound)
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 4, len(lens) - 1))
    total = int(offs[-1] + lens[-1])
    arena = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    dev.synth_fill_device(arena[:total], 0x5EED + bound)
    o = torch.from_numpy(offs).cuda()
    l = torch.from_numpy(lens.astype(np.int32)).cuda()
    packed = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    default = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    dev.batch_device(arena, o, l, packed, max_length=bound)
    dev.batch_device(arena, o, l, default)
    torch.cuda.synchronize()
    got = packed.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, default.cpu().numpy().view(np.uint32))
    host = dev.synth_fill(total, 0x5EED + bound)
    pick = np.unique(np.linspace(0, len(lens) - 1, 20_000).astype(np.int64))
    np.testing.assert_array_equal(got[pick], oracle_c.batch(host, offs[pick], lens[pick]))
    del arena


def test_full_size_c3_digest(dev, oracle_c, digests):
    """C3 at BASELINE size (Zipf 64 B..1 MiB, ~4 GiB, any alignment)."""
    d = digests["C3"]
    lens = dev.zipf_lengths(d["target"], d["len_seed"])
    assert len(lens) == d["count"] and int(lens.sum()) == d["total_bytes"]
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1].astype(np.int64))
    arena = torch.empty(d["total_bytes"] + 64, dtype=torch.uint8, device="cuda")
    dev.synth_fill_device(arena[: d["total_bytes"]], d["seed"])
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    dev.batch_device(arena, torch.from_numpy(offs).cuda(), torch.from_numpy(lens.view(np.int32)).cuda(),
                     out)
    torch.cuda.synchronize()
    got = _digest(oracle_c.crc32, out.cpu().numpy().view(np.uint32))
    assert got == {k: d[k] for k in ("count", "xor", "crc_of_crcs")}


def test_max_sizes_digest(dev, oracle_c, digests):
    """The interface's size limits on a 4.5 GiB device arena: one record of
    2^32 - 1 bytes (the largest u32 length: every wave of the grid cuts it,
    the tail pool is off for it), an 8 MiB payload past the 4 GiB offset mark,
    a record straddling that mark, an empty one, one ending at the arena's
    last byte, 5,000 small ones beyond 4 GiB -- against the reference's crcs
    (tests/golden/make_golden.py --only-max, pinned by the oracle as well)"""
    sys.path.insert(0, str(GOLDEN))
    from make_golden import max_case
    d = digests["MAX"]
    total, offs, lens = max_case()
    assert total == d["total_bytes"]
    arena = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    dev.synth_fill_device(arena[:total], d["seed"])
    out = torch.empty(len(lens), dtype=torch.int32, device="cuda")
    dev.batch_device(arena, torch.from_numpy(offs.view(np.int64)).cuda(),
                     torch.from_numpy(lens.view(np.int32)).cuda(), out)
    torch.cuda.synchronize()
    crcs = out.cpu().numpy().view(np.uint32)
    assert [f"{int(c):08x}" for c in crcs[:5]] == d["first"]
    assert _digest(oracle_c.crc32, crcs) == {k: d[k] for k in ("count", "xor", "crc_of_crcs")}
    del arena


def test_repeat_is_deterministic(dev):
    arena = oracle.splitmix_bytes(3 << 20, 16)
    rng = np.random.default_rng(16)
    lens = rng.integers(0, 1 << 20, 50)
    offs = np.array([rng.integers(0, (3 << 20) - l) for l in lens])
    a = gpu_batch(dev, arena, offs, lens)
    for _ in range(3):
        np.testing.assert_array_equal(gpu_batch(dev, arena, offs, lens), a)


def _tail_pool_batch(seed: int, big: int):
    """~450 MB batch, above the tail pool's size threshold (4096 units per
    wave): 60k empty records first (their static slices hold no segment, so
    those waves start in the pool), mixed sizes, one `big` record."""
    rng = np.random.default_rng(seed)
    lens = np.concatenate([np.zeros(60_000, np.int64), rng.integers(0, 256 << 10, 3000), [big],
                           rng.integers(0, 5000, 20_000)])
    gaps = rng.integers(0, 24, len(lens))
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1] + gaps[:-1])
    offs += 5
    arena = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 16, seed)
    return arena, offs, lens


def test_tail_pool_batches(dev, oracle_c):
    """The default kernel's tail pool (chunks claimed by atomic counters whose
    launch parity alternates): A (largest record 512 KiB, pool on: < 64 chunks of ≈ 600 units) and B (one
    64 MiB record: more chunks than the guard allows per record, pool off),
    launched alternately so each counter parity is reused, bit-exact every time."""
    cases = [_tail_pool_batch(41, 512 << 10), _tail_pool_batch(42, 64 << 20)]
    want = [oracle_c.batch(a, o, l) for a, o, l in cases]
    for _ in range(2):
        for (a, o, l), w in zip(cases, want):
            np.testing.assert_array_equal(gpu_batch(dev, a, o, l), w)


# ------------------------------------------------------ integrity tool ------

TOOL_CASES = ["mixed", "zipf_small", "fixed_4k", "corrupt_payload", "corrupt_crc", "multi_errors",
              "truncated_payload", "truncated_header", "bad_magic", "bad_version", "header_only"]


NO_PAYLOAD_CASES = {"bad_magic", "bad_version", "header_only"}  # the tool never reaches a checksum


def split_trace(err):
    """(stderr without the ZDBCRC_TOOL_TRACE lines, the checksum engines those lines name)"""
    text = err if isinstance(err, str) else err.decode()
    lines = text.splitlines(keepends=True)
    engines = [ln.split("checksum engine ")[1].split(",")[0] for ln in lines if "checksum engine " in ln]
    rest = "".join(ln for ln in lines if not ln.startswith("[trace]"))
    return (rest if isinstance(err, str) else rest.encode()), engines


@pytest.mark.parametrize("engine", ["hip", "auto"])
@pytest.mark.parametrize("name", TOOL_CASES)
def test_tool_gpu_engine_matches_reference(tmp_path, datafile_cases, name, engine, monkeypatch):
    """every golden datafile through the GPU engine (auto: with the GPU
    start-up forced and waited for) -- and the tool's trace proves that the
    HIP engine did the checksum"""
    from test_tool_cpu import expected, run_tool
    monkeypatch.setenv("ZDBCRC_AUTO_START_GPU", "1")  # auto: start the GPU even for a small scan, and wait for it
    monkeypatch.setenv("ZDBCRC_TOOL_TRACE", "1")
    out, err, code = run_tool(name, tmp_path, engine)
    err, engines = split_trace(err)
    eout, eerr = expected(name)
    assert out == eout
    assert err == eerr
    assert code == {c["name"]: c for c in datafile_cases}[name]["exit"]
    assert engines == ([] if name in NO_PAYLOAD_CASES else ["hip"])


@pytest.fixture(scope="module")
def big_datafile(tmp_path_factory):
    """a 256 MiB datafile (65,000 x 4 KiB values) written through
    the reference libzdb (oracle/_ref/gen_datafile_ref), three payload bytes
    flipped, and the reference integrity-check's output on it"""
    if not (oracle.REF_GEN.exists() and oracle.REF_INTEGRITY.exists()):
        pytest.skip("oracle/_ref not built")
    d = tmp_path_factory.mktemp("big")
    subprocess.run([str(oracle.REF_GEN), str(d), "fixed", "65000", "99", "4096"], check=True, capture_output=True)
    d0 = d / "data" / "default" / "d0"
    img = bytearray(d0.read_bytes())
    import zdbcrc
    recs, _ = zdbcrc.datafile_walk(bytes(img))
    for k in (17, 30_000, 64_999):
        img[int(recs["payload_offset"][k]) + 100] ^= 0x21
    d0.write_bytes(bytes(img))
    os.symlink("d0", d / "data" / "default" / "zdb-data-0")
    p = subprocess.run([str(oracle.REF_INTEGRITY), str(d / "data" / "default" / "zdb-data-0")], capture_output=True,
                       env=dict(os.environ, TZ="UTC"), timeout=120)
    assert p.returncode == 3
    return d / "data" / "default" / "zdb-data-0", p


@pytest.mark.parametrize("engine", ["hip", "auto"])
def test_tool_gpu_256MiB_matches_reference(big_datafile, engine):
    """the GPU tool on a reference-written 256 MiB datafile (three corrupt
    payloads): stdout, stderr and exit status of the reference tool (auto: with
    its own start-up policy, i.e. the scalar engine for one 256 MiB file)"""
    import re
    path, ref = big_datafile
    from test_tool_cpu import TOOL
    p = subprocess.run([str(TOOL), f"--engine={engine}", str(path)], capture_output=True,
                       env=dict(os.environ, TZ="UTC", ZDBCRC_TOOL_TRACE="1"), timeout=120)
    t = re.compile(rb"\[\s*\d+\.\d{6}\]")
    err, engines = split_trace(p.stderr)
    assert p.returncode == ref.returncode == 3
    assert t.sub(b"[T]", p.stdout) == t.sub(b"[T]", ref.stdout)
    assert err == ref.stderr
    # hip: the GPU did it; auto: one 256 MiB file is below the start-up policy's threshold
    assert engines == (["hip"] if engine == "hip" else ["cpu"])
    if engine == "hip":  # f1: the file buffer was pinned in place and went over in one direct DMA
        assert b"buffer pinned: yes" in p.stderr


def test_tool_gpu_pinned_streaming_ingest(big_datafile):
    """f1 ingest: one worker, the same 256 MiB datafile three times -- once the
    GPU is up, the worker's buffer is pinned in place and every 32 MiB read is
    streamed to the device as a direct DMA while the next is read (trace:
    streamed, buffer pinned); the reports are the reference's, three times"""
    import re
    path, ref = big_datafile
    from test_tool_cpu import TOOL
    p = subprocess.run([str(TOOL), "--engine=hip", "--jobs=1", str(path), str(path), str(path)], capture_output=True,
                       env=dict(os.environ, TZ="UTC", ZDBCRC_TOOL_TRACE="1"), timeout=120)
    t = re.compile(rb"\[\s*\d+\.\d{6}\]")
    err, engines = split_trace(p.stderr)
    assert p.returncode == 9  # 3 corrupt payloads per file
    assert t.sub(b"[T]", p.stdout) == t.sub(b"[T]", ref.stdout) * 3
    assert err == ref.stderr * 3
    assert engines == ["hip"] * 3
    files = [ln for ln in p.stderr.decode().splitlines() if ln.startswith("[trace]") and "buffer pinned" in ln]
    assert len(files) == 3
    assert all("buffer pinned: yes" in ln for ln in files)
    assert "streamed: yes" in files[-1]  # the GPU was up before the last file's first read


@pytest.fixture(scope="module", params=["max8MiB", "zipf160MiB"])
def large_value_datafile(request, tmp_path_factory):
    """reference-written datafiles of large values: 24 values of exactly
    ZDB_DATA_MAX_PAYLOAD (libzdb/data.h:6, 8 MiB) and a 160 MiB SURVEY §8(d)
    C3 mix (up to 1 MiB per value); payload bytes flipped at the first byte,
    the last byte and inside of several values, including the largest; the
    reference integrity-check's output on each"""
    if not (oracle.REF_GEN.exists() and oracle.REF_INTEGRITY.exists()):
        pytest.skip("oracle/_ref not built")
    d = tmp_path_factory.mktemp(request.param)
    if request.param == "max8MiB":
        args = ["fixed", "24", "7", str(8 << 20)]
    else:
        args = ["zipf", "1000000", "8", str(160 << 20)]
    subprocess.run([str(oracle.REF_GEN), str(d), *args], check=True, capture_output=True)
    d0 = d / "data" / "default" / "d0"
    img = bytearray(d0.read_bytes())
    import zdbcrc
    recs, _ = zdbcrc.datafile_walk(bytes(img))
    off = recs["payload_offset"].astype(np.int64)
    ln = recs["datalength"].astype(np.int64)
    big = int(np.argmax(ln))
    flips = {0: 0, big: int(ln[big]) - 1, len(ln) // 2: int(ln[len(ln) // 2]) // 2,
             len(ln) - 1: int(ln[-1]) - 1}
    for k, at in flips.items():
        img[int(off[k]) + at] ^= 0x40
    d0.write_bytes(bytes(img))
    os.symlink("d0", d / "data" / "default" / "zdb-data-0")
    p = subprocess.run([str(oracle.REF_INTEGRITY), str(d / "data" / "default" / "zdb-data-0")], capture_output=True,
                       env=dict(os.environ, TZ="UTC"), timeout=120)
    assert p.returncode == len(flips)  # the tool exits with its error count
    return d / "data" / "default" / "zdb-data-0", p


@pytest.mark.parametrize("engine", ["hip", "auto"])
def test_tool_gpu_large_values_match_reference(large_value_datafile, engine):
    """the GPU tool on 8 MiB (maximum) and Zipf-mixed values: the reference
    tool's stdout, stderr and exit status (auto: GPU start forced)"""
    import re
    path, ref = large_value_datafile
    from test_tool_cpu import TOOL
    p = subprocess.run([str(TOOL), f"--engine={engine}", str(path)], capture_output=True,
                       env=dict(os.environ, TZ="UTC", ZDBCRC_AUTO_START_GPU="1", ZDBCRC_TOOL_TRACE="1"),
                       timeout=120)
    t = re.compile(rb"\[\s*\d+\.\d{6}\]")
    err, engines = split_trace(p.stderr)
    assert p.returncode == ref.returncode
    assert t.sub(b"[T]", p.stdout) == t.sub(b"[T]", ref.stdout)
    assert err == ref.stderr
    assert engines == ["hip"]


@pytest.mark.parametrize("jobs", [1, 3])
def test_tool_gpu_multi_file_scan(tmp_path, datafile_cases, jobs):
    """several datafiles in one run, worker threads sharing the GPU: every
    report identical to the reference run on that file (tests/test_tool_multi.py)"""
    from test_tool_multi import MULTI, check_multi
    check_multi(MULTI, tmp_path, "hip", datafile_cases, [f"--jobs={jobs}"])


def test_tool_gpu_multi_file_fatal(tmp_path):
    from test_tool_cpu import expected
    from test_tool_multi import run_multi
    names = ["mixed", "corrupt_crc", "truncated_payload", "multi_errors", "zipf_small"]
    out, err, code = run_multi(names, tmp_path, "hip", ["--jobs=4"])
    assert out == "".join(expected(n)[0] for n in names[:3])
    assert err == "".join(expected(n)[1] for n in names[:3])
    assert code == 1


# ------------------------------------------------------------------ C4 -------

def test_c4_device_image_and_verify(dev, oracle_c):
    """bench.c4_build_device writes the same bytes as the host construction
    (which the reference tool accepts, tests/test_c4.py), its crcs match the
    oracle, and verify_device flags exactly the corrupted records."""
    import bench
    lay = bench.c4_layout(1, files=3, file_cap=6 << 20)
    seed = bench.C4_SEED + 1
    img, poff, plen, expected, crcs = bench.c4_build_device(lay, seed)
    host = bench.c4_image_host(lay, seed, crcs)
    np.testing.assert_array_equal(img[: lay["total"]].cpu().numpy(), host)
    np.testing.assert_array_equal(crcs, oracle_c.batch(host, lay["payload_off"], lay["lens"]))
    np.testing.assert_array_equal(expected.cpu().numpy().view(np.uint32), crcs)
    n = len(lay["lens"])
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    mism = torch.zeros(64, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    dev.verify_device(img, poff, plen, expected, out, mism, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    bad = [r for r in (3, n // 2, n - 1) if lay["lens"][r] > 0]
    for r in bad:
        img[int(lay["payload_off"][r]) + int(lay["lens"][r]) // 2] ^= 0x40
    dev.verify_device(img, poff, plen, expected, out, mism, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == len(bad)
    assert sorted(mism[: len(bad)].cpu().tolist()) == sorted(bad)


def test_full_size_c4_shard_digest(dev, digests):
    """The rank-0 C4 shard (64 datafiles, ~16 GiB in HBM) against the digest
    the reference computed on the CPU (tests/golden/make_golden.py)."""
    import bench
    d = digests["C4"]
    lay = bench.c4_layout(0)
    assert lay["total"] == d["image_bytes"] and len(lay["lens"]) == d["count"]
    img, poff, plen, expected, crcs = bench.c4_build_device(lay, bench.C4_SEED)
    assert bench.digest(crcs) == {k: d[k] for k in ("count", "xor", "crc_of_crcs")}
    out = torch.empty(len(crcs), dtype=torch.int32, device="cuda")
    mism = torch.zeros(16, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    dev.verify_device(img, poff, plen, expected, out, mism, cnt)
    torch.cuda.synchronize()
    assert int(cnt.item()) == 0
    del img
    torch.cuda.empty_cache()


def _check_real(img: np.ndarray, off: int, crc32) -> int:
    """data_check_real (data.c:533-571) on an in-memory image: -1 on a short
    header or payload read, else payload crc == header integrity."""
    if off + 18 > len(img):
        return -1
    idlen = int(img[off])
    dlen = int(img[off + 1:off + 5].view("<u4")[0])
    integ = int(img[off + 9:off + 13].view("<u4")[0])
    p = off + 18 + idlen
    if dlen == 0:  # read(fd, buf, 0) == 0 succeeds past EOF too: crc(empty) = 0
        return int(integ == 0)
    if p + dlen > len(img):
        return -1
    return int(crc32(img[p:p + dlen]) == integ)


@pytest.mark.parametrize("name", ["mixed", "zipf_small", "fixed_4k", "corrupt_payload", "corrupt_crc",
                                  "multi_errors", "truncated_payload"])
def test_batched_check_device(dev, oracle_c, name):
    """f4: batched CHECK over a reference-written datafile image in HBM, one
    launch for every record the index would point at, plus offsets whose
    header or payload leaves the image (-1) and the file header itself."""
    img = np.fromfile(GOLDEN / "datafiles" / f"{name}.d0", dtype=np.uint8)
    recs, _ = dev.datafile_walk(img)
    offs = [int(o) for o in recs["header_offset"]] + [0, 28, len(img) - 5, len(img) - 18, len(img) + 100]
    want = np.array([_check_real(img, o, oracle_c.crc32) for o in offs], np.int32)
    d_img = torch.from_numpy(img.copy()).cuda()
    d_off = torch.tensor(offs, dtype=torch.int64, device="cuda")
    res = torch.full((len(offs),), 7, dtype=torch.int32, device="cuda")
    dev.datafile_check_device(d_img, d_off, res)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.cpu().numpy(), want)
    if name.startswith("corrupt") or name == "multi_errors":
        assert (want[:len(recs)] == 0).any()


@pytest.mark.parametrize("integrity,want", [(0, 1), (7, 0)])
def test_batched_check_empty_payload_key_past_end(dev, oracle_c, integrity, want):
    """An entry with datalength 0 whose key runs past the end of the image:
    data_check_real's payload read of 0 bytes succeeds, so the result is
    crc(empty) == integrity (data.c:546-570), not a short read."""
    img = np.fromfile(GOLDEN / "datafiles" / "mixed.d0", dtype=np.uint8)
    tail = np.frombuffer(dev.encode_entry(b"", 0, 28, integrity), np.uint8).copy()
    tail[0] = 200  # idlength: the key would end 200 bytes past the image
    full = np.concatenate([img, tail])
    offs = [len(img)]
    assert _check_real(full, len(img), oracle_c.crc32) == want
    d_img = torch.from_numpy(full).cuda()
    res = torch.full((1,), 7, dtype=torch.int32, device="cuda")
    dev.datafile_check_device(d_img, torch.tensor(offs, dtype=torch.int64, device="cuda"), res)
    torch.cuda.synchronize()
    assert int(res.cpu()[0]) == want


@pytest.mark.parametrize("case", ["fixed4k", "fixed4k_misaligned", "small_mixed", "hint_too_small"])
def test_small_record_shape(dev, oracle_c, case):
    """zdb_crc32_batch_device_sized with a 4 KiB bound (the packed kernel in
    rows of 16 lanes) is bit-exact -- also when the caller's bound is wrong
    (a 300 KiB record under a 4 KiB hint only costs speed)"""
    rng = np.random.default_rng(7)
    if case.startswith("fixed4k"):
        n = 3000
        lens = np.full(n, 4096, np.int64)
        stride = 4096 if case == "fixed4k" else 4096 + 26
        offs = np.arange(n, dtype=np.int64) * stride + (0 if case == "fixed4k" else 26)
    else:
        lens = rng.integers(0, 4097, 5000).astype(np.int64)
        if case == "hint_too_small":
            lens[1234] = 300_000
        offs = np.zeros(len(lens), np.int64)
        offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 5, len(lens) - 1))
    total = int(offs[-1] + lens[-1])
    arena = oracle.splitmix_bytes(total, 0x5A11)
    a = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    a[:total] = torch.from_numpy(arena).cuda()
    o = torch.from_numpy(offs).cuda()
    l = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.full((len(lens),), -1, dtype=torch.int32, device="cuda")
    want = oracle_c.batch(arena, offs, lens)
    for _ in range(2):  # both counter parities of the tail pool
        dev.batch_device(a, o, l, out, max_length=4096)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    # the host-buffer entry picks the shape from the lengths it is given
    np.testing.assert_array_equal(dev.batch_host(arena, offs.astype(np.uint64), lens.astype(np.uint32)), want)


def _packed_cases():
    """crafted batches for the packed kernel (records <= 4 KiB: one per row
    of 4 / 8 / 16 lanes by the bound; dword-anchored grid, piece 0 shifted up
    when a record starts in the first 16 bytes of a page)"""
    rng = np.random.default_rng(5)
    out = {}
    lens = np.arange(0, 301)
    out["every_len_0_300"] = (np.cumsum(np.concatenate([[1], lens[:-1] + 3])), lens, 2048)
    lens = np.full(64 * 16, 2048)
    out["2k_every_alignment"] = (np.array([4096 * 2 * i + (i % 64) for i in range(len(lens))]), lens, 2048)
    offs, ls = [], []
    for p in range(64):
        for a in range(16):
            for L in (1, 2, 3, 5, 17, 100, 2047, 2045):
                offs.append(4096 * (p * 4 + 1) + a)
                ls.append(L)
    out["page_start_records"] = (np.array(offs), np.array(ls), 2048)
    out["arena_start"] = (np.array([0, 1, 2, 3, 5, 9, 15, 0, 3]), np.array([100, 1, 2, 3, 7, 13, 1, 2048, 2045]), 2048)
    lens = rng.integers(0, 2049, 200_000)
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 5, len(lens) - 1))
    out["random_0_2k"] = (offs, lens, 2048)
    lens = np.concatenate([rng.integers(0, 300, 5000), [1 << 20, 3 << 20, 4096, 2049], rng.integers(0, 2049, 5000)])
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1] + 1)
    out["hint_too_small"] = (offs, lens, 2048)  # the bound is wrong: still exact
    lens = np.full(1 << 16, 64)
    out["fixed_64B"] = (np.arange(1 << 16, dtype=np.int64) * 64, lens, 64)
    # row widths by bound: <= 512 B rows of 4 lanes, <= 2 KiB rows of 8, <= 4 KiB rows of 16
    for bound in (256, 1024, 4096):
        lens = rng.integers(0, bound + 1, 100_000)
        offs = np.zeros(len(lens), np.int64)
        offs[1:] = np.cumsum(lens[:-1] + rng.integers(0, 5, len(lens) - 1))
        out[f"random_0_{bound}"] = (offs, lens, bound)
        offs, ls = [], []
        for p in range(32):
            for a in range(16):
                for L in (0, 1, 2, 3, 5, 17, 100, bound - 3, bound):
                    offs.append(4096 * (p * 4 + 1) + a)
                    ls.append(L)
        out[f"page_start_{bound}"] = (np.array(offs), np.array(ls), bound)
        lens = np.concatenate([rng.integers(0, bound, 3000), [1 << 20, 70_000, bound + 1], rng.integers(0, bound, 3000)])
        offs = np.zeros(len(lens), np.int64)
        offs[1:] = np.cumsum(lens[:-1] + 1)
        out[f"hint_too_small_{bound}"] = (offs, lens, bound)  # a wrong bound: still exact
    return out


PACKED_CASES = _packed_cases()


@pytest.mark.parametrize("case", list(PACKED_CASES))
def test_packed_kernel_small_records(dev, oracle_c, case):
    """batches whose records are known to be <= 2 KiB take the packed kernel
    (zdb_crc32_batch_device_sized, and the host-buffer entry, which measures
    the bound itself): bit-exact against the oracle on every crafted case,
    over both tail-pool counter parities"""
    offs, lens, bound = PACKED_CASES[case]
    offs = np.asarray(offs, np.int64)
    lens = np.asarray(lens, np.int64)
    total = int((offs + lens).max())
    arena = oracle.splitmix_bytes(total, 77)
    a = torch.zeros(total + 64, dtype=torch.uint8, device="cuda")
    a[:total] = torch.from_numpy(arena).cuda()
    o = torch.from_numpy(offs).cuda()
    l = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.full((len(lens),), -1, dtype=torch.int32, device="cuda")
    want = oracle_c.batch(arena, offs, lens)
    for _ in range(2):
        dev.batch_device(a, o, l, out, max_length=bound)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want)
    if lens.max() <= 4096:  # the host entry takes the packed kernel (its row width) from the lengths themselves
        np.testing.assert_array_equal(dev.batch_host(arena, offs.astype(np.uint64), lens.astype(np.uint32)), want)


@pytest.mark.parametrize("case", ["one_256KiB", "eight_256KiB", "mixed_small", "at_buffer_end"])
def test_host_batch_zero_copy(dev, oracle_c, case):
    """zdb_crc32_batch over an arena in zdb_crc32_host_alloc memory: the
    kernel reads it in place over PCIe (no staging copy) with a launch sized
    to the batch -- bit-exact, including a record that ends at the last byte
    the caller asked for"""
    rng = np.random.default_rng(11)
    V = 256 * 1024
    if case == "one_256KiB":
        offs, lens = np.array([0]), np.array([V])
    elif case == "eight_256KiB":
        offs, lens = np.arange(8) * V + 3, np.full(8, V)
    elif case == "mixed_small":
        lens = rng.integers(0, 9000, 700)
        offs = np.zeros(len(lens), np.int64)
        offs[1:] = np.cumsum(lens[:-1] + 1)
    else:
        lens = np.array([1, 4096, 333, 70_001])
        offs = np.array([0, 5, 4200, 0])
    total = int((offs + lens).max())
    pin = dev.PinnedBuffer(total)
    try:
        pin.array[:total] = oracle.splitmix_bytes(total, 0xC5 + len(case))
        if case == "at_buffer_end":
            offs = offs.copy()
            offs[-1] = total - int(lens[-1])  # ends exactly at the end of the allocation
        arena = pin.array[:total]
        want = oracle_c.batch(np.ascontiguousarray(arena), np.asarray(offs, np.int64), np.asarray(lens, np.int64))
        for _ in range(3):
            got = dev.batch_host(arena, np.asarray(offs, np.uint64), np.asarray(lens, np.uint32))
            np.testing.assert_array_equal(got, want)
    finally:
        pin.free()


def test_host_batch_mailbox_sizes_interleaved(dev, oracle_c):
    """small host batches (at most 1,024 records) return through the mailbox,
    whose device result buffer publish_kernel re-zeroes after each batch;
    larger ones through a copy.  Batches of growing and shrinking size,
    across the 1,024 boundary, pinned and pageable, with empty records and a
    record that spans many waves, must all stay exact: a word left over from a
    previous batch would show up as a wrong checksum in the next one"""
    rng = np.random.default_rng(23)
    total = 6 << 20
    pin = dev.PinnedBuffer(total)
    try:
        pin.array[:total] = oracle.splitmix_bytes(total, 0x3A11)
        plain = np.array(pin.array[:total])  # pageable copy: the staging path
        for n in (1, 7, 1024, 3, 1025, 1024, 64, 4000, 2, 1):
            lens = rng.integers(0, 3000, n)
            lens[rng.random(n) < 0.1] = 0
            if n == 3:
                lens[1] = 5 << 20  # one record over many waves: cut partials XORed into out[]
            offs = rng.integers(0, total - lens.max() - 1, n)
            want = oracle_c.batch(plain, offs.astype(np.int64), lens.astype(np.int64))
            for arena in (pin.array[:total], plain):
                got = dev.batch_host(arena, offs.astype(np.uint64), lens.astype(np.uint32))
                np.testing.assert_array_equal(got, want, err_msg=f"n={n}")
    finally:
        pin.free()


@pytest.mark.parametrize("batch,datasize", [(1, 600_000), (64, 600_000), (4096, 256 << 20)])
def test_set_pipeline_gpu_engine_matches_reference_daemon(tmp_path, batch, datasize):
    """f2: the two-phase SET batch with the GPU engine (values checksummed in
    place in the pinned receive buffer) against the reference zdbd: replies
    and datafiles byte-identical (timestamps aside), rotation included"""
    from test_set_pipeline import ZDBD, build_stream, run_harness, run_reference_zdbd, without_clock
    if not ZDBD.exists():
        pytest.skip("oracle/_ref/zdbd not built")
    stream, nreq = build_stream(5 + batch)
    reps, ref_files = run_reference_zdbd(stream, nreq, tmp_path, datasize)
    out, files, stats = run_harness(stream, tmp_path, datasize, "hip", batch)
    assert '"engine": "hip"' in stats
    assert out == b"".join(reps)
    assert sorted(files) == sorted(ref_files)
    for name in files:
        assert without_clock(files[name]) == without_clock(ref_files[name]), name


def test_set_pipeline_gpu_seq_mode_timestamps_and_api(tmp_path):
    """a9 with the GPU engine: the sequential handler and timestamped /
    malformed SETs against the reference zdbd started in sequential and user
    mode, and zdb_api_set's crc-only UP_TO_DATE against the reference library
    (tests/test_set_pipeline.py check_extra_modes)"""
    from test_set_pipeline import API_REF, ZDBD, check_extra_modes
    if not (ZDBD.exists() and API_REF.exists()):
        pytest.skip("oracle/_ref not built")
    check_extra_modes(tmp_path, "hip", batch=16)


@pytest.mark.parametrize("engine", ["hip", "auto"])
def test_set_pipeline_gpu_large_values(tmp_path, engine):
    """values up to the 8 MiB maximum payload (data.h:6) through the GPU
    engine, datafile rotation between them: the reference zdbd's replies and
    datafiles"""
    import json
    from test_set_pipeline import ZDBD, build_stream_large, run_harness, run_reference_zdbd, without_clock
    if not ZDBD.exists():
        pytest.skip("oracle/_ref/zdbd not built")
    stream, nreq = build_stream_large(9)
    reps, ref_files = run_reference_zdbd(stream, nreq, tmp_path, 20 << 20)
    out, files, stats = run_harness(stream, tmp_path, 20 << 20, engine, 16, from_file=True)
    st = json.loads(stats.strip().splitlines()[-1])
    assert st["engine"] == engine and st["gpu_batches"] > 0
    assert out == b"".join(reps)
    assert sorted(files) == sorted(ref_files) and len(files) > 1
    for name in files:
        assert without_clock(files[name]) == without_clock(ref_files[name]), name


def test_set_pipeline_auto_engine_splits_batches(tmp_path):
    """--engine=auto: batches of at least 512 KiB of values on the GPU, the
    smaller ones on the scalar engine, replies and datafiles still those of
    the reference zdbd"""
    import json
    from test_set_pipeline import ZDBD, build_stream, run_harness, run_reference_zdbd, without_clock
    if not ZDBD.exists():
        pytest.skip("oracle/_ref/zdbd not built")
    stream, nreq = build_stream(31)  # 4 of its 17 batches of 24 reach 512 KiB
    reps, ref_files = run_reference_zdbd(stream, nreq, tmp_path, 600_000)
    out, files, stats = run_harness(stream, tmp_path, 600_000, "auto", 24, from_file=True)
    st = json.loads(stats.strip().splitlines()[-1])
    assert st["engine"] == "auto" and 0 < st["gpu_batches"] < st["batches"]
    assert out == b"".join(reps)
    assert sorted(files) == sorted(ref_files)
    for name in files:
        assert without_clock(files[name]) == without_clock(ref_files[name]), name


@pytest.mark.parametrize("name", ["clean", "damaged", "cut", "stops_at_bad_file"])
def test_index_verify_gpu_engine(tmp_path, name):
    """f4: zdb-index-verify with the GPU engine against the reference
    index-rebuild + index-dump (tests/test_index_verify.py)"""
    from test_index_verify import NAMESPACES, REF, make_ns, oracle_corrupt, reference_live, tool_live
    if not (REF / "index-rebuild").exists():
        pytest.skip("oracle/_ref index tools not built")
    ns = make_ns(tmp_path, NAMESPACES[name])
    want = reference_live(tmp_path, ns)
    live, corrupt, p = tool_live(ns, "hip")
    assert live == want
    assert corrupt == oracle_corrupt(ns, live)
    assert p.returncode == len(corrupt)
