"""GPU tests of f3 (record-boundary discovery, 0-db_amd/csrc/datafile_hip.hip)
and the device-resident integrity scan built on it: the device walk must
equal the serial walk (zdb_datafile_walk, pinned to the reference tool's
output on the same files) on every golden datafile -- truncated, corrupt and
malformed ones included -- at chunk sizes that cut records every way, on
stores of several files, on files whose `previous` chain is broken (serial
re-walk fallback) and on a C4-shaped store; the scan's mismatch list must be
exactly the records whose stored crc the reference tool rejects."""
from __future__ import annotations

import sys

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from test_walk_model import CASES, serial

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.fail("no GPU visible to torch (tests marked gpu must run on the MI355X box)")
    import zdbcrc
    return zdbcrc


def store(dev, images, gap=13, capacity=None):
    """files back to back in one device image, `gap` junk bytes between them"""
    offs, parts, pos = [], [], 0
    for im in images:
        offs.append(pos)
        parts.append(im)
        pad = np.full(gap, 0xA5, np.uint8)
        parts.append(pad)
        pos += len(im) + gap
    host = np.concatenate(parts + [np.zeros(64, np.uint8)]) if parts else np.zeros(64, np.uint8)
    t = torch.from_numpy(host).cuda()
    cap = capacity if capacity is not None else sum(len(im) // 18 + 1 for im in images)
    return dev.DeviceStore(t, offs, [len(im) for im in images], cap), offs


def walked(st, n):
    eo = st.entry_off[:n].cpu().numpy()
    po = st.payload_off[:n].cpu().numpy()
    pl = st.payload_len[:n].cpu().numpy().view(np.uint32)
    ex = st.expected[:n].cpu().numpy().view(np.uint32)
    return [(int(a), int(b), int(c), int(d)) for a, b, c, d in zip(eo, po, pl, ex)]


def file_results(st):
    rec = st.file_records.cpu().numpy()
    return rec, st.file_status.cpu().numpy()[:st.nfiles], st.rewalks.cpu().numpy()


@pytest.mark.parametrize("chunk", [1024, 4096, 65536, 0])
@pytest.mark.parametrize("name", CASES)
def test_device_walk_equals_serial(dev, name, chunk):
    img = np.fromfile(GOLDEN / "datafiles" / f"{name}.d0", dtype=np.uint8)
    st, offs = store(dev, [img])
    st.walk(chunk)
    torch.cuda.synchronize()
    rec, status, _ = file_results(st)
    want, wst = serial(img)
    assert int(status[0]) == wst
    assert int(rec[1]) == len(want)
    assert walked(st, len(want)) == want


def test_device_walk_many_files_one_image(dev):
    """every golden file (and the mixed file 3 times) as one store: file
    order, per-file status and absolute offsets"""
    names = CASES + ["mixed", "mixed"]
    imgs = [np.fromfile(GOLDEN / "datafiles" / f"{n}.d0", dtype=np.uint8) for n in names]
    st, offs = store(dev, imgs)
    st.walk(2048)
    torch.cuda.synchronize()
    rec, status, _ = file_results(st)
    allw = []
    for i, im in enumerate(imgs):
        w, s = serial(im)
        assert int(status[i]) == s, names[i]
        assert int(rec[i]) == len(allw)
        allw += [(a + offs[i], b + offs[i], c, d) for a, b, c, d in w]
    assert int(rec[-1]) == len(allw)
    assert walked(st, len(allw)) == allw


def test_device_walk_more_files_than_one_stitch_block(dev):
    """300 files (the stitch kernel folds the file prefix into its one block
    up to 256 files; beyond that the prefix is a kernel of its own): every
    golden file repeated, record offsets, per-file status and totals"""
    names = (CASES * 28)[:300]
    imgs = [np.fromfile(GOLDEN / "datafiles" / f"{n}.d0", dtype=np.uint8) for n in names]
    st, offs = store(dev, imgs)
    st.walk(65536)
    torch.cuda.synchronize()
    rec, status, rew = file_results(st)
    allw = []
    for i, im in enumerate(imgs):
        w, s = serial(im)
        assert int(status[i]) == s, names[i]
        assert int(rec[i]) == len(allw)
        allw += [(a + offs[i], b + offs[i], c, d) for a, b, c, d in w]
    assert int(rec[len(imgs)]) == len(allw)
    assert walked(st, len(allw)) == allw


def test_device_walk_broken_previous_chain(dev):
    img = np.fromfile(GOLDEN / "datafiles" / "zipf_small.d0", dtype=np.uint8).copy()
    recs, _ = dev.datafile_walk(img)
    for h in recs["header_offset"]:
        img[int(h) + 5:int(h) + 9] = np.frombuffer(np.uint32(0xDEADBEEF).tobytes(), np.uint8)
    st, _ = store(dev, [img])
    st.walk(4096)
    torch.cuda.synchronize()
    rec, status, redo = file_results(st)
    want, wst = serial(img)
    assert (int(status[0]), int(rec[1])) == (wst, len(want))
    assert walked(st, len(want)) == want
    # no back-pointer confirms a header: the relaxed second search found the
    # chunk starts (the serial fallback: test_device_walk_unfiltered_headers)
    assert int(redo[-1]) == 0


def test_device_walk_scrambled_previous_256MiB(dev, tmp_path):
    """f3's worst case: a 256 MiB reference-written datafile (65,000 x 4 KiB
    values, oracle/_ref/gen_datafile_ref) whose `previous` fields are all
    scrambled -- no back-pointer confirms any header, so every chunk used to
    be re-walked serially (one dependent load per record).  The relaxed
    second search (forward_ok: four headers in a row that parse and fit)
    finds every chunk's start again: same records as the serial walk, no
    re-walked chunk, and a walk time of the order of the host walk's.  The
    timings land in gpurun_out/f3_worst_case.json."""
    import json
    import subprocess
    import time
    import oracle
    import zdbcrc
    if not oracle.REF_GEN.exists():
        pytest.skip("oracle/_ref not built")
    subprocess.run([str(oracle.REF_GEN), str(tmp_path), "fixed", "65000", "7", "4096"], check=True,
                   capture_output=True)
    img = np.fromfile(tmp_path / "data" / "default" / "d0", dtype=np.uint8).copy()
    recs, _ = dev.datafile_walk(img)
    rng = np.random.default_rng(3)
    for h in recs["header_offset"]:
        img[int(h) + 5:int(h) + 9] = rng.integers(0, 256, 4, dtype=np.uint8)
    t0 = time.perf_counter()
    zdbcrc.datafile_walk(img)  # the host walk (datafile.c), for scale
    host_s = time.perf_counter() - t0
    want, wst = serial(img)
    st, _ = store(dev, [img])
    st.walk()
    torch.cuda.synchronize()
    rec, status, redo = file_results(st)
    assert (int(status[0]), int(rec[1])) == (wst, len(want)) and len(want) == 65000
    assert walked(st, len(want)) == want
    assert int(redo[-1]) == 0  # no chunk fell back to the serial re-walk
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        ev0.record()
        st.walk()
        ev1.record()
        torch.cuda.synchronize()
        ts.append(ev0.elapsed_time(ev1))
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    (out / "f3_worst_case.json").write_text(json.dumps({
        "file_bytes": int(len(img)), "records": len(want), "device_walk_ms": sorted(ts),
        "host_walk_ms": round(host_s * 1e3, 2), "rewalked_chunks": int(redo[-1])}) + "\n")


def test_device_walk_unfiltered_headers(dev):
    img = np.fromfile(GOLDEN / "datafiles" / "fixed_4k.d0", dtype=np.uint8).copy()
    recs, _ = dev.datafile_walk(img)
    for h in recs["header_offset"]:
        img[int(h) + 13] = 0xFF  # flags the filter rejects
    st, _ = store(dev, [img])
    st.walk(1024)
    torch.cuda.synchronize()
    rec, status, redo = file_results(st)
    want, wst = serial(img)
    assert walked(st, len(want)) == want and int(status[0]) == wst
    assert int(redo[-1]) > 0


def test_device_walk_bound_and_capacity(dev):
    img = np.fromfile(GOLDEN / "datafiles" / "mixed.d0", dtype=np.uint8)
    st, _ = store(dev, [img])
    dev._check(dev._walk_device(st.image.data_ptr(), st.file_off.data_ptr(), st.file_len.data_ptr(), 1, 1024,
                                1024, st.entry_off.data_ptr(), st.payload_off.data_ptr(), st.payload_len.data_ptr(),
                                st.expected.data_ptr(), st.capacity, st.file_records.data_ptr(),
                                st.file_status.data_ptr(), st.rewalks.data_ptr(), None), "walk")
    torch.cuda.synchronize()
    assert int(st.file_status.cpu()[0]) == dev.WALK_EXCEEDS_BOUND
    small, _ = store(dev, [img], capacity=5)
    with pytest.raises(dev.ZdbCrcError, match="capacity"):
        small.scan(2048)
    # the verify ran on the device-side count bounded by the capacity: the
    # first 5 records are checked (mixed.d0 is clean: computed == stored)
    want, _ = serial(img)
    assert small.computed[:5].cpu().numpy().view(np.uint32).tolist() == [w[3] for w in want[:5]]
    assert dev._walk_device(None, None, None, 1, 1, 0, None, None, None, None, 0, None, None, None, None) == -2
    # a size query (capacity 0): the walk's count comes back with ENOSPC
    q, _ = store(dev, [img], capacity=0)
    with pytest.raises(dev.ZdbCrcError, match=f"{len(want)} records > capacity 0"):
        q.scan(2048)
    # a store too large for the launch grids is refused up front (2^24 files of one chunk)
    assert dev._walk_device(st.image.data_ptr(), st.file_off.data_ptr(), st.file_len.data_ptr(), 1 << 24,
                            1024, 1024, st.entry_off.data_ptr(), st.payload_off.data_ptr(),
                            st.payload_len.data_ptr(), st.expected.data_ptr(), st.capacity,
                            st.file_records.data_ptr(), st.file_status.data_ptr(), st.rewalks.data_ptr(),
                            None) == -2


@pytest.mark.parametrize("name", ["mixed", "zipf_small", "corrupt_payload", "corrupt_crc", "multi_errors",
                                  "truncated_payload"])
def test_device_scan_mismatches(dev, datafile_cases, name):
    """scan = walk + checksum + compare: the mismatch count is the reference
    tool's error count (for the truncated file: the errors before the record
    that ends its run), and the listed records are exactly the bad ones"""
    img = np.fromfile(GOLDEN / "datafiles" / f"{name}.d0", dtype=np.uint8)
    st, _ = store(dev, [img])
    n = st.scan(4096)
    torch.cuda.synchronize()
    want, _ = serial(img)
    assert n == len(want)
    import oracle
    orc = oracle.Oracle()
    bad = sorted(i for i, (_, po, pl, ex) in enumerate(want) if pl and orc.crc32(img[po:po + pl]) != ex)
    cnt = int(st.mismatch_count.cpu()[0])
    assert sorted(st.mismatch[:cnt].cpu().numpy().tolist()) == bad
    exit_code = {c["name"]: c["exit"] for c in datafile_cases}[name]
    if name != "truncated_payload":
        assert cnt == exit_code


def test_device_scan_c4_shaped_store(dev):
    """a C4-shaped store (bench.c4_layout: reference-valid datafiles of
    C3-distributed payloads, 8-byte keys) at 6 files x 8 MiB: the walk finds
    exactly the layout's entries, the scan reports no mismatch, and after
    flipping one payload byte in three records exactly those three"""
    sys.path.insert(0, str(ROOT))
    import bench
    import zdbcrc
    lay = bench.c4_layout(0, files=6, file_cap=8 << 20)
    arena = zdbcrc.synth_fill(lay["total"], 77)
    crcs = np.array([zdbcrc.crc32(arena[o:o + l]) for o, l in zip(lay["payload_off"], lay["lens"])], np.uint32)
    img = bench.c4_image_host(lay, 77, crcs)
    t = torch.from_numpy(np.concatenate([img, np.zeros(64, np.uint8)])).cuda()
    st = dev.DeviceStore(t, lay["file_off"], lay["file_size"], capacity=len(crcs) + 10)
    n = st.scan(1 << 20)
    assert n == len(crcs)
    np.testing.assert_array_equal(st.entry_off[:n].cpu().numpy(), lay["entry_off"])
    assert int(st.mismatch_count.cpu()[0]) == 0
    assert (st.file_status.cpu().numpy() == 0).all()
    assert int(st.rewalks.cpu()[-1]) == 0  # zdbd-shaped files: every chunk speculated right
    np.testing.assert_array_equal(st.computed[:n].cpu().numpy().view(np.uint32), crcs)
    hit = [5, len(crcs) // 2, len(crcs) - 1]
    for r in hit:
        t[int(lay["payload_off"][r])] ^= 0x40
    st.scan(1 << 20)
    cnt = int(st.mismatch_count.cpu()[0])
    assert sorted(st.mismatch[:cnt].cpu().numpy().tolist()) == hit


def test_device_scan_small_value_store_default_chunks(dev):
    """a store of 4 KiB values (C2u-shaped datafiles, 4 x 64 MiB) through the
    default chunk size -- chosen from the store's record density by the
    sampling kernel (512 KiB here instead of 8 MiB: ~2,000 dependent hops per
    chain otherwise) -- and at two fixed sizes: the same entries as the
    layout, every chunk speculated right, no mismatch; then one flipped byte"""
    sys.path.insert(0, str(ROOT))
    import bench
    files, cap, val = 4, 64 << 20, 4096
    per = (cap - bench.FILE_HDR) // (bench.ENTRY_HDR + bench.C4_KEY + val)
    n = per * files
    step = bench.ENTRY_HDR + bench.C4_KEY + val
    file_of = np.repeat(np.arange(files), per)
    rel = bench.FILE_HDR + (np.arange(n) % per) * step
    fsize = np.full(files, bench.FILE_HDR + per * step, np.int64)
    file_off = np.concatenate([[0], np.cumsum(fsize[:-1])])
    entry_off = file_off[file_of] + rel
    lay = {"lens": np.full(n, val, np.int64), "entry_off": entry_off,
           "payload_off": entry_off + bench.ENTRY_HDR + bench.C4_KEY,
           "prev": np.where(np.arange(n) % per == 0, 0, rel - step), "file_of": file_of, "file_off": file_off,
           "file_size": fsize, "total": int(file_off[-1] + fsize[-1])}
    img, _, _, _, crcs = bench.c4_build_device(lay, 0x5A11)
    st = dev.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=n + 10)
    for chunk in (0, 8 << 20, 256 << 10):
        assert st.scan(chunk) == n
        np.testing.assert_array_equal(st.entry_off[:n].cpu().numpy(), lay["entry_off"])
        assert int(st.mismatch_count.cpu()[0]) == 0
        assert int(st.rewalks.cpu()[-1]) == 0
        np.testing.assert_array_equal(st.computed[:n].cpu().numpy().view(np.uint32), crcs)
    img[int(lay["payload_off"][n // 3]) + 7] ^= 0x10
    st.scan()
    cnt = int(st.mismatch_count.cpu()[0])
    assert st.mismatch[:cnt].cpu().numpy().tolist() == [n // 3]


def test_device_scan_files_over_2GiB(dev):
    """two C4-shaped datafiles of ~3 GiB each (entry offsets past 2^31, the
    top of a datafile's u32 offsets in reach): the walk finds exactly the
    layout's entries with every chunk speculated right, and the scan matches
    every stored crc"""
    sys.path.insert(0, str(ROOT))
    import bench
    lay = bench.c4_layout(5, files=2, file_cap=3 << 30)
    assert lay["file_size"].max() > (5 << 29)  # positions beyond 2.5 GiB in both files
    img, _, _, _, crcs = bench.c4_build_device(lay, 0x2B16)
    st = dev.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=len(crcs) + 10)
    n = st.scan()
    assert n == len(crcs)
    np.testing.assert_array_equal(st.entry_off[:n].cpu().numpy(), lay["entry_off"])
    assert (st.file_status.cpu().numpy() == 0).all()
    assert int(st.rewalks.cpu()[-1]) == 0
    assert int(st.mismatch_count.cpu()[0]) == 0
    np.testing.assert_array_equal(st.computed[:n].cpu().numpy().view(np.uint32), crcs)
    del img, st


@pytest.mark.parametrize("chunk", [1024, 4096])
def test_device_scan_many_small_chunks(dev, chunk):
    """16 C4-shaped datafiles of 8 MiB walked in 1 KiB / 4 KiB chunks: more
    than 65,536 chunks at 1 KiB (the walk then keeps 64 record slots per
    chunk instead of 512, and overfull chunks are emitted by a second walk)"""
    sys.path.insert(0, str(ROOT))
    import bench
    lay = bench.c4_layout(6, files=16, file_cap=8 << 20)
    img, _, _, _, crcs = bench.c4_build_device(lay, 0x1C)
    st = dev.DeviceStore(img, lay["file_off"], lay["file_size"], capacity=len(crcs) + 10)
    n = st.scan(chunk)
    assert n == len(crcs)
    np.testing.assert_array_equal(st.entry_off[:n].cpu().numpy(), lay["entry_off"])
    np.testing.assert_array_equal(st.payload_off[:n].cpu().numpy(), lay["payload_off"])
    assert (st.file_status.cpu().numpy() == 0).all()
    assert int(st.mismatch_count.cpu()[0]) == 0
    np.testing.assert_array_equal(st.computed[:n].cpu().numpy().view(np.uint32), crcs)
