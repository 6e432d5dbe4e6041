"""CPU tests of the product library's host side: the scalar drop-in engine,
the GF(2) helpers, the C ABI surface, the datafile walk/encoders and the
synthetic-input generators.  No GPU call is made here."""
from __future__ import annotations

import re
import subprocess
import sys

import numpy as np
import pytest

import oracle
import zdbcrc
from conftest import GOLDEN, ROOT, kat_bytes


# ---------------------------------------------------------------- ABI -------

def _declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(zdb_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def test_every_declared_symbol_is_exported():
    declared = _declared_functions()
    assert len(declared) >= 20
    assert declared == set(zdbcrc.EXPORTED)
    for name in declared:
        assert hasattr(zdbcrc._lib, name), name


def test_library_exports_exactly_the_abi():
    """libzdbcrc.so exports the include/*.h functions and nothing else: the
    A/B kernel variants, probe kernels and zdbcrc_debug_* hooks live in
    libzdbcrc_diag.so only (its version script), and no ZDBCRC_VARIANT knob
    can reach the product."""
    lib = ROOT / "0-db_amd" / "lib" / "libzdbcrc.so"
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if ln.strip()}
    assert exported == _declared_functions()
    blob = lib.read_bytes()
    assert b"ZDBCRC_VARIANT" not in blob and b"zdbcrc_debug" not in blob
    diag = ROOT / "0-db_amd" / "lib" / "libzdbcrc_diag.so"
    dout = subprocess.run(["nm", "-D", "--defined-only", str(diag)], capture_output=True, text=True,
                          check=True).stdout
    assert "zdbcrc_debug_set_variant" in dout


def test_host_batch_rejects_overflowing_descriptor_before_hip():
    """zdb_crc32_batch: offset + length must not wrap around u64 (offset near
    UINT64_MAX is EINVAL), and the check runs before HIP is initialised."""
    code = ("import sys, numpy as np; sys.path.insert(0, %r); import zdbcrc; "
            "a = np.zeros(64, np.uint8); o = np.array([2**64 - 2], np.uint64); "
            "l = np.array([4], np.uint32); out = np.zeros(1, np.uint32); "
            "rc = zdbcrc._batch_host(a.ctypes.data, a.size, o.ctypes.data, l.ctypes.data, out.ctypes.data, 1); "
            "o3 = np.array([61], np.uint64); "
            "rc3 = zdbcrc._batch_host(a.ctypes.data, a.size, o3.ctypes.data, l.ctypes.data, out.ctypes.data, 1); "
            "print(rc, rc3, zdbcrc.gpu_initialized())"
            % str(ROOT / "0-db_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["-2", "-2", "False"]


def test_scalar_path_never_touches_hip():
    # key hashing / CHECK must not initialise the GPU (fork safety)
    code = ("import sys; sys.path.insert(0, %r); import zdbcrc; "
            "zdbcrc.crc32(b'k'*255); zdbcrc.checksum_crc32(b'x'*4096); zdbcrc.shift(1, 100); "
            "zdbcrc.datafile_walk(open(%r,'rb').read()); "
            "print(zdbcrc.gpu_initialized(), zdbcrc.batch_engine())"
            % (str(ROOT / "0-db_amd"), str(GOLDEN / "datafiles" / "mixed.d0")))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["False", "uninitialized"]


# ------------------------------------------------------- scalar engine ------

def test_engine_value():
    assert zdbcrc.engine_value() == "sse42"


@pytest.mark.parametrize("engine,flags", [("armv8", ["-msse4.2", "-DZDBCRC_ARMV8_EMULATE"]),
                                          ("software", ["-mno-sse4.2"]),
                                          ("sse42", ["-msse4.2"])])
def test_every_engine_of_the_drop_in(tmp_path, kats, vectors, engine, flags):
    """The three compile-time engines of crc32.c:94-155 (sse42, armv8,
    software) built from crc32_cpu.c: engine name and values.  There is no
    AArch64 compiler in this image, so the armv8 loop is built with its ACLE
    intrinsics spelled by their SSE4.2 twins (ZDBCRC_ARMV8_EMULATE)."""
    import ctypes as C
    src = ROOT / "0-db_amd" / "csrc"
    so = tmp_path / f"libcpu_{engine}.so"
    subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-std=gnu11", "-I", str(ROOT / "include"), "-I", str(src),
                    *flags, "-o", str(so), str(src / "crc32_cpu.c"), str(src / "crc32c_gf2.c"), "-lpthread"],
                   check=True)
    lib = C.CDLL(str(so))
    lib.zdb_crc32_engine_value.restype = C.c_char_p
    lib.zdb_crc32.restype = C.c_uint32
    lib.zdb_crc32.argtypes = [C.c_void_p, C.c_ssize_t]
    assert lib.zdb_crc32_engine_value().decode() == engine
    for e in kats:
        d = np.frombuffer(kat_bytes(e), np.uint8)
        assert lib.zdb_crc32(d.ctypes.data if d.size else None, d.size) == int(e["crc"], 16), e["name"]
    lens, seeds, crcs = vectors
    for n, sd, c in list(zip(lens, seeds, crcs))[::7]:
        if n > 70_000:
            continue
        buf = np.zeros(int(n) + 16, dtype=np.uint8)
        for mis in (0, 3, 9):
            buf[mis:mis + n] = oracle.splitmix_bytes(int(n), int(sd))
            assert lib.zdb_crc32(buf[mis:].ctypes.data, int(n)) == int(c)


def test_scalar_known_answers(kats):
    for e in kats:
        data = kat_bytes(e)
        assert zdbcrc.crc32(data) == int(e["crc"], 16), e["name"]
        assert zdbcrc.checksum_crc32(data) == int(e["crc"], 16), e["name"]


def test_scalar_vectors_all_alignments(vectors):
    lens, seeds, crcs = vectors
    for n, s, c in zip(lens, seeds, crcs):
        if n > 70_000:
            continue
        buf = np.zeros(int(n) + 16, dtype=np.uint8)
        data = oracle.splitmix_bytes(int(n), int(s))
        for mis in (0, 1, 7, 13):
            buf[mis:mis + n] = data
            assert zdbcrc.crc32(buf[mis:mis + n]) == int(c)


def test_negative_length_is_zero():
    assert zdbcrc._crc32(None, -5) == 0


# ----------------------------------------------------------- GF(2) ----------

def test_combine_and_shift(oracle_c):
    rng = np.random.default_rng(3)
    for _ in range(200):
        a = oracle.splitmix_bytes(int(rng.integers(0, 3000)), int(rng.integers(1 << 30)))
        b = oracle.splitmix_bytes(int(rng.integers(0, 3000)), int(rng.integers(1 << 30)))
        ca, cb = oracle_c.crc32(a), oracle_c.crc32(b)
        assert zdbcrc.combine(ca, cb, len(b)) == oracle_c.crc32(np.concatenate([a, b]))
        n = int(rng.integers(-100_000, 100_000))
        assert zdbcrc.shift(zdbcrc.shift(ca, n), -n) == ca
        # shift over n zero bytes == crc of data followed by n zeros
        k = int(rng.integers(0, 500))
        assert zdbcrc.shift(ca, k) == oracle_c.crc32(np.concatenate([a, np.zeros(k, np.uint8)]))


def test_zero_prefix_invariance(oracle_c):
    d = oracle.splitmix_bytes(777, 1)
    assert oracle_c.crc32(np.concatenate([np.zeros(333, np.uint8), d])) == oracle_c.crc32(d)


def test_large_shift_matches_repeated():
    c = 0x12345678
    x = c
    for _ in range(16):
        x = zdbcrc.shift(x, 1 << 20)
    assert zdbcrc.shift(c, 16 << 20) == x


# --------------------------------------------------------- synthetic --------

@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 63, 64, 65, 1000, 4097, 1 << 20])
def test_synth_matches_restatement(n):
    np.testing.assert_array_equal(zdbcrc.synth_fill(n, 0xABC + n), oracle.splitmix_bytes(n, 0xABC + n))


def test_zipf_recipe():
    lens = zdbcrc.zipf_lengths(256 << 20, 0xC3C3C3)
    assert lens.min() >= 64 and lens.max() <= 1 << 20
    assert lens.sum() >= 256 << 20
    # ~78 % of records <= 4 KiB, ~79 % of bytes in records >= 256 KiB
    assert 0.70 < (lens <= 4096).mean() < 0.85
    big = lens[lens >= 256 * 1024].sum() / lens.sum()
    assert 0.70 < big < 0.88
    np.testing.assert_array_equal(lens, zdbcrc.zipf_lengths(256 << 20, 0xC3C3C3))


# ---------------------------------------------------------- datafile --------

@pytest.mark.parametrize("name", ["mixed", "zipf_small", "fixed_4k", "corrupt_payload",
                                  "truncated_payload", "truncated_header", "bad_magic",
                                  "bad_version", "header_only"])
def test_walk_matches_oracle_scan(oracle_c, name):
    img = (GOLDEN / "datafiles" / f"{name}.d0").read_bytes()
    recs, status = zdbcrc.datafile_walk(img)
    orecs, _, fatal = oracle_c.integrity_scan(img)
    assert status == fatal
    assert len(recs) == len(orecs)
    for f in ("header_offset", "payload_offset", "datalength", "integrity", "previous", "idlength",
              "flags"):
        np.testing.assert_array_equal(recs[f].astype(np.uint64), orecs[f].astype(np.uint64), f)


def test_reencode_is_byte_identical():
    """Encoding every walked record back (header + key + payload) reproduces
    the reference-written datafile byte for byte (data.c:594-633 framing)."""
    img = (GOLDEN / "datafiles" / "mixed.d0").read_bytes()
    recs, status = zdbcrc.datafile_walk(img)
    assert status == 0
    out = bytearray(img[:28])
    assert zdbcrc.encode_header(0)[:8] == img[:8]
    for r in recs:
        h = int(r["header_offset"])
        key = img[h + 18:h + 18 + int(r["idlength"])]
        out += zdbcrc.encode_entry(key, int(r["datalength"]), int(r["previous"]), int(r["integrity"]),
                                   int(r["flags"]), int(r["timestamp"]))
        p = int(r["payload_offset"])
        out += img[p:p + int(r["datalength"])]
    assert bytes(out) == img


def test_deleted_entries_present():
    img = (GOLDEN / "datafiles" / "mixed.d0").read_bytes()
    recs, _ = zdbcrc.datafile_walk(img)
    deleted = recs[recs["flags"] & 1 == 1]
    assert len(deleted) == 2
    assert (deleted["datalength"] == 0).all() and (deleted["integrity"] == 0).all()


def test_encode_batch_matches_reference_inserts():
    """zdb_datafile_encode_batch == successive reference data_insert calls
    (fixed_4k.d0 was written by libzdb; timestamps are taken from the file)."""
    img = (GOLDEN / "datafiles" / "fixed_4k.d0").read_bytes()
    recs, status = zdbcrc.datafile_walk(img)
    assert status == 0
    arr = np.frombuffer(img, np.uint8)
    keys = [img[int(r["header_offset"]) + 18:int(r["payload_offset"])] for r in recs]
    out, prev, eo = zdbcrc.encode_batch(keys, arr, recs["payload_offset"], recs["datalength"],
                                        recs["integrity"], file_offset=28, previous=0,
                                        timestamp=int(recs["timestamp"][0]))
    got = bytearray(img[:28] + out)
    for r in recs:  # the reference stamps each insert with time(NULL)
        h = int(r["header_offset"])
        got[h + 14:h + 18] = img[h + 14:h + 18]
    assert bytes(got) == img
    assert prev == int(recs["header_offset"][-1])
    np.testing.assert_array_equal(eo, recs["header_offset"])


def test_check_device_argument_errors_without_gpu():
    """zdb_datafile_check_device: an empty batch is a no-op and null device
    pointers are rejected before HIP is touched (CPU-only: no compute call)."""
    f = zdbcrc._check_device
    assert f(None, 0, None, None, 0, None) == 0
    assert f(None, 100, None, None, 5, None) == -2  # ZDB_CRC32_EINVAL (zdb_crc32.h)
    code = ("import sys; sys.path.insert(0, %r); import zdbcrc; "
            "zdbcrc._check_device(None, 0, None, None, 0, None); print(zdbcrc.gpu_initialized())"
            % str(ROOT / "0-db_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["False"]
