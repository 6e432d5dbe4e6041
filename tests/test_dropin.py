"""The scalar drop-in linked the way INTEGRATION.md §1 says: the reference's
own libzdb objects (compiled from /root/reference/libzdb by oracle/Makefile)
archived into libzdb.a with crc32.o replaced by 0-db_amd/lib/crc32_cpu.o,
then the reference integrity-check (tools/integrity-check/Makefile links
libzdb.a statically) and the fixture generator (zdb_api_set -> data_insert)
linked against that archive (`make -C oracle dropin`).

* the swapped tool's stdout / stderr / exit status on every golden datafile
  equal the unmodified reference tool's captured ones;
* a datafile written through the swapped libzdb carries the same stored crcs
  (and the same bytes, timestamps aside) as one written by the reference
  libzdb, and the unmodified reference tool finds it clean.
CPU only (no GPU is touched by the drop-in)."""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

import oracle
import zdbcrc
from conftest import GOLDEN
from test_tool_cpu import CASES, TIMELOG, expected

DROPIN = Path(oracle.__file__).resolve().parent / "_ref" / "dropin"
TOOL = DROPIN / "integrity-check"
GEN = DROPIN / "gen_datafile"

pytestmark = pytest.mark.skipif(not (TOOL.exists() and GEN.exists() and oracle.REF_GEN.exists()),
                                reason="make -C oracle ref dropin (needs /root/reference at build time)")


def test_dropin_archive_has_no_reference_crc32():
    out = subprocess.run(["ar", "t", str(DROPIN / "libzdb.a")], capture_output=True, text=True,
                         check=True).stdout.split()
    assert "crc32.o" not in out and "crc32_cpu.o" in out
    syms = subprocess.run(["nm", str(TOOL)], capture_output=True, text=True, check=True).stdout
    # zdb_crc32 comes from the drop-in (its software-table builder rides along)
    assert " T zdb_crc32\n" in syms and "zdbcrc_build_tables" in syms


@pytest.mark.parametrize("name", CASES)
def test_swapped_reference_tool_matches_reference(tmp_path, datafile_cases, name):
    d = tmp_path / name
    d.mkdir()
    shutil.copy(GOLDEN / "datafiles" / f"{name}.d0", d / "d0")
    os.symlink("d0", d / "zdb-data-0")
    p = subprocess.run([str(TOOL), str(d / "zdb-data-0")], capture_output=True, cwd=d,
                       env=dict(os.environ, TZ="UTC"), timeout=120)
    norm = lambda s: TIMELOG.sub("[T]", s.decode().replace(str(d), "@DIR@"))
    eout, eerr = expected(name)
    assert norm(p.stdout) == eout
    assert norm(p.stderr) == eerr
    assert p.returncode == {c["name"]: c["exit"] for c in datafile_cases}[name]


def _generate(gen: Path, mode: str, count: int, seed: int, size: int) -> bytes:
    with tempfile.TemporaryDirectory() as td:
        subprocess.run([str(gen), td, mode, str(count), str(seed), str(size)], check=True, capture_output=True)
        return (Path(td) / "data" / "default" / "d0").read_bytes()


def _without_clock(img: bytes) -> bytes:
    """zero the wall-clock fields: file header created/opened (data.h:41-42)
    and each entry's timestamp (data.h:64)"""
    b = bytearray(img)
    b[8:24] = bytes(16)
    recs, status = zdbcrc.datafile_walk(img)
    assert status == 0
    for h in recs["header_offset"]:
        b[int(h) + 14:int(h) + 18] = bytes(4)
    return bytes(b)


@pytest.mark.parametrize("mode,count,seed,size", [("mixed", 100, 7, 0), ("zipf", 400, 11, 300_000),
                                                  ("fixed", 64, 13, 4096)])
def test_swapped_libzdb_writes_reference_datafiles(tmp_path, mode, count, seed, size):
    ref = _generate(oracle.REF_GEN, mode, count, seed, size)
    swp = _generate(GEN, mode, count, seed, size)
    assert _without_clock(swp) == _without_clock(ref)
    recs, _ = zdbcrc.datafile_walk(swp)
    live = recs[recs["datalength"] > 0]
    assert len(live) > 0
    # the stored crcs are the reference's values for those payloads
    arr = np.frombuffer(swp, np.uint8)
    want = oracle.Oracle().batch(arr, live["payload_offset"].astype(np.int64), live["datalength"].astype(np.int64))
    np.testing.assert_array_equal(live["integrity"], want)
    # and the unmodified reference tool finds the file clean
    d = tmp_path / "d"
    d.mkdir()
    (d / "d0").write_bytes(swp)
    os.symlink("d0", d / "zdb-data-0")
    p = subprocess.run([str(oracle.REF_INTEGRITY), str(d / "zdb-data-0")], capture_output=True, timeout=120)
    assert p.returncode == 0 and b"integrity check failed" not in p.stderr
