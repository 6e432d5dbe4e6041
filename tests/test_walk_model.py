"""The f3 walk algorithm (tests/walk_model.py, the CPU model of the kernels in
0-db_amd/csrc/datafile_hip.hip) against the serial walk on every golden
datafile, at chunk sizes that cut records every way, on files whose
`previous` chain is broken (forcing serial re-walks), and on files that are
not zdbd-shaped (headers the filter rejects)."""
from __future__ import annotations

import numpy as np
import pytest

import zdbcrc
from conftest import GOLDEN
from walk_model import device_walk

CASES = ["mixed", "zipf_small", "fixed_4k", "corrupt_payload", "corrupt_crc", "multi_errors",
         "truncated_payload", "truncated_header", "bad_magic", "bad_version", "header_only"]


def serial(img: np.ndarray):
    recs, status = zdbcrc.datafile_walk(img)
    out = []
    for r in recs:
        ln = int(r["datalength"])
        full = ln > 0 and int(r["payload_offset"]) + ln <= len(img)
        out.append((int(r["header_offset"]), int(r["payload_offset"]), ln if full else 0,
                    int(r["integrity"]) if full else 0))
    return out, status


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("chunk", [1024, 4096, 65536])
def test_model_equals_serial_walk(name, chunk):
    img = np.fromfile(GOLDEN / "datafiles" / f"{name}.d0", dtype=np.uint8)
    recs, st, _ = device_walk(img, chunk)
    want, wst = serial(img)
    assert st == wst
    assert recs == want


def test_model_broken_previous_chain_rewalks():
    """`previous` fields scrambled (as a rewriting tool could leave them):
    every speculative start fails validation, the stitch re-walks serially
    and the result is still the serial walk's."""
    img = np.fromfile(GOLDEN / "datafiles" / "mixed.d0", dtype=np.uint8).copy()
    recs, _ = zdbcrc.datafile_walk(img)
    for h in recs["header_offset"]:
        img[int(h) + 5:int(h) + 9] = np.frombuffer(np.uint32(0xDEADBEEF).tobytes(), np.uint8)
    got, st, redo = device_walk(img, 1024)
    want, wst = serial(img)
    assert (got, st) == (want, wst)
    assert redo > 0


def test_model_unfiltered_headers():
    """headers the filter rejects (flags 0xFF): exact through re-walks"""
    img = np.fromfile(GOLDEN / "datafiles" / "fixed_4k.d0", dtype=np.uint8).copy()
    recs, _ = zdbcrc.datafile_walk(img)
    for h in recs["header_offset"]:
        img[int(h) + 13] = 0xFF
    got, st, redo = device_walk(img, 1024)
    assert (got, st) == serial(img)
    assert redo > 0


def test_model_max_len_bound():
    img = np.fromfile(GOLDEN / "datafiles" / "mixed.d0", dtype=np.uint8)
    _, st, _ = device_walk(img, 1024, max_len=1024)
    assert st == 4  # ZDB_WALK_EXCEEDS_BOUND
