"""Pin the oracle: the C restatement (oracle/crc32c_oracle.c), the numpy /
pure-Python restatements, and -- where it was built -- the real reference
(oracle/_ref) against the golden fixtures that the reference produced
(tests/golden/make_golden.py).  CPU only."""
from __future__ import annotations

import numpy as np
import pytest

import oracle
from conftest import GOLDEN, kat_bytes

POLY = 0x82F63B78


def test_table_is_crc32c_reflected(oracle_c):
    t = oracle_c.table()
    # crc32.c:16-81 spot values
    assert t[0] == 0 and t[1] == 0xF26B8303 and t[128] == POLY and t[255] == 0xAD7D5351


def test_known_answers(oracle_c, kats):
    for e in kats:
        data = kat_bytes(e)
        assert len(data) == e["length"]
        assert oracle_c.crc32(data) == int(e["crc"], 16), e["name"]


def test_documented_answers(oracle_c):
    # values quoted in SURVEY §0 / §8(c), measured there on the reference
    assert oracle_c.crc32(b"123456789") == 0x58E3FA20  # not standard CRC-32C (0xE3069283)
    assert oracle_c.crc32(b"world") == 0x74D8F77B
    assert oracle_c.crc32(b"") == 0
    assert oracle_c.crc32(b"\x00" * 999) == 0


def test_python_restatement_small(kats):
    for e in kats:
        if e["length"] <= 1024:
            assert oracle.crc32_py(kat_bytes(e)) == int(e["crc"], 16), e["name"]


def test_random_vectors(oracle_c, vectors):
    lens, seeds, crcs = vectors
    for n, s, c in zip(lens, seeds, crcs):
        assert oracle_c.crc32(oracle.splitmix_bytes(int(n), int(s))) == int(c), int(n)


def test_batch_matches_scalar(oracle_c):
    arena = oracle.splitmix_bytes(10_000, 5)
    rng = np.random.default_rng(0)
    lens = rng.integers(0, 2000, 50)
    offs = np.array([rng.integers(0, 10_000 - l) for l in lens])
    got = oracle_c.batch(arena, offs, lens)
    for o, l, g in zip(offs, lens, got):
        assert g == oracle_c.crc32(arena[o:o + l].tobytes())


def test_reference_agrees_with_restatement(reference, oracle_c):
    assert reference.engine() == "sse42"
    rng = np.random.default_rng(7)
    arena = oracle.splitmix_bytes(1 << 20, 99)
    lens = rng.integers(0, 70_000, 64)
    offs = np.array([rng.integers(0, (1 << 20) - l) for l in lens])
    np.testing.assert_array_equal(reference.batch(arena, offs, lens), oracle_c.batch(arena, offs, lens))
    np.testing.assert_array_equal(reference.batch(arena, offs, lens, threads=4),
                                  oracle_c.batch(arena, offs, lens))


@pytest.mark.parametrize("name", ["mixed", "zipf_small", "fixed_4k", "corrupt_payload",
                                  "corrupt_crc", "multi_errors", "truncated_payload",
                                  "truncated_header", "bad_magic", "bad_version", "header_only"])
def test_integrity_scan_restatement(oracle_c, datafile_cases, name):
    case = {c["name"]: c for c in datafile_cases}[name]
    img = (GOLDEN / "datafiles" / f"{name}.d0").read_bytes()
    recs, errors, fatal = oracle_c.integrity_scan(img)
    stdout = (GOLDEN / "datafiles" / f"{name}.stdout").read_text()
    stderr = (GOLDEN / "datafiles" / f"{name}.stderr").read_text()
    # the reference prints one "data entry" block per walked record
    assert stdout.count("[+] data entry: ") == len(recs)
    assert stdout.count("data crc       : ok, match") == int((recs["status"] == 1).sum())
    assert stderr.count("integrity check failed") == errors
    if fatal == 0:
        assert case["exit"] == errors
    else:
        assert case["exit"] == 1
    if fatal == 1:
        assert "data header read failed" in stderr
    if fatal == 2:
        assert "payload entry read failed" in stderr
    if fatal == 3:
        assert "invalid header" in stdout or "unsupported version" in stdout
    # each reported mismatch carries (computed, expected) in that order
    bad = recs[recs["status"] == 0]
    for r in bad:
        assert f"{r['computed']:08x} <> {r['integrity']:08x}" in stderr
