"""The kernel's algorithm, replayed on the CPU (tests/kernel_model.py) with
the library's real table image, against the oracle.  Covers the math of
crc32_hip.hip -- lane mapping, supersteps, edge masks, trailing-pad removal,
segment splits across waves and the atomic-XOR recombination -- without a
GPU.  The GPU tests check the HIP implementation of the same algorithm."""
from __future__ import annotations

import numpy as np
import pytest

import kernel_model as km
import oracle
import zdbcrc


@pytest.fixture(scope="module")
def tab():
    t = zdbcrc.table_image()
    assert len(t) == km.TABLE_DW
    return t


def _case(seed, nrec, maxlen, arena_len):
    rng = np.random.default_rng(seed)
    arena = oracle.splitmix_bytes(arena_len, seed)
    lens = rng.integers(0, maxlen + 1, nrec)
    offs = np.array([rng.integers(0, arena_len - l + 1) for l in lens])
    return arena, offs, lens


def test_table_spot_values(tab):
    # slot K-1 of the data tables is plain crc of a piece with one slice set
    piece = np.zeros(16, np.uint8)
    piece[0] = 1
    assert tab[km.OFF_T + ((km.K - 1) * km.PCH + 0) * 32 + 1] == oracle.crc32_py(piece.tobytes())
    # lane 63 is not shifted at all
    for v in range(32):
        assert tab[km.OFF_L + (0 * 32 + v) * 64 + 63] == v


@pytest.mark.parametrize("base", [0, 5, 15])
def test_edges_and_small(oracle_c, tab, base):
    arena = oracle.splitmix_bytes(5000, 11)
    lens = [0, 1, 2, 3, 4, 5, 8, 15, 16, 17, 20, 31, 32, 33, 47, 48, 49, 63, 64, 65]
    offs = [(7 * i) % 3000 for i in range(len(lens))]
    got = km.batch(arena, offs, lens, tab, base_addr=base)
    np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


@pytest.mark.parametrize("max_waves,min_units", [(4096, 256), (5, 16), (11, 1), (2, 1)])
def test_random_split_geometries(oracle_c, tab, max_waves, min_units):
    arena, offs, lens = _case(max_waves * 7 + min_units, 24, 9000, 60_000)
    got = km.batch(arena, offs, lens, tab, max_waves=max_waves, min_units=min_units, base_addr=3)
    np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


def test_multi_superstep_record(oracle_c, tab):
    # > K KiB so the register is advanced across supersteps; split 3 ways
    arena = oracle.splitmix_bytes(40_000, 21)
    offs, lens = [13, 100], [33_333, 5_000]
    for mw, mu in ((4096, 256), (3, 1)):
        got = km.batch(arena, offs, lens, tab, max_waves=mw, min_units=mu)
        np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


# ------------------------------------------------------------------ v4 -------

@pytest.mark.parametrize("max_waves,seed", [(4096, 1), (5, 2), (2, 3), (64, 4)])
def test_v4_random_geometries(oracle_c, tab, max_waves, seed):
    arena, offs, lens = _case(max_waves * 13 + seed, 24, 20_000, 80_000)
    got = km.batch_v4(arena, offs, lens, tab, max_waves=max_waves, base_addr=seed, seed=seed)
    np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


def test_v4_split_large_record(oracle_c, tab):
    arena = oracle.splitmix_bytes(300_000, 5)
    offs, lens = [7, 0, 299_000], [290_000, 100, 1000]
    for mw in (3, 17, 4096):
        got = km.batch_v4(arena, offs, lens, tab, max_waves=mw, base_addr=9, seed=mw)
        np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


@pytest.mark.parametrize("kind", ["zipf", "fixed4k", "single", "tiny"])
def test_v4_partition_exact(kind):
    """Every piece of every record is in exactly one chunk segment, at the
    full-size wave count; edges inside a record fall on np - 256 k."""
    if kind == "zipf":
        lens = zdbcrc.zipf_lengths(512 << 20, 0xC3C3C3)
    elif kind == "fixed4k":
        lens = np.full(131_072, 4096)
    elif kind == "single":
        lens = np.array([1 << 30])
    else:
        lens = np.arange(1, 200) % 7
    lens = np.asarray(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) + 3
    A = offs
    units = np.where(lens > 0, ((A + lens - 1) >> 4) - (A >> 4) + 1, 0) + km.UNIT_OVH
    us = np.zeros(len(lens) + 1, dtype=np.int64)
    us[1:] = np.cumsum(units)
    covered = np.zeros(len(lens), dtype=np.int64)
    last_pb = np.zeros(len(lens), dtype=np.int64)
    nseg = 0
    for _, r, pa, pb, np_ in km.v4_segments(us, 6144):
        assert pa == last_pb[r], (r, pa, last_pb[r])  # chunks visit a record in order, no gap/overlap
        assert (np_ - pb) % 256 == 0 and (pa == 0 or (np_ - pa) % 256 == 0)
        if np_ <= 256:
            assert pa == 0 and pb == np_
        last_pb[r] = pb
        covered[r] += pb - pa
        nseg += 1
    np.testing.assert_array_equal(covered, units - km.UNIT_OVH)
    assert nseg >= int((lens > 0).sum())
