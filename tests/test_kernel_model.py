"""The kernel's algorithm, replayed on the CPU (tests/kernel_model.py) with
the library's real table image, against the oracle.  Covers the math of
crc32_hip.hip -- lane mapping, supersteps, edge masks, trailing-pad removal,
segment splits across waves and the atomic-XOR recombination -- without a
GPU.  The GPU tests check the HIP implementation of the same algorithm."""
from __future__ import annotations

import ctypes

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


def test_windows_cover_every_piece_bit_once():
    bits = [km.window_bit(j, t) for j in range(km.PCH) for t in range(5)]
    used = sorted(b for b in bits if b >= 0)
    assert used == list(range(128))
    # the library's table builder uses the same map (internal symbol: the
    # diagnostic build exports it, the product library does not)
    diag = ctypes.CDLL(str(zdbcrc.LIB_PATH.parent / "libzdbcrc_diag.so"))
    f = diag.zdbcrc_window_bit
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_int, ctypes.c_int]
    assert [f(j, t) for j in range(km.PCH) for t in range(5)] == bits


def test_table_spot_values(tab):
    # slot K-1 of the data tables is plain crc of a piece with one window bit set
    for j, t in ((0, 0), (5, 3), (16, 0), (23, 4), (24, 1), (25, 3)):
        b = km.window_bit(j, t)
        piece = np.zeros(16, np.uint8)
        piece[b >> 3] = 1 << (b & 7)
        assert tab[km.OFF_T + ((km.K - 1) * km.PCH + j) * 32 + (1 << t)] == oracle.crc32_py(piece.tobytes())
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


def test_radix_shift_tables(tab):
    """R[j][d] tables == zdb_crc32_shift by 16 * d * 256^j bytes."""
    rng = np.random.default_rng(8)
    for q in [1, 255, 256, 257, 65535, 65536, 1 << 24, (1 << 28) + 1, 0xFFFFFFFF]:
        x = int(rng.integers(1, 1 << 32))
        assert km.shift_pieces(x, q, tab) == zdbcrc.shift(x, 16 * q)


def test_record_relative_grid(oracle_c, tab):
    # 1 KiB-multiple records at misaligned addresses take the record-relative
    # piece grid (one step fewer); neighbours of other lengths stay aligned
    arena = oracle.splitmix_bytes(30_000, 33)
    lens = [4096, 1024, 2048, 4096 - 16, 4096 + 16, 1000, 4096, 17]
    offs = [26, 4200, 5301, 7400, 11533, 16000, 17013, 21111]
    for r, (o, L) in enumerate(zip(offs, lens)):
        if L % 1024 == 0 and o % 16:
            assert km.record_pieces(o, L) == L // 16 < km.pieces_aligned(o, L)
    # records of 64 KiB and more: loads start at the dword below the record
    # (h = A mod 4 bytes masked, the last h bytes folded in at the end)
    big = oracle.splitmix_bytes(300_000, 34)
    blens = [65536, 1024, 131072, 65536 + 16]
    boffs = [13, 65600, 66627, 197710]
    assert all(km.record_pieces(o, L) == L // 16 for o, L in zip(boffs, blens) if L % 1024 == 0)
    for base in (0, 1, 2, 3):
        for mw, mu in ((4096, 256), (9, 1)):
            got = km.batch(big, boffs, blens, tab, max_waves=mw, min_units=mu, base_addr=base)
            np.testing.assert_array_equal(got, oracle_c.batch(big, boffs, blens))
    for base in (0, 1, 2, 3):
        for mw, mu in ((4096, 256), (7, 1)):
            got = km.batch(arena, offs, lens, tab, max_waves=mw, min_units=mu, base_addr=base)
            np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


@pytest.mark.parametrize("dyn,cpw,pools", [(6, 4, 4), (8, 3, 2), (16, 1, 1), (2, 5, 4)])
def test_tail_pool_ranges(oracle_c, tab, dyn, cpw, pools):
    """The tail pool (crc_batch_kernel_v3 DYN): static slices + pool chunks
    tile the unit space exactly once, and the checksums match the oracle."""
    arena, offs, lens = _case(100 + dyn, 40, 3000, 60_000)
    units = np.array([km.record_pieces(3 + int(o), int(l)) if l else 0 for o, l in zip(offs, lens)]) + km.UNIT_OVH
    total = int(units.sum())
    rs = km.ranges(total, 16, int(units.max()), 16, dyn=dyn, cpw=cpw, pools=pools, dyn_min_units=8,
                   max_chunks_per_record=1 << 30)
    assert len(rs) > 16 or dyn == 16  # the pool ran (dyn 16: all of it)
    edges = sorted(rs)
    assert edges[0][0] == 0 and edges[-1][1] == total
    assert all(a[1] == b[0] for a, b in zip(edges, edges[1:]))
    got = km.batch(arena, offs, lens, tab, max_waves=16, min_units=1, base_addr=3, dyn=dyn, cpw=cpw,
                   pools=pools, dyn_min_units=8, max_chunks_per_record=1 << 30)
    np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


def test_tail_pool_guard():
    """No pool below 4096 units per wave, or when one record would span more
    than 64 chunks (its cut partials would serialise on one atomic)."""
    assert len(km.ranges(4096 * 16 - 1, 16, 100, 16, dyn=6)) == 16
    assert len(km.ranges(10 ** 7, 16, 100, 16, dyn=6, pools=8)) > 16
    chunk = 10 ** 7 * 6 // 16 // (4 * 16)
    assert len(km.ranges(10 ** 7, 16, 64 * chunk + 1, 16, dyn=6, pools=8)) == 16


@pytest.mark.parametrize("rw", [32, 16, 8, 4])
@pytest.mark.parametrize("force_shifted_first", [False, True])
@pytest.mark.parametrize("base", [0, 1, 2, 3, 13])
def test_packed_small_records(oracle_c, tab, base, force_shifted_first, rw):
    """the packed small-record kernel's math (rows of rw = 16 / 8 / 4 lanes,
    16 rw bytes per slot, dword-anchored grid + h-byte fold, packets as long as
    their longest record): lengths 0..4 KiB at every alignment, including
    records shorter than their fold and packets mixing supersteps; and the
    first-piece path the kernel takes when a piece would start in the page below"""
    rng = np.random.default_rng(300 + base)
    lens = np.concatenate([np.arange(0, 40), rng.integers(0, 4097, 120), [4096] * 8, [4095, 4097, 1024, 1023, 1025]])
    rng.shuffle(lens)
    gaps = rng.integers(0, 7, len(lens))
    offs = np.zeros(len(lens), np.int64)
    offs[1:] = np.cumsum(lens[:-1] + gaps[:-1])
    offs += 1
    arena = oracle.splitmix_bytes(int(offs[-1] + lens[-1]) + 16, 300 + base)
    got = km.packed_batch(arena, offs, lens, tab, base_addr=base, force_shifted_first=force_shifted_first, rw=rw)
    np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))


@pytest.mark.parametrize("rw", [32, 16, 8, 4])
def test_packed_long_record_in_packet(oracle_c, tab, rw):
    """a record longer than 4 KiB (a wrong max_length hint) stretches its packet: still exact"""
    lens = np.array([5, 70_000, 4096, 0, 33, 9000])
    offs = np.array([0, 7, 70_011, 74_200, 74_200, 74_300])
    arena = oracle.splitmix_bytes(90_000, 9)
    np.testing.assert_array_equal(km.packed_batch(arena, offs, lens, tab, rw=rw), oracle_c.batch(arena, offs, lens))


@pytest.mark.parametrize("rw", [32, 16, 4])
def test_packed_loads_stay_in_bounds(oracle_c, tab, rw):
    """every load the packed kernel issues (empty positions included) stays in
    A's 4 KiB page from A's 16-byte block on and below the 16-byte boundary
    after the record (packed_row_crc asserts it): records at the first bytes
    of pages, with every short length"""
    offs, lens = [], []
    for pg in range(1, 6):
        for a in range(16):
            for L in (1, 2, 3, 4, 5, 13, 17, 100, 1000, 4093, 4096):
                offs.append(4096 * 3 * pg + a)
                lens.append(L)
    offs, lens = np.array(offs), np.array(lens)
    arena = oracle.splitmix_bytes(int(offs.max() + lens.max()) + 32, 5)
    got = km.packed_batch(arena, offs, lens, tab, base_addr=1 << 20, rw=rw)
    np.testing.assert_array_equal(got, oracle_c.batch(arena, offs, lens))
