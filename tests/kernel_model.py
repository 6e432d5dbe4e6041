"""CPU model of crc_batch_kernel (0-db_amd/csrc/crc32_hip.hip), in numpy.

It replays the kernel's exact algorithm -- unit scan, per-wave unit slices,
segment walk, end-aligned lane mapping, supersteps of K slots, 5-bit table
lookups from the host-built table image, lane placement, trailing-pad removal
and the generic piece shift -- so the math can be checked against the oracle
on a machine without a GPU.  The GPU tests then check the HIP code itself.
"""
from __future__ import annotations

import numpy as np

K, PCH, SCH, WAVE = 4, 26, 7, 64
OFF_T = 0
OFF_W = OFF_T + K * PCH * 32
OFF_L = OFF_W + SCH * 32
LDS_DW = OFF_L + SCH * 32 * WAVE
OFF_Z = LDS_DW
OFF_R = OFF_Z + 16 * SCH * 32
RDIG = 4
OFF_F = OFF_R + RDIG * 256 * SCH * 32
OFF_TP = OFF_F + 4 * SCH * 32  # packed kernel: [K][PCH][32] slot tables (256 B per slot)
OFF_WP = OFF_TP + K * PCH * 32   # [SCH][32] advance over one packed superstep (1 KiB)
OFF_LP = OFF_WP + SCH * 32       # [SCH][32][32] placement of lane l & 31 in its row of 16
OFF_TE = OFF_LP + SCH * 32 * 32  # rows of 8 lanes: slot tables (128 B per slot)
OFF_WE = OFF_TE + K * PCH * 32   # ... advance over 512 B
OFF_TQ = OFF_WE + SCH * 32       # rows of 4 lanes: slot tables (64 B per slot)
OFF_WQ = OFF_TQ + K * PCH * 32   # ... advance over 256 B
OFF_TT = OFF_WQ + SCH * 32       # rows of 32 lanes: slot tables (512 B per slot)
OFF_WT = OFF_TT + K * PCH * 32   # ... advance over 2 KiB
OFF_LT = OFF_WT + SCH * 32       # ... placement of lane l & 31 in its row of 32
TABLE_DW = OFF_LT + SCH * 32 * 32
PK_TABLES = {32: (OFF_TT, OFF_WT), 16: (OFF_TP, OFF_WP), 8: (OFF_TE, OFF_WE), 4: (OFF_TQ, OFF_WQ)}
UNIT_OVH = 384
DWG_MIN_BYTES = 64 * 1024  # record-relative grids this long load from the dword below the record
MIN_UNITS_PER_WAVE = 256

LANES = np.arange(WAVE, dtype=np.int64)


def window_bit(j: int, t: int) -> int:
    """Piece bit behind index bit t of lookup window j (-1: unused), as
    zdbcrc_window_bit in 0-db_amd/csrc/crc32c_gf2.c defines the windows."""
    if j < 16:  # A: bits [8n+2, 8n+7) of dword j/4
        return 32 * (j >> 2) + 8 * (j & 3) + 2 + t
    if j < 24:  # B: rotl3(w_a) | rotl5(w_b), byte n
        a, n = (0 if j < 20 else 2), (j - 16) & 3
        return [32 * a + ((8 * n + 31) & 31), 32 * a + 8 * n, 32 * a + 8 * n + 1,
                32 * (a + 1) + 8 * n, 32 * (a + 1) + 8 * n + 1][t]
    m = 2 * (j - 24)  # C: bit 7 of bytes m, m+1 of w1 and w3
    return [32 + 8 * m + 7, 96 + 8 * m + 7, 32 + 8 * (m + 1) + 7, 96 + 8 * (m + 1) + 7, -1][t]


_WIN = np.array([[window_bit(j, t) for t in range(5)] for j in range(PCH)], dtype=np.int64)


def _slices128(words: np.ndarray) -> np.ndarray:
    """words: [64, 4] uint32 -> [64, 26] window indices of the 128-bit piece."""
    bits = np.unpackbits(words.astype("<u4").view(np.uint8), axis=1, bitorder="little").astype(np.int64)
    out = np.zeros((len(words), PCH), dtype=np.int64)
    for t in range(5):
        col = _WIN[:, t]
        out |= np.where(col >= 0, bits[:, np.maximum(col, 0)], 0) << t
    return out


def _slices32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    return np.stack([((x >> np.uint64(5 * c)) & np.uint64(31)).astype(np.int64) for c in range(SCH)], 1)


def _uniform_shift(x: int, tab: np.ndarray, base: int) -> int:
    r = 0
    for c in range(SCH):
        r ^= int(tab[base + c * 32 + ((x >> (5 * c)) & 31)])
    return r


def shift_pieces(x: int, q: int, tab: np.ndarray) -> int:
    """x shifted over q pieces: one radix-256 digit per table (seg_value_v3)."""
    j = 0
    while q:
        if q & 255:
            x = _uniform_shift(x, tab, OFF_R + (j * 256 + (q & 255)) * SCH * 32)
        q >>= 8
        j += 1
    return x


def _keep_mask(lo: int, hi: int, k: int) -> int:
    a, b = lo - 4 * k, hi - 4 * k
    mh = 0xFFFFFFFF if b >= 4 else 0 if b <= 0 else (1 << (8 * b)) - 1
    ml = 0xFFFFFFFF if a <= 0 else 0 if a >= 4 else (0xFFFFFFFF << (8 * a)) & 0xFFFFFFFF
    return mh & ml


def segment_crc(mem: np.ndarray, base_addr: int, P0: int, pa: int, pb: int, np_: int, lo0: int,
                hi_last: int, tab: np.ndarray) -> int:
    nps = pb - pa
    T = (nps + 63) // 64
    S = (T + K - 1) // K
    t0 = S * K - T
    base_j = pb - 64 * S * K
    acc = np.zeros(WAVE, dtype=np.uint32)
    for ss in range(S):
        if ss:
            sl = _slices32(acc)
            acc = np.bitwise_xor.reduce(tab[OFF_W + np.arange(SCH) * 32 + sl], axis=1).astype(np.uint32)
        for i in range(K):
            t = ss * K + i
            if t < t0:
                continue
            jj = base_j + 64 * t + LANES
            words = np.zeros((WAVE, 4), dtype=np.uint32)
            for l in range(WAVE):
                j = int(jj[l])
                if j < pa:
                    continue
                addr = P0 + 16 * j - base_addr
                wv = mem[addr:addr + 16].view("<u4").copy()
                if j == 0 or j == np_ - 1:
                    lo = lo0 if j == 0 else 0
                    hi = hi_last if j == np_ - 1 else 16
                    for k in range(4):
                        wv[k] &= np.uint32(_keep_mask(lo, hi, k))
                words[l] = wv
            sl = _slices128(words)
            idx = OFF_T + (i * PCH + np.arange(PCH)) * 32 + sl
            acc ^= np.bitwise_xor.reduce(tab[idx], axis=1).astype(np.uint32)
    sl = _slices32(acc)
    idx = OFF_L + (np.arange(SCH)[None, :] * 32 + sl) * WAVE + LANES[:, None]
    placed = np.bitwise_xor.reduce(tab[idx], axis=1)
    return int(np.bitwise_xor.reduce(placed))


def pieces_aligned(a: int, L: int) -> int:
    return ((a + L - 1) >> 4) - (a >> 4) + 1


def record_pieces(a: int, L: int) -> int:
    """Piece count of a record (crc32_hip.hip record_pieces): the 16-byte
    address grid, or the record-relative grid when L % 16 == 0 and that saves
    a 1 KiB step."""
    na, nr = pieces_aligned(a, L), L >> 4
    return nr if (L & 15) == 0 and (nr + 63) >> 6 < (na + 63) >> 6 else na


def ranges(total: int, nwaves: int, max_units: int, max_waves: int, dyn: int = 0, cpw: int = 4,
           pools: int = 8, dyn_min_units: int = 4096, max_chunks_per_record: int = 64) -> list:
    """The unit ranges the kernel's waves walk: static slices of the first
    (16 - dyn)/16 of [0, total), then the tail pool's chunks (pool p of
    `pools`, cpw chunks per wave) when the guards of crc_batch_kernel_v3 let
    the pool run.  Which wave claims a chunk does not change the result (cut
    partials are XORed), so the model only needs the ranges."""
    dyn_on = (dyn > 0 and total >= dyn_min_units * max_waves and
              max_units <= max_chunks_per_record * (total * dyn // 16 // (cpw * nwaves)))
    ts = total - total * dyn // 16 if dyn_on else total
    out = [(ts * gw // nwaves, ts * (gw + 1) // nwaves) for gw in range(nwaves)]
    if dyn_on:
        td = total - ts
        nch = cpw * (nwaves // pools)
        for p in range(pools):
            p0 = ts + td * p // pools
            pl = ts + td * (p + 1) // pools - p0
            out += [(p0 + pl * c // nch, p0 + pl * (c + 1) // nch) for c in range(nch)]
    return [(ub, ue) for ub, ue in out if ub < ue]


def batch(arena: np.ndarray, offsets, lengths, tab: np.ndarray, max_waves: int = 4096,
          min_units: int = MIN_UNITS_PER_WAVE, base_addr: int = 0, **pool) -> np.ndarray:
    """out[r] as crc_batch_kernel computes it.  base_addr is the (virtual)
    address of arena[0]; pieces are aligned on absolute addresses.  `pool`:
    the tail-pool parameters of `ranges` (default: no pool)."""
    offsets = np.asarray(offsets, dtype=np.int64)
    lengths = np.asarray(lengths, dtype=np.int64)
    n = len(offsets)
    out = np.zeros(n, dtype=np.uint32)
    if n == 0:
        return out
    # memory with slack so aligned reads never leave the buffer
    pad_lo = (base_addr & 15) + 16
    mem = np.zeros(pad_lo + len(arena) + 32, dtype=np.uint8)
    mem[pad_lo:pad_lo + len(arena)] = arena
    mem_base = base_addr - pad_lo  # absolute address of mem[0]

    A = base_addr + offsets
    units = np.array([record_pieces(int(a), int(L)) if L > 0 else 0 for a, L in zip(A, lengths)],
                     dtype=np.int64) + UNIT_OVH
    unit_start = np.zeros(n + 1, dtype=np.int64)
    unit_start[1:] = np.cumsum(units)
    total = int(unit_start[n])
    nwaves = min(max_waves, (total + min_units - 1) // min_units)
    for ub, ue in ranges(total, nwaves, int(units.max()), max_waves, **pool):
        r = int(np.searchsorted(unit_start, ub, side="right") - 1)
        while True:
            us = int(unit_start[r]) + UNIT_OVH
            ur = int(unit_start[r + 1])
            s_lo, s_hi = max(ub, us), min(ue, ur)
            if s_hi > s_lo:
                a = int(A[r])
                aend = a + int(lengths[r])
                np_ = ur - us
                rel = np_ != pieces_aligned(a, aend - a)
                h = a & 3 if rel and aend - a >= DWG_MIN_BYTES else 0  # loads from the dword below
                P0 = a - h if rel else a & ~15
                z = 0 if rel else P0 + 16 * np_ - aend
                pa, pb = s_lo - us, s_hi - us
                x = segment_crc(mem, mem_base, P0, pa, pb, np_, h if rel else a & 15, 16 - z, tab)
                if h:  # the record's last h bytes: crc(X || y) = shift(crc(X) ^ y, h)
                    y = 0
                    if pb == np_:
                        y = int.from_bytes(mem[aend - h - mem_base:aend - mem_base].tobytes(), "little")
                    x = _uniform_shift(x ^ y, tab, OFF_F + h * SCH * 32)
                elif z:
                    x = _uniform_shift(x, tab, OFF_Z + z * SCH * 32)
                x = shift_pieces(x, np_ - pb, tab)
                out[r] ^= np.uint32(x)  # store for whole records == xor into 0
            if ur >= ue or r + 1 >= n:
                break
            r += 1
    return out


# ------------------------------------------------------------ packed kernel --

def packed_geometry(A: int, L: int, rw: int = 16) -> dict:
    """One record's grid in crc_packed_kernel: pieces end at the dword Ep at or
    below the record's end E; the h = min(E & 3, L) bytes after it are folded
    in at the end, crc(X || y) = shift(crc(X) ^ y, h); piece 0 starts lo0
    bytes before the record (those bytes are masked off)."""
    E = A + L
    h = min(E & 3, L)
    Ep = E - h
    np_ = (L - h + 15) >> 4
    pps = K * rw  # pieces of a row per superstep
    return {"E": E, "h": h, "Ep": Ep, "np": np_, "lo0": 16 * np_ - (L - h), "S": (np_ + pps - 1) // pps}


def packed_row_crc(mem: np.ndarray, mem_base: int, A: int, L: int, S: int, row: int, tab: np.ndarray,
                   force_shifted_first: bool = False, rw: int = 16) -> int:
    """The crc one row of rw lanes computes for record (A, L) in a packet of S
    supersteps (S >= the record's own): with P = 4 rw pieces per superstep,
    position q = P s + rw i + l holds piece k = q - (P S - np) (k < 0: empty),
    loaded from Ep - 16 (P S - q).
    force_shifted_first: load every first piece the way the kernel loads one
    that starts in an unmapped page (the aligned block holding A, moved up)."""
    g = packed_geometry(A, L, rw)
    P = K * rw
    off_t, off_w = PK_TABLES[rw]
    kbase = P * S - g["np"]
    # what the kernel may read: A's 4 KiB page from A's 16-byte block on, up to
    # the 16-byte boundary after the record's last byte
    lo_ok, hi_ok = ((A & ~15) & ~4095), (g["E"] + 15) & ~15
    F0 = g["Ep"] - 16 * g["np"]
    d = (A & ~15) - F0 if g["np"] and F0 < (A & ~15) and (A & ~15) % 4096 == 0 else 0

    def check(addr: int, n: int):
        assert lo_ok <= addr and addr + n <= hi_ok, (A, L, addr, n)

    if g["h"]:
        check(g["Ep"] & ~3, 4)
    acc = np.zeros(rw, dtype=np.uint32)
    for s in range(S):
        if s:
            sl = _slices32(acc)
            acc = np.bitwise_xor.reduce(tab[off_w + np.arange(SCH) * 32 + sl], axis=1).astype(np.uint32)
        for i in range(K):
            words = np.zeros((rw, 4), dtype=np.uint32)
            for l16 in range(rw):
                q = P * s + rw * i + l16
                k = q - kbase
                if g["np"]:  # the kernel's load: positions k <= 0 read piece 0 (at F0 + d)
                    check(F0 + d if k <= 0 else g["Ep"] - 16 * (P * S - q), 16)
                if k < 0:
                    continue
                addr = g["Ep"] - 16 * (P * S - q)
                if k == 0 and force_shifted_first and addr < (A & ~15):
                    blk = mem[(A & ~15) - mem_base:(A & ~15) - mem_base + 16]
                    d = (A & ~15) - addr  # the block holds piece bytes [d, 16)
                    b = np.zeros(16, np.uint8)
                    b[d:] = blk[:16 - d]
                else:
                    b = mem[addr - mem_base:addr - mem_base + 16].copy()
                if k == 0:
                    b[:g["lo0"]] = 0
                words[l16] = b.view("<u4")
            sl = _slices128(words)
            idx = off_t + (i * PCH + np.arange(PCH)) * 32 + sl
            acc ^= np.bitwise_xor.reduce(tab[idx], axis=1).astype(np.uint32)
    sl = _slices32(acc)
    lanes = rw * row + np.arange(rw, dtype=np.int64)
    # LP column of lane l: l & 31 for rows of 16, else 16 - rw + l mod rw (+16 in the upper half);
    # rows of 32 read LT at column l & 31
    col = lanes & 31 if rw >= 16 else (16 - rw) + lanes % rw + (lanes & 16)
    idx = (OFF_LT if rw == 32 else OFF_LP) + (np.arange(SCH)[None, :] * 32 + sl) * 32 + col[:, None]
    x = int(np.bitwise_xor.reduce(np.bitwise_xor.reduce(tab[idx], axis=1)))
    if g["h"]:
        y = int.from_bytes(mem[g["Ep"] - mem_base:g["E"] - mem_base].tobytes(), "little")
        x = _uniform_shift(x ^ y, tab, OFF_F + g["h"] * SCH * 32)
    return x


def packed_batch(arena: np.ndarray, offsets, lengths, tab: np.ndarray, base_addr: int = 0,
                 force_shifted_first: bool = False, rw: int = 16) -> np.ndarray:
    """out[r] as crc_packed_kernel<RW = rw> computes it: records 64 / rw at a
    time (rows of a wave), every packet as many supersteps as its longest record."""
    nr = 64 // rw
    offsets = np.asarray(offsets, dtype=np.int64)
    lengths = np.asarray(lengths, dtype=np.int64)
    n = len(offsets)
    out = np.zeros(n, dtype=np.uint32)
    pad_lo = (base_addr & 15) + 32
    mem = np.zeros(pad_lo + len(arena) + 32, dtype=np.uint8)
    mem[pad_lo:pad_lo + len(arena)] = arena
    mem_base = base_addr - pad_lo
    for r0 in range(0, n, nr):
        recs = [(base_addr + int(offsets[r]), int(lengths[r])) for r in range(r0, min(n, r0 + nr))]
        S = max(max(packed_geometry(a, L, rw)["S"] for a, L in recs), 1)
        for g, (a, L) in enumerate(recs):
            out[r0 + g] = packed_row_crc(mem, mem_base, a, L, S, g, tab, force_shifted_first, rw)
    return out
