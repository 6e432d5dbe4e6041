"""CPU model of the f3 device walk (0-db_amd/csrc/datafile_hip.hip): the same
chunked speculative search, chain walk and exact stitch, step for step, in
plain Python -- so the algorithm is checked against the serial walk
(zdb_datafile_walk, itself pinned to the reference tool's output) on the CPU,
and the GPU tests then check the kernels against both.  Test infrastructure."""
from __future__ import annotations

import numpy as np

NONE = -1
CONT, OK, SHORT_HEADER, SHORT_PAYLOAD, BAD_DESCRIPTOR, EXCEEDS = -1, 0, 1, 2, 3, 4
MAXL, MAXF = 8 << 20, 3


def _le32(f: np.ndarray, p: int) -> int:
    b = f[p:p + 4]
    b = np.concatenate([b, np.zeros(4 - len(b), np.uint8)])  # images are readable past their end
    return int(b.view("<u4")[0])


def _byte(f: np.ndarray, p: int) -> int:
    return int(f[p]) if p < len(f) else 0


def hop(f, ln, pos):
    hlen = 18 + int(f[pos])
    if pos + hlen > ln:
        return SHORT_HEADER, 0, 0
    L = _le32(f, pos + 1)
    nxt = pos + hlen
    if L:
        if nxt + L > ln:
            return SHORT_PAYLOAD, nxt, L
        nxt += L
    return CONT, nxt, L


def walk_chain(f, ln, pos, cend, emit=None):
    count, st = 0, CONT
    while pos < cend:
        if pos >= ln:
            st = OK
            break
        s, nxt, L = hop(f, ln, pos)
        if s == SHORT_HEADER:
            st = s
            break
        if emit is not None:
            full = s == CONT and L > 0
            emit.append((pos, pos + 18 + int(f[pos]), L if full else 0, _le32(f, pos + 9) if full else 0))
        count += 1
        if s == SHORT_PAYLOAD:
            st = s
            break
        pos = nxt
    if st == CONT and pos >= ln:
        st = OK
    return count, pos, st


def plausible_successor(f, ln, p, idl, L):
    q = p + 18 + idl + L
    if q == ln:
        return True
    if q + 18 > ln:
        return False
    return _le32(f, q + 5) == (p & 0xFFFFFFFF)


SB, NF, NB = 8192, 2, 2  # search block bytes per wave, forward / backward waves per chunk


def candidate(f, ln, p):
    """filter: top byte of datalength 0 (L < 16 MiB; the writer caps at 8 MiB,
    data.h:6), flags <= 3 (data.h:47-51), the entry's own `previous` before it
    (data.c:601), then the successor's back-pointer"""
    return (_byte(f, p + 4) == 0 and _byte(f, p + 13) <= MAXF and _le32(f, p + 5) < p
            and plausible_successor(f, ln, p, int(f[p]), _le32(f, p + 1)))


def search(f, ln, c0, C):
    """the first entry header at or past c0, as walk_search_kernel finds it:
    forward from c0 and backward from c0 (the header of the entry straddling
    c0, whose end is the answer) in rounds of NF / NB blocks of SB bytes,
    whichever direction hits in the earlier round (forward on a tie)"""
    if ln < 18:
        return NONE
    lim = min(c0 + C, ln - 17)
    fwd = next((p for p in range(c0, lim) if candidate(f, ln, p)), NONE)
    k_end = max(0, -(-(lim - c0) // (NF * SB)) - 1)  # the last forward round
    rf = (fwd - c0) // (NF * SB) if fwd != NONE else None
    kmax = k_end if rf is None else rf - 1  # the backward search decides only in an earlier round
    lo = max(27, c0 - 1 - (kmax + 1) * NB * SB)
    bwd = next((p for p in range(c0 - 1, lo, -1) if candidate(f, ln, p)), NONE) if kmax >= 0 else NONE
    rb = ((c0 - 1 - bwd) // SB) // NB if bwd != NONE else None
    if rb is not None and rb <= kmax:
        e = bwd + 18 + int(f[bwd]) + _le32(f, bwd + 1)
        if e >= c0:
            return e if e < lim else NONE
    return fwd


def device_walk(f: np.ndarray, C: int, max_len: int | None = None):
    """-> (records [(entry, payload_off, plen, expected)], status, rewalks)"""
    ln = len(f)
    cpf = max(1, -(-(max_len if max_len is not None else ln) // C))
    # A1 + A2
    spec = []
    for c in range(cpf):
        c0 = c * C
        st, start = CONT, NONE
        if c == 0:
            if ln < 28 or bytes(f[:4]) != b"DAT0" or _le32(f, 4) != 3:
                st = BAD_DESCRIPTOR
            else:
                start = 28
        elif c0 < ln:
            start = search(f, ln, c0, C)
        if start != NONE:
            cnt, ex, st = walk_chain(f, ln, start, c0 + C)
            spec.append((start, ex, cnt, st))
        else:
            spec.append((NONE, 0, 0, st))
    # B
    if ln > cpf * C:
        return [], EXCEEDS, 0
    st, pos = CONT, 28
    if spec[0][3] == BAD_DESCRIPTOR:
        st = BAD_DESCRIPTOR
    true_start, redo = [], 0
    for c in range(cpf):
        cend = (c + 1) * C
        if st != CONT or pos >= cend:
            true_start.append(NONE)
            continue
        true_start.append(pos)
        s0, ex, cnt, cs = spec[c]
        if s0 != pos:
            cnt, ex, cs = walk_chain(f, ln, pos, cend)
            redo += 1
        pos, st = ex, cs
    # C
    recs = []
    for c in range(cpf):
        if true_start[c] != NONE:
            walk_chain(f, ln, true_start[c], (c + 1) * C, emit=recs)
    return recs, (OK if st == CONT else st), redo
