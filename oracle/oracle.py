"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Python handle on the CPU checkers.  Imported only by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg -- never by the
product (0-db_amd/).

* ``liboracle.so`` (oracle/crc32c_oracle.c): the from-scratch C restatement
  of libzdb/crc32.c:84-91 and of integrity-check.c:59-105.
* ``libzdbref.so`` (oracle/_ref/, optional): the REAL reference
  libzdb/crc32.c compiled from /root/reference by oracle/Makefile, plus a
  batch driver (oracle/ref_batch.c).  Present wherever it was built here; it
  travels to the GPU box inside the gpurun snapshot.
* ``splitmix_bytes`` / ``crc32_py``: numpy / pure-Python restatements used to
  regenerate fixture inputs and cross-check small cases.

Parity is PINNED: tests/test_oracle.py checks all of the above against
tests/golden/, produced by running the reference itself (make_golden.py).
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ORACLE_SO = HERE / "_build" / "liboracle.so"
REF_SO = HERE / "_ref" / "libzdbref.so"
REF_INTEGRITY = HERE / "_ref" / "integrity-check"
REF_GEN = HERE / "_ref" / "gen_datafile_ref"

POLY = 0x82F63B78

RECORD_DTYPE = np.dtype([
    ("header_offset", "<u8"), ("payload_offset", "<u8"), ("idlength", "<u4"),
    ("datalength", "<u4"), ("previous", "<u4"), ("integrity", "<u4"), ("flags", "<u4"),
    ("computed", "<u4"), ("status", "<i4"), ("pad", "<u4"),
])


def _load(path: Path):
    if not path.exists():
        raise FileNotFoundError(f"{path} missing: run `make -C oracle` (and `make -C oracle ref`)")
    return C.CDLL(str(path))


class Oracle:
    """The C restatement (always available once `make -C oracle` ran)."""

    def __init__(self):
        lib = _load(ORACLE_SO)
        lib.oracle_crc32.restype = C.c_uint32
        lib.oracle_crc32.argtypes = [C.c_void_p, C.c_size_t]
        lib.oracle_crc32_batch.restype = None
        lib.oracle_crc32_batch.argtypes = [C.c_void_p] * 4 + [C.c_size_t]
        lib.oracle_table_entry.restype = C.c_uint32
        lib.oracle_table_entry.argtypes = [C.c_int]
        lib.oracle_integrity_scan.restype = C.c_long
        lib.oracle_integrity_scan.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_long,
                                              C.POINTER(C.c_int), C.POINTER(C.c_int)]
        lib.oracle_record_size.restype = C.c_long
        assert lib.oracle_record_size() == RECORD_DTYPE.itemsize
        self.lib = lib

    def crc32(self, data) -> int:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        return int(self.lib.oracle_crc32(a.ctypes.data if a.size else None, a.size))

    def batch(self, arena: np.ndarray, offsets, lengths) -> np.ndarray:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        out = np.zeros(len(offsets), dtype=np.uint32)
        self.lib.oracle_crc32_batch(arena.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                                    out.ctypes.data, len(offsets))
        return out

    def table(self) -> np.ndarray:
        return np.array([self.lib.oracle_table_entry(i) for i in range(256)], dtype=np.uint32)

    def integrity_scan(self, image) -> tuple[np.ndarray, int, int]:
        img = np.frombuffer(bytes(image), dtype=np.uint8) if not isinstance(image, np.ndarray) else image
        cap = img.size // 18 + 2
        recs = np.zeros(cap, dtype=RECORD_DTYPE)
        err = C.c_int(0)
        fatal = C.c_int(0)
        n = self.lib.oracle_integrity_scan(img.ctypes.data, img.size, recs.ctypes.data, cap,
                                           C.byref(err), C.byref(fatal))
        return recs[:n], err.value, fatal.value


class Reference:
    """The real libzdb/crc32.c (oracle/_ref/libzdbref.so)."""

    def __init__(self):
        lib = _load(REF_SO)
        lib.zdb_crc32.restype = C.c_uint32
        lib.zdb_crc32.argtypes = [C.c_void_p, C.c_ssize_t]
        lib.ref_crc32_batch.restype = None
        lib.ref_crc32_batch.argtypes = [C.c_void_p] * 4 + [C.c_size_t]
        lib.ref_crc32_batch_mt.restype = C.c_int
        lib.ref_crc32_batch_mt.argtypes = [C.c_void_p] * 4 + [C.c_size_t, C.c_int]
        lib.ref_engine.restype = C.c_char_p
        self.lib = lib

    @staticmethod
    def available() -> bool:
        return REF_SO.exists()

    def engine(self) -> str:
        return self.lib.ref_engine().decode()

    def crc32(self, data) -> int:
        a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        return int(self.lib.zdb_crc32(a.ctypes.data if a.size else None, a.size))

    def batch(self, arena: np.ndarray, offsets, lengths, threads: int = 1) -> np.ndarray:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        out = np.zeros(len(offsets), dtype=np.uint32)
        if threads <= 1:
            self.lib.ref_crc32_batch(arena.ctypes.data, offsets.ctypes.data, lengths.ctypes.data,
                                     out.ctypes.data, len(offsets))
        else:
            rc = self.lib.ref_crc32_batch_mt(arena.ctypes.data, offsets.ctypes.data,
                                             lengths.ctypes.data, out.ctypes.data, len(offsets),
                                             threads)
            assert rc == 0
        return out


# ------------------------------------------------------------ restatements --

GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def splitmix_bytes(nbytes: int, seed: int) -> np.ndarray:
    """Byte i = byte (i % 8) of LE mix64(seed + (i//8 + 1) * golden) -- the
    definition include/zdb_crc32.h documents for zdb_synth_fill."""
    words = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(1, words + 1, dtype=np.uint64)
        w = _mix64(np.uint64(seed) + idx * GOLDEN)
    return w.astype("<u8").view(np.uint8)[:nbytes].copy()


def crc32_py(data: bytes, crc: int = 0) -> int:
    """Bitwise restatement (pure Python, small inputs only)."""
    for b in data:
        crc ^= b
        for _ in range(8):
            crc = (crc >> 1) ^ (POLY if crc & 1 else 0)
    return crc
