"""ctypes binding of libzdbcrc.so (the C ABI in include/zdb_crc32.h and
include/zdb_datafile.h) for the Python test-suite, bench.py and
__graft_entry__.py.

The product is the C library; this module only marshals pointers.  It never
computes a checksum itself and never falls back to anything: if the shared
library is missing it raises at import, and every batched call raises
``ZdbCrcError`` on a non-zero status.

Device buffers are passed as torch tensors (torch is plumbing here: device
memory, streams, torch.distributed); the library sees raw pointers and the
raw hipStream_t of torch's current stream.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ZDBCRC_LIB", HERE / "lib" / "libzdbcrc.so"))

if not LIB_PATH.exists():
    raise ImportError(
        f"libzdbcrc.so not found at {LIB_PATH}: build it with `make -C 0-db_amd` "
        "(or __graft_entry__.build()); there is no fallback implementation")

# torch's wheel carries its own HIP runtime (libamdhip64.so + its own HSA
# runtime) beside the ROCm one this library links (libamdhip64.so.7).  The
# two coexist in one process only when torch's is loaded first (the other
# order leaves this library without a device), so load torch, when it is
# installed, before the library.  Importing torch does not initialise a GPU.
try:
    import torch  # noqa: F401
except ImportError:
    pass

_lib = C.CDLL(str(LIB_PATH))

u8p = C.POINTER(C.c_uint8)
vp = C.c_void_p


def _fn(name, restype, *argtypes):
    f = getattr(_lib, name)
    f.restype = restype
    f.argtypes = list(argtypes)
    return f


# scalar drop-ins (crc32.h:5,8; api.h:72)
_engine_value = _fn("zdb_crc32_engine_value", C.c_char_p)
_crc32 = _fn("zdb_crc32", C.c_uint32, vp, C.c_ssize_t)
_checksum = _fn("zdb_checksum_crc32", C.c_uint32, vp, C.c_ssize_t)
_shift = _fn("zdb_crc32_shift", C.c_uint32, C.c_uint32, C.c_int64)
_combine = _fn("zdb_crc32_combine", C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64)
_table_image = _fn("zdb_crc32_table_image", C.c_size_t, vp, C.c_size_t)

# batched GPU entries
_strerror = _fn("zdb_crc32_strerror", C.c_char_p, C.c_int)
_batch_engine = _fn("zdb_crc32_batch_engine", C.c_char_p)
_gpu_initialized = _fn("zdb_crc32_gpu_initialized", C.c_int)
_batch_device = _fn("zdb_crc32_batch_device", C.c_int, vp, vp, vp, vp, C.c_size_t, vp)
_batch_device_sized = _fn("zdb_crc32_batch_device_sized", C.c_int, vp, vp, vp, vp, C.c_size_t, C.c_uint32, vp)
_verify_device = _fn("zdb_crc32_verify_device", C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_uint32,
                     C.c_size_t, vp)
_batch_host = _fn("zdb_crc32_batch", C.c_int, vp, C.c_size_t, vp, vp, vp, C.c_size_t)
_check_device = _fn("zdb_datafile_check_device", C.c_int, vp, C.c_uint64, vp, vp, C.c_size_t, vp)
_walk_device = _fn("zdb_datafile_walk_device", C.c_int, vp, vp, vp, C.c_uint32, C.c_uint64, C.c_uint32, vp, vp,
                   vp, vp, C.c_uint64, vp, vp, vp, vp)


class ScanBuffers(C.Structure):
    """zdb_scan_buffers_t (include/zdb_datafile.h)"""
    _fields_ = [("entry_off", vp), ("payload_off", vp), ("payload_len", vp), ("expected", vp), ("computed", vp),
                ("capacity", C.c_uint64), ("file_records", vp), ("file_status", vp), ("rewalks", vp),
                ("mismatch", vp), ("mismatch_count", vp), ("max_mismatch", C.c_uint32)]


_scan_device = _fn("zdb_datafile_scan_device", C.c_int, vp, vp, vp, C.c_uint32, C.c_uint64, C.c_uint32,
                   C.POINTER(ScanBuffers), C.POINTER(C.c_uint64), vp)
_host_alloc = _fn("zdb_crc32_host_alloc", vp, C.c_size_t)
_host_free = _fn("zdb_crc32_host_free", None, vp)
_set_timing = _fn("zdb_crc32_set_timing", None, C.c_int)
_kernel_stats = _fn("zdb_crc32_kernel_stats", C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64))

# synthetic inputs
_synth_fill = _fn("zdb_synth_fill", None, vp, C.c_size_t, C.c_uint64)
_synth_fill_device = _fn("zdb_synth_fill_device", C.c_int, vp, C.c_size_t, C.c_uint64, vp)
_zipf = _fn("zdb_synth_zipf_lengths", C.c_size_t, vp, C.c_size_t, C.c_uint64, C.c_uint64)

# datafile framing
_walk = _fn("zdb_datafile_walk", C.c_long, vp, C.c_size_t, vp, C.c_long, C.POINTER(C.c_int))
_encode_entry = _fn("zdb_datafile_encode_entry", C.c_size_t, vp, vp, C.c_uint8, C.c_uint32, C.c_uint32,
                    C.c_uint32, C.c_uint8, C.c_uint32)
_encode_header = _fn("zdb_datafile_encode_header", C.c_size_t, vp, C.c_uint32)
_encode_batch = _fn("zdb_datafile_encode_batch", C.c_size_t, vp, C.c_size_t, C.c_uint64, vp, vp, vp, vp, vp,
                    vp, vp, C.c_size_t, C.c_uint32, C.POINTER(C.c_uint32), vp)

#: every symbol include/*.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "zdb_crc32_engine_value", "zdb_crc32", "zdb_checksum_crc32", "zdb_crc32_shift",
    "zdb_crc32_combine", "zdb_crc32_table_image", "zdb_crc32_strerror", "zdb_crc32_batch_engine",
    "zdb_crc32_gpu_initialized", "zdb_crc32_batch_device", "zdb_crc32_batch_device_sized",
    "zdb_crc32_verify_device",
    "zdb_crc32_batch", "zdb_crc32_device_count", "zdb_crc32_use_device", "zdb_crc32_host_alloc",
    "zdb_crc32_host_free", "zdb_crc32_host_register", "zdb_crc32_host_unregister", "zdb_crc32_set_timing",
    "zdb_crc32_kernel_stats", "zdb_synth_fill", "zdb_synth_fill_device", "zdb_synth_zipf_lengths",
    "zdb_datafile_walk", "zdb_datafile_encode_entry", "zdb_datafile_encode_header",
    "zdb_datafile_payloads", "zdb_datafile_encode_batch", "zdb_datafile_check_device",
    "zdb_datafile_walk_device", "zdb_datafile_scan_device", "zdb_crc32_stream_open", "zdb_crc32_stream_begin",
    "zdb_crc32_stream_append", "zdb_crc32_stream_checksum", "zdb_crc32_stream_close",
]

RECORD_DTYPE = np.dtype([
    ("header_offset", "<u8"), ("payload_offset", "<u8"), ("datalength", "<u4"),
    ("integrity", "<u4"), ("previous", "<u4"), ("timestamp", "<u4"), ("idlength", "u1"),
    ("flags", "u1"), ("pad", "u1", (6,)),
])
assert RECORD_DTYPE.itemsize == 40

WALK_OK, WALK_SHORT_HEADER, WALK_SHORT_PAYLOAD, WALK_BAD_DESCRIPTOR, WALK_EXCEEDS_BOUND = 0, 1, 2, 3, 4
ENOSPC = -5


class ZdbCrcError(RuntimeError):
    pass


def _check(rc: int, what: str):
    if rc != 0:
        raise ZdbCrcError(f"{what}: {_strerror(rc).decode()} ({rc})")


def _ptr(buf) -> int:
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            raise ValueError("array must be C-contiguous")
        return buf.ctypes.data
    if isinstance(buf, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(buf, dtype=np.uint8)
        return arr.ctypes.data
    raise TypeError(type(buf))


# ---------------------------------------------------------------- scalar --

def engine_value() -> str:
    return _engine_value().decode()


def crc32(data) -> int:
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return int(_crc32(arr.ctypes.data if arr.size else None, arr.size))


def checksum_crc32(data) -> int:
    arr = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return int(_checksum(arr.ctypes.data if arr.size else None, arr.size))


def shift(crc: int, nbytes: int) -> int:
    return int(_shift(crc, nbytes))


def combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(_combine(crc_a, crc_b, len_b))


def table_image() -> np.ndarray:
    n = _table_image(None, 0)
    img = np.zeros(n, dtype=np.uint32)
    _table_image(img.ctypes.data, n)
    return img


# ----------------------------------------------------------------- batch --

def batch_engine() -> str:
    return _batch_engine().decode()


def gpu_initialized() -> bool:
    return bool(_gpu_initialized())


def _stream_handle(stream) -> int | None:
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def _dev_check(t, dtype, name):
    import torch
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


def batch_device(arena, offsets, lengths, out, stream=None, max_length: int | None = None):
    """out[r] = zdb_crc32(arena[offsets[r]:][:lengths[r]]) on the GPU (async).
    max_length: an upper bound of the lengths the caller knows
    (zdb_crc32_batch_device_sized), None = unknown."""
    import torch
    _dev_check(arena, torch.uint8, "arena")
    _dev_check(offsets, torch.int64, "offsets")
    _dev_check(lengths, torch.int32, "lengths")
    _dev_check(out, torch.int32, "out")
    n = offsets.numel()
    if lengths.numel() != n or out.numel() < n:
        raise ValueError("descriptor sizes differ")
    if max_length is None:
        _check(_batch_device(arena.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), out.data_ptr(), n,
                             _stream_handle(stream)), "zdb_crc32_batch_device")
    else:
        _check(_batch_device_sized(arena.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), out.data_ptr(), n,
                                   max_length, _stream_handle(stream)), "zdb_crc32_batch_device_sized")
    return out


def datafile_check_device(image, record_offsets, result, stream=None):
    """Batched CHECK (data_check_real, data.c:533-571) over a device-resident
    datafile image: result[i] = 1 / 0 / -1 (match / mismatch / short read)."""
    import torch
    for t, d, nm in ((image, torch.uint8, "image"), (record_offsets, torch.int64, "record_offsets"),
                     (result, torch.int32, "result")):
        _dev_check(t, d, nm)
    _check(_check_device(image.data_ptr(), image.numel(), record_offsets.data_ptr(), result.data_ptr(),
                         record_offsets.numel(), _stream_handle(stream)), "zdb_datafile_check_device")


class DeviceStore:
    """A store of datafile images in device memory (torch tensors) and the
    buffers of a device walk / scan over it (f3: zdb_datafile_walk_device,
    zdb_datafile_scan_device)."""

    def __init__(self, image, file_off, file_len, capacity: int, max_mismatch: int = 1024):
        import torch
        _dev_check(image, torch.uint8, "image")
        self.image = image
        self.file_off = torch.as_tensor(np.asarray(file_off, np.int64)).cuda()
        self.file_len = torch.as_tensor(np.asarray(file_len, np.int64)).cuda()
        self.nfiles = len(file_off)
        self.max_file_len = int(np.max(file_len)) if len(file_len) else 0
        dv = image.device
        self.capacity = capacity
        self.entry_off = torch.zeros(max(capacity, 1), dtype=torch.int64, device=dv)
        self.payload_off = torch.zeros(max(capacity, 1), dtype=torch.int64, device=dv)
        self.payload_len = torch.zeros(max(capacity, 1), dtype=torch.int32, device=dv)
        self.expected = torch.zeros(max(capacity, 1), dtype=torch.int32, device=dv)
        self.computed = torch.zeros(max(capacity, 1), dtype=torch.int32, device=dv)
        self.file_records = torch.zeros(self.nfiles + 1, dtype=torch.int64, device=dv)
        self.file_status = torch.zeros(max(self.nfiles, 1), dtype=torch.int32, device=dv)
        self.rewalks = torch.zeros(self.nfiles + 1, dtype=torch.int32, device=dv)
        self.mismatch = torch.zeros(max(max_mismatch, 1), dtype=torch.int32, device=dv)
        self.mismatch_count = torch.zeros(1, dtype=torch.int32, device=dv)
        self.max_mismatch = max_mismatch
        self.buffers = ScanBuffers(
            self.entry_off.data_ptr(), self.payload_off.data_ptr(), self.payload_len.data_ptr(),
            self.expected.data_ptr(), self.computed.data_ptr(), capacity, self.file_records.data_ptr(),
            self.file_status.data_ptr(), self.rewalks.data_ptr(), self.mismatch.data_ptr(),
            self.mismatch_count.data_ptr(), max_mismatch)

    def walk(self, chunk_bytes: int = 0, stream=None):
        """async: descriptors of every record, in file order"""
        _check(_walk_device(self.image.data_ptr(), self.file_off.data_ptr(), self.file_len.data_ptr(), self.nfiles,
                            self.max_file_len, chunk_bytes, self.entry_off.data_ptr(), self.payload_off.data_ptr(),
                            self.payload_len.data_ptr(), self.expected.data_ptr(), self.capacity,
                            self.file_records.data_ptr(), self.file_status.data_ptr(), self.rewalks.data_ptr(),
                            _stream_handle(stream)), "zdb_datafile_walk_device")

    def scan(self, chunk_bytes: int = 0, stream=None) -> int:
        """walk + checksum + compare (synchronises once); returns the record count"""
        n = C.c_uint64(0)
        rc = _scan_device(self.image.data_ptr(), self.file_off.data_ptr(), self.file_len.data_ptr(), self.nfiles,
                          self.max_file_len, chunk_bytes, C.byref(self.buffers), C.byref(n), _stream_handle(stream))
        if rc == ENOSPC:
            raise ZdbCrcError(f"zdb_datafile_scan_device: {n.value} records > capacity {self.capacity}")
        _check(rc, "zdb_datafile_scan_device")
        return n.value


def verify_device(arena, offsets, lengths, expected, out, mismatch, count, stream=None):
    import torch
    for t, d, nm in ((arena, torch.uint8, "arena"), (offsets, torch.int64, "offsets"),
                     (lengths, torch.int32, "lengths"), (expected, torch.int32, "expected"),
                     (out, torch.int32, "out"), (mismatch, torch.int32, "mismatch"),
                     (count, torch.int32, "count")):
        _dev_check(t, d, nm)
    n = offsets.numel()
    _check(_verify_device(arena.data_ptr(), offsets.data_ptr(), lengths.data_ptr(), expected.data_ptr(),
                          out.data_ptr(), mismatch.data_ptr(), count.data_ptr(), mismatch.numel(), n,
                          _stream_handle(stream)), "zdb_crc32_verify_device")


def batch_host(arena: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> np.ndarray:
    """Host buffers in, host crcs out (synchronous).  An arena inside a
    PinnedBuffer is read in place by the kernel (zero-copy), any other one is
    staged; batches of at most 1,024 records return through the mailbox."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    out = np.zeros(len(offsets), dtype=np.uint32)
    _check(_batch_host(arena.ctypes.data, arena.size, offsets.ctypes.data, lengths.ctypes.data,
                       out.ctypes.data, len(offsets)), "zdb_crc32_batch")
    return out


class PinnedBuffer:
    """Pinned host staging (zdb_crc32_host_alloc) exposed as a numpy array."""

    def __init__(self, nbytes: int):
        self.nbytes = nbytes
        self.ptr = _host_alloc(nbytes)
        if not self.ptr:
            raise ZdbCrcError("zdb_crc32_host_alloc failed")
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            _host_free(self.ptr)
            self.ptr = None


def set_timing(enable: bool):
    _set_timing(1 if enable else 0)


def kernel_stats():
    ms = C.c_double(0)
    n = C.c_uint64(0)
    _check(_kernel_stats(C.byref(ms), C.byref(n)), "zdb_crc32_kernel_stats")
    return ms.value, n.value


# ------------------------------------------------------------- synthetic --

def synth_fill(nbytes: int, seed: int) -> np.ndarray:
    buf = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        _synth_fill(buf.ctypes.data, nbytes, seed)
    return buf


def synth_fill_device(t, seed: int, stream=None):
    import torch
    _dev_check(t, torch.uint8, "buffer")
    _check(_synth_fill_device(t.data_ptr(), t.numel(), seed, _stream_handle(stream)),
           "zdb_synth_fill_device")


def zipf_lengths(target_bytes: int, seed: int, max_n: int | None = None) -> np.ndarray:
    if max_n is None:
        max_n = max(16, target_bytes // 64 + 16)
    out = np.empty(max_n, dtype=np.uint32)
    n = _zipf(out.ctypes.data, max_n, target_bytes, seed)
    return out[:n].copy()


# -------------------------------------------------------------- datafile --

def datafile_walk(image) -> tuple[np.ndarray, int]:
    img = np.frombuffer(image, dtype=np.uint8) if not isinstance(image, np.ndarray) else image
    st = C.c_int(0)
    n = _walk(img.ctypes.data, img.size, None, 0, C.byref(st))
    recs = np.zeros(max(n, 1), dtype=RECORD_DTYPE)
    n2 = _walk(img.ctypes.data, img.size, recs.ctypes.data, n, C.byref(st))
    assert n2 == n
    return recs[:n], st.value


def encode_header(fileid: int = 0) -> bytes:
    buf = np.zeros(28, dtype=np.uint8)
    _encode_header(buf.ctypes.data, fileid)
    return buf.tobytes()


def encode_entry(key: bytes, datalength: int, previous: int, integrity: int, flags: int = 0,
                 timestamp: int = 0) -> bytes:
    buf = np.zeros(18 + len(key), dtype=np.uint8)
    k = np.frombuffer(key, dtype=np.uint8) if key else None
    n = _encode_entry(buf.ctypes.data, k.ctypes.data if k is not None else None, len(key), datalength,
                      previous, integrity, flags, timestamp)
    return buf[:n].tobytes()


def encode_batch(keys: list[bytes], values: np.ndarray, value_offsets, value_lengths, crcs, file_offset: int,
                 previous: int = 0, timestamp: int = 0):
    """In-order append of n entries (data_insert semantics) -> (bytes, previous, entry_offsets)."""
    kl = np.array([len(k) for k in keys], dtype=np.uint8)
    ko = np.zeros(len(keys), dtype=np.uint64)
    if len(keys) > 1:
        ko[1:] = np.cumsum(kl[:-1], dtype=np.uint64)
    kb = np.frombuffer(b"".join(keys) or b"\0", dtype=np.uint8)
    vo = np.ascontiguousarray(value_offsets, dtype=np.uint64)
    vl = np.ascontiguousarray(value_lengths, dtype=np.uint32)
    cr = np.ascontiguousarray(crcs, dtype=np.uint32)
    cap = int(vl.sum(dtype=np.uint64)) + int(kl.sum()) + 18 * len(keys)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    prev = C.c_uint32(previous)
    eo = np.zeros(len(keys), dtype=np.uint64)
    n = _encode_batch(out.ctypes.data, cap, file_offset, kb.ctypes.data, ko.ctypes.data, kl.ctypes.data,
                      values.ctypes.data, vo.ctypes.data, vl.ctypes.data, cr.ctypes.data, len(keys), timestamp,
                      C.byref(prev), eo.ctypes.data)
    if n != cap:
        raise ZdbCrcError("zdb_datafile_encode_batch: capacity")
    return out[:n].tobytes(), prev.value, eo
