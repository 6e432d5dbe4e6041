/*
 * zdb_crc32.h -- C ABI of the MI355X-native batched record checksum for 0-db.
 *
 * Library: 0-db_amd/lib/libzdbcrc.so (build: make -C 0-db_amd).
 * No torch types, no HIP types: plain pointers, sizes and an opaque stream.
 *
 * Checksum function everywhere: 0-db's "crc32" = CRC-32C (reflected poly
 * 0x82F63B78) with initial register 0 and NO final XOR (libzdb/crc32.c:84-110).
 * It is not the standard CRC-32C ("123456789" -> 0x58e3fa20, not 0xe3069283).
 */
#ifndef ZDB_CRC32_AMD_H
#define ZDB_CRC32_AMD_H

#include <stdint.h>
#include <stddef.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------
 * 1. Drop-in scalar entry points (CPU only, never initialise the GPU).
 *    Bit-exact replacements for the reference symbols; link this library (or
 *    its crc32_cpu.o) in place of libzdb/crc32.o.
 * ------------------------------------------------------------------------ */

/* replaces crc32.h:5 / crc32.c:133-143 -- "sse42" or "software" */
char *zdb_crc32_engine_value();

/* replaces crc32.h:8 / crc32.c:145-155; length <= 0 returns 0 */
uint32_t zdb_crc32(const uint8_t *bytes, ssize_t length);

/* replaces api.h:72 / api.c:470-472 (the tools' entry point) */
uint32_t zdb_checksum_crc32(const uint8_t *bytes, ssize_t length);

/* GF(2) helpers (new): register advanced over nbytes zero bytes (nbytes < 0
 * applies the inverse), and crc(A||B) from crc(A), crc(B), |B|. */
uint32_t zdb_crc32_shift(uint32_t crc, int64_t nbytes);
uint32_t zdb_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* Introspection: writes the host-built table image that the kernel stages
 * (layout: 0-db_amd/csrc/crc32c_gf2.h) when dwords is large enough; returns
 * the image size in dwords.  Used by the CPU model of the kernel in tests. */
size_t zdb_crc32_table_image(uint32_t *dst, size_t dwords);

/* ------------------------------------------------------------------------
 * 2. Batched GPU entry points (new, additive).
 *    One call checksums n independent records of an arena:
 *        out[r] = zdb_crc32(arena + offsets[r], lengths[r])
 *    This is the batched form of every payload caller: SET
 *    (commands_set.c:106, :216; api.c:124, :204), CHECK (data.c:564) and the
 *    integrity scan (integrity-check.c:90).
 *    HIP is initialised lazily on the first batched call (after any fork).
 *    Errors are returned, never hidden: there is no CPU fallback inside.
 * ------------------------------------------------------------------------ */

#define ZDB_CRC32_OK            0
#define ZDB_CRC32_ENODEV       -1  /* no usable gfx950 device / HIP runtime */
#define ZDB_CRC32_EINVAL       -2  /* bad argument                          */
#define ZDB_CRC32_ENOMEM       -3  /* device allocation failed              */
#define ZDB_CRC32_ELAUNCH      -4  /* kernel launch / runtime error         */
#define ZDB_CRC32_ENOSPC       -5  /* caller's output buffers too small     */

const char *zdb_crc32_strerror(int code);

/* "hip-gfx950" once a device is bound, "uninitialized" before */
const char *zdb_crc32_batch_engine(void);

/* 1 when this process has initialised HIP through this library */
int zdb_crc32_gpu_initialized(void);

/* Device-resident batch.  All pointers are device pointers on the calling
 * thread's current HIP device; `stream` is a hipStream_t (NULL = default
 * stream).  Asynchronous: results are valid once the stream has reached the
 * point of the call.  Records may start and end at any byte alignment and may
 * overlap; lengths may be 0 (crc 0).  The arena must stay readable up to the
 * 16-byte boundary that follows each record's last byte (true for any
 * allocation from hipMalloc).  n < 2^32 (ZDB_CRC32_EINVAL otherwise). */
int zdb_crc32_batch_device(const uint8_t *d_arena, const uint64_t *d_offsets,
                           const uint32_t *d_lengths, uint32_t *d_out,
                           size_t n, void *stream);

/* As zdb_crc32_batch_device, for a caller that knows an upper bound of its
 * record lengths (max_length, 0 = unknown): batches of records <= 4 KiB
 * (fixed-size values, pipelined small SETs) take the packed kernel, one
 * record per row of 16 lanes (4 per wave); <= 2 KiB rows of 8 lanes, <= 512 B
 * rows of 4 (8 / 16 records per wave).  Exact for any input; a record longer
 * than the bound only costs speed.  The host-buffer entry points measure the
 * bound themselves. */
int zdb_crc32_batch_device_sized(const uint8_t *d_arena, const uint64_t *d_offsets,
                                 const uint32_t *d_lengths, uint32_t *d_out,
                                 size_t n, uint32_t max_length, void *stream);

/* Device-resident verify: as zdb_crc32_batch_device, then compares with
 * d_expected[r] (the stored `integrity` field, data.h:60).  Mismatching record
 * indices are appended (unordered) to d_mismatch[0..max_mismatch) and
 * counted in *d_mismatch_count (device u32, zeroed by this call). */
int zdb_crc32_verify_device(const uint8_t *d_arena, const uint64_t *d_offsets,
                            const uint32_t *d_lengths, const uint32_t *d_expected,
                            uint32_t *d_out, uint32_t *d_mismatch,
                            uint32_t *d_mismatch_count, uint32_t max_mismatch,
                            size_t n, void *stream);

/* Host-buffer batch: out[r] for host descriptors over a host arena,
 * synchronous.  An arena inside memory from zdb_crc32_host_alloc is read by
 * the kernel in place over PCIe (zero-copy: one launch, one small copy back);
 * any other arena is staged to the device first.  The launch is sized to
 * the batch (one 256 KiB value does not start the whole persistent grid). */
int zdb_crc32_batch(const uint8_t *arena, size_t arena_len, const uint64_t *offsets,
                    const uint32_t *lengths, uint32_t *out, size_t n);

/* ------------------------------------------------------------------------
 * 2b. Host -> device ingest stream (f1: datafiles on disk).
 *     A device image filled chunk by chunk through a ring of pinned staging
 *     slots: each append copies into the next free slot and queues its H2D
 *     copy, so the caller's next read overlaps the previous transfer; then
 *     one batched checksum over the image.  One stream per host thread, on
 *     the device current at open.
 * ------------------------------------------------------------------------ */
#define ZDB_CRC32_STREAM_MAX_SLOTS 8

typedef struct zdb_crc32_stream_t zdb_crc32_stream_t;

/* NULL on failure (no device, bad arguments: 4 KiB <= slot_bytes, 2 <= slots
 * <= ZDB_CRC32_STREAM_MAX_SLOTS) */
zdb_crc32_stream_t *zdb_crc32_stream_open(size_t slot_bytes, int slots);

/* start a new image of image_bytes (waits for the previous one's copies) */
int zdb_crc32_stream_begin(zdb_crc32_stream_t *s, size_t image_bytes);

/* append n bytes at the end of the image (EINVAL past image_bytes).  A
 * source inside pinned memory (zdb_crc32_host_alloc, zdb_crc32_host_register)
 * is copied by one DMA straight from it with no staging copy and no wait: it
 * must then stay unchanged until the next begin or checksum on the stream. */
int zdb_crc32_stream_append(zdb_crc32_stream_t *s, const uint8_t *src, size_t n);

/* out[r] = zdb_crc32(image + offsets[r], lengths[r]) over the bytes appended
 * so far (EINVAL for a record past them); synchronous */
int zdb_crc32_stream_checksum(zdb_crc32_stream_t *s, const uint64_t *offsets, const uint32_t *lengths,
                              uint32_t *out, size_t n);

void zdb_crc32_stream_close(zdb_crc32_stream_t *s);

/* Number of usable HIP devices (initialises HIP; 0 when there is none). */
int zdb_crc32_device_count(void);

/* Bind the calling thread's batched calls to device `device` (HIP's
 * per-thread current device; one host thread per GPU for multi-GPU scans --
 * calls on different devices run concurrently). */
int zdb_crc32_use_device(int device);

/* pinned host memory for the host-buffer path (readable 64 bytes past
 * `bytes`; batches over it are zero-copy) */
void *zdb_crc32_host_alloc(size_t bytes);
void zdb_crc32_host_free(void *p);

/* pin existing host memory [p, p + bytes) in place (e.g. a reader's
 * huge-page buffer, so that a datafile is read straight into DMA-able
 * memory: f1 ingest); batches whose arena lies inside it (16 bytes readable
 * past the arena) are zero-copy, stream appends from it are direct DMAs.
 * Unregister before unmapping or reusing the range for anything else. */
int zdb_crc32_host_register(void *p, size_t bytes);
void zdb_crc32_host_unregister(void *p);

/* Instrumentation: when enabled, the main kernel of every batched call is
 * bracketed by HIP events on the caller's stream; the accumulated time of
 * completed launches is returned by zdb_crc32_kernel_stats (synchronises on
 * the recorded events). */
void zdb_crc32_set_timing(int enable);
int zdb_crc32_kernel_stats(double *total_ms, uint64_t *launches);

/* ------------------------------------------------------------------------
 * 3. Deterministic synthetic inputs (bench / tests on both hosts).
 *    Byte i of a filled buffer is byte (i mod 8) of the little-endian word
 *    splitmix64_mix(seed + (i/8 + 1) * 0x9E3779B97F4A7C15).
 * ------------------------------------------------------------------------ */
void zdb_synth_fill(uint8_t *buf, size_t len, uint64_t seed);
int zdb_synth_fill_device(uint8_t *d_buf, size_t len, uint64_t seed, void *stream);

/* SURVEY §8(d) C3 recipe: bucket k in 0..14 with P(k) ~ (k+1)^-1.1, size
 * uniform in [64*2^k, 64*2^(k+1)), capped at 1 MiB, drawn until the running
 * total reaches target_bytes (or max_n records).  Returns the count. */
size_t zdb_synth_zipf_lengths(uint32_t *lengths, size_t max_n,
                              uint64_t target_bytes, uint64_t seed);

#ifdef __cplusplus
}
#endif

#endif
