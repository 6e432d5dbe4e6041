/*
 * zdb_datafile.h -- 0-db datafile framing and the host-side record walk that
 * feeds the batched GPU checksum (library: 0-db_amd/lib/libzdbcrc.so).
 *
 * On-disk format, datafile version 3 (libzdb/libzdb.h:29), little endian,
 * packed:
 *   data_header_t       (libzdb/data.h:38-45) 28 bytes: "DAT0", u32 version,
 *                        u64 created, u64 opened, u32 fileid
 *   data_entry_header_t (libzdb/data.h:56-65) 18 bytes: u8 idlength,
 *                        u32 datalength, u32 previous, u32 integrity,
 *                        u8 flags, u32 timestamp; then id[idlength], then
 *                        datalength payload bytes.
 * `integrity` (byte 9 of the entry header) is zdb_crc32(payload).
 */
#ifndef ZDB_DATAFILE_AMD_H
#define ZDB_DATAFILE_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZDB_DATAFILE_VERSION   3
#define ZDB_DATA_HEADER_SIZE  28
#define ZDB_ENTRY_HEADER_SIZE 18
#define ZDB_ENTRY_DELETED      1  /* data.h:48 */
#define ZDB_ENTRY_TRUNCATED    2  /* data.h:49 */

typedef struct zdb_record_t {
    uint64_t header_offset;   /* offset of the entry header in the file   */
    uint64_t payload_offset;  /* offset of the payload                    */
    uint32_t datalength;      /* payload bytes                            */
    uint32_t integrity;       /* stored crc                               */
    uint32_t previous;        /* previous entry offset                    */
    uint32_t timestamp;
    uint8_t idlength;
    uint8_t flags;
    uint8_t pad[6];
} zdb_record_t;

/* walk status, mirroring how tools/integrity-check stops */
#define ZDB_WALK_OK             0  /* clean end of file (integrity-check.c:59)        */
#define ZDB_WALK_SHORT_HEADER   1  /* "data header read failed" (:68-69)              */
#define ZDB_WALK_SHORT_PAYLOAD  2  /* "payload entry read failed" (:87-88)            */
#define ZDB_WALK_BAD_DESCRIPTOR 3  /* short file header, magic or version (data.c:197-206) */
#define ZDB_WALK_EXCEEDS_BOUND  4  /* device walk only: file longer than the caller's max_file_len */

/* Walk the entry headers of an in-memory datafile image (the serial chain of
 * integrity-check.c:59-69 / data.c:306-311).  Fills up to max_records
 * descriptors in file order and returns the number of records walked
 * (including the one that stopped a SHORT_PAYLOAD walk); pass recs = NULL to
 * count only. */
long zdb_datafile_walk(const uint8_t *image, size_t len, zdb_record_t *recs, long max_records,
                       int *status);

/* Encode one entry header + key at dst (data_insert, data.c:594-633; the
 * caller passes the payload crc, as data.c:606 takes source->crc).  Returns
 * bytes written (18 + idlength). */
size_t zdb_datafile_encode_entry(uint8_t *dst, const uint8_t *id, uint8_t idlength, uint32_t datalength,
                                 uint32_t previous, uint32_t integrity, uint8_t flags, uint32_t timestamp);

/* Encode the 28-byte file header (data_initialize, data.c: created/opened 0). */
size_t zdb_datafile_encode_header(uint8_t *dst, uint32_t fileid);

/* SET-path batching hook (the in-order second phase of a pipelined SET
 * batch): append n entries to a datafile image at dst (capacity cap bytes),
 * exactly as n successive data_insert calls would (data.c:594-633): header
 * with the caller-computed crc (from zdb_crc32_batch*), key, payload;
 * `previous` chains each entry to the one before, starting from *previous
 * (the offset of the last entry already in the file), and file_offset is
 * the offset at which dst will be written.  key i is keys[key_offsets[i] ..
 * + key_lengths[i]], value i is values[value_offsets[i] .. + value_lengths[i]].
 * Entry i's file offset is written to entry_offsets[i] (may be NULL) and
 * *previous is updated.  Returns bytes written, 0 if cap is too small. */
size_t zdb_datafile_encode_batch(uint8_t *dst, size_t cap, uint64_t file_offset, const uint8_t *keys,
                                 const uint64_t *key_offsets, const uint8_t *key_lengths,
                                 const uint8_t *values, const uint64_t *value_offsets,
                                 const uint32_t *value_lengths, const uint32_t *crcs, size_t n,
                                 uint32_t timestamp, uint32_t *previous, uint64_t *entry_offsets);

/* Gather descriptors for the batched checksum: records with datalength > 0
 * (integrity-check.c:81-82 skips empty ones).  Returns the count written. */
size_t zdb_datafile_payloads(const zdb_record_t *recs, size_t nrecs, uint64_t *offsets, uint32_t *lengths,
                             uint32_t *expected, uint32_t *record_index);

/* Batched CHECK (f4): data_check_real (data.c:533-571, the CHECK command,
 * commands_dataset.c:54-102) for n index-given record offsets at once, over a
 * datafile image resident in device memory (d_image[0..image_len)).  For
 * record i: decode the entry header at d_offsets[i], checksum its payload on
 * the GPU and compare with the header's integrity field.  d_result[i] (device
 * i32) = 1 when they match, 0 when not, -1 when the header or the payload
 * does not fit in the image (the reference's short-read -1).  Enqueued on
 * `stream` (a hipStream_t, NULL = default); HIP errors are returned, there
 * is no CPU fallback. */
int zdb_datafile_check_device(const uint8_t *d_image, uint64_t image_len, const uint64_t *d_offsets,
                              int32_t *d_result, size_t n, void *stream);

/* f3 -- record-boundary discovery on the GPU (the serial chain of
 * integrity-check.c:59-69 / data.c:306-311, found without it): nfiles
 * datafile images in device memory, file i at d_image + d_file_off[i] of
 * d_file_len[i] bytes (device arrays; every file <= max_file_len <= 4 GiB,
 * the image readable 16 bytes past each file's end).  Each file is cut into
 * chunks of chunk_bytes (a power of two >= 1 KiB; 0 = 8 MiB) whose chains
 * are discovered speculatively (header filter + the next entry's `previous`
 * back-pointer) and stitched exactly from offset 28; a chunk whose guess is
 * wrong is re-walked serially, so the result is always the serial walk's.
 *
 * Outputs (device, written on `stream`, asynchronous):
 *   d_file_records[nfiles + 1]  exclusive prefix of the files' record counts
 *                               (entry nfiles = total records);
 *   d_file_status[nfiles]       ZDB_WALK_* of each file, as zdb_datafile_walk;
 *   d_rewalks[nfiles + 1]       chunks re-walked serially per file (+ total);
 *   up to `capacity` records in file order: d_entry_off (image offset of the
 *   entry header), d_payload_off, d_payload_len and d_expected (the stored
 *   integrity).  d_payload_len / d_expected are 0 for records the
 *   integrity check skips (datalength 0, integrity-check.c:81-82) and for a
 *   payload cut by the end of the file (ZDB_WALK_SHORT_PAYLOAD), so the
 *   descriptors feed zdb_crc32_verify_device as they are. */
int zdb_datafile_walk_device(const uint8_t *d_image, const uint64_t *d_file_off, const uint64_t *d_file_len,
                             uint32_t nfiles, uint64_t max_file_len, uint32_t chunk_bytes, uint64_t *d_entry_off,
                             uint64_t *d_payload_off, uint32_t *d_payload_len, uint32_t *d_expected,
                             uint64_t capacity, uint64_t *d_file_records, int32_t *d_file_status,
                             uint32_t *d_rewalks, void *stream);

/* device buffers of a device-resident integrity scan (all device pointers) */
typedef struct zdb_scan_buffers_t {
    uint64_t *entry_off;      /* [capacity]                                  */
    uint64_t *payload_off;    /* [capacity]                                  */
    uint32_t *payload_len;    /* [capacity]                                  */
    uint32_t *expected;       /* [capacity] stored integrity (0 if skipped)  */
    uint32_t *computed;       /* [capacity] crc of each payload              */
    uint64_t capacity;
    uint64_t *file_records;   /* [nfiles + 1]                                */
    int32_t *file_status;     /* [nfiles]                                    */
    uint32_t *rewalks;        /* [nfiles + 1]                                */
    uint32_t *mismatch;       /* [max_mismatch] record indices, unordered    */
    uint32_t *mismatch_count; /* [1]                                         */
    uint32_t max_mismatch;
} zdb_scan_buffers_t;

/* The integrity scan of a whole store, device-resident (tools/integrity-check
 * over every file: integrity-check.c:59-105): zdb_datafile_walk_device, then
 * the batched checksum + compare (zdb_crc32_verify_device) over the walked
 * records -- the record count stays in device memory between the two -- and
 * one synchronisation at the end that returns it (*n_records).
 * Returns ZDB_CRC32_ENOSPC (with *n_records set; computed / mismatch then
 * cover the first `capacity` records only) when capacity is too small. */
int zdb_datafile_scan_device(const uint8_t *d_image, const uint64_t *d_file_off, const uint64_t *d_file_len,
                             uint32_t nfiles, uint64_t max_file_len, uint32_t chunk_bytes,
                             const zdb_scan_buffers_t *buffers, uint64_t *n_records, void *stream);

#ifdef __cplusplus
}
#endif

#endif
