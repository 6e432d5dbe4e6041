/*
 * Datafile framing and header walk (see include/zdb_datafile.h).
 *
 * The walk is the host half of the integrity scan: it turns the serial chain
 * of entry headers (each header gives the next offset: integrity-check.c:59-69,
 * data.c:306-311) into descriptors (payload offset, length, stored crc) that
 * the GPU checksums in one batch.  It reads an image already in memory -- no
 * per-record read()/lseek() syscalls, which are ~70 % of the reference tool's
 * time.
 */
#include <stdint.h>
#include <string.h>

#include "zdb_datafile.h"

static uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static void wr32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

long zdb_datafile_walk(const uint8_t *image, size_t len, zdb_record_t *recs, long max_records, int *status) {
    int dummy;
    if (!status)
        status = &dummy;
    *status = ZDB_WALK_OK;
    if (len < ZDB_DATA_HEADER_SIZE || memcmp(image, "DAT0", 4) != 0 ||
        rd32(image + 4) != ZDB_DATAFILE_VERSION) {
        *status = ZDB_WALK_BAD_DESCRIPTOR;
        return 0;
    }
    size_t pos = ZDB_DATA_HEADER_SIZE;
    long count = 0;
    while (pos < len) {
        const uint8_t *h = image + pos;
        size_t hlen = ZDB_ENTRY_HEADER_SIZE + (size_t)h[0];
        if (pos + hlen > len) {
            *status = ZDB_WALK_SHORT_HEADER;
            return count;
        }
        zdb_record_t rec;
        memset(&rec, 0, sizeof(rec));
        rec.header_offset = pos;
        rec.idlength = h[0];
        rec.datalength = rd32(h + 1);
        rec.previous = rd32(h + 5);
        rec.integrity = rd32(h + 9);
        rec.flags = h[13];
        rec.timestamp = rd32(h + 14);
        rec.payload_offset = pos + hlen;
        if (recs && count < max_records)
            recs[count] = rec;
        count++;
        pos += hlen;
        if (rec.datalength) {
            if (pos + rec.datalength > len) {
                *status = ZDB_WALK_SHORT_PAYLOAD;
                return count;
            }
            pos += rec.datalength;
        }
    }
    return count;
}

size_t zdb_datafile_encode_entry(uint8_t *dst, const uint8_t *id, uint8_t idlength, uint32_t datalength,
                                 uint32_t previous, uint32_t integrity, uint8_t flags, uint32_t timestamp) {
    dst[0] = idlength;
    wr32(dst + 1, datalength);
    wr32(dst + 5, previous);
    wr32(dst + 9, integrity);
    dst[13] = flags;
    wr32(dst + 14, timestamp);
    if (idlength)
        memcpy(dst + ZDB_ENTRY_HEADER_SIZE, id, idlength);
    return ZDB_ENTRY_HEADER_SIZE + (size_t)idlength;
}

size_t zdb_datafile_encode_header(uint8_t *dst, uint32_t fileid) {
    memcpy(dst, "DAT0", 4);
    wr32(dst + 4, ZDB_DATAFILE_VERSION);
    memset(dst + 8, 0, 16); /* created / opened = 0 (data.c data_initialize) */
    wr32(dst + 24, fileid);
    return ZDB_DATA_HEADER_SIZE;
}

size_t zdb_datafile_payloads(const zdb_record_t *recs, size_t nrecs, uint64_t *offsets, uint32_t *lengths,
                             uint32_t *expected, uint32_t *record_index) {
    size_t m = 0;
    for (size_t i = 0; i < nrecs; i++) {
        if (!recs[i].datalength)
            continue;
        offsets[m] = recs[i].payload_offset;
        lengths[m] = recs[i].datalength;
        if (expected)
            expected[m] = recs[i].integrity;
        if (record_index)
            record_index[m] = (uint32_t)i;
        m++;
    }
    return m;
}

size_t zdb_datafile_encode_batch(uint8_t *dst, size_t cap, uint64_t file_offset, const uint8_t *keys,
                                 const uint64_t *key_offsets, const uint8_t *key_lengths,
                                 const uint8_t *values, const uint64_t *value_offsets,
                                 const uint32_t *value_lengths, const uint32_t *crcs, size_t n,
                                 uint32_t timestamp, uint32_t *previous, uint64_t *entry_offsets) {
    size_t pos = 0;
    uint32_t prev = previous ? *previous : 0;
    for (size_t i = 0; i < n; i++) {
        const size_t need = ZDB_ENTRY_HEADER_SIZE + key_lengths[i] + (size_t)value_lengths[i];
        if (pos + need > cap)
            return 0;
        const uint64_t here = file_offset + pos;
        pos += zdb_datafile_encode_entry(dst + pos, keys + key_offsets[i], key_lengths[i], value_lengths[i],
                                         prev, crcs[i], 0, timestamp);
        if (value_lengths[i])
            memcpy(dst + pos, values + value_offsets[i], value_lengths[i]);
        pos += value_lengths[i];
        if (entry_offsets)
            entry_offsets[i] = here;
        prev = (uint32_t)here; /* root->previous = offset (data.c:630) */
    }
    if (previous)
        *previous = prev;
    return pos;
}
