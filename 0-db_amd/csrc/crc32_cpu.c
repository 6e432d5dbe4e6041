/*
 * Scalar (CPU) engine behind the drop-in entry points.
 *
 * Replaces libzdb/crc32.c as a link-time drop-in (crc32.h:5,8; api.h:72).
 * This path never initialises HIP: it serves the latency-bound callers -- the
 * key hash on every GET/SET/DEL (index.c:419-421) and single-record CHECK
 * (data.c:564) -- and is safe before zdbd's daemonize() fork (redis.c:1365).
 * Batched payload checksums go to the GPU entry points in crc32_hip.hip.
 *
 * Function: CRC-32C, reflected polynomial 0x82F63B78, initial register 0,
 * no final XOR (crc32.c:84-110).  Engines:
 *   "sse42"    one _mm_crc32_u64 dependency chain over 8-byte words, then
 *              bytes (the reference leaves a full last word to its byte loop,
 *              crc32.c:102; same value, so this engine keeps it in the chain);
 *   "software" byte table generated from the polynomial.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <sys/types.h>

#include "crc32c_gf2.h"

#ifdef __SSE4_2__
#include <nmmintrin.h>
#endif

char *zdb_crc32_engine_value() {
#ifdef __SSE4_2__
    return "sse42";
#else
    return "software";
#endif
}

uint32_t zdb_crc32(const uint8_t *bytes, ssize_t length) {
    if (length <= 0)
        return 0;
    size_t n = (size_t)length;
#ifdef __SSE4_2__
    uint64_t h = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, bytes + i, 8);
        h = _mm_crc32_u64(h, w);
    }
    uint32_t c = (uint32_t)h;
    for (; i < n; i++)
        c = _mm_crc32_u8(c, bytes[i]);
    return c;
#else
    return zdbcrc_update_bytes(0, bytes, n);
#endif
}

uint32_t zdb_checksum_crc32(const uint8_t *bytes, ssize_t length) {
    return zdb_crc32(bytes, length);
}

/* ---- GF(2) helpers exported through include/zdb_crc32.h ---------------- */

uint32_t zdb_crc32_shift(uint32_t crc, int64_t nbytes) {
    return zdbcrc_shift(crc, nbytes);
}

uint32_t zdb_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return zdbcrc_combine(crc_a, crc_b, len_b);
}

size_t zdb_crc32_table_image(uint32_t *dst, size_t dwords) {
    if (dst && dwords >= ZDBCRC_TABLE_DW)
        zdbcrc_build_tables(dst);
    return ZDBCRC_TABLE_DW;
}
