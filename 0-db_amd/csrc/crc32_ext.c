/*
 * The rest of libzdbcrc.so's scalar ABI (include/zdb_crc32.h), kept out of
 * crc32_cpu.o so that object defines exactly what libzdb/crc32.c defines:
 *   zdb_checksum_crc32 -- the tools' entry point (api.h:72 / api.c:470-472),
 *                         exported here for programs that link libzdbcrc.so
 *                         instead of libzdb (in libzdb it stays api.c's);
 *   GF(2) helpers and the kernel's table image (new).
 */
#include <stdint.h>
#include <stddef.h>
#include <sys/types.h>

#include "crc32c_gf2.h"
#include "zdb_crc32.h"

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
