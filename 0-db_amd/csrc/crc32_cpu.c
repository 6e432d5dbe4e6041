/*
 * Scalar (CPU) engine behind the drop-in entry points.
 *
 * Replaces libzdb/crc32.c as a link-time drop-in (crc32.h:5,8): this file
 * (plus crc32c_gf2.c for the software engine's table) defines exactly the
 * two symbols crc32.c defines, so lib/crc32_cpu.o can take crc32.o's place in
 * libzdb.a without clashing with api.o's zdb_checksum_crc32 (api.c:470-472,
 * which keeps calling zdb_crc32).  oracle/Makefile `dropin` links it so.
 * This path never initialises HIP: it serves the latency-bound callers -- the
 * key hash on every GET/SET/DEL (index.c:419-421) and single-record CHECK
 * (data.c:564) -- and is safe before zdbd's daemonize() fork (redis.c:1365).
 * Batched payload checksums go to the GPU entry points in crc32_hip.hip.
 *
 * Function: CRC-32C, reflected polynomial 0x82F63B78, initial register 0,
 * no final XOR (crc32.c:84-130).  Engines, chosen at compile time in the
 * reference's order (crc32.c:133-155):
 *   "sse42"    one _mm_crc32_u64 dependency chain over 8-byte words, then
 *              bytes (the reference leaves a full last word to its byte loop,
 *              crc32.c:102; same value, so this engine keeps it in the chain);
 *   "armv8"    the same chain with the ACLE __crc32cd / __crc32cb
 *              instructions (crc32.c:115-130), on AArch64 with +crc;
 *   "software" byte table generated from the polynomial.
 *
 * ZDBCRC_ARMV8_EMULATE (tests only, tests/test_host.py): builds the armv8
 * engine on x86 with the two ACLE intrinsics spelled by their SSE4.2 twins
 * (same polynomial, same reflected 8-byte/1-byte register update), so its
 * loop and engine name are exercised where no AArch64 compiler exists.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <sys/types.h>

#include "crc32c_gf2.h"

#if defined(ZDBCRC_ARMV8_EMULATE)
#include <nmmintrin.h>
#define ZDBCRC_ENGINE_ARMV8 1
static inline uint32_t zdbcrc_crc32cd(uint32_t c, uint64_t w) { return (uint32_t)_mm_crc32_u64(c, w); }
static inline uint32_t zdbcrc_crc32cb(uint32_t c, uint8_t b) { return _mm_crc32_u8(c, b); }
#elif defined(__SSE4_2__)
#include <nmmintrin.h>
#define ZDBCRC_ENGINE_SSE42 1
#elif defined(__ARM_FEATURE_CRC32)
#include <arm_acle.h>
#define ZDBCRC_ENGINE_ARMV8 1
#define zdbcrc_crc32cd __crc32cd
#define zdbcrc_crc32cb __crc32cb
#endif

char *zdb_crc32_engine_value() {
#if defined(ZDBCRC_ENGINE_SSE42)
    return "sse42";
#elif defined(ZDBCRC_ENGINE_ARMV8)
    return "armv8";
#else
    return "software";
#endif
}

uint32_t zdb_crc32(const uint8_t *bytes, ssize_t length) {
    if (length <= 0)
        return 0;
    size_t n = (size_t)length;
#if defined(ZDBCRC_ENGINE_SSE42)
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
#elif defined(ZDBCRC_ENGINE_ARMV8)
    uint32_t c = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) { /* unaligned-safe word load (the reference casts, crc32.c:116) */
        uint64_t w;
        memcpy(&w, bytes + i, 8);
        c = zdbcrc_crc32cd(c, w);
    }
    for (; i < n; i++)
        c = zdbcrc_crc32cb(c, bytes[i]);
    return c;
#else
    return zdbcrc_update_bytes(0, bytes, n);
#endif
}
