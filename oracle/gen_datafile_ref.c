/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Fixture generator: writes real 0-db datafiles through the REFERENCE
 * library (libzdb objects compiled from /root/reference/libzdb by
 * oracle/Makefile into oracle/_ref/), so the datafile framing and the stored
 * `integrity` CRCs are produced by the reference code itself:
 *   zdb_api_set (api.c:268-306) -> api_set_handler_userkey (api.c:108-167,
 *   crc at :124) -> data_insert (data.c:594-633, header->integrity at :606).
 *   zdb_api_del (data_delete, data.c:653-671) writes datalength 0 / crc 0.
 *
 * The embedding follows examples/zdb-example.c, with the index mode set
 * explicitly (the default MIX mode indexes past the handler
 * table, bootstrap.c:46 / api.c:260-265).
 *
 * usage: gen_datafile_ref <rootdir> <mode> <count> <seed> [size]
 *   mode fixed : <count> values of exactly <size> bytes
 *   mode zipf  : SURVEY §8(d) C3 recipe until <size> payload bytes (cap count)
 *   mode mixed : small fixture mix -- short/long/empty-key-ish values, an
 *                overwrite and deletions
 * The datafile lands in <rootdir>/data/default/d0.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <math.h>
#include "libzdb.h"

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void fill(uint8_t *buf, size_t len, uint64_t seed) {
    for (size_t i = 0; i < len; i += 8) {
        uint64_t w = mix64(seed + (i / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        for (size_t k = 0; k < 8 && i + k < len; k++)
            buf[i + k] = (uint8_t)(w >> (8 * k));
    }
}

static uint64_t rng_state;
static uint64_t rng_next(void) {
    rng_state += 0x9E3779B97F4A7C15ULL;
    return mix64(rng_state);
}

static size_t zipf_size(void) {
    /* bucket k in 0..14 with P(k) ~ (k+1)^-1.1, size uniform in
     * [64*2^k, 64*2^(k+1)), capped at 1 MiB */
    double w[15], tot = 0;
    for (int k = 0; k < 15; k++) { w[k] = pow(k + 1, -1.1); tot += w[k]; }
    double u = (double)(rng_next() >> 11) / 9007199254740992.0 * tot;
    int k = 0;
    for (; k < 14; k++) { if (u < w[k]) break; u -= w[k]; }
    size_t lo = (size_t)64 << k, hi = (size_t)64 << (k + 1);
    size_t s = lo + rng_next() % (hi - lo);
    return s > (1u << 20) ? (1u << 20) : s;
}

static void set_one(namespace_t *ns, uint32_t idx, size_t size, uint64_t seed, uint8_t *buf) {
    char key[32];
    int klen = snprintf(key, sizeof(key), "k%u", idx);
    fill(buf, size, seed ^ ((uint64_t)idx << 32));
    zdb_api_t *reply = zdb_api_set(ns, key, klen, buf, size);
    zdb_api_reply_free(reply);
}

int main(int argc, char *argv[]) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s rootdir fixed|zipf|mixed count seed [size]\n", argv[0]);
        return 1;
    }
    char datapath[512], indexpath[512];
    snprintf(datapath, sizeof(datapath), "%s/data", argv[1]);
    snprintf(indexpath, sizeof(indexpath), "%s/index", argv[1]);
    const char *mode = argv[2];
    long count = atol(argv[3]);
    uint64_t seed = strtoull(argv[4], NULL, 0);
    size_t size = argc > 5 ? strtoull(argv[5], NULL, 0) : 4096;
    rng_state = seed;

    zdb_settings_t *settings = zdb_initialize();
    zdb_id_set("oracle-fixture");
    settings->datapath = datapath;
    settings->indexpath = indexpath;
    settings->mode = ZDB_MODE_KEY_VALUE;
    settings->datasize = (size_t)1 << 31; /* never rotate inside one fixture */
    zdb_open(settings);
    namespace_t *ns = namespace_get_default();

    uint8_t *buf = malloc(8u << 20);
    if (!strcmp(mode, "fixed")) {
        for (long i = 0; i < count; i++)
            set_one(ns, (uint32_t)i, size, seed, buf);
    } else if (!strcmp(mode, "zipf")) {
        size_t total = 0;
        for (long i = 0; i < count && total < size; i++) {
            size_t s = zipf_size();
            set_one(ns, (uint32_t)i, s, seed, buf);
            total += s;
        }
    } else if (!strcmp(mode, "mixed")) {
        /* lengths that exercise the sse42 loop edges (crc32.c:101-108):
         * 1..9 bytes, multiples of 8, odd sizes, a 64 KiB value */
        static const size_t sizes[] = {1, 2, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65,
                                       100, 255, 256, 1000, 1023, 1024, 1025,
                                       4095, 4096, 4097, 12345, 65536};
        long n = (long)(sizeof(sizes) / sizeof(sizes[0]));
        for (long i = 0; i < n && i < count; i++)
            set_one(ns, (uint32_t)i, sizes[i], seed, buf);
        /* overwrite k3 with a different value: a second entry for the key */
        set_one(ns, 3, 333, seed + 1, buf);
        /* delete two keys: datalength-0 entries, flags DELETED (data.c:653-671) */
        zdb_api_reply_free(zdb_api_del(ns, "k5", 2));
        zdb_api_reply_free(zdb_api_del(ns, "k11", 3));
        set_one(ns, 1000, 777, seed, buf);
    } else {
        fprintf(stderr, "unknown mode %s\n", mode);
        return 1;
    }
    free(buf);
    zdb_close(settings);
    return 0;
}
