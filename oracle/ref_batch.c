/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * Batch driver around the REFERENCE zdb_crc32 (libzdb/crc32.c:145-155,
 * compiled unmodified from /root/reference by oracle/Makefile into
 * oracle/_ref/).  It is the "reference" CPU baseline that bench.py times
 * beside the GPU kernel, and the generator of golden vectors
 * (tests/golden/make_golden.py).  Each call is exactly one zdb_crc32 call,
 * like the reference callers (commands_set.c:106, integrity-check.c:90).
 */
#include <stdint.h>
#include <stddef.h>
#include <pthread.h>
#include <sys/types.h>

uint32_t zdb_crc32(const uint8_t *bytes, ssize_t length);
char *zdb_crc32_engine_value();

void ref_crc32_batch(const uint8_t *arena, const uint64_t *offsets,
                     const uint32_t *lengths, uint32_t *out, size_t n) {
    for (size_t r = 0; r < n; r++)
        out[r] = zdb_crc32(arena + offsets[r], (ssize_t)lengths[r]);
}

typedef struct shard_t {
    const uint8_t *arena;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint32_t *out;
    size_t lo, hi;
} shard_t;

static void *shard_main(void *p) {
    shard_t *s = (shard_t *)p;
    for (size_t r = s->lo; r < s->hi; r++)
        s->out[r] = zdb_crc32(s->arena + s->offsets[r], (ssize_t)s->lengths[r]);
    return NULL;
}

/* one contiguous shard of records per thread ("one shard each") */
int ref_crc32_batch_mt(const uint8_t *arena, const uint64_t *offsets,
                       const uint32_t *lengths, uint32_t *out, size_t n, int threads) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    shard_t sh[256];
    for (int t = 0; t < threads; t++) {
        sh[t].arena = arena; sh[t].offsets = offsets; sh[t].lengths = lengths; sh[t].out = out;
        sh[t].lo = n * (size_t)t / (size_t)threads;
        sh[t].hi = n * (size_t)(t + 1) / (size_t)threads;
        if (pthread_create(&tid[t], NULL, shard_main, &sh[t]) != 0)
            return -1;
    }
    for (int t = 0; t < threads; t++)
        pthread_join(tid[t], NULL);
    return 0;
}

const char *ref_engine(void) { return zdb_crc32_engine_value(); }
