/*
 * TEST DOUBLE -- a stand-in for libzdbcrc.so's GPU entry points, so the
 * integrity tool's multi-GPU orchestration (worker -> device mapping, the
 * start-up thread, the ingest stream calls) is testable on a machine without
 * a GPU (tests/test_tool_multi.py).  It pretends to have
 * $ZDBCRC_STUB_DEVICES devices, logs every device bind and checksum call to
 * $ZDBCRC_STUB_LOG, and checksums on the CPU with the scalar drop-in engine
 * (crc32_cpu.c).  Never shipped, never loaded outside that test.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>

#include "zdb_crc32.h"

static __thread int t_dev = 0;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

static void logf_(const char *fmt, int a, long b) {
    const char *p = getenv("ZDBCRC_STUB_LOG");
    if (!p)
        return;
    pthread_mutex_lock(&mu);
    FILE *f = fopen(p, "a");
    if (f) {
        fprintf(f, fmt, a, b);
        fclose(f);
    }
    pthread_mutex_unlock(&mu);
}

const char *zdb_crc32_strerror(int code) { return code ? "stub error" : "ok"; }

int zdb_crc32_device_count(void) {
    const char *e = getenv("ZDBCRC_STUB_DEVICES");
    return e ? atoi(e) : 1;
}

int zdb_crc32_use_device(int d) {
    if (d < 0 || d >= zdb_crc32_device_count())
        return ZDB_CRC32_EINVAL;
    t_dev = d;
    logf_("bind %d %ld\n", d, (long)pthread_self() % 100000);
    return 0;
}

int zdb_crc32_batch(const uint8_t *arena, size_t arena_len, const uint64_t *offsets, const uint32_t *lengths,
                    uint32_t *out, size_t n) {
    (void)arena_len;
    for (size_t i = 0; i < n; i++)
        out[i] = zdb_crc32(arena + offsets[i], (ssize_t)lengths[i]);
    return 0;
}

struct zdb_crc32_stream_t {
    int dev;
    uint8_t *img;
    size_t cap, fill;
};

zdb_crc32_stream_t *zdb_crc32_stream_open(size_t slot_bytes, int slots) {
    (void)slot_bytes;
    (void)slots;
    zdb_crc32_stream_t *s = calloc(1, sizeof(*s));
    s->dev = t_dev;
    logf_("open %d %ld\n", t_dev, 0);
    return s;
}

int zdb_crc32_stream_begin(zdb_crc32_stream_t *s, size_t n) {
    free(s->img);
    s->img = malloc(n + 16);
    s->cap = n;
    s->fill = 0;
    return s->img ? 0 : ZDB_CRC32_ENOMEM;
}

int zdb_crc32_stream_append(zdb_crc32_stream_t *s, const uint8_t *src, size_t n) {
    if (n > s->cap - s->fill)
        return ZDB_CRC32_EINVAL;
    memcpy(s->img + s->fill, src, n);
    s->fill += n;
    return 0;
}

int zdb_crc32_stream_checksum(zdb_crc32_stream_t *s, const uint64_t *offsets, const uint32_t *lengths,
                              uint32_t *out, size_t n) {
    logf_("checksum %d %ld\n", s->dev, (long)n);
    for (size_t i = 0; i < n; i++) {
        if (offsets[i] > s->fill || lengths[i] > s->fill - offsets[i])
            return ZDB_CRC32_EINVAL;
        out[i] = zdb_crc32(s->img + offsets[i], (ssize_t)lengths[i]);
    }
    return 0;
}

void zdb_crc32_stream_close(zdb_crc32_stream_t *s) {
    free(s->img);
    free(s);
}
