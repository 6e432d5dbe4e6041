/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * The embedded API's SET (zdb_api_set, api.c:268-306, and its handlers
 * api.c:108-256) driven by the REFERENCE library (libzdb objects compiled
 * from /root/reference/libzdb by oracle/Makefile into oracle/_ref/) over a
 * stream of pipelined RESP "SET key value" requests on stdin, one reply line
 * per request -- the reference side of `zdb-set-pipeline --api`
 * (tests/test_set_pipeline.py):
 *   BUFFER <hex>    the key written (user mode) or the 8-byte sequential id
 *   UP_TO_DATE      crc equal to the existing entry's (api.c:129-131, :204-207)
 *   FAILURE <msg>   zdb_api_reply_error
 *   INSERT_DENIED   sequential mode, unknown key (api.c:178-179)
 *   INTERNAL_ERROR
 *
 * usage: api_set_ref <rootdir> user|seq <datasize> <replies-file>   < requests
 * The datafiles land in <rootdir>/data/default/d*; the library logs on
 * stdout, so the reply lines go to their own file.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <strings.h>
#include "libzdb.h"

static uint8_t *slurp(size_t *len) {
    size_t cap = 1 << 20, n = 0;
    uint8_t *b = malloc(cap);
    for (;;) {
        if (n == cap) {
            cap *= 2;
            b = realloc(b, cap);
        }
        size_t got = fread(b + n, 1, cap - n, stdin);
        if (!got)
            break;
        n += got;
    }
    *len = n;
    return b;
}

/* "$<len>\r\n" at *p: the length, *p moved past the line */
static long bulk_len(const uint8_t **p, const uint8_t *end, char c) {
    if (*p >= end || **p != c)
        return -1;
    const uint8_t *q = *p + 1;
    long v = 0;
    while (q < end && *q >= '0' && *q <= '9')
        v = v * 10 + (*q++ - '0');
    if (q + 1 >= end || q[0] != '\r' || q[1] != '\n')
        return -1;
    *p = q + 2;
    return v;
}

int main(int argc, char *argv[]) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s rootdir user|seq datasize replies-file < requests\n", argv[0]);
        return 1;
    }
    FILE *out = fopen(argv[4], "w");
    if (!out)
        return 1;
    char datapath[512], indexpath[512];
    snprintf(datapath, sizeof(datapath), "%s/data", argv[1]);
    snprintf(indexpath, sizeof(indexpath), "%s/index", argv[1]);
    zdb_settings_t *settings = zdb_initialize();
    zdb_id_set("oracle-api-set");
    settings->datapath = datapath;
    settings->indexpath = indexpath;
    settings->mode = strcmp(argv[2], "seq") == 0 ? ZDB_MODE_SEQUENTIAL : ZDB_MODE_KEY_VALUE;
    settings->datasize = strtoull(argv[3], NULL, 0);
    zdb_open(settings);
    namespace_t *ns = namespace_get_default();

    size_t len;
    uint8_t *buf = slurp(&len);
    const uint8_t *p = buf, *end = buf + len;
    while (p < end) {
        const uint8_t *arg[3];
        long alen[3];
        if (bulk_len(&p, end, '*') != 3) {
            fprintf(stderr, "bad request\n");
            return 2;
        }
        for (int i = 0; i < 3; i++) {
            alen[i] = bulk_len(&p, end, '$');
            if (alen[i] < 0 || end - p < alen[i] + 2) {
                fprintf(stderr, "bad request\n");
                return 2;
            }
            arg[i] = p;
            p += alen[i] + 2;
        }
        zdb_api_t *r = zdb_api_set(ns, (void *)arg[1], (size_t)alen[1], (void *)arg[2], (size_t)alen[2]);
        switch (r->status) {
        case ZDB_API_BUFFER: {
            zdb_api_buffer_t *b = r->payload;
            fprintf(out, "BUFFER ");
            for (size_t i = 0; i < b->size; i++)
                fprintf(out, "%02x", b->payload[i]);
            fprintf(out, "\n");
            break;
        }
        case ZDB_API_UP_TO_DATE: fprintf(out, "UP_TO_DATE\n"); break;
        case ZDB_API_FAILURE: fprintf(out, "FAILURE %s\n", (char *)r->payload); break;
        case ZDB_API_INSERT_DENIED: fprintf(out, "INSERT_DENIED\n"); break;
        default: fprintf(out, "%s\n", zdb_api_debug_type(r->status) + 8); break;
        }
        zdb_api_reply_free(r);
    }
    free(buf);
    fclose(out);
    zdb_close(settings);
    return 0;
}
