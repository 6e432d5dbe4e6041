/*
 * zdb-set-pipeline -- the SET path of zdbd with two-phase batching of
 * pipelined requests, as a stand-alone harness
 * over the same on-disk format.
 *
 * zdbd answers one request at a time: for every SET it computes the payload
 * crc (commands_set.c:106), compares with the existing entry (crc, length,
 * then memcmp: commands_set.c:52-74, :111-116), appends header + key +
 * payload to the datafile (data_insert, data.c:594-633), indexes and replies
 * (commands_set.c:162-168).  Pipelined SETs arrive together in one
 * redis_chunk_read (redis.c:736-789), so they can be handled in two phases:
 *
 *   phase 1  parse every complete SET of the receive buffer and checksum all
 *            their values in ONE batched call (zdb_crc32_batch).  The
 *            receive buffer is pinned (zdb_crc32_host_alloc), so the GPU
 *            reads the values in place: no staging copy, one launch;
 *   phase 2  in request order, exactly what zdbd does per request: datafile
 *            rotation before the insert (commands_set.c:370-373, where the
 *            new file's first entry keeps the previous file's last offset as
 *            `previous`, data.c:283-315), compare with the existing entry,
 *            append (headers with the phase-1 crcs), index, reply -- and one
 *            write() per datafile per batch instead of two per SET.
 *
 * Replies and datafiles are byte-identical to the reference daemon's for the
 * same request stream (timestamps aside): tests/test_set_pipeline.py runs
 * the reference zdbd (oracle/_ref/zdbd/zdb) beside it.
 *
 *   usage: zdb-set-pipeline [--engine=hip|cpu|auto] [--mode=user|seq] [--api]
 *                           [--datasize=BYTES] [--batch=N] [--stats] <datadir>
 *                           < requests   > replies
 *
 * --engine=auto checksums a batch on the GPU when its values total at least
 * AUTO_GPU_MIN_BYTES and with the scalar engine below that (one 256 KiB value
 * costs 35 us through the GPU and 21 us on one core), and
 * runs on the scalar engine alone when no GPU is usable.
 *
 * Handlers (the daemon's table, commands_set.c:285-290):
 *   --mode=user  redis_set_handler_userkey, commands_set.c:76-171 (default)
 *   --mode=seq   redis_set_handler_sequential, commands_set.c:173-283: the
 *                key is index_next_id (index.c:404-408) unless the request
 *                names an existing id (8 bytes, index_get_handler_sequential,
 *                index_get.c:16-59), "-Invalid key, only update authorized"
 *                otherwise; an update appends the replaced entry, flagged
 *                deleted, at the next id (index_update_entry_sequential,
 *                index_set.c:321-356), so that id is skipped; the reply is
 *                the 8-byte id.
 * Arguments (command_set, commands_set.c:292-323): 4 arguments carry an
 * admin timestamp (timestamp_from_set, :16-29; every client is admin when
 * zdbd runs without --admin, redis.c:903); any count but 3 or 4 is
 * "-Unexpected arguments" (commands.c:25-29).
 * --api: the embedded API's SET instead (zdb_api_set, api.c:268-306, and its
 * handlers api.c:108-256): no RESP reply but one line per request (BUFFER
 * <hex> / UP_TO_DATE / FAILURE <message> / INSERT_DENIED), "unchanged" on
 * crc equality alone (api.c:129-131, :204-211: no length or memcmp check),
 * timestamps from the clock, no argument-count or key-length checks (3-argument
 * SETs with keys of at most 255 bytes only).
 *
 * Any other command ends the run with exit status 2.  The datafiles are
 * <datadir>/d<id>, created from d0 on.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <libgen.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "zdb_crc32.h"
#include "zdb_datafile.h"

#define RECV_CAP (64u << 20)       /* pinned receive buffer                 */
#define MAX_PAYLOAD (8u << 20)     /* redis.h:160 / data.h:6                */
#define MAX_KEY 255                /* index.h:264                           */
#define AUTO_GPU_MIN_BYTES (512u << 10) /* --engine=auto crossover */

static void die(const char *msg) {
    fprintf(stderr, "[-] zdb-set-pipeline: %s\n", msg);
    exit(1);
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

/* ---- GPU engine (dlopen'ed, like zdb-integrity-check) ------------------- */

typedef struct {
    int (*batch)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t);
    const char *(*strerror)(int);
    void *(*host_alloc)(size_t);
    int (*device_count)(void);
} gpu_api_t;

static gpu_api_t g_gpu;

static int load_gpu(void) {
    const char *env = getenv("ZDBCRC_LIB");
    char path[4096];
    if (env) {
        snprintf(path, sizeof(path), "%s", env);
    } else {
        char exe[4096];
        ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
        if (n <= 0)
            return 0;
        exe[n] = 0;
        snprintf(path, sizeof(path), "%s/../lib/libzdbcrc.so", dirname(exe));
    }
    void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h)
        return 0;
    g_gpu.batch = (int (*)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *,
                           size_t))dlsym(h, "zdb_crc32_batch");
    g_gpu.strerror = (const char *(*)(int))dlsym(h, "zdb_crc32_strerror");
    g_gpu.host_alloc = (void *(*)(size_t))dlsym(h, "zdb_crc32_host_alloc");
    g_gpu.device_count = (int (*)(void))dlsym(h, "zdb_crc32_device_count");
    return g_gpu.batch && g_gpu.strerror && g_gpu.host_alloc && g_gpu.device_count && g_gpu.device_count() > 0;
}

/* ---- in-memory index: key -> (crc, length, file, offset) ----------------- */

typedef struct {
    uint8_t *key; /* NULL = empty slot */
    uint8_t klen;
    uint32_t crc, length, fileid;
    uint64_t offset; /* entry header offset in d<fileid> */
} idx_entry_t;

static idx_entry_t *g_idx;
static size_t g_idx_cap, g_idx_n;

static uint64_t key_hash(const uint8_t *k, size_t n) {
    uint64_t h = 1469598103934665603ull; /* FNV-1a: a host hash table, not 0-db's bucket hash */
    for (size_t i = 0; i < n; i++)
        h = (h ^ k[i]) * 1099511628211ull;
    return h;
}

static idx_entry_t *idx_find(const uint8_t *k, uint8_t n, int insert) {
    if (insert && 2 * (g_idx_n + 1) > g_idx_cap) {
        size_t ncap = g_idx_cap ? 2 * g_idx_cap : 1024;
        idx_entry_t *t = calloc(ncap, sizeof(*t));
        if (!t)
            die("out of memory");
        for (size_t i = 0; i < g_idx_cap; i++) {
            if (!g_idx[i].key)
                continue;
            size_t j = key_hash(g_idx[i].key, g_idx[i].klen) & (ncap - 1);
            while (t[j].key)
                j = (j + 1) & (ncap - 1);
            t[j] = g_idx[i];
        }
        free(g_idx);
        g_idx = t;
        g_idx_cap = ncap;
    }
    if (!g_idx_cap)
        return NULL;
    size_t j = key_hash(k, n) & (g_idx_cap - 1);
    while (g_idx[j].key) {
        if (g_idx[j].klen == n && memcmp(g_idx[j].key, k, n) == 0)
            return &g_idx[j];
        j = (j + 1) & (g_idx_cap - 1);
    }
    if (!insert)
        return NULL;
    g_idx[j].key = malloc(n ? n : 1);
    if (!g_idx[j].key)
        die("out of memory");
    memcpy(g_idx[j].key, k, n);
    g_idx[j].klen = n;
    g_idx_n++;
    return &g_idx[j];
}

/* sequential mode: entry id -> (crc, length, file, offset), or a deleted
 * placeholder (the replaced entry an update appends at the next id) */
typedef struct {
    uint32_t crc, length, fileid;
    uint64_t offset;
    int deleted;
} seq_entry_t;

static seq_entry_t *g_seq;
static uint64_t g_seq_n, g_seq_cap; /* g_seq_n = index_next_id */

static seq_entry_t *seq_push(void) {
    if (g_seq_n == g_seq_cap) {
        g_seq_cap = g_seq_cap ? 2 * g_seq_cap : 1024;
        g_seq = realloc(g_seq, g_seq_cap * sizeof(*g_seq));
        if (!g_seq)
            die("out of memory");
    }
    memset(&g_seq[g_seq_n], 0, sizeof(*g_seq));
    return &g_seq[g_seq_n++];
}

/* index_get in sequential mode: an 8-byte id below the next id whose entry is live */
static seq_entry_t *seq_find(const uint8_t *k, uint32_t n) {
    if (n != 8)
        return NULL;
    uint64_t id;
    memcpy(&id, k, 8);
    if (id >= g_seq_n || g_seq[id].deleted)
        return NULL;
    return &g_seq[id];
}

/* ---- datafiles ------------------------------------------------------------- */

typedef struct {
    char dir[4096];
    uint64_t datasize;   /* --datasize: split threshold (zdbd.c --datasize)      */
    uint32_t fileid;     /* current datafile                                    */
    int fd;
    uint64_t size;       /* data_next_offset: bytes in the file incl. pending   */
    uint64_t flushed;    /* bytes already written                               */
    uint32_t previous;   /* root->previous (data.c:605, :630)                   */
    uint8_t *pend;       /* bytes appended this batch, not yet written           */
    size_t npend, cap_pend;
} store_t;

static void store_write_all(store_t *s) {
    size_t done = 0;
    while (done < s->npend) {
        ssize_t w = write(s->fd, s->pend + done, s->npend - done);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            die("datafile write failed");
        }
        done += (size_t)w;
    }
    s->flushed += s->npend;
    s->npend = 0;
}

static void store_open(store_t *s, uint32_t id) {
    char path[4200];
    snprintf(path, sizeof(path), "%s/d%u", s->dir, id);
    s->fd = open(path, O_CREAT | O_RDWR | O_APPEND | O_TRUNC, 0600);
    if (s->fd < 0)
        die("cannot create datafile");
    /* data_initialize (data.c): "DAT0", version, created, opened, fileid */
    uint8_t h[ZDB_DATA_HEADER_SIZE];
    zdb_datafile_encode_header(h, id);
    const uint64_t t = (uint64_t)time(NULL);
    memcpy(h + 8, &t, 8);
    memcpy(h + 16, &t, 8);
    if (write(s->fd, h, sizeof(h)) != (ssize_t)sizeof(h))
        die("datafile header write failed");
    s->fileid = id;
    s->size = s->flushed = ZDB_DATA_HEADER_SIZE;
}

static uint8_t *store_reserve(store_t *s, size_t more) {
    if (s->npend + more > s->cap_pend) {
        size_t cap = s->cap_pend ? s->cap_pend : (1u << 20);
        while (cap < s->npend + more)
            cap *= 2;
        s->pend = realloc(s->pend, cap);
        if (!s->pend)
            die("out of memory");
        s->cap_pend = cap;
    }
    return s->pend + s->npend;
}

/* the stored payload of an index entry (data_get, data.c:464-504): from the
 * bytes of this batch not written yet, or from its datafile */
static int store_read_payload(store_t *s, const idx_entry_t *e, uint8_t *dst) {
    const uint64_t p = e->offset + ZDB_ENTRY_HEADER_SIZE + e->klen;
    if (e->fileid == s->fileid && p >= s->flushed) {
        memcpy(dst, s->pend + (p - s->flushed), e->length);
        return 1;
    }
    char path[4200];
    snprintf(path, sizeof(path), "%s/d%u", s->dir, e->fileid);
    int fd = open(path, O_RDONLY);
    if (fd < 0)
        return 0;
    ssize_t got = pread(fd, dst, e->length, (off_t)p);
    close(fd);
    return got == (ssize_t)e->length;
}

/* ---- RESP parsing ---------------------------------------------------------- */

typedef struct {
    uint64_t key_off, val_off; /* offsets in the receive buffer */
    uint32_t klen, vlen;
    int argc;                  /* 2..5 (argv[0] = SET) */
    int64_t timestamp;         /* argc == 4: atoll(argv[3]) */
} set_req_t;

static int parse_int(const uint8_t *p, const uint8_t *end, long *v, const uint8_t **next) {
    long x = 0;
    const uint8_t *q = p;
    while (q < end && *q >= '0' && *q <= '9')
        x = x * 10 + (*q++ - '0');
    if (q == p || q + 1 >= end)
        return q + 1 >= end ? 0 : -1;
    if (q[0] != '\r' || q[1] != '\n')
        return -1;
    *v = x;
    *next = q + 2;
    return 1;
}

/* one complete "*N $3 SET $k key $v value [$t timestamp]" at p, N = 2..5:
 * 1 parsed, 0 incomplete, -1 bad or another command */
static int parse_set(const uint8_t *base, const uint8_t *p, const uint8_t *end, set_req_t *r, const uint8_t **next) {
    if (p >= end)
        return 0;
    if (*p != '*')
        return -1;
    long argc;
    int rc = parse_int(p + 1, end, &argc, &p);
    if (rc <= 0)
        return rc;
    if (argc < 2 || argc > 5)
        return -1;
    const uint8_t *arg[5];
    long len[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < argc; i++) {
        if (p >= end)
            return 0;
        if (*p != '$')
            return -1;
        rc = parse_int(p + 1, end, &len[i], &p);
        if (rc <= 0)
            return rc;
        if (len[i] < 0 || (i == 2 && len[i] > (long)MAX_PAYLOAD))
            return -1;
        if (end - p < len[i] + 2)
            return 0;
        arg[i] = p;
        p += len[i];
        if (p[0] != '\r' || p[1] != '\n')
            return -1;
        p += 2;
    }
    if (!((len[0] == 3 && strncasecmp((const char *)arg[0], "SET", 3) == 0) ||
          (len[0] == 4 && strncasecmp((const char *)arg[0], "SETX", 4) == 0)))
        return -1;
    r->argc = (int)argc;
    r->key_off = (uint64_t)(arg[1] - base);
    r->klen = (uint32_t)len[1];
    r->val_off = argc > 2 ? (uint64_t)(arg[2] - base) : r->key_off;
    r->vlen = argc > 2 ? (uint32_t)len[2] : 0;
    r->timestamp = 0;
    if (argc == 4) { /* timestamp_from_set: atoll of the argument (commands_set.c:22-23) */
        char t[64];
        const size_t tl = (size_t)len[3] < sizeof(t) - 1 ? (size_t)len[3] : sizeof(t) - 1;
        memcpy(t, arg[3], tl);
        t[tl] = 0;
        r->timestamp = atoll(t);
    }
    *next = p;
    return 1;
}

/* ---- the two phases ----------------------------------------------------------- */

typedef struct {
    int use_gpu;  /* GPU engine loaded                        */
    int auto_min; /* --engine=auto: small batches on the CPU  */
    int seq;      /* --mode=seq: the sequential handler        */
    int api;      /* --api: zdb_api_set semantics and replies  */
    size_t batch;
    int stats;
    double t_crc, t_apply, t_crc_warm;
    uint64_t sets, batches, unchanged, bytes, sets_warm, gpu_batches;
} run_t;

static void reply(FILE *out, const char *s, size_t n) {
    if (fwrite(s, 1, n, out) != n)
        die("reply write failed");
}
#define REPLY_LIT(out, lit) reply((out), (lit), sizeof(lit) - 1)

static void process(run_t *run, store_t *st, const uint8_t *buf, set_req_t *req, size_t n, uint32_t *crc,
                    uint64_t *voff, uint32_t *vlen, FILE *out, uint8_t *cmpbuf) {
    /* phase 1: every value of the batch in one checksum call */
    const double t0 = now_s();
    for (size_t i = 0; i < n; i++) {
        voff[i] = req[i].val_off;
        vlen[i] = req[i].vlen;
    }
    size_t span = 0, total = 0;
    for (size_t i = 0; i < n; i++) {
        if (voff[i] + vlen[i] > span)
            span = voff[i] + vlen[i];
        total += vlen[i];
    }
    if (run->use_gpu && (!run->auto_min || total >= AUTO_GPU_MIN_BYTES)) {
        run->gpu_batches++;
        int rc = g_gpu.batch(buf, span, voff, vlen, crc, n);
        if (rc) {
            fprintf(stderr, "[-] zdb-set-pipeline: GPU engine failed: %s\n", g_gpu.strerror(rc));
            exit(1);
        }
    } else {
        for (size_t i = 0; i < n; i++)
            crc[i] = zdb_crc32(buf + voff[i], (ssize_t)vlen[i]);
    }
    const double t1 = now_s();

    /* phase 2: in request order, as zdbd handles each SET */
    for (size_t i = 0; i < n; i++) {
        const uint8_t *key = buf + req[i].key_off;
        const uint32_t klen = req[i].klen, L = req[i].vlen;
        if (!run->api) {
            /* command_set's checks (commands_set.c:295-311, commands.c:25-29) */
            if (req[i].argc != 3 && req[i].argc != 4) {
                REPLY_LIT(out, "-Unexpected arguments\r\n");
                continue;
            }
            if (klen > MAX_KEY) {
                REPLY_LIT(out, "-Key too large\r\n");
                continue;
            }
        }
        /* the existing entry: index_get (commands_set.c:338-342; api.c:279-283) */
        idx_entry_t *e = NULL;
        seq_entry_t *q = NULL;
        if (klen) {
            if (run->seq)
                q = seq_find(key, klen);
            else
                e = idx_find(key, (uint8_t)klen, 0);
        }
        const int exists = e || q;
        const uint32_t ex_crc = e ? e->crc : q ? q->crc : 0, ex_len = e ? e->length : q ? q->length : 0;
        /* datafile rotation before the handler (commands_set.c:370-373, api.c:299-303) */
        if (st->size + L > st->datasize) {
            store_write_all(st);
            close(st->fd);
            store_open(st, st->fileid + 1); /* root->previous carries over (data.c:283-315) */
        }
        /* the handler's own first check */
        if (!run->seq && klen == 0) { /* commands_set.c:85-88, api.c:109-110 */
            if (run->api)
                REPLY_LIT(out, "FAILURE Invalid argument, key needed\n");
            else
                REPLY_LIT(out, "-Invalid argument, key needed\r\n");
            continue;
        }
        if (run->seq && klen && !exists) { /* commands_set.c:182-185, api.c:178-179 */
            if (run->api)
                REPLY_LIT(out, "INSERT_DENIED\n");
            else
                REPLY_LIT(out, "-Invalid key, only update authorized\r\n");
            continue;
        }
        /* unchanged payload: the daemon checks crc, then length and bytes
         * (commands_set.c:52-74, :111-116, :221-227); the API the crc alone
         * (api.c:129-131, :204-207) */
        if (exists && ex_crc == crc[i]) {
            int same = run->api;
            if (!same && ex_len == L) {
                idx_entry_t tmp;
                const idx_entry_t *src = e;
                if (q) {
                    tmp.klen = 8;
                    tmp.length = q->length;
                    tmp.fileid = q->fileid;
                    tmp.offset = q->offset;
                    src = &tmp;
                }
                same = store_read_payload(st, src, cmpbuf) && memcmp(cmpbuf, buf + voff[i], L) == 0;
            }
            if (same) {
                if (run->api)
                    REPLY_LIT(out, "UP_TO_DATE\n");
                else
                    REPLY_LIT(out, "$-1\r\n");
                run->unchanged++;
                continue;
            }
        }
        /* the key written: the user's, or the sequential id (index_next_id,
         * or the existing entry's id on an update) */
        uint8_t idbuf[8];
        const uint8_t *wkey = key;
        uint32_t wklen = klen;
        uint64_t id = g_seq_n;
        if (run->seq) {
            if (q)
                id = (uint64_t)(q - g_seq);
            memcpy(idbuf, &id, 8);
            wkey = idbuf;
            wklen = 8;
        }
        /* data_insert (data.c:594-633): header with this batch's crc, key, payload */
        const uint32_t ts = (uint32_t)(req[i].argc == 4 ? req[i].timestamp : (int64_t)time(NULL));
        const uint64_t offset = st->size;
        uint8_t *dst = store_reserve(st, ZDB_ENTRY_HEADER_SIZE + wklen + L);
        const size_t hl = zdb_datafile_encode_entry(dst, wkey, (uint8_t)wklen, L, st->previous, crc[i], 0, ts);
        memcpy(dst + hl, buf + voff[i], L);
        st->npend += hl + L;
        st->size += hl + L;
        st->previous = (uint32_t)offset;
        /* index_set (commands_set.c:151, :262) */
        if (run->seq) {
            if (q) { /* the replaced entry goes to the next id, flagged deleted */
                seq_push()->deleted = 1;
                q = &g_seq[id]; /* (seq_push may have moved the array) */
            } else {
                q = seq_push();
            }
            q->crc = crc[i];
            q->length = L;
            q->fileid = st->fileid;
            q->offset = offset;
        } else {
            if (!e)
                e = idx_find(key, (uint8_t)klen, 1);
            e->crc = crc[i];
            e->length = L;
            e->fileid = st->fileid;
            e->offset = offset;
        }
        /* reply: the key as a bulk string (commands_set.c:162-168, :274-280) */
        if (run->api) {
            static const char hx[] = "0123456789abcdef";
            REPLY_LIT(out, "BUFFER ");
            for (uint32_t b = 0; b < wklen; b++) {
                const char c2[2] = {hx[wkey[b] >> 4], hx[wkey[b] & 15]};
                reply(out, c2, 2);
            }
            REPLY_LIT(out, "\n");
        } else {
            char head[32];
            int hn = snprintf(head, sizeof(head), "$%u\r\n", wklen);
            reply(out, head, (size_t)hn);
            reply(out, (const char *)wkey, wklen);
            REPLY_LIT(out, "\r\n");
        }
        run->bytes += L;
    }
    store_write_all(st); /* one append per batch */
    fflush(out);
    run->t_crc += t1 - t0;
    run->t_apply += now_s() - t1;
    if (run->batches > 0) { /* steady state: every batch after the first */
        run->t_crc_warm += t1 - t0;
        run->sets_warm += n;
    }
    run->sets += n;
    run->batches++;
}

int main(int argc, char **argv) {
    run_t run;
    memset(&run, 0, sizeof(run));
    run.use_gpu = 1;
    run.batch = 4096;
    uint64_t datasize = 256ull << 20; /* ZDB_DEFAULT_DATA_MAXSIZE, data.h:5 */
    int argi = 1;
    while (argi < argc && strncmp(argv[argi], "--", 2) == 0) {
        if (!strcmp(argv[argi], "--engine=cpu"))
            run.use_gpu = 0, run.auto_min = 0;
        else if (!strcmp(argv[argi], "--engine=hip"))
            run.use_gpu = 1, run.auto_min = 0;
        else if (!strcmp(argv[argi], "--engine=auto"))
            run.use_gpu = 1, run.auto_min = 1;
        else if (!strcmp(argv[argi], "--mode=user"))
            run.seq = 0;
        else if (!strcmp(argv[argi], "--mode=seq"))
            run.seq = 1;
        else if (!strcmp(argv[argi], "--api"))
            run.api = 1;
        else if (!strncmp(argv[argi], "--datasize=", 11) && atoll(argv[argi] + 11) > 0)
            datasize = (uint64_t)atoll(argv[argi] + 11);
        else if (!strncmp(argv[argi], "--batch=", 8) && atol(argv[argi] + 8) > 0)
            run.batch = (size_t)atol(argv[argi] + 8);
        else if (!strcmp(argv[argi], "--stats"))
            run.stats = 1;
        else
            break;
        argi++;
    }
    if (argc - argi != 1) {
        fprintf(stderr,
                "Usage: %s [--engine=hip|cpu|auto] [--mode=user|seq] [--api] [--datasize=BYTES] [--batch=N] [--stats] "
                "<datadir>\n",
                argv[0]);
        return 1;
    }
    if (run.use_gpu && !load_gpu()) {
        if (!run.auto_min)
            die("GPU engine unavailable (use --engine=cpu)");
        run.use_gpu = 0; /* auto: the scalar engine alone */
    }

    store_t st;
    memset(&st, 0, sizeof(st));
    snprintf(st.dir, sizeof(st.dir), "%s", argv[argi]);
    st.datasize = datasize;
    mkdir(st.dir, 0700);
    store_open(&st, 0);

    /* the receive buffer: pinned when the GPU checksums the values in place */
    uint8_t *buf = run.use_gpu ? g_gpu.host_alloc(RECV_CAP) : malloc(RECV_CAP);
    uint8_t *cmpbuf = malloc(MAX_PAYLOAD);
    set_req_t *req = malloc(sizeof(set_req_t) * run.batch);
    uint32_t *crc = malloc(sizeof(uint32_t) * run.batch);
    uint64_t *voff = malloc(sizeof(uint64_t) * run.batch);
    uint32_t *vlen = malloc(sizeof(uint32_t) * run.batch);
    if (!buf || !cmpbuf || !req || !crc || !voff || !vlen)
        die("out of memory");
    if (run.use_gpu) { /* bring the device up before the first request (code object, tables) */
        uint64_t o = 0;
        uint32_t l = 64, c = 0;
        memset(buf, 0, 64);
        if (g_gpu.batch(buf, 64, &o, &l, &c, 1) != 0)
            die("GPU engine failed to start (use --engine=cpu)");
    }

    size_t fill = 0, pos = 0;
    int eof = 0, status = 0;
    while (!eof || pos < fill) {
        /* redis_chunk_read: take what the socket (stdin) has */
        if (!eof && fill < RECV_CAP) {
            ssize_t got = read(0, buf + fill, RECV_CAP - fill);
            if (got < 0 && errno != EINTR)
                die("read failed");
            if (got == 0)
                eof = 1;
            if (got > 0)
                fill += (size_t)got;
        }
        /* phase 1 + 2 over the complete SETs in the buffer (up to --batch) */
        size_t n = 0;
        int bad = 0;
        while (n < run.batch) {
            const uint8_t *next;
            int rc = parse_set(buf, buf + pos, buf + fill, &req[n], &next);
            if (rc == 0)
                break;
            if (rc < 0) {
                bad = 1;
                break;
            }
            pos = (size_t)(next - buf);
            n++;
        }
        if (n)
            process(&run, &st, buf, req, n, crc, voff, vlen, stdout, cmpbuf);
        if (bad) {
            fprintf(stderr, "[-] zdb-set-pipeline: unsupported or malformed request at byte %zu\n", pos);
            status = 2;
            break;
        }
        if (n == 0 && (eof || fill == RECV_CAP)) {
            if (pos < fill && (eof || pos == 0)) {
                fprintf(stderr, "[-] zdb-set-pipeline: truncated request at the end of the stream\n");
                status = 2;
                break;
            }
        }
        /* keep the partial request at the front of the buffer */
        if (pos > 0 && (n == 0 || fill - pos < (RECV_CAP >> 2))) {
            memmove(buf, buf + pos, fill - pos);
            fill -= pos;
            pos = 0;
        }
    }
    store_write_all(&st);
    close(st.fd);
    if (run.stats)
        fprintf(stderr,
                "{\"engine\": \"%s\", \"sets\": %llu, \"batches\": %llu, \"gpu_batches\": %llu, \"unchanged\": %llu, "
                "\"payload_bytes\": %llu, \"crc_s\": %.6f, \"apply_s\": %.6f, \"crc_s_after_first_batch\": %.6f, "
                "\"sets_after_first_batch\": %llu}\n",
                run.use_gpu ? (run.auto_min ? "auto" : "hip") : "cpu", (unsigned long long)run.sets,
                (unsigned long long)run.batches, (unsigned long long)run.gpu_batches, (unsigned long long)run.unchanged, (unsigned long long)run.bytes, run.t_crc, run.t_apply, run.t_crc_warm,
                (unsigned long long)run.sets_warm);
    fflush(stdout);
    _exit(status); /* the HIP runtime needs no teardown here */
}
