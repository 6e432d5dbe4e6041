/*
 * zdb-index-verify -- the index-rebuild scan of a namespace's datafiles with
 * the payload check that tools/index-rebuild leaves out.
 *
 * index-rebuild (tools/index-rebuild/index-rebuild.c:56-147) walks d0, d1,
 * ... until a file is missing or has a bad header (index_data_jump_to,
 * :14-52), and for every entry either deletes the key (DATA_ENTRY_DELETED)
 * or sets it to the entry (offset, length, and the stored `integrity`,
 * copied without being checked: :94), stopping a file's pass at the first
 * entry newer than --time (:79-82).  It never reads a payload.
 *
 * This tool replays exactly that walk and that set/delete sequence, and
 * checks the payload crc of every entry the rebuilt index points at -- all
 * payloads of a datafile in one batched checksum (zdb_crc32_batch, GPU) --
 * so a rebuild from damaged datafiles no longer indexes corrupt values
 * silently.
 *
 *   usage: zdb-index-verify [--engine=hip|cpu] [--time=T] [--list] <datadir>
 *
 * <datadir> holds the namespace's datafiles (index-rebuild --data <root>
 * --namespace <ns> reads <root>/<ns>/d<N>).  --list prints every live key
 * (file order).  Each corrupt live entry gets one line on stderr; the exit
 * status is their count (at most 255), 1 on a short entry header (the
 * rebuild's zdb_diep, :72-73).
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
#include <unistd.h>

#include "zdb_crc32.h"
#include "zdb_datafile.h"

typedef struct {
    int (*batch)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t);
    const char *(*strerror)(int);
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
    g_gpu.device_count = (int (*)(void))dlsym(h, "zdb_crc32_device_count");
    return g_gpu.batch && g_gpu.strerror && g_gpu.device_count && g_gpu.device_count() > 0;
}

/* one indexed entry: where the rebuilt index points, and what its payload is */
typedef struct {
    uint8_t *key;
    uint8_t klen;
    uint8_t live;
    uint32_t fileid, length, stored, computed;
    uint64_t offset; /* entry header offset in d<fileid> */
    int cut;         /* payload cut by the end of the file */
} entry_t;

static entry_t *g_map;
static size_t g_cap, g_n;

static uint64_t key_hash(const uint8_t *k, size_t n) {
    uint64_t h = 1469598103934665603ull; /* FNV-1a: a host hash table */
    for (size_t i = 0; i < n; i++)
        h = (h ^ k[i]) * 1099511628211ull;
    return h;
}

static entry_t *map_slot(const uint8_t *k, uint8_t n) {
    if (2 * (g_n + 1) > g_cap) {
        size_t ncap = g_cap ? 2 * g_cap : 1024;
        entry_t *t = calloc(ncap, sizeof(*t));
        if (!t) {
            perror("calloc");
            exit(1);
        }
        for (size_t i = 0; i < g_cap; i++) {
            if (!g_map[i].key)
                continue;
            size_t j = key_hash(g_map[i].key, g_map[i].klen) & (ncap - 1);
            while (t[j].key)
                j = (j + 1) & (ncap - 1);
            t[j] = g_map[i];
        }
        free(g_map);
        g_map = t;
        g_cap = ncap;
    }
    size_t j = key_hash(k, n) & (g_cap - 1);
    while (g_map[j].key) {
        if (g_map[j].klen == n && memcmp(g_map[j].key, k, n) == 0)
            return &g_map[j];
        j = (j + 1) & (g_cap - 1);
    }
    g_map[j].key = malloc(n ? n : 1);
    if (!g_map[j].key) {
        perror("malloc");
        exit(1);
    }
    memcpy(g_map[j].key, k, n);
    g_map[j].klen = n;
    g_n++;
    return &g_map[j];
}

static uint8_t *read_file(const char *path, size_t *len) {
    int fd = open(path, O_RDONLY);
    if (fd < 0)
        return NULL;
    struct stat sb;
    if (fstat(fd, &sb) != 0) {
        close(fd);
        return NULL;
    }
    uint8_t *buf = malloc((size_t)sb.st_size + 16);
    size_t got = 0;
    while (buf && got < (size_t)sb.st_size) {
        ssize_t r = pread(fd, buf + got, (size_t)sb.st_size - got, (off_t)got);
        if (r <= 0)
            break;
        got += (size_t)r;
    }
    close(fd);
    *len = got;
    return buf;
}

static int cmp_entry(const void *a, const void *b) {
    const entry_t *x = *(entry_t *const *)a, *y = *(entry_t *const *)b;
    if (x->fileid != y->fileid)
        return x->fileid < y->fileid ? -1 : 1;
    return x->offset < y->offset ? -1 : x->offset > y->offset;
}

int main(int argc, char **argv) {
    int use_gpu = 1, list = 0;
    long long tlimit = 0;
    int argi = 1;
    while (argi < argc && strncmp(argv[argi], "--", 2) == 0) {
        if (!strcmp(argv[argi], "--engine=cpu"))
            use_gpu = 0;
        else if (!strcmp(argv[argi], "--engine=hip"))
            use_gpu = 1;
        else if (!strncmp(argv[argi], "--time=", 7))
            tlimit = atoll(argv[argi] + 7);
        else if (!strcmp(argv[argi], "--list"))
            list = 1;
        else
            break;
        argi++;
    }
    if (argc - argi != 1) {
        fprintf(stderr, "Usage: %s [--engine=hip|cpu] [--time=T] [--list] <datadir>\n", argv[0]);
        return 1;
    }
    if (use_gpu && !load_gpu()) {
        fprintf(stderr, "[-] zdb-index-verify: GPU engine unavailable (use --engine=cpu)\n");
        return 1;
    }
    const char *dir = argv[argi];
    uint64_t total = 0;
    int fatal = 0;
    for (uint32_t fileid = 0; !fatal; fileid++) {
        char path[4200];
        snprintf(path, sizeof(path), "%s/d%u", dir, fileid);
        size_t len = 0;
        uint8_t *img = read_file(path, &len);
        if (!img)
            break; /* index_data_jump_to: no such file ends the rebuild */
        int status = 0;
        long n = zdb_datafile_walk(img, len, NULL, 0, &status);
        if (status == ZDB_WALK_BAD_DESCRIPTOR) { /* bad header: the rebuild stops here too */
            free(img);
            break;
        }
        zdb_record_t *recs = calloc((size_t)(n > 0 ? n : 1), sizeof(zdb_record_t));
        n = zdb_datafile_walk(img, len, recs, n, &status);
        /* every payload of the file in one batch (cut ones are checked as far as they go) */
        uint64_t *offs = malloc(sizeof(uint64_t) * (size_t)(n + 1));
        uint32_t *lens = malloc(sizeof(uint32_t) * (size_t)(n + 1));
        uint32_t *crc = malloc(sizeof(uint32_t) * (size_t)(n + 1));
        for (long i = 0; i < n; i++) {
            offs[i] = recs[i].payload_offset;
            const uint64_t avail = recs[i].payload_offset <= len ? len - recs[i].payload_offset : 0;
            lens[i] = recs[i].datalength <= avail ? recs[i].datalength : (uint32_t)avail;
        }
        if (n > 0) {
            if (use_gpu) {
                int rc = g_gpu.batch(img, len, offs, lens, crc, (size_t)n);
                if (rc) {
                    fprintf(stderr, "[-] zdb-index-verify: GPU engine failed: %s\n", g_gpu.strerror(rc));
                    return 1;
                }
            } else {
                for (long i = 0; i < n; i++)
                    crc[i] = zdb_crc32(img + offs[i], (ssize_t)lens[i]);
            }
        }
        /* the rebuild's pass over this file (index-rebuild.c:56-120) */
        long used = 0;
        for (long i = 0; i < n; i++) {
            const zdb_record_t *r = &recs[i];
            if (tlimit > 0 && (long long)r->timestamp > tlimit)
                break; /* timestamp limit: this file's pass stops (:79-82) */
            entry_t *e = map_slot(img + r->header_offset + ZDB_ENTRY_HEADER_SIZE, r->idlength);
            if (r->flags & ZDB_ENTRY_DELETED) {
                e->live = 0;
            } else {
                e->live = 1;
                e->fileid = fileid;
                e->offset = r->header_offset;
                e->length = r->datalength;
                e->stored = r->integrity;
                e->computed = crc[i];
                e->cut = lens[i] != r->datalength;
            }
            used++;
        }
        if (status == ZDB_WALK_SHORT_HEADER && (tlimit <= 0 || used == n))
            fatal = 1; /* "data header read failed": zdb_diep in the rebuild */
        printf("[+] index-verify: datafile %s: %ld entries\n", path, used);
        total += (uint64_t)used;
        free(recs);
        free(offs);
        free(lens);
        free(crc);
        free(img);
    }
    if (fatal) {
        fprintf(stderr, "[-] zdb-index-verify: data header read failed\n");
        return 1;
    }
    /* the live keys the rebuilt index holds, in file order */
    entry_t **live = malloc(sizeof(entry_t *) * (g_n + 1));
    size_t nlive = 0, bad = 0;
    for (size_t i = 0; i < g_cap; i++)
        if (g_map[i].key && g_map[i].live)
            live[nlive++] = &g_map[i];
    qsort(live, nlive, sizeof(entry_t *), cmp_entry);
    for (size_t i = 0; i < nlive; i++) {
        const entry_t *e = live[i];
        const int ok = !e->cut && e->computed == e->stored;
        if (list) {
            printf("live 0x");
            for (uint8_t k = 0; k < e->klen; k++)
                printf("%02x", e->key[k]);
            printf(" %u %llu %u %08x %s\n", e->fileid, (unsigned long long)e->offset, e->length, e->stored,
                   ok ? "ok" : "CORRUPT");
        }
        if (!ok) {
            fprintf(stderr, "[-] index-verify: corrupt payload: datafile %u, offset %llu, key 0x", e->fileid,
                    (unsigned long long)e->offset);
            for (uint8_t k = 0; k < e->klen; k++)
                fprintf(stderr, "%02x", e->key[k]);
            fprintf(stderr, ": %08x <> %08x%s\n", e->computed, e->stored, e->cut ? " (payload cut short)" : "");
            bad++;
        }
    }
    printf("[+] index-verify: %llu entries, %zu live keys, %zu corrupt\n", (unsigned long long)total, nlive, bad);
    fflush(stdout);
    fflush(stderr);
    _exit(bad > 255 ? 255 : (int)bad);
}
