/*
 * zdb-integrity-check -- GPU counterpart of 0-db's tools/integrity-check.
 *
 * Same command line, stdout, stderr and exit status as the reference tool
 * (tools/integrity-check/integrity-check.c:30-166), but restructured for the
 * MI355X: the datafile is read into memory with one large read, the host walks
 * the entry headers (zdb_datafile_walk), every payload checksum is computed in
 * ONE batched GPU call (zdb_crc32_batch -> crc32_hip.hip), and the report is
 * formatted in a single buffer.  The reference does 4 syscalls and ~7 printf
 * per record around one CPU crc each (integrity-check.c:59-105).
 *
 *   usage: zdb-integrity-check [--engine=hip|cpu] <dir>/zdb-data-<id>
 *
 * --engine=cpu selects the scalar drop-in engine (zdb_crc32, crc32_cpu.c)
 * explicitly, e.g. to time the reference-compatible CPU path.  The default
 * engine is the GPU; if it cannot run, the tool says so and exits 1 -- it
 * never falls back silently.
 *
 * Observable behaviour mirrored from the reference:
 *   - the argument must exist and its basename start with "zdb-data-"
 *     (:121-133), but the file actually read is "<dir>/d<id>" (data.c:135);
 *   - header validation messages (data.c:197-206) go to stdout with the
 *     elapsed-time prefix and colours of zdb_danger (libzdb.h:152);
 *   - per record: 7 report lines, "data crc : ok, match" on stdout or
 *     "[-] integrity check failed: <computed> <> <expected>" on stderr;
 *     records with datalength 0 are not checked (:81-82);
 *   - a short header or payload read ends the run via zdb_diep (exit 1) with
 *     a message carrying strerror(errno) -- errno is whatever the last failing
 *     libc call left (in practice the localtime() zone lookup), SURVEY App.A.6;
 *   - exit status = number of mismatches (:162-165), reported as
 *     "[-] data file inconsistency: %d error(s)".
 *
 * Linking: the header walk and the scalar engine are linked in statically;
 * libzdbcrc.so (HIP) is dlopen'ed only when the GPU engine is about to run,
 * after the header report, so the HIP runtime's own start-up (which touches
 * the time-zone state) happens where the reference's process does nothing.
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
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include "zdb_crc32.h"
#include "zdb_datafile.h"

#define COLOR_RED "\033[31;1m"
#define COLOR_YELLOW "\033[33;1m"
#define COLOR_RESET "\033[0m"

static struct timeval g_inittime;

static void timelog(FILE *fp) {
    struct timeval n;
    gettimeofday(&n, NULL);
    double v = (double)(n.tv_usec - g_inittime.tv_usec) / 1000000 + (double)(n.tv_sec - g_inittime.tv_sec);
    fprintf(fp, "[% 15.6f]", v);
}

static void warnp(const char *str, int err) {
    timelog(stderr);
    fprintf(stderr, COLOR_YELLOW "[-] %s: %s" COLOR_RESET "\n", str, strerror(err));
}

/* ---- report buffer ------------------------------------------------------ */

typedef struct {
    char *p;
    size_t n, cap;
} outbuf_t;

static void ob_reserve(outbuf_t *b, size_t more) {
    if (b->n + more <= b->cap)
        return;
    size_t cap = b->cap ? b->cap * 2 : (1u << 20);
    while (cap < b->n + more)
        cap *= 2;
    b->p = realloc(b->p, cap);
    if (!b->p) {
        perror("realloc");
        exit(EXIT_FAILURE);
    }
    b->cap = cap;
}

static void ob_str(outbuf_t *b, const char *s) {
    size_t l = strlen(s);
    ob_reserve(b, l);
    memcpy(b->p + b->n, s, l);
    b->n += l;
}

static void ob_u64(outbuf_t *b, uint64_t v) {
    char tmp[24];
    int i = 0;
    do {
        tmp[i++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    ob_reserve(b, (size_t)i);
    while (i)
        b->p[b->n++] = tmp[--i];
}

static const char hexdig[] = "0123456789abcdef";

static void ob_hex32(outbuf_t *b, uint32_t v, int width) {
    char tmp[8];
    int i = 0;
    do {
        tmp[i++] = hexdig[v & 15];
        v >>= 4;
    } while (v);
    ob_reserve(b, 8);
    for (int k = i; k < width; k++)
        b->p[b->n++] = '0';
    while (i)
        b->p[b->n++] = tmp[--i];
}

static void ob_flush(outbuf_t *b) {
    if (b->n)
        fwrite(b->p, 1, b->n, stdout);
    b->n = 0;
}

/* ---- GPU engine, resolved at run time ------------------------------------ */

typedef struct {
    int (*batch)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t);
    const char *(*strerror)(int);
    void *(*host_alloc)(size_t);
} gpu_api_t;

static int load_gpu(gpu_api_t *api) {
    const char *env = getenv("ZDBCRC_LIB");
    char path[4096];
    if (env) {
        snprintf(path, sizeof(path), "%s", env);
    } else {
        char exe[4096];
        ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
        if (n <= 0)
            return -1;
        exe[n] = 0;
        snprintf(path, sizeof(path), "%s/../lib/libzdbcrc.so", dirname(exe));
    }
    void *h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "[-] zdb-integrity-check: cannot load %s: %s\n", path, dlerror());
        return -1;
    }
    api->batch = (int (*)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *,
                          size_t))dlsym(h, "zdb_crc32_batch");
    api->strerror = (const char *(*)(int))dlsym(h, "zdb_crc32_strerror");
    api->host_alloc = (void *(*)(size_t))dlsym(h, "zdb_crc32_host_alloc");
    return (api->batch && api->strerror && api->host_alloc) ? 0 : -1;
}

/* ---- file loading --------------------------------------------------------- */

static uint8_t *load_file(int fd, size_t *len, const gpu_api_t *gpu, int *read_errno) {
    struct stat sb;
    *read_errno = 0;
    if (fstat(fd, &sb) != 0) {
        *read_errno = errno;
        return NULL;
    }
    size_t size = (size_t)sb.st_size;
    uint8_t *buf = gpu ? gpu->host_alloc(size + 16) : malloc(size + 16);
    if (!buf) {
        *read_errno = ENOMEM;
        return NULL;
    }
    size_t got = 0;
    while (got < size) {
        ssize_t r = read(fd, buf + got, size - got);
        if (r < 0) {
            *read_errno = errno;
            break;
        }
        if (r == 0)
            break;
        got += (size_t)r;
    }
    *len = got;
    return buf;
}

static void usage(const char *prog) {
    fprintf(stderr, "Usage: %s data-filename\n", prog);
    exit(EXIT_FAILURE);
}

int main(int argc, char *argv[]) {
    int use_gpu = 1;
    int argi = 1;
    while (argi < argc && strncmp(argv[argi], "--", 2) == 0) {
        if (!strcmp(argv[argi], "--engine=cpu"))
            use_gpu = 0;
        else if (!strcmp(argv[argi], "--engine=hip"))
            use_gpu = 1;
        else
            usage(argv[0]);
        argi++;
    }
    if (argc - argi < 1)
        usage(argv[0]);

    char *filename = argv[argi];
    printf("[+] checking data integrity of: %s\n", filename);

    struct stat sb;
    if (stat(filename, &sb) != 0 || S_ISDIR(sb.st_mode)) {
        fprintf(stderr, "[-] %s: invalid target file\n", filename);
        exit(EXIT_FAILURE);
    }

    char *filedir = dirname(strdup(filename));
    char *datafile = basename(filename);
    if (strncmp(datafile, "zdb-data-", 9)) {
        fprintf(stderr, "[-] integrity-check: data filename seems wrong\n");
        exit(EXIT_FAILURE);
    }
    uint32_t dataid = (uint32_t)atoi(datafile + 9);

    printf("[+] datafile path: %s\n", filedir);
    printf("[+] datafile name: %s\n", datafile);
    printf("[+] datafile id  : %d\n", (int)dataid);
    gettimeofday(&g_inittime, NULL);

    /* the file actually read is <dir>/d<id> (data.c:135) */
    char path[4096];
    snprintf(path, sizeof(path), "%s/d%u", filedir, dataid);
    int errors = 0;
    int fd = open(path, O_RDONLY);
    if (fd < 0) {
        warnp(path, errno);
        errors = 1;
        fflush(stdout);
        fprintf(stderr, "[-] data file inconsistency: %d error(s)\n", errors);
        return errors;
    }

    /* descriptor load + validate (data.c:177-209), before anything touches
     * the GPU so that errno evolves as in the reference process */
    uint8_t hdr[ZDB_DATA_HEADER_SIZE];
    if (pread(fd, hdr, sizeof(hdr), 0) != (ssize_t)sizeof(hdr)) {
        close(fd);
        fflush(stdout);
        fprintf(stderr, "[-] data file inconsistency: %d error(s)\n", 1);
        return 1;
    }
    uint32_t version;
    memcpy(&version, hdr + 4, 4);
    if (memcmp(hdr, "DAT0", 4)) {
        timelog(stdout);
        printf(COLOR_RED "[-] %s: invalid header, wrong magic" COLOR_RESET "\n", path);
        fflush(stdout);
        fprintf(stderr, "[-] data file inconsistency: %d error(s)\n", 1);
        return 1;
    }
    if (version != ZDB_DATAFILE_VERSION) {
        timelog(stdout);
        printf(COLOR_RED "[-] %s: unsupported version detected" COLOR_RESET "\n", path);
        timelog(stdout);
        printf(COLOR_RED "[-] file version: %d, supported version: %d" COLOR_RESET "\n", (int)version,
               ZDB_DATAFILE_VERSION);
        fflush(stdout);
        fprintf(stderr, "[-] data file inconsistency: %d error(s)\n", 1);
        return 1;
    }

    uint64_t created, opened;
    memcpy(&created, hdr + 8, 8);
    memcpy(&opened, hdr + 16, 8);
    char datestr[64];
    printf("[+] integrity-check: header seems correct\n");
    /* zdb_header_date takes a uint32_t epoch (libzdb.c:156) */
    errno = 0;
    time_t t = (time_t)(uint32_t)created;
    strftime(datestr, sizeof(datestr), "%F %T", localtime(&t));
    printf("[+] integrity-check: created at: %s\n", datestr);
    t = (time_t)(uint32_t)opened;
    strftime(datestr, sizeof(datestr), "%F %T", localtime(&t));
    printf("[+] integrity-check: last open: %s\n", datestr);
    const int stale_errno = errno; /* what zdb_diep would report below */

    gpu_api_t gpu = {0};
    if (use_gpu && load_gpu(&gpu) != 0) {
        fflush(stdout);
        fprintf(stderr, "[-] zdb-integrity-check: GPU engine unavailable (use --engine=cpu)\n");
        return EXIT_FAILURE;
    }

    size_t len = 0;
    int read_errno = 0;
    uint8_t *image = load_file(fd, &len, use_gpu ? &gpu : NULL, &read_errno);
    close(fd);
    if (!image) {
        warnp(path, read_errno);
        return EXIT_FAILURE;
    }

    /* header walk -> descriptors */
    int status = 0;
    long nrec = zdb_datafile_walk(image, len, NULL, 0, &status);
    zdb_record_t *recs = calloc((size_t)(nrec > 0 ? nrec : 1), sizeof(zdb_record_t));
    nrec = zdb_datafile_walk(image, len, recs, nrec, &status);

    /* payloads present in full are checksummed in one batch */
    long nfull = (status == ZDB_WALK_SHORT_PAYLOAD) ? nrec - 1 : nrec;
    uint64_t *offs = malloc(sizeof(uint64_t) * (size_t)(nfull + 1));
    uint32_t *lens = malloc(sizeof(uint32_t) * (size_t)(nfull + 1));
    uint32_t *idx = malloc(sizeof(uint32_t) * (size_t)(nfull + 1));
    uint32_t *crc = malloc(sizeof(uint32_t) * (size_t)(nfull + 1));
    size_t m = zdb_datafile_payloads(recs, (size_t)nfull, offs, lens, NULL, idx);
    if (m) {
        if (use_gpu) {
            int rc = gpu.batch(image, len, offs, lens, crc, m);
            if (rc) {
                fflush(stdout);
                fprintf(stderr, "[-] zdb-integrity-check: GPU engine failed: %s (use --engine=cpu)\n",
                        gpu.strerror(rc));
                return EXIT_FAILURE;
            }
        } else {
            for (size_t i = 0; i < m; i++)
                crc[i] = zdb_crc32(image + offs[i], (ssize_t)lens[i]);
        }
    }

    outbuf_t ob = {0};
    size_t k = 0;
    for (long i = 0; i < nrec; i++) {
        const zdb_record_t *r = &recs[i];
        const uint8_t *h = image + r->header_offset;
        ob_str(&ob, "[+] data entry: ");
        ob_u64(&ob, (uint64_t)(i + 1));
        ob_str(&ob, ", id length: ");
        ob_u64(&ob, r->idlength);
        ob_str(&ob, "\n[+]   expected length: ");
        ob_u64(&ob, r->datalength);
        ob_str(&ob, ", current offset: ");
        ob_u64(&ob, r->header_offset);
        ob_str(&ob, "\n[+]   previous offset: ");
        ob_u64(&ob, r->previous);
        ob_str(&ob, "\n[+]   expected crc   : ");
        ob_hex32(&ob, r->integrity, 8);
        ob_str(&ob, "\n[+]   entry flags    : 0x");
        ob_hex32(&ob, r->flags, 1);
        ob_str(&ob, "\n[+]   entry key      : 0x");
        ob_reserve(&ob, 2u * r->idlength + 1);
        for (uint32_t b = 0; b < r->idlength; b++) {
            ob.p[ob.n++] = hexdig[h[ZDB_ENTRY_HEADER_SIZE + b] >> 4];
            ob.p[ob.n++] = hexdig[h[ZDB_ENTRY_HEADER_SIZE + b] & 15];
        }
        ob.p[ob.n++] = '\n';

        if (r->datalength == 0)
            continue;
        if (i >= nfull) { /* short payload: zdb_diep (integrity-check.c:87-88) */
            ob_flush(&ob);
            fflush(stdout);
            warnp("payload entry read failed", stale_errno);
            exit(EXIT_FAILURE);
        }
        if (crc[k] != r->integrity) {
            ob_flush(&ob);
            fflush(stdout);
            fprintf(stderr, "[-] integrity check failed: %08x <> %08x\n", crc[k], r->integrity);
            errors += 1;
        } else {
            ob_str(&ob, "[+]   data crc       : ok, match\n");
        }
        k++;
    }
    ob_flush(&ob);
    if (status == ZDB_WALK_SHORT_HEADER) { /* integrity-check.c:68-69 */
        fflush(stdout);
        warnp("data header read failed", stale_errno);
        exit(EXIT_FAILURE);
    }
    fflush(stdout);
    if (errors)
        fprintf(stderr, "[-] data file inconsistency: %d error(s)\n", errors);
    return errors;
}
