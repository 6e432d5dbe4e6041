/*
 * zdb-integrity-check -- GPU counterpart of 0-db's tools/integrity-check.
 *
 * Same command line, stdout, stderr and exit status as the reference tool
 * (tools/integrity-check/integrity-check.c:30-166) for one datafile, but
 * restructured for the MI355X: the datafile is read with large reads and
 * streamed into a device image, the host walks the entry headers
 * (zdb_datafile_walk), every payload checksum is computed in ONE batched GPU
 * pass over the image (crc32_hip.hip), and the report is formatted in a
 * single buffer.  The
 * reference does 4 syscalls and ~7 printf per record around one CPU crc each
 * (integrity-check.c:59-105).
 *
 *   usage: zdb-integrity-check [--engine=hip|cpu|auto] [--jobs=J] [--gpus=G]
 *                              <dir>/zdb-data-<id> [<dir>/zdb-data-<id> ...]
 *
 * Engines:
 *   hip  every checksum on the GPU; if the GPU cannot run, the tool says so
 *        and exits 1 -- it never falls back silently;
 *   cpu  the scalar drop-in engine (zdb_crc32, crc32_cpu.c), e.g. to time the
 *        reference-compatible CPU path;
 *   auto (default) the scalar engine when the whole scan would finish on the workers'
 *        cores before the GPU could pay for its start-up (HIP start-up costs
 *        ~0.2 s, longer than reading and checking one 256 MiB datafile on a
 *        core: DESIGN.md §7; AUTO_* below); otherwise the GPU is started and
 *        takes every file read after it is up, the scalar engine the files
 *        before.  Both engines are bit-exact, so the report does not depend
 *        on the choice.
 *
 * Ingest: the GPU runtime is brought up on a thread of its
 * own at start, while the workers read.  Each worker reads its file in 32 MiB
 * preads into one reused buffer and, once the GPU is up, streams every chunk
 * into a device image through a ring of pinned slots
 * (zdb_crc32_stream_append: the H2D copy of a chunk overlaps the read of the
 * next); the host walks the headers (zdb_datafile_walk) and one batched
 * checksum over the device image (zdb_crc32_stream_checksum) gives every
 * payload crc.
 *
 * Several datafiles (the store-wide scan): each file's
 * report is exactly what one reference run on that file prints, and the
 * reports appear in argument order.  J worker threads (default: 1 for one
 * file, min(files, 8) otherwise) each read, walk and checksum whole files
 * concurrently; worker w runs its batches on GPU w mod G (default G = every
 * visible GPU) -- datafiles are independent (records never span files,
 * api.c:300-303), so the scan shards with no device-to-device exchange.  The
 * exit status is the total mismatch count over all files (the reference's
 * per-file status, summed), saturated at 255 so that a multiple of 256 never
 * reads as 0; a fatal error in one file (zdb_diep: short header
 * or payload, exit 1) ends the run after the reports of the files before it.
 *
 * Observable behaviour mirrored from the reference, per file:
 *   - the argument must exist and its basename start with "zdb-data-"
 *     (:121-133), but the file actually read is "<dir>/d<id>" (data.c:135);
 *   - header validation messages (data.c:197-206) go to stdout with the
 *     elapsed-time prefix and colours of zdb_danger (libzdb.h:152);
 *   - per record: 7 report lines, "data crc : ok, match" on stdout or
 *     "[-] integrity check failed: <computed> <> <expected>" on stderr;
 *     records with datalength 0 are not checked (:81-82);
 *   - a short header or payload read ends the run via zdb_diep (exit 1) with
 *     a message carrying strerror(errno) -- errno is whatever the last failing
 *     libc call left in a fresh process (in practice the time-zone lookup of
 *     the first localtime(), captured once at start-up), SURVEY App.A.6;
 *   - exit status = number of mismatches (:162-165), reported as
 *     "[-] data file inconsistency: %d error(s)".
 *
 * Linking: the header walk and the scalar engine are linked in statically;
 * libzdbcrc.so (HIP) is dlopen'ed only when the GPU engine is first needed.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <libgen.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include "zdb_crc32.h"
#include "zdb_datafile.h"

#define COLOR_RED "\033[31;1m"
#define COLOR_YELLOW "\033[33;1m"
#define COLOR_RESET "\033[0m"

#define FATAL_EXIT 0x100 /* result flag: the reference process would have exited here */

/* ---- per-file report: stdout bytes with stderr lines anchored in them ---- */

typedef struct {
    char *p;
    size_t n, cap;
} outbuf_t;

static void ob_reserve(outbuf_t *b, size_t more) {
    if (b->n + more <= b->cap)
        return;
    size_t cap = b->cap ? b->cap * 2 : (1u << 16);
    while (cap < b->n + more)
        cap *= 2;
    b->p = realloc(b->p, cap);
    if (!b->p) {
        perror("realloc");
        exit(EXIT_FAILURE);
    }
    b->cap = cap;
}

static void ob_mem(outbuf_t *b, const char *s, size_t l) {
    ob_reserve(b, l);
    memcpy(b->p + b->n, s, l);
    b->n += l;
}

static void ob_str(outbuf_t *b, const char *s) { ob_mem(b, s, strlen(s)); }

static void ob_printf(outbuf_t *b, const char *fmt, ...) {
    char tmp[8192];
    va_list ap;
    va_start(ap, fmt);
    int l = vsnprintf(tmp, sizeof(tmp), fmt, ap);
    va_end(ap);
    if (l > 0)
        ob_mem(b, tmp, (size_t)l < sizeof(tmp) ? (size_t)l : sizeof(tmp) - 1);
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

typedef struct {
    outbuf_t out;   /* everything the file's run writes to stdout            */
    outbuf_t err;   /* everything it writes to stderr, line after line       */
    size_t *anchor; /* anchor[i]: stdout bytes written before stderr line i  */
    size_t *eend;   /* eend[i]: end of stderr line i in err                  */
    size_t nerr, cap_err;
    int status;     /* errors for this file, | FATAL_EXIT (exit code in low bits) */
    struct timeval t0; /* the file's zdb_inittime (elapsed-time prefix origin) */
} report_t;

static void rep_err(report_t *r, const char *fmt, ...) {
    if (r->nerr == r->cap_err) {
        r->cap_err = r->cap_err ? 2 * r->cap_err : 16;
        r->anchor = realloc(r->anchor, r->cap_err * sizeof(size_t));
        r->eend = realloc(r->eend, r->cap_err * sizeof(size_t));
        if (!r->anchor || !r->eend) {
            perror("realloc");
            exit(EXIT_FAILURE);
        }
    }
    char tmp[8192];
    va_list ap;
    va_start(ap, fmt);
    int l = vsnprintf(tmp, sizeof(tmp), fmt, ap);
    va_end(ap);
    if (l > 0)
        ob_mem(&r->err, tmp, (size_t)l < sizeof(tmp) ? (size_t)l : sizeof(tmp) - 1);
    r->anchor[r->nerr] = r->out.n;
    r->eend[r->nerr] = r->err.n;
    r->nerr++;
}

/* write the report to the real streams, keeping the stdout/stderr order */
static void rep_emit(report_t *r) {
    size_t pos = 0, epos = 0;
    for (size_t i = 0; i < r->nerr; i++) {
        if (r->anchor[i] > pos)
            fwrite(r->out.p + pos, 1, r->anchor[i] - pos, stdout);
        pos = r->anchor[i];
        fflush(stdout);
        fwrite(r->err.p + epos, 1, r->eend[i] - epos, stderr);
        epos = r->eend[i];
    }
    if (r->out.n > pos)
        fwrite(r->out.p + pos, 1, r->out.n - pos, stdout);
    fflush(stdout);
}

static void rep_free(report_t *r) {
    free(r->out.p);
    free(r->err.p);
    free(r->anchor);
    free(r->eend);
    memset(r, 0, sizeof(*r));
}

static double elapsed(const report_t *r) {
    struct timeval n;
    gettimeofday(&n, NULL);
    return (double)(n.tv_usec - r->t0.tv_usec) / 1000000 + (double)(n.tv_sec - r->t0.tv_sec);
}

/* zdb_warnp (libzdb.c:110-115): elapsed-time prefix, yellow, strerror */
static void rep_warnp(report_t *r, const char *str, int err) {
    rep_err(r, "[% 15.6f]" COLOR_YELLOW "[-] %s: %s" COLOR_RESET "\n", elapsed(r), str, strerror(err));
}

/* zdb_danger (libzdb.h:152) to stdout */
static void rep_danger(report_t *r, const char *fmt, const char *a, int b, int c) {
    ob_printf(&r->out, "[% 15.6f]", elapsed(r));
    ob_str(&r->out, COLOR_RED);
    ob_printf(&r->out, fmt, a, b, c);
    ob_str(&r->out, COLOR_RESET "\n");
}

/* ---- GPU engine, resolved at run time ------------------------------------ */

typedef struct {
    int (*batch)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t);
    const char *(*strerror)(int);
    int (*device_count)(void);
    int (*use_device)(int);
    zdb_crc32_stream_t *(*stream_open)(size_t, int);
    int (*stream_begin)(zdb_crc32_stream_t *, size_t);
    int (*stream_append)(zdb_crc32_stream_t *, const uint8_t *, size_t);
    int (*stream_checksum)(zdb_crc32_stream_t *, const uint64_t *, const uint32_t *, uint32_t *, size_t);
    void (*stream_close)(zdb_crc32_stream_t *);
    int (*host_register)(void *, size_t); /* optional: pinned reads (f1) */
    void (*host_unregister)(void *);
} gpu_api_t;

static gpu_api_t g_gpu;
static int g_gpu_ok = -1; /* -1 not tried / in progress, 0 failed, 1 up */
static int g_gpu_count = 0;
static int g_gpu_devices = 0; /* devices the workers are spread over */
static pthread_mutex_t g_gpu_mu = PTHREAD_MUTEX_INITIALIZER;
static pthread_cond_t g_gpu_cv = PTHREAD_COND_INITIALIZER;
static double g_gpu_t0, g_gpu_t_count, g_gpu_t_up; /* start-up thread timeline (--trace) */
static double g_t_main;                            /* process timeline origin (--trace) */

#define ENGINE_CPU 0
#define ENGINE_HIP 1
#define ENGINE_AUTO 2

/* --engine=auto: bring the GPU up only when the scan can gain from it.  A
 * worker checksums host memory at AUTO_CPU_GIBS on the scalar engine; the GPU
 * engine pays AUTO_GPU_START_S of runtime start-up and moves the bytes over
 * PCIe at AUTO_PCIE_GIBS (DESIGN.md §7.1 measures all three), so the GPU is
 * started only when bytes / (workers * cpu) > start + bytes / pcie. */
/* With J workers the rule can only hold when J * AUTO_CPU_GIBS < AUTO_PCIE_GIBS,
 * i.e. for at most 3 workers: a scan with 4 or more workers stays on the
 * scalar engine whatever its size (the host checksums faster than PCIe moves
 * the bytes). */
#define AUTO_CPU_GIBS 10.0
#define AUTO_GPU_START_S 0.30 /* HIP start-up 150-340 ms + exit, profiles/r3/tool_timeline.jsonl */
#define AUTO_PCIE_GIBS 40.0

#define READ_CHUNK (32u << 20)  /* pread size: one H2D chunk per read */
#define SLOT_BYTES (8u << 20)   /* pinned staging slot (when buffers cannot be pinned in place) */
#define SLOTS 4
#define SLOT_BYTES_PINNED (1u << 20) /* the ring is only a fallback when buffers are pinned in place */
#define SLOTS_PINNED 2
#define MAX_PREPARED 256       /* worker streams the start-up thread opens ahead */

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + (double)t.tv_nsec * 1e-9;
}

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
    if (!h) {
        fprintf(stderr, "[-] zdb-integrity-check: cannot load %s: %s\n", path, dlerror());
        return 0;
    }
    g_gpu.batch = (int (*)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *,
                           size_t))dlsym(h, "zdb_crc32_batch");
    g_gpu.strerror = (const char *(*)(int))dlsym(h, "zdb_crc32_strerror");
    g_gpu.device_count = (int (*)(void))dlsym(h, "zdb_crc32_device_count");
    g_gpu.use_device = (int (*)(int))dlsym(h, "zdb_crc32_use_device");
    g_gpu.stream_open = (zdb_crc32_stream_t * (*)(size_t, int)) dlsym(h, "zdb_crc32_stream_open");
    g_gpu.stream_begin = (int (*)(zdb_crc32_stream_t *, size_t))dlsym(h, "zdb_crc32_stream_begin");
    g_gpu.stream_append =
        (int (*)(zdb_crc32_stream_t *, const uint8_t *, size_t))dlsym(h, "zdb_crc32_stream_append");
    g_gpu.stream_checksum = (int (*)(zdb_crc32_stream_t *, const uint64_t *, const uint32_t *, uint32_t *,
                                     size_t))dlsym(h, "zdb_crc32_stream_checksum");
    g_gpu.stream_close = (void (*)(zdb_crc32_stream_t *))dlsym(h, "zdb_crc32_stream_close");
    g_gpu.host_register = (int (*)(void *, size_t))dlsym(h, "zdb_crc32_host_register");
    g_gpu.host_unregister = (void (*)(void *))dlsym(h, "zdb_crc32_host_unregister");
    if (!g_gpu.host_register || !g_gpu.host_unregister)
        g_gpu.host_register = NULL;
    if (!g_gpu.batch || !g_gpu.strerror || !g_gpu.device_count || !g_gpu.use_device || !g_gpu.stream_open ||
        !g_gpu.stream_begin || !g_gpu.stream_append || !g_gpu.stream_checksum || !g_gpu.stream_close)
        return 0;
    g_gpu_count = g_gpu.device_count();
    return g_gpu_count > 0;
}

/* what the start-up thread prepares besides the devices */
typedef struct {
    int gpus;        /* --gpus */
    int jobs;        /* worker threads */
    size_t max_file; /* largest file of the scan (device image size) */
} gpu_prep_t;

static int g_pin_off = -1; /* ZDBCRC_TOOL_PIN=0: no in-place pinning (measurement A/B) */
static int pin_off(void) {
    if (g_pin_off < 0) {
        const char *e = getenv("ZDBCRC_TOOL_PIN");
        g_pin_off = e && e[0] == '0';
    }
    return g_pin_off;
}

static zdb_crc32_stream_t *g_pre_stream[MAX_PREPARED]; /* worker j's ingest stream, opened ahead */
static double g_gpu_t_dev;                             /* devices up (before the streams) */

/* the GPU start-up thread: load the library, bring every device the workers
 * will use up (code object, tables, workspace: one tiny batch each), then
 * open every worker's ingest stream with its device image sized for the
 * largest file -- while the workers read their first files, so that a worker
 * that finds the GPU up only pins its buffer and copies (the eight workers'
 * stream set-up otherwise contends in the runtime right when the GPU comes up:
 * 70-160 ms per worker, profiles/r3/tool_timeline.jsonl) */
static void *gpu_init_main(void *arg) {
    const gpu_prep_t *prep = (const gpu_prep_t *)arg;
    const int want = prep->gpus;
    g_gpu_t0 = now_s();
    int ok = load_gpu();
    g_gpu_t_count = now_s();
    if (ok) {
        g_gpu_devices = want > 0 && want < g_gpu_count ? want : g_gpu_count;
        for (int d = 0; ok && d < g_gpu_devices; d++) {
            uint8_t b[64] = {0};
            uint64_t o = 0;
            uint32_t l = 64, c = 0;
            ok = g_gpu.use_device(d) == 0 && g_gpu.batch(b, sizeof(b), &o, &l, &c, 1) == 0;
        }
    }
    g_gpu_t_dev = now_s();
    const int pinned = g_gpu.host_register && !pin_off();
    for (int j = 0; ok && j < prep->jobs && j < MAX_PREPARED; j++) {
        if (g_gpu.use_device(j % g_gpu_devices) != 0)
            break;
        zdb_crc32_stream_t *st = g_gpu.stream_open(pinned ? SLOT_BYTES_PINNED : SLOT_BYTES, pinned ? SLOTS_PINNED : SLOTS);
        if (st && prep->max_file && g_gpu.stream_begin(st, prep->max_file) != 0) {
            g_gpu.stream_close(st);
            st = NULL;
        }
        g_pre_stream[j] = st; /* NULL: the worker opens its own */
    }
    pthread_mutex_lock(&g_gpu_mu);
    g_gpu_t_up = now_s();
    g_gpu_ok = ok;
    pthread_cond_broadcast(&g_gpu_cv);
    pthread_mutex_unlock(&g_gpu_mu);
    return NULL;
}

/* 1 up, 0 failed, -1 still starting (wait = 0) */
static int gpu_state(int wait) {
    pthread_mutex_lock(&g_gpu_mu);
    while (wait && g_gpu_ok < 0)
        pthread_cond_wait(&g_gpu_cv, &g_gpu_mu);
    const int st = g_gpu_ok;
    pthread_mutex_unlock(&g_gpu_mu);
    return st;
}

/* ---- scan configuration and per-worker state ----------------------------- */

typedef struct {
    int engine;        /* ENGINE_*                                             */
    int gpus;          /* devices to spread the workers over (0 = all)        */
    int stale_errno;   /* errno a fresh process has after its first localtime */
    int trace;         /* ZDBCRC_TOOL_TRACE: per-file phase times on stderr   */
    int auto_wait;     /* ZDBCRC_AUTO_START_GPU=1 (tests): auto waits for the
                          GPU start-up instead of taking the scalar engine for
                          files whose checksum starts before it is up        */
} config_t;

typedef struct {
    int id;
    int device;        /* -1 until the thread has bound its GPU               */
    uint8_t *buf;      /* file image, reused from file to file                */
    size_t cap;
    int pinned;        /* buf is registered with the GPU runtime: reads land
                          in DMA-able memory and stream appends are direct  */
    zdb_crc32_stream_t *stream; /* this worker's device image + pinned ring   */
} worker_t;

/* the worker's file image: anonymous memory backed by transparent huge
 * pages where the kernel allows it (a 256 MiB read otherwise takes 65,536
 * first-touch page faults, and the faults of concurrent workers serialise on
 * the process's memory map); reused from file to file */
static uint8_t *worker_buffer(worker_t *w, size_t size) {
    if (w->cap >= size)
        return w->buf;
    if (w->pinned) {
        g_gpu.host_unregister(w->buf);
        w->pinned = 0;
    }
    if (w->buf)
        munmap(w->buf, w->cap);
    const size_t huge = 2u << 20;
    size_t cap = (size + (size >> 3) + huge) & ~(huge - 1);
    void *p = mmap(NULL, cap, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
        w->buf = NULL;
        w->cap = 0;
        return NULL;
    }
    madvise(p, cap, MADV_HUGEPAGE);
    w->buf = p;
    w->cap = cap;
    return w->buf;
}

/* the worker's ingest stream on its GPU (worker w on device w mod G) */
static int worker_stream(worker_t *w, report_t *r) {
    if (w->stream)
        return 1;
    if (w->device < 0 && w->id < MAX_PREPARED && g_pre_stream[w->id]) { /* opened by the start-up thread */
        w->device = w->id % g_gpu_devices;
        if (g_gpu.use_device(w->device) == 0) {
            w->stream = g_pre_stream[w->id];
            g_pre_stream[w->id] = NULL;
            return 1;
        }
    }
    if (w->device < 0) {
        w->device = w->id % g_gpu_devices;
        int rc = g_gpu.use_device(w->device);
        if (rc) {
            rep_err(r, "[-] zdb-integrity-check: GPU %d: %s (use --engine=cpu)\n", w->device, g_gpu.strerror(rc));
            return 0;
        }
    }
    const int pinned = g_gpu.host_register && !pin_off();
    w->stream = g_gpu.stream_open(pinned ? SLOT_BYTES_PINNED : SLOT_BYTES, pinned ? SLOTS_PINNED : SLOTS);
    if (!w->stream) {
        rep_err(r, "[-] zdb-integrity-check: GPU %d: cannot open an ingest stream (use --engine=cpu)\n", w->device);
        return 0;
    }
    return 1;
}

/* pin the worker's file buffer in place once the GPU is up (f1): the next
 * reads land in DMA-able memory and every appended chunk is one direct H2D
 * copy, overlapping the read of the next chunk -- no staging copy.  Failure
 * only leaves the staged path. */
static void worker_pin(worker_t *w, report_t *r, double *pin_ms) {
    if (pin_off() || w->pinned || !w->buf || !g_gpu.host_register || !worker_stream(w, r))
        return;
    const double t0 = now_s();
    w->pinned = g_gpu.host_register(w->buf, w->cap) == 0;
    *pin_ms += (now_s() - t0) * 1e3;
}

/* ---- one datafile, as one reference run would report it ---------------- */

static void check_file(const config_t *cfg, worker_t *w, const char *filename, report_t *r) {
    gettimeofday(&r->t0, NULL);
    ob_printf(&r->out, "[+] checking data integrity of: %s\n", filename);

    struct stat sb;
    if (stat(filename, &sb) != 0 || S_ISDIR(sb.st_mode)) {
        rep_err(r, "[-] %s: invalid target file\n", filename);
        r->status = FATAL_EXIT | EXIT_FAILURE;
        return;
    }
    char *dup1 = strdup(filename), *dup2 = strdup(filename);
    const char *filedir = dirname(dup1);
    const char *datafile = basename(dup2);
    if (strncmp(datafile, "zdb-data-", 9)) {
        rep_err(r, "[-] integrity-check: data filename seems wrong\n");
        r->status = FATAL_EXIT | EXIT_FAILURE;
        free(dup1);
        free(dup2);
        return;
    }
    uint32_t dataid = (uint32_t)atoi(datafile + 9);
    ob_printf(&r->out, "[+] datafile path: %s\n", filedir);
    ob_printf(&r->out, "[+] datafile name: %s\n", datafile);
    ob_printf(&r->out, "[+] datafile id  : %d\n", (int)dataid);
    gettimeofday(&r->t0, NULL);

    /* the file actually read is <dir>/d<id> (data.c:135) */
    char path[4096];
    snprintf(path, sizeof(path), "%s/d%u", filedir, dataid);
    free(dup1);
    free(dup2);
    int fd = open(path, O_RDONLY);
    if (fd < 0) {
        rep_warnp(r, path, errno);
        rep_err(r, "[-] data file inconsistency: %d error(s)\n", 1);
        r->status = 1;
        return;
    }

    /* descriptor load + validate (data.c:177-209) */
    uint8_t hdr[ZDB_DATA_HEADER_SIZE];
    if (pread(fd, hdr, sizeof(hdr), 0) != (ssize_t)sizeof(hdr)) {
        close(fd);
        rep_err(r, "[-] data file inconsistency: %d error(s)\n", 1);
        r->status = 1;
        return;
    }
    uint32_t version;
    memcpy(&version, hdr + 4, 4);
    if (memcmp(hdr, "DAT0", 4)) {
        close(fd);
        rep_danger(r, "[-] %s: invalid header, wrong magic", path, 0, 0);
        rep_err(r, "[-] data file inconsistency: %d error(s)\n", 1);
        r->status = 1;
        return;
    }
    if (version != ZDB_DATAFILE_VERSION) {
        close(fd);
        rep_danger(r, "[-] %s: unsupported version detected", path, 0, 0);
        ob_printf(&r->out, "[% 15.6f]", elapsed(r));
        ob_printf(&r->out, COLOR_RED "[-] file version: %d, supported version: %d" COLOR_RESET "\n", (int)version,
                  ZDB_DATAFILE_VERSION);
        rep_err(r, "[-] data file inconsistency: %d error(s)\n", 1);
        r->status = 1;
        return;
    }

    uint64_t created, opened;
    memcpy(&created, hdr + 8, 8);
    memcpy(&opened, hdr + 16, 8);
    char datestr[64];
    struct tm tmv;
    ob_str(&r->out, "[+] integrity-check: header seems correct\n");
    /* zdb_header_date takes a uint32_t epoch (libzdb.c:156) */
    time_t t = (time_t)(uint32_t)created;
    strftime(datestr, sizeof(datestr), "%F %T", localtime_r(&t, &tmv));
    ob_printf(&r->out, "[+] integrity-check: created at: %s\n", datestr);
    t = (time_t)(uint32_t)opened;
    strftime(datestr, sizeof(datestr), "%F %T", localtime_r(&t, &tmv));
    ob_printf(&r->out, "[+] integrity-check: last open: %s\n", datestr);

    /* the file in 32 MiB reads; once the GPU is up, each chunk is streamed
     * into the worker's device image as soon as it is read */
    const double t_read = now_s();
    size_t len = 0, sent = 0;
    int read_errno = 0, streaming = 0, gpu_failed = 0;
    double pin_ms = 0;
    uint8_t *image = NULL;
    size_t size = 0;
    if (fstat(fd, &sb) != 0) {
        read_errno = errno;
    } else if (!(image = worker_buffer(w, (size_t)sb.st_size + 16))) {
        read_errno = ENOMEM;
    } else {
        size = (size_t)sb.st_size;
        if (cfg->engine != ENGINE_CPU && gpu_state(0) == 1)
            worker_pin(w, r, &pin_ms);
        while (len < size) {
            ssize_t got = pread(fd, image + len, size - len > READ_CHUNK ? READ_CHUNK : size - len, (off_t)len);
            if (got < 0) {
                read_errno = errno;
                break;
            }
            if (got == 0)
                break;
            len += (size_t)got;
            if (cfg->engine != ENGINE_CPU && !streaming && !gpu_failed && gpu_state(0) == 1) {
                if (worker_stream(w, r) && g_gpu.stream_begin(w->stream, size) == 0) {
                    streaming = 1;
                    worker_pin(w, r, &pin_ms); /* the GPU came up during this file */
                } else {
                    gpu_failed = 1;
                }
            }
            if (streaming) {
                if (g_gpu.stream_append(w->stream, image + sent, len - sent) != 0) {
                    gpu_failed = 1;
                    streaming = 0;
                }
                sent = len;
            }
        }
    }
    close(fd);
    if (read_errno) {
        rep_warnp(r, path, read_errno);
        r->status = FATAL_EXIT | EXIT_FAILURE;
        return;
    }
    const double t_walk = now_s();

    /* header walk -> descriptors */
    int status = 0;
    long nrec = zdb_datafile_walk(image, len, NULL, 0, &status);
    zdb_record_t *recs = calloc((size_t)(nrec > 0 ? nrec : 1), sizeof(zdb_record_t));
    nrec = zdb_datafile_walk(image, len, recs, nrec, &status);

    /* payloads present in full are checksummed in one batch */
    long nfull = (status == ZDB_WALK_SHORT_PAYLOAD) ? nrec - 1 : nrec;
    uint64_t *offs = malloc(sizeof(uint64_t) * (size_t)(nfull + 1));
    uint32_t *lens = malloc(sizeof(uint32_t) * (size_t)(nfull + 1));
    uint32_t *crc = malloc(sizeof(uint32_t) * (size_t)(nfull + 1));
    size_t m = zdb_datafile_payloads(recs, (size_t)nfull, offs, lens, NULL, NULL);
    int errors = 0;
    const double t_sum = now_s();
    const char *engine_used = "none";
    double gpu_wait_ms = 0;
    if (m) {
        /* hip: always the GPU (waiting for it to come up); auto: the GPU if
         * it is up by now, the scalar engine otherwise */
        int use_gpu = 0;
        if (cfg->engine == ENGINE_HIP) {
            const double t_wait = now_s();
            const int up = gpu_state(1);
            gpu_wait_ms = (now_s() - t_wait) * 1e3;
            if (up != 1) {
                rep_err(r, "[-] zdb-integrity-check: GPU engine unavailable (use --engine=cpu)\n");
                r->status = FATAL_EXIT | EXIT_FAILURE;
                goto out;
            }
            use_gpu = 1;
        } else if (cfg->engine == ENGINE_AUTO) {
            use_gpu = !gpu_failed && (streaming || gpu_state(cfg->auto_wait) == 1);
        }
        if (use_gpu) {
            int rc = 0;
            if (gpu_failed || !worker_stream(w, r)) {
                rc = ZDB_CRC32_ELAUNCH;
            } else if (!streaming) {
                worker_pin(w, r, &pin_ms); /* read before the GPU was up: pinned in place, one DMA */
                rc = g_gpu.stream_begin(w->stream, len);
                if (!rc)
                    rc = g_gpu.stream_append(w->stream, image, len);
            } else if (sent < len) {
                rc = g_gpu.stream_append(w->stream, image + sent, len - sent);
            }
            if (!rc)
                rc = g_gpu.stream_checksum(w->stream, offs, lens, crc, m);
            if (rc) {
                rep_err(r, "[-] zdb-integrity-check: GPU engine failed: %s (use --engine=cpu)\n",
                        g_gpu.strerror ? g_gpu.strerror(rc) : "library not loaded");
                r->status = FATAL_EXIT | EXIT_FAILURE;
                goto out;
            }
            engine_used = "hip";
        } else {
            for (size_t i = 0; i < m; i++)
                crc[i] = zdb_crc32(image + offs[i], (ssize_t)lens[i]);
            engine_used = "cpu";
        }
    }
    const double t_fmt = now_s();
    if (cfg->trace && m)
        fprintf(stderr, "[trace] %s: checksum engine %s, %zu payloads\n", filename, engine_used, m);

    outbuf_t *ob = &r->out;
    size_t k = 0;
    for (long i = 0; i < nrec; i++) {
        const zdb_record_t *e = &recs[i];
        const uint8_t *h = image + e->header_offset;
        ob_str(ob, "[+] data entry: ");
        ob_u64(ob, (uint64_t)(i + 1));
        ob_str(ob, ", id length: ");
        ob_u64(ob, e->idlength);
        ob_str(ob, "\n[+]   expected length: ");
        ob_u64(ob, e->datalength);
        ob_str(ob, ", current offset: ");
        ob_u64(ob, e->header_offset);
        ob_str(ob, "\n[+]   previous offset: ");
        ob_u64(ob, e->previous);
        ob_str(ob, "\n[+]   expected crc   : ");
        ob_hex32(ob, e->integrity, 8);
        ob_str(ob, "\n[+]   entry flags    : 0x");
        ob_hex32(ob, e->flags, 1);
        ob_str(ob, "\n[+]   entry key      : 0x");
        ob_reserve(ob, 2u * e->idlength + 1);
        for (uint32_t b = 0; b < e->idlength; b++) {
            ob->p[ob->n++] = hexdig[h[ZDB_ENTRY_HEADER_SIZE + b] >> 4];
            ob->p[ob->n++] = hexdig[h[ZDB_ENTRY_HEADER_SIZE + b] & 15];
        }
        ob->p[ob->n++] = '\n';

        if (e->datalength == 0)
            continue;
        if (i >= nfull) { /* short payload: zdb_diep (integrity-check.c:87-88) */
            rep_warnp(r, "payload entry read failed", cfg->stale_errno);
            r->status = FATAL_EXIT | EXIT_FAILURE;
            goto out;
        }
        if (crc[k] != e->integrity) {
            rep_err(r, "[-] integrity check failed: %08x <> %08x\n", crc[k], e->integrity);
            errors += 1;
        } else {
            ob_str(ob, "[+]   data crc       : ok, match\n");
        }
        k++;
    }
    if (status == ZDB_WALK_SHORT_HEADER) { /* integrity-check.c:68-69 */
        rep_warnp(r, "data header read failed", cfg->stale_errno);
        r->status = FATAL_EXIT | EXIT_FAILURE;
        goto out;
    }
    if (errors)
        rep_err(r, "[-] data file inconsistency: %d error(s)\n", errors);
    r->status = errors;
    if (cfg->trace)
        fprintf(stderr,
                "[trace] %s: %zu B, engine %s, worker %d, %.1f..%.1f ms, read %.2f ms (streamed: %s, buffer pinned: "
                "%s, pinning %.2f ms), walk %.2f ms, checksum %.2f ms (of which waiting for the GPU start-up %.2f "
                "ms), format %.2f ms\n",
                filename, len, engine_used, w->id, (t_read - g_t_main) * 1e3, (now_s() - g_t_main) * 1e3,
                (t_walk - t_read) * 1e3, streaming ? "yes" : "no", w->pinned ? "yes" : "no", pin_ms,
                (t_sum - t_walk) * 1e3, (t_fmt - t_sum) * 1e3, gpu_wait_ms, (now_s() - t_fmt) * 1e3);
out:
    free(recs);
    free(offs);
    free(lens);
    free(crc);
}

/* ---- the scan: J workers, reports emitted in argument order ------------- */

typedef struct {
    const config_t *cfg;
    char **files;
    int nfiles;
    report_t *reports;
    int *done;
    int next;
    int stop; /* a fatal report was produced: files after it are not needed */
    pthread_mutex_t mu;
    pthread_cond_t cv;
} scan_t;

typedef struct {
    scan_t *scan;
    worker_t w;
} worker_arg_t;

static void *worker_main(void *p) {
    worker_arg_t *a = p;
    scan_t *s = a->scan;
    for (;;) {
        pthread_mutex_lock(&s->mu);
        int i = s->stop ? s->nfiles : s->next++;
        pthread_mutex_unlock(&s->mu);
        if (i >= s->nfiles)
            break;
        check_file(s->cfg, &a->w, s->files[i], &s->reports[i]);
        pthread_mutex_lock(&s->mu);
        s->done[i] = 1;
        if (s->reports[i].status & FATAL_EXIT)
            s->stop = 1;
        pthread_cond_broadcast(&s->cv);
        pthread_mutex_unlock(&s->mu);
    }
    /* a worker that used the GPU leaves its stream, pinned buffer and
     * device image to the process's end: main ends GPU runs with _exit, and
     * unpinning or freeing ~300 MiB per worker would only delay that */
    if (a->w.buf && !a->w.stream && !a->w.pinned)
        munmap(a->w.buf, a->w.cap);
    return NULL;
}

static void usage(const char *prog) {
    fprintf(stderr, "Usage: %s data-filename\n", prog);
    exit(EXIT_FAILURE);
}

int main(int argc, char *argv[]) {
    g_t_main = now_s();
    config_t cfg = {ENGINE_AUTO, 0, 0, getenv("ZDBCRC_TOOL_TRACE") != NULL, 0};
    int jobs = 0;
    int argi = 1;
    while (argi < argc && strncmp(argv[argi], "--", 2) == 0) {
        if (!strcmp(argv[argi], "--engine=cpu"))
            cfg.engine = ENGINE_CPU;
        else if (!strcmp(argv[argi], "--engine=hip"))
            cfg.engine = ENGINE_HIP;
        else if (!strcmp(argv[argi], "--engine=auto"))
            cfg.engine = ENGINE_AUTO;
        else if (!strncmp(argv[argi], "--jobs=", 7) && atoi(argv[argi] + 7) > 0)
            jobs = atoi(argv[argi] + 7);
        else if (!strncmp(argv[argi], "--gpus=", 7) && atoi(argv[argi] + 7) > 0)
            cfg.gpus = atoi(argv[argi] + 7);
        else
            usage(argv[0]);
        argi++;
    }
    if (argc - argi < 1)
        usage(argv[0]);

    /* errno of a fresh process after its first time-zone lookup (what the
     * reference's zdb_diep reports for short reads, SURVEY App.A.6) */
    {
        errno = 0;
        time_t t = 0;
        localtime(&t);
        localtime(&t);
        cfg.stale_errno = errno;
    }

    int njobs = jobs > 0 ? jobs : (argc - argi < 8 ? argc - argi : 8);
    if (njobs > argc - argi)
        njobs = argc - argi;
    const char *force_gpu = getenv("ZDBCRC_AUTO_START_GPU"); /* tests: start the GPU whatever the size */
    cfg.auto_wait = force_gpu && force_gpu[0] == '1';
    if (cfg.engine == ENGINE_AUTO && !cfg.auto_wait) {
        double gib = 0;
        for (int i = argi; i < argc; i++) {
            struct stat fst;
            if (stat(argv[i], &fst) == 0)
                gib += (double)fst.st_size / (double)(1u << 30);
        }
        if (gib / (njobs * AUTO_CPU_GIBS) <= AUTO_GPU_START_S + gib / AUTO_PCIE_GIBS)
            g_gpu_ok = 0; /* the scalar engine finishes first: no GPU start-up */
        if (cfg.trace)
            fprintf(stderr, "[trace] auto engine: %.2f GiB over %d worker(s): %s\n", gib, njobs,
                    g_gpu_ok == 0 ? "scalar engine (the GPU start-up would not pay)" : "GPU once it is up");
    }

    /* GPU start-up overlaps the reads (the thread is never joined: a
     * worker that needs the GPU waits for it; exit does not) */
    static gpu_prep_t prep;
    prep.gpus = cfg.gpus;
    prep.jobs = njobs;
    for (int i = argi; i < argc; i++) {
        struct stat fst;
        if (stat(argv[i], &fst) == 0 && (size_t)fst.st_size > prep.max_file)
            prep.max_file = (size_t)fst.st_size;
    }
    if (cfg.engine == ENGINE_HIP || (cfg.engine == ENGINE_AUTO && g_gpu_ok != 0)) {
        pthread_t gt;
        if (pthread_create(&gt, NULL, gpu_init_main, &prep) != 0)
            g_gpu_ok = 0;
        else
            pthread_detach(gt);
    }

    scan_t s;
    memset(&s, 0, sizeof(s));
    s.cfg = &cfg;
    s.files = argv + argi;
    s.nfiles = argc - argi;
    s.reports = calloc((size_t)s.nfiles, sizeof(report_t));
    s.done = calloc((size_t)s.nfiles, sizeof(int));
    pthread_mutex_init(&s.mu, NULL);
    pthread_cond_init(&s.cv, NULL);
    if (jobs <= 0)
        jobs = s.nfiles < 8 ? s.nfiles : 8;
    if (jobs > s.nfiles)
        jobs = s.nfiles;

    worker_arg_t *wa = calloc((size_t)jobs, sizeof(worker_arg_t));
    pthread_t *th = calloc((size_t)jobs, sizeof(pthread_t));
    for (int j = 0; j < jobs; j++) {
        wa[j].scan = &s;
        wa[j].w.id = j;
        wa[j].w.device = -1;
    }
    if (jobs == 1) {
        worker_main(&wa[0]); /* one file or --jobs=1: no extra thread */
    } else {
        for (int j = 0; j < jobs; j++)
            pthread_create(&th[j], NULL, worker_main, &wa[j]);
    }

    long total = 0;
    for (int i = 0; i < s.nfiles; i++) {
        pthread_mutex_lock(&s.mu);
        while (!s.done[i])
            pthread_cond_wait(&s.cv, &s.mu);
        pthread_mutex_unlock(&s.mu);
        report_t *r = &s.reports[i];
        rep_emit(r);
        const int st = r->status;
        rep_free(r);
        if (st & FATAL_EXIT) {
            /* zdb_diep / exit(EXIT_FAILURE) in the reference run; _exit: other
             * workers may still be inside a GPU call, no teardown under them */
            fflush(stdout);
            fflush(stderr);
            _exit(st & 0xFF);
        }
        total += st;
    }
    if (jobs > 1)
        for (int j = 0; j < jobs; j++)
            pthread_join(th[j], NULL);
    /* one file: the reference's status (error count; the OS keeps its low 8
     * bits, integrity-check.c:162-165).  Several files: saturate at 255 so a
     * total that is a multiple of 256 cannot read as a clean store. */
    const int code = s.nfiles > 1 ? (total > 255 ? 255 : (int)total) : (int)(total > 0x7FFFFFFF ? 0x7FFFFFFF : total);
    free(s.reports);
    free(s.done);
    free(wa);
    free(th);
    if (cfg.trace && cfg.engine != ENGINE_CPU) {
        pthread_mutex_lock(&g_gpu_mu);
        if (g_gpu_ok >= 0 && g_gpu_t0 > 0)
            fprintf(stderr,
                    "[trace] GPU start-up: thread at %.1f ms, library load + device count %.2f ms, first batch %.2f "
                    "ms, worker streams %.2f ms, up at %.1f ms; reports done at %.1f ms\n",
                    (g_gpu_t0 - g_t_main) * 1e3, (g_gpu_t_count - g_gpu_t0) * 1e3, (g_gpu_t_dev - g_gpu_t_count) * 1e3,
                    (g_gpu_t_up - g_gpu_t_dev) * 1e3, (g_gpu_t_up - g_t_main) * 1e3, (now_s() - g_t_main) * 1e3);
        pthread_mutex_unlock(&g_gpu_mu);
    }
    if (cfg.engine != ENGINE_CPU) {
        /* the GPU start-up thread may still be inside the HIP runtime (auto
         * engine, nothing needed it): end without running teardown under it */
        fflush(stdout);
        fflush(stderr);
        _exit(code & 0xFF);
    }
    return code;
}
