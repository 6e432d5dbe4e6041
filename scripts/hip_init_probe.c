/* Start-up costs of the GPU engine as the integrity tool sees them (f1):
 * dlopen of libzdbcrc.so, first device query, device bind, first batch
 * (table upload + workspace + code object), pinned allocations. */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    const char *lib = argc > 1 ? argv[1] : "0-db_amd/lib/libzdbcrc.so";
    double t0 = now();
    void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!h) { fprintf(stderr, "%s\n", dlerror()); return 1; }
    double t1 = now();
    int (*count)(void) = dlsym(h, "zdb_crc32_device_count");
    int (*use)(int) = dlsym(h, "zdb_crc32_use_device");
    int (*batch)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t) = dlsym(h, "zdb_crc32_batch");
    void *(*halloc)(size_t) = dlsym(h, "zdb_crc32_host_alloc");
    void (*hfree)(void *) = dlsym(h, "zdb_crc32_host_free");
    int n = count();
    double t2 = now();
    use(0);
    double t3 = now();
    uint8_t buf[4096];
    memset(buf, 7, sizeof(buf));
    uint64_t off = 0;
    uint32_t len = 4096, out = 0;
    int rc = batch(buf, sizeof(buf), &off, &len, &out, 1);
    double t4 = now();
    rc |= batch(buf, sizeof(buf), &off, &len, &out, 1);
    double t5 = now();
    void *p32 = halloc(32u << 20);
    double t6 = now();
    void *p288 = halloc(288u << 20);
    double t7 = now();
    memset(p288, 1, 288u << 20);
    double t8 = now();
    void *m288 = malloc(288u << 20);
    memset(m288, 1, 288u << 20);
    double t9 = now();
    hfree(p32);
    hfree(p288);
    printf("{\"devices\": %d, \"rc\": %d, \"dlopen_ms\": %.2f, \"device_count_ms\": %.2f, \"use_device_ms\": %.2f, "
           "\"first_batch_ms\": %.2f, \"second_batch_ms\": %.3f, \"host_alloc_32MiB_ms\": %.2f, "
           "\"host_alloc_288MiB_ms\": %.2f, \"touch_pinned_288MiB_ms\": %.2f, \"malloc_touch_288MiB_ms\": %.2f}\n",
           n, rc, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3,
           (t6 - t5) * 1e3, (t7 - t6) * 1e3, (t8 - t7) * 1e3, (t9 - t8) * 1e3);
    return 0;
}
