/* Where the GPU engine's start-up time goes (f1): the HIP runtime
 * calls the first zdb_crc32_batch makes, timed one by one in a fresh process
 * before the library's own first batch, which is then left with the table
 * image, its code object and its first launches.
 *   build: hipcc -O2 scripts/hip_init_breakdown.cpp -ldl -o <out>
 *   run:   <out> [libzdbcrc.so]  -> one JSON line */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(int argc, char **argv) {
    const char *lib = argc > 1 ? argv[1] : "0-db_amd/lib/libzdbcrc.so";
    double t[16];
    int k = 0;
    t[k++] = now();
    void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        fprintf(stderr, "%s\n", dlerror());
        return 1;
    }
    t[k++] = now();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1)
        return 2;
    t[k++] = now();
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    t[k++] = now();
    void *d = nullptr;
    hipMalloc(&d, 1u << 20);
    t[k++] = now();
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    t[k++] = now();
    void *hp = nullptr;
    hipHostMalloc(&hp, 1u << 16, hipHostMallocMapped | hipHostMallocCoherent);
    t[k++] = now();
    hipMemcpyAsync(d, hp, 4096, hipMemcpyHostToDevice, st);
    hipStreamSynchronize(st);
    t[k++] = now();
    int (*batch)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t) =
        (int (*)(const uint8_t *, size_t, const uint64_t *, const uint32_t *, uint32_t *, size_t))dlsym(
            h, "zdb_crc32_batch");
    uint8_t buf[64];
    memset(buf, 7, sizeof(buf));
    uint64_t off = 0;
    uint32_t len = 64, out = 0;
    int rc = batch(buf, sizeof(buf), &off, &len, &out, 1);
    t[k++] = now();
    rc |= batch(buf, sizeof(buf), &off, &len, &out, 1);
    t[k++] = now();
    printf("{\"rc\": %d, \"dlopen_ms\": %.2f, \"hipGetDeviceCount_ms\": %.2f, \"hipGetDeviceProperties_ms\": %.2f, "
           "\"hipMalloc_ms\": %.2f, \"hipStreamCreate_ms\": %.2f, \"hipHostMalloc_mapped_ms\": %.2f, "
           "\"first_copy_ms\": %.2f, \"lib_first_batch_ms\": %.2f, \"lib_second_batch_ms\": %.3f}\n",
           rc, (t[1] - t[0]) * 1e3, (t[2] - t[1]) * 1e3, (t[3] - t[2]) * 1e3, (t[4] - t[3]) * 1e3,
           (t[5] - t[4]) * 1e3, (t[6] - t[5]) * 1e3, (t[7] - t[6]) * 1e3, (t[8] - t[7]) * 1e3,
           (t[9] - t[8]) * 1e3);
    return 0;
}
