// process exit cost after GPU work: HIP init, then optional device
// allocations, registered (pinned) host memory, a copy and a kernel, then
// _exit; the caller times the whole process.  usage: exit_probe dev_mib
// pin_mib copy(0/1) threads
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <pthread.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>

static size_t g_dev, g_pin;
static int g_copy;

__global__ void touch(unsigned char *p, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        p[i] = (unsigned char)i;
}

static void *work(void *) {
    unsigned char *d = nullptr;
    if (g_dev && hipMalloc(&d, g_dev) != hipSuccess)
        std::abort();
    unsigned char *h = nullptr;
    if (g_pin) {
        h = (unsigned char *)mmap(nullptr, g_pin, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        madvise(h, g_pin, MADV_HUGEPAGE);
        std::memset(h, 1, g_pin);
        if (hipHostRegister(h, g_pin, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess)
            std::abort();
    }
    if (g_copy && d && h) {
        size_t n = g_dev < g_pin ? g_dev : g_pin;
        hipMemcpy(d, h, n, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(touch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, d, n);
        hipDeviceSynchronize();
    }
    return nullptr;
}

int main(int argc, char **argv) {
    if (argc < 5)
        return 2;
    g_dev = (size_t)atol(argv[1]) << 20;
    g_pin = (size_t)atol(argv[2]) << 20;
    g_copy = atoi(argv[3]);
    int nt = atoi(argv[4]);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n < 1)
        return 3;
    pthread_t t[64];
    for (int i = 0; i < nt; i++)
        pthread_create(&t[i], nullptr, work, nullptr);
    for (int i = 0; i < nt; i++)
        pthread_join(t[i], nullptr);
    std::fflush(stdout);
    _exit(0);
}
