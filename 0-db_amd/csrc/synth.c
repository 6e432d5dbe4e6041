/*
 * Deterministic synthetic inputs: identical bytes and record
 * sizes on every host, so the GPU box regenerates exactly what the fixtures
 * in this repository were computed on.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void zdb_synth_fill(uint8_t *buf, size_t len, uint64_t seed) {
    size_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t w = mix64(seed + (i / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        for (int k = 0; k < 8; k++)
            buf[i + k] = (uint8_t)(w >> (8 * k));
    }
    if (i < len) {
        uint64_t w = mix64(seed + (i / 8 + 1) * 0x9E3779B97F4A7C15ULL);
        for (int k = 0; i + k < len; k++)
            buf[i + k] = (uint8_t)(w >> (8 * k));
    }
}

size_t zdb_synth_zipf_lengths(uint32_t *lengths, size_t max_n, uint64_t target_bytes, uint64_t seed) {
    double w[15], tot = 0;
    for (int k = 0; k < 15; k++) {
        w[k] = pow((double)(k + 1), -1.1);
        tot += w[k];
    }
    uint64_t state = seed;
    uint64_t total = 0;
    size_t n = 0;
    while (n < max_n && total < target_bytes) {
        state += 0x9E3779B97F4A7C15ULL;
        double u = (double)(mix64(state) >> 11) / 9007199254740992.0 * tot;
        int k = 0;
        for (; k < 14; k++) {
            if (u < w[k])
                break;
            u -= w[k];
        }
        uint64_t lo = (uint64_t)64 << k, hi = (uint64_t)64 << (k + 1);
        state += 0x9E3779B97F4A7C15ULL;
        uint64_t s = lo + mix64(state) % (hi - lo);
        if (s > (1u << 20))
            s = 1u << 20;
        lengths[n++] = (uint32_t)s;
        total += s;
    }
    return n;
}
