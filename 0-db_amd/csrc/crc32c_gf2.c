/*
 * GF(2) toolkit and kernel table image -- see crc32c_gf2.h.
 *
 * Register convention is the reference's reflected one (crc32.c:16-91): bit 31
 * of the register is the coefficient of x^0, and one zero-bit step is
 * r = (r >> 1) ^ (r & 1 ? POLY : 0), i.e. a multiplication by x mod P.
 */
#include "crc32c_gf2.h"

#include <pthread.h>
#include <string.h>

static uint32_t byte_table[256];
static uint32_t xpow2[64];    /* x^(2^k) mod P             */
static uint32_t xinvpow2[64]; /* x^(-(2^k)) mod P          */
static pthread_once_t gf2_once = PTHREAD_ONCE_INIT;

/* a * b mod P, both reflected (bit 31 = x^0) */
static uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    if (a == 0)
        return 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0)
                break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ ZDBCRC_POLY : (b >> 1);
    }
    return p;
}

/* inverse of the one-bit step: recovers r from (r >> 1) ^ (r & 1 ? P : 0).
 * P has bit 31 set and (r >> 1) never does, so bit 31 tells the low bit. */
static uint32_t unstep(uint32_t r) {
    uint32_t lsb = r >> 31;
    return ((r ^ (lsb ? ZDBCRC_POLY : 0)) << 1) | lsb;
}

static void gf2_init(void) {
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++)
            c = (c & 1) ? (c >> 1) ^ ZDBCRC_POLY : (c >> 1);
        byte_table[i] = c;
    }
    xpow2[0] = 1u << 30;             /* x^1  */
    xinvpow2[0] = unstep(1u << 31);  /* x^-1 */
    for (int k = 1; k < 64; k++) {
        xpow2[k] = multmodp(xpow2[k - 1], xpow2[k - 1]);
        xinvpow2[k] = multmodp(xinvpow2[k - 1], xinvpow2[k - 1]);
    }
}

static void gf2_ready(void) { pthread_once(&gf2_once, gf2_init); }

/* x^e mod P (inverse powers when inv) */
static uint32_t xpow(uint64_t e, int inv) {
    const uint32_t *tab = inv ? xinvpow2 : xpow2;
    uint32_t p = 1u << 31; /* x^0 */
    for (int k = 0; e; k++, e >>= 1)
        if (e & 1)
            p = multmodp(tab[k], p);
    return p;
}

uint32_t zdbcrc_shift(uint32_t crc, int64_t nbytes) {
    gf2_ready();
    if (nbytes == 0 || crc == 0)
        return crc;
    if (nbytes > 0)
        return multmodp(xpow((uint64_t)nbytes * 8u, 0), crc);
    return multmodp(xpow((uint64_t)(-nbytes) * 8u, 1), crc);
}

uint32_t zdbcrc_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
    return zdbcrc_shift(crc_a, (int64_t)len_b) ^ crc_b;
}

uint32_t zdbcrc_update_bytes(uint32_t crc, const uint8_t *p, size_t n) {
    gf2_ready();
    for (size_t i = 0; i < n; i++)
        crc = byte_table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return crc;
}

int zdbcrc_window_bit(int j, int t) {
    if (j < 0 || j >= ZDBCRC_PCH || t < 0 || t >= 5)
        return -1;
    if (j < 16) /* A */
        return 32 * (j >> 2) + 8 * (j & 3) + 2 + t;
    if (j < 24) { /* B: u = rotl3(w_a) | rotl5(w_b), byte n, bits [2,7) */
        const int a = j < 20 ? 0 : 2, n = (j - 16) & 3;
        switch (t) {
        case 0: return 32 * a + ((8 * n + 31) & 31);
        case 1: return 32 * a + 8 * n;
        case 2: return 32 * a + 8 * n + 1;
        case 3: return 32 * (a + 1) + 8 * n;
        default: return 32 * (a + 1) + 8 * n + 1;
        }
    }
    /* C: z2 bits [2,6) (j = 24) and [18,22) (j = 25) */
    {
        const int m = 2 * (j - 24); /* byte of w1/w3 behind index bits 0,1 */
        switch (t) {
        case 0: return 32 + 8 * m + 7;
        case 1: return 96 + 8 * m + 7;
        case 2: return 32 + 8 * (m + 1) + 7;
        case 3: return 96 + 8 * (m + 1) + 7;
        default: return -1;
        }
    }
}

/* crc (from 0) of a 16-byte piece whose only set bits are window j's bits selected by v */
static uint32_t piece_window_crc(uint32_t v, int j) {
    uint8_t piece[16];
    memset(piece, 0, sizeof(piece));
    for (int t = 0; t < 5; t++) {
        const int b = zdbcrc_window_bit(j, t);
        if (((v >> t) & 1) && b >= 0)
            piece[b >> 3] |= (uint8_t)(1u << (b & 7));
    }
    return zdbcrc_update_bytes(0, piece, 16);
}

/* register slice v at bit 5c, as a 32-bit value (bits past 31 dropped) */
static uint32_t reg_slice(uint32_t v, int c) {
    return (uint32_t)(((uint64_t)v << (5 * c)) & 0xFFFFFFFFu);
}

/* dst[v * stride] for v < 32 from the images of the 5 unit vectors: every
 * table below is GF(2)-linear in v, so one XOR per entry replaces a multiply */
static void fill_linear(uint32_t *dst, size_t stride, const uint32_t basis[5]) {
    dst[0] = 0;
    for (uint32_t v = 1; v < 32; v++) {
        const int t = __builtin_ctz(v);
        dst[v * stride] = dst[(v & (v - 1)) * stride] ^ basis[t];
    }
}

void zdbcrc_build_tables(uint32_t *img) {
    gf2_ready();
    memset(img, 0, sizeof(uint32_t) * ZDBCRC_TABLE_DW);
    uint32_t b[5];

    for (int i = 0; i < ZDBCRC_K; i++) {
        const uint32_t m = xpow(8 * 1024 * (uint64_t)(ZDBCRC_K - 1 - i), 0);
        for (int c = 0; c < ZDBCRC_PCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, piece_window_crc(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_T + (i * ZDBCRC_PCH + c) * 32, 1, b);
        }
    }

    const uint32_t mw = xpow(8 * 1024 * (uint64_t)ZDBCRC_K, 0);
    for (int c = 0; c < ZDBCRC_SCH; c++) {
        for (int t = 0; t < 5; t++)
            b[t] = multmodp(mw, reg_slice(1u << t, c));
        fill_linear(img + ZDBCRC_OFF_W + c * 32, 1, b);
    }

    for (int l = 0; l < ZDBCRC_WAVE; l++) {
        const uint32_t m = xpow(8 * 16 * (uint64_t)(ZDBCRC_WAVE - 1 - l), 0);
        for (int c = 0; c < ZDBCRC_SCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, reg_slice(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_L + c * 32 * ZDBCRC_WAVE + l, ZDBCRC_WAVE, b);
        }
    }

    for (int z = 0; z < 16; z++) {
        const uint32_t m = xpow(8 * (uint64_t)z, 1);
        for (int c = 0; c < ZDBCRC_SCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, reg_slice(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_Z + (z * ZDBCRC_SCH + c) * 32, 1, b);
        }
    }

    for (int j = 0; j < ZDBCRC_RDIG; j++)
        for (uint32_t d = 0; d < 256; d++) {
            const uint32_t m = xpow((uint64_t)d << (8 * j + 7), 0); /* x^(8 * 16 * d * 256^j) */
            for (int c = 0; c < ZDBCRC_SCH; c++) {
                for (int t = 0; t < 5; t++)
                    b[t] = multmodp(m, reg_slice(1u << t, c));
                fill_linear(img + ZDBCRC_OFF_R + ((j * 256 + d) * ZDBCRC_SCH + c) * 32, 1, b);
            }
        }

    for (int h = 0; h < 4; h++) {
        const uint32_t m = xpow(8 * (uint64_t)h, 0);
        for (int c = 0; c < ZDBCRC_SCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, reg_slice(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_F + (h * ZDBCRC_SCH + c) * 32, 1, b);
        }
    }

    /* packed kernel: rows of 16 lanes, 256 B per slot */
    for (int i = 0; i < ZDBCRC_K; i++) {
        const uint32_t m = xpow(8 * 256 * (uint64_t)(ZDBCRC_K - 1 - i), 0);
        for (int c = 0; c < ZDBCRC_PCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, piece_window_crc(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_TP + (i * ZDBCRC_PCH + c) * 32, 1, b);
        }
    }
    const uint32_t mwp = xpow(8 * 256 * (uint64_t)ZDBCRC_K, 0);
    for (int c = 0; c < ZDBCRC_SCH; c++) {
        for (int t = 0; t < 5; t++)
            b[t] = multmodp(mwp, reg_slice(1u << t, c));
        fill_linear(img + ZDBCRC_OFF_WP + c * 32, 1, b);
    }
    /* other row widths: 8 lanes (128 B per slot), 4 lanes (64 B), 32 lanes (512 B) */
    for (int nr = 0; nr < 3; nr++) {
        const uint64_t slot = nr == 0 ? 128 : nr == 1 ? 64 : 512;
        uint32_t *const tt = img + (nr == 0 ? ZDBCRC_OFF_TE : nr == 1 ? ZDBCRC_OFF_TQ : ZDBCRC_OFF_TT);
        uint32_t *const tw = img + (nr == 0 ? ZDBCRC_OFF_WE : nr == 1 ? ZDBCRC_OFF_WQ : ZDBCRC_OFF_WT);
        for (int i = 0; i < ZDBCRC_K; i++) {
            const uint32_t m = xpow(8 * slot * (uint64_t)(ZDBCRC_K - 1 - i), 0);
            for (int c = 0; c < ZDBCRC_PCH; c++) {
                for (int t = 0; t < 5; t++)
                    b[t] = multmodp(m, piece_window_crc(1u << t, c));
                fill_linear(tt + (i * ZDBCRC_PCH + c) * 32, 1, b);
            }
        }
        const uint32_t mw2 = xpow(8 * slot * (uint64_t)ZDBCRC_K, 0);
        for (int c = 0; c < ZDBCRC_SCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(mw2, reg_slice(1u << t, c));
            fill_linear(tw + c * 32, 1, b);
        }
    }
    for (int l = 0; l < 32; l++) {
        const uint32_t m = xpow(8 * 16 * (uint64_t)(15 - (l & 15)), 0);
        for (int c = 0; c < ZDBCRC_SCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, reg_slice(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_LP + c * 32 * 32 + l, 32, b);
        }
    }
    for (int l = 0; l < 32; l++) {
        const uint32_t m = xpow(8 * 16 * (uint64_t)(31 - l), 0);
        for (int c = 0; c < ZDBCRC_SCH; c++) {
            for (int t = 0; t < 5; t++)
                b[t] = multmodp(m, reg_slice(1u << t, c));
            fill_linear(img + ZDBCRC_OFF_LT + c * 32 * 32 + l, 32, b);
        }
    }
}
