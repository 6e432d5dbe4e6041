/*
 * GF(2) toolkit for 0-db's checksum (CRC-32C, reflected poly 0x82F63B78,
 * init 0, no final XOR -- libzdb/crc32.c:84-110).
 *
 * Because the reference starts from 0 and applies no final XOR
 * (crc32.c:85, :97), the checksum is a pure GF(2)-linear map of the data:
 *   crc(A || B)   = shift(crc(A), |B|) ^ crc(B)
 *   crc(0^k || A) = crc(A)
 * where shift(c, n) advances the register over n zero bytes, i.e. multiplies
 * by x^(8n) mod P.  P has a nonzero constant term, so shift(c, -n) exists.
 * Everything the GPU kernel does rests on these two identities; the tables it
 * reads are built here on the host (see zdbcrc_build_tables).
 */
#ifndef ZDBCRC_GF2_H
#define ZDBCRC_GF2_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZDBCRC_POLY 0x82F63B78u

/* register advanced over n zero bytes (n < 0: the inverse map) */
uint32_t zdbcrc_shift(uint32_t crc, int64_t nbytes);

/* crc(A || B) from crc(A), crc(B), |B| */
uint32_t zdbcrc_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* byte-at-a-time update from an arbitrary register value (table engine) */
uint32_t zdbcrc_update_bytes(uint32_t crc, const uint8_t *p, size_t n);

/* ---- kernel table image (layout shared with crc32_hip.hip) ---------------
 * All tables map a 5-bit slice of their operand to its 32-bit contribution;
 * the operand is the XOR of its slices' contributions (linearity).  32-entry
 * tables of dwords occupy exactly the 32 LDS banks of a ds_read_b32 lane
 * group, so a lookup wave-instruction is conflict-free whatever the data.
 */
#define ZDBCRC_K         4   /* pieces (16 B) per lane per superstep      */
#define ZDBCRC_PCH      26   /* 5-bit slices of a 128-bit piece (25x5+3)  */
#define ZDBCRC_SCH       7   /* 5-bit slices of a 32-bit register (6x5+2) */
#define ZDBCRC_WAVE     64
#define ZDBCRC_RDIG      4   /* radix-256 digits of a piece count (< 2^32) */

/* dword offsets inside the image */
#define ZDBCRC_OFF_T    0                                              /* [K][PCH][32]      */
#define ZDBCRC_OFF_W    (ZDBCRC_OFF_T + ZDBCRC_K * ZDBCRC_PCH * 32)    /* [SCH][32]         */
#define ZDBCRC_OFF_L    (ZDBCRC_OFF_W + ZDBCRC_SCH * 32)               /* [SCH][32][64]     */
#define ZDBCRC_LDS_DW   (ZDBCRC_OFF_L + ZDBCRC_SCH * 32 * ZDBCRC_WAVE) /* end of LDS image  */
#define ZDBCRC_OFF_Z    ZDBCRC_LDS_DW                                  /* [16][SCH][32]     */
#define ZDBCRC_OFF_R    (ZDBCRC_OFF_Z + 16 * ZDBCRC_SCH * 32)          /* [RDIG][256][SCH][32] */
#define ZDBCRC_TABLE_DW (ZDBCRC_OFF_R + ZDBCRC_RDIG * 256 * ZDBCRC_SCH * 32)

/*
 * T[i][c][v] : crc of a 16-byte piece whose only set bits are v << 5c,
 *              then shifted by 1024*(K-1-i) bytes (slot i of a superstep)
 * W[c][v]    : shift(v << 5c, 1024*K)          (register across a superstep)
 * L[c][v][l] : shift(v << 5c, 16*(63-l))       (lane l's final placement)
 * Z[z][c][v] : shift(v << 5c, -z), z = 0..15   (trailing pad removal)
 * R[j][d][c][v] : shift(v << 5c, 16 * d * 256^j) (shift by a piece count,
 *              one radix-256 digit per table: at most 4 dependent rounds)
 */
void zdbcrc_build_tables(uint32_t *image /* ZDBCRC_TABLE_DW dwords */);

#ifdef __cplusplus
}
#endif

#endif
