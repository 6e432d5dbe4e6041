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
#define ZDBCRC_PCH      26   /* lookup windows of a 128-bit piece        */
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
#define ZDBCRC_OFF_F    (ZDBCRC_OFF_R + ZDBCRC_RDIG * 256 * ZDBCRC_SCH * 32) /* [4][SCH][32] */
/* packed small-record kernel (crc_packed_kernel): four records per wave, one
 * per row of 16 lanes; its LDS image is the contiguous range [OFF_F, TABLE_DW) */
#define ZDBCRC_OFF_TP   (ZDBCRC_OFF_F + 4 * ZDBCRC_SCH * 32)                /* [K][PCH][32]      */
#define ZDBCRC_OFF_WP   (ZDBCRC_OFF_TP + ZDBCRC_K * ZDBCRC_PCH * 32)        /* [SCH][32]         */
#define ZDBCRC_OFF_LP   (ZDBCRC_OFF_WP + ZDBCRC_SCH * 32)                   /* [SCH][32][32]     */
#define ZDBCRC_PK_LDS_DW (ZDBCRC_OFF_LP + ZDBCRC_SCH * 32 * 32 - ZDBCRC_OFF_F)
/* the same kernel with narrower rows (8 / 4 lanes: 8 / 16 records per wave):
 * its slot and advance tables; F and LP are shared */
#define ZDBCRC_OFF_TE   (ZDBCRC_OFF_LP + ZDBCRC_SCH * 32 * 32)              /* [K][PCH][32] rows of 8 */
#define ZDBCRC_OFF_WE   (ZDBCRC_OFF_TE + ZDBCRC_K * ZDBCRC_PCH * 32)        /* [SCH][32]            */
#define ZDBCRC_OFF_TQ   (ZDBCRC_OFF_WE + ZDBCRC_SCH * 32)                   /* [K][PCH][32] rows of 4 */
#define ZDBCRC_OFF_WQ   (ZDBCRC_OFF_TQ + ZDBCRC_K * ZDBCRC_PCH * 32)        /* [SCH][32]            */
/* rows of 32 lanes (two records per wave): slot, advance and placement tables */
#define ZDBCRC_OFF_TT   (ZDBCRC_OFF_WQ + ZDBCRC_SCH * 32)                   /* [K][PCH][32]         */
#define ZDBCRC_OFF_WT   (ZDBCRC_OFF_TT + ZDBCRC_K * ZDBCRC_PCH * 32)        /* [SCH][32]            */
#define ZDBCRC_OFF_LT   (ZDBCRC_OFF_WT + ZDBCRC_SCH * 32)                   /* [SCH][32][32]        */
#define ZDBCRC_TABLE_DW (ZDBCRC_OFF_LT + ZDBCRC_SCH * 32 * 32)

/*
 * Piece windows.  A 16-byte piece (dwords w0..w3, little endian) is covered
 * by 26 lookup windows chosen so that the kernel extracts most indices with
 * ONE VALU op (an SDWA byte select + AND 0x7C gives bits [8n+2, 8n+7) of a
 * dword already scaled to a dword address):
 *   j  0..15  A: bits [8n+2, 8n+7) of w_k            (k = j/4, n = j%4)
 *   j 16..19  B: byte n of u1 = rotl3(w0) on 0x1C1C1C1C | rotl5(w1) elsewhere
 *   j 20..23  B: byte n of u2, the same from (w2, w3)
 *              -> index bits: w_a bit 8n-1 (mod 32), 8n, 8n+1, w_b bit 8n, 8n+1
 *   j 24..25  C: z = (w1 >> 5) on 0x04040404 | (w3 >> 4) elsewhere,
 *              z2 = rotr6(z) on 0x00300030 | z elsewhere; bits [2,6) and
 *              [18,22) of z2 -> w1 bit 8m+7, w3 bit 8m+7 for m = 2c', 2c'+1
 * zdbcrc_window_bit(j, t) is the piece bit behind index bit t of window j
 * (-1 for the unused 5th bit of the C windows); the tables below are built
 * from it, and the kernel's extraction (crc32_hip.hip piece_contrib) and the
 * CPU model (tests/kernel_model.py) follow the same map.
 */
int zdbcrc_window_bit(int j, int t);

/*
 * T[i][j][v] : crc of a 16-byte piece whose only set bits are those of
 *              window j selected by v, then shifted by 1024*(K-1-i) bytes
 *              (slot i of a superstep)
 * W[c][v]    : shift(v << 5c, 1024*K)          (register across a superstep)
 * L[c][v][l] : shift(v << 5c, 16*(63-l))       (lane l's final placement)
 * Z[z][c][v] : shift(v << 5c, -z), z = 0..15   (trailing pad removal)
 * R[j][d][c][v] : shift(v << 5c, 16 * d * 256^j) (shift by a piece count,
 *              one radix-256 digit per table: at most 4 dependent rounds)
 * F[h][c][v] : shift(v << 5c, h), h = 0..3     (a record-relative grid loaded
 *              from the dword below the record: its last h bytes y are folded
 *              in at the end as crc(X || y) = shift(crc(X) ^ y, h))
 * Packed kernel (a row of 16 lanes walks one record, 256 B per slot, 1 KiB
 * per superstep):
 * TP[i][j][v]: as T, shifted by 256*(K-1-i) bytes
 * WP[c][v]   : shift(v << 5c, 1024)           (row register across a superstep)
 * LP[c][v][l]: shift(v << 5c, 16*(15-(l&15))), l = lane & 31 (lane l's
 *              placement in its row; 32 columns so that bank = lane & 31)
 * Rows of RW = 8 / 4 lanes (16 RW bytes per slot, 64 RW per superstep):
 * TE, TQ[i][j][v]: as T, shifted by 16 RW (K-1-i) bytes
 * WE, WQ[c][v]   : shift(v << 5c, 64 RW)
 * (placement by 16 (RW-1-l) bytes reads LP's column 16 - RW + l)
 * Rows of 32 lanes: TT (512 B per slot), WT (2 KiB), and
 * LT[c][v][l]    : shift(v << 5c, 16*(31-l)), l = lane & 31
 */
void zdbcrc_build_tables(uint32_t *image /* ZDBCRC_TABLE_DW dwords */);

#ifdef __cplusplus
}
#endif

#endif
