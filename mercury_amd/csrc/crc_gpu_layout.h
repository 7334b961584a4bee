/*
 * crc_gpu_layout.h -- table packs shared by the host table generator
 * (crc_tables.c) and the CDNA4 kernels (mchecksum_gpu.hip).
 *
 * Notation (reflected CRC of width W, register r):
 *   Z(r)   = one zero byte through the register  = (r >> 8) ^ T0[r & 0xFF]
 *   F      = Z^(16G): advance by one step block of 16*G bytes, where G is
 *            the number of lanes that cooperate on one payload and every
 *            lane loads 16 contiguous bytes per step (one dwordx4).
 * A lane keeps one independent sub-stream per W-bit word of its 16-byte
 * piece (4 for CRC-32C, 2 for CRC-64); sub-stream q = (lane * 16 + word
 * offset) / (W/8) advances by s <- F(s ^ w) every step (uniform stride, so
 * the stride is folded into the lookup tables).  At the end the payload's
 * register is  XOR_q Z^(-q*W/8)(S_q)  (tree combine, ops below), then
 * Z^(-t) undoes the t trailing pad bytes of the 16-byte-aligned window.
 */
#ifndef CRC_GPU_LAYOUT_H
#define CRC_GPU_LAYOUT_H

#include <stdint.h>

#define CRC_GPU_MAX_LOG2G 6 /* G in {1,2,...,64} lanes per payload        */
#define CRC_GPU_NTAIL 16    /* Z^(-t), t = 0..15                           */

/* ---- CRC-32C (W = 32): byte tables, 4 per step, 32-bank replicated in LDS */
/* ops: [0] Z^-4, [1] Z^-8, [2+k] Z^-(16*2^k) (k < log2G), then the tails.   */
#define CRC32_NOPS_MAX (2 + CRC_GPU_MAX_LOG2G + CRC_GPU_NTAIL)
typedef struct {
    uint32_t main[4][256];            /* main[p][b] = Z^(16G-p)(b)          */
    uint32_t ops[CRC32_NOPS_MAX][8][16]; /* ops[o][h][v] = M_o(v << 4h)     */
    uint32_t zinit[4];                /* Z^n(init), n = 0..3 (n < 4 payloads) */
    uint32_t xorout;
    uint32_t init;
    uint32_t log2g;
    uint32_t nops;
    /* Two-level lane combine (log2g == 6 only): XOR_l Z^(-16 l)(v_l) over the
     * 64 lanes as Z^(-128 a) o Z^(-16 b), l = 8a + b -- one lane-dependent
     * operator per level instead of six butterfly levels.  Interleaved
     * [level][h][v][i] = M_{level,i}(v << 4h), M_{0,i} = Z^(-16 i),
     * M_{1,i} = Z^(-128 i), so lanes with different operators i read
     * different LDS banks.                                                   */
    uint32_t lv[2][8][16][8];
} crc32_gpu_pack_t;

/* ---- CRC-64 (W = 64): nibble tables, 16 per step, 32-bank replicated ---- */
/* ops: [0] Z^-8, [1+k] Z^-(16*2^k), then the tails.                         */
#define CRC64_NOPS_MAX (1 + CRC_GPU_MAX_LOG2G + CRC_GPU_NTAIL)
typedef struct {
    uint64_t main[16][16];            /* main[2p+h][v] = Z^(16G-p)(v << 4h) */
    uint64_t ops[CRC64_NOPS_MAX][16][16]; /* ops[o][h][v] = M_o(v << 4h)    */
    uint64_t zinit[8];                /* Z^n(init), n = 0..7                */
    uint64_t xorout;
    uint64_t init;
    uint32_t log2g;
    uint32_t nops;
    /* Fewer-lookup form of the same step fold F = Z^(16G) (12 lookups per
     * 64-bit word instead of 16): bits 3..7 of byte j index a 32-entry table,
     * bits 0..2 of bytes i and i+4 together a 64-entry table.              */
    uint64_t f5[8][32];               /* f5[j][v] = F(v << (8j + 3))         */
    uint64_t f6[4][64];               /* f6[i][v] = F((v&7) << 8i | (v>>3) << (8i+32)) */
} crc64_gpu_pack_t;

/* ---- register shifts Z^n for 0 <= n < 2^48 (scatter-gather combine) ----- */
/* Z^n = prod over base-16 digits d_k of n of Z^(d_k * 16^k): at most 12
 * operator applications.  op[k][d-1] = nibble tables of Z^(d * 16^k).       */
#define CRC_SHIFT_DIGITS 12
typedef struct {
    uint32_t op[CRC_SHIFT_DIGITS][15][8][16];
} crc32_shift_pack_t;
typedef struct {
    uint64_t op[CRC_SHIFT_DIGITS][15][16][16];
} crc64_shift_pack_t;

#ifdef __cplusplus
extern "C" {
#endif

/* Reflected CRC model as the kernels see it.  msb = 1: an MSB-first model
 * (refin = refout = false), run as the reflected model of the same polynomial
 * over bit-reversed bytes -- with every operator conjugated by R, the bit
 * reversal within each byte of the register (R o Z o R), so the kernels XOR
 * the data bytes in unchanged; rinit and xorout are then given in that R
 * domain, and the kernel's output v is the CRC byte-swapped (reflect_W(R(v))
 * = bswap(v)): the host swaps the outputs after the launch. */
typedef struct {
    int width;        /* 32 or 64 */
    uint64_t rpoly;   /* reflected polynomial */
    uint64_t rinit;   /* initial register in reflected form */
    uint64_t xorout;
    int msb;
} crc_rmodel_t;

/* Host generators (crc_tables.c). Return 0 on success. */
uint64_t crc_rev_bytes(int w, uint64_t v);
int crc32_gpu_pack_build(const crc_rmodel_t *m, int log2g, crc32_gpu_pack_t *out);
int crc64_gpu_pack_build(const crc_rmodel_t *m, int log2g, crc64_gpu_pack_t *out);
int crc32_shift_pack_build(const crc_rmodel_t *m, crc32_shift_pack_t *out);
int crc64_shift_pack_build(const crc_rmodel_t *m, crc64_shift_pack_t *out);

/* GF(2) operator helpers (W x W bit matrices stored as W column words). */
void crc_op_zero_byte(const crc_rmodel_t *m, uint64_t *col);
void crc_op_identity(int w, uint64_t *col);
uint64_t crc_op_apply(int w, const uint64_t *col, uint64_t x);
void crc_op_mul(int w, const uint64_t *a, const uint64_t *b, uint64_t *out); /* out = a o b */
void crc_op_pow(int w, const uint64_t *a, uint64_t n, uint64_t *out);
int crc_op_inv(int w, const uint64_t *a, uint64_t *out);
/* Z^n for signed n (negative = inverse). */
int crc_op_zpow(const crc_rmodel_t *m, int64_t n, uint64_t *out);

#ifdef __cplusplus
}
#endif
#endif
