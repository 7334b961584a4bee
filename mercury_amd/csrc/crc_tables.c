/*
 * crc_tables.c -- host-side GF(2) operator algebra and the lookup-table packs
 * the CDNA4 batch kernels stage into LDS (layout: crc_gpu_layout.h).
 *
 * A CRC register update is linear over GF(2), so every "advance by n bytes"
 * (Z^n) and its inverse is a W x W bit matrix.  Tables are those matrices
 * evaluated on byte/nibble basis values, so one table lookup applies a
 * fixed operator to 8 (or 4) bits of the register at once.
 */
#include "crc_gpu_layout.h"

#include <string.h>

static uint64_t
wmask(int w)
{
    return w == 64 ? ~0ULL : ((1ULL << w) - 1);
}

/* One zero byte through the reflected register. */
static uint64_t
zero_byte(const crc_rmodel_t *m, uint64_t r)
{
    int k;

    for (k = 0; k < 8; k++)
        r = (r & 1) ? ((r >> 1) ^ m->rpoly) : (r >> 1);
    return r & wmask(m->width);
}

/* Bit reversal within each byte of a w-bit value (the R of crc_rmodel_t). */
uint64_t
crc_rev_bytes(int w, uint64_t v)
{
    uint64_t r = 0;
    int b, k;

    for (b = 0; b < w / 8; b++)
        for (k = 0; k < 8; k++)
            if ((v >> (8 * b + k)) & 1)
                r |= 1ULL << (8 * b + 7 - k);
    return r;
}

void
crc_op_zero_byte(const crc_rmodel_t *m, uint64_t *col)
{
    int i;

    for (i = 0; i < m->width; i++)
        col[i] = m->msb ? crc_rev_bytes(m->width, zero_byte(m, 1ULL << ((i & ~7) | (7 - (i & 7)))))
                        : zero_byte(m, 1ULL << i);
}

void
crc_op_identity(int w, uint64_t *col)
{
    int i;

    for (i = 0; i < w; i++)
        col[i] = 1ULL << i;
}

uint64_t
crc_op_apply(int w, const uint64_t *col, uint64_t x)
{
    uint64_t r = 0;
    int i;

    for (i = 0; i < w; i++)
        if ((x >> i) & 1)
            r ^= col[i];
    return r;
}

void
crc_op_mul(int w, const uint64_t *a, const uint64_t *b, uint64_t *out)
{
    uint64_t tmp[64];
    int i;

    for (i = 0; i < w; i++)
        tmp[i] = crc_op_apply(w, a, b[i]);
    memcpy(out, tmp, sizeof(uint64_t) * (size_t) w);
}

void
crc_op_pow(int w, const uint64_t *a, uint64_t n, uint64_t *out)
{
    uint64_t base[64], acc[64];

    memcpy(base, a, sizeof(uint64_t) * (size_t) w);
    crc_op_identity(w, acc);
    while (n) {
        if (n & 1)
            crc_op_mul(w, base, acc, acc);
        crc_op_mul(w, base, base, base);
        n >>= 1;
    }
    memcpy(out, acc, sizeof(uint64_t) * (size_t) w);
}

/* Gauss-Jordan over GF(2).  Returns 0 on success, -1 if singular. */
int
crc_op_inv(int w, const uint64_t *a, uint64_t *out)
{
    uint64_t row[64], inv[64];
    int r, c, i;

    /* row r of A: bit i = bit r of column i */
    for (r = 0; r < w; r++) {
        row[r] = 0;
        for (i = 0; i < w; i++)
            if ((a[i] >> r) & 1)
                row[r] |= 1ULL << i;
        inv[r] = 1ULL << r;
    }
    for (c = 0; c < w; c++) {
        int piv = -1;
        for (r = c; r < w; r++)
            if ((row[r] >> c) & 1) {
                piv = r;
                break;
            }
        if (piv < 0)
            return -1;
        if (piv != c) {
            uint64_t t = row[c];
            row[c] = row[piv];
            row[piv] = t;
            t = inv[c];
            inv[c] = inv[piv];
            inv[piv] = t;
        }
        for (r = 0; r < w; r++)
            if (r != c && ((row[r] >> c) & 1)) {
                row[r] ^= row[c];
                inv[r] ^= inv[c];
            }
    }
    /* inv holds rows of A^-1; convert to columns */
    for (i = 0; i < w; i++) {
        out[i] = 0;
        for (r = 0; r < w; r++)
            if ((inv[r] >> i) & 1)
                out[i] |= 1ULL << r;
    }
    return 0;
}

int
crc_op_zpow(const crc_rmodel_t *m, int64_t n, uint64_t *out)
{
    uint64_t z[64];

    crc_op_zero_byte(m, z);
    if (n < 0) {
        uint64_t zi[64];
        if (crc_op_inv(m->width, z, zi) != 0)
            return -1;
        crc_op_pow(m->width, zi, (uint64_t) (-n), out);
    } else {
        crc_op_pow(m->width, z, (uint64_t) n, out);
    }
    return 0;
}

/* ---------------------------------------------------------------------- */

static int
fill_nibble_op32(const crc_rmodel_t *m, int64_t n, uint32_t tab[8][16])
{
    uint64_t op[64];
    int h, v;

    if (crc_op_zpow(m, n, op) != 0)
        return -1;
    for (h = 0; h < 8; h++)
        for (v = 0; v < 16; v++)
            tab[h][v] = (uint32_t) crc_op_apply(32, op, (uint64_t) v << (4 * h));
    return 0;
}

static int
fill_nibble_op64(const crc_rmodel_t *m, int64_t n, uint64_t tab[16][16])
{
    uint64_t op[64];
    int h, v;

    if (crc_op_zpow(m, n, op) != 0)
        return -1;
    for (h = 0; h < 16; h++)
        for (v = 0; v < 16; v++)
            tab[h][v] = crc_op_apply(64, op, (uint64_t) v << (4 * h));
    return 0;
}

int
crc32_gpu_pack_build(const crc_rmodel_t *m, int log2g, crc32_gpu_pack_t *out)
{
    const int64_t step = 16LL << log2g;
    uint64_t op[64];
    int p, b, k, t, o = 0;

    if (!m || !out || m->width != 32 || log2g < 0 || log2g > CRC_GPU_MAX_LOG2G)
        return -1;
    memset(out, 0, sizeof(*out));
    for (p = 0; p < 4; p++) {
        if (crc_op_zpow(m, step - p, op) != 0)
            return -1;
        for (b = 0; b < 256; b++)
            out->main[p][b] = (uint32_t) crc_op_apply(32, op, (uint64_t) b);
    }
    if (fill_nibble_op32(m, -4, out->ops[o++]) || fill_nibble_op32(m, -8, out->ops[o++]))
        return -1;
    for (k = 0; k < log2g; k++)
        if (fill_nibble_op32(m, -(16LL << k), out->ops[o++]))
            return -1;
    for (t = 0; t < CRC_GPU_NTAIL; t++)
        if (fill_nibble_op32(m, -(int64_t) t, out->ops[o++]))
            return -1;
    for (k = 0; k < 4; k++) {
        if (crc_op_zpow(m, k, op) != 0)
            return -1;
        out->zinit[k] = (uint32_t) crc_op_apply(32, op, m->rinit);
    }
    if (log2g == 6) {
        int lvl, i, h, v;
        for (lvl = 0; lvl < 2; lvl++)
            for (i = 0; i < 8; i++) {
                if (crc_op_zpow(m, -(int64_t) i * (lvl ? 128 : 16), op) != 0)
                    return -1;
                for (h = 0; h < 8; h++)
                    for (v = 0; v < 16; v++)
                        out->lv[lvl][h][v][i] = (uint32_t) crc_op_apply(32, op, (uint64_t) v << (4 * h));
            }
    }
    out->xorout = (uint32_t) m->xorout;
    out->init = (uint32_t) m->rinit;
    out->log2g = (uint32_t) log2g;
    out->nops = (uint32_t) o;
    return 0;
}

int
crc64_gpu_pack_build(const crc_rmodel_t *m, int log2g, crc64_gpu_pack_t *out)
{
    const int64_t step = 16LL << log2g;
    uint64_t op[64];
    int p, h, v, k, t, o = 0;

    if (!m || !out || m->width != 64 || log2g < 0 || log2g > CRC_GPU_MAX_LOG2G)
        return -1;
    memset(out, 0, sizeof(*out));
    for (p = 0; p < 8; p++) {
        if (crc_op_zpow(m, step - p, op) != 0)
            return -1;
        for (h = 0; h < 2; h++)
            for (v = 0; v < 16; v++)
                out->main[2 * p + h][v] = crc_op_apply(64, op, (uint64_t) v << (4 * h));
    }
    if (crc_op_zpow(m, step, op) != 0)
        return -1;
    for (p = 0; p < 8; p++)
        for (v = 0; v < 32; v++)
            out->f5[p][v] = crc_op_apply(64, op, (uint64_t) v << (8 * p + 3));
    for (p = 0; p < 4; p++)
        for (v = 0; v < 64; v++)
            out->f6[p][v] = crc_op_apply(64, op, ((uint64_t) (v & 7) << (8 * p)) |
                                                     ((uint64_t) (v >> 3) << (8 * p + 32)));
    if (fill_nibble_op64(m, -8, out->ops[o++]))
        return -1;
    for (k = 0; k < log2g; k++)
        if (fill_nibble_op64(m, -(16LL << k), out->ops[o++]))
            return -1;
    for (t = 0; t < CRC_GPU_NTAIL; t++)
        if (fill_nibble_op64(m, -(int64_t) t, out->ops[o++]))
            return -1;
    for (k = 0; k < 8; k++) {
        if (crc_op_zpow(m, k, op) != 0)
            return -1;
        out->zinit[k] = crc_op_apply(64, op, m->rinit);
    }
    out->xorout = m->xorout;
    out->init = m->rinit;
    out->log2g = (uint32_t) log2g;
    out->nops = (uint32_t) o;
    return 0;
}

/* Z^(d * 16^k) for d = 1..15, k < CRC_SHIFT_DIGITS, by repeated products of
 * Z^(16^k) (no per-entry matrix powers). */
static int
shift_ops(const crc_rmodel_t *m, void (*emit)(void *, int, int, const uint64_t *), void *out)
{
    uint64_t base[64], cur[64], nxt[64];
    int k, d, w = m->width;

    crc_op_zero_byte(m, base); /* Z^(16^0) */
    for (k = 0; k < CRC_SHIFT_DIGITS; k++) {
        memcpy(cur, base, sizeof(cur));
        for (d = 1; d <= 15; d++) {
            emit(out, k, d, cur);
            crc_op_mul(w, cur, base, nxt);
            memcpy(cur, nxt, sizeof(cur));
        }
        memcpy(base, cur, sizeof(base)); /* Z^(16^(k+1)) = Z^(16 * 16^k) */
    }
    return 0;
}

static void
emit32(void *o, int k, int d, const uint64_t *op)
{
    crc32_shift_pack_t *out = (crc32_shift_pack_t *) o;
    int h, v;
    for (h = 0; h < 8; h++)
        for (v = 0; v < 16; v++)
            out->op[k][d - 1][h][v] = (uint32_t) crc_op_apply(32, op, (uint64_t) v << (4 * h));
}

static void
emit64(void *o, int k, int d, const uint64_t *op)
{
    crc64_shift_pack_t *out = (crc64_shift_pack_t *) o;
    int h, v;
    for (h = 0; h < 16; h++)
        for (v = 0; v < 16; v++)
            out->op[k][d - 1][h][v] = crc_op_apply(64, op, (uint64_t) v << (4 * h));
}

int
crc32_shift_pack_build(const crc_rmodel_t *m, crc32_shift_pack_t *out)
{
    if (!m || !out || m->width != 32)
        return -1;
    return shift_ops(m, emit32, out);
}

int
crc64_shift_pack_build(const crc_rmodel_t *m, crc64_shift_pack_t *out)
{
    if (!m || !out || m->width != 64)
        return -1;
    return shift_ops(m, emit64, out);
}
