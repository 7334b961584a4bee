/*
 * crc_oracle.c -- CPU restatement of mchecksum's CRC methods (TEST ONLY).
 * See crc_oracle.h for what is restated, from where, and the pinning status.
 *
 * Call sites whose semantics this follows:
 *   src/mercury_proc.c:387-406  hg_proc_checksum_update: update(data, n) on
 *                               exactly the n serialized bytes, in order
 *   src/mercury_proc.c:358-384  hg_proc_flush: get(..., MCHECKSUM_FINALIZE)
 *   src/mercury_proc.h:124-143,162-181  HG_PROC_TYPE/BYTES: memcpy then update
 * so the checksum of an encoded proc buffer is the CRC of its bytes
 * buf[0:size_used), which is what these functions compute.
 */
#define _GNU_SOURCE
#include "crc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static const oracle_model_t g_models[] = {
    /* name              width poly                   refin refout init                   xorout                 check */
    {"crc32c",              32, 0x1EDC6F41ULL,          1, 1, 0xFFFFFFFFULL,          0xFFFFFFFFULL,          0xE3069283ULL},
    {"crc32",               32, 0x04C11DB7ULL,          1, 1, 0xFFFFFFFFULL,          0xFFFFFFFFULL,          0xCBF43926ULL},
    {"crc64-xz",            64, 0x42F0E1EBA9EA3693ULL,  1, 1, ~0ULL,                  ~0ULL,                  0x995DC9BBDF1939FAULL},
    {"crc64-ecma182",       64, 0x42F0E1EBA9EA3693ULL,  0, 0, 0ULL,                   0ULL,                   0x6C40DF5F0B497347ULL},
    {"crc64-go-iso",        64, 0x000000000000001BULL,  1, 1, ~0ULL,                  ~0ULL,                  0xB90956C775A41001ULL},
    {"crc64-jones",         64, 0xAD93D23594C935A9ULL,  1, 1, 0ULL,                   0ULL,                   0xE9C6D914C4B8D9CAULL},
    {"crc16-arc",           16, 0x8005ULL,              1, 1, 0ULL,                   0ULL,                   0xBB3DULL},
    {"crc16-ibm-3740",      16, 0x1021ULL,              0, 0, 0xFFFFULL,              0ULL,                   0x29B1ULL},
    {"crc16-xmodem",        16, 0x1021ULL,              0, 0, 0ULL,                   0ULL,                   0x31C3ULL},
    {"crc16-kermit",        16, 0x1021ULL,              1, 1, 0ULL,                   0ULL,                   0x2189ULL},
    {"crc16-umts",          16, 0x8005ULL,              0, 0, 0ULL,                   0ULL,                   0xFEE8ULL},
    {"crc16-t10-dif",       16, 0x8BB7ULL,              0, 0, 0ULL,                   0ULL,                   0xD0DBULL},
    {NULL, 0, 0, 0, 0, 0, 0, 0},
};

const oracle_model_t *
oracle_models(void)
{
    return g_models;
}

const oracle_model_t *
oracle_model_by_name(const char *name)
{
    const oracle_model_t *m;

    if (!name)
        return NULL;
    /* mchecksum method names map onto the default variants. */
    if (strcmp(name, "crc64") == 0)
        name = "crc64-xz";
    else if (strcmp(name, "crc16") == 0)
        name = "crc16-t10-dif";
    for (m = g_models; m->name; m++)
        if (strcmp(m->name, name) == 0)
            return m;
    return NULL;
}

static uint64_t
width_mask(int width)
{
    return width == 64 ? ~0ULL : ((1ULL << width) - 1);
}

static uint64_t
reflect_bits(uint64_t v, int nbits)
{
    uint64_t r = 0;
    int i;

    for (i = 0; i < nbits; i++)
        if (v & (1ULL << i))
            r |= 1ULL << (nbits - 1 - i);
    return r;
}

/* ---------------------------------------------------------------------- */
/* Bitwise: the literal Rocksoft definition (register in direct form).     */
/* ---------------------------------------------------------------------- */

uint64_t
oracle_reg_init(const oracle_model_t *m)
{
    return m->init & width_mask(m->width);
}

uint64_t
oracle_reg_update(const oracle_model_t *m, uint64_t reg, const void *data, size_t n)
{
    const uint8_t *d = (const uint8_t *) data;
    const uint64_t mask = width_mask(m->width);
    const uint64_t top = 1ULL << (m->width - 1);
    size_t i;
    int k;

    for (i = 0; i < n; i++) {
        uint8_t b = m->refin ? (uint8_t) reflect_bits(d[i], 8) : d[i];
        reg ^= (uint64_t) b << (m->width - 8);
        for (k = 0; k < 8; k++)
            reg = (reg & top) ? ((reg << 1) ^ m->poly) : (reg << 1);
        reg &= mask;
    }
    return reg;
}

uint64_t
oracle_reg_final(const oracle_model_t *m, uint64_t reg)
{
    if (m->refout)
        reg = reflect_bits(reg, m->width);
    return (reg ^ m->xorout) & width_mask(m->width);
}

uint64_t
oracle_crc_bitwise(const oracle_model_t *m, const void *data, size_t n)
{
    return oracle_reg_final(m, oracle_reg_update(m, oracle_reg_init(m), data, n));
}

/* ---------------------------------------------------------------------- */
/* Sarwate byte table, built from the bitwise model.                       */
/* ---------------------------------------------------------------------- */

#define MAX_TABLES 16
static struct {
    const oracle_model_t *m;
    uint64_t t[256];
    int reflected;
} g_tables[MAX_TABLES];
static int g_ntables;
static pthread_mutex_t g_table_lock = PTHREAD_MUTEX_INITIALIZER;

static const uint64_t *
table_for(const oracle_model_t *m, int *reflected)
{
    int i;
    const uint64_t *t = NULL;

    pthread_mutex_lock(&g_table_lock);
    for (i = 0; i < g_ntables; i++)
        if (g_tables[i].m == m) {
            t = g_tables[i].t;
            *reflected = g_tables[i].reflected;
            break;
        }
    if (!t && g_ntables < MAX_TABLES) {
        /* A reflected model (refin == refout) runs on the reflected register
         * with the reflected polynomial; table[b] = register after feeding
         * byte b into a zero register.  A direct model runs MSB-first. */
        int refl = m->refin && m->refout;
        uint64_t *tt = g_tables[g_ntables].t;
        uint64_t mask = width_mask(m->width);
        int b, k;

        for (b = 0; b < 256; b++) {
            if (refl) {
                uint64_t rp = reflect_bits(m->poly, m->width);
                uint64_t r = (uint64_t) b;
                for (k = 0; k < 8; k++)
                    r = (r & 1) ? ((r >> 1) ^ rp) : (r >> 1);
                tt[b] = r & mask;
            } else {
                uint64_t top = 1ULL << (m->width - 1);
                uint64_t r = (uint64_t) b << (m->width - 8);
                for (k = 0; k < 8; k++)
                    r = (r & top) ? ((r << 1) ^ m->poly) : (r << 1);
                tt[b] = r & mask;
            }
        }
        g_tables[g_ntables].m = m;
        g_tables[g_ntables].reflected = refl;
        t = tt;
        *reflected = refl;
        g_ntables++;
    }
    pthread_mutex_unlock(&g_table_lock);
    return t;
}

uint64_t
oracle_crc_table(const oracle_model_t *m, const void *data, size_t n)
{
    const uint8_t *d = (const uint8_t *) data;
    const uint64_t mask = width_mask(m->width);
    int refl = 0;
    const uint64_t *t = table_for(m, &refl);
    uint64_t reg;
    size_t i;

    if (!t || (m->refin != m->refout))
        return oracle_crc_bitwise(m, data, n);
    if (refl) {
        reg = reflect_bits(m->init & mask, m->width);
        for (i = 0; i < n; i++)
            reg = (reg >> 8) ^ t[(reg ^ d[i]) & 0xFF];
        /* reg is already the reflected register == refout form */
        return (reg ^ m->xorout) & mask;
    }
    reg = m->init & mask;
    for (i = 0; i < n; i++)
        reg = ((reg << 8) ^ t[((reg >> (m->width - 8)) ^ d[i]) & 0xFF]) & mask;
    return (reg ^ m->xorout) & mask;
}

/* ---------------------------------------------------------------------- */
/* Slicing-by-8 for reflected models (the CPU baseline's table path): eight */
/* tables T_k[b] = the Sarwate table advanced by k more zero bytes, so one  */
/* 8-byte step costs 8 lookups instead of 8 dependent ones.  Checked        */
/* against the bitwise model in oracle_selftest.c and tests/test_oracle.py. */
/* ---------------------------------------------------------------------- */

#define MAX_SLICE 16
static struct {
    const oracle_model_t *m;
    uint64_t t[8][256];
} g_slice[MAX_SLICE];
static int g_nslice;

static const uint64_t (*slice_for(const oracle_model_t *m))[256]
{
    int i, refl = 0, b, k;
    const uint64_t (*r)[256] = NULL;
    const uint64_t *t = table_for(m, &refl);

    if (!t || !refl)
        return NULL;
    pthread_mutex_lock(&g_table_lock);
    for (i = 0; i < g_nslice; i++)
        if (g_slice[i].m == m)
            r = (const uint64_t (*)[256]) g_slice[i].t;
    if (!r && g_nslice < MAX_SLICE) {
        uint64_t (*tt)[256] = g_slice[g_nslice].t;
        for (b = 0; b < 256; b++)
            tt[0][b] = t[b];
        for (k = 1; k < 8; k++)
            for (b = 0; b < 256; b++)
                tt[k][b] = (tt[k - 1][b] >> 8) ^ t[tt[k - 1][b] & 0xFF];
        g_slice[g_nslice].m = m;
        r = (const uint64_t (*)[256]) tt;
        g_nslice++;
    }
    pthread_mutex_unlock(&g_table_lock);
    return r;
}

uint64_t
oracle_crc_slice8(const oracle_model_t *m, const void *data, size_t n)
{
    const uint8_t *d = (const uint8_t *) data;
    const uint64_t mask = width_mask(m->width);
    const uint64_t (*t)[256] = slice_for(m);
    uint64_t reg;

    if (!t || m->refin != m->refout)
        return oracle_crc_table(m, data, n);
    reg = reflect_bits(m->init & mask, m->width);
    while (n >= 8) {
        uint64_t x;
        memcpy(&x, d, 8); /* little-endian host */
        x ^= reg;
        reg = t[7][x & 0xFF] ^ t[6][(x >> 8) & 0xFF] ^ t[5][(x >> 16) & 0xFF] ^ t[4][(x >> 24) & 0xFF] ^
              t[3][(x >> 32) & 0xFF] ^ t[2][(x >> 40) & 0xFF] ^ t[1][(x >> 48) & 0xFF] ^ t[0][x >> 56];
        d += 8;
        n -= 8;
    }
    while (n--)
        reg = (reg >> 8) ^ t[0][(reg ^ *d++) & 0xFF];
    return (reg ^ m->xorout) & mask;
}

/* ---------------------------------------------------------------------- */
/* Hardware oracle: SSE4.2 crc32 (Castagnoli polynomial by definition).    */
/* ---------------------------------------------------------------------- */

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) static uint32_t
crc32c_sse42_impl(const uint8_t *d, size_t n)
{
    uint64_t c = 0xFFFFFFFFu;

    while (n && ((uintptr_t) d & 7)) {
        c = __builtin_ia32_crc32qi((uint32_t) c, *d++);
        n--;
    }
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, d, 8);
        c = __builtin_ia32_crc32di(c, w);
        d += 8;
        n -= 8;
    }
    while (n--) {
        c = __builtin_ia32_crc32qi((uint32_t) c, *d++);
    }
    return (uint32_t) c ^ 0xFFFFFFFFu;
}
#endif

uint32_t
oracle_crc32c_sse42(const void *data, size_t n, int *ok)
{
#if defined(__x86_64__)
    __builtin_cpu_init();
    if (__builtin_cpu_supports("sse4.2")) {
        if (ok)
            *ok = 1;
        return crc32c_sse42_impl((const uint8_t *) data, n);
    }
#endif
    if (ok)
        *ok = 0;
    (void) data;
    (void) n;
    return 0;
}

/* ---------------------------------------------------------------------- */
/* Synthetic data.                                                         */
/* ---------------------------------------------------------------------- */

uint64_t
oracle_splitmix64(uint64_t x)
{
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void
oracle_fill_splitmix(void *dst, size_t nbytes, uint64_t seed, uint64_t first_word)
{
    uint8_t *p = (uint8_t *) dst;
    size_t nw = nbytes / 8, i;

    for (i = 0; i < nw; i++) {
        uint64_t w = oracle_splitmix64(seed ^ (first_word + i));
        memcpy(p + 8 * i, &w, 8); /* little-endian host */
    }
    if (nbytes & 7) {
        uint64_t w = oracle_splitmix64(seed ^ (first_word + nw));
        memcpy(p + 8 * nw, &w, nbytes & 7);
    }
}

void
oracle_varlen_offsets(uint64_t seed, size_t count, uint64_t min_len,
    uint64_t max_len, uint64_t *offsets)
{
    uint64_t span = max_len - min_len + 1, lseed = seed ^ ORACLE_LEN_SALT;
    size_t i;

    offsets[0] = 0;
    for (i = 0; i < count; i++)
        offsets[i + 1] = offsets[i] + min_len + oracle_splitmix64(lseed ^ i) % span;
}

/* ---------------------------------------------------------------------- */
/* Batches (pthreads over payloads).                                       */
/* ---------------------------------------------------------------------- */

static uint64_t
one_crc(const oracle_model_t *m, int variant, const void *d, size_t n)
{
    switch (variant) {
        case 1: {
            int ok = 0;
            uint32_t c = oracle_crc32c_sse42(d, n, &ok);
            return ok ? c : oracle_crc_table(m, d, n);
        }
        case 2:
            return oracle_crc_bitwise(m, d, n);
        case 3:
            return oracle_crc_slice8(m, d, n);
        default:
            return oracle_crc_table(m, d, n);
    }
}

struct batch_job {
    const oracle_model_t *m;
    int variant;
    const uint8_t *base;
    size_t stride, len;
    const uint64_t *offsets;
    uint64_t seed; /* splitmix-generated mode when gen != 0 */
    int gen;
    size_t first, count;
    uint64_t *out;
    int tid, nthreads;
};

static void *
batch_worker(void *arg)
{
    struct batch_job *j = (struct batch_job *) arg;
    size_t lo = j->count * (size_t) j->tid / (size_t) j->nthreads;
    size_t hi = j->count * (size_t) (j->tid + 1) / (size_t) j->nthreads;
    uint8_t *tmp = NULL;
    size_t i;

    if (j->gen) {
        tmp = (uint8_t *) malloc(j->len + 16);
        if (!tmp)
            return (void *) 1;
    }
    for (i = lo; i < hi; i++) {
        size_t idx = j->first + i;
        if (j->gen) {
            uint64_t start = (uint64_t) idx * j->stride;
            uint64_t w0 = start / 8, skip = start % 8;
            oracle_fill_splitmix(tmp, j->len + skip, j->seed, w0);
            j->out[i] = one_crc(j->m, j->variant, tmp + skip, j->len);
        } else if (j->offsets) {
            j->out[i] = one_crc(j->m, j->variant, j->base + j->offsets[idx],
                (size_t) (j->offsets[idx + 1] - j->offsets[idx]));
        } else {
            j->out[i] = one_crc(j->m, j->variant, j->base + idx * j->stride, j->len);
        }
    }
    free(tmp);
    return NULL;
}

static int
run_batch(struct batch_job *proto, int nthreads)
{
    pthread_t th[256];
    struct batch_job jobs[256];
    int t, rc = 0;

    if (nthreads <= 0)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    for (t = 0; t < nthreads; t++) {
        jobs[t] = *proto;
        jobs[t].tid = t;
        jobs[t].nthreads = nthreads;
    }
    if (nthreads == 1)
        return batch_worker(&jobs[0]) ? -1 : 0;
    for (t = 0; t < nthreads; t++)
        if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0)
            return -1;
    for (t = 0; t < nthreads; t++) {
        void *r = NULL;
        pthread_join(th[t], &r);
        if (r)
            rc = -1;
    }
    return rc;
}

int
oracle_batch_fixed(const oracle_model_t *m, int variant, const void *base,
    size_t stride, size_t len, size_t count, uint64_t *out, int nthreads)
{
    struct batch_job j;

    if (!m || (!base && count) || (!out && count))
        return -1;
    memset(&j, 0, sizeof(j));
    j.m = m;
    j.variant = variant;
    j.base = (const uint8_t *) base;
    j.stride = stride;
    j.len = len;
    j.count = count;
    j.out = out;
    return run_batch(&j, nthreads);
}

int
oracle_batch_offsets(const oracle_model_t *m, int variant, const void *base,
    const uint64_t *offsets, size_t count, uint64_t *out, int nthreads)
{
    struct batch_job j;

    if (!m || !offsets || (!out && count))
        return -1;
    memset(&j, 0, sizeof(j));
    j.m = m;
    j.variant = variant;
    j.base = (const uint8_t *) base;
    j.offsets = offsets;
    j.count = count;
    j.out = out;
    return run_batch(&j, nthreads);
}

int
oracle_splitmix_batch_fixed(const oracle_model_t *m, int variant,
    uint64_t seed, size_t stride, size_t len, size_t first, size_t count,
    uint64_t *out, int nthreads)
{
    struct batch_job j;

    if (!m || (!out && count))
        return -1;
    memset(&j, 0, sizeof(j));
    j.m = m;
    j.variant = variant;
    j.seed = seed;
    j.gen = 1;
    j.stride = stride;
    j.len = len;
    j.first = first;
    j.count = count;
    j.out = out;
    return run_batch(&j, nthreads);
}
