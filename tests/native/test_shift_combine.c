/*
 * test_shift_combine.c -- the host half of the scatter-gather algebra that
 * mchecksum_gpu_ext.hip runs on the device, checked on the CPU:
 *  1. the base-16 shift tables (crc32/64_shift_pack_build) apply Z^n exactly
 *     like the GF(2) matrix power crc_op_zpow, for n up to 2^44;
 *  2. the object formula  CRC = Z^N(init) ^ XOR_c Z^after_c(L(chunk_c)) ^ xorout
 *     (L = CRC with zero init, no xorout; chunks of <= 256 KiB of every
 *     segment) equals the streaming API's CRC of the concatenated segments,
 *     for crc32c and crc64 over random segment lists.
 * The streaming API (mchecksum_cpu.c) is itself pinned to the oracle.
 */
#include <mchecksum.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc_gpu_layout.h"
#include "mchecksum_models.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
}

static uint64_t shift(int w, const void *sp, uint64_t x, uint64_t n) {
    for (int k = 0; n; k++, n >>= 4) {
        unsigned d = (unsigned) (n & 15u);
        if (!d)
            continue;
        uint64_t r = 0;
        if (w == 32) {
            const crc32_shift_pack_t *p = sp;
            for (int h = 0; h < 8; h++) r ^= p->op[k][d - 1][h][(x >> (4 * h)) & 15u];
        } else {
            const crc64_shift_pack_t *p = sp;
            for (int h = 0; h < 16; h++) r ^= p->op[k][d - 1][h][(x >> (4 * h)) & 15u];
        }
        x = r;
    }
    return x;
}

static uint64_t api_crc(const char *method, const unsigned char *p, size_t n) {
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    uint64_t v = 0;
    mchecksum_init(method, &c);
    mchecksum_update(c, p, n);
    mchecksum_get(c, &v, mchecksum_get_size(c), MCHECKSUM_FINALIZE);
    mchecksum_destroy(c);
    return v;
}

int main(void) {
    int fails = 0;
    const size_t chunk = 256u << 10, total = 3u << 20;
    unsigned char *buf = malloc(total), *cat = malloc(total);
    for (size_t i = 0; i < total; i++) buf[i] = (unsigned char) next();
    for (int w = 32; w <= 64; w += 32) {
        const char *method = w == 32 ? "crc32c" : "crc64";
        const mck_model_t *m = &mck_models[mck_model_index(method)];
        crc_rmodel_t rm = {m->width, mck_reflect(m->poly, m->width), mck_reflect(m->init, m->width), m->xorout};
        void *sp = calloc(1, w == 32 ? sizeof(crc32_shift_pack_t) : sizeof(crc64_shift_pack_t));
        if ((w == 32 ? crc32_shift_pack_build(&rm, sp) : crc64_shift_pack_build(&rm, sp)) != 0) {
            printf("FAIL shift pack build w=%d\n", w);
            return 1;
        }
        const uint64_t mask = w == 32 ? 0xFFFFFFFFull : ~0ull;
        uint64_t op[64];
        for (int t = 0; t < 300; t++) {
            uint64_t n = t < 40 ? (uint64_t) t : next() & ((1ull << 44) - 1), x = next() & mask;
            crc_op_zpow(&rm, (int64_t) n, op);
            if (shift(w, sp, x, n) != crc_op_apply(w, op, x)) {
                printf("FAIL shift w=%d n=%llu\n", w, (unsigned long long) n);
                fails++;
            }
        }
        for (int trial = 0; trial < 40; trial++) {
            int nseg = (int) (next() % 6);
            size_t N = 0, off[6], len[6];
            for (int s = 0; s < nseg; s++) {
                static const size_t pool[] = {0, 1, 3, 8, 100, 4095, 262143, 262144, 262145, 600001};
                len[s] = pool[next() % 10];
                off[s] = next() % (total - len[s]);
                memcpy(cat + N, buf + off[s], len[s]);
                N += len[s];
            }
            /* device formula, chunk by chunk */
            uint64_t v = shift(w, sp, rm.rinit, N) ^ rm.xorout, pos = 0;
            for (int s = 0; s < nseg; s++)
                for (size_t o = 0; o < len[s]; o += chunk) {
                    size_t n = len[s] - o < chunk ? len[s] - o : chunk;
                    /* L(M) = CRC(M) ^ xorout ^ Z^|M|(init) */
                    uint64_t L = api_crc(method, buf + off[s] + o, n) ^ rm.xorout ^ shift(w, sp, rm.rinit, n);
                    pos += n;
                    v ^= shift(w, sp, L, N - pos);
                }
            if (v != api_crc(method, cat, N)) {
                printf("FAIL combine w=%d trial %d\n", w, trial);
                fails++;
            }
        }
        free(sp);
    }
    free(buf);
    free(cat);
    if (fails)
        return 1;
    printf("shift/combine: all checks passed\n");
    return 0;
}
