/*
 * mchecksum_models.c -- variant catalogue and method-name resolution.
 * Parameters are the public CRC catalogue entries.
 */
#define _GNU_SOURCE
#include "mchecksum_models.h"
#include "crc_gpu_layout.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

const mck_model_t mck_models[MCK_NMODELS] = {
    /* name             width poly                   refl init    xorout */
    {"crc32c",           32, 0x1EDC6F41ULL,          1, 0xFFFFFFFFULL, 0xFFFFFFFFULL},
    {"crc32",            32, 0x04C11DB7ULL,          1, 0xFFFFFFFFULL, 0xFFFFFFFFULL},
    {"crc64-xz",         64, 0x42F0E1EBA9EA3693ULL,  1, ~0ULL,         ~0ULL},
    {"crc64-ecma182",    64, 0x42F0E1EBA9EA3693ULL,  0, 0ULL,          0ULL},
    {"crc64-go-iso",     64, 0x000000000000001BULL,  1, ~0ULL,         ~0ULL},
    {"crc64-jones",      64, 0xAD93D23594C935A9ULL,  1, 0ULL,          0ULL},
    {"crc16-arc",        16, 0x8005ULL,              1, 0ULL,          0ULL},
    {"crc16-ibm-3740",   16, 0x1021ULL,              0, 0xFFFFULL,     0ULL},
    {"crc16-xmodem",     16, 0x1021ULL,              0, 0ULL,          0ULL},
    {"crc16-kermit",     16, 0x1021ULL,              1, 0ULL,          0ULL},
    {"crc16-umts",       16, 0x8005ULL,              0, 0ULL,          0ULL},
    {"crc16-t10-dif",    16, 0x8BB7ULL,              0, 0ULL,          0ULL},
};

#define MCK_DEFAULT_CRC64 "crc64-xz"
#define MCK_DEFAULT_CRC16 "crc16-t10-dif"

static int
find(const char *name)
{
    int i;

    for (i = 0; i < MCK_NMODELS; i++)
        if (strcmp(mck_models[i].name, name) == 0)
            return i;
    return -1;
}

int
mck_model_index(const char *hash_method)
{
    const char *name = hash_method;
    int idx;

    if (!name)
        return -1;
    if (strcmp(name, "crc64") == 0) {
        const char *env = getenv("MCHECKSUM_CRC64_VARIANT");
        name = MCK_DEFAULT_CRC64;
        if (env && strncmp(env, "crc64-", 6) == 0 && find(env) >= 0)
            name = env;
    } else if (strcmp(name, "crc16") == 0) {
        const char *env = getenv("MCHECKSUM_CRC16_VARIANT");
        name = MCK_DEFAULT_CRC16;
        if (env && strncmp(env, "crc16-", 6) == 0 && find(env) >= 0)
            name = env;
    }
    idx = find(name);
    return idx;
}

uint64_t
mck_reflect(uint64_t v, int nbits)
{
    uint64_t r = 0;
    int i;

    for (i = 0; i < nbits; i++)
        if (v & (1ULL << i))
            r |= 1ULL << (nbits - 1 - i);
    return r;
}

/* Byte tables of Z^256 and Z^512 on the CRC-32C register. */
static uint32_t g_shift[2][4][256];
static pthread_once_t g_shift_once = PTHREAD_ONCE_INIT;

static void
build_shift(void)
{
    const crc_rmodel_t m = {32, 0x82F63B78ULL, 0xFFFFFFFFULL, 0xFFFFFFFFULL, 0};
    uint64_t op[64];
    int s, p, b;

    for (s = 0; s < 2; s++) {
        crc_op_zpow(&m, s ? 512 : 256, op);
        for (p = 0; p < 4; p++)
            for (b = 0; b < 256; b++)
                g_shift[s][p][b] = (uint32_t) crc_op_apply(32, op, (uint64_t) b << (8 * p));
    }
}

static uint64_t
shift_apply(int s, uint64_t c)
{
    pthread_once(&g_shift_once, build_shift);
    return (uint64_t) (g_shift[s][0][c & 0xFF] ^ g_shift[s][1][(c >> 8) & 0xFF] ^
                       g_shift[s][2][(c >> 16) & 0xFF] ^ g_shift[s][3][(c >> 24) & 0xFF]);
}

uint64_t
mck_crc32c_shift512(uint64_t c)
{
    return shift_apply(1, c);
}

uint64_t
mck_crc32c_shift256(uint64_t c)
{
    return shift_apply(0, c);
}
