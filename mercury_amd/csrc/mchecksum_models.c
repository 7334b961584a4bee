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

/* ------------------------------------------------------------ settings -- */

static int
env_int(const char *var, int lo, int hi)
{
    const char *e = getenv(var);
    long v;

    if (!e || !e[0])
        return -1;
    v = strtol(e, NULL, 10);
    return v < lo || v > hi ? -1 : (int) v;
}

static int
env_variant(const char *var, const char *family, const char *dflt)
{
    const char *e = getenv(var);

    if (e && strncmp(e, family, 6) == 0 && find(e) >= 0)
        return find(e);
    return find(dflt);
}

static mck_settings_t *
settings_from_env(void)
{
    mck_settings_t *s = calloc(1, sizeof(*s));
    const char *e;

    if (!s)
        return NULL;
    s->crc64_idx = env_variant("MCHECKSUM_CRC64_VARIANT", "crc64-", MCK_DEFAULT_CRC64);
    s->crc16_idx = env_variant("MCHECKSUM_CRC16_VARIANT", "crc16-", MCK_DEFAULT_CRC16);
    e = getenv("MCHECKSUM_LOG_LEVEL");
    s->log_quiet = e && (strcmp(e, "none") == 0 || strcmp(e, "0") == 0);
    s->gpu_log2g = env_int("MCHECKSUM_GPU_LOG2G", 0, CRC_GPU_MAX_LOG2G);
    s->gpu_light = env_int("MCHECKSUM_GPU_LIGHT", 0, 1);
    s->gpu_nt = env_int("MCHECKSUM_GPU_NT", 0, 1);
    s->gpu_split = env_int("MCHECKSUM_GPU_SPLIT", 0, 1);
    s->gpu_split_lds = env_int("MCHECKSUM_GPU_SPLIT_LDS", 0, 1) != 0;
    s->gpu_force_generic = env_int("MCHECKSUM_GPU_FORCE_GENERIC", 0, 1) == 1;
    s->gpu_xdr_fast = env_int("MCHECKSUM_GPU_XDR_FAST", 0, 1);
    e = getenv("MCHECKSUM_GPU_SEG_MAP_CAP");
    s->gpu_seg_map_cap = e && e[0] ? strtoull(e, NULL, 10) : UINT64_MAX;
    e = getenv("MCHECKSUM_GPU_QUEUE_SLOTS");
    s->gpu_queue_slots = e && e[0] && atol(e) > 0 ? (uint32_t) atol(e) : 0;
    e = getenv("MCHECKSUM_GPU_QFAULT_MODE");
    s->qfault_mode = !e                                  ? 0
                     : strcmp(e, "stall") == 0           ? 1
                     : strcmp(e, "scanstall") == 0       ? 2
                     : strcmp(e, "stall+scanstall") == 0 ? 3
                                                         : 0;
    e = getenv("MCHECKSUM_GPU_QFAULT_SCAN");
    s->qfault_scan = e && e[0] ? strtoull(e, NULL, 10) : UINT64_MAX;
    return s;
}

/* The current snapshot.  A reload publishes a new one and never frees the
 * old (a concurrent reader may still hold it): reloads are for tests and
 * tuning tools, a few per process. */
static const mck_settings_t *_Atomic g_settings;
static pthread_once_t g_settings_once = PTHREAD_ONCE_INIT;
static pthread_mutex_t g_settings_mu = PTHREAD_MUTEX_INITIALIZER;
/* the defaults, if the first snapshot cannot be allocated */
static mck_settings_t g_settings_fallback = {.gpu_log2g = -1, .gpu_light = -1, .gpu_nt = -1, .gpu_split = -1,
                                             .gpu_split_lds = 1, .gpu_xdr_fast = -1,
                                             .gpu_seg_map_cap = UINT64_MAX, .qfault_scan = UINT64_MAX};

static void
settings_init(void)
{
    const mck_settings_t *s = settings_from_env();

    if (!s) {
        g_settings_fallback.crc64_idx = find(MCK_DEFAULT_CRC64);
        g_settings_fallback.crc16_idx = find(MCK_DEFAULT_CRC16);
        s = &g_settings_fallback;
    }
    __atomic_store_n(&g_settings, s, __ATOMIC_RELEASE);
}

const mck_settings_t *
mck_settings(void)
{
    pthread_once(&g_settings_once, settings_init);
    return __atomic_load_n(&g_settings, __ATOMIC_ACQUIRE);
}

void
mck_settings_reload(void)
{
    const mck_settings_t *s;

    pthread_once(&g_settings_once, settings_init);
    pthread_mutex_lock(&g_settings_mu);
    s = settings_from_env();
    if (s)
        __atomic_store_n(&g_settings, s, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&g_settings_mu);
}

int
mck_model_index(const char *hash_method)
{
    if (!hash_method)
        return -1;
    if (strcmp(hash_method, "crc64") == 0)
        return mck_settings()->crc64_idx;
    if (strcmp(hash_method, "crc16") == 0)
        return mck_settings()->crc16_idx;
    return find(hash_method);
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
