/*
 * mchecksum_models.h -- the CRC variants libmchecksum implements and how the
 * mchecksum method names map onto them.
 *
 * "crc32c" is CRC-32C (Castagnoli, RFC 3720) -- a standard, pinned.
 * "crc64" and "crc16": the upstream mchecksum variants are not recoverable
 * (its source is absent from the reference tree), so the
 * defaults below are choices, labelled "parity unpinned" in DESIGN.md, and
 * can be re-pointed at run time without rebuilding:
 *     MCHECKSUM_CRC64_VARIANT=crc64-ecma182 (or any crc64-* name below)
 *     MCHECKSUM_CRC16_VARIANT=crc16-arc     (or any crc16-* name below)
 */
#ifndef MCHECKSUM_MODELS_H
#define MCHECKSUM_MODELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const char *name;
    int width;      /* 16, 32 or 64 */
    uint64_t poly;  /* normal (MSB-first) polynomial, x^width term implied */
    int reflected;  /* refin == refout == 1 */
    uint64_t init;  /* direct-form initial register */
    uint64_t xorout;
} mck_model_t;

#define MCK_NMODELS 12
extern const mck_model_t mck_models[MCK_NMODELS];

/* Environment settings, read ONCE per process at first use into an
 * immutable snapshot (no getenv on the call path: getenv races setenv in a
 * multithreaded Mercury process); mck_settings_reload() publishes a fresh
 * snapshot (mchecksum_gpu_reload_settings(): tests and tuning tools that
 * change the environment).  -1 = "not set: the library decides". */
typedef struct {
    int crc64_idx, crc16_idx;   /* MCHECKSUM_CRC64_VARIANT / _CRC16_VARIANT, resolved */
    int log_quiet;              /* MCHECKSUM_LOG_LEVEL=none|0 */
    /* MCHECKSUM_GPU_* overrides of the batch path's launch policy (A/B
     * tools and tests; the defaults are the measured best) */
    int gpu_log2g;              /* _LOG2G: lanes per payload for fixed batches */
    int gpu_light;              /* _LIGHT: small-batch layout 0/1 */
    int gpu_nt;                 /* _NT: non-temporal payload loads 0/1 */
    int gpu_split;              /* _SPLIT: split CRC-64 pieces 0/1 */
    int gpu_split_lds;          /* _SPLIT_LDS=0: pieces combine through a zeroed output */
    int gpu_force_generic;      /* _FORCE_GENERIC=1: no aligned fixed path */
    int gpu_xdr_fast;           /* _XDR_FAST: XDR throughput layout 0/1 */
    uint64_t gpu_seg_map_cap;   /* _SEG_MAP_CAP: cap on the chunk map (UINT64_MAX: none) */
    uint32_t gpu_queue_slots;   /* _QUEUE_SLOTS: smaller slot pool (0: default) */
    int qfault_mode;            /* test builds: _QFAULT_MODE (0 give-up, 1 stall, 2 scanstall, 3 both) */
    uint64_t qfault_scan;       /* test builds: _QFAULT_SCAN (UINT64_MAX: none) */
} mck_settings_t;
const mck_settings_t *mck_settings(void);
void mck_settings_reload(void);

/* Resolve a method name ("crc32c", "crc64", "crc16" or a variant name) to an
 * index into mck_models, honouring the *_VARIANT settings.
 * Returns -1 for unknown names. */
int mck_model_index(const char *hash_method);

uint64_t mck_reflect(uint64_t v, int nbits);

/* Z^512 and Z^256 applied to a CRC-32C register (3-way SSE4.2 combine). */
uint64_t mck_crc32c_shift512(uint64_t c);
uint64_t mck_crc32c_shift256(uint64_t c);

#ifdef __cplusplus
}
#endif
#endif
