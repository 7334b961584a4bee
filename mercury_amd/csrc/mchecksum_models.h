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

/* Resolve a method name ("crc32c", "crc64", "crc16" or a variant name) to an
 * index into mck_models, honouring the *_VARIANT environment overrides.
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
