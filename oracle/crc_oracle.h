/*
 * crc_oracle.h -- CPU restatement of the mchecksum CRC arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under mercury_amd/ (the product) may
 * include, link or call this code.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg use it, and only as the checker.
 *
 * What it restates.  Mercury calls the third-party module mchecksum
 * (git submodule src/mchecksum, .gitmodules:4-6; pinned version unrecoverable,
 * "Update to mchecksum v2.0" in Documentation/CHANGES_v2.2.0.md:63) with the
 * methods "crc16", "crc32c" and "crc64":
 *   - src/mercury_proc.c:54-63     hash enum -> method name
 *   - src/mercury_proc.c:398       mchecksum_update per serialized field
 *   - src/mercury_proc.c:374       mchecksum_get(..., MCHECKSUM_FINALIZE)
 *   - src/mercury_core_header.c:24 "crc16" over the core header fields
 * The mchecksum source is absent from /root/reference, so the algorithm is
 * restated from the published CRC definitions (Rocksoft/Williams model):
 *   - crc32c : CRC-32C / iSCSI, RFC 3720 sec. B.4 -- PINNED (standard, RFC
 *              vectors, and the x86 SSE4.2 crc32 instruction, which computes
 *              exactly this CRC in hardware).
 *   - crc64  : CRC-64/XZ (ECMA-182, reflected, init/xorout all-ones) by
 *              default -- PARITY UNPINNED (upstream variant unknown here).
 *   - crc16  : CRC-16/T10-DIF by default -- PARITY UNPINNED.
 * Every catalogue variant in SURVEY.md Appendix A is available through the
 * parameterised model so a later round can re-pin without code changes.
 */
#ifndef CRC_ORACLE_H
#define CRC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const char *name;
    int width;       /* 8..64 */
    uint64_t poly;   /* normal (MSB-first) form, without the x^width term */
    int refin;       /* reflect each input byte */
    int refout;      /* reflect the final register */
    uint64_t init;   /* initial register value (direct form) */
    uint64_t xorout; /* final XOR */
    uint64_t check;  /* catalogue CRC of ASCII "123456789" */
} oracle_model_t;

/* Catalogue of models. Terminated by name == NULL. */
const oracle_model_t *oracle_models(void);
const oracle_model_t *oracle_model_by_name(const char *name);

/* Bit-at-a-time, literally the Rocksoft definition.  Slow; small inputs. */
uint64_t oracle_crc_bitwise(const oracle_model_t *m, const void *data, size_t n);

/* Streaming form of the bitwise model: reg = oracle_reg_init(m);
 * reg = oracle_reg_update(m, reg, d, n) ...; crc = oracle_reg_final(m, reg). */
uint64_t oracle_reg_init(const oracle_model_t *m);
uint64_t oracle_reg_update(const oracle_model_t *m, uint64_t reg, const void *data, size_t n);
uint64_t oracle_reg_final(const oracle_model_t *m, uint64_t reg);

/* Byte-at-a-time table form (Sarwate), derived from the bitwise model at
 * run time; checked against it in tests.  Used for large fixtures. */
uint64_t oracle_crc_table(const oracle_model_t *m, const void *data, size_t n);
/* slicing-by-8 (reflected models; others fall back to the byte table) */
uint64_t oracle_crc_slice8(const oracle_model_t *m, const void *data, size_t n);

/* Independent hardware oracle: x86 SSE4.2 crc32 instruction (CRC-32C).
 * Returns 0 and sets *ok = 0 when the CPU lacks SSE4.2. */
uint32_t oracle_crc32c_sse42(const void *data, size_t n, int *ok);

/* Synthetic payload bytes: little-endian 64-bit words
 * splitmix64(seed ^ (first_word + i)).  Writes nbytes bytes (nbytes need not
 * be a multiple of 8; the last word is truncated). */
uint64_t oracle_splitmix64(uint64_t x);
void oracle_fill_splitmix(void *dst, size_t nbytes, uint64_t seed, uint64_t first_word);

/* Variable-length batch layout (config C4): len_i = 64 + splitmix64(lseed ^ i)
 * % 65473, packed back to back; offsets[0] = 0, offsets[i+1] = offsets[i]+len_i.
 * lseed = seed ^ ORACLE_LEN_SALT. */
#define ORACLE_LEN_SALT 0x4C454E4754480000ULL
void oracle_varlen_offsets(uint64_t seed, size_t count, uint64_t min_len,
    uint64_t max_len, uint64_t *offsets /* count + 1 */);

/* Batch CRC over host buffers with nthreads pthreads (nthreads <= 0: 1).
 * variant: 0 = table (Sarwate), 1 = SSE4.2 (crc32c only), 2 = bitwise.
 * out receives count values as uint64 (low bits hold the CRC).
 * Returns 0 on success, -1 on bad arguments. */
int oracle_batch_fixed(const oracle_model_t *m, int variant, const void *base,
    size_t stride, size_t len, size_t count, uint64_t *out, int nthreads);
int oracle_batch_offsets(const oracle_model_t *m, int variant, const void *base,
    const uint64_t *offsets, size_t count, uint64_t *out, int nthreads);

/* Generate-and-checksum for a fixed-size splitmix batch without holding the
 * whole batch in memory: payload i occupies bytes [i*stride, i*stride+len) of
 * a virtual buffer filled by oracle_fill_splitmix(seed, word 0).  Computes
 * payloads [first, first+count).  Used by the parity tests at full sizes. */
int oracle_splitmix_batch_fixed(const oracle_model_t *m, int variant,
    uint64_t seed, size_t stride, size_t len, size_t first, size_t count,
    uint64_t *out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
