/*
 * oracle_selftest.c -- pins the oracle before anything trusts it (TEST ONLY).
 *
 *  1. every catalogue model reproduces its published check value
 *     (CRC of ASCII "123456789");
 *  2. CRC-32C reproduces the four RFC 3720 sec. B.4 vectors;
 *  3. the table form equals the bitwise form on random data for every model;
 *  4. CRC-32C equals the SSE4.2 crc32 instruction on random data, lengths
 *     0..4100 at every start offset 0..15.
 * Exit status 0 = all pinned.
 */
#include "crc_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int failures;

#define CHECK(cond, ...)                                                       \
    do {                                                                       \
        if (!(cond)) {                                                         \
            fprintf(stderr, "FAIL: " __VA_ARGS__);                             \
            fprintf(stderr, "\n");                                             \
            failures++;                                                        \
        }                                                                      \
    } while (0)

int
main(void)
{
    const oracle_model_t *m;
    const oracle_model_t *c32 = oracle_model_by_name("crc32c");
    uint8_t buf[4200 + 16], v[32];
    size_t n, off;
    int i, ok = 0;

    for (m = oracle_models(); m->name; m++) {
        uint64_t c = oracle_crc_bitwise(m, "123456789", 9);
        CHECK(c == m->check, "%s check 0x%llx != 0x%llx", m->name,
            (unsigned long long) c, (unsigned long long) m->check);
        c = oracle_crc_table(m, "123456789", 9);
        CHECK(c == m->check, "%s table check 0x%llx", m->name, (unsigned long long) c);
    }

    memset(v, 0, 32);
    CHECK(oracle_crc_bitwise(c32, v, 32) == 0x8A9136AAu, "rfc3720 zeros");
    memset(v, 0xFF, 32);
    CHECK(oracle_crc_bitwise(c32, v, 32) == 0x62A8AB43u, "rfc3720 ones");
    for (i = 0; i < 32; i++)
        v[i] = (uint8_t) i;
    CHECK(oracle_crc_bitwise(c32, v, 32) == 0x46DD794Eu, "rfc3720 ascending");
    for (i = 0; i < 32; i++)
        v[i] = (uint8_t) (31 - i);
    CHECK(oracle_crc_bitwise(c32, v, 32) == 0x113FDB5Cu, "rfc3720 descending");

    oracle_fill_splitmix(buf, sizeof(buf), 0x4D43310000000000ULL, 0);
    for (m = oracle_models(); m->name; m++)
        for (n = 0; n < 300; n += 7)
            CHECK(oracle_crc_table(m, buf + (n % 13), n) ==
                      oracle_crc_bitwise(m, buf + (n % 13), n),
                "%s table!=bitwise n=%zu", m->name, n);
    for (m = oracle_models(); m->name; m++)
        for (n = 0; n < 300; n += 5)
            CHECK(oracle_crc_slice8(m, buf + (n % 11), n) ==
                      oracle_crc_bitwise(m, buf + (n % 11), n),
                "%s slice8!=bitwise n=%zu", m->name, n);

    oracle_crc32c_sse42("", 0, &ok);
    if (ok) {
        for (off = 0; off < 16; off++)
            for (n = 0; n <= 4100; n += (n < 80 ? 1 : 37))
                CHECK(oracle_crc32c_sse42(buf + off, n, NULL) ==
                          (uint32_t) oracle_crc_table(c32, buf + off, n),
                    "sse42 != table off=%zu n=%zu", off, n);
    } else {
        fprintf(stderr, "note: no SSE4.2 on this CPU; hardware cross-check skipped\n");
    }

    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("oracle pinned: %s\n", ok ? "catalogue+rfc3720+sse4.2" : "catalogue+rfc3720");
    return 0;
}
