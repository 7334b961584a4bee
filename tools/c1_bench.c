/*
 * c1_bench.c -- BASELINE configs[0] on the host: CRC-32C of 1024 x 4 KiB
 * buffers through libmchecksum's streaming API the way Mercury's proc layer
 * drives it for hg_perf_proc_iovec (Testing/perf/hg/mercury_perf.c:897-923):
 * reset, update(u32 length field), update(raw bytes), get(FINALIZE).
 * One object, one thread (an RPC handler).  Timing: CLOCK_MONOTONIC
 * (as src/util/mercury_time.h:257-260).
 * usage: c1_bench COUNT LENGTH STEPS WARMUP < payload bytes (COUNT*LENGTH)
 * prints: seconds crc_first crc_xor
 */
#define _POSIX_C_SOURCE 199309L
#include <mchecksum.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static double
now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + (double) ts.tv_nsec * 1e-9;
}

int
main(int argc, char **argv)
{
    size_t count, length, i;
    int steps, warmup, s;
    unsigned char *buf;
    uint32_t *crcs, len32, x = 0;
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    double t0 = 0, t1;

    if (argc < 5)
        return 2;
    count = strtoul(argv[1], NULL, 0);
    length = strtoul(argv[2], NULL, 0);
    steps = atoi(argv[3]);
    warmup = atoi(argv[4]);
    buf = malloc(count * length);
    crcs = calloc(count, sizeof(*crcs));
    if (!buf || !crcs || fread(buf, 1, count * length, stdin) != count * length)
        return 3;
    if (mchecksum_init("crc32c", &c) != 0)
        return 4;
    len32 = (uint32_t) length;
    for (s = -warmup; s < steps; s++) {
        if (s == 0)
            t0 = now();
        for (i = 0; i < count; i++) {
            mchecksum_reset(c);
            mchecksum_update(c, &len32, sizeof(len32));
            mchecksum_update(c, buf + i * length, length);
            mchecksum_get(c, &crcs[i], sizeof(uint32_t), MCHECKSUM_FINALIZE);
        }
    }
    t1 = now();
    for (i = 0; i < count; i++)
        x ^= crcs[i];
    printf("%.9f %u %u\n", t1 - t0, crcs[0], x);
    mchecksum_destroy(c);
    free(buf);
    free(crcs);
    return 0;
}
