/* cpu_batch.c -- the PRODUCT's CPU path over a batch, for bench.py's
 * cpu_baseline breakdown ("product_<n>threads"): libmchecksum's streaming API
 * (init / reset / update / get(FINALIZE), include/mchecksum.h) on every
 * payload, payloads split into contiguous ranges over n pthreads, one
 * mchecksum object per thread.  This is what a Mercury build linked against
 * libmchecksum.so does per serialized buffer (src/mercury_proc.c:358-406),
 * minus Mercury: for crc32c/crc64 it runs the AVX-512 VPCLMULQDQ fold on
 * updates >= 1 KiB (mercury_amd/csrc/mchecksum_cpu.c).  Not part of the ABI;
 * built as build/libcpu_batch.so and loaded by bench.py with ctypes.
 *
 * Outputs are the mchecksum_get bytes widened to u64 (host order). */
#include <mchecksum.h>

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

struct job {
    const char *method;
    const uint8_t *base;
    const uint64_t *off; /* NULL: fixed stride */
    size_t stride, len, first, count;
    uint64_t *out;
    int rc;
};

static void *run(void *p) {
    struct job *j = p;
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    if (mchecksum_init(j->method, &c) != 0) {
        j->rc = -1;
        return NULL;
    }
    const int size = mchecksum_get_size(c);
    for (size_t i = j->first; i < j->first + j->count; i++) {
        const uint8_t *p0;
        size_t n;
        if (j->off) {
            p0 = j->base + j->off[i];
            n = (size_t)(j->off[i + 1] - j->off[i]);
        } else {
            p0 = j->base + i * j->stride;
            n = j->len;
        }
        uint64_t v = 0;
        mchecksum_reset(c);
        mchecksum_update(c, p0, n);
        if (mchecksum_get(c, &v, (size_t)size, MCHECKSUM_FINALIZE) != 0) {
            j->rc = -1;
            break;
        }
        j->out[i] = v;
    }
    mchecksum_destroy(c);
    return NULL;
}

static int batch(const char *method, const uint8_t *base, const uint64_t *off, size_t stride, size_t len,
                 size_t count, uint64_t *out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if ((size_t)nthreads > count) nthreads = count ? (int)count : 1;
    struct job *jobs = calloc((size_t)nthreads, sizeof(*jobs));
    pthread_t *th = calloc((size_t)nthreads, sizeof(*th));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1;
    }
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        const size_t lo = count * (size_t)t / (size_t)nthreads, hi = count * (size_t)(t + 1) / (size_t)nthreads;
        jobs[t] = (struct job){method, base, off, stride, len, lo, hi - lo, out, 0};
        if (t && pthread_create(&th[t], NULL, run, &jobs[t]) != 0) jobs[t].rc = -2;
    }
    run(&jobs[0]);
    for (int t = 1; t < nthreads; t++)
        if (jobs[t].rc != -2) pthread_join(th[t], NULL);
    for (int t = 0; t < nthreads; t++) rc |= jobs[t].rc;
    free(jobs);
    free(th);
    return rc;
}

__attribute__((visibility("default"))) int cpu_batch_fixed(const char *method, const uint8_t *base, size_t stride,
                                                            size_t len, size_t count, uint64_t *out, int nthreads) {
    return batch(method, base, NULL, stride, len, count, out, nthreads);
}

__attribute__((visibility("default"))) int cpu_batch_offsets(const char *method, const uint8_t *base,
                                                              const uint64_t *offsets, size_t count, uint64_t *out,
                                                              int nthreads) {
    return batch(method, base, offsets, 0, 0, count, out, nthreads);
}
