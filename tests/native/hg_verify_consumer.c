/*
 * hg_verify_consumer.c -- a compiled consumer of the batch ABI
 * (<mchecksum_gpu.h>), written as the binding a Mercury maintainer would add
 * (INTEGRATION.md section 3): it finds libmchecksum through
 * cmake/mchecksum-config.cmake (tests/native/hg_consumer/CMakeLists.txt),
 * hipMallocs a drained receive buffer of Mercury-shaped messages, and checks
 * them on a real hipStream_t with mchecksum_gpu_verify_messages and
 * mchecksum_gpu_verify_core_headers.
 *
 * Message i (request): a 16-byte core header -- hg, protocol, id (u64
 * big-endian), flags, cookie, CRC16 (u16 big-endian at byte 12) over the
 * HOST-order field values (/root/reference/src/mercury_core_header.c:175-230,
 * HG_CORE_HEADER_CHECKSUM_UPDATE :46-55) -- then the 4-byte HG header holding
 * the payload's CRC32C in network order (/root/reference/src/mercury_header.c:
 * 111-112), then the serialized payload.
 *
 * The verdicts it must reproduce are the reference's per-message checks,
 * computed here on the host through the streaming API the way Mercury does:
 * hg_proc_checksum_verify (/root/reference/src/mercury_proc.c:433-472)
 * memcmps the hash that mchecksum_get(FINALIZE) returns after the payload was
 * streamed through mchecksum_update, and hg_core_header_request_proc (:175-230)
 * compares the CRC16 of the decoded fields with the wire value.  Planted
 * corruption: a payload bit, a stored payload hash, a core-header field, a
 * core-header hash, and a message too short for its headers.
 *
 * Without a HIP device every entry point must refuse with
 * MCHECKSUM_GPU_ENODEV (no host fallback); the program then prints NODEV and
 * exits 0 (the CPU test run).  Exit status: 0 pass, non-zero the failed step.
 */
#include <mchecksum.h>
#include <mchecksum_gpu.h>

#include <hip/hip_runtime_api.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NMSG 4096
#define HDR 16
#define HGH 4

static uint64_t rng_state = 0x4D43310000000006ull;
static uint64_t
next_u64(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* mchecksum over one buffer, the way hg_proc_flush computes it */
static int
stream_hash(const char *method, const void *p, size_t n, void *out, size_t out_size)
{
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    if (mchecksum_init(method, &c) != 0)
        return -1;
    if (n && mchecksum_update(c, p, n) != 0)
        return -1;
    if (mchecksum_get(c, out, out_size, MCHECKSUM_FINALIZE) != 0)
        return -1;
    return mchecksum_destroy(c);
}

/* The core header's CRC16 over the host-order field values, field by field
 * as HG_CORE_HEADER_PROC streams them (an update per field). */
static uint16_t
core_header_crc16(uint8_t hg, uint8_t protocol, uint64_t id, uint8_t flags, uint8_t cookie)
{
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
    uint16_t h = 0;
    if (mchecksum_init("crc16", &c) != 0)
        return 0;
    mchecksum_update(c, &hg, 1);
    mchecksum_update(c, &protocol, 1);
    mchecksum_update(c, &id, 8); /* host order: the decoded value */
    mchecksum_update(c, &flags, 1);
    mchecksum_update(c, &cookie, 1);
    mchecksum_get(c, &h, sizeof(h), MCHECKSUM_FINALIZE);
    mchecksum_destroy(c);
    return h;
}

static void
put_be(uint8_t *p, uint64_t v, int n)
{
    for (int k = 0; k < n; k++)
        p[k] = (uint8_t)(v >> (8 * (n - 1 - k)));
}
static uint64_t
get_be(const uint8_t *p, int n)
{
    uint64_t v = 0;
    for (int k = 0; k < n; k++)
        v = v << 8 | p[k];
    return v;
}

/* hg_core_header_request_proc(HG_DECODE) + hg_proc_checksum_verify on the host:
 * the reference verdicts (1 = HG_CHECKSUM_ERROR / too short). */
static void
host_verdicts(const uint8_t *buf, const uint64_t *off, size_t n, uint8_t *hdr_bad, uint8_t *pay_bad)
{
    for (size_t i = 0; i < n; i++) {
        const uint8_t *m = buf + off[i];
        const uint64_t len = off[i + 1] - off[i];
        if (len < HDR) {
            hdr_bad[i] = 1;
        } else {
            const uint64_t id = get_be(m + 2, 8);
            const uint16_t h = core_header_crc16(m[0], m[1], id, m[10], m[11]);
            hdr_bad[i] = h != (uint16_t) get_be(m + 12, 2);
        }
        if (len < HDR + HGH) {
            pay_bad[i] = 1;
        } else {
            uint32_t h = 0, wire = (uint32_t) get_be(m + HDR, 4);
            stream_hash("crc32c", m + HDR + HGH, len - HDR - HGH, &h, sizeof(h));
            pay_bad[i] = memcmp(&h, &wire, sizeof(h)) != 0; /* hash bytes as hg_proc holds them */
        }
    }
}

#define HIPCHK(x)                                                               \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 20;                                                          \
        }                                                                       \
    } while (0)

int
main(void)
{
    if (!mchecksum_gpu_available()) {
        /* no host fallback: every entry point refuses */
        uint8_t st = 0;
        uint32_t bad = 0;
        uint64_t off[2] = {0, 0};
        int rc1 = mchecksum_gpu_verify_messages("crc32c", off, off, 1, HDR + HGH, HDR, &st, &bad, NULL);
        int rc2 = mchecksum_gpu_verify_core_headers("crc16", MCHECKSUM_GPU_CORE_HEADER_REQUEST, off, off, 1, &st,
                                                    &bad, NULL);
        if (rc1 != MCHECKSUM_GPU_ENODEV || rc2 != MCHECKSUM_GPU_ENODEV) {
            fprintf(stderr, "no device, but rc %d / %d\n", rc1, rc2);
            return 2;
        }
        printf("NODEV: verify_messages and verify_core_headers refused with MCHECKSUM_GPU_ENODEV\n");
        return 0;
    }

    /* the drained receive buffer: NMSG requests, payloads 0 B .. 16 KiB */
    uint64_t *off = malloc((NMSG + 1) * sizeof(uint64_t));
    size_t total = 0;
    off[0] = 0;
    for (size_t i = 0; i < NMSG; i++) {
        size_t pay = (size_t)(next_u64() % 16385);
        if (i % 97 == 5)
            pay = 0; /* an empty payload */
        size_t len = HDR + HGH + pay;
        if (i == 13)
            len = HDR + 2; /* too short for its HG header */
        if (i == 14)
            len = 9; /* too short for its core header */
        total += len;
        off[i + 1] = total;
    }
    uint8_t *buf = calloc(total + 64, 1);
    for (size_t i = 0; i < NMSG; i++) {
        uint8_t *m = buf + off[i];
        const uint64_t len = off[i + 1] - off[i];
        for (uint64_t k = 0; k < len; k++)
            m[k] = (uint8_t) next_u64();
        if (len < HDR)
            continue;
        const uint8_t hg = 'H' << 1 | 1, proto = 4, flags = (uint8_t) i, cookie = (uint8_t)(i >> 8);
        const uint64_t id = next_u64();
        m[0] = hg;
        m[1] = proto;
        put_be(m + 2, id, 8);
        m[10] = flags;
        m[11] = cookie;
        put_be(m + 12, core_header_crc16(hg, proto, id, flags, cookie), 2);
        m[14] = m[15] = 0;
        if (len < HDR + HGH)
            continue;
        uint32_t h = 0; /* hg_set_struct: the payload hash, network order in the HG header */
        if (stream_hash("crc32c", m + HDR + HGH, len - HDR - HGH, &h, sizeof(h)) != 0)
            return 3;
        put_be(m + HDR, h, 4);
    }
    /* planted corruption */
    buf[off[3] + HDR + HGH + 1] ^= 0x20;   /* payload bit: payload fails */
    buf[off[7] + HDR + 2] ^= 0x01;         /* stored payload hash: payload fails */
    buf[off[11] + 10] ^= 0x80;             /* a core-header field: header fails */
    buf[off[12] + 13] ^= 0x04;             /* the core-header hash: header fails */

    uint8_t *want_hdr = calloc(NMSG, 1), *want_pay = calloc(NMSG, 1);
    host_verdicts(buf, off, NMSG, want_hdr, want_pay);
    size_t want_nhdr = 0, want_npay = 0;
    for (size_t i = 0; i < NMSG; i++) {
        want_nhdr += want_hdr[i];
        want_npay += want_pay[i];
    }
    if (!want_pay[3] || !want_pay[7] || !want_hdr[11] || !want_hdr[12] || !want_pay[13] || !want_hdr[14] ||
        want_pay[11] || want_hdr[3]) {
        fprintf(stderr, "host verdicts do not show the planted corruption\n");
        return 4;
    }

    /* device side: one buffer, its message table, a real stream */
    void *d_buf = NULL, *d_off = NULL, *d_st = NULL, *d_cnt = NULL;
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&d_buf, total + 64));
    HIPCHK(hipMalloc(&d_off, (NMSG + 1) * sizeof(uint64_t)));
    HIPCHK(hipMalloc(&d_st, 2 * NMSG));
    HIPCHK(hipMalloc(&d_cnt, 2 * sizeof(uint32_t)));
    HIPCHK(hipMemcpyAsync(d_buf, buf, total + 64, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_off, off, (NMSG + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_cnt, 0, 2 * sizeof(uint32_t), s));
    HIPCHK(hipMemsetAsync(d_st, 0xAB, 2 * NMSG, s));
    if (mchecksum_gpu_prepare("crc32c") != MCHECKSUM_GPU_OK || mchecksum_gpu_prepare("crc16") != MCHECKSUM_GPU_OK) {
        fprintf(stderr, "prepare: %s\n", mchecksum_gpu_last_error());
        return 5;
    }
    uint8_t *d_st_hdr = d_st, *d_st_pay = (uint8_t *) d_st + NMSG;
    uint32_t *d_nhdr = d_cnt, *d_npay = (uint32_t *) d_cnt + 1;
    int rc = mchecksum_gpu_verify_core_headers("crc16", MCHECKSUM_GPU_CORE_HEADER_REQUEST, d_buf, d_off, NMSG, d_st_hdr,
                                               d_nhdr, s);
    if (rc != MCHECKSUM_GPU_OK) {
        fprintf(stderr, "verify_core_headers rc %d: %s\n", rc, mchecksum_gpu_last_error());
        return 6;
    }
    rc = mchecksum_gpu_verify_messages("crc32c", d_buf, d_off, NMSG, HDR + HGH, HDR, d_st_pay, d_npay, s);
    if (rc != MCHECKSUM_GPU_OK) {
        fprintf(stderr, "verify_messages rc %d: %s\n", rc, mchecksum_gpu_last_error());
        return 7;
    }
    uint8_t *st = malloc(2 * NMSG);
    uint32_t cnt[2];
    HIPCHK(hipMemcpyAsync(st, d_st, 2 * NMSG, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cnt, d_cnt, sizeof(cnt), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    size_t diff_hdr = 0, diff_pay = 0;
    for (size_t i = 0; i < NMSG; i++) {
        diff_hdr += st[i] != want_hdr[i];
        diff_pay += st[NMSG + i] != want_pay[i];
        if ((st[i] != want_hdr[i] || st[NMSG + i] != want_pay[i]) && diff_hdr + diff_pay <= 4)
            fprintf(stderr, "message %zu: gpu hdr %u pay %u, host hdr %u pay %u\n", i, st[i], st[NMSG + i],
                    want_hdr[i], want_pay[i]);
    }
    printf("gpu: %d messages (%zu bytes) on a hipStream_t: core-header statuses %zu differ, payload statuses %zu "
           "differ; flagged %u / %u (host %zu / %zu)\n",
           NMSG, total, diff_hdr, diff_pay, cnt[0], cnt[1], want_nhdr, want_npay);
    if (diff_hdr || diff_pay || cnt[0] != want_nhdr || cnt[1] != want_npay)
        return 8;
    HIPCHK(hipFree(d_buf));
    HIPCHK(hipFree(d_off));
    HIPCHK(hipFree(d_st));
    HIPCHK(hipFree(d_cnt));
    HIPCHK(hipStreamDestroy(s));
    printf("PASS\n");
    return 0;
}
