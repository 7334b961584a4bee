/*
 * test_mchecksum_api.c -- the drop-in mchecksum ABI exercised the way Mercury
 * does (C, no Python), modelled on Testing/unit/hg/test_proc.c:79-227:
 *   encode a proc buffer field by field (HG_PROC_TYPE: memcpy + update,
 *   src/mercury_proc.h:124-143), flush (get FINALIZE, src/mercury_proc.c:374),
 *   "send" (memcpy), decode with the same per-field updates, verify with memcmp
 *   (hg_proc_checksum_verify, src/mercury_proc.c:433-472).
 * Adds what test_proc lacks: the pinned CRC-32C value of the encoded bytes,
 * the save_ptr/restore_ptr pattern of bulk-handle procs (src/mercury_proc_bulk.c),
 * a corrupted-transfer case, every method's size, destroy(NULL), and distinct
 * objects used concurrently from 8 threads (Mercury's progress + handler
 * threads).  Built plain, with ASan+UBSan and with TSan (tests/test_native_api.py).
 */
#include <mchecksum.h>

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int failures;
#define CHECK(c, msg)                                                          \
    do {                                                                       \
        if (!(c)) {                                                            \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, msg);      \
            failures++;                                                        \
        }                                                                      \
    } while (0)

struct proc {
    unsigned char *buf, *ptr;
    int encode;
    mchecksum_object_t ck;
    unsigned char hash[8];
    size_t hash_size;
};

static void
proc_reset(struct proc *p, unsigned char *buf, int encode)
{
    p->buf = p->ptr = buf;
    p->encode = encode;
    mchecksum_reset(p->ck);
    memset(p->hash, 0, sizeof(p->hash));
}

/* HG_PROC_TYPE / HG_PROC_BYTES in the non-XDR build */
static void
proc_bytes(struct proc *p, void *data, size_t n)
{
    if (p->encode)
        memcpy(p->ptr, data, n);
    else
        memcpy(data, p->ptr, n);
    p->ptr += n;
    mchecksum_update(p->ck, data, n);
}

static int
proc_flush(struct proc *p)
{
    return mchecksum_get(p->ck, p->hash, p->hash_size, MCHECKSUM_FINALIZE);
}

struct uint_struct {
    uint8_t v8;
    uint16_t v16;
    uint32_t v32;
    uint64_t v64;
};

static void
proc_uint_struct(struct proc *p, struct uint_struct *s)
{
    proc_bytes(p, &s->v8, 1);
    proc_bytes(p, &s->v16, 2);
    proc_bytes(p, &s->v32, 4);
    proc_bytes(p, &s->v64, 8);
}

static void
test_proc_uint(void)
{
    struct proc p;
    struct uint_struct in = {1, 2, 3, 4}, out = {0, 0, 0, 0};
    unsigned char in_buf[4096] = {0}, out_buf[4096] = {0}, sent[8];
    uint32_t h;

    CHECK(mchecksum_init("crc32c", &p.ck) == 0, "init crc32c");
    p.hash_size = mchecksum_get_size(p.ck);
    CHECK(p.hash_size == 4, "crc32c size");
    proc_reset(&p, in_buf, 1);
    proc_uint_struct(&p, &in);
    CHECK(proc_flush(&p) == 0, "flush");
    memcpy(sent, p.hash, p.hash_size);
    memcpy(&h, p.hash, 4);
    /* CRC-32C of 01 | 02 00 | 03 00 00 00 | 04 00*7 (tests/golden/test_proc.json) */
    CHECK(h == 0xEE017DA0u, "pinned crc32c of the uint struct image");

    memcpy(out_buf, in_buf, sizeof(in_buf)); /* simulate RPC copy */
    proc_reset(&p, out_buf, 0);
    proc_uint_struct(&p, &out);
    CHECK(proc_flush(&p) == 0, "flush decode");
    CHECK(memcmp(sent, p.hash, p.hash_size) == 0, "verify");
    CHECK(out.v8 == 1 && out.v16 == 2 && out.v32 == 3 && out.v64 == 4, "values survive");

    out_buf[5] ^= 0x40; /* one flipped bit in transit -> HG_CHECKSUM_ERROR */
    proc_reset(&p, out_buf, 0);
    proc_uint_struct(&p, &out);
    proc_flush(&p);
    CHECK(memcmp(sent, p.hash, p.hash_size) != 0, "corruption detected");
    mchecksum_destroy(p.ck);
}

static void
test_proc_string(void)
{
    /* hg_string_t "Hello": u64 length incl. NUL, bytes, is_const, is_owned
     * (src/proc_extra/mercury_proc_string.c:30-54) */
    struct proc p;
    unsigned char buf[64] = {0};
    uint64_t len = 6;
    char s[6] = "Hello";
    uint8_t is_const = 0, is_owned = 0;
    uint32_t h;

    CHECK(mchecksum_init("crc32c", &p.ck) == 0, "init");
    p.hash_size = 4;
    proc_reset(&p, buf, 1);
    proc_bytes(&p, &len, 8);
    proc_bytes(&p, s, 6);
    proc_bytes(&p, &is_const, 1);
    proc_bytes(&p, &is_owned, 1);
    proc_flush(&p);
    memcpy(&h, p.hash, 4);
    CHECK(h == 0x74AB61ACu, "pinned crc32c of the string image");
    mchecksum_destroy(p.ck);
}

/* hg_proc_save_ptr / hg_proc_restore_ptr as hg_proc_hg_bulk_t uses them
 * (src/mercury_proc_bulk.c:82-93 encode, :111-125 decode;
 * src/mercury_proc.c:277-335): save_ptr reserves buf_size bytes WITHOUT
 * hashing, the serializer fills them, restore_ptr hashes that same region.
 * The proc checksum must still equal one CRC over buf[0 : size_used) -- the
 * invariant the whole-buffer GPU batch entry points rely on. */
static unsigned char *
proc_save_ptr(struct proc *p, size_t n)
{
    unsigned char *r = p->ptr;
    p->ptr += n;
    return r;
}

static void
proc_restore_ptr(struct proc *p, const void *data, size_t n)
{
    mchecksum_update(p->ck, data, n);
}

static void
test_proc_bulk_save_restore(void)
{
    struct proc p;
    unsigned char in_buf[512] = {0}, out_buf[512] = {0}, sent[4];
    uint8_t flags = 3;
    uint64_t buf_size = 77, got_size = 0;
    uint32_t whole = 0, h = 0;
    size_t used, i;
    unsigned char *region;
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;

    CHECK(mchecksum_init("crc32c", &p.ck) == 0, "init");
    p.hash_size = 4;
    proc_reset(&p, in_buf, 1);
    proc_bytes(&p, &flags, 1);          /* a field before the handle */
    proc_bytes(&p, &buf_size, 8);       /* hg_proc_uint64_t(proc, &buf_size) */
    region = proc_save_ptr(&p, buf_size);
    for (i = 0; i < buf_size; i++)      /* HG_Bulk_serialize(buf, buf_size, ...) */
        region[i] = (unsigned char) (i * 37 + 11);
    proc_restore_ptr(&p, region, buf_size);
    proc_bytes(&p, &flags, 1);          /* and one after it */
    proc_flush(&p);
    used = (size_t) (p.ptr - p.buf);
    memcpy(sent, p.hash, 4);
    memcpy(&h, p.hash, 4);
    mchecksum_init("crc32c", &c);
    mchecksum_update(c, in_buf, used);  /* what a whole-buffer batch kernel hashes */
    mchecksum_get(c, &whole, 4, MCHECKSUM_FINALIZE);
    mchecksum_destroy(c);
    CHECK(used == 1 + 8 + 77 + 1, "size_used");
    CHECK(h == whole, "save_ptr/restore_ptr checksum == CRC of buf[0:size_used)");

    memcpy(out_buf, in_buf, used);      /* the receiver: decode, save_ptr, restore_ptr, verify */
    proc_reset(&p, out_buf, 0);
    proc_bytes(&p, &flags, 1);
    proc_bytes(&p, &got_size, 8);
    region = proc_save_ptr(&p, got_size);
    proc_restore_ptr(&p, region, got_size);
    proc_bytes(&p, &flags, 1);
    proc_flush(&p);
    CHECK(got_size == 77 && memcmp(sent, p.hash, 4) == 0, "decode side verifies");

    out_buf[40] ^= 1;                   /* a bit flipped inside the saved region */
    proc_reset(&p, out_buf, 0);
    proc_bytes(&p, &flags, 1);
    proc_bytes(&p, &got_size, 8);
    region = proc_save_ptr(&p, got_size);
    proc_restore_ptr(&p, region, got_size);
    proc_bytes(&p, &flags, 1);
    proc_flush(&p);
    CHECK(memcmp(sent, p.hash, 4) != 0, "corruption in the saved region detected");
    mchecksum_destroy(p.ck);
}

static void
test_methods_and_edges(void)
{
    static const struct {
        const char *m;
        size_t size;
        uint64_t check;
    } tab[] = {{"crc16", 2, 0xD0DB}, {"crc32c", 4, 0xE3069283u}, {"crc64", 8, 0x995DC9BBDF1939FAull}};
    size_t i;

    for (i = 0; i < sizeof(tab) / sizeof(tab[0]); i++) {
        mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
        uint64_t v = 0;
        unsigned char small[1];
        CHECK(mchecksum_init(tab[i].m, &c) == 0, tab[i].m);
        CHECK(mchecksum_get_size(c) == tab[i].size, "size");
        mchecksum_update(c, "1234", 4);
        mchecksum_update(c, "56789", 5);
        CHECK(mchecksum_get(c, &v, tab[i].size, MCHECKSUM_FINALIZE) == 0, "get");
        CHECK(v == tab[i].check, "catalogue check value through the ABI");
        CHECK(mchecksum_get(c, small, 1, MCHECKSUM_FINALIZE) != 0, "get into a too-small buffer fails");
        mchecksum_destroy(c);
    }
    {
        mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
        CHECK(mchecksum_init("adler32-nope", &c) != 0, "unknown method fails");
        CHECK(c == MCHECKSUM_OBJECT_NULL, "object untouched");
        CHECK(mchecksum_destroy(MCHECKSUM_OBJECT_NULL) == 0, "destroy(NULL) ok");
    }
}

/* Distinct objects from concurrent threads (no shared mutable state). */
#define NT 8
#define NB 64
static unsigned char g_data[NB][5000];
static uint32_t g_want[NB];

static void *
worker(void *arg)
{
    long t = (long) arg;
    int rep, b;
    mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;

    if (mchecksum_init("crc32c", &c) != 0)
        return (void *) 1;
    for (rep = 0; rep < 50; rep++)
        for (b = (int) t; b < NB; b += NT) {
            uint32_t h;
            size_t n = 100 + (size_t) b * 70, off = 0;
            mchecksum_reset(c);
            while (off < n) { /* per-field style: 1..8-byte updates plus a tail */
                size_t f = 1 + (off % 8);
                if (off + f > n)
                    f = n - off;
                mchecksum_update(c, g_data[b] + off, f);
                off += f;
            }
            mchecksum_get(c, &h, 4, MCHECKSUM_FINALIZE);
            if (h != g_want[b]) {
                mchecksum_destroy(c);
                return (void *) 2;
            }
        }
    mchecksum_destroy(c);
    return NULL;
}

static void
test_threads(void)
{
    pthread_t th[NT];
    long t;
    int b, i;

    for (b = 0; b < NB; b++) {
        mchecksum_object_t c = MCHECKSUM_OBJECT_NULL;
        for (i = 0; i < 5000; i++)
            g_data[b][i] = (unsigned char) (b * 131 + i * 7 + (i >> 5));
        mchecksum_init("crc32c", &c);
        mchecksum_update(c, g_data[b], 100 + (size_t) b * 70);
        mchecksum_get(c, &g_want[b], 4, MCHECKSUM_FINALIZE);
        mchecksum_destroy(c);
    }
    for (t = 0; t < NT; t++)
        pthread_create(&th[t], NULL, worker, (void *) t);
    for (t = 0; t < NT; t++) {
        void *r = NULL;
        pthread_join(th[t], &r);
        CHECK(r == NULL, "thread result");
    }
}

/* Large updates take the carry-less-multiply fold on AVX-512 VPCLMULQDQ CPUs
 * (crc32c from 1 KiB, other reflected models from 256 B); 1..8-byte field
 * updates never do.  Both must give the same value at every length. */
static void
test_fold_vs_fields(void)
{
    static const char *methods[] = {"crc32c", "crc64", "crc32", "crc16-arc"};
    static unsigned char buf[9000];
    size_t i, m, n;

    for (i = 0; i < sizeof(buf); i++)
        buf[i] = (unsigned char) (i * 197 + (i >> 7) * 13 + 5);
    for (m = 0; m < sizeof(methods) / sizeof(methods[0]); m++)
        for (n = 0; n + 3 <= sizeof(buf); n += 61) {
            mchecksum_object_t a = MCHECKSUM_OBJECT_NULL, b = MCHECKSUM_OBJECT_NULL;
            uint64_t ha = 0, hb = 0;
            size_t off = 0;
            CHECK(mchecksum_init(methods[m], &a) == 0 && mchecksum_init(methods[m], &b) == 0, "init");
            mchecksum_update(a, buf + 3, n); /* odd start: unaligned loads */
            while (off < n) {
                size_t f = 1 + (off % 8);
                if (off + f > n)
                    f = n - off;
                mchecksum_update(b, buf + 3 + off, f);
                off += f;
            }
            mchecksum_get(a, &ha, sizeof(ha), MCHECKSUM_FINALIZE);
            mchecksum_get(b, &hb, sizeof(hb), MCHECKSUM_FINALIZE);
            CHECK(ha == hb, "whole update (fold) == per-field updates");
            mchecksum_destroy(a);
            mchecksum_destroy(b);
        }
}

int
main(void)
{
    test_fold_vs_fields();
    test_proc_uint();
    test_proc_string();
    test_proc_bulk_save_restore();
    test_methods_and_edges();
    test_threads();
    if (failures) {
        fprintf(stderr, "%d failures\n", failures);
        return 1;
    }
    printf("mchecksum ABI: all checks passed\n");
    return 0;
}
