// kernel_emulator.cpp -- TEST ONLY.  Scalar emulation of the lane-parallel
// batch-CRC algorithm that mercury_amd/csrc/mchecksum_gpu.hip runs on CDNA4,
// using the very same host-built table packs (crc_tables.c).  It validates the
// algebra (window alignment, sub-stream folding, tree combine, tail undo,
// init handling) on the CPU against the oracle; the GPU parity tests then
// cover what is GPU-specific (LDS layout, v_perm addressing, shuffles).
#include "../../mercury_amd/csrc/crc_gpu_layout.h"
#include "../../mercury_amd/csrc/crc_gpu_mask.h"
#include "../../oracle/crc_oracle.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static uint32_t op32(const crc32_gpu_pack_t &pk, int o, uint32_t x) {
    uint32_t r = 0;
    for (int h = 0; h < 8; h++) r ^= pk.ops[o][h][(x >> (4 * h)) & 15];
    return r;
}
static uint64_t op64(const crc64_gpu_pack_t &pk, int o, uint64_t x) {
    uint64_t r = 0;
    for (int h = 0; h < 16; h++) r ^= pk.ops[o][h][(x >> (4 * h)) & 15];
    return r;
}

// Raw little-endian word at absolute position wa of buf[0, nbuf) (bytes past
// the buffer read as 0) -- neighbouring payloads' bytes included, exactly as
// the kernel's aligned loads see them; edge handling is crc_gpu_mask.h's.
template <typename T>
static T raw_word(const uint8_t *buf, int64_t nbuf, int64_t wa) {
    T w = 0;
    for (int i = 0; i < (int)sizeof(T); i++)
        if (wa + i >= 0 && wa + i < nbuf) w |= (T)buf[wa + i] << (8 * i);
    return w;
}

// End of the step grid: the payload's end rounded up to 16 B, or -- with
// EMU_GRID_ALIGN=128, the one-payload-per-wave loops (G = 64) of round 3 --
// to the 128-B line, so every step covers whole lines.
static int64_t grid_end(int64_t end, int log2g) {
    const char *e = getenv("EMU_GRID_ALIGN");
    const int64_t al = log2g == 6 && e && atoi(e) == 128 ? 128 : 16;
    return (end + al - 1) & ~(al - 1);
}

// CRC of payload buf[start, start+len) as the kernel computes it.
extern "C" uint32_t emu_crc32(const crc32_gpu_pack_t *pk, const uint8_t *buf, int64_t nbuf, int64_t start,
                              int64_t len) {
    const int log2g = (int)pk->log2g, G = 1 << log2g;
    const int64_t step = 16LL * G;
    int64_t a0 = start & ~15LL, a1 = grid_end(start + len, log2g), t = a1 - (start + len);
    int64_t W = a1 - a0, K = (W + step - 1) / step, r0 = W - K * step;
    int64_t hs = start - a0, he = start + len - a0;
    std::vector<uint32_t> S(4 * G, 0);
    for (int64_t k = 0; k < K; k++)
        for (int l = 0; l < G; l++) {
            int64_t pc = r0 + k * step + 16 * l;
            uint32_t w[4] = {0, 0, 0, 0};
            if (pc >= 0)
                for (int j = 0; j < 4; j++) w[j] = raw_word<uint32_t>(buf, nbuf, a0 + pc + 4 * j);
            if (!mck_piece_clean(pc, hs, he, 4))
                for (int j = 0; j < 4; j++) w[j] = mck_mask32(w[j], pc - hs + 4 * j, len, pk->init);
            for (int j = 0; j < 4; j++) {
                uint32_t x = S[4 * l + j] ^ w[j];
                S[4 * l + j] = pk->main[0][x & 255] ^ pk->main[1][(x >> 8) & 255] ^ pk->main[2][(x >> 16) & 255] ^
                               pk->main[3][x >> 24];
            }
        }
    std::vector<uint32_t> X(G);
    for (int l = 0; l < G; l++) {
        uint32_t a = S[4 * l] ^ op32(*pk, 0, S[4 * l + 1]);
        uint32_t b = S[4 * l + 2] ^ op32(*pk, 0, S[4 * l + 3]);
        X[l] = a ^ op32(*pk, 1, b);
    }
    if (log2g == 6 && !getenv("EMU_BUTTERFLY")) {  // two-level combine (throughput layout, G = 64)
        uint32_t acc = 0;
        for (int a = 0; a < 8; a++) {
            uint32_t grp = 0;
            for (int b = 0; b < 8; b++) {
                uint32_t r = 0;
                for (int h = 0; h < 8; h++) r ^= pk->lv[0][h][(X[8 * a + b] >> (4 * h)) & 15][b];
                grp ^= r;
            }
            uint32_t r = 0;
            for (int h = 0; h < 8; h++) r ^= pk->lv[1][h][(grp >> (4 * h)) & 15][a];
            acc ^= r;
        }
        X[0] = acc;
    } else {
        for (int k = 0; k < log2g; k++) {  // butterfly, as the shuffles do it
            std::vector<uint32_t> Y(G);
            for (int l = 0; l < G; l++) {
                uint32_t other = X[l ^ (1 << k)];
                bool bit = (l >> k) & 1;
                uint32_t lo = bit ? other : X[l], hi = bit ? X[l] : other;
                Y[l] = lo ^ op32(*pk, 2 + k, hi);
            }
            X = Y;
        }
    }
    // pad undo Z^-t, t = 16q + r (q > 0 only on the 128-B grid, G = 64)
    uint32_t r = op32(*pk, 2 + log2g + (int)(t & 15), X[0]);
    for (int k = 0; k < 3; k++)
        if ((t >> (4 + k)) & 1) r = op32(*pk, 2 + k, r);
    if (len < 4) r ^= pk->zinit[len];
    return r ^ pk->xorout;
}

extern "C" uint64_t emu_crc64(const crc64_gpu_pack_t *pk, const uint8_t *buf, int64_t nbuf, int64_t start,
                              int64_t len) {
    const int log2g = (int)pk->log2g, G = 1 << log2g;
    const int64_t step = 16LL * G;
    int64_t a0 = start & ~15LL, a1 = grid_end(start + len, log2g), t = a1 - (start + len);
    int64_t W = a1 - a0, K = (W + step - 1) / step, r0 = W - K * step;
    int64_t hs = start - a0, he = start + len - a0;
    std::vector<uint64_t> S(2 * G, 0);
    for (int64_t k = 0; k < K; k++)
        for (int l = 0; l < G; l++) {
            int64_t pc = r0 + k * step + 16 * l;
            uint64_t w[2] = {0, 0};
            if (pc >= 0)
                for (int j = 0; j < 2; j++) w[j] = raw_word<uint64_t>(buf, nbuf, a0 + pc + 8 * j);
            if (!mck_piece_clean(pc, hs, he, 8))
                for (int j = 0; j < 2; j++) w[j] = mck_mask64(w[j], pc - hs + 8 * j, len, pk->init);
            for (int j = 0; j < 2; j++) {
                uint64_t x = S[2 * l + j] ^ w[j], r = 0, r6 = 0;
                for (int p = 0; p < 8; p++)
                    for (int h = 0; h < 2; h++) r ^= pk->main[2 * p + h][(x >> (8 * p + 4 * h)) & 15];
                // the kernels' 12-lookup form (f5 / f6) of the same fold
                for (int p = 0; p < 8; p++) r6 ^= pk->f5[p][(x >> (8 * p + 3)) & 31];
                for (int i = 0; i < 4; i++)
                    r6 ^= pk->f6[i][((x >> (8 * i)) & 7) | (((x >> (8 * i + 32)) & 7) << 3)];
                if (r6 != r) {
                    std::fprintf(stderr, "emu_crc64: the f5/f6 fold differs from the nibble fold\n");
                    std::abort();
                }
                S[2 * l + j] = r6;
            }
        }
    std::vector<uint64_t> X(G);
    for (int l = 0; l < G; l++) X[l] = S[2 * l] ^ op64(*pk, 0, S[2 * l + 1]);
    for (int k = 0; k < log2g; k++) {
        std::vector<uint64_t> Y(G);
        for (int l = 0; l < G; l++) {
            uint64_t other = X[l ^ (1 << k)];
            bool bit = (l >> k) & 1;
            uint64_t lo = bit ? other : X[l], hi = bit ? X[l] : other;
            Y[l] = lo ^ op64(*pk, 1 + k, hi);
        }
        X = Y;
    }
    uint64_t r = op64(*pk, 1 + log2g + (int)(t & 15), X[0]);
    for (int k = 0; k < 3; k++)
        if ((t >> (4 + k)) & 1) r = op64(*pk, 1 + k, r);
    if (len < 8) r ^= pk->zinit[len];
    return r ^ pk->xorout;
}

#ifdef EMULATOR_MAIN
int main() {
    const oracle_model_t *m32 = oracle_model_by_name("crc32c");
    const oracle_model_t *m64 = oracle_model_by_name("crc64");
    crc_rmodel_t r32 = {32, 0x82F63B78ULL, 0xFFFFFFFFULL, 0xFFFFFFFFULL};
    crc_rmodel_t r64 = {64, 0xC96C5795D7870F42ULL, ~0ULL, ~0ULL};
    std::vector<uint8_t> buf(70000);
    oracle_fill_splitmix(buf.data(), buf.size(), 0x1234, 0);
    int fails = 0, n = 0;
    for (int lg = 0; lg <= 6; lg++) {
        static crc32_gpu_pack_t p32;
        static crc64_gpu_pack_t p64;
        if (crc32_gpu_pack_build(&r32, lg, &p32) || crc64_gpu_pack_build(&r64, lg, &p64)) {
            printf("pack build failed\n");
            return 1;
        }
        for (int64_t len : {0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 31, 63, 64, 65, 255, 256, 1023, 1024, 1025, 4096, 4097,
                            65535, 65536})
            for (int64_t start : {0, 1, 2, 3, 4, 5, 7, 8, 11, 12, 13, 15, 16, 33}) {
                if (start + len > (int64_t)buf.size()) continue;
                uint32_t e32 = (uint32_t)oracle_crc_table(m32, buf.data() + start, len);
                uint64_t e64 = oracle_crc_table(m64, buf.data() + start, len);
                uint32_t g32 = emu_crc32(&p32, buf.data(), (int64_t)buf.size(), start, len);
                uint64_t g64 = emu_crc64(&p64, buf.data(), (int64_t)buf.size(), start, len);
                n++;
                if (e32 != g32) { fails++; if (fails < 10) printf("crc32 lg=%d len=%ld start=%ld %08x vs %08x\n", lg, (long)len, (long)start, g32, e32); }
                if (e64 != g64) { fails++; if (fails < 10) printf("crc64 lg=%d len=%ld start=%ld %016lx vs %016lx\n", lg, (long)len, (long)start, (unsigned long)g64, (unsigned long)e64); }
            }
    }
    // MSB-first model (CRC-64/ECMA-182, refin = refout = false): the kernels run
    // the reflected model of the same polynomial conjugated by the per-byte bit
    // reversal R (crc_gpu_layout.h); the output is the CRC byte-swapped
    const oracle_model_t *me = oracle_model_by_name("crc64-ecma182");
    auto refl = [](uint64_t v, int w) { uint64_t r = 0; for (int i = 0; i < w; i++) if ((v >> i) & 1) r |= 1ULL << (w - 1 - i); return r; };
    crc_rmodel_t rme = {64, refl(0x42F0E1EBA9EA3693ULL, 64), crc_rev_bytes(64, refl(0, 64)), crc_rev_bytes(64, refl(0, 64)), 1};
    for (int lg : {0, 3, 6}) {
        static crc64_gpu_pack_t pe;
        if (crc64_gpu_pack_build(&rme, lg, &pe)) {
            printf("msb pack build failed\n");
            return 1;
        }
        for (int64_t len : {0, 1, 7, 8, 9, 63, 64, 65, 1023, 1024, 4097, 65536})
            for (int64_t start : {0, 1, 5, 8, 13, 16}) {
                uint64_t e = oracle_crc_table(me, buf.data() + start, len);
                uint64_t g = __builtin_bswap64(emu_crc64(&pe, buf.data(), (int64_t)buf.size(), start, len));
                n++;
                if (e != g) { fails++; if (fails < 10) printf("crc64-ecma182 lg=%d len=%ld start=%ld %016lx vs %016lx\n", lg, (long)len, (long)start, (unsigned long)g, (unsigned long)e); }
            }
    }
    // MSB-first models with non-zero init and/or xorout (not in the product
    // catalogue): their init and xorout map into the byte-reversed
    // register domain exactly as mchecksum_gpu.hip's gpu_rmodel does --
    // rinit = R(reflect(init)), xorout = R(reflect(xorout)).  Catalogue
    // check values pin the synthetic models themselves.
    static const oracle_model_t msbz[] = {
        {"crc64-we", 64, 0x42F0E1EBA9EA3693ULL, 0, 0, ~0ULL, ~0ULL, 0x62EC59E3F1A4F00AULL},
        {"crc32-bzip2", 32, 0x04C11DB7ULL, 0, 0, 0xFFFFFFFFULL, 0xFFFFFFFFULL, 0xFC891918ULL},
        {"crc32-mpeg2", 32, 0x04C11DB7ULL, 0, 0, 0xFFFFFFFFULL, 0ULL, 0x0376E6E7ULL},
    };
    for (const oracle_model_t &mm : msbz) {
        if (oracle_crc_bitwise(&mm, "123456789", 9) != mm.check) {
            fails++;
            printf("%s: check value differs\n", mm.name);
            continue;
        }
        const int w = mm.width;
        crc_rmodel_t rm = {w, refl(mm.poly, w), crc_rev_bytes(w, refl(mm.init, w)), crc_rev_bytes(w, refl(mm.xorout, w)), 1};
        for (int lg : {0, 3, 6}) {
            static crc32_gpu_pack_t q32;
            static crc64_gpu_pack_t q64;
            if (w == 32 ? crc32_gpu_pack_build(&rm, lg, &q32) : crc64_gpu_pack_build(&rm, lg, &q64)) {
                printf("%s pack build failed\n", mm.name);
                return 1;
            }
            for (int64_t len : {0, 1, 3, 4, 5, 7, 8, 9, 63, 64, 65, 1023, 1024, 4097, 65536})
                for (int64_t start : {0, 1, 5, 8, 13, 16}) {
                    const uint64_t e = oracle_crc_table(&mm, buf.data() + start, len);
                    const uint64_t g = w == 32 ? __builtin_bswap32(emu_crc32(&q32, buf.data(), (int64_t)buf.size(), start, len))
                                               : __builtin_bswap64(emu_crc64(&q64, buf.data(), (int64_t)buf.size(), start, len));
                    n++;
                    if (e != g) { fails++; if (fails < 10) printf("%s lg=%d len=%ld start=%ld %016lx vs %016lx\n", mm.name, lg, (long)len, (long)start, (unsigned long)g, (unsigned long)e); }
                }
        }
    }
    printf("%d cases, %d failures\n", n, fails);
    return fails != 0;
}
#endif

// ctypes entry points for tests/test_emulator.py
extern "C" void *emu_pack32(int log2g) {
    auto *p = new crc32_gpu_pack_t;
    crc_rmodel_t r = {32, 0x82F63B78ULL, 0xFFFFFFFFULL, 0xFFFFFFFFULL};
    if (crc32_gpu_pack_build(&r, log2g, p)) { delete p; return nullptr; }
    return p;
}
extern "C" void *emu_pack64(int log2g) {
    auto *p = new crc64_gpu_pack_t;
    crc_rmodel_t r = {64, 0xC96C5795D7870F42ULL, ~0ULL, ~0ULL};
    if (crc64_gpu_pack_build(&r, log2g, p)) { delete p; return nullptr; }
    return p;
}
extern "C" void emu_pack_free32(void *p) { delete (crc32_gpu_pack_t *)p; }
extern "C" void emu_pack_free64(void *p) { delete (crc64_gpu_pack_t *)p; }
