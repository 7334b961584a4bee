// Host check of the split CRC-64 queue plan (crc_gpu_device.h, SplitPlan):
// for many batch shapes and grids, the chunks tile the units exactly once,
// the units tile every payload's bytes exactly once (pieces of len / 2^psl),
// and whenever whole() is true every
// chunk holds whole payloads -- at most kSplitAcc, distinct mod kSplitAcc --
// which the in-workgroup combine needs.  Built with hipcc for the host only.
#include "crc_gpu_device.h"

#include <cstdio>
#include <vector>

static int fails = 0;
#define CHECK(c, ...)                       \
    do {                                    \
        if (!(c)) {                         \
            if (fails++ < 10) {             \
                printf("FAIL: " __VA_ARGS__); \
                printf("\n");               \
            }                               \
        }                                   \
    } while (0)

int main() {
    const uint32_t grids[] = {1, 3, 8, 64, 255, 256, 512};
    const uint64_t counts[] = {1, 2, 5, 63, 100, 1000, 2048, 8192, 20000};
    const uint32_t psls[] = {1, 2, 3, 4, 6};
    int shapes = 0, whole = 0;
    for (uint32_t grid : grids)
        for (uint64_t count : counts)
            for (uint32_t psl : psls) {
                const SplitPlan P(count, psl, grid);
                shapes++;
                // chunks tile [0, n)
                uint64_t next = 0;
                for (uint64_t id = 0; id < P.nch; id++) {
                    const uint64_t st = P.start(id), sz = P.size(id);
                    CHECK(st == next, "chunk %llu starts at %llu, expected %llu", (unsigned long long)id,
                          (unsigned long long)st, (unsigned long long)next);
                    CHECK(sz <= (1u << P.cl), "chunk larger than its slots");
                    next = st + sz < P.n ? st + sz : P.n;
                }
                CHECK(next == P.n, "chunks end at %llu of %llu units (grid %u count %llu psl %u)",
                      (unsigned long long)next, (unsigned long long)P.n, grid, (unsigned long long)count, psl);
                // units tile every payload in pieces of len / 2^psl
                const uint32_t gran = 1u << P.psl;
                std::vector<uint8_t> cover(count * gran, 0);
                for (uint64_t u = 0; u < P.n; u++) {
                    uint64_t p;
                    uint32_t q;
                    P.unit(u, &p, &q);
                    CHECK(p < count && q < gran, "unit %llu out of range", (unsigned long long)u);
                    if (p >= count) continue;
                    cover[p * gran + q]++;
                }
                for (uint64_t i = 0; i < cover.size(); i++)
                    CHECK(cover[i] == 1, "granule %llu covered %d times (grid %u count %llu psl %u)",
                          (unsigned long long)i, cover[i], grid, (unsigned long long)count, psl);
                if (!P.whole()) continue;
                whole++;
                for (uint64_t id = 0; id < P.nch; id++) {
                    const uint64_t st = P.start(id), en = st + P.size(id) < P.n ? st + P.size(id) : P.n;
                    std::vector<uint64_t> pays;
                    std::vector<uint32_t> seen;
                    for (uint64_t u = st; u < en; u++) {
                        uint64_t p;
                        uint32_t q;
                        P.unit(u, &p, &q);
                        if (pays.empty() || pays.back() != p) {
                            pays.push_back(p);
                            seen.push_back(0);
                        }
                        seen.back()++;
                        CHECK(q + 1 == seen.back(), "pieces of a payload out of order in a chunk");
                    }
                    CHECK(pays.size() <= kSplitAcc, "chunk with %zu payloads", pays.size());
                    for (size_t k = 0; k < pays.size(); k++) {
                        CHECK(seen[k] == gran, "payload %llu split over chunks (%u of %u pieces)",
                              (unsigned long long)pays[k], seen[k], gran);
                        for (size_t j = 0; j < k; j++)
                            CHECK((pays[j] & (kSplitAcc - 1)) != (pays[k] & (kSplitAcc - 1)),
                                  "two payloads of a chunk share an accumulator");
                    }
                }
            }
    // C3's shape: 4 pieces per payload, whole-payload chunks
    const SplitPlan c3(8192, 2, 256);
    CHECK(c3.whole() && c3.n == 8192 * 4 && c3.cl == 5 && c3.sl == 2, "C3 plan: n %llu cl %u sl %u",
          (unsigned long long)c3.n, c3.cl, c3.sl);
    printf("split plan: %d shapes (%d whole-chunk), %d failures\n", shapes, whole, fails);
    return fails ? 1 : 0;
}
