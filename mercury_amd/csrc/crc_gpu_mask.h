/*
 * crc_gpu_mask.h -- edge handling of the batch kernels, shared verbatim by the
 * HIP kernels and the CPU emulator (tests/native/kernel_emulator.cpp) so the
 * emulator checks the exact code the GPU runs.
 *
 * A kernel reads whole aligned words; for a word whose first byte sits at
 * payload-relative position lo (it may be negative or past the end):
 *   - bytes outside the payload [0, len) are cleared (leading bytes before the
 *     payload keep the zero register at zero; trailing pad bytes are undone
 *     later by the Z^-t operator);
 *   - for len >= W/8 the initial register is XORed into payload bytes
 *     [0, W/8): R(init, M) == R(0, M ^ init) for a W-bit CRC.
 * Word byte i holds payload byte lo + i, so init byte j lands on word byte
 * j - lo: a right shift by lo bytes when lo >= 0, a left shift otherwise.
 */
#ifndef CRC_GPU_MASK_H
#define CRC_GPU_MASK_H

#include <stdint.h>

#if defined(__HIPCC__)
#    define MCK_HD __host__ __device__ __forceinline__
#else
#    define MCK_HD static inline
#endif

MCK_HD uint32_t
mck_mask32(uint32_t w, int64_t lo, int64_t len, uint32_t init)
{
    if (lo >= len || lo <= -4)
        return 0;
    const int sc = lo < 0 ? (int) (-lo) : 0;
    const int64_t e = lo + 4 - len;
    const int ec = e > 0 ? (int) e : 0;
    w &= (0xFFFFFFFFu << (8 * sc)) & (0xFFFFFFFFu >> (8 * ec));
    if (len >= 4 && lo < 4)
        w ^= lo >= 0 ? (init >> (8 * (int) lo)) : (init << (8 * (int) (-lo)));
    return w;
}

MCK_HD uint64_t
mck_mask64(uint64_t w, int64_t lo, int64_t len, uint64_t init)
{
    if (lo >= len || lo <= -8)
        return 0;
    const int sc = lo < 0 ? (int) (-lo) : 0;
    const int64_t e = lo + 8 - len;
    const int ec = e > 0 ? (int) e : 0;
    w &= (~0ULL << (8 * sc)) & (~0ULL >> (8 * ec));
    if (len >= 8 && lo < 8)
        w ^= lo >= 0 ? (init >> (8 * (int) lo)) : (init << (8 * (int) (-lo)));
    return w;
}

/* True when a 16-byte piece at payload-window offset pc (window offsets are
 * relative to the aligned window start a0; the payload is [hs, he)) needs no
 * edge handling: it lies wholly inside the payload and past the init bytes. */
MCK_HD int
mck_piece_clean(int64_t pc, int64_t hs, int64_t he, int wbytes)
{
    return pc >= hs + wbytes && pc + 16 <= he;
}

#endif
