/*
 * mchecksum_gpu.h -- MI355X batch entry points of libmchecksum.
 *
 * These are ADDITIONAL extern "C" entry points next to the unchanged
 * mchecksum streaming API (<mchecksum.h>).  Where Mercury streams the bytes
 * of one serialized proc buffer through mchecksum_update/get
 * (src/mercury_proc.c:387-406, 358-384), a batch entry point computes the
 * same value for many independent, device-resident payloads at once:
 *
 *   value[i] == mchecksum_get() after mchecksum_update(payload_i, len_i)
 *
 * bit for bit, for every method the GPU supports (every 32/64-bit catalogue
 * method: crc32c, crc32, crc64 and its variants, MSB-first ECMA-182 included).  The
 * whole-buffer form is exact because, in Mercury's default non-XDR build, the
 * proc checksum is the CRC of the contiguous serialized bytes
 * buf[0 : hg_proc_get_size_used) (src/mercury_proc.h:124-143,162-181;
 * SURVEY.md 0.4).  It is NOT exact for a Mercury built with XDR encoding:
 * hash such buffers with mchecksum_gpu_checksum_xdr() below.
 *
 * Memory: dev_base, dev_offsets and dev_out are device pointers (hipMalloc or
 * any device-accessible allocation).  Payload bytes are read in aligned
 * 16-byte granules, so the allocation must be readable up to the next 16-byte
 * boundary after the last payload byte (hipMalloc allocations always are).
 * dev_out receives `count` host-order integers of the method's size
 * (uint32_t for crc32c, uint64_t for crc64).
 *
 * Streams: `stream` is a hipStream_t (NULL = the default stream).  Calls are
 * asynchronous and capture-safe once mchecksum_gpu_prepare() has run for the
 * method on the current device (it uploads the lookup tables).  Large batches
 * balance their payloads through a device-side work-queue slot: each launch
 * takes an idle one of the device's 2048 slots and holds it until it
 * completes (a HIP event recorded by the launch's completion, queried without
 * blocking), so no slot ever serves two launches at once -- whatever the
 * streams, host threads, stream handle reuse or hipStreamDestroy timing.
 * Calls captured into a hipGraph, and calls that find the oldest in-flight
 * slots all still busy with no idle one left, take a plain static split of
 * the batch instead: a graph replays its captured arguments, possibly on two
 * execs at once, so no slot could be exclusive to it.  Destroying a stream
 * with calls in flight follows the HIP rules for the memory those calls use;
 * the library itself keeps no per-stream state.
 *
 * Fail closed: every wait on the device is bounded, and so is every call.  A
 * wait gives up after 1 s of real time (time the wave spends switched out of
 * the GPU does not count); once one wait of a call has given up, every other
 * wait of that call gives up at once (the launch's abort flag; a segments
 * call whose scan gave up hashes nothing more), so a call that meets any
 * number of stalls still returns within about one deadline.  A call in which
 * a wait gave up (a protocol fault; 0 in every test run) adds 1 -- once per
 * call -- to the error word set with mchecksum_gpu_set_error_word(), adds
 * `count` to the mismatch counter of a verify call and marks every payload it
 * cannot vouch for with status 1, so unhashed bytes never read as verified.
 *
 * Settings: the MCHECKSUM_* environment variables (variants, log level, the
 * MCHECKSUM_GPU_* launch-policy overrides of the A/B tools) are read once,
 * at the library's first use, never on the call path.
 *
 * There is NO host fallback: without a usable HIP device every call returns
 * MCHECKSUM_GPU_ENODEV.
 */
#ifndef MCHECKSUM_GPU_H
#define MCHECKSUM_GPU_H

#include <stddef.h>
#include <stdint.h>

#include "mchecksum.h"

#define MCHECKSUM_GPU_OK        0
#define MCHECKSUM_GPU_EINVAL    (-1) /* bad argument */
#define MCHECKSUM_GPU_ENODEV    (-2) /* no usable HIP device */
#define MCHECKSUM_GPU_EMETHOD   (-3) /* method not supported on GPU (16-bit methods on the
                                         payload paths; MSB-first ones on XDR) */
#define MCHECKSUM_GPU_EHIP      (-4) /* HIP runtime error (see error string) */

#ifdef __cplusplus
extern "C" {
#endif

/* 1 if a HIP device is usable by this process, else 0. */
MCHECKSUM_PUBLIC int
mchecksum_gpu_available(void);

/* Build and upload the lookup tables for hash_method on the current device:
 * the payload kernels' packs and the Z^n shift pack (32/64-bit models), or
 * the core-header byte table (16-bit models).  Optional (done lazily on first
 * use); call it before hipGraph capture -- a first use inside a capture
 * would upload tables there and invalidate the capture. */
MCHECKSUM_PUBLIC int
mchecksum_gpu_prepare(const char *hash_method);

/* Fixed-size batch: payload i = dev_base[i*stride, i*stride + len), i < count.
 * (Every batch entry point takes at most 2^31 payloads per call.) */
MCHECKSUM_PUBLIC int
mchecksum_gpu_checksum_fixed(const char *hash_method, const void *dev_base,
    size_t stride, size_t len, size_t count, void *dev_out, void *stream);

/* Variable-size batch: payload i = dev_base[dev_offsets[i], dev_offsets[i+1]),
 * i < count; dev_offsets holds count + 1 non-decreasing byte offsets
 * (the C4 "offsets table" layout; payloads may start at any byte). */
MCHECKSUM_PUBLIC int
mchecksum_gpu_checksum_offsets(const char *hash_method, const void *dev_base,
    const uint64_t *dev_offsets, size_t count, void *dev_out, void *stream);

/* Batched verify of received payloads against expected values (e.g. the
 * payload hash carried in the 4-byte HG header, src/mercury_header.c:111-112,
 * after ntohl): dev_status[i] = 1 if CRC(payload i) != dev_expected[i] else 0,
 * and *dev_mismatches (device uint32) is incremented by the number of
 * mismatches (caller zeroes it).  dev_expected holds host-order values of the
 * method's size.  Either status pointer may be NULL. */
MCHECKSUM_PUBLIC int
mchecksum_gpu_verify_offsets(const char *hash_method, const void *dev_base,
    const uint64_t *dev_offsets, size_t count, const void *dev_expected,
    uint8_t *dev_status, uint32_t *dev_mismatches, void *stream);

/* Batched verify of received RPC messages in place.
 * Message i = dev_buf[dev_msg_offsets[i], dev_msg_offsets[i+1]) as it sits in
 * an NA multi-recv buffer (src/mercury_core.c:2092-2132, 4667-4714): headers,
 * then the serialized payload from payload_offset on.  The expected CRC is
 * the network-order u32 at hash_offset -- in Mercury the HG header's payload
 * hash (src/mercury_header.c:111-112) right after the 16-byte core header, so
 * hash_offset = 16 and payload_offset = 20 for HG_INPUT without user offset.
 * dev_status[i] = 1 when the payload CRC differs (what hg_get_struct reports
 * as HG_CHECKSUM_ERROR, src/mercury.c:565-573) or the message is shorter than
 * payload_offset; *dev_mismatches is incremented per failure.  crc32c only
 * (the header slot is 32 bits). */
MCHECKSUM_PUBLIC int
mchecksum_gpu_verify_messages(const char *hash_method, const void *dev_buf,
    const uint64_t *dev_msg_offsets, size_t count, size_t payload_offset,
    size_t hash_offset, uint8_t *dev_status, uint32_t *dev_mismatches,
    void *stream);

/* Scatter-gather objects: object j is the
 * concatenation, in order, of segments [dev_obj_first[j], dev_obj_first[j+1])
 * of the segment list (dev_seg_addr[s], dev_seg_len[s]) -- the shape of a bulk
 * handle's segments, HG_Bulk_create(count, buf_ptrs, buf_sizes)
 * (src/mercury_bulk.h:55,79), registered as device memory (hg_bulk_attr
 * mem_type HG_MEM_TYPE_ROCM, src/mercury_types.h:38,44-47).  dev_out[j] =
 * mchecksum_get() after one mchecksum_update() per segment of object j
 * (count = nobj host-order values; an object with no bytes gets the CRC of the
 * empty message).  All arrays are device-resident: dev_seg_addr holds device
 * addresses (each segment readable to its next 16-byte boundary),
 * dev_obj_first holds nobj + 1 non-decreasing indices <= nseg; segments
 * outside [first[0], first[nobj]) are ignored.  dev_work: caller-owned device
 * scratch (8-byte aligned) of at least mchecksum_gpu_segments_work_size(nseg)
 * bytes, not shared with a concurrent call (SIZE_MAX for nseg > 2^40, which
 * is rejected).  Every 32/64-bit method.  Segments are
 * cut into 256 KiB chunks hashed in parallel and recombined with GF(2) shift
 * operators, so one huge segment still spreads over the whole GPU. */
MCHECKSUM_PUBLIC size_t
mchecksum_gpu_segments_work_size(size_t nseg);

MCHECKSUM_PUBLIC int
mchecksum_gpu_checksum_segments(const char *hash_method,
    const uint64_t *dev_seg_addr, const uint64_t *dev_seg_len, size_t nseg,
    const uint64_t *dev_obj_first, size_t nobj, void *dev_work,
    size_t work_size, void *dev_out, void *stream);

/* Batched check of Mercury core headers for received
 * messages in device memory: message i = dev_buf[dev_msg_offsets[i],
 * dev_msg_offsets[i+1]) starts with the 16-byte core header that
 * hg_core_header_request_proc / _response_proc encode
 * (src/mercury_core_header.c:175-289).  The 16-bit hash_method ("crc16") is
 * recomputed over the host-order field values exactly as those functions
 * stream them into mchecksum_update and compared with the big-endian hash on
 * the wire (request: offset 12, response: offset 4).  dev_status[i] = 1 on a
 * mismatch or a message shorter than 16 bytes (HG_CHECKSUM_ERROR /
 * HG_INVALID_ARG in Mercury); *dev_mismatches is incremented per failure. */
#define MCHECKSUM_GPU_CORE_HEADER_REQUEST  0
#define MCHECKSUM_GPU_CORE_HEADER_RESPONSE 1
MCHECKSUM_PUBLIC int
mchecksum_gpu_verify_core_headers(const char *hash_method, int kind,
    const void *dev_buf, const uint64_t *dev_msg_offsets, size_t count,
    uint8_t *dev_status, uint32_t *dev_mismatches, void *stream);

/* XDR-mode proc checksum.  In a Mercury built with
 * MERCURY_USE_XDR (HG_HAS_XDR) the serialized buffer holds XDR -- every
 * integer big-endian and rounded up to 4 bytes, byte arrays zero-padded to a
 * multiple of 4 -- while the proc checksum covers the HOST-order field values
 * (src/mercury_proc.h:110-122,147-160).  The whole-buffer entry points above
 * are exact only for the default non-XDR encoding; they cannot tell an XDR
 * buffer apart and must not be used on one.  This entry point takes the
 * message's field schema instead, the sequence of hg_proc_* calls its proc
 * function makes:
 *   MCHECKSUM_XDR_INT         size 1, 2, 4 or 8: hg_proc_[u]int<8*size>_t
 *                             (wire: 4 or 8 bytes big-endian; hashed: the
 *                             size little-endian bytes of the value)
 *   MCHECKSUM_XDR_OPAQUE      size bytes of hg_proc_bytes/raw/memcpy (wire:
 *                             the bytes + zero pad to a multiple of 4)
 *   MCHECKSUM_XDR_OPAQUE_LEN  as OPAQUE, byte count = the value of the last
 *                             INT field (hg_string_t: u64 length, then bytes)
 *   MCHECKSUM_XDR_RAW         size bytes reserved by hg_proc_save_ptr and
 *                             hashed by hg_proc_restore_ptr (exact size, no
 *                             XDR rounding; src/mercury_proc.c:277-335)
 *   MCHECKSUM_XDR_RAW_LEN     as RAW, size = the last INT field's value
 *                             (bulk handles, src/mercury_proc_bulk.c:91-125)
 *   MCHECKSUM_XDR_SKIP_IF_ZERO if the last INT field was 0, skip the next
 *                             `size` schema entries (an empty hg_string_t
 *                             carries no bytes and no flags)
 * Message i = dev_buf[dev_msg_offsets[i], dev_msg_offsets[i+1]) starting
 * where the proc buffer starts; dev_out[i] = the value hg_proc_checksum_get
 * returns for it (host-order, method size).  dev_status[i] (optional) = 1
 * when the schema runs past the message (dev_out[i] is then 0).  At most 64
 * schema entries; reflected 32/64-bit methods (crc32c, crc64). */
#define MCHECKSUM_XDR_INT          0
#define MCHECKSUM_XDR_OPAQUE       1
#define MCHECKSUM_XDR_OPAQUE_LEN   2
#define MCHECKSUM_XDR_RAW          3
#define MCHECKSUM_XDR_RAW_LEN      4
#define MCHECKSUM_XDR_SKIP_IF_ZERO 5
typedef struct mchecksum_xdr_field {
    uint32_t kind;
    uint32_t size;
} mchecksum_xdr_field_t;

MCHECKSUM_PUBLIC int
mchecksum_gpu_checksum_xdr(const char *hash_method,
    const mchecksum_xdr_field_t *fields, size_t nfields, const void *dev_buf,
    const uint64_t *dev_msg_offsets, size_t count, void *dev_out,
    uint8_t *dev_status, void *stream);

/* Lanes cooperating on one payload that checksum_fixed would choose for
 * this length (1..64) in a batch large enough to fill the device; a smaller
 * batch gets more lanes per payload until it fills every wave slot (a small
 * one in the light layout may get fewer).  For reporting; -1 on error. */
MCHECKSUM_PUBLIC int
mchecksum_gpu_lanes_per_payload(const char *hash_method, size_t len);

/* Fail-closed report for the batch calls this host thread makes from now on:
 * each call whose launch could not hash every payload adds 1 to *dev_word
 * (a device-resident uint32_t the caller owns, zeroes and reads after the
 * calls' streams are synchronized).  The word is captured by value into
 * graph-captured calls.  NULL (the default) turns the report off; the
 * process-wide count mchecksum_gpu_queue_faults() is always kept. */
MCHECKSUM_PUBLIC int
mchecksum_gpu_set_error_word(uint32_t *dev_word);

/* Human-readable text for the last error on this thread. */
MCHECKSUM_PUBLIC const char *
mchecksum_gpu_last_error(void);

/* Re-read the MCHECKSUM_* environment settings (normally read once, at first
 * use) for calls made from now on -- for tests and tuning tools that change
 * the environment between calls; calls already made are not affected. */
MCHECKSUM_PUBLIC void
mchecksum_gpu_reload_settings(void);

/* Diagnostics: the number of work-queue protocol faults the batch kernels
 * counted on the current device since the library was loaded (0 in a
 * healthy run; every wait inside a launch is bounded, and a wait that gives
 * up is counted here instead of hanging the GPU).  Synchronizes the device.
 * Returns -1 without a usable device. */
MCHECKSUM_PUBLIC long long
mchecksum_gpu_queue_faults(void);

/* Diagnostics: work-queue slot bookkeeping of the current device since the
 * library was loaded, written to stats[0 .. min(n, MCHECKSUM_GPU_QSTAT_COUNT)):
 * launches given a slot, launches that took the static split for want of one
 * (graph captures, no idle slot), slots returned to the idle pool once their
 * launch had completed, busy in-flight slots looked at while reaping, and
 * slots handed out and not yet reaped.  Host-side counters only: no device
 * sync. */
#define MCHECKSUM_GPU_QSTAT_SLOT 0
#define MCHECKSUM_GPU_QSTAT_NOSLOT 1
#define MCHECKSUM_GPU_QSTAT_REAPED 2
#define MCHECKSUM_GPU_QSTAT_BUSY_SKIP 3
#define MCHECKSUM_GPU_QSTAT_IN_FLIGHT 4
#define MCHECKSUM_GPU_QSTAT_COUNT 5
MCHECKSUM_PUBLIC int
mchecksum_gpu_queue_stats(long long *stats, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* MCHECKSUM_GPU_H */
