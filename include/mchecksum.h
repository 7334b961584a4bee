/*
 * mchecksum.h -- drop-in replacement for the public header of the mchecksum
 * library that Mercury links when built with MERCURY_USE_CHECKSUMS=ON.
 *
 * The upstream module (git submodule src/mchecksum, .gitmodules:4-6) is absent
 * from the reference tree, so this surface is exactly the one Mercury's call
 * sites bind; each declaration cites the call it serves.
 * Mercury includes it as <mchecksum.h> (src/mercury_proc.c:12-14,
 * src/mercury_core_header.c:11-13) and stores `struct mchecksum_object *`
 * (src/mercury_proc.h:613, src/mercury_core_header.h:67).
 *
 * Methods: "crc16", "crc32c", "crc64" (src/mercury_proc.c:54-63,
 * src/mercury_core_header.c:24).  Catalogue variant names such as
 * "crc64-xz" or "crc16-arc" are accepted too (see DESIGN.md "Variants").
 *
 * Conventions: int return codes, 0 = success, non-zero = failure (Mercury
 * tests rc != 0: src/mercury_proc.c:70-72,206-208,374-377,398-400).
 * update() borrows a HOST pointer for the duration of the call.  get() writes
 * the CRC as a host-order integer of get_size() bytes.  One object is used by
 * one thread at a time; distinct objects may be used concurrently.
 *
 * Large device-resident batches go through the additional entry points in
 * <mchecksum_gpu.h>, which produce the identical values on MI355X.
 */
#ifndef MCHECKSUM_H
#define MCHECKSUM_H

#include <stddef.h>

#if defined(_WIN32)
#    define MCHECKSUM_PUBLIC
#else
#    define MCHECKSUM_PUBLIC __attribute__((visibility("default")))
#endif

#define MCHECKSUM_SUCCESS 0
#define MCHECKSUM_FAIL    (-1)

/* Only flag Mercury passes to mchecksum_get (src/mercury_proc.c:374,
 * src/mercury_core_header.c:210,266). */
#define MCHECKSUM_NOFINALIZE 0
#define MCHECKSUM_FINALIZE   1

typedef struct mchecksum_object *mchecksum_object_t;
/* Compared with == / != by Mercury (src/mercury_proc.c:201,367,393). */
#define MCHECKSUM_OBJECT_NULL ((mchecksum_object_t) 0)

#ifdef __cplusplus
extern "C" {
#endif

/* hg_proc_create (src/mercury_proc.c:70), hg_core_header_*_init
 * (src/mercury_core_header.c:98,114). */
MCHECKSUM_PUBLIC int
mchecksum_init(const char *hash_method, mchecksum_object_t *checksum);

/* Called unconditionally, also with MCHECKSUM_OBJECT_NULL
 * (src/mercury_proc.c:93,136; src/mercury_core_header.c:127,139). */
MCHECKSUM_PUBLIC int
mchecksum_destroy(mchecksum_object_t checksum);

/* hg_proc_reset (src/mercury_proc.c:206); core header (src/mercury_core_header.c:189,251). */
MCHECKSUM_PUBLIC int
mchecksum_reset(mchecksum_object_t checksum);

/* hg_proc_create sizes the hash buffer from it (src/mercury_proc.c:74):
 * 2 for crc16, 4 for crc32c, 8 for crc64. */
MCHECKSUM_PUBLIC size_t
mchecksum_get_size(mchecksum_object_t checksum);

/* hg_proc_flush (src/mercury_proc.c:374) and the core header
 * (src/mercury_core_header.c:210,266).  Fails if size < get_size().
 * Idempotent: calling it twice without update returns the same value. */
MCHECKSUM_PUBLIC int
mchecksum_get(mchecksum_object_t checksum, void *buf, size_t size, int finalize);

/* hg_proc_checksum_update (src/mercury_proc.c:398) once per serialized
 * field; core header fields (src/mercury_core_header.c:49). */
MCHECKSUM_PUBLIC int
mchecksum_update(mchecksum_object_t checksum, const void *data, size_t size);

#ifdef __cplusplus
}
#endif

#endif /* MCHECKSUM_H */
