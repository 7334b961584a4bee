#!/usr/bin/env python3
"""Writes tests/golden/*.json -- small committed fixtures (TEST INFRASTRUCTURE).

Pins, in order of strength:
  catalogue.json  published check values (CRC of ASCII "123456789") for every
                  variant in SURVEY.md Appendix A -- literal values from the
                  public CRC catalogue, NOT produced by the oracle;
  rfc3720.json    the four CRC-32C vectors of RFC 3720 sec. B.4 (literal);
  test_proc.json  the byte images Mercury's only checksum test serializes
                  (Testing/unit/hg/test_proc.c:186-227: {u8 1, u16 2, u32 3,
                  u64 4} and hg_string_t "Hello"), with their CRCs; CRC-32C
                  cross-checked against the SSE4.2 instruction at generation;
  vectors.json    seeded splitmix payloads (lengths/offsets from SURVEY.md
                  8(c)) with CRCs per method; CRC-32C cross-checked by SSE4.2,
                  CRC-64/CRC-16 marked parity-unpinned (upstream variant
                  unknown);
  stream_split.json  update(a); update(b) == update(a||b) split points;
  core_headers.json  Mercury core-header request/response images with their
                  CRC-16 for every catalogue variant (core_header_fixtures).
The reference's own tests hold no CRC values, so nothing
here comes from the reference; the data are generated from seeds.
"""
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# Public CRC catalogue (width, poly, refin, refout, init, xorout, check).
CATALOGUE = {
    "crc32c": (32, 0x1EDC6F41, True, True, 0xFFFFFFFF, 0xFFFFFFFF, 0xE3069283),
    "crc32": (32, 0x04C11DB7, True, True, 0xFFFFFFFF, 0xFFFFFFFF, 0xCBF43926),
    "crc64-xz": (64, 0x42F0E1EBA9EA3693, True, True, 2**64 - 1, 2**64 - 1, 0x995DC9BBDF1939FA),
    "crc64-ecma182": (64, 0x42F0E1EBA9EA3693, False, False, 0, 0, 0x6C40DF5F0B497347),
    "crc64-go-iso": (64, 0x1B, True, True, 2**64 - 1, 2**64 - 1, 0xB90956C775A41001),
    "crc64-jones": (64, 0xAD93D23594C935A9, True, True, 0, 0, 0xE9C6D914C4B8D9CA),
    "crc16-arc": (16, 0x8005, True, True, 0, 0, 0xBB3D),
    "crc16-ibm-3740": (16, 0x1021, False, False, 0xFFFF, 0, 0x29B1),
    "crc16-xmodem": (16, 0x1021, False, False, 0, 0, 0x31C3),
    "crc16-kermit": (16, 0x1021, True, True, 0, 0, 0x2189),
    "crc16-umts": (16, 0x8005, False, False, 0, 0, 0xFEE8),
    "crc16-t10-dif": (16, 0x8BB7, False, False, 0, 0, 0xD0DB),
}
RFC3720 = [
    ("32 bytes of 0x00", "00" * 32, 0x8A9136AA),
    ("32 bytes of 0xFF", "ff" * 32, 0x62A8AB43),
    ("0x00..0x1F ascending", bytes(range(32)).hex(), 0x46DD794E),
    ("0x1F..0x00 descending", bytes(range(31, -1, -1)).hex(), 0x113FDB5C),
]
METHODS = ["crc32c", "crc64", "crc16"]


def test_proc_images():
    """Byte images of Mercury's test_proc payloads in the default non-XDR,
    little-endian build: each hg_proc_<type> memcpy's the host value
    (src/mercury_proc.h:124-143); hg_string_t = u64 length incl. NUL, the
    bytes, then u8 is_const, u8 is_owned (src/proc_extra/mercury_proc_string.c:30-54)."""
    uint_struct = struct.pack("<BHIQ", 1, 2, 3, 4)
    s = b"Hello\x00"
    string_obj = struct.pack("<Q", len(s)) + s + b"\x00\x00"
    return {"uint_struct": (uint_struct, [1, 2, 4, 8]), "string_hello": (string_obj, [8, 6, 1, 1])}


CRC16_VARIANTS = [k for k in CATALOGUE if k.startswith("crc16-")]


def core_header_fixtures():
    """Mercury core headers as hg_core_header_request_proc / _response_proc
    encode them (src/mercury_core_header.c:175-289): the CRC16 runs over the
    HOST-order field values in proc order (HG_CORE_HEADER_CHECKSUM_UPDATE,
    :48-55) -- request hg u8, protocol u8, id u64, flags u8, cookie u8 (12 B);
    response ret_code i8, flags u8, cookie u16 (4 B) -- and the wire carries
    the fields big-endian (:26-36) with the u16 hash big-endian right after the
    last field (request offset 12, response offset 4: the response's u64 pad
    is never proc'd), in a 16-byte header (src/mercury_core_header.h:23-40).
    One hash per CRC-16 catalogue variant (which one upstream mchecksum's
    "crc16" is stays unpinned)."""
    rng_vals = []
    x = 0x4D43484452000001
    for i in range(16):  # seeded field values, edges first
        x = O.splitmix64(x)
        rng_vals.append(x)
    reqs = [(0x48 | 0x47, 5, 0, 0, 0), (0xFF, 0xFF, 2**64 - 1, 0xFF, 0xFF), (0x4F, 5, 0x0123456789ABCDEF, 0x81, 0x22)]
    reqs += [(v & 0xFF, (v >> 8) & 0xFF, O.splitmix64(v), (v >> 16) & 0xFF, (v >> 24) & 0xFF) for v in rng_vals[:8]]
    resps = [(0, 0, 0), (-1, 0xFF, 0xFFFF), (-128, 0x01, 0x1234), (127, 0x80, 0x8000)]
    resps += [(((v & 0xFF) ^ 0x80) - 0x80, (v >> 8) & 0xFF, (v >> 16) & 0xFFFF) for v in rng_vals[8:]]
    out = {"source": "src/mercury_core_header.c:175-289 encodings; CRC16 of the host-order field image per "
                     "CRC-16 catalogue variant (oracle bitwise model); upstream crc16 variant: parity unpinned",
           "request": [], "response": []}
    for hg, proto, rid, flags, cookie in reqs:
        img = struct.pack("<BBQBB", hg, proto, rid, flags, cookie)
        e = {"fields": [hg, proto, hex(rid), flags, cookie], "image": img.hex(), "hash_offset": 12,
             "wire_fields": struct.pack(">BBQBB", hg, proto, rid, flags, cookie).hex()}
        for v in CRC16_VARIANTS:
            e[v] = hex(O.crc(v, img, variant="bitwise"))
            assert int(e[v], 16) == O.crc(v, img)
        out["request"].append(e)
    for ret, flags, cookie in resps:
        img = struct.pack("<bBH", ret, flags, cookie)
        e = {"fields": [ret, flags, cookie], "image": img.hex(), "hash_offset": 4,
             "wire_fields": struct.pack(">bBH", ret, flags, cookie).hex()}
        for v in CRC16_VARIANTS:
            e[v] = hex(O.crc(v, img, variant="bitwise"))
            assert int(e[v], 16) == O.crc(v, img)
        out["response"].append(e)
    return out


def test_proc_xdr():
    """The same payloads serialized with MERCURY_USE_XDR (src/mercury_proc.h:
    110-122,147-160): u8/u16/u32 as 4-byte big-endian words, u64 as 8; the
    string's bytes through xdr_opaque (zero pad to 4), its two u8 flags as
    4-byte words.  Schema kinds: include/mchecksum_gpu.h MCHECKSUM_XDR_*."""
    st = [(O.XDR_INT, 1), (O.XDR_INT, 2), (O.XDR_INT, 4), (O.XDR_INT, 8)]
    sg = [(O.XDR_INT, 8), (O.XDR_SKIP_IF_ZERO, 3), (O.XDR_OPAQUE_LEN, 0), (O.XDR_INT, 1), (O.XDR_INT, 1)]
    return {"uint_struct": (st, O.xdr_encode(st, [1, 2, 3, 4])),
            "string_hello": (sg, O.xdr_encode(sg, [6, b"Hello\x00", 0, 0]))}


def main():
    os.makedirs(OUT, exist_ok=True)
    cat = {k: {"width": w, "poly": hex(p), "refin": ri, "refout": ro, "init": hex(i), "xorout": hex(x),
               "check": hex(c)} for k, (w, p, ri, ro, i, x, c) in CATALOGUE.items()}
    json.dump({"source": "public CRC catalogue (SURVEY.md Appendix A); check = CRC(ASCII '123456789')",
               "models": cat}, open(os.path.join(OUT, "catalogue.json"), "w"), indent=1)
    json.dump({"source": "RFC 3720 sec. B.4 (iSCSI CRC-32C examples)",
               "vectors": [{"name": n, "hex": h, "crc32c": hex(c)} for n, h, c in RFC3720]},
              open(os.path.join(OUT, "rfc3720.json"), "w"), indent=1)

    tp = {}
    xdr = test_proc_xdr()
    for name, (img, fields) in test_proc_images().items():
        c32 = O.crc("crc32c", img)
        assert c32 == O.crc("crc32c", img, variant="sse42")
        schema, wire = xdr[name]
        assert O.xdr_hashed_stream(schema, wire) == img  # XDR mode hashes the same host values
        tp[name] = {"hex": img.hex(), "field_sizes": fields,
                    **{m: hex(O.crc(m, img)) for m in METHODS},
                    "xdr_hex": wire.hex(), "xdr_schema": [list(f) for f in schema]}
    json.dump({"source": "Testing/unit/hg/test_proc.c:186-227 payload images (non-XDR, little-endian)",
               "pinned": {"crc32c": "RFC 3720 standard + SSE4.2", "crc64": "parity unpinned (CRC-64/XZ default)",
                          "crc16": "parity unpinned (CRC-16/T10-DIF default)"},
               "xdr": "xdr_hex: the payload as MERCURY_USE_XDR serializes it (src/mercury_proc.h:110-160); "
                      "its proc checksum is the CRC of hex (the host-order values)",
               "payloads": tp}, open(os.path.join(OUT, "test_proc.json"), "w"), indent=1)

    lengths = [0, 1, 3, 7, 8, 9, 63, 64, 65, 4095, 4096, 4097, 65535, 65536]
    vecs = []
    seed = 0x4D43310000000000
    for li, n in enumerate(lengths):
        for off in (0, 1, 5, 15) if n < 65535 else (0, 7):
            buf = O.splitmix_bytes(off + n, seed ^ (li << 8) ^ off)
            data = buf[off:off + n]
            e = {"seed": hex(seed ^ (li << 8) ^ off), "offset": off, "length": n}
            for m in METHODS:
                e[m] = hex(O.crc(m, data))
            assert int(e["crc32c"], 16) == O.crc("crc32c", data, variant="sse42")
            vecs.append(e)
    json.dump({"source": "payload = splitmix_bytes(offset+length, seed)[offset:]; oracle CRCs; "
                         "crc32c cross-checked with SSE4.2 at generation",
               "vectors": vecs}, open(os.path.join(OUT, "vectors.json"), "w"), indent=1)

    json.dump(core_header_fixtures(), open(os.path.join(OUT, "core_headers.json"), "w"), indent=1)

    splits = []
    buf = O.splitmix_bytes(5000, 77)
    for cuts in ([0], [1], [3, 4], [7, 8, 9], [100, 1000, 4096], [4999]):
        splits.append({"seed": hex(77), "length": 5000, "cuts": cuts,
                       **{m: hex(O.crc(m, buf)) for m in METHODS}})
    json.dump({"source": "streaming-split invariance: update(a); update(b) == update(a||b)", "cases": splits},
              open(os.path.join(OUT, "stream_split.json"), "w"), indent=1)
    print("wrote", sorted(os.listdir(OUT)))


if __name__ == "__main__":
    main()
