"""Mercury core-header CRC16 fixtures (tests/golden/core_headers.json, written
by oracle/gen_golden.py) against the oracle and the drop-in library's
streaming API, for every CRC-16 catalogue variant.

The library is fed exactly as hg_core_header_request_proc / _response_proc
feed mchecksum: reset, one update per field with the HOST-order value, get
(src/mercury_core_header.c:48-55, 175-289).  Which CRC-16 upstream mchecksum's
"crc16" is remains parity unpinned; every candidate is pinned to its published
check value in test_oracle.py."""
import json
import os
import struct

import pytest

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "core_headers.json")))
VARIANTS = ["crc16-arc", "crc16-ibm-3740", "crc16-xmodem", "crc16-kermit", "crc16-umts", "crc16-t10-dif"]
REQ_FIELDS = ("<B", "<B", "<Q", "<B", "<B")   # hg, protocol, id, flags, cookie
RESP_FIELDS = ("<b", "<B", "<H")              # ret_code, flags, cookie


def _field_values(kind, e):
    v = [int(x, 16) if isinstance(x, str) else x for x in e["fields"]]
    return list(zip(REQ_FIELDS if kind == "request" else RESP_FIELDS, v))


@pytest.mark.parametrize("kind", ["request", "response"])
def test_fixture_images_match_the_encoding(kind):
    for e in GOLD[kind]:
        img = b"".join(struct.pack(f, v) for f, v in _field_values(kind, e))
        assert img.hex() == e["image"]
        wire = b"".join(struct.pack(">" + f[1], v) for f, v in _field_values(kind, e))
        assert wire.hex() == e["wire_fields"] and len(wire) == e["hash_offset"]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("kind", ["request", "response"])
def test_fixtures_oracle_and_streaming_api(oracle_mod, product_lib, kind, variant, monkeypatch):
    from mercury_amd import Checksum
    monkeypatch.setenv("MCHECKSUM_CRC16_VARIANT", variant)
    ck = Checksum("crc16")
    for e in GOLD[kind]:
        img = bytes.fromhex(e["image"])
        want = int(e[variant], 16)
        assert oracle_mod.crc(variant, img) == want
        assert oracle_mod.crc(variant, img, variant="bitwise") == want
        ck.reset()
        for f, v in _field_values(kind, e):  # HG_CORE_HEADER_PROC: one update per field
            ck.update(struct.pack(f, v))
        assert ck.get() == want, (kind, variant, e["fields"])
