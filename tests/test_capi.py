"""The drop-in C ABI: libmchecksum.so loads, exports every symbol the public
headers declare, and the streaming API behaves the way Mercury's call sites
need (CPU only; no compute on a GPU here).

Call sites mirrored: hg_proc_create / reset / flush / checksum_get /
checksum_verify (src/mercury_proc.c:34-99,151-217,358-472) and the per-field
updates of HG_PROC_TYPE / HG_PROC_BYTES (src/mercury_proc.h:124-143,162-181).
"""
import ctypes
import json
import os
import re
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _declared_functions():
    names = set()
    for h in ("mchecksum.h", "mchecksum_gpu.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        for m in re.finditer(r"^MCHECKSUM_PUBLIC\s+[\w\s\*]+?\n?\s*(\w+)\s*\(", txt, re.M):
            names.add(m.group(1))
    return names


def test_header_declares_the_mercury_surface():
    names = _declared_functions()
    # every entry point Mercury binds
    for n in ("mchecksum_init", "mchecksum_destroy", "mchecksum_reset", "mchecksum_get_size", "mchecksum_get",
              "mchecksum_update"):
        assert n in names
    txt = open(os.path.join(ROOT, "include", "mchecksum.h")).read()
    assert "#define MCHECKSUM_FINALIZE" in txt and "#define MCHECKSUM_OBJECT_NULL" in txt
    assert "typedef struct mchecksum_object *mchecksum_object_t" in txt


def test_library_exports_every_declared_symbol(product_lib):
    from mercury_amd import _lib
    names = _declared_functions()
    assert names == set(_lib.STREAMING_SYMBOLS) | set(_lib.GPU_SYMBOLS)
    for n in names:
        assert hasattr(product_lib, n), n
    # and nothing else leaks with default visibility besides them
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert names <= exported
    assert not {e for e in exported if e.startswith(("crc_", "mck_"))}, "internal helpers must stay hidden"


def test_no_gpu_means_loud_failure_not_fallback(product_lib):
    """On a box without a HIP device the batch path must fail, never compute
    on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    L = product_lib
    assert L.mchecksum_gpu_available() == 0
    out = ctypes.create_string_buffer(64)
    data = ctypes.create_string_buffer(b"x" * 64)
    rc = L.mchecksum_gpu_checksum_fixed(b"crc32c", data, 64, 64, 1, out, None)
    assert rc == -2  # MCHECKSUM_GPU_ENODEV
    assert L.mchecksum_gpu_prepare(b"crc32c") == -2
    offs = (ctypes.c_uint64 * 2)(0, 64)
    assert L.mchecksum_gpu_checksum_offsets(b"crc32c", data, offs, 1, out, None) == -2
    assert b"device" in L.mchecksum_gpu_last_error()


def test_batch_arguments_rejected_before_any_device_work(product_lib):
    """Bad batch arguments give MCHECKSUM_GPU_EINVAL (-1) and a reason,
    whether or not a device is present (checked before device detection)."""
    L = product_lib
    buf = ctypes.create_string_buffer(64)
    offs = (ctypes.c_uint64 * 2)(0, 64)
    cases = [
        (lambda: L.mchecksum_gpu_checksum_fixed(b"crc32c", None, 64, 64, 1, buf, None), "NULL"),
        (lambda: L.mchecksum_gpu_checksum_fixed(b"crc32c", buf, 64, 64, 1, None, None), "NULL"),
        (lambda: L.mchecksum_gpu_checksum_fixed(b"crc32c", buf, 32, 64, 2, buf, None), "stride"),
        (lambda: L.mchecksum_gpu_checksum_fixed(b"crc32c", buf, 64, 64, (1 << 31) + 1, buf, None), "2^31"),
        (lambda: L.mchecksum_gpu_checksum_fixed(b"crc32c", buf, 1 << 62, 64, 8, buf, None), "overflows"),
        (lambda: L.mchecksum_gpu_checksum_offsets(b"crc32c", buf, None, 1, buf, None), "NULL"),
        (lambda: L.mchecksum_gpu_checksum_offsets(b"crc32c", buf, offs, (1 << 31) + 1, buf, None), "2^31"),
        (lambda: L.mchecksum_gpu_verify_offsets(b"crc32c", buf, offs, 1, None, None, None, None), "NULL"),
        (lambda: L.mchecksum_gpu_verify_messages(b"crc32c", buf, offs, 1, 18, 16, None, None, None), "hash_offset"),
    ]
    ws = L.mchecksum_gpu_segments_work_size
    ws.restype = ctypes.c_size_t
    # P, C, ragged flag, fault claim, call count, spare, per scan block a
    # look-back descriptor (8), segment -> (object, its first[] bounds, its head
    # segment) (u64 words), then the chunk -> segment map (u32, 4 per segment +
    # 64 Ki; none past 2^32 segments)
    assert ws(4) == 8 * (2 * 5 + 4 + 8 + 4 * 4) + 4 * (4 * 4 + 65536) and ws((1 << 40) + 1) == (1 << 64) - 1
    n = 1 << 32
    assert ws(n) == 8 * (2 * (n + 1) + 4 + 8 * (n // 1024) + 4 * n)
    first = (ctypes.c_uint64 * 2)(0, 1)
    cases += [
        (lambda: L.mchecksum_gpu_checksum_segments(b"crc64", offs, offs, 1, first, 1, buf, 8, buf, None), "workspace"),
        (lambda: L.mchecksum_gpu_checksum_segments(b"crc64", offs, offs, (1 << 40) + 1, first, 1, buf, 64, buf, None),
         "2^40"),
        (lambda: L.mchecksum_gpu_verify_core_headers(b"crc16", 7, buf, offs, 1, None, None, None), "kind"),
    ]
    for call, why in cases:
        assert call() == -1, why
        assert why.encode() in L.mchecksum_gpu_last_error(), (why, L.mchecksum_gpu_last_error())
    # an empty batch is valid with NULL buffers (the offsets table included):
    # never EINVAL -- 0 with a device, ENODEV without one
    assert L.mchecksum_gpu_checksum_fixed(b"crc32c", None, 0, 0, 0, None, None) in (0, -2)
    assert L.mchecksum_gpu_checksum_offsets(b"crc32c", None, None, 0, None, None) in (0, -2)
    assert L.mchecksum_gpu_verify_offsets(b"crc64", None, None, 0, None, None, None, None) in (0, -2)
    assert L.mchecksum_gpu_verify_messages(b"crc32c", None, None, 0, 20, 16, None, None, None) in (0, -2)


def test_lanes_per_payload_heuristic(product_lib):
    f = product_lib.mchecksum_gpu_lanes_per_payload
    assert f(b"crc32c", 65536) == 64
    # CRC-32 (round-6 sweeps on cold lines): 16 steps per payload from 1 KiB to
    # under 8 KiB, then ~32 steps per payload
    assert [f(b"crc32c", n) for n in (1024, 2048, 4096, 6144, 8192, 16384, 32768)] == [4, 8, 16, 16, 16, 32, 64]
    assert f(b"crc32c", 512) == 2
    # CRC-64: about 128 steps per payload, 4 lanes at least
    assert [f(b"crc64", n) for n in (1024, 4096, 16384, 65536, 262144)] == [4, 4, 8, 32, 64]
    assert f(b"crc64", 1 << 20) == 64
    assert f(b"crc32c", 64) == 1
    assert f(b"crc16", 4096) == -1  # crc16 has no GPU kernel (CPU header path only)
    assert f(b"nope", 4096) == -1


def test_init_destroy_reset_get_size(product_lib):
    from mercury_amd import Checksum
    sizes = {"crc16": 2, "crc32c": 4, "crc64": 8, "crc64-ecma182": 8, "crc16-arc": 2, "crc32": 4}
    for m, s in sizes.items():
        c = Checksum(m)
        assert c.get_size() == s
        c.close()
    obj = ctypes.c_void_p()
    assert product_lib.mchecksum_init(b"sha1", ctypes.byref(obj)) != 0
    assert product_lib.mchecksum_init(None, ctypes.byref(obj)) != 0
    assert product_lib.mchecksum_init(b"crc32c", None) != 0
    # destroy(NULL) is called unconditionally by Mercury (src/mercury_proc.c:93,136)
    assert product_lib.mchecksum_destroy(None) == 0
    assert product_lib.mchecksum_reset(None) != 0
    assert product_lib.mchecksum_get_size(None) == 0


def test_get_contract(product_lib):
    from mercury_amd import Checksum
    c = Checksum("crc32c")
    c.update(b"123456789")
    # too-small buffer fails (Mercury sizes the hash from get_size)
    buf = ctypes.create_string_buffer(8)
    assert product_lib.mchecksum_get(c._obj, buf, 3, 1) != 0
    assert product_lib.mchecksum_get(c._obj, None, 4, 1) != 0
    # host-order integer, idempotent, finalize flag does not change the value
    a = c.get_bytes()
    assert a == c.get_bytes() == c.get_bytes(finalize=0) == struct.pack("<I", 0xE3069283)
    assert c.get_bytes(size=8)[:4] == a
    c.reset()
    assert c.get() == 0  # CRC-32C of the empty message
    c.update(b"")
    assert c.get() == 0
    assert product_lib.mchecksum_update(c._obj, None, 5) != 0


def test_catalogue_through_the_abi(product_lib):
    from mercury_amd import checksum
    cat = json.load(open(os.path.join(GOLDEN, "catalogue.json")))["models"]
    for name, m in cat.items():
        assert checksum(name, b"123456789") == int(m["check"], 16), name
    assert checksum("crc64", b"123456789") == int(cat["crc64-xz"]["check"], 16)
    assert checksum("crc16", b"123456789") == int(cat["crc16-t10-dif"]["check"], 16)


def test_variant_environment_override(product_lib, monkeypatch):
    from mercury_amd import checksum
    cat = json.load(open(os.path.join(GOLDEN, "catalogue.json")))["models"]
    monkeypatch.setenv("MCHECKSUM_CRC64_VARIANT", "crc64-ecma182")
    monkeypatch.setenv("MCHECKSUM_CRC16_VARIANT", "crc16-arc")
    assert checksum("crc64", b"123456789") == int(cat["crc64-ecma182"]["check"], 16)
    assert checksum("crc16", b"123456789") == int(cat["crc16-arc"]["check"], 16)
    monkeypatch.setenv("MCHECKSUM_CRC64_VARIANT", "crc16-arc")  # wrong family: ignored
    assert checksum("crc64", b"123456789") == int(cat["crc64-xz"]["check"], 16)


@pytest.mark.parametrize("method", ["crc32c", "crc64", "crc16", "crc32", "crc64-ecma182", "crc16-arc", "crc64-go-iso",
                                    "crc64-jones", "crc16-kermit"])
def test_streaming_matches_oracle_random(product_lib, oracle_mod, method):
    from mercury_amd import Checksum
    buf = oracle_mod.splitmix_bytes(200000, 0xABC)
    rng = np.random.default_rng(1)
    for _ in range(60):
        off = int(rng.integers(0, 32))
        n = int(rng.integers(0, 150000)) if rng.random() < 0.3 else int(rng.integers(0, 2000))
        d = buf[off:off + n]
        c = Checksum(method)
        cuts = sorted(set(int(x) for x in rng.integers(0, n + 1, size=int(rng.integers(0, 6)))))
        prev = 0
        for cut in cuts + [n]:
            c.update(d[prev:cut].tobytes())
            prev = cut
        assert c.get() == oracle_mod.crc(method, d), (method, off, n, cuts)


_PATH_LENS = (0, 1, 767, 768, 769, 1023, 1024, 1025, 1536, 2304, 4096, 5000, 9999, 65536 + 13, 262144 + 255)


def test_sse42_and_software_paths_agree(product_lib, oracle_mod):
    """Every CPU path agrees with the oracle's bitwise model, for crc32c and
    crc64: the AVX-512 VPCLMULQDQ fold (default where the CPU has it), the
    SSE4.2 3-way interleave + shift combine / slicing-by-8
    (MCHECKSUM_DISABLE_CLMUL=1) and the slicing path
    (MCHECKSUM_DISABLE_SSE42=1) -- each knob is read once per process, so each
    path runs in a subprocess, on lengths around every path's thresholds, at
    an odd start offset, whole and as a 3-way split update."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from mercury_amd import checksum, Checksum\n"
            "from oracle import oracle as O\n"
            "buf = O.splitmix_bytes(300000, 0x55)\n"
            "out = []\n"
            "for m in ('crc32c', 'crc64'):\n"
            "  for n in %r:\n"
            "    d = buf[3:3 + n].tobytes()\n"
            "    c = Checksum(m); c.update(d[:n // 3]); c.update(d[n // 3:n - 7]); c.update(d[n - 7:] if n >= 7 else b'')\n"
            "    out.append('%%d/%%d' %% (checksum(m, d), c.get() if n >= 7 else checksum(m, d)))\n"
            "print(','.join(out))\n") % (ROOT, _PATH_LENS)
    outs = []
    for env in ({}, {"MCHECKSUM_DISABLE_CLMUL": "1"}, {"MCHECKSUM_DISABLE_SSE42": "1"}):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           env={**os.environ, **env})
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.strip())
    buf = oracle_mod.splitmix_bytes(300000, 0x55)
    want = ",".join("%d/%d" % ((oracle_mod.crc(m, buf[3:3 + n], "bitwise"),) * 2)
                    for m in ("crc32c", "crc64") for n in _PATH_LENS)
    assert outs == [want] * 3


def test_stream_split_fixture(product_lib):
    from mercury_amd import Checksum
    from oracle import oracle as O
    for case in json.load(open(os.path.join(GOLDEN, "stream_split.json")))["cases"]:
        buf = O.splitmix_bytes(case["length"], int(case["seed"], 16)).tobytes()
        for m in ("crc32c", "crc64", "crc16"):
            c = Checksum(m)
            prev = 0
            for cut in case["cuts"] + [case["length"]]:
                c.update(buf[prev:cut])
                prev = cut
            assert c.get() == int(case[m], 16)


class _Proc:
    """Minimal restatement of the hg_proc encode/decode + checksum flow
    (src/mercury_proc.c:151-217, 358-472; src/mercury_proc.h:124-181) on top
    of the drop-in library, to show the per-field streaming CRC equals the
    whole-buffer CRC the GPU batch path computes."""

    def __init__(self, method="crc32c"):
        from mercury_amd import Checksum
        self.ck = Checksum(method)
        self.hash = b""

    def reset(self, buf: bytearray):
        self.buf, self.pos = buf, 0
        self.ck.reset()
        self.hash = bytes(self.ck.get_size())

    def proc(self, fmt, value=None):
        n = struct.calcsize(fmt)
        if value is not None:  # HG_ENCODE: memcpy into buffer
            self.buf[self.pos:self.pos + n] = struct.pack(fmt, value)
        data = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        self.ck.update(data)  # HG_PROC_CHECKSUM_UPDATE on the same n bytes
        return struct.unpack(fmt, data)[0]

    def flush(self):
        self.hash = self.ck.get_bytes()


def test_proc_roundtrip_like_test_proc(product_lib, oracle_mod):
    """Testing/unit/hg/test_proc.c:79-147 with the uint struct {1,2,3,4}."""
    tp = json.load(open(os.path.join(GOLDEN, "test_proc.json")))["payloads"]["uint_struct"]
    p = _Proc()
    buf = bytearray(4096)
    p.reset(buf)
    for fmt, v in (("<B", 1), ("<H", 2), ("<I", 3), ("<Q", 4)):
        p.proc(fmt, v)
    p.flush()
    sent_hash = p.hash
    assert bytes(buf[:p.pos]).hex() == tp["hex"]
    assert int.from_bytes(sent_hash, "little") == int(tp["crc32c"], 16) == oracle_mod.crc("crc32c", buf[:p.pos])
    # decode side verifies
    recv = bytearray(buf)
    p.reset(recv)
    assert [p.proc(f) for f in ("<B", "<H", "<I", "<Q")] == [1, 2, 3, 4]
    p.flush()
    assert p.hash == sent_hash  # hg_proc_checksum_verify: memcmp
    # one flipped bit in transit -> HG_CHECKSUM_ERROR
    recv[6] ^= 0x20
    p.reset(recv)
    for f in ("<B", "<H", "<I", "<Q"):
        p.proc(f)
    p.flush()
    assert p.hash != sent_hash
