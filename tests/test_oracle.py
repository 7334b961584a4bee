"""The oracle is pinned before anything trusts it (CPU only).

Pins: the public catalogue check values, RFC 3720 sec. B.4 vectors, and the
x86 SSE4.2 crc32 instruction (CRC-32C in hardware).  The reference holds no
CRC known-answer values (its only checksum test, Testing/unit/hg/test_proc.c:
87-138, checks encode == decode), so CRC-64 / CRC-16 stay "parity unpinned".
"""
import json
import os
import subprocess

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load(name):
    return json.load(open(os.path.join(GOLDEN, name)))


def test_selftest_binary(oracle_mod):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "oracle", "_build", "oracle_selftest")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "oracle pinned" in r.stdout


@pytest.mark.parametrize("variant", ["bitwise", "table"])
def test_catalogue_check_values(oracle_mod, variant):
    cat = _load("catalogue.json")["models"]
    assert len(cat) == 12
    for name, m in cat.items():
        assert oracle_mod.crc(name, b"123456789", variant) == int(m["check"], 16), name


def test_catalogue_parameters_match_oracle(oracle_mod):
    cat = _load("catalogue.json")["models"]
    for m in oracle_mod.models():
        e = cat[m.name.decode()]
        assert (m.width, m.poly, bool(m.refin), bool(m.refout), m.init, m.xorout) == (
            e["width"], int(e["poly"], 16), e["refin"], e["refout"], int(e["init"], 16), int(e["xorout"], 16))


def test_rfc3720_vectors(oracle_mod):
    for v in _load("rfc3720.json")["vectors"]:
        data = bytes.fromhex(v["hex"])
        for variant in ("bitwise", "table", "sse42"):
            assert oracle_mod.crc("crc32c", data, variant) == int(v["crc32c"], 16), (v["name"], variant)


def test_sse42_cross_check_random(oracle_mod):
    buf = oracle_mod.splitmix_bytes(70000, 0xC0FFEE)
    rng = np.random.default_rng(0)
    for _ in range(300):
        off = int(rng.integers(0, 16))
        n = int(rng.integers(0, 69000))
        d = buf[off:off + n]
        assert oracle_mod.crc("crc32c", d, "sse42") == oracle_mod.crc("crc32c", d, "table")


def test_vectors_fixture(oracle_mod):
    for v in _load("vectors.json")["vectors"]:
        buf = oracle_mod.splitmix_bytes(v["offset"] + v["length"], int(v["seed"], 16))
        d = buf[v["offset"]:]
        for m in ("crc32c", "crc64", "crc16"):
            assert oracle_mod.crc(m, d) == int(v[m], 16), (v, m)
        if v["length"] <= 4097:
            assert oracle_mod.crc("crc32c", d, "bitwise") == int(v["crc32c"], 16)


def test_test_proc_images(oracle_mod):
    tp = _load("test_proc.json")["payloads"]
    for name, p in tp.items():
        img = bytes.fromhex(p["hex"])
        assert sum(p["field_sizes"]) == len(img)
        for m in ("crc32c", "crc64", "crc16"):
            assert oracle_mod.crc(m, img, "bitwise") == int(p[m], 16)


def test_splitmix_layout(oracle_mod):
    # little-endian words splitmix64(seed ^ word_index), any byte window
    b = oracle_mod.splitmix_bytes(24, 5, first_word=10)
    for i in range(3):
        assert int.from_bytes(b[8 * i:8 * i + 8].tobytes(), "little") == oracle_mod.splitmix64(5 ^ (10 + i))
    full = oracle_mod.splitmix_bytes(1000, 9)
    part = oracle_mod.splitmix_bytes(1000 - 80, 9, first_word=10)
    assert np.array_equal(full[80:], part)


def test_varlen_offsets_layout(oracle_mod):
    off = oracle_mod.varlen_offsets(0x4D43310000000004, 10000)
    lens = np.diff(off.astype(np.int64))
    assert off[0] == 0 and lens.min() >= 64 and lens.max() <= 65536
    assert abs(lens.mean() - (64 + 65536) / 2) < 1000


def test_batch_helpers_agree(oracle_mod):
    buf = oracle_mod.splitmix_bytes(300 * 1000, 3)
    a = oracle_mod.batch_fixed("crc32c", buf, 1000, 999, 300, nthreads=4)
    b = oracle_mod.batch_fixed("crc32c", buf, 1000, 999, 300, variant="sse42", nthreads=3)
    assert np.array_equal(a, b)
    c = oracle_mod.splitmix_batch_fixed("crc64", 3, 1000, 999, 5, 20, nthreads=2)
    assert np.array_equal(c, oracle_mod.batch_fixed("crc64", buf[5000:], 1000, 999, 20))
    off = np.arange(0, 300 * 1000 + 1, 1000, dtype=np.uint64)
    d = oracle_mod.batch_offsets("crc32c", buf, off, nthreads=5)
    assert np.array_equal(d, oracle_mod.batch_fixed("crc32c", buf, 1000, 1000, 300))


def test_slice8_equals_bitwise_for_every_reflected_model(oracle_mod):
    """The CPU baseline's slicing-by-8 path (bench.py cpu_baseline for crc64)
    equals the literal bitwise model, at every length 0..70 and unaligned starts."""
    import numpy as np
    buf = oracle_mod.splitmix_bytes(4096, 0x51CE)
    for m in ("crc32c", "crc32", "crc64", "crc64-xz", "crc64-jones", "crc64-go-iso", "crc16-arc", "crc16-kermit"):
        for n in list(range(0, 71)) + [1000, 4093]:
            for off in (0, 3):
                d = buf[off:off + n]
                assert oracle_mod.crc(m, d, variant="slice8") == oracle_mod.crc(m, d, variant="bitwise"), (m, n, off)
    big = oracle_mod.splitmix_bytes(1 << 20, 3)
    assert oracle_mod.batch_fixed("crc64", big, 1 << 18, 1 << 18, 4, variant="slice8").tolist() == \
        oracle_mod.batch_fixed("crc64", big, 1 << 18, 1 << 18, 4, variant="table").tolist()
