"""GPU against committed data: the batch kernels reproduce the CRCs stored in
tests/golden/ -- no live oracle in the loop.

* vectors.json: 60 seeded payloads (lengths 0..65536, start offsets 0..15),
  payload = splitmix_bytes(offset + length, seed)[offset:] with its crc32c
  and crc64 (= CRC-64/XZ, the default variant) written at generation time
  (oracle/gen_golden.py).  The bytes are made on the device by the product's
  own splitmix generator (libmchecksum_bench.so), and every payload sits at
  its recorded offset from a 16-byte boundary, through checksum_fixed (one
  call per payload), checksum_offsets (all 60 in one batch, each behind a
  gap payload so it keeps its offset) and verify_offsets (every status 0
  against the committed values).
* rfc3720.json: RFC 3720 sec. B.4's four 32-byte iSCSI vectors (crc32c).
* catalogue.json: the published check value CRC("123456789") of every
  32/64-bit catalogue model the GPU serves, MSB-first ECMA-182 included.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
VMETHODS = [("crc32c", "crc32c"), ("crc64", "crc64"), ("crc64-xz", "crc64")]


def _load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def vectors():
    return _load("vectors.json")["vectors"]


@pytest.fixture(autouse=True)
def _default_variants(monkeypatch):
    # "crc64" must mean the default CRC-64/XZ the fixture was made with
    monkeypatch.delenv("MCHECKSUM_CRC64_VARIANT", raising=False)
    monkeypatch.delenv("MCHECKSUM_GPU_LIGHT", raising=False)
    monkeypatch.delenv("MCHECKSUM_GPU_LOG2G", raising=False)


def _slot_bytes(v):
    return (int(v["offset"]) + int(v["length"]) + 15) // 16 * 16 + 16


@pytest.fixture(scope="module")
def device_vectors(gpu, vectors):
    """One device buffer holding every vector's bytes in its own 16-B aligned
    slot (made by the device generator from the vector's seed); returns the
    buffer and each payload's (start, length)."""
    import torch
    sizes = [_slot_bytes(v) for v in vectors]
    starts = np.concatenate([[0], np.cumsum(sizes)])
    buf = torch.zeros(int(starts[-1]) + 64, dtype=torch.uint8, device="cuda")
    spans = []
    for v, s, n in zip(vectors, starts[:-1], sizes):
        gpu.fill_splitmix(buf[int(s):int(s) + n], int(v["seed"], 16))
        spans.append((int(s) + int(v["offset"]), int(v["length"])))
    torch.cuda.synchronize()
    return buf, spans


def _want(vectors, key):
    return np.array([int(v[key], 16) for v in vectors], dtype=np.uint64)


@pytest.mark.parametrize("method,key", VMETHODS)
def test_vectors_one_call_each(gpu, vectors, device_vectors, method, key):
    buf, spans = device_vectors
    got = []
    for (a, n) in spans:
        got.append(int(gpu.as_unsigned(gpu.checksum_fixed(method, buf[a:], n, count=1))[0]))
    want = _want(vectors, key)
    bad = [i for i in range(len(want)) if got[i] != int(want[i])]
    assert not bad, [(vectors[i]["length"], vectors[i]["offset"], hex(got[i]), vectors[i][key]) for i in bad[:5]]


def _gap_offsets(spans):
    """offsets of a batch alternating gap, payload: payload j is entry 2j+1."""
    off = [0]
    for (a, n) in spans:
        off.append(a)
        off.append(a + n)
    return np.array(off, dtype=np.int64)


@pytest.mark.parametrize("method,key", VMETHODS)
def test_vectors_offsets_batch(gpu, vectors, device_vectors, method, key):
    import torch
    buf, spans = device_vectors
    off = _gap_offsets(spans)
    got = gpu.as_unsigned(gpu.checksum_offsets(method, buf, torch.from_numpy(off).cuda(), offsets_host=off))
    assert np.array_equal(got[1::2].astype(np.uint64), _want(vectors, key))


def test_vectors_offsets_batch_throughput_layout(gpu, vectors):
    """The 60 payloads laid out 20 times over (each copy in its own slots, at
    its recorded offsets) as one 2400-entry batch: past 1024 entries, so the
    throughput layout and the work queue run."""
    import torch
    reps = 20
    sizes = [_slot_bytes(v) for v in vectors] * reps
    starts = np.concatenate([[0], np.cumsum(sizes)])
    buf = torch.zeros(int(starts[-1]) + 64, dtype=torch.uint8, device="cuda")
    spans = []
    for k, (s, n) in enumerate(zip(starts[:-1], sizes)):
        v = vectors[k % len(vectors)]
        gpu.fill_splitmix(buf[int(s):int(s) + n], int(v["seed"], 16))
        spans.append((int(s) + int(v["offset"]), int(v["length"])))
    off = _gap_offsets(spans)
    offs = torch.from_numpy(off).cuda()
    for method, key in (("crc32c", "crc32c"), ("crc64", "crc64")):
        got = gpu.as_unsigned(gpu.checksum_offsets(method, buf, offs, offsets_host=off))
        assert np.array_equal(got[1::2].astype(np.uint64), np.tile(_want(vectors, key), reps)), method


@pytest.mark.parametrize("method,key", [("crc32c", "crc32c"), ("crc64", "crc64")])
def test_vectors_verify_against_committed(gpu, vectors, device_vectors, method, key):
    import torch
    buf, spans = device_vectors
    off = _gap_offsets(spans)
    want = _want(vectors, key)
    dt = torch.int32 if method == "crc32c" else torch.int64
    exp = np.zeros(len(off) - 1, dtype=np.uint64)
    exp[1::2] = want
    # gap entries: expect what the device computes for them (not under test)
    gaps = gpu.as_unsigned(gpu.checksum_offsets(method, buf, torch.from_numpy(off).cuda()))
    exp[0::2] = gaps[0::2]
    exp_t = torch.from_numpy(exp.astype(np.uint32 if dt == torch.int32 else np.uint64).view(
        np.int32 if dt == torch.int32 else np.int64)).cuda()
    st, m = gpu.verify_offsets(method, buf, torch.from_numpy(off).cuda(), exp_t)
    assert int(m.item()) == 0 and int(st.sum().item()) == 0
    # one committed value off by one bit: exactly that payload fails
    exp2 = exp.copy()
    exp2[2 * 17 + 1] ^= 1
    exp_t2 = torch.from_numpy(exp2.astype(np.uint32 if dt == torch.int32 else np.uint64).view(
        np.int32 if dt == torch.int32 else np.int64)).cuda()
    st2, m2 = gpu.verify_offsets(method, buf, torch.from_numpy(off).cuda(), exp_t2)
    assert int(m2.item()) == 1 and np.nonzero(st2.cpu().numpy())[0].tolist() == [2 * 17 + 1]


def test_rfc3720_vectors(gpu):
    import torch
    for v in _load("rfc3720.json")["vectors"]:
        host = np.frombuffer(bytes.fromhex(v["hex"]), dtype=np.uint8)
        for shift in (0, 3, 15):  # aligned and unaligned starts
            t = torch.zeros(host.size + 64, dtype=torch.uint8, device="cuda")
            t[shift:shift + host.size].copy_(torch.from_numpy(host.copy()))
            got = int(gpu.as_unsigned(gpu.checksum_fixed("crc32c", t[shift:], host.size, count=1))[0])
            assert got == int(v["crc32c"], 16), (v["name"], shift, hex(got))


def test_catalogue_check_values(gpu):
    """CRC("123456789") of every 32/64-bit catalogue model, one call each and
    as a 3000-payload fixed batch (16-B stride) of the same string."""
    import torch
    cat = _load("catalogue.json")["models"]
    msg = np.frombuffer(b"123456789", dtype=np.uint8)
    names = [n for n, m in cat.items() if m["width"] in (32, 64)]
    assert {"crc32c", "crc32", "crc64-xz", "crc64-ecma182", "crc64-go-iso", "crc64-jones"} <= set(names)
    one = torch.zeros(64, dtype=torch.uint8, device="cuda")
    one[:9].copy_(torch.from_numpy(msg.copy()))
    n = 3000
    many = torch.from_numpy(np.tile(np.concatenate([msg, np.zeros(7, np.uint8)]), n)).cuda()
    for name in names:
        check = int(cat[name]["check"], 16)
        got = int(gpu.as_unsigned(gpu.checksum_fixed(name, one, 9, count=1))[0])
        assert got == check, (name, hex(got))
        gotn = gpu.as_unsigned(gpu.checksum_fixed(name, many, 9, count=n, stride=16))
        assert np.all(gotn.astype(np.uint64) == check), name
