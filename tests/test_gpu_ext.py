"""GPU parity of the 8(f) entry points (mchecksum_gpu_ext.hip) through the C ABI.

* checksum_segments: scatter-gather objects (a bulk handle's segment list,
  HG_Bulk_create(count, buf_ptrs, buf_sizes), src/mercury_bulk.h:55) -- the
  value must equal the oracle CRC of the concatenated bytes and the streaming
  API fed one update per segment.
* verify_core_headers: Mercury core headers encoded as
  hg_core_header_request_proc / _response_proc do it
  (src/mercury_core_header.c:175-289), hashed by the ORACLE over the
  host-order field values for every CRC-16 catalogue variant (and the
  committed request/response fixtures), then corrupted in known places.
"""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host(t):
    return t.cpu().numpy()


@pytest.fixture
def buf(gpu):
    import torch
    n = 24 << 20
    t = torch.empty(n + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, 0x5E6)
    return t


def _objects(rng, buf_len, nobj, max_seg=6, lens=None):
    """Random segment views (offset, length) grouped into objects."""
    segs, first = [], [0]
    pool = lens or [0, 1, 3, 7, 8, 15, 16, 17, 63, 64, 100, 1000, 4095, 4096, 4097, 65536, 100003, 262143, 262144,
                    262145, 600000, 1 << 20, (1 << 20) + 5]
    for _ in range(nobj):
        for _ in range(int(rng.integers(0, max_seg + 1))):
            ln = int(pool[int(rng.integers(0, len(pool)))])
            off = int(rng.integers(0, buf_len - ln))
            segs.append((off, ln))
        first.append(len(segs))
    return segs, first


def _want(oracle_mod, method, host, segs, first):
    out = []
    for j in range(len(first) - 1):
        b = b"".join(host[o:o + n].tobytes() for o, n in segs[first[j]:first[j + 1]])
        out.append(oracle_mod.crc(method, np.frombuffer(b, dtype=np.uint8)))
    return out


# the chunk map serves the CRC-64 queue pass only: its caps are CRC-64 cases
@pytest.mark.parametrize("method,map_cap", [("crc32c", None), ("crc64", None), ("crc64-ecma182", None),
                                            ("crc64", "0"), ("crc64", "40")])
def test_segments_random_objects(gpu, buf, oracle_mod, method, map_cap, monkeypatch):
    """map_cap: the CRC-64 queue pass finds each chunk's segment in the scan's
    chunk map; "0" forces the search over the chunk prefix sums, "40" a map
    too small for the list (searched too, after partial map writes)."""
    if map_cap is not None:
        monkeypatch.setenv("MCHECKSUM_GPU_SEG_MAP_CAP", map_cap)
    rng = np.random.default_rng(77 if method == "crc32c" else 78)
    host = _host(buf)
    segs, first = _objects(rng, buf.numel() - 64, 120)
    views = [buf[o:o + n] for o, n in segs]
    got = gpu.as_unsigned(gpu.checksum_segments(method, views, first))
    assert got.tolist() == _want(oracle_mod, method, host, segs, first)


@pytest.mark.parametrize("method,map_cap", [("crc32c", None), ("crc64", None), ("crc64", "0")])
def test_segments_one_huge_segment_and_chunk_edges(gpu, buf, oracle_mod, method, map_cap, monkeypatch):
    """One 20 MiB segment (80 chunks) and objects whose segment lengths sit on
    and around the 256 KiB chunk size; map_cap "0": chunk -> segment by search."""
    if map_cap is not None:
        monkeypatch.setenv("MCHECKSUM_GPU_SEG_MAP_CAP", map_cap)
    host = _host(buf)
    big = [(3, 20 << 20)]
    got = gpu.as_unsigned(gpu.checksum_segments(method, [buf[3:3 + (20 << 20)]]))
    assert got.tolist() == _want(oracle_mod, method, host, big, [0, 1])
    k = 256 << 10
    segs = [(11, k - 1), (5000, k), (9, k + 1), (77, 2 * k), (1 << 20, 3 * k + 13), (0, 0), (123, 1)]
    first = [0, 1, 2, 3, 4, 5, 7, 7]
    got = gpu.as_unsigned(gpu.checksum_segments(method, [buf[o:o + n] for o, n in segs], first))
    assert got.tolist() == _want(oracle_mod, method, host, segs, first)


def test_segments_match_streaming_api_and_edges(gpu, buf):
    """Per-segment mchecksum_update (what a host would do) equals the GPU value;
    empty objects give the CRC of the empty message; segments outside
    [first[0], first[-1]) are ignored."""
    from mercury_amd import Checksum
    host = _host(buf)
    rng = np.random.default_rng(5)
    segs, first = _objects(rng, 1 << 20, 30, lens=[0, 1, 2, 5, 9, 31, 200, 5000, 70000])
    for method in ("crc32c", "crc64"):
        got = gpu.as_unsigned(gpu.checksum_segments(method, [buf[o:o + n] for o, n in segs], first))
        for j in range(len(first) - 1):
            ck = Checksum(method)
            for o, n in segs[first[j]:first[j + 1]]:
                ck.update(host[o:o + n].tobytes())
            assert int(got[j]) == ck.get()
        # objects over a sub-range of the list
        sub = [3, 5, 5, 9]
        got2 = gpu.as_unsigned(gpu.checksum_segments(method, [buf[o:o + n] for o, n in segs], sub))
        for j in range(len(sub) - 1):
            ck = Checksum(method)
            for o, n in segs[sub[j]:sub[j + 1]]:
                ck.update(host[o:o + n].tobytes())
            assert int(got2[j]) == ck.get()
    empty = gpu.as_unsigned(gpu.checksum_segments("crc32c", [], [0, 0, 0]))
    assert empty.tolist() == [Checksum("crc32c").get()] * 2


def test_segments_reject_bad_arguments(gpu, buf):
    with pytest.raises(gpu.GpuChecksumError):
        gpu.checksum_segments("crc32c", [buf[:10]], [0, 2])
    with pytest.raises(gpu.GpuChecksumError):
        gpu.checksum_segments("crc16", [buf[:10]])  # no GPU segment kernel for 16-bit models
    L = gpu._lib()
    rc = L.mchecksum_gpu_checksum_segments(b"crc32c", buf.data_ptr(), buf.data_ptr(), 4, buf.data_ptr(), 1,
                                           buf.data_ptr(), 8, buf.data_ptr(), None)
    assert rc == -1  # workspace smaller than mchecksum_gpu_segments_work_size(4)


# ------------------------------------------------------------ core headers --
#
# The expected hashes come straight from the oracle (oracle.crc over the
# host-order field image each proc function streams into mchecksum_update,
# src/mercury_core_header.c:193-205 / 255-261), for every CRC-16 catalogue
# variant, plus the committed request/response fixtures
# (tests/golden/core_headers.json, oracle/gen_golden.py).

CRC16_VARIANTS = ["crc16-arc", "crc16-ibm-3740", "crc16-xmodem", "crc16-kermit", "crc16-umts", "crc16-t10-dif"]


def _request(rng, oracle_mod, variant):
    hg, proto, rid, flags, cookie = 0x48 | 0x47, 5, int(rng.integers(0, 2**63)), int(rng.integers(0, 256)), \
        int(rng.integers(0, 256))
    img = struct.pack("<BBQBB", hg, proto, rid, flags, cookie)  # HG_CORE_HEADER_CHECKSUM_UPDATE: host order
    h = oracle_mod.crc(variant, img)
    wire = struct.pack(">BBQBBH", hg, proto, rid, flags, cookie, h) + b"\0\0"  # hash union is 4 bytes
    assert len(wire) == 16
    return wire


def _response(rng, oracle_mod, variant):
    ret, flags, cookie = int(rng.integers(-128, 128)), int(rng.integers(0, 256)), int(rng.integers(0, 65536))
    img = struct.pack("<bBH", ret, flags, cookie)
    h = oracle_mod.crc(variant, img)
    wire = struct.pack(">bBHH", ret, flags, cookie, h) + b"\0" * 10  # pad is never proc'd: hash lands at 4
    assert len(wire) == 16
    return wire


def _golden_headers(kind, variant):
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "core_headers.json")))
    out = []
    for e in g[kind]:
        wire = bytes.fromhex(e["wire_fields"]) + struct.pack(">H", int(e[variant], 16))
        out.append(wire + b"\0" * (16 - len(wire)))
    return out


@pytest.mark.parametrize("variant", [None] + CRC16_VARIANTS)
@pytest.mark.parametrize("kind", ["request", "response"])
def test_core_headers(gpu, oracle_mod, kind, variant, monkeypatch):
    import torch
    if variant:
        monkeypatch.setenv("MCHECKSUM_CRC16_VARIANT", variant)
    name = variant or "crc16-t10-dif"  # the library's default "crc16"
    rng = np.random.default_rng(31 if kind == "request" else 32)
    gold = _golden_headers(kind, name)
    msgs = [bytearray(h) for h in gold]
    for i in range(3000 - len(gold)):
        hdr = (_request if kind == "request" else _response)(rng, oracle_mod, name)
        body = rng.integers(0, 256, size=int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        msgs.append(bytearray(hdr + body))
    hash_at = 12 if kind == "request" else 4
    flips = {7: 1, 100: hash_at, 101: hash_at + 1, 2500: 0, 2999: 3}   # covered bytes -> must fail
    quiet = {50: 14 if kind == "request" else 8}                        # pad byte -> must pass
    for i, b in list(flips.items()) + list(quiet.items()):
        msgs[i][b] ^= 0x10
    msgs[1234] = msgs[1234][:15]                                       # shorter than the header
    off = np.zeros(len(msgs) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    data = torch.zeros(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    data[:int(off[-1])].copy_(torch.from_numpy(np.frombuffer(b"".join(msgs), dtype=np.uint8).copy()))
    status, mism = gpu.verify_core_headers(data, torch.from_numpy(off.astype(np.int64)).cuda(), kind=kind,
                                           offsets_host=off)
    bad = sorted(np.nonzero(status.cpu().numpy())[0].tolist())
    assert bad == sorted(list(flips) + [1234])
    assert int(mism.item()) == len(flips) + 1


def test_core_header_values_pinned_to_oracle(oracle_mod):
    """The product's streaming CRC16 (fed field by field, as the proc code
    does) equals the oracle's on a request image (default crc16 =
    CRC-16/T10-DIF, parity unpinned vs upstream mchecksum)."""
    from mercury_amd import Checksum
    img = struct.pack("<BBQBB", 0x4F, 5, 0x0123456789ABCDEF, 0x81, 0x22)
    ck = Checksum("crc16")
    for a, b in ((0, 1), (1, 2), (2, 10), (10, 11), (11, 12)):
        ck.update(img[a:b])
    assert ck.get() == oracle_mod.crc("crc16", np.frombuffer(img, dtype=np.uint8))


def test_core_headers_reject_wide_methods(gpu):
    import torch
    data = torch.zeros(64, dtype=torch.uint8, device="cuda")
    offs = torch.tensor([0, 16], dtype=torch.int64, device="cuda")
    with pytest.raises(gpu.GpuChecksumError):
        gpu.verify_core_headers(data, offs, method="crc32c")
    with pytest.raises(gpu.GpuChecksumError):
        gpu.verify_core_headers(data, offs, kind="reply")


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
@pytest.mark.parametrize("layout", ["per5", "one_object", "empties_subrange"])
def test_segments_long_lists_multi_block_scan(gpu, buf, oracle_mod, method, layout):
    """300000 short segments: the single-pass scan runs in 293 blocks, each
    looking back over up to 292 predecessors (windows of 64).  Object tables:
    5 segments each; ONE object over all 293 blocks (every block's objects are
    found by the 64-ary search, the object's rows written across blocks); and
    runs of empty objects with a table covering only part of the list
    (segments outside it belong to no object)."""
    host = _host(buf)
    rng = np.random.default_rng(91)
    lens = rng.integers(0, 65, 300000)
    offs = rng.integers(0, buf.numel() - 128, 300000)
    if layout == "per5":
        first = list(range(0, 300001, 5))
    elif layout == "one_object":
        first = [0, 300000]
    else:
        cuts = np.sort(rng.integers(1000, 299000, 20000))
        cuts = np.repeat(cuts, rng.integers(1, 4, cuts.size))  # repeated cuts: runs of empty objects
        first = [1000] + [int(x) for x in cuts] + [299000]
    views = [buf[int(o):int(o) + int(n)] for o, n in zip(offs, lens)]
    got = gpu.as_unsigned(gpu.checksum_segments(method, views, first))
    nobj = len(first) - 1
    check = sorted(set(list(range(0, nobj, max(1, nobj // 600))) + [nobj - 1]))
    if layout == "empties_subrange":
        check += [j for j in range(nobj) if first[j] == first[j + 1]][:50]
    for j in check:
        b = b"".join(host[int(offs[s]):int(offs[s]) + int(lens[s])].tobytes() for s in range(first[j], first[j + 1]))
        assert int(got[j]) == oracle_mod.crc(method, np.frombuffer(b, dtype=np.uint8)), j
    segs = [(16 * int(o), 4096) for o in rng.integers(0, (buf.numel() - 8192) // 16, 3000)]
    first = list(range(0, 3001, 3))
    got = gpu.as_unsigned(gpu.checksum_segments(method, [buf[o:o + n] for o, n in segs], first))
    assert got.tolist() == _want(oracle_mod, method, host, segs, first)


@pytest.mark.parametrize("method", ["crc32c", "crc64", "crc64-ecma182"])
def test_segments_leading_empty_segments_across_scan_blocks(gpu, buf, oracle_mod, method):
    """The object's head chunk (the one that starts from the register init):
    the scan records each object's first non-empty segment when the object
    starts in the same 1024-segment scan block; objects that start in an
    earlier block fall back to comparing byte offsets.  Heads after leading
    empty segments -- inside the block, in the next block, two blocks on --
    and multi-chunk head segments (only their first chunk is the head)."""
    host = _host(buf)
    rng = np.random.default_rng(2024)
    n = 3200
    lens = [int(x) for x in rng.integers(1, 300, n)]
    for s in range(1000, 1024):   # object A = [1000, 1030): head in block 1
        lens[s] = 0
    for s in range(1030, 2053):   # object B = [1030, 2100): head two blocks on
        lens[s] = 0
    lens[2053] = 600000           # a 3-chunk head segment
    lens[10] = lens[11] = 0       # object [10, 20): head inside block 0
    lens[12] = (256 << 10) + 7
    lens[3070] = lens[3071] = 0   # object [3070, 3080): starts and heads in block 2
    offs = [int(o) for o in rng.integers(0, buf.numel() - 600064, n)]
    segs = list(zip(offs, lens))
    first = sorted(set([0, 10, 20, 500, 1000, 1030, 2100, 2500, 3070, 3080, n]))
    got = gpu.as_unsigned(gpu.checksum_segments(method, [buf[o:o + ln] for o, ln in segs], first))
    assert got.tolist() == _want(oracle_mod, method, host, segs, first)


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_segments_large_batch_non_temporal(gpu, buf, oracle_mod, method):
    """>= 512 MiB in one call takes the non-temporal loads (decided on the
    device from the scan's total): 640 segments of 1 MiB, views that reuse the
    24 MiB buffer at 16-B aligned offsets, 4 per object, plus a few ragged ones."""
    rng = np.random.default_rng(91 if method == "crc32c" else 92)
    host = _host(buf)
    mib = 1 << 20
    segs = [(16 * int(rng.integers(0, (buf.numel() - 64 - mib) // 16)), mib) for _ in range(640)]
    segs[5] = (segs[5][0] + 3, mib - 7)  # ragged: takes the generic pass
    first = list(range(0, 641, 4))
    got = gpu.as_unsigned(gpu.checksum_segments(method, [buf[o:o + n] for o, n in segs], first)).tolist()
    for j in (0, 1, 17, 80, 159):
        assert got[j] == _want(oracle_mod, method, host, segs[first[j]:first[j + 1]], [0, 4])[0], j


def test_segment_batch_raw_stream_destroyed_between_calls(gpu, buf, oracle_mod):
    """A SegmentBatch called on a raw hipStream_t that the caller then destroys,
    and next on another raw stream: the guard event of the first call was
    recorded right after it (a raw handle may be gone by the next call), so
    the second call waits on it safely and both results equal the oracle."""
    import ctypes
    import os
    import torch
    L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    L.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    L.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    host = _host(buf)
    rng = np.random.default_rng(405)
    segs, first = _objects(rng, buf.numel() - 64, 60)
    batch = gpu.SegmentBatch([buf[o:o + n] for o, n in segs], first)
    want = _want(oracle_mod, "crc64", host, segs, first)
    outs = []
    torch.cuda.synchronize()
    for rep in range(6):
        h = ctypes.c_void_p()
        assert L.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0
        o = torch.zeros(len(first) - 1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()  # o's zeroing done before the raw stream writes it
        batch.checksum("crc64", out=o, stream=h.value)
        assert L.hipStreamDestroy(h.value) == 0  # with the call possibly still in flight
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs:
        assert gpu.as_unsigned(o).tolist() == want


@pytest.mark.parametrize("how", ["external", "current"])
def test_segment_batch_external_stream_destroyed_between_calls(gpu, buf, oracle_mod, how):
    """As above, with the raw handle wrapped in torch.cuda.ExternalStream --
    passed as `stream` ("external") or made the current stream with
    torch.cuda.stream(...) and stream=None ("current"): torch does not own
    such a stream, so the guard event is recorded right after each call, never
    later on a handle the caller has destroyed."""
    import ctypes
    import os
    import torch
    L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    L.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    L.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    host = _host(buf)
    rng = np.random.default_rng(406)
    segs, first = _objects(rng, buf.numel() - 64, 60)
    batch = gpu.SegmentBatch([buf[o:o + n] for o, n in segs], first)
    want = _want(oracle_mod, "crc64", host, segs, first)
    outs = []
    torch.cuda.synchronize()
    for rep in range(6):
        h = ctypes.c_void_p()
        assert L.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0
        o = torch.zeros(len(first) - 1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        ext = torch.cuda.ExternalStream(h.value)
        if how == "external":
            batch.checksum("crc64", out=o, stream=ext)
        else:
            with torch.cuda.stream(ext):
                batch.checksum("crc64", out=o)
        assert batch._last[2] is not None, "no guard event recorded after a call on a stream torch does not own"
        del ext
        assert L.hipStreamDestroy(h.value) == 0  # with the call possibly still in flight
        outs.append(o)
    torch.cuda.synchronize()
    for o in outs:
        assert gpu.as_unsigned(o).tolist() == want
    # a pool stream still defers its event to the switch (no per-call marker)
    s1 = torch.cuda.Stream()
    o = torch.zeros(len(first) - 1, dtype=torch.int64, device="cuda")
    batch.checksum("crc64", out=o, stream=s1)
    assert batch._last[2] is None
    torch.cuda.synchronize()
    assert gpu.as_unsigned(o).tolist() == want


def test_segment_batch_calls_on_two_streams(gpu, buf, oracle_mod):
    """One SegmentBatch used on two streams back to back: the calls share its
    workspace, so the second waits for the first (gpu.SegmentBatch) and both
    results equal the oracle."""
    import torch
    host = _host(buf)
    rng = np.random.default_rng(404)
    segs, first = _objects(rng, buf.numel() - 64, 60)
    batch = gpu.SegmentBatch([buf[o:o + n] for o, n in segs], first)
    want = _want(oracle_mod, "crc64", host, segs, first)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = []
    for rep in range(20):
        o1 = torch.zeros(len(first) - 1, dtype=torch.int64, device="cuda")
        o2 = torch.zeros(len(first) - 1, dtype=torch.int64, device="cuda")
        batch.checksum("crc64", out=o1, stream=s1)
        batch.checksum("crc64", out=o2, stream=s2)
        outs += [o1, o2]
    torch.cuda.synchronize()
    for o in outs:
        assert gpu.as_unsigned(o).tolist() == want


# Small lists around one scan block (<= 1024 segments per scan block): the
# scan launch's look-back over one, exactly one and one-past-one blocks.
@pytest.mark.parametrize("method", ["crc32c", "crc64", "crc64-ecma182"])
@pytest.mark.parametrize("shape", ["one_segment", "few", "exactly_one_block", "one_past"])
def test_segments_around_one_scan_block(gpu, buf, oracle_mod, method, shape):
    host = _host(buf)
    import zlib
    rng = np.random.default_rng(zlib.crc32(f"{method}/{shape}".encode()))
    if shape == "one_segment":
        segs, first = [(5, 300000)], [0, 1]
    elif shape == "few":
        segs, first = _objects(rng, buf.numel() - 64, 3, max_seg=3)
    else:
        n = 1024 if shape == "exactly_one_block" else 1025
        lens = [int(x) for x in rng.choice([0, 1, 17, 1024, 4096, 70000], n)]
        segs = [(int(rng.integers(0, buf.numel() - 64 - ln)), ln) for ln in lens]
        first = sorted(set([0, n] + [int(x) for x in rng.integers(0, n, 40)]))
    want = _want(oracle_mod, method, host, segs, first)
    views = [buf[o:o + n] for o, n in segs]
    assert gpu.as_unsigned(gpu.checksum_segments(method, views, first)).tolist() == want


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_segments_one_workspace_different_lists(gpu, buf, oracle_mod, method):
    """One caller workspace reused by calls with different small lists, back to
    back on one stream: every call must see its own scan (epoch-tagged
    look-back descriptors, never the previous call's maps)."""
    import torch
    from mercury_amd import _lib
    L = _lib.load_library()
    host = _host(buf)
    rng = np.random.default_rng(2026)
    lists = []
    for k in range(4):
        segs, first = _objects(rng, buf.numel() - 64, 20 + 7 * k, max_seg=5)
        meta = torch.from_numpy(np.concatenate([
            np.asarray([buf.data_ptr() + o for o, _ in segs], dtype=np.uint64).view(np.int64),
            np.asarray([n for _, n in segs], dtype=np.int64), np.asarray(first, dtype=np.int64)])).cuda()
        lists.append((segs, first, meta, _want(oracle_mod, method, host, segs, first)))
    nmax = max(len(s) for s, _, _, _ in lists)
    work = torch.empty((L.mchecksum_gpu_segments_work_size(nmax) + 7) // 8, dtype=torch.int64, device="cuda")
    outs = []
    for rep in range(12):
        segs, first, meta, want = lists[rep % len(lists)]
        n, nobj, base = len(segs), len(first) - 1, meta.data_ptr()
        out = torch.empty(nobj, dtype=torch.int64 if method == "crc64" else torch.int32, device="cuda")
        assert L.mchecksum_gpu_checksum_segments(method.encode(), base, base + 8 * n, n, base + 16 * n, nobj,
                                                 work.data_ptr(), work.numel() * 8, out.data_ptr(),
                                                 torch.cuda.current_stream().cuda_stream) == 0
        outs.append((out, want))
    torch.cuda.synchronize()
    for rep, (out, want) in enumerate(outs):
        assert gpu.as_unsigned(out).tolist() == want, rep
