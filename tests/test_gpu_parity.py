"""GPU parity: the MI355X batch kernels vs the CPU oracle, bit for bit.

Every case runs through the C ABI (libmchecksum.so, via mercury_amd.gpu) on
device-resident bytes and compares with oracle/ on the same bytes.  Sizes the
oracle finishes in seconds are compared exhaustively; here the full BASELINE
shapes add size-independent properties (determinism, single-bit corruption
detected exactly where injected), and test_gpu_full_shapes.py checks every
payload of them against the oracle.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_C2 = 0x4D43310000000002
SEED_C3 = 0x4D43310000000003
SEED_C4 = 0x4D43310000000004
SEED_METRIC = 0x4D43310000000005
# crc32 (IEEE, reflected) and crc64-ecma182 (MSB-first: run as the reflected
# model conjugated by the per-byte bit reversal, outputs byte-swapped --
# crc_gpu_layout.h) cover the other catalogue forms the GPU path takes
METHODS = ["crc32c", "crc64", "crc32", "crc64-ecma182"]


def _dev_bytes(torch, host: np.ndarray, pad: int = 64):
    t = torch.zeros(host.size + pad, dtype=torch.uint8, device="cuda")
    if host.size:
        t[:host.size].copy_(torch.from_numpy(np.array(host, dtype=np.uint8)))
    return t


def _setenv(k, v):
    """Set (or with v None, clear) a library setting; the library reads them
    once, so it re-reads them here (conftest.reload_library_settings)."""
    from conftest import reload_library_settings
    if v is None:
        os.environ.pop(k, None)
    else:
        os.environ[k] = v
    reload_library_settings()


def _force_log2g(lg):
    _setenv("MCHECKSUM_GPU_LOG2G", None if lg is None else str(lg))


@pytest.fixture(autouse=True)
def _clean_env():
    yield
    for k in ("MCHECKSUM_GPU_LOG2G", "MCHECKSUM_GPU_FORCE_GENERIC", "MCHECKSUM_GPU_LIGHT"):
        _setenv(k, None)


@pytest.fixture(params=["full", "light"])
def layout(request):
    """Both CRC-32C table layouts: the 32x-replicated throughput layout and the
    light small-batch layout (MCHECKSUM_GPU_LIGHT forces the choice)."""
    _setenv("MCHECKSUM_GPU_LIGHT", "1" if request.param == "light" else "0")
    yield request.param
    _setenv("MCHECKSUM_GPU_LIGHT", None)


def test_selfcheck_small_known_answers(gpu, oracle_mod):
    import torch
    # catalogue check string and RFC 3720 vectors through the batch kernel
    cases = [b"123456789", bytes(32), b"\xff" * 32, bytes(range(32)), bytes(range(31, -1, -1))]
    want32 = [0xE3069283, 0x8A9136AA, 0x62A8AB43, 0x46DD794E, 0x113FDB5C]
    for data, w in zip(cases, want32):
        h = np.frombuffer(data, dtype=np.uint8)
        t = _dev_bytes(torch, h)
        got = gpu.as_unsigned(gpu.checksum_fixed("crc32c", t, len(data), count=1))[0]
        assert got == w, (data, hex(got), hex(w))
        got64 = gpu.as_unsigned(gpu.checksum_fixed("crc64", t, len(data), count=1))[0]
        assert got64 == oracle_mod.crc("crc64", data)
    t = _dev_bytes(torch, np.frombuffer(b"123456789", dtype=np.uint8))
    assert gpu.as_unsigned(gpu.checksum_fixed("crc64", t, 9, count=1))[0] == 0x995DC9BBDF1939FA


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("length,stride", [
    (4096, 4096), (65536, 65536), (1024, 1024), (256, 256), (16, 16),
    (4096, 4100), (1000, 1000), (3, 7), (0, 16), (1, 1), (17, 33), (65537, 65552), (4095, 4096), (100000, 100003),
])
def test_fixed_every_lane_width(gpu, oracle_mod, method, length, stride, layout):
    import torch
    count = 67
    nbytes = (count - 1) * stride + length
    host = oracle_mod.splitmix_bytes(nbytes + 16, SEED_C2 ^ length ^ (stride << 20))[:nbytes]
    t = _dev_bytes(torch, host)
    want = oracle_mod.batch_fixed(method, host, stride, length, count, nthreads=8)
    for lg in [None, 0, 1, 2, 3, 4, 5, 6]:
        _force_log2g(lg)
        got = gpu.as_unsigned(gpu.checksum_fixed(method, t, length, count=count, stride=stride))
        torch.cuda.synchronize()
        bad = np.nonzero(got.astype(np.uint64) != want)[0]
        assert bad.size == 0, f"lg={lg} first bad payload {bad[:5]}"


@pytest.mark.parametrize("method", METHODS)
def test_fixed_unaligned_base_generic_path(gpu, oracle_mod, method, layout):
    import torch
    length, count = 4096, 40
    host = oracle_mod.splitmix_bytes(count * length + 64, SEED_C2)
    t = _dev_bytes(torch, host)
    for shift in [1, 3, 8, 15]:
        view = t[shift:shift + count * length]
        want = oracle_mod.batch_fixed(method, host[shift:], length, length, count)
        got = gpu.as_unsigned(gpu.checksum_fixed(method, view, length, count=count))
        assert np.array_equal(got.astype(np.uint64), want), shift
    # the generic path forced on aligned data gives the same values
    _setenv("MCHECKSUM_GPU_FORCE_GENERIC", "1")
    want = oracle_mod.batch_fixed(method, host, length, length, count)
    got = gpu.as_unsigned(gpu.checksum_fixed(method, t, length, count=count))
    assert np.array_equal(got.astype(np.uint64), want)


@pytest.mark.parametrize("method", METHODS)
def test_offsets_varlen_c4_layout(gpu, oracle_mod, method, layout):
    import torch
    count = 3000  # C4 shape, scaled: U[64 B, 64 KiB] packed at byte granularity
    off = oracle_mod.varlen_offsets(SEED_C4, count)
    host = oracle_mod.splitmix_bytes(int(off[-1]) + 16, SEED_C4)[:int(off[-1])]
    t = _dev_bytes(torch, host)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    want = oracle_mod.batch_offsets(method, host, off, nthreads=8)
    got = gpu.as_unsigned(gpu.checksum_offsets(method, t, offs, offsets_host=off))
    bad = np.nonzero(got.astype(np.uint64) != want)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("method", METHODS)
def test_offsets_edge_cases(gpu, oracle_mod, method, layout):
    import torch
    rng = np.random.default_rng(7)
    lens = [0, 0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 0, 31, 32, 33, 63, 64, 65, 1023, 1024, 1025, 0]
    lens += list(rng.integers(0, 40, size=300)) + [70000, 0, 131072, 5]
    off = np.zeros(len(lens) + 1, dtype=np.uint64)
    off[1:] = np.cumsum(np.array(lens, dtype=np.uint64))
    host = oracle_mod.splitmix_bytes(int(off[-1]) + 16, 99)[:int(off[-1])]
    t = _dev_bytes(torch, host)
    want = oracle_mod.batch_offsets(method, host, off)
    got = gpu.as_unsigned(gpu.checksum_offsets(method, t, torch.from_numpy(off.astype(np.int64)).cuda(),
                                               offsets_host=off))
    bad = np.nonzero(got.astype(np.uint64) != want)[0]
    assert bad.size == 0, [(int(i), lens[i]) for i in bad[:10]]
    # fewer payloads than waves, and a single payload
    one = off[:2].copy()
    got1 = gpu.as_unsigned(gpu.checksum_offsets(method, t, torch.from_numpy(one.astype(np.int64)).cuda()))
    assert got1[0] == want[0]


@pytest.mark.parametrize("method", METHODS)
def test_all_zero_and_all_ones_batches(gpu, oracle_mod, method):
    import torch
    for fill in (0x00, 0xFF):
        length, count = 65536, 32
        host = np.full(length * count, fill, dtype=np.uint8)
        t = _dev_bytes(torch, host)
        want = oracle_mod.batch_fixed(method, host, length, length, count)
        got = gpu.as_unsigned(gpu.checksum_fixed(method, t, length, count=count))
        assert np.array_equal(got.astype(np.uint64), want)
        assert len(set(got.tolist())) == 1


def test_verify_detects_single_bit_corruption(gpu, oracle_mod, layout):
    import torch
    count = 500
    off = oracle_mod.varlen_offsets(SEED_C4 ^ 1, count)
    host = oracle_mod.splitmix_bytes(int(off[-1]) + 16, 5)[:int(off[-1])]
    t = _dev_bytes(torch, host)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    expected = gpu.checksum_offsets("crc32c", t, offs)
    status, mism = gpu.verify_offsets("crc32c", t, offs, expected)
    assert int(mism.item()) == 0 and int(status.sum().item()) == 0
    victims = [0, 17, 250, count - 1]
    rng = np.random.default_rng(3)
    for v in victims:
        pos = int(off[v]) + int(rng.integers(0, int(off[v + 1] - off[v])))
        t[pos] ^= 1 << int(rng.integers(0, 8))
    status, mism = gpu.verify_offsets("crc32c", t, offs, expected)
    assert int(mism.item()) == len(victims)
    assert sorted(np.nonzero(status.cpu().numpy())[0].tolist()) == victims


def test_c2_shape_exhaustive(gpu, oracle_mod):
    """C2: 65536 x 4 KiB CRC-32C, every payload checked."""
    import torch
    count, length = 65536, 4096
    t = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, SEED_C2)
    got = gpu.as_unsigned(gpu.checksum_fixed("crc32c", t, length, count=count))
    host = t[:count * length].cpu().numpy()
    assert np.array_equal(host[:4096], oracle_mod.splitmix_bytes(4096, SEED_C2))  # device generator == host
    want = oracle_mod.batch_fixed("crc32c", host, length, length, count, variant="sse42", nthreads=16)
    assert np.array_equal(got.astype(np.uint64), want)


def test_metric_shape_sampled_and_deterministic(gpu, oracle_mod):
    """Headline workload: 65536 x 64 KiB CRC-32C (4 GiB device-resident)."""
    import torch
    count, length = 65536, 65536
    t = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, SEED_METRIC)
    a = gpu.checksum_fixed("crc32c", t, length, count=count)
    b = gpu.checksum_fixed("crc32c", t, length, count=count)
    got = gpu.as_unsigned(a)
    assert torch.equal(a, b)
    rng = np.random.default_rng(11)
    idx = np.unique(np.concatenate([[0, 1, count - 1], rng.integers(0, count, 509)]))
    for i in idx:
        want = oracle_mod.splitmix_batch_fixed("crc32c", SEED_METRIC, length, length, int(i), 1)[0]
        assert got[i] == want, int(i)
    # a single flipped bit anywhere changes exactly that payload's CRC
    pos = 12345 * length + 777
    t[pos] ^= 0x10
    c = gpu.as_unsigned(gpu.checksum_fixed("crc32c", t, length, count=count))
    diff = np.nonzero(c != got)[0]
    assert diff.tolist() == [12345]
    del t


def test_c3_crc64_segments_sampled(gpu, oracle_mod):
    """C3: 8192 x 1 MiB CRC-64 bulk segments."""
    import torch
    count, length = 8192, 1 << 20
    t = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(t, SEED_C3)
    got = gpu.as_unsigned(gpu.checksum_fixed("crc64", t, length, count=count))
    rng = np.random.default_rng(13)
    idx = np.unique(np.concatenate([[0, count - 1], rng.integers(0, count, 30)]))
    want = {int(i): oracle_mod.splitmix_batch_fixed("crc64", SEED_C3, length, length, int(i), 1)[0] for i in idx}
    for i, w in want.items():
        assert got[i] == w, i
    del t


def test_gpu_matches_streaming_api(gpu, oracle_mod):
    """The batch value equals what the drop-in streaming API returns."""
    import torch
    from mercury_amd import Checksum
    host = oracle_mod.splitmix_bytes(20000, 42)
    t = _dev_bytes(torch, host)
    for method in METHODS:
        got = gpu.as_unsigned(gpu.checksum_fixed(method, t, 20000, count=1))[0]
        c = Checksum(method)
        for a, b in [(0, 1), (1, 9), (9, 4096), (4096, 20000)]:  # per-field style updates
            c.update(host[a:b].tobytes())
        assert c.get() == got


@pytest.mark.parametrize("count,length,extra,method", [(37, 512 << 10, 0, "crc64"), (5, 2 << 20, 4096, "crc64"),
                                                       (3, 16 << 20, 16, "crc64"), (1, 1 << 20, 0, "crc64"),
                                                       (9, 1 << 20, 0, "crc64"), (9, 1 << 20, 0, "crc64-ecma182")])
def test_crc64_split_pieces(gpu, oracle_mod, monkeypatch, count, length, extra, method):
    """CRC-64 payloads of whole 256 KiB pieces go to the work queue piece by
    piece and are recombined with Z^n shifts (crc64_batch_kernel<..., SPLIT>):
    forced on with MCHECKSUM_GPU_SPLIT=1 at these small sizes, equal to the
    oracle and to the unsplit kernel (MCHECKSUM_GPU_SPLIT=0)."""
    import torch
    stride = length + extra
    host = oracle_mod.splitmix_bytes(stride * (count - 1) + length, 0x5B17 + count)
    dev = _dev_bytes(torch, host)
    want = oracle_mod.batch_fixed(method, host, stride, length, count, nthreads=8)
    stale = torch.full((count,), -1, dtype=torch.int64, device="cuda")  # the split path zeroes out[] itself
    monkeypatch.setenv("MCHECKSUM_GPU_SPLIT", "1")
    got = gpu.as_unsigned(gpu.checksum_fixed(method, dev, length, count=count, stride=stride, out=stale))
    monkeypatch.setenv("MCHECKSUM_GPU_SPLIT", "0")
    plain = gpu.as_unsigned(gpu.checksum_fixed(method, dev, length, count=count, stride=stride))
    assert np.array_equal(got.astype(np.uint64), want)
    assert np.array_equal(plain.astype(np.uint64), want)


def test_msb_first_method_verify(gpu, oracle_mod):
    """MSB-first methods: checksum outputs are byte-swapped after the launch,
    verify swaps the kernel's value before comparing (BatchArgs::bswap) --
    both agree with the oracle, and a flipped bit is flagged where it is."""
    import torch
    rng = np.random.default_rng(11)
    off = np.zeros(401, dtype=np.uint64)
    off[1:] = np.cumsum(rng.integers(0, 9000, 400))
    host = oracle_mod.splitmix_bytes(int(off[-1]) + 16, 3)[:int(off[-1])]
    t = _dev_bytes(torch, host)
    offs = torch.from_numpy(off.astype(np.int64)).cuda()
    want = oracle_mod.batch_offsets("crc64-ecma182", host, off, nthreads=8)
    got = gpu.as_unsigned(gpu.checksum_offsets("crc64-ecma182", t, offs))
    assert np.array_equal(got.astype(np.uint64), want)
    exp = torch.from_numpy(want.astype(np.uint64).view(np.int64)).cuda()
    st, bad = gpu.verify_offsets("crc64-ecma182", t, offs, exp)
    assert int(bad.item()) == 0 and int(st.sum().item()) == 0
    victim = int(np.nonzero(np.diff(off) > 0)[0][7])
    t[int(off[victim])] ^= 0x20
    st, bad = gpu.verify_offsets("crc64-ecma182", t, offs, exp)
    assert int(bad.item()) == 1 and np.nonzero(st.cpu().numpy())[0].tolist() == [victim]


def test_strided_out_is_refused(gpu):
    """the kernels write `count` contiguous values at
    out.data_ptr(), so a strided out view is refused on every entry point
    that takes one, before any launch."""
    import torch
    data = torch.zeros(8 * 4096 + 64, dtype=torch.uint8, device="cuda")
    offs = torch.arange(0, 9 * 4096, 4096, dtype=torch.int64, device="cuda")
    strided = torch.empty(16, dtype=torch.int32, device="cuda")[::2]
    assert strided.numel() == 8 and not strided.is_contiguous()
    with pytest.raises(gpu.GpuChecksumError, match="contiguous"):
        gpu.checksum_fixed("crc32c", data, 4096, count=8, out=strided)
    with pytest.raises(gpu.GpuChecksumError, match="contiguous"):
        gpu.checksum_offsets("crc32c", data, offs, out=strided)
    with pytest.raises(gpu.GpuChecksumError, match="contiguous"):
        gpu.checksum_xdr("crc32c", data, offs, [(2, 0)], out=strided)
