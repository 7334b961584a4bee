"""Fail-closed work queue (include/mchecksum_gpu.h, "Fail closed").

build/libmchecksum_qfault.so is libmchecksum built with -DMCK_QFAULT_TEST=1:
in every launch that takes the work queue, workgroup 3 gives up the first unit
of its second chunk, exactly as a wave whose bounded wait timed out would
(crc_gpu_device.h, for_each_unit).  Such a launch must never report unhashed
bytes as good -- the contract hg_get_struct relies on when it turns a failed
check into HG_CHECKSUM_ERROR (/root/reference/src/mercury.c:565-573):

* checksum calls add 1 to the caller's error word (mchecksum_gpu_set_error_word);
* verify calls add `count` to the mismatch counter, and every payload's status
  ends as its true verdict or 1 -- never a stale 0 (status is pre-filled with 0
  here, so only the kernel can have flagged it).

Reference values come from the product library (itself checked against the
oracle by the parity suites).
"""
import ctypes
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QLIB = os.path.join(ROOT, "build", "libmchecksum_qfault.so")


@pytest.fixture(scope="module")
def qlib(gpu):
    assert os.path.exists(QLIB), "build/libmchecksum_qfault.so missing: run make"
    L = ctypes.CDLL(QLIB)
    c = ctypes
    L.mchecksum_gpu_prepare.argtypes = [c.c_char_p]
    L.mchecksum_gpu_checksum_offsets.argtypes = [c.c_char_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p,
                                                 c.c_void_p]
    L.mchecksum_gpu_checksum_fixed.argtypes = [c.c_char_p, c.c_void_p, c.c_size_t, c.c_size_t, c.c_size_t,
                                               c.c_void_p, c.c_void_p]
    L.mchecksum_gpu_verify_offsets.argtypes = [c.c_char_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p,
                                               c.c_void_p, c.c_void_p, c.c_void_p]
    L.mchecksum_gpu_checksum_segments.argtypes = [c.c_char_p, c.c_void_p, c.c_void_p, c.c_size_t, c.c_void_p,
                                                  c.c_size_t, c.c_void_p, c.c_size_t, c.c_void_p, c.c_void_p]
    L.mchecksum_gpu_segments_work_size.argtypes = [c.c_size_t]
    L.mchecksum_gpu_segments_work_size.restype = c.c_size_t
    L.mchecksum_gpu_set_error_word.argtypes = [c.c_void_p]
    L.mchecksum_gpu_queue_faults.restype = c.c_longlong
    L.mchecksum_gpu_reload_settings.restype = None
    return L


@pytest.fixture(autouse=True)
def _qlib_settings(request):
    """The fault-injecting library reads its MCHECKSUM_GPU_QFAULT_* settings
    once, like the product library: re-read them after each test has set
    (monkeypatch, undone by now) or left them."""
    yield
    if "qlib" in request.fixturenames:
        request.getfixturevalue("qlib").mchecksum_gpu_reload_settings()


def _qsetenv(monkeypatch, qlib, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    qlib.mchecksum_gpu_reload_settings()


@pytest.fixture(scope="module")
def batch(gpu):
    """20000 payloads U[64 B, 8 KiB] packed at byte granularity: > 1024 payloads,
    so the throughput layout with the work queue runs."""
    import torch
    rng = np.random.default_rng(2024)
    lens = rng.integers(64, 8193, 20000)
    off = np.zeros(len(lens) + 1, dtype=np.int64)
    off[1:] = np.cumsum(lens)
    data = torch.empty(int(off[-1]) + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, 0xFA17)
    return data, torch.from_numpy(off).cuda()


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_checksum_fault_bumps_error_word(gpu, qlib, batch, method):
    import torch
    data, offs = batch
    n = offs.numel() - 1
    want = gpu.checksum_offsets(method, data, offs)
    out = ~want  # every entry wrong until a launch writes it
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    faults0 = qlib.mchecksum_gpu_queue_faults()
    assert qlib.mchecksum_gpu_prepare(method.encode()) == 0
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        rc = qlib.mchecksum_gpu_checksum_offsets(method.encode(), data.data_ptr(), offs.data_ptr(), n,
                                                 out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert rc == 0
    torch.cuda.synchronize()
    assert int(word.item()) == 1, "a launch that dropped a unit must bump the error word"
    assert qlib.mchecksum_gpu_queue_faults() - faults0 == 1
    lost = np.nonzero((out != want).cpu().numpy())[0]
    assert len(lost) == 1, lost[:8]  # exactly the injected unit went unhashed; the rest is right


def test_verify_fault_fails_closed(gpu, qlib, batch):
    import torch
    data, offs = batch
    n = offs.numel() - 1
    truth = gpu.checksum_offsets("crc32c", data, offs)
    expected = truth.clone()
    bad = np.arange(0, n, 7)
    expected[torch.from_numpy(bad).cuda()] ^= 0x100  # a genuine mismatch every 7th payload
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")  # stale "pass" everywhere
    mism = torch.zeros(1, dtype=torch.int32, device="cuda")
    assert qlib.mchecksum_gpu_verify_offsets(b"crc32c", data.data_ptr(), offs.data_ptr(), n, expected.data_ptr(),
                                             status.data_ptr(), mism.data_ptr(),
                                             torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert int(mism.item()) >= n, "a faulted verify must not read as clean"
    assert set(np.unique(st).tolist()) <= {0, 1}
    assert np.all(st[bad] == 1), "a real mismatch read as verified"
    # every 0 is a payload whose bytes really match; the unhashed one is among
    # the 1s (the status sweep left it flagged)
    ok = st == 0
    assert np.array_equal(expected.cpu().numpy()[ok], truth.cpu().numpy()[ok])
    assert int((st == 1).sum()) > len(bad)


def test_large_fixed_batch_fault(gpu, qlib):
    """A >= 512 MiB aligned CRC-32C batch (non-temporal loads) also takes the
    queue: same report."""
    import torch
    count, length = 8192, 65536
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, 0x5EED)
    want = gpu.checksum_fixed("crc32c", data, length, count=count)
    out = ~want
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        assert qlib.mchecksum_gpu_checksum_fixed(b"crc32c", data.data_ptr(), length, length, count, out.data_ptr(),
                                                 torch.cuda.current_stream().cuda_stream) == 0
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    torch.cuda.synchronize()
    assert int(word.item()) == 1
    assert int((out != want).sum().item()) == 1


def test_segment_chunk_queue_fault(gpu, qlib):
    """The CRC-64 scatter-gather chunk pass (mchecksum_gpu_ext.hip, seg_kernel
    with the work queue) in the fault-injecting build: the dropped chunk leaves
    exactly one object wrong, the caller's error word gets +1, and the
    process-wide fault count (which sums both translation units' counters)
    rises by one."""
    import torch
    nobj, nseg_per, seg = 128, 4, 1 << 20  # 2048 aligned 256 KiB chunks: two+ per workgroup
    data = torch.empty(nobj * nseg_per * seg + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, 0x5E6F)
    segs = [data[i * seg:(i + 1) * seg] for i in range(nobj * nseg_per)]
    first = np.arange(0, nobj * nseg_per + 1, nseg_per)
    batch = gpu.SegmentBatch(segs, first)
    want = batch.checksum("crc64").clone()
    torch.cuda.synchronize()
    out = ~want
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    n = batch.nseg
    base = batch.meta.data_ptr()
    faults0 = qlib.mchecksum_gpu_queue_faults()
    assert qlib.mchecksum_gpu_prepare(b"crc64") == 0
    work = torch.empty((qlib.mchecksum_gpu_segments_work_size(n) + 7) // 8, dtype=torch.int64, device="cuda")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        rc = qlib.mchecksum_gpu_checksum_segments(b"crc64", base, base + 8 * n, n, base + 16 * n, batch.nobj,
                                                  work.data_ptr(), work.numel() * 8, out.data_ptr(),
                                                  torch.cuda.current_stream().cuda_stream)
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert rc == 0
    torch.cuda.synchronize()
    assert int(word.item()) == 1, "a chunk pass that dropped a chunk must bump the error word"
    assert qlib.mchecksum_gpu_queue_faults() - faults0 == 1, "the segment kernels' fault count must be reported"
    lost = np.nonzero((out != want).cpu().numpy())[0]
    assert len(lost) == 1, lost[:8]


def test_product_library_reports_no_fault(gpu, batch):
    """The same calls through the product library: error word stays 0."""
    import torch
    data, offs = batch
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    gpu.set_error_word(word)
    try:
        for method in ("crc32c", "crc64"):
            gpu.checksum_offsets(method, data, offs)
        exp = gpu.checksum_offsets("crc32c", data, offs)
        st, m = gpu.verify_offsets("crc32c", data, offs, exp)
    finally:
        gpu.set_error_word(None)
    torch.cuda.synchronize()
    assert int(word.item()) == 0 and int(m.item()) == 0 and int(st.sum().item()) == 0


def test_segment_scan_lookback_fault(gpu, qlib, monkeypatch):
    """The one-launch segment scan's look-back in the fault-injecting build
    (MCHECKSUM_GPU_QFAULT_SCAN=1: scan block 1 gives up its wait): the call
    returns, and the caller's error word reports the failed scan once: the
    chunk pass sees the scan's fault claim and hashes nothing (so its own
    injected drop never happens either) -- one increment per call."""
    import torch
    _qsetenv(monkeypatch, qlib, MCHECKSUM_GPU_QFAULT_SCAN="1")
    nseg = 3000  # three scan blocks
    data = torch.empty(nseg * 4096 + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, 0x5CA1)
    segs = [data[i * 4096:(i + 1) * 4096] for i in range(nseg)]
    batch = gpu.SegmentBatch(segs, np.arange(0, nseg + 1, 3))
    torch.cuda.synchronize()
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    n, base = batch.nseg, batch.meta.data_ptr()
    out = torch.zeros(batch.nobj, dtype=torch.int64, device="cuda")
    faults0 = qlib.mchecksum_gpu_queue_faults()
    assert qlib.mchecksum_gpu_prepare(b"crc64") == 0
    work = torch.empty((qlib.mchecksum_gpu_segments_work_size(n) + 7) // 8, dtype=torch.int64, device="cuda")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        rc = qlib.mchecksum_gpu_checksum_segments(b"crc64", base, base + 8 * n, n, base + 16 * n, batch.nobj,
                                                  work.data_ptr(), work.numel() * 8, out.data_ptr(),
                                                  torch.cuda.current_stream().cuda_stream)
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert rc == 0
    torch.cuda.synchronize()
    assert int(word.item()) == 1, "a failed call must bump the error word exactly once"
    assert qlib.mchecksum_gpu_queue_faults() - faults0 >= 1


# Deadline waits (crc_gpu_device.h, Deadline): 1 s of the 100 MHz real-time
# counter, and once one wait of a call has given up every other one gives up
# at once (the abort flag; a segments call whose scan failed hashes nothing).
# A call whose waits are never satisfied returns within about one deadline
# and reports itself failed -- whatever the per-poll cost under contention.
STALL_MAX_S = 1.5


def _timed(fn):
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


@pytest.mark.parametrize("method", ["crc32c", "crc64"])
def test_ring_entry_never_published_times_out(gpu, qlib, batch, method, monkeypatch):
    """MCHECKSUM_GPU_QFAULT_MODE=stall: workgroup 3 never publishes its third
    chunk, so its waves wait on that ring entry until the deadline.  The other
    workgroups take every unit (no chunk is lost), so every CRC is right -- and
    the call still reports the failed wait on the error word, exactly once."""
    import torch
    data, offs = batch
    n = offs.numel() - 1
    want = gpu.checksum_offsets(method, data, offs)
    out = ~want
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    faults0 = qlib.mchecksum_gpu_queue_faults()
    assert qlib.mchecksum_gpu_prepare(method.encode()) == 0
    _qsetenv(monkeypatch, qlib, MCHECKSUM_GPU_QFAULT_MODE="stall")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        rc = []
        dt = _timed(lambda: rc.append(qlib.mchecksum_gpu_checksum_offsets(
            method.encode(), data.data_ptr(), offs.data_ptr(), n, out.data_ptr(),
            torch.cuda.current_stream().cuda_stream)))
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert rc == [0]
    print(f"stalled launch returned after {dt:.3f} s")
    assert 0.9 <= dt <= STALL_MAX_S, f"deadline wait took {dt:.3f} s"
    assert int(word.item()) == 1, "a launch whose waves timed out must bump the error word once"
    assert qlib.mchecksum_gpu_queue_faults() - faults0 >= 1
    assert torch.equal(out, want), "no unit is lost by the stall: every CRC must be right"


def test_verify_with_stalled_entry_never_reads_clean(gpu, qlib, batch, monkeypatch):
    """A verify launch whose waves time out: the mismatch count covers the
    batch and every status ends flagged or truly verified -- never a stale 0."""
    import torch
    data, offs = batch
    n = offs.numel() - 1
    truth = gpu.checksum_offsets("crc32c", data, offs)
    expected = truth.clone()
    bad = np.arange(3, n, 11)
    expected[torch.from_numpy(bad).cuda()] ^= 0x4000
    status = torch.zeros(n, dtype=torch.uint8, device="cuda")
    mism = torch.zeros(1, dtype=torch.int32, device="cuda")
    _qsetenv(monkeypatch, qlib, MCHECKSUM_GPU_QFAULT_MODE="stall")
    dt = _timed(lambda: qlib.mchecksum_gpu_verify_offsets(
        b"crc32c", data.data_ptr(), offs.data_ptr(), n, expected.data_ptr(), status.data_ptr(), mism.data_ptr(),
        torch.cuda.current_stream().cuda_stream))
    assert dt <= STALL_MAX_S, f"deadline wait took {dt:.3f} s"
    st = status.cpu().numpy()
    assert int(mism.item()) >= n
    assert np.all(st[bad] == 1), "a real mismatch read as verified"
    ok = st == 0
    assert np.array_equal(expected.cpu().numpy()[ok], truth.cpu().numpy()[ok])


def test_scan_descriptor_never_published_times_out(gpu, qlib, monkeypatch):
    """MCHECKSUM_GPU_QFAULT_SCAN=1 with MCHECKSUM_GPU_QFAULT_MODE=scanstall: scan
    block 1 never publishes its look-back descriptor, so the blocks after it
    wait until their deadlines.  The call returns within the bound and the
    error word reports it once, however many scan blocks gave up."""
    import torch
    nseg = 6000  # six scan blocks: 2..5 may all give up
    data = torch.empty(nseg * 4096 + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, 0x5CA2)
    segs = [data[i * 4096:(i + 1) * 4096] for i in range(nseg)]
    batch = gpu.SegmentBatch(segs, np.arange(0, nseg + 1, 3))
    torch.cuda.synchronize()
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    n, base = batch.nseg, batch.meta.data_ptr()
    out = torch.zeros(batch.nobj, dtype=torch.int64, device="cuda")
    faults0 = qlib.mchecksum_gpu_queue_faults()
    assert qlib.mchecksum_gpu_prepare(b"crc64") == 0
    work = torch.empty((qlib.mchecksum_gpu_segments_work_size(n) + 7) // 8, dtype=torch.int64, device="cuda")
    _qsetenv(monkeypatch, qlib, MCHECKSUM_GPU_QFAULT_SCAN="1", MCHECKSUM_GPU_QFAULT_MODE="scanstall")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        rc = []
        dt = _timed(lambda: rc.append(qlib.mchecksum_gpu_checksum_segments(
            b"crc64", base, base + 8 * n, n, base + 16 * n, batch.nobj, work.data_ptr(), work.numel() * 8,
            out.data_ptr(), torch.cuda.current_stream().cuda_stream)))
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert rc == [0]
    print(f"stalled scan returned after {dt:.3f} s")
    assert 0.9 <= dt <= STALL_MAX_S, f"deadline wait took {dt:.3f} s"
    assert int(word.item()) == 1, "a scan whose look-back timed out must bump the error word once"
    assert qlib.mchecksum_gpu_queue_faults() - faults0 >= 1


def _seg_call(gpu, qlib, nseg, seed, word, stream=None):
    """A CRC-64 segments call of nseg 4 KiB segments (3 per object) through the
    fault-injecting library; returns (callable issuing it, out, keep-alive)."""
    import torch
    data = torch.empty(nseg * 4096 + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, seed)
    segs = [data[i * 4096:(i + 1) * 4096] for i in range(nseg)]
    batch = gpu.SegmentBatch(segs, np.arange(0, nseg + 1, 3))
    n, base = batch.nseg, batch.meta.data_ptr()
    out = torch.zeros(batch.nobj, dtype=torch.int64, device="cuda")
    assert qlib.mchecksum_gpu_prepare(b"crc64") == 0
    work = torch.empty((qlib.mchecksum_gpu_segments_work_size(n) + 7) // 8, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()

    def call():
        s = stream if stream is not None else torch.cuda.current_stream()
        return qlib.mchecksum_gpu_checksum_segments(b"crc64", base, base + 8 * n, n, base + 16 * n, batch.nobj,
                                                    work.data_ptr(), work.numel() * 8, out.data_ptr(), s.cuda_stream)
    return call, out, (data, segs, batch, work)


def test_two_stalls_in_one_segments_call_cost_one_deadline(gpu, qlib, monkeypatch):
    """MCHECKSUM_GPU_QFAULT_MODE=stall+scanstall injects a
    scan stall (block 1 never publishes its descriptor) AND a ring stall
    (workgroup 3 never publishes a chunk) into one segments call.  Round 5
    spent a deadline on each (3.000 s in pytest_r05a.log); now the scan's
    give-up claims the call's fault and the chunk pass hashes nothing, so the
    call returns within one deadline and the error word rises exactly once."""
    import torch
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    call, out, keep = _seg_call(gpu, qlib, 6000, 0x5CA3, word)
    faults0 = qlib.mchecksum_gpu_queue_faults()
    _qsetenv(monkeypatch, qlib, MCHECKSUM_GPU_QFAULT_SCAN="1", MCHECKSUM_GPU_QFAULT_MODE="stall+scanstall")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        rc = []
        dt = _timed(lambda: rc.append(call()))
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert rc == [0]
    print(f"two stalls in one call returned after {dt:.3f} s")
    assert 0.9 <= dt <= STALL_MAX_S, f"the call took {dt:.3f} s"
    assert int(word.item()) == 1, "one failed call, one increment"
    assert qlib.mchecksum_gpu_queue_faults() - faults0 >= 1


def test_scan_fault_reported_on_every_graph_replay(gpu, qlib, monkeypatch):
    """a captured segments call replays its captured epoch, so the
    scan's fault claim is keyed by the epoch AND the workspace's call count
    (bumped by every scan): each replay whose scan gives up adds 1 to the
    error word, and so does each eager call on the same workspace."""
    import torch
    word = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    call, out, keep = _seg_call(gpu, qlib, 3000, 0x5CA4, word, stream=s)
    _qsetenv(monkeypatch, qlib, MCHECKSUM_GPU_QFAULT_SCAN="1")
    qlib.mchecksum_gpu_set_error_word(word.data_ptr())
    try:
        for _ in range(2):  # eager: +1 each
            assert call() == 0
        torch.cuda.synchronize()
        assert int(word.item()) == 2
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            assert call() == 0
        torch.cuda.synchronize()
        base = int(word.item())  # (capture itself launches nothing)
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
    finally:
        qlib.mchecksum_gpu_set_error_word(None)
    assert int(word.item()) - base == 3, "every failed replay must report"
