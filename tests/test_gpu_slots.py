"""Work-queue slot lifecycle.

A slot (crc_gpu_device.h: the work-queue counters) belongs to one stream at a
time (mchecksum_gpu.hip, queue_slot):

* a stream keeps its slot across launches (they never overlap);
* once all 2048 slots are owned, a new stream takes over the least recently
  used slot whose issued launches have all completed (the kernels count each
  completed launch in the slot) -- a busy one is passed over;
* a stream destroyed with launches in flight: hipStreamDestroy returns only
  after its work has completed, so a new stream that receives the same handle
  (and thereby the slot) never overlaps the old stream's launches.

Reference values come from the oracle or from a first launch (itself
oracle-checked).  The threading contract these serve is SURVEY.md 8(b)
(distinct objects used concurrently, /root/reference/src/CMakeLists.txt:22-27).
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NOT_READY = 600  # hipErrorNotReady


@pytest.fixture(scope="module")
def hip():
    import torch
    L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    vp = ctypes.c_void_p
    L.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    L.hipStreamDestroy.argtypes = [vp]
    L.hipStreamSynchronize.argtypes = [vp]
    L.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    L.hipEventRecord.argtypes = [vp, vp]
    L.hipEventQuery.argtypes = [vp]
    L.hipEventDestroy.argtypes = [vp]
    return L


def _stream(hip):
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0  # hipStreamNonBlocking
    return s.value


def _event(hip):
    e = ctypes.c_void_p()
    assert hip.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0  # hipEventDisableTiming
    return e.value


@pytest.fixture(scope="module")
def small_batch(gpu, oracle_mod):
    """2000 payloads U[64 B, 1 KiB], byte-packed: > 1024 payloads, so the
    throughput layout with the work queue runs (one slot per launch)."""
    import torch
    rng = np.random.default_rng(77)
    off = np.zeros(2001, dtype=np.int64)
    off[1:] = np.cumsum(rng.integers(64, 1025, 2000))
    host = oracle_mod.splitmix_bytes(int(off[-1]), 0x51075)
    data = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
    want = oracle_mod.batch_offsets("crc32c", host, off.astype(np.uint64))
    return data, torch.from_numpy(off).cuda(), want


@pytest.mark.parametrize("alive", [1, 2500])
def test_stream_churn_keeps_the_queue_path(gpu, hip, small_batch, alive):
    """5000 streams created, used once and destroyed `alive` iterations later
    (1: the runtime hands the freed handle straight back; 2500: more distinct
    streams than slots, so owners must be recycled): every launch still gets a
    slot, and every result is exact."""
    import torch
    data, offs, want = small_batch
    n = offs.numel() - 1
    outs = torch.empty((5000, n), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    st0 = gpu.queue_stats()
    live, handles = [], set()
    for i in range(5000):
        s = _stream(hip)
        handles.add(s)
        gpu.checksum_offsets("crc32c", data, offs, out=outs[i], stream=s)
        live.append(s)
        if len(live) >= alive:
            assert hip.hipStreamDestroy(live.pop(0)) == 0
    for s in live:
        assert hip.hipStreamDestroy(s) == 0
    torch.cuda.synchronize()
    st1 = gpu.queue_stats()
    print(f"{len(handles)} distinct handles, stats {st0} -> {st1}")
    assert st1["slot"] - st0["slot"] == 5000, (st0, st1)
    assert st1["noslot"] == st0["noslot"], (st0, st1)
    if alive > 2048:
        assert len(handles) > 2048
        # (handles already owning a slot before the test need no reclaim)
        assert st1["reclaim"] - st0["reclaim"] >= len(handles) - 2048 - st0["owners"], (st0, st1)
    assert st1["owners"] <= 2048
    bad = torch.nonzero((outs != torch.from_numpy(want.astype(np.uint32).view(np.int32)).cuda()).any(dim=1))
    assert bad.numel() == 0, bad.flatten()[:8].tolist()


def test_destroy_with_launches_in_flight(gpu, hip, oracle_mod):
    """Destroy a stream right after queueing large batches on it, create a
    new one (often with the same handle, hence the same slot) and use it at
    once: hipStreamDestroy must have waited for the old work, and both
    streams' results are exact."""
    import torch
    count, length, seed = 16384, 65536, 0xDE57  # 1 GiB: non-temporal, work queue
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    gpu.fill_splitmix(data, seed)
    ref = gpu.checksum_fixed("crc32c", data, length, count=count)
    torch.cuda.synchronize()
    got = gpu.as_unsigned(ref)
    for i in np.random.default_rng(5).integers(0, count, 16):
        assert got[i] == oracle_mod.splitmix_batch_fixed("crc32c", seed, length, length, int(i), 1)[0]
    outs = [torch.empty(count, dtype=torch.int32, device="cuda") for _ in range(21)]
    reused = 0
    for trial in range(3):
        s1 = _stream(hip)
        for k in range(20):
            gpu.checksum_fixed("crc32c", data, length, count=count, out=outs[k], stream=s1)
        ev = _event(hip)
        assert hip.hipEventRecord(ev, s1) == 0
        pending = hip.hipEventQuery(ev) == NOT_READY
        assert hip.hipStreamDestroy(s1) == 0
        # the destroyed stream's work is complete once destroy has returned
        assert hip.hipEventQuery(ev) == 0, "hipStreamDestroy returned with the stream's launches in flight"
        s2 = _stream(hip)
        reused += s2 == s1
        gpu.checksum_fixed("crc32c", data, length, count=count, out=outs[20], stream=s2)
        assert hip.hipStreamSynchronize(s2) == 0
        assert hip.hipStreamDestroy(s2) == 0
        assert hip.hipEventDestroy(ev) == 0
        for k, o in enumerate(outs):
            assert torch.equal(o, ref), (trial, k, pending)
    print(f"handle reused in {reused}/3 trials")


def test_full_table_passes_over_a_busy_slot(gpu, hip, small_batch):
    """With every slot owned, a new stream must not take the least recently
    used slot while that slot's stream still has a launch queued behind a
    long-running kernel; it takes the next idle one."""
    import torch
    data, offs, want = small_batch
    n = offs.numel() - 1
    want_t = torch.from_numpy(want.astype(np.uint32).view(np.int32)).cuda()
    streams = [_stream(hip) for _ in range(2048)]
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    try:
        for s in streams:  # afterwards the 2048 slots all belong to these streams, streams[0]'s the LRU
            gpu.checksum_offsets("crc32c", data, offs, out=out, stream=s)
        torch.cuda.synchronize()
        # streams[0]: a long sleep kernel, then a launch on its slot -> the slot
        # stays busy (issued > completed) until the sleep ends
        # (calibrate torch's sleep kernel: cycles per second of its clock)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(50_000_000)
        b.record()
        torch.cuda.synchronize()
        per_s = 50_000_000 / max(a.elapsed_time(b) * 1e-3, 1e-6)
        ext = torch.cuda.ExternalStream(streams[0])
        ev = _event(hip)
        with torch.cuda.stream(ext):
            torch.cuda._sleep(int(8 * per_s))  # ~8 s, far longer than the 2047 launches below
            busy_out = torch.empty(n, dtype=torch.int32, device="cuda")
            gpu.checksum_offsets("crc32c", data, offs, out=busy_out, stream=streams[0])
        assert hip.hipEventRecord(ev, streams[0]) == 0
        # ... then touch every other owner, so streams[0]'s slot is the LRU again
        for s in streams[1:]:
            gpu.checksum_offsets("crc32c", data, offs, out=out, stream=s)
        for s in streams[1:]:
            assert hip.hipStreamSynchronize(s) == 0
        if hip.hipEventQuery(ev) != NOT_READY:
            pytest.skip("the sleep kernel ended before the new stream arrived")
        st0 = gpu.queue_stats()
        x = _stream(hip)
        xo = torch.empty(n, dtype=torch.int32, device="cuda")
        gpu.checksum_offsets("crc32c", data, offs, out=xo, stream=x)
        st1 = gpu.queue_stats()
        assert st1["busy_skip"] - st0["busy_skip"] >= 1, (st0, st1)
        assert st1["reclaim"] - st0["reclaim"] == 1 and st1["slot"] - st0["slot"] == 1, (st0, st1)
        assert hip.hipStreamSynchronize(x) == 0
        assert hip.hipStreamSynchronize(streams[0]) == 0
        assert torch.equal(xo, want_t) and torch.equal(busy_out, want_t) and torch.equal(out, want_t)
        assert hip.hipStreamDestroy(x) == 0
        assert hip.hipEventDestroy(ev) == 0
    finally:
        torch.cuda.synchronize()
        for s in streams:
            hip.hipStreamDestroy(s)
