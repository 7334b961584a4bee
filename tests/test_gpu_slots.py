"""Work-queue slot lifecycle (round 4: a pool of idle slots).

A slot (crc_gpu_device.h: the work-queue counters of two banks) serves one
launch at a time (mchecksum_gpu.hip, queue_slot):

* every eager queue launch takes an idle slot from the device's pool and holds
  it until the launch completes -- the HIP event recorded by the launch's own
  completion (hipExtLaunchKernel's stop event), queried without blocking when
  the slot is reaped back into the pool;
* no stream owns a slot, so nothing rests on stream handles: a stream created
  after another was destroyed may get the same handle, and hipStreamDestroy
  need not wait for the old stream's launches (HIP does not promise it does);
* a slot whose launch is still queued is passed over; with no idle slot left
  and the oldest in-flight slots all busy, a launch takes the static split.

Reference values come from the oracle or from a first launch (itself
oracle-checked).  The threading contract these serve is SURVEY.md 8(b)
(distinct objects used concurrently, /root/reference/src/CMakeLists.txt:22-27).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
    (1: the runtime hands the freed handle straight back; 2500: more live
    streams than slots): every launch gets a slot -- the pool is reaped as
    launches complete -- and every result is exact."""
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
    assert st1["reaped"] - st0["reaped"] >= 5000 - 2048, (st0, st1)
    assert st1["in_flight"] <= 2048
    bad = torch.nonzero((outs != torch.from_numpy(want.astype(np.uint32).view(np.int32)).cuda()).any(dim=1))
    assert bad.numel() == 0, bad.flatten()[:8].tolist()


def test_destroy_with_launches_in_flight(gpu, hip, oracle_mod):
    """Destroy a stream right after queueing large batches on it, create a
    new one (often with the same handle) and use it at once: the new stream's
    launch takes an idle slot, never one of the old stream's in-flight ones,
    and both streams' results are exact -- whether or not hipStreamDestroy
    waited for the old work (recorded, not relied on)."""
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
    reused = waited = 0
    for trial in range(3):
        s1 = _stream(hip)
        st0 = gpu.queue_stats()
        for k in range(20):
            gpu.checksum_fixed("crc32c", data, length, count=count, out=outs[k], stream=s1)
        ev = _event(hip)
        assert hip.hipEventRecord(ev, s1) == 0
        pending = hip.hipEventQuery(ev) == NOT_READY
        assert hip.hipStreamDestroy(s1) == 0
        waited += hip.hipEventQuery(ev) == 0  # observed ROCm behaviour, not relied on
        s2 = _stream(hip)
        reused += s2 == s1
        gpu.checksum_fixed("crc32c", data, length, count=count, out=outs[20], stream=s2)
        st1 = gpu.queue_stats()
        assert st1["slot"] - st0["slot"] == 21, (st0, st1)  # 21 launches, 21 slots
        assert hip.hipStreamSynchronize(s2) == 0
        assert hip.hipStreamDestroy(s2) == 0
        assert hip.hipEventDestroy(ev) == 0
        for k, o in enumerate(outs):
            assert torch.equal(o, ref), (trial, k, pending)
    print(f"handle reused in {reused}/3 trials; hipStreamDestroy had waited in {waited}/3")


POOL = r"""
import os, sys, time
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from mercury_amd import gpu as G
from oracle import oracle as O
NSLOTS = int(os.environ["MCHECKSUM_GPU_QUEUE_SLOTS"])
rng = np.random.default_rng(77)
off = np.zeros(2001, dtype=np.int64)
off[1:] = np.cumsum(rng.integers(64, 1025, 2000))
host = O.splitmix_bytes(int(off[-1]), 0x51075)
data = torch.from_numpy(np.concatenate([host, np.zeros(64, np.uint8)])).cuda()
offs = torch.from_numpy(off).cuda()
want = torch.from_numpy(O.batch_offsets("crc32c", host, off.astype(np.uint64)).astype(np.uint32).view(np.int32)).cuda()
n = 2000
gate = G.HostGate()
A = torch.cuda.Stream()
G.checksum_offsets("crc32c", data, offs, stream=A); torch.cuda.synchronize()  # warm-up


def done_within(ev, seconds):
    t0 = time.monotonic()
    while not ev.query() and time.monotonic() - t0 < seconds:
        time.sleep(0.0005)
    return ev.query()


# B: a stream on another hardware queue than A (GPU_MAX_HW_QUEUES = 4 queues
# are shared round-robin by the process's streams): with A held by the gate,
# a candidate whose small kernel completes does not sit behind A.
gate.hold(A)
B, tried = None, 0
for prio in (0, -1):
    for _ in range(8):
        cand = torch.cuda.Stream(priority=prio)
        tried += 1
        with torch.cuda.stream(cand):
            x = torch.ones(4, device="cuda") * 2
            ev = torch.cuda.Event(); ev.record(cand)
        if done_within(ev, 0.5):
            B = cand
            break
    if B is not None:
        break
gate.release(); torch.cuda.synchronize()
assert not gate.expired
assert B is not None, f"no stream of {tried} runs beside a held stream"
print("B found after", tried, "candidates")

# 1) A held by the gate, then NSLOTS + 3 queue launches behind it: the first
#    NSLOTS take every slot; the last 3 find none idle (all in flight, busy)
#    and take the static split
st0 = G.queue_stats()
outs = torch.zeros((NSLOTS + 3, n), dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
gate.hold(A)
with torch.cuda.stream(A):
    for k in range(NSLOTS + 3):
        G.checksum_offsets("crc32c", data, offs, out=outs[k], stream=A)
    ev_a = torch.cuda.Event(); ev_a.record(A)
st1 = G.queue_stats()
held = not ev_a.query()
gate.release(); torch.cuda.synchronize()
assert held and not gate.expired
assert st1["slot"] - st0["slot"] == NSLOTS and st1["noslot"] - st0["noslot"] == 3, (st0, st1)
assert st1["in_flight"] == NSLOTS and st1["busy_skip"] > st0["busy_skip"], (st0, st1)
assert bool((outs == want).all()), torch.nonzero((outs != want).any(dim=1)).tolist()

# 2) once they have completed, the pool is reaped: a launch gets a slot again
st2 = G.queue_stats()
o = G.checksum_offsets("crc32c", data, offs, stream=B); torch.cuda.synchronize()
st3 = G.queue_stats()
assert st3["slot"] - st2["slot"] == 1 and st3["reaped"] > st2["reaped"], (st2, st3)
assert torch.equal(o, want)


def blocked_oldest(nheld, nb):
    # nheld launches held behind the gate on A (the oldest slots in flight),
    # then nb launches on B one at a time, each completed before the next:
    # every B launch must get a slot -- the reaper passes the held ones over
    # and finds B's completed slots behind them
    s0 = G.queue_stats()
    xa = torch.zeros((nheld, n), dtype=torch.int32, device="cuda")
    ob = torch.zeros((nb, n), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    gate.hold(A)
    with torch.cuda.stream(A):
        for k in range(nheld):
            G.checksum_offsets("crc32c", data, offs, out=xa[k], stream=A)
        ev_a = torch.cuda.Event(); ev_a.record(A)
    for k in range(nb):
        G.checksum_offsets("crc32c", data, offs, out=ob[k], stream=B)
        ev_b = torch.cuda.Event(); ev_b.record(B)
        assert done_within(ev_b, 5), f"B launch {k} did not complete beside the held stream"
    s1 = G.queue_stats()
    still = not ev_a.query()
    gate.release(); torch.cuda.synchronize()
    assert still and not gate.expired, "A was released before B finished"
    assert bool((ob == want).all()) and bool((xa == want).all())
    assert s1["slot"] - s0["slot"] == nheld + nb and s1["noslot"] == s0["noslot"], (nheld, s0, s1)
    # the held slots were looked at and passed over: once per call after the
    # slots in flight at the start (older than the held ones) are reaped
    assert s1["busy_skip"] - s0["busy_skip"] >= nb - s0["in_flight"], (nheld, s0, s1)
    return s0, s1


# 3) one busy slot passed over while B cycles through the pool 3 times
print("one held", blocked_oldest(1, 3 * NSLOTS))
# 4) ADVICE r4: as many held launches as one reap looks at (8) at the head of
#    the FIFO: busy slots rotate to its back, so B's completed ones are still
#    reaped once the idle stack runs out (before: every later launch took the
#    static split until A was released)
if NSLOTS >= 16:
    print("eight held", blocked_oldest(8, 3 * NSLOTS))
gate.close()
assert G.queue_faults() == 0
print("pool ok", NSLOTS)
"""


def test_pool_hands_no_busy_slot_out():
    """A fresh process with a 16-slot pool (MCHECKSUM_GPU_QUEUE_SLOTS=16),
    streams held by a host-released gate kernel (not a timed sleep), and a
    second stream probed to run beside the held one: launches queued behind
    the gate take every slot and the rest take the static split; the pool
    refills once they complete; a slot whose launch is held is passed over
    while other launches cycle through the pool -- also with eight held
    launches at the head of the in-flight FIFO.  Every result is exact.
    One process, one conclusive outcome (round 4 retried in a second process
    when the two streams shared a hardware queue)."""
    r = subprocess.run([sys.executable, "-c", POOL, ROOT], capture_output=True, text=True, timeout=200,
                       env=dict(os.environ, MCHECKSUM_GPU_QUEUE_SLOTS="16", MCHECKSUM_GPU_LIGHT="0"))
    print(r.stdout[-3000:])
    assert r.returncode == 0 and "pool ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


def test_sticky_error_before_a_queue_launch(gpu, hip, small_batch):
    """a failed HIP call earlier on this thread leaves a sticky
    error.  A queue launch must take its status from its own launch call, not
    from hipGetLastError(): otherwise the enqueued kernel would read as failed,
    its slot would be taken back while it runs and handed to the next launch,
    which would count in a bank whose tickets were never zeroed (skipped
    payloads, no fault).  Both launches succeed and are exact."""
    import torch
    data, offs, want = small_batch
    n = offs.numel() - 1
    want_t = torch.from_numpy(want.astype(np.uint32).view(np.int32)).cuda()
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipGetLastError.restype = ctypes.c_int
    s = _stream(hip)
    try:
        for rep in range(3):
            outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(2)]
            torch.cuda.synchronize()
            st0 = gpu.queue_stats()
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), 1 << 62) != 0  # out of memory: sticky last error
            try:
                for o in outs:
                    gpu.checksum_offsets("crc32c", data, offs, out=o, stream=s)
            finally:
                hip.hipGetLastError()  # clear it before torch checks its own launches
            st1 = gpu.queue_stats()
            assert st1["slot"] - st0["slot"] == 2, (st0, st1)
            assert hip.hipStreamSynchronize(s) == 0
            for o in outs:
                assert torch.equal(o, want_t), rep
    finally:
        hip.hipStreamDestroy(s)
