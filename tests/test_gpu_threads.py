"""Batch entry points called from several host threads at once, the way
Mercury's RPC handler threads would (Testing/unit/hg/mercury_unit.c:347-356:
a handler thread pool).  A fresh process starts 8 threads that make their
first library calls together, so the lazy per-device setup (table packs,
work-queue ring; guarded by one mutex) and the work-queue slot allocation run
concurrently.  Each thread uses its own stream and checks every result
against the oracle."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, threading
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from mercury_amd import gpu as G
from oracle import oracle as O
host = O.splitmix_bytes(32 << 20, 31337)
dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
rng = np.random.default_rng(5)
jobs = []
for k in range(8):
    method = ("crc32c", "crc64")[k % 2]
    offs = np.zeros(2001, dtype=np.uint64)
    offs[1:] = np.cumsum(rng.integers(0, 8192, 2000))
    jobs.append((method, offs, torch.from_numpy(offs.astype(np.int64)).cuda(),
                 O.batch_offsets(method, host, offs, nthreads=4),
                 O.batch_fixed(method, host, 4096, 4096, 4096, nthreads=4)))
torch.cuda.synchronize()
barrier = threading.Barrier(8)
errors = []

def worker(k):
    method, offs, offs_d, want_o, want_f = jobs[k]
    s = torch.cuda.Stream()
    try:
        barrier.wait()
        for it in range(20):
            with torch.cuda.stream(s):
                o = G.checksum_offsets(method, dev, offs_d, stream=s)
                f = G.checksum_fixed(method, dev, 4096, count=4096, stream=s)
            s.synchronize()
            if not np.array_equal(G.as_unsigned(o).astype(np.uint64), want_o):
                errors.append((k, it, "offsets"))
            if not np.array_equal(G.as_unsigned(f).astype(np.uint64), want_f):
                errors.append((k, it, "fixed"))
    except Exception as e:  # reported below
        errors.append((k, repr(e)))

th = [threading.Thread(target=worker, args=(k,)) for k in range(8)]
for t in th:
    t.start()
for t in th:
    t.join(timeout=90)
assert not any(t.is_alive() for t in th), "a worker thread did not finish"
assert not errors, errors[:5]
assert G.queue_faults() == 0
print("threads ok")
"""


def test_eight_host_threads_first_calls_together(gpu):
    r = subprocess.run([sys.executable, "-c", SCRIPT, ROOT], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MCHECKSUM_GPU_LIGHT="0"))
    assert r.returncode == 0 and "threads ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


SHARED = r"""
import sys, threading
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from mercury_amd import gpu as G
from oracle import oracle as O
host = O.splitmix_bytes(8 << 20, 4242)
dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
rng = np.random.default_rng(9)
offs = np.zeros(3001, dtype=np.uint64)
offs[1:] = np.cumsum(rng.integers(0, 2048, 3000))
offs_d = torch.from_numpy(offs.astype(np.int64)).cuda()
want = O.batch_offsets("crc32c", host, offs, nthreads=4)
s = torch.cuda.Stream()  # ONE stream shared by every thread
ITERS, NT = 60, 8
outs = torch.zeros((NT, ITERS, 3000), dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
barrier = threading.Barrier(NT)
errors = []

def worker(k):
    try:
        barrier.wait()
        for it in range(ITERS):
            G.checksum_offsets("crc32c", dev, offs_d, out=outs[k, it], stream=s)
    except Exception as e:  # reported below
        errors.append((k, repr(e)))

th = [threading.Thread(target=worker, args=(k,)) for k in range(NT)]
for t in th:
    t.start()
for t in th:
    t.join(timeout=90)
assert not any(t.is_alive() for t in th), "a worker thread did not finish"
s.synchronize()
assert not errors, errors[:5]
w = torch.from_numpy(want.astype(np.uint32).view(np.int32)).cuda()
bad = torch.nonzero((outs != w).any(dim=2)).tolist()
assert not bad, bad[:8]
assert G.queue_faults() == 0
print("shared stream ok", G.queue_stats())
"""


def test_threads_sharing_one_stream_alternate_the_slot_banks(gpu):
    """8 host threads launch 480 queue batches onto ONE stream at once: each
    launch holds a slot of its own from the pool until it completes
    (queue_slot), so no two of them -- queued back to back on the stream, or
    racing on the host -- ever count in one slot's banks.  Every result is
    exact and no queue wait gave up."""
    r = subprocess.run([sys.executable, "-c", SHARED, ROOT], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MCHECKSUM_GPU_LIGHT="0"))
    assert r.returncode == 0 and "shared stream ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


PERTHREAD = r"""
import sys, threading, ctypes, os
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from mercury_amd import gpu as G
from oracle import oracle as O
hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
PER_THREAD = 2  # hipStreamPerThread
host = O.splitmix_bytes(8 << 20, 777)
dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
rng = np.random.default_rng(3)
offs = np.zeros(3001, dtype=np.uint64)
offs[1:] = np.cumsum(rng.integers(0, 2048, 3000))
offs_d = torch.from_numpy(offs.astype(np.int64)).cuda()
want = torch.from_numpy(O.batch_offsets("crc32c", host, offs, nthreads=4).astype(np.uint32).view(np.int32)).cuda()
ITERS, NT = 40, 4
outs = torch.zeros((NT, ITERS, 3000), dtype=torch.int32, device="cuda")
torch.cuda.synchronize()
st0 = G.queue_stats()
barrier = threading.Barrier(NT)
errors = []

def worker(k):
    try:
        torch.cuda.set_device(0)
        barrier.wait()
        for it in range(ITERS):
            G.checksum_offsets("crc32c", dev, offs_d, out=outs[k, it], stream=PER_THREAD)
        assert hip.hipStreamSynchronize(PER_THREAD) == 0  # this thread's own per-thread stream
    except Exception as e:  # reported below
        errors.append((k, repr(e)))

th = [threading.Thread(target=worker, args=(k,)) for k in range(NT)]
for t in th:
    t.start()
for t in th:
    t.join(timeout=90)
assert not any(t.is_alive() for t in th), "a worker thread did not finish"
torch.cuda.synchronize()
assert not errors, errors[:5]
st1 = G.queue_stats()
bad = torch.nonzero((outs != want).any(dim=2)).tolist()
assert not bad, bad[:8]
assert st1["slot"] - st0["slot"] == NT * ITERS and st1["noslot"] == st0["noslot"], (st0, st1)
assert G.queue_faults() == 0
print("per-thread ok", st0, st1)
"""


def test_per_thread_default_stream_takes_the_queue(gpu):
    """hipStreamPerThread is one handle naming a different stream in every host
    thread.  Round 3 gave its launches no slot (a slot per handle could have
    served two threads' launches at once); with slots held per launch (round
    4) they take the work queue like any other eager launch: 4 threads x 40
    queue batches on it, every one with a slot, every result exact."""
    r = subprocess.run([sys.executable, "-c", PERTHREAD, ROOT], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MCHECKSUM_GPU_LIGHT="0"))
    assert r.returncode == 0 and "per-thread ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
