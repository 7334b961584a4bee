"""Stress the batch kernels' dynamic work queue: many launches of random
shapes (fixed, offsets and scatter-gather batches, both methods, every
lanes-per-payload width, both load policies) on the throughput layout, each checked bit for bit against the CPU
oracle, with a host watchdog (a launch not done after 20 s ends the process
with exit 3 instead of waiting on a wedged GPU).  Ends with the device's
queue fault count (must be 0)."""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _wait(torch, tag, streams=(None,)):
    evs = []
    for st in streams:
        ev = torch.cuda.Event()
        ev.record(st)
        evs.append(ev)
    t0 = time.time()
    while not all(ev.query() for ev in evs):
        if time.time() - t0 > 20:
            print("HUNG", tag, flush=True)
            os._exit(3)
        time.sleep(0.002)


@pytest.mark.parametrize("n_iter", [240])
def test_dynamic_queue_random_shapes(gpu, oracle_mod, n_iter, monkeypatch):
    import torch
    G, O = gpu, oracle_mod
    rng = np.random.default_rng(12345)
    monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", "0")
    host = O.splitmix_bytes(64 << 20, 99)
    dev = torch.from_numpy(host).cuda()
    dev = torch.cat([dev, torch.zeros(64, dtype=torch.uint8, device="cuda")])
    bad = 0
    t0 = time.time()
    for it in range(n_iter):
        method = ("crc32c", "crc64")[it % 2]
        r = rng.random()
        if r < 0.2:
            # scatter-gather objects: the CRC-64 aligned chunk pass takes the
            # queue (chunk -> segment map), interleaved on the stream's slot
            # with the fixed and offsets launches
            nobj = int(rng.choice([1, 5, 40, 300]))
            seg_lens = rng.choice([0, 64, 1024, 4096, 262144, 300000, 1 << 20], size=3 * nobj)
            starts = [int(rng.integers(0, (64 << 20) - int(n) - 64)) // 16 * 16 + int(rng.choice([0, 0, 0, 5]))
                      for n in seg_lens]
            first = np.arange(0, 3 * nobj + 1, 3)
            batch = G.SegmentBatch([dev[a:a + int(n)] for a, n in zip(starts, seg_lens)], first)
            got = batch.checksum(method)
            _wait(torch, (it, method, "segments", nobj))
            want = np.array([O.crc(method, np.concatenate([host[starts[3 * j + q]:starts[3 * j + q] + int(seg_lens[3 * j + q])]
                                                            for q in range(3)]))
                             for j in range(nobj)], dtype=np.uint64)
            tag = ("segments", nobj)
        elif r < 0.6:
            length = int(rng.choice([0, 1, 16, 1000, 4096, 4100, 16384, 65536, 100003]))
            stride = length + int(rng.choice([0, 0, 16, 3]))
            maxc = max(1, (64 << 20) // max(stride, 1) - 1)
            count = int(min(maxc, rng.choice([1, 2, 15, 16, 17, 67, 255, 256, 1000, 4097, 20000])))
            if length == 0:
                stride = 16
            lg = rng.choice([None, 0, 2, 4, 6])
            if lg is None:
                monkeypatch.delenv("MCHECKSUM_GPU_LOG2G", raising=False)
            else:
                monkeypatch.setenv("MCHECKSUM_GPU_LOG2G", str(lg))
            # NT forces the large-batch kernels (CRC-32C aligned ones take the queue)
            monkeypatch.setenv("MCHECKSUM_GPU_NT", str(int(rng.integers(0, 2))))
            got = G.checksum_fixed(method, dev, length, count=count, stride=stride)
            _wait(torch, (it, method, "fixed", length, stride, count, lg))
            want = O.batch_fixed(method, host, stride, length, count, nthreads=8)
            tag = ("fixed", length, stride, count, lg)
        else:
            count = int(rng.choice([1, 3, 16, 17, 100, 1025, 5000, 20000]))
            lens = rng.integers(0, int(rng.choice([64, 4096, 65536])), count)
            offs = np.zeros(count + 1, dtype=np.uint64)
            offs[1:] = np.cumsum(lens)
            if offs[-1] >= (64 << 20):
                continue
            offs += np.uint64(rng.integers(0, 16))
            got = G.checksum_offsets(method, dev, torch.from_numpy(offs.astype(np.int64)).cuda(), offsets_host=offs)
            _wait(torch, (it, method, "offsets", count))
            want = O.batch_offsets(method, host, offs, nthreads=8)
            tag = ("offsets", count)
        g = G.as_unsigned(got).astype(np.uint64)
        nb = int(np.count_nonzero(g != want))
        if nb:
            bad += 1
            print("MISMATCH", it, method, tag, nb, flush=True)
        if it % 50 == 0:
            print(f"iter {it} ok ({time.time() - t0:.1f} s)", flush=True)
    faults = G.queue_faults()
    print(f"done {n_iter} launches, {bad} mismatching, queue faults {faults}", flush=True)
    assert bad == 0 and faults == 0


def test_queue_slot_survives_graph_replay(gpu, oracle_mod, monkeypatch):
    """Captured calls (an offsets batch and an NT fixed batch, both queue
    kernels) replay with the static split -- no slot is baked into the graph
    -- and every replay hashes the whole batch again."""
    import torch
    G, O = gpu, oracle_mod
    monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", "0")
    monkeypatch.setenv("MCHECKSUM_GPU_NT", "1")
    host = O.splitmix_bytes(8 << 20, 4242)
    dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
    rng = np.random.default_rng(7)
    offs = np.zeros(3001, dtype=np.uint64)
    offs[1:] = np.cumsum(rng.integers(0, 2048, 3000))
    offs_d = torch.from_numpy(offs.astype(np.int64)).cuda()
    G.prepare("crc32c")
    out_o = torch.zeros(3000, dtype=torch.int32, device="cuda")
    out_f = torch.zeros(2048, dtype=torch.int32, device="cuda")
    G.checksum_offsets("crc32c", dev, offs_d, out=out_o, offsets_host=offs)  # validate once, eager
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        G.checksum_offsets("crc32c", dev, offs_d, out=out_o)
        G.checksum_fixed("crc32c", dev, 4096, count=2048, out=out_f)
    want_o = O.batch_offsets("crc32c", host, offs, nthreads=8)
    want_f = O.batch_fixed("crc32c", host, 4096, 4096, 2048, nthreads=8)
    for _ in range(4):
        out_o.zero_()
        out_f.zero_()
        g.replay()
        _wait(torch, "graph replay")
        assert np.array_equal(G.as_unsigned(out_o).astype(np.uint64), want_o)
        assert np.array_equal(G.as_unsigned(out_f).astype(np.uint64), want_f)
    assert G.queue_faults() == 0


def test_concurrent_streams_get_distinct_slots(gpu, oracle_mod, monkeypatch):
    """Queue-driven launches on four streams at once (each stream has a slot
    of its own) all return the oracle's values."""
    import torch
    G, O = gpu, oracle_mod
    monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", "0")
    host = O.splitmix_bytes(16 << 20, 5151)
    dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
    rng = np.random.default_rng(3)
    tables, outs, wants = [], [], []
    for k in range(4):
        offs = np.zeros(4001, dtype=np.uint64)
        offs[1:] = np.cumsum(rng.integers(0, 4000, 4000))
        offs += np.uint64(k * 997)
        tables.append((offs, torch.from_numpy(offs.astype(np.int64)).cuda()))
        wants.append(O.batch_offsets("crc64" if k % 2 else "crc32c", host, offs, nthreads=8))
    G.prepare("crc32c")
    G.prepare("crc64")
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(4)]
    for rep in range(3):
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                outs.append(G.checksum_offsets("crc64" if k % 2 else "crc32c", dev, tables[k][1], stream=s))
        _wait(torch, "concurrent streams", streams)
        torch.cuda.synchronize()
    for i, o in enumerate(outs):
        assert np.array_equal(G.as_unsigned(o).astype(np.uint64), wants[i % 4]), i
    assert G.queue_faults() == 0


def test_graph_slot_is_never_reused_by_eager_launches(gpu, oracle_mod, monkeypatch):
    """4300 eager queue launches on one stream while a captured launch of the
    same kernel keeps replaying on another: the graph never touches the eager
    stream's slot, and neither side loses or repeats a unit."""
    import torch
    G, O = gpu, oracle_mod
    monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", "0")
    host = O.splitmix_bytes(8 << 20, 777)
    dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
    rng = np.random.default_rng(21)
    tabs = []
    for _ in range(2):
        offs = np.zeros(2049, dtype=np.uint64)
        offs[1:] = np.cumsum(rng.integers(0, 2048, 2048))
        tabs.append((offs, torch.from_numpy(offs.astype(np.int64)).cuda()))
    want_g = O.batch_offsets("crc32c", host, tabs[0][0], nthreads=8)
    want_e = O.batch_offsets("crc32c", host, tabs[1][0], nthreads=8)
    G.prepare("crc32c")
    out_g = torch.zeros(2048, dtype=torch.int32, device="cuda")
    outs_e = [torch.zeros(2048, dtype=torch.int32, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    s, e = torch.cuda.Stream(), torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        G.checksum_offsets("crc32c", dev, tabs[0][1], out=out_g)
    torch.cuda.synchronize()
    bad = 0
    for i in range(4300):
        with torch.cuda.stream(e):
            G.checksum_offsets("crc32c", dev, tabs[1][1], out=outs_e[i % 2], stream=e)
        if i % 100 == 0:
            with torch.cuda.stream(s):
                g.replay()
        if i % 500 == 499:
            _wait(torch, ("eager", i), (s, e))
            torch.cuda.synchronize()
            bad += int(not np.array_equal(G.as_unsigned(out_g).astype(np.uint64), want_g))
            bad += sum(int(not np.array_equal(G.as_unsigned(o).astype(np.uint64), want_e)) for o in outs_e)
    _wait(torch, "final", (s, e))
    torch.cuda.synchronize()
    assert bad == 0 and G.queue_faults() == 0


def test_captured_launches_replayed_concurrently_stay_correct(gpu, oracle_mod, monkeypatch):
    """Graph-captured launches get no work-queue slot and take the static split
    (crc_gpu_device.h, "Exclusivity"): two offsets graphs, a split CRC-64 graph
    (pieces XORed into a zeroed output, MCHECKSUM_GPU_SPLIT=1) and a
    scatter-gather graph (chunks XORed into out[]) replayed at the same time on
    four streams, next to eager queue launches on a fifth, keep returning the
    oracle's values.  (Round 2's shared-slot ownership failed this: a replay
    whose early workgroups found the slot busy and later ones found it free
    never released it, and its next replay skipped units -- 1 bad batch in 400.)"""
    import torch
    G, O = gpu, oracle_mod
    monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", "0")
    host = O.splitmix_bytes(8 << 20, 31337)
    dev = torch.cat([torch.from_numpy(host).cuda(), torch.zeros(64, dtype=torch.uint8, device="cuda")])
    rng = np.random.default_rng(5)
    tabs, wants, outs = [], [], []
    for k in range(2):
        offs = np.zeros(3001, dtype=np.uint64)
        offs[1:] = np.cumsum(rng.integers(0, 2600, 3000))
        tabs.append(torch.from_numpy(offs.astype(np.int64)).cuda())
        wants.append(O.batch_offsets("crc32c", host, offs, nthreads=8))
        outs.append(torch.zeros(3000, dtype=torch.int32, device="cuda"))
    # split CRC-64: 16 payloads of 512 KiB (2 pieces each)
    want_sp = O.batch_fixed("crc64", host, 512 << 10, 512 << 10, 16, nthreads=8)
    out_sp = torch.zeros(16, dtype=torch.int64, device="cuda")
    # scatter-gather: 24 objects of 3 segments (256 KiB + 40 KiB + 4 KiB) from anywhere
    seg_lens = [256 << 10, 40 << 10, 4 << 10]
    starts = rng.integers(0, (8 << 20) - (256 << 10), 72) // 16 * 16
    segs = [dev[int(a):int(a) + seg_lens[q % 3]] for q, a in enumerate(starts)]
    batch = G.SegmentBatch(segs, np.arange(0, 73, 3))
    want_sg = [O.crc("crc64", np.concatenate([host[int(starts[3 * j + q]):int(starts[3 * j + q]) + seg_lens[q]]
                                               for q in range(3)])) for j in range(24)]
    out_sg = torch.zeros(24, dtype=torch.int64, device="cuda")
    G.prepare("crc32c")
    G.prepare("crc64")
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(5)]
    calls = [lambda: G.checksum_offsets("crc32c", dev, tabs[0], out=outs[0]),
             lambda: G.checksum_offsets("crc32c", dev, tabs[1], out=outs[1]),
             lambda: G.checksum_fixed("crc64", dev, 512 << 10, count=16, out=out_sp),
             lambda: batch.checksum("crc64", out=out_sg)]
    graphs = []
    monkeypatch.setenv("MCHECKSUM_GPU_SPLIT", "1")
    for k, f in enumerate(calls):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(streams[k]), torch.cuda.graph(g, stream=streams[k]):
            f()
        graphs.append(g)
    torch.cuda.synchronize()
    eager_out = torch.zeros(3000, dtype=torch.int32, device="cuda")
    bad = {"offsets0": 0, "offsets1": 0, "split64": 0, "segments": 0, "eager": 0}
    for rep in range(150):
        for o in outs + [out_sp, out_sg, eager_out]:
            o.zero_()
        torch.cuda.synchronize()
        for k, g in enumerate(graphs):
            with torch.cuda.stream(streams[k]):
                g.replay()
        with torch.cuda.stream(streams[4]):
            G.checksum_offsets("crc32c", dev, tabs[rep % 2], out=eager_out, stream=streams[4])
        _wait(torch, ("captured", rep), streams)
        for k in range(2):
            bad[f"offsets{k}"] += int(not np.array_equal(G.as_unsigned(outs[k]).astype(np.uint64), wants[k]))
        bad["split64"] += int(not np.array_equal(G.as_unsigned(out_sp), want_sp))
        bad["segments"] += int(not np.array_equal(G.as_unsigned(out_sg), np.asarray(want_sg, dtype=np.uint64)))
        bad["eager"] += int(not np.array_equal(G.as_unsigned(eager_out).astype(np.uint64), wants[rep % 2]))
    assert sum(bad.values()) == 0 and G.queue_faults() == 0, bad
