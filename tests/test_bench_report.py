"""bench.py's N > 1 JSON line on the CPU: 2 gloo ranks each checksum their
share of one global batch (the oracle standing in for the GPU kernels on a
CPU-only box), gather it with bench.gather_shares, and rank 0 builds the line
with bench.report -- the same code the GPU run executes after timing.  The line
must carry the CPU baseline (timed on rank 0's host at N > 1 too), a parity
verdict from the ORACLE over every share, and a labelled roofline.traffic."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


LAYOUTS = {
    # name: (bench config, method, global count, payload length, seed, layout)
    "fixed": ("c5", "crc32c", 96, 65536, 0x4D43310000000005, "fixed"),
    # the default at every N: the headline's per-GPU batch (weak scaling),
    # here 48 payloads per rank -- global count 96 over 2 ranks
    "weak_fixed": ("metric", "crc32c", 96, 65536, 0x4D43310000000005, "fixed"),
    "offsets": ("c4", "crc32c", 300, None, 0x4D43310000000004, "offsets"),
    "messages": ("msgs", "crc32c", 300, None, 0x4D43310000000004, "messages"),
    "segments": ("seg", "crc64", 6, 1 << 20, 0x4D43310000000003, "segments"),
}


def _share_crcs(O, bench, name, rank, world):
    """(local CRC array, plan, rank-local offsets) of this rank's share."""
    from mercury_amd.shard import batch_shard
    from mercury_amd.workload import segment_slots, varlen_offsets
    cfg, method, gc, length, seed, layout = LAYOUTS[name]
    if layout == "fixed":
        plan = batch_shard(rank, world, gc, length)
        local = O.splitmix_bytes(plan.nbytes, seed, first_word=plan.first_word)
        return O.batch_fixed(method, local, length, length, plan.count), plan, None
    if layout == "segments":  # weak: gc objects per rank from seed ^ rank
        slots = segment_slots(seed ^ rank, gc * bench.SEGS_PER_OBJECT)
        crcs = [O.crc(method, bench._segment_object_bytes(O, seed ^ rank, length, j, slots)) for j in range(gc)]
        return np.array(crcs, dtype=np.uint64), None, None
    plan = batch_shard(rank, world, gc, offsets_global=varlen_offsets(seed, gc))
    local = O.splitmix_bytes(plan.nbytes, seed, first_word=plan.first_word)
    if layout == "offsets":
        return O.batch_offsets(method, local, plan.offsets), plan, plan.offsets
    inter = np.empty(2 * plan.count + 1, dtype=np.uint64)  # sender pieces: header, payload
    inter[0::2] = plan.offsets
    inter[1::2] = plan.offsets[:-1] + np.uint64(20)
    return O.batch_offsets(method, local, inter), plan, plan.offsets


def _worker(name, corrupt, rank, world, port, q):
    sys.path.insert(0, ROOT)
    from types import SimpleNamespace

    import torch
    import torch.distributed as dist

    import bench
    from oracle import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg, method, gc, length, seed, layout = LAYOUTS[name]
    crcs, plan, off = _share_crcs(O, bench, name, rank, world)
    if corrupt and rank == 1:
        crcs = crcs.copy()
        crcs[1 if layout == "messages" else 0] ^= np.uint64(1)  # the first payload of rank 1's share
    dt = np.int32 if method == "crc32c" else np.int64
    t = torch.from_numpy(crcs.astype(np.uint32 if method == "crc32c" else np.uint64).view(dt).copy())
    count = plan.count if plan is not None else gc
    counts = plan.counts if plan is not None else [gc] * world
    if layout == "messages":
        counts = [2 * c for c in counts]
    full = bench.gather_shares(dist, t, counts, world, torch.device("cpu"))
    if rank == 0:
        got = full.numpy().view(np.uint32 if method == "crc32c" else np.uint64)
        args = SimpleNamespace(steps=3, warmup=1, cpu_seconds=0.05, parity_samples=16, no_cpu_baseline=False)
        payload_bytes = count * length if length else int(off[-1] - off[0])
        r = SimpleNamespace(
            config=cfg, method=method, seed=seed, length=length, layout=layout, strong=cfg in bench.STRONG,
            global_count=gc if layout != "segments" else gc * world, count=count, plan=plan,
            payload_bytes=payload_bytes, alg_bytes=payload_bytes + 4 * count, gib_s=1.0, wall_max=0.003,
            kern_ms_max=1.0, achieved=1.0, per_rank=[[0.003, 1.0]] * world, world=world, got=got, offsets_host=off,
            verify_note=None, lanes=64, pcis=[f"0000:{0x11 * (i + 1):02x}:00" for i in range(world)])
        q.put(bench.report(args, r))
    dist.barrier()
    dist.destroy_process_group()


def _run(name, corrupt=False):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(name, corrupt, r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    return q.get()


@pytest.mark.parametrize("name", sorted(LAYOUTS))
def test_two_rank_line_has_baseline_oracle_parity_and_traffic(name):
    res = _run(name)
    cb = res["cpu_baseline"]
    assert cb["kind"] == "port" and cb["unit"] == "GiB/s" and cb["value"] > 0 and cb["cores"] >= 1
    assert cb["sample"] and "breakdown_GiB_s" in cb
    # the product's own CPU path (libmchecksum streaming API on the same
    # sample, oracle-checked) beside the oracle port, at full width and 1 thread
    bd = cb["breakdown_GiB_s"]
    prod = {k: v for k, v in bd.items() if k.startswith("product_")}
    assert f"product_{cb['cores']}thread{'s' if cb['cores'] > 1 else ''}" in prod and "product_1thread" in prod, bd
    assert all(v and v > 0 for v in prod.values()), (bd, cb.get("product_note"))
    assert res["parity"].startswith("bit-exact (") and "across all 2 shares vs oracle" in res["parity"], res["parity"]
    assert res["n_gpus"] == 2 and res["world_size"] == 2 and len(res["per_rank"]) == 2
    # every rank's PCI address is in the line (bench.py gathers them; distinct on RCCL runs)
    assert [p["pci"] for p in res["per_rank"]] == ["0000:11:00", "0000:22:00"]
    roof = res["roofline"]
    assert roof["traffic"] is not None and "rank 0's share" in roof["traffic_source"], roof
    assert res["scaling"] == ("weak" if name in ("segments", "weak_fixed") else "strong")


def test_default_multi_gpu_line_is_the_per_gpu_headline():
    """bench.py --gpus N defaults to the headline's 65536 x 64 KiB per rank at
    every N (weak scaling), so the driver's 1/2/4/8 series is one per-GPU
    workload: the 2-rank line names 48 payloads on rank 0 out of 96 in all."""
    import bench
    assert bench.CONFIGS["metric"][1:3] == (65536, 65536) and "metric" not in bench.STRONG
    res = _run("weak_fixed")
    assert res["scaling"] == "weak" and res["metric"].endswith("64K x 64 KiB payloads")
    cfg = res["config"]
    assert cfg["payloads_rank0"] == 48 and cfg["global_batch"] == 96 and cfg["bytes_rank0"] == 48 * 65536
    assert "48 x 65536 B payloads per GPU (96 in all over 2 GPUs)" in cfg["workload"], cfg["workload"]


@pytest.mark.parametrize("name", ["fixed", "messages"])
def test_two_rank_line_flags_a_wrong_share(name):
    """A wrong CRC in rank 1's share reads as a mismatch, not as bit-exact."""
    res = _run(name, corrupt=True)
    assert res["parity"].startswith("MISMATCH 1/") and "across all 2 shares" in res["parity"], res["parity"]


def _e2e_record(O, count=64, length=4096, cpu_n=16, seed=0x4D43310000000005):
    """An e2e record as bench.run_e2e leaves it for e2e_finish, built on the
    CPU: the host bytes, the legs' CRCs (oracle values standing in for the
    GPU's) and the product CPU path's CRCs of the first cpu_n payloads."""
    hb = O.splitmix_bytes(count * length, seed)
    want = O.batch_fixed("crc32c", hb, length, length, count).astype(np.uint32)
    rec = {"staged": {}, "h2d_only": {}, "zero_copy": {},
           "cpu_same_bytes": {"cores": 1, "product_crcs": want[:cpu_n].astype(np.uint64)},
           "_crcs": {"staged": want.copy(), "zero_copy": want.copy()}, "_host": hb,
           "_shape": ("crc32c", count, length, cpu_n)}
    return rec, want


def test_e2e_finish_bit_exact_and_detects_a_wrong_crc():
    """bench.e2e_finish: both host-memory legs are compared with the
    device-resident CRCs on every payload and with the oracle on sampled
    payloads of the host bytes; a single wrong CRC turns the verdict."""
    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle as O

    class A:
        no_cpu_baseline = False

    rec, want = _e2e_record(O)
    out = bench.e2e_finish(rec, want.copy(), A())
    assert out["parity"].startswith("bit-exact"), out["parity"]
    assert "64/64 equal the device-resident" in out["parity"]
    assert out["cpu_same_bytes"]["oracle_GiB_s"] > 0
    assert not any(k.startswith("_") for k in out)

    rec, want = _e2e_record(O)
    rec["_crcs"]["zero_copy"][17] ^= 1
    out = bench.e2e_finish(rec, want.copy(), A())
    assert out["parity"].startswith("MISMATCH") and "zero_copy: 63/64" in out["parity"]

    rec, want = _e2e_record(O)
    rec["_crcs"]["staged"][0] ^= 0x80000000  # also sampled by the oracle leg
    out = bench.e2e_finish(rec, want.copy(), A())
    assert out["parity"].startswith("MISMATCH")
