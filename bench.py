#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X mchecksum batch path.

Metric (BASELINE.json): GiB/s checksummed (device-resident), CRC32c,
64K x 64 KiB payloads.  One "step" = one batch launch over the whole
per-GPU batch (65536 payloads of 64 KiB = 4 GiB), inputs already in HBM.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
each rank owns a contiguous shard of a global batch (weak scaling: per-GPU
work fixed), generated on its own device; no collective in the timed region.
After timing, RCCL all_gather of the per-shard CRC arrays to check the
gathered result and an all_reduce(MAX) of the timings.

Prints ONE JSON line on rank 0 (contract in the task statement), with
`roofline` (HIP-event kernel time vs HBM peak) and `cpu_baseline` (oracle on
this host's cores, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0
SEGS_PER_OBJECT = 4  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md:36

CONFIGS = {
    # name: (method, count, length, seed, layout)
    "metric": ("crc32c", 65536, 65536, 0x4D43310000000005, "fixed"),
    "c2": ("crc32c", 65536, 4096, 0x4D43310000000002, "fixed"),
    "c3": ("crc64", 8192, 1 << 20, 0x4D43310000000003, "fixed"),
    "c4": ("crc32c", 262144, None, 0x4D43310000000004, "offsets"),
    # 8(f) 2: C3's bytes as bulk-handle segment lists -- 8192 objects x 4
    # segments of 256 KiB scattered over the buffer (permuted slots)
    "seg": ("crc64", 8192, 1 << 20, 0x4D43310000000003, "segments"),
    # C5: the 2^20 x 64 KiB global batch (64 GiB) split over the ranks --
    # strong scaling (8 GiB per GPU at 8 GPUs; all of it on one GPU at N=1)
    "c5": ("crc32c", 1 << 20, 65536, 0x4D43310000000005, "fixed"),
    # 8(f) 1: C4's packets as Mercury messages (16 B core header, 4 B HG header
    # carrying the network-order payload CRC, payload) verified in place --
    # the batched hg_get_struct checksum check
    "msgs": ("crc32c", 262144, None, 0x4D43310000000004, "messages"),
    # BASELINE configs[0]: host CPU, through the drop-in streaming API
    "c1": ("crc32c", 1024, 4096, 0x4D43310000000001, "cpu"),
}
# configs whose count is the GLOBAL batch, split over the ranks (strong
# scaling); the others give every rank a batch of that size (weak scaling)
STRONG = {"c5", "c4", "msgs"}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); without torchrun in the environment bench.py starts them itself")
    p.add_argument("--steps", type=int, default=50)
    # 40: the clock settles after ~30 back-to-back launches (per-launch times
    # 0.62 -> 0.75 -> 0.62 ms over the first 30, profiles/r01/launch_series_metric.json)
    p.add_argument("--warmup", type=int, default=40)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS),
                   help="default: the headline (metric) at 1 GPU, C5's 2^20 x 64 KiB global batch split over "
                        "the ranks at N > 1")
    p.add_argument("--streams", type=int, default=1,
                   help="issue consecutive steps round-robin on this many streams (independent batches, "
                        "fixed and offsets layouts)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the CPU baseline sample")
    p.add_argument("--parity-samples", type=int, default=64)
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL (default); gloo only to rehearse the multi-rank flow on one GPU")
    return p.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """`bench.py --gpus N` outside torchrun: start the N ranks as a child
    torch.distributed.run (127.0.0.1 rendezvous) BEFORE this process touches
    the GPU, and return its exit code.  Ranks then see WORLD_SIZE = N."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only (RCCL, CUDA-tensor sharing)
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if args.config is None:
        args.config = "metric" if args.gpus == 1 else "c5"
    if CONFIGS[args.config][4] == "cpu":
        return bench_c1(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local % torch.cuda.device_count())
        # The communication libraries may print connection notices on file
        # descriptor 1 (gloo's "[Gloo] Rank 0 is connected to ..."), which
        # would corrupt the one-JSON-line stdout contract: point fd 1 at
        # stderr while the group comes up.
        sys.stdout.flush()
        saved_fd = os.dup(1)
        os.dup2(2, 1)
        try:
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group("gloo")
            dist.barrier()  # connections are made by the first collective at the latest
        finally:
            sys.stdout.flush()
            os.dup2(saved_fd, 1)
            os.close(saved_fd)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from mercury_amd import gpu as G
    from mercury_amd.shard import batch_shard
    from mercury_amd.workload import varlen_offsets

    method, count, length, seed, layout = CONFIGS[args.config]
    strong = args.config in STRONG
    # ONE global batch, split into contiguous rank shares (mercury_amd.shard):
    # strong configs split their own count; weak ones grow it with the ranks
    global_count = count if strong else count * world
    plan = None
    if layout == "fixed":
        plan = batch_shard(rank, world, global_count, length)
    elif layout in ("offsets", "messages"):
        plan = batch_shard(rank, world, global_count, offsets_global=varlen_offsets(seed, global_count))
    if plan is not None:
        count = plan.count
    stream = torch.cuda.current_stream()
    G.prepare(method)

    # ---- this rank's share of the global batch, generated on the device ----
    if layout == "fixed":
        data = torch.empty(plan.nbytes + 64, dtype=torch.uint8, device=dev)
        G.fill_splitmix(data, seed, first_word=plan.first_word)  # the global stream's bytes
        offsets_dev = offsets_host = None
        payload_bytes = plan.nbytes
        run = lambda out: G.checksum_fixed(method, data, length, count=count, out=out)  # noqa: E731
    elif layout == "segments":  # per-rank objects (weak): scattered segment lists
        from mercury_amd.workload import segment_slots
        seg_len = length // SEGS_PER_OBJECT
        payload_bytes = count * length
        data = torch.empty(payload_bytes + 64, dtype=torch.uint8, device=dev)
        G.fill_splitmix(data, seed ^ rank)
        slots = segment_slots(seed ^ rank, count * SEGS_PER_OBJECT)
        batch = G.SegmentBatch([data[int(q) * seg_len:(int(q) + 1) * seg_len] for q in slots],
                               np.arange(0, count * SEGS_PER_OBJECT + 1, SEGS_PER_OBJECT))
        offsets_dev = offsets_host = None
        run = lambda out: batch.checksum(method, out=out)  # noqa: E731
    elif layout == "messages":
        msg_host = plan.offsets
        payload_bytes = int(msg_host[-1] - msg_host[0])
        data = torch.empty(plan.nbytes + 64, dtype=torch.uint8, device=dev)
        G.fill_splitmix(data, seed, first_word=plan.first_word)
        # sender side (hg_set_struct): CRC of each payload = message bytes
        # [20, len); one offsets batch over the interleaved table
        # (header_i, payload_i, ...), the checker's layout as well
        offsets_host = np.empty(2 * count + 1, dtype=np.uint64)
        offsets_host[0::2] = msg_host
        offsets_host[1::2] = msg_host[:-1] + np.uint64(20)
        sender = G.checksum_offsets(method, data, torch.from_numpy(offsets_host.astype(np.int64)).to(dev),
                                    offsets_host=offsets_host)
        # ... stored network-order in each message's HG header (bytes 16..19)
        msg_dev = torch.from_numpy(msg_host.astype(np.int64)).to(dev)
        crc = sender[1::2].to(torch.int64) & 0xFFFFFFFF
        for k in range(4):
            data[msg_dev[:-1] + 16 + k] = ((crc >> (24 - 8 * k)) & 0xFF).to(torch.uint8)
        offsets_dev = msg_dev
        status = torch.empty(count, dtype=torch.uint8, device=dev)
        mism = torch.zeros(1, dtype=torch.int32, device=dev)
        G.verify_messages(data, msg_dev, status=status, mismatches=mism, offsets_host=msg_host)  # validates once
        run = lambda out: G.verify_messages(data, msg_dev, status=status, mismatches=mism)  # noqa: E731
    else:
        offsets_host = plan.offsets
        payload_bytes = int(offsets_host[-1] - offsets_host[0])
        data = torch.empty(plan.nbytes + 64, dtype=torch.uint8, device=dev)
        G.fill_splitmix(data, seed, first_word=plan.first_word)
        offsets_dev = torch.from_numpy(offsets_host.astype(np.int64)).to(dev)
        G.checksum_offsets(method, data, offsets_dev, offsets_host=offsets_host)  # validates the table once
        run = lambda out: G.checksum_offsets(method, data, offsets_dev, out=out)  # noqa: E731
    out = torch.empty(count, dtype=G.out_dtype(method), device=dev)
    if args.streams > 1 and layout not in ("fixed", "offsets"):
        raise SystemExit(f"--streams > 1 needs a fixed or offsets layout (config {args.config} shares scratch)")
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(args.streams - 1)]
    outs = [out] + [torch.empty_like(out) for _ in range(args.streams - 1)]
    torch.cuda.synchronize()

    def step(i):  # step i: one batch, on stream i % S with its own output
        s = streams[i % len(streams)]
        with torch.cuda.stream(s):
            run(outs[i % len(streams)])
        return s

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()

    # Device time of the timed region: ONE HIP event pair on the launch stream
    # around the K back-to-back launches (other streams join it), so
    # kernel_ms = region / K.  An event pair around every launch would put
    # two timestamp packets between consecutive kernels: +2.6 us on C2's
    # 42.2 us launches (rocprofv3 kernel trace, profiles/r02/c2_kernel_steady.json).
    ev_start, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_start.record(streams[0])
    for s in streams[1:]:
        s.wait_event(ev_start)
    for i in range(args.steps):
        step(i)
    for s in streams[1:]:
        joined = torch.cuda.Event()
        joined.record(s)
        streams[0].wait_event(joined)
    ev_end.record(streams[0])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev_start.elapsed_time(ev_end) / args.steps

    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=coll_dev)
    per_rank = [t.clone() for _ in range(world)]
    if world > 1:
        dist.all_gather(per_rank, t)
    per_rank = [[float(x[0]), float(x[1])] for x in per_rank]
    wall_max = max(w for w, _ in per_rank)
    kern_ms_max = max(k for _, k in per_rank)

    # ---- gathered result (outside the timed region) ----------------------
    crcs = out
    verify_note = None
    if layout == "messages":
        # every timed verify passed (the mismatch counter accumulates over all
        # launches), and one flipped payload bit is caught exactly where it is
        bad_before = int(mism.item())
        victim = count // 3
        pos = int(msg_host[victim]) + 20 + (int(msg_host[victim + 1] - msg_host[victim]) - 20) // 2
        data[pos] ^= 0x10
        st, m2 = G.verify_messages(data, offsets_dev)
        flagged = torch.nonzero(st).flatten().tolist()
        data[pos] ^= 0x10
        verify_note = (f"{args.steps + args.warmup + 1} verify launches: {bad_before} mismatches; one flipped bit "
                       f"flagged {flagged} (expected [{victim}])")
        crcs = sender  # the sender-side CRCs, checked against the oracle below
    if world > 1 and layout != "messages":
        # RCCL all_gather of the per-rank CRC arrays (padded to the largest
        # shard: ranks may hold different counts), then trimmed in rank order
        counts = plan.counts if plan is not None else [count] * world
        mine = torch.zeros(max(counts), dtype=crcs.dtype, device=coll_dev)
        mine[:count] = crcs[:count].to(coll_dev)
        gathered = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
        crcs = torch.cat([g[:c] for g, c in zip(gathered, counts)])
    got = G.as_unsigned(crcs) if rank == 0 else None

    bytes_all = torch.tensor([float(payload_bytes)], dtype=torch.float64, device=coll_dev)
    if world > 1:
        dist.all_reduce(bytes_all)
    total_bytes = float(bytes_all[0]) * args.steps  # every rank checksummed its shard once per step
    gib_s = total_bytes / wall_max / 2**30
    out_bytes = count * (4 if G.out_dtype(method) == torch.int32 else 8)
    alg_bytes = payload_bytes + out_bytes + (8 * (count + 1) if layout == "offsets" else 0) + \
        (16 * count * SEGS_PER_OBJECT + 8 * (count + 1) if layout == "segments" else 0)
    if layout == "messages":  # messages read (headers included), 1 status byte each, the offsets table
        alg_bytes = payload_bytes + count + 8 * (count + 1)
    achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9

    result = None
    if rank == 0:
        # HBM bytes per launch cannot be counted inside this process: they come
        # from the committed rocprofv3 PMC passes of this same command
        # (tools/gpu_pmc_traffic.sh -> profiles/pmc_traffic_<config>.json)
        traffic, traffic_src = None, None
        pmc = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}.json")
        if os.path.exists(pmc) and world == 1:
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
                traffic_src = (f"profiles/pmc_traffic_{args.config}.json (rocprofv3 FETCH_SIZE + WRITE_SIZE passes "
                               "of this config, committed; not measured in this run)")
            except Exception:
                traffic = None
        metric = {"metric": "GiB/s checksummed (device-resident), CRC32c, 64K x 64 KiB payloads",
                  "c5": "GiB/s checksummed (device-resident), CRC32c, 1M x 64 KiB payloads split over the GPUs (C5)"}
        result = {
            "metric": metric.get(args.config, f"GiB/s checksummed (device-resident), {args.config}"),
            "value": round(gib_s, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 bytes generated on device)",
            "config": {"workload": f"{args.config}: {method} over {global_count} x "
                       f"{length if length else 'U[64B,64KiB]'} B payloads"
                       + (" (offsets table)" if layout == "offsets" else "")
                       + (" as Mercury messages, verified in place" if layout == "messages" else "")
                       + (f" ({SEGS_PER_OBJECT} scattered segments each)" if layout == "segments" else "")
                       + (f", one global batch split over {world} GPUs" if world > 1 and layout != "segments"
                          else f", per GPU" if world > 1 else ""),
                       "method": method, "global_batch": global_count, "payloads_rank0": count,
                       "payload_bytes": length, "bytes_rank0": payload_bytes,
                       "lanes_per_payload": G.lanes_per_payload(method, length or 65536) if layout == "fixed" else 64,
                       "parallelism": f"shard{world}"},
            "world_size": dist.get_world_size() if world > 1 else 1,
            "per_rank": [{"rank": r, "wall_ms_per_step": round(w / args.steps * 1e3, 4), "kernel_ms": round(k, 4)}
                         for r, (w, k) in enumerate(per_rank)],
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_ms": round(kern_ms_max, 4), "algorithmic_bytes_per_launch": alg_bytes},
        }
        if world == 1 and not args.no_cpu_baseline:
            # the only leg that runs the oracle: timed on a bounded sample, and
            # the checker of the GPU's values (that sample + random payloads)
            result["cpu_baseline"], result["parity"] = cpu_baseline(
                method, seed, length, offsets_host, got, args.cpu_seconds, args.parity_samples,
                segments=layout == "segments")
        elif world > 1 and layout == "messages":
            result["parity"] = "per-rank verify counters (see verify)"
        elif world > 1:
            result["parity"] = cross_rank_check(G, method, seed, length, got, world, dev, args.parity_samples,
                                                layout, global_count, count)
        else:
            result["parity"] = "unchecked (--no-cpu-baseline)"
        if verify_note:
            result["verify"] = verify_note
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


def bench_c1(args):
    """C1 (BASELINE configs[0]): CRC-32C of 1024 x 4 KiB host buffers through
    libmchecksum's streaming API as Mercury's proc layer drives it
    (tools/c1_bench.c, C, one thread).  No GPU.  The reference's own mchecksum
    is absent, so the baseline beside it is the oracle's SSE4.2 path."""
    import struct
    import subprocess
    from oracle import oracle as O
    method, count, length, seed, _ = CONFIGS["c1"]
    exe = os.path.join(ROOT, "build", "c1_bench")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", ROOT, "build/c1_bench"], check=True)
    host = O.splitmix_bytes(count * length, seed)
    steps = max(args.steps, 200)
    r = subprocess.run([exe, str(count), str(length), str(steps), str(args.warmup)], input=host.tobytes(),
                       capture_output=True, check=True)
    el, first, xsum = r.stdout.decode().split()
    el = float(el)
    want = [O.crc(method, struct.pack("<I", length) + host[i * length:(i + 1) * length].tobytes())
            for i in range(count)]
    wx = 0
    for w in want:
        wx ^= w
    ok = int(first) == want[0] and int(xsum) == wx
    ref_t0 = time.perf_counter()
    for _ in range(steps):
        O.batch_fixed(method, host, length, length, count, variant="sse42", nthreads=1)
    ref_el = time.perf_counter() - ref_t0
    res = {"metric": "GiB/s checksummed on the host CPU through the mchecksum API, c1",
           "value": round(count * (length + 4) * steps / el / 2**30, 3), "unit": "GiB/s", "n_gpus": 0,
           "steps": steps, "warmup": args.warmup, "ms_per_step": round(el / steps * 1e3, 4),
           "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "u8",
           "data": "synthetic (splitmix64 bytes)",
           "config": {"workload": "crc32c, 1024 x (4 B length field + 4 KiB raw bytes) via reset/update/update/get",
                      "threads": 1, "driver": "tools/c1_bench.c"},
           "parity": "bit-exact (all 1024 payloads: first + xor-sum vs oracle)" if ok else "MISMATCH",
           "cpu_baseline": {"value": round(count * length * steps / ref_el / 2**30, 3), "unit": "GiB/s",
                            "cores": 1, "kind": "port", "variant": "x86 SSE4.2 crc32 instruction (oracle)",
                            "sample": f"{steps} passes over the same 1024 x 4 KiB buffers"}}
    print(json.dumps(res), flush=True)
    return res


def _segment_object_bytes(O, seed, length, j, slots):
    """Host bytes of object j of the segments layout (oracle generator)."""
    seg = length // SEGS_PER_OBJECT
    return np.concatenate([O.splitmix_bytes(seg, seed, first_word=int(slots[j * SEGS_PER_OBJECT + q]) * seg // 8)
                           for q in range(SEGS_PER_OBJECT)])


def _cpu_quota():
    """The cgroup v2 CPU limit as (CPUs,), e.g. cpu.max "1600000 100000" -> (16.0,); None if unlimited."""
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q and q[0] != "max":
            return (int(q[0]) / int(q[1]),)
    except (OSError, ValueError, IndexError, ZeroDivisionError):
        pass
    return None


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(method, seed, length, offsets_host, got, budget_s, samples, segments=False):
    """The CPU leg (N=1, rank 0): the oracle (CPU restatement of mchecksum --
    the reference's own mchecksum is absent, so kind = "port") timed on this
    host's cores over a bounded sample of the same workload (the first n
    payloads), whose CRCs then check the GPU's values for those payloads; plus
    `samples` random payloads from the whole batch."""
    from oracle import oracle as O
    # `nproc` threads (BASELINE.md "Thread counts"): every CPU this process may
    # run on -- capped by the cgroup CPU quota when the box sets one (the GPU
    # box grants 16 CPUs of a 128-thread host: 256 threads on that quota ran
    # 4x slower than 16)
    affinity = len(os.sched_getaffinity(0))
    quota = _cpu_quota()
    threads = max(1, min(256, affinity, int(quota[0]) if quota else affinity))
    variant = "sse42" if method == "crc32c" else "slice8"
    slots = None
    if segments:
        from mercury_amd.workload import segment_slots
        slots = segment_slots(seed, len(got) * SEGS_PER_OBJECT)
        n = 256
        host = np.concatenate([_segment_object_bytes(O, seed, length, j, slots) for j in range(n)])
        runv = lambda k, v, th: O.batch_fixed(method, host, length, length, k, variant=v, nthreads=th)  # noqa: E731
        sample_bytes = n * length
        what = f"the first {n} objects ({SEGS_PER_OBJECT} x {length // SEGS_PER_OBJECT} B segments, gathered)"
    elif offsets_host is None:
        n = 4096 if length <= 65536 else 256
        host = O.splitmix_bytes(n * length, seed)
        runv = lambda k, v, th: O.batch_fixed(method, host, length, length, k, variant=v, nthreads=th)  # noqa: E731
        sample_bytes = n * length
        what = f"{n} x {length} B"
    else:
        n = int(np.searchsorted(offsets_host, np.uint64(256 << 20)))  # ~256 MiB of whole payloads
        host = O.splitmix_bytes(int(offsets_host[n]), seed)
        sub = np.ascontiguousarray(offsets_host[:n + 1])
        runv = lambda k, v, th: O.batch_offsets(method, host, sub[:k + 1], variant=v, nthreads=th)  # noqa: E731
        sample_bytes = int(offsets_host[n])
        what = f"the first {n} payloads ({sample_bytes} B) of the offsets layout"
    run = lambda k: runv(k, variant, threads)  # noqa: E731
    for _ in range(3):  # warm-ups
        run(n)
    # per-pass CLOCK_MONOTONIC times (time.perf_counter), >= 20 passes and the
    # wall budget (1.5 s x 16 threads: ~24 s of CPU work); the value is the
    # median pass
    laps, t0 = [], time.perf_counter()
    while True:
        ta = time.perf_counter()
        want = run(n)
        laps.append(time.perf_counter() - ta)
        el = time.perf_counter() - t0
        if (el >= budget_s and len(laps) >= 20) or (el >= 4 * budget_s and len(laps) >= 5) or len(laps) >= 20000:
            break
    med = float(np.median(laps))
    base = {"value": round(sample_bytes / med / 2**30, 2), "unit": "GiB/s", "cores": threads, "kind": "port",
            "variant": "x86 SSE4.2 crc32 instruction" if variant == "sse42" else "slicing-by-8 tables",
            "sample": f"median of {len(laps)} passes over {what} of the same splitmix payloads "
                      f"({el:.2f} s wall, {threads} threads)"}
    base["cpus_visible"] = f"{affinity} in the affinity mask" + (f", cgroup quota {quota[0]:g} CPUs" if quota else "")
    # the other CPU paths on the same sample: 1 thread, and the
    # table path next to SSE4.2 for CRC-32C
    legs = [(variant, 1), ("table", threads)]  # 1 thread; the byte-table (Sarwate) path at full width
    breakdown = {}
    for v, th in legs:
        p2, t2 = 0, time.perf_counter()
        while True:
            runv(n, v, th)
            p2 += 1
            e2 = time.perf_counter() - t2
            if e2 >= budget_s / 3 or p2 >= 50:
                break
        breakdown[f"{v}_{th}thread{'s' if th > 1 else ''}"] = round(p2 * sample_bytes / e2 / 2**30, 2)
    base["breakdown_GiB_s"] = breakdown
    base["cpu_model"] = _cpu_model()

    bad = int(np.count_nonzero(got[:n] != want))
    rng = np.random.default_rng(1234)
    total = len(got)
    idx = np.unique(np.concatenate([[total - 1], rng.integers(n, total, samples)])) if total > n else []
    for gi in idx:
        gi = int(gi)
        if segments:
            w = O.crc(method, _segment_object_bytes(O, seed, length, gi, slots))
        elif offsets_host is None:
            w = O.splitmix_batch_fixed(method, seed, length, length, gi, 1)[0]
        else:
            lo, hi = int(offsets_host[gi]), int(offsets_host[gi + 1])
            w0 = lo // 8
            b = O.splitmix_bytes(hi - w0 * 8, seed, first_word=w0)
            w = O.crc(method, b[lo - w0 * 8:])
        bad += int(got[gi] != w)
    checked = n + len(idx)
    parity = f"bit-exact ({checked} payloads vs oracle)" if bad == 0 else f"MISMATCH {bad}/{checked}"
    return base, parity


def cross_rank_check(G, method, seed, length, got, world, dev, samples, layout, global_count, count0):
    """N>1 (rank 0): regenerate sampled payloads of EVERY rank's share on rank
    0's GPU and recompute them through the same entry point; the gathered CRCs
    (global payload order) must agree.  Kernel parity itself is the N=1 oracle
    check and tests/."""
    if got is None:
        return None
    import torch
    from mercury_amd.workload import varlen_offsets
    rng = np.random.default_rng(4321)
    bad = checked = 0
    if layout == "segments":  # weak: rank r's objects from seed ^ r, count0 per rank
        from mercury_amd.workload import segment_slots
        seg = length // SEGS_PER_OBJECT
        for r in range(world):
            slots = segment_slots(seed ^ r, count0 * SEGS_PER_OBJECT)
            for i in np.unique(np.concatenate([[0, count0 - 1], rng.integers(0, count0, max(1, samples // world))])):
                parts = []
                for q in range(SEGS_PER_OBJECT):
                    t = torch.empty(seg + 64, dtype=torch.uint8, device=dev)
                    G.fill_splitmix(t, seed ^ r, first_word=int(slots[int(i) * SEGS_PER_OBJECT + q]) * seg // 8)
                    parts.append(t[:seg])
                bad += int(G.as_unsigned(G.checksum_segments(method, parts))[0] != got[r * count0 + int(i)])
                checked += 1
    else:
        off = varlen_offsets(seed, global_count) if layout == "offsets" else None
        idx = np.unique(np.concatenate([[0, global_count - 1], rng.integers(0, global_count, samples)]))
        for i in idx:
            i = int(i)
            if off is None:
                buf = torch.empty(length + 64, dtype=torch.uint8, device=dev)
                G.fill_splitmix(buf, seed, first_word=i * length // 8)
                v = G.checksum_fixed(method, buf, length, count=1)
            else:
                lo, hi = int(off[i]), int(off[i + 1])
                w0 = lo // 8
                buf = torch.empty(hi - w0 * 8 + 64, dtype=torch.uint8, device=dev)
                G.fill_splitmix(buf, seed, first_word=w0)
                t = torch.tensor([lo - w0 * 8, hi - w0 * 8], dtype=torch.int64, device=dev)
                v = G.checksum_offsets(method, buf, t)
            bad += int(G.as_unsigned(v)[0] != got[i])
            checked += 1
    return (f"consistent ({checked} payloads across all {world} shares recomputed on rank 0)" if bad == 0
            else f"MISMATCH {bad}/{checked} across shards")


if __name__ == "__main__":
    main()
