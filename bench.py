#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X mchecksum batch path.

Metric (BASELINE.json): GiB/s checksummed (device-resident), CRC32c,
64K x 64 KiB payloads.  One "step" = one batch launch over the whole
per-GPU batch (65536 payloads of 64 KiB = 4 GiB), inputs already in HBM.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N,
or bench.py --gpus N, which starts those ranks itself): each rank owns a
contiguous share of ONE global batch, generated on its own device; no
collective in the timed region.  By default every rank's share is the
headline's 65536 x 64 KiB (weak scaling: the global batch is N x 4 GiB), so
the 1/2/4/8 series is one per-GPU workload; --config c5 splits C5's fixed
2^20 x 64 KiB batch instead (strong).  After timing: RCCL all_gather of the
per-share CRC arrays (global payload order) and of the timings.  Under
torchrun the process group is formed at every world size, 1 included.

Prints ONE JSON line on rank 0 (contract in the task statement), with
`roofline` (HIP-event kernel time vs HBM peak; `traffic` from the committed
PMC profile, scaled to rank 0's share at N > 1) and `cpu_baseline` (the
oracle timed on this host's cores, at every N, on rank 0 after timing) --
the oracle also checks the gathered CRCs of every share (`parity`).
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md:36
SEGS_PER_OBJECT = 4

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
    # 8(f) 4: C4's payloads as hg_perf_proc_iovec messages serialized in XDR
    # mode (Testing/perf/hg/mercury_perf.c:897-923; src/mercury_proc.h:110-160):
    # a big-endian u32 length, the bytes, zero pad to 4 -- while the checksum
    # covers the host-order length and the bytes (mchecksum_gpu_checksum_xdr)
    "xdr": ("crc32c", 262144, None, 0x4D43310000000004, "xdr"),
}
# configs whose count is the GLOBAL batch, split over the ranks (strong
# scaling); the others give every rank a batch of that size (weak scaling)
STRONG = {"c5", "c4", "msgs", "xdr"}
# hg_perf_proc_iovec's XDR schema: INT(4) length, OPAQUE_LEN bytes
XDR_IOVEC = [(0, 4), (2, 0)]


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); without torchrun in the environment bench.py starts them itself")
    p.add_argument("--steps", type=int, default=50)
    # 40: the clock settles after ~30 back-to-back launches (per-launch times
    # 0.62 -> 0.75 -> 0.62 ms over the first 30, profiles/r01/launch_series_metric.json)
    p.add_argument("--warmup", type=int, default=40)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS),
                   help="default: the headline (metric), 65536 x 64 KiB per GPU at every N (weak scaling); "
                        "c5 = C5's 2^20 x 64 KiB global batch split over the ranks (strong scaling)")
    p.add_argument("--streams", type=int, default=1,
                   help="issue consecutive steps round-robin on this many streams (independent batches, "
                        "fixed and offsets layouts)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=1.5, help="wall budget of the CPU baseline sample")
    p.add_argument("--parity-samples", type=int, default=64)
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="nccl = RCCL (default); gloo only to rehearse the multi-rank flow on one GPU")
    p.add_argument("--no-c5-strong", action="store_true",
                   help="skip the c5_strong sub-record of the default (headline) run")
    p.add_argument("--no-e2e", action="store_true",
                   help="skip the e2e sub-record of the default (headline) run at N=1 (host memory -> GPU -> host)")
    p.add_argument("--e2e-reps", type=int, default=5, help="timed passes per e2e leg (median reported)")
    p.add_argument("--rotate", type=int, default=None,
                   help="fixed layouts: step i reads batch i %% R of R equal batches at distinct addresses, so no "
                        "launch re-reads what the previous one left in the 256 MiB Infinity Cache "
                        "(default: 4 for c2, whose 256 MiB batch fits that cache; 1 otherwise)")
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
        # every N runs the headline's per-GPU batch (65536 x 64 KiB per rank,
        # weak scaling), so the driver's 1/2/4/8 series is one workload
        args.config = "metric"
    if CONFIGS[args.config][4] == "cpu":
        return bench_c1(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Under torchrun (WORLD_SIZE set) the process group is formed at every
    # world size, 1 included: `torchrun --nproc-per-node 1 bench.py` runs the
    # same RCCL calls as the 8-GPU run (init, all_gather, all_reduce).
    dist_on = env_world is not None
    ndev = torch.cuda.device_count()  # (counting devices does not initialise the GPU)
    if dist_on:
        # one GPU per rank: a node with more ranks than GPUs is refused (round 4
        # mapped ranks modulo the count); only the gloo rehearsal may share one.
        # Per node (LOCAL_WORLD_SIZE): a multi-node run has more ranks in all
        # than one node has GPUs.
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if args.backend == "nccl" and (local >= ndev or local_world > ndev):
            sys.exit(f"bench.py: {local_world} ranks on this node (LOCAL_RANK {local}) but {ndev} GPU(s) visible: "
                     "one GPU per rank")
        torch.cuda.set_device(local if args.backend == "nccl" else local % max(ndev, 1))
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
        # the line reports the group's own size and rank, not the environment's
        world, rank = dist.get_world_size(), dist.get_rank()
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")
    # every rank's PCI address and host, gathered into the line: N distinct
    # GPUs took part (the same PCI address on two hosts is two GPUs)
    import socket
    import zlib
    host = socket.gethostname()
    pci = [float(x) for x in pci_address(torch, dev)] + [float(zlib.crc32(host.encode()))]
    if dist_on:
        pt = torch.tensor(pci, dtype=torch.float64, device=coll_dev)
        allp = [torch.empty_like(pt) for _ in range(world)]
        dist.all_gather(allp, pt)
        keys = [tuple(p.tolist()) for p in allp]
    else:
        keys = [tuple(pci)]
    pcis = [pci_string(k[:3]) for k in keys]
    if args.backend == "nccl" and len(set(keys)) != world:
        sys.exit(f"bench.py: ranks share a GPU ({pcis}): one GPU per rank")

    # The sub-records run before the headline, so the headline's dispatches
    # are the last of their kernel in a profile of this command, in the order
    # e2e, c5_strong, headline: with the PCIe-bound e2e second between
    # c5_strong and the headline, the headline measured ~1% lower and noisier
    # (0.837-0.856 vs 0.854-0.857 on one box, profiles/r06/order/).
    e2e = None
    if args.config == "metric" and not args.no_e2e and world == 1:
        # north_star's end-to-end rate: the headline's bytes starting and
        # ending in host memory (NA recv buffers / hg_proc buffers)
        e2e = run_e2e(args, torch, dev)
    c5_strong = None
    if args.config == "metric" and not args.no_c5_strong:
        # BASELINE configs[4] in the same run, whatever flags the driver
        # passes: C5's fixed 2^20 x 64 KiB batch split over the ranks (strong
        # scaling)
        c5_strong = run_c5_strong(args, torch, dist, dist_on, rank, world, dev, coll_dev)

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
    elif layout == "xdr":
        plan = batch_shard(rank, world, global_count, offsets_global=xdr_offsets(seed, global_count))
    if plan is not None:
        count = plan.count
    stream = torch.cuda.current_stream()
    G.prepare(method)

    rotate = args.rotate if args.rotate is not None else (4 if args.config == "c2" else 1)
    if rotate < 1 or (rotate > 1 and layout != "fixed"):
        raise SystemExit("--rotate needs R >= 1, and R > 1 a fixed layout")
    datas = None
    # ---- this rank's share of the global batch, generated on the device ----
    if layout == "fixed":
        # R copies of the share at distinct addresses (R > 1: every launch
        # reads cold lines -- the previous launch read another copy)
        datas = [torch.empty(plan.nbytes + 64, dtype=torch.uint8, device=dev) for _ in range(rotate)]
        for d in datas:
            G.fill_splitmix(d, seed, first_word=plan.first_word)  # the global stream's bytes
        data = datas[0]
        offsets_dev = offsets_host = None
        payload_bytes = plan.nbytes
        run = lambda out, b=0: G.checksum_fixed(method, datas[b], length, count=count, out=out)  # noqa: E731
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
    elif layout == "xdr":
        # the rank's messages: splitmix bytes, then each message's big-endian
        # length word and zero pad written over them
        from mercury_amd.workload import varlen_lengths
        offsets_host = plan.offsets
        payload_bytes = int(offsets_host[-1] - offsets_host[0])  # message bytes (read)
        data = torch.empty(plan.nbytes + 64, dtype=torch.uint8, device=dev)
        G.fill_splitmix(data, seed, first_word=plan.first_word)
        lens = varlen_lengths(seed, global_count)[plan.first:plan.first + count].astype(np.int64)
        msg_dev = torch.from_numpy(offsets_host.astype(np.int64)).to(dev)
        lens_dev = torch.from_numpy(lens).to(dev)
        for k in range(4):
            data[msg_dev[:-1] + k] = ((lens_dev >> (24 - 8 * k)) & 0xFF).to(torch.uint8)
        for k in range(1, 4):  # pad bytes: 4 + len .. 4 + RNDUP(len)
            sel = (-lens_dev) % 4 >= k
            data[(msg_dev[:-1] + 4 + lens_dev + k - 1)[sel]] = 0
        offsets_dev = msg_dev
        xout = torch.empty(count, dtype=G.out_dtype(method), device=dev)
        G.checksum_xdr(method, data, msg_dev, XDR_IOVEC, offsets_host=offsets_host, out=xout)  # validates once
        run = lambda out: G.checksum_xdr(method, data, msg_dev, XDR_IOVEC, out=out)  # noqa: E731
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
    # S > 1: S pool streams, none of them the default stream -- HIP's null
    # stream is ordered against the others, so a pair that includes it never
    # overlaps (round 5: +-0 either way without a profiler)
    streams = [stream] if args.streams == 1 else [torch.cuda.Stream(device=dev) for _ in range(args.streams)]
    outs = [out] + [torch.empty_like(out) for _ in range(args.streams - 1)]
    torch.cuda.synchronize()

    def step(i):  # step i: one batch (copy i % R), on stream i % S with its own output
        s = streams[i % len(streams)]
        with torch.cuda.stream(s):
            if rotate > 1:
                run(outs[i % len(streams)], i % rotate)
            else:
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
    if dist_on:
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
    if dist_on:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev_start.elapsed_time(ev_end) / args.steps

    rotation = None
    if rotate > 1:
        # every copy gives the same CRCs, and the replay figure of copy 0 alone
        # (each launch re-reads what the last one left in the Infinity Cache),
        # kept only as a labelled cache-warm number
        outs_r = [torch.empty_like(out) for _ in range(rotate)]
        for b in range(rotate):
            run(outs_r[b], b)
        same = all(torch.equal(outs_r[0], o) for o in outs_r[1:])
        for _ in range(args.warmup):
            run(out, 0)
        ew0, ew1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ew0.record()
        for _ in range(args.steps):
            run(out, 0)
        ew1.record()
        torch.cuda.synchronize()
        warm_ms = ew0.elapsed_time(ew1) / args.steps
        rotation = {"copies": rotate, "bytes_per_copy": payload_bytes, "copies_agree": same,
                    "cache_warm": {"kernel_ms": round(warm_ms, 4),
                                   "GiB_s": round(payload_bytes / (warm_ms * 1e-3) / 2**30, 2),
                                   "note": "replay of ONE copy back to back (Infinity-Cache warm; not HBM evidence)"}}

    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=coll_dev)
    per_rank = [t.clone() for _ in range(world)]
    if dist_on:
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
    if dist_on:
        # RCCL all_gather of the per-rank CRC arrays (padded to the largest
        # shard: ranks may hold different counts), then trimmed in rank order:
        # the global batch's CRCs in global payload order (messages: the
        # sender's interleaved header/payload pieces, two per message)
        counts = plan.counts if plan is not None else [count] * world
        if layout == "messages":
            counts = [2 * c for c in counts]
        crcs = gather_shares(dist, crcs, counts, world, coll_dev)
    got = G.as_unsigned(crcs) if rank == 0 else None

    bytes_all = torch.tensor([float(payload_bytes)], dtype=torch.float64, device=coll_dev)
    if dist_on:
        dist.all_reduce(bytes_all)
    total_bytes = float(bytes_all[0]) * args.steps  # every rank checksummed its shard once per step
    gib_s = total_bytes / wall_max / 2**30
    out_bytes = count * (4 if G.out_dtype(method) == torch.int32 else 8)
    alg_bytes = payload_bytes + out_bytes + (8 * (count + 1) if layout in ("offsets", "xdr") else 0) + \
        (16 * count * SEGS_PER_OBJECT + 8 * (count + 1) if layout == "segments" else 0)
    if layout == "messages":  # messages read (headers included), 1 status byte each, the offsets table
        alg_bytes = payload_bytes + count + 8 * (count + 1)
    achieved = alg_bytes / (kern_ms_max * 1e-3) / 1e9

    result = None
    if rank == 0:
        from types import SimpleNamespace
        result = report(args, SimpleNamespace(
            config=args.config, method=method, seed=seed, length=length, layout=layout, strong=strong,
            global_count=global_count, count=count, plan=plan, payload_bytes=payload_bytes, alg_bytes=alg_bytes,
            gib_s=gib_s, wall_max=wall_max, kern_ms_max=kern_ms_max, achieved=achieved, per_rank=per_rank,
            world=world, got=got, offsets_host=offsets_host, verify_note=verify_note,
            process_group=dist.get_backend() if dist_on else None, pcis=pcis,
            lanes=G.lanes_per_payload(method, length or 65536) if layout == "fixed" else 64))
        if c5_strong is not None:
            if not args.no_cpu_baseline:
                c5_strong["parity"] = c5_parity(c5_strong.pop("_got"), c5_strong.pop("_firsts"), args.parity_samples)
            c5_strong.pop("_got", None)
            c5_strong.pop("_firsts", None)
            result["c5_strong"] = c5_strong
        if rotation is not None:
            result["rotation"] = rotation
            result["roofline"]["cache"] = (f"cold: step i reads copy i % {rotate} of {rotate} at distinct addresses "
                                           f"({rotate * payload_bytes / 2**20:.0f} MiB in all)")
        if e2e is not None:
            result["e2e"] = e2e_finish(e2e, got, args)
        print(json.dumps(result), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    return result


def report(args, r):
    """Rank 0's JSON line of one run (r: the run's shape, shares, timings and
    gathered CRCs, assembled by main).  The oracle runs here, after timing, at
    every N: the CPU baseline, and the parity check of every rank's share."""
    traffic, traffic_src = pmc_traffic(r.config, r.world, r.alg_bytes)
    metric = {"metric": "GiB/s checksummed (device-resident), CRC32c, 64K x 64 KiB payloads",
              "c5": "GiB/s checksummed (device-resident), CRC32c, 1M x 64 KiB payloads split over the GPUs (C5)"}
    per_gpu = r.global_count // r.world if not r.strong else r.global_count
    workload = (f"{r.config}: {r.method} over {per_gpu if not r.strong else r.global_count} x "
                f"{r.length if r.length else 'U[64B,64KiB]'} B payloads"
                + (" (offsets table)" if r.layout == "offsets" else "")
                + (" as Mercury messages, verified in place" if r.layout == "messages" else "")
                + (" as hg_perf_proc_iovec messages in XDR mode" if r.layout == "xdr" else "")
                + (f" ({SEGS_PER_OBJECT} scattered segments each)" if r.layout == "segments" else "")
                + (f", one global batch split over {r.world} GPUs" if r.world > 1 and r.strong
                   else f" per GPU ({r.global_count} in all over {r.world} GPUs)" if r.world > 1 else ""))
    result = {
        "metric": metric.get(r.config, f"GiB/s checksummed (device-resident), {r.config}"),
        "value": round(r.gib_s, 2),
        "unit": "GiB/s",
        "n_gpus": r.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(r.wall_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if r.strong else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (splitmix64 bytes generated on device)",
        "config": {"workload": workload, "method": r.method, "global_batch": r.global_count,
                   "payloads_rank0": r.count, "payload_bytes": r.length, "bytes_rank0": r.payload_bytes,
                   "lanes_per_payload": r.lanes, "parallelism": f"shard{r.world}",
                   **({"streams": args.streams} if getattr(args, "streams", 1) > 1 else {})},
        "world_size": r.world,
        "process_group": getattr(r, "process_group", None),
        "per_rank": [dict({"rank": i, "wall_ms_per_step": round(w / args.steps * 1e3, 4), "kernel_ms": round(k, 4)},
                          **({"pci": r.pcis[i]} if getattr(r, "pcis", None) else {}))
                     for i, (w, k) in enumerate(r.per_rank)],
        "roofline": {"bound": "hbm", "achieved": round(r.achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(r.achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel_ms": round(r.kern_ms_max, 4), "algorithmic_bytes_per_launch": r.alg_bytes},
    }
    if not args.no_cpu_baseline:
        # the only leg that runs the oracle: timed on a bounded sample on this
        # host's cores, and the checker of the gathered CRCs -- that sample,
        # the first and last payload of every rank's share and random payloads
        # of the whole global batch
        result["cpu_baseline"], result["parity"] = cpu_baseline(
            r.method, r.seed, r.length, global_offsets(r.layout, r.seed, r.global_count, r.offsets_host), r.got,
            args.cpu_seconds, args.parity_samples, segments=r.layout == "segments",
            world=r.world, count0=r.count, share_firsts=share_firsts(r.plan, r.layout, r.world, r.count),
            xdr=r.layout == "xdr")
    else:
        result["parity"] = "unchecked (--no-cpu-baseline)"
    if getattr(args, "streams", 1) > 1:
        # consecutive steps overlap pairwise on the GPU: kernel_ms is the event
        # region over the steps, not one dispatch's duration (a rocprof trace
        # shows each dispatch ~S times as long)
        result["roofline"]["kernel_ms_is"] = f"event region / steps ({args.streams} streams overlap)"
    if r.verify_note:
        result["verify"] = r.verify_note
    return result


def pci_address(torch, dev):
    """(domain, bus, device) of the rank's GPU (-1 where torch does not say)."""
    p = torch.cuda.get_device_properties(dev)
    return tuple(int(getattr(p, k, -1)) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))


def pci_string(v):
    d, b, f = (int(x) for x in v)
    return f"{d:04x}:{b:02x}:{f:02x}" if min(d, b, f) >= 0 else "unknown"


C5 = "c5"


def run_c5_strong(args, torch, dist, dist_on, rank, world, dev, coll_dev):
    """The c5_strong sub-record of the default run: BASELINE configs[4] --
    CRC-32C over 2^20 x 64 KiB payloads, ONE global batch split into
    contiguous rank shares (2^20 / N per rank) -- timed the same way as the
    headline (barrier + synchronize around K back-to-back launches, max over
    ranks), its CRCs gathered over the process group for the oracle check."""
    from mercury_amd import gpu as G
    from mercury_amd.shard import batch_shard
    method, gcount, length, seed, _ = CONFIGS[C5]
    plan = batch_shard(rank, world, gcount, length)
    data = torch.empty(plan.nbytes + 64, dtype=torch.uint8, device=dev)
    G.fill_splitmix(data, seed, first_word=plan.first_word)
    out = torch.empty(plan.count, dtype=G.out_dtype(method), device=dev)
    G.prepare(method)
    for _ in range(args.warmup):
        G.checksum_fixed(method, data, length, count=plan.count, out=out)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        G.checksum_fixed(method, data, length, count=plan.count, out=out)
    ev1.record()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=coll_dev)
    per_rank = [t.clone() for _ in range(world)]
    crcs = out
    if dist_on:
        dist.all_gather(per_rank, t)
        crcs = gather_shares(dist, out, plan.counts, world, coll_dev)
    per_rank = [[float(x[0]), float(x[1])] for x in per_rank]
    got = G.as_unsigned(crcs) if rank == 0 else None
    del data, out
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    wall_max = max(w for w, _ in per_rank)
    kern_max = max(k for _, k in per_rank)
    total = float(gcount) * length * args.steps
    alg = plan.nbytes + 4 * plan.count  # rank 0's share: payload bytes + 4-byte CRCs
    return {
        "config": C5,
        "metric": "GiB/s checksummed (device-resident), CRC32c, 1M x 64 KiB payloads split over the GPUs (C5)",
        "workload": (f"c5: {method} over {gcount} x {length} B payloads, one global batch split over {world} "
                     f"GPU{'s' if world > 1 else ''} ({plan.count} on rank 0)"),
        "value": round(total / wall_max / 2**30, 2),
        "unit": "GiB/s",
        "scaling": "strong",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall_max / args.steps * 1e3, 4),
        "kernel_ms": round(kern_max, 4),
        "roofline_frac": round(alg / (kern_max * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "per_rank": [{"rank": i, "wall_ms_per_step": round(w / args.steps * 1e3, 4), "kernel_ms": round(k, 4)}
                     for i, (w, k) in enumerate(per_rank)],
        "_got": got,
        "_firsts": share_firsts(plan, "fixed", world, plan.count),
    }


PCIE_GEN5_X16_GBS = 63.0  # 32 GT/s x 16 lanes, 128b/130b encoding, per direction


def _hip():
    """libamdhip64 (the one torch loaded) for the host-memory calls torch does not wrap."""
    import ctypes
    import torch
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    vp = ctypes.c_void_p
    lib.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
    lib.hipHostGetDevicePointer.restype = ctypes.c_int
    return lib


def run_e2e(args, torch, dev):
    """The e2e sub-record of the default run (N = 1): the headline's 65536 x
    64 KiB payloads starting and ending in HOST memory, as Mercury's NA recv
    buffers and hg_proc buffers are (src/mercury_core.c:4667-4714 hands the
    received bytes to the proc layer).  Three legs over the same pinned 4 GiB,
    each the median of --e2e-reps timed passes after one untimed pass:

      staged    -- H2D in 128 MiB chunks on a copy stream, double-buffered
                   against the batch kernel on a compute stream, and D2H of
                   each chunk's CRCs: the copy engine and the kernel overlap;
      h2d_only  -- the same chunked H2D alone (this link's measured ceiling);
      zero_copy -- one batch call on the pinned buffer's device alias: the
                   kernel reads the bytes over PCIe, no staging copy.

    Beside them the host CPU over the same pinned bytes (the product's
    streaming API on the box's cores, and the oracle), so the crossover is
    in the line.  The CRCs are compared after the headline (e2e_finish)."""
    import ctypes
    from mercury_amd import gpu as G
    method, count, length, seed, _ = CONFIGS["metric"]
    chunk = 128 << 20
    total = count * length
    nchunks, per = total // chunk, chunk // length
    G.prepare(method)
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    stage = torch.empty(chunk + 64, dtype=torch.uint8, device=dev)
    for i in range(nchunks):  # the headline's bytes (same splitmix stream), made on the device
        G.fill_splitmix(stage, seed, first_word=i * chunk // 8)
        host[i * chunk:(i + 1) * chunk].copy_(stage[:chunk])
    torch.cuda.synchronize()
    del stage
    dbuf = [torch.empty(chunk + 64, dtype=torch.uint8, device=dev) for _ in range(2)]
    dout = [torch.empty(per, dtype=torch.int32, device=dev) for _ in range(2)]
    hout = torch.empty(count, dtype=torch.int32, pin_memory=True)
    zout = torch.empty(count, dtype=torch.int32, device=dev)
    s_copy, s_comp = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)

    def staged():
        copied = [torch.cuda.Event() for _ in range(2)]
        free = [torch.cuda.Event() for _ in range(2)]
        for e in free:
            e.record(s_comp)
        for i in range(nchunks):
            b = i % 2
            s_copy.wait_event(free[b])  # the kernel is done with buffer b
            with torch.cuda.stream(s_copy):
                dbuf[b][:chunk].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)
                copied[b].record(s_copy)
            s_comp.wait_event(copied[b])
            G.checksum_fixed(method, dbuf[b], length, count=per, out=dout[b], stream=s_comp)
            with torch.cuda.stream(s_comp):
                hout[i * per:(i + 1) * per].copy_(dout[b], non_blocking=True)
            free[b].record(s_comp)

    def h2d_only():
        with torch.cuda.stream(s_copy):
            for i in range(nchunks):
                dbuf[i % 2][:chunk].copy_(host[i * chunk:(i + 1) * chunk], non_blocking=True)

    hip = _hip()
    alias = ctypes.c_void_p()
    zc_err = hip.hipHostGetDevicePointer(ctypes.byref(alias), ctypes.c_void_p(host.data_ptr()), 0)
    lib = G._lib()

    def zero_copy():
        rc = lib.mchecksum_gpu_checksum_fixed(method.encode(), alias.value, length, length, count, zout.data_ptr(),
                                              s_comp.cuda_stream)
        if rc:
            raise G.GpuChecksumError(f"zero-copy batch call rc={rc}")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        laps = []
        for _ in range(max(1, args.e2e_reps)):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            laps.append(time.perf_counter() - t0)
        med = float(np.median(laps))
        return {"GiB_s": round(total / med / 2**30, 2), "GB_s": round(total / med / 1e9, 2),
                "pcie_frac": round(total / med / 1e9 / PCIE_GEN5_X16_GBS, 4), "ms": round(med * 1e3, 2),
                "ms_min": round(min(laps) * 1e3, 2), "ms_max": round(max(laps) * 1e3, 2), "reps": len(laps)}

    rec = {"workload": f"{method} over {count} x {length} B payloads in pinned host memory (the headline's bytes), "
                       "CRCs back in host memory",
           "pcie_spec_GB_s": PCIE_GEN5_X16_GBS,
           "staged": dict(timed(staged), chunk_bytes=chunk, streams="copy + compute, double-buffered"),
           "h2d_only": dict(timed(h2d_only), chunk_bytes=chunk)}
    rec["staged"]["of_h2d_only"] = round(rec["h2d_only"]["ms"] / rec["staged"]["ms"], 4)
    if zc_err == 0:
        rec["zero_copy"] = dict(timed(zero_copy), how="hipHostGetDevicePointer alias of the pinned buffer, one call")
    else:
        rec["zero_copy"] = {"skipped": f"hipHostGetDevicePointer error {zc_err}"}
    # host CPU over the same pinned bytes: the first 4096 payloads (256 MiB)
    cpu_n = 4096
    hb = host.numpy()
    threads = _cpu_threads()
    cpu = {"sample": f"the first {cpu_n} payloads ({cpu_n * length >> 20} MiB) of the same pinned buffer",
           "cores": threads}
    try:
        pv = product_batch(method, hb[:cpu_n * length], threads, count=cpu_n, length=length)
        cpu["product_crcs"] = pv
        cpu["product_GiB_s"] = round(_rate(lambda: product_batch(method, hb[:cpu_n * length], threads, count=cpu_n,
                                                                 length=length), cpu_n * length), 2)
    except OSError as e:
        cpu["product_GiB_s"] = None
        cpu["product_note"] = f"product CPU path not timed: {e}"
    rec["cpu_same_bytes"] = cpu
    rec["_crcs"] = {"staged": hout.numpy().view(np.uint32).copy(), "zero_copy": G.as_unsigned(zout)
                    if zc_err == 0 else None}
    rec["_host"] = hb
    rec["_shape"] = (method, count, length, cpu_n)
    del dbuf, dout
    torch.cuda.synchronize()
    return rec


def _rate(fn, nbytes, budget_s=0.5):
    """GiB/s of fn over nbytes: passes until budget_s, at least 3."""
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        el = time.perf_counter() - t0
        if el >= budget_s and n >= 3:
            return n * nbytes / el / 2**30


def e2e_finish(rec, got, args):
    """The e2e CRCs against the headline's device-resident CRCs (every
    payload; those are oracle-checked in `parity`) and, independently, the
    oracle over sampled payloads of the pinned host bytes themselves."""
    from oracle import oracle as O
    method, count, length, cpu_n = rec.pop("_shape")
    crcs, hb = rec.pop("_crcs"), rec.pop("_host")
    notes, ok = [], True
    for leg in ("staged", "zero_copy"):
        c = crcs.get(leg)
        if c is None:
            continue
        bad = int(np.count_nonzero(c.astype(np.uint64) != np.asarray(got[:count]).astype(np.uint64)))
        ok &= bad == 0
        notes.append(f"{leg}: {count - bad}/{count} equal the device-resident CRCs")
    rng = np.random.default_rng(0xE2E)
    idx = sorted(set([0, count - 1]) | set(int(i) for i in rng.integers(0, count, 62)))
    obad = sum(int(crcs["staged"][i]) != O.crc(method, hb[i * length:(i + 1) * length]) for i in idx)
    ok &= obad == 0
    notes.append(f"{len(idx) - obad}/{len(idx)} sampled payloads of the pinned bytes equal the oracle")
    cpu = rec["cpu_same_bytes"]
    pv = cpu.pop("product_crcs", None)
    if pv is not None:
        n = len(pv)
        pbad = int(np.count_nonzero(pv.astype(np.uint64) != crcs["staged"][:n].astype(np.uint64)))
        ok &= pbad == 0
        notes.append(f"product CPU path: {n - pbad}/{n} equal the staged GPU CRCs")
    rec["parity"] = ("bit-exact: " if ok else "MISMATCH: ") + "; ".join(notes)
    if not args.no_cpu_baseline:
        # the oracle on the same sample, on the same cores (kind "port": the
        # reference's own mchecksum is absent)
        sub = hb[:cpu_n * length]
        threads = cpu["cores"]
        cpu["oracle_GiB_s"] = round(_rate(lambda: O.batch_fixed(method, sub, length, length, cpu_n,
                                                                variant="sse42", nthreads=threads),
                                          cpu_n * length), 2)
        cpu["oracle_variant"] = "x86 SSE4.2 crc32 instruction"
    return rec


def _cpu_threads():
    """Every CPU this process may use, capped by the cgroup quota (cpu_baseline's rule)."""
    affinity = len(os.sched_getaffinity(0))
    quota = _cpu_quota()
    return max(1, min(256, affinity, int(quota[0]) if quota else affinity))


def c5_parity(got, firsts, samples):
    """The c5_strong CRCs vs the oracle (rank 0, after timing): the first and
    last payload of every rank's share and `samples` random payloads of the
    global batch, regenerated from the splitmix stream on the host."""
    from oracle import oracle as O
    method, gcount, length, seed, _ = CONFIGS[C5]
    rng = np.random.default_rng(0xC5)
    idx = sorted(set(firsts) | set(int(i) for i in rng.integers(0, gcount, samples)))
    bad = [i for i in idx if int(got[i]) != int(O.splitmix_batch_fixed(method, seed, length, length, i, 1)[0])]
    if bad:
        return f"MISMATCH {len(bad)}/{len(idx)} sampled payloads (first {bad[:4]}) vs oracle"
    return f"bit-exact ({len(idx)} payloads: both ends of every share + {samples} random, vs oracle)"


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


def cpu_baseline(method, seed, length, offsets_host, got, budget_s, samples, segments=False, world=1, count0=None,
                 share_firsts=(), xdr=False):
    """The CPU leg (rank 0, after timing, at every N): the oracle (CPU
    restatement of mchecksum -- the reference's own mchecksum is absent, so
    kind = "port") timed on this host's cores over a bounded sample of the
    same workload (the first n payloads of the global batch), whose CRCs then
    check the gathered GPU values for those payloads; plus the first and last
    payload of every rank's share (share_firsts) and `samples` random payloads
    of the whole global batch.  `got`: the gathered CRCs in global order;
    offsets_host: the global offsets table (None for fixed layouts); segments:
    rank r's count0 objects come from seed ^ r (weak scaling); xdr: the
    messages of the xdr config, whose checksum covers the host-order length
    and the payload bytes (the oracle is timed over those hashed streams --
    the CRC work of an XDR build's mchecksum_update calls, not its XDR
    decoding -- and the rate is quoted in message bytes, like the GPU's)."""
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
    count0 = len(got) if count0 is None else count0
    if segments:
        from mercury_amd.workload import segment_slots
        slots = segment_slots(seed, count0 * SEGS_PER_OBJECT)
        rank_slots = {0: slots}
        n = min(256, count0)
        host = np.concatenate([_segment_object_bytes(O, seed, length, j, slots) for j in range(n)])
        runv = lambda k, v, th: O.batch_fixed(method, host, length, length, k, variant=v, nthreads=th)  # noqa: E731
        prod = lambda th: product_batch(method, host, th, count=n, length=length)  # noqa: E731
        sample_bytes = n * length
        what = f"the first {n} objects ({SEGS_PER_OBJECT} x {length // SEGS_PER_OBJECT} B segments, gathered)"
    elif xdr:
        import struct
        from mercury_amd.workload import varlen_lengths
        xlens = varlen_lengths(seed, len(offsets_host) - 1).astype(np.int64)
        n = min(int(np.searchsorted(offsets_host, np.uint64(256 << 20))), len(offsets_host) - 1)
        raw = O.splitmix_bytes(int(offsets_host[n]), seed)
        parts = []
        for i in range(n):
            o = int(offsets_host[i]) + 4
            parts += [np.frombuffer(struct.pack("<I", int(xlens[i])), dtype=np.uint8), raw[o:o + int(xlens[i])]]
        host = np.concatenate(parts)
        hoff = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(np.uint64(4) + xlens[:n].astype(np.uint64), out=hoff[1:])
        runv = lambda k, v, th: O.batch_offsets(method, host, hoff[:k + 1], variant=v, nthreads=th)  # noqa: E731
        prod = lambda th: product_batch(method, host, th, offsets=hoff)  # noqa: E731
        sample_bytes = int(offsets_host[n])
        what = (f"the first {n} messages ({sample_bytes} B): the hashed streams (host-order length + payload "
                f"bytes) an XDR build feeds mchecksum_update")

        def xdr_message(gi):  # the message's bytes as the device holds them, and its hashed stream
            lo, hi, ln = int(offsets_host[gi]), int(offsets_host[gi + 1]), int(xlens[gi])
            w0 = lo // 8
            b = O.splitmix_bytes(hi - w0 * 8, seed, first_word=w0)[lo - w0 * 8:]
            payload = b[4:4 + ln].tobytes()
            msg = struct.pack(">I", ln) + payload + bytes(hi - lo - 4 - ln)
            return msg, struct.pack("<I", ln) + payload
    elif offsets_host is None:
        n = min(4096 if length <= 65536 else 256, len(got))
        host = O.splitmix_bytes(n * length, seed)
        runv = lambda k, v, th: O.batch_fixed(method, host, length, length, k, variant=v, nthreads=th)  # noqa: E731
        prod = lambda th: product_batch(method, host, th, count=n, length=length)  # noqa: E731
        sample_bytes = n * length
        what = f"{n} x {length} B"
    else:
        n = min(int(np.searchsorted(offsets_host, np.uint64(256 << 20))), len(offsets_host) - 1)  # ~256 MiB
        host = O.splitmix_bytes(int(offsets_host[n]), seed)
        sub = np.ascontiguousarray(offsets_host[:n + 1])
        runv = lambda k, v, th: O.batch_offsets(method, host, sub[:k + 1], variant=v, nthreads=th)  # noqa: E731
        prod = lambda th: product_batch(method, host, th, offsets=sub)  # noqa: E731
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
    # ... and the PRODUCT's own CPU path on the same sample (libmchecksum's
    # streaming API, one object per thread: the AVX-512 VPCLMULQDQ fold for
    # updates >= 1 KiB; tools/cpu_batch.c), at full width and on one thread --
    # what the host can actually do, next to the oracle port above.  Its CRCs
    # must equal the oracle's.
    for th in (threads, 1):
        key = f"product_{th}thread{'s' if th > 1 else ''}"
        try:
            pv = prod(th)
        except OSError as e:  # build/libcpu_batch.so absent
            breakdown[key] = None
            base["product_note"] = f"product CPU path not timed: {e}"
            break
        if not np.array_equal(pv.astype(want.dtype), want):
            breakdown[key] = None
            base["product_note"] = "product CPU path disagrees with the oracle"
            break
        p2, t2 = 0, time.perf_counter()
        while True:
            prod(th)
            p2 += 1
            e2 = time.perf_counter() - t2
            if e2 >= budget_s / 3 or p2 >= 200:
                break
        breakdown[key] = round(p2 * sample_bytes / e2 / 2**30, 2)
    base["breakdown_GiB_s"] = breakdown
    base["cpu_model"] = _cpu_model()

    bad = int(np.count_nonzero(got[:n] != want))
    rng = np.random.default_rng(1234)
    total = len(got)
    idx = np.unique(np.concatenate([[total - 1], np.asarray(share_firsts, dtype=np.int64),
                                    rng.integers(n, total, samples)]).astype(np.int64)) if total > n else []
    idx = [int(i) for i in idx if int(i) >= n]
    for gi in idx:
        gi = int(gi)
        if xdr:
            w = O.crc(method, xdr_message(gi)[1])
        elif segments:
            r, j = divmod(gi, count0)
            if r not in rank_slots:
                rank_slots[r] = segment_slots(seed ^ r, count0 * SEGS_PER_OBJECT)
            w = O.crc(method, _segment_object_bytes(O, seed ^ r, length, j, rank_slots[r]))
        elif offsets_host is None:
            w = O.splitmix_batch_fixed(method, seed, length, length, gi, 1)[0]
        else:
            lo, hi = int(offsets_host[gi]), int(offsets_host[gi + 1])
            w0 = lo // 8
            b = O.splitmix_bytes(hi - w0 * 8, seed, first_word=w0)
            w = O.crc(method, b[lo - w0 * 8:])
        bad += int(got[gi] != w)
    if xdr:  # the oracle's XDR restatement (decode the wire bytes by the schema) on one message
        msg, stream = xdr_message(0)
        schema = [(O.XDR_INT, 4), (O.XDR_OPAQUE_LEN, 0)]
        bad += int(O.xdr_hashed_stream(schema, msg) != stream or O.crc(method, stream) != got[0])
    checked = n + len(idx)
    where = f" across all {world} shares" if world > 1 else ""
    parity = f"bit-exact ({checked} payloads{where} vs oracle)" if bad == 0 else f"MISMATCH {bad}/{checked}{where}"
    return base, parity


_CPU_BATCH = None


def product_batch(method, host, threads, count=None, length=None, offsets=None):
    """CRCs (u64) of the product's CPU streaming path over a host batch:
    fixed (count x length, packed) or an offsets table (build/libcpu_batch.so,
    tools/cpu_batch.c, on `threads` pthreads)."""
    import ctypes
    global _CPU_BATCH
    if _CPU_BATCH is None:
        L = ctypes.CDLL(os.path.join(ROOT, "build", "libcpu_batch.so"))
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.cpu_batch_fixed.argtypes = [ctypes.c_char_p, vp, sz, sz, sz, vp, ctypes.c_int]
        L.cpu_batch_offsets.argtypes = [ctypes.c_char_p, vp, vp, sz, vp, ctypes.c_int]
        _CPU_BATCH = L
    host = np.ascontiguousarray(host)
    if offsets is not None:
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        count = len(offsets) - 1
        out = np.zeros(count, dtype=np.uint64)
        rc = _CPU_BATCH.cpu_batch_offsets(method.encode(), host.ctypes.data, offsets.ctypes.data, count,
                                          out.ctypes.data, threads)
    else:
        out = np.zeros(count, dtype=np.uint64)
        rc = _CPU_BATCH.cpu_batch_fixed(method.encode(), host.ctypes.data, length, length, count, out.ctypes.data,
                                        threads)
    if rc != 0:
        raise RuntimeError(f"cpu_batch {method}: rc {rc}")
    return out


def xdr_offsets(seed, count):
    """Message offsets of the xdr config: message i = 4-byte length + C4's
    len_i payload bytes + zero pad to a multiple of 4 (xdr_opaque)."""
    from mercury_amd.workload import varlen_lengths
    lens = varlen_lengths(seed, count)
    off = np.zeros(count + 1, dtype=np.uint64)
    np.cumsum(np.uint64(4) + (lens + np.uint64(3)) // np.uint64(4) * np.uint64(4), out=off[1:])
    return off


def gather_shares(dist, crcs, counts, world, coll_dev):
    """all_gather of the per-rank CRC arrays, padded to the largest share
    (ranks may hold different counts), trimmed and concatenated in rank order
    -- shares are contiguous ranges of the global batch, so the result is in
    global payload order."""
    import torch
    rank = dist.get_rank()
    mine = torch.zeros(max(counts), dtype=crcs.dtype, device=coll_dev)
    mine[:counts[rank]] = crcs[:counts[rank]].to(coll_dev)
    gathered = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(gathered, mine)
    return torch.cat([g[:c] for g, c in zip(gathered, counts)])


def global_offsets(layout, seed, global_count, offsets_host):
    """The host offsets table of the WHOLE global batch, for the oracle check
    (None for fixed-size layouts): C4's packed layout regenerated from its seed;
    for messages the sender's interleaved (header, payload) pieces."""
    from mercury_amd.workload import varlen_offsets
    if layout == "offsets":
        return varlen_offsets(seed, global_count)
    if layout == "xdr":
        return xdr_offsets(seed, global_count)
    if layout == "messages":
        msg = varlen_offsets(seed, global_count)
        inter = np.empty(2 * global_count + 1, dtype=np.uint64)
        inter[0::2] = msg
        inter[1::2] = msg[:-1] + np.uint64(20)
        return inter
    return None


def share_firsts(plan, layout, world, count0):
    """Indices (into the gathered CRC array) of the first and last payload of
    every rank's share, so the oracle check touches every share."""
    if layout == "segments":  # weak: count0 objects per rank
        firsts, counts = [r * count0 for r in range(world)], [count0] * world
    elif plan is not None:
        firsts, counts = plan.firsts, plan.counts
    else:
        firsts, counts = [0], [count0]
    if layout == "messages":  # two pieces per message; the payload piece is the odd one
        firsts, counts = [2 * f for f in firsts], [2 * c for c in counts]
    idx = [f for f, c in zip(firsts, counts) if c] + [f + c - 1 for f, c in zip(firsts, counts) if c]
    return sorted(set(idx))


def pmc_traffic(config, world, alg_bytes):
    """roofline.traffic: HBM bytes per launch cannot be counted inside this
    process -- they come from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of this config (tools/gpu_pass.sh PART=pmc ->
    profiles/pmc_traffic_<config>.json).  At N > 1 the profile (one GPU, the
    whole batch) is scaled to rank 0's share by its traffic/algorithmic
    ratio.  (None, reason) when there is no profile."""
    rel = f"profiles/pmc_traffic_{config}.json"
    path = os.path.join(ROOT, rel)
    if not os.path.exists(path):
        return None, f"no committed PMC profile for {config} ({rel})"
    try:
        prof = json.load(open(path))
        if world == 1:
            return prof["hbm_bytes_per_launch"], (f"{rel} (rocprofv3 FETCH_SIZE + WRITE_SIZE passes of this config, "
                                                  "committed; not measured in this run)")
        ratio = float(prof["hbm_bytes_per_launch"]) / float(prof["algorithmic_bytes_per_launch"])
        return round(ratio * alg_bytes), (f"rank 0's share: its algorithmic bytes x {ratio:.5f}, the "
                                          f"traffic/algorithmic ratio of {rel} (one GPU, whole batch, rocprofv3 "
                                          "PMC passes, committed); not measured in this run")
    except (OSError, ValueError, KeyError, ZeroDivisionError) as e:
        return None, f"{rel} unreadable: {e}"


if __name__ == "__main__":
    main()
