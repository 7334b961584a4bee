"""N > 1 path on the CPU: world_size 2 over gloo.  Each rank checksums its own
shard (through the drop-in library's streaming API, standing in for the GPU
kernel on a CPU-only box), the CRC arrays are all_gathered as bench.py does
with RCCL, and rank 0 checks the gathered batch against the oracle."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, length, seed, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    from mercury_amd import checksum
    from mercury_amd.shard import fixed_shard
    from oracle import oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = fixed_shard(rank, world, total)
    # this rank's bytes: words starting at first*length/8 of the global stream
    host = O.splitmix_bytes(n * length, seed, first_word=first * length // 8)
    mine = torch.tensor([checksum("crc32c", host[i * length:(i + 1) * length].tobytes()) for i in range(n)],
                        dtype=torch.int64)
    sizes = [fixed_shard(r, world, total)[1] for r in range(world)]
    gathered = [torch.zeros(s, dtype=torch.int64) for s in sizes]
    dist.all_gather(gathered, mine) if len(set(sizes)) == 1 else [
        dist.broadcast(gathered[r], src=r) if r != rank else dist.broadcast(mine, src=r) for r in range(world)]
    if len(set(sizes)) != 1:
        gathered[rank] = mine
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        full = torch.cat(gathered).numpy().astype(np.uint64)
        want = O.splitmix_batch_fixed("crc32c", seed, length, length, 0, total)
        q.put((bool(np.array_equal(full, want)), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [64, 63])
def test_two_rank_shard_and_gather(total):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, 4096, 0x4D43310000000005, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    ok, tmax = q.get()
    assert ok and tmax == 2.0


def test_fixed_shard_partition():
    from mercury_amd.shard import fixed_shard
    for total in (0, 1, 7, 65536, 1048576):
        for world in (1, 2, 3, 8):
            spans = [fixed_shard(r, world, total) for r in range(world)]
            assert sum(n for _, n in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))


def test_byte_balanced_cuts(oracle_mod):
    from mercury_amd.shard import byte_balanced_cuts
    off = oracle_mod.varlen_offsets(0x4D43310000000004, 262144)
    for world in (1, 2, 4, 8):
        cuts = byte_balanced_cuts(off, world)
        assert cuts[0] == 0 and cuts[-1] == 262144 and np.all(np.diff(cuts) >= 0)
        b = np.array([int(off[cuts[r + 1]] - off[cuts[r]]) for r in range(world)])
        assert b.max() - b.min() <= 2 * 65536  # equal bytes up to one payload per cut
