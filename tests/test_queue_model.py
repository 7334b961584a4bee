"""CPU model of the batch kernels' work-queue protocol (crc_gpu_device.h:
WgQueue, wg_fetch, wg_publish, for_each_unit), run under random interleavings
of every wave's shared-memory steps.  Checks what the GPU relies on: every
unit is processed exactly once, no wait can block forever, and every launch
leaves the bank the slot's next launch counts in at zero (two banks per slot,
round 3: launch s counts in bank s & 1 and its first workgroup zeroes the
other).  The host learns that a slot's launch has completed from the HIP event
its completion records (round 4; queue_slot in mchecksum_gpu.hip) -- here, from
every wave of the launch having returned.

Each wave is a generator that yields at every access to shared state (LDS or
the global slot), so a seeded scheduler explores many orders of the same
steps the device code takes.  A launch without a slot (graph captures, the
per-thread stream, streams past the table: crc_gpu_device.h "Exclusivity")
takes the static split and never touches any slot; the fail-closed fault flag
is modelled too.  Fetch triggers, chunk sizes (chunk_log2, the
eighth-size tail chunks of ChunkPlan), the
round-robin sub-queues, the LDS ring recycling and the bank zeroing mirror the
device code one to one.
"""
import random

import pytest

QSUB, RING, NOCH = 8, 8, 0xFFFFFFFF


def chunk_log2(n, grid, max_log2=5):
    share = n // (4 * grid)
    lg = 0
    while lg < max_log2 and (2 << lg) <= share:
        lg += 1
    return lg


class Bank:
    def __init__(self):
        self.sub = [0] * QSUB          # sub-queue tickets
        self.fault = 0                 # first faulting wave of the launch

    def zero(self):  # wg_queue_init, workgroup 0: the protocol lines only
        self.sub = [0] * QSUB
        self.fault = 0

    def clean(self):
        return self.sub == [0] * QSUB and self.fault == 0


class Slot:
    def __init__(self):
        self.banks = [Bank(), Bank()]
        self.issued = 0       # launches handed this slot (host: SlotState::seq)

    def clean(self):
        """Ready for the next launch (the previous one has completed): the bank
        it will count in is zeroed."""
        return self.banks[self.issued & 1].clean()


class Lds:
    def __init__(self):
        self.slot = 0
        self.drained = 0
        self.reads = [0] * RING
        self.entry = [(0xFFFFFFFF, 0)] * RING
        self.busy = False
        self.ready = False  # wg_queue_init done (the kernel's barrier)


def run_model(n, grid, waves_per_wg, seed, slot=None, max_steps=2_000_000, drop=None):
    """One launch; returns (sorted processed units, slot)."""
    res = run_launches([dict(n=n, grid=grid, wpw=waves_per_wg, drop=drop)], seed, slot, max_steps)
    return res[0]["units"], res[0]["slot"]


def run_launches(launches, seed, slot=None, max_steps=4_000_000):
    """Several launches, their waves interleaved at random: at most one uses the
    slot (the host never hands one slot to two launches that can overlap); the
    others have none (no_slot=True).  drop=(wg, seq): that workgroup's wave
    taking slot 0 of chunk `seq` gives up (MCK_QFAULT_TEST)."""
    assert sum(not spec.get("no_slot") for spec in launches) <= 1
    rnd = random.Random(seed)
    slot = slot or Slot()
    gens = []
    results = []
    for spec in launches:
        r = dict(units=[], slot=slot, faulted_waves=0, first_faults=0, busy_wgs=0)
        results.append(r)
        bank = None
        if not spec.get("no_slot"):  # queue_slot: bank issued & 1, then count the launch
            bank = (slot.banks[slot.issued & 1], slot.banks[(slot.issued & 1) ^ 1])
            slot.issued += 1
        gens += _launch(spec, bank, rnd, r)
    steps = 0
    while gens:
        g = rnd.choice(gens)
        try:
            next(g)
        except StopIteration:
            gens.remove(g)
        steps += 1
        assert steps < max_steps, "no progress: a wait never ends"
    for r in results:
        r["units"].sort()
    return results


def _launch(spec, bank, rnd, res):
    n, grid, waves_per_wg, drop = spec["n"], spec["grid"], spec["wpw"], spec.get("drop")
    cl = chunk_log2(n, grid)
    cu, lead = 1 << cl, max(1, (1 << cl) // 4) if (1 << cl) > 4 else 1
    # ChunkPlan: full chunks, then about one full chunk per workgroup of units
    # in eighth chunks (MCK_QTAIL_SHIFT = 3)
    sl = cl - 3 if cl >= 3 else cl
    tail = grid << cl
    nbig = (n - tail) >> cl if n > tail else 0
    big_end = nbig << cl
    nch = nbig + ((n - big_end + (1 << sl) - 1) >> sl)

    def start(cid):
        return cid << cl if cid < nbig else big_end + ((cid - nbig) << sl)

    def size(cid):
        return 1 << cl if cid < nbig else 1 << sl
    done_units = res["units"]
    lds = [Lds() for _ in range(grid)]
    cur, other = bank if bank else (None, None)

    def fetch(L, b):  # wg_fetch
        home = b % QSUB
        d = L.drained
        while d < QSUB:
            # crc_gpu_device.h MCK_STEAL_ROT: a workgroup's victims after its
            # home are the other seven rotated by (b / QSUB) % 7
            k = home if d == 0 else (home + 1 + (d - 1 + (b // QSUB) % (QSUB - 1)) % (QSUB - 1)) % QSUB
            t = cur.sub[k]
            cur.sub[k] += 1
            yield
            if k + t * QSUB < nch:
                return k + t * QSUB
            L.drained = max(L.drained, d + 1)
            yield
            d = max(L.drained, d + 1)
        return NOCH

    def publish(L, seq, cid):  # wg_publish
        r = seq % RING
        if seq >= RING:
            while L.reads[r] != cu:
                yield
        L.reads[r] = 0
        yield
        L.entry[r] = (seq, cid)
        yield

    def wave(b, w):  # for_each_unit<true>
        L = lds[b]
        while not L.ready:  # the kernel's first barrier
            yield
        if L.busy:  # no slot: static split
            nw = grid * waves_per_wg
            u = b * waves_per_wg + w
            while u < n:
                done_units.append(u)
                u += nw
                yield
            return
        flt = False
        while True:
            t = L.slot
            L.slot += 1
            yield
            seq, r = t >> cl, (t >> cl) % RING
            while L.entry[r][0] != seq:
                yield
            e = L.entry[r]
            L.reads[r] += 1
            yield
            if (t & (cu - 1)) == cu - lead:
                nid = NOCH if e[1] == NOCH else (yield from fetch(L, b))
                yield from publish(L, seq + 1, nid)
            if drop is not None and (b, seq) == drop and (t & (cu - 1)) == 0:
                flt = True  # injected give-up: this unit is never hashed
                e = (seq, NOCH)
            if e[1] == NOCH:
                break
            k = t & (cu - 1)
            u = start(e[1]) + k if k < size(e[1]) else n
            if u < n:
                done_units.append(u)
                for _ in range(rnd.randint(0, 40)):
                    yield
        if flt:
            res["faulted_waves"] += 1
            first = cur.fault == 0  # atomicCAS(fault, 0, 1)
            cur.fault = 1
            yield
            res["first_faults"] += first

    def init(b):  # wg_queue_init (thread 0 of the workgroup, before the barrier)
        L = lds[b]
        L.busy = bool(spec.get("no_slot"))
        if L.busy:
            res["busy_wgs"] += 1
        else:
            if b == 0:
                other.zero()  # the slot's next launch counts there
                yield
            yield from publish(L, 0, (yield from fetch(L, b)))
        yield
        L.ready = True

    return [init(b) for b in range(grid)] + [wave(b, w) for b in range(grid) for w in range(waves_per_wg)]


@pytest.mark.parametrize("n,grid", [(1, 1), (2, 3), (17, 1), (67, 2), (67, 5), (100, 3), (257, 8), (1000, 9),
                                    (4096, 1), (4096, 16), (20000, 8)])
def test_every_unit_once_and_slot_reset(n, grid):
    slot = Slot()
    for seed in range(3):
        units, slot = run_model(n, grid, 4, seed * 7919 + n, slot)  # reused by the next launch
        assert units == list(range(n))
        assert slot.clean()


def test_chunk_size_rule():
    # C4 (262144 units, 256 workgroups): 32-unit chunks; C3-sized fixed batch at
    # 512 workgroups: 4; a small batch: single units
    assert 1 << chunk_log2(262144, 256) == 32
    assert 1 << chunk_log2(8192, 512) == 4
    assert 1 << chunk_log2(100, 256) == 1


@pytest.mark.parametrize("n,grid", [(67, 2), (5000, 4), (262144 // 64, 8)])
def test_sixteen_waves_per_workgroup(n, grid):
    units, slot = run_model(n, grid, 16, n + grid)
    assert units == list(range(n))
    assert slot.clean()


@pytest.mark.parametrize("seed", range(16))
def test_slotless_launch_beside_a_queue_launch(seed):
    """A launch without a slot (e.g. a graph replay) runs at the same time as a
    queue launch on the slot: each hashes every unit exactly once (the
    XOR-accumulating kernels need exactly once), and the slot is clean for the
    stream's next launch."""
    a = dict(n=700, grid=4, wpw=4)
    b = dict(n=500, grid=3, wpw=4, no_slot=True)
    ra, rb = run_launches([a, b], seed * 31 + 7)
    assert ra["units"] == list(range(700)) and rb["units"] == list(range(500))
    assert rb["busy_wgs"] == 3 and ra["busy_wgs"] == 0
    assert ra["slot"].clean()


@pytest.mark.parametrize("n,grid,drop", [(2000, 4, (1, 1)), (5000, 8, (3, 1)), (300, 2, (0, 2))])
def test_injected_give_up_is_reported_once(n, grid, drop):
    """MCK_QFAULT_TEST: the dropped unit is the only one not hashed, exactly one
    wave claims the launch's fault flag (it runs fail_closed), and the slot is
    clean for the next launch."""
    r = run_launches([dict(n=n, grid=grid, wpw=4, drop=drop)], n + grid)[0]
    assert r["faulted_waves"] == 1 and r["first_faults"] == 1
    missing = set(range(n)) - set(r["units"])
    assert len(missing) == 1 and len(r["units"]) == n - 1
    assert r["slot"].clean()


def test_fault_flag_is_cleared_before_its_bank_is_reused():
    """A launch that faults leaves its bank's fault flag set; the slot's next
    launch (other bank) zeroes it, so the launch after that -- back on the
    faulted bank -- starts clean and claims no fault it did not have."""
    slot = Slot()
    r = run_launches([dict(n=900, grid=4, wpw=4, drop=(2, 1))], 11, slot)[0]
    assert r["first_faults"] == 1 and slot.banks[0].fault == 1
    for seed in (12, 13, 14):
        r = run_launches([dict(n=900, grid=4, wpw=4)], seed, slot)[0]
        assert r["units"] == list(range(900)) and r["first_faults"] == 0
        assert slot.clean()
    assert slot.banks[0].fault == 0 and slot.issued == 4
