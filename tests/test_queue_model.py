"""CPU model of the batch kernels' work-queue protocol (crc_gpu_device.h:
WgQueue, wg_fetch, wg_publish, for_each_unit), run under random interleavings
of every wave's shared-memory steps.  Checks what the GPU relies on: every
unit is processed exactly once, no wait can block forever, and every launch
leaves the bank the slot's next launch counts in at zero (two banks per slot,
round 3: launch s counts in bank s & 1 and its first workgroup zeroes the
other).  The host learns that a slot's launch is done with the slot from the
HIP event its completion records (round 4) or, in MCK_SLOT_DONE=1 builds
(crc_gpu_device.h "Completion without an event"), from the slot's completion
word -- modelled here, as the stricter of the two: every wave counts itself
out of its workgroup, the workgroup's last wave counts the workgroup out of its
sub-queue group, the group's last out of the launch, and the launch's last
workgroup bumps the slot's launch count and stores it to host-mapped memory
(crc_gpu_device.h slot_exit).  The model checks that the word is stored once
per launch, after the launch's last access to the slot, and that a launch
handed the slot at that moment -- while the previous one's waves still run --
is exact.

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
        self.zero()

    def zero(self):  # wg_queue_init, workgroup 0: the protocol lines only
        self.sub = [0] * QSUB          # sub-queue tickets
        self.fault = 0                 # first faulting wave of the launch
        self.exit_group = [0] * QSUB   # workgroups counted out, per sub-queue group
        self.exit_top = 0              # groups counted out

    def clean(self):
        return self.sub == [0] * QSUB and self.fault == 0 and self.exit_group == [0] * QSUB and self.exit_top == 0


class Slot:
    def __init__(self):
        self.banks = [Bank(), Bank()]
        self.issued = 0       # launches handed this slot (host: SlotState::seq)
        self.launches = 0     # device: the slot's completed-launch line (kQLaunchLine)
        self.done = 0         # host-mapped completion word (DevCtx::slot_done)

    def clean(self):
        """Ready for the next launch (the previous one has completed): the bank
        it will count in is zeroed."""
        return self.banks[self.issued & 1].clean()


class Lds:
    def __init__(self):
        self.exits = 0
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
    slot at a time (the host hands a slot to a launch only once the previous
    launch's completion word says it is done with it); the others have none
    (no_slot=True).  after_done=True: the launch is issued on the slot at the
    moment the previous slot launch stores its completion word -- the host's
    reap -- while that launch's waves may still run.  drop=(wg, seq): that
    workgroup's wave taking slot 0 of chunk `seq` gives up (MCK_QFAULT_TEST)."""
    rnd = random.Random(seed)
    slot = slot or Slot()
    clock = [0]
    gens = []
    results = []
    pending = []

    def issue(spec):
        r = dict(units=[], slot=slot, faulted_waves=0, first_faults=0, busy_wgs=0, last_access=-1, done_at=[])
        results.append(r)
        bank = None
        if not spec.get("no_slot"):  # queue_slot: bank issued & 1, then count the launch
            assert slot.done == slot.issued, "slot handed out while a launch still holds it"
            bank = (slot.banks[slot.issued & 1], slot.banks[(slot.issued & 1) ^ 1])
            slot.issued += 1
        gens.extend(_launch(spec, bank, rnd, r, slot, clock))

    for spec in launches:
        if spec.get("after_done"):
            pending.append(spec)
        else:
            issue(spec)
    while gens or pending:
        if pending and slot.done == slot.issued:
            issue(pending.pop(0))
            continue
        assert gens, "a launch never stored its completion word"
        g = rnd.choice(gens)
        try:
            next(g)
        except StopIteration:
            gens.remove(g)
        clock[0] += 1
        assert clock[0] < max_steps, "no progress: a wait never ends"
    for r in results:
        r["units"].sort()
    return results


def _launch(spec, bank, rnd, res, slot, clock):
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

    def touch():  # an access to the slot's lines
        res["last_access"] = clock[0]

    def fetch(L, b):  # wg_fetch
        home = b % QSUB
        d = L.drained
        while d < QSUB:
            # crc_gpu_device.h MCK_STEAL_ROT: a workgroup's victims after its
            # home are the other seven rotated by (b / QSUB) % 7
            k = home if d == 0 else (home + 1 + (d - 1 + (b // QSUB) % (QSUB - 1)) % (QSUB - 1)) % QSUB
            t = cur.sub[k]
            cur.sub[k] += 1
            touch()
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
            touch()
            yield
            res["first_faults"] += first
        # slot_exit: this wave, its workgroup, its group, the launch
        L.exits += 1
        last_wave = L.exits == waves_per_wg
        yield
        if not last_wave:
            return
        g = b % QSUB
        in_group, groups = (grid - g + QSUB - 1) // QSUB, min(grid, QSUB)
        old = cur.exit_group[g]
        cur.exit_group[g] += 1
        touch()
        yield
        if old != in_group - 1:
            return
        old = cur.exit_top
        cur.exit_top += 1
        touch()
        yield
        if old != groups - 1:
            return
        slot.launches += 1
        n_done = slot.launches
        touch()
        yield
        slot.done = n_done  # the host-mapped word
        res["done_at"].append(clock[0])
        for _ in range(rnd.randint(0, 20)):  # the launch's last waves may still run
            yield

    def init(b):  # wg_queue_init (thread 0 of the workgroup, before the barrier)
        L = lds[b]
        L.busy = bool(spec.get("no_slot"))
        if L.busy:
            res["busy_wgs"] += 1
        else:
            if b == 0:
                other.zero()  # the slot's next launch counts there
                touch()
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


@pytest.mark.parametrize("n,grid,wpw", [(1, 1, 1), (67, 5, 4), (1000, 9, 4), (5000, 8, 16), (20000, 12, 4),
                                        (3000, 17, 2)])
def test_completion_word_after_the_last_slot_access(n, grid, wpw):
    """The launch's last workgroup stores the slot's launch count once, after
    every access of the launch to the slot's lines (sub-queue tickets, the
    fault flag, the exit counters, the next bank's zeroing)."""
    slot = Slot()
    for seed in range(3):
        r = run_launches([dict(n=n, grid=grid, wpw=wpw)], seed * 104729 + n, slot)[0]
        assert r["units"] == list(range(n))
        assert len(r["done_at"]) == 1 and r["done_at"][0] > r["last_access"]
        assert slot.done == slot.issued == seed + 1


@pytest.mark.parametrize("seed", range(12))
def test_next_launch_takes_the_slot_at_the_completion_word(seed):
    """The host reaps the slot the moment the word is stored and hands it to the
    next launch, whose waves then run beside the previous launch's last ones:
    both hash every unit exactly once, and each stores its word once."""
    specs = [dict(n=900, grid=6, wpw=4), dict(n=700, grid=5, wpw=4, after_done=True),
             dict(n=1300, grid=9, wpw=2, after_done=True, drop=(1, 1)), dict(n=40, grid=3, wpw=4, after_done=True)]
    res = run_launches(specs, seed * 7 + 3)
    assert [r["units"] for r in res[:2]] == [list(range(900)), list(range(700))]
    assert len(res[2]["units"]) == 1299 and res[2]["first_faults"] == 1
    assert res[3]["units"] == list(range(40))
    assert all(len(r["done_at"]) == 1 for r in res)
    assert res[0]["slot"].done == res[0]["slot"].issued == 4
