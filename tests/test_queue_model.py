"""CPU model of the batch kernels' work-queue protocol (crc_gpu_device.h:
WgQueue, wg_fetch, wg_publish, for_each_unit), run under random interleavings
of every wave's shared-memory steps.  Checks what the GPU relies on: every
unit is processed exactly once, no wait can block forever, and every launch
leaves the bank the slot's next launch counts in at zero (two banks per slot,
round 3: launch s counts in bank s & 1 and its first workgroup zeroes the
other).  The host learns that a slot's launch is done with the slot from the
HIP event its completion records (round 4), so the next launch on a slot
starts after every wave of the previous one has ended.  Bounded waits are
modelled in poll counts: a wait still unmet after `deadline` polls gives up
and raises the launch's abort flag (round 6), and every other wait of the
launch then gives up at its next clock read -- so a launch with a stall spends
one deadline, not one per wait.

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
        self.abort = 0                 # a wait of the launch gave up

    def clean(self):
        return self.sub == [0] * QSUB and self.fault == 0 and self.abort == 0


class Slot:
    def __init__(self):
        self.banks = [Bank(), Bank()]
        self.issued = 0       # launches handed this slot (host: SlotState::seq)
        self.active = False   # a launch on the slot has waves left (its completion event not yet recorded)

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


def run_launches(launches, seed, slot=None, max_steps=4_000_000, deadline=20_000):
    """Several launches, their waves interleaved at random.  At most one uses the
    slot at a time: a slot launch (no_slot absent) is issued only once every
    wave of the previous one has ended (its completion event); launches with
    no_slot=True take the static split beside it.  drop=(wg, seq): that
    workgroup's wave taking slot 0 of chunk `seq` gives up (MCK_QFAULT_TEST
    give-up).  stall=(wg, seq): that workgroup never publishes chunk seq + 1,
    so the waves that take its slots wait out the deadline (MCK_QFAULT_TEST
    "stall")."""
    rnd = random.Random(seed)
    slot = slot or Slot()
    clock = [0]
    results = []
    pending = list(launches)
    live = []  # [generators, result, uses_slot]

    def issue(spec):
        r = dict(units=[], slot=slot, faulted_waves=0, first_faults=0, busy_wgs=0, gave_up_at=[], ended_at=0)
        results.append(r)
        bank = None
        if not spec.get("no_slot"):  # queue_slot: bank issued & 1, then count the launch
            assert not slot.active, "slot handed out while a launch still holds it"
            bank = (slot.banks[slot.issued & 1], slot.banks[(slot.issued & 1) ^ 1])
            slot.issued += 1
            slot.active = True
        live.append([_launch(spec, bank, rnd, r, clock, deadline), r, bank is not None])

    while live or pending:
        while pending and (pending[0].get("no_slot") or not slot.active):
            issue(pending.pop(0))
        launch = rnd.choice(live)
        gens = launch[0]
        g = rnd.choice(gens)
        try:
            next(g)
        except StopIteration:
            gens.remove(g)
        clock[0] += 1
        assert clock[0] < max_steps, "no progress: a wait never ends"
        if not gens:
            live.remove(launch)
            launch[1]["ended_at"] = clock[0]
            if launch[2]:
                slot.active = False  # the completion event
    for r in results:
        r["units"].sort()
    return results


def _launch(spec, bank, rnd, res, clock, deadline):
    n, grid, waves_per_wg, drop, stall = spec["n"], spec["grid"], spec["wpw"], spec.get("drop"), spec.get("stall")
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

    def wait(cond):
        """A bounded wait (crc_gpu_device.h Deadline): True when cond() holds,
        False once it gave up -- after `deadline` polls, or at the next poll
        once the launch's abort flag is up (every 16th poll reads it)."""
        polls = 0
        while not cond():
            polls += 1
            if polls >= deadline or (polls % 16 == 1 and cur.abort):
                cur.abort = 1  # raise_abort
                res["gave_up_at"].append(clock[0])
                return False
            yield
        return True

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

    def publish(L, seq, cid):  # wg_publish; False when its wait gave up
        r = seq % RING
        ok = True
        if seq >= RING:
            ok = yield from wait(lambda: L.reads[r] == cu)
        L.reads[r] = 0
        yield
        L.entry[r] = (seq, cid)
        yield
        return ok

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
            if (yield from wait(lambda: L.entry[r][0] == seq)):
                e = L.entry[r]
            else:
                e = (seq, NOCH)
                flt = True
            L.reads[r] += 1
            yield
            if (t & (cu - 1)) == cu - lead:
                stalled = stall is not None and (b, seq) == stall
                nid = NOCH if e[1] == NOCH or stalled else (yield from fetch(L, b))
                if not stalled and not (yield from publish(L, seq + 1, nid)):
                    flt = True
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


@pytest.mark.parametrize("seed", range(8))
def test_next_slot_launch_after_completion(seed):
    """Slot launches back to back (each issued at its predecessor's completion
    event), one with a give-up, beside a slot-less launch: every launch hashes
    each unit exactly once (the give-up's one unit aside) and the slot is clean
    after each."""
    specs = [dict(n=900, grid=6, wpw=4), dict(n=500, grid=3, wpw=4, no_slot=True), dict(n=700, grid=5, wpw=4),
             dict(n=1300, grid=9, wpw=2, drop=(1, 1)), dict(n=40, grid=3, wpw=4)]
    res = run_launches(specs, seed * 7 + 3)
    assert [r["units"] for r in res[:3]] == [list(range(900)), list(range(500)), list(range(700))]
    assert len(res[3]["units"]) == 1299 and res[3]["first_faults"] == 1
    assert res[4]["units"] == list(range(40))
    assert res[0]["slot"].issued == 4 and res[0]["slot"].clean()


@pytest.mark.parametrize("n,grid,wpw,stall", [(2000, 4, 4, (1, 0)), (5000, 8, 4, (3, 1)), (3000, 3, 16, (0, 2))])
def test_stall_costs_one_deadline(n, grid, wpw, stall):
    """A workgroup that never publishes a chunk (MCK_QFAULT_TEST "stall"): its
    waves that take that chunk's slots wait out ONE deadline, the first give-up
    raises the abort flag, and every other wait of the launch then gives up at
    its next clock read -- the launch ends well within two deadlines, one wave
    claims the fault, no unit is hashed twice, and the slot is clean after."""
    deadline = 20_000
    r = run_launches([dict(n=n, grid=grid, wpw=wpw, stall=stall)], n + grid, deadline=deadline)[0]
    assert r["first_faults"] == 1 and r["faulted_waves"] >= 1
    assert len(r["units"]) == len(set(r["units"])) and set(r["units"]) <= set(range(n))
    assert r["gave_up_at"], "the stalled wait never gave up"
    first = min(r["gave_up_at"])
    # after the first give-up, every other waiting wave gives up within a few
    # polls of its next clock read (16 polls), not after its own deadline
    assert max(r["gave_up_at"]) - first < deadline // 2
    assert r["ended_at"] - first < deadline // 2
    assert r["slot"].banks[0].fault == 1 and r["slot"].banks[0].abort == 1  # zeroed by the slot's next launch
    assert r["slot"].clean()
    nxt = run_launches([dict(n=300, grid=2, wpw=4)], 5, r["slot"])[0]
    assert nxt["units"] == list(range(300)) and nxt["first_faults"] == 0


# ---- split CRC-64 pieces, pipelined (round 6) -------------------------------
# crc64_batch_kernel<..., SPLIT>: unit u = piece (u % 2^psl) of payload
# u >> psl.  A wave takes its NEXT piece (slot, ring entry, read counted at
# once) as soon as its current piece's step loop ends, then combines the
# current one and accumulates it into the workgroup's LDS entry
# (seq % NA, payload % 16), owned by the chunk (tag seq + 1) until its last
# piece stores the CRC.  Checked here under random interleavings: every
# payload's pieces are all accumulated and its CRC stored exactly once, no
# wait blocks forever, and no entry is ever claimed by a newer chunk while an
# older one holds it (the device turns that into a fault).
NA, ACC = 32, 16


def _split_model(count, psl, grid, wpw, seed, max_steps=6_000_000, deadline=200_000):
    n = count << psl
    pieces = 1 << psl
    rnd = random.Random(seed)
    cl = chunk_log2(n, grid)
    cu, lead = 1 << cl, (1 << cl) // 4 if (1 << cl) > 4 else 1
    sl = cl - 3 if cl >= 3 else cl
    assert (1 << psl) <= (1 << sl) and (1 << cl) // (1 << psl) <= ACC, "not a whole-payload plan"
    tail = grid << cl
    nbig = (n - tail) >> cl if n > tail else 0
    big_end = nbig << cl
    nch = nbig + ((n - big_end + (1 << sl) - 1) >> sl)

    def start(cid):
        return cid << cl if cid < nbig else big_end + ((cid - nbig) << sl)

    def size(cid):
        return 1 << cl if cid < nbig else 1 << sl
    bank = Bank()
    lds = [Lds() for _ in range(grid)]
    acc = [[dict(tag=0, cnt=0) for _ in range(NA * ACC)] for _ in range(grid)]
    stored = [0] * count
    got = [0] * count
    res = dict(faults=0, newer=0)

    def wait(cond):
        polls = 0
        while not cond():
            polls += 1
            if polls >= deadline:
                res["faults"] += 1
                return False
            yield
        return True

    def fetch(L, b):
        home = b % QSUB
        d = L.drained
        while d < QSUB:
            k = home if d == 0 else (home + 1 + (d - 1 + (b // QSUB) % (QSUB - 1)) % (QSUB - 1)) % QSUB
            t = bank.sub[k]
            bank.sub[k] += 1
            yield
            if k + t * QSUB < nch:
                return k + t * QSUB
            L.drained = max(L.drained, d + 1)
            yield
            d = max(L.drained, d + 1)
        return NOCH

    def publish(L, seq, cid):
        r = seq % RING
        if seq >= RING:
            yield from wait(lambda: L.reads[r] == cu)
        L.reads[r] = 0
        yield
        L.entry[r] = (seq, cid)
        yield

    def take(L, b):  # UnitTaker::take_unit: (unit, seq) or None
        while True:
            t = L.slot
            L.slot += 1
            yield
            seq, r = t >> cl, (t >> cl) % RING
            if not (yield from wait(lambda: L.entry[r][0] == seq)):
                return None
            e = L.entry[r]
            L.reads[r] += 1  # counted at once: no deferred reader
            yield
            if (t & (cu - 1)) == cu - lead:
                nid = NOCH if e[1] == NOCH else (yield from fetch(L, b))
                yield from publish(L, seq + 1, nid)
            if e[1] == NOCH:
                return None
            k = t & (cu - 1)
            if k < size(e[1]):
                return start(e[1]) + k, seq

    def accumulate(b, u, seq):
        p = u >> psl
        ent = acc[b][(seq % NA) * ACC + (p % ACC)]
        me = seq + 1
        while True:
            tg = ent["tag"]
            if tg == me:
                break
            if tg == 0:  # CAS 0 -> me
                ent["tag"] = me
                yield
                break
            if tg > me:
                res["newer"] += 1
                return
            if not (yield from wait(lambda: ent["tag"] in (0, me))):
                return
        got[p] += 1
        ent["cnt"] += 1
        yield
        if ent["cnt"] == pieces:
            stored[p] += 1
            ent["cnt"] = 0
            yield
            ent["tag"] = 0
            yield

    def wave(b, w):
        L = lds[b]
        while not L.ready:
            yield
        cur = yield from take(L, b)
        while cur is not None:
            for _ in range(rnd.randint(0, 60)):  # the piece's step loop
                yield
            nxt = yield from take(L, b)  # the next piece's loads go out here
            for _ in range(rnd.randint(0, 6)):  # combine + shift
                yield
            yield from accumulate(b, *cur)
            cur = nxt

    def init(b):
        L = lds[b]
        yield from publish(L, 0, (yield from fetch(L, b)))
        yield
        L.ready = True

    gens = [init(b) for b in range(grid)] + [wave(b, w) for b in range(grid) for w in range(wpw)]
    steps = 0
    while gens:
        g = rnd.choice(gens)
        try:
            next(g)
        except StopIteration:
            gens.remove(g)
        steps += 1
        assert steps < max_steps, "no progress"
    return stored, got, res


@pytest.mark.parametrize("count,psl,grid,wpw", [(64, 2, 2, 4), (200, 2, 3, 8), (8192 // 16, 2, 4, 16),
                                                (300, 1, 4, 4), (128, 2, 1, 16), (40, 2, 1, 4)])
def test_split_pipelined_pieces_combine_exactly_once(count, psl, grid, wpw):
    for seed in range(3):
        stored, got, res = _split_model(count, psl, grid, wpw, seed * 131 + count)
        assert res == dict(faults=0, newer=0), res
        assert got == [1 << psl] * count, "a payload missed or doubled a piece"
        assert stored == [1] * count, "a payload's CRC not stored exactly once"
