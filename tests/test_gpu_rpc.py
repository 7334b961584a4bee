"""Mercury-shaped end-to-end check of the batched verify path.

Sender side, as hg_set_struct does it (src/mercury.c:597-791): serialize the
proc fields -- here hg_perf_proc_iovec's layout, u32 length then the raw bytes
(Testing/perf/hg/mercury_perf.c:897-923) -- streaming each field through the
drop-in mchecksum API (src/mercury_proc.h:124-181), finalize, and store the
CRC network-order in the 4-byte HG header (src/mercury_header.c:111-112)
behind the 16-byte core header.  Messages are packed back to back as in an NA
multi-recv buffer (src/mercury_core.c:4667-4714).  Receiver side: one
mchecksum_gpu_verify_messages call instead of per-handle decode + verify
(src/mercury.c:565-573); it must flag exactly the corrupted messages.
"""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CORE_HDR, HG_HDR = 16, 4


def _encode_message(rng, payload_len):
    from mercury_amd import Checksum
    raw = rng.integers(0, 256, size=payload_len, dtype=np.uint8).tobytes()
    ck = Checksum("crc32c")
    body = b""
    for field in (struct.pack("<I", payload_len), raw):  # hg_proc_uint32_t, hg_proc_raw
        body += field
        ck.update(field)
    crc = ck.get()
    core = rng.integers(0, 256, size=CORE_HDR, dtype=np.uint8).tobytes()
    return core + struct.pack(">I", crc) + body, crc


def _batch(rng, n):
    msgs, crcs = [], []
    for i in range(n):
        ln = int(rng.integers(0, 9000)) if i % 7 else int(rng.integers(0, 70000))
        m, c = _encode_message(rng, ln)
        msgs.append(m)
        crcs.append(c)
    off = np.zeros(n + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(m) for m in msgs])
    return b"".join(msgs), off, crcs


@pytest.mark.parametrize("light", ["0", "1"])
def test_verify_messages_in_place(gpu, oracle_mod, light, monkeypatch):
    monkeypatch.setenv("MCHECKSUM_GPU_LIGHT", light)
    import torch
    rng = np.random.default_rng(2024)
    buf, off, crcs = _batch(rng, 700)
    host = np.frombuffer(buf, dtype=np.uint8).copy()
    t = torch.zeros(host.size + 64, dtype=torch.uint8, device="cuda")
    t[:host.size].copy_(torch.from_numpy(host))
    offs = torch.from_numpy(off.astype(np.int64)).cuda()

    status, mism = gpu.verify_messages(t, offs, offsets_host=off)
    assert int(mism.item()) == 0 and int(status.sum().item()) == 0

    # the sender-side (per-field streaming) hash equals the whole-payload CRC
    pay = [(int(off[i]) + CORE_HDR + HG_HDR, int(off[i + 1])) for i in range(len(off) - 1)]
    for i in (0, 1, 350, 699):
        assert oracle_mod.crc("crc32c", host[pay[i][0]:pay[i][1]]) == crcs[i]

    # faults: flipped payload bit, flipped header-hash bit, flipped core-header
    # bit (not covered by the payload CRC), truncated message
    t2 = t.clone()
    t2[pay[10][0] + 3] ^= 0x01
    t2[int(off[20]) + CORE_HDR + 1] ^= 0x80
    t2[int(off[30]) + 2] ^= 0x04          # core header only: payload check passes
    status, mism = gpu.verify_messages(t2, offs, offsets_host=off)
    bad = sorted(np.nonzero(status.cpu().numpy())[0].tolist())
    assert bad == [10, 20] and int(mism.item()) == 2

    trunc = np.array([0, 10, 10 + int(off[1])], dtype=np.uint64)  # a 10-byte "message" then message 0 moved
    t3 = torch.zeros(int(trunc[-1]) + 64, dtype=torch.uint8, device="cuda")
    t3[10:int(trunc[-1])].copy_(t[:int(off[1])])
    status, mism = gpu.verify_messages(t3, torch.from_numpy(trunc.astype(np.int64)).cuda(), offsets_host=trunc)
    assert status.cpu().tolist() == [1, 0] and int(mism.item()) == 1


def test_checksum_offsets_reproduces_sender_hash(gpu):
    """mchecksum_gpu_checksum_offsets over the payload ranges yields exactly the
    values the sender stored (what hg_set_struct writes, src/mercury.c:699-707)."""
    import torch
    rng = np.random.default_rng(99)
    buf, off, crcs = _batch(rng, 300)
    host = np.frombuffer(buf, dtype=np.uint8).copy()
    t = torch.zeros(host.size + 64, dtype=torch.uint8, device="cuda")
    t[:host.size].copy_(torch.from_numpy(host))
    # payload table: [msg + 20, next msg) -- an offsets table with gaps is
    # expressed by checksumming each payload separately through pairs
    starts = off[:-1] + CORE_HDR + HG_HDR
    pair = np.empty(2 * (len(off) - 1), dtype=np.uint64)
    pair[0::2], pair[1::2] = starts, off[1:]
    got_all = gpu.as_unsigned(gpu.checksum_offsets("crc32c", t, torch.from_numpy(pair.astype(np.int64)).cuda()))
    assert got_all[0::2].tolist() == crcs


def test_verify_messages_rejects_bad_layout(gpu):
    import torch
    t = torch.zeros(128, dtype=torch.uint8, device="cuda")
    offs = torch.tensor([0, 64], dtype=torch.int64, device="cuda")
    with pytest.raises(gpu.GpuChecksumError):
        gpu.verify_messages(t, offs, payload_offset=18, hash_offset=16)  # hash overlaps payload
    with pytest.raises(gpu.GpuChecksumError):
        gpu.verify_messages(t, offs, method="crc64")
