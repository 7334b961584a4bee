"""CPU emulation of the exact lane-parallel algorithm the gfx950 kernels run
(same host-built table packs, same edge-handling code in crc_gpu_mask.h),
checked against the oracle for every lanes-per-payload width, many lengths and
every start alignment.  GPU-only details (LDS replication, v_perm addressing,
shuffles) are covered by the -m gpu parity tests."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "tests", "native", "kernel_emulator.cpp"),
       os.path.join(ROOT, "mercury_amd", "csrc", "crc_tables.c"),
       os.path.join(ROOT, "oracle", "crc_oracle.c")]
OUT = os.path.join(ROOT, "build", "test")


@pytest.fixture(scope="module")
def emu():
    os.makedirs(OUT, exist_ok=True)
    so = os.path.join(OUT, "libemu.so")
    if not os.path.exists(so) or any(os.path.getmtime(s) > os.path.getmtime(so) for s in SRC):
        subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-x", "c++", SRC[0], "-x", "c", SRC[1], SRC[2],
                        "-o", so, "-lpthread"], check=True, capture_output=True)
    L = ctypes.CDLL(so)
    L.emu_pack32.restype = ctypes.c_void_p
    L.emu_pack64.restype = ctypes.c_void_p
    L.emu_pack32.argtypes = L.emu_pack64.argtypes = [ctypes.c_int]
    L.emu_crc32.restype = ctypes.c_uint32
    L.emu_crc64.restype = ctypes.c_uint64
    for f in (L.emu_crc32, L.emu_crc64):
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
    return L


def test_emulator_main_binary():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "emu_main")
    subprocess.run(["g++", "-O2", "-DEMULATOR_MAIN", "-x", "c++", SRC[0], "-x", "c", SRC[1], SRC[2], "-o", exe,
                    "-lpthread"], check=True, capture_output=True)
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 0 and " 0 failures" in r.stdout, r.stdout


@pytest.mark.parametrize("log2g", range(7))
def test_emulated_kernel_equals_oracle(emu, oracle_mod, log2g):
    p32, p64 = emu.emu_pack32(log2g), emu.emu_pack64(log2g)
    assert p32 and p64
    buf = oracle_mod.splitmix_bytes(140000, 0x77 + log2g)
    rng = np.random.default_rng(log2g)
    for _ in range(120):
        start = int(rng.integers(0, 40))
        n = int(rng.integers(0, 130000)) if rng.random() < 0.25 else int(rng.integers(0, 600))
        d = buf[start:start + n]
        assert emu.emu_crc32(p32, buf.ctypes.data, buf.size, start, n) == oracle_mod.crc("crc32c", d), (start, n)
        assert emu.emu_crc64(p64, buf.ctypes.data, buf.size, start, n) == oracle_mod.crc("crc64", d), (start, n)


@pytest.mark.parametrize("log2g", [6])
def test_emulated_128b_grid_equals_oracle(emu, oracle_mod, log2g, monkeypatch):
    """The one-payload-per-wave loops end their step grid on a 128-B line
    (round 3, crc_gpu_device.h kGridAlign): up to 127 pad bytes, undone by the
    tail table and the butterfly operators.  Every start alignment and lengths
    around each multiple of 16 and 128."""
    monkeypatch.setenv("EMU_GRID_ALIGN", "128")
    p32, p64 = emu.emu_pack32(log2g), emu.emu_pack64(log2g)
    buf = oracle_mod.splitmix_bytes(140000, 0x128)
    lens = sorted({0, 1, 3, 4, 7, 8, 9, 15, 16, 17} | {m + d for m in (127, 128, 255, 256, 1024, 1151, 4096, 65536)
                                                        for d in (-1, 0, 1)})
    for start in list(range(0, 130, 7)) + [1023, 4097]:
        for n in lens:
            d = buf[start:start + n]
            assert emu.emu_crc32(p32, buf.ctypes.data, buf.size, start, n) == oracle_mod.crc("crc32c", d), (start, n)
            assert emu.emu_crc64(p64, buf.ctypes.data, buf.size, start, n) == oracle_mod.crc("crc64", d), (start, n)
