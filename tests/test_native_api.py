"""The drop-in ABI from C, as Mercury uses it (tests/native/test_mchecksum_api.c):
linked against libmchecksum.so, and rebuilt from the CPU sources with
host-only ASan+UBSan and with TSan (the reference CI's sanitizer matrix,
.github/workflows/ci.yml:81-117)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "test")
TEST = os.path.join(ROOT, "tests", "native", "test_mchecksum_api.c")
CPU_SRC = [os.path.join(ROOT, "mercury_amd", "csrc", f) for f in ("mchecksum_cpu.c", "mchecksum_models.c",
                                                                   "crc_tables.c")]
INC = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "mercury_amd", "csrc")]


def _run(exe, env=None):
    r = subprocess.run([exe], capture_output=True, text=True, env={**os.environ, **(env or {})}, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout


def test_against_shared_library(product_lib):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "test_api_so")
    lib = os.path.join(ROOT, "mercury_amd", "lib")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", *INC, TEST, "-o", exe, "-L" + lib, "-lmchecksum",
                    "-Wl,-rpath," + lib, "-lpthread"], check=True)
    _run(exe)


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_sanitized_cpu_build(san):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "test_api_" + san.replace(",", "_"))
    subprocess.run(["gcc", "-O1", "-g", "-std=c11", "-fno-omit-frame-pointer", "-fsanitize=" + san,
                    "-fno-sanitize-recover=all", *INC, TEST, *CPU_SRC, "-o", exe, "-lpthread"], check=True)
    _run(exe, {"MCHECKSUM_LOG_LEVEL": "none"})


def test_scatter_gather_algebra():
    """Host half of mchecksum_gpu_checksum_segments: shift tables and the
    chunk-combine formula vs the streaming API (tests/native/test_shift_combine.c)."""
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "test_shift_combine")
    src = os.path.join(ROOT, "tests", "native", "test_shift_combine.c")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", *INC, src, *CPU_SRC, "-o", exe, "-lpthread"], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all checks passed" in r.stdout
