"""The split CRC-64 queue plan (crc_gpu_device.h SplitPlan: chunks of whole
payloads in 256 KiB pieces, eighth-size tail chunks) checked on the host: chunks tile the units once, units tile every
payload's bytes once, and a plan that claims whole-payload chunks (the
in-workgroup combine) has them.  The GPU side is tests/test_gpu_split64.py and
the C3 full-shape parity test."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "split_plan.cpp")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not installed")
def test_split_plan_tiles_units_and_payloads(tmp_path):
    exe = str(tmp_path / "split_plan")
    subprocess.run([HIPCC, "-O1", "-std=c++17", "--offload-arch=gfx950",
                    "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "mercury_amd", "csrc"), SRC,
                    "-o", exe], check=True, capture_output=True, timeout=600)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failures" in r.stdout
