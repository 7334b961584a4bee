"""The batch ABI from C on the MI355X: build/hg_verify_consumer
(tests/native/hg_verify_consumer.c, built by `make` through
cmake/mchecksum-config.cmake) hipMallocs a drained receive buffer of 4096
Mercury request messages -- core header with its CRC16, HG header with the
network-order payload CRC32C, payload -- with planted corruption, verifies it
with mchecksum_gpu_verify_core_headers and mchecksum_gpu_verify_messages on a
hipStream_t it created, and compares every status and both mismatch counts
with the verdicts Mercury's own per-message checks give through the streaming
API (hg_core_header_request_proc, /root/reference/src/mercury_core_header.c:
175-230; hg_proc_checksum_verify, /root/reference/src/mercury_proc.c:433-472)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "hg_verify_consumer")


def test_c_consumer_verifies_like_mercury(gpu):
    assert os.access(EXE, os.X_OK), "build/hg_verify_consumer missing: run make"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout and "statuses 0 differ, payload statuses 0 differ" in r.stdout
