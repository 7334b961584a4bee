"""bench.py's RCCL leg on the one-GPU box.

`torchrun --nproc-per-node 1 bench.py --gpus 1` forms the process group with
the nccl (= RCCL) backend even at world size 1 (bench.py: the group exists
whenever WORLD_SIZE is set), so the calls the driver's 8-GPU run makes --
init_process_group("nccl", device_id=...), the device all_gather of the
padded CRC shares, the float64 all_reduce of the byte count and the timing
gather -- execute here before that run does.  The line must carry the CPU
baseline and an oracle parity verdict over the gathered CRCs.

Requirement: BASELINE.json configs[4] (C5 sharded via RCCL), SURVEY.md 8(e).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(config, extra=()):
    import torch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()  # the child allocates its own batch (C5: 64 GiB)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--config", config, "--steps", "3", "--warmup", "2", "--cpu-seconds", "0.3",
           "--parity-samples", "16", *extra]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    print(r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # the one-JSON-line contract, RCCL notices kept off stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("config", ["c5", "metric"])
def test_one_rank_nccl_line(config):
    res = _torchrun(config)
    print(json.dumps(res))
    assert res["world_size"] == 1 and res["n_gpus"] == 1
    assert res["process_group"] == "nccl"
    cb = res["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    assert res["parity"].startswith("bit-exact (") and res["parity"].endswith("vs oracle)"), res["parity"]
    assert res["value"] > 0 and res["roofline"]["frac"] > 0
    assert res["scaling"] == ("strong" if config == "c5" else "weak")
    # the group's own world size, and the GPU each rank ran on
    assert [p["rank"] for p in res["per_rank"]] == [0] and res["per_rank"][0]["pci"] != "unknown", res["per_rank"]
    if config == "metric":
        # BASELINE configs[4] measured in the same run whatever the flags:
        # C5's 2^20 x 64 KiB global batch split over the ranks
        c5 = res["c5_strong"]
        assert c5["config"] == "c5" and c5["scaling"] == "strong" and c5["n_gpus"] == 1, c5
        assert "1048576 x 65536 B payloads" in c5["workload"] and "(1048576 on rank 0)" in c5["workload"], c5
        assert c5["value"] > 0 and 0 < c5["roofline_frac"] < 1 and len(c5["per_rank"]) == 1
        assert c5["parity"].startswith("bit-exact ("), c5["parity"]
    else:
        assert "c5_strong" not in res
