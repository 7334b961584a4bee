#!/usr/bin/env python3
"""DIAGNOSTIC: what a headline-shaped launch (256 x 1024-thread workgroups,
140 KiB LDS each) costs with no payload work.  Needs
  make variants VARIANTS="base:-DMCK_EMPTY=0 e1:-DMCK_EMPTY=1 e2:-DMCK_EMPTY=2"
(e2: return at kernel entry; e1: return after the LDS table fill; only on the
static path, MCHECKSUM_GPU_NT=0).  Median HIP-event time per launch, us."""
import ctypes, json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from ab_variants import load  # noqa: E402
from mercury_amd import gpu as G  # noqa: E402


def main():
    count, length = 65536, 65536
    data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(data, 5)
    out = torch.empty(count, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    libs = {n: load(os.path.join(ROOT, "build", "variants", f"libmchecksum_{n}.so")) for n in ("e2", "e1", "base")}
    for L in libs.values():
        assert L.mchecksum_gpu_prepare(b"crc32c") == 0
    res = {}
    for nt in ("0", "1"):
        os.environ["MCHECKSUM_GPU_NT"] = nt
        for _ in range(3):
            for n, L in libs.items():
                for _ in range(10):
                    L.mchecksum_gpu_checksum_fixed(b"crc32c", data.data_ptr(), length, length, count, out.data_ptr(), s)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
                for a, b in ev:
                    a.record()
                    L.mchecksum_gpu_checksum_fixed(b"crc32c", data.data_ptr(), length, length, count, out.data_ptr(), s)
                    b.record()
                torch.cuda.synchronize()
                res.setdefault(f"{n}_nt{nt}", []).append(round(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3, 2))
    print(json.dumps(res), flush=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "empty_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
