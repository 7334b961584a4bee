#!/usr/bin/env python3
"""Batch rate of every 32/64-bit catalogue method on the GPU path, C3's shape
(8192 x 1 MiB) and the headline's (65536 x 64 KiB), interleaved in one
process: an MSB-first method (crc64-ecma182) runs the reflected kernels on
conjugated tables plus one byte-swap launch.  Median of 20 launches after 10
warm-ups, HIP events on the launch stream; first payloads checked against the
oracle.  Writes gpurun_out/variant_rate.json."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    res = {}
    for shape, (count, length) in {"c3": (8192, 1 << 20), "metric": (65536, 65536)}.items():
        data = torch.empty(count * length + 64, dtype=torch.uint8, device="cuda")
        G.fill_splitmix(data, 0x4D43310000000003)
        head = data[:4 * length].cpu().numpy()
        for rnd in range(2):
            for m in ("crc32c", "crc32", "crc64", "crc64-ecma182", "crc64-go-iso", "crc64-jones"):
                out = torch.empty(count, dtype=G.out_dtype(m), device="cuda")
                for _ in range(10):
                    G.checksum_fixed(m, data, length, count=count, out=out)
                ts = []
                for _ in range(20):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(); G.checksum_fixed(m, data, length, count=count, out=out); b.record()
                    b.synchronize(); ts.append(a.elapsed_time(b))
                got = G.as_unsigned(out[:4]).astype(np.uint64).tolist()
                want = [O.crc(m, head[i * length:(i + 1) * length]) for i in range(4)]
                ms = float(np.median(ts))
                res[f"{shape}/{m}"] = {"ms": round(ms, 4), "GB_s": round(count * length / ms / 1e6, 1),
                                       "oracle_ok": got == want}
        print(json.dumps({k: v for k, v in res.items() if k.startswith(shape)}), flush=True)
        del data
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "variant_rate.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
