#!/usr/bin/env python3
"""Device time per call of the offsets-table entry points on small batches of
4 KiB messages (HIP events, median of 50): checksum_offsets over the whole
messages, checksum_offsets over the payloads (byte 20 on), verify_offsets,
verify_messages -- per layout policy (argv[1]: default / 0 / 1)."""
import json, os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G  # noqa: E402


def dev_us(f):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for a, b in ev:
        a.record(s)
        f()
        b.record(s)
    torch.cuda.synchronize()
    return round(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3, 2)


def main():
    L = G._lib()
    length = 4096
    big = torch.empty(16384 * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(big, 3)
    for light in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["default"]):
        if light == "default":
            os.environ.pop("MCHECKSUM_GPU_LIGHT", None)
        else:
            os.environ["MCHECKSUM_GPU_LIGHT"] = light
        L.mchecksum_gpu_reload_settings()
        for count in (64, 1024, 4096, 16384):
            off = torch.arange(0, (count + 1) * length, length, dtype=torch.int64, device="cuda")
            pay = torch.empty(2 * count, dtype=torch.int64, device="cuda")
            pay[0::2] = off[:-1] + 20
            pay[1::2] = off[1:]
            out = torch.empty(2 * count, dtype=torch.int32, device="cuda")
            exp = torch.zeros(count, dtype=torch.int32, device="cuda")
            st = torch.empty(count, dtype=torch.uint8, device="cuda")
            bad = torch.zeros(1, dtype=torch.int32, device="cuda")
            h = torch.cuda.current_stream().cuda_stream
            m = b"crc32c"
            r = {"light": light, "messages": count,
                 "checksum_offsets_us": dev_us(lambda: L.mchecksum_gpu_checksum_offsets(m, big.data_ptr(), off.data_ptr(), count, out.data_ptr(), h)),
                 "checksum_payload_pairs_us": dev_us(lambda: L.mchecksum_gpu_checksum_offsets(m, big.data_ptr(), pay.data_ptr(), 2 * count - 1, out.data_ptr(), h)),
                 "verify_offsets_us": dev_us(lambda: L.mchecksum_gpu_verify_offsets(m, big.data_ptr(), off.data_ptr(), count, exp.data_ptr(), st.data_ptr(), bad.data_ptr(), h)),
                 "verify_messages_us": dev_us(lambda: L.mchecksum_gpu_verify_messages(m, big.data_ptr(), off.data_ptr(), count, 20, 16, st.data_ptr(), bad.data_ptr(), h))}
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
