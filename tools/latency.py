#!/usr/bin/env python3
"""Small-batch latency of the batch entry points: per-call device time (HIP
events) and host wall time per call, eager launches vs hipGraph replay
(torch.cuda.CUDAGraph capturing the C-ABI call on the capture stream), and
verify_messages over n 4 KiB messages; per layout policy (argv[1]: a comma
list of default / 0 / 1 = MCHECKSUM_GPU_LIGHT unset / off / on)."""
import json, os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mercury_amd import gpu as G

def main():
    length = 4096
    res = []
    G.prepare("crc32c")
    big = torch.empty(16384 * length + 64, dtype=torch.uint8, device="cuda")
    G.fill_splitmix(big, 1)
    for light in sys.argv[1].split(",") if len(sys.argv) > 1 else ("default", "0", "1"):
      if light == "default":
          os.environ.pop("MCHECKSUM_GPU_LIGHT", None)
      else:
          os.environ["MCHECKSUM_GPU_LIGHT"] = light
      G._lib().mchecksum_gpu_reload_settings()  # (the library reads its settings once)
      for count in (1, 8, 64, 256, 1024, 4096, 8192, 16384):
          out = torch.empty(count, dtype=torch.int32, device="cuda")
          f = lambda: G.checksum_fixed("crc32c", big, length, count=count, out=out)
          for _ in range(5):
              f()
          torch.cuda.synchronize()
          s = torch.cuda.current_stream()
          ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
          for a, b in ev:
              a.record(s); f(); b.record(s)
          torch.cuda.synchronize()
          dev_us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
          n = 200
          t0 = time.perf_counter()
          for _ in range(n):
              f()
          issue_us = (time.perf_counter() - t0) / n * 1e6  # host cost of one call (queue not full)
          torch.cuda.synchronize()
          eager_us = (time.perf_counter() - t0) / n * 1e6
          # the C-ABI call alone (no torch wrapper): host cost of the entry point
          L = G._lib()
          h = torch.cuda.current_stream().cuda_stream
          t1 = time.perf_counter()
          for _ in range(n):
              L.mchecksum_gpu_checksum_fixed(b"crc32c", big.data_ptr(), length, length, count, out.data_ptr(), h)
          capi_us = (time.perf_counter() - t1) / n * 1e6
          torch.cuda.synchronize()
          g = torch.cuda.CUDAGraph()
          with torch.cuda.graph(g):
              f()
          ref = out.clone()
          g.replay(); torch.cuda.synchronize()
          same = bool(torch.equal(ref, out))
          t0 = time.perf_counter()
          for _ in range(n):
              g.replay()
          torch.cuda.synchronize()
          graph_us = (time.perf_counter() - t0) / n * 1e6
          r = {"light": light, "payloads": count, "bytes": count * length, "device_us": round(dev_us, 2),
               "eager_wall_us_per_call": round(eager_us, 2), "host_issue_us": round(issue_us, 2), "capi_issue_us": round(capi_us, 2), "graph_wall_us_per_replay": round(graph_us, 2),
               "graph_result_identical": same, "GBps_device": round(count * length / dev_us / 1e3, 1)}
          print(json.dumps(r), flush=True)
          res.append(r)
    # Mercury's receive side: a drained buffer of n request messages of 4 KiB
    # verified in place (mchecksum_gpu_verify_messages), device time per call
    L = G._lib()
    for light in sys.argv[1].split(",") if len(sys.argv) > 1 else ("default", "0", "1"):
        if light == "default":
            os.environ.pop("MCHECKSUM_GPU_LIGHT", None)
        else:
            os.environ["MCHECKSUM_GPU_LIGHT"] = light
        L.mchecksum_gpu_reload_settings()
        for count in (1, 64, 256, 1024, 4096):
            off = torch.arange(0, (count + 1) * length, length, dtype=torch.int64, device="cuda")
            status = torch.empty(count, dtype=torch.uint8, device="cuda")
            bad = torch.zeros(1, dtype=torch.int32, device="cuda")
            h = torch.cuda.current_stream().cuda_stream
            f = lambda: L.mchecksum_gpu_verify_messages(b"crc32c", big.data_ptr(), off.data_ptr(), count, 20, 16,
                                                        status.data_ptr(), bad.data_ptr(), h)
            for _ in range(5):
                assert f() == 0
            torch.cuda.synchronize()
            s_ = torch.cuda.current_stream()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
            for a, b in ev:
                a.record(s_); f(); b.record(s_)
            torch.cuda.synchronize()
            dev_us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
            r = {"light": light, "messages": count, "bytes": count * length, "verify_messages_device_us": round(dev_us, 2)}
            print(json.dumps(r), flush=True)
            res.append(r)
    json.dump(res, open(os.path.join(ROOT, "gpurun_out", "latency.json"), "w"), indent=1)

if __name__ == "__main__":
    main()
