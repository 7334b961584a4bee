#!/bin/bash
# CPU streaming-path throughput on this host: bench.py's C1 config (1024 x 4 KiB
# through reset/update/update/get, one thread) with each CRC-32C path the
# library can pick (MCHECKSUM_DISABLE_CLMUL / _SSE42), plus large single updates.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}; cd "$R"; mkdir -p gpurun_out
for v in default 1 sse_off; do
  case $v in default) E="";; 1) E="MCHECKSUM_DISABLE_CLMUL=1";; sse_off) E="MCHECKSUM_DISABLE_SSE42=1";; esac
  env $E timeout -k 10 120 python bench.py --config c1 > gpurun_out/c1_$v.json || exit 1
  echo "$v $(python -c "import json; d=json.load(open('gpurun_out/c1_$v.json')); print(d['value'], d['unit'], d['parity'], 'oracle', d['cpu_baseline']['value'])")"
done
gcc -O2 -Iinclude tools/cpu_update_bench.c -o gpurun_out/cpu_update_bench -Lmercury_amd/lib -lmchecksum -Wl,-rpath,$R/mercury_amd/lib || exit 1
for m in crc32c crc64 crc32; do for n in 4096 65536 1048576; do
  for v in default 1; do
    case $v in default) E="";; 1) E="MCHECKSUM_DISABLE_CLMUL=1";; esac
    echo "$v $(env $E timeout -k 10 60 gpurun_out/cpu_update_bench $m $n $((2000000000 / n)))" || exit 1
  done
done; done
grep -m1 "model name" /proc/cpuinfo
