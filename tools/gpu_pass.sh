#!/bin/bash
# GPU passes (gpurun).  PART selects one or more (space-separated), in order:
#   tests    -- the whole -m gpu suite (TESTS: only those files)
#   driver   -- the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   bench    -- bench.py --config C per CONFIGS (BENCH_ARGS appended)
#   trace    -- rocprofv3 --kernel-trace --stats of bench.py per CONFIGS
#   pmc      -- FETCH_SIZE / WRITE_SIZE passes per CONFIGS -> pmc_traffic_<config>.json
#               (KR_ARGS appended to tools/kernel_run.py, e.g. "--rotate 4")
#   ab       -- in-process A/B (tools/ab_variants.py) of AB_VARIANTS on AB_CONFIGS
#   sq       -- SQ / LDS / clock counters (three --pmc passes) per CONFIGS
# Output: gpurun_out/$TAG (default r06).  Every GPU step has its own time limit;
# the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"
O="$R/gpurun_out/${TAG:-r06}"
mkdir -p "$O"
step() { echo "== $1 $(date +%T)"; }
fail_log() { grep -E "Error|assert|FAILED|^E " "$1" | head -60; }
for P in ${PART:-tests}; do
if [ "$P" = tests ]; then
  step "pytest -m gpu ${TESTS:-tests}"
  timeout -k 10 ${PT_TOTAL:-1100} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout ${PT:-300} \
    --timeout-method thread > $O/pytest_${PTAG:-gpu}.log 2>&1; rc=$?
  tail -5 $O/pytest_${PTAG:-gpu}.log
  [ $rc -eq 0 ] || { fail_log $O/pytest_${PTAG:-gpu}.log; exit $rc; }
fi
if [ "$P" = driver ]; then
  step "driver's command"
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err \
    || { tail -20 $O/bench_driver.err; exit 1; }
  cat $O/bench_driver.json
fi
if [ "$P" = bench ]; then
  for c in ${CONFIGS:-metric}; do
    step "bench $c"
    timeout -k 10 400 python bench.py --config $c ${BENCH_ARGS:-} > $O/bench_$c.json 2> $O/bench_$c.err \
      || { tail -20 $O/bench_$c.err; exit 1; }
    cat $O/bench_$c.json
  done
fi
if [ "$P" = trace ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-metric}; do
    step "kernel trace $c"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o bench -- \
      python3 $R/bench.py --config $c ${BENCH_ARGS:-} > $O/prof_bench_$c.json 2> $O/prof_bench_$c.err \
      || { tail $O/prof_bench_$c.err; exit 1; }
    cat $O/prof_bench_$c.json
  done
  cd "$R"
fi
if [ "$P" = pmc ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-c2}; do
    step "pmc $c"
    timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tr_${c}_f -o p -- \
      python3 $R/tools/kernel_run.py --config $c --iters 8 ${KR_ARGS:-} > $O/tr_${c}_f.log 2>&1 || { tail $O/tr_${c}_f.log; exit 1; }
    timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tr_${c}_w -o p -- \
      python3 $R/tools/kernel_run.py --config $c --iters 8 ${KR_ARGS:-} > $O/tr_${c}_w.log 2>&1 || { tail $O/tr_${c}_w.log; exit 1; }
    k=batch_kernel; pc=1; [ "$c" = xdr ] && k=xdr_fast_kernel
    [ "$c" = seg ] && k=seg_ && pc=2  # one-launch scan + chunk pass per call
    python3 $R/tools/pmc_traffic.py $O/tr_${c}_f $O/tr_${c}_w $k $O/pmc_traffic_$c.json $(python3 $R/tools/alg_bytes.py $c) \
      $pc $((4 * pc)) || exit 1
  done
  cd "$R"
fi
if [ "$P" = ab ]; then
  step "ab ${AB_CONFIGS:-c3}"
  timeout -k 10 700 python tools/ab_variants.py --config ${AB_CONFIGS:-c3} --variants ${AB_VARIANTS:-prev cur} \
    ${AB_ENV:-} --rounds ${AB_ROUNDS:-6} --iters ${AB_ITERS:-10} ${AB_ARGS:-} \
    --out $O/ab_${AB_TAG:-r06}.json > $O/ab_${AB_TAG:-r06}.log 2>&1; rc=$?
  grep -v amdgpu.ids $O/ab_${AB_TAG:-r06}.log | tail -40; [ $rc -eq 0 ] || exit $rc
fi
if [ "$P" = sq ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-c3}; do
    i=0
    for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_CYCLES" \
               "SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
               "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD"; do
      i=$((i+1))
      step "sq $c pass $i"
      kt=""; [ $i = 1 ] && kt="--kernel-trace"
      timeout -s KILL 120 rocprofv3 --pmc $set $kt --output-format csv -d $O/sq_${c}_$i -o p -- \
        python3 $R/tools/kernel_run.py --config $c --iters ${SQ_ITERS:-6} > $O/sq_${c}_$i.log 2>&1 \
        || { echo "sq $c $i failed"; tail -5 $O/sq_${c}_$i.log; exit 1; }
    done
    python3 $R/tools/pmc_summary.py $O/sq_${c}_1 $O/sq_${c}_2 $O/sq_${c}_3 > $O/sq_$c.txt || exit 1
    cat $O/sq_$c.txt
  done
  cd "$R"
fi
done
