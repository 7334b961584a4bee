#!/bin/bash
# Round-5 GPU passes.  PART selects one:
#   tests  -- new slot / fail-closed tests first, then the whole -m gpu suite
#   ab     -- in-process A/B (tools/ab_variants.py): AB_VARIANTS of build/variants
#             (default: working tree "cur" vs last commit "prev") plus the
#             env pseudo-variants in AB_ENV, on AB_CONFIGS
#   bench  -- bench.py per CONFIGS into gpurun_out/r05/bench_<config>.json
#   trace  -- rocprofv3 kernel-trace summaries of bench.py per CONFIGS
#   xcd    -- per-XCD end time and shader clock (tools/xcd_clock.py, trace build)
#   pmc    -- FETCH_SIZE / WRITE_SIZE passes per CONFIGS -> pmc_traffic_<config>.json
#   probe  -- tools/stream_probe (stream ids vs handles, completion-evidence cost)
#   nccl   -- torchrun --nproc-per-node 1 bench.py (RCCL process group at world 1) per CONFIGS
#   newtests -- TESTS (space-separated test files) only
#   sq     -- SQ / LDS / clock counters (three --pmc passes, GRBM_GUI_ACTIVE with a
#             kernel trace) per CONFIGS over PMC_KERNELS -> sq_<config>.txt
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd "$R"; mkdir -p gpurun_out/r05
O="$R/gpurun_out/r05"
step() { echo "== $1 $(date +%T)"; }
for P in ${PART:-tests}; do
if [ "$P" = probe ]; then
  step "stream probe"
  timeout -k 10 120 ./build/stream_probe > $O/stream_probe.log 2>&1; rc=$?
  cat $O/stream_probe.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$P" = newtests ]; then
  step "tests $TESTS"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout ${PT:-150} --timeout-method thread > $O/pytest_${TAG:-new}.log 2>&1; rc=$?
  tail -15 $O/pytest_${TAG:-new}.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|^E " $O/pytest_${TAG:-new}.log | head -60; exit $rc; }
fi
if [ "$P" = nccl ]; then
  for c in ${CONFIGS:-c5}; do
    step "torchrun 1 rank nccl $c"
    timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29533 \
      bench.py --gpus 1 --config $c ${BENCH_ARGS:-} > $O/bench_nccl_1rank_$c.json 2> $O/bench_nccl_1rank_$c.err || { tail -30 $O/bench_nccl_1rank_$c.err; exit 1; }
    cat $O/bench_nccl_1rank_$c.json
  done
fi
if [ "$P" = tests ]; then
  step "new tests"
  timeout -k 10 600 python -u -m pytest tests/test_gpu_slots.py tests/test_gpu_fail_closed.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > $O/pytest_new.log 2>&1; rc=$?
  tail -15 $O/pytest_new.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|^E " $O/pytest_new.log | head -60; exit $rc; }
  step "full suite"
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1; rc=$?
  tail -5 $O/pytest_gpu.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|^E " $O/pytest_gpu.log | head -60; exit $rc; }
fi
if [ "$P" = ab ]; then
  step "ab ${AB_CONFIGS:-c2,metric}"
  timeout -k 10 600 python tools/ab_variants.py --config ${AB_CONFIGS:-c2,metric} --variants ${AB_VARIANTS:-prev cur} \
    ${AB_ENV:-} --rounds ${AB_ROUNDS:-6} --iters ${AB_ITERS:-10} \
    --out $O/ab_${AB_TAG:-r05}.json > $O/ab_${AB_TAG:-r05}.log 2>&1; rc=$?
  grep -v amdgpu.ids $O/ab_${AB_TAG:-r05}.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "$P" = xdrtest ]; then
  step "xdr tests"
  timeout -k 10 600 python -u -m pytest tests/test_xdr.py -m gpu -x -v --timeout 300 --timeout-method thread \
    > $O/pytest_xdr.log 2>&1; rc=$?
  tail -5 $O/pytest_xdr.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED|^E " $O/pytest_xdr.log | head -60; exit $rc; }
fi
if [ "$P" = bench ]; then
  for c in ${CONFIGS:-metric c2}; do
    step "bench $c"
    timeout -k 10 300 python bench.py --config $c ${BENCH_ARGS:-} > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
    cat $O/bench_$c.json
  done
fi
if [ "$P" = driver ]; then
  step "bench driver-style"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
  cat $O/bench_driver.json
fi
if [ "$P" = xcd ]; then
  step "xcd clock ${XCD_CONFIGS:-c2}"
  timeout -k 10 300 python tools/xcd_clock.py ${XCD_CONFIGS:-c2} --out $O/xcd_clock.json > $O/xcd_clock.log 2>&1; rc=$?
  grep -v amdgpu.ids $O/xcd_clock.log | tail -25; [ $rc -eq 0 ] || exit $rc
fi
if [ "$P" = trace ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-c2}; do
    step "kernel trace $c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o bench -- python3 $R/bench.py --config $c ${BENCH_ARGS:-} > $O/prof_bench_$c.json 2> $O/prof_bench_$c.err || { tail $O/prof_bench_$c.err; exit 1; }
    cat $O/prof_bench_$c.json
  done
  cd "$R"
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
      timeout -s KILL 120 rocprofv3 --pmc $set $kt --output-format csv -d $O/sq_${c}_$i -o p -- python3 $R/tools/kernel_run.py --config $c --iters ${SQ_ITERS:-6} > $O/sq_${c}_$i.log 2>&1 || { echo "sq $c $i failed"; tail -5 $O/sq_${c}_$i.log; exit 1; }
    done
    python3 $R/tools/pmc_summary.py $O/sq_${c}_1 $O/sq_${c}_2 $O/sq_${c}_3 > $O/sq_$c.txt || exit 1
    cat $O/sq_$c.txt
  done
  cd "$R"
fi
if [ "$P" = pmc ]; then
  cd /tmp && export TMPDIR=/tmp
  for c in ${CONFIGS:-c4}; do
    step "pmc $c"
    timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/tr_${c}_f -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/tr_${c}_f.log 2>&1 || { tail $O/tr_${c}_f.log; exit 1; }
    timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/tr_${c}_w -o p -- python3 $R/tools/kernel_run.py --config $c --iters 4 > $O/tr_${c}_w.log 2>&1 || { tail $O/tr_${c}_w.log; exit 1; }
    k=batch_kernel; pc=1; [ "$c" = xdr ] && k=xdr_fast_kernel
    [ "$c" = seg ] && k=seg_ && pc=2  # one-launch scan + chunk pass per call
    python3 $R/tools/pmc_traffic.py $O/tr_${c}_f $O/tr_${c}_w $k $O/pmc_traffic_$c.json $(python3 $R/tools/alg_bytes.py $c) $pc $((4 * pc)) || exit 1
  done
  cd "$R"
fi
done
