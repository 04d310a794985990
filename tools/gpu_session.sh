#!/bin/bash
# One GPU-box session, parameterised (replaces the per-round tools/gpu_r0*.sh scripts).
#
#   OUT=gpurun_out/<tag> STAGES="smoke tests suite bench" bash tools/gpu_session.sh
#
# Stages, run in the order given; each GPU step has its own time limit, and a fault, abort,
# segfault or time-out stops the session (no further GPU step after it):
#   smoke            __graft_entry__.smoke()
#   tests            pytest -m gpu on TESTS (files / node ids, default: the whole tests/ tree),
#                    filtered by TESTS_K (pytest -k) when set
#   suite            the whole -m gpu suite (as the driver runs it, -x)
#   bench            python bench.py $BENCH_ARGS > $OUT/bench.json
#   ab               interleaved A/B: for each of AB_ROUNDS rounds, bench.py $AB_ARGS once per
#                    CASR_OPTS value in AB_OPTS (';'-separated; "-" = defaults) -> $OUT/ab_<i>_<r>.json
#   counters         rocprofv3 -L (the counters this box can collect) -> $OUT/counters.txt
#   pmc              PMC passes of tools/probes/one_step.py (PMC_MODES: greedy and/or beam) with the
#                    counter sets in PMC_SETS (';'-separated passes) into $OUT/pmc<PMC_TAG>_<mode>;
#                    CASR_OPTS=$PMC_OPTS (default REC_COOP=0, the ordinary recurrence launch: DESIGN
#                    3.2, a cooperative launch (REC_COOP=1) ends in SIGSEGV under rocprofv3)
#   profbeam         rocprofv3 kernel trace + stats of tools/probes/one_step.py at beam 8, B = 256 and 128
#   probe            python $PROBE once (tools/probes/*.py)
#   ablibs           tools/probes/ab_libs.sh (LIBS, AB_ARGS, AB_ROUNDS): interleaved library-build A/B
#   trace            tools/rec_trace.py
#   prof             rocprofv3 kernel trace + stats of bench.py (greedy only) on the shipped
#                    recurrence launch (round 6: chained ordinary, REC_COOP=2); its exit status is
#                    recorded (must be the LAST stage)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/session}
mkdir -p "$OUT"
STAGES="${STAGES:-smoke suite bench}"
FAULT_RE='illegal memory access|HSA_STATUS_ERROR|Memory access fault|hipErrorIllegalAddress|core dumped|Aborted'
stop_on() {  # $1 = rc, $2 = stage, $3 = log
  if [ -n "$3" ] && grep -Eq "$FAULT_RE" "$3"; then
    echo "[$2] GPU fault in $3: stopping the session"; exit 99
  fi
  [ "$1" = 0 ] && return 0
  echo "[$2] rc=$1: stopping the session"; tail -30 "$3"; exit "$1"
}
PYTEST="python -u -m pytest -x -v --timeout ${TEST_TIMEOUT:-300} --timeout-method thread -p no:cacheprovider"
for s in $STAGES; do
  case $s in
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
      rc=$?; tail -1 $OUT/smoke.log; stop_on $rc smoke $OUT/smoke.log ;;
    tests)
      timeout -k 10 ${TESTS_LIMIT:-900} $PYTEST -m gpu ${TESTS:-tests} ${TESTS_K:+-k "$TESTS_K"} > $OUT/tests.log 2>&1
      rc=$?; grep -E "PASSED|FAILED|ERROR|SKIPPED" $OUT/tests.log | sed 's/^tests\///' | tail -60; tail -1 $OUT/tests.log
      stop_on $rc tests $OUT/tests.log ;;
    suite)
      timeout -k 10 1000 $PYTEST -m gpu tests > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -1 $OUT/pytest_gpu.log; stop_on $rc suite $OUT/pytest_gpu.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; stop_on $rc bench $OUT/bench.err
      python tools/bench_line.py $OUT/bench.json ;;
    ab)
      IFS=';' read -r -a opts <<< "${AB_OPTS:--}"
      for r in $(seq 1 ${AB_ROUNDS:-2}); do
        for i in "${!opts[@]}"; do
          o="${opts[$i]}"; [ "$o" = "-" ] && o=""
          CASR_OPTS="$o" timeout -k 10 300 python bench.py --steps ${AB_STEPS:-20} --warmup 3 --no-configs \
            --no-cpu-baseline --no-f32-compare ${AB_ARGS} > $OUT/ab_${i}_$r.json 2> $OUT/ab.err
          rc=$?; stop_on $rc ab $OUT/ab.err
          echo -n "[$r] opts='$o' "; python tools/bench_line.py $OUT/ab_${i}_$r.json
        done
      done ;;
    counters)
      timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
      rc=$?; grep -ciE "counter|name" $OUT/counters.txt; stop_on $rc counters $OUT/counters.txt ;;
    pmc)
      DEFSETS="${PMC_SETS:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE}"
      for mode in ${PMC_MODES:-greedy beam}; do
        mv_="PMC_SETS_$mode"  # per-mode counter sets (PMC_SETS_greedy=...), else the common ones
        IFS=';' read -r -a sets <<< "${!mv_:-$DEFSETS}"
        P=$OUT/pmc${PMC_TAG}_$mode
        mkdir -p $P
        if [ $mode = beam ]; then export BEAM=8 B=256; elif [ $mode = beam128 ]; then export BEAM=8 B=128;
        else unset BEAM; export B=256; fi
        for i in "${!sets[@]}"; do
          CASR_OPTS=${PMC_OPTS:-REC_COOP=0} timeout -s KILL 120 rocprofv3 --pmc ${sets[$i]} --output-format csv -d $P/p$i -o p$i -- \
            python3 tools/probes/one_step.py > $P/p$i.log 2>&1
          rc=$?; stop_on $rc "pmc $mode ${sets[$i]}" $P/p$i.log
        done
      done
      unset BEAM B ;;
    profbeam)
      # kernel trace + stats of beam 8 at B = 256 (the metric's beam line) and at B = 128 (config 3),
      # tools/probes/one_step.py, ordinary recurrence launch (a cooperative launch ends in SIGSEGV at
      # exit under rocprofv3)
      for bb in ${PROF_BATCHES:-256 128}; do
        BEAM=${PROF_BEAM:-8} B=$bb STEPS=${PROF_STEPS:-6} CASR_OPTS=REC_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats \
          --output-format csv -d $OUT/profbeam$bb -o run -- python3 tools/probes/one_step.py > $OUT/profbeam$bb.log 2>&1
        rc=$?; stop_on $rc "profbeam $bb" $OUT/profbeam$bb.log
        python tools/prof_by_grid.py $OUT/profbeam$bb/run_kernel_trace.csv 30 > $OUT/prof_by_grid_beam$bb.txt 2>&1
        head -12 $OUT/prof_by_grid_beam$bb.txt
      done ;;
    probe)
      # PROBE = a python script (tools/probes/...) or a probe binary built in the container, run once
      case $PROBE in
        *.py) timeout -k 10 ${PROBE_LIMIT:-300} python -u $PROBE > $OUT/probe.log 2>&1 ;;
        *) (cd $(dirname $PROBE) && timeout -k 10 ${PROBE_LIMIT:-300} ./$(basename $PROBE) $PROBE_ARGS) > $OUT/probe.log 2>&1 ;;
      esac
      rc=$?; tail -20 $OUT/probe.log; stop_on $rc probe $OUT/probe.log ;;
    ablibs)
      OUT=$OUT/ablibs timeout -k 10 ${ABLIBS_LIMIT:-600} bash tools/probes/ab_libs.sh > $OUT/ablibs.log 2>&1
      rc=$?; cat $OUT/ablibs.log | tail -20; stop_on $rc ablibs $OUT/ablibs.log ;;
    trace)
      timeout -k 10 300 python tools/rec_trace.py > $OUT/rec_trace.txt 2>&1
      rc=$?; tail -20 $OUT/rec_trace.txt; stop_on $rc trace $OUT/rec_trace.txt ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py --steps 20 --warmup 2 --streams 1 --no-beam --no-configs --no-f32-compare --no-cpu-baseline \
        > $OUT/prof_bench.json 2> $OUT/prof.err
      echo "rocprofv3 kernel trace of the default recurrence launch: exit status $?" | tee $OUT/prof_rc.txt
      python tools/prof_by_grid.py $OUT/prof/run_kernel_trace.csv 30 > $OUT/prof_by_grid.txt 2>&1
      head -14 $OUT/prof_by_grid.txt
      break ;;
  esac
done
echo "session done"
