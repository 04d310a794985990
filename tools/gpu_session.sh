#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault / abort / timeout stops the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STAGES="${STAGES:-pytest smoke bench prof}"
FAULT_RE='illegal memory access|HSA_STATUS_ERROR|Memory access fault|hipErrorIllegalAddress|core dumped|Aborted'
stop_on_fault() {  # $1 = rc, $2 = stage, $3 = log
  if [ -n "$3" ] && grep -Eq "$FAULT_RE" "$3"; then
    echo "[$2] GPU fault in $3: stopping the session"; exit 99
  fi
  case "$1" in
    0) return 0 ;;
    1) [ "$2" = pytest ] && { echo "[$2] test failures (rc=1), continuing"; return 0; } ;;
  esac
  echo "[$2] rc=$1: stopping the session"; exit "$1"
}
for s in $STAGES; do
  case $s in
    pytest)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -5 $OUT/pytest_gpu.log; stop_on_fault $rc pytest $OUT/pytest_gpu.log ;;
    pytestall)
      timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
      rc=$?; tail -15 $OUT/pytest_gpu.log; stop_on_fault $rc pytest $OUT/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; tail -3 $OUT/smoke.log; stop_on_fault $rc smoke $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
      rc=$?; cat $OUT/bench.json; tail -3 $OUT/bench.err; stop_on_fault $rc bench $OUT/bench.err ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-configs ${PROF_ARGS} > $OUT/prof_bench.json 2> $OUT/prof.err
      rc=$?; tail -3 $OUT/prof.err; stop_on_fault $rc prof $OUT/prof.err
      python tools/prof_by_grid.py $OUT/prof/run_kernel_trace.csv 30 > $OUT/prof_by_grid.txt 2>&1
      head -12 $OUT/prof_by_grid.txt ;;
    trace)
      timeout -k 10 300 python tools/rec_trace.py > $OUT/rec_trace.txt 2>&1
      rc=$?; cat $OUT/rec_trace.txt; stop_on_fault $rc trace $OUT/rec_trace.txt ;;
  esac
done
echo "session done"
