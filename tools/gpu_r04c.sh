#!/bin/bash
# Round-4 pass c: log-mel front end (tests + line + profile), then the cooperative-launch exit probe
# under rocprofv3: a bare HIP program (no casr code) launching one trivial kernel plainly, then
# cooperatively (last: the run that may end in SIGSEGV).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_frontend.log 2>&1 || { tail -40 $O/pytest_frontend.log; exit 1; }
tail -2 $O/pytest_frontend.log
bash tools/probes/logmel_profile.sh || exit 1
timeout -k 10 200 python tools/probes/dg_trace.py > $O/dg_trace_greedy.txt 2>&1 || { tail -5 $O/dg_trace_greedy.txt; exit 1; }
cat $O/dg_trace_greedy.txt
for mode in plain coop; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/coop_$mode -o run -- \
    ./tools/probes/coop_exit_probe $mode > $O/coop_$mode.log 2>&1
  echo "coop_exit_probe $mode under rocprofv3: exit status $?" | tee -a $O/coop_rc.txt
  grep -v "^    @" $O/coop_$mode.log | tail -4
done
