#!/bin/bash
# Round-4 pass f: log-mel (front-end tests, line, profile) and the greedy decode phase trace with
# the folded attention's prologue sub-phases (select / cell / query).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frontend.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_frontend.log 2>&1 || { tail -40 $O/pytest_frontend.log; exit 1; }
tail -1 $O/pytest_frontend.log
bash tools/probes/logmel_profile.sh || exit 1
timeout -k 10 200 python tools/probes/dg_trace.py > $O/dg_trace_greedy.txt 2>&1 || { tail -5 $O/dg_trace_greedy.txt; exit 1; }
head -12 $O/dg_trace_greedy.txt
timeout -k 10 120 ./tools/probes/logmel_variants > $O/logmel_variants.txt 2>&1 || { tail -5 $O/logmel_variants.txt; exit 1; }
cat $O/logmel_variants.txt
