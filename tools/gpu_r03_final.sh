#!/bin/bash
# Round-3 evidence on the current code: the whole -m gpu suite, smoke, then profile_r03.sh
# (bench line, rocprofv3 kernel trace + stats, PMC passes) into gpurun_out/r03
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r03/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke.log 2>&1 || { tail -5 gpurun_out/r03/smoke.log; exit 1; }
tail -1 gpurun_out/r03/smoke.log
bash tools/probes/profile_r03.sh
