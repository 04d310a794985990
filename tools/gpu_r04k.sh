#!/bin/bash
# Round-4 pass k: fused decode GEMM phase trace of one mid-decode step (CASR_DG_TRACE_STEP), by
# column-block kind and XCD, greedy and beam 8 at B = 256.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
CASR_DG_TRACE_STEP=20 NTN=7 timeout -k 10 150 python tools/probes/dg_trace.py > $O/greedy_step20.txt 2>&1 || { tail -5 $O/greedy_step20.txt; exit 1; }
grep -A12 "^proj (greedy)" $O/greedy_step20.txt
CASR_DG_TRACE_STEP=20 NTN=14 BEAM=1 BB=256 K=8 timeout -k 10 150 python tools/probes/dg_trace.py > $O/beam_step20.txt 2>&1 || { tail -5 $O/beam_step20.txt; exit 1; }
grep -A12 "^proj (beam)" $O/beam_step20.txt
