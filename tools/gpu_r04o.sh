#!/bin/bash
# Round-4 pass o: log-mel kernel at 5 and 6 waves per SIMD (__launch_bounds__ minimum; the
# compiler spills 36 / 51 VGPRs to reach them) against the shipped 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 120 ./tools/probes/logmel_variants_lb > $O/logmel_variants_lb.txt 2>&1 || { tail -5 $O/logmel_variants_lb.txt; exit 1; }
cat $O/logmel_variants_lb.txt
