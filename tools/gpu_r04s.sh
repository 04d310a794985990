#!/bin/bash
# Round-4 pass s: the fused image's gate tiles aligned to a whole wave column (pad, the tree) against
# HEAD (head): the -m gpu suite on the tree, step-20 fused-GEMM traces by block kind, interleaved
# bench runs (greedy + beam lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
L=chinese-asr_amd/casr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cp $L/libcasr_hip.so /tmp/casr_base.so
restore() { cp /tmp/casr_base.so $L/libcasr_hip.so; touch $L/libcasr_hip.so; }
use() { cp $L/libcasr_hip_$1.so $L/libcasr_hip.so; touch $L/libcasr_hip.so; }
for n in pad head; do
  use $n
  CASR_DG_TRACE_STEP=20 NTN=14 BEAM=1 BB=256 K=8 timeout -k 10 150 python tools/probes/dg_trace.py > $O/beam_$n.txt 2>&1 || { tail -5 $O/beam_$n.txt; restore; exit 1; }
  echo "== $n"; grep -A12 "^proj (beam)" $O/beam_$n.txt | grep -v "start\|prologue\|first"
done
for n in head pad head pad head pad; do
  use $n
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-configs --no-cpu-baseline --no-f32-compare > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; restore; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$n.json')); b=d['beam']; print('$n greedy', round(d['ms_per_step'],3), d['kernel_breakdown_ms']['proj'], '| beam', round(b['ms_per_step'],3), b['kernel_breakdown_ms']['proj'], b['device_ms_per_step']['median'])"
done
restore
