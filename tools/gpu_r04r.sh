#!/bin/bash
# Round-4 pass r: greedy attention prologue with the bulk loads held behind a first barrier (the
# tree) against the previous order (headattn): the -m gpu suite on the tree, greedy phase traces of
# both, interleaved bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
L=chinese-asr_amd/casr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cp $L/libcasr_hip.so /tmp/casr_base.so
restore() { cp /tmp/casr_base.so $L/libcasr_hip.so; touch $L/libcasr_hip.so; }
use() { case $1 in base*) cp /tmp/casr_base.so $L/libcasr_hip.so;; *) cp $L/libcasr_hip_$1.so $L/libcasr_hip.so;; esac; touch $L/libcasr_hip.so; }
for n in base headattn; do
  use $n
  timeout -k 10 150 python tools/probes/dg_trace.py > $O/greedy_$n.txt 2>&1 || { tail -5 $O/greedy_$n.txt; restore; exit 1; }
  echo "== $n"; grep -A10 "^attention (greedy)" $O/greedy_$n.txt
done
for n in headattn base headattn base headattn base; do
  use $n
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-beam --no-configs --no-cpu-baseline --no-f32-compare > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; restore; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', round(d['ms_per_step'],3), d['device_ms_per_step']['median'], d['kernel_breakdown_ms']['attention'])"
done
restore
