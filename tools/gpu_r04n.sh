#!/bin/bash
# Round-4 pass n: recurrence pacing re-sweep on the round-4 code (CASR_OPT_REC_SLEEP x
# CASR_OPT_REC_POLL_GAP, two interleaved rounds; defaults 1 / 2), greedy bench line only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
for rnd in 1 2; do
  for sl in 0 1 2; do
    for gp in 1 2 3; do
      n=s${sl}g${gp}r${rnd}
      CASR_OPTS=REC_SLEEP=$sl,REC_POLL_GAP=$gp timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-beam --no-configs \
        --no-cpu-baseline --no-f32-compare > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
      python -c "import json; d=json.load(open('$O/b_$n.json')); print('$n', round(d['ms_per_step'],3), d['device_ms_per_step']['median'], d['kernel_breakdown_ms']['rec_step'], d['roofline'].get('avg_launch_us'))"
    done
  done
done
