#!/bin/bash
# Interleaved A/B of library builds on one box: for each round, each name in $LIBS ("base" = the
# tree's build, else chinese-asr_amd/casr/libcasr_hip_<name>.so) replaces libcasr_hip.so and runs
# bench.py $AB_ARGS; one summary line per run (tools/bench_line.py).  Restores the base build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/ablibs}
mkdir -p $O
L=chinese-asr_amd/casr
cp $L/libcasr_hip.so /tmp/casr_base.so
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for n in ${LIBS:-base}; do
    if [ "$n" = base ]; then cp /tmp/casr_base.so $L/libcasr_hip.so; else cp $L/libcasr_hip_$n.so $L/libcasr_hip.so; fi
    touch $L/libcasr_hip.so
    timeout -k 10 300 python bench.py --steps ${AB_STEPS:-10} --warmup 3 --no-configs --no-cpu-baseline --no-f32-compare \
      ${AB_ARGS} > $O/ab_${n}_$r.json 2> $O/ab.err || { tail -5 $O/ab.err; cp /tmp/casr_base.so $L/libcasr_hip.so; exit 1; }
    echo -n "[$r] $n: "; python tools/bench_line.py $O/ab_${n}_$r.json
  done
done
cp /tmp/casr_base.so $L/libcasr_hip.so
touch $L/libcasr_hip.so
