# Kernel-trace timelines of the greedy headline: one batch in flight and two, the
# ordinary recurrence launch (REC_COOP=0: a cooperative launch ends in SIGSEGV under rocprofv3)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/timeline}
mkdir -p $O
for n in 1 2; do
  CASR_OPTS=REC_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/s$n -o run -- \
    python3 bench.py --steps 20 --warmup 2 --streams $n --no-beam --no-configs --no-f32-compare --no-cpu-baseline \
    > $O/bench_s$n.json 2> $O/s$n.err || exit $?
  python tools/pipeline_timeline.py $O/s$n/run_kernel_trace.csv --window ${WINDOW:-120} > $O/timeline_s$n.txt
  cat $O/timeline_s$n.txt
done
