# Round-end evidence on one box: bench line (with the CPU baseline), rocprofv3 kernel stats of
# a short bench, PMC passes of one greedy step, recurrence phase trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
python tools/prof_by_grid.py $O/prof/run_kernel_trace.csv 30 > $O/prof_by_grid.txt 2>&1
head -14 $O/prof_by_grid.txt
bash tools/probes/pmc_passes.sh || exit 1
python tools/pmc_summary.py $O/pmc --json $O/pmc_traffic.json > $O/pmc_summary.txt 2>&1
head -16 $O/pmc_summary.txt
timeout -k 10 300 python tools/rec_trace.py > $O/rec_trace.txt 2>&1 && grep -v amdgpu.ids $O/rec_trace.txt
