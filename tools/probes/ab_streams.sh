cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/r06af
for r in 1 2 3; do for n in 2 3; do
  timeout -k 10 300 python bench.py --no-beam --no-configs --no-f32-compare --no-cpu-baseline --streams $n > gpurun_out/r06af/s${n}_$r.json 2> gpurun_out/r06af/err.txt || exit $?
  echo -n "[$r] streams=$n "; python tools/bench_line.py gpurun_out/r06af/s${n}_$r.json | cut -c1-40
done; done
