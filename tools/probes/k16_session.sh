# The fused beam select at k = 16 (CELL 4 with 8 rows per block): its parity tests, then BASELINE
# config 5 (beam 16 + second pass) timed with the select fused (default) and as launches
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/k16}
mkdir -p $O
OUT=$O STAGES='tests' TESTS='tests/test_gpu_parity.py tests/test_gpu_select_paths.py tests/test_gpu_scale.py' \
  TESTS_K='select_in_attention or fused_select or config5' bash tools/gpu_session.sh || exit $?
for r in 1 2; do for o in "" "FUSE_SELECT=0"; do
  CASR_OPTS="$o" timeout -k 10 400 python bench.py --no-beam --no-f32-compare --no-cpu-baseline > $O/b.json 2> $O/err.txt || exit $?
  python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); c=d['config5_beam16_lm']; print('[$r] opts=$o config5', round(c['ms_per_batch'], 2), 'host', round(c['host_ms_per_batch_rank0'], 2), 'config4', round(d['config4_beam8_sharded']['ms_per_batch'], 2))"
done; done
