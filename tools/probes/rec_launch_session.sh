# CASR_OPT_REC_COOP: the chained ordinary launch (2, default) against the cooperative launch (1):
# recurrence parity tests, batches-in-flight tests, interleaved A/B serial and two in flight, and a
# rocprofv3 kernel trace of the default bench (its exit status recorded)
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/rec_launch}
mkdir -p $O
OUT=$O STAGES='tests' TESTS='tests/test_gpu_parity.py tests/test_gpu_pipeline.py' \
  TESTS_K='persistent or cooperative or pacing or in_flight or shard_decoder' bash tools/gpu_session.sh || exit $?
OUT=$O/s1 STAGES='ab' AB_ROUNDS=3 AB_OPTS='-;REC_COOP=1' AB_ARGS='--no-beam --streams 1' bash tools/gpu_session.sh || exit $?
OUT=$O/s2 STAGES='ab' AB_ROUNDS=3 AB_OPTS='-;REC_COOP=1' AB_ARGS='--streams 2 --beam-streams 2' bash tools/gpu_session.sh || exit $?
OUT=$O STAGES='prof' bash tools/gpu_session.sh
