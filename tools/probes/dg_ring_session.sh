# Greedy fused GEMM ring depth (CASR_DG_GREEDY_S builds: 32-deep stages on a ring of S buffers
# instead of 64-deep on three): interleaved library A/B, then the parity tests of the greedy fold
# on the S = 6 build
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/dg_ring}
mkdir -p $O
OUT=$O LIBS="base s6 s5" AB_ROUNDS=2 AB_ARGS="--no-beam --streams 1" timeout -k 10 600 bash tools/probes/ab_libs.sh > $O/ablibs.log 2>&1 || { tail -5 $O/ablibs.log; exit 1; }
cat $O/ablibs.log
L=chinese-asr_amd/casr
cp $L/libcasr_hip.so /tmp/casr_base_keep.so
cp $L/libcasr_hip_s6.so $L/libcasr_hip.so && touch $L/libcasr_hip.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_fullbatch.py tests/test_gpu_parity.py -k "headline_greedy or fold or ksplit or greedy_golden" > $O/tests_s6.log 2>&1
rc=$?
cp /tmp/casr_base_keep.so $L/libcasr_hip.so && touch $L/libcasr_hip.so
tail -3 $O/tests_s6.log
exit $rc
