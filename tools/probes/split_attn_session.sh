# Split-T greedy attention at B = 32 (CASR_OPT_ATTN_SPLIT): phase traces per split count, then an
# interleaved A/B of the split counts on the config-2 bench line
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/split}
mkdir -p $O
for s in ${SPLITS_TRACE:-0 2 4 8}; do
  CASR_OPTS=ATTN_SPLIT=$s B=32 timeout -k 10 200 python tools/probes/dg_trace.py > $O/trace_b32_s$s.txt 2>&1 || exit $?
  head -12 $O/trace_b32_s$s.txt | tail -11
done
OUT=$O STAGES='ab' AB_ROUNDS=${AB_ROUNDS:-2} AB_OPTS="${AB_OPTS:-ATTN_SPLIT=0;ATTN_SPLIT=2;ATTN_SPLIT=3;ATTN_SPLIT=4;ATTN_SPLIT=8}" \
  AB_ARGS='--batch 32 --no-beam --streams 1' bash tools/gpu_session.sh
