# decode-GEMM phase traces (dg_trace.py, beam) for ablation builds: each name in $LIBS
# (files in chinese-asr_amd/casr/) replaces libcasr_hip.so in turn; "base" = the tree's build
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=chinese-asr_amd/casr
cp $L/libcasr_hip.so /tmp/casr_base.so
for n in $LIBS; do
  if [ "$n" = base ]; then cp /tmp/casr_base.so $L/libcasr_hip.so; else cp $L/$n $L/libcasr_hip.so; fi
  touch $L/libcasr_hip.so
  echo "== $n"
  BEAM=1 timeout -k 10 150 python tools/probes/dg_trace.py > gpurun_out/dgd_$n.txt 2>&1 || { tail -5 gpurun_out/dgd_$n.txt; cp /tmp/casr_base.so $L/libcasr_hip.so; exit 1; }
  grep -A5 "^dec_lstm (beam)\|^proj (beam)\|^dec_lstm (greedy)\|^proj (greedy)" gpurun_out/dgd_$n.txt | grep "beam\|greedy\|k loop\|block "
done
cp /tmp/casr_base.so $L/libcasr_hip.so
touch $L/libcasr_hip.so
