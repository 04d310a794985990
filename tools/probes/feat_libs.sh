# rocprofv3 kernel stats of tools/probes/feat_probe.py for each library in $LIBS ("base" = the tree's)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out
L=chinese-asr_amd/casr
cp $L/libcasr_hip.so /tmp/casr_base.so
for n in $LIBS; do
  if [ "$n" = base ]; then cp /tmp/casr_base.so $L/libcasr_hip.so; else cp $L/$n $L/libcasr_hip.so; fi
  touch $L/libcasr_hip.so
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_$n -o fp -- python3 tools/probes/feat_probe.py > gpurun_out/fp_$n.log 2>&1 || { tail -3 gpurun_out/fp_$n.log; break; }
  echo "== $n"; grep -h "features" gpurun_out/fp_$n/*kernel_stats.csv | cut -d, -f1-4
done
cp /tmp/casr_base.so $L/libcasr_hip.so
touch $L/libcasr_hip.so
