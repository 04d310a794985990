# recurrence phase traces under the workgroup-layout knob (diagnostic)
cd $GRAFT_REPO_ROOT
for L in 1 2 3; do  # 32x16 16x32 16x16
  CASR_OPTS=REC_LAYOUT=$L timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_$L.txt 2>&1 || exit 1
  echo "== $L"; grep -v amdgpu.ids gpurun_out/rt_$L.txt
done
