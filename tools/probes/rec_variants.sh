# recurrence phase traces under the tuning knobs (diagnostic): default layout, 16x32, f32 arithmetic
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_base.txt 2>&1 || exit 1
CASR_REC_LAYOUT=16x32 timeout -k 10 200 python tools/rec_trace.py > gpurun_out/rt_1632.txt 2>&1 || exit 1
for f in base 1632; do echo "== $f"; grep -v amdgpu.ids gpurun_out/rt_$f.txt; done
