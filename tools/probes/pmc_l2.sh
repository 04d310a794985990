# L2 hit / miss and fabric read counters per kernel (one pass each), for $ONE_STEP_ENV (e.g.
# "B=128 BEAM=8"); summaries under gpurun_out/pmcl2
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmcl2
mkdir -p $O
export $ONE_STEP_ENV
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/h -o h -- python3 $R/tools/probes/one_step.py > $O/h.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum --output-format csv -d $O/r -o r -- python3 $R/tools/probes/one_step.py > $O/r.log 2>&1
echo rc=$?
