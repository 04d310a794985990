# Round-4 evidence on one box (profiles/r04): PMC passes of two greedy steps and of two beam 8
# B = 256 steps, a kernel trace of three beam 8 B = 256 steps, then (last) the rocprofv3 kernel
# trace + stats of a greedy-only bench run on the shipped default launch.
# The PMC and beam-trace runs use the ordinary recurrence launch (CASR_OPTS=REC_COOP=0: the same
# kernel, grid and code; only the launch API differs): a process that made a cooperative launch ends
# in SIGSEGV under rocprofv3 after its results are written (ROCm teardown, reproduced without casr
# code by tools/probes/coop_exit_probe.hip), and no GPU step may follow a SIGSEGV in
# one call, so the cooperative (default) run is the last step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
R=$GRAFT_REPO_ROOT
export CASR_OPTS=REC_COOP=0
for mode in greedy beam; do
  P=$O/pmc_$mode
  mkdir -p $P
  if [ $mode = beam ]; then export BEAM=8 B=256; else unset BEAM; export B=256; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $P/p1 -o p1 -- python3 $R/tools/probes/one_step.py > $P/p1.log 2>&1 || { tail -3 $P/p1.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/p2 -o p2 -- python3 $R/tools/probes/one_step.py > $P/p2.log 2>&1 || { tail -3 $P/p2.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/p3 -o p3 -- python3 $R/tools/probes/one_step.py > $P/p3.log 2>&1 || { tail -3 $P/p3.log; exit 1; }
done
unset BEAM
python tools/pmc_summary.py $O/pmc_greedy --json $O/pmc_traffic.json > $O/pmc_summary.txt 2>&1
python tools/pmc_summary.py $O/pmc_beam --json $O/pmc_traffic_beam.json > $O/pmc_summary_beam.txt 2>&1
head -14 $O/pmc_summary.txt
head -14 $O/pmc_summary_beam.txt
STEPS=3 BEAM=8 B=256 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_beam -o run -- \
  python3 $R/tools/probes/one_step.py > $O/prof_beam.log 2>&1 || { tail -5 $O/prof_beam.log; exit 1; }
python tools/prof_by_grid.py $O/prof_beam/run_kernel_trace.csv 30 > $O/prof_beam_by_grid.txt 2>&1
head -12 $O/prof_beam_by_grid.txt
unset CASR_OPTS
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 bench.py --steps 20 --warmup 2 --no-beam --no-configs --no-f32-compare --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo "rocprofv3 kernel trace of the default (cooperative) launch: exit status $?" | tee $O/prof_rc.txt
python tools/prof_by_grid.py $O/prof/run_kernel_trace.csv 30 > $O/prof_by_grid.txt 2>&1
head -12 $O/prof_by_grid.txt
