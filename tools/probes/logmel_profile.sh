#!/bin/bash
# log-mel front end at B = 256 x 8 s: HIP-event line, rocprofv3 kernel trace + stats, PMC
# FETCH_SIZE / WRITE_SIZE passes (gpurun_out/logmel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/logmel
mkdir -p $O
timeout -k 10 200 python tools/probes/logmel_probe.py > $O/line.json 2> $O/line.err || { tail -5 $O/line.err; exit 1; }
cat $O/line.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/probes/logmel_probe.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep -h "log_mel" $O/prof/run_kernel_stats.csv | cut -d, -f1-8
export ITERS=2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p2 -o p2 -- python3 tools/probes/logmel_probe.py > $O/p2.log 2>&1 || { tail -3 $O/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p3 -o p3 -- python3 tools/probes/logmel_probe.py > $O/p3.log 2>&1 || { tail -3 $O/p3.log; exit 1; }
python3 - <<'PY'
import csv, glob
for tag in ("p2", "p3"):
    for f in glob.glob(f"gpurun_out/logmel/{tag}/*counter_collection.csv"):
        vals = {}
        for r in csv.DictReader(open(f)):
            if "log_mel" in r.get("Kernel_Name", ""):
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        for k, v in vals.items():
            print(tag, k, "per launch (KB, mean of", len(v), "):", round(sum(v) / len(v), 1))
PY
