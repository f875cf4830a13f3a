#!/bin/bash
# kernel trace of the llm-qa service under Poisson 320 q/s (overload): GPU occupancy of the
# continuous-batching loop (scripts/serve_trace.py)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 700 python -u "$ROOT/benchmarks/bench_serving.py" --entry launch --rate 320 --requests 1200 --max-batch 256 \
  --modes continuous --server-log "$ROOT/gpurun_out/r3c_serve_prof_srv.log" \
  --launch-prefix "rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/prof_serve -o run --output-format csv --" \
  > "$ROOT/gpurun_out/r3c_serve_prof.log" 2>&1; rc=$?
cd "$ROOT"; tail -c 800 gpurun_out/r3c_serve_prof.log; [ $rc -eq 0 ] || exit $rc
sleep 5
TR=$(ls gpurun_out/prof_serve/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$TR" ] || { echo "no trace"; ls -R gpurun_out/prof_serve | head; exit 1; }
python scripts/serve_trace.py "$TR" --trim-s 0.5 --top 45 --skip-tuning > gpurun_out/r3c_serve_trace.txt && python scripts/serve_trace.py "$TR" --trim-s 0 --top 8 > gpurun_out/r3c_serve_trace_all.txt; cat gpurun_out/r3c_serve_trace.txt; head -12 gpurun_out/r3c_serve_trace_all.txt
python - "$TR" <<'PY' > gpurun_out/r3c_serve_pids.txt
import csv, sys, collections
c = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    c[(r.get('Process_Id') or r.get('Pid') or '?', r['Kernel_Name'][:60])] += 1
for k, v in c.most_common(40):
    print(v, k)
PY
ls -la gpurun_out/prof_serve; python - "$TR" <<'PY'
import csv, gzip, sys
w = gzip.open("gpurun_out/prof_serve/kernels_min.csv.gz", "wt")
for r in csv.DictReader(open(sys.argv[1])):
    w.write(f"{r['Start_Timestamp']},{r['End_Timestamp']},{r['Kernel_Name'][:48]}\n")
w.close()
PY
ls -la gpurun_out/prof_serve; rm -f gpurun_out/prof_serve/*kernel_trace.csv
