#!/bin/bash
# Kernel + ROCTX marker trace of a short bench run, then the host spans around the largest
# GPU-idle gaps (scripts/gap_context.py).  Usage (via gpurun): bash scripts/prof_markers.sh [tag]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ROOT=$(pwd)
TAG=${1:-mk}
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DOCQA_TRACE=1 DOCQA_ROCTX=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace -d "$ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 3 --warmup 2 > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT"
KT=$(ls gpurun_out/prof_$TAG/*kernel_trace.csv | head -1)
MT=$(ls gpurun_out/prof_$TAG/*marker_api_trace.csv | head -1)
python scripts/gap_context.py "$KT" "$MT" --gaps ${GAPS:-4} --window-ms ${WINDOW_MS:-2300} --min-us 500 > gpurun_out/prof_${TAG}_gaps.txt 2>&1
head -1 "$KT" > gpurun_out/prof_${TAG}_kernel_columns.txt; rm -f gpurun_out/prof_$TAG/*kernel_trace.csv
head -60 gpurun_out/prof_${TAG}_gaps.txt
