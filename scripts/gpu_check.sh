#!/bin/bash
# Round-1 GPU check: build, kernel numerics, generator probe, rocprof summary.
# Every GPU step has its own time limit; stop at the first fault/abort/timeout.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -c "from __graft_entry__ import build; build()" > gpurun_out/build.log 2>&1 || exit 3
if [ "$SKIP_PYTEST" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$KBENCH_ARGS" ]; then
  timeout -k 10 600 python benchmarks/bench_kernels.py $KBENCH_ARGS > gpurun_out/kbench.log 2>&1
  rc=$?; echo "kbench rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROBE_ARGS" ]; then
  timeout -k 10 600 python scripts/gen_probe.py $PROBE_ARGS > gpurun_out/gen_probe.log 2>&1
  rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 900 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 600 python -c "from __graft_entry__ import smoke; smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$PROF_ARGS" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/${PROF_SCRIPT:-scripts/gen_probe.py}" $PROF_ARGS > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "prof rc=$rc"
  rm -f "$GRAFT_REPO_ROOT"/gpurun_out/prof/*kernel_trace.csv
fi
exit 0
