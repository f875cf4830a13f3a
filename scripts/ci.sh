#!/bin/bash
# CI entry point -- the equivalent of the reference's Jenkinsfile (venv -> install ->
# pytest with junit + coverage -> quality gate; Jenkinsfile:18-102), for this repo:
#   1. build the gfx950 HIP extension in-tree (hipcc cross-compiles without a GPU);
#   2. run the CPU suite with a JUnit report and the line-coverage gate (scripts/covgate.py);
#   3. on a machine with an MI355X (or with DOCQA_CI_GPU=1), the GPU suite as well.
# Reports land in ci_out/ (junit-cpu.xml, coverage.xml, junit-gpu.xml).
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p ci_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
COV_MIN=${DOCQA_COV_MIN:-70}
python -c "import __graft_entry__ as g; g.build()" > ci_out/build.log 2>&1 || { tail -40 ci_out/build.log; exit 1; }
PYTHONPATH=scripts python -m pytest tests -m "not gpu" -q -p covgate \
  --junitxml=ci_out/junit-cpu.xml --docqa-cov-min "$COV_MIN" --docqa-cov-xml ci_out/coverage.xml
if [ "${DOCQA_CI_GPU:-0}" = "1" ] || python -c "import torch,sys; sys.exit(0 if torch.cuda.is_available() else 1)"; then
  python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --junitxml=ci_out/junit-gpu.xml
fi
echo "CI passed"
