#!/bin/bash
# same-box A/B of decode knobs on the unique-question headline (bench.py defaults, 6 timed steps);
# a knob value the code rejects (Python exception, rc 1) is logged and skipped; any other failure
# (fault, abort, time limit) ends the script
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/r3d_knob_ab.log
: > $out
run() {
  echo "== $*" >> $out
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 --steps 6 --warmup 2 > gpurun_out/r3d_knob_last.log 2>&1
  rc=$?
  tail -1 gpurun_out/r3d_knob_last.log | python3 -c "import sys,json
try:
  d=json.loads(sys.stdin.read()); print('   q/s %.2f  p50 %.0f ms  prefill %.1f  decode %.1f' % (d['value'], d['p50_latency_ms'], d['engine_ms_per_batch']['prefill'], d['engine_ms_per_batch']['decode']))
except Exception as e: print('   no JSON', e)" >> $out
  echo "   rc=$rc" >> $out
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run BASE=1
run DOCQA_MID_WG_CAP=256
run DOCQA_MID_WG_CAP=192
run DOCQA_GROUP_TILES=8
run DOCQA_GROUP_TILES=16
run DOCQA_LM_HEAD_CFG=5
run DOCQA_PIPELINE_LEAD=2
run DOCQA_GROUP_DEFER=1
run BASE=2
cat $out
