#!/bin/bash
# end-of-round-6 evidence on one box: rocprofv3 kernel stats of the headline (for the roofline
# table; only the stats CSV is kept), then the headline at the driver's settings, batch 1 and
# the reference template
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/final
[ "${PROFILE_ONLY:-0}" = 1 ] && out=gpurun_out/final_prof
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 1 > $out/prof_bench.log 2>&1 || { tail -20 $out/prof_bench.log; exit 1; }
find /tmp/prof -name "*kernel_stats.csv" -exec cp {} $out/ \;
ls $out
[ "${PROFILE_ONLY:-0}" = 1 ] && exit 0
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/head.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 1 --steps 5 --warmup 2 > $out/b1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --template reference --steps 5 --warmup 2 > $out/ref.log 2>&1 || exit 1
grep -h '"metric"' $out/head.log $out/b1.log $out/ref.log | cut -c1-160
