set -o pipefail
mkdir -p gpurun_out
for t in 512 128 64 32; do
  DOCQA_DECODE_WG_TARGET=$t timeout -k 10 240 python -u bench.py --batch 1 --steps 3 --warmup 1 > gpurun_out/b1_wg$t.log 2>&1 || exit 1
  echo "wg $t: $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/b1_wg$t.log) $(grep -o '"decode": [0-9.]*' gpurun_out/b1_wg$t.log)"
done
