# serving A/B: admission batching vs mixed prefill/decode steps at small
# token budgets, reference prompt over HTTP, offered 60 and 100 q/s
set -o pipefail
mkdir -p gpurun_out
run() {
  tag=$1; shift
  env "$@" timeout -k 10 420 python -u benchmarks/bench_serving.py --rate 60,100 --requests 1500 --max-batch 256 \
      --ignore-eos --modes continuous --server-log gpurun_out/srv_$tag.log > gpurun_out/serve_$tag.log 2>&1 || return 1
  echo "== $tag"; grep -h '^{' gpurun_out/serve_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    if 'offered_rate' in d:
        print(d['offered_rate'], d['value'], d['p50_latency_ms'], d['p90_latency_ms'], d.get('scheduler', {}).get('steps'))"
}
run base DOCQA_MIXED_PREFILL=0 || exit 1
run mixed512 DOCQA_MIXED_PREFILL=1 DOCQA_CHUNK_TOKENS=512 || exit 1
run mixed1024 DOCQA_MIXED_PREFILL=1 DOCQA_CHUNK_TOKENS=1024 || exit 1
