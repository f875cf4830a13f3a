"""Rehearse the driver's bench.py contract on CPU: single process and a 2-rank torchrun
(gloo) with the index sharded across ranks, tiny models.  Checks the one-JSON-line output
and its required keys, so the round-end multi-GPU scaling run cannot fail on plumbing."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}
ARGS = ["--device", "cpu", "--llm", "tiny", "--embed", "tiny-bert", "--notes", "8", "--batch", "3",
        "--max-new-tokens", "3", "--steps", "2", "--warmup", "1", "--max-context", "1024"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _last_json(out: str) -> dict:
    lines = [l for l in out.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_single_process_cpu():
    env = dict(os.environ, WORLD_SIZE="1")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", *ARGS], cwd=ROOT,
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d) and d["n_gpus"] == 1 and d["value"] > 0
    assert "retrieval_check" not in d          # one GPU: no sharded index to verify


def test_bench_two_ranks_gloo_sharded_index():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--gpus", "2", *ARGS]            # WORLD_SIZE > 1: the retrieval check runs by default
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 6 and d["config"]["parallelism"] == "dp2"
    assert d["retrieval_check"] == {"rows": 3, "k": 3, "bad_rows_max_over_ranks": 0}


def test_bench_eight_ranks_gloo_sharded_index():
    """The driver's 8-GPU scaling command shape (torchrun --nproc-per-node 8 bench.py --gpus 8)
    rehearsed on gloo: 8 data-parallel ranks, the index sharded x8 (all-gather of queries and
    top-k), MAX-over-ranks timing, one JSON line with the whole-job aggregate."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--gpus", "8", *ARGS]            # the driver's exact command: self-verifying by default
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 24 and d["config"]["parallelism"] == "dp8"
    assert d["value"] > 0 and d["workload"]["unique_question_frac"] == 1.0
    assert d["retrieval_check"]["bad_rows_max_over_ranks"] == 0
    assert d["retrieval_check"]["rows"] == 3


def test_pipeline_bench_tp2_gloo_sharded_index():
    """Config-5 pipeline benchmark (ingest -> deid -> embed -> sharded kNN -> TP generate)
    as 2 gloo ranks: TP=2 generator, index sharded over both ranks with replicated queries."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           str(ROOT / "benchmarks" / "bench_pipeline.py"), "--device", "cpu", "--llm", "tiny",
           "--embed", "tiny-bert", "--ner", "tiny-bert", "--notes", "24", "--batch", "3",
           "--steps", "1", "--warmup", "1", "--max-new-tokens", "3", "--max-context", "1024"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "tp2" and d["value"] > 0
    assert d["ingest_docs_per_sec"] > 0 and d["config"]["index"] == "flat-L2 sharded x2"


def test_pipeline_bench_tp8_gloo_replicated_index():
    """Config 5 at its real parallel shape: 8 ranks, TP=8 over the 70B GQA layout at toy
    width (test-tp8), index sharded over all 8 ranks with replicated queries."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           str(ROOT / "benchmarks" / "bench_pipeline.py"), "--device", "cpu", "--llm", "test-tp8",
           "--embed", "tiny-bert", "--ner", "tiny-bert", "--notes", "24", "--batch", "2",
           "--steps", "1", "--warmup", "1", "--max-new-tokens", "2", "--max-context", "1024"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=1200, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "tp8" and d["value"] > 0
    assert d["config"]["index"] == "flat-L2 sharded x8"


def test_serving_bench_through_service_launcher():
    """bench_serving's default entry: the services launcher in a child process group
    (TP 2 under torchrun, gloo), Poisson arrivals over HTTP POST /ask/."""
    env = dict(os.environ, PYTHONPATH=str(ROOT))
    cmd = [sys.executable, str(ROOT / "benchmarks" / "bench_serving.py"), "--entry", "launch", "--tiny",
           "--device", "cpu", "--requests", "16", "--warmup", "4", "--rate", "20", "--max-new-tokens", "6",
           "--max-batch", "8", "--modes", "continuous", "--notes", "40", "--gpus", "2", "--tp", "2",
           "--port-offset", str(21000 + os.getpid() % 5000)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["errors"] == 0 and out["requests"] == 16 and out["tp"] == 2
    assert out["entry"].startswith("services.launch") and out["p50_latency_ms"] > 0
    assert "steady_state_qps" in out and out["steady_window_s"] >= 0
