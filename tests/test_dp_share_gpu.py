"""The data-parallel headline path on GPU kernels, rehearsed on the one-GPU box: bench.py
under torchrun with two ranks that both bind cuda:0 (``--share-gpu``, gloo process group).
Each rank holds a full generator replica and one shard of the flat index; the sharded kNN
all-gathers every rank's top-k, the timing bracket is barrier + synchronize on both sides
and the MAX over ranks -- the same code the driver's 8-GPU scaling run executes with one
GPU per rank over RCCL."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 8])
def test_bench_dp_shared_gpu(world):
    """bench.py's DP path (the driver's --gpus N command) with every rank on cuda:0: the
    sharded index's per-batch all-gathers run on the IPC peer-memory gather, at the default
    wait bound, and the sharded retrieval equals an unsharded flat search."""
    # default gather bound (DOCQA_SHARD_GATHER_TIMEOUT_MS): no test-only override
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0",
               GPU_MAX_HW_QUEUES="1", DOCQA_AR_MAX_WG="32")   # ranks share one GPU: keep every rank's queue resident
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "DOCQA_AR_TIMEOUT_MS", "DOCQA_SHARD_GATHER_TIMEOUT_MS"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--gpus", str(world), "--share-gpu", "--llm", "llama3-1b-test", "--batch", "16", "--max-new-tokens", "8",
           "--steps", "2", "--warmup", "1", "--notes", "200", "--kv-mem-fraction", "0.02",
           "--check-retrieval"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=420, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == world and out["config"]["parallelism"] == f"dp{world}"
    assert out["config"]["global_batch"] == 16 * world and out["value"] > 0
    assert "IPC all-gather unavailable" not in r.stdout + r.stderr
    assert out["workload"]["unique_question_frac"] == 1.0
    # every rank's sharded top-3 (IPC gathers + merge) equals one unsharded exact search
    assert out["retrieval_check"]["rows"] == 16 and out["retrieval_check"]["bad_rows_max_over_ranks"] == 0
