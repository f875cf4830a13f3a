"""IPC all-reduce (csrc/kernels/allreduce.hip): one-shot and two-shot, bf16 partials and
fp32 split-K slabs, plain and with the fused residual + RMSNorm, against the fp32
reference, + HIP-graph replay -- at 2 and 4 ranks.  On the 1-GPU box every rank shares
cuda:0 and reaches the others' staging through HIP IPC, which checks the protocol (flags,
call epochs, double buffering, column chunks); xGMI timing needs a multi-GPU node."""
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


@pytest.mark.parametrize("world", [2, 4])
def test_custom_all_reduce(world):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0",
               GPU_MAX_HW_QUEUES="1", DOCQA_AR_MAX_WG="32",   # ranks share one GPU: keep every rank's queue resident
               DOCQA_AR_TIMEOUT_MS=os.environ.get("DOCQA_AR_TIMEOUT_MS", "20000"))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tests" / "custom_ar_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.count(" ok") == world
