"""One-shot IPC all-reduce (csrc/kernels/allreduce.hip): 2 ranks x many sizes x 12
iterations (double-buffer parity, device-side epochs) + HIP-graph replay.  On the 1-GPU
box both ranks share cuda:0 and reach each other's staging through HIP IPC, which checks
the protocol (flags, epochs, slicing); xGMI cache behaviour needs a multi-GPU node."""
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


def test_custom_all_reduce_two_ranks():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tests" / "custom_ar_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.count(" ok") == 2
