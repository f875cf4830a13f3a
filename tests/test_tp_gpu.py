"""Tensor-parallel Llama on GPU kernels (TP=2 and TP=4, every rank on the 1-GPU box's
cuda:0): column/row-parallel projections on the decode / prefill GEMM kernels, the IPC
all-reduce with the residual + RMSNorm fused (one-shot at decode, two-shot at prefill),
vocab-parallel logits and the packed-key greedy pick -- must match the TP=1 model's
prefill and decode logits, and every rank must generate the same tokens."""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("preset,tp", [("llama3-1b-test", 2), ("test-tp8", 4)])
def test_tp_matches_tp1(tmp_path, preset, tp):
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from test_models_gpu import _decode_logits, _prefill_logits, _rel

    from docqa_amd import ops
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    assert ops.load_native()
    cfg = LlamaConfig.preset(preset)
    m = LlamaModel(cfg, device="cuda", seed=9)
    sd_path, out_path = tmp_path / "sd.pt", tmp_path / "out.pt"
    torch.save(m.export_state_dict_hf(), sd_path)
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist() for n in (9, 130, 300)]
    kv = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, 64).caches
    p1, tables = _prefill_logits(m, kv, prompts, 64)
    d1 = _decode_logits(m, kv, prompts, tables, [5, 6, 7], 64)
    del m, kv
    torch.cuda.empty_cache()
    # every rank shares cuda:0.  With HIP's default 4 hardware queues per process, 4 ranks
    # oversubscribe the GPU's queue slots: the scheduler leaves a rank's queue unmapped while
    # the others' all-reduce kernels spin on it, so that rank "never arrives" (round 3's
    # spin-limit hits; round 4: rank 0 absent > 30 s at the first call, profiles/
    # r4_ar_skew_default_hwq_tp4_fail.txt).  One queue per process keeps every rank resident:
    # the longest peer wait drops to ~35 ms (profiles/r4_ar_skew_hwq1_tp.log).  Rarely a
    # shared-GPU rank still stalls for > 2 s (one failure in five suites, rank 0 at its 4th
    # call), so the bound here is 20 s; one process per GPU keeps the 500 ms default.
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", GPU_MAX_HW_QUEUES="1", DOCQA_AR_MAX_WG="32",
               DOCQA_AR_TIMEOUT_MS=os.environ.get("DOCQA_AR_TIMEOUT_MS", "20000"))
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(tp),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "tests" / "tp_gpu_worker.py"),
           str(sd_path), str(out_path), preset, str(tp)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    if r.returncode != 0:
        # the workers' tracebacks sit in the middle of torchrun's output: keep all of it
        dump = ROOT / "gpurun_out" / f"tp_gpu_worker_{preset}_{tp}.log"
        dump.parent.mkdir(exist_ok=True)
        dump.write_text(r.stdout + "\n---- stderr ----\n" + r.stderr)
        errs = [ln for ln in r.stderr.splitlines() if "Error" in ln or "error" in ln]
        raise AssertionError(f"torchrun rc {r.returncode}; error lines: {errs[:12]}; full log: {dump}")
    out = torch.load(out_path, weights_only=True)
    assert _rel(out["prefill"], p1.float().cpu()) < 0.03
    assert _rel(out["decode"], d1.float().cpu()) < 0.03
    waits = [int(Path(f"{out_path}.wait{r}").read_text()) for r in range(tp)]
    print(f"[tp{tp} {preset}] longest peer wait per rank (us): {waits}", flush=True)
    toks = [torch.load(f"{out_path}.tok{r}", weights_only=True) for r in range(tp)]
    assert all(t == toks[0] for t in toks[1:])
    assert all(0 <= x < cfg.vocab_size for row in toks[0] for x in row)
