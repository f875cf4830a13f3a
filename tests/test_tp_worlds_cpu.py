"""Tensor parallelism beyond 2 ranks on CPU (gloo): the Llama-3-70B GQA shape at toy
width (``test-tp8``: 32 query / 8 KV heads of 128) generated at TP = 4 and 8 and as TP = 4
x DP = 2, every configuration token-exact against the single-process model -- the same
column / row-parallel layers, fused residual + RMSNorm consumers of the row-parallel
all-reduces and packed-key vocab-parallel argmax the 8-GPU runs take over RCCL."""
import os
import socket

import torch
import torch.multiprocessing as mp

PROMPTS = [[1, 2, 3, 4, 5], list(range(7, 40)), [9] * 12 + [10, 11], list(range(100, 180))]
NEW = 6


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, tp, sd_path, out_path):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.parallel import comm

    ps = comm.init_distributed(tp_size=tp, backend="gloo")
    m = LlamaModel(LlamaConfig.preset("test-tp8"), device="cpu", dtype=torch.float32, init=False)
    m.load_state_dict_hf(torch.load(sd_path, weights_only=True))
    assert m.hq == 32 // tp and m.hkv == 8 // tp and m.lm_head.shape[0] % 256 == 0
    eng = LLMEngine(m, max_batch=4, max_context=256, block_size=16, use_graphs=False)
    mine = PROMPTS[ps.dp_rank::ps.dp_size]          # each DP replica serves its own requests
    out = eng.generate(mine, SamplingParams(max_new_tokens=NEW, stop_on_eos=False))
    if ps.tp_rank == 0:
        torch.save(out, f"{out_path}.{ps.dp_rank}")
    comm.destroy()


def _expected(tmp_path):
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.parallel import comm

    comm.destroy()
    ref = LlamaModel(LlamaConfig.preset("test-tp8"), device="cpu", dtype=torch.float32, seed=5)
    sd_path = tmp_path / "sd.pt"
    torch.save(ref.export_state_dict_hf(), sd_path)
    eng = LLMEngine(ref, max_batch=4, max_context=256, block_size=16, use_graphs=False)
    return sd_path, eng.generate(PROMPTS, SamplingParams(max_new_tokens=NEW, stop_on_eos=False))


def _run(tmp_path, world, tp):
    sd_path, expect = _expected(tmp_path)
    out = tmp_path / "out"
    mp.start_processes(_worker, args=(world, _free_port(), tp, str(sd_path), str(out)), nprocs=world,
                       join=True, start_method="spawn")
    dp = world // tp
    for d in range(dp):
        got = torch.load(f"{out}.{d}", weights_only=True)
        assert got == expect[d::dp], (world, tp, d)


def test_tp8_matches_single_process(tmp_path):
    _run(tmp_path, 8, 8)


def test_tp4_matches_single_process(tmp_path):
    _run(tmp_path, 4, 4)


def test_tp4_x_dp2_matches_single_process(tmp_path):
    _run(tmp_path, 8, 4)
