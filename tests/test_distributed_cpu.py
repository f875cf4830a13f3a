"""Multi-process distributed paths on CPU (gloo, world_size 2), as the GPU runs use them
over RCCL: tensor-parallel Llama forward (column/row-parallel layers + all-reduce +
vocab-parallel LM head) and the sharded vector index (all-gather queries, local search,
all-gather top-k, merge)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port, tp):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    from docqa_amd.parallel import comm

    return comm.init_distributed(tp_size=tp, backend="gloo")


def _tp_worker(rank, world, port, sd_path, out_path):
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.parallel import comm

    _init(rank, world, port, tp=world)
    torch.manual_seed(0)
    cfg = LlamaConfig.preset("tiny")
    m = LlamaModel(cfg, device="cpu", dtype=torch.float32, init=False)
    m.load_state_dict_hf(torch.load(sd_path, weights_only=True))
    eng = LLMEngine(m, max_batch=4, max_context=128, block_size=16, use_graphs=False)
    out = eng.generate([[1, 2, 3, 4, 5], list(range(7, 40))], SamplingParams(max_new_tokens=6, stop_on_eos=False))
    if rank == 0:
        torch.save(out, out_path)
    comm.destroy()


def test_tensor_parallel_matches_single_process(tmp_path):
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.parallel import comm

    comm.destroy()
    cfg = LlamaConfig.preset("tiny")
    ref = LlamaModel(cfg, device="cpu", dtype=torch.float32, seed=11)
    sd = ref.export_state_dict_hf()
    sd_path, out_path = tmp_path / "sd.pt", tmp_path / "out.pt"
    torch.save(sd, sd_path)
    eng = LLMEngine(ref, max_batch=4, max_context=128, block_size=16, use_graphs=False)
    expect = eng.generate([[1, 2, 3, 4, 5], list(range(7, 40))], SamplingParams(max_new_tokens=6, stop_on_eos=False))
    mp.start_processes(_tp_worker, args=(2, _free_port(), str(sd_path), str(out_path)), nprocs=2,
                       join=True, start_method="spawn")
    assert torch.load(out_path, weights_only=True) == expect


def _shard_worker(rank, world, port, data_path, out_path):
    from docqa_amd.index.flat import FlatIndex
    from docqa_amd.index.sharded import ShardedFlatIndex
    from docqa_amd.parallel import comm

    _init(rank, world, port, tp=1)
    d = torch.load(data_path, weights_only=True)
    xb, xq = d["xb"], d["xq"]
    n = xb.shape[0]
    lo, hi = n * rank // world, n * (rank + 1) // world
    local = FlatIndex(xb.shape[1], "l2", device="cpu")
    local.add(xb[lo:hi])
    idx = ShardedFlatIndex(local)
    assert idx.ntotal == n and idx.id_offset == lo
    myq = xq[rank::world]                     # uneven query counts per rank
    D, I = idx.search(myq, 5)
    torch.save({"D": D, "I": I}, f"{out_path}.{rank}")
    comm.destroy()


def test_sharded_index_matches_flat(tmp_path):
    from docqa_amd.index.flat import FlatIndex

    g = torch.Generator().manual_seed(0)
    xb = torch.randn(1001, 32, generator=g)
    xq = torch.randn(7, 32, generator=g)
    data, out = tmp_path / "d.pt", tmp_path / "o"
    torch.save({"xb": xb, "xq": xq}, data)
    mp.start_processes(_shard_worker, args=(2, _free_port(), str(data), str(out)), nprocs=2,
                       join=True, start_method="spawn")
    full = FlatIndex(32, "l2", device="cpu")
    full.add(xb)
    for r in range(2):
        got = torch.load(f"{out}.{r}", weights_only=True)
        D, I = full.search(xq[r::2], 5)
        assert torch.equal(got["I"], I)
        torch.testing.assert_close(got["D"], D, rtol=1e-4, atol=1e-4)
