"""Worker for test_tp_gpu: one rank of a TP=2 Llama (llama3-1b-test) on the 1-GPU box --
both ranks on cuda:0, gloo for the process group, the one-shot IPC all-reduce for the
per-layer TP all-reduces.  Rank 0 saves the full (vocab-gathered) logits."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch


def main():
    sd_path, out_path = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)
    from docqa_amd import ops
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.parallel import comm
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from test_models_gpu import _decode_logits, _prefill_logits

    assert ops.load_native()
    comm.init_distributed(tp_size=2, backend="gloo")
    car = comm.enable_custom_all_reduce(force=True)
    assert car is not None
    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", init=False)
    m.load_state_dict_hf(torch.load(sd_path, weights_only=True))
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, 32000, (n,), generator=g).tolist() for n in (9, 130, 300)]
    BS = 64
    kv = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    p, tables = _prefill_logits(m, kv, prompts, BS)
    d = _decode_logits(m, kv, prompts, tables, [5, 6, 7], BS)
    p, d = m.full_logits(p), m.full_logits(d)
    torch.cuda.synchronize()
    car.check()
    if comm.state().rank == 0:
        torch.save({"prefill": p.float().cpu(), "decode": d.float().cpu()}, out_path)
    comm.destroy()


if __name__ == "__main__":
    main()
