"""Worker for test_tp_gpu: one rank of a TP=N Llama on the 1-GPU box -- every rank on
cuda:0, gloo for the process group, the IPC all-reduce (one-shot / two-shot, residual +
RMSNorm fused) for the row-parallel projections.  Rank 0 saves the full (vocab-gathered)
prefill / decode logits; every rank saves the tokens of a HIP-graph-captured greedy
generation (they must agree across ranks)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch


def main():
    sd_path, out_path, preset, tp = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    torch.cuda.set_device(0)
    from docqa_amd import ops
    from docqa_amd.engine.kv_cache import KVCache
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.parallel import comm
    sys.path.insert(0, str(Path(__file__).resolve().parent))
    from test_models_gpu import _decode_logits, _prefill_logits

    assert ops.load_native()
    ps = comm.init_distributed(tp_size=tp, backend="gloo")
    car = comm.enable_custom_all_reduce(force=True)
    assert car is not None
    cfg = LlamaConfig.preset(preset)
    m = LlamaModel(cfg, device="cuda", init=False)
    m.load_state_dict_hf(torch.load(sd_path, weights_only=True))
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist() for n in (9, 130, 300)]
    BS = 64
    kv = KVCache(m.cfg.layers, 64, m.hkv, m.cfg.head_dim, BS).caches
    p, tables = _prefill_logits(m, kv, prompts, BS)
    d = _decode_logits(m, kv, prompts, tables, [5, 6, 7], BS)
    p, d = m.full_logits(p), m.full_logits(d)
    del kv
    # graph-captured greedy decode through the engine (fused LM-head argmax + packed-key pick)
    eng = LLMEngine(m, max_batch=8, max_context=512, use_graphs=True)
    gen_prompts = [torch.randint(0, cfg.vocab_size, (n,), generator=g).tolist() for n in (5, 17, 64, 100, 33, 8)]
    toks = eng.generate(gen_prompts, SamplingParams(max_new_tokens=8, stop_on_eos=False))
    torch.cuda.synchronize()
    # the longest any workgroup waited for a peer: ranks time-sliced on ONE GPU arrive far
    # apart (a peer's queue may not be mapped while this rank spins); printed for the log
    Path(f"{out_path}.wait{ps.rank}").write_text(str(car.max_wait_us()))
    car.check()
    torch.save(toks, f"{out_path}.tok{ps.rank}")
    if ps.rank == 0:
        torch.save({"prefill": p.float().cpu(), "decode": d.float().cpu()}, out_path)
    comm.destroy()


if __name__ == "__main__":
    main()
