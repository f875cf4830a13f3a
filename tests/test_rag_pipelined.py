"""The pipelined RAG loop (side-stream embed/kNN, reservation on the prep thread,
launch-before-collect, collector thread) answers exactly what the plain sequential
``answer_batch`` loop answers, batch for batch.

Both loops see the same prefix-cache history (a batch's prefixes are registered at launch,
before the next batch reserves), so their kernels run on identical inputs and greedy token
streams compare exactly even for random-init weights (decode-GEMM autotuning is off: two
stacks could time their way to different tile configs).  The GPU case runs the full decode
path: native kernels, HIP graphs, grouped/split cascade decode, token-granular prefix
copies."""
import pytest
import torch


def _stack(llm, device):
    from docqa_amd.pipeline.builder import StackConfig, build_stack

    # a KV pool far larger than the three batches: with a tight pool the pipelined loop,
    # holding two batches while a third reserves, evicts cached prefixes at timing-
    # dependent moments, and a prefix recomputed at another prefill length rounds
    # differently (the sequential loop never holds more than one batch)
    sc = StackConfig(llm=llm, n_notes=60, max_batch=8, max_context=2048,
                     kv_mem_fraction=0.02 if device == "cuda" else None)
    pipe, _ = build_stack(sc, device=device, log=lambda *a: None)
    return pipe


def _check(llm, device, n_batches=3, bs=8, new=12):
    from docqa_amd.engine.llm_engine import SamplingParams
    from docqa_amd.text.synthetic import synthetic_questions

    qs = synthetic_questions(n_batches * bs, seed=3)
    batches = [qs[i * bs:(i + 1) * bs] for i in range(n_batches)]
    sp = SamplingParams(max_new_tokens=new, stop_on_eos=False)
    seq_pipe = _stack(llm, device)
    seq = [seq_pipe.answer_batch(b, sp) for b in batches]
    pl_pipe = _stack(llm, device)
    out = list(pl_pipe.answer_pipelined(batches, sp))
    assert len(out) == n_batches
    for bi, (ref, (ans, st, lat)) in enumerate(zip(seq, out)):
        bad = [(r, next(j for j, (x, y) in enumerate(zip(a.token_ids, b.token_ids)) if x != y))
               for r, (a, b) in enumerate(zip(ans, ref)) if a.token_ids != b.token_ids]
        assert not bad, f"batch {bi}: (row, first differing step) {bad}"
        assert [a.sources for a in ans] == [a.sources for a in ref]
        assert [a.answer for a in ans] == [a.answer for a in ref]
        assert lat > 0 and st.generate_s > 0
    for p in (seq_pipe, pl_pipe):
        eng = p.engine
        if device != "cpu":
            torch.cuda.synchronize()
        if eng.tail is not None:
            eng.tail.clear()
        assert eng.kv.allocator.num_free() == eng.kv.num_blocks   # every block returned
    # the shared chat prefix / retrieved notes were served from the prefix cache
    assert pl_pipe.engine.stats.cached_tokens == seq_pipe.engine.stats.cached_tokens > 0


def test_pipelined_matches_sequential_cpu(monkeypatch):
    monkeypatch.setenv("DOCQA_TUNE_DECODE", "0")
    _check("tiny", "cpu", new=4)


@pytest.mark.gpu
def test_pipelined_matches_sequential_gpu(monkeypatch):
    monkeypatch.setenv("DOCQA_TUNE_DECODE", "0")
    from docqa_amd import ops

    assert ops.load_native(build_if_missing=False)
    _check("llama3-1b-test", "cuda")
    assert ops.native_loaded()


def test_pipelined_with_pool_for_one_batch_cpu(monkeypatch):
    """KV pool that holds ONE batch (no prefix cache): the pipelined loop must not fail
    when batch i+1 cannot be reserved while batch i runs -- it collects batch i first
    (answer_pipelined MemoryError) -- and still answers like the sequential loop."""
    monkeypatch.setenv("DOCQA_TUNE_DECODE", "0")
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.text.synthetic import synthetic_questions

    bs, new, nb = 4, 4, 3
    qs = synthetic_questions(nb * bs, seed=5)
    batches = [qs[i * bs:(i + 1) * bs] for i in range(nb)]
    sp = SamplingParams(max_new_tokens=new, stop_on_eos=False)
    outs = []
    for mode in ("seq", "pipe"):
        pipe = _stack("tiny", "cpu")
        needs = []
        for b in batches:
            _, I = pipe.index.search(pipe.embed(b), pipe.k)
            prompts = pipe.build_prompts(b, I.tolist())
            needs.append(sum((len(p) + new + 63) // 64 for p in prompts))
        blocks = max(needs)
        assert 2 * min(needs) > blocks              # two batches never fit together
        pipe.engine = LLMEngine(pipe.engine.model, max_batch=bs, max_context=2048, use_graphs=False,
                                num_blocks=blocks, prefix_cache=False)
        if mode == "seq":
            outs.append([[a.token_ids for a in pipe.answer_batch(b, sp)] for b in batches])
        else:
            outs.append([[a.token_ids for a in ans] for ans, _, _ in pipe.answer_pipelined(batches, sp)])
        assert pipe.engine.kv.allocator.num_free() == blocks
    assert outs[0] == outs[1]
