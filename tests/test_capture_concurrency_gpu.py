"""Decode-graph capture beside a busy second thread (the llm-qa service shape: the
scheduler thread captures a batch bucket lazily while the front end's prep thread embeds,
searches and copies results to the host on its own stream).  The capture must neither be
invalidated by the other thread's syncs nor fail them, and the graphs must replay the
eager tokens."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_capture_while_other_thread_syncs():
    from docqa_amd import ops
    from docqa_amd.engine.llm_engine import LLMEngine, SamplingParams
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    assert ops.load_native()
    m = LlamaModel(LlamaConfig.preset("llama3-1b-test"), device="cuda", seed=3)
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(3, 30000, (n,), generator=g).tolist() for n in (7, 40, 90, 130, 65)]
    params = SamplingParams(max_new_tokens=6, stop_on_eos=False)
    ref = LLMEngine(m, max_batch=8, max_context=512, use_graphs=False).generate(prompts, params)

    stop, errors = threading.Event(), []

    def busy():
        s = torch.cuda.Stream()
        x = torch.randn(4096, 256, device="cuda")
        try:
            with torch.cuda.stream(s):
                while not stop.is_set():
                    y = (x @ x.t()).sum(1)
                    y.tolist()                      # a device -> host sync, as I.tolist() in qa.py
        except Exception as e:                      # noqa: BLE001 -- reported below
            errors.append(e)

    t = threading.Thread(target=busy)
    t.start()
    try:
        eng = LLMEngine(m, max_batch=8, max_context=512, use_graphs=True)
        out = eng.generate(prompts, params)          # captures the bucket's graph lazily
    finally:
        stop.set()
        t.join(timeout=60)
    assert not errors, errors
    assert out == ref
