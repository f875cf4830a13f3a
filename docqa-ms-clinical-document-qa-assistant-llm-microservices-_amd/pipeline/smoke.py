"""One tiny end-to-end QA step of the flagship stack on the GPU (used by
``__graft_entry__.smoke``): MiniLM embed -> flat kNN -> Llama-3-8B prefill + 4 decode
steps through the HIP-graph engine, all on the native kernels."""
from __future__ import annotations

import torch

from ..engine.llm_engine import SamplingParams
from ..text.synthetic import synthetic_questions
from .builder import StackConfig, build_stack


def run_smoke(device: str = "cuda", llm: str = "llama3-8b") -> dict:
    from .. import ops

    sc = StackConfig(llm=llm, n_notes=20, max_batch=2, max_context=1024)
    pipe, info = build_stack(sc, device=device)
    qs = synthetic_questions(2, seed=1)
    ans = pipe.answer_batch(qs, SamplingParams(max_new_tokens=4, stop_on_eos=False))
    assert len(ans) == 2 and all(len(a.sources) == 3 for a in ans)
    assert all(len(a.token_ids) == 4 for a in ans)
    if device != "cpu":
        torch.cuda.synchronize()
        assert ops.native_loaded(), "native kernels were not used"
    return {"sources": ans[0].sources, "tokens": ans[0].token_ids, **info}
