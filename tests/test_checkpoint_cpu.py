"""Hugging Face checkpoint IO (models/checkpoint.py): a Llama model written as
config.json + safetensors (single file and sharded with an index) loads back to the same
logits; a BERT / sentence-transformers layout and a token-classification head map onto
the encoder kernels' layout.  Random tiny models on CPU (no hub is reachable)."""
import json

import torch


def _llama_logits(model, ids):
    from docqa_amd.models.llama import AttnMeta

    T = len(ids)
    meta = AttnMeta(prefill=True, positions=torch.arange(T, dtype=torch.int32),
                    slot_mapping=torch.arange(T, dtype=torch.int32),
                    cu_seqlens=torch.tensor([0, T], dtype=torch.int32), max_len=T)
    shape = (1, model.hkv, 64, model.cfg.head_dim)
    caches = [(torch.zeros(shape, dtype=model.dtype), torch.zeros(shape, dtype=model.dtype))
              for _ in model.layers]
    return model.forward(torch.tensor(ids, dtype=torch.int32), meta, caches)


def test_llama_roundtrip_single_and_sharded(tmp_path):
    from safetensors.torch import save_file

    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    m = LlamaModel(LlamaConfig.preset("tiny"), device="cpu", seed=3)
    ids = [1, 17, 230, 4000, 9, 77]
    ref = _llama_logits(m, ids)
    ck.save_llama(m, tmp_path / "one")
    assert ck.is_checkpoint(tmp_path / "one")
    m1 = ck.resolve_llama(tmp_path / "one", device="cpu")
    assert m1.cfg.layers == m.cfg.layers and m1.cfg.kv_heads == m.cfg.kv_heads
    assert torch.equal(_llama_logits(m1, ids), ref)
    # sharded layout: two files + model.safetensors.index.json
    sd = m.export_state_dict_hf()
    keys = sorted(sd)
    half = len(keys) // 2
    d = tmp_path / "sharded"
    d.mkdir()
    (d / "config.json").write_text((tmp_path / "one" / "config.json").read_text())
    parts = {"model-00001-of-00002.safetensors": keys[:half], "model-00002-of-00002.safetensors": keys[half:]}
    for f, ks in parts.items():
        save_file({k: sd[k].contiguous() for k in ks}, str(d / f))
    (d / "model.safetensors.index.json").write_text(json.dumps(
        {"weight_map": {k: f for f, ks in parts.items() for k in ks}}))
    lazy = ck.LazySafetensors(d)
    assert len(lazy) == len(sd) and "model.norm.weight" in lazy
    m2 = ck.load_llama(d, device="cpu")
    assert torch.equal(_llama_logits(m2, ids), ref)
    # preset names still give random-init architectures
    assert ck.resolve_llama_config("tiny").hidden == 256


def _bert_hf_state(enc, prefix=""):
    sd = {prefix + "embeddings.word_embeddings.weight": enc.wte,
          prefix + "embeddings.position_embeddings.weight": enc.wpe,
          prefix + "embeddings.token_type_embeddings.weight": enc.wtt,
          prefix + "embeddings.LayerNorm.weight": enc.emb_g, prefix + "embeddings.LayerNorm.bias": enc.emb_b}
    H = enc.cfg.hidden
    for i, L in enumerate(enc.layers):
        p = f"{prefix}encoder.layer.{i}."
        for j, n in enumerate(("query", "key", "value")):
            sd[p + f"attention.self.{n}.weight"] = L["qkv_w"][j * H:(j + 1) * H]
            sd[p + f"attention.self.{n}.bias"] = L["qkv_b"][j * H:(j + 1) * H]
        sd.update({p + "attention.output.dense.weight": L["o_w"], p + "attention.output.dense.bias": L["o_b"],
                   p + "attention.output.LayerNorm.weight": L["ln1_g"], p + "attention.output.LayerNorm.bias": L["ln1_b"],
                   p + "intermediate.dense.weight": L["up_w"], p + "intermediate.dense.bias": L["up_b"],
                   p + "output.dense.weight": L["down_w"], p + "output.dense.bias": L["down_b"],
                   p + "output.LayerNorm.weight": L["ln2_g"], p + "output.LayerNorm.bias": L["ln2_b"]})
    return {k: v.contiguous().clone() for k, v in sd.items()}


def _bert_hf_config(cfg):
    return {"vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden, "num_hidden_layers": cfg.layers,
            "num_attention_heads": cfg.heads, "intermediate_size": cfg.intermediate,
            "max_position_embeddings": cfg.max_position, "type_vocab_size": cfg.type_vocab,
            "layer_norm_eps": cfg.eps}


def test_sentence_transformers_encoder_layout(tmp_path):
    from safetensors.torch import save_file

    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.bert import BertConfig, BertEncoder

    cfg = BertConfig.preset("tiny-bert")
    enc = BertEncoder(cfg, device="cpu", seed=5)
    d = tmp_path / "minilm"
    d.mkdir()
    (d / "config.json").write_text(json.dumps(_bert_hf_config(cfg)))
    (d / "modules.json").write_text(json.dumps([{"type": "sentence_transformers.models.Transformer"},
                                                {"type": "sentence_transformers.models.Pooling"},
                                                {"type": "sentence_transformers.models.Normalize"}]))
    (d / "1_Pooling").mkdir()
    (d / "1_Pooling" / "config.json").write_text(json.dumps({"pooling_mode_mean_tokens": True}))
    save_file(_bert_hf_state(enc), str(d / "model.safetensors"))
    got = ck.resolve_bert(d, device="cpu")
    assert got.cfg.pooling == "mean" and got.cfg.normalize
    toks = [[2, 100, 200, 3], [2, 55, 3]]
    assert torch.allclose(got.encode(toks), enc.encode(toks))


def test_token_classifier_head_and_labels(tmp_path):
    from safetensors.torch import save_file

    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.bert import BertConfig, BertTokenClassifier

    cfg = BertConfig.preset("tiny-bert")
    labels = ["O", "B-PERSON", "I-PERSON", "B-DATE_TIME"]
    clf = BertTokenClassifier(cfg, labels, device="cpu", seed=7)
    d = tmp_path / "ner"
    d.mkdir()
    hf = _bert_hf_config(cfg)
    hf["id2label"] = {str(i): lab for i, lab in enumerate(labels)}
    (d / "config.json").write_text(json.dumps(hf))
    sd = _bert_hf_state(clf, prefix="bert.")
    sd["classifier.weight"] = clf.cls_w[:len(labels)].clone()
    sd["classifier.bias"] = clf.cls_b[:len(labels)].clone()
    save_file(sd, str(d / "model.safetensors"))
    got = ck.load_bert_token_classifier(d, ["unused"], device="cpu")
    assert got.labels == labels
    toks = [[2, 100, 200, 300, 3]]
    assert got.predict(toks) == clf.predict(toks)


def test_stack_runs_from_checkpoint_directories(tmp_path):
    """build_stack with LLM / embedder given as checkpoint directories (what a user with real
    weights passes via LLM_MODEL / EMBED_MODEL) answers a question end to end."""
    from safetensors.torch import save_file

    from docqa_amd.engine.llm_engine import SamplingParams
    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.bert import BertConfig, BertEncoder
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.pipeline.builder import StackConfig, build_stack

    ck.save_llama(LlamaModel(LlamaConfig.preset("tiny"), device="cpu", seed=1), tmp_path / "llm")
    cfg = BertConfig.preset("tiny-bert")
    d = tmp_path / "emb"
    d.mkdir()
    (d / "config.json").write_text(json.dumps(_bert_hf_config(cfg)))
    save_file(_bert_hf_state(BertEncoder(cfg, device="cpu", seed=2)), str(d / "model.safetensors"))
    pipe, info = build_stack(StackConfig(llm=str(tmp_path / "llm"), embed=str(d), n_notes=8, max_batch=4,
                                         max_context=2048, use_graphs=False), device="cpu", log=lambda *a: None)
    assert pipe.engine.model.cfg.name == "llm" and pipe.encoder.cfg.hidden == cfg.hidden
    ans = pipe.answer_batch(["Quelle plante pour le syndrome ?"], SamplingParams(max_new_tokens=4, stop_on_eos=False))
    assert len(ans) == 1 and len(ans[0].token_ids) == 4 and len(ans[0].sources) == 3


def test_llama3_rope_scaling_inv_freq_closed_form():
    """Llama-3.1 rope_scaling (type llama3) against the closed-form per-frequency rule."""
    import math

    from docqa_amd.ops import reference as ref

    sc = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
          "original_max_position_embeddings": 8192}
    got = ref.rope_inv_freq(128, 500000.0, sc)
    for i, g in enumerate(got.tolist()):
        f = 500000.0 ** (-(2 * i) / 128)
        wl = 2 * math.pi / f
        if wl < 8192 / 4.0:
            want = f                       # high frequency: kept
        elif wl > 8192 / 1.0:
            want = f / 8.0                 # low frequency: divided by factor
        else:
            s = (8192 / wl - 1.0) / (4.0 - 1.0)
            want = (1 - s) * f / 8.0 + s * f
        assert abs(g - want) <= 1e-12 * max(1.0, abs(want)), (i, g, want)
    # the scaled table differs from the plain one only in the low/medium bands
    plain = ref.rope_inv_freq(128, 500000.0)
    assert torch.equal(got[:20], plain[:20]) and not torch.equal(got, plain)
    assert torch.allclose(ref.rope_inv_freq(64, 1e4, {"type": "linear", "factor": 2.0}),
                          ref.rope_inv_freq(64, 1e4) / 2)
    cs = ref.rope_cos_sin(16, 128, 500000.0, scaling=sc)
    assert torch.allclose(cs[5, 64:], torch.sin(5 * got).float())


def test_llama_config_from_hf_refuses_unsupported():
    import pytest

    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.llama import LlamaConfig

    base = ck.llama_config_to_hf(LlamaConfig.preset("tiny"))
    cfg = ck.llama_config_from_hf(dict(base, rope_scaling={"rope_type": "llama3", "factor": 32.0,
                                                            "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                                            "original_max_position_embeddings": 8192}))
    assert cfg.rope_scaling["factor"] == 32.0
    # Mistral (the reference's generator) loads; its sliding window is recorded
    m = ck.llama_config_from_hf(dict(base, model_type="mistral", sliding_window=4096))
    assert m.sliding_window == 4096
    for bad in (dict(base, model_type="qwen2"), dict(base, attention_bias=True), dict(base, mlp_bias=True),
                dict(base, rope_scaling={"rope_type": "yarn", "factor": 4.0}), dict(base, hidden_act="gelu")):
        with pytest.raises(NotImplementedError):
            ck.llama_config_from_hf(bad)


def test_engine_refuses_context_beyond_sliding_window():
    import pytest

    from docqa_amd.engine.llm_engine import LLMEngine
    from docqa_amd.models.llama import LlamaConfig, LlamaModel

    cfg = LlamaConfig.preset("tiny")
    cfg.sliding_window = 256
    model = LlamaModel(cfg, device="cpu", seed=0)
    with pytest.raises(ValueError):
        LLMEngine(model, max_batch=2, max_context=512, use_graphs=False)
    LLMEngine(model, max_batch=2, max_context=256, use_graphs=False)


def test_rope_scaled_checkpoint_round_trip(tmp_path):
    """A llama3-scaled checkpoint round-trips and the model uses the scaled table."""
    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.llama import LlamaConfig, LlamaModel
    from docqa_amd.ops import reference as ref

    cfg = LlamaConfig.preset("tiny")
    cfg.rope_scaling = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                        "high_freq_factor": 4.0, "original_max_position_embeddings": 64}
    ck.save_llama(LlamaModel(cfg, device="cpu", seed=1), tmp_path / "m")
    got = ck.load_llama(tmp_path / "m", device="cpu")
    assert got.cfg.rope_scaling == cfg.rope_scaling
    want = ref.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, scaling=cfg.rope_scaling)
    assert torch.equal(got.cos_sin, want)


def test_mistral_preset_matches_hf_config():
    """The reference's generator (ChatOllama(model="mistral"), llm-qa/main.py:69) as a preset:
    the Mistral-7B v0.3 HF config.json maps onto exactly LlamaConfig.preset("mistral-7b")."""
    from docqa_amd.models import checkpoint as ck
    from docqa_amd.models.llama import LlamaConfig

    hf = {"architectures": ["MistralForCausalLM"], "model_type": "mistral", "vocab_size": 32768,
          "hidden_size": 4096, "intermediate_size": 14336, "num_hidden_layers": 32, "num_attention_heads": 32,
          "num_key_value_heads": 8, "head_dim": 128, "rope_theta": 1000000.0, "rms_norm_eps": 1e-05,
          "max_position_embeddings": 32768, "bos_token_id": 1, "eos_token_id": 2, "sliding_window": None,
          "hidden_act": "silu", "tie_word_embeddings": False}
    got = ck.llama_config_from_hf(hf)
    want = LlamaConfig.preset("mistral-7b")
    for f in ("vocab_size", "hidden", "intermediate", "layers", "heads", "kv_heads", "head_dim", "rope_theta",
              "rms_eps", "max_position", "bos_token_id", "eos_token_id", "sliding_window"):
        assert getattr(got, f) == getattr(want, f), f
    assert 7.0e9 < want.num_params() < 7.5e9
