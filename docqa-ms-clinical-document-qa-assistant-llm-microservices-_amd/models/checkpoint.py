"""Hugging Face checkpoint IO for the generator and the encoders.

The reference downloads its weights through its runtimes (MiniLM from the HF hub inside
sentence-transformers, semantic-indexer/indexer.py:21; Mistral pulled by Ollama,
llm-qa/main.py:66-69).  Here a model name is either a preset (random-init weights of that
architecture -- no hub is reachable offline) or a local Hugging Face checkpoint
directory: ``config.json`` + ``model.safetensors`` or sharded
``model-0000x-of-0000y.safetensors`` with ``model.safetensors.index.json``.

Tensors are read lazily, one at a time (:class:`LazySafetensors`), and moved straight
to the GPU shard that needs them, so a 70B checkpoint (141 GB) never has to fit in host
RAM.  Only safetensors are read -- no pickle-based formats.
"""
from __future__ import annotations

import json
import os
from collections.abc import Mapping
from pathlib import Path

import torch

from ..ops import reference as ref
from .bert import BertConfig, BertEncoder, BertTokenClassifier
from .llama import LlamaConfig, LlamaModel


class LazySafetensors(Mapping):
    """Read-only mapping name -> tensor over the safetensors files of a checkpoint dir;
    each access opens the owning file and reads that tensor only."""

    def __init__(self, path):
        from safetensors import safe_open

        self._open = safe_open
        p = Path(path)
        idx = p / "model.safetensors.index.json"
        self._where: dict[str, Path] = {}
        if idx.exists():
            wm = json.loads(idx.read_text())["weight_map"]
            self._where = {k: p / f for k, f in wm.items()}
        else:
            files = sorted(p.glob("*.safetensors"))
            if not files:
                raise FileNotFoundError(f"no .safetensors files in {p}")
            for f in files:
                with safe_open(str(f), framework="pt") as h:
                    for k in h.keys():
                        self._where[k] = f

    def __getitem__(self, key: str) -> torch.Tensor:
        with self._open(str(self._where[key]), framework="pt") as h:
            return h.get_tensor(key)

    def __iter__(self):
        return iter(self._where)

    def __len__(self) -> int:
        return len(self._where)

    def __contains__(self, key) -> bool:
        return key in self._where


def is_checkpoint(name_or_path) -> bool:
    p = Path(str(name_or_path))
    return p.is_dir() and (p / "config.json").exists()


# --------------------------------------------------------------------------- Llama
# decoder families whose weights map 1:1 onto models/llama.py (Mistral-7B is the
# reference's generator, llm-qa/main.py:69; Llama-3 the BASELINE.json one)
SUPPORTED_DECODERS = ("llama", "mistral")


def llama_config_from_hf(hf: dict, name: str = "hf") -> LlamaConfig:
    """Hugging Face config.json -> :class:`LlamaConfig`.  Refuses what the decoder would
    otherwise load silently wrong: other model types (e.g. Qwen2 with q/k/v biases),
    ``attention_bias`` / ``mlp_bias``, and unsupported ``rope_scaling`` types."""
    mt = hf.get("model_type", "llama")
    if mt not in SUPPORTED_DECODERS:
        raise NotImplementedError(f"model_type {mt!r} is not supported (supported: {SUPPORTED_DECODERS})")
    for flag in ("attention_bias", "mlp_bias"):
        if hf.get(flag):
            raise NotImplementedError(f"{flag}=true checkpoints are not supported (no bias terms in the decoder)")
    if hf.get("hidden_act", "silu") not in ("silu", "swish"):
        raise NotImplementedError(f"hidden_act {hf['hidden_act']!r} is not supported (SwiGLU only)")
    scaling = hf.get("rope_scaling") or None
    if scaling is not None:
        ref.rope_inv_freq(8, 10000.0, scaling)   # raises on an unsupported type / missing keys
    heads = hf["num_attention_heads"]
    eos = hf.get("eos_token_id", 128009)
    if isinstance(eos, list):
        eos = eos[-1]
    return LlamaConfig(name=name, vocab_size=hf["vocab_size"], hidden=hf["hidden_size"],
                       intermediate=hf["intermediate_size"], layers=hf["num_hidden_layers"],
                       heads=heads, kv_heads=hf.get("num_key_value_heads", heads),
                       head_dim=hf.get("head_dim") or hf["hidden_size"] // heads,
                       rope_theta=float(hf.get("rope_theta", 10000.0)),
                       rms_eps=float(hf.get("rms_norm_eps", 1e-5)),
                       max_position=hf.get("max_position_embeddings", 8192),
                       bos_token_id=hf.get("bos_token_id", 128000), eos_token_id=eos,
                       rope_scaling=scaling, sliding_window=hf.get("sliding_window"))


def llama_config_to_hf(cfg: LlamaConfig) -> dict:
    return {"architectures": ["LlamaForCausalLM"], "model_type": "llama",
            "vocab_size": cfg.vocab_size, "hidden_size": cfg.hidden,
            "intermediate_size": cfg.intermediate, "num_hidden_layers": cfg.layers,
            "num_attention_heads": cfg.heads, "num_key_value_heads": cfg.kv_heads,
            "head_dim": cfg.head_dim, "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.rms_eps,
            "max_position_embeddings": cfg.max_position, "bos_token_id": cfg.bos_token_id,
            "eos_token_id": cfg.eos_token_id, "torch_dtype": "bfloat16", "tie_word_embeddings": False,
            "rope_scaling": cfg.rope_scaling, "attention_bias": False, "mlp_bias": False,
            "hidden_act": "silu"}


def load_llama(path, device="cuda", dtype=torch.bfloat16) -> LlamaModel:
    """LlamaForCausalLM checkpoint -> this rank's shard of :class:`LlamaModel` (TP from
    the current process groups)."""
    p = Path(path)
    cfg = llama_config_from_hf(json.loads((p / "config.json").read_text()), name=p.name)
    model = LlamaModel(cfg, device=device, dtype=dtype, init=False)
    model.load_state_dict_hf(LazySafetensors(p))
    return model


def save_llama(model: LlamaModel, path) -> None:
    """Write a TP=1 model as a Hugging Face checkpoint (config.json + model.safetensors)."""
    from safetensors.torch import save_file

    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    (p / "config.json").write_text(json.dumps(llama_config_to_hf(model.cfg), indent=1))
    save_file({k: v.contiguous() for k, v in model.export_state_dict_hf().items()},
              str(p / "model.safetensors"))


def resolve_llama_config(name_or_path) -> LlamaConfig:
    if is_checkpoint(name_or_path):
        p = Path(str(name_or_path))
        return llama_config_from_hf(json.loads((p / "config.json").read_text()), name=p.name)
    return LlamaConfig.preset(str(name_or_path))


def resolve_llama(name_or_path, device="cuda", seed: int = 0) -> LlamaModel:
    """A checkpoint directory -> its weights; a preset name -> random-init weights.
    ``DOCQA_LLM_DTYPE`` (bfloat16 | float32; default bfloat16): the weight / KV dtype --
    float32 for CPU rehearsals that compare TP = N against TP = 1 token for token (bf16
    rounds each TP split's sums differently, which flips near-tied greedy picks of a
    random-init model)."""
    dtype = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "float32": torch.float32,
             "fp32": torch.float32}[os.environ.get("DOCQA_LLM_DTYPE", "bfloat16")]
    if is_checkpoint(name_or_path):
        return load_llama(name_or_path, device=device, dtype=dtype)
    return LlamaModel(LlamaConfig.preset(str(name_or_path)), device=device, dtype=dtype, seed=seed)


# --------------------------------------------------------------------------- BERT
def bert_config_from_hf(hf: dict, name: str = "hf", pooling: str = "mean", normalize: bool = True,
                        max_seq_len: int = 256) -> BertConfig:
    return BertConfig(name=name, vocab_size=hf["vocab_size"], hidden=hf["hidden_size"],
                      layers=hf["num_hidden_layers"], heads=hf["num_attention_heads"],
                      intermediate=hf["intermediate_size"],
                      max_position=hf.get("max_position_embeddings", 512),
                      type_vocab=hf.get("type_vocab_size", 2), eps=float(hf.get("layer_norm_eps", 1e-12)),
                      pooling=pooling, normalize=normalize, max_seq_len=max_seq_len)


def _st_pooling(p: Path) -> tuple[str, bool]:
    """sentence-transformers layout: pooling mode from 1_Pooling/config.json, L2 norm if a
    Normalize module is listed (modules.json); plain BERT: mean + normalise."""
    pooling, normalize = "mean", True
    pc = p / "1_Pooling" / "config.json"
    if pc.exists():
        c = json.loads(pc.read_text())
        pooling = "cls" if c.get("pooling_mode_cls_token") else "mean"
    mods = p / "modules.json"
    if mods.exists():
        normalize = any("Normalize" in m.get("type", "") for m in json.loads(mods.read_text()))
    return pooling, normalize


def _bert_prefix(sd: Mapping) -> str:
    for pre in ("", "bert.", "model."):
        if pre + "embeddings.word_embeddings.weight" in sd:
            return pre
    raise KeyError("no BERT embeddings in the checkpoint")


def load_bert_encoder(path, device="cuda") -> BertEncoder:
    """BertModel / sentence-transformers checkpoint -> :class:`BertEncoder`."""
    p = Path(path)
    pooling, normalize = _st_pooling(p)
    cfg = bert_config_from_hf(json.loads((p / "config.json").read_text()), name=p.name,
                              pooling=pooling, normalize=normalize)
    enc = BertEncoder(cfg, device=device)
    sd = LazySafetensors(p)
    enc.load_state_dict_hf(sd, prefix=_bert_prefix(sd))
    return enc


def load_bert_token_classifier(path, labels: list[str], device="cuda", dtype=None) -> BertTokenClassifier:
    """BertForTokenClassification checkpoint (the NER de-identifier) ->
    :class:`BertTokenClassifier`; ``labels`` in the checkpoint's id2label order."""
    p = Path(path)
    hf = json.loads((p / "config.json").read_text())
    cfg = bert_config_from_hf(hf, name=p.name, pooling="cls", normalize=False, max_seq_len=512)
    if "id2label" in hf:
        labels = [hf["id2label"][str(i)] for i in range(len(hf["id2label"]))]
    if dtype is None:
        dtype = torch.bfloat16 if str(device).startswith("cuda") else torch.float32
    clf = BertTokenClassifier(cfg, labels, device=device, dtype=dtype)
    sd = LazySafetensors(p)
    clf.load_state_dict_hf(sd, prefix=_bert_prefix(sd))
    n = len(clf.labels)
    clf.cls_w[:n] = sd["classifier.weight"].to(device=clf.device, dtype=clf.dtype)
    clf.cls_b[:n] = sd["classifier.bias"].to(device=clf.device, dtype=clf.dtype)
    return clf


def resolve_bert_config(name_or_path) -> BertConfig:
    if is_checkpoint(name_or_path):
        p = Path(str(name_or_path))
        pooling, normalize = _st_pooling(p)
        return bert_config_from_hf(json.loads((p / "config.json").read_text()), name=p.name,
                                   pooling=pooling, normalize=normalize)
    return BertConfig.preset(str(name_or_path))


def resolve_bert(name_or_path, device="cuda", seed: int = 0) -> BertEncoder:
    if is_checkpoint(name_or_path):
        return load_bert_encoder(name_or_path, device=device)
    return BertEncoder(BertConfig.preset(str(name_or_path)), device=device, seed=seed)


def use_checkpoint_tokenizers(llm, embed) -> None:
    """Point the tokenizers at the checkpoints' own ``tokenizer.json`` (the chat BPE of the
    generator, the WordPiece vocab of the embedder) unless set explicitly."""
    import os

    for name, var in ((llm, "DOCQA_CHAT_TOKENIZER_JSON"), (embed, "DOCQA_WORDPIECE_JSON")):
        tj = tokenizer_json(name)
        if tj:
            os.environ.setdefault(var, tj)


def tokenizer_json(name_or_path) -> str | None:
    """tokenizer.json of a checkpoint directory, if present (for DOCQA_*_TOKENIZER_JSON)."""
    if is_checkpoint(name_or_path):
        f = Path(str(name_or_path)) / "tokenizer.json"
        if f.exists():
            return str(f)
    return None


__all__ = ["LazySafetensors", "is_checkpoint", "load_llama", "save_llama", "resolve_llama",
           "resolve_llama_config", "load_bert_encoder", "load_bert_token_classifier", "resolve_bert",
           "resolve_bert_config", "tokenizer_json", "use_checkpoint_tokenizers", "llama_config_from_hf", "bert_config_from_hf"]
