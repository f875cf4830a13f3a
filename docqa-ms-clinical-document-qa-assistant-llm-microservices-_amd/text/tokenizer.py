"""Offline tokenizers.

No Hugging Face hub is reachable, so both tokenizers are trained (with the Rust
``tokenizers`` library) on the deterministic synthetic clinical corpus and cached under
``build/tokenizers``:

  * :func:`wordpiece` -- BERT WordPiece (lower-cased, like all-MiniLM-L6-v2's
    ``bert-base-uncased`` vocab), ids < 30522, [CLS] ... [SEP] framing;
  * :func:`chat_bpe` -- byte-level BPE with Llama-3 chat special tokens
    (``<|begin_of_text|>``, ``<|start_header_id|>``, ``<|end_header_id|>``,
    ``<|eot_id|>``), mapped onto the ids the random-init Llama-3 model uses.

When real tokenizer files exist (``DOCQA_WORDPIECE_JSON`` / ``DOCQA_CHAT_TOKENIZER_JSON``)
they are loaded instead.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors, trainers

_CACHE = Path(__file__).resolve().parents[2] / "build" / "tokenizers"
# trained vocabularies shipped with the package: the WordPiece trainer is not deterministic
# across processes (tie order), so a box that trained its own vocabulary tokenised -- and
# retrieved, and prompted -- differently from the next; every box now loads these
_ASSETS = Path(__file__).resolve().parent / "assets"
_lock = threading.Lock()
_instances: dict = {}

CHAT_SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>",
                 "<|end_header_id|>", "<|eot_id|>", "<|pad|>"]


def _train_wordpiece(vocab_size: int) -> Tokenizer:
    from .synthetic import corpus_text

    tok = Tokenizer(models.WordPiece(unk_token="[UNK]"))
    tok.normalizer = normalizers.BertNormalizer(lowercase=True, strip_accents=False)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tok.decoder = decoders.WordPiece()
    tr = trainers.WordPieceTrainer(vocab_size=vocab_size, min_frequency=1,
                                   special_tokens=["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"])
    tok.train_from_iterator(corpus_text(), tr)
    cls, sep = tok.token_to_id("[CLS]"), tok.token_to_id("[SEP]")
    tok.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
        special_tokens=[("[CLS]", cls), ("[SEP]", sep)])
    return tok


def _train_bpe(vocab_size: int) -> Tokenizer:
    from .synthetic import corpus_text

    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab_size, min_frequency=2, special_tokens=CHAT_SPECIALS,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus_text(), tr)
    return tok


def _cached(name: str, env: str, train, vocab_size: int) -> Tokenizer:
    with _lock:
        key = (name, vocab_size)
        if key in _instances:
            return _instances[key]
        path = os.environ.get(env)
        if path and Path(path).exists():
            tok = Tokenizer.from_file(path)
        elif (_ASSETS / f"{name}-{vocab_size}.json").exists():
            tok = Tokenizer.from_file(str(_ASSETS / f"{name}-{vocab_size}.json"))
        else:
            f = _CACHE / f"{name}-{vocab_size}.json"
            if f.exists():
                tok = Tokenizer.from_file(str(f))
            else:
                tok = train(vocab_size)
                _CACHE.mkdir(parents=True, exist_ok=True)
                tmp = f.with_suffix(f".tmp{os.getpid()}")
                tok.save(str(tmp))
                os.replace(tmp, f)
        _instances[key] = tok
        return tok


class WordPieceTokenizer:
    def __init__(self, vocab_size: int = 30522, max_len: int = 256):
        self.tok = _cached("wordpiece", "DOCQA_WORDPIECE_JSON", _train_wordpiece, vocab_size)
        self.max_len = max_len

    @property
    def vocab_size(self) -> int:
        return self.tok.get_vocab_size()

    def encode(self, text: str) -> list[int]:
        ids = self.tok.encode(text).ids
        if len(ids) > self.max_len:  # keep [CLS] ... truncated ... [SEP]
            ids = ids[: self.max_len - 1] + ids[-1:]
        return ids

    def encode_batch(self, texts: list[str]) -> list[list[int]]:
        out = []
        for e in self.tok.encode_batch(texts):
            ids = e.ids
            if len(ids) > self.max_len:
                ids = ids[: self.max_len - 1] + ids[-1:]
            out.append(ids)
        return out


class ChatTokenizer:
    """Byte-level BPE with Llama-3 chat framing.  Special tokens are remapped onto the
    Llama-3 special-id range (128000+) so the model config keeps Llama-3's ids."""

    LLAMA3_SPECIAL = {"<|begin_of_text|>": 128000, "<|end_of_text|>": 128001,
                      "<|start_header_id|>": 128006, "<|end_header_id|>": 128007,
                      "<|eot_id|>": 128009, "<|pad|>": 128004}

    def __init__(self, vocab_size: int = 32000, model_vocab: int = 128256):
        self.tok = _cached("chatbpe", "DOCQA_CHAT_TOKENIZER_JSON", _train_bpe, vocab_size)
        self.model_vocab = model_vocab
        self._to_model = {}
        self._from_model = {}
        for s, mid in self.LLAMA3_SPECIAL.items():
            tid = self.tok.token_to_id(s)
            if tid is not None and model_vocab >= 128256:
                self._to_model[tid] = mid
                self._from_model[mid] = tid
        self.n = self.tok.get_vocab_size()

    def special(self, name: str) -> int:
        tid = self.tok.token_to_id(name)
        return self._to_model.get(tid, tid)

    @property
    def eos_id(self) -> int:
        return self.special("<|eot_id|>")

    def encode(self, text: str) -> list[int]:
        return [self._to_model.get(i, i) for i in self.tok.encode(text).ids]

    def encode_many(self, texts: list[str]) -> list[list[int]]:
        """:meth:`encode` of many texts in one ``encode_batch`` call (parallel in the Rust
        tokenizer); identical ids."""
        tm = self._to_model
        return [[tm.get(i, i) for i in e.ids] for e in self.tok.encode_batch(list(texts))]

    def chat_prompt(self, user: str, system: str | None = None) -> list[int]:
        s = self.special
        ids = [s("<|begin_of_text|>")]
        if system:
            ids += [s("<|start_header_id|>")] + self.encode("system") + [s("<|end_header_id|>")]
            ids += self.encode("\n\n" + system) + [s("<|eot_id|>")]
        ids += [s("<|start_header_id|>")] + self.encode("user") + [s("<|end_header_id|>")]
        ids += self.encode("\n\n" + user) + [s("<|eot_id|>")]
        ids += [s("<|start_header_id|>")] + self.encode("assistant") + [s("<|end_header_id|>")]
        ids += self.encode("\n\n")
        return ids

    def chat_messages(self, messages: list[dict]) -> list[int]:
        """Llama-3 framing of a whole conversation (Ollama /api/chat ``messages``: role
        system / user / assistant / tool, content) ending in the assistant header, so the
        model continues as the assistant.  One user message (+ optional system first) gives
        exactly :meth:`chat_prompt`'s ids."""
        s = self.special
        ids = [s("<|begin_of_text|>")]
        for m in messages:
            ids += [s("<|start_header_id|>")] + self.encode(str(m.get("role", "user"))) + [s("<|end_header_id|>")]
            ids += self.encode("\n\n" + str(m.get("content", ""))) + [s("<|eot_id|>")]
        ids += [s("<|start_header_id|>")] + self.encode("assistant") + [s("<|end_header_id|>")]
        ids += self.encode("\n\n")
        return ids

    def decode(self, ids: list[int]) -> str:
        keep = []
        for i in ids:
            if i in self._from_model:
                continue  # drop special tokens
            if 0 <= i < self.n:
                keep.append(i)
        return self.tok.decode(keep)

    def encode_batch_chat(self, users: list[str]) -> list[list[int]]:
        """chat_prompt for many user turns: the user texts are tokenised in one
        ``encode_batch`` call (parallel in the Rust tokenizer) and the constant framing
        tokens once -- identical ids to per-prompt :meth:`chat_prompt`."""
        if not users:
            return []
        s = self.special
        head = [s("<|begin_of_text|>"), s("<|start_header_id|>")] + self.encode("user") + [s("<|end_header_id|>")]
        tail = ([s("<|eot_id|>"), s("<|start_header_id|>")] + self.encode("assistant")
                + [s("<|end_header_id|>")] + self.encode("\n\n"))
        m = self._to_model
        bodies = [[m.get(i, i) for i in e.ids] for e in self.tok.encode_batch(["\n\n" + u for u in users])]
        return [head + b + tail for b in bodies]
