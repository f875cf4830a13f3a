"""Llama-3 decoder (8B / 70B / test sizes) for the llm-qa generator.

MI355X-first layout:
  * fused projections: one [(Hq + 2*Hkv)*D, H] QKV GEMM and one [2I, H] gate|up GEMM
    per layer, all on the hand-written MFMA GEMMs (prefill: pgemm.hip 256 x 256 with SwiGLU
    in the gate|up epilogue; decode: dgemm.hip <= 192 rows, mgemm.hip 193..512 rows, split-K
    fp32 slabs consumed by the fused RoPE + KV-cache write and residual + RMSNorm kernels;
    the LM head with the greedy argmax fused in at every bucket);
  * the residual stream is updated inside the fused add+RMSNorm kernel, so each layer
    costs 2 GEMM-epilogue-free passes over the hidden state instead of 4;
  * attention reads Q/K/V straight out of the packed QKV buffer (prefill: MFMA flash
    kernel; decode: paged split-K GQA kernel over a [blocks, Hkv, BS, D] cache);
  * tensor parallelism is Megatron-style: column-parallel QKV / gate|up, row-parallel
    O / down followed by one all-reduce each (RCCL over xGMI), vocab-parallel LM head
    whose argmax is resolved with a [B, 2] all-gather instead of gathering logits;
  * with 288 GB of HBM per GPU the 8B model (16 GB bf16) is replicated per GPU (TP=1,
    request-level data parallel) and 70B (140 GB) runs TP=8 (17.6 GB/GPU).

Weights are random-initialised on the device (no checkpoints are reachable offline);
``models/checkpoint.py`` loads Hugging Face Llama checkpoints (safetensors) when one is
available: pass the checkpoint directory wherever a preset name is accepted.

Reference parity: replaces the Ollama/llama.cpp Mistral-7B generator behind
``ChatOllama(model="mistral", temperature=0)`` (llm-qa/main.py:66-69).
"""
from __future__ import annotations

import math
import os
import zlib
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel import comm

# cascade decode over a library-GEMM QKV: DOCQA_CASCADE_ROPE=1 fuses RoPE + the new
# token's cache write into the cascade kernels (ops.paged_decode_cascade_rope).  Off by
# default: measured 2.5 % slower per decode step at batch 256 than the separate rope_cache
# launch (the ring's fused preamble delays its K/V stream; profiles/r1_cascade_rope_ab.log)
_CASCADE_ROPE = os.environ.get("DOCQA_CASCADE_ROPE", "0") == "1"
# last prefill layer on the logits rows only (forward(): trim)
_PREFILL_TRIM = os.environ.get("DOCQA_PREFILL_TRIM", "1") != "0"
# grouped decode reading the QKV slabs itself (ops.paged_decode_grouped_fused): off -- every
# group workgroup's slab loads + new-token write ahead of its first K/V stage cost more than the
# rope_cache_splitk launch saved (decode 1148-1151 vs 1120-1122 ms per batch same-box,
# profiles/r4_group_fused_ab.log)
_GROUP_FUSED = os.environ.get("DOCQA_GROUP_FUSED", "0") == "1"
# short prefills (<= ops.MID_M_MAX tokens) on the decode projection plans (forward())
_PREFILL_MID = os.environ.get("DOCQA_PREFILL_MID", "1") != "0"


@dataclass
class LlamaConfig:
    name: str = "llama3-8b"
    vocab_size: int = 128256
    hidden: int = 4096
    intermediate: int = 14336
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    bos_token_id: int = 128000
    eos_token_id: int = 128009
    # Hugging Face rope_scaling dict (None, "linear" or "llama3"; ops.reference.rope_inv_freq)
    rope_scaling: dict | None = None
    # Mistral-style sliding-window attention span (None = full causal attention); the
    # engine refuses a context longer than the window since its kernels attend to all of it
    sliding_window: int | None = None

    @staticmethod
    def preset(name: str) -> "LlamaConfig":
        if name in ("llama3-8b", "llama-3-8b", "8b"):
            return LlamaConfig()
        if name in ("llama3-70b", "llama-3-70b", "70b"):
            return LlamaConfig(name="llama3-70b", hidden=8192, intermediate=28672, layers=80,
                               heads=64, kv_heads=8)
        if name in ("mistral-7b", "mistral"):
            # the reference's own generator: ChatOllama(model="mistral") (llm-qa/main.py:69)
            # pulls Mistral-7B-Instruct v0.3 -- the Llama block with a 32768-token vocabulary,
            # rope theta 1e6 and full causal attention (v0.1's 4096-token sliding window is
            # gone); HF checkpoints of either version load through models/checkpoint.py
            return LlamaConfig(name="mistral-7b", vocab_size=32768, rope_theta=1e6, max_position=32768,
                               bos_token_id=1, eos_token_id=2)
        if name == "llama3-1b-test":  # mid-size config for kernel/engine tests on GPU
            return LlamaConfig(name=name, vocab_size=32000, hidden=2048, intermediate=8192,
                               layers=4, heads=16, kv_heads=4, max_position=4096,
                               bos_token_id=1, eos_token_id=2)
        if name == "test-tp8":
            # Llama-3-70B's GQA shape (8 KV heads, 128-d heads) at toy width: every TP degree
            # 1 / 2 / 4 / 8 shards it, so the TP=8 paths run in CPU and one-GPU tests; a vocab
            # that is not a multiple of 8 x 256 exercises the padded last LM-head shard
            return LlamaConfig(name=name, vocab_size=4000, hidden=1024, intermediate=2048,
                               layers=2, heads=32, kv_heads=8, head_dim=128, max_position=2048,
                               bos_token_id=1, eos_token_id=2)
        if name == "tiny":
            return LlamaConfig(name="tiny", vocab_size=4096, hidden=256, intermediate=512,
                               layers=2, heads=4, kv_heads=2, head_dim=128, max_position=2048,
                               bos_token_id=1, eos_token_id=2)
        if name == "tiny-8k":   # tiny with Llama-3's 8192-token window (long-prompt service tests)
            return LlamaConfig(name="tiny-8k", vocab_size=4096, hidden=256, intermediate=512,
                               layers=2, heads=4, kv_heads=2, head_dim=128, max_position=8192,
                               bos_token_id=1, eos_token_id=2)
        raise ValueError(f"unknown llama preset {name}")

    def num_params(self) -> int:
        H, I, D = self.hidden, self.intermediate, self.head_dim
        per_layer = H * (self.heads + 2 * self.kv_heads) * D + self.heads * D * H + 3 * H * I + 2 * H
        return self.layers * per_layer + 2 * self.vocab_size * H + H


@dataclass
class AttnMeta:
    """Per-forward attention metadata (all int32 device tensors)."""
    prefill: bool
    positions: torch.Tensor                 # [T]
    slot_mapping: torch.Tensor              # [T]
    cu_seqlens: torch.Tensor | None = None  # [B+1] (prefill)
    max_len: int = 0                        # (prefill)
    block_tables: torch.Tensor | None = None  # [B, maxb] (decode)
    context_lens: torch.Tensor | None = None  # [B] (decode; includes the new token)
    max_context: int = 0                    # (decode) graph-capture bound
    prefix_lens: torch.Tensor | None = None  # [B] (prefill with prefix-cache hits)
    # (decode, cascade) prompt prefix shared by every row: its block ids [maxb] and its
    # length [1] (multiple of the block size), attended once for the whole batch
    shared_table: torch.Tensor | None = None
    shared_len: torch.Tensor | None = None
    cascade_chunks: int = 8
    # (decode) workgroup dispatch order: int32 permutation of the rows, longest context
    # first (LPT), so short sequences fill the last launch round; None: row order
    seq_order: torch.Tensor | None = None
    # (decode, cascade) rows packed in groups of <= 4 sharing prefix-cache blocks
    # (ops.paged_decode_cascade_grouped); None: per-row suffix attention
    decode_groups: torch.Tensor | None = None
    # decode_groups is a deferred split plan (ops.split_decode_groups(defer=True))
    decode_defer: bool = False
    # ... a split plan whose items start at block 0 (the groups attend the shared prefix)
    decode_inline: bool = False


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 init: bool = True):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        ps = comm.state()
        self.tp = ps.tp_size
        self.tp_rank = ps.tp_rank
        if cfg.heads % self.tp or cfg.kv_heads % self.tp or cfg.intermediate % self.tp:
            raise ValueError("heads / kv_heads / intermediate must divide the TP size")
        self.hq = cfg.heads // self.tp
        self.hkv = cfg.kv_heads // self.tp
        self.inter = cfg.intermediate // self.tp
        self.vocab_shard = (cfg.vocab_size + self.tp - 1) // self.tp
        if self.tp > 1:
            # whole 256-row tiles for the fused LM-head argmax kernel (mgemm.hip); the padded
            # rows (ids >= vocab_size, on the last rank only) are zero and never picked
            self.vocab_shard = (self.vocab_shard + 255) // 256 * 256
        self.vocab_start = self.tp_rank * self.vocab_shard
        # ids this rank's LM-head shard holds
        self.vocab_valid = max(0, min(cfg.vocab_size - self.vocab_start, self.vocab_shard))
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.cos_sin = ops.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta, self.device,
                                        scaling=cfg.rope_scaling)
        self.layers: list[dict] = []
        self._tick = None      # decode attention's last-arriver merge tickets (ops.decode_ticket)
        self._ntick = None     # fused projection + add + RMSNorm ticket word (ops.dgemm_add_rmsnorm)
        if init:
            self._random_init(seed)

    # ------------------------------------------------------------------ weights
    def _random_init(self, seed: int) -> None:
        """Random weights (no checkpoints offline) that are TP-INVARIANT: every weight is
        generated in fixed global blocks (per head for q / k / v / o, per 64 rows or columns
        of the MLP, per 256 vocab rows of the LM head), each from its own seeded stream, so
        a rank's shard holds exactly the bits the TP = 1 model has at those positions -- TP
        runs and services are then token-exact against TP = 1 by construction."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        std = 0.02
        out_std = std / math.sqrt(2 * cfg.layers)
        H, D, r = cfg.hidden, cfg.head_dim, self.tp_rank

        def gen(key, shape, s=std):
            g.manual_seed((seed * 1_000_003 + zlib.crc32(repr(key).encode())) & 0x7FFFFFFFFFFF)
            t = torch.empty(*shape, device=dev, dtype=dt)
            t.normal_(0.0, s, generator=g)
            return t

        def rows(key, lo, hi, width, blk, s=std):       # global rows [lo, hi) in blocks
            return torch.cat([gen(key + (b,), (blk, width), s) for b in range(lo // blk, hi // blk)])

        ib = 64 if self.inter % 64 == 0 else 8            # MLP block (divides every TP shard)
        self.embed = gen(("embed",), (cfg.vocab_size, H))
        self.final_norm = torch.ones(H, device=dev, dtype=dt)
        # vocab block: the same for every TP degree (shards start at multiples of 256)
        vb = next(b for b in (256, 8, 1) if cfg.vocab_size % b == 0)
        self.lm_head = rows(("lm",), self.vocab_start, self.vocab_start + self.vocab_shard, H, vb)
        if self.vocab_valid < self.vocab_shard:
            self.lm_head[self.vocab_valid:] = 0
        i0, i1 = r * self.inter, (r + 1) * self.inter
        for li in range(cfg.layers):
            q = rows((li, "q"), r * self.hq * D, (r + 1) * self.hq * D, H, D)
            k = rows((li, "k"), r * self.hkv * D, (r + 1) * self.hkv * D, H, D)
            v = rows((li, "v"), r * self.hkv * D, (r + 1) * self.hkv * D, H, D)
            o = rows((li, "o"), r * self.hq * D, (r + 1) * self.hq * D, H, D, out_std).t()   # columns
            gt = rows((li, "gate"), i0, i1, H, ib)
            up = rows((li, "up"), i0, i1, H, ib)
            dn = rows((li, "down"), i0, i1, H, ib, out_std).t()
            self.layers.append({
                "in_norm": torch.ones(H, device=dev, dtype=dt),
                "qkv": torch.cat([q, k, v]).contiguous(),
                "o": o.contiguous(),
                "post_norm": torch.ones(H, device=dev, dtype=dt),
                # rows interleaved in blocks of 8 (gate, up): the decode GEMMs' fused SwiGLU
                "gate_up": ops.glu_interleave(gt, up).contiguous(),
                "down": dn.contiguous(),
            })

    def load_state_dict_hf(self, sd: dict) -> None:
        """Map a Hugging Face LlamaForCausalLM state dict (full, un-sharded) onto this
        rank's shards."""
        cfg, D, r, tp = self.cfg, self.cfg.head_dim, self.tp_rank, self.tp
        dev, dt = self.device, self.dtype

        def get(k):
            return sd[k].to(device=dev, dtype=dt)

        self.embed = get("model.embed_tokens.weight")
        self.final_norm = get("model.norm.weight")
        lm = get("lm_head.weight") if "lm_head.weight" in sd else self.embed
        pad = self.vocab_shard * tp - lm.shape[0]
        if pad:
            lm = torch.cat([lm, lm.new_zeros(pad, lm.shape[1])])
        self.lm_head = lm[r * self.vocab_shard:(r + 1) * self.vocab_shard].contiguous()
        self.layers = []
        for i in range(cfg.layers):
            p = f"model.layers.{i}."
            q = get(p + "self_attn.q_proj.weight").view(cfg.heads, D, -1)[r * self.hq:(r + 1) * self.hq]
            k = get(p + "self_attn.k_proj.weight").view(cfg.kv_heads, D, -1)[r * self.hkv:(r + 1) * self.hkv]
            v = get(p + "self_attn.v_proj.weight").view(cfg.kv_heads, D, -1)[r * self.hkv:(r + 1) * self.hkv]
            o = get(p + "self_attn.o_proj.weight")[:, r * self.hq * D:(r + 1) * self.hq * D]
            gt = get(p + "mlp.gate_proj.weight")[r * self.inter:(r + 1) * self.inter]
            up = get(p + "mlp.up_proj.weight")[r * self.inter:(r + 1) * self.inter]
            dn = get(p + "mlp.down_proj.weight")[:, r * self.inter:(r + 1) * self.inter]
            self.layers.append({
                "in_norm": get(p + "input_layernorm.weight"),
                "qkv": torch.cat([q.reshape(-1, cfg.hidden), k.reshape(-1, cfg.hidden),
                                  v.reshape(-1, cfg.hidden)]).contiguous(),
                "o": o.contiguous(),
                "post_norm": get(p + "post_attention_layernorm.weight"),
                # rows interleaved in blocks of 8 (gate, up): the decode GEMM's fused SwiGLU
                # epilogue pairs them inside one MFMA tile (csrc/kernels/dgemm.hip)
                "gate_up": ops.glu_interleave(gt, up).contiguous(),
                "down": dn.contiguous(),
            })

    def export_state_dict_hf(self) -> dict:
        """Inverse of :meth:`load_state_dict_hf` for an un-sharded (TP=1) model."""
        if self.tp != 1:
            raise ValueError("export requires TP=1")
        cfg, D = self.cfg, self.cfg.head_dim
        sd = {"model.embed_tokens.weight": self.embed, "model.norm.weight": self.final_norm,
              "lm_head.weight": self.lm_head[: cfg.vocab_size]}
        for i, L in enumerate(self.layers):
            p = f"model.layers.{i}."
            q, k, v = L["qkv"].split([self.hq * D, self.hkv * D, self.hkv * D])
            g, u = ops.glu_split(L["gate_up"])
            sd.update({p + "self_attn.q_proj.weight": q, p + "self_attn.k_proj.weight": k,
                       p + "self_attn.v_proj.weight": v, p + "self_attn.o_proj.weight": L["o"],
                       p + "mlp.gate_proj.weight": g, p + "mlp.up_proj.weight": u,
                       p + "mlp.down_proj.weight": L["down"],
                       p + "input_layernorm.weight": L["in_norm"],
                       p + "post_attention_layernorm.weight": L["post_norm"]})
        return {k: t.detach().cpu() for k, t in sd.items()}

    def weight_bytes(self) -> int:
        n = self.embed.numel() + self.lm_head.numel() + self.final_norm.numel()
        for L in self.layers:
            n += sum(t.numel() for t in L.values())
        return n * self.embed.element_size()

    # ------------------------------------------------------------------ forward
    def forward(self, input_ids: torch.Tensor, meta: AttnMeta, kv_caches: list,
                logits_index: torch.Tensor | None = None, greedy_ids: bool = False) -> torch.Tensor:
        """input_ids [T] int32 -> logits [R, vocab_shard] for the rows selected by
        ``logits_index`` (all rows if None).  kv_caches: list of (k_cache, v_cache).
        ``greedy_ids``: return the greedy token ids int64 [R] instead (the LM head's argmax
        is fused into its GEMM where :func:`ops.lm_head_argmax_ok`)."""
        cfg = self.cfg
        D, hq, hkv, eps = cfg.head_dim, self.hq, self.hkv, cfg.rms_eps
        h, x = ops.embed_rmsnorm(input_ids, self.embed, self.layers[0]["in_norm"], eps)
        residual = h
        nl = len(self.layers)
        # decode steps stream every weight once: per projection the mid-M MFMA GEMM
        # (mgemm.hip, 129..512 rows where it wins -- ops.mid_plan) or the skinny
        # weight-streaming kernel (dgemm.hip, <= 192 rows -- ops.decode_plan) emits fp32
        # split-K slabs straight into the fused consumers: RoPE + KV write for QKV, and for the
        # row-parallel O / down the (TP all-reduce +) residual add + RMSNorm
        # (comm.tp_add_rmsnorm); split 0 = library GEMM + plain consumer.  Prefill (large M):
        # the 256 x 256 MFMA GEMM (pgemm.hip) with SwiGLU fused into the gate|up epilogue.
        decode = not meta.prefill
        lin = ops.decode_linear if decode else ops.prefill_linear
        M = x.shape[0]
        plans = {}
        # a short prefill (<= ops.MID_M_MAX prompt tokens: batch-1 serving) has the decode
        # step's shape -- too few rows for the 256 x 256 prefill GEMM's tiles -- so it takes
        # the same split-K projection plans and fused consumers (RoPE + KV write, add + norm)
        # (ops.prefill_route mirrors the prefill plan choices below for the GEMM probes and
        # tests/test_pgemm_gpu.py::test_prefill_route_products -- keep the two in step)
        small = (not decode and x.is_cuda and _PREFILL_MID and M <= ops.MID_M_MAX)
        if (decode or small) and self.layers:
            L0 = self.layers[0]
            cascade = decode and meta.shared_len is not None
            # bf16 split-K slabs (ops.SLAB_BF16) where the consumer is the RoPE + cache-write
            # kernel (QKV) or the TP = 1 add + RMSNorm (O / down); the fused attention kernels
            # that read QKV slabs themselves take fp32 only
            s16 = x.is_cuda and self.tp == 1 and ops.SLAB_BF16
            qkv_rope = (not decode or
                        (not (meta.decode_groups is not None and meta.decode_inline and _GROUP_FUSED
                              and meta.slot_mapping is not None) if cascade
                         else not (meta.block_tables is not None and kv_caches
                                   and ops.fused_decode_ok(kv_caches[0][0], meta.block_tables))))
            b16 = {"qkv": s16 and qkv_rope, "o": s16, "down": s16}
            for k in ("qkv", "o", "down"):
                Sg, R = ops.gemv_plan(M, *L0[k].shape) if x.is_cuda else (0, 0)
                if Sg:
                    # one row: the register-streaming GEMV (no LDS ring) -- QKV / O
                    plans[k] = (Sg, lambda a, w, S=Sg, R=R: ops.gemv_partial(a, w, S, R))
                    continue
                S, c = ops.mid_plan(M, *L0[k].shape)
                if S and b16[k] and S > 1:
                    plans[k] = (S, lambda a, w, S=S, c=c: ops.mgemm_partial(a, w, S, c, bf16=True))
                elif S:
                    plans[k] = (S, lambda a, w, S=S, c=c: (ops.mgemm_partial(a, w, S, c) if S > 1
                                                          else ops.mgemm_partial(a, w, 1, c).float()[None]))
                else:
                    S, t = ops.decode_plan(M, *L0[k].shape)
                    plans[k] = (S, lambda a, w, S=S, t=t: ops.dgemm_partial(a, w, S, t))
            if small and M > 256 and "down" in plans:
                # a 257..512-token prefill's down projection (decode buckets keep their plan):
                # the 256 x 256 kernel's S=8 slabs where K is long -- 8B: 66.1 vs the mid-M
                # kernel's S=4 77.5 and hipBLASLt's 97.4 us at 512 rows
                # (profiles/r6_prefill_mid_plans.log); the 70B TP-8 shard keeps mid_plan's
                Sd = ops.down_small_split(M, *L0["down"].shape)
                if Sd:
                    plans["down"] = (Sd, lambda a, w, S=Sd: ops.pgemm_partial(a, w, S))
            Sg, cg = ops.mid_plan(M, *L0["gate_up"].shape, glu=True)
            if decode and x.is_cuda and ops.gemv_glu_ok(M, *L0["gate_up"].shape):
                glu = ops.gemv_glu        # one row: the register-streaming GEMV with SwiGLU
            elif small and (ops.pgemm_ok(M, *L0["gate_up"].shape)
                          or ops.prefill_split_plan(M, *L0["gate_up"].shape, glu=True)):
                # 256 x 256 tiles with SwiGLU (104 vs 141 us at M = 512), or their split-K
                # slabs into the SwiGLU consumer where too few tiles (the 70B TP-8 shard)
                glu = ops.prefill_glu
            elif decode and s16 and ops.glu_split16_plan(M, *L0["gate_up"].shape)[0]:
                S2, c2 = ops.glu_split16_plan(M, *L0["gate_up"].shape)
                glu = lambda a, w, S=S2, c=c2: ops.glu_split16(a, w, S, c)  # noqa: E731
            else:
                glu = (lambda a, w: ops.mgemm_glu(a, w, cg)) if Sg else ops.glu_linear
        else:
            glu = ops.prefill_glu
            if self.layers and x.is_cuda and not decode:
                # 513..2048-token prefills: split-K slab plans where they win with the consumer
                L0 = self.layers[0]
                s16 = self.tp == 1 and ops.SLAB_BF16      # bf16 slabs: see the decode plans above
                for k in ("qkv", "o", "down"):
                    S, c = ops.prefill_plan(M, *L0[k].shape)
                    if S >= 2:
                        plans[k] = (S, lambda a, w, S=S, c=c, b=s16: ops.mgemm_partial(a, w, S, c, bf16=b))
                    elif not S:
                        # narrow tensor-parallel shards: the 256 x 256 tiles split over K
                        Sp = ops.prefill_split_plan(M, *L0[k].shape)
                        if Sp:
                            plans[k] = (Sp, lambda a, w, S=Sp: ops.pgemm_partial(a, w, S))
        if self.tp > 1 and not x.is_cuda:
            # CPU TP rehearsal: row-parallel partials as fp32 slabs, all-reduced before the one
            # bf16 rounding (comm.tp_add_rmsnorm), so TP = N tracks TP = 1's rounding
            for k in ("o", "down"):
                if not plans.get(k, (0, None))[0]:
                    plans[k] = (1, lambda a, w: F.linear(a.float(), w.float())[None])
        # batch 1 (<= ops.NORM_FUSE_ROWS rows, TP = 1): O / down with the residual add + RMSNorm
        # in the projection's own last workgroup -- no add_rmsnorm_splitk launch
        nf = {}
        if decode and self.tp == 1 and self.layers and x.is_cuda:
            L0 = self.layers[0]
            for k in ("o", "down"):
                S = ops.dgemm_norm_plan(M, *L0[k].shape)
                if S:
                    nf[k] = S
            if nf and self._ntick is None:
                self._ntick = torch.zeros(1, dtype=torch.int32, device=self.device)
        sq, qkv_part = plans.get("qkv", (0, None))
        so, o_part = plans.get("o", (0, None))
        sd, down_part = plans.get("down", (0, None))
        cascade = decode and meta.shared_len is not None
        trim = (not decode and _PREFILL_TRIM and x.is_cuda and logits_index is not None and self.layers
                and meta.block_tables is not None and meta.prefix_lens is not None
                and logits_index.numel() == meta.block_tables.shape[0] and M > logits_index.numel())
        # batch 1 (one row, TP = 1, skinny-kernel plans): the gate|up and the next layer's QKV
        # projection build their input row themselves -- residual add + RMSNorm of the previous
        # projection's slabs, in LDS, under their first weight stages (dgemm.hip XNormIn) --
        # so no add_rmsnorm launch runs between projections; the residual ping-pongs between
        # two buffers (one workgroup writes the new one while the others read the old)
        xn = (decode and self.tp == 1 and not nf and x.is_cuda and sq and so and sd
              and self.layers and ops.xn_ok(M, self.cfg.hidden)
              and not ops.mid_plan(M, *self.layers[0]["gate_up"].shape, glu=True)[0])
        res2 = torch.empty_like(residual) if xn else None
        pd = None   # XN: the previous layer's down-projection slabs
        for i, L in enumerate(self.layers):
            kc, vc = kv_caches[i]
            if sq:
                if xn and pd is not None:
                    Sg, R = ops.gemv_plan(M, *L["qkv"].shape)
                    if Sg == sq:
                        qkv_slabs = ops.gemv_partial_xn(pd, residual, res2, L["in_norm"], eps, L["qkv"], sq, R)
                    else:
                        qkv_slabs = ops.dgemm_partial_xn(pd, residual, res2, L["in_norm"], eps, L["qkv"], sq)
                    residual, res2 = res2, residual
                else:
                    qkv_slabs = qkv_part(x, L["qkv"])
            if cascade:
                # shared-prefix decode: RoPE + cache write, then prefix-once + suffix attention
                if (sq and meta.decode_groups is not None and meta.decode_inline and x.is_cuda
                        and _GROUP_FUSED and meta.slot_mapping is not None):
                    # the group kernel reads the QKV slabs itself (RoPE + new-token cache write)
                    a = ops.paged_decode_grouped_fused(qkv_slabs, meta.positions, self.cos_sin, meta.slot_mapping,
                                                       kc, vc, meta.block_tables, meta.context_lens, hq,
                                                       self.scale, meta.shared_table, meta.shared_len,
                                                       meta.cascade_chunks, meta.decode_groups, self._decode_tick(M))
                elif sq:
                    qkv = ops.rope_cache_splitk(qkv_slabs, meta.positions,
                                                self.cos_sin, meta.slot_mapping, kc, vc, hq, hkv, D)
                    if meta.decode_groups is not None:
                        a = ops.paged_decode_cascade_grouped(qkv, kc, vc, meta.block_tables, meta.context_lens,
                                                             hq, self.scale, meta.shared_table, meta.shared_len,
                                                             meta.cascade_chunks, meta.decode_groups,
                                                             meta.decode_defer,
                                                             self._decode_tick(M) if x.is_cuda else None,
                                                             meta.decode_inline)
                    else:
                        a = ops.paged_decode_cascade(qkv, kc, vc, meta.block_tables, meta.context_lens, hq,
                                                     meta.max_context, self.scale, meta.shared_table,
                                                     meta.shared_len, meta.cascade_chunks, meta.seq_order)
                elif not _CASCADE_ROPE:
                    qkv = lin(x, L["qkv"])
                    ops.rope_cache(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc, hq, hkv, D)
                    if meta.decode_groups is not None:
                        a = ops.paged_decode_cascade_grouped(qkv, kc, vc, meta.block_tables, meta.context_lens,
                                                             hq, self.scale, meta.shared_table, meta.shared_len,
                                                             meta.cascade_chunks, meta.decode_groups,
                                                             meta.decode_defer,
                                                             self._decode_tick(M) if x.is_cuda else None,
                                                             meta.decode_inline)
                    else:
                        a = ops.paged_decode_cascade(qkv, kc, vc, meta.block_tables, meta.context_lens, hq,
                                                     meta.max_context, self.scale, meta.shared_table,
                                                     meta.shared_len, meta.cascade_chunks, meta.seq_order)
                else:
                    # library-GEMM QKV: RoPE + new-token cache write fused into the cascade kernels
                    a = ops.paged_decode_cascade_rope(lin(x, L["qkv"]), meta.positions, self.cos_sin,
                                                      meta.slot_mapping, kc, vc, meta.block_tables,
                                                      meta.context_lens, hq, meta.max_context, self.scale,
                                                      meta.shared_table, meta.shared_len,
                                                      meta.cascade_chunks, meta.seq_order)
                qkv = None
            elif decode and sq and ops.fused_decode_ok(kc, meta.block_tables):
                # QKV partials -> RoPE + new-token cache write + attention, one launch
                a = ops.paged_decode_fused(qkv_slabs, meta.positions, self.cos_sin,
                                           meta.slot_mapping, kc, vc, meta.block_tables, meta.context_lens,
                                           hq, meta.max_context, self.scale, meta.seq_order,
                                           self._decode_tick(M) if x.is_cuda else None)
                qkv = None
            elif sq:
                qkv = ops.rope_cache_splitk(qkv_slabs, meta.positions, self.cos_sin,
                                            meta.slot_mapping, kc, vc, hq, hkv, D)
            else:
                qkv = lin(x, L["qkv"])
                ops.rope_cache(qkv, meta.positions, self.cos_sin, meta.slot_mapping, kc, vc, hq, hkv, D)
            if trim and i == nl - 1 and qkv is not None:
                # last layer of a prefill whose logits are wanted for a few rows only: every
                # token's K/V is in the cache now; only the selected rows go on through
                # attention, O and the MLP (their outputs are the only ones anything reads)
                # -- each selected row is its sequence's last token, so its attention over
                # the paged cache is exactly the decode attention at that context length
                ctx = meta.prefix_lens + (meta.cu_seqlens[1:] - meta.cu_seqlens[:-1])
                a = ops.paged_decode(qkv.index_select(0, logits_index).contiguous(), kc, vc, meta.block_tables,
                                     ctx, hq, meta.block_tables.shape[1] * kc.shape[2], self.scale)
                residual = residual.index_select(0, logits_index)
                logits_index = None
                qkv = None
            if qkv is None:
                pass
            elif meta.prefill and meta.prefix_lens is not None:
                # prompt prefix already in the paged cache: attend over cache (prefix + new)
                a = ops.flash_prefill_paged(qkv, meta.cu_seqlens, meta.max_len, hq, hkv, D, self.scale,
                                            kc, vc, meta.block_tables, meta.prefix_lens)
            elif meta.prefill:
                a = ops.flash_prefill(qkv, meta.cu_seqlens, meta.max_len, hq, hkv, D, self.scale, True)
            else:
                a = ops.paged_decode(qkv, kc, vc, meta.block_tables, meta.context_lens, hq,
                                     meta.max_context, self.scale, meta.seq_order)
            nxt = self.layers[i + 1]["in_norm"] if i + 1 < nl else self.final_norm
            if xn:
                if ops.gemv_glu_ok(M, *L["gate_up"].shape):
                    g = ops.gemv_glu_xn(o_part(a, L["o"]), residual, res2, L["post_norm"], eps, L["gate_up"])
                else:
                    g = ops.dgemm_glu_xn(o_part(a, L["o"]), residual, res2, L["post_norm"], eps, L["gate_up"])
                residual, res2 = res2, residual
                pd = down_part(g, L["down"])
                if i + 1 == nl:
                    x = ops.add_rmsnorm_splitk(pd, residual, nxt, eps)
                continue
            # row-parallel O: (TP all-reduce +) residual add + RMSNorm in one consumer
            if "o" in nf:
                x = ops.dgemm_add_rmsnorm(a, L["o"], nf["o"], residual, L["post_norm"], eps, self._ntick)
            else:
                x = comm.tp_add_rmsnorm(o_part(a, L["o"]) if so else lin(a, L["o"]), residual, L["post_norm"], eps)
            g = glu(x, L["gate_up"])
            if "down" in nf:
                x = ops.dgemm_add_rmsnorm(g, L["down"], nf["down"], residual, nxt, eps, self._ntick)
            else:
                x = comm.tp_add_rmsnorm(down_part(g, L["down"]) if sd else lin(g, L["down"]), residual, nxt, eps)
        if logits_index is not None:
            x = x.index_select(0, logits_index)
        if greedy_ids:
            return self.greedy_ids(x)
        return ops.lm_head_logits(x, self.lm_head)

    def forward_mixed(self, input_ids: torch.Tensor, n_dec: int, dmeta: AttnMeta, pmeta: AttnMeta,
                      kv_caches: list, logits_index: torch.Tensor, return_logits: bool = False) -> torch.Tensor:
        """One forward over decode rows AND a prefill chunk (continuous batching without the
        prefill stall): rows [0, n_dec) are decode slots (one new token each, paged decode
        attention over their cache -- ``dmeta``, the decode step's metadata), rows
        [n_dec, T) are prompt-chunk tokens (``pmeta``: positions / slots / cu_seqlens /
        block_tables / prefix_lens of the chunk; attention over cached prefix + chunk).
        Every projection runs ONCE over all T rows -- the decode rows ride in the prefill
        GEMMs' weight pass -- and only attention is split by row kind.  Returns the greedy
        ids of the rows in ``logits_index``.
        Reference parity: the service loop the reference runs one request at a time
        (llm-qa/main.py:111-117)."""
        cfg = self.cfg
        D, hq, hkv, eps = cfg.head_dim, self.hq, self.hkv, cfg.rms_eps
        h, x = ops.embed_rmsnorm(input_ids, self.embed, self.layers[0]["in_norm"], eps)
        residual = h
        positions = torch.cat([dmeta.positions, pmeta.positions]) if n_dec else pmeta.positions
        slots = torch.cat([dmeta.slot_mapping, pmeta.slot_mapping]) if n_dec else pmeta.slot_mapping
        nl = len(self.layers)
        M = x.shape[0]
        for i, L in enumerate(self.layers):
            kc, vc = kv_caches[i]
            qkv = ops.prefill_linear(x, L["qkv"])
            ops.rope_cache(qkv, positions, self.cos_sin, slots, kc, vc, hq, hkv, D)
            parts = []
            if n_dec:
                parts.append(self._attend_decode(qkv[:n_dec], dmeta, kc, vc, n_dec))
            parts.append(ops.flash_prefill_paged(qkv[n_dec:], pmeta.cu_seqlens, pmeta.max_len, hq, hkv, D,
                                                 self.scale, kc, vc, pmeta.block_tables, pmeta.prefix_lens))
            a = torch.cat(parts) if len(parts) > 1 else parts[0]
            nxt = self.layers[i + 1]["in_norm"] if i + 1 < nl else self.final_norm
            x = comm.tp_add_rmsnorm(ops.prefill_linear(a, L["o"]), residual, L["post_norm"], eps)
            g = ops.prefill_glu(x, L["gate_up"])
            x = comm.tp_add_rmsnorm(ops.prefill_linear(g, L["down"]), residual, nxt, eps)
        assert x.shape[0] == M
        if return_logits:          # tests: the selected rows' logits instead of their greedy ids
            return ops.lm_head_logits(x.index_select(0, logits_index).contiguous(), self.lm_head)
        return self.greedy_ids(x.index_select(0, logits_index))

    def _attend_decode(self, qkv: torch.Tensor, meta: AttnMeta, kc, vc, M: int) -> torch.Tensor:
        """Decode attention of post-RoPE bf16 QKV rows whose new K/V are already in the
        cache: the grouped / plain cascade kernels when the step attends a shared prefix,
        else per-row paged decode (the same dispatch as :meth:`forward`'s library-GEMM
        branch)."""
        hq = self.hq
        if meta.shared_len is not None:
            if meta.decode_groups is not None:
                return ops.paged_decode_cascade_grouped(qkv, kc, vc, meta.block_tables, meta.context_lens, hq,
                                                        self.scale, meta.shared_table, meta.shared_len,
                                                        meta.cascade_chunks, meta.decode_groups, meta.decode_defer,
                                                        self._decode_tick(M) if qkv.is_cuda else None,
                                                        meta.decode_inline)
            return ops.paged_decode_cascade(qkv, kc, vc, meta.block_tables, meta.context_lens, hq,
                                            meta.max_context, self.scale, meta.shared_table, meta.shared_len,
                                            meta.cascade_chunks, meta.seq_order)
        return ops.paged_decode(qkv, kc, vc, meta.block_tables, meta.context_lens, hq, meta.max_context,
                                self.scale, meta.seq_order)

    def _decode_tick(self, B: int):
        """Ticket words for the fused decode attention's in-kernel partition merge, shared
        by every layer (the launches are stream-ordered and each re-arms its words).  The
        grouped kernel indexes them by plan row, and a plan holds up to
        bucket x DOCQA_GROUP_CAP_MULT rows (engine/llm_engine.py), so the buffer is sized for
        the largest bucket x that multiple ONCE, before any graph is captured, and never
        reallocated: a captured graph keeps pointing at it."""
        import os

        mult = max(1, int(os.environ.get("DOCQA_GROUP_CAP_MULT", "1")))
        need = max(B, 1) * mult * self.hkv
        if self._tick is None:
            self._tick = ops.decode_ticket(max(B, 4096) * mult * self.hkv, self.device)
        if self._tick.numel() < need:
            raise RuntimeError(f"decode ticket buffer holds {self._tick.numel()} words, a {B}-row bucket "
                               f"needs {need}: raise the first bucket size (buffers are never regrown)")
        return self._tick

    def greedy_ids(self, x: torch.Tensor) -> torch.Tensor:
        """Greedy token ids int64 [R] of the final normed hidden rows ``x``: the LM-head GEMM
        with its argmax fused (mgemm.hip EPI_ARGMAX, no [R, vocab] logits) where the shape
        allows, the vocab-parallel pick resolved by one packed-key MAX all-reduce at TP > 1."""
        R = x.shape[0]
        N, K = self.lm_head.shape
        fused = ops.lm_head_argmax_ok(R, N, K) or (self.tp > 1 and 0 < R <= ops.MID_M_MAX
                                                   and ops.lm_head_argmax_shape_ok(N, K))
        if self.tp == 1:
            if fused:
                return ops.lm_head_argmax(x, self.lm_head, self.cfg.vocab_size)
            return self.greedy(ops.lm_head_logits(x, self.lm_head))
        if fused and self.vocab_valid > 0:
            ids, vals = ops.lm_head_argmax(x, self.lm_head, self.vocab_valid, with_values=True)
        else:
            logits = ops.lm_head_logits(x, self.lm_head)[:, : max(1, self.vocab_valid)]
            ids = ops.argmax(logits)
            vals = logits.gather(1, ids[:, None])[:, 0].float()
        if self.vocab_valid == 0:
            vals = torch.full_like(vals, float("-inf"))
        return comm.tp_argmax(vals, ids + self.vocab_start)

    def greedy(self, logits: torch.Tensor) -> torch.Tensor:
        """argmax over the (possibly vocab-parallel) logits -> int64 [R]."""
        if self.tp == 1:
            return ops.argmax(logits)
        valid = logits[:, : max(1, self.vocab_valid)]
        idx = ops.argmax(valid)
        val = valid.gather(1, idx[:, None])[:, 0].float()
        if self.vocab_valid == 0:
            val = torch.full_like(val, float("-inf"))
        return comm.tp_argmax(val, idx + self.vocab_start)

    def full_logits(self, logits: torch.Tensor) -> torch.Tensor:
        full = comm.tp_all_gather_last(logits)
        return full[:, : self.cfg.vocab_size]
