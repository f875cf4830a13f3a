"""Plain-PyTorch (fp32-accumulating) reference implementations of every native op.

These serve two purposes:
  * the numerics oracle the GPU tests compare the HIP kernels against;
  * the CPU execution path, so services, models and the distributed code can be
    exercised in CI without a GPU.  On a GPU tensor the dispatcher in
    ``docqa_amd.ops`` never falls back here: it raises if the native extension is
    missing (see ``ops/__init__.py``).
Layouts mirror the kernels exactly (paged cache ``[num_blocks, Hkv, BS, D]``, packed
QKV rows ``[(Hq + 2*Hkv) * D]``, FAISS distance conventions).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rmsnorm(x, w, eps):
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype)


def add_rmsnorm(x, residual, w, eps):
    s = (x.float() + residual.float()).to(x.dtype)
    residual.copy_(s)
    return rmsnorm(s, w, eps)


def layernorm(x, residual, gamma, beta, eps):
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
    return F.layer_norm(xf, (x.shape[-1],), gamma.float(), beta.float(), eps).to(x.dtype)


def rope_inv_freq(head_dim: int, theta: float, scaling: dict | None = None) -> torch.Tensor:
    """fp64 RoPE inverse frequencies, with Hugging Face ``rope_scaling`` applied.

    * ``None`` / ``"default"``: theta^(-2i/d).
    * ``"linear"``: every frequency divided by ``factor`` (position interpolation).
    * ``"llama3"`` (Llama-3.1 / 3.2): wavelengths longer than
      ``original_max_position_embeddings / low_freq_factor`` are divided by ``factor``,
      shorter than ``.../high_freq_factor`` kept, and the band between is blended with
      ``s = (L_orig / wavelen - low) / (high - low)``: ``(1 - s) * f / factor + s * f``.
    Anything else raises: a checkpoint must not load with silently wrong positions."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if not scaling:
        return inv
    kind = scaling.get("rope_type", scaling.get("type", "default"))
    if kind == "default":
        return inv
    factor = float(scaling["factor"])
    if kind == "linear":
        return inv / factor
    if kind == "llama3":
        low, high = float(scaling["low_freq_factor"]), float(scaling["high_freq_factor"])
        orig = float(scaling["original_max_position_embeddings"])
        wavelen = 2 * math.pi / inv
        scaled = torch.where(wavelen > orig / low, inv / factor, inv)
        smooth = (orig / wavelen - low) / (high - low)
        blended = (1 - smooth) * scaled / factor + smooth * scaled
        medium = (wavelen >= orig / high) & (wavelen <= orig / low)
        return torch.where(medium, blended, scaled)
    raise NotImplementedError(f"rope_scaling type {kind!r} is not supported")


def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None,
                 scaling: dict | None = None) -> torch.Tensor:
    """fp32 table [max_pos, head_dim]: first half cos, second half sin (rotate-half RoPE)."""
    inv_freq = rope_inv_freq(head_dim, theta, scaling)
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv_freq)
    return torch.cat([freqs.cos(), freqs.sin()], dim=-1).float().to(device)


def rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D):
    T = qkv.shape[0]
    x = qkv.view(T, Hq + 2 * Hkv, D)
    cs = cos_sin[positions.long()]  # [T, D]
    half = D // 2
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    qk = x[:, : Hq + Hkv].float()
    x1, x2 = qk[..., :half], qk[..., half:]
    rot = torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(qkv.dtype)
    x[:, : Hq + Hkv] = rot
    if slot_mapping is not None:
        BS = k_cache.shape[2]
        sm = slot_mapping.long()
        valid = sm >= 0
        sm = sm[valid]
        blk, off = sm // BS, sm % BS
        k = x[valid, Hq : Hq + Hkv]
        v = x[valid, Hq + Hkv :]
        k_cache[blk, :, off] = k
        v_cache[blk, :, off] = v


def silu_mul(gu, interleaved: bool = False):
    """SwiGLU; ``interleaved``: gate|up rows in blocks of 8 (glu_interleave layout)."""
    if interleaved:
        v = gu.float().unflatten(-1, (-1, 2, 8))
        g, u = v[..., 0, :].flatten(-2), v[..., 1, :].flatten(-2)
    else:
        g, u = gu.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gu.dtype)


def glu_interleave(gate, up):
    """[I, K] gate and up -> [2I, K] with rows in blocks of 8: g0..g7 u0..u7 g8..g15 ..."""
    I, K = gate.shape
    return torch.stack([gate.view(I // 8, 8, K), up.view(I // 8, 8, K)], 1).reshape(2 * I, K)


def glu_split(gu):
    """Inverse of :func:`glu_interleave`."""
    v = gu.view(-1, 2, 8, gu.shape[-1])
    return v[:, 0].reshape(-1, gu.shape[-1]), v[:, 1].reshape(-1, gu.shape[-1])


def bias_act(x, bias, residual, gelu):
    y = x.float()
    if residual is not None:
        y = y + residual.float()
    y = y + bias.float()
    if gelu:
        y = F.gelu(y)  # erf form
    return y.to(x.dtype)


def linear_fused(x, w, bias, residual, epi):
    """epi: 0 none, 1 bias, 2 bias+gelu, 3 bias+residual (fp32 accumulate, bf16 out)."""
    y = x.float() @ w.float().T
    if epi >= 1:
        y = y + bias.float()
    if epi == 2:
        y = F.gelu(y)
    if epi == 3:
        y = y + residual.float()
    return y.to(x.dtype)


def embedding(ids, table):
    return table[ids.long()]


def bert_embed_ln(ids, pos, token_type, wte, wpe, wtt, gamma, beta, eps):
    tt = token_type.long() if token_type is not None else torch.zeros_like(ids, dtype=torch.long)
    e = wte[ids.long()].float() + wpe[pos.long()].float() + wtt[tt].float()
    return F.layer_norm(e, (wte.shape[1],), gamma.float(), beta.float(), eps).to(wte.dtype)


def argmax(logits):
    return logits.float().argmax(dim=-1)


def token_cls_argmax(h, w, bias, n_valid):
    logits = h.float() @ w[:n_valid].float().t() + bias[:n_valid].float()
    return logits.argmax(dim=-1)


def sample(logits, inv_temp, top_k, top_p, u):
    out = torch.empty(logits.shape[0], dtype=torch.long, device=logits.device)
    for r in range(logits.shape[0]):
        x = logits[r].float() * float(inv_temp[r])
        k = int(top_k[r])
        if 0 < k < x.numel():
            th = torch.topk(x, k).values[-1]
            x = torch.where(x >= th, x, torch.full_like(x, -math.inf))
        p = torch.softmax(x, -1)
        tp = float(top_p[r])
        if 0.0 < tp < 1.0:
            sp, si = torch.sort(p, descending=True)
            keep = torch.cumsum(sp, 0) - sp < tp
            mask = torch.zeros_like(p, dtype=torch.bool)
            mask[si[keep]] = True
            p = torch.where(mask, p, torch.zeros_like(p))
            p = p / p.sum()
        c = torch.cumsum(p, 0)
        idx = int(torch.searchsorted(c, torch.tensor([float(u[r])], device=c.device)).clamp(max=x.numel() - 1))
        out[r] = idx
    return out


def paged_decode(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context, scale):
    B = q.shape[0]
    NB, Hkv, BS, D = k_cache.shape
    G = Hq // Hkv
    out = torch.empty(B, Hq * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        L = int(context_lens[b])
        nblk = (L + BS - 1) // BS
        blocks = block_tables[b, :nblk].long()
        k = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :L].float()
        v = v_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :L].float()
        qb = q[b, : Hq * D].view(Hkv, G, D).float()
        s = torch.einsum("hgd,htd->hgt", qb, k) * scale
        p = torch.softmax(s, -1)
        o = torch.einsum("hgt,htd->hgd", p, v)
        out[b] = o.reshape(-1).to(q.dtype)
    return out


def paged_decode_cascade(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context, scale,
                         prefix_table, prefix_len, nchunk=8):
    """Cascade decode attention: keys [0, P) come from the shared ``prefix_table`` blocks,
    keys [P, L) from each sequence's own block table (one softmax over both)."""
    B = q.shape[0]
    NB, Hkv, BS, D = k_cache.shape
    G = Hq // Hkv
    P = int(prefix_len.reshape(-1)[0])
    pb = prefix_table.reshape(-1)[: P // BS].long()
    kp = k_cache[pb].permute(1, 0, 2, 3).reshape(Hkv, -1, D).float()
    vp = v_cache[pb].permute(1, 0, 2, 3).reshape(Hkv, -1, D).float()
    out = torch.zeros(B, Hq * D, dtype=q.dtype, device=q.device)
    for b in range(B):
        L = int(context_lens[b])
        if L <= P:
            continue
        nblk = (L + BS - 1) // BS
        blocks = block_tables[b, P // BS:nblk].long()
        ks = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, -1, D)[:, : L - P].float()
        vs = v_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, -1, D)[:, : L - P].float()
        k, v = torch.cat([kp, ks], 1), torch.cat([vp, vs], 1)
        qb = q[b, : Hq * D].view(Hkv, G, D).float()
        p = torch.softmax(torch.einsum("hgd,htd->hgt", qb, k) * scale, -1)
        out[b] = torch.einsum("hgt,htd->hgd", p, v).reshape(-1).to(q.dtype)
    return out


def flash_prefill(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, causal):
    T = qkv.shape[0]
    x = qkv.view(T, Hq + 2 * Hkv, D)
    G = Hq // Hkv
    out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    cu = cu_seqlens.tolist()
    for b in range(len(cu) - 1):
        s0, s1 = cu[b], cu[b + 1]
        L = s1 - s0
        if L == 0:
            continue
        q = x[s0:s1, :Hq].float().transpose(0, 1)  # [Hq, L, D]
        k = x[s0:s1, Hq : Hq + Hkv].float().transpose(0, 1).repeat_interleave(G, 0)
        v = x[s0:s1, Hq + Hkv :].float().transpose(0, 1).repeat_interleave(G, 0)
        s = torch.einsum("hld,hmd->hlm", q, k) * scale
        if causal:
            mask = torch.ones(L, L, dtype=torch.bool, device=qkv.device).triu(1)
            s = s.masked_fill(mask, -math.inf)
        o = torch.einsum("hlm,hmd->hld", torch.softmax(s, -1), v)
        out[s0:s1] = o.transpose(0, 1).reshape(L, Hq * D).to(qkv.dtype)
    return out


def flash_prefill_paged(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, k_cache, v_cache,
                        block_tables, ctx_start):
    """Causal attention of the new tokens over (cached prefix + new) keys read from the
    paged cache (the new keys must already be written there)."""
    T = qkv.shape[0]
    x = qkv.view(T, Hq + 2 * Hkv, D)
    G = Hq // Hkv
    BS = k_cache.shape[2]
    out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    cu = cu_seqlens.tolist()
    for b in range(len(cu) - 1):
        s0, s1 = cu[b], cu[b + 1]
        L = s1 - s0
        if L == 0:
            continue
        P0 = int(ctx_start[b])
        Lk = P0 + L
        nblk = (Lk + BS - 1) // BS
        blocks = block_tables[b, :nblk].long()
        k = k_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :Lk].float()
        v = v_cache[blocks].permute(1, 0, 2, 3).reshape(Hkv, nblk * BS, D)[:, :Lk].float()
        k = k.repeat_interleave(G, 0)
        v = v.repeat_interleave(G, 0)
        q = x[s0:s1, :Hq].float().transpose(0, 1)
        s = torch.einsum("hld,hmd->hlm", q, k) * scale
        qpos = torch.arange(P0, Lk, device=qkv.device)[:, None]
        kpos = torch.arange(Lk, device=qkv.device)[None, :]
        s = s.masked_fill(kpos > qpos, -math.inf)
        o = torch.einsum("hlm,hmd->hld", torch.softmax(s, -1), v)
        out[s0:s1] = o.transpose(0, 1).reshape(L, Hq * D).to(qkv.dtype)
    return out


def knn(xb, xb_norms, xq, k, inner_product, id_offset):
    """FAISS IndexFlat semantics: L2 -> ascending squared distances, IP -> descending."""
    nq = xq.shape[0]
    N = xb.shape[0]
    D = torch.full((nq, k), -3.4028234663852886e38 if inner_product else 3.4028234663852886e38,
                   dtype=torch.float32, device=xq.device)
    I = torch.full((nq, k), -1, dtype=torch.long, device=xq.device)
    if N == 0 or nq == 0:
        return D, I
    xbf = xb.float()
    xqf = xq.float()
    ip = xqf @ xbf.T
    if inner_product:
        vals, idx = torch.topk(ip, min(k, N), dim=1, largest=True)
    else:
        norms = xb_norms.float() if xb_norms is not None else (xbf * xbf).sum(1)
        d = (xqf * xqf).sum(1, keepdim=True) + norms[None, :] - 2 * ip
        vals, idx = torch.topk(d, min(k, N), dim=1, largest=False)
    D[:, : vals.shape[1]] = vals
    I[:, : idx.shape[1]] = idx + id_offset
    return D, I


def pool_l2(h, cu_seqlens, mean, normalize):
    cu = cu_seqlens.tolist()
    out = torch.zeros(len(cu) - 1, h.shape[-1], dtype=torch.float32, device=h.device)
    for b in range(len(cu) - 1):
        s0, s1 = cu[b], cu[b + 1]
        if s1 > s0:
            out[b] = h[s0:s1].float().mean(0) if mean else h[s0].float()
    if normalize:
        out = F.normalize(out, dim=-1, eps=1e-12)
    return out


def decode_slots(block_tables, positions, valid, BS: int):
    blk = torch.gather(block_tables, 1, (positions // BS).long().clamp(max=block_tables.shape[1] - 1)[:, None])[:, 0]
    return torch.where(valid.bool(), blk * BS + positions % BS, torch.full_like(blk, -1)).int()


def decode_advance(nxt, out, tokens, positions, context_lens, valid) -> None:
    out.copy_(nxt)
    tokens.copy_(nxt.int())
    positions.add_(valid)
    context_lens.add_(valid)


def coarse_probes(xq, centroids, cnorm, nprobe: int):
    """fp32 reference of csrc/kernels/coarse.hip: ||c||^2 - 2 q.c per (query, centroid),
    the nprobe smallest in ascending order, ties to the lower centroid id (stable sort)."""
    d = cnorm.float()[None, :] - 2.0 * (xq.float() @ centroids.float().t())
    order = torch.sort(d, dim=1, stable=True).indices
    return order[:, :nprobe].contiguous()
