"""Persistent decode-layer chain (mgemm.hip mgemm_chain_kernel) vs the six standalone
launches it replaces (O split-K -> add+RMSNorm -> gate|up+SwiGLU -> down split-K ->
add+RMSNorm -> next QKV split-K), Llama-3-8B shapes at the bench's decode bucket, weights of
NL distinct layers (436 MB each, past the 256 MB MALL), both captured in HIP graphs of NL
layers so launch overhead is the graph's, as in the engine.  Prints one JSON line per M.
Usage: python scripts/chain_probe.py [M ...]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops

ops.load_native()
ops._CHAIN = True
nat = torch.ops.docqa
H, Ko, inter, Nq, NL, eps = 4096, 4096, 14336, 6144, 8, 1e-5


def w(n, k):
    return (torch.randn(n, k, device="cuda") / k ** 0.5).bfloat16()


layers = [dict(o=w(H, Ko), gate_up=w(2 * inter, H), down=w(H, inter), qkv=w(Nq, H),
               post=torch.ones(H, device="cuda").bfloat16(), nxt=torch.ones(H, device="cuda").bfloat16())
          for _ in range(NL)]
ctr = torch.zeros(NL, 16, dtype=torch.int32, device="cuda")


def timed(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps / NL    # us per layer


for M in [int(a) for a in sys.argv[1:]] or [256]:
    plan = ops.chain_plan(M, H, Ko, 2 * inter, Nq)
    S_o, c_o, S_d, c_d, S_q, c_q = plan
    a = torch.randn(M, Ko, device="cuda").bfloat16()
    res = torch.randn(M, H, device="cuda").bfloat16()

    def seq():
        for L in layers:
            x1 = nat.add_rmsnorm_splitk(nat.mgemm(a, L["o"], S_o, c_o), res, L["post"], eps)
            g = nat.mgemm_glu(x1, L["gate_up"], 2)
            x2 = nat.add_rmsnorm_splitk(nat.mgemm(g, L["down"], S_d, c_d), res, L["nxt"], eps)
            nat.mgemm(x2, L["qkv"], S_q, c_q)

    def chain():
        for i, L in enumerate(layers):
            ops.mgemm_chain(a, L["o"], res, L["post"], L["gate_up"], L["down"], L["nxt"], L["qkv"], ctr[i], plan, eps)

    t_seq = timed(seq)
    t_chain = timed(chain)
    t_seq2 = timed(seq)
    t_chain2 = timed(chain)
    err = int(ctr[:, 12].sum())
    print(json.dumps({"M": M, "plan": plan, "seq_us_per_layer": round(min(t_seq, t_seq2), 1),
                      "chain_us_per_layer": round(min(t_chain, t_chain2), 1),
                      "speedup": round(min(t_seq, t_seq2) / min(t_chain, t_chain2), 3), "chain_errors": err}),
          flush=True)

# per-item timeline of one chain launch (s_memrealtime, 100 MHz): phase spans, item compute,
# the dependency wait, the publish (release fence + counter)
if True:
    M = 256
    plan = ops.chain_plan(M, H, Ko, 2 * inter, Nq)
    a = torch.randn(M, Ko, device="cuda").bfloat16()
    res = torch.randn(M, H, device="cuda").bfloat16()
    tr = torch.zeros(4096 * 6, dtype=torch.int64, device="cuda")
    for rep in range(3):
        L = layers[rep % NL]
        tr.zero_()
        nat.mgemm_chain(a, L["o"], res, L["post"], L["gate_up"], L["down"], L["nxt"], L["qkv"], ctr[0], *plan, eps, tr)
        torch.cuda.synchronize()
    t = tr.view(-1, 6).cpu()
    t = t[t[:, 5] > 0]
    base = int(t[:, 2].min())
    names = ["O", "norm1", "gate_up", "down", "norm2", "qkv"]
    for p in range(6):
        r = t[t[:, 0] == p].double()
        if not len(r):
            continue
        us = lambda v: round(float(v) / 100.0, 2)   # noqa: E731  (10 ns ticks -> us)
        print(json.dumps({"phase": names[p], "items": len(r), "first_ready_us": us(r[:, 3].min() - base),
                          "last_done_us": us(r[:, 5].max() - base),
                          "compute_med_us": us((r[:, 4] - r[:, 3]).median()),
                          "compute_max_us": us((r[:, 4] - r[:, 3]).max()),
                          "wait_med_us": us((r[:, 3] - r[:, 2]).median()),
                          "publish_med_us": us((r[:, 5] - r[:, 4]).median()),
                          "publish_max_us": us((r[:, 5] - r[:, 4]).max())}), flush=True)

    # the slow items of each phase: which workgroups / XCDs / tickets
    for p in (0, 2, 3):
        idx = (t[:, 0] == p).nonzero()[:, 0]
        r = t[idx]
        comp = (r[:, 4] - r[:, 3]).double() / 100.0
        xcc = (r[:, 1] >> 16) & 15
        wg = r[:, 1] & 0xFFFF
        order = comp.argsort(descending=True)[:12]
        print(json.dumps({"phase": names[p], "slowest": [[int(idx[j]), int(wg[j]), int(xcc[j]), round(float(comp[j]), 1),
                                                          round(float(r[j, 3] - base) / 100.0, 1)] for j in order],
                          "per_xcc_med_us": [round(float(comp[xcc == x].median()), 1) if (xcc == x).any() else None
                                             for x in range(8)],
                          "per_xcc_max_us": [round(float(comp[xcc == x].max()), 1) if (xcc == x).any() else None
                                             for x in range(8)]}), flush=True)
