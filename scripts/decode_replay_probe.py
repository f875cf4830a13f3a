"""Replay the grouped cascade decode attention on a REAL bench batch layout (tables, context
lengths and group plan dumped by the engine with DOCQA_DECODE_DUMP=<dir>), caches rotated
past the MALL, and report time / TB/s plus the per-workgroup timeline (g_group_trace):
prologue (tile list + Q), first-tile latency, streaming loop, epilogue, and how busy the
CUs are over the kernel's span.

Usage: python scripts/decode_replay_probe.py <dump-dir> [step-offset]"""
import json
import math
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch

from docqa_amd import ops


def graph_time(fn, copies, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(copies):
            fn(i)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(copies):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * copies)


def main():
    d = torch.load(os.path.join(sys.argv[1], "decode_batch.pt"), weights_only=True)
    t_off = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    assert ops.load_native()
    tables, lens, bp = d["tables"], d["lens"], d["bp"]
    B = len(tables)
    BS, Hq, Hkv, D = d["block_size"], d["hq"], d["hkv"], d["head_dim"]
    nblk, maxb = d["num_blocks"], d["max_blocks_per_seq"]
    used = sorted({b for t in tables for b in t})
    # compact the pool to the blocks the batch uses (same per-row sharing structure)
    remap = {b: i for i, b in enumerate(used)}
    nb = len(used)
    copies = max(2, (1 << 30) // (2 * nb * Hkv * BS * D * 2) + 1)
    caches = [(torch.randn(nb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16),
               torch.randn(nb, Hkv, BS, D, device="cuda", dtype=torch.bfloat16)) for _ in range(copies)]
    bt = torch.zeros(bp, maxb, dtype=torch.int32)
    for i, t in enumerate(tables):
        bt[i, :len(t)] = torch.tensor([remap[b] for b in t], dtype=torch.int32)
    bt = bt.cuda()
    cl = torch.zeros(bp, dtype=torch.int32)
    cl[:B] = torch.tensor([n + t_off for n in lens], dtype=torch.int32)
    cl = cl.cuda()
    q = torch.randn(bp, (Hq + 2 * Hkv) * D, device="cuda", dtype=torch.bfloat16)
    ns = d["nshared"]
    st = torch.zeros(maxb, dtype=torch.int32)
    st[:ns] = bt[0, :ns].cpu()
    st = st.cuda()
    sl = torch.tensor([ns * BS], dtype=torch.int32, device="cuda")
    groups = d["groups"].cuda()
    tick = ops.decode_ticket(max(bp, 4096) * Hkv, "cuda")
    scale = 1 / math.sqrt(D)
    nchunk = d["cascade_chunks"]
    inline = d["inline"]

    def run(i):
        kc, vc = caches[i % copies]
        return ops.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, st, sl, nchunk, groups, False,
                                                tick, inline)

    sweep = os.environ.get("DOCQA_REPLAY_ITEMS", "")
    if sweep and groups.dim() == 3 and groups.shape[0] == 2:
        # re-plan the same batch for other item-count targets (llm_engine.set_groups' rule:
        # END lengths, the tiles budget giving the most items within the target)
        end = [n + d.get("max_new_tokens", 128) for n in lens]
        skip = 0 if inline else d["nshared"]
        quads = ops.pack_decode_groups(tables, end, d["nshared"], BS, (bp + 1) // 2)
        for target in [int(x) for x in sweep.split(",")]:
            plan, best = None, -1
            for budget in (4, 6, 8, 12, 16, 24, 32, 40, 48, 64, 80, 96, 128, 160, 192, 256, 384, 512):
                p = ops.split_decode_groups(quads, tables, end, skip, BS, bp, budget)
                n_it = int((p[0, :, :4] >= 0).any(1).sum())
                if n_it <= target and n_it > best:
                    plan, best = p, n_it
            if plan is None:
                continue
            gp = plan.cuda()

            def run_p(i, gp=gp):
                kc, vc = caches[i % copies]
                return ops.paged_decode_cascade_grouped(q, kc, vc, bt, cl, Hq, scale, st, sl, nchunk, gp, False,
                                                        tick, inline)

            for v in [int(x) for x in os.environ.get("DOCQA_REPLAY_WAVES", "-1").split(",")]:
                was = torch.ops.docqa.set_group_wave(v)
                print(json.dumps({"sweep_target": target, "items": best, "us": round(graph_time(run_p, copies), 1),
                                  "wave": int(torch.ops.docqa.set_group_wave(-1))}), flush=True)
                torch.ops.docqa.set_group_wave(was)
    distinct = len({b for t, L in zip(tables, cl[:B].tolist()) for b in t[:(L + BS - 1) // BS]})
    kv_bytes = distinct * Hkv * BS * D * 2 * 2
    us = graph_time(run, copies)
    out = {"B": B, "bp": bp, "t_off": t_off, "distinct_blocks": distinct, "kv_MB": round(kv_bytes / 1e6, 1),
           "us": round(us, 1), "TBps": round(kv_bytes / us / 1e6, 2), "nshared": ns, "copies": copies,
           "items": int((groups[0, :, :4] >= 0).any(1).sum()) if groups.dim() == 3 else None,
           "env": {k: v for k, v in os.environ.items() if k.startswith("DOCQA_GROUP")}}
    # timeline
    nwg = Hkv * (groups.shape[1] if groups.dim() == 3 else groups.numel() // 4)
    buf = torch.zeros(nwg * 8, dtype=torch.int64, device="cuda")
    torch.ops.docqa.set_decode_trace(buf)
    run(0)
    torch.cuda.synchronize()
    torch.ops.docqa.set_decode_trace(None)
    tr = buf.view(nwg, 8).cpu()
    live = tr[tr[:, 0] > 0]
    if live.shape[0]:
        t0 = int(live[:, 0].min())
        span = (int(live[:, 4].max()) - t0) / 100.0         # us (100 MHz)
        pro = (live[:, 1] - live[:, 0]).float() / 100
        first = (live[:, 2] - live[:, 1]).float() / 100
        loop = (live[:, 3] - live[:, 2]).float() / 100
        epi = (live[:, 4] - live[:, 3]).float() / 100
        tiles = live[:, 5].float()
        work = live[tiles > 0]
        dur = (live[:, 4] - live[:, 0]).float() / 100
        per_tile = (loop[tiles > 1] / (tiles[tiles > 1] - 1)).median().item() if (tiles > 1).any() else 0
        start = (live[:, 0] - t0).float() / 100
        # concurrency: workgroups in flight at 20 sample points
        samples = []
        for k in range(20):
            tt = t0 + int(k * span * 100 / 20)
            samples.append(int(((live[:, 0] <= tt) & (live[:, 4] >= tt)).sum()))
        out["trace"] = {
            "workgroups": int(live.shape[0]), "with_tiles": int(work.shape[0]), "span_us": round(span, 1),
            "tiles_mean": round(tiles.mean().item(), 1), "tiles_max": int(tiles.max()),
            "dur_us_p50": round(dur.median().item(), 1), "dur_us_max": round(dur.max().item(), 1),
            "prologue_us_p50": round(pro.median().item(), 2), "first_tile_us_p50": round(first.median().item(), 2),
            "loop_us_p50": round(loop.median().item(), 1), "epilogue_us_p50": round(epi.median().item(), 2),
            "epilogue_us_max": round(epi.max().item(), 2), "per_tile_us_p50": round(per_tile, 3),
            "last_start_us": round(start.max().item(), 1), "inflight_wgs": samples,
            "sum_prologue_frac": round((pro.sum() / dur.sum()).item(), 3),
            "sum_first_frac": round((first.sum() / dur.sum()).item(), 3),
            "sum_epilogue_frac": round((epi.sum() / dur.sum()).item(), 3),
            "xcc_counts": torch.bincount(live[:, 7], minlength=8).tolist(),
        }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
