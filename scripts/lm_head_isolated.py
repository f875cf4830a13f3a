"""The batch-256 LM head (mgemm.hip cfg 6, fused greedy argmax) alone, weights cycled past
the 256 MB MALL: the isolated arm of the in-step vs isolated PMC comparison
(scripts/instep_vs_isolated_pmc.sh).  python scripts/lm_head_isolated.py [iters]"""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from docqa_amd import ops  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    assert ops.load_native()
    nat = torch.ops.docqa
    g = torch.Generator(device="cuda").manual_seed(0)
    M, N, K = 256, 128256, 4096
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    ws = [(torch.randn(N, K, device="cuda", generator=g) * 0.02).to(torch.bfloat16) for _ in range(3)]
    for i in range(iters):
        nat.mgemm_argmax(x, ws[i % 3], N, 6)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    main()
