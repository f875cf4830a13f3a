"""Operator dispatch: GPU tensors -> hand-written gfx950 HIP kernels (torch.ops.docqa.*),
CPU tensors -> the fp32 PyTorch reference in :mod:`docqa_amd.ops.reference`.

The native library is built in-tree by :mod:`docqa_amd.ops.build` into
``ops/_docqa_C.so``.  On a GPU tensor there is deliberately NO silent fallback: if the
extension is missing the op raises, so a GPU run can never pass on eager PyTorch by
accident.  Set ``DOCQA_FORCE_REFERENCE=1`` to route GPU tensors through the reference
(numerics debugging only).
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

from . import reference as ref

# DOCQA_NATIVE_LIB: load another build of the extension (same-box A/B of two kernel builds)
_LIB_PATH = Path(os.environ.get("DOCQA_NATIVE_LIB") or Path(__file__).resolve().parent / "_docqa_C.so")
_lock = threading.Lock()
_loaded = False
_load_error: str | None = None
_FORCE_REF = os.environ.get("DOCQA_FORCE_REFERENCE", "0") == "1"


def library_path() -> Path:
    return _LIB_PATH


def load_native(build_if_missing: bool = False) -> bool:
    """Load ``_docqa_C.so`` (optionally building it first). Returns True on success."""
    global _loaded, _load_error
    if _loaded:
        return True
    with _lock:
        if _loaded:
            return True
        if not _LIB_PATH.exists() and build_if_missing:
            from .build import build

            build(verbose=False)
        if not _LIB_PATH.exists():
            _load_error = f"native library not built: {_LIB_PATH} (run python -m docqa_amd.ops.build)"
            return False
        try:
            torch.ops.load_library(str(_LIB_PATH))
            _loaded = True
        except Exception as e:  # pragma: no cover - surfaced by native()
            _load_error = f"failed to load {_LIB_PATH}: {e}"
        return _loaded


def native_loaded() -> bool:
    return _loaded


def _native():
    if not _loaded and not load_native():
        raise RuntimeError(f"docqa native kernels unavailable on a GPU tensor: {_load_error}")
    return torch.ops.docqa


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda and not _FORCE_REF


class use_reference:
    """Context manager: route GPU tensors through the PyTorch reference (model-level
    numerics tests compare a whole forward on native vs reference ops)."""

    def __enter__(self):
        global _FORCE_REF
        self._prev = _FORCE_REF
        _FORCE_REF = True
        return self

    def __exit__(self, *exc):
        global _FORCE_REF
        _FORCE_REF = self._prev
        return False


# ----------------------------------------------------------------------------- norms
def rmsnorm(x, w, eps: float):
    if _gpu(x):
        return _native().rmsnorm(x.contiguous(), w, eps)
    return ref.rmsnorm(x, w, eps)


def add_rmsnorm(x, residual, w, eps: float):
    """residual <- residual + x (in place, bf16); returns rmsnorm(residual) * w."""
    if _gpu(x):
        return _native().add_rmsnorm(x.contiguous(), residual, w, eps)
    return ref.add_rmsnorm(x, residual, w, eps)


def layernorm(x, residual, gamma, beta, eps: float):
    if _gpu(x):
        return _native().layernorm(x.contiguous(), residual, gamma, beta, eps)
    return ref.layernorm(x, residual, gamma, beta, eps)


# ----------------------------------------------------------------------------- rope / kv
def rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D):
    if _gpu(qkv):
        if slot_mapping is None:
            k_cache = v_cache = qkv  # unused placeholders
        _native().rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
        return
    ref.rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)


rope_cos_sin = ref.rope_cos_sin


# ----------------------------------------------------------------------------- activations
def silu_mul(gu, interleaved: bool = False):
    if _gpu(gu):
        return _native().silu_mul(gu.contiguous(), interleaved)
    return ref.silu_mul(gu, interleaved)


glu_interleave, glu_split = ref.glu_interleave, ref.glu_split


def glu_linear(x, w_il):
    """silu(x Wg^T) * (x Wu^T) for 8-interleaved gate|up weights at <= 128 decode rows: the
    skinny fused-SwiGLU decode GEMM (dgemm.hip); 129..512 rows take the mid-M kernel
    (:func:`mid_plan`), so no decode bucket runs the library GEMM.  Measured vs hipBLASLt +
    silu_mul at M = 64 / 96 / 128: 50.9 / 60.0 / 63.1 us vs 56.4 / 57.6 / 59.7
    (profiles/r4_lm_head_probe.log)."""
    if _gpu(x):
        N, K = w_il.shape
        if x.numel() // K <= 128 and N % 64 == 0 and K % 512 == 0:
            return _native().dgemm_glu(x.contiguous(), w_il)
    return silu_mul(torch.nn.functional.linear(x, w_il), interleaved=True)


def bias_act(x, bias, residual=None, gelu: bool = False):
    if _gpu(x):
        return _native().bias_act(x.contiguous(), bias, residual, gelu)
    return ref.bias_act(x, bias, residual, gelu)


# ----------------------------------------------------------------------------- fused GEMM
EPI_NONE, EPI_BIAS, EPI_BIAS_GELU, EPI_BIAS_RES, EPI_GLU = 0, 1, 2, 3, 4


def linear_fused(x, w, bias=None, residual=None, epi: int = EPI_BIAS):
    """act(x @ w^T + bias) (+ residual) on the hand-written MFMA GEMM (N % 128 == 0,
    K % 64 == 0); other shapes fall back to hipBLASLt + the element-wise kernel."""
    if _gpu(x):
        N, K = w.shape
        if N % 128 == 0 and K % 64 == 0:
            return _native().gemm(x.contiguous(), w, bias, residual, epi)
        y = torch.nn.functional.linear(x, w)
        if epi == EPI_NONE:
            return y
        return bias_act(y, bias, residual if epi == EPI_BIAS_RES else None, epi == EPI_BIAS_GELU)
    return ref.linear_fused(x, w, bias, residual, epi)


def _splits_for(N: int, K: int, tile: int, min_wgs: int = 192) -> int:
    """Smallest split-K count giving >= ``min_wgs`` workgroups of ``tile`` weight rows
    (whole 512-deep ring turns per slice)."""
    tiles, S = N // tile, 1
    while tiles * S < min_wgs and K % (2 * S) == 0 and (K // (2 * S)) % 512 == 0:
        S *= 2
    return S if K % S == 0 and (K // S) % 512 == 0 else 0


def decode_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(split-K count, weight rows per workgroup) of the skinny decode GEMM
    (csrc/kernels/dgemm.hip) for an [M, K] x [N, K]^T projection; split 0 where hipBLASLt
    is faster or the shape is unsupported.

    Measured per Llama-3-8B projection (profiles/r1_bench_kernels_dgemm.json at M <= 64,
    profiles/r1_dgemm_m128_sweep.log at 65-128 rows, weights rotated past the MALL): the
    LM head and, above 32 rows, gate|up stay on hipBLASLt; at <= 64 rows QKV / O / down use
    64-row tiles with the smallest split giving >= 192 workgroups; at 65-128 rows 128-row
    tiles (X re-read from L2 half as often) where such a split exists (QKV S=4: 21.9 us vs
    hipBLASLt 25.2 at M=128; O S=8: 17.2 vs 24.4), else 64-row tiles (down S=4: 40.7 vs 75.1)."""
    if M > 192 or N % 64 or N >= 65536 or (N >= 16384 and M > 32):
        return 0, 64
    if M > 128:
        # 129-192 rows (three m-tiles per wave, 64-row tiles only): only where a split gives
        # a full round of 256 workgroups -- O 21.8 us vs tuned hipBLASLt 23.9, down 54.2 vs
        # 65.3 at M=192; QKV (192 workgroups at S=2: 33.7 vs 27.3) stays on hipBLASLt
        # (profiles/r1_dgemm_m192_sweep.log)
        S = _splits_for(N, K, 64)
        return (S, 64) if S and (N // 64) * S >= 256 else (0, 64)
    # (QKV at S=4 times 11.6 vs 13.4 us alone at M = 1, profiles/r4_b1_decode_gemm_split_probe.log,
    # but the fused attention then sums twice the slabs: batch-1 decode 471-473 vs 468-470 ms
    # per query, profiles/r4_b1_ab.log -- S=2 stays)
    if M <= 64:
        return _splits_for(N, K, 64), 64
    S64 = _splits_for(N, K, 64)
    if N % 128 == 0:
        S = _splits_for(N, K, 128)
        # 128-row tiles, unless they need more than 4 split-K slabs where 64-row tiles fill
        # the chip with <= 4: the fused consumer re-reads every fp32 slab (O at M=128:
        # S=8 t128 17.2 us + 16.8 MB of slabs vs S=4 t64 16.5 us + 8.4 MB)
        if S and (N // 128) * S >= 192 and not (S > 4 and 0 < S64 <= 4 and (N // 64) * S64 >= 192):
            return S, 128
    return S64, 64


def decode_splits(M: int, N: int, K: int) -> int:
    """Split-K count of :func:`decode_plan` (0: use hipBLASLt)."""
    return decode_plan(M, N, K)[0]


def decode_linear(x, w):
    """x @ w^T for a decode step (<= 128 rows): the skinny weight-streaming MFMA kernel
    where it beats hipBLASLt on MI355X, else F.linear."""
    if _gpu(x):
        N, K = w.shape
        S = decode_splits(x.numel() // K, N, K)
        if S:
            return _native().dgemm(x.contiguous(), w, S)
    return torch.nn.functional.linear(x, w)


def dgemm_partial(x, w, splits: int, tile_rows: int = 64):
    """Split-K partial slabs [S, M, N] fp32 of x @ w^T (combine fused into the consumer:
    add_rmsnorm_splitk / rope_cache_splitk); tile_rows 64 or 128 weight rows per workgroup."""
    if _gpu(x):
        return _native().dgemm_partial(x.contiguous(), w, splits, tile_rows)
    K = w.shape[1]
    xs = x.float().reshape(-1, splits, K // splits)
    ws = w.float().reshape(-1, splits, K // splits)
    return torch.einsum("msk,nsk->smn", xs, ws).contiguous()


MID_M_MIN, MID_M_MAX = 129, 512
_MID_OFF = os.environ.get("DOCQA_MID_GEMM", "1") == "0"
_MID_CFG = int(os.environ.get("DOCQA_MID_CFG", "2"))
_MID_NARROW = os.environ.get("DOCQA_MID_NARROW", "1") == "1"
_MID_WG_CAP = int(os.environ.get("DOCQA_MID_WG_CAP", "224"))
_L2_XCD_BYTES = 4 << 20          # one XCD's L2 (MI355X_MICROARCH.md)


def mid_plan(M: int, N: int, K: int, glu: bool = False) -> tuple[int, int]:
    """(split-K count, kernel variant) of the mid-M decode GEMM (csrc/kernels/mgemm.hip) for
    an [M, K] x [N, K]^T projection at 129..512 rows; (0, 0) where it does not apply.
    ``glu``: the plan is for the fused-SwiGLU gate|up launch (mgemm_glu), which never
    splits K and has no 64-wide (cfg 7) variant -- only a non-zero S means "use it".

    Every workgroup owns all 256 rows of an m-tile x 128 weight rows; S is the largest
    divisor of K / 128 keeping (N / 128) x m-tiles x S <= 224 workgroups (one round on the
    256 CUs; fewer, larger slabs for the consumer where a round is already full).
    Measured at M = 256 against hipBLASLt (scripts/mgemm_probe.py, weights rotated past the
    MALL; profiles/r2_mgemm_probe_m256_v5.log): QKV S=4 21.9 us vs 43.1, O S=4 20.3 vs
    26.8 (S=8: 20.8 with twice the slab bytes), down S=7 40.1 vs 63.3, fused SwiGLU gate|up
    S=1 75.4 vs 67.8 + a 5.9 us silu_mul + a [M, 2I] round trip."""
    if _MID_OFF or not (MID_M_MIN <= M <= MID_M_MAX) or N % 128 or K % 128:
        return 0, 0
    # 129..192 rows: QKV / O / down gain over the skinny kernel and hipBLASLt (QKV 20.2-20.8
    # vs 27.7-33.4 us; profiles/r4_lm_head_probe.log, r2_mgemm_probe_m128_192.log); the wide
    # gate|up with fused SwiGLU is at parity with hipBLASLt + silu_mul (62.3 / 64.7 vs
    # 62.4 / 66.5 us at M = 160 / 192) and takes it too
    tiles = (N // 128) * ((M + 255) // 256)
    kb = K // 128
    S = max(s for s in range(1, kb + 1) if kb % s == 0 and (s == 1 or tiles * s <= _MID_WG_CAP))
    if glu:
        return S, _MID_CFG
    if _MID_CFG == 2 and M * K * 2 > _L2_XCD_BYTES and kb % 8 == 0 and tiles * 8 <= 256 and S < 8:
        # activations larger than one XCD's L2 (down: 256 x 14336 bf16 = 7.3 MB): 8 slices,
        # one per XCD (mgemm.hip remap 1), so each L2 holds only its 0.9 MB slice of X --
        # down S=8 40.5 vs S=7 44.1 us, 46.4 vs 48.8 with the add+norm consumer
        # (profiles/r5_mid_consumer_probe.log)
        return 8, _MID_CFG
    if _MID_CFG == 2 and _MID_NARROW and S > 1 and tiles * S <= 128 and N % 64 == 0:
        # the split left half the chip idle (O: 32 tiles x S=4): 64-wide tiles (cfg 7) at
        # the same split fill it with the same slab bytes -- O 17.5 vs 20.7 us
        # (profiles/r2_mgemm_probe_bn64.log)
        return S, 7
    if _MID_CFG == 2 and _MID_NARROW and S == 1 and tiles * 2 <= 256 and N % 64 == 0:
        # no split under the cap (the 70B TP-8 O / down shards, 128 tiles at 257..512 rows):
        # twice the workgroups -- short K (O, 1024) by 64-wide tiles, 22.6 vs 26.3 us at 512
        # rows (hipBLASLt 23.2), long K (down, 3584) by a 2-way split, 46.5 vs 58.8 (46.1)
        # (profiles/r6_prefill_mid_plans.log)
        return (2, 2) if K >= 2048 and kb % 2 == 0 else (1, 7)
    return S, _MID_CFG


# bf16 split-K slabs for the mid-M decode GEMM's fused consumers (RoPE + cache write, add +
# RMSNorm) at TP = 1: half the slab bytes the GEMM writes and its consumer reads; each
# partial is rounded to bf16 once before the consumer's fp32 sum (as a bf16 all-reduce
# rounds each rank's partial)
SLAB_BF16 = os.environ.get("DOCQA_SLAB_BF16", "1") == "1"


def mgemm_partial(x, w, splits: int, cfg: int = 0, bf16: bool = False):
    """Split-K partial slabs [S, M, N] fp32 (``bf16``: bf16) of x @ w^T on the mid-M decode
    GEMM (S = 1 without ``bf16``: the bf16 product [M, N])."""
    if _gpu(x):
        if bf16:
            return _native().mgemm_slab16(x.contiguous(), w, splits, cfg)
        return _native().mgemm(x.contiguous(), w, splits, cfg)
    if splits == 1 and not bf16:
        return torch.nn.functional.linear(x, w)
    K = w.shape[1]
    xs = x.float().reshape(-1, splits, K // splits)
    ws = w.float().reshape(-1, splits, K // splits)
    out = torch.einsum("msk,nsk->smn", xs, ws).contiguous()
    return out.to(torch.bfloat16) if bf16 else out


def pgemm_partial(x, w, splits: int):
    """Split-K partial slabs [S, M, N] fp32 of x @ w^T on the 256 x 256 prefill GEMM."""
    if _gpu(x):
        return _native().pgemm_partial(x.contiguous(), w, splits)
    K = w.shape[1]
    xs = x.float().reshape(-1, splits, K // splits)
    ws = w.float().reshape(-1, splits, K // splits)
    return torch.einsum("msk,nsk->smn", xs, ws).contiguous()


def mgemm_glu(x, w_il, cfg: int = 0):
    """silu(x Wg^T) * (x Wu^T) for 8-interleaved gate|up weights on the mid-M decode GEMM."""
    if _gpu(x):
        return _native().mgemm_glu(x.contiguous(), w_il, cfg)
    return silu_mul(torch.nn.functional.linear(x, w_il), interleaved=True)


# batch-256 decode gate|up as 256-wide tiles split over K into bf16 slabs + the split-K
# SwiGLU consumer (act.hip silu_mul_splitk16) instead of the fused-SwiGLU 128-wide tiles: X
# is re-read from L2 112 instead of 224 times (scripts/gateup_split_probe.py, cold weights:
# GEMM 64.3 us at cfg 6 S=2 vs 78.8 us fused)
_GLU_SPLIT16 = os.environ.get("DOCQA_GLU_SPLIT16", "0") == "1"


def glu_split16_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(S, cfg) of the split bf16-slab gate|up (:func:`glu_split16`) for an [M, K] x [N, K]^T
    gate|up at TP = 1, or (0, 0): one 256-row m-tile (193..256 rows), 256-wide tiles, two K
    slices -- (N / 256) x 2 workgroups must fit one round of the chip."""
    if not (SLAB_BF16 and _GLU_SPLIT16) or not (193 <= M <= 256):
        return 0, 0
    if N % 256 or K % 256 or (N // 256) * 2 > 256:
        return 0, 0
    return 2, 6


def glu_split16(x, w_il, S: int, cfg: int):
    """silu(x Wg^T) * (x Wu^T) from S bf16 split-K slabs (mgemm cfg ``cfg``)."""
    if _gpu(x):
        return _native().silu_mul_splitk(_native().mgemm_slab16(x.contiguous(), w_il, S, cfg))
    return silu_mul(torch.nn.functional.linear(x, w_il), interleaved=True)


# ----------------------------------------------------------------------------- prefill GEMM
_PGEMM_OFF = os.environ.get("DOCQA_PGEMM", "1") == "0"
# below this many 256 x 256 tiles the 128 x 128 encoder GEMM (gemm.hip, 4x the workgroups)
# fills the chip better (scripts/pgemm_probe.py)
_PGEMM_MIN_TILES = int(os.environ.get("DOCQA_PGEMM_MIN_TILES", "128"))


def pgemm_ok(M: int, N: int, K: int) -> bool:
    """Shapes the prefill GEMM (csrc/kernels/pgemm.hip) takes: N % 256, K % 128, 32-bit
    row offsets, and enough 256 x 256 tiles to fill the chip."""
    return (not _PGEMM_OFF and M > 0 and N % 256 == 0 and K % 128 == 0
            and max(M, N) * K * 2 < (1 << 32) and ((M + 255) // 256) * (N // 256) >= _PGEMM_MIN_TILES)


PREFILL_MID_MAX = 2048
# Mid-M prefill (513..2048 packed prompt tokens; the Llama-3-70B TP-8 shards from 257 rows):
# every projection on the hand-written kernels -- no library GEMM.  Measured WITH each
# projection's consumer and weights rotated past the MALL (scripts/prefill_mid_probe.py,
# profiles/r6_prefill_mid_plans.log): where the 256 x 256 tiles cannot fill the 256 CUs the
# K dimension is split into fp32 slabs (pgemm.hip EPI_PARTIAL, one K slice per XCD group)
# that the consumer which runs anyway sums -- RoPE + KV write (QKV), residual add + RMSNorm
# (O / down), SwiGLU (gate|up: act.hip silu_mul_splitk) -- :func:`prefill_split_plan`; a
# few measured shapes keep the mid-M kernel (:func:`prefill_plan`).  What the forward runs
# (:func:`prefill_route`) against hipBLASLt + the same consumer at 512..2048 rows: 0.93..1.47x,
# 36 of 40 (shape, M) points >= 0.95x.
_PREFILL_SPLIT_MIN_K = 1024       # K per slice below this loses to fewer slices (O at 512 rows: S=8 42.0 vs S=4 37.5 us)


_PREFILL_PLANS = os.environ.get("DOCQA_PREFILL_PLANS", "1") != "0"


def prefill_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(split-K count, mgemm cfg) of a 513..2048-row prefill projection on the mid-M kernel,
    (0, 0) for the 256 x 256 kernel (split-K slabs where :func:`prefill_split_plan` says so,
    else bf16 tiles).  S >= 2: fp32 slabs into the split-K consumers (RoPE + KV write, add +
    RMSNorm); S == 1: the bf16 product.  Since round 6 the 256 x 256 split plans take every
    shape they apply to except the two points measured faster here (8B O and the 70B TP-8
    down shard at 769..1024 rows, profiles/r6_prefill_mid_plans.log); the remaining rules
    are round 4's (profiles/r4_prefill_mid_probe.log) for shapes no split plan takes."""
    if not _PREFILL_PLANS or _MID_OFF or not (MID_M_MAX < M <= PREFILL_MID_MAX) or N % 128 or K % 128:
        return 0, 0
    if 769 <= M <= 1024 and (N, K) in ((4096, 4096), (8192, 3584)):
        # the two measured points where the mid-M kernel beats the split 256 x 256 tiles:
        # 8B O S=2 48.5 vs pgemm S=4 50.9 us, 70B TP-8 down S=1 71.9 vs pgemm S=2 75.4
        return (2, 2) if N == 4096 else (1, 2)
    if prefill_split_plan(M, N, K):
        return 0, 0
    if N < 4096:
        # narrow N (the 70B TP-8 QKV shard, N 1280 x K 8192): the mid-M kernel's few 128-wide
        # tiles lose to the 256 x 256 kernel's split-K (profiles/r4_pgemm_mid_probe.log)
        return 0, 0
    if N >= 6144 and K <= 4096:          # QKV-like: wide N
        return (1, 2) if M <= 1024 else (0, 0)
    if M <= 1024 and (K // 128) % 2 == 0:
        return 2, 2
    return 1, 2


def prefill_split_plan(M: int, N: int, K: int, glu: bool = False) -> int:
    """Split-K count for a prefill projection whose 256 x 256 tiles cannot fill the chip:
    the largest S (<= DOCQA_PREFILL_SPLIT_MAX) with tiles x S <= 256 workgroups and >= 1024
    of K per slice.  The fp32 slabs [S, M, N] go straight into the split-K consumer that runs
    anyway (RoPE + KV write, (TP all-reduce +) add + RMSNorm, SwiGLU).  Measured with the
    consumer (profiles/r6_prefill_mid_plans.log): 8B down S=4 93.8 vs hipBLASLt 115.9 us at
    768 rows, QKV S=2 55.3 vs 55.2, O S=4 42.3 vs 40.3; 70B TP-8 gate|up S=4 69.2 vs 84.2 at
    512 rows, QKV shard S=8 32.2 vs 35.8.  0: no split (enough tiles, or not a pgemm shape).
    ``glu``: the gate|up shard's S (consumer silu_mul_splitk), from 257 rows (measured at
    512+; below that the decode-sized mid-M SwiGLU kernel keeps it).  DOCQA_PREFILL_SPLIT=0
    disables."""
    if (not _PREFILL_SPLIT or _PGEMM_OFF or M <= 0 or N % 256 or K % 256
            or max(M, N) * K * 2 >= (1 << 32)):
        return 0
    if M <= MID_M_MAX and not (N < 4096 or (glu and M > 256)):
        return 0          # decode-sized M: the mid-M kernel's plans (mid_plan)
    tiles = ((M + 255) // 256) * (N // 256)
    S = 1
    while (S < _PREFILL_SPLIT_MAX and tiles * S * 2 <= 256 and K % (128 * S * 2) == 0
           and K // (S * 2) >= _PREFILL_SPLIT_MIN_K):
        S *= 2
    return S if S >= 2 else 0


def down_small_split(M: int, N: int, K: int) -> int:
    """Split-K count of a 257..512-row prefill's down projection on the 256 x 256 kernel
    (long K: the 8B down, 14336): S=8 slabs into add + RMSNorm, 67.5 vs 77.5 us for the mid-M
    kernel's S=4 and 98.7 for hipBLASLt at 512 rows (profiles/r6_prefill_mid_plans.log).
    0 where it does not apply (fewer than 4 slices of >= 1024)."""
    if not (256 < M <= MID_M_MAX) or _PGEMM_OFF or not _PREFILL_SPLIT or N % 256 or K % 256:
        return 0
    tiles = ((M + 255) // 256) * (N // 256)
    S = 1
    while S < 8 and tiles * S * 2 <= 256 and K % (128 * S * 2) == 0 and K // (S * 2) >= _PREFILL_SPLIT_MIN_K:
        S *= 2
    return S if S >= 4 else 0


_PREFILL_SPLIT = os.environ.get("DOCQA_PREFILL_SPLIT", "1") != "0"
_PREFILL_SPLIT_MAX = int(os.environ.get("DOCQA_PREFILL_SPLIT_MAX", "8"))


def prefill_linear(x, w):
    """x @ w^T for the prefill projections (M = packed prompt tokens) on the hand-written
    MFMA GEMMs: the mid-M kernel's bf16 product where :func:`prefill_plan` says so, the
    256 x 256 8-phase kernel (pgemm.hip) where it has enough tiles, else the 128 x 128
    kernel (gemm.hip); hipBLASLt only for shapes none takes."""
    if _gpu(x):
        N, K = w.shape
        M = x.numel() // K
        S, cfg = prefill_plan(M, N, K)
        if S == 1:
            return _native().mgemm(x.contiguous(), w, 1, cfg)
        Sp = prefill_split_plan(M, N, K)
        if Sp:
            # a caller without a split-K consumer (the mixed prefill/decode forward): the
            # slabs summed here, still ahead of the 128 x 128 kernel at these shapes
            return _native().pgemm_partial(x.contiguous(), w, Sp).sum(0).to(torch.bfloat16)
        if pgemm_ok(M, N, K):
            return _native().pgemm(x.contiguous(), w, 0)
        if N % 128 == 0 and K % 64 == 0:
            return _native().gemm(x.contiguous(), w, None, None, EPI_NONE)
    return torch.nn.functional.linear(x, w)


def prefill_route(M: int, N: int, K: int, glu: bool = False, down: bool = False):
    """(label, fn(x, w)) of what a prefill projection of M rows runs in models/llama.py
    (its per-forward plan logic, mirrored here for probes): split-K slab plans return the
    fp32 slabs [S, M, N] their consumer sums; ``down``: the 257..512-row down override."""
    nat = _native
    if glu:
        if M <= MID_M_MAX and not (pgemm_ok(M, N, K) or prefill_split_plan(M, N, K, glu=True)):
            Sg, cg = mid_plan(M, N, K, glu=True)
            if Sg:
                return f"mgemm_glu c{cg}", lambda x, w: nat().mgemm_glu(x.contiguous(), w, cg)
            return "glu_linear", glu_linear
        Sg = prefill_split_plan(M, N, K, glu=True)
        return (f"pgemm S{Sg}+silu_splitk" if Sg else "prefill_glu"), prefill_glu
    if down and M <= MID_M_MAX and M > 256 and down_small_split(M, N, K):
        Sd = down_small_split(M, N, K)
        return f"pgemm S{Sd}", lambda x, w: nat().pgemm_partial(x.contiguous(), w, Sd)
    if M <= MID_M_MAX:
        S, c = mid_plan(M, N, K)
        if S:
            return f"mgemm S{S} c{c}", lambda x, w: nat().mgemm(x.contiguous(), w, S, c)
        S, t = decode_plan(M, N, K)
        return f"dgemm S{S} t{t}", lambda x, w: dgemm_partial(x, w, S, t)
    S, c = prefill_plan(M, N, K)
    if S >= 2:
        return f"mgemm S{S} c{c}", lambda x, w: nat().mgemm(x.contiguous(), w, S, c)
    if not S:
        Sp = prefill_split_plan(M, N, K)
        if Sp:
            return f"pgemm S{Sp}", lambda x, w: nat().pgemm_partial(x.contiguous(), w, Sp)
    return "prefill_linear", prefill_linear


_GLU128 = os.environ.get("DOCQA_GLU128", "1") != "0"


def prefill_glu(x, w_il):
    """silu(x Wg^T) * (x Wu^T) for 8-interleaved gate|up weights at prefill sizes: SwiGLU
    fused into the 256 x 256 GEMM's epilogue (no [M, 2I] round trip through HBM)."""
    if _gpu(x):
        N, K = w_il.shape
        M = x.numel() // K
        S = prefill_split_plan(M, N, K, glu=True)
        if S:
            # too few 256 x 256 tiles (the 70B TP-8 shard: 56 at 512 rows): K split into fp32
            # slabs, summed by the SwiGLU consumer -- 69.2 vs hipBLASLt + silu_mul 84.2 us
            return _native().silu_mul_splitk(_native().pgemm_partial(x.contiguous(), w_il, S))
        if pgemm_ok(M, N, K):
            return _native().pgemm(x.contiguous(), w_il, 1)
        if (_GLU128 and N % 128 == 0 and K % 64 == 0 and ((M + 255) // 256) * (N // 128) < 128
                and ((M + 127) // 128) * (N // 128) >= 192):
            # too few 256 x 256 tiles, and the 256 x 128 kernel would leave half the CUs idle:
            # the 128 x 128 tiles with the SwiGLU epilogue (gemm.hip EPI_GLU) -- 70B TP-8
            # gate|up shard at 512 rows 90.8 us vs 106.1 (256 x 128) and 132.7 (256 x 256);
            # hipBLASLt + silu_mul 64.6 (profiles/r5_pgemm_70b_split_probe.log)
            return _native().gemm(x.contiguous(), w_il, None, None, EPI_GLU)
        if N % 128 == 0 and K % 128 == 0:
            return _native().mgemm_glu(x.contiguous(), w_il, 2)
    return silu_mul(prefill_linear(x, w_il), interleaved=True)


# LM head: 256-wide tiles (mgemm.hip cfg 6) halve the X re-reads of the 1002-tile vocab
# sweep -- 281 vs 326 us with the argmax fused at M = 256 (profiles/r2_mgemm_probe_m256_v6.log)
_LM_CFG = int(os.environ.get("DOCQA_LM_HEAD_CFG", "6"))
_GEMV_LM = os.environ.get("DOCQA_GEMV_LM", "1") != "0"


def lm_head_argmax(x, w, n_valid: int, cfg: int = -1, with_values: bool = False):
    """Greedy token ids argmax(bf16(x @ w[:n_valid]^T)) with the LM-head GEMM and the argmax
    fused (mgemm.hip EPI_ARGMAX): the [M, vocab] logits never reach HBM.  ``with_values``:
    (ids, picked logit fp32) -- a vocab-parallel shard's candidates for comm.tp_argmax."""
    if _gpu(x):
        N, K = w.shape
        if (_GEMV_LM and x.numel() == K and N % 16 == 0 and K % 2048 == 0 and K // 2048 <= 2
                and n_valid > 0):
            # one row: the register-streaming GEMV with the argmax in its epilogue
            # (profiles/r6_b1_lm_head_gemv_ab.log)
            ids, vals = _native().gemv_argmax_val(x.contiguous(), w, int(n_valid))
            return (ids, vals) if with_values else ids
        if x.numel() // K <= 32 and N % 64 == 0 and K % 512 == 0:
            # <= 32 rows (batch-1 decode included): the skinny weight-streaming kernel with
            # the argmax in its epilogue (dgemm.hip EPI_ARGMAX) -- 197.6 / 203.4 us at M = 1 /
            # 32 vs hipBLASLt + argmax 190.1 / 201.3; from 33 rows the mid-M kernel's 256-row
            # tiles stream the vocab once (256-275 us flat; profiles/r4_lm_head_probe.log)
            ids, vals = _native().dgemm_argmax_val(x.contiguous(), w, int(n_valid))
            return (ids, vals) if with_values else ids
        if cfg < 0:
            cfg = _LM_CFG if w.shape[0] % 256 == 0 else _MID_CFG
        if with_values:
            return _native().mgemm_argmax_val(x.contiguous(), w, int(n_valid), cfg)
        return _native().mgemm_argmax(x.contiguous(), w, int(n_valid), cfg)
    logits = torch.nn.functional.linear(x, w[:n_valid])
    ids = ref.argmax(logits)
    if with_values:
        return ids, logits.gather(1, ids[:, None])[:, 0].float()
    return ids


def lm_head_logits(x, w):
    """bf16 logits x @ w^T of the LM head for SAMPLED rows (temperature > 0: the Ollama
    API's options), on the hand-written GEMMs at every row count: the skinny
    weight-streaming kernel up to 192 rows (dgemm.hip, one pass over the vocab), the mid-M
    kernel with 256-wide tiles up to 512, the prefill kernels
    beyond -- no library GEMM.  Greedy rows never get here: their
    argmax is fused into the GEMM (:func:`lm_head_argmax`)."""
    if _gpu(x):
        N, K = w.shape
        M = x.numel() // K
        if 0 < M <= 192 and N % 64 == 0 and K % 512 == 0:
            return _native().dgemm(x.contiguous(), w, 1)
        if 0 < M <= MID_M_MAX and N % 128 == 0 and K % 128 == 0 and not _MID_OFF:
            cfg = _LM_CFG if N % 256 == 0 else _MID_CFG
            return _native().mgemm(x.contiguous(), w, 1, cfg)
        return prefill_linear(x, w)
    return torch.nn.functional.linear(x, w)


def lm_head_argmax_shape_ok(N: int, K: int) -> bool:
    return not _MID_OFF and N % 128 == 0 and K % 128 == 0


def lm_head_argmax_ok(M: int, N: int, K: int) -> bool:
    """Fused LM head + argmax at every decode bucket: dgemm.hip up to 32 rows, mgemm.hip
    from 33 to 512 (no [M, vocab] logits, no library GEMM)."""
    if M <= 32 and N % 64 == 0 and K % 512 == 0:
        return M > 0
    return not _MID_OFF and 0 < M <= MID_M_MAX and N % 128 == 0 and K % 128 == 0


def embed_rmsnorm(ids, table, w, eps: float):
    """(h, x): h = table[ids] (the residual stream), x = rmsnorm(h) * w -- the Llama input
    embedding and the first layer's norm in one launch."""
    if _gpu(table):
        return _native().embed_rmsnorm(ids.contiguous(), table, w, float(eps))
    h = embedding(ids, table)
    return h, rmsnorm(h, w, eps)


_XN = os.environ.get("DOCQA_DECODE_XN", "1") != "0"


def xn_ok(M: int, K: int) -> bool:
    """Batch-1 projections that build their own input row (residual add + RMSNorm of the
    previous projection's slabs, in LDS) -- :func:`dgemm_partial_xn`, :func:`dgemm_glu_xn`."""
    return _XN and M == 1 and K <= 4096 and K % 512 == 0


def dgemm_partial_xn(Pin, res_in, res_out, gamma, eps: float, w, splits: int):
    """Split-K slabs of x @ w^T for the one row x = rmsnorm(res_in + bf16(sum Pin)) * gamma,
    built inside the projection (no add_rmsnorm launch); res_out <- res_in + bf16(sum Pin)
    (a second buffer -- every workgroup still reads res_in)."""
    if _gpu(Pin):
        return _native().dgemm_partial_xn(Pin, res_in, res_out, gamma, float(eps), w, int(splits))
    res_out.copy_(res_in)
    x = ref.add_rmsnorm(Pin.sum(0).to(res_out.dtype).view_as(res_out), res_out, gamma, eps)
    return torch.nn.functional.linear(x.float(), w.float())[None].reshape(1, 1, -1).expand(splits, 1, -1) / splits


def dgemm_glu_xn(Pin, res_in, res_out, gamma, eps: float, w_il):
    """silu(x Wg^T) * (x Wu^T) for x = rmsnorm(res_in + bf16(sum Pin)) * gamma (one row, built
    in-kernel); res_out <- res_in + bf16(sum Pin)."""
    if _gpu(Pin):
        return _native().dgemm_glu_xn(Pin, res_in, res_out, gamma, float(eps), w_il)
    res_out.copy_(res_in)
    x = ref.add_rmsnorm(Pin.sum(0).to(res_out.dtype).view_as(res_out), res_out, gamma, eps)
    return silu_mul(torch.nn.functional.linear(x, w_il), interleaved=True)


_GEMV = os.environ.get("DOCQA_GEMV", "1") != "0"


_GEMV_DOWN = os.environ.get("DOCQA_GEMV_DOWN", "1") == "1"
_GEMV_R = int(os.environ.get("DOCQA_GEMV_R", "8"))   # rows per workgroup, K <= 4096 (A/B knob)


def gemv_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(split-K count, weight rows per workgroup) of the batch-1 register-streaming GEMV
    (dgemm.hip gemv_kernel: every lane issues all its weight loads at once, no LDS ring)
    for a one-row projection; (0, 0) where the ring kernel stays.  Measured at M = 1 on the
    Llama-3-8B projections, weights rotated past the MALL (profiles/r6_gemv_probe.log): O
    7.8 vs 8.8 us for the ring kernel's plan; the QKV with its input row built in-kernel
    (XNormIn: every workgroup runs that prologue, so few wide workgroups win) 13.3 vs 15.4
    at 8 rows per workgroup, no split (17.9 at 4 rows x 2 slices).  The down projection
    (K 14336) alone is 21.3 vs the ring's 20.9 us, but on the GEMV (4 rows, no split) it
    hands the next QKV ONE slab to build its input row from instead of four: with the
    non-temporal weight loads, batch-1 p50 454 -> 431 ms (profiles/r6_b1_nt_down_ab.log;
    DOCQA_GEMV_DOWN=0 keeps the ring).  DOCQA_GEMV=0 disables."""
    if not _GEMV or M != 1 or N % 8 or K % 2048:
        return 0, 0
    if K > 8192:
        # one slab for the next QKV's in-kernel input row instead of the ring's four
        return (1, 4) if _GEMV_DOWN and K // 2048 == 7 else (0, 0)
    return (1, _GEMV_R) if K <= 4096 else ((2, 8) if K % 4096 == 0 else (0, 0))


def gemv_glu_ok(M: int, N: int, K: int) -> bool:
    """The batch-1 gate|up projection with SwiGLU on the GEMV (one 16-row gate|up group per
    workgroup): 41.1 vs 47.6 us for the ring kernel at Llama-3-8B (profiles/r6_gemv_probe.log)."""
    return _GEMV and M == 1 and N % 16 == 0 and K % 2048 == 0 and (K // 2048) in (1, 2)


def gemv_glu(x, w_il):
    """silu(x Wg^T) * (x Wu^T) for one row on the batch-1 GEMV (:func:`gemv_glu_ok`)."""
    if _gpu(x):
        return _native().gemv(x.contiguous(), w_il, 1, 16, True)
    return glu_linear(x, w_il)


def gemv_partial(x, w, splits: int, rows: int):
    """fp32 slabs [S, 1, N] of one row x @ w^T on the batch-1 GEMV (:func:`gemv_plan`)."""
    if _gpu(x):
        return _native().gemv(x.contiguous(), w, int(splits), int(rows), False)
    return dgemm_partial(x, w, splits, 64)


def gemv_partial_xn(Pin, res_in, res_out, gamma, eps: float, w, splits: int, rows: int):
    """:func:`dgemm_partial_xn` (input row built in-kernel) on the batch-1 GEMV."""
    if _gpu(Pin):
        return _native().gemv_xn(Pin, res_in, res_out, gamma, float(eps), w, int(splits), int(rows), False)
    return dgemm_partial_xn(Pin, res_in, res_out, gamma, eps, w, splits)


def gemv_glu_xn(Pin, res_in, res_out, gamma, eps: float, w_il):
    """:func:`dgemm_glu_xn` (input row built in-kernel, SwiGLU epilogue) on the batch-1 GEMV."""
    if _gpu(Pin):
        return _native().gemv_xn(Pin, res_in, res_out, gamma, float(eps), w_il, 1, 16, True)
    return dgemm_glu_xn(Pin, res_in, res_out, gamma, eps, w_il)


NORM_FUSE_ROWS = 4
# off by default: the last-workgroup add + RMSNorm tail (one workgroup reading every slab at
# agent scope) costs more than the add_rmsnorm_splitk launch it replaces -- batch-1 p50
# 511.5 ms with it vs 492.0 without (profiles/r4_b1_ab.log)
_NORM_FUSE = os.environ.get("DOCQA_DGEMM_NORM", "0") == "1"


def dgemm_norm_plan(M: int, N: int, K: int) -> int:
    """Split count of the few-row projection with the residual add + RMSNorm fused into its
    last workgroup (dgemm.hip NormArgs), 0 where it does not apply (more than
    NORM_FUSE_ROWS rows, N > 8192, no skinny-kernel plan, DOCQA_DGEMM_NORM=0)."""
    if not _NORM_FUSE or not (0 < M <= NORM_FUSE_ROWS) or N > 8192 or N % 64:
        return 0
    S, t = decode_plan(M, N, K)
    return S if t == 64 else 0


def dgemm_add_rmsnorm(x, w, splits: int, residual, gamma, eps: float, tick):
    """residual <- residual + bf16(x @ w^T); returns rmsnorm(residual) * gamma -- the
    split-K projection and the add + norm in one launch (few rows, :func:`dgemm_norm_plan`).
    ``tick``: one zeroed int32 word (the kernel re-arms it)."""
    if _gpu(x):
        return _native().dgemm_add_rmsnorm(x.contiguous(), w, int(splits), residual, gamma, float(eps), tick)
    y = torch.nn.functional.linear(x.float(), w.float()).to(residual.dtype)
    return ref.add_rmsnorm(y, residual, gamma, eps)


def add_rmsnorm_splitk(P, residual, w, eps: float):
    """residual <- residual + bf16(sum_s P[s]); returns rmsnorm(residual) * w."""
    if _gpu(P):
        return _native().add_rmsnorm_splitk(P, residual, w, eps)
    return ref.add_rmsnorm(P.float().sum(0).to(residual.dtype).view_as(residual), residual, w, eps)


def paged_decode_fused(P, positions, cos_sin, slot_mapping, k_cache, v_cache, block_tables,
                       context_lens, Hq, max_context, scale, order=None, tick=None):
    """Decode attention straight from the QKV projection's split-K partial slabs: RoPE,
    paged-cache write of the new token and attention in one launch (attn_decode.hip ring
    kernel, FUSED mode).  Same result as rope_cache_splitk + paged_decode.
    ``tick``: a zeroed int32 buffer of >= B x Hkv entries (:func:`decode_ticket`) -- split
    context partitions are then merged by their last workgroup, no second launch."""
    if _gpu(P):
        return _native().paged_decode_fused(P, positions, cos_sin, slot_mapping, k_cache, v_cache,
                                            block_tables, context_lens, Hq, max_context, scale, order,
                                            tick)
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    qkv = rope_cache_splitk(P, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
    return ref.paged_decode(qkv, k_cache, v_cache, block_tables, context_lens, Hq, max_context, scale)


_LAST_MERGE = os.environ.get("DOCQA_DECODE_LAST_MERGE", "1") != "0"


def decode_ticket(n: int, device) -> torch.Tensor | None:
    """Zeroed int32 ticket words for the last-arriver partition merge of the decode
    attention kernels (one per sequence x KV head; the kernel re-arms them).  None when
    DOCQA_DECODE_LAST_MERGE=0 (separate reduce launch)."""
    if not _LAST_MERGE:
        return None
    return torch.zeros(n, dtype=torch.int32, device=device)


def fused_decode_ok(k_cache, block_tables) -> bool:
    """Shapes the fused decode attention kernel supports (head_dim 128, 64-token blocks,
    <= 256 blocks per sequence)."""
    return k_cache.shape[2] == 64 and k_cache.shape[3] == 128 and block_tables.shape[1] <= 256


def rope_cache_splitk(P, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D):
    """Packed bf16 QKV <- rope(bf16(sum_s P[s])) with the paged-cache write (rope_cache)."""
    if _gpu(P):
        if slot_mapping is None:
            k_cache = v_cache = P
        return _native().rope_cache_splitk(P, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
    # the model dtype: bf16 on the GPU path, fp32 for CPU reference models
    qkv = P.float().sum(0).to(k_cache.dtype if slot_mapping is not None else torch.bfloat16)
    ref.rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
    return qkv


# ----------------------------------------------------------------------------- embeddings
def embedding(ids, table):
    if _gpu(table):
        return _native().embedding(ids, table)
    return ref.embedding(ids, table)


def bert_embed_ln(ids, pos, token_type, wte, wpe, wtt, gamma, beta, eps):
    if _gpu(wte):
        return _native().bert_embed_ln(ids, pos, token_type, wte, wpe, wtt, gamma, beta, eps)
    return ref.bert_embed_ln(ids, pos, token_type, wte, wpe, wtt, gamma, beta, eps)


# ----------------------------------------------------------------------------- sampling
def decode_slots(block_tables, positions, valid, BS: int):
    """Paged-cache slot of each decode row's next token, -1 for padded rows."""
    if _gpu(block_tables):
        return _native().decode_slots(block_tables, positions, valid, BS)
    return ref.decode_slots(block_tables, positions, valid, BS)


def decode_advance(nxt, out, tokens, positions, context_lens, valid) -> None:
    """In place: out <- nxt, tokens <- nxt, positions / context_lens += valid."""
    if _gpu(nxt):
        _native().decode_advance(nxt, out, tokens, positions, context_lens, valid)
        return
    ref.decode_advance(nxt, out, tokens, positions, context_lens, valid)


def argmax(logits):
    if _gpu(logits):
        return _native().argmax(logits)
    return ref.argmax(logits)


def token_cls_argmax(h, w, bias, n_valid: int):
    """Fused token-classification head + argmax: argmax_n(h @ w[:n_valid].T + bias)."""
    if _gpu(h):
        return _native().token_cls_argmax(h, w, bias, int(n_valid))
    return ref.token_cls_argmax(h, w, bias, n_valid)


def sample(logits, inv_temp, top_k, top_p, u):
    if _gpu(logits):
        return _native().sample(logits.float().contiguous(), inv_temp, top_k, top_p, u)
    return ref.sample(logits, inv_temp, top_k, top_p, u)


# ----------------------------------------------------------------------------- attention
def paged_decode(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context, scale, order=None):
    """``order``: optional int32 permutation of the rows -- the workgroup dispatch order
    (longest context first); results do not depend on it."""
    if _gpu(q):
        return _native().paged_decode(q, k_cache, v_cache, block_tables, context_lens, Hq,
                                      max_context, scale, order)
    return ref.paged_decode(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context, scale)


def cascade_ok(k_cache, block_tables, Hq: int) -> bool:
    """Shapes the cascade (shared-prefix) decode path supports: Llama-3 GQA (4 query heads
    per KV head), head_dim 128, 64-token blocks, <= 256 blocks per sequence (the CPU
    reference path takes any GQA shape)."""
    if not _gpu(k_cache):
        return Hq % k_cache.shape[1] == 0
    return (k_cache.shape[2] == 64 and k_cache.shape[3] == 128 and Hq == 4 * k_cache.shape[1]
            and block_tables.shape[1] <= 256)


def paged_decode_cascade_rope(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, block_tables,
                              context_lens, Hq, max_context, scale, prefix_table, prefix_len,
                              nchunk: int = 8, order=None):
    """Cascade decode over the unrotated packed QKV rows of a library GEMM: RoPE, the new
    token's paged-cache write and the attention inside the cascade kernels (the prefix
    kernel rotates queries on load, the ring kernel rotates its queries and writes / attends
    the new K/V from registers).  ``qkv`` may be rotated in place (fallback path)."""
    if _gpu(qkv):
        return _native().paged_decode_cascade_rope(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache,
                                                   block_tables, context_lens, Hq, max_context, scale,
                                                   prefix_table, prefix_len, nchunk, order)
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    ref.rope_cache(qkv, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
    return ref.paged_decode_cascade(qkv, k_cache, v_cache, block_tables, context_lens, Hq, max_context,
                                    scale, prefix_table, prefix_len, nchunk)


def paged_decode_cascade(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context, scale,
                         prefix_table, prefix_len, nchunk: int = 8, order=None):
    """Decode attention with the batch's shared prompt prefix attended once for all rows
    (csrc/include/docqa_cascade.h): keys [0, prefix_len) from ``prefix_table``, keys
    [prefix_len, L) from each row's block table.  Same result as :func:`paged_decode`
    when the prefix blocks are the ones every row's table starts with."""
    if _gpu(q):
        return _native().paged_decode_cascade(q, k_cache, v_cache, block_tables, context_lens, Hq,
                                              max_context, scale, prefix_table, prefix_len, nchunk, order)
    return ref.paged_decode_cascade(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context,
                                    scale, prefix_table, prefix_len, nchunk)


def paged_decode_cascade_grouped(q, k_cache, v_cache, block_tables, context_lens, Hq, scale,
                                 prefix_table, prefix_len, nchunk: int, groups, defer: bool = False,
                                 tick=None, inline_prefix: bool = False):
    """Cascade decode with the suffix attention of rows that share prefix-cache KV blocks
    done together (csrc/kernels/attn_decode.hip paged_decode_group_kernel): ``groups``
    int32 [ngroups * 4] packs every row into one group of <= 4 (-1 = empty slot), and a
    block shared by k rows of a group is read once instead of k times.  Same result as
    :func:`paged_decode_cascade` for any packing.  ``groups`` may also be a split plan
    int32 [2, cap, 8] from :func:`split_decode_groups` (long groups over several
    workgroups, partials merged by log-sum-exp); ``defer``: that plan was built with
    ``split_decode_groups(defer=True)`` (the prefix kernel then runs on a side stream).
    ``tick``: zeroed int32 ticket words (>= cap x Hkv, :func:`decode_ticket`) -- a split
    plan's groups are then merged by their last work item instead of a merge launch.
    ``inline_prefix``: the split plan's items start at block 0 (built with skip 0), so the
    groups attend the shared prefix themselves -- no prefix kernel."""
    if _gpu(q):
        if groups.dim() == 3:
            return _native().paged_decode_cascade_split(q, k_cache, v_cache, block_tables, context_lens, Hq,
                                                        scale, prefix_table, prefix_len, nchunk, groups,
                                                        defer and groups.shape[0] == 2, tick,
                                                        bool(inline_prefix) and groups.shape[0] == 2)
        return _native().paged_decode_cascade_grouped(q, k_cache, v_cache, block_tables, context_lens, Hq,
                                                      scale, prefix_table, prefix_len, nchunk, groups)
    max_context = block_tables.shape[1] * k_cache.shape[2]
    return ref.paged_decode_cascade(q, k_cache, v_cache, block_tables, context_lens, Hq, max_context,
                                    scale, prefix_table, prefix_len, nchunk)


def paged_decode_grouped_fused(P, positions, cos_sin, slot_mapping, k_cache, v_cache, block_tables, context_lens,
                               Hq, scale, prefix_table, prefix_len, nchunk: int, plan, tick=None):
    """Grouped decode attention straight from the QKV projection's split-K slabs (split plan
    built from block 0, no prefix kernel): each workgroup rotates the query rows it needs and
    the item holding a row's new token writes its rotated K / V to the paged cache first --
    the same result as :func:`rope_cache_splitk` + :func:`paged_decode_cascade_grouped`
    (``inline_prefix``), one launch and the bf16 QKV round trip fewer."""
    if _gpu(P):
        return _native().paged_decode_grouped_fused(P, positions, cos_sin, slot_mapping, k_cache, v_cache,
                                                    block_tables, context_lens, Hq, scale, prefix_table,
                                                    prefix_len, nchunk, plan, tick)
    Hkv, D = k_cache.shape[1], k_cache.shape[3]
    qkv = rope_cache_splitk(P, positions, cos_sin, slot_mapping, k_cache, v_cache, Hq, Hkv, D)
    return paged_decode_cascade_grouped(qkv, k_cache, v_cache, block_tables, context_lens, Hq, scale, prefix_table,
                                        prefix_len, nchunk, plan, False, tick, True)


GROUP_MAX_BLOCKS = 64   # block positions one grouped-decode work item covers (attn_decode.hip kGroupMaxPos)


def grouped_decode_ok(k_cache, block_tables, Hq: int, max_blocks: int | None = None) -> bool:
    """Shapes the grouped cascade kernel supports: cascade shapes and rows of <= 64 blocks --
    ``max_blocks``, the most any row of the batch reaches by the end of its decode, or else
    the block table's width (its capacity)."""
    nb = block_tables.shape[1] if max_blocks is None else max_blocks
    return cascade_ok(k_cache, block_tables, Hq) and nb <= GROUP_MAX_BLOCKS


def pack_decode_groups(tables: list[list[int]], lens: list[int], skip: int, block_size: int,
                       cap: int) -> list[list[int]]:
    """Pack the rows of a decode batch into groups of <= 4 for the grouped decode kernel:
    rows are sorted by their block ids beyond the ``skip`` cascade-prefix blocks (rows whose
    prompts share prefix-cache blocks become neighbours), clusters of rows sharing their
    first such block stay together where they fit, and the groups are ordered by distinct
    blocks, largest first (LPT).  Falls back to plain consecutive quads when the packing
    would exceed ``cap`` groups."""
    n = len(tables)
    if n == 0:
        return []
    # sort key: block ids relabelled by first occurrence (row-major), so the packing -- and
    # with it each row's split points and partial-merge order -- depends only on which rows
    # share blocks, never on the physical ids the allocator handed out (a pipelined run
    # frees batch i-1 and reserves batch i+1 on two threads in a timing-dependent order)
    label: dict[int, int] = {}
    for t in tables:
        for b in t[skip:]:
            label.setdefault(b, len(label))
    keyed = [[label[b] for b in t[skip:]] for t in tables]
    idx = sorted(range(n), key=lambda i: keyed[i])

    def first(i):
        return tables[i][skip] if len(tables[i]) > skip else -1 - i

    clusters, cur = [], [idx[0]]
    for a, b in zip(idx, idx[1:]):
        if first(a) == first(b) and first(a) >= 0:
            cur.append(b)
        else:
            clusters.append(cur)
            cur = [b]
    clusters.append(cur)
    quads, cur = [], []
    for cl in clusters:
        while len(cl) > 4:
            quads.append(cl[:4])
            cl = cl[4:]
        if len(cur) + len(cl) > 4:
            quads.append(cur)
            cur = []
        cur = cur + cl
    if cur:
        quads.append(cur)
    if len(quads) > cap:
        quads = [idx[i:i + 4] for i in range(0, n, 4)]

    def work(qd):
        blocks = set()
        for r in qd:
            nb = (lens[r] + block_size - 1) // block_size
            blocks.update(tables[r][skip:nb])
        return len(blocks)

    quads.sort(key=work, reverse=True)
    return quads


def kv_copy_rows(pools: list, copies: list, ptrs: torch.Tensor | None = None) -> None:
    """K/V rows [0, m) of block src -> the same rows of block dst in every paged pool
    (``pools``: [(k, v)] per layer, [num_blocks, Hkv, BS, D]; ``copies``: [(src, dst, m)]).
    GPU: one launch of csrc/kernels/rope_cache.hip kv_copy_rows over all pools (``ptrs``:
    int64 device addresses of the pools in (k_0, v_0, k_1, ...) order, built by the
    caller once); CPU: tensor indexing."""
    if not copies:
        return
    k0 = pools[0][0]
    if _gpu(k0):
        if ptrs is None:
            ptrs = torch.tensor([t.data_ptr() for kv in pools for t in kv], dtype=torch.int64, device=k0.device)
        tab = torch.tensor(copies, dtype=torch.int32).pin_memory().to(k0.device, non_blocking=True)
        _native().kv_copy_rows(ptrs, tab, k0.shape[0], k0.shape[1], k0.shape[2], k0.shape[3])
        return
    src = torch.tensor([s for s, _, m in copies for _ in range(m)], dtype=torch.long, device=k0.device)
    dst = torch.tensor([d for _, d, m in copies for _ in range(m)], dtype=torch.long, device=k0.device)
    rows = torch.tensor([i for _, _, m in copies for i in range(m)], dtype=torch.long, device=k0.device)
    for kc, vc in pools:
        kc[dst, :, rows] = kc[src, :, rows]
        vc[dst, :, rows] = vc[src, :, rows]


def group_tiles_by_position(tables: list[list[int]], lens: list[int], rows: list[int], skip: int,
                            block_size: int) -> list[tuple[int, int]]:
    """(block position, 32-token K/V tiles) the grouped decode kernel streams for ``rows``
    at each position beyond the ``skip`` cascade-prefix blocks: one or two tiles (by the
    longest length among the rows reading it) per DISTINCT block id at that position."""
    half = block_size // 2
    rl = [(tables[r], lens[r]) for r in rows]
    nb = max((L + block_size - 1) // block_size for _, L in rl)
    out = []
    for pos in range(skip, nb):
        lo = pos * block_size
        live: dict[int, int] = {}
        for t, L in rl:
            if lo < L and pos < len(t):
                b = t[pos]
                if live.get(b, 0) < L:
                    live[b] = L
        if live:
            thr = lo + half
            out.append((pos, len(live) + sum(1 for L in live.values() if L > thr)))
    return out


def remap_plan_rows(plan: torch.Tensor, plan_ids: list, ids: list) -> torch.Tensor | None:
    """A split plan (:func:`split_decode_groups`, [2 or 3, cap, 8]) built for rows with
    request ids ``plan_ids``, re-targeted at rows ``ids`` after requests RETIRED and the
    survivors were compacted: each row id in columns 0..3 of the items and merges becomes
    the survivor's new index, or -1 if it retired.  None if ``ids`` holds a request the plan
    does not know (an admission: re-plan).  Positions and split points stay valid -- they
    depend only on each survivor's blocks and END length -- and every item of a group
    carries the group's rows, so a fully retired group's items all exit before drawing a
    merge ticket."""
    pos = {rid: i for i, rid in enumerate(plan_ids)}
    if not all(rid in pos for rid in ids):
        return None
    n = len(plan_ids)
    m = torch.full((n + 1,), -1, dtype=torch.int32)
    if ids:
        m[torch.tensor([pos[rid] for rid in ids], dtype=torch.long)] = torch.arange(len(ids), dtype=torch.int32)
    out = plan.clone()
    cols = plan[:2, :, :4].long()
    out[:2, :, :4] = torch.where(cols >= 0, m[cols.clamp(min=0, max=n)], torch.full_like(plan[:2, :, :4], -1))
    return out


def persist_bins(cap: int, Hkv: int) -> int:
    """Workgroups per KV head of the persistent grouped decode (attn_decode.hip
    group_persist_bins): ~3 per CU chip-wide, at least one per quad of ``cap`` rows."""
    nb = max(768 // max(1, Hkv), (cap + 3) // 4)
    return min(nb, cap)


BIN_ITEMS, BIN_MAX_TILES = 8, 512    # attn_decode.hip kBinItems / kBinMaxTiles


def split_decode_groups(quads: list[list[int]], tables: list[list[int]], lens: list[int], skip: int,
                        block_size: int, cap: int, tiles_per_item: int = 12, bins: int = 0,
                        defer: bool = False, per_quad: list | None = None) -> torch.Tensor:
    """Split plan for the grouped cascade decode (``paged_decode_cascade_grouped`` with a
    [2, cap, 8] int32 ``groups``): every group of :func:`pack_decode_groups` is cut at block
    positions into work items of about ``tiles_per_item`` K/V tiles (``lens``: the lengths
    at the END of decode, so an item's range stays valid for every step), one workgroup per
    item and KV head.  A group that needs one item finishes in its workgroup; the items of
    a longer group write partials that a merge kernel combines.  Items are ordered largest
    first (LPT).  plan[0]: items (4 rows, first position, end position, slot or -1, 0);
    plan[1]: merges (4 rows, first slot, slots, 0, 0) -- at most (cap + 1) // 2 of them
    (the merge kernel's grid).

    ``bins`` > 0: the PERSISTENT plan [3, cap, 8] instead -- every item writes a partial
    (slot = its index), every group has a merge row, and plan[2] packs the items into
    ``bins`` (:func:`persist_bins`) workgroups of <= 8 items and <= 512 tiles each, greedy
    longest-first onto the least-loaded bin, so each workgroup streams ~total / bins tiles
    through one ring.

    ``defer``: every item writes a partial and every group has a merge row (at most ``cap``),
    as in the persistent plan, so no item reads the cascade-prefix partials and the prefix
    kernel runs on a side stream beside the group kernel (attn_decode.hip, DOCQA_GROUP_DEFER).

    ``per_quad``: :func:`group_tiles_by_position` of each quad, precomputed (a caller that
    tries several budgets for one batch computes them once -- they do not depend on it)."""
    budget = max(1, tiles_per_item)
    all_partial = bool(bins) or defer
    if per_quad is None:
        per_quad = [group_tiles_by_position(tables, lens, list(qd), skip, block_size) for qd in quads]
    while True:
        items, merges, nslot = [], [], 0
        for qd, per in zip(quads, per_quad):
            rows4 = (list(qd) + [-1] * 4)[:4]
            cuts, acc, start = [], 0, skip
            for pos, t in per:
                if acc and acc + t > budget:
                    cuts.append((start, pos, acc))
                    start, acc = pos, 0
                acc += t
            end = max((lens[r] + block_size - 1) // block_size for r in qd)
            cuts.append((start, max(end, start + 1), acc))
            # an item of a merged group carries its merge row (column 7) for the
            # last-arriver merge inside the group kernel
            if all_partial:
                merges.append(rows4 + [nslot, len(cuts), 0, 0])
                for lo, hi, t in cuts:
                    items.append((t, rows4 + [lo, hi, nslot, len(merges) - 1]))
                    nslot += 1
            elif len(cuts) == 1:
                items.append((cuts[0][2], rows4 + [skip, 1 << 20, -1, 0]))
            else:
                merges.append(rows4 + [nslot, len(cuts), 0, 0])
                for lo, hi, t in cuts:
                    items.append((t, rows4 + [lo, hi, nslot, len(merges) - 1]))
                    nslot += 1
        fits = len(items) <= cap and len(merges) <= (cap if all_partial else (cap + 1) // 2)
        if fits and bins:
            nb = min(bins, cap)
            fits = len(items) <= nb * BIN_ITEMS and all(t <= BIN_MAX_TILES for t, _ in items)
        if fits:
            break
        if budget > 1 << 20:
            raise ValueError(f"split_decode_groups: {len(quads)} groups exceed the plan capacity {cap}")
        budget *= 2
    if not bins:
        items.sort(key=lambda it: -it[0])
        plan = torch.full((2, cap, 8), -1, dtype=torch.int32)
        plan[:, :, 4:] = 0
        if items:
            plan[0, :len(items)] = torch.tensor([it[1] for it in items], dtype=torch.int32)
        if merges:
            plan[1, :len(merges)] = torch.tensor(merges, dtype=torch.int32)
        return plan
    nb = min(bins, cap)
    load, members = [0] * nb, [[] for _ in range(nb)]
    for i in sorted(range(len(items)), key=lambda i: -items[i][0]):
        t = items[i][0]
        best = min((b for b in range(nb) if len(members[b]) < BIN_ITEMS and load[b] + t <= BIN_MAX_TILES),
                   key=lambda b: load[b], default=None)
        if best is None:    # every bin full: the plan cannot hold this batch
            raise ValueError("split_decode_groups: items exceed the persistent bins")
        members[best].append(i)
        load[best] += t
    plan = torch.full((3, cap, 8), -1, dtype=torch.int32)
    plan[:2, :, 4:] = 0
    plan[0, len(items):, 6] = -1           # unused item rows: no slot
    if items:
        plan[0, :len(items)] = torch.tensor([it[1] for it in items], dtype=torch.int32)
    if merges:
        plan[1, :len(merges)] = torch.tensor(merges, dtype=torch.int32)
    for b, mem in enumerate(members):
        # a bin streams its items in index order: keep them position-ordered per group
        for j, i in enumerate(sorted(mem)):
            plan[2, b, j] = i
    return plan


def flash_prefill(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, causal=True):
    if _gpu(qkv):
        return _native().flash_prefill(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, causal)
    return ref.flash_prefill(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, causal)


def flash_prefill_paged(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, k_cache, v_cache,
                        block_tables, ctx_start):
    if _gpu(qkv):
        return _native().flash_prefill_paged(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, k_cache,
                                             v_cache, block_tables, ctx_start)
    return ref.flash_prefill_paged(qkv, cu_seqlens, max_len, Hq, Hkv, D, scale, k_cache, v_cache,
                                   block_tables, ctx_start)


# ----------------------------------------------------------------------------- search
def knn(xb, xb_norms, xq, k: int, inner_product: bool = False, id_offset: int = 0):
    if _gpu(xb):
        return _native().knn(xb, xb_norms, xq.float().contiguous(), k, inner_product, id_offset)
    return ref.knn(xb, xb_norms, xq, k, inner_product, id_offset)


def fp32_matmul_nt(x, w):
    """Exact fp32 ``x @ w.T`` on the coarse quantizer's MFMA tiles (coarse.hip) -- the IVF-PQ
    query pre-rotation on the GPU without a library GEMM; torch on the CPU."""
    if _gpu(x) and x.shape[1] % 8 == 0 and x.shape[1] <= 1280:
        return _native().fp32_gemm_nt(x.float().contiguous(), w.float().contiguous())
    return x.float() @ w.float().t()


def coarse_probes(xq, centroids, cnorm, nprobe: int):
    """IVF coarse quantizer: int64 [nq, nprobe] nearest centroids by squared L2, ascending,
    ties to the lower centroid id.  GPU: csrc/kernels/coarse.hip (MFMA fp32 distances +
    radix select, nprobe <= 512); nprobe <= 64 may also use :func:`knn`.  Shapes outside
    the kernel's envelope (nprobe > 512, d > 1280 or d % 8 != 0 -- recall sweeps, wide
    embeddings) take the fp32 reference on the same device instead of failing."""
    d = int(centroids.shape[1])
    nprobe = int(min(int(nprobe), int(centroids.shape[0])))
    if _gpu(xq) and nprobe <= 512 and d % 8 == 0 and d <= 1280:
        return _native().coarse_probes(xq.float().contiguous(), centroids, cnorm, nprobe)
    return ref.coarse_probes(xq, centroids, cnorm, nprobe)


# ----------------------------------------------------------------------------- pooling
def pool_l2(h, cu_seqlens, mean: bool = True, normalize: bool = True):
    if _gpu(h):
        return _native().pool_l2(h.contiguous(), cu_seqlens, mean, normalize)
    return ref.pool_l2(h, cu_seqlens, mean, normalize)


# eager-load when a GPU is present so an import on the box fails loudly if unbuilt
if torch.cuda.is_available() and not _FORCE_REF:
    load_native()
