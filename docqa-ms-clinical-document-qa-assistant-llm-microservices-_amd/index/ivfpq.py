"""IVF-PQ index (FAISS ``IndexIVFPQ`` semantics: squared L2, residual PQ, 8-bit codes),
HBM-resident, for the multi-million-vector semantic-indexer configuration.

Layout on the GPU: coarse centroids [nlist, d] fp32, PQ codebook [M, 256, d/M] fp32,
codes of all lists concatenated and sorted by list [N, M] uint8 with list offsets
[nlist + 1] int64 and stored ids [N] int64.  At 10M x 768-d with M=64 the codes take
640 MB -- a fraction of one MI355X's 288 GB, so an 8-GPU node holds 3.5B vectors.

Search = coarse flat kNN (q vs centroids, top-nprobe; MFMA kernel) + the precomputed-table
ADC scan (``ivfpq.hip`` ivfpq_scan_pt_kernel): ||q - c_l - r^||^2 splits into ||q||^2 -
2<q, c_l> (one dot product per probe), ||c_l + r^||^2 (``norms``, stored per vector at add
time) and -2 sum_m <q_m, pq[m][code_m]> (one fp16 LUT per QUERY, shared by all its probes),
so no per-(query, list) table is rebuilt; candidates pass an LDS threshold buffer with
radix-select compaction, then one merge launch maps positions to ids.
``DOCQA_IVFPQ_SCAN=lut`` keeps the per-item-LUT kernel (exact fp32 ADC, no norms needed).
Training = GPU k-means (coarse) + per-subspace k-means (PQ); encoding = one kernel.

FAISS file format (``IvPQ``) read/write: header + nlist/nprobe + flat quantizer +
direct map + by_residual + code_size + ProductQuantizer + ArrayInvertedLists ("ilar",
"full"/"sprs" size lists, then per list codes and ids), following faiss's
index_write.cpp layout.  No IVF-PQ fixture ships with the reference, so byte-level
parity with FAISS itself is "parity unpinned" (round-trip tested only).
"""
from __future__ import annotations

import io
import os
import struct

import numpy as np
import torch

from .. import ops
from . import faiss_io
from .kmeans import assign, kmeans, kmeans_subspaces


def pca_rotation(x: torch.Tensor, M: int) -> torch.Tensor:
    """Orthogonal [d, d] pre-rotation for PQ (applied as x @ R): the principal directions of
    ``x``, dealt to the M sub-quantizers round-robin (PCA direction r -> sub-space r % M), so
    each sub-space gets an equal share of the variance.  L2 distances are unchanged; the
    codebooks stop spending most of their bits on the handful of sub-spaces that would
    otherwise hold the dominant directions (random-init sentence embeddings: one direction
    carries ~40 % of the variance; recall@10 0.78 -> 0.93 at nprobe 64 with exact refine,
    profiles/r3_ivfpq_rotation_probe.log)."""
    x = x.double()
    xc = x - x.mean(0, keepdim=True)
    cov = xc.t() @ xc / max(1, x.shape[0] - 1)
    _, vec = torch.linalg.eigh(cov)                        # ascending eigenvalues
    vec = vec.flip(1)
    d = x.shape[1]
    order = torch.tensor([r for j in range(M) for r in range(j, d, M)], device=vec.device)
    return vec[:, order].float().contiguous()


def probes_per_workgroup(nq: int, nprobe: int) -> int:
    """Probed lists per scan workgroup: enough workgroups to fill the chip several times
    over (~4096: two 57 KB-LDS workgroups per CU x 256 CUs x 8 rounds) without re-loading
    each query's 48 KB LUT for only a list or two (DOCQA_IVFPQ_PC overrides)."""
    env = os.environ.get("DOCQA_IVFPQ_PC")
    if env:
        return max(1, int(env))
    chunks = max(1, min(nprobe, -(-4096 // max(1, nq))))
    return -(-nprobe // chunks)


# auto scan: above this E||c||^2 / E||r^||^2 the exact-fp32 LUT kernel is used
_PT_MAX_RATIO = float(os.environ.get("DOCQA_IVFPQ_PT_MAX_RATIO", "32"))


class IVFPQIndex:
    def __init__(self, d: int, nlist: int, M: int, nbits: int = 8, device="cuda", rotation: str = "none"):
        if nbits != 8:
            raise ValueError("only 8-bit PQ codes are supported")
        if d % M:
            raise ValueError("d must be divisible by M")
        if rotation not in ("none", "pca"):
            raise ValueError(f"unknown PQ pre-rotation {rotation!r}")
        self.d, self.nlist, self.M = d, nlist, M
        self.dsub = d // M
        self.device = torch.device(device)
        self.nprobe = 16
        self.rotation = rotation
        # orthogonal pre-transform R [d, d] (x -> x @ R), FAISS IndexPreTransform(LinearTransform)
        self.rot: torch.Tensor | None = None
        self.centroids: torch.Tensor | None = None
        self.pq: torch.Tensor | None = None
        self.codes = torch.empty(0, M, dtype=torch.uint8, device=self.device)
        self.ids = torch.empty(0, dtype=torch.long, device=self.device)
        self.list_off = torch.zeros(nlist + 1, dtype=torch.long, device=self.device)
        # ||c_list + r^_i||^2 per stored vector (list-major like codes); rebuilt lazily after
        # a FAISS load, which stores no such term
        self.norms: torch.Tensor | None = torch.empty(0, dtype=torch.float32, device=self.device)
        self.ntotal = 0

    @property
    def is_trained(self) -> bool:
        return self.centroids is not None and self.pq is not None

    # ------------------------------------------------------------------ build
    def _in(self, x) -> torch.Tensor:
        """Vectors into the index's (rotated) space."""
        x = torch.as_tensor(x).to(self.device, torch.float32)
        if self.rot is None:
            return x
        # x @ R as x @ (R^T)^T on the fp32 MFMA tiles of coarse.hip (no library GEMM on the
        # search path); R^T cached per rotation tensor
        if getattr(self, "_rot_src", None) is not self.rot:
            self._rot_t, self._rot_src = self.rot.t().contiguous(), self.rot
        return ops.fp32_matmul_nt(x, self._rot_t)

    def train(self, x, niter: int = 20, seed: int = 0) -> None:
        x = torch.as_tensor(x).to(self.device, torch.float32)
        # stored ||c + r^||^2 belong to the old quantizers: rebuilt from the codes on the next
        # precomputed-table search (they were rebuilt only on a row-count change)
        self.norms = None
        if self.rotation == "pca":
            self.rot = pca_rotation(x, self.M).to(self.device)
            x = x @ self.rot
        self.centroids = kmeans(x, self.nlist, niter, seed)
        _, a = assign(x, self.centroids)
        resid = x - self.centroids.index_select(0, a)
        self.pq = kmeans_subspaces(resid, self.M, 256, max(10, niter // 2), seed + 1).contiguous()

    def encode(self, x: torch.Tensor, a: torch.Tensor) -> torch.Tensor:
        if self.device.type == "cuda":
            return ops._native().pq_encode(x.contiguous(), self.centroids, a.contiguous(), self.pq)
        r = (x - self.centroids.index_select(0, a)).view(-1, self.M, 1, self.dsub)
        dist = ((r - self.pq[None]) ** 2).sum(-1)           # [n, M, 256]
        return dist.argmin(-1).to(torch.uint8)

    def add(self, x, ids=None, batch: int = 1 << 20) -> None:
        if not self.is_trained:
            raise RuntimeError("train() first")
        x = torch.as_tensor(x)
        n = x.shape[0]
        if ids is None:
            ids = torch.arange(self.ntotal, self.ntotal + n, dtype=torch.long)
        ids = torch.as_tensor(ids, dtype=torch.long).to(self.device)
        new_codes, new_lists = [], []
        for i in range(0, n, batch):
            xb = self._in(x[i:i + batch])
            _, a = assign(xb, self.centroids)
            new_codes.append(self.encode(xb, a))
            new_lists.append(a)
        new_norms = [self.recon_norms(c, a) for c, a in zip(new_codes, new_lists)]
        old_norms = [self._norms()] if self.ntotal else []
        codes = torch.cat([self._list_major_codes(), *new_codes]) if self.ntotal else torch.cat(new_codes)
        lists = torch.cat([self._row_lists(), *new_lists]) if self.ntotal else torch.cat(new_lists)
        allids = torch.cat([self.ids, ids]) if self.ntotal else ids
        order = torch.argsort(lists, stable=True)
        self.codes = codes.index_select(0, order).contiguous()
        self.ids = allids.index_select(0, order).contiguous()
        self.norms = torch.cat([*old_norms, *new_norms]).index_select(0, order).contiguous()
        counts = torch.bincount(lists, minlength=self.nlist)
        self.list_off = torch.zeros(self.nlist + 1, dtype=torch.long, device=self.device)
        self.list_off[1:] = torch.cumsum(counts, 0)
        self.ntotal += n

    def _list_major_codes(self):
        return self.codes

    def recon_norms(self, codes: torch.Tensor, lists: torch.Tensor, batch: int = 1 << 18) -> torch.Tensor:
        """||c_list + r^||^2 of encoded vectors (r^ = the PQ reconstruction of the residual):
        the per-vector term of the precomputed-table distance."""
        out = torch.empty(codes.shape[0], dtype=torch.float32, device=codes.device)
        m_idx = torch.arange(self.M, device=codes.device)
        for i in range(0, codes.shape[0], batch):
            c = codes[i:i + batch].long()
            r = self.pq[m_idx[None, :], c].reshape(c.shape[0], self.d)      # [n, d]
            x = r + self.centroids.index_select(0, lists[i:i + batch])
            out[i:i + batch] = (x * x).sum(1)
        return out

    def _norms(self) -> torch.Tensor:
        if self.norms is None or self.norms.shape[0] != self.codes.shape[0]:
            self.norms = self.recon_norms(self.codes, self._row_lists()).contiguous()
        return self.norms

    def _row_lists(self):
        counts = self.list_off[1:] - self.list_off[:-1]
        return torch.repeat_interleave(torch.arange(self.nlist, device=self.device), counts)

    # ------------------------------------------------------------------ search
    def search(self, xq, k: int, nprobe: int | None = None):
        nprobe = min(nprobe or self.nprobe, self.nlist)
        xq = self._in(xq).contiguous()
        cn = (self.centroids ** 2).sum(1)
        if nprobe <= 64 and self.device.type == "cuda":
            _, probes = ops.knn(self.centroids, cn, xq, nprobe, False, 0)
        else:   # wide probes (the 10M operating points: nprobe 128..512): coarse.hip
            probes = ops.coarse_probes(xq, self.centroids, cn, nprobe)
        if self.device.type == "cuda":
            if self.scan_mode() == "lut":
                return ops._native().ivfpq_search(xq, self.centroids, self.pq, self.codes, self.ids,
                                                  self.list_off, probes.contiguous(), k)
            return ops._native().ivfpq_search_pt(xq, self.centroids, self.pq, self.codes, self._norms(),
                                                 self.ids, self.list_off, probes.contiguous(), k,
                                                 probes_per_workgroup(xq.shape[0], probes.shape[1]))
        return self._search_reference(xq, probes, k)

    def scan_mode(self) -> str:
        """``pt`` (precomputed tables: fp16 per-query LUT + stored norms) or ``lut`` (exact
        fp32 per-(query, list) LUT).  DOCQA_IVFPQ_SCAN=pt|lut forces one; ``auto`` (default)
        takes ``pt`` unless the vectors sit far from the origin relative to their residual
        spread: the pt decomposition ||q||^2 - 2<q, c> + ||c + r^||^2 - 2 sum <q_m, pq>
        cancels terms of size ||x||^2 down to a distance of size ||r||^2, so its fp16 LUT
        error grows with that ratio (unit-norm embeddings sit at ~2-4, an offset
        cloud at 400 measured 2.4e-3 relative distance error,
        tests/test_ivfpq_gpu.py::test_precomputed_table_scan_unnormalised_offset_vectors)."""
        mode = os.environ.get("DOCQA_IVFPQ_SCAN", "auto")
        if mode in ("pt", "lut"):
            return mode
        if getattr(self, "_auto_src", None) is not (self.centroids, self.pq):
            cn = float((self.centroids.float() ** 2).sum(1).mean())
            rn = float((self.pq.float() ** 2).sum(-1).mean(1).sum())      # E||r^||^2 over the M sub-spaces
            self._auto_mode = "lut" if cn > _PT_MAX_RATIO * max(rn, 1e-30) else "pt"
            self._auto_src = (self.centroids, self.pq)
        return self._auto_mode

    def _search_reference(self, xq, probes, k):
        nq = xq.shape[0]
        D = torch.full((nq, k), float("inf"))
        I = torch.full((nq, k), -1, dtype=torch.long)
        off = self.list_off.tolist()
        for q in range(nq):
            cand_d, cand_i = [], []
            for l in probes[q].tolist():
                if l < 0 or off[l] == off[l + 1]:
                    continue
                r = (xq[q] - self.centroids[l]).view(self.M, 1, self.dsub)
                lut = ((r - self.pq) ** 2).sum(-1)               # [M, 256]
                c = self.codes[off[l]:off[l + 1]].long()          # [n, M]
                dist = lut.gather(1, c.T).sum(0)                  # [n]
                cand_d.append(dist)
                cand_i.append(self.ids[off[l]:off[l + 1]])
            if cand_d:
                dd, ii = torch.cat(cand_d), torch.cat(cand_i)
                v, p = torch.topk(dd, min(k, dd.numel()), largest=False)
                D[q, :v.numel()] = v
                I[q, :v.numel()] = ii[p]
        return D, I

    # ------------------------------------------------------------------ FAISS IO
    def to_bytes(self) -> bytes:
        """FAISS bytes: ``IvPQ``, wrapped as IndexPreTransform(LinearTransform) -- ``IxPT`` +
        ``LTra`` with A = R^T, no bias -- when the index has a pre-rotation (faiss
        index_write.cpp write_VectorTransform layout)."""
        body = self._ivfpq_bytes()
        if self.rot is None:
            return body
        w = io.BytesIO()
        w.write(b"IxPT")
        faiss_io.write_header(w, self.d, self.ntotal, True, faiss_io.METRIC_L2)
        w.write(struct.pack("<i", 1))                        # chain length
        w.write(b"LTra")
        w.write(struct.pack("<B", 0))                        # have_bias
        faiss_io.write_vector(w, self.rot.t().contiguous().float().cpu().numpy().reshape(-1))   # A [d_out, d_in]
        faiss_io.write_vector(w, np.zeros(0, dtype=np.float32))                                # b
        w.write(struct.pack("<iiB", self.d, self.d, 1))     # d_in, d_out, is_trained
        w.write(body)
        return w.getvalue()

    def _ivfpq_bytes(self) -> bytes:
        w = io.BytesIO()
        w.write(b"IvPQ")
        faiss_io.write_header(w, self.d, self.ntotal, True, faiss_io.METRIC_L2)
        w.write(struct.pack("<QQ", self.nlist, self.nprobe))
        w.write(faiss_io.flat_bytes(self.centroids.float().cpu().numpy(), faiss_io.METRIC_L2))
        w.write(struct.pack("<b", 0))                        # direct map: NoMap
        faiss_io.write_vector(w, np.zeros(0, dtype=np.int64))
        w.write(struct.pack("<B", 1))                        # by_residual
        w.write(struct.pack("<Q", self.M))                   # code_size (8-bit codes)
        w.write(struct.pack("<QQQ", self.d, self.M, 8))      # ProductQuantizer d, M, nbits
        faiss_io.write_vector(w, self.pq.float().cpu().numpy().reshape(-1))
        w.write(b"ilar")
        w.write(struct.pack("<QQ", self.nlist, self.M))
        sizes = (self.list_off[1:] - self.list_off[:-1]).cpu().numpy().astype(np.uint64)
        w.write(b"full")
        faiss_io.write_vector(w, sizes)
        codes = self.codes.cpu().numpy()
        ids = self.ids.cpu().numpy().astype(np.int64)
        off = self.list_off.cpu().numpy()
        for l in range(self.nlist):
            a, b = int(off[l]), int(off[l + 1])
            if b > a:
                w.write(codes[a:b].tobytes())
                w.write(ids[a:b].tobytes())
        return w.getvalue()

    def save(self, path) -> None:
        faiss_io.atomic_write(path, self.to_bytes())

    @classmethod
    def load(cls, path, device="cuda") -> "IVFPQIndex":
        data = faiss_io.read_index(path)
        if not isinstance(data, cls):
            raise ValueError("not an IVF-PQ index")
        return data.to(device)

    def to(self, device) -> "IVFPQIndex":
        self.device = torch.device(device)
        for name in ("rot", "centroids", "pq", "codes", "ids", "list_off", "norms"):
            t = getattr(self, name)
            if t is not None:
                setattr(self, name, t.to(self.device))
        return self


def read_ivfpq_body(r: faiss_io.Reader) -> IVFPQIndex:
    d, ntotal, _, metric, _ = faiss_io.read_header(r)
    nlist, nprobe = r.unpack("<QQ")
    qfourcc = r.read(4)
    quant = faiss_io.read_flat(r, qfourcc)
    dm_type, = r.unpack("<b")
    r.vector(np.int64)
    if dm_type == 2:  # hashtable direct map: key/value vectors
        r.vector(np.int64)
    by_residual, = r.unpack("<B")
    code_size, = r.unpack("<Q")
    pq_d, M, nbits = r.unpack("<QQQ")
    cent = r.vector(np.float32)
    if nbits != 8 or not by_residual:
        raise ValueError("only 8-bit residual IVF-PQ is supported")
    if r.read(4) != b"ilar":
        raise ValueError("unsupported inverted-list storage")
    il_nlist, il_code_size = r.unpack("<QQ")
    kind = r.read(4)
    sizes_raw = r.vector(np.uint64).astype(np.int64)
    if kind == b"full":
        sizes = sizes_raw
    elif kind == b"sprs":
        sizes = np.zeros(il_nlist, dtype=np.int64)
        sizes[sizes_raw[0::2]] = sizes_raw[1::2]
    else:
        raise ValueError(f"unknown inverted-list kind {kind!r}")
    codes, ids = [], []
    for l in range(il_nlist):
        n = int(sizes[l])
        if n:
            codes.append(r.array(np.uint8, n * int(il_code_size)).reshape(n, int(il_code_size)))
            ids.append(r.array(np.int64, n))
    idx = IVFPQIndex(d, int(nlist), int(M), 8, device="cpu")
    idx.nprobe = int(nprobe)
    idx.centroids = torch.from_numpy(quant.xb.copy())
    idx.pq = torch.from_numpy(cent.reshape(int(M), 256, d // int(M)).copy())
    idx.codes = torch.from_numpy(np.concatenate(codes)) if codes else torch.empty(0, int(M), dtype=torch.uint8)
    idx.ids = torch.from_numpy(np.concatenate(ids)) if ids else torch.empty(0, dtype=torch.long)
    off = np.zeros(int(nlist) + 1, dtype=np.int64)
    off[1:] = np.cumsum(sizes)
    idx.list_off = torch.from_numpy(off)
    idx.ntotal = int(ntotal)
    return idx


def read_pretransform_body(r: faiss_io.Reader) -> IVFPQIndex:
    """``IxPT`` (IndexPreTransform) with one orthogonal ``LTra`` (no bias) over an IVF-PQ:
    the rotation becomes the index's pre-rotation R = A^T."""
    read_header = faiss_io.read_header
    d, _, _, _, _ = read_header(r)
    nt, = r.unpack("<i")
    if nt != 1:
        raise ValueError("IxPT: one linear transform supported")
    kind = r.read(4)
    if kind not in (b"LTra", b"Pcam", b"rrot"):
        raise ValueError(f"IxPT: unsupported vector transform {kind!r}")
    if kind == b"Pcam":
        raise ValueError("IxPT: PCAMatrix transforms are not supported")
    have_bias, = r.unpack("<B")
    A = r.vector(np.float32)
    b = r.vector(np.float32)
    d_in, d_out, _ = r.unpack("<iiB")
    if have_bias and b.size and np.any(b != 0):
        raise ValueError("IxPT: a biased linear transform is not supported")
    if d_in != d_out or A.size != d_in * d_out:
        raise ValueError("IxPT: only square (rotation) transforms are supported")
    sub = faiss_io.read_index_from(r)
    if not isinstance(sub, IVFPQIndex):
        raise ValueError("IxPT: only an IVF-PQ sub-index is supported")
    sub.rotation = "pca"
    sub.rot = torch.from_numpy(A.reshape(d_out, d_in).T.copy())
    return sub
