// bindings.cpp -- registers the gfx950 kernels as torch operators (torch.ops.docqa.*).
//
// Ops allocate their outputs through the PyTorch caching allocator and launch on the
// current HIP stream, so they run under torch.cuda.graph capture (HIP graphs) and on
// the side streams the pipeline uses for embed/search/generate overlap.
#include <torch/library.h>
#include <algorithm>
#include <tuple>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include "docqa_kernels.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_GPU(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_ALIGN16(t) \
  TORCH_CHECK((reinterpret_cast<uintptr_t>((t).data_ptr()) & 15u) == 0, \
              #t " must be 16-byte aligned (storage offset a multiple of 16 bytes)")
// DOCQA_KERNEL_DEBUG=1: synchronous kernel checking (the HIP_LAUNCH_BLOCKING of this
// extension): after every op that is not being graph-captured, the stream
// is synchronised and any asynchronous fault is reported with the op's name -- a
// faulting kernel is named by the op that launched it, not by a later unrelated sync.
static bool kernel_debug() {
  static const bool on = [] {
    const char* e = getenv("DOCQA_KERNEL_DEBUG");
    return e && atoi(e) != 0;
  }();
  return on;
}

static void debug_sync(const char* name) {
  hipStream_t s = stream();
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return;
  const hipError_t e = hipStreamSynchronize(s);
  TORCH_CHECK(e == hipSuccess, "docqa kernel ", name, " faulted (DOCQA_KERNEL_DEBUG): ", hipGetErrorString(e));
}

#define CHECK_RC(rc, name)                                                                 \
  do {                                                                                     \
    const int rc__ = (rc);                                                                 \
    TORCH_CHECK(rc__ == 0, "docqa kernel " name " failed with code ", rc__);               \
    if (kernel_debug()) debug_sync(name);                                                  \
  } while (0)

at::Tensor rmsnorm(const at::Tensor& x, const at::Tensor& w, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  const int H = x.size(-1);
  TORCH_CHECK(w.numel() == H, "rmsnorm weight size mismatch");
  c10::DeviceGuard g(x.device());
  auto out = at::empty_like(x);
  const int rows = x.numel() / H;
  CHECK_RC(docqa_rmsnorm(x.data_ptr(), w.data_ptr(), out.data_ptr(), rows, H, (float)eps, stream()), "rmsnorm");
  return out;
}

at::Tensor add_rmsnorm(const at::Tensor& x, at::Tensor residual, const at::Tensor& w, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_BF16(w);
  CHECK_CONTIG(x); CHECK_CONTIG(residual);
  TORCH_CHECK(x.sizes() == residual.sizes(), "add_rmsnorm shape mismatch");
  const int H = x.size(-1);
  c10::DeviceGuard g(x.device());
  auto out = at::empty_like(x);
  CHECK_RC(docqa_add_rmsnorm(x.data_ptr(), residual.data_ptr(), w.data_ptr(), out.data_ptr(),
                             x.numel() / H, H, (float)eps, stream()), "add_rmsnorm");
  return out;
}

at::Tensor layernorm(const at::Tensor& x, const c10::optional<at::Tensor>& residual,
                     const at::Tensor& gamma, const at::Tensor& beta, double eps) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(gamma); CHECK_BF16(beta);
  const int H = x.size(-1);
  const void* rp = nullptr;
  if (residual.has_value()) {
    CHECK_BF16(*residual); CHECK_CONTIG(*residual);
    TORCH_CHECK(residual->sizes() == x.sizes(), "layernorm residual shape mismatch");
    rp = residual->data_ptr();
  }
  c10::DeviceGuard g(x.device());
  auto out = at::empty_like(x);
  CHECK_RC(docqa_layernorm(x.data_ptr(), rp, gamma.data_ptr(), beta.data_ptr(), out.data_ptr(),
                           x.numel() / H, H, (float)eps, stream()), "layernorm");
  return out;
}

void rope_cache(at::Tensor qkv, const at::Tensor& positions, const at::Tensor& cos_sin,
                const c10::optional<at::Tensor>& slot_mapping, at::Tensor k_cache,
                at::Tensor v_cache, int64_t Hq, int64_t Hkv, int64_t D) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_I32(positions);
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat, "cos_sin must be fp32");
  TORCH_CHECK(qkv.stride(-1) == 1, "qkv rows must be contiguous");
  TORCH_CHECK(qkv.size(-1) == (Hq + 2 * Hkv) * D, "qkv width mismatch");
  const int T = qkv.numel() / qkv.size(-1);
  const int* sm = nullptr;
  int BS = 1;
  if (slot_mapping.has_value()) {
    CHECK_I32(*slot_mapping);
    sm = slot_mapping->data_ptr<int>();
    CHECK_BF16(k_cache); CHECK_BF16(v_cache);
    BS = k_cache.size(2);  // [num_blocks, Hkv, BS, D]
  }
  c10::DeviceGuard g(qkv.device());
  CHECK_RC(docqa_rope_cache(qkv.data_ptr(), positions.data_ptr<int>(), cos_sin.data_ptr<float>(),
                            sm, sm ? k_cache.data_ptr() : nullptr, sm ? v_cache.data_ptr() : nullptr,
                            T, Hq, Hkv, D, qkv.size(-1), BS, stream()), "rope_cache");
}

// token-granular prefix copies: K/V rows [0, m) of block src -> block dst in every pool
// (caches: int64 [2 L] device addresses of the [num_blocks, Hkv, BS, D] bf16 pools,
// tab: int32 [n, 3] (src, dst, m))
void kv_copy_rows(const at::Tensor& caches, const at::Tensor& tab, int64_t num_blocks, int64_t Hkv, int64_t BS,
                  int64_t D) {
  CHECK_GPU(caches); CHECK_GPU(tab); CHECK_I32(tab); CHECK_CONTIG(tab); CHECK_CONTIG(caches);
  TORCH_CHECK(caches.scalar_type() == at::kLong && caches.dim() == 1, "caches: int64 [2 L] addresses");
  TORCH_CHECK(tab.dim() == 2 && tab.size(1) == 3, "tab: [n, 3] (src, dst, rows)");
  c10::DeviceGuard g(tab.device());
  CHECK_RC(docqa_kv_copy_rows(reinterpret_cast<const uint64_t*>(caches.data_ptr<int64_t>()), (int)caches.numel(),
                              tab.data_ptr<int>(), (int)tab.size(0), (int)num_blocks, (int)Hkv, (int)BS, (int)D,
                              stream()),
           "kv_copy_rows");
}

// split-K partial slabs P [S, rows, H] fp32 -> residual += bf16(sum P); rmsnorm(residual) * w
at::Tensor add_rmsnorm_splitk(const at::Tensor& P, at::Tensor residual, const at::Tensor& w, double eps) {
  CHECK_GPU(P); CHECK_CONTIG(P); CHECK_BF16(residual); CHECK_CONTIG(residual); CHECK_BF16(w);
  TORCH_CHECK((P.scalar_type() == at::kFloat || P.scalar_type() == at::kBFloat16) && P.dim() == 3,
              "partials must be fp32 or bf16 [S, rows, H]");
  TORCH_CHECK(P.size(1) * P.size(2) == residual.numel() && P.size(2) == residual.size(-1),
              "add_rmsnorm_splitk shape mismatch");
  c10::DeviceGuard g(P.device());
  auto out = at::empty_like(residual);
  if (P.scalar_type() == at::kBFloat16)
    CHECK_RC(docqa_add_rmsnorm_splitk16(P.data_ptr(), P.size(0), residual.data_ptr(), w.data_ptr(),
                                        out.data_ptr(), P.size(1), P.size(2), (float)eps, stream()),
             "add_rmsnorm_splitk");
  else
    CHECK_RC(docqa_add_rmsnorm_splitk(P.data_ptr<float>(), P.size(0), residual.data_ptr(), w.data_ptr(),
                                      out.data_ptr(), P.size(1), P.size(2), (float)eps, stream()),
             "add_rmsnorm_splitk");
  return out;
}

// split-K partial slabs P [S, T, (Hq+2Hkv)*D] fp32 -> packed bf16 qkv (rotated) + cache write
at::Tensor rope_cache_splitk(const at::Tensor& P, const at::Tensor& positions, const at::Tensor& cos_sin,
                             const c10::optional<at::Tensor>& slot_mapping, at::Tensor k_cache,
                             at::Tensor v_cache, int64_t Hq, int64_t Hkv, int64_t D) {
  CHECK_GPU(P); CHECK_CONTIG(P); CHECK_I32(positions);
  TORCH_CHECK((P.scalar_type() == at::kFloat || P.scalar_type() == at::kBFloat16) && P.dim() == 3,
              "partials must be fp32 or bf16 [S, T, width]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat, "cos_sin must be fp32");
  TORCH_CHECK(P.size(2) == (Hq + 2 * Hkv) * D, "qkv width mismatch");
  const int T = P.size(1);
  const int* sm = nullptr;
  int BS = 1;
  if (slot_mapping.has_value()) {
    CHECK_I32(*slot_mapping);
    sm = slot_mapping->data_ptr<int>();
    CHECK_BF16(k_cache); CHECK_BF16(v_cache);
    BS = k_cache.size(2);
  }
  c10::DeviceGuard g(P.device());
  auto qkv = at::empty({T, P.size(2)}, P.options().dtype(at::kBFloat16));
  if (P.scalar_type() == at::kBFloat16)
    CHECK_RC(docqa_rope_cache_splitk16(P.data_ptr(), P.size(0), qkv.data_ptr(), positions.data_ptr<int>(),
                                       cos_sin.data_ptr<float>(), sm, sm ? k_cache.data_ptr() : nullptr,
                                       sm ? v_cache.data_ptr() : nullptr, T, Hq, Hkv, D, P.size(2), BS,
                                       stream()), "rope_cache_splitk");
  else
    CHECK_RC(docqa_rope_cache_splitk(P.data_ptr<float>(), P.size(0), qkv.data_ptr(), positions.data_ptr<int>(),
                                     cos_sin.data_ptr<float>(), sm, sm ? k_cache.data_ptr() : nullptr,
                                     sm ? v_cache.data_ptr() : nullptr, T, Hq, Hkv, D, P.size(2), BS,
                                     stream()), "rope_cache_splitk");
  return qkv;
}

// split-K SwiGLU consumer: P [S, T, 2I] fp32 slabs of an 8-interleaved gate|up projection
// -> [T, I] bf16 silu(gate) * up
at::Tensor silu_mul_splitk(const at::Tensor& P) {
  CHECK_GPU(P); CHECK_CONTIG(P); CHECK_ALIGN16(P);
  TORCH_CHECK((P.scalar_type() == at::kFloat || P.scalar_type() == at::kBFloat16) && P.dim() == 3,
              "silu_mul_splitk: float32 or bf16 [S, T, 2I]");
  const int S = P.size(0), T = P.size(1), I2 = P.size(2);
  TORCH_CHECK(I2 % 16 == 0, "silu_mul_splitk: 2I % 16");
  c10::DeviceGuard g(P.device());
  auto out = at::empty({T, I2 / 2}, P.options().dtype(at::kBFloat16));
  if (P.scalar_type() == at::kBFloat16)
    CHECK_RC(docqa_silu_mul_splitk16(P.data_ptr(), out.data_ptr(), S, T, I2 / 2, stream()), "silu_mul_splitk");
  else
    CHECK_RC(docqa_silu_mul_splitk(P.data_ptr<float>(), out.data_ptr(), S, T, I2 / 2, stream()), "silu_mul_splitk");
  return out;
}

at::Tensor silu_mul(const at::Tensor& gu, bool interleaved) {
  CHECK_GPU(gu); CHECK_BF16(gu); CHECK_CONTIG(gu);
  const int I2 = gu.size(-1);
  auto sizes = gu.sizes().vec();
  sizes.back() = I2 / 2;
  c10::DeviceGuard g(gu.device());
  auto out = at::empty(sizes, gu.options());
  CHECK_RC(docqa_silu_mul(gu.data_ptr(), out.data_ptr(), gu.numel() / I2, I2 / 2, interleaved ? 1 : 0,
                          stream()), "silu_mul");
  return out;
}

at::Tensor bias_act(const at::Tensor& x, const at::Tensor& bias,
                    const c10::optional<at::Tensor>& residual, bool gelu) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_CONTIG(x); CHECK_BF16(bias);
  const int N = x.size(-1);
  TORCH_CHECK(bias.numel() == N, "bias size mismatch");
  const void* rp = nullptr;
  if (residual.has_value()) { CHECK_BF16(*residual); CHECK_CONTIG(*residual); rp = residual->data_ptr(); }
  c10::DeviceGuard g(x.device());
  auto out = at::empty_like(x);
  CHECK_RC(docqa_bias_act(x.data_ptr(), bias.data_ptr(), rp, out.data_ptr(), x.numel() / N, N,
                          gelu ? 1 : 0, stream()), "bias_act");
  return out;
}

at::Tensor embedding(const at::Tensor& ids, const at::Tensor& table) {
  CHECK_GPU(ids); CHECK_I32(ids); CHECK_BF16(table); CHECK_CONTIG(table);
  const int H = table.size(1);
  auto sizes = ids.sizes().vec();
  sizes.push_back(H);
  c10::DeviceGuard g(ids.device());
  auto out = at::empty(sizes, table.options());
  CHECK_RC(docqa_embedding(ids.data_ptr<int>(), table.data_ptr(), out.data_ptr(), ids.numel(), H, (int)table.size(0), stream()), "embedding");
  return out;
}

// (h, x): h = table[ids] (residual stream), x = rmsnorm(h) * w
std::tuple<at::Tensor, at::Tensor> embed_rmsnorm(const at::Tensor& ids, const at::Tensor& table, const at::Tensor& w,
                                                 double eps) {
  CHECK_GPU(ids); CHECK_I32(ids); CHECK_CONTIG(ids); CHECK_BF16(table); CHECK_CONTIG(table); CHECK_BF16(w);
  const int H = table.size(1);
  TORCH_CHECK(w.numel() == H, "embed_rmsnorm: weight of H");
  auto sizes = ids.sizes().vec();
  sizes.push_back(H);
  c10::DeviceGuard g(ids.device());
  auto h = at::empty(sizes, table.options());
  auto x = at::empty(sizes, table.options());
  CHECK_RC(docqa_embed_rmsnorm(ids.data_ptr<int>(), table.data_ptr(), w.data_ptr(), h.data_ptr(), x.data_ptr(),
                               ids.numel(), H, (int)table.size(0), (float)eps, stream()), "embed_rmsnorm");
  return {h, x};
}

at::Tensor bert_embed_ln(const at::Tensor& ids, const at::Tensor& pos,
                         const c10::optional<at::Tensor>& token_type, const at::Tensor& wte,
                         const at::Tensor& wpe, const at::Tensor& wtt, const at::Tensor& gamma,
                         const at::Tensor& beta, double eps) {
  CHECK_GPU(ids); CHECK_I32(ids); CHECK_I32(pos); CHECK_BF16(wte);
  const int H = wte.size(1);
  const int* tt = nullptr;
  if (token_type.has_value()) { CHECK_I32(*token_type); tt = token_type->data_ptr<int>(); }
  c10::DeviceGuard g(ids.device());
  auto out = at::empty({ids.numel(), H}, wte.options());
  CHECK_RC(docqa_bert_embed_ln(ids.data_ptr<int>(), pos.data_ptr<int>(), tt, wte.data_ptr(),
                               wpe.data_ptr(), wtt.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                               out.data_ptr(), ids.numel(), H, (float)eps, stream()), "bert_embed_ln");
  return out;
}

// decode-step state: paged-cache slot of every row's next token (-1: padded row)
at::Tensor decode_slots(const at::Tensor& block_tables, const at::Tensor& positions,
                        const at::Tensor& valid, int64_t BS) {
  CHECK_GPU(block_tables);
  TORCH_CHECK(block_tables.scalar_type() == at::kInt && positions.scalar_type() == at::kInt &&
                  valid.scalar_type() == at::kInt, "decode_slots: int32 tensors");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.is_contiguous() && positions.is_contiguous() &&
                  valid.is_contiguous(), "decode_slots: contiguous [B, maxb], [B], [B]");
  const int B = block_tables.size(0);
  TORCH_CHECK(positions.numel() == B && valid.numel() == B, "decode_slots: B mismatch");
  c10::DeviceGuard g(block_tables.device());
  auto slots = at::empty({B}, positions.options());
  CHECK_RC(docqa_decode_slots(block_tables.data_ptr<int>(), block_tables.size(1), positions.data_ptr<int>(),
                              valid.data_ptr<int>(), slots.data_ptr<int>(), B, (int)BS, stream()),
           "decode_slots");
  return slots;
}

// out <- nxt, tokens <- nxt, positions += valid, context_lens += valid (in place)
void decode_advance(const at::Tensor& nxt, at::Tensor out, at::Tensor tokens, at::Tensor positions,
                    at::Tensor context_lens, const at::Tensor& valid) {
  CHECK_GPU(nxt);
  const int B = nxt.numel();
  TORCH_CHECK(nxt.scalar_type() == at::kLong && out.scalar_type() == at::kLong &&
                  tokens.scalar_type() == at::kInt && positions.scalar_type() == at::kInt &&
                  context_lens.scalar_type() == at::kInt && valid.scalar_type() == at::kInt,
              "decode_advance: int64 nxt/out, int32 state");
  TORCH_CHECK(out.numel() == B && tokens.numel() == B && positions.numel() == B &&
                  context_lens.numel() == B && valid.numel() == B, "decode_advance: B mismatch");
  TORCH_CHECK(nxt.is_contiguous() && out.is_contiguous() && tokens.is_contiguous() &&
                  positions.is_contiguous() && context_lens.is_contiguous() && valid.is_contiguous(),
              "decode_advance: contiguous tensors");
  c10::DeviceGuard g(nxt.device());
  CHECK_RC(docqa_decode_advance(nxt.data_ptr<int64_t>(), out.data_ptr<int64_t>(), tokens.data_ptr<int>(),
                                positions.data_ptr<int>(), context_lens.data_ptr<int>(), valid.data_ptr<int>(),
                                B, stream()), "decode_advance");
}

at::Tensor argmax(const at::Tensor& logits) {
  CHECK_GPU(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "argmax wants [rows, V] with unit stride");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || logits.scalar_type() == at::kFloat, "argmax: bf16 or fp32 logits");
  const int rows = logits.size(0), V = logits.size(1);
  int splits = (V + 8191) / 8192;
  if (splits > 64) splits = 64;
  if (splits < 1) splits = 1;
  c10::DeviceGuard g(logits.device());
  auto ws_v = at::empty({rows * splits}, logits.options().dtype(at::kFloat));
  auto ws_i = at::empty({rows * splits}, logits.options().dtype(at::kInt));
  auto out = at::empty({rows}, logits.options().dtype(at::kLong));
  CHECK_RC(docqa_argmax(logits.data_ptr(), rows, V, logits.stride(0), bf ? 1 : 0,
                        ws_v.data_ptr<float>(), ws_i.data_ptr<int>(), splits,
                        out.data_ptr<int64_t>(), stream()), "argmax");
  return out;
}

// fused NER head + argmax: h [T, H] bf16 (row stride may exceed H), w [NL, H] bf16 with
// NL in {8, 16, 32} (zero-padded label rows), bias [NL] bf16; labels >= n_valid never win
at::Tensor token_cls_argmax(const at::Tensor& h, const at::Tensor& w, const at::Tensor& bias,
                            int64_t n_valid) {
  CHECK_GPU(h); CHECK_GPU(w); CHECK_GPU(bias);
  CHECK_BF16(h); CHECK_BF16(w); CHECK_BF16(bias);
  CHECK_CONTIG(w); CHECK_CONTIG(bias);
  TORCH_CHECK(h.dim() == 2 && h.stride(1) == 1, "token_cls_argmax wants h [T, H] with unit stride");
  TORCH_CHECK(w.dim() == 2 && w.size(1) == h.size(1), "token_cls_argmax: w [NL, H] must match h");
  TORCH_CHECK(bias.numel() == w.size(0), "token_cls_argmax: bias [NL]");
  CHECK_ALIGN16(h); CHECK_ALIGN16(w); CHECK_ALIGN16(bias);
  const int T = h.size(0), H = h.size(1), NL = w.size(0);
  c10::DeviceGuard g(h.device());
  auto out = at::empty({T}, h.options().dtype(at::kLong));
  CHECK_RC(docqa_token_cls_argmax(h.data_ptr(), h.stride(0), w.data_ptr(), bias.data_ptr(), NL,
                                  (int)n_valid, T, H, out.data_ptr<int64_t>(), stream()),
           "token_cls_argmax");
  return out;
}

at::Tensor sample(const at::Tensor& logits, const at::Tensor& inv_temp, const at::Tensor& top_k,
                  const at::Tensor& top_p, const at::Tensor& u) {
  CHECK_GPU(logits);
  TORCH_CHECK(logits.scalar_type() == at::kFloat && logits.dim() == 2 && logits.stride(1) == 1,
              "sample wants fp32 [rows, V]");
  CHECK_I32(top_k);
  c10::DeviceGuard g(logits.device());
  auto out = at::empty({logits.size(0)}, logits.options().dtype(at::kLong));
  CHECK_RC(docqa_sample(logits.data_ptr<float>(), logits.size(0), logits.size(1), logits.stride(0),
                        inv_temp.data_ptr<float>(), top_k.data_ptr<int>(), top_p.data_ptr<float>(),
                        u.data_ptr<float>(), out.data_ptr<int64_t>(), stream()), "sample");
  return out;
}

// optional LPT dispatch order of the decode workgroups (int32 permutation of [0, B))
static const int* order_ptr(const c10::optional<at::Tensor>& order, int B) {
  if (!order.has_value() || !order->defined()) return nullptr;
  TORCH_CHECK(order->scalar_type() == at::kInt && order->is_contiguous() && order->numel() == B,
              "order: contiguous int32 [B]");
  return order->data_ptr<int>();
}

at::Tensor paged_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                        const at::Tensor& block_tables, const at::Tensor& context_lens,
                        int64_t Hq, int64_t max_context, double scale,
                        const c10::optional<at::Tensor>& order) {
  // q: [B, >= Hq*D] rows (e.g. the packed QKV buffer), caches [NB, Hkv, BS, D]
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(context_lens); CHECK_CONTIG(block_tables);
  TORCH_CHECK(q.stride(-1) == 1, "q rows must be contiguous");
  const int B = q.size(0);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  const int max_parts = docqa_decode_splits(B, Hkv, max_context);
  c10::DeviceGuard g(q.device());
  auto out = at::empty({B, Hq * D}, q.options());
  auto tmp_out = at::empty({B, Hq, max_parts, D}, q.options().dtype(at::kFloat));
  auto tmp_ml = at::empty({B, Hq, max_parts, 2}, q.options().dtype(at::kFloat));
  CHECK_RC(docqa_paged_decode(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                              block_tables.data_ptr<int>(), block_tables.size(1),
                              context_lens.data_ptr<int>(), out.data_ptr(), Hq * D,
                              tmp_out.data_ptr<float>(), tmp_ml.data_ptr<float>(), B, Hq, Hkv, D,
                              BS, max_parts, (float)scale, order_ptr(order, B), stream()), "paged_decode");
  return out;
}

// cascade decode attention: the prompt prefix shared by every sequence of the batch
// (prefix_table: its block ids, prefix_len: device scalar, multiple of 64) is attended once
// for all rows by the MFMA prefix kernel; each sequence's suffix by the ring kernel
at::Tensor paged_decode_cascade(const at::Tensor& q, at::Tensor k_cache, at::Tensor v_cache,
                                const at::Tensor& block_tables, const at::Tensor& context_lens,
                                int64_t Hq, int64_t max_context, double scale,
                                const at::Tensor& prefix_table, const at::Tensor& prefix_len,
                                int64_t nchunk, const c10::optional<at::Tensor>& order) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(context_lens); CHECK_CONTIG(block_tables);
  CHECK_I32(prefix_table); CHECK_I32(prefix_len); CHECK_CONTIG(prefix_table);
  TORCH_CHECK(q.stride(-1) == 1, "q rows must be contiguous");
  const int B = q.size(0);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(D == 128 && BS == 64 && Hq == 4 * Hkv, "cascade decode: head_dim 128, 64-token blocks, GQA 4");
  TORCH_CHECK(block_tables.size(1) <= 256, "cascade decode: <= 256 blocks per sequence");
  TORCH_CHECK(prefix_table.numel() >= 1 && prefix_len.numel() == 1, "cascade decode: prefix table / length");
  const int max_parts = docqa_decode_splits(B, Hkv, max_context);
  c10::DeviceGuard g(q.device());
  auto out = at::empty({B, Hq * D}, q.options());
  auto f32 = q.options().dtype(at::kFloat);
  auto tmp_out = at::empty({B, Hq, max_parts, D}, f32);
  auto tmp_ml = at::empty({B, Hq, max_parts, 2}, f32);
  auto pacc = at::empty({nchunk, B, Hq, D}, f32);
  auto pml = at::empty({nchunk, B, Hq, 2}, f32);
  CHECK_RC(docqa_paged_decode_cascade(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                      block_tables.data_ptr<int>(), block_tables.size(1),
                                      context_lens.data_ptr<int>(), out.data_ptr(), Hq * D,
                                      tmp_out.data_ptr<float>(), tmp_ml.data_ptr<float>(), B, Hq, Hkv, BS,
                                      max_parts, (float)scale, prefix_table.data_ptr<int>(),
                                      prefix_len.data_ptr<int>(), (int)nchunk, pacc.data_ptr<float>(),
                                      pml.data_ptr<float>(), order_ptr(order, B), stream()),
           "paged_decode_cascade");
  return out;
}

// cascade decode with the rows packed into groups of <= 4 by shared prefix-cache blocks
// (groups [ngroups, 4] int32 row ids, -1 = none): each shared block is read once per group
at::Tensor paged_decode_cascade_grouped(const at::Tensor& q, at::Tensor k_cache, at::Tensor v_cache,
                                        const at::Tensor& block_tables, const at::Tensor& context_lens,
                                        int64_t Hq, double scale, const at::Tensor& prefix_table,
                                        const at::Tensor& prefix_len, int64_t nchunk, const at::Tensor& groups) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(context_lens); CHECK_CONTIG(block_tables);
  CHECK_I32(prefix_table); CHECK_I32(prefix_len); CHECK_CONTIG(prefix_table);
  CHECK_I32(groups); CHECK_CONTIG(groups);
  TORCH_CHECK(q.stride(-1) == 1, "q rows must be contiguous");
  const int B = q.size(0);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(D == 128 && BS == 64 && Hq == 4 * Hkv, "grouped decode: head_dim 128, 64-token blocks, GQA 4");
  TORCH_CHECK(block_tables.size(1) <= 256, "grouped decode: block table <= 256 wide (rows <= 64 blocks: the caller)");
  TORCH_CHECK(context_lens.numel() == B && block_tables.size(0) >= B, "grouped decode: B rows");
  TORCH_CHECK(groups.numel() % 4 == 0 && groups.numel() >= 4, "groups: [ngroups, 4]");
  TORCH_CHECK(prefix_table.numel() >= 1 && prefix_len.numel() == 1, "cascade decode: prefix table / length");
  c10::DeviceGuard g(q.device());
  auto out = at::empty({B, Hq * D}, q.options());
  auto f32 = q.options().dtype(at::kFloat);
  auto pacc = at::empty({nchunk, B, Hq, D}, f32);
  auto pml = at::empty({nchunk, B, Hq, 2}, f32);
  CHECK_RC(docqa_paged_decode_cascade_grouped(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                              block_tables.data_ptr<int>(), block_tables.size(1),
                                              context_lens.data_ptr<int>(), out.data_ptr(), Hq * D, B, Hq, Hkv,
                                              BS, (float)scale, prefix_table.data_ptr<int>(),
                                              prefix_len.data_ptr<int>(), (int)nchunk, pacc.data_ptr<float>(),
                                              pml.data_ptr<float>(), groups.data_ptr<int>(),
                                              (int)(groups.numel() / 4), stream()),
           "paged_decode_cascade_grouped");
  return out;
}

// grouped cascade decode with long groups split over several workgroups: plan [2, cap, 8]
// int32 = work items (4 row ids, first / end block position, partial slot or -1, 0) and
// merges (4 row ids, first slot, slots, 0, 0) -- ops.split_decode_groups
// grouped decode straight from the QKV projection's split-K slabs P [S, B, (Hq + 2 Hkv) 128]:
// RoPE + the new token's cache write inside the group kernel (split plan from block 0)
at::Tensor paged_decode_grouped_fused(const at::Tensor& P, const at::Tensor& positions, const at::Tensor& cos_sin,
                                      const at::Tensor& slot_mapping, at::Tensor k_cache, at::Tensor v_cache,
                                      const at::Tensor& block_tables, const at::Tensor& context_lens, int64_t Hq,
                                      double scale, const at::Tensor& prefix_table, const at::Tensor& prefix_len,
                                      int64_t nchunk, const at::Tensor& plan, const c10::optional<at::Tensor>& tick) {
  CHECK_GPU(P); CHECK_CONTIG(P); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(positions); CHECK_I32(slot_mapping); CHECK_I32(block_tables); CHECK_I32(context_lens);
  CHECK_CONTIG(block_tables); CHECK_I32(prefix_table); CHECK_I32(prefix_len); CHECK_I32(plan); CHECK_CONTIG(plan);
  TORCH_CHECK(P.scalar_type() == at::kFloat && P.dim() == 3, "fused grouped decode: slabs fp32 [S, B, width]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat, "cos_sin must be fp32");
  const int B = P.size(1);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(D == 128 && BS == 64 && Hq == 4 * Hkv && P.size(2) == (Hq + 2 * Hkv) * D,
              "fused grouped decode: head_dim 128, 64-token blocks, GQA 4, packed QKV width");
  TORCH_CHECK(block_tables.size(1) <= 256 && context_lens.numel() == B && block_tables.size(0) >= B &&
              positions.numel() >= B && slot_mapping.numel() >= B, "fused grouped decode: B rows, block table <= 256 wide");
  TORCH_CHECK(plan.dim() == 3 && plan.size(0) == 2 && plan.size(2) == 8, "fused grouped decode: split plan [2, cap, 8]");
  const int cap = plan.size(1);
  c10::DeviceGuard g(P.device());
  auto out = at::empty({B, Hq * D}, P.options().dtype(at::kBFloat16));
  auto f32 = P.options();
  auto ws_acc = at::empty({cap, Hkv, 16, D}, f32);
  auto ws_ml = at::empty({cap, Hkv, 16, 2}, f32);
  int* tick_ptr = nullptr;
  if (tick && tick->defined()) {
    CHECK_GPU((*tick)); CHECK_I32((*tick));
    TORCH_CHECK(tick->numel() >= (int64_t)cap * Hkv, "fused grouped decode: tick needs cap * Hkv entries");
    tick_ptr = tick->data_ptr<int>();
  }
  const int* pp = plan.data_ptr<int>();
  CHECK_RC(docqa_paged_decode_cascade_split(nullptr, 0, k_cache.data_ptr(), v_cache.data_ptr(),
                                            block_tables.data_ptr<int>(), block_tables.size(1),
                                            context_lens.data_ptr<int>(), out.data_ptr(), Hq * D, B, Hq, Hkv, BS,
                                            (float)scale, prefix_table.data_ptr<int>(), prefix_len.data_ptr<int>(),
                                            (int)nchunk, nullptr, nullptr, pp, pp + 8 * cap, cap,
                                            ws_acc.data_ptr<float>(), ws_ml.data_ptr<float>(), 0, stream(), tick_ptr, 1,
                                            P.data_ptr<float>(), P.size(0), positions.data_ptr<int>(),
                                            cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int>()),
           "paged_decode_grouped_fused");
  return out;
}

at::Tensor paged_decode_cascade_split(const at::Tensor& q, at::Tensor k_cache, at::Tensor v_cache,
                                      const at::Tensor& block_tables, const at::Tensor& context_lens,
                                      int64_t Hq, double scale, const at::Tensor& prefix_table,
                                      const at::Tensor& prefix_len, int64_t nchunk, const at::Tensor& plan,
                                      bool defer, const c10::optional<at::Tensor>& tick, bool inline_prefix) {
  CHECK_GPU(q); CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(context_lens); CHECK_CONTIG(block_tables);
  CHECK_I32(prefix_table); CHECK_I32(prefix_len); CHECK_CONTIG(prefix_table);
  CHECK_I32(plan); CHECK_CONTIG(plan);
  TORCH_CHECK(q.stride(-1) == 1, "q rows must be contiguous");
  const int B = q.size(0);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(D == 128 && BS == 64 && Hq == 4 * Hkv, "split decode: head_dim 128, 64-token blocks, GQA 4");
  TORCH_CHECK(block_tables.size(1) <= 256, "split decode: block table <= 256 wide (rows <= 64 blocks: the caller)");
  TORCH_CHECK(k_cache.size(0) < (1 << 20), "split decode: < 2^20 KV blocks (packed tile lists)");
  TORCH_CHECK(context_lens.numel() == B && block_tables.size(0) >= B, "split decode: B rows");
  TORCH_CHECK(plan.dim() == 3 && plan.size(0) >= 2 && plan.size(0) <= 3 && plan.size(2) == 8 && plan.size(1) >= 1,
              "plan: [2, cap, 8] (split) or [3, cap, 8] (persistent bins)");
  TORCH_CHECK(prefix_table.numel() >= 1 && prefix_len.numel() == 1, "cascade decode: prefix table / length");
  const int cap = plan.size(1);
  c10::DeviceGuard g(q.device());
  auto out = at::empty({B, Hq * D}, q.options());
  auto f32 = q.options().dtype(at::kFloat);
  auto pacc = at::empty({nchunk, B, Hq, D}, f32);
  auto pml = at::empty({nchunk, B, Hq, 2}, f32);
  auto ws_acc = at::empty({cap, Hkv, 16, D}, f32);
  auto ws_ml = at::empty({cap, Hkv, 16, 2}, f32);
  const int* pp = plan.data_ptr<int>();
  int* tick_ptr = nullptr;   // split groups merged by their last item (zeroed int32 [cap * Hkv])
  if (tick && tick->defined()) {
    CHECK_GPU((*tick)); CHECK_I32((*tick));
    TORCH_CHECK(tick->numel() >= (int64_t)cap * Hkv, "split decode: tick needs cap * Hkv entries");
    tick_ptr = tick->data_ptr<int>();
  }
  if (plan.size(0) == 3) {
    CHECK_RC(docqa_paged_decode_cascade_persist(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                                block_tables.data_ptr<int>(), block_tables.size(1),
                                                context_lens.data_ptr<int>(), out.data_ptr(), Hq * D, B, Hq, Hkv,
                                                BS, (float)scale, prefix_table.data_ptr<int>(),
                                                prefix_len.data_ptr<int>(), (int)nchunk, pacc.data_ptr<float>(),
                                                pml.data_ptr<float>(), pp, pp + 8 * cap, pp + 16 * cap, cap,
                                                ws_acc.data_ptr<float>(), ws_ml.data_ptr<float>(), stream()),
             "paged_decode_cascade_persist");
    return out;
  }
  CHECK_RC(docqa_paged_decode_cascade_split(q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                            block_tables.data_ptr<int>(), block_tables.size(1),
                                            context_lens.data_ptr<int>(), out.data_ptr(), Hq * D, B, Hq, Hkv,
                                            BS, (float)scale, prefix_table.data_ptr<int>(),
                                            prefix_len.data_ptr<int>(), (int)nchunk, pacc.data_ptr<float>(),
                                            pml.data_ptr<float>(), pp, pp + 8 * cap, cap, ws_acc.data_ptr<float>(),
                                            ws_ml.data_ptr<float>(), defer ? 1 : 0, stream(), tick_ptr,
                                            inline_prefix ? 1 : 0),
           "paged_decode_cascade_split");
  return out;
}

// cascade decode over the UNROTATED packed QKV of a library GEMM: RoPE, the new token's
// cache write and the attention in the cascade kernels (fallback: rope_cache in place)
at::Tensor paged_decode_cascade_rope(at::Tensor qkv, const at::Tensor& positions, const at::Tensor& cos_sin,
                                     const at::Tensor& slot_mapping, at::Tensor k_cache, at::Tensor v_cache,
                                     const at::Tensor& block_tables, const at::Tensor& context_lens,
                                     int64_t Hq, int64_t max_context, double scale,
                                     const at::Tensor& prefix_table, const at::Tensor& prefix_len,
                                     int64_t nchunk, const c10::optional<at::Tensor>& order) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(positions); CHECK_I32(slot_mapping); CHECK_I32(block_tables); CHECK_I32(context_lens);
  CHECK_CONTIG(block_tables); CHECK_I32(prefix_table); CHECK_I32(prefix_len); CHECK_CONTIG(prefix_table);
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be [B, width] with unit stride");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat, "cos_sin must be fp32");
  const int B = qkv.size(0);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(D == 128 && BS == 64 && Hq == 4 * Hkv, "cascade decode: head_dim 128, 64-token blocks, GQA 4");
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * D, "qkv rows narrower than the packed QKV width");
  TORCH_CHECK(positions.numel() == B && slot_mapping.numel() == B && context_lens.numel() == B,
              "positions / slot_mapping / context_lens must have B entries");
  TORCH_CHECK(block_tables.size(1) <= 256, "cascade decode: <= 256 blocks per sequence");
  TORCH_CHECK(prefix_table.numel() >= 1 && prefix_len.numel() == 1, "cascade decode: prefix table / length");
  const int max_parts = docqa_decode_splits(B, Hkv, max_context);
  c10::DeviceGuard g(qkv.device());
  auto out = at::empty({B, Hq * D}, qkv.options());
  auto f32 = qkv.options().dtype(at::kFloat);
  auto tmp_out = at::empty({B, Hq, max_parts, D}, f32);
  auto tmp_ml = at::empty({B, Hq, max_parts, 2}, f32);
  auto pacc = at::empty({nchunk, B, Hq, D}, f32);
  auto pml = at::empty({nchunk, B, Hq, 2}, f32);
  CHECK_RC(docqa_paged_decode_cascade_rope(qkv.data_ptr(), qkv.stride(0), positions.data_ptr<int>(),
                                           cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int>(),
                                           k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                           block_tables.size(1), context_lens.data_ptr<int>(), out.data_ptr(),
                                           Hq * D, tmp_out.data_ptr<float>(), tmp_ml.data_ptr<float>(), B, Hq,
                                           Hkv, BS, max_parts, (float)scale, prefix_table.data_ptr<int>(),
                                           prefix_len.data_ptr<int>(), (int)nchunk, pacc.data_ptr<float>(),
                                           pml.data_ptr<float>(), order_ptr(order, B), stream()),
           "paged_decode_cascade_rope");
  return out;
}

// decode step attention fed by the QKV projection's split-K partial slabs: RoPE + cache
// write of the new token + paged attention in one launch (ring kernel)
at::Tensor paged_decode_fused(const at::Tensor& P, const at::Tensor& positions, const at::Tensor& cos_sin,
                              const at::Tensor& slot_mapping, at::Tensor k_cache, at::Tensor v_cache,
                              const at::Tensor& block_tables, const at::Tensor& context_lens,
                              int64_t Hq, int64_t max_context, double scale,
                              const c10::optional<at::Tensor>& order, const c10::optional<at::Tensor>& tick) {
  CHECK_GPU(P); CHECK_CONTIG(P); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(positions); CHECK_I32(slot_mapping); CHECK_I32(block_tables); CHECK_I32(context_lens);
  CHECK_CONTIG(block_tables);
  TORCH_CHECK(P.scalar_type() == at::kFloat && P.dim() == 3, "partials must be fp32 [S, B, width]");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat, "cos_sin must be fp32");
  const int B = P.size(1);
  const int Hkv = k_cache.size(1), BS = k_cache.size(2), D = k_cache.size(3);
  TORCH_CHECK(D == 128 && P.size(2) == (Hq + 2 * Hkv) * D, "fused decode: head_dim 128, packed QKV width");
  const int max_parts = docqa_decode_splits(B, Hkv, max_context);
  c10::DeviceGuard g(P.device());
  auto out = at::empty({B, Hq * D}, P.options().dtype(at::kBFloat16));
  auto tmp_out = at::empty({B, Hq, max_parts, D}, P.options());
  auto tmp_ml = at::empty({B, Hq, max_parts, 2}, P.options());
  // tick: zeroed int32 [>= B * Hkv] owned by the caller (the kernel re-arms it): the split
  // partitions are merged by their last workgroup instead of a second launch
  int* tick_ptr = nullptr;
  if (tick && tick->defined()) {
    CHECK_GPU((*tick)); CHECK_I32((*tick));
    TORCH_CHECK(tick->numel() >= (int64_t)B * Hkv, "paged_decode_fused: tick needs B * Hkv entries");
    tick_ptr = tick->data_ptr<int>();
  }
  CHECK_RC(docqa_paged_decode_fused(P.data_ptr<float>(), P.size(0), positions.data_ptr<int>(),
                                    cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int>(),
                                    k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                    block_tables.size(1), context_lens.data_ptr<int>(), out.data_ptr(),
                                    Hq * D, tmp_out.data_ptr<float>(), tmp_ml.data_ptr<float>(), B, Hq,
                                    Hkv, BS, max_parts, (float)scale, order_ptr(order, B), stream(), tick_ptr),
           "paged_decode_fused");
  return out;
}

at::Tensor flash_prefill(const at::Tensor& qkv, const at::Tensor& cu_seqlens, int64_t max_len,
                         int64_t Hq, int64_t Hkv, int64_t D, double scale, bool causal) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_I32(cu_seqlens);
  TORCH_CHECK(qkv.stride(-1) == 1 && qkv.size(-1) == (Hq + 2 * Hkv) * D, "qkv layout mismatch");
  const int T = qkv.numel() / qkv.size(-1);
  const int B = cu_seqlens.numel() - 1;
  c10::DeviceGuard g(qkv.device());
  auto out = at::empty({T, Hq * D}, qkv.options());
  CHECK_RC(docqa_flash_prefill(qkv.data_ptr(), qkv.size(-1), cu_seqlens.data_ptr<int>(),
                               out.data_ptr(), Hq * D, B, max_len, Hq, Hkv, D, (float)scale,
                               causal ? 1 : 0, stream()), "flash_prefill");
  return out;
}

at::Tensor flash_prefill_paged(const at::Tensor& qkv, const at::Tensor& cu_seqlens, int64_t max_len,
                               int64_t Hq, int64_t Hkv, int64_t D, double scale,
                               const at::Tensor& k_cache, const at::Tensor& v_cache,
                               const at::Tensor& block_tables, const at::Tensor& ctx_start) {
  CHECK_GPU(qkv); CHECK_BF16(qkv); CHECK_I32(cu_seqlens); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(ctx_start); CHECK_CONTIG(block_tables);
  TORCH_CHECK(qkv.stride(-1) == 1 && qkv.size(-1) == (Hq + 2 * Hkv) * D, "qkv layout mismatch");
  TORCH_CHECK(k_cache.size(1) == Hkv && k_cache.size(3) == D, "cache layout mismatch");
  const int T = qkv.numel() / qkv.size(-1);
  const int B = cu_seqlens.numel() - 1;
  TORCH_CHECK(block_tables.size(0) == B && ctx_start.numel() == B, "per-sequence metadata mismatch");
  c10::DeviceGuard g(qkv.device());
  auto out = at::empty({T, Hq * D}, qkv.options());
  CHECK_RC(docqa_flash_prefill_paged(qkv.data_ptr(), qkv.size(-1), cu_seqlens.data_ptr<int>(),
                                     out.data_ptr(), Hq * D, B, max_len, Hq, Hkv, D, (float)scale,
                                     k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr<int>(),
                                     block_tables.size(1), ctx_start.data_ptr<int>(), k_cache.size(2),
                                     stream()), "flash_prefill_paged");
  return out;
}

// epilogue: 0 none, 1 bias, 2 bias+gelu, 3 bias+residual
at::Tensor gemm(const at::Tensor& a, const at::Tensor& w, const c10::optional<at::Tensor>& bias,
                const c10::optional<at::Tensor>& residual, int64_t epi) {
  CHECK_GPU(a); CHECK_BF16(a); CHECK_BF16(w); CHECK_CONTIG(a); CHECK_CONTIG(w);
  const int K = a.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "gemm: K mismatch");
  const int M = a.numel() / K;
  const void* bp = nullptr;
  const void* rp = nullptr;
  if (bias.has_value()) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N, "bias size"); bp = bias->data_ptr(); }
  if (residual.has_value()) { CHECK_BF16(*residual); CHECK_CONTIG(*residual); rp = residual->data_ptr(); }
  TORCH_CHECK(epi != 4 || N % 128 == 0, "gemm: the SwiGLU epilogue needs 8-interleaved gate|up rows, N % 128");
  auto sizes = a.sizes().vec();
  sizes.back() = epi == 4 ? N / 2 : N;   // 4: SwiGLU over 8-interleaved gate|up -> [.., N / 2]
  c10::DeviceGuard g(a.device());
  auto out = at::empty(sizes, a.options());
  CHECK_RC(docqa_gemm(a.data_ptr(), w.data_ptr(), bp, rp, out.data_ptr(), M, N, K, (int)epi, stream()), "gemm");
  return out;
}

// skinny decode projection Y = X . W^T for M <= 128 rows (splits = 0: auto split-K)
// decode gate|up projection with fused SwiGLU: x [M, K], w [2I, K] (8-interleaved) -> [M, I]
at::Tensor dgemm_glu(const at::Tensor& x, const at::Tensor& w) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && N % 16 == 0, "dgemm_glu: shape mismatch");
  const int M = x.numel() / K;
  TORCH_CHECK(M <= 256, "dgemm_glu: at most 256 rows");
  auto sizes = x.sizes().vec();
  sizes.back() = N / 2;
  c10::DeviceGuard g(x.device());
  auto out = at::empty(sizes, x.options());
  if (M > 128) {   // past the skinny kernel's rows: the mid-M kernel's fused SwiGLU
    CHECK_RC(docqa_mgemm_glu(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, 0, stream()), "dgemm_glu");
    return out;
  }
  CHECK_RC(docqa_dgemm_glu(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, stream()), "dgemm_glu");
  return out;
}

// split-K partial slabs only: [S, M, N] fp32 (S >= 1), combine fused into the consumer
at::Tensor dgemm_partial(const at::Tensor& x, const at::Tensor& w, int64_t splits, int64_t tile_rows) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "dgemm_partial: K mismatch");
  const int M = x.numel() / K;
  TORCH_CHECK(M <= 256 && splits >= 1, "dgemm_partial: at most 256 rows, splits >= 1");
  c10::DeviceGuard g(x.device());
  auto part = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
  if (M > 192) {   // past the skinny kernel's rows: the mid-M kernel's split-K slabs
    CHECK_RC(docqa_mgemm(x.data_ptr(), w.data_ptr(), nullptr, part.data_ptr<float>(), M, N, K, (int)splits, 0,
                         stream()), "dgemm_partial");
    return part;
  }
  CHECK_RC(docqa_dgemm_partial(x.data_ptr(), w.data_ptr(), part.data_ptr<float>(), M, N, K, (int)splits,
                               (int)tile_rows, stream()), "dgemm_partial");
  return part;
}

// few-row split-K projection + residual add + RMSNorm in one launch (last-arriver epilogue):
// residual <- residual + bf16(x w^T); returns rmsnorm(residual) * gamma
at::Tensor dgemm_add_rmsnorm(const at::Tensor& x, const at::Tensor& w, int64_t splits, at::Tensor residual,
                             const at::Tensor& gamma, double eps, at::Tensor tick) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_BF16(residual); CHECK_CONTIG(residual); CHECK_BF16(gamma); CHECK_I32(tick); CHECK_GPU(tick);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "dgemm_add_rmsnorm: K mismatch");
  const int M = x.numel() / K;
  TORCH_CHECK(residual.numel() == (int64_t)M * N && gamma.numel() == N && tick.numel() >= 1,
              "dgemm_add_rmsnorm: residual [M, N], gamma [N], one ticket word");
  c10::DeviceGuard g(x.device());
  auto part = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
  auto out = at::empty_like(residual);
  CHECK_RC(docqa_dgemm_add_rmsnorm(x.data_ptr(), w.data_ptr(), part.data_ptr<float>(), M, N, K, (int)splits,
                                   residual.data_ptr(), gamma.data_ptr(), out.data_ptr(), (float)eps,
                                   tick.data_ptr<int>(), stream()), "dgemm_add_rmsnorm");
  return out;
}

// batch-1 projection whose input row is built in-kernel from the previous projection's slabs:
// x = rmsnorm(res_in + bf16(sum Pin)) * gamma, res_out <- res_in + bf16(sum Pin)
static void check_xn(const at::Tensor& Pin, const at::Tensor& res_in, const at::Tensor& res_out,
                     const at::Tensor& gamma, const at::Tensor& w) {
  CHECK_GPU(Pin); CHECK_CONTIG(Pin); CHECK_BF16(res_in); CHECK_BF16(res_out); CHECK_BF16(gamma); CHECK_BF16(w);
  CHECK_CONTIG(res_in); CHECK_CONTIG(res_out); CHECK_CONTIG(w);
  TORCH_CHECK(Pin.scalar_type() == at::kFloat && Pin.dim() == 3 && Pin.size(1) == 1, "xn: slabs fp32 [S, 1, K]");
  const int64_t K = w.size(1);
  TORCH_CHECK(Pin.size(2) == K && res_in.numel() == K && res_out.numel() == K && gamma.numel() == K,
              "xn: one row of K");
  TORCH_CHECK(res_in.data_ptr() != res_out.data_ptr(), "xn: res_out must be a second buffer");
}

at::Tensor dgemm_partial_xn(const at::Tensor& Pin, const at::Tensor& res_in, at::Tensor res_out,
                            const at::Tensor& gamma, double eps, const at::Tensor& w, int64_t splits) {
  check_xn(Pin, res_in, res_out, gamma, w);
  const int N = w.size(0), K = w.size(1);
  c10::DeviceGuard g(Pin.device());
  auto part = at::empty({splits, 1, N}, Pin.options());
  CHECK_RC(docqa_dgemm_partial_xn(Pin.data_ptr<float>(), Pin.size(0), res_in.data_ptr(), res_out.data_ptr(),
                                  gamma.data_ptr(), (float)eps, w.data_ptr(), part.data_ptr<float>(), N, K,
                                  (int)splits, stream()), "dgemm_partial_xn");
  return part;
}

at::Tensor dgemm_glu_xn(const at::Tensor& Pin, const at::Tensor& res_in, at::Tensor res_out, const at::Tensor& gamma,
                        double eps, const at::Tensor& w) {
  check_xn(Pin, res_in, res_out, gamma, w);
  const int N = w.size(0), K = w.size(1);
  c10::DeviceGuard g(Pin.device());
  auto out = at::empty({1, N / 2}, res_in.options());
  CHECK_RC(docqa_dgemm_glu_xn(Pin.data_ptr<float>(), Pin.size(0), res_in.data_ptr(), res_out.data_ptr(),
                              gamma.data_ptr(), (float)eps, w.data_ptr(), out.data_ptr(), N, K, stream()),
           "dgemm_glu_xn");
  return out;
}

// batch-1 GEMV (dgemm.hip gemv_kernel: weight rows streamed straight into VGPRs): fp32
// slabs [S, 1, N] of x . w^T (rows weight rows per workgroup), or with glu the SwiGLU row
// [1, N / 2] of an 8-interleaved gate|up weight
at::Tensor gemv(const at::Tensor& x, const at::Tensor& w, int64_t splits, int64_t rows, bool glu) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w); CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && x.numel() == K, "gemv: one row, K mismatch");
  c10::DeviceGuard g(x.device());
  at::Tensor out = glu ? at::empty({1, N / 2}, x.options()) : at::empty({splits, 1, N}, x.options().dtype(at::kFloat));
  CHECK_RC(docqa_gemv(x.data_ptr(), w.data_ptr(), glu ? out.data_ptr() : nullptr,
                      glu ? nullptr : out.data_ptr<float>(), N, K, (int)splits, (int)rows, glu ? 1 : 0, nullptr, 0,
                      nullptr, nullptr, nullptr, 0.f, stream()), "gemv");
  return out;
}

// batch-1 GEMV whose input row is rmsnorm(res_in + bf16(sum Pin)) * gamma built in LDS
// (XNormIn); res_out <- res_in + bf16(sum Pin)
at::Tensor gemv_xn(const at::Tensor& Pin, const at::Tensor& res_in, at::Tensor res_out, const at::Tensor& gamma,
                   double eps, const at::Tensor& w, int64_t splits, int64_t rows, bool glu) {
  check_xn(Pin, res_in, res_out, gamma, w);
  const int N = w.size(0), K = w.size(1);
  c10::DeviceGuard g(Pin.device());
  at::Tensor out = glu ? at::empty({1, N / 2}, res_in.options()) : at::empty({splits, 1, N}, Pin.options());
  CHECK_RC(docqa_gemv(nullptr, w.data_ptr(), glu ? out.data_ptr() : nullptr, glu ? nullptr : out.data_ptr<float>(),
                      N, K, (int)splits, (int)rows, glu ? 1 : 0, Pin.data_ptr<float>(), Pin.size(0), res_in.data_ptr(),
                      res_out.data_ptr(), gamma.data_ptr(), (float)eps, stream()), "gemv_xn");
  return out;
}

at::Tensor dgemm(const at::Tensor& x, const at::Tensor& w, int64_t splits) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "dgemm: K mismatch");
  const int M = x.numel() / K;
  TORCH_CHECK(M <= 256, "dgemm: at most 256 rows");
  const int S = splits > 0 ? (int)splits : docqa_dgemm_splits(N, K);
  auto sizes = x.sizes().vec();
  sizes.back() = N;
  c10::DeviceGuard g(x.device());
  auto out = at::empty(sizes, x.options());
  if (M > 192) {   // past the skinny kernel's rows: the mid-M kernel, bf16 out
    CHECK_RC(docqa_mgemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), nullptr, M, N, K, 1, 0, stream()), "dgemm");
    return out;
  }
  at::Tensor part;
  if (S > 1) part = at::empty({S, M, N}, x.options().dtype(at::kFloat));
  CHECK_RC(docqa_dgemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), S > 1 ? part.data_ptr<float>() : nullptr,
                       M, N, K, S, stream()), "dgemm");
  return out;
}

// mid-M decode GEMM (193..512 rows): splits == 1 -> bf16 [.., N]; splits > 1 -> fp32
// split-K slabs [S, M, N] for the fused consumers (add_rmsnorm_splitk / rope_cache_splitk)
at::Tensor mgemm(const at::Tensor& x, const at::Tensor& w, int64_t splits, int64_t cfg) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "mgemm: K mismatch");
  const int M = x.numel() / K;
  TORCH_CHECK(splits >= 1, "mgemm: splits >= 1");
  c10::DeviceGuard g(x.device());
  at::Tensor out;
  if (splits == 1) {
    auto sizes = x.sizes().vec();
    sizes.back() = N;
    out = at::empty(sizes, x.options());
    CHECK_RC(docqa_mgemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), nullptr, M, N, K, 1, (int)cfg, stream()),
             "mgemm");
  } else {
    out = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
    CHECK_RC(docqa_mgemm(x.data_ptr(), w.data_ptr(), nullptr, out.data_ptr<float>(), M, N, K, (int)splits,
                         (int)cfg, stream()), "mgemm");
  }
  return out;
}

// mid-M decode GEMM -> bf16 split-K slabs [S, M, N] (the bf16-slab consumers)
at::Tensor mgemm_slab16(const at::Tensor& x, const at::Tensor& w, int64_t splits, int64_t cfg) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "mgemm_slab16: K mismatch");
  const int M = x.numel() / K;
  TORCH_CHECK(splits >= 1, "mgemm_slab16: splits >= 1");
  c10::DeviceGuard g(x.device());
  auto out = at::empty({splits, M, N}, x.options());
  CHECK_RC(docqa_mgemm_slab16(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, (int)splits, (int)cfg,
                              stream()), "mgemm_slab16");
  return out;
}

// mid-M gate|up projection with fused SwiGLU: x [M, K], w [2I, K] (8-interleaved) -> [M, I]
at::Tensor mgemm_glu(const at::Tensor& x, const at::Tensor& w, int64_t cfg) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && N % 16 == 0, "mgemm_glu: shape mismatch");
  const int M = x.numel() / K;
  auto sizes = x.sizes().vec();
  sizes.back() = N / 2;
  c10::DeviceGuard g(x.device());
  auto out = at::empty(sizes, x.options());
  CHECK_RC(docqa_mgemm_glu(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, (int)cfg, stream()), "mgemm_glu");
  return out;
}

int64_t mgemm_tile_n(int64_t cfg) { return docqa_mgemm_tile_n((int)cfg); }


// layout probe: x [M, K] / w [N, K] views with row strides >= K (stride(1) == 1); glu: the
// SwiGLU epilogue over 8-interleaved gate|up rows -> [M, N / 2]; else splits >= 2 -> fp32
// slabs [S, M, N], splits == 1 -> bf16 [M, N]
at::Tensor mgemm_ld(const at::Tensor& x, const at::Tensor& w, int64_t splits, int64_t cfg, bool glu) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.stride(1) == 1 && w.stride(1) == 1, "mgemm_ld: 2-D row views");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && splits >= 1, "mgemm_ld: shape");
  c10::DeviceGuard g(x.device());
  at::Tensor out;
  if (glu) {
    out = at::empty({M, N / 2}, x.options());
    CHECK_RC(docqa_mgemm_ld(x.data_ptr(), (int)x.stride(0), w.data_ptr(), (int)w.stride(0), out.data_ptr(), nullptr,
                            M, N, K, 1, (int)cfg, 1, stream()), "mgemm_ld");
  } else if (splits == 1) {
    out = at::empty({M, N}, x.options());
    CHECK_RC(docqa_mgemm_ld(x.data_ptr(), (int)x.stride(0), w.data_ptr(), (int)w.stride(0), out.data_ptr(), nullptr,
                            M, N, K, 1, (int)cfg, 0, stream()), "mgemm_ld");
  } else {
    out = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
    CHECK_RC(docqa_mgemm_ld(x.data_ptr(), (int)x.stride(0), w.data_ptr(), (int)w.stride(0), nullptr,
                            out.data_ptr<float>(), M, N, K, (int)splits, (int)cfg, 0, stream()), "mgemm_ld");
  }
  return out;
}

// LM head + greedy pick: argmax over the first n_valid columns of bf16(x . w^T) -> int64 [M]
at::Tensor mgemm_argmax(const at::Tensor& x, const at::Tensor& w, int64_t n_valid, int64_t cfg) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0), bn = docqa_mgemm_tile_n((int)cfg);   // weight-tile rows
  TORCH_CHECK(w.size(1) == K && bn > 0 && N % bn == 0, "mgemm_argmax: shape mismatch");
  const int M = x.numel() / K;
  c10::DeviceGuard g(x.device());
  auto out = at::empty({M}, x.options().dtype(at::kLong));
  auto ws_v = at::empty({M, N / bn}, x.options().dtype(at::kFloat));
  auto ws_i = at::empty({M, N / bn}, x.options().dtype(at::kInt));
  CHECK_RC(docqa_mgemm_argmax(x.data_ptr(), w.data_ptr(), out.data_ptr<int64_t>(), nullptr, ws_v.data_ptr<float>(),
                              ws_i.data_ptr<int>(), M, N, K, (int)n_valid, (int)cfg, stream()), "mgemm_argmax");
  return out;
}

// the same with the picked logit per row (vocab-parallel LM head: the TP group compares them)
std::tuple<at::Tensor, at::Tensor> mgemm_argmax_val(const at::Tensor& x, const at::Tensor& w, int64_t n_valid,
                                                    int64_t cfg) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0), bn = docqa_mgemm_tile_n((int)cfg);
  TORCH_CHECK(w.size(1) == K && bn > 0 && N % bn == 0, "mgemm_argmax_val: shape mismatch");
  const int M = x.numel() / K;
  c10::DeviceGuard g(x.device());
  auto out = at::empty({M}, x.options().dtype(at::kLong));
  auto outv = at::empty({M}, x.options().dtype(at::kFloat));
  auto ws_v = at::empty({M, N / bn}, x.options().dtype(at::kFloat));
  auto ws_i = at::empty({M, N / bn}, x.options().dtype(at::kInt));
  CHECK_RC(docqa_mgemm_argmax(x.data_ptr(), w.data_ptr(), out.data_ptr<int64_t>(), outv.data_ptr<float>(),
                              ws_v.data_ptr<float>(), ws_i.data_ptr<int>(), M, N, K, (int)n_valid, (int)cfg,
                              stream()), "mgemm_argmax_val");
  return {out, outv};
}

// LM head + greedy pick at <= 192 rows on the skinny decode GEMM (dgemm.hip EPI_ARGMAX)
std::tuple<at::Tensor, at::Tensor> dgemm_argmax_val(const at::Tensor& x, const at::Tensor& w, int64_t n_valid) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && N % 64 == 0 && K % 512 == 0, "dgemm_argmax: N % 64, K % 512");
  const int M = x.numel() / K;
  TORCH_CHECK(M <= 192, "dgemm_argmax: at most 192 rows");
  c10::DeviceGuard g(x.device());
  auto out = at::empty({M}, x.options().dtype(at::kLong));
  auto outv = at::empty({M}, x.options().dtype(at::kFloat));
  auto ws_v = at::empty({M, N / 64}, x.options().dtype(at::kFloat));
  auto ws_i = at::empty({M, N / 64}, x.options().dtype(at::kInt));
  CHECK_RC(docqa_dgemm_argmax(x.data_ptr(), w.data_ptr(), out.data_ptr<int64_t>(), outv.data_ptr<float>(),
                              ws_v.data_ptr<float>(), ws_i.data_ptr<int>(), M, N, K, (int)n_valid, stream()),
           "dgemm_argmax");
  return {out, outv};
}

// batch-1 LM head + greedy pick on the register-streaming GEMV (dgemm.hip EPI_ARGMAX)
std::tuple<at::Tensor, at::Tensor> gemv_argmax_val(const at::Tensor& x, const at::Tensor& w, int64_t n_valid) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(x.numel() == K && w.size(1) == K, "gemv_argmax: one row");
  TORCH_CHECK(N % 16 == 0 && K % 2048 == 0 && K / 2048 <= 2, "gemv_argmax: N % 16, K 2048 or 4096");
  c10::DeviceGuard g(x.device());
  auto out = at::empty({1}, x.options().dtype(at::kLong));
  auto outv = at::empty({1}, x.options().dtype(at::kFloat));
  auto ws_v = at::empty({N / 16}, x.options().dtype(at::kFloat));
  auto ws_i = at::empty({N / 16}, x.options().dtype(at::kInt));
  CHECK_RC(docqa_gemv_argmax(x.data_ptr(), w.data_ptr(), out.data_ptr<int64_t>(), outv.data_ptr<float>(),
                             ws_v.data_ptr<float>(), ws_i.data_ptr<int>(), N, K, (int)n_valid, stream()),
           "gemv_argmax");
  return {out, outv};
}

// prefill GEMM (pgemm.hip, 256 x 256 tiles): epi 0 -> x . w^T bf16 [.., N]; epi 1 -> fused
// SwiGLU over 8-interleaved gate|up rows -> [.., N / 2]
at::Tensor pgemm(const at::Tensor& x, const at::Tensor& w, int64_t epi) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K, "pgemm: K mismatch");
  TORCH_CHECK(epi == 0 || epi == 1, "pgemm: epi must be 0 (bf16) or 1 (SwiGLU)");
  const int M = x.numel() / K;
  TORCH_CHECK(M == 0 || docqa_pgemm_ok(M, N, K), "pgemm: unsupported shape M=", M, " N=", N, " K=", K,
              " (N % 256, K % 128, 32-bit row offsets)");
  auto sizes = x.sizes().vec();
  sizes.back() = epi == 1 ? N / 2 : N;
  c10::DeviceGuard g(x.device());
  auto out = at::empty(sizes, x.options());
  CHECK_RC(docqa_pgemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), nullptr, M, N, K, 1, (int)epi, stream()), "pgemm");
  return out;
}

// split-K fp32 slabs [S, M, N] of x . w^T on the 256 x 256 kernel (decode-sized M)
at::Tensor pgemm_partial(const at::Tensor& x, const at::Tensor& w, int64_t splits) {
  CHECK_GPU(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  CHECK_ALIGN16(x); CHECK_ALIGN16(w);
  const int K = x.size(-1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && splits >= 1 && K % (splits * 128) == 0, "pgemm_partial: shape / splits");
  const int M = x.numel() / K;
  TORCH_CHECK(M == 0 || docqa_pgemm_ok(M, N, K), "pgemm_partial: unsupported shape");
  c10::DeviceGuard g(x.device());
  auto out = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
  CHECK_RC(docqa_pgemm(x.data_ptr(), w.data_ptr(), nullptr, out.data_ptr<float>(), M, N, K, (int)splits, 2,
                       stream()), "pgemm_partial");
  return out;
}

int64_t group_persist_bins(int64_t cap, int64_t Hkv) { return docqa_group_persist_bins((int)cap, (int)Hkv); }

// diagnostics: per-workgroup timeline of the grouped decode kernel into buf (int64
// [>= workgroups x 8], see attn_decode.hip g_group_trace); None turns it off
void set_decode_trace(const c10::optional<at::Tensor>& buf) {
  long long* p = nullptr;
  if (buf.has_value()) {
    CHECK_GPU(*buf); CHECK_CONTIG(*buf);
    TORCH_CHECK(buf->scalar_type() == at::kLong, "set_decode_trace: int64 buffer");
    p = (long long*)buf->data_ptr<int64_t>();
  }
  CHECK_RC(docqa_set_decode_trace(p), "set_decode_trace");
}

// grouped decode kernel choice for split plans: 1 = wave-parallel, 0 = cooperative, -1 =
// query; returns the previous setting
int64_t set_group_wave(int64_t on) { return docqa_set_group_wave((int)on); }

bool pgemm_ok(int64_t M, int64_t N, int64_t K) { return docqa_pgemm_ok((int)M, (int)N, (int)K); }

std::tuple<at::Tensor, at::Tensor> knn(const at::Tensor& xb, const at::Tensor& xb_norms,
                                       const at::Tensor& xq, int64_t k, bool inner_product,
                                       int64_t id_offset) {
  CHECK_GPU(xb); CHECK_CONTIG(xb); CHECK_CONTIG(xq);
  TORCH_CHECK(xq.scalar_type() == at::kFloat, "queries must be fp32");
  const bool bf = xb.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || xb.scalar_type() == at::kFloat, "database must be fp32 or bf16");
  TORCH_CHECK(xb.size(1) == xq.size(1), "dimension mismatch");
  TORCH_CHECK(k >= 1 && docqa_knn_kpad(k) > 0, "k must be in [1, 64]");
  const int N = xb.size(0), d = xb.size(1), nq = xq.size(0);
  c10::DeviceGuard g(xb.device());
  auto out_d = at::empty({nq, k}, xq.options());
  auto out_i = at::empty({nq, k}, xq.options().dtype(at::kLong));
  if (N == 0 || nq == 0) {
    out_d.fill_(inner_product ? -3.4028234663852886e38 : 3.4028234663852886e38);
    out_i.fill_(-1);
    return {out_d, out_i};
  }
  const int nblk = docqa_knn_workspace_blocks(N);
  const int kp = docqa_knn_kpad(k);
  auto ws_d = at::empty({nq, nblk, kp}, xq.options());
  auto ws_i = at::empty({nq, nblk, kp}, xq.options().dtype(at::kInt));
  const float* norms = inner_product ? nullptr : xb_norms.data_ptr<float>();
  CHECK_RC(docqa_knn(xb.data_ptr(), norms, N, d, bf ? 1 : 0, xq.data_ptr<float>(), nq, k,
                     inner_product ? 1 : 0, ws_d.data_ptr<float>(), ws_i.data_ptr<int>(), nblk,
                     out_d.data_ptr<float>(), out_i.data_ptr<int64_t>(), id_offset, stream()), "knn");
  return {out_d, out_i};
}

// IVF coarse quantizer, wide probes: int64 [nq, nprobe] nearest centroids (ascending, ties
// to the lower id) for nprobe <= 512
// exact fp32 x @ w^T on the coarse quantizer's MFMA tiles (the IVF-PQ query pre-rotation)
at::Tensor fp32_gemm_nt(const at::Tensor& x, const at::Tensor& w) {
  CHECK_GPU(x); CHECK_GPU(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.scalar_type() == at::kFloat && w.scalar_type() == at::kFloat && x.dim() == 2 && w.dim() == 2 &&
              x.size(1) == w.size(1), "fp32_gemm_nt: fp32 [M, K] x [N, K]");
  TORCH_CHECK(x.size(1) % 8 == 0 && (size_t)32 * x.size(1) * 4 <= 160 * 1024, "fp32_gemm_nt: K % 8 == 0, K <= 1280");
  c10::DeviceGuard g(x.device());
  auto out = at::empty({x.size(0), w.size(0)}, x.options());
  CHECK_RC(docqa_fp32_gemm_nt(x.data_ptr<float>(), x.size(0), x.size(1), w.data_ptr<float>(), w.size(0),
                              out.data_ptr<float>(), stream()), "fp32_gemm_nt");
  return out;
}

at::Tensor coarse_probes(const at::Tensor& xq, const at::Tensor& cent, const at::Tensor& cnorm, int64_t nprobe) {
  CHECK_GPU(xq); CHECK_GPU(cent); CHECK_GPU(cnorm);
  CHECK_CONTIG(xq); CHECK_CONTIG(cent); CHECK_CONTIG(cnorm);
  TORCH_CHECK(xq.scalar_type() == at::kFloat && cent.scalar_type() == at::kFloat && cnorm.scalar_type() == at::kFloat,
              "coarse_probes: fp32 operands");
  TORCH_CHECK(xq.dim() == 2 && cent.dim() == 2 && xq.size(1) == cent.size(1) && cnorm.numel() == cent.size(0),
              "coarse_probes: shape mismatch");
  const int nq = xq.size(0), d = xq.size(1), nlist = cent.size(0);
  TORCH_CHECK(nprobe >= 1 && nprobe <= 512 && nprobe <= nlist, "coarse_probes: 1 <= nprobe <= min(512, nlist)");
  TORCH_CHECK(d % 8 == 0 && (size_t)32 * d * 4 <= 160 * 1024, "coarse_probes: d % 8 == 0, d <= 1280");
  c10::DeviceGuard g(xq.device());
  auto ws = at::empty({nq, nlist}, xq.options());
  auto probes = at::empty({nq, nprobe}, xq.options().dtype(at::kLong));
  CHECK_RC(docqa_coarse_probes(cent.data_ptr<float>(), cnorm.data_ptr<float>(), nlist, d, xq.data_ptr<float>(), nq,
                               (int)nprobe, ws.data_ptr<float>(), probes.data_ptr<int64_t>(), stream()),
           "coarse_probes");
  return probes;
}

at::Tensor pool_l2(const at::Tensor& h, const at::Tensor& cu_seqlens, bool mean, bool normalize) {
  CHECK_GPU(h); CHECK_BF16(h); CHECK_CONTIG(h); CHECK_I32(cu_seqlens);
  const int H = h.size(-1);
  const int B = cu_seqlens.numel() - 1;
  c10::DeviceGuard g(h.device());
  auto out = at::empty({B, H}, h.options().dtype(at::kFloat));
  CHECK_RC(docqa_pool_l2(h.data_ptr(), cu_seqlens.data_ptr<int>(), B, H, mean ? 1 : 0,
                         normalize ? 1 : 0, out.data_ptr<float>(), stream()), "pool_l2");
  return out;
}

std::tuple<at::Tensor, at::Tensor> ivfpq_search(const at::Tensor& xq, const at::Tensor& centroids,
                                                const at::Tensor& pq, const at::Tensor& codes,
                                                const at::Tensor& ids, const at::Tensor& list_off,
                                                const at::Tensor& probes, int64_t k) {
  CHECK_GPU(xq); CHECK_CONTIG(xq); CHECK_CONTIG(centroids); CHECK_CONTIG(pq); CHECK_CONTIG(codes);
  CHECK_CONTIG(probes);
  TORCH_CHECK(xq.scalar_type() == at::kFloat && centroids.scalar_type() == at::kFloat &&
              pq.scalar_type() == at::kFloat, "ivfpq: fp32 queries / centroids / codebook");
  TORCH_CHECK(codes.scalar_type() == at::kByte, "codes must be uint8");
  TORCH_CHECK(ids.scalar_type() == at::kLong && list_off.scalar_type() == at::kLong &&
              probes.scalar_type() == at::kLong, "ids / list offsets / probes must be int64");
  const int nq = xq.size(0), d = xq.size(1), nprobe = probes.size(1), M = pq.size(0);
  TORCH_CHECK(pq.size(1) == 256 && pq.size(2) * M == d, "pq codebook must be [M, 256, d/M]");
  TORCH_CHECK(codes.size(1) == M, "codes must be [N, M]");
  TORCH_CHECK(k >= 1 && k <= 64, "k must be in [1, 64]");
  const int kp = k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64;
  c10::DeviceGuard g(xq.device());
  auto out_d = at::empty({nq, k}, xq.options());
  auto out_i = at::empty({nq, k}, xq.options().dtype(at::kLong));
  auto ws_d = at::empty({nq, nprobe, kp}, xq.options());
  auto ws_i = at::empty({nq, nprobe, kp}, xq.options().dtype(at::kInt));
  CHECK_RC(docqa_ivfpq_search(xq.data_ptr<float>(), centroids.data_ptr<float>(), pq.data_ptr<float>(),
                              codes.data_ptr<uint8_t>(), ids.data_ptr<int64_t>(),
                              list_off.data_ptr<int64_t>(), probes.data_ptr<int64_t>(), nq, nprobe, d,
                              M, k, ws_d.data_ptr<float>(), ws_i.data_ptr<int>(),
                              out_d.data_ptr<float>(), out_i.data_ptr<int64_t>(), stream()), "ivfpq_search");
  return {out_d, out_i};
}

std::tuple<at::Tensor, at::Tensor> ivfpq_search_pt(const at::Tensor& xq, const at::Tensor& centroids,
                                                   const at::Tensor& pq, const at::Tensor& codes,
                                                   const at::Tensor& norms, const at::Tensor& ids,
                                                   const at::Tensor& list_off, const at::Tensor& probes, int64_t k,
                                                   int64_t pc) {
  CHECK_GPU(xq); CHECK_CONTIG(xq); CHECK_CONTIG(centroids); CHECK_CONTIG(pq); CHECK_CONTIG(codes);
  CHECK_CONTIG(probes); CHECK_CONTIG(norms); CHECK_CONTIG(ids); CHECK_CONTIG(list_off);
  TORCH_CHECK(xq.scalar_type() == at::kFloat && centroids.scalar_type() == at::kFloat &&
              pq.scalar_type() == at::kFloat && norms.scalar_type() == at::kFloat,
              "ivfpq_pt: fp32 queries / centroids / codebook / norms");
  TORCH_CHECK(codes.scalar_type() == at::kByte, "codes must be uint8");
  TORCH_CHECK(ids.scalar_type() == at::kLong && list_off.scalar_type() == at::kLong &&
              probes.scalar_type() == at::kLong, "ids / list offsets / probes must be int64");
  const int nq = xq.size(0), d = xq.size(1), nprobe = probes.size(1), M = pq.size(0);
  TORCH_CHECK(pq.size(1) == 256 && pq.size(2) * M == d, "pq codebook must be [M, 256, d/M]");
  TORCH_CHECK(codes.size(1) == M && norms.size(0) == codes.size(0) && ids.size(0) == codes.size(0),
              "codes [N, M], norms [N], ids [N]");
  TORCH_CHECK(centroids.size(1) == d && list_off.size(0) == centroids.size(0) + 1, "centroids / list offsets");
  TORCH_CHECK(probes.size(0) == nq, "probes must be [nq, nprobe]");
  TORCH_CHECK(M % 4 == 0 && (size_t)M * 512 + 1024 * 8 + 272 * 4 <= 160 * 1024, "ivfpq_pt: M % 4 == 0, M <= 300");
  TORCH_CHECK(k >= 1 && k <= 64, "k must be in [1, 64]");
  TORCH_CHECK(pc >= 1, "probes per workgroup must be >= 1");
  const int kp = k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64;
  const int nchunk = (nprobe + (int)pc - 1) / (int)pc;
  c10::DeviceGuard g(xq.device());
  auto out_d = at::empty({nq, k}, xq.options());
  auto out_i = at::empty({nq, k}, xq.options().dtype(at::kLong));
  auto lut = at::empty({nq, M, 256}, xq.options().dtype(at::kHalf));
  auto base = at::empty({nq, nprobe}, xq.options());
  auto ws_d = at::empty({nq, nchunk, kp}, xq.options());
  auto ws_i = at::empty({nq, nchunk, kp}, xq.options().dtype(at::kInt));
  CHECK_RC(docqa_ivfpq_search_pt(xq.data_ptr<float>(), centroids.data_ptr<float>(), pq.data_ptr<float>(),
                                 codes.data_ptr<uint8_t>(), norms.data_ptr<float>(), ids.data_ptr<int64_t>(),
                                 list_off.data_ptr<int64_t>(), probes.data_ptr<int64_t>(), nq, nprobe, d, M, k,
                                 (int)pc, lut.data_ptr(), base.data_ptr<float>(), ws_d.data_ptr<float>(),
                                 ws_i.data_ptr<int>(), out_d.data_ptr<float>(), out_i.data_ptr<int64_t>(), stream()),
           "ivfpq_search_pt");
  return {out_d, out_i};
}

std::tuple<at::Tensor, at::Tensor> refine_flat(const at::Tensor& xb, const at::Tensor& xq, const at::Tensor& cand,
                                               int64_t k, bool ip) {
  CHECK_GPU(xb); CHECK_CONTIG(xb); CHECK_CONTIG(xq); CHECK_CONTIG(cand);
  TORCH_CHECK(xb.scalar_type() == at::kFloat || xb.scalar_type() == at::kBFloat16, "refine: fp32 / bf16 vectors");
  TORCH_CHECK(xq.scalar_type() == at::kFloat && cand.scalar_type() == at::kLong, "refine: fp32 queries, int64 ids");
  TORCH_CHECK(xb.dim() == 2 && xq.dim() == 2 && xq.size(1) == xb.size(1) && cand.size(0) == xq.size(0),
              "refine: xb [N, d], xq [nq, d], cand [nq, kc]");
  TORCH_CHECK(cand.size(1) >= 1 && cand.size(1) <= 64 && k >= 1, "refine: 1..64 candidates per query");
  const int nq = xq.size(0), d = xq.size(1);
  c10::DeviceGuard g(xq.device());
  auto out_d = at::empty({nq, k}, xq.options());
  auto out_i = at::empty({nq, k}, xq.options().dtype(at::kLong));
  CHECK_RC(docqa_refine_flat(xb.data_ptr(), xb.scalar_type() == at::kBFloat16 ? 1 : 0, xb.size(0),
                             xq.data_ptr<float>(), cand.data_ptr<int64_t>(), nq, cand.size(1), d, k, ip ? 1 : 0,
                             out_d.data_ptr<float>(), out_i.data_ptr<int64_t>(), stream()),
           "refine_flat");
  return {out_d, out_i};
}

at::Tensor pq_encode(const at::Tensor& x, const at::Tensor& centroids, const at::Tensor& assign,
                     const at::Tensor& pq) {
  CHECK_GPU(x); CHECK_CONTIG(x); CHECK_CONTIG(centroids); CHECK_CONTIG(pq); CHECK_CONTIG(assign);
  TORCH_CHECK(assign.scalar_type() == at::kLong, "assign must be int64");
  const int n = x.size(0), d = x.size(1), M = pq.size(0);
  c10::DeviceGuard g(x.device());
  auto codes = at::empty({n, M}, x.options().dtype(at::kByte));
  CHECK_RC(docqa_pq_encode(x.data_ptr<float>(), centroids.data_ptr<float>(), assign.data_ptr<int64_t>(),
                           pq.data_ptr<float>(), n, d, M, codes.data_ptr<uint8_t>(), stream()), "pq_encode");
  return codes;
}

// ---- one-shot IPC all-reduce (kernels/allreduce.hip): raw device pointers travel as int64
int64_t ar_region_bytes(int64_t max_elems) { return (int64_t)docqa_ar_region_bytes((size_t)max_elems); }

int64_t ar_alloc(int64_t bytes) {
  void* p = nullptr;
  TORCH_CHECK(docqa_ar_alloc((size_t)bytes, &p) == 0, "ar_alloc: hipExtMallocWithFlags(uncached) failed");
  return (int64_t)(uintptr_t)p;
}

void ar_free(int64_t ptr) { TORCH_CHECK(docqa_ar_free((void*)(uintptr_t)ptr) == 0, "ar_free failed"); }

at::Tensor ar_ipc_handle(int64_t ptr) {
  auto h = at::empty({64}, at::TensorOptions().dtype(at::kByte));
  TORCH_CHECK(docqa_ar_ipc_handle((void*)(uintptr_t)ptr, h.data_ptr()) == 0, "hipIpcGetMemHandle failed");
  return h;
}

int64_t ar_ipc_open(const at::Tensor& handle) {
  TORCH_CHECK(handle.numel() == 64 && handle.scalar_type() == at::kByte && !handle.is_cuda(),
              "ipc handle must be 64 host bytes");
  void* p = nullptr;
  TORCH_CHECK(docqa_ar_ipc_open(handle.contiguous().data_ptr(), &p) == 0, "hipIpcOpenMemHandle failed");
  return (int64_t)(uintptr_t)p;
}

void ar_ipc_close(int64_t ptr) { TORCH_CHECK(docqa_ar_ipc_close((void*)(uintptr_t)ptr) == 0, "ipc close failed"); }

// x: bf16 [M, H] partial (slabs false) or fp32 split-K slabs [S, M, H] (slabs true); residual /
// w given: residual <- residual + allreduce(x) in place and the RMSNorm of it is returned,
// else the all-reduced sum.  mode 0 one-shot, 1 two-shot (kernels/allreduce.hip).
at::Tensor ar_run(const at::Tensor& x, bool slabs, const c10::optional<at::Tensor>& residual,
                  const c10::optional<at::Tensor>& w, double eps, int64_t rank, std::vector<int64_t> regions,
                  int64_t max_elems, int64_t mode, at::Tensor ctr, at::Tensor err, int64_t timeout_us) {
  CHECK_GPU(x); CHECK_CONTIG(x); CHECK_ALIGN16(x);
  TORCH_CHECK(ctr.scalar_type() == at::kInt && ctr.numel() >= 4 && err.scalar_type() == at::kInt,
              "ctr int32[4] / err int32[1]");
  TORCH_CHECK(regions.size() >= 1 && regions.size() <= 8, "1..8 ranks");
  const int H = x.size(-1);
  int S = 0, M;
  if (slabs) {
    TORCH_CHECK(x.scalar_type() == at::kFloat && x.dim() == 3, "slabs must be fp32 [S, M, H]");
    S = x.size(0);
    M = x.size(1);
  } else {
    CHECK_BF16(x);
    M = x.numel() / H;
  }
  const bool fused = residual.has_value();
  TORCH_CHECK(fused == w.has_value(), "residual and w go together");
  if (fused) {
    CHECK_BF16(*residual); CHECK_CONTIG(*residual); CHECK_BF16(*w); CHECK_CONTIG(*w);
    TORCH_CHECK(residual->numel() == (int64_t)M * H && w->numel() == H, "ar_run: residual / w shape");
  }
  std::vector<void*> ptrs;
  for (auto r : regions) ptrs.push_back((void*)(uintptr_t)r);
  c10::DeviceGuard g(x.device());
  at::Tensor out;
  if (mode == 2) {   // all-gather: [nranks, ..x's shape]
    TORCH_CHECK(!slabs && !fused, "ar_run gather takes a bf16 payload only");
    auto sizes = x.sizes().vec();
    sizes.insert(sizes.begin(), (int64_t)regions.size());
    out = at::empty(sizes, x.options());
  } else {
    out = slabs ? at::empty({M, H}, x.options().dtype(at::kBFloat16)) : at::empty_like(x);
  }
  CHECK_RC(docqa_ar_run(x.data_ptr(), S, out.data_ptr(), fused ? residual->data_ptr() : nullptr,
                        fused ? w->data_ptr() : nullptr, (float)eps, M, H, (int)rank, (int)regions.size(),
                        ptrs.data(), (size_t)max_elems, (int)mode, (unsigned*)ctr.data_ptr(),
                        (unsigned*)err.data_ptr(), (long long)timeout_us, stream()), "ar_run");
  return out;
}

}  // namespace

TORCH_LIBRARY(docqa, m) {
  m.def("rmsnorm(Tensor x, Tensor w, float eps) -> Tensor");
  m.def("add_rmsnorm(Tensor x, Tensor(a!) residual, Tensor w, float eps) -> Tensor");
  m.def("layernorm(Tensor x, Tensor? residual, Tensor gamma, Tensor beta, float eps) -> Tensor");
  m.def("rope_cache(Tensor(a!) qkv, Tensor positions, Tensor cos_sin, Tensor? slot_mapping, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, int D) -> ()");
  m.def("silu_mul(Tensor gu, bool interleaved=False) -> Tensor");
  m.def("silu_mul_splitk(Tensor P) -> Tensor");
  m.def("bias_act(Tensor x, Tensor bias, Tensor? residual, bool gelu) -> Tensor");
  m.def("embedding(Tensor ids, Tensor table) -> Tensor");
  m.def("bert_embed_ln(Tensor ids, Tensor pos, Tensor? token_type, Tensor wte, Tensor wpe, "
        "Tensor wtt, Tensor gamma, Tensor beta, float eps) -> Tensor");
  m.def("argmax(Tensor logits) -> Tensor");
  m.def("token_cls_argmax(Tensor h, Tensor w, Tensor bias, int n_valid) -> Tensor");
  m.def("decode_slots(Tensor block_tables, Tensor positions, Tensor valid, int BS) -> Tensor");
  m.def("decode_advance(Tensor nxt, Tensor(a!) out, Tensor(b!) tokens, Tensor(c!) positions, Tensor(d!) context_lens, Tensor valid) -> ()");
  m.def("sample(Tensor logits, Tensor inv_temp, Tensor top_k, Tensor top_p, Tensor u) -> Tensor");
  m.def("paged_decode(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor context_lens, int Hq, int max_context, float scale, Tensor? order=None) -> Tensor");
  m.def("flash_prefill(Tensor qkv, Tensor cu_seqlens, int max_len, int Hq, int Hkv, int D, "
        "float scale, bool causal) -> Tensor");
  m.def("knn(Tensor xb, Tensor xb_norms, Tensor xq, int k, bool inner_product, int id_offset) "
        "-> (Tensor, Tensor)");
  m.def("pool_l2(Tensor h, Tensor cu_seqlens, bool mean, bool normalize) -> Tensor");
  m.def("coarse_probes(Tensor xq, Tensor cent, Tensor cnorm, int nprobe) -> Tensor");
  m.def("fp32_gemm_nt(Tensor x, Tensor w) -> Tensor");
  m.def("ivfpq_search(Tensor xq, Tensor centroids, Tensor pq, Tensor codes, Tensor ids, "
        "Tensor list_off, Tensor probes, int k) -> (Tensor, Tensor)");
  m.def("ivfpq_search_pt(Tensor xq, Tensor centroids, Tensor pq, Tensor codes, Tensor norms, Tensor ids, "
        "Tensor list_off, Tensor probes, int k, int pc) -> (Tensor, Tensor)");
  m.def("refine_flat(Tensor xb, Tensor xq, Tensor cand, int k, bool ip) -> (Tensor, Tensor)");
  m.def("pq_encode(Tensor x, Tensor centroids, Tensor assign, Tensor pq) -> Tensor");
  m.def("gemm(Tensor a, Tensor w, Tensor? bias, Tensor? residual, int epi) -> Tensor");
  m.def("flash_prefill_paged(Tensor qkv, Tensor cu_seqlens, int max_len, int Hq, int Hkv, int D, "
        "float scale, Tensor k_cache, Tensor v_cache, Tensor block_tables, Tensor ctx_start) -> Tensor");
  m.def("dgemm(Tensor x, Tensor w, int splits) -> Tensor");
  m.def("dgemm_partial(Tensor x, Tensor w, int splits, int tile_rows=64) -> Tensor");
  m.def("embed_rmsnorm(Tensor ids, Tensor table, Tensor w, float eps) -> (Tensor, Tensor)");
  m.def("dgemm_partial_xn(Tensor Pin, Tensor res_in, Tensor(a!) res_out, Tensor gamma, float eps, Tensor w, "
        "int splits) -> Tensor");
  m.def("dgemm_glu_xn(Tensor Pin, Tensor res_in, Tensor(a!) res_out, Tensor gamma, float eps, Tensor w) -> Tensor");
  m.def("gemv(Tensor x, Tensor w, int splits=1, int rows=16, bool glu=False) -> Tensor");
  m.def("gemv_xn(Tensor Pin, Tensor res_in, Tensor(a!) res_out, Tensor gamma, float eps, Tensor w, int splits=1, int rows=16, bool glu=False) -> Tensor");
  m.def("dgemm_add_rmsnorm(Tensor x, Tensor w, int splits, Tensor(a!) residual, Tensor gamma, float eps, "
        "Tensor(t!) tick) -> Tensor");
  m.def("dgemm_glu(Tensor x, Tensor w) -> Tensor");
  m.def("mgemm(Tensor x, Tensor w, int splits, int cfg=0) -> Tensor");
  m.def("mgemm_slab16(Tensor x, Tensor w, int splits, int cfg=0) -> Tensor");
  m.def("mgemm_glu(Tensor x, Tensor w, int cfg=0) -> Tensor");
  m.def("mgemm_tile_n(int cfg) -> int", &mgemm_tile_n);
  m.def("mgemm_argmax(Tensor x, Tensor w, int n_valid, int cfg=0) -> Tensor");
  m.def("dgemm_argmax_val(Tensor x, Tensor w, int n_valid) -> (Tensor, Tensor)");
  m.def("gemv_argmax_val(Tensor x, Tensor w, int n_valid) -> (Tensor, Tensor)");
  m.def("pgemm(Tensor x, Tensor w, int epi=0) -> Tensor");
  m.def("pgemm_partial(Tensor x, Tensor w, int splits) -> Tensor");
  m.def("mgemm_argmax_val(Tensor x, Tensor w, int n_valid, int cfg=0) -> (Tensor, Tensor)");
  m.def("pgemm_ok(int M, int N, int K) -> bool", &pgemm_ok);
  m.def("mgemm_ld(Tensor x, Tensor w, int splits, int cfg, bool glu) -> Tensor");
  m.def("group_persist_bins(int cap, int Hkv) -> int", &group_persist_bins);
  m.def("set_decode_trace(Tensor? buf) -> ()", &set_decode_trace);
  m.def("set_group_wave(int on) -> int", &set_group_wave);
  m.def("paged_decode_cascade(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor context_lens, int Hq, int max_context, float scale, Tensor prefix_table, Tensor prefix_len, "
        "int nchunk, Tensor? order=None) -> Tensor");
  m.def("paged_decode_cascade_grouped(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor context_lens, int Hq, float scale, Tensor prefix_table, Tensor prefix_len, int nchunk, "
        "Tensor groups) -> Tensor");
  m.def("kv_copy_rows(Tensor caches, Tensor tab, int num_blocks, int Hkv, int BS, int D) -> ()");
  m.def("paged_decode_cascade_split(Tensor q, Tensor k_cache, Tensor v_cache, Tensor block_tables, "
        "Tensor context_lens, int Hq, float scale, Tensor prefix_table, Tensor prefix_len, int nchunk, "
        "Tensor plan, bool defer=False, Tensor(t!)? tick=None, bool inline_prefix=False) -> Tensor");
  m.def("paged_decode_grouped_fused(Tensor P, Tensor positions, Tensor cos_sin, Tensor slot_mapping, "
        "Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor block_tables, Tensor context_lens, int Hq, float scale, "
        "Tensor prefix_table, Tensor prefix_len, int nchunk, Tensor plan, Tensor(t!)? tick=None) -> Tensor");
  m.def("paged_decode_cascade_rope(Tensor(a!) qkv, Tensor positions, Tensor cos_sin, Tensor slot_mapping, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, Tensor block_tables, Tensor context_lens, int Hq, "
        "int max_context, float scale, Tensor prefix_table, Tensor prefix_len, int nchunk, "
        "Tensor? order=None) -> Tensor");
  m.def("paged_decode_fused(Tensor P, Tensor positions, Tensor cos_sin, Tensor slot_mapping, "
        "Tensor(a!) k_cache, Tensor(b!) v_cache, Tensor block_tables, Tensor context_lens, int Hq, "
        "int max_context, float scale, Tensor? order=None, Tensor(t!)? tick=None) -> Tensor");
  m.def("ar_run(Tensor x, bool slabs, Tensor(r!)? residual, Tensor? w, float eps, int rank, int[] regions, "
        "int max_elems, int mode, Tensor(a!) ctr, Tensor(b!) err, int timeout_us=500000) -> Tensor");
  m.def("ar_region_bytes(int max_elems) -> int", &ar_region_bytes);
  m.def("ar_alloc(int bytes) -> int", &ar_alloc);
  m.def("ar_free(int ptr) -> ()", &ar_free);
  m.def("ar_ipc_handle(int ptr) -> Tensor", &ar_ipc_handle);
  m.def("ar_ipc_open(Tensor handle) -> int", &ar_ipc_open);
  m.def("ar_ipc_close(int ptr) -> ()", &ar_ipc_close);
  m.def("add_rmsnorm_splitk(Tensor P, Tensor(a!) residual, Tensor w, float eps) -> Tensor");
  m.def("rope_cache_splitk(Tensor P, Tensor positions, Tensor cos_sin, Tensor? slot_mapping, "
        "Tensor(b!) k_cache, Tensor(c!) v_cache, int Hq, int Hkv, int D) -> Tensor");
}

TORCH_LIBRARY_IMPL(docqa, CUDA, m) {
  m.impl("rmsnorm", &rmsnorm);
  m.impl("add_rmsnorm", &add_rmsnorm);
  m.impl("layernorm", &layernorm);
  m.impl("rope_cache", &rope_cache);
  m.impl("silu_mul", &silu_mul);
  m.impl("silu_mul_splitk", &silu_mul_splitk);
  m.impl("bias_act", &bias_act);
  m.impl("embedding", &embedding);
  m.impl("bert_embed_ln", &bert_embed_ln);
  m.impl("argmax", &argmax);
  m.impl("token_cls_argmax", &token_cls_argmax);
  m.impl("decode_slots", &decode_slots);
  m.impl("decode_advance", &decode_advance);
  m.impl("sample", &sample);
  m.impl("paged_decode", &paged_decode);
  m.impl("flash_prefill", &flash_prefill);
  m.impl("knn", &knn);
  m.impl("pool_l2", &pool_l2);
  m.impl("ivfpq_search", &ivfpq_search);
  m.impl("ivfpq_search_pt", &ivfpq_search_pt);
  m.impl("refine_flat", &refine_flat);
  m.impl("pq_encode", &pq_encode);
  m.impl("gemm", &gemm);
  m.impl("flash_prefill_paged", &flash_prefill_paged);
  m.impl("dgemm", &dgemm);
  m.impl("dgemm_partial", &dgemm_partial);
  m.impl("embed_rmsnorm", &embed_rmsnorm);
  m.impl("dgemm_partial_xn", &dgemm_partial_xn);
  m.impl("dgemm_glu_xn", &dgemm_glu_xn);
  m.impl("gemv", &gemv);
  m.impl("gemv_xn", &gemv_xn);
  m.impl("dgemm_add_rmsnorm", &dgemm_add_rmsnorm);
  m.impl("dgemm_glu", &dgemm_glu);
  m.impl("mgemm", &mgemm);
  m.impl("mgemm_slab16", &mgemm_slab16);
  m.impl("mgemm_glu", &mgemm_glu);
  m.impl("mgemm_argmax", &mgemm_argmax);
  m.impl("pgemm", &pgemm);
  m.impl("mgemm_ld", &mgemm_ld);
  m.impl("pgemm_partial", &pgemm_partial);
  m.impl("mgemm_argmax_val", &mgemm_argmax_val);
  m.impl("coarse_probes", &coarse_probes);
  m.impl("fp32_gemm_nt", &fp32_gemm_nt);
  m.impl("dgemm_argmax_val", &dgemm_argmax_val);
  m.impl("gemv_argmax_val", &gemv_argmax_val);
  m.impl("paged_decode_fused", &paged_decode_fused);
  m.impl("paged_decode_cascade", &paged_decode_cascade);
  m.impl("paged_decode_cascade_rope", &paged_decode_cascade_rope);
  m.impl("paged_decode_cascade_grouped", &paged_decode_cascade_grouped);
  m.impl("paged_decode_cascade_split", &paged_decode_cascade_split);
  m.impl("paged_decode_grouped_fused", &paged_decode_grouped_fused);
  m.impl("kv_copy_rows", &kv_copy_rows);
  m.impl("ar_run", &ar_run);
  m.impl("add_rmsnorm_splitk", &add_rmsnorm_splitk);
  m.impl("rope_cache_splitk", &rope_cache_splitk);
}
