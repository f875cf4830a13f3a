// docqa_kernels.h -- host launchers of the gfx950 kernels (raw pointers + stream).
// Every launcher returns 0 on success, a negative value for an unsupported shape and a
// hipError_t for a failed launch.  They allocate nothing and never synchronise, so they
// can be captured into HIP graphs (cdna_hip_programming.md Guideline 9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

int docqa_rmsnorm(const void* x, const void* w, void* out, int rows, int H, float eps,
                  hipStream_t s);
int docqa_add_rmsnorm(const void* x, void* residual, const void* w, void* out, int rows, int H,
                      float eps, hipStream_t s);
int docqa_layernorm(const void* x, const void* residual, const void* g, const void* b, void* out,
                    int rows, int H, float eps, hipStream_t s);

int docqa_kv_copy_rows(const uint64_t* caches, int ntensors, const int* tab, int n, int nblocks, int Hkv, int BS,
                       int D, hipStream_t s);
int docqa_rope_cache(void* qkv, const int* positions, const float* cos_sin,
                     const int* slot_mapping, void* k_cache, void* v_cache, int T, int Hq,
                     int Hkv, int D, int row_stride, int BS, hipStream_t s);

int docqa_silu_mul(const void* gu, void* out, int T, int I, int interleaved, hipStream_t s);
int docqa_silu_mul_splitk16(const void* P, void* out, int S, int T, int I, hipStream_t s);
int docqa_silu_mul_splitk(const float* P, void* out, int S, int T, int I, hipStream_t s);
int docqa_bias_act(const void* x, const void* bias, const void* res, void* out, int T, int N,
                   int gelu, hipStream_t s);

int docqa_embedding(const int* ids, const void* table, void* out, int T, int H, int V, hipStream_t s);
int docqa_decode_slots(const int* block_tables, int maxb, const int* positions, const int* valid,
                       int* slots, int B, int BS, hipStream_t s);
int docqa_decode_advance(const int64_t* nxt, int64_t* out, int* tokens, int* positions,
                         int* context_lens, const int* valid, int B, hipStream_t s);
int docqa_bert_embed_ln(const int* ids, const int* pos, const int* tt, const void* wte,
                        const void* wpe, const void* wtt, const void* g, const void* b, void* out,
                        int T, int H, float eps, hipStream_t s);
int docqa_argmax(const void* logits, int rows, int V, int ld, int is_bf16, float* ws_v, int* ws_i,
                 int splits, int64_t* out, hipStream_t s);
int docqa_token_cls_argmax(const void* h, int ldh, const void* w, const void* bias, int n_rows,
                           int n_valid, int T, int H, int64_t* out, hipStream_t s);
int docqa_sample(const float* logits, int rows, int V, int ld, const float* inv_temp,
                 const int* top_k, const float* top_p, const float* u, int64_t* out,
                 hipStream_t s);

int docqa_paged_decode(const void* q, int q_stride, const void* k_cache, const void* v_cache,
                       const int* block_tables, int maxb, const int* context_lens, void* out,
                       int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                       int D, int BS, int max_parts, float scale, const int* order, hipStream_t s);
int docqa_decode_splits(int B, int Hkv, int max_context);
int docqa_paged_decode_cascade(const void* q, int q_stride, void* k_cache, void* v_cache,
                               const int* block_tables, int maxb, const int* context_lens, void* out,
                               int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                               int BS, int max_parts, float scale, const int* prefix_table,
                               const int* plen, int nchunk, float* pacc, float* pml, const int* order,
                               hipStream_t s);
int docqa_paged_decode_cascade_grouped(const void* q, int q_stride, void* k_cache, void* v_cache,
                                       const int* block_tables, int maxb, const int* context_lens,
                                       void* out, int out_stride, int B, int Hq, int Hkv, int BS,
                                       float scale, const int* prefix_table, const int* plen, int nchunk,
                                       float* pacc, float* pml, const int* groups, int ngroups,
                                       hipStream_t s);
int docqa_paged_decode_cascade_split(const void* q, int q_stride, void* k_cache, void* v_cache,
                                     const int* block_tables, int maxb, const int* context_lens,
                                     void* out, int out_stride, int B, int Hq, int Hkv, int BS,
                                     float scale, const int* prefix_table, const int* plen, int nchunk,
                                     float* pacc, float* pml, const int* items, const int* merges, int cap,
                                     float* ws_acc, float* ws_ml, int defer,
                                     hipStream_t s, int* tick = nullptr, int inline_prefix = 0,
                                     const float* fP = nullptr, int fS = 0, const int* positions = nullptr,
                                     const float* cos_sin = nullptr, const int* slot_mapping = nullptr);
int docqa_paged_decode_cascade_persist(const void* q, int q_stride, void* k_cache, void* v_cache,
                                       const int* block_tables, int maxb, const int* context_lens,
                                       void* out, int out_stride, int B, int Hq, int Hkv, int BS,
                                       float scale, const int* prefix_table, const int* plen, int nchunk,
                                       float* pacc, float* pml, const int* items, const int* merges,
                                       const int* bins, int cap, float* ws_acc, float* ws_ml, hipStream_t s);
int docqa_group_persist_bins(int cap, int Hkv);
int docqa_set_decode_trace(long long* buf);
int docqa_set_group_wave(int on);   // -1: query only; returns the previous setting
int docqa_paged_decode_cascade_rope(void* qkv, int q_stride, const int* positions,
                                    const float* cos_sin, const int* slot_mapping, void* k_cache,
                                    void* v_cache, const int* block_tables, int maxb,
                                    const int* context_lens, void* out, int out_stride,
                                    float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv, int BS,
                                    int max_parts, float scale, const int* prefix_table,
                                    const int* plen, int nchunk, float* pacc, float* pml,
                                    const int* order, hipStream_t s);

int docqa_flash_prefill(const void* qkv, int row_stride, const int* cu_seqlens, void* out,
                        int o_stride, int B, int max_len, int Hq, int Hkv, int head_dim,
                        float scale, int causal, hipStream_t s);

int docqa_flash_prefill_paged(const void* qkv, int row_stride, const int* cu_seqlens, void* out,
                              int o_stride, int B, int max_len, int Hq, int Hkv, int head_dim,
                              float scale, const void* k_cache, const void* v_cache,
                              const int* block_tables, int maxb, const int* ctx_start, int BS,
                              hipStream_t s);

int docqa_dgemm_partial(const void* X, const void* W, float* P, int M, int N, int K, int S,
                        int tile_rows, hipStream_t s);
int docqa_add_rmsnorm_splitk(const float* P, int S, void* residual, const void* w, void* out,
                             int rows, int H, float eps, hipStream_t s);
int docqa_rope_cache_splitk(const float* P, int S, void* qkv_out, const int* positions,
                            const float* cos_sin, const int* slot_mapping, void* k_cache,
                            void* v_cache, int T, int Hq, int Hkv, int D, int row_stride, int BS,
                            hipStream_t s);
int docqa_add_rmsnorm_splitk16(const void* P, int S, void* residual, const void* w, void* out,
                               int rows, int H, float eps, hipStream_t s);
int docqa_rope_cache_splitk16(const void* P, int S, void* qkv_out, const int* positions,
                              const float* cos_sin, const int* slot_mapping, void* k_cache,
                              void* v_cache, int T, int Hq, int Hkv, int D, int row_stride, int BS,
                              hipStream_t s);
size_t docqa_ar_region_bytes(size_t max_elems);
int docqa_ar_alloc(size_t bytes, void** ptr);
int docqa_ar_free(void* ptr);
int docqa_ar_ipc_handle(void* ptr, void* handle_out);
int docqa_ar_ipc_open(const void* handle, void** ptr);
int docqa_ar_ipc_close(void* ptr);
int docqa_ar_run(const void* in, int S, void* out, void* residual, const void* w, float eps, int M, int H,
                 int rank, int nranks, void* const* regions, size_t max_elems, int mode, unsigned* ctr,
                 unsigned* err, long long timeout_us, hipStream_t s);
int docqa_paged_decode_fused(const float* P, int S, const int* positions, const float* cos_sin,
                             const int* slot_mapping, void* k_cache, void* v_cache,
                             const int* block_tables, int maxb, const int* context_lens, void* out,
                             int out_stride, float* tmp_out, float* tmp_ml, int B, int Hq, int Hkv,
                             int BS, int max_parts, float scale, const int* order, hipStream_t s,
                             int* tick = nullptr);
int docqa_dgemm_splits(int N, int K);
int docqa_dgemm_glu(const void* X, const void* W, void* Y, int M, int N, int K, hipStream_t s);
int docqa_dgemm_add_rmsnorm(const void* X, const void* W, float* P, int M, int N, int K, int S, void* residual,
                            const void* gamma, void* out, float eps, int* tick, hipStream_t s);
int docqa_dgemm_partial_xn(const float* Pin, int Sin, const void* res_in, void* res_out, const void* gamma,
                           float eps, const void* W, float* P, int N, int K, int S, hipStream_t s);
int docqa_dgemm_glu_xn(const float* Pin, int Sin, const void* res_in, void* res_out, const void* gamma, float eps,
                       const void* W, void* Y, int N, int K, hipStream_t s);
// batch-1 GEMV (dgemm.hip gemv_kernel): epi 0 fp32 slabs P [S, 1, N], epi 1 SwiGLU Y [1, N / 2];
// Pin != null: the input row from the previous projection's slabs (XNormIn)
int docqa_gemv(const void* X, const void* W, void* Y, float* P, int N, int K, int S, int R, int epi,
               const float* Pin, int Sin, const void* res_in, void* res_out, const void* gamma, float eps,
               hipStream_t s);
int docqa_embed_rmsnorm(const int* ids, const void* table, const void* w, void* h, void* x, int T, int H, int V,
                        float eps, hipStream_t s);
int docqa_fp32_gemm_nt(const float* x, int nq, int d, const float* w, int n, float* out, hipStream_t s);
int docqa_gemv_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int N, int K,
                      int n_valid, hipStream_t s);
int docqa_dgemm_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int M,
                       int N, int K, int n_valid, hipStream_t s);
int docqa_dgemm(const void* X, const void* W, void* Y, float* partial, int M, int N, int K, int S,
                hipStream_t s);
int docqa_gemm(const void* A, const void* W, const void* bias, const void* res, void* C, int M,
               int N, int K, int epi, hipStream_t s);
int docqa_mgemm(const void* X, const void* W, void* Y, float* P, int M, int N, int K, int S, int cfg,
                hipStream_t s);
int docqa_mgemm_slab16(const void* X, const void* W, void* Y, int M, int N, int K, int S, int cfg,
                       hipStream_t s);
int docqa_mgemm_glu(const void* X, const void* W, void* Y, int M, int N, int K, int cfg, hipStream_t s);
int docqa_mgemm_argmax(const void* X, const void* W, int64_t* out, float* outv, float* ws_v, int* ws_i, int M,
                       int N, int K, int n_valid, int cfg, hipStream_t s);
int docqa_mgemm_tile_n(int cfg);
int docqa_mgemm_ld(const void* X, int ldx, const void* W, int ldw, void* Y, float* P, int M, int N, int K, int S,
                   int cfg, int glu, hipStream_t s);
// IVF coarse quantizer for wide probes (coarse.hip): nprobe <= 512 nearest centroids per query
int docqa_coarse_probes(const float* cent, const float* cnorm, int nlist, int d, const float* xq, int nq,
                        int nprobe, float* ws, int64_t* probes, hipStream_t s);
bool docqa_pgemm_ok(int M, int N, int K);
int docqa_pgemm(const void* A, const void* W, void* C, float* P, int M, int N, int K, int S, int epi,
                hipStream_t s);
int docqa_knn_workspace_blocks(int N);
int docqa_knn_kpad(int k);
int docqa_knn(const void* xb, const float* norms, int N, int d, int is_bf16, const float* xq,
              int nq, int k, int metric_ip, float* ws_d, int* ws_i, int nblk, float* out_d,
              int64_t* out_i, int64_t id_offset, hipStream_t s);

int docqa_ivfpq_search(const float* xq, const float* centroids, const float* pq,
                       const uint8_t* codes, const int64_t* ids, const int64_t* list_off,
                       const int64_t* probes, int nq, int nprobe, int d, int M, int k,
                       float* ws_d, int* ws_i, float* out_d, int64_t* out_i, hipStream_t s);
// precomputed-table scan: norms [N] = ||c_list + r^||^2; lut_ws >= nq*M*256 halves, base_ws >=
// nq*nprobe floats, ws_d / ws_i >= nq*ceil(nprobe/pc)*kpad (kpad = k rounded up to 8/16/32/64)
int docqa_ivfpq_search_pt(const float* xq, const float* centroids, const float* pq, const uint8_t* codes,
                          const float* norms, const int64_t* ids, const int64_t* list_off, const int64_t* probes,
                          int nq, int nprobe, int d, int M, int k, int pc, void* lut_ws, float* base_ws,
                          float* ws_d, int* ws_i, float* out_d, int64_t* out_i, hipStream_t s);
// exact re-rank of <= 64 candidate ids per query against stored vectors (fp32 or bf16 rows)
int docqa_refine_flat(const void* xb, int xb_bf16, int64_t ntotal, const float* xq, const int64_t* cand, int nq,
                      int kc, int d, int k, int ip, float* out_d, int64_t* out_i, hipStream_t s);
int docqa_pq_encode(const float* x, const float* centroids, const int64_t* assign, const float* pq,
                    int n, int d, int M, uint8_t* codes, hipStream_t s);

int docqa_pool_l2(const void* h, const int* cu, int B, int H, int mean, int normalize, float* out,
                  hipStream_t s);
