// docqa_cascade.h -- shared-prefix ("cascade") decode attention, the pieces both kernels
// need (attn_prefill.hip computes the prefix partials, attn_decode.hip merges them).
//
// Every prompt of a RAG decode batch starts with the same instruction template, and the
// prefix cache maps that template to ONE set of physical KV blocks.  Plain paged decode
// re-reads those blocks once per sequence (B x Lp tokens of K/V per layer); here the
// shared prefix is attended once for all B x Hq query rows -- an MFMA flash kernel over
// the prefix keys, split into `nchunk` key chunks -- and the ring decode kernel attends
// only each sequence's own suffix [Lp, L), merging the chunk partials by log-sum-exp
// before it normalises.  Exactly the same softmax, ~Lp/L fewer K/V bytes per step.
#pragma once

namespace docqa {

constexpr int kCascadeMaxChunks = 16;

struct CascadeIn {        // prefix partials consumed by the decode kernel / merge kernel
  const float* acc;       // [nchunk, B, Hq, D] un-normalised sum p * v
  const float* ml;        // [nchunk, B, Hq, 2] (running max in log2 units, sum p)
  const int* plen;        // device scalar: shared prefix length (multiple of 64); null: none
  int nchunk;
  // dispatch order of the decode workgroups: grid row y serves sequence order[y] (a
  // permutation, longest context first -- LPT -- so the short sequences fill the tail of
  // the last launch round); null: identity.  Not a cascade input, but every decode kernel
  // launch carries this struct.
  const int* order = nullptr;
};

struct CascadeOut {       // prefix partials produced by the MFMA prefix kernel
  float* acc;
  float* ml;
  const int* plen;
  int nchunk;
  int rows;               // B: query rows = decode sequences
  // fused RoPE: the query rows are the library GEMM's unrotated QKV; rotate them on load
  // (null: already rotated)
  const int* positions = nullptr;
  const float* cos_sin = nullptr;
};

// keys per chunk (a multiple of the 64-key tile) and chunks holding >= 1 key
__host__ __device__ inline int cascade_chunk(int Lp, int nchunk) {
  int c = (Lp + nchunk - 1) / nchunk;
  c = (c + 63) / 64 * 64;
  return c < 64 ? 64 : c;
}
__host__ __device__ inline int cascade_parts(int Lp, int nchunk) {
  if (Lp <= 0) return 0;
  const int c = cascade_chunk(Lp, nchunk);
  return (Lp + c - 1) / c;
}

}  // namespace docqa
