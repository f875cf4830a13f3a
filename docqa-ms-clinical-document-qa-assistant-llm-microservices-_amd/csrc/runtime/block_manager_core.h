// block_manager_core.h -- the paged-KV block allocator + content-hashed prefix cache,
// free of torch so the same code is linked into the torch custom class
// (block_manager.cpp) and into the host sanitizer stress test
// (csrc/tests/block_manager_stress.cpp: ThreadSanitizer and ASan/UBSan builds, run by
// tests/test_native_sanitizers.py -- SURVEY.md §5.2 race detection).
//
// * alloc/free/share: O(1) free-list allocator over the HBM-resident KV block pool;
//   refcounts let several sequences share prompt-prefix blocks.
// * prefix cache: every FULL block of a prompt is keyed by a chained 64-bit hash of
//   (parent block hash, the block's token ids).  Cached blocks whose refcount drops to
//   zero stay resident in an LRU list and are evicted only when the free list runs dry.
// Thread-safe (one mutex).
#pragma once

#include <algorithm>
#include <cstdint>
#include <iterator>
#include <list>
#include <mutex>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace docqa_rt {


inline uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
  h *= 0xff51afd7ed558ccdULL;
  return h ^ (h >> 33);
}

class BlockManagerCore {
 public:
  explicit BlockManagerCore(int64_t num_blocks, int64_t block_size)
      : n_(num_blocks), bs_(block_size), ref_(num_blocks, 0), hash_of_(num_blocks, 0),
        cached_(num_blocks, false) {
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back(b);
  }

  int64_t num_free() {
    std::lock_guard<std::mutex> g(mu_);
    return (int64_t)free_.size() + (int64_t)lru_.size();
  }
  int64_t num_blocks() const { return n_; }
  int64_t block_size() const { return bs_; }

  std::vector<int64_t> alloc(int64_t n) {
    std::lock_guard<std::mutex> g(mu_);
    if (n > (int64_t)free_.size() + (int64_t)lru_.size())
      throw std::runtime_error("KV cache exhausted");
    std::vector<int64_t> out;
    out.reserve(n);
    for (int64_t i = 0; i < n; ++i) out.push_back(take_one());
    return out;
  }

  void share(const std::vector<int64_t>& blocks) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto b : blocks) {
      check(b);
      if (ref_[b] == 0 && cached_[b]) lru_erase(b);
      ++ref_[b];
    }
  }

  void free(const std::vector<int64_t>& blocks) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto b : blocks) {
      check(b);
      if (ref_[b] <= 0) throw std::runtime_error("double free of KV block");
      if (--ref_[b] == 0) {
        if (cached_[b]) {
          lru_.push_back(b);
          lru_pos_[b] = std::prev(lru_.end());
        } else {
          free_.push_back(b);
        }
      }
    }
  }

  // Longest cached prefix of `tokens` in whole blocks; the returned blocks are shared
  // (refcount +1) on behalf of the caller.
  std::vector<int64_t> match_prefix(const std::vector<int64_t>& tokens) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<int64_t> out;
    uint64_t h = 0x243f6a8885a308d3ULL;
    const int64_t full = (int64_t)tokens.size() / bs_;
    for (int64_t i = 0; i < full; ++i) {
      h = block_hash(h, tokens, i);
      auto it = table_.find(h);
      if (it == table_.end()) break;
      const int64_t b = it->second;
      if (ref_[b] == 0) lru_erase(b);
      ++ref_[b];
      out.push_back(b);
    }
    ++lookups_;
    hit_blocks_ += (int64_t)out.size();
    return out;
  }

  // Publish the full blocks of a prompt (blocks[i] holds tokens[i*bs, (i+1)*bs)).
  void register_prefix(const std::vector<int64_t>& tokens, const std::vector<int64_t>& blocks) {
    std::lock_guard<std::mutex> g(mu_);
    uint64_t h = 0x243f6a8885a308d3ULL;
    const int64_t full = std::min<int64_t>((int64_t)tokens.size() / bs_, (int64_t)blocks.size());
    for (int64_t i = 0; i < full; ++i) {
      h = block_hash(h, tokens, i);
      const int64_t b = blocks[i];
      check(b);
      if (table_.count(h) || cached_[b]) continue;
      table_[h] = b;
      hash_of_[b] = h;
      cached_[b] = true;
    }
  }

  // Batched reservation with caller-computed block keys (one call for a whole batch:
  // the per-call cost of the bound methods, not the hashing, dominated 256 single calls).
  // Prompt i has nb[i] full-block keys in `keys` (chained: key j covers tokens
  // [0, (j+1) bs)), lens[i] tokens and needs need[i] blocks: its longest cached key prefix
  // is shared (the last hit is dropped when it would cover the whole prompt -- >= 1 token
  // is always recomputed), then fresh blocks complete the table.  Returns
  // [hits_0 .. hits_{B-1}, table_0 (need_0 ids), ..., table_{B-1}].  All or nothing: on
  // exhaustion every block taken or shared for the batch is released and it throws.
  std::vector<int64_t> match_alloc_batch(const std::vector<int64_t>& keys, const std::vector<int64_t>& nb,
                                         const std::vector<int64_t>& lens, const std::vector<int64_t>& need) {
    std::lock_guard<std::mutex> g(mu_);
    const size_t B = nb.size();
    if (lens.size() != B || need.size() != B) throw std::runtime_error("match_alloc_batch: sizes");
    std::vector<int64_t> out(B);
    size_t total = 0;
    for (size_t i = 0; i < B; ++i) total += (size_t)need[i];
    out.reserve(B + total);
    size_t off = 0;
    try {
      for (size_t i = 0; i < B; ++i) {
        if (off + (size_t)nb[i] > keys.size()) throw std::runtime_error("match_alloc_batch: keys");
        int64_t hits = 0;
        for (int64_t j = 0; j < nb[i] && hits < need[i]; ++j) {
          auto it = table_.find((uint64_t)keys[off + j]);
          if (it == table_.end()) break;
          const int64_t b = it->second;
          if (ref_[b] == 0) lru_erase(b);
          ++ref_[b];
          out.push_back(b);
          ++hits;
        }
        if (hits > 0 && hits * bs_ >= lens[i]) {
          release_one(out.back());
          out.pop_back();
          --hits;
        }
        ++lookups_;
        hit_blocks_ += hits;
        out[i] = hits;
        const int64_t fresh = need[i] - hits;
        if (fresh > (int64_t)free_.size() + (int64_t)lru_.size()) throw std::runtime_error("KV cache exhausted");
        for (int64_t j = 0; j < fresh; ++j) out.push_back(take_one());
        off += (size_t)nb[i];
      }
    } catch (...) {
      for (size_t k = B; k < out.size(); ++k) release_one(out[k]);
      throw;
    }
    return out;
  }

  // Publish the first nb[i] blocks of table i under its caller-computed keys (the keys
  // match_alloc_batch looks up); tables flat with ntab[i] ids each.
  void register_batch(const std::vector<int64_t>& keys, const std::vector<int64_t>& nb,
                      const std::vector<int64_t>& tables, const std::vector<int64_t>& ntab) {
    std::lock_guard<std::mutex> g(mu_);
    size_t ko = 0, to = 0;
    for (size_t i = 0; i < nb.size(); ++i) {
      const int64_t full = std::min(nb[i], ntab[i]);
      if (ko + (size_t)nb[i] > keys.size() || to + (size_t)ntab[i] > tables.size())
        throw std::runtime_error("register_batch: sizes");
      for (int64_t j = 0; j < full; ++j) {
        const uint64_t h = (uint64_t)keys[ko + j];
        const int64_t b = tables[to + j];
        check(b);
        if (table_.count(h) || cached_[b]) continue;
        table_[h] = b;
        hash_of_[b] = h;
        cached_[b] = true;
      }
      ko += (size_t)nb[i];
      to += (size_t)ntab[i];
    }
  }

  std::vector<int64_t> stats() {
    std::lock_guard<std::mutex> g(mu_);
    return {(int64_t)free_.size(), (int64_t)lru_.size(), (int64_t)table_.size(), lookups_, hit_blocks_};
  }

 private:
  uint64_t block_hash(uint64_t parent, const std::vector<int64_t>& t, int64_t i) const {
    uint64_t h = parent;
    for (int64_t j = i * bs_; j < (i + 1) * bs_; ++j) h = mix(h, (uint64_t)t[j]);
    return h;
  }
  void release_one(int64_t b) {   // free() of one block, lock held
    if (ref_[b] <= 0) throw std::runtime_error("double free of KV block");
    if (--ref_[b] == 0) {
      if (cached_[b]) {
        lru_.push_back(b);
        lru_pos_[b] = std::prev(lru_.end());
      } else {
        free_.push_back(b);
      }
    }
  }
  void check(int64_t b) const {
    if (b < 0 || b >= n_) throw std::runtime_error("KV block id out of range");
  }
  void lru_erase(int64_t b) {
    auto it = lru_pos_.find(b);
    if (it != lru_pos_.end()) {
      lru_.erase(it->second);
      lru_pos_.erase(it);
    }
  }
  int64_t take_one() {
    int64_t b;
    if (!free_.empty()) {
      b = free_.back();
      free_.pop_back();
    } else {  // evict the least recently released cached block
      b = lru_.front();
      lru_.pop_front();
      lru_pos_.erase(b);
      table_.erase(hash_of_[b]);
      cached_[b] = false;
    }
    ref_[b] = 1;
    return b;
  }

  int64_t n_, bs_;
  std::vector<int64_t> free_;
  std::vector<int64_t> ref_;
  std::vector<uint64_t> hash_of_;
  std::vector<bool> cached_;
  std::unordered_map<uint64_t, int64_t> table_;
  std::list<int64_t> lru_;
  std::unordered_map<int64_t, std::list<int64_t>::iterator> lru_pos_;
  std::mutex mu_;
  int64_t lookups_ = 0, hit_blocks_ = 0;
};


}  // namespace docqa_rt
