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
