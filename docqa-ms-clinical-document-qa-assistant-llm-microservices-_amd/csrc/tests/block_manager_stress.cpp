// block_manager_stress.cpp -- host stress test of the KV block manager core, built with
// ThreadSanitizer (data races) and with AddressSanitizer + UndefinedBehaviorSanitizer
// (memory errors, UB) by tests/test_native_sanitizers.py.  Host code only: GPU sanitizer
// builds are not available on the MI355X pool.
//
// T threads each run sequences of: match_prefix on one of a few shared "templates" +
// alloc of the remainder + register_prefix + (sometimes) share/free of a sibling's blocks
// + free -- the access pattern of concurrent schedulers sharing one KV pool with the
// RAG prefix cache.  Invariants checked at the end: every block is back (free or
// evictable), the prefix table only names evictable blocks, and the hit counters add up.
#include "../runtime/block_manager_core.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

using docqa_rt::BlockManagerCore;

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 8;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  const int64_t NB = argc > 3 ? atoi(argv[3]) : 48, BS = 16;   // small pool: eviction + OOM paths
  BlockManagerCore bm(NB, BS);
  std::vector<std::vector<int64_t>> templates(4);
  for (int k = 0; k < 4; ++k)
    for (int i = 0; i < (3 + k) * BS; ++i) templates[k].push_back(1000 * k + i);
  std::atomic<long> oom{0}, ops{0};
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) {
    th.emplace_back([&, t] {
      std::mt19937 rng(1234 + t);
      for (int it = 0; it < iters; ++it) {
        const auto& tpl = templates[rng() % templates.size()];
        std::vector<int64_t> prompt = tpl;
        const int extra = 1 + rng() % 40;
        for (int i = 0; i < extra; ++i) prompt.push_back(rng() % 50000);
        std::vector<int64_t> blocks;
        if (it % 2) {   // the engine's batched, caller-keyed path (match_alloc_batch / register_batch)
          std::vector<int64_t> keys;
          uint64_t h = 7;
          for (size_t j = 0; j + BS <= prompt.size(); j += BS) {
            for (size_t q = j; q < j + BS; ++q) h = docqa_rt::mix(h, (uint64_t)prompt[q]);
            keys.push_back((int64_t)h);
          }
          const int64_t total = ((int64_t)prompt.size() + 8 + BS - 1) / BS;
          std::vector<int64_t> out;
          try {
            out = bm.match_alloc_batch(keys, {(int64_t)keys.size()}, {(int64_t)prompt.size()}, {total});
          } catch (const std::runtime_error&) {
            ++oom;
            continue;
          }
          blocks.assign(out.begin() + 1, out.end());
          if ((int64_t)blocks.size() != total || out[0] * BS >= (int64_t)prompt.size()) {
            fprintf(stderr, "match_alloc_batch: bad table\n");
            std::abort();
          }
          bm.register_batch(keys, {(int64_t)keys.size()}, blocks, {total});
        } else {
          blocks = bm.match_prefix(prompt);
          const int64_t need = ((int64_t)prompt.size() + 8 + BS - 1) / BS - (int64_t)blocks.size();
          try {
            auto nb = bm.alloc(need);
            blocks.insert(blocks.end(), nb.begin(), nb.end());
          } catch (const std::runtime_error&) {
            ++oom;
            bm.free(blocks);
            continue;
          }
          bm.register_prefix(prompt, blocks);
        }
        if (rng() % 4 == 0) {         // a second holder of the prompt's leading blocks
          std::vector<int64_t> head(blocks.begin(), blocks.begin() + std::min<size_t>(2, blocks.size()));
          bm.share(head);
          bm.free(head);
        }
        bm.free(blocks);
        ++ops;
      }
    });
  }
  for (auto& x : th) x.join();
  auto st = bm.stats();   // free, evictable, cached, lookups, hit_blocks
  const bool all_back = st[0] + st[1] == NB;
  const bool table_ok = st[2] <= st[1];
  const bool lookups_ok = st[3] == (long)T * iters;
  printf("threads=%d iters=%d ops=%ld oom=%ld free=%ld evictable=%ld cached=%ld lookups=%ld hits=%ld\n", T, iters,
         ops.load(), oom.load(), (long)st[0], (long)st[1], (long)st[2], (long)st[3], (long)st[4]);
  if (!all_back || !table_ok || !lookups_ok || st[4] == 0) {
    fprintf(stderr, "invariant violated: all_back=%d table_ok=%d lookups_ok=%d\n", all_back, table_ok, lookups_ok);
    return 1;
  }
  // double free must be detected, not corrupt the pool
  auto b = bm.alloc(1);
  bm.free(b);
  try {
    bm.free(b);
    fprintf(stderr, "double free not detected\n");
    return 1;
  } catch (const std::runtime_error&) {
  }
  // exhaustion, deterministically (the threaded phase hits it only when threads overlap):
  // a request for more than the pool throws and leaves every block where it was
  try {
    auto all = bm.alloc(NB + 1);
    fprintf(stderr, "allocation past the pool not refused\n");
    return 1;
  } catch (const std::runtime_error&) {
  }
  auto st2 = bm.stats();
  if (st2[0] + st2[1] != NB) {
    fprintf(stderr, "refused allocation leaked blocks\n");
    return 1;
  }
  puts("OK");
  return 0;
}
