// block_manager.cpp -- torch.classes.docqa_rt.BlockManager: the native paged-KV block
// allocator with reference counts and a content-addressed prefix cache
// (block_manager_core.h).  When a new prompt starts with the same tokens as a cached one
// (the fixed RAG instruction template every /ask/ request shares), its leading blocks are
// reused instead of recomputed.
//
// Reference parity: no KV cache exists in the reference (generation is delegated to
// Ollama, llm-qa/main.py:69); this is the MI355X-native serving runtime around it.
#include <torch/custom_class.h>
#include <torch/library.h>

#include "block_manager_core.h"

namespace {

// torch's class_ binds methods of the registered class itself, so the core is held by
// composition and every method forwards
struct BlockManager : torch::CustomClassHolder {
  BlockManager(int64_t num_blocks, int64_t block_size) : core(num_blocks, block_size) {}
  int64_t num_free() { return core.num_free(); }
  int64_t num_blocks() { return core.num_blocks(); }
  int64_t block_size() { return core.block_size(); }
  std::vector<int64_t> alloc(int64_t n) { return core.alloc(n); }
  void share(std::vector<int64_t> b) { core.share(b); }
  void free(std::vector<int64_t> b) { core.free(b); }
  std::vector<int64_t> match_prefix(std::vector<int64_t> t) { return core.match_prefix(t); }
  void register_prefix(std::vector<int64_t> t, std::vector<int64_t> b) { core.register_prefix(t, b); }
  std::vector<int64_t> match_alloc_batch(std::vector<int64_t> keys, std::vector<int64_t> nb,
                                         std::vector<int64_t> lens, std::vector<int64_t> need) {
    return core.match_alloc_batch(keys, nb, lens, need);
  }
  void register_batch(std::vector<int64_t> keys, std::vector<int64_t> nb, std::vector<int64_t> tables,
                      std::vector<int64_t> ntab) {
    core.register_batch(keys, nb, tables, ntab);
  }
  std::vector<int64_t> stats() { return core.stats(); }
  docqa_rt::BlockManagerCore core;
};

}  // namespace

TORCH_LIBRARY(docqa_rt, m) {
  m.class_<BlockManager>("BlockManager")
      .def(torch::init<int64_t, int64_t>())
      .def("num_free", &BlockManager::num_free)
      .def("num_blocks", &BlockManager::num_blocks)
      .def("block_size", &BlockManager::block_size)
      .def("alloc", &BlockManager::alloc)
      .def("share", &BlockManager::share)
      .def("free", &BlockManager::free)
      .def("match_prefix", &BlockManager::match_prefix)
      .def("register_prefix", &BlockManager::register_prefix)
      .def("match_alloc_batch", &BlockManager::match_alloc_batch)
      .def("register_batch", &BlockManager::register_batch)
      .def("stats", &BlockManager::stats);
}
