// Split-K scratch descriptor shared by host code (engine, bindings) and gemm.h.
#pragma once
#include <stddef.h>

namespace ddl {

// Partial slab + per-tile arrival tickets (zeroed once at allocation; each split-K
// reducer re-arms its ticket).
struct SplitScratch {
  void* slab = nullptr;   // float4 elements
  size_t slab_f4 = 0;
  int* tickets = nullptr;
  int max_tiles = 0;
};

}  // namespace ddl
