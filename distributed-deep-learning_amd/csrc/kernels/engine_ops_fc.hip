// Explicit instantiations of the engine GEMM launches: OP_FC2_DGRAD, OP_FC2_WGRAD, OP_FC1_DGRAD, OP_FC1_WGRAD.
#include "engine_impl.h"

namespace ddl {

template void run_op_inst<OP_FC2_DGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_FC2_WGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_FC1_DGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_FC1_WGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_dual_inst<OP_FC2_DGRAD, OP_FC2_WGRAD>(Engine&, const float*, int, const uint32_t*,
                                                  hipStream_t);
template void run_dual_inst<OP_FC1_DGRAD, OP_FC1_WGRAD>(Engine&, const float*, int, const uint32_t*,
                                                  hipStream_t);

bool run_fc2_deferred(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st) {
  e.fc2_slab = nullptr;
  if (e.cfg[OP_FC2_FWD] != 3) return false;
  const auto p = make_policy<OP_FC2_FWD>(e, B, x, seed, true);
  SubGrid g;
  launch_gemm<TILE_3>(p, e.splits[OP_FC2_FWD], e.wide[OP_FC2_FWD], e.scratch[0], st, &g);
  if (g.nblocks > 0 && g.mode == 2) {
    if (g.gz > 32) {  // (the head replicates the 4- and 16-lane reduce orders only)
      launch_reduce<TILE_3>(p, g, st);
      return true;
    }
    e.fc2_slab = reinterpret_cast<const float*>(g.slab);
    e.fc2_S = g.gz;
    e.fc2_gx = g.gx;
    e.fc2_ntiles = g.gx * g.gy;
  }
  return true;
}

void run_fc2_reduce(Engine& e, const uint32_t* seed, int B, hipStream_t st) {
  if (!e.fc2_slab) return;
  const auto p = make_policy<OP_FC2_FWD>(e, B, nullptr, seed, true);
  SubGrid g;
  g.slab = reinterpret_cast<float4*>(const_cast<float*>(e.fc2_slab));
  g.gz = e.fc2_S;
  g.gx = e.fc2_gx;
  g.gy = e.fc2_ntiles / e.fc2_gx;
  g.mode = 2;
  g.nblocks = g.gx * g.gy * g.gz;
  launch_reduce<TILE_3>(p, g, st);
  e.fc2_slab = nullptr;
}

}  // namespace ddl
