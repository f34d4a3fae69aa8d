// Explicit instantiations of the engine GEMM launches: OP_CONV1_FWD, OP_CONV2_FWD, OP_CONV3_FWD, OP_CONV4_FWD, OP_FC1_FWD, OP_FC2_FWD.
#include "engine_impl.h"

namespace ddl {

template void run_op_inst<OP_CONV1_FWD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_CONV2_FWD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_CONV3_FWD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_CONV4_FWD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_FC1_FWD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_FC2_FWD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);

bool run_fc2_fwd_partials(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st) {
  e.fc2_part.slab = nullptr;
  if (e.cfg[OP_FC2_FWD] != 3 || e.workers[OP_FC2_FWD] > 0) return false;
  const auto p = make_policy<OP_FC2_FWD>(e, B, x, seed, true);
  const SubGrid g = plan_gemm<32, 32, 32>(p, e.sarg(OP_FC2_FWD), 0, e.wide[OP_FC2_FWD],
                                          e.scratch[0]);
  // the head's fixed 16-lane reduction tree and 32x32 fragment decode
  if (g.streamk || g.mode != 2 || g.nblocks == 0 || g.gz <= 4 || g.gz > 16 || p.N != HK)
    return false;
  DDL_LAUNCH((gemm_f32_kernel<TILE_3, std::decay_t<decltype(p)>>), dim3(g.gx, g.gy, g.gz),
             dim3(64), 0, st, p, g.kchunk, g.mode, g.slab, g.tickets, g.xcd);
  e.fc2_part.slab = reinterpret_cast<const float*>(g.slab);
  e.fc2_part.S = g.gz;
  e.fc2_part.gx = g.gx;
  e.fc2_part.ntiles = g.gx * g.gy;
  return true;
}

}  // namespace ddl
