// The fused fc chain launch (fc_chain.h): fc1 forward .. fc1 backward of one training step.
#include <stdlib.h>

#include "engine_impl.h"
#include "fc_chain.h"

namespace ddl {

void run_fc_chain(Engine& e, const int64_t* labels, int B, const uint32_t* seed, hipStream_t st) {
  if (B > 32 * kFcRowTiles) throw std::runtime_error("fc chain: batch > 128");
  FcChain a;
  const auto f1 = make_policy<OP_FC1_FWD>(e, B, nullptr, seed, true);
  const auto f2 = make_policy<OP_FC2_FWD>(e, B, nullptr, seed, true);
  a.f1 = {f1.M, f1.N, f1.K, f1.in, f1.w, f1.bias, f1.out, f1.seed, f1.layer, f1.thr24,
          f1.inv_keep, f1.seed_v};
  a.f2 = {f2.M, f2.N, f2.K, f2.in, f2.w, f2.bias, f2.out, f2.seed, f2.layer, f2.thr24,
          f2.inv_keep, f2.seed_v};
  int M, N, K;
  Engine::op_shape(OP_FC2_DGRAD, B, &M, &N, &K);
  a.d2 = {{M, N, K, e.dpre2fc, e.P[10]}, e.h1, e.inv_keep, e.dpre1fc};
  Engine::op_shape(OP_FC2_WGRAD, B, &M, &N, &K);
  a.w2 = {M, N, K, 1024, e.h1, e.dpre2fc, e.G[10], e.G[11]};
  Engine::op_shape(OP_FC1_DGRAD, B, &M, &N, &K);
  a.d1 = {{M, N, K, e.dpre1fc, e.P[8]}, e.c4, e.d4};
  Engine::op_shape(OP_FC1_WGRAD, B, &M, &N, &K);
  a.w1 = {M, N, K, 1024, e.p4, e.dpre1fc, e.G[8], e.G[9]};
  a.w3 = e.P[12];
  a.b3 = e.P[13];
  a.labels = labels;
  a.dlog = e.dlog;
  a.loss = e.loss;
  a.dpre2 = e.dpre2fc;
  a.gw3 = e.G[12];
  a.gb3 = e.G[13];
  a.inv_batch = 1.f / (float)B;
  a.thr24 = e.thr24;
  a.inv_keep = e.inv_keep;
  a.B = B;
  a.ctr = e.fc_ctr;
  a.timeout_ticks = (long long)(2.0 * 1e8);  // 2 s (wall_clock64: 100 MHz); healthy: us
  a.stamps = e.fc_stamps;
  using T = GemmTile<32, 32, 32, 1, 1, FcFwd<true, false, true>>;
  constexpr int L = T::LDS_F4 > 256 ? T::LDS_F4 : 256;
  static int grid = 0;
  if (!grid) {  // persistent: as many workgroups as can be resident (any count is correct)
    int per_cu = 0, dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fc_chain_kernel<L>,
                                                       kFcWaves * 64, 0);
    grid = std::max(1, std::min(per_cu, 2)) * std::max(cus, 1);
    if (const char* g = getenv("DDL_FC_CHAIN_GRID")) grid = atoi(g);
    grid = std::min(grid, kFcItems);
  }
  DDL_LAUNCH(fc_chain_kernel<L>, dim3(grid), dim3(kFcWaves * 64), 0, st, a);
  DDL_CHECK_LAUNCH();
}

}  // namespace ddl
