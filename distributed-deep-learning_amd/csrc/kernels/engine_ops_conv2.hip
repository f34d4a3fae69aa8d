// Explicit instantiations of the engine GEMM launches: OP_CONV2_DGRAD, OP_CONV2_WGRAD, OP_CONV1_WGRAD.
#include "engine_impl.h"

namespace ddl {

template void run_op_inst<OP_CONV2_DGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_CONV2_WGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_op_inst<OP_CONV1_WGRAD>(Engine&, const float*, int, const uint32_t*, bool, hipStream_t,
                                  int);
template void run_dual_inst<OP_CONV2_DGRAD, OP_CONV2_WGRAD>(Engine&, const float*, int, const uint32_t*,
                                                  hipStream_t);
template void run_dual_then_inst<OP_CONV2_DGRAD, OP_CONV2_WGRAD, OP_CONV1_WGRAD>(
    Engine&, const float*, int, const uint32_t*, hipStream_t);

}  // namespace ddl
