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

}  // namespace ddl
