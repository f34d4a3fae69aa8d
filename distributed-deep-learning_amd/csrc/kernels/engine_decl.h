// Declarations of the engine's kernel-instantiating entry points (defined in
// engine_impl.h, explicitly instantiated in engine_ops_*.hip; called from engine.hip).
#pragma once
#include "api.h"

namespace ddl {

template <int OP>
void run_op_inst(Engine& e, const float* x, int B, const uint32_t* seed, bool train,
                 hipStream_t st, int si);
template <int OA, int OB>
void run_dual_inst(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st);
template <int OA, int OB, int ON>
void run_dual_then_inst(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st);
// fc2 forward with its mode-2 reduce left pending in e.fc2_* (false: not applicable, nothing
// launched); fc2's pending reduce as its own launch
bool run_fc2_deferred(Engine& e, const float* x, int B, const uint32_t* seed, hipStream_t st);
void run_fc2_reduce(Engine& e, const uint32_t* seed, int B, hipStream_t st);

}  // namespace ddl
