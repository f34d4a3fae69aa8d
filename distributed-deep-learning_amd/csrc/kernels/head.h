// Classifier-head device code shared by head.hip (stand-alone kernels) and the engine's dual
// launch (fc3 weight gradient as extra blocks).  Semantics: model.py:85-92, SURVEY.md §2.6
// F19-F22, B1-B3.
#pragma once
#include "common.h"

namespace ddl {

constexpr int HK = 512;  // fc3 input width
constexpr int HC = 10;   // classes

// dW3_aug row i (i == HK: the bias row of ones) = sum_b [h2;1][b, i] * dlog[b, :], one wave
// per row: lanes stride the batch, the 10 class partials are reduced across the wave.
DDL_DEV void head_wgrad_row(const float* __restrict__ h2, const float* __restrict__ dlog, int B,
                            int i, float* __restrict__ gw, float* __restrict__ gb) {
  const int lane = threadIdx.x & 63;
  float acc[HC];
#pragma unroll
  for (int c = 0; c < HC; ++c) acc[c] = 0.f;
  for (int b = lane; b < B; b += 64) {
    const float hv = i < HK ? h2[(size_t)b * HK + i] : 1.f;
    const float* dl = dlog + (size_t)b * HC;
#pragma unroll
    for (int c = 0; c < HC; ++c) acc[c] = fmaf(hv, dl[c], acc[c]);
  }
#pragma unroll
  for (int c = 0; c < HC; ++c) {
    acc[c] = wave_sum(acc[c]);
  }
  if (lane < HC) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < HC; ++c)
      if (c == lane) v = acc[c];
    if (i < HK) gw[i * HC + lane] = v;
    else gb[lane] = v;
  }
}

// fc3 weight gradient as auxiliary blocks of a one-wave GEMM launch (gemm_dual_kernel's AUX):
// it needs dlog of every sample, so it cannot live in the per-sample head kernel; riding in
// the next launch (fc2's dual dgrad+wgrad, which needs only dh2) saves the head's second launch.
struct HeadWgradAux {
  const float* h2 = nullptr;
  const float* dlog = nullptr;
  int B = 0;
  float* gw = nullptr;
  float* gb = nullptr;
  int nblk = 0;    // HK + 1 rows (one wave each) when active, 0 otherwise
  int first_ = 0;  // after the GEMM blocks
  DDL_DEV void run(int b) const {
    if (b <= HK) head_wgrad_row(h2, dlog, B, b, gw, gb);
  }
};

}  // namespace ddl
