// conv1 forward (5x5 SAME, 1 -> 32 channels) + bias + ReLU + 2x2 max-pool, as a direct kernel
// over an LDS-staged image band (model.py:24-31).
//
// Through the GEMM engine conv1 is M = B*784 rows, N = 32, K = 25: one K tile whose im2col
// gather (CIN = 1: four range-checked scalar loads per float4, tap decode per element) costs
// ~47 VALU per MFMA and leaves the launch gather-bound (profiles/r3_pmc.md).  Here a workgroup
// stages a band of 18 input rows (14 output rows = 7 pooled rows, 2-row halo each side) of one
// image in LDS once, every wave keeps its 13 weight pairs in registers, and each MFMA's A
// operand is ONE ds_read at (lane's pixel + tap offset): 13 v_mfma_f32_32x32x2_f32 per 32x32
// output tile, K = 26 (tap 25 is a zero weight).  Output rows are pool-window-major (row
// i = 4 * window + q) so a lane's four consecutive accumulator rows are one 2x2 window and the
// pool + code run in registers, exactly as ConvFwd::epi (layers.h).
#include "api.h"
#include "common.h"
#include "layers.h"
#include "conv1.h"

namespace ddl {

namespace {

constexpr int kC1Rows = 18;                      // staged input rows per band
// staged row pitch: 28 + 2 + 2 columns used; 48 = 16 mod 32, so the two image rows a half-wave's
// ds_read_b32 touches (a 2x2 pool window spans rows y, y + 1) fall in disjoint bank halves
// (ds_read_b32 serves 32 lanes at a time, bank = dword mod 32; pitch 32 put them 2-way)
constexpr int kC1Pitch = 48;
constexpr int kC1Windows = 7 * 14;               // pool windows per band
constexpr int kC1Tiles = (kC1Windows + 7) / 8;   // 32-row MFMA tiles per band (13)

}  // namespace

__global__ void __launch_bounds__(64 * kC1Tiles)
conv1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                 const float* __restrict__ bias, float* __restrict__ out,
                 uint8_t* __restrict__ code) {
  __shared__ float T[kC1Rows * kC1Pitch];
  const int b = blockIdx.x, band = blockIdx.y;  // pooled rows [7 band, 7 band + 7)
  const int y0 = 14 * band - 2;                 // image row of T row 0; T col c = image col c - 2
  const float* img = x + (size_t)b * 784;
  for (int e = threadIdx.x; e < kC1Rows * kC1Pitch; e += blockDim.x) {
    const int iy = y0 + e / kC1Pitch, ix = e % kC1Pitch - 2;
    T[e] = ((unsigned)iy < 28u && (unsigned)ix < 28u) ? img[iy * 28 + ix] : 0.f;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = lane & 31, hk = lane >> 5;  // A row / B column, and the k parity of this lane
  // B operand: W1[k][col] for k = 2 * step + hk (k = 25: zero)
  float wv[13];
#pragma unroll
  for (int s = 0; s < 13; ++s) {
    const int k = 2 * s + hk;
    wv[s] = k < 25 ? w[k * 32 + col] : 0.f;
  }
  // A operand row `col` of this wave's tile: window wave*8 + col/4, pool position q = col%4
  const int win = wave * 8 + (col >> 2);
  const int wr = win < kC1Windows ? win : 0;  // rows past the band's windows compute window 0
  const int q = col & 3;
  const int ly = 2 * (wr / 14) + (q >> 1), lx = 2 * (wr % 14) + (q & 1);
  const float* trow = T + ly * kC1Pitch + lx;  // tap (0, 0) of this output pixel
  __syncthreads();
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
  for (int s = 0; s < 13; ++s) {
    const int k0 = 2 * s, k1 = 2 * s + 1;
    const int o0 = (k0 / 5) * kC1Pitch + k0 % 5;
    const int o1 = k1 < 25 ? (k1 / 5) * kC1Pitch + k1 % 5 : 0;
    acc = mfma32x32x2(trow[hk ? o1 : o0], wv[s], acc);
  }
  // lane: channel col, accumulator rows 8g + 4hk + r = window wave*8 + 2g + hk, q = r
  const float bb = bias[col];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int wg = wave * 8 + 2 * g + hk;
    if (wg >= kC1Windows) continue;
    float best = -INFINITY;
    int arg = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float val = acc[4 * g + r] + bb;
      if (val > best) { best = val; arg = r; }
    }
    const int py = 7 * band + wg / 14, px = wg % 14;
    out[map_off<14, 32, true>(b, py, px, col)] = best > 0.f ? best : 0.f;
    if (code)
      code[((size_t)(b * 14 + py) * 14 + px) * 32 + col] = best > 0.f ? (uint8_t)arg : (uint8_t)0xFF;
  }
}

void launch_conv1_fwd(const float* x, const float* w, const float* bias, float* out,
                      uint8_t* code, int B, hipStream_t st) {
  if (B <= 0) return;
  DDL_LAUNCH(conv1_fwd_kernel, dim3(B, 2), dim3(64 * kC1Tiles), 0, st, x, w, bias, out, code);
}

bool conv1_wgrad_fits(int B, size_t slab_floats, int max_tickets) {
  return conv1_wgrad_direct_ok(B, slab_floats, max_tickets);
}

// conv1's weight gradient alone (conv1.h; no reduce of another problem in the launch)
void launch_conv1_wgrad_only(const float* x, const float* d1, int B, float* gw, float* gb,
                             float* part, int* tickets, hipStream_t st) {
  if (B <= 0) return;
  using C = TileCfg<32, 32, 32, 1, 1>;
  launch_conv1_wgrad<C, WgradConv1>(WgradConv1{}, SubGrid(), x, d1, B, gw, gb, part, tickets, st);
}

}  // namespace ddl
