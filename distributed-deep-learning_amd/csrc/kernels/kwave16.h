// The 16-row K-wave launch of the fc forwards (CFG_KW16).
#pragma once
#include "gemm.h"

namespace ddl {

// K-wave launch on 16-row tiles (v_mfma_f32_16x16x4_f32), for the skinny fc GEMMs at M = batch:
// at M = 100 the 32-row tiles leave 4 of 128 rows useful in the last tile and 128 workgroups for
// 256 CUs; 16-row tiles give 7 x N/32 workgroups with 12 of 112 rows idle.  A workgroup of KW
// waves owns the 16x32 output tile, wave w runs 1/KW of the K range.  MFMA step s (0..7) of a
// 32-deep K tile feeds k = 8h + s from lane group h = lane >> 4 (the MFMA's own k index), so a
// lane's A values of a tile are 8 consecutive k of its row (two 16-byte loads).  N-contiguous B
// stages through the wave's own LDS image (rows k of 32 columns; the two 16-column halves of
// rows with bit 3 set swapped, so the lane groups h = 0 / 1 of a ds_read_b32 hit opposite bank
// halves); K-contiguous B loads straight into registers.  The KW accumulators are summed through
// LDS in wave order and the policy's column-wise epilogue runs in the same launch.
// floats of LDS a KW-wave 16-row K-wave tile needs (N-contiguous B: one 32 x 36 image per wave;
// K-contiguous B: the reduction buffer only)
template <int KW, class P>
constexpr int kw16_lds_floats() {
  return P::B_KCONTIG ? KW * 8 * 64 : KW * 32 * 36;
}
// One 16x32 tile (bx, by) by the KW waves of this workgroup (lds: kw16_lds_floats floats)
template <int KW, class P>
DDL_DEV void kw16_body(const P& p, int bx, int by, float* lds) {
  static_assert(P::A_KCONTIG, "K-contiguous A");
  constexpr int BK = 32, PB = 36;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int m_blk = bx * 16, n_blk = by * 32;
  const int r = lane & 15, h = lane >> 4;
  const int kc = ((p.K + KW - 1) / KW + BK - 1) / BK * BK;
  const int kb = wave * kc, ke = min(p.K, kb + kc);
  const auto a0 = p.prepA(m_blk + r, 8 * h), a1 = p.prepA(m_blk + r, 8 * h + 4);
  f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (P::B_KCONTIG) {
    const auto b00 = p.prepB(n_blk + r, 8 * h), b01 = p.prepB(n_blk + r, 8 * h + 4);
    const auto b10 = p.prepB(n_blk + 16 + r, 8 * h), b11 = p.prepB(n_blk + 16 + r, 8 * h + 4);
    for (int k0 = kb; k0 < ke; k0 += BK) {
      const float4 A0 = p.loadA(a0, k0), A1 = p.loadA(a1, k0);
      const float4 B00 = p.loadB(b00, k0), B01 = p.loadB(b01, k0);
      const float4 B10 = p.loadB(b10, k0), B11 = p.loadB(b11, k0);
      const float av[8] = {A0.x, A0.y, A0.z, A0.w, A1.x, A1.y, A1.z, A1.w};
      const float bv0[8] = {B00.x, B00.y, B00.z, B00.w, B01.x, B01.y, B01.z, B01.w};
      const float bv1[8] = {B10.x, B10.y, B10.z, B10.w, B11.x, B11.y, B11.z, B11.w};
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) {
        c0 = mfma16x16x4(av[s2], bv0[s2], c0);
        c1 = mfma16x16x4(av[s2], bv1[s2], c1);
      }
    }
  } else {
    float* img = lds + wave * BK * PB;
    typename P::BInfo bi[4];
    int off[4];
#pragma unroll
    for (int it = 0; it < 4; ++it) {
      const int sl = it * 64 + lane, kk = sl >> 3, nq = sl & 7;
      bi[it] = p.prepB(n_blk + 4 * nq, kk);
      off[it] = kk * PB + ((4 * nq) ^ (((kk >> 3) & 1) << 4));
    }
    float4 A0, A1, Bt[4];
    auto gload = [&](int k0) {
      A0 = p.loadA(a0, k0);
      A1 = p.loadA(a1, k0);
#pragma unroll
      for (int it = 0; it < 4; ++it) Bt[it] = p.loadB(bi[it], k0);
    };
    if (kb < ke) gload(kb);
    for (int k0 = kb; k0 < ke; k0 += BK) {
      // (one wave: its LDS ops run in order, so these stores follow the last tile's reads)
#pragma unroll
      for (int it = 0; it < 4; ++it) *reinterpret_cast<float4*>(img + off[it]) = Bt[it];
      const float av[8] = {A0.x, A0.y, A0.z, A0.w, A1.x, A1.y, A1.z, A1.w};
      float bv0[8], bv1[8];
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) {
        const int k = 8 * h + s2, sw = (h & 1) << 4;
        bv0[s2] = img[k * PB + (r ^ sw)];
        bv1[s2] = img[k * PB + ((16 + r) ^ sw)];
      }
      if (k0 + BK < ke) gload(k0 + BK);  // the next tile's loads under this tile's MFMAs
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) {
        c0 = mfma16x16x4(av[s2], bv0[s2], c0);
        c1 = mfma16x16x4(av[s2], bv1[s2], c1);
      }
    }
  }
  __syncthreads();  // every wave is past its image reads: the images become the sum buffer
  float* red = lds;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[(wave * 8 + i) * 64 + lane] = c0[i];
    red[(wave * 8 + 4 + i) * 64 + lane] = c1[i];
  }
  __syncthreads();
  if (wave < 2) {  // wave j finishes the 16-column half j: rows 4h .. 4h + 3 of column 16j + r
    const int j = wave;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int ww = 0; ww < KW; ++ww)
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += red[(ww * 8 + 4 * j + i) * 64 + lane];
    const int n = n_blk + 16 * j + r, m0 = m_blk + 4 * h;
    if (n < p.N && m0 < p.M) p.epi(m0, n, f32x4{v[0], v[1], v[2], v[3]});
  }
}

template <int KW, class P>
__global__ void __launch_bounds__(KW * 64) gemm_kw16_kernel(P p) {
  __shared__ float lds[kw16_lds_floats<KW, P>()];
  kw16_body<KW, P>(p, blockIdx.x, blockIdx.y, lds);
}

template <class P>
inline void launch_gemm_kw16(const P& p, int waves, hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0) return;
  const dim3 grid((p.M + 15) / 16, (p.N + 31) / 32);
  switch (waves) {
    case 4: DDL_LAUNCH((gemm_kw16_kernel<4, P>), grid, dim3(256), 0, stream, p); break;
    case 16: DDL_LAUNCH((gemm_kw16_kernel<16, P>), grid, dim3(1024), 0, stream, p); break;
    default: DDL_LAUNCH((gemm_kw16_kernel<8, P>), grid, dim3(512), 0, stream, p);
  }
}

}  // namespace ddl
