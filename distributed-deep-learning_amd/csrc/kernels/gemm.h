// Generic FP32 MFMA GEMM engine for gfx950: C[M,N] = sum_k A[m,k] * B[k,n].
//
// Every conv / fc forward, data-gradient and weight-gradient of the MNIST CNN is one
// instantiation of this kernel with a *problem* policy P that supplies:
//   * operand gathers: P::prepA(mn) -> per-thread info hoisted out of the K loop, then
//     P::loadA(info, k) returning 4 consecutive elements along the operand's contiguous
//     global direction (A_KCONTIG / B_KCONTIG); same for B.  Implicit-GEMM im2col,
//     transposed weights and pool-window row orders are just address functions — nothing
//     is materialised;
//   * a fused epilogue P::epi(m0, n, f32x4 rows m0..m0+3) (bias / ReLU / max-pool with
//     argmax code / dropout / pool-backward scatter / dW+db split).  The 32x32 MFMA C
//     layout gives each lane 4 groups of 4 consecutive rows of one column; with M
//     enumerated pool-window-major each group is exactly one 2x2 pool window.
//
// Math: v_mfma_f32_32x32x2_f32 (exact fp32; gfx950 has no xf32; 64-cycle issue and
// dependent latency, so one accumulator chain per fragment runs at the full rate).
// Tiling: BM x BN block tile, BK-deep K step, WM x WN waves (wave64), wave tile
// (BM/WM) x (BN/WN) of 32x32 fragments.  LDS double buffer + register prefetch of the next
// K tile (one barrier per K step); the LDS fragment reads of K sub-step r+1 are issued
// before the MFMAs of sub-step r.  LDS operand images follow global contiguity so the
// global->LDS copy is a straight float4 store:
//   K-contiguous operand -> [mn][BK+4]   one ds_read_b128 per 4 MFMAs: lane half
//                                        h = l>>5 owns k = 8r+4h .. 8r+4h+3 of every
//                                        8-deep sub-step (MFMA s pairs k = 8r+s and
//                                        8r+4+s); stride BK+4 is bank-conflict free for
//                                        the four 16-lane b128 groups
//   MN-contiguous operand -> [BK][mn+4]  ds_read_b32; the two 32-lane halves read rows
//                                        4 apart (separate conflict groups)
//
// Split-K (gridDim.z = S > 1), deterministic, no float atomics:
//   mode 1: every split stores its fp32 partial fragments (float4 per lane, coalesced)
//     and takes an arrival ticket; the last arriver of a tile sums the S partials in z
//     order and runs the fused epilogue (MI355X guide §5, in-launch split-K reduction:
//     agent-scope release before the ticket, acquire in the reducer).
//   mode 2: partials only; splitk_wide_reduce sums them with RL lanes per output element
//     and runs the epilogue.
#pragma once
#include "common.h"
#include "scratch.h"

namespace ddl {

typedef float f32x16 __attribute__((ext_vector_type(16)));

DDL_DEV f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN>
struct TileGeo {
  static constexpr int NW = WM * WN;
  static constexpr int WTM = BM / WM, WTN = BN / WN;
  static constexpr int TM = WTM / 32, TN = WTN / 32;
  static constexpr int FRAGS = TM * TN;
  // float4 elements of one split's partial tile: 4 float4 per fragment per lane
  static constexpr int PART4 = NW * FRAGS * 4 * 64;
};

template <int BM, int BN, int BK, int WM, int WN, class P>
__global__ void __launch_bounds__(WM * WN * 64)
gemm_f32_kernel(P p, int kchunk, int mode, float4* __restrict__ slab, int* __restrict__ tickets) {
  using G = TileGeo<BM, BN, WM, WN>;
  constexpr int NT = WM * WN * 64;
  constexpr bool AK = P::A_KCONTIG;
  constexpr bool BKC = P::B_KCONTIG;
  constexpr int SA = AK ? (BK + 4) : (BM + 4);
  constexpr int A_ELEMS = AK ? BM * SA : BK * SA;
  constexpr int SB = BKC ? (BK + 4) : (BN + 4);
  constexpr int B_ELEMS = BKC ? BN * SB : BK * SB;
  constexpr int WTM = G::WTM, WTN = G::WTN, TM = G::TM, TN = G::TN;
  constexpr int FA = (BM * BK / 4) / NT;
  constexpr int FB = (BN * BK / 4) / NT;
  constexpr int R = BK / 8;
  static_assert(FA >= 1 && FA * NT == BM * BK / 4, "A tile must split evenly over threads");
  static_assert(FB >= 1 && FB * NT == BN * BK / 4, "B tile must split evenly over threads");
  static_assert(TM * 32 == WTM && TN * 32 == WTN, "wave tile must be 32-multiples");
  static_assert(BK % 8 == 0, "BK must be a multiple of 8");

  // One-wave blocks need neither a second LDS buffer nor barriers: a wave's LDS ops execute
  // in order, so the next tile's ds_writes cannot overtake this tile's ds_reads.  Halving
  // the LDS footprint doubles the resident waves per CU (LDS was the occupancy limit).
  constexpr bool SOLO = (NT == 64);
  constexpr int NBUF = SOLO ? 1 : 2;
  __shared__ float4 lds4[(NBUF * (A_ELEMS + B_ELEMS)) / 4];
  float* const As0 = reinterpret_cast<float*>(lds4);
  float* const Bs0 = As0 + NBUF * A_ELEMS;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m_blk = blockIdx.x * BM;
  const int n_blk = blockIdx.y * BN;
  const int kb = blockIdx.z * kchunk;
  const int ke = min(p.K, kb + kchunk);
  const int nk = (ke - kb + BK - 1) / BK;

  // ---- per-thread hoisted gather state ------------------------------------------------------
  // Loader protocol: prepX(mn, kk) fixes a thread's row/column (group) and its k offset
  // inside every K tile; loadX(info, k0) gathers at tile base k0 (wave-uniform, a multiple
  // of BK = 32), so per-tile index math that depends only on k0 runs on the scalar unit.
  typename P::AInfo ai[FA];
  typename P::BInfo bi[FB];
  int a_off[FA], b_off[FB];
#pragma unroll
  for (int it = 0; it < FA; ++it) {
    const int idx = tid + it * NT;
    if constexpr (AK) {
      const int kq = idx % (BK / 4), row = idx / (BK / 4);
      ai[it] = p.prepA(m_blk + row, kq * 4);
      a_off[it] = row * SA + kq * 4;
    } else {
      const int mq = idx % (BM / 4), kk = idx / (BM / 4);
      ai[it] = p.prepA(m_blk + mq * 4, kk);
      a_off[it] = kk * SA + mq * 4;
    }
  }
#pragma unroll
  for (int it = 0; it < FB; ++it) {
    const int idx = tid + it * NT;
    if constexpr (BKC) {
      const int kq = idx % (BK / 4), row = idx / (BK / 4);
      bi[it] = p.prepB(n_blk + row, kq * 4);
      b_off[it] = row * SB + kq * 4;
    } else {
      const int nq = idx % (BN / 4), kk = idx / (BN / 4);
      bi[it] = p.prepB(n_blk + nq * 4, kk);
      b_off[it] = kk * SB + nq * 4;
    }
  }

  float4 ra[FA], rb[FB];
  auto gload = [&](int k0) {
#pragma unroll
    for (int it = 0; it < FA; ++it) ra[it] = p.loadA(ai[it], k0);
#pragma unroll
    for (int it = 0; it < FB; ++it) rb[it] = p.loadB(bi[it], k0);
  };
  auto sstore = [&](int buf) {
    float* As = As0 + buf * A_ELEMS;
    float* Bs = Bs0 + buf * B_ELEMS;
#pragma unroll
    for (int it = 0; it < FA; ++it) *reinterpret_cast<float4*>(As + a_off[it]) = ra[it];
#pragma unroll
    for (int it = 0; it < FB; ++it) *reinterpret_cast<float4*>(Bs + b_off[it]) = rb[it];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

  const int lr = lane & 31;   // fragment row / column
  const int lh = lane >> 5;   // k half

  // fragment fetch of K sub-step r from LDS buffer (As, Bs)
  auto fetch = [&](const float* As, const float* Bs, int r, float (&av)[TM][4], float (&bv)[TN][4]) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * WTM + i * 32 + lr;
      if constexpr (AK) {
        const float4 t = *reinterpret_cast<const float4*>(As + row * SA + r * 8 + 4 * lh);
        av[i][0] = t.x; av[i][1] = t.y; av[i][2] = t.z; av[i][3] = t.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) av[i][s] = As[(r * 8 + 4 * lh + s) * SA + row];
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = wn * WTN + j * 32 + lr;
      if constexpr (BKC) {
        const float4 t = *reinterpret_cast<const float4*>(Bs + col * SB + r * 8 + 4 * lh);
        bv[j][0] = t.x; bv[j][1] = t.y; bv[j][2] = t.z; bv[j][3] = t.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) bv[j][s] = Bs[(r * 8 + 4 * lh + s) * SB + col];
      }
    }
  };

  if (nk > 0) {
    gload(kb);
    sstore(0);
  }
  if constexpr (!SOLO) __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = SOLO ? 0 : (kt & 1);
    if (kt + 1 < nk) gload(kb + (kt + 1) * BK);
    const float* As = As0 + cur * A_ELEMS;
    const float* Bs = Bs0 + cur * B_ELEMS;
    float av[2][TM][4], bv[2][TN][4];
    fetch(As, Bs, 0, av[0], bv[0]);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r + 1 < R) fetch(As, Bs, r + 1, av[(r + 1) & 1], bv[(r + 1) & 1]);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = mfma32x32x2(av[r & 1][i][s], bv[r & 1][j][s], acc[i][j]);
    }
    if (kt + 1 < nk) sstore(SOLO ? 0 : (cur ^ 1));
    if constexpr (!SOLO) __syncthreads();
  }

  if (mode != 0) {
    // ---- split-K: publish this split's partial fragments ------------------------------------
    const int tile = blockIdx.y * gridDim.x + blockIdx.x;
    const int ntiles = gridDim.x * gridDim.y;
    const int S = gridDim.z;
    constexpr int WPART = TM * TN * 4 * 64;  // float4 per wave
    float4* mine = slab + ((size_t)blockIdx.z * ntiles + tile) * G::PART4 + wave * WPART + lane;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x16& v = acc[i][j];
          mine[((i * TN + j) * 4 + g) * 64] =
              make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
        }
    if (mode == 2) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(lds4);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int prev = __hip_atomic_fetch_add(&tickets[tile], 1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == S - 1;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tickets[tile] = 0;  // re-arm for the next launch (kernel boundary orders it)
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    const float4* base = slab + (size_t)tile * G::PART4 + wave * WPART + lane;
    const size_t zstride = (size_t)ntiles * G::PART4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
    for (int z = 0; z < S; ++z) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const float4 t = base[z * zstride + ((i * TN + j) * 4 + g) * 64];
            acc[i][j][4 * g] += t.x; acc[i][j][4 * g + 1] += t.y;
            acc[i][j][4 * g + 2] += t.z; acc[i][j][4 * g + 3] += t.w;
          }
    }
  }

  // ---- fused epilogue: each lane owns 4 groups of 4 consecutive rows of one column ----------
#pragma unroll
  for (int i = 0; i < TM; ++i) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n_blk + wn * WTN + j * 32 + lr;
      if (n >= p.N) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int m0 = m_blk + wm * WTM + i * 32 + 8 * g + 4 * lh;
        if (m0 < p.M) {
          const f32x16& v = acc[i][j];
          p.epi(m0, n, f32x4{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]});
        }
      }
    }
  }
}

// Wide split-K reduce (mode 2): RL lanes cooperate on one float4 output element.
template <int BM, int BN, int WM, int WN, int RL, class P>
__global__ void __launch_bounds__(256)
splitk_wide_reduce(P p, const float4* __restrict__ slab, int S, int gx, int ntiles) {
  using G = TileGeo<BM, BN, WM, WN>;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  const int elem = gid / RL;
  const int sub = gid % RL;
  const int nelem = ntiles * G::PART4;
  const bool valid = elem < nelem;
  const int e = valid ? elem : 0;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  const size_t zstride = (size_t)ntiles * G::PART4;
  for (int z = sub; z < S; z += RL) {
    const float4 t = slab[z * zstride + e];
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
#pragma unroll
  for (int off = RL / 2; off > 0; off >>= 1) {
    s.x += __shfl_xor(s.x, off, 64);
    s.y += __shfl_xor(s.y, off, 64);
    s.z += __shfl_xor(s.z, off, 64);
    s.w += __shfl_xor(s.w, off, 64);
  }
  if (!valid || sub != 0) return;
  const int tile = e / G::PART4;
  int r = e % G::PART4;
  constexpr int WPART = G::FRAGS * 4 * 64;
  const int wave = r / WPART;
  r %= WPART;
  const int fg = r / 64, lane = r % 64;
  const int frag = fg / 4, g = fg % 4;
  const int i = frag / G::TN, j = frag % G::TN;
  const int wm = wave / WN, wn = wave % WN;
  const int bx = tile % gx, by = tile / gx;
  const int m0 = bx * BM + wm * G::WTM + i * 32 + 8 * g + 4 * (lane >> 5);
  const int n = by * BN + wn * G::WTN + j * 32 + (lane & 31);
  if (n < p.N && m0 < p.M) p.epi(m0, n, f32x4{s.x, s.y, s.z, s.w});
}

template <int BK>
inline int splitk_kchunk(int K, int splits) {
  if (splits <= 1) return K;
  const int per = (K + splits - 1) / splits;
  const int kc = ((per + BK - 1) / BK) * BK;
  return kc < BK ? BK : kc;
}

template <int BK>
inline int splitk_z(int K, int splits) {
  if (splits <= 1) return 1;
  const int kc = splitk_kchunk<BK>(K, splits);
  const int z = (K + kc - 1) / kc;
  return z < 1 ? 1 : z;
}

// float4 partial-slab elements a launch needs
template <int BM, int BN, int BK, int WM, int WN>
inline size_t splitk_slab_f4(int M, int N, int K, int splits) {
  const int z = splitk_z<BK>(K, splits);
  if (z <= 1) return 0;
  const size_t tiles = (size_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  return (size_t)z * tiles * TileGeo<BM, BN, WM, WN>::PART4;
}

// wide_thr: z > wide_thr uses mode 2 (separate wide reduce), else mode 1 (last arriver).
template <int BM, int BN, int BK, int WM, int WN, class P>
inline void launch_gemm(const P& p, int splits, int wide_thr, const SplitScratch& sc,
                        hipStream_t stream) {
  if (p.M <= 0 || p.N <= 0) return;
  const int z = splitk_z<BK>(p.K, splits);
  const int kchunk = z > 1 ? splitk_kchunk<BK>(p.K, splits) : p.K;
  const int gx = (p.M + BM - 1) / BM, gy = (p.N + BN - 1) / BN;
  const int mode = z == 1 ? 0 : (z > wide_thr ? 2 : 1);
  dim3 grid(gx, gy, z);
  hipLaunchKernelGGL((gemm_f32_kernel<BM, BN, BK, WM, WN, P>), grid, dim3(WM * WN * 64), 0,
                     stream, p, kchunk, mode, reinterpret_cast<float4*>(sc.slab), sc.tickets);
  if (mode == 2) {
    using G = TileGeo<BM, BN, WM, WN>;
    const int ntiles = gx * gy;
    const size_t nelem = (size_t)ntiles * G::PART4;
    const float4* s4 = reinterpret_cast<const float4*>(sc.slab);
    if (z > 32) {
      const size_t th = nelem * 64;
      hipLaunchKernelGGL((splitk_wide_reduce<BM, BN, WM, WN, 64, P>), dim3((th + 255) / 256),
                         dim3(256), 0, stream, p, s4, z, gx, ntiles);
    } else if (z > 4) {
      const size_t th = nelem * 16;
      hipLaunchKernelGGL((splitk_wide_reduce<BM, BN, WM, WN, 16, P>), dim3((th + 255) / 256),
                         dim3(256), 0, stream, p, s4, z, gx, ntiles);
    } else {
      const size_t th = nelem * 4;
      hipLaunchKernelGGL((splitk_wide_reduce<BM, BN, WM, WN, 4, P>), dim3((th + 255) / 256),
                         dim3(256), 0, stream, p, s4, z, gx, ntiles);
    }
  }
}

}  // namespace ddl
