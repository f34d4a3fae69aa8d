// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DDL_DEV __device__ __forceinline__
#define DDL_HD __host__ __device__ __forceinline__

#include <hip/hip_ext.h>

namespace ddl {
// Completion event bound to the engine's kernel launches (host thread-local).  While set, a
// DDL_LAUNCH records it through the kernel's OWN dispatch packet (hipExtLaunchKernelGGL stop
// event) instead of a separate hipEventRecord marker packet.  A marker after the segment cost
// ~5 us of compute-queue idle per issue point (forced-rehearsal timelines) — and so does every
// kernel that carries the event, so a scope binds it to ONE launch: `target` (its index in the
// scope), or every launch when target < 0.  The scope reports how many launches it saw and
// which one got the event, so a caller that predicted the last launch wrong can fall back to
// a marker (SyncRunner::step).
struct StopCtl {
  hipEvent_t ev = nullptr;
  int target = -1;  // launch index to bind (< 0: all)
  int n = 0;        // launches issued in the scope
  int bound = -1;   // index of the last launch that got the event
};
inline StopCtl& stop_ctl() {
  static thread_local StopCtl c;
  return c;
}
// the event for the next launch, or null (advances the scope's launch count)
inline hipEvent_t take_stop_event() {
  StopCtl& c = stop_ctl();
  if (!c.ev) return nullptr;
  const int i = c.n++;
  if (c.target >= 0 && i != c.target) return nullptr;
  c.bound = i;
  return c.ev;
}
// RAII: the DDL_LAUNCHes inside the scope carry `ev` (launch `target` only, or all)
struct StopEventScope {
  explicit StopEventScope(hipEvent_t ev, int target = -1) {
    stop_ctl() = StopCtl{ev, target, 0, -1};
  }
  ~StopEventScope() { stop_ctl() = StopCtl{}; }
  int launches() const { return stop_ctl().n; }
  int bound() const { return stop_ctl().bound; }
  StopEventScope(const StopEventScope&) = delete;
  StopEventScope& operator=(const StopEventScope&) = delete;
};
}  // namespace ddl

#define DDL_LAUNCH(kernel, grid, block, shmem, stream, ...)                                     \
  do {                                                                                          \
    if (hipEvent_t ddl_ev_ = ::ddl::take_stop_event())                                          \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, nullptr, ddl_ev_, 0,             \
                            __VA_ARGS__);                                                       \
    else                                                                                        \
      hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                      \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------------
// Dropout RNG — bit-identical to ops/rng.py (lowbias32 finalizer on (index ^ layer_key)).
// TF1 tf.nn.dropout keeps an element when uniform >= rate (mnist_sync/model/model.py:73-74).
// ---------------------------------------------------------------------------------------------
DDL_DEV uint32_t ddl_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// key = mix(seed + layer * 0x9E3779B9) is computed on the host (ops/rng.py:layer_key).
DDL_DEV bool ddl_keep(uint32_t key, uint32_t idx, uint32_t thr24) {
  return (ddl_mix32(idx ^ key) >> 8) >= thr24;
}

// f32-input / f32-accumulate MFMA, 16x16x4 (exact fp32, 64 FLOP/clk/SIMD on gfx950).
// Lane l holds A[l&15][k=l>>4] and B[k=l>>4][l&15]; C/D: col = l&15, row = (l>>4)*4 + reg.
DDL_DEV f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// TF1 ApplyAdam update of one element (TF's update form, documented in optim.hip).
DDL_DEV void adam1(float& w, float g, float& m, float& v, float lr_t, float c1, float c2,
                   float eps) {
  m += (g - m) * c1;
  v += (g * g - v) * c2;
  w -= lr_t * m / (sqrtf(v) + eps);
}

// Momentum SGD of one element (mu = 0: plain SGD).  The roundings are pinned (one product, one
// fma each) so every kernel that applies it — the flat optimizer, the xGMI owner update, the
// async PS apply — gives the same bits whatever the compiler's contraction choices.
DDL_DEV void momentum1(float& w, float g, float& m, float lr, float mu, float scale) {
  m = __fmaf_rn(m, mu, __fmul_rn(g, scale));
  w = __fmaf_rn(-lr, m, w);
}

// Sum over aligned groups of RL lanes (RL = 1, 2, 4, ..., 64), returned in every lane of the
// group.  DPP adds inside each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror: after the quad steps every lane of a quad holds the quad's sum, so the mirrors
// pair whole partial sums), then the row sums of a 32 / 64 group by v_readlane.  Replaces
// __shfl_xor trees: each step of those is a ds_bpermute through the LDS pipe, and hipcc issued
// chains of them one lgkmcnt(0) wait at a time (the fused head spent ~4.6 us per sample on 60
// of them).  All 64 lanes of the wave must be active.
template <int CTRL>
DDL_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v),
                                                               CTRL, 0xF, 0xF, true));
}
DDL_DEV float rdlane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
template <int RL>
DDL_DEV float group_sum(float v) {
  static_assert(RL >= 1 && RL <= 64 && (RL & (RL - 1)) == 0, "power-of-two lane groups");
  if constexpr (RL >= 2) v += dpp_f<0xB1>(v);
  if constexpr (RL >= 4) v += dpp_f<0x4E>(v);
  if constexpr (RL >= 8) v += dpp_f<0x141>(v);
  if constexpr (RL >= 16) v += dpp_f<0x140>(v);
  if constexpr (RL == 32) {
    const float lo = rdlane_f(v, 0) + rdlane_f(v, 16), hi = rdlane_f(v, 32) + rdlane_f(v, 48);
    v = (threadIdx.x & 32) ? hi : lo;
  }
  if constexpr (RL == 64)
    v = (rdlane_f(v, 0) + rdlane_f(v, 16)) + (rdlane_f(v, 32) + rdlane_f(v, 48));
  return v;
}
DDL_DEV float wave_sum(float v) { return group_sum<64>(v); }

// 4x4 transpose inside each lane quad: lane qi (= lane & 3) holds a0..a3 (rows 0..3 of column
// qi) and gets row qi of columns 0..3.  Round k: every lane sends a[(qi + k) & 3]; DPP
// quad_perm makes lane qi read lane (qi - k) & 3, whose value is its a[qi] = element (qi, that
// column).  Every lane of the wave must be active.
template <int CTRL>
DDL_DEV float quad_rot(float v) { return dpp_f<CTRL>(v); }
DDL_DEV float4 quad_transpose(float a0, float a1, float a2, float a3, int qi) {
  auto pick = [&](int s) { return s == 0 ? a0 : s == 1 ? a1 : s == 2 ? a2 : a3; };
  float b[4];
  b[0] = b[1] = b[2] = b[3] = 0.f;
  const float own = pick(qi);
  const float r1 = quad_rot<0x93>(pick((qi + 1) & 3));  // quad_perm [3, 0, 1, 2]
  const float r2 = quad_rot<0x4E>(pick((qi + 2) & 3));  // quad_perm [2, 3, 0, 1]
  const float r3 = quad_rot<0x39>(pick((qi + 3) & 3));  // quad_perm [1, 2, 3, 0]
#pragma unroll
  for (int c = 0; c < 4; ++c)
    b[c] = c == qi ? own : c == ((qi + 3) & 3) ? r1 : c == ((qi + 2) & 3) ? r2 : r3;
  return make_float4(b[0], b[1], b[2], b[3]);
}

DDL_DEV float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// ---------------------------------------------------------------------------------------------
// Raw buffer loads (MI355X guide T8): 32-bit offsets against a wave-uniform descriptor, and
// the hardware range check returns 0 for any offset past num_records.  Gathers with padding
// (SAME conv halos, tile edges) therefore need no branches or predicated zero-fill: an
// out-of-range element simply gets offset kOOB.  Descriptors are built from kernel
// arguments only, so they stay in SGPRs (guide T20).
// ---------------------------------------------------------------------------------------------
typedef __amdgpu_buffer_rsrc_t brsrc_t;
constexpr int kOOB = 0x7FFFFFF0;

DDL_DEV brsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                           0x00020000);
}
DDL_DEV float4 bload4(brsrc_t r, int byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0);
  return *reinterpret_cast<float4*>(&v);
}
// per-lane offset + wave-uniform (SGPR) offset: the gather's per-K-tile part rides in the
// instruction's soffset field, no VALU add.  Only for offsets known to be in range.
DDL_DEV float4 bload4_so(brsrc_t r, int voff_bytes, int soff_bytes) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff_bytes, soff_bytes, 0);
  return *reinterpret_cast<float4*>(&v);
}
DDL_DEV float bload1(brsrc_t r, int byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0);
  return __builtin_bit_cast(float, v);
}
DDL_DEV float bload1_so(brsrc_t r, int voff_bytes, int soff_bytes) {
  auto v = __builtin_amdgcn_raw_buffer_load_b32(r, voff_bytes, soff_bytes, 0);
  return __builtin_bit_cast(float, v);
}

// Write-through (sc1) 16-B store / load pair for data handed to another workgroup inside
// one launch (MI355X guide §6 Guideline 16, R1): the stores need no agent-scope release (an
// L2 writeback) and the consumer's sc1 loads bypass its possibly-stale L1, so it needs no
// acquire either.  aux bit 16 = sc1.
DDL_DEV void bstore4_sc1(brsrc_t r, int byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                         r, byte_off, 0, 16);
}
DDL_DEV float4 bload4_sc1(brsrc_t r, int byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16);
  return *reinterpret_cast<float4*>(&v);
}

// System-coherent (sc0 | sc1) 16-B store / load: data for another GPU (xGMI peer memory) or
// the host.  A write-through store is counted complete (vmcnt) only once the memory side has
// acknowledged it, so a drained wave's payload is globally visible before any flag it stores
// next (guide G16 at system scope).
DDL_DEV void bstore4_sys(brsrc_t r, int byte_off, float4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v),
                                         r, byte_off, 0, 1 | 16);
}
DDL_DEV float4 bload4_sys(brsrc_t r, int byte_off) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 1 | 16);
  return *reinterpret_cast<float4*>(&v);
}
DDL_DEV void drain_vmem() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 4-byte forms of the same pair (and plain 4-byte store / int load through a descriptor)
DDL_DEV float bload1_sc1(brsrc_t r, int byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 16));
}
DDL_DEV void bstore1_sc1(brsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, byte_off, 0, 16);
}
DDL_DEV void bstore1(brsrc_t r, int byte_off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, byte_off, 0, 0);
}
DDL_DEV int bload1i(brsrc_t r, int byte_off) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA (MI355X guide: `buffer_load_dwordx4 ... lds`): a 16-byte gather per lane that lands
// in LDS at (wave-uniform base + lane * 16) without passing through VGPRs.  Issued from inline
// asm so hipcc's wait-count pass does not see an LDS write it cannot disambiguate (the builtin
// made it wait vmcnt(0) before every ds_read, draining tiles still in flight): the caller counts
// completion itself (vm_wait<N>) and retires its own reads of a buffer (lgkm_wait0) before
// re-staging it.  M0 is written and restored inside the statement (guide: M0 is reserved).
// ---------------------------------------------------------------------------------------------
struct Gather16 {  // what a policy's 16-byte operand load reads: descriptor + offsets
  brsrc_t r;
  int voff;  // per lane (kOOB: the range check returns zeros)
  int soff;  // wave-uniform
};
DDL_DEV uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
DDL_DEV void dma16(const Gather16& g, uint32_t lds_dst) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "buffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g.voff), "s"(g.r), "s"(lds_dst), "s"(__builtin_amdgcn_readfirstlane(g.soff))
      : "memory");
}
template <int N>
DDL_DEV void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else static_assert(N == 0 || N == 8, "add the count you need");
}
DDL_DEV void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

DDL_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

DDL_DEV float f4get(const float4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

#define DDL_CHECK_LAUNCH() (void)hipGetLastError()
