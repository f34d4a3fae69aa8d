// Per-block timestamps of the split-K dual launches (diagnostic build only: DDL_STAMPS=1 via
// DDL_BUILD_TAG=stamp DDL_EXTRA_CFLAGS=-DDDL_STAMPS=1, loaded with DDL_SO=_C_stamp.so).
//
// Each split-K block of a dual launch records, from lane 0 of its wave, 8 words: its start and
// end on the 100 MHz constant clock (s_memrealtime) and on the shader clock (s_memtime), the
// hardware slot it ran on (HW_ID: wave / SIMD / CU / SH / SE, and the XCC id), the number of
// 32-deep K tiles it ran and its (bx, by, bz) tile coordinates.  scripts/stamp_report.py turns
// them into per-launch spans, block-length spread, per-SIMD occupancy and tail.  In the default
// build none of this exists (DDL_STAMPS = 0).
#pragma once
#include <stdint.h>

#include <vector>

#ifndef DDL_STAMPS
#define DDL_STAMPS 0
#endif

namespace ddl {

struct StampRec {     // one launch's sub-grid in the stamp buffer
  int64_t off;        // first block's record index
  int nblocks, sub, gx, gy, gz;
};
struct StampState {
  unsigned long long* buf = nullptr;  // device, 8 words per block
  int64_t cap = 0, next = 0;          // records
  std::vector<StampRec> log;
};
inline StampState& stamp_state() {
  static StampState s;
  return s;
}
// the stamp area of the next sub-grid (null when stamping is off or the buffer is full)
inline unsigned long long* stamp_slot(int nblocks, int sub, int gx, int gy, int gz) {
  StampState& s = stamp_state();
  if (!s.buf || nblocks <= 0 || s.next + nblocks > s.cap) return nullptr;
  unsigned long long* p = s.buf + s.next * 8;
  s.log.push_back({s.next, nblocks, sub, gx, gy, gz});
  s.next += nblocks;
  return p;
}

#if DDL_STAMPS && defined(__HIPCC__)  // device half (gemm.h, after common.h)
struct Stamp {
  unsigned long long real, cyc;
};
DDL_DEV Stamp stamp_now() {
  return {__builtin_amdgcn_s_memrealtime(), __builtin_amdgcn_s_memtime()};
}
// mid (optional): the 100 MHz times at which the main loop ended and the split-K partial was
// stored with its ticket back (splitk_body); they replace the shader-clock pair in r[2], r[3]
DDL_DEV void stamp_block(unsigned long long* buf, int vb, const Stamp& s0, int nkt, int bx, int by,
                         int bz, const unsigned long long* mid = nullptr) {
  if (!buf || threadIdx.x != 0) return;
  const Stamp s1 = stamp_now();
  const unsigned hw = __builtin_amdgcn_s_getreg(0xf804);   // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg(0xf814);  // HW_REG_XCC_ID
  unsigned long long* r = buf + (size_t)vb * 8;
  r[0] = s0.real;
  r[1] = s1.real;
  r[2] = mid ? mid[0] : s0.cyc;
  r[3] = mid ? mid[1] : s1.cyc;
  r[4] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
  r[5] = (unsigned long long)nkt;
  r[6] = (unsigned long long)bx | ((unsigned long long)by << 32);
  r[7] = (unsigned long long)bz;
}
#endif

}  // namespace ddl
