// roctx phase ranges for the native runtime ("roctx ranges per phase").
//
// DDL_TRACE=1 turns them on (the same switch as the Python ranges in utils/tracing.py).  The
// roctx library is resolved at run time — rocprofiler-sdk's librocprofiler-sdk-roctx first
// (what `rocprofv3 --marker-trace` records), else roctracer's libroctx64 (the one torch's nvtx
// ranges go through) — so the extension has no link-time dependency on either and costs one
// predictable branch per range when tracing is off.  Ranges are host-side: they bracket the
// ENQUEUE of a phase's kernels; the kernel trace of the same run gives their GPU times.
#pragma once
#include <dlfcn.h>
#include <stdlib.h>

namespace ddl {

struct RoctxApi {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  bool on = false;
};

inline const RoctxApi& roctx() {
  static RoctxApi api = [] {
    RoctxApi a;
    const char* e = getenv("DDL_TRACE");
    if (!e || e[0] != '1') return a;
    const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                          "libroctx64.so.4", "libroctx64.so"};
    for (const char* l : libs) {
      void* h = dlopen(l, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      a.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      a.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (a.push && a.pop) {
        a.on = true;
        break;
      }
    }
    return a;
  }();
  return api;
}

// RAII range; `name` must outlive the push call only (roctx copies it)
struct TraceRange {
  bool on;
  explicit TraceRange(const char* name) : on(roctx().on) {
    if (on) roctx().push(name);
  }
  ~TraceRange() {
    if (on) roctx().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace ddl
