// RCCL entry points for the native runtime (runner.hip, rccl_async.hip), resolved from the
// librccl instance torch already loaded: torch's ProcessGroupNCCL and our communicators must
// share ONE RCCL (a second copy from /opt/rocm would run its own proxy threads / shm / device
// state).  Declarations come from the header; the NCCL API of these calls is identical across
// the 2.26 (torch) / 2.27 (ROCm 7.2) builds.
#pragma once
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

#include <hip/hip_runtime.h>

namespace ddl {

struct RcclApi {
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclReduceScatter) ReduceScatter = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclReduce) Reduce = nullptr;
  decltype(&ncclBroadcast) Broadcast = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
};

inline const RcclApi& rccl() {
  static RcclApi api = [] {
    RcclApi a;
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) throw std::runtime_error(std::string("cannot locate librccl: ") + dlerror());
    auto sym = [&](const char* n) {
      void* f = dlsym(h, n);
      if (!f) throw std::runtime_error(std::string("librccl lacks ") + n);
      return f;
    };
    a.GetUniqueId = (decltype(a.GetUniqueId))sym("ncclGetUniqueId");
    a.CommInitRank = (decltype(a.CommInitRank))sym("ncclCommInitRank");
    a.CommDestroy = (decltype(a.CommDestroy))sym("ncclCommDestroy");
    a.GetErrorString = (decltype(a.GetErrorString))sym("ncclGetErrorString");
    a.ReduceScatter = (decltype(a.ReduceScatter))sym("ncclReduceScatter");
    a.AllGather = (decltype(a.AllGather))sym("ncclAllGather");
    a.AllReduce = (decltype(a.AllReduce))sym("ncclAllReduce");
    a.Reduce = (decltype(a.Reduce))sym("ncclReduce");
    a.Broadcast = (decltype(a.Broadcast))sym("ncclBroadcast");
    a.Send = (decltype(a.Send))sym("ncclSend");
    a.Recv = (decltype(a.Recv))sym("ncclRecv");
    a.GroupStart = (decltype(a.GroupStart))sym("ncclGroupStart");
    a.GroupEnd = (decltype(a.GroupEnd))sym("ncclGroupEnd");
    a.CommGetAsyncError = (decltype(a.CommGetAsyncError))sym("ncclCommGetAsyncError");
    a.CommAbort = (decltype(a.CommAbort))sym("ncclCommAbort");
    return a;
  }();
  return api;
}

#define RCCL_CHECK(x)                                                                 \
  do {                                                                                \
    ncclResult_t r_ = (x);                                                            \
    if (r_ != ncclSuccess)                                                            \
      throw std::runtime_error(std::string("RCCL: ") + #x + ": " +                     \
                               ::ddl::rccl().GetErrorString(r_));                      \
  } while (0)
#define HIP_CHECK(x)                                                                  \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess)                                                             \
      throw std::runtime_error(std::string("HIP: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

}  // namespace ddl
