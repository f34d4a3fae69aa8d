// Cost of a cross-stream hand-off point on the producer stream: a hipEventRecord marker between
// two kernels vs the same event attached to the producing kernel's launch (hipExtLaunchKernelGGL
// stopEvent, the kernel's own completion signal), over event flags and consumer set-ups.  The
// consumer stream waits on the event and runs a short kernel each time, like the W > 1 step's
// exchange stream.  Prints us per step (4 producer kernels, 3 hand-offs) per variant, twice.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/event_probe scripts/event_probe.hip && /tmp/event_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("%s failed: %s\n", #x, hipGetErrorString(e_));                \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// ~busy work: each block spins for `iters` dependent FMAs, then stores
__global__ void work(float* out, int iters) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i) a = fmaf(a, b, 1e-7f);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

struct Variant {
  const char* name;
  int handoff;      // 0 none, 1 marker (hipEventRecord), 2 stop event on the kernel launch
  unsigned flags;   // event creation flags
  int consumer;     // 0: nobody waits, 1: consumer stream waits + runs a kernel
  int hiprio;       // consumer stream at high priority (the runner's comm stream)
};

int main() {
  float *buf, *buf2;
  CK(hipMalloc(&buf, 4096 * 256 * sizeof(float)));
  CK(hipMalloc(&buf2, 64 * 256 * sizeof(float)));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  hipStream_t s1, s2, s2h;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  CK(hipStreamCreateWithPriority(&s2h, hipStreamNonBlocking, hi));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const unsigned DT = hipEventDisableTiming;
  const Variant vs[] = {
      {"no hand-off", 0, DT, 0, 0},
      {"marker, sysfence, consumer", 1, DT, 1, 1},
      {"marker, no-sysfence, consumer", 1, DT | hipEventDisableSystemFence, 1, 1},
      {"stop, sysfence, consumer", 2, DT, 1, 1},
      {"stop, no-sysfence, consumer", 2, DT | hipEventDisableSystemFence, 1, 1},
      {"stop, release-to-device, consumer", 2, DT | hipEventReleaseToDevice, 1, 1},
      {"stop, no-sysfence, no consumer", 2, DT | hipEventDisableSystemFence, 0, 1},
      {"marker, no-sysfence, no consumer", 1, DT | hipEventDisableSystemFence, 0, 1},
      {"stop, no-sysfence, consumer lo-prio", 2, DT | hipEventDisableSystemFence, 1, 0},
  };
  const int blocks = 2048, iters = 4000, steps = 200, seg = 4;
  for (int rep = 0; rep < 2; ++rep) {
    for (const Variant& v : vs) {
      hipEvent_t ev[4];
      for (int i = 0; i < 4; ++i) CK(hipEventCreateWithFlags(&ev[i], v.flags));
      hipStream_t sc = v.hiprio ? s2h : s2;
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, s1));
      for (int st = 0; st < steps; ++st) {
        for (int k = 0; k < seg; ++k) {
          const bool h = v.handoff && k < seg - 1;
          if (h && v.handoff == 2)
            hipExtLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s1, nullptr, ev[k], 0, buf,
                                  iters);
          else
            hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s1, buf, iters);
          if (h && v.handoff == 1) CK(hipEventRecord(ev[k], s1));
          if (h && v.consumer) {
            CK(hipStreamWaitEvent(sc, ev[k], 0));
            hipLaunchKernelGGL(work, dim3(64), dim3(256), 0, sc, buf2, iters / 4);
          }
        }
        if (v.handoff && v.consumer) {  // the producer waits for the consumer at step end
          CK(hipEventRecord(ev[3], sc));
          CK(hipStreamWaitEvent(s1, ev[3], 0));
        }
      }
      CK(hipEventRecord(t1, s1));
      CK(hipEventSynchronize(t1));
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      printf("%-40s %8.2f us/step\n", v.name, 1e3f * ms / steps);
      for (int i = 0; i < 4; ++i) CK(hipEventDestroy(ev[i]));
    }
  }
  return 0;
}
