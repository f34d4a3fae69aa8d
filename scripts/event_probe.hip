// Cost of a cross-stream hand-off point on the producer stream: a hipEventRecord marker between
// two kernels vs the same event attached to the producing kernel's launch (hipExtLaunchKernelGGL
// stopEvent, the kernel's own completion signal).  The consumer stream waits on the event and
// runs a short kernel each time, like the W > 1 step's exchange stream.
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

int main() {
  float *buf, *buf2;
  CK(hipMalloc(&buf, 4096 * 256 * sizeof(float)));
  CK(hipMalloc(&buf2, 64 * 256 * sizeof(float)));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev[4], t0, t1;
  for (int i = 0; i < 4; ++i)
    CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming | hipEventDisableSystemFence));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const int blocks = 2048, iters = 4000, steps = 200, seg = 4;
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(t0, s1));
      for (int st = 0; st < steps; ++st) {
        for (int k = 0; k < seg; ++k) {
          if (mode == 2 && k < seg - 1) {  // stop event on the kernel's own completion signal
            hipExtLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s1, nullptr, ev[k], 0, buf,
                                  iters);
          } else {
            hipLaunchKernelGGL(work, dim3(blocks), dim3(256), 0, s1, buf, iters);
          }
          if (mode == 1 && k < seg - 1) CK(hipEventRecord(ev[k], s1));  // marker packet
          if (mode > 0 && k < seg - 1) {
            CK(hipStreamWaitEvent(s2, ev[k], 0));
            hipLaunchKernelGGL(work, dim3(64), dim3(256), 0, s2, buf2, iters / 4);
          }
        }
        if (mode > 0) {  // the producer waits for the consumer at the end of the step
          CK(hipEventRecord(ev[3], s2));
          CK(hipStreamWaitEvent(s1, ev[3], 0));
        }
      }
      CK(hipEventRecord(t1, s1));
      CK(hipEventSynchronize(t1));
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      const char* name[] = {"no hand-off", "hipEventRecord marker", "ext-launch stop event"};
      printf("%-24s %.2f us/step\n", name[mode], 1e3f * ms / steps);
    }
  }
  return 0;
}
