// Round-4 experiment: the host-side floor of one synchronous call (C2's 10M select-project is
// ~45 us of kernels inside a ~62-87 us call). Times, median of many: an empty launch followed by
// hipEventSynchronize / hipStreamSynchronize / a spin on a pinned word the kernel stores, and the
// same with two launches (the two-pass shape). Build: hipcc --offload-arch=gfx950 -O2 -o
// tools/_build/exp_sync_latency tools/exp_sync_latency.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__global__ void k_empty(unsigned long long* flag, unsigned long long v) {
  if (flag && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
    __atomic_store_n(flag, v, __ATOMIC_RELEASE);  // vector store to host-coherent pinned memory
  }
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned long long* pin;
  CK(hipHostMalloc((void**)&pin, 64, hipHostMallocCoherent | hipHostMallocMapped));
  unsigned long long* dpin;
  CK(hipHostGetDevicePointer((void**)&dpin, pin, 0));
  unsigned long long* dbuf;
  CK(hipMalloc((void**)&dbuf, 64));
  const int reps = 2000;
  const int grid = 610;
  auto bench = [&](const char* name, int mode, int launches) {
    std::vector<double> t;
    for (int r = 0; r < reps + 50; ++r) {
      volatile unsigned long long* vp = pin;
      *vp = 0;
      const double t0 = now_us();
      for (int l = 0; l < launches; ++l)
        hipLaunchKernelGGL(k_empty, dim3(grid), dim3(1024), 0, s, (mode == 2 && l == launches - 1) ? dpin : nullptr,
                           (unsigned long long)(r + 1));
      if (mode == 0) {
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
      } else if (mode == 1) {
        CK(hipStreamSynchronize(s));
      } else if (mode == 2) {
        while (*vp != (unsigned long long)(r + 1)) {
        }
      } else if (mode == 3) {
        CK(hipMemcpyAsync(pin + 1, dbuf, 8, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
      }
      const double t1 = now_us();
      if (r >= 50) t.push_back(t1 - t0);
      if (mode == 2) CK(hipStreamSynchronize(s));  // drain before the next rep
    }
    std::sort(t.begin(), t.end());
    printf("{\"case\": \"%s\", \"launches\": %d, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f}\n", name,
           launches, t[t.size() / 2], t[t.size() / 10], t[t.size() * 9 / 10]);
    fflush(stdout);
  };
  for (int launches : {1, 2}) {
    bench("event_sync", 0, launches);
    bench("stream_sync", 1, launches);
    bench("spin_pinned", 2, launches);
    bench("memcpy_d2h_stream_sync", 3, launches);
  }
  return 0;
}
