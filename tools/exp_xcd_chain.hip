// Round-4 experiment: latency of one hop of a look-back style chain (wait for the predecessor's
// status word, then publish one's own), across the chip vs inside one XCD. Far: consecutive
// workgroups (which the dispatcher places on different XCDs), agent-scope loads and stores (they
// go past the XCD's L2). Near: each workgroup reads its XCD from HW_REG_XCC_ID, takes a ticket in
// its XCD's chain, and its status words are read and written with workgroup-scope atomics
// (L1-bypassing loads, write-through stores: served by the XCD's own L2), which is coherent here
// because only that XCD ever touches them. Build: hipcc --offload-arch=gfx950 -O2 -o
// tools/_build/exp_xcd_chain tools/exp_xcd_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr unsigned kSpinCap = 1u << 22;  // bounded spins: a missing predecessor flags and exits

__device__ inline unsigned xcc_id() { return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11)) & 7u; }

// laps x grid hops; WG b owns hops b, b + grid, ...
__global__ void k_far(unsigned long long* st, unsigned laps, unsigned long long* err) {
  if (threadIdx.x != 0) return;
  const unsigned g = gridDim.x, b = blockIdx.x;
  for (unsigned l = 0; l < laps; ++l) {
    const unsigned h = l * g + b;
    if (h > 0) {
      unsigned s = 0;
      while (__hip_atomic_load(&st[h - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0 && ++s < kSpinCap) {
      }
      if (s >= kSpinCap) {
        atomicAdd(err, 1ull);
        return;
      }
    }
    __hip_atomic_store(&st[h], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// per XCD: laps x (workgroups on it) hops; tickets from tick[xcc]
__global__ void k_near(unsigned long long* st, unsigned* tick, unsigned laps, unsigned stride,
                       unsigned long long* err, unsigned* per_xcd) {
  if (threadIdx.x != 0) return;
  const unsigned x = xcc_id();
  const unsigned t = atomicAdd(&tick[x], 1u);
  __syncthreads();
  const unsigned gx = per_xcd[x];  // workgroups this XCD runs (counted by a first launch)
  unsigned long long* sx = st + (size_t)x * stride;
  for (unsigned l = 0; l < laps; ++l) {
    const unsigned h = l * gx + t;
    if (h > 0) {
      unsigned s = 0;
      while (__hip_atomic_load(&sx[h - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0 && ++s < kSpinCap) {
      }
      if (s >= kSpinCap) {
        atomicAdd(err, 1ull);
        return;
      }
    }
    __hip_atomic_store(&sx[h], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

__global__ void k_count(unsigned* per_xcd) {
  if (threadIdx.x == 0) atomicAdd(&per_xcd[xcc_id()], 1u);
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const unsigned grid = prop.multiProcessorCount;  // one 64-thread workgroup per CU-equivalent
  const unsigned laps = 16, stride = 1 << 16;
  unsigned long long *st, *err;
  unsigned *tick, *per;
  CK(hipMalloc(&st, (size_t)8 * stride * 8));
  CK(hipMalloc(&err, 8));
  CK(hipMalloc(&tick, 64));
  CK(hipMalloc(&per, 64));
  CK(hipMemset(per, 0, 64));
  hipLaunchKernelGGL(k_count, dim3(grid), dim3(64), 0, 0, per);
  unsigned hper[8];
  CK(hipMemcpy(hper, per, 32, hipMemcpyDeviceToHost));
  printf("{\"grid\": %u, \"per_xcd\": [%u,%u,%u,%u,%u,%u,%u,%u]}\n", grid, hper[0], hper[1], hper[2], hper[3], hper[4],
         hper[5], hper[6], hper[7]);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int mode = 0; mode < 2; ++mode) {
    std::vector<float> ts;
    unsigned long long herr = 0;
    for (int rep = 0; rep < 12; ++rep) {
      CK(hipMemset(st, 0, (size_t)8 * stride * 8));
      CK(hipMemset(err, 0, 8));
      CK(hipMemset(tick, 0, 64));
      CK(hipEventRecord(a, 0));
      if (mode == 0) hipLaunchKernelGGL(k_far, dim3(grid), dim3(64), 0, 0, st, laps, err);
      else hipLaunchKernelGGL(k_near, dim3(grid), dim3(64), 0, 0, st, tick, laps, stride, err, per);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      unsigned long long e;
      CK(hipMemcpy(&e, err, 8, hipMemcpyDeviceToHost));
      herr += e;
      if (rep >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double med = ts[ts.size() / 2] * 1e3;  // us
    unsigned mx = 0;
    for (int x = 0; x < 8; ++x) mx = std::max(mx, hper[x]);
    const double hops = mode == 0 ? (double)laps * grid : (double)laps * mx;
    printf("{\"chain\": \"%s\", \"hops\": %.0f, \"kernel_us\": %.1f, \"ns_per_hop\": %.1f, \"stalls\": %llu}\n",
           mode == 0 ? "far (agent scope, consecutive workgroups)" : "near (workgroup scope, one XCD's L2)", hops, med,
           med * 1e3 / hops, herr);
    fflush(stdout);
  }
  return 0;
}
