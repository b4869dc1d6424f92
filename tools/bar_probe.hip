// bar_probe.hip -- can the host write device memory directly (large BAR), and
// how fast is a host-written flag seen by a polling kernel?  Tool, not product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <time.h>
#include <immintrin.h>

static double now() { timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }

__global__ void echo(uint64_t *in, uint64_t *out, int rounds) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();
  for (int r = 1; r <= rounds; ++r) {
    while (__hip_atomic_load(in, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != (uint64_t)r) {
      if (wall_clock64() - t0 > 200000000ull) return;   // 2 s
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(out, (uint64_t)r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static int pingpong(const char *name, uint64_t *in_host, uint64_t *in_dev, uint64_t *out_host, uint64_t *out_dev,
                    bool fence = false) {
  const int rounds = 2000;
  *(volatile uint64_t *)in_host = 0;
  *(volatile uint64_t *)out_host = 0;
  hipLaunchKernelGGL(echo, dim3(1), dim3(64), 0, 0, in_dev, out_dev, rounds);
  double t0 = now();
  for (int r = 1; r <= rounds; ++r) {
    __atomic_store_n(in_host, (uint64_t)r, __ATOMIC_RELEASE);
    if (fence) _mm_sfence();   // flush the write-combining buffer (BAR mappings are WC)
    double ts = now();
    while (__atomic_load_n(out_host, __ATOMIC_ACQUIRE) != (uint64_t)r) {
      if (now() - ts > 1.0) { printf("%s: timeout at round %d\n", name, r); hipDeviceSynchronize(); return 1; }
    }
  }
  double t1 = now();
  hipDeviceSynchronize();
  printf("{\"probe\": \"%s\", \"round_trip_us\": %.3f}\n", name, (t1 - t0) / rounds * 1e6);
  return 0;
}

int main() {
  // host-memory flags (coherent, mapped)
  uint64_t *hin, *hout, *hin_d, *hout_d;
  hipHostMalloc(&hin, 64, hipHostMallocMapped | hipHostMallocCoherent);
  hipHostMalloc(&hout, 64, hipHostMallocMapped | hipHostMallocCoherent);
  hipHostGetDevicePointer((void **)&hin_d, hin, 0);
  hipHostGetDevicePointer((void **)&hout_d, hout, 0);
  pingpong("in=host out=host", hin, hin_d, hout, hout_d);
  // device fine-grained memory for the doorbell, written by the host through the BAR
  uint64_t *din = nullptr;
  hipError_t e = hipExtMallocWithFlags((void **)&din, 4096, hipDeviceMallocFinegrained);
  printf("hipExtMallocWithFlags(finegrained): %s ptr %p\n", hipGetErrorString(e), (void *)din);
  if (e == hipSuccess) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, din) == hipSuccess) printf("hostPointer %p devicePointer %p\n", a.hostPointer, a.devicePointer);
    fflush(stdout);
    pingpong("in=device(BAR) out=host", din, din, hout, hout_d);
    pingpong("in=device(BAR)+sfence out=host", din, din, hout, hout_d, true);
  }
  return 0;
}
