// Diagnostic: latency of one dependent load chain (pointer chase, one lane) over a
// 1 MB buffer that fits L2, by load kind: plain, non-temporal, agent-scope
// relaxed atomic (global_load ... sc1), and over 512 MB (HBM / memory-side cache).
// Answers: does a device-scope (sc1) load of an L2-resident line cost an L2 hit
// or a trip past L2?
// Build: hipcc --offload-arch=gfx950 -O3 -o build/probe_sc1_latency tools/probe_sc1_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int KIND>
__global__ void k_chase(const uint64_t* __restrict__ next, uint64_t start, int steps, uint64_t* out, long long* cyc) {
  uint64_t p = start;
  // warm pass (fills the caches the load kind allows)
  for (int i = 0; i < steps; ++i) p = next[p];
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < steps; ++i) {
    if (KIND == 0) p = next[p];
    if (KIND == 1) p = __builtin_nontemporal_load(next + p);
    if (KIND == 2) p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const long long t1 = __builtin_amdgcn_s_memrealtime();
  out[0] = p;
  cyc[0] = t1 - t0;
}

int main() {
  for (long bytes : {1L << 20, 512L << 20}) {
    const long n = bytes / 8;
    uint64_t* h = new uint64_t[n];
    // a random cycle over cache-line-spaced slots (stride 16 elements = 128 B)
    const long slots = n / 16;
    long* perm = new long[slots];
    for (long i = 0; i < slots; ++i) perm[i] = i;
    uint64_t s = 88172645463325252ull;
    for (long i = slots - 1; i > 0; --i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      const long j = (long)(s % (uint64_t)(i + 1));
      const long t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
    for (long i = 0; i < slots; ++i) h[perm[i] * 16] = perm[(i + 1) % slots] * 16;
    uint64_t *d, *out;
    long long* cyc;
    (void)hipMalloc(&d, bytes);
    (void)hipMalloc(&out, 8);
    (void)hipMalloc(&cyc, 8);
    (void)hipMemcpy(d, h, bytes, hipMemcpyHostToDevice);
    const int steps = 4000;
    const char* nm[] = {"plain", "nontemporal", "agent-scope atomic (sc1)"};
    for (int kind = 0; kind < 3; ++kind) {
      long long best = 1LL << 62;
      for (int rep = 0; rep < 3; ++rep) {
        if (kind == 0) k_chase<0><<<1, 1>>>(d, perm[0] * 16, steps, out, cyc);
        if (kind == 1) k_chase<1><<<1, 1>>>(d, perm[0] * 16, steps, out, cyc);
        if (kind == 2) k_chase<2><<<1, 1>>>(d, perm[0] * 16, steps, out, cyc);
        long long c;
        (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        if (c < best) best = c;
      }
      // s_memrealtime: 100 MHz
      printf("%4ld MB  %-26s %7.1f ns per load\n", bytes >> 20, nm[kind], best * 10.0 / steps);
    }
    (void)hipFree(d);
    delete[] h;
    delete[] perm;
  }
  return 0;
}
