// Diagnostic: HBM read rate of 2 GiB by access pattern (16-byte non-temporal loads).
//   A: grid-stride over the whole buffer (all workgroups sweep memory together)
//   B: workgroup b reads its own contiguous 1 MiB, 4 KiB per step
//   C: as B, wave w reads 2 KiB sub-blocks of each 8 KiB step (k_vstream's per-wave rows)
//   D: as C with four steps in flight per wave (k_vstream's U = 4)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_stream tools/probe_stream.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dv2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_a(const dv2* __restrict__ src, double* out, long n) {
  double acc = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    dv2 v = __builtin_nontemporal_load(src + i);
    acc += v.x + v.y;
  }
  if (acc == -1.0) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_b(const dv2* __restrict__ src, double* out, long per_wg) {
  const dv2* p = src + blockIdx.x * per_wg;
  double acc = 0.0;
  for (long i = threadIdx.x; i < per_wg; i += 256) {
    dv2 v = __builtin_nontemporal_load(p + i);
    acc += v.x + v.y;
  }
  if (acc == -1.0) out[0] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void k_c(const dv2* __restrict__ src, double* out, long per_wg) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const dv2* p = src + blockIdx.x * per_wg;
  double acc = 0.0;
  // step = 512 dv2 (8 KiB); wave w takes dv2 [128 w, 128 w + 128) of it, two loads per lane
  for (long s = 0; s < per_wg; s += 512L * U) {
    dv2 v[2 * U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      v[2 * u] = __builtin_nontemporal_load(p + s + 512L * u + 128 * w + l);
      v[2 * u + 1] = __builtin_nontemporal_load(p + s + 512L * u + 128 * w + 64 + l);
    }
#pragma unroll
    for (int u = 0; u < 2 * U; ++u) acc += v[u].x * v[u].y;
  }
  if (acc == -1.0) out[0] = acc;
}

int main() {
  const long n = 1L << 27;   // dv2 elements: 2 GiB
  dv2* buf;
  double* out;
  hipMalloc(&buf, n * 16);
  hipMalloc(&out, 64);
  hipMemset(buf, 0, n * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int nwg = 2048;
  const long per = n / nwg;
  for (int kind = 0; kind < 5; ++kind) {
    float best = 1e9f;
    for (int rep = 0; rep < 12; ++rep) {
      hipEventRecord(e0, 0);
      if (kind == 0) k_a<<<nwg, 256>>>(buf, out, n);
      if (kind == 1) k_b<<<nwg, 256>>>(buf, out, per);
      if (kind == 2) k_c<1><<<nwg, 256>>>(buf, out, per);
      if (kind == 3) k_c<4><<<nwg, 256>>>(buf, out, per);
      if (kind == 4) k_c<8><<<nwg, 256>>>(buf, out, per);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep > 1 && ms < best) best = ms;
    }
    const char* nm[] = {"A grid-stride", "B wg-contiguous", "C per-wave U=1", "D per-wave U=4", "E per-wave U=8"};
    printf("%-18s %8.1f us  %6.2f TB/s\n", nm[kind], best * 1e3, n * 16.0 / (best * 1e-3) / 1e12);
  }
  return 0;
}
