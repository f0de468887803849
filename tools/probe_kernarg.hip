// Probe: does a launch with a large by-value kernel argument (8 descriptors of
// 1152 bytes, the batched lattice step's GPDesc array) reach the kernel intact?
// Each workgroup checks every 8-byte word of its descriptor against a pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int NB>
struct Pack { uint64_t w[NB][144]; };
template <int NB>
__global__ void k_probe(const Pack<NB> p, int* bad) {
  const uint64_t* d = p.w[blockIdx.x];
  for (int i = threadIdx.x; i < 144; i += blockDim.x)
    if (d[i] != (uint64_t)(blockIdx.x * 1000003ull + i * 7919ull + 1)) atomicAdd(bad, 1);
}
template <int NB>
int run() {
  Pack<NB> p;
  for (int b = 0; b < NB; ++b)
    for (int i = 0; i < 144; ++i) p.w[b][i] = b * 1000003ull + i * 7919ull + 1;
  int* bad;
  hipMalloc(&bad, sizeof(int));
  hipMemset(bad, 0, sizeof(int));
  hipLaunchKernelGGL(k_probe<NB>, dim3(NB), dim3(64), 0, 0, p, bad);
  hipError_t e = hipGetLastError();
  hipError_t e2 = hipDeviceSynchronize();
  int h = -1;
  hipMemcpy(&h, bad, sizeof(int), hipMemcpyDeviceToHost);
  printf("NB=%d bytes=%zu launch=%s sync=%s bad=%d\n", NB, sizeof(Pack<NB>), hipGetErrorString(e), hipGetErrorString(e2), h);
  hipFree(bad);
  return (e == hipSuccess && e2 == hipSuccess && h == 0) ? 0 : 1;
}
int main() {
  int r = run<1>();
  r |= run<3>();
  r |= run<4>();
  r |= run<8>();
  return r;
}
