// Diagnostic: time k_potrf_diag (one 64x64 diagonal block per GP) with phase stamps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMFGP_STAMPS tools/bench_diag.hip -o tools/bench_diag
#include "../mfgp_coverage_amd/csrc/mfgp_kernels.hip"
#include <cstdio>
#include <cstring>
#include <vector>
#include <cmath>
using namespace mfgp;
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
int main() {
  const int64_t N = 200, ld = 256; const int B = 8;
  std::vector<double> A(ld * ld, 0.0);
  for (int i = 0; i < N; i++) for (int j = 0; j < N; j++) {
    double dx = (i % 17) * 0.05 - (j % 17) * 0.05, dy = (i / 17) * 0.05 - (j / 17) * 0.05;
    A[j * ld + i] = 0.1 * exp(-0.5 * (dx * dx + dy * dy) / 0.04) + (i == j ? 0.01 : 0.0);
  }
  double *dA, *dL; int* st; GPDesc* dd; long long* dS;
  CK(hipMalloc(&dA, sizeof(double) * ld * ld * B)); CK(hipMalloc(&dL, sizeof(double) * 4 * TILE * B));
  CK(hipMalloc(&st, sizeof(int) * B)); CK(hipMalloc(&dd, sizeof(GPDesc) * B)); CK(hipMalloc(&dS, 8 * 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dS, sizeof(dS)));
  std::vector<GPDesc> hd(B);
  for (int b = 0; b < B; b++) {
    CK(hipMemcpy(dA + b * ld * ld, A.data(), sizeof(double) * ld * ld, hipMemcpyHostToDevice));
    GPDesc& d = hd[b]; std::memset((void*)&d, 0, sizeof(d));
    d.A = dA + b * ld * ld; d.Linv = dL + b * 4 * TILE; d.status = st + b; d.ld = ld; d.N = N; d.NL = 0; d.M = 0;
  }
  CK(hipMemcpy(dd, hd.data(), sizeof(GPDesc) * B, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int it = 0; it < 5; it++) (void)launch_potrf_diag(dd, B, 0, 0);
  CK(hipDeviceSynchronize());
  const int R = 200; float ms;
  CK(hipEventRecord(e0));
  for (int it = 0; it < R; it++) (void)launch_potrf_diag(dd, B, 0, 0);
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
  long long s[64]; CK(hipMemcpy(s, dS, 8 * 64, hipMemcpyDeviceToHost));
  printf("k_potrf_diag: %.2f us per launch (B=%d, back-to-back)\n", 1e3 * ms / R, B);
  const char* nm[] = {"start","load","a0","b0","c0","a1","b1","c1","a2","b2","c2","a3","b3","c3","inv1","inv2","inv3","store"};
  int ids[] = {0,1,2,3,4,5,6,7,8,9,10,11,12,13,15,16,17,18};
  for (int q = 1; q < 18; q++) printf("  %-9s %7lld cycles\n", nm[q], s[ids[q]] - s[ids[q-1]]);
  printf("  total     %7lld cycles\n", s[18] - s[0]);
  // empty-ish kernel for launch overhead reference
  return 0;
}
