// Probe 2: f64 MFMA cycles/instruction (s_memtime), in-kernel clock (s_memtime vs
// s_memrealtime @100 MHz), and MFMA + VALU co-execution (waves split by role).
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_f64_rates.hip -o tools/probe_f64_rates
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

// role: 0 = all MFMA, 1 = all VALU, 2 = even waves MFMA / odd waves VALU
template <int ROLE>
__global__ __launch_bounds__(256) void mix_k(double* out, long long* stamps, int iters) {
  const int l = threadIdx.x, w = threadIdx.x >> 6;
  const bool do_mfma = ROLE == 0 || (ROLE == 2 && (w & 1) == 0);
  double a = 1.0 + 1e-9 * l, b = 1.0 - 1e-9 * l;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double v0 = l, v1 = l + 1, v2 = l + 2, v3 = l + 3, v4 = l + 4, v5 = l + 5, v6 = l + 6, v7 = l + 7;
  const double m = 0.999999, cc = 1e-9;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  if (do_mfma) {
    for (int i = 0; i < iters; i++) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
  } else {
    for (int i = 0; i < iters; i++) {  // 8 independent chains x 2 = 16 FMAs = 32 flops/lane per iter
      v0 = fma(v0, m, cc); v1 = fma(v1, m, cc); v2 = fma(v2, m, cc); v3 = fma(v3, m, cc);
      v4 = fma(v4, m, cc); v5 = fma(v5, m, cc); v6 = fma(v6, m, cc); v7 = fma(v7, m, cc);
      v0 = fma(v0, m, cc); v1 = fma(v1, m, cc); v2 = fma(v2, m, cc); v3 = fma(v3, m, cc);
      v4 = fma(v4, m, cc); v5 = fma(v5, m, cc); v6 = fma(v6, m, cc); v7 = fma(v7, m, cc);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + l] = s[0] + s[1] + s[2] + s[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7;
  if (l == 0 && blockIdx.x == 0) { stamps[0] = t1 - t0; stamps[1] = r1 - r0; }
}

template <int ROLE>
int run(const char* name, int nb, int iters, double* dO, long long* dS, int wpb_mfma, int wpb_valu) {
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
  mix_k<ROLE><<<nb, 256>>>(dO, dS, 64); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); mix_k<ROLE><<<nb, 256>>>(dO, dS, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  long long st[2]; CK(hipMemcpy(st, dS, 16, hipMemcpyDeviceToHost));
  double fm = (double)nb * wpb_mfma * iters * 4 * 2048.0, fv = (double)nb * wpb_valu * 64 * iters * 32.0;
  printf("%-22s %8.3f ms  MFMA %6.2f TF  VALU %6.2f TF  total %6.2f TF  clock %.0f MHz  cyc/iter(wave0) %.1f\n", name, ms,
         fm / ms / 1e9, fv / ms / 1e9, (fm + fv) / ms / 1e9, 100.0 * st[0] / (double)st[1], (double)st[0] / iters);
  return 0;
}

int main() {
  int dev; CK(hipGetDevice(&dev)); hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, dev));
  double* dO; long long* dS;
  int nb1 = p.multiProcessorCount;  // 1 block (4 waves) per CU
  CK(hipMalloc(&dO, (size_t)p.multiProcessorCount * 8 * 256 * 8)); CK(hipMalloc(&dS, 16));
  for (int bpc : {1, 2, 4, 8}) {
    int nb = nb1 * bpc; char n[64];
    snprintf(n, 64, "mfma  %d blk/CU", bpc); run<0>(n, nb, 4096, dO, dS, 4, 0);
    snprintf(n, 64, "valu  %d blk/CU", bpc); run<1>(n, nb, 4096, dO, dS, 0, 4);
    snprintf(n, 64, "mixed %d blk/CU", bpc); run<2>(n, nb, 4096, dO, dS, 2, 2);
  }
  return 0;
}
