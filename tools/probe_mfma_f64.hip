// Probe: v_mfma_f64_16x16x4_f64 operand/accumulator lane layout and the f64 MFMA /
// f64 exp throughput on gfx950. Used once to pin the fragment maps the kernels rely on.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mfma_f64.hip -o /tmp/probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__global__ void layout_k(const double* A, const double* B, double* C) {
  int l = threadIdx.x;
  // assumed A map: lane l holds A[l&15][l>>4]; B map: B[l>>4][l&15]
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) C[l * 4 + r] = acc[r];
}

__global__ __launch_bounds__(256) void mfma_rate_k(double* out, int iters) {
  int l = threadIdx.x;
  double a = 1.0 + 1e-9 * l, b = 1.0 - 1e-9 * l;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < iters; i++) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 256 + l] = s[0] + s[1] + s[2] + s[3];
}

__global__ __launch_bounds__(256) void exp_rate_k(double* out, int iters) {
  int l = threadIdx.x + blockIdx.x * 256;
  double x = -1e-3 * (l & 1023), s = 0;
  for (int i = 0; i < iters; i++) { s += exp(x); x -= 1e-7; }
  out[l] = s;
}

__global__ __launch_bounds__(256) void fma_rate_k(double* out, int iters) {
  int l = threadIdx.x + blockIdx.x * 256;
  double a0 = l, a1 = l + 1, a2 = l + 2, a3 = l + 3, m = 0.999999, c = 1e-9;
  for (int i = 0; i < iters; i++) {
    a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
  }
  out[l] = a0 + a1 + a2 + a3;
}

int main() {
  std::vector<double> A(64), B(64), C(256), R(256);
  for (int i = 0; i < 16; i++) for (int k = 0; k < 4; k++) A[i * 4 + k] = i * 7 + k * 3 + 1;
  for (int k = 0; k < 4; k++) for (int j = 0; j < 16; j++) B[k * 16 + j] = k * 100 + j * 5 + 2;
  for (int i = 0; i < 16; i++) for (int j = 0; j < 16; j++) {
    double s = 0; for (int k = 0; k < 4; k++) s += A[i * 4 + k] * B[k * 16 + j]; R[i * 16 + j] = s; }
  double *dA, *dB, *dC, *dO;
  CK(hipMalloc(&dA, 64 * 8)); CK(hipMalloc(&dB, 64 * 8)); CK(hipMalloc(&dC, 256 * 8));
  CK(hipMemcpy(dA, A.data(), 64 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), 64 * 8, hipMemcpyHostToDevice));
  layout_k<<<1, 64>>>(dA, dB, dC);
  CK(hipMemcpy(C.data(), dC, 256 * 8, hipMemcpyDeviceToHost));
  int ok_guide = 1, ok_f32style = 1;
  for (int l = 0; l < 64; l++) for (int r = 0; r < 4; r++) {
    int col = l & 15;
    int row_g = (l >> 4) + 4 * r, row_f = (l >> 4) * 4 + r;
    if (C[l * 4 + r] != R[row_g * 16 + col]) ok_guide = 0;
    if (C[l * 4 + r] != R[row_f * 16 + col]) ok_f32style = 0;
  }
  printf("layout: guide-map(row=(l>>4)+4r) %s ; f32-map(row=4(l>>4)+r) %s\n", ok_guide ? "MATCH" : "no", ok_f32style ? "MATCH" : "no");
  for (int l = 0; l < 64; l += 13) {
    printf(" lane %2d:", l);
    for (int r = 0; r < 4; r++) {
      int found = -1; for (int q = 0; q < 256; q++) if (R[q] == C[l * 4 + r]) { found = q; break; }
      printf(" r%d->(%d,%d)", r, found / 16, found % 16);
    }
    printf("\n");
  }
  int dev; CK(hipGetDevice(&dev)); hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, dev));
  int nb = p.multiProcessorCount * 8; const int iters = 4096;
  CK(hipMalloc(&dO, (size_t)nb * 256 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
  mfma_rate_k<<<nb, 256>>>(dO, 16); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); mfma_rate_k<<<nb, 256>>>(dO, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  double fl = (double)nb * 4 /*waves*/ * iters * 4 * 2048.0;
  printf("CUs %d clock %d kHz: f64 MFMA 16x16x4 rate %.2f TFLOP/s (%.3f ms)\n", p.multiProcessorCount, p.clockRate, fl / ms / 1e9, ms);
  CK(hipEventRecord(e0)); fma_rate_k<<<nb, 256>>>(dO, iters); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  fl = (double)nb * 256 * iters * 4 * 2.0;
  printf("f64 VALU fma rate %.2f TFLOP/s\n", fl / ms / 1e9);
  CK(hipEventRecord(e0)); exp_rate_k<<<nb, 256>>>(dO, 256); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("f64 exp rate %.3f Gexp/s\n", (double)nb * 256 * 256 / ms / 1e6);
  return ok_guide ? 0 : 2;
}
