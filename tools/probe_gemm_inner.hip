// Probe 3: f64 GEMM inner loops on LDS-resident operands (no global traffic):
// VALU register-blocked outer products vs v_mfma_f64_16x16x4f64.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_gemm_inner.hip -o tools/probe_gemm_inner
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double rnd(unsigned e, unsigned salt) {
  unsigned x = e * 2654435761u ^ salt; x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  unsigned y = x * 2246822519u + 0x9e3779b9u; y ^= y >> 16;
  return ((double)x / 4294967296.0 - 0.5) + ((double)y / 4294967296.0) * 1e-7;
}
#ifdef RANDOM_DATA
#define FILL_A(e) rnd(e, 17u)
#define FILL_B(e) rnd(e, 91u)
#else
#define FILL_A(e) (1e-3 * ((e) % 97))
#define FILL_B(e) (1e-3 * ((e) % 89))
#endif

#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

// VALU: 256 threads, 128x128 output tile, thread = 8x8 block; K-step 16 in LDS, swept `reps` times.
template <int TM>
__global__ __launch_bounds__(256) void valu_k(double* out, int reps) {
  constexpr int BMt = 16 * TM;  // 128 for TM=8
  __shared__ double As[16][BMt], Bs[16][BMt];
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  for (int e = t; e < 16 * BMt; e += 256) { As[e / BMt][e % BMt] = FILL_A(e); Bs[e / BMt][e % BMt] = FILL_B(e); }
  __syncthreads();
  double c[TM][TM] = {};
  for (int rp = 0; rp < reps; ++rp) {
#pragma unroll 4
    for (int k = 0; k < 16; ++k) {
      double a[TM], b[TM];
#pragma unroll
      for (int i = 0; i < TM; i += 2) { double2 v = *(const double2*)&As[k][ty * TM + i]; a[i] = v.x; a[i + 1] = v.y; }
#pragma unroll
      for (int j = 0; j < TM; j += 2) { double2 v = *(const double2*)&Bs[k][tx * TM + j]; b[j] = v.x; b[j + 1] = v.y; }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) c[i][j] = fma(a[i], b[j], c[i][j]);
    }
  }
  double s = 0; for (int i = 0; i < TM; ++i) for (int j = 0; j < TM; ++j) s += c[i][j];
  out[blockIdx.x * 256 + t] = s;
}

// MFMA: 256 threads, 64x64 output tile (4 waves x 32x32 = 2x2 MFMA tiles), K-step 64 in LDS.
__global__ __launch_bounds__(256) void mfma_k(double* out, int reps) {
  __shared__ double As[64 * 64], Bs[64 * 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1, r = lane & 15, q = lane >> 4;
  for (int e = t; e < 4096; e += 256) { As[e] = FILL_A(e); Bs[e] = FILL_B(e); }
  __syncthreads();
  d4 c[2][2] = {};
  for (int rp = 0; rp < reps; ++rp) {
#pragma unroll 4
    for (int k0 = 0; k0 < 64; k0 += 4) {
      const int k = k0 + q;
      double a0 = As[k * 64 + ((wm * 32 + r) ^ ((k & 1) << 4))], a1 = As[k * 64 + ((wm * 32 + 16 + r) ^ ((k & 1) << 4))];
      double b0 = Bs[k * 64 + ((wn * 32 + r) ^ ((k & 1) << 4))], b1 = Bs[k * 64 + ((wn * 32 + 16 + r) ^ ((k & 1) << 4))];
      c[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, c[0][0], 0, 0, 0);
      c[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, c[0][1], 0, 0, 0);
      c[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, c[1][0], 0, 0, 0);
      c[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, c[1][1], 0, 0, 0);
    }
  }
  d4 s = c[0][0] + c[0][1] + c[1][0] + c[1][1];
  out[blockIdx.x * 256 + t] = s[0] + s[1] + s[2] + s[3];
}

// MFMA with 4x2 tiles per wave (64x32 per wave, 128x64 per WG)
__global__ __launch_bounds__(256) void mfma42_k(double* out, int reps) {
  __shared__ double As[64 * 128], Bs[64 * 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1, r = lane & 15, q = lane >> 4;
  for (int e = t; e < 8192; e += 256) As[e] = FILL_A(e);
  for (int e = t; e < 4096; e += 256) Bs[e] = FILL_B(e);
  __syncthreads();
  d4 c[4][2] = {};
  for (int rp = 0; rp < reps; ++rp) {
#pragma unroll 2
    for (int k0 = 0; k0 < 64; k0 += 4) {
      const int k = k0 + q;
      double a[4], b[2];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = As[k * 128 + ((wm * 64 + m * 16 + r) ^ ((k & 1) << 4))];
#pragma unroll
      for (int n = 0; n < 2; ++n) b[n] = Bs[k * 64 + ((wn * 32 + n * 16 + r) ^ ((k & 1) << 4))];
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) c[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[m], b[n], c[m][n], 0, 0, 0);
    }
  }
  d4 s = {};
  for (int m = 0; m < 4; ++m) for (int n = 0; n < 2; ++n) s += c[m][n];
  out[blockIdx.x * 256 + t] = s[0] + s[1] + s[2] + s[3];
}

int main() {
  double* dO; CK(hipMalloc(&dO, 256 * 16 * 256 * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
  for (int bpc : {1, 2, 3, 4}) {
    int nb = 256 * bpc;
    int reps = 256;
    valu_k<8><<<nb, 256>>>(dO, 4); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); valu_k<8><<<nb, 256>>>(dO, reps); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    double fl = (double)nb * 128 * 128 * 16 * 2.0 * reps;
    printf("VALU 8x8/thr  128x128/WG  %d WG/CU: %6.2f TF (%.3f ms)\n", bpc, fl / ms / 1e9, ms);
    mfma_k<<<nb, 256>>>(dO, 4); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); mfma_k<<<nb, 256>>>(dO, reps / 4); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = (double)nb * 64 * 64 * 64 * 2.0 * (reps / 4);
    printf("MFMA 2x2/wave  64x64/WG   %d WG/CU: %6.2f TF (%.3f ms)\n", bpc, fl / ms / 1e9, ms);
    mfma42_k<<<nb, 256>>>(dO, 4); CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0)); mfma42_k<<<nb, 256>>>(dO, reps / 4); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    fl = (double)nb * 128 * 64 * 64 * 2.0 * (reps / 4);
    printf("MFMA 4x2/wave 128x64/WG   %d WG/CU: %6.2f TF (%.3f ms)\n", bpc, fl / ms / 1e9, ms);
  }
  // sustained: ~15 ms launches back to back (DVFS settles)
  for (int rep = 0; rep < 3; ++rep) {
    int nb = 512, reps = 256 * 12;
    CK(hipEventRecord(e0)); mfma_k<<<nb, 256>>>(dO, reps); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    double fl = (double)nb * 64 * 64 * 64 * 2.0 * reps;
    printf("sustained MFMA 2x2/wave 2 WG/CU: %6.2f TF (%.3f ms)\n", fl / ms / 1e9, ms);
  }
  return 0;
}
