// Probe: the 4x4x4 f64 MFMA (v_mfma_f64_4x4x4_4b_f64) on gfx950 -- its operand /
// accumulator lane maps (one-hot products, every (a-lane, b-lane) pair in one launch)
// and its issue rate against v_mfma_f64_16x16x4_f64. For the w units of the lattice
// step, whose 16-row A operand holds only k <= 8 live rows.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_mfma4.hip -o /tmp/probe_mfma4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

// wave p*64+q: a = one-hot at lane p (value 1), b = one-hot at lane q (value 1);
// out[(p*64+q)*64 + l] = c of lane l
// BC: the A broadcast (cbsz = 2: every block takes block abid's A)
template <int BC, int ABID>
__global__ void onehot_k(double* out) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  const int p = wv >> 6, q = wv & 63;
  const double a = l == p ? 1.0 : 0.0, b = l == q ? 1.0 : 0.0;
  const double c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, BC, ABID, 0);
  out[(size_t)wv * 64 + l] = c;
}

template <bool SMALL>
__global__ __launch_bounds__(256) void rate_k(double* out, long long* st, int iters) {
  const int l = threadIdx.x;
  const double a = 1.0 + 1e-9 * l, b = 1.0 - 1e-9 * l;
  long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
  if constexpr (SMALL) {
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0, c7 = 0;
    for (int i = 0; i < iters; i++) {
      c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c3, 0, 0, 0);
      c4 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c4, 0, 0, 0);
      c5 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c5, 0, 0, 0);
      c6 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c6, 0, 0, 0);
      c7 = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c7, 0, 0, 0);
    }
    s = c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7;
  } else {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    for (int i = 0; i < iters; i++) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    d4 t = c0 + c1 + c2 + c3;
    s = t[0] + t[1] + t[2] + t[3];
  }
  long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + l] = s;
  if (l == 0 && blockIdx.x == 0) {
    st[0] = t1 - t0;
    st[1] = r1 - r0;
  }
}

// random operands (per lane, from memory), 4 rotating values: the power / toggling
// state of a real GEMM (the 16x16x4 form ran faster on random data)
template <bool SMALL>
__global__ __launch_bounds__(256) void rate_rand_k(const double* __restrict__ rnd, double* out, int iters) {
  const int l = threadIdx.x;
  double a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = rnd[((blockIdx.x * 256 + l) * 8 + i) & ((1 << 20) - 1)];       // (the buffer holds 2^20)
    b[i] = rnd[((blockIdx.x * 256 + l) * 8 + 4 + i) & ((1 << 20) - 1)];
  }
  double s = 0.0;
  if constexpr (SMALL) {
    double c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = 0.0;
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[4 * i + j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], b[j], c[4 * i + j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s += c[i];
  } else {
    d4 c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[it & 3], b[j], c[j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  }
  out[blockIdx.x * 256 + l] = s;
}

// LDS-fed: per K4 step a wave reads its operands from LDS (random data) -- the
// 16x16x4 form one A and four B values per lane for 4 instructions (16 rows x 64
// columns), the 4x4x4 form four A and four B values for 16 instructions (the same
// 16 x 64 outputs)
template <bool SMALL>
__global__ __launch_bounds__(256) void rate_lds_k(const double* __restrict__ rnd, double* out, int iters) {
  __shared__ double sh[4096];
  const int l = threadIdx.x, lane = l & 63, w = l >> 6;
  for (int e = l; e < 4096; e += 256) sh[e] = rnd[(blockIdx.x * 4096 + e) & ((1 << 20) - 1)];
  __syncthreads();
  double s = 0.0;
  const double* A = sh + w * 1024;
  const double* B = sh + ((w + 1) & 3) * 1024;
  if constexpr (SMALL) {
    double c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = 0.0;
    for (int it = 0; it < iters; it++) {
      const int kk = ((it & 15) << 2) + (lane >> 4);
      double a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = A[kk * 16 + 4 * i + (lane & 3)];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = B[kk * 16 + ((lane + 16 * j) & 15) ];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[4 * i + j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], b[j], c[4 * i + j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) s += c[i];
  } else {
    d4 c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) c[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; it++) {
      const int kk = ((it & 15) << 2) + (lane >> 4);
      const double a = A[kk * 16 + (lane & 15)];
      double b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = B[kk * 16 + ((lane + 16 * j) & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[j], c[j], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  }
  out[blockIdx.x * 256 + l] = s;
}

int main() {
  int dev; CK(hipGetDevice(&dev)); hipDeviceProp_t pr; CK(hipGetDeviceProperties(&pr, dev));
  double* d; CK(hipMalloc(&d, sizeof(double) * 4096 * 64));
  long long* st; CK(hipMalloc(&st, 16));
  std::vector<double> h(4096 * 64);
  for (int v = 0; v < 3; ++v) {
    if (v == 0) onehot_k<0, 0><<<1024, 256>>>(d);
    else if (v == 1) onehot_k<2, 1><<<1024, 256>>>(d);
    else onehot_k<2, 3><<<1024, 256>>>(d);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, sizeof(double) * h.size(), hipMemcpyDeviceToHost));
    // every (a-lane p, b-lane q) whose product lands somewhere: "p q -> l"
    int n = 0;
    printf("variant %s\n", v == 0 ? "cbsz 0" : (v == 1 ? "cbsz 2 abid 1" : "cbsz 2 abid 3"));
    for (int p = 0; p < 64; ++p)
      for (int q = 0; q < 64; ++q)
        for (int l = 0; l < 64; ++l)
          if (h[(size_t)(p * 64 + q) * 64 + l] != 0.0) {
            printf("map a%d b%d -> c%d (%g)\n", p, q, l, h[(size_t)(p * 64 + q) * 64 + l]);
            ++n;
          }
    printf("products landing: %d\n", n);
  }
  const int nb = pr.multiProcessorCount * 4, iters = 4096;
  for (int small = 0; small < 2; ++small) {
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
    if (small) rate_k<true><<<nb, 256>>>(d, st, 64); else rate_k<false><<<nb, 256>>>(d, st, 64);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    if (small) rate_k<true><<<nb, 256>>>(d, st, iters); else rate_k<false><<<nb, 256>>>(d, st, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    long long cyc[2]; CK(hipMemcpy(cyc, st, 16, hipMemcpyDeviceToHost));
    // MACs per instruction: 4x4x4 x 4 blocks = 256; 16x16x4 = 1024
    const double macs = small ? (double)nb * 4 * iters * 8 * 256 : (double)nb * 4 * iters * 4 * 1024;
    printf("%s: %.3f ms, %.2f TF (2 flop per MAC), wave0 %.1f cycles per instruction, clock %.0f MHz\n",
           small ? "4x4x4_4b " : "16x16x4  ", ms, 2 * macs / ms / 1e9, (double)cyc[0] / iters / (small ? 8 : 4),
           100.0 * cyc[0] / (double)cyc[1]);
  }
  // random operands: registers, then LDS-fed
  double* rnd; CK(hipMalloc(&rnd, sizeof(double) * (1 << 20)));
  {
    std::vector<double> hr(1 << 20);
    unsigned x = 12345;
    for (auto& v : hr) { x = x * 1664525u + 1013904223u; v = 1.0 + (x >> 8) * (1.0 / 16777216.0); }
    CK(hipMemcpy(rnd, hr.data(), sizeof(double) * hr.size(), hipMemcpyHostToDevice));
  }
  for (int kind = 0; kind < 2; ++kind)
    for (int small = 0; small < 2; ++small) {
      hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); float ms;
      auto go = [&](int it) {
        if (kind == 0) { if (small) rate_rand_k<true><<<nb, 256>>>(rnd, d, it); else rate_rand_k<false><<<nb, 256>>>(rnd, d, it); }
        else { if (small) rate_lds_k<true><<<nb, 256>>>(rnd, d, it); else rate_lds_k<false><<<nb, 256>>>(rnd, d, it); }
      };
      go(64); CK(hipDeviceSynchronize());
      const int it = 2048;
      CK(hipEventRecord(e0)); go(it); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      // MACs per wave-iteration: 16 x 256 (4x4x4) or 4 x 1024 (16x16x4): 4096 either way
      const double macs = (double)nb * 4 * it * 4096;
      printf("%s %s: %.3f ms, %.2f TF\n", kind == 0 ? "random regs" : "random LDS ", small ? "4x4x4_4b" : "16x16x4 ",
             ms, 2 * macs / ms / 1e9);
    }
  return 0;
}
