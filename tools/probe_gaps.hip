// Diagnostic: gaps between dependent kernels on one stream, by launch shape.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_gaps tools/probe_gaps.hip
// Run under rocprofv3 --kernel-trace and read start/end timestamps per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_tiny(double* p) {
  if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

template <int LDSD>
__global__ __launch_bounds__(256) void k_wide(double* p, int iters) {
  __shared__ double s[LDSD];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  double a = s[(threadIdx.x + 1) & 255];
  for (int i = 0; i < iters; ++i) a = a * 1.0000001 + 1e-9;
  if (a == -1.0) p[blockIdx.x] = a;
}

typedef double dv2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_stream(const dv2* __restrict__ src, double* out, long n) {
  double acc = 0.0;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    dv2 v = __builtin_nontemporal_load(src + i);
    acc += v.x + v.y;
  }
  if (acc == -1.0) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_write(double* dst, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = (double)i;
}

int main() {
  double *p, *big, *w;
  hipMalloc(&p, 1 << 20);
  const long n2 = 1L << 27;   // 2 GiB of double2
  hipMalloc(&big, n2 * 16);
  hipMemset(big, 0, n2 * 16);
  hipMalloc(&w, 16L << 20);
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int rep = 0; rep < 20; ++rep) {
    k_tiny<<<1, 64, 0, s>>>(p);
    k_tiny<<<1, 64, 0, s>>>(p);
    k_wide<4880><<<2048, 256, 0, s>>>(p, 10);       // 39 KB LDS, short
    k_tiny<<<1, 64, 0, s>>>(p);
    k_wide<256><<<2048, 256, 0, s>>>(p, 10);        // little LDS
    k_tiny<<<1, 64, 0, s>>>(p);
    k_stream<<<2048, 256, 0, s>>>(reinterpret_cast<const dv2*>(big), p, n2);
    k_tiny<<<1, 64, 0, s>>>(p);
    k_write<<<2048, 256, 0, s>>>(w, 2L << 20);       // 16 MB of dirty lines
    k_tiny<<<1, 64, 0, s>>>(p);
    k_wide<256><<<64, 256, 0, s>>>(p, 10);
    k_tiny<<<1, 64, 0, s>>>(p);
  }
  hipStreamSynchronize(s);
  printf("done\n");
  return 0;
}
