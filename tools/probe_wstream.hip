// Diagnostic: the lattice step's F stream in isolation. B x 16.6 MB of F (B = 8:
// 133 MB) read once by NWG workgroups of 256 threads, each a contiguous share in
// 16 KB steps (lane: 64 bytes = four 16-byte loads per step), U steps in flight
// per wave, plain or non-temporal loads. Answers: what rate can a ~20-40 us
// stream of this size reach, and does it depend on the workgroup count, the
// depth in flight or the load kind.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/probe_wstream tools/probe_wstream.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double dv2 __attribute__((ext_vector_type(2)));

template <int U, bool NTL>
__global__ __launch_bounds__(256) void k_w(const dv2* __restrict__ src, double* out, long per_wg) {
  const int tid = threadIdx.x;
  const dv2* p = src + blockIdx.x * per_wg;
  double acc = 0.0;
  // step = 1024 dv2 (16 KiB): lane tid reads dv2 tid, tid + 256, tid + 512, tid + 768
  for (long s = 0; s < per_wg; s += 1024L * U) {
    dv2 v[4 * U];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long e = s + 1024L * u + 256 * j + tid;
        const long ee = e < per_wg ? e : per_wg - 1;
        v[4 * u + j] = NTL ? __builtin_nontemporal_load(p + ee) : p[ee];
      }
#pragma unroll
    for (int u = 0; u < 4 * U; ++u) acc += v[u].x * v[u].y;
  }
  if (acc == -1.0) out[0] = acc;
}

// the w unit's loop shape: 512-byte rows, a 16-row step gives wave w rows 4 w + q,
// lane (r, q) the 16-byte pairs r and 16 + r of its row; RG steps per batch, two
// batches in flight; f64 MFMA 16x16x4 on each pair (A from a small table: plain
// or agent-scope atomic loads)
typedef double d4 __attribute__((ext_vector_type(4)));
template <int RG, bool NTL, bool SC1>
__global__ __launch_bounds__(256) void k_wl(const dv2* __restrict__ src, const double* __restrict__ tab, double* out,
                                            long rows_per_wg) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, q = lane >> 4;
  const long row0 = blockIdx.x * rows_per_wg;
  const long T = rows_per_wg / (16 * RG);
  d4 acc[4] = {};
  auto ld = [&](long t, dv2 (&f)[RG][2], double (&a)[RG]) {
#pragma unroll
    for (int x = 0; x < RG; ++x) {
      const long i = row0 + 16 * RG * t + 16 * x + 4 * w + q;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const dv2* pp = src + i * 32 + 16 * hh + r;
        f[x][hh] = NTL ? __builtin_nontemporal_load(pp) : *pp;
      }
      const double* pa = tab + ((i & 4095) * 16 + r);
      a[x] = SC1 ? __hip_atomic_load(pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *pa;
    }
  };
  auto cmp = [&](const dv2 (&f)[RG][2], const double (&a)[RG]) {
#pragma unroll
    for (int x = 0; x < RG; ++x)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        acc[2 * hh] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], f[x][hh].x, acc[2 * hh], 0, 0, 0);
        acc[2 * hh + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], f[x][hh].y, acc[2 * hh + 1], 0, 0, 0);
      }
  };
  dv2 fA[RG][2], fB[RG][2];
  double aA[RG], aB[RG];
  ld(0, fA, aA);
  for (long t = 0; t < T; t += 2) {
    ld(t + 1 < T ? t + 1 : T - 1, fB, aB);
    cmp(fA, aA);
    if (t + 1 >= T) break;
    ld(t + 2 < T ? t + 2 : T - 1, fA, aA);
    cmp(fB, aB);
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == -1.0) out[0] = s;
}

template <int RG, bool NTL, bool SC1>
float run_wl(const dv2* buf, const double* tab, double* out, long bytes, int nwg) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long rows = bytes / 512 / nwg / (16 * RG) * (16 * RG);
  float best = 1e9f;
  for (int rep = 0; rep < 20; ++rep) {
    hipEventRecord(e0, 0);
    k_wl<RG, NTL, SC1><<<nwg, 256>>>(buf, tab, out, rows);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep > 2 && ms < best) best = ms;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best * (double)bytes / (rows * 512.0 * nwg);   // scaled to the whole size
}

template <int U, bool NTL>
float run(const dv2* buf, double* out, long n, int nwg) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const long per = n / nwg;
  float best = 1e9f;
  for (int rep = 0; rep < 20; ++rep) {
    hipEventRecord(e0, 0);
    k_w<U, NTL><<<nwg, 256>>>(buf, out, per);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep > 2 && ms < best) best = ms;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best;
}

int main() {
  const long nmax = 1L << 26;   // dv2: 1 GiB
  dv2* buf;
  double* out;
  hipMalloc(&buf, nmax * 16);
  hipMalloc(&out, 64);
  hipMemset(buf, 0, nmax * 16);
  const long sizes[] = {133L << 20, 1L << 30};
  for (long bytes : sizes) {
    const long n = bytes / 16;
    for (int nwg : {256, 512, 1024, 2048}) {
      float t[6] = {run<1, true>(buf, out, n, nwg), run<2, true>(buf, out, n, nwg), run<4, true>(buf, out, n, nwg),
                    run<1, false>(buf, out, n, nwg), run<2, false>(buf, out, n, nwg), run<4, false>(buf, out, n, nwg)};
      printf("%5ld MB nwg %4d |", bytes >> 20, nwg);
      const char* nm[] = {"nt U1", "nt U2", "nt U4", "pl U1", "pl U2", "pl U4"};
      for (int i = 0; i < 6; ++i) printf(" %s %6.1f us %5.2f TB/s |", nm[i], t[i] * 1e3, bytes / (t[i] * 1e-3) / 1e12);
      printf("\n");
    }
  }
  double* tab;
  hipMalloc(&tab, 4096 * 16 * 8);
  hipMemset(tab, 0, 4096 * 16 * 8);
  for (int nwg : {256, 272, 512, 1024}) {
    const long bytes = 133L << 20;
    float t[5] = {run_wl<2, true, true>(buf, tab, out, bytes, nwg), run_wl<2, false, true>(buf, tab, out, bytes, nwg),
                  run_wl<2, true, false>(buf, tab, out, bytes, nwg), run_wl<1, true, true>(buf, tab, out, bytes, nwg),
                  run_wl<4, true, true>(buf, tab, out, bytes, nwg)};
    const char* nm[] = {"RG2 nt sc1", "RG2 pl sc1", "RG2 nt pl", "RG1 nt sc1", "RG4 nt sc1"};
    printf("w-like 133 MB nwg %4d |", nwg);
    for (int i = 0; i < 5; ++i) printf(" %s %6.1f us %5.2f TB/s |", nm[i], t[i] * 1e3, bytes / (t[i] * 1e-3) / 1e12);
    printf("\n");
  }
  return 0;
}
