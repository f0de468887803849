// Diagnostic: the lattice step's w-unit loop in isolation (the F stream and its
// MFMAs, no hand-offs): B GPs x U units per GP, grid (GP, unit) as in k_inc_lat,
// each unit an equal share of the GP's F in pair order (CUR = 1) or of a flat
// contiguous copy of the same bytes (CUR = 0); DEPTH steps in flight per wave;
// L21c loads agent-scope (SC1) or plain; F loads non-temporal (NTL) or plain.
// Build: hipcc --offload-arch=gfx950 -O3 -o build/probe_wloop tools/probe_wloop.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef double dv2 __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));

__host__ __device__ inline int64_t fblk_off(int64_t jb, int64_t ld) { return 64 * jb * ld - 2048 * jb * (jb - 1); }

template <int DEPTH, bool SC1, bool NTL, bool CUR>
__global__ __launch_bounds__(256) void k_wloop(const double* const* __restrict__ Fs, const double* const* __restrict__ Ls,
                                                double* out, int64_t n0, int64_t ld, int U) {
  const int64_t g = blockIdx.x, u = blockIdx.y;
  const double* F = Fs[g];
  const double* l21c = Ls[g];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, r = lane & 15, q = lane >> 4;
  const int64_t nwb = (n0 + 63) / 64, C = (n0 + 15) / 16;
  const int64_t K2 = 2 * C - 4 * (nwb - 1);
  const int64_t S = (nwb / 2) * K2 + (nwb & 1) * (C - 4 * (nwb / 2));
  const int64_t s0 = u * S / U, s1 = (u + 1) * S / U, T = s1 - s0;
  const int64_t p0 = s0 / K2, rem0 = s0 - p0 * K2;
  const bool odd0 = rem0 >= C - 4 * p0;
  struct Cur {
    int64_t jb, st, nb, p;
    bool odd;
  };
  Cur cl{odd0 ? nwb - 1 - p0 : p0, odd0 ? rem0 - (C - 4 * p0) : rem0, 0, p0, odd0};
  cl.nb = C - 4 * cl.jb;
  int64_t flat = s0;   // CUR = 0: step index into a contiguous run
  auto adv = [&](Cur& c) {
    if (++c.st == c.nb) {
      c.st = 0;
      if (c.odd) {
        ++c.p;
        c.jb = c.p;
      } else {
        c.jb = nwb - 1 - c.p;
      }
      c.odd = !c.odd;
      c.nb = C - 4 * c.jb;
    }
  };
  auto row_of = [&](const Cur& c) { return 64 * c.jb + 16 * c.st + 4 * w + q; };
  auto load = [&](dv2 (&f)[2], double& a) {
    const dv2* Fr;
    int64_t i;
    if (CUR) {
      i = row_of(cl);
      const int64_t ii = i < n0 ? i : n0 - 1;
      Fr = reinterpret_cast<const dv2*>(F + fblk_off(cl.jb, ld) + (ii - 64 * cl.jb) * 64 + 2 * r);
    } else {
      i = (flat * 16 + 4 * w + q) % n0;
      Fr = reinterpret_cast<const dv2*>(F + (flat * 16 + 4 * w + q) * 64 + 2 * r);
    }
    f[0] = NTL ? __builtin_nontemporal_load(Fr) : Fr[0];
    f[1] = NTL ? __builtin_nontemporal_load(Fr + 16) : Fr[16];
    const double* pa = l21c + (i < n0 ? i : n0 - 1) * 16 + r;
    a = SC1 ? __hip_atomic_load(pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *pa;
  };
  int64_t tl = 0;
  auto next = [&]() {
    if (tl + 1 < T) {
      adv(cl);
      ++flat;
      ++tl;
    }
  };
  d4 acc[4] = {};
  dv2 fb[DEPTH][2];
  double ab[DEPTH];
#pragma unroll
  for (int b = 0; b + 1 < DEPTH; ++b) {
    load(fb[b], ab[b]);
    next();
  }
  for (int64_t t0 = 0; t0 < T; t0 += DEPTH) {
#pragma unroll
    for (int b = 0; b < DEPTH; ++b) {
      const int64_t t = t0 + b;
      load(fb[(b + DEPTH - 1) % DEPTH], ab[(b + DEPTH - 1) % DEPTH]);
      next();
      const double av = t < T ? ab[b] : 0.0;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        acc[2 * hh] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, fb[b][hh].x, acc[2 * hh], 0, 0, 0);
        acc[2 * hh + 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, fb[b][hh].y, acc[2 * hh + 1], 0, 0, 0);
      }
    }
  }
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  if (s == -12345.0) out[0] = s;
}

__global__ void k_fill(double* p, int64_t n) {
  for (int64_t i = blockIdx.x * 256L + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5;
}
__global__ void k_pollute(const double* p, int64_t n, double* out) {
  double s = 0.0;
  for (int64_t i = blockIdx.x * 256L + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) s += p[i];
  if (s == -1.0) out[1] = s;
}

template <int DEPTH, bool SC1, bool NTL, bool CUR>
float run(const double* const* F, const double* const* l21, double* out, int B, int U, int64_t n0, int64_t ld,
          const double* pol = nullptr, int64_t npol = 0) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9f;
  for (int rep = 0; rep < 20; ++rep) {
    if (pol) k_pollute<<<1024, 256>>>(pol, npol, out);
    (void)hipEventRecord(e0, 0);
    k_wloop<DEPTH, SC1, NTL, CUR><<<dim3(B, U), 256>>>(F, l21, out, n0, ld, U);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 2 && ms < best) best = ms;
  }
  return best * 1e3f;
}

int main() {
  const int64_t n0 = 2040;
  const int Bmax = 8;
  double* out;
  (void)hipMalloc(&out, 64);
  const int64_t nwb = (n0 + 63) / 64, C = (n0 + 15) / 16;
  const double mb = (double)(nwb * C - 2 * nwb * (nwb - 1)) * 16 * 512 / 1e6;   // F bytes per GP (MB)
  const int64_t npol = 1L << 27;   // 1 GiB
  double* pol;
  (void)hipMalloc(&pol, 8 * npol);
  k_fill<<<4096, 256>>>(pol, npol);
  for (int64_t ld : {2048L, 3072L}) {
    double *Fh[Bmax], *Lh[Bmax];
    for (int g = 0; g < Bmax; ++g) {
      (void)hipMalloc(&Fh[g], sizeof(double) * fblk_off(ld / 64, ld));
      (void)hipMalloc(&Lh[g], sizeof(double) * ld * 16);
      k_fill<<<1024, 256>>>(Fh[g], fblk_off(ld / 64, ld));
      k_fill<<<64, 256>>>(Lh[g], ld * 16);
      double* junk;
      (void)hipMalloc(&junk, 64 << 20);   // other allocations between them
    }
    double **F, **L;
    (void)hipMalloc(&F, sizeof(double*) * Bmax);
    (void)hipMalloc(&L, sizeof(double*) * Bmax);
    (void)hipMemcpy(F, Fh, sizeof(Fh), hipMemcpyHostToDevice);
    (void)hipMemcpy(L, Lh, sizeof(Lh), hipMemcpyHostToDevice);
    for (int B : {8, 1}) {
      const int U = 256 / B;
      float t[6] = {run<6, true, true, true>(F, L, out, B, U, n0, ld),       run<6, true, false, true>(F, L, out, B, U, n0, ld),
                    run<6, true, true, true>(F, L, out, B, 2 * U, n0, ld),   run<6, true, false, true>(F, L, out, B, 2 * U, n0, ld),
                    run<6, true, false, true>(F, L, out, B, 2 * U, n0, ld, pol, npol / 8),
                    run<6, true, false, true>(F, L, out, B, 2 * U, n0, ld, pol, npol)};
      const char* nm[] = {"D6 nt", "D6 plain", "D6 2U nt", "D6 2U plain", "D6 2U plain +128MB", "D6 2U plain +1GB"};
      printf("ld %ld B %d U/GP %3d |", (long)ld, B, U);
      for (int i = 0; i < 6; ++i) printf(" %s %5.1f us %4.2f TB/s |", nm[i], t[i], B * mb / t[i]);
      printf("\n");
    }
  }
  return 0;
}
