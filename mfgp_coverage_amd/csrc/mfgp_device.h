// Device-side helpers shared by the HIP translation units of libmfgp_hip.so
// (mfgp_kernels.hip, mfgp_nlml.hip): f64 MFMA tile products, LDS tile staging,
// the SE kernel in the reference's operation order (gaussian_process.py:66-79)
// and the K entries of gp:253-254 / gp:523-529.
#pragma once
#include <climits>
#include <hip/hip_runtime.h>

#include "mfgp_internal.h"

namespace mfgp {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double dv2 __attribute__((ext_vector_type(2)));
typedef float fv2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// Generic -> global address space, so loads/stores through descriptor pointers
// are emitted as global_* (vmcnt only) instead of flat_* (vmcnt + lgkmcnt).
#define GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GLOBAL T* gp(T* p) {
  return (GLOBAL T*)p;
}
template <class T>
__device__ __forceinline__ const GLOBAL T* gp(const T* p) {
  return (const GLOBAL T*)p;
}

__device__ __forceinline__ int swz(int k, int i) { return k * NB + (i ^ ((k & 1) << 4)); }

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// v_mfma_f64_4x4x4_4b_f64: four independent 4 x 4 x 4 blocks; lane l = 16 k + 4 blk + r
// holds A_blk[r][k] and B_blk[k][r], and C lane 16 i + 4 blk + j holds C_blk[i][j]
// (tools/probe_mfma4.hip, one-hot products); 1.64x the multiply-adds per cycle of
// the 16x16x4 form on gfx950
__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// exact f32 (v_mfma_f32_16x16x4_f32 = an fmaf chain). A/B lane maps as the f64
// form; C/D: lane (r, g) register v holds row 4g + v, column r (the f64 form:
// row g + 4v).
__device__ __forceinline__ f4 mfma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Per-wave 32x32 accumulator = 2x2 MFMA tiles of 16x16.
struct Acc {
  d4 c[2][2];
};

__device__ __forceinline__ void acc_zero(Acc& a) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) a.c[m][n] = d4{0.0, 0.0, 0.0, 0.0};
}

// acc (+/-)= A[64x64] * B[64x64] restricted to this wave's 32x32 output block.
// As[swz(k,i)] = A[i][k], Bs[swz(k,j)] = B[k][j].
template <bool NEG>
__device__ __forceinline__ void tile_mma(const double* __restrict__ As, const double* __restrict__ Bs,
                                         Acc& acc, int wm, int wn, int lane) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll 4
  for (int k0 = 0; k0 < NB; k0 += 4) {
    const int k = k0 + q;
    double a0 = As[swz(k, wm * 32 + r)];
    double a1 = As[swz(k, wm * 32 + 16 + r)];
    const double b0 = Bs[swz(k, wn * 32 + r)];
    const double b1 = Bs[swz(k, wn * 32 + 16 + r)];
    if (NEG) {
      a0 = -a0;
      a1 = -a1;
    }
    acc.c[0][0] = mfma(a0, b0, acc.c[0][0]);
    acc.c[0][1] = mfma(a0, b1, acc.c[0][1]);
    acc.c[1][0] = mfma(a1, b0, acc.c[1][0]);
    acc.c[1][1] = mfma(a1, b1, acc.c[1][1]);
  }
}

// Ts[swz(k,i)] = G[(c0+k)*ld + r0 + i], k,i in [0,64): a column-major 64x64 tile,
// each source column becoming one k-row. 16-byte loads, coalesced along i.
__device__ __forceinline__ void load_tile_cm(double* __restrict__ Ts, const double* __restrict__ G,
                                             int64_t ld, int64_t r0, int64_t c0, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int k = p * 8 + (tid >> 5);
    const int i = (tid & 31) * 2;
    const dv2 v = *reinterpret_cast<const GLOBAL dv2*>(gp(G) + (c0 + k) * ld + r0 + i);
    *reinterpret_cast<dv2*>(Ts + swz(k, i)) = v;
  }
}

// Register staging of a column-major 64x64 tile (issue-early / write-late):
// fetch_tile_cm issues the 8 16-byte global loads per thread; store_tile writes
// them to the swizzled k-major LDS image once the buffer is free.
struct Stage {
  dv2 v[8];
};

__device__ __forceinline__ void fetch_tile_cm(Stage& st, const double* __restrict__ G, int64_t ld, int64_t r0,
                                              int64_t c0, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int k = p * 8 + (tid >> 5);
    const int i = (tid & 31) * 2;
    st.v[p] = *reinterpret_cast<const GLOBAL dv2*>(gp(G) + (c0 + k) * ld + r0 + i);
  }
}

__device__ __forceinline__ void store_tile(double* __restrict__ Ts, const Stage& st, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int k = p * 8 + (tid >> 5);
    const int i = (tid & 31) * 2;
    *reinterpret_cast<dv2*>(Ts + swz(k, i)) = st.v[p];
  }
}

// stage one 64x64 operand tile through registers (8 16-byte loads per thread)
struct TileRegs {
  dv2 v[8];
};
__device__ __forceinline__ void tile_fetch(TileRegs& t, const double* __restrict__ G, int64_t ld, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) t.v[p] = *reinterpret_cast<const GLOBAL dv2*>(gp(G) + (p * 8 + (tid >> 5)) * ld + (tid & 31) * 2);
}
// the tile's memory rows become k-rows: Ts[swz(k, i)] = G[k * ld + i]
__device__ __forceinline__ void tile_put_k(double* __restrict__ Ts, const TileRegs& t, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int k = p * 8 + (tid >> 5), i = (tid & 31) * 2;
    *reinterpret_cast<dv2*>(Ts + swz(k, i)) = t.v[p];
  }
}
// transposed: Ts[swz(k, i)] = G[i * ld + k]
__device__ __forceinline__ void tile_put_t(double* __restrict__ Ts, const TileRegs& t, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int i = p * 8 + (tid >> 5), k = (tid & 31) * 2;
    Ts[swz(k, i)] = t.v[p].x;
    Ts[swz(k + 1, i)] = t.v[p].y;
  }
}

constexpr int PW = 128;                  // row width of the predict L image (= PRB)
typedef __attribute__((address_space(3))) void* lds_vptr;

__device__ __forceinline__ int swzp(int k, int i) { return k * PW + (i ^ ((k & 1) << 4)); }

// DMA kn rows of 128 doubles into a swizzled [kn][128] LDS image:
// dst[swzp(k, i)] = G[(c0 + k) * ld + r0 + i]. One wave-instruction moves one 1 KB row.
__device__ __forceinline__ void dma_rows128(double* dst, const double* __restrict__ G, int64_t ld, int64_t r0,
                                            int64_t c0, int kn, int w, int lane) {
  for (int k = w; k < kn; k += PNT / 64) {
    const int i = (2 * lane) ^ ((k & 1) << 4);
    const double* src = G + (c0 + k) * ld + r0 + i;
    __builtin_amdgcn_global_load_lds((const GLOBAL void*)src, (lds_vptr)(dst + k * PW), 16, 0, 0);
  }
}

// DMA kn rows of 64 doubles into a swizzled [kn][64] LDS image:
// dst[swz(k, i)] = G[(c0 + k) * ld + r0 + i]. One wave-instruction moves two rows.
__device__ __forceinline__ void dma_rows64(double* dst, const double* __restrict__ G, int64_t ld, int64_t r0,
                                           int64_t c0, int kn, int w, int lane) {
  for (int p = w; p < kn / 2; p += PNT / 64) {
    const int k = 2 * p + (lane >> 5);
    const int i = ((lane & 31) * 2) ^ ((k & 1) << 4);
    const double* src = G + (c0 + k) * ld + r0 + i;
    __builtin_amdgcn_global_load_lds((const GLOBAL void*)src, (lds_vptr)(dst + 2 * p * NB), 16, 0, 0);
  }
}

__device__ __forceinline__ void vm_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// C/D element (mt, nt, v) of this lane <-> tile (row, col).
__device__ __forceinline__ int acc_row(int wm, int mt, int q, int v) { return wm * 32 + mt * 16 + q + 4 * v; }
__device__ __forceinline__ int acc_col(int wn, int nt, int r) { return wn * 32 + nt * 16 + r; }

// ---------------------------------------------------------------------------
// Squared-exponential kernel, gaussian_process.py:66-79, in the reference's
// operation order: scale each coordinate by the length scale (a division),
// subtract, square, sum over D = 2, exp(-0.5 * .), times the output scale.
// No FMA contraction, so the rounding matches NumPy's elementwise ops.
// ---------------------------------------------------------------------------
__device__ __forceinline__ double se_scaled(double ax, double ay, double bx, double by, double s) {
#pragma clang fp contract(off)
  const double dx = ax - bx;
  const double dy = ay - by;
  const double d2 = dx * dx + dy * dy;
  return s * exp(-0.5 * d2);
}

__device__ __forceinline__ double div_(double a, double b) {
#pragma clang fp contract(off)
  return a / b;
}

// K entry (i, j), both < N, jitter and noise included (gp:253-254 / gp:523-529).
// pi / pj: the rows' coordinates (x, y).
__device__ __forceinline__ double k_entry_pts(const Hyp& h, int64_t NL, int64_t gi, const double* pi, int64_t gj,
                                              const double* pj) {
#pragma clang fp contract(off)
  const double xi = pi[0], yi = pi[1];
  const double xj = pj[0], yj = pj[1];
  const double kl = se_scaled(div_(xi, h.lL), div_(yi, h.lL), div_(xj, h.lL), div_(yj, h.lL), h.sL);
  double v;
  if (h.kind == 0) {
    v = kl;
    if (gi == gj) v = (v + h.noiseL) + h.jitter;
  } else {
    const bool li = gi < NL, lj = gj < NL;
    if (li && lj) {
      v = kl;                                            // K_LL (gp:523)
      if (gi == gj) v = (v + h.noiseL) + h.jitter;
    } else if (li != lj) {
      v = h.rho * kl;                                    // K_LH (gp:524)
    } else {
      const double kh = se_scaled(div_(xi, h.lH), div_(yi, h.lH), div_(xj, h.lH), div_(yj, h.lH), h.sH);
      v = h.rho2 * kl + kh;                              // K_HH (gp:525-526)
      if (gi == gj) v = (v + h.noiseH) + h.jitter;
    }
  }
  return v;
}
__device__ __forceinline__ double k_entry(const Hyp& h, const double* __restrict__ X, int64_t NL, int64_t gi,
                                          int64_t gj) {
  return k_entry_pts(h, NL, gi, X + 2 * gi, gj, X + 2 * gj);
}

__device__ __forceinline__ void tri_index(int64_t t, int& I, int& J) {
  int i = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
  while ((int64_t)(i + 1) * (i + 2) / 2 <= t) ++i;
  while ((int64_t)i * (i + 1) / 2 > t) --i;
  I = i;
  J = (int)(t - (int64_t)i * (i + 1) / 2);
}

}  // namespace mfgp
