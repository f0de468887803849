// HIP kernels of the GP posterior update for gfx950 (MI355X), fp64.
//
// Reference path (MSU-dcypherlab/mfgp-coverage, gaussian_process.py):
//   k_assemble    <- kernel(X,X) + sigma_n I + jitter I, SF gp:253-254, MF gp:523-529
//                    (+ one augmented row r = y - m so the factor also yields z = L^-1 r)
//   k_potrf_diag  \
//   k_panel        > np.linalg.cholesky (gp:254, gp:529), blocked right-looking, NB = 64,
//   k_syrk        /  with the explicit inverse of every diagonal block kept for the solves
//   k_predict     <- predict (gp:121-148 / gp:401-438): psi = k(X*,X) generated in registers,
//                    V = L^-1 psi^T by blocked forward substitution on f64 MFMA, and the
//                    epilogue mu = m + V^T z (= m + psi alpha), var = k** - colsum(V o V)
//                    (= diag(k** - psi K^-1 psi^T)); the M x M matrices of the reference
//                    are never formed.
//
// Matrices are column-major; 64x64 operand tiles are staged "k-major" in LDS,
// As[k][i], with an XOR swizzle of bit 4 of the column on odd k so that the
// ds_read_b64 fragment loads of v_mfma_f64_16x16x4f64 are bank-conflict free.
// f64 MFMA fragment maps (pinned on the hardware by tools/probe_mfma_f64.hip):
//   A[i][k]: lane l holds A[l&15][l>>4];  B[k][j]: lane l holds B[l>>4][l&15];
//   C/D:     lane l, reg v holds C[(l>>4) + 4v][l&15].
#include <climits>
#include <cstring>
#include "mfgp_internal.h"
#include "mfgp_device.h"

namespace mfgp {

// Diagnostic phase stamps (tools/bench_diag.hip builds with -DMFGP_STAMPS); no-op otherwise.
#ifdef MFGP_STAMPS
__device__ long long* g_stamps;
#define STAMP(id)                                                                        \
  do {                                                                                   \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_stamps[id] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(id) \
  do {            \
  } while (0)
#endif
// k_inc_stream timeline stamps (GP 0 only; diagnostic builds)
#ifdef MFGP_STAMPS
#define FSTAMP(id)                                                                                 \
  do {                                                                                             \
    if (threadIdx.x == 0 && blockIdx.x == 0)                                                       \
      atomicMax((unsigned long long*)&g_stamps[id], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
  } while (0)
// per-workgroup k_inc_stream trace: g_stamps[64 + 8 * (linear WG id) + slot]
#define WTRACE(slot)                                                                                 \
  do {                                                                                               \
    if (threadIdx.x == 0) {                                                                          \
      long long* wt_ = g_stamps + 64 + 8 * (blockIdx.y * gridDim.x + blockIdx.x);                     \
      wt_[slot] = __builtin_amdgcn_s_memrealtime();                                                  \
      if ((slot) == 0)                                                                               \
        wt_[7] = ((long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32) |                       \
                 (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));                                \
    }                                                                                                \
  } while (0)
// the lattice step's second launch (k_lat_gemm2/3): its workgroups at role 1024 + tile
#define WTRACE2(slot)                                                                                \
  do {                                                                                               \
    if (threadIdx.x == 0) {                                                                          \
      long long* wt_ = g_stamps + 64 + 8 * ((1024 + blockIdx.y) * gridDim.x + blockIdx.x);                       \
      wt_[slot] = __builtin_amdgcn_s_memrealtime();                                                  \
      if ((slot) == 0)                                                                               \
        wt_[7] = ((long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32) |                       \
                 (unsigned)__builtin_amdgcn_s_getreg(4 | (31 << 11));                                \
    }                                                                                                \
  } while (0)
#else
#define FSTAMP(id) \
  do {             \
  } while (0)
#define WTRACE(slot) \
  do {               \
  } while (0)
#define WTRACE2(slot) \
  do {                \
  } while (0)
#endif
#ifndef MFGP_SPIN_SLEEP
#define MFGP_SPIN_SLEEP 16
#endif

// (shared device helpers: mfgp_device.h)

// ---------------------------------------------------------------------------
// Assembly: lower-triangular tiles of the augmented matrix
//   [ K + (sigma_n + jitter) I   .  ]   rows 0..N-1
//   [ (y - m)^T                  1  ]   row N  (its pivot is forced to 1)
//   [ 0                          I  ]   padding up to a multiple of NB
// Grid (tiles, batch); 256 threads; thread -> (row i = tid & 63, column group).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(NT) void k_assemble(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t N = d.N, NL = d.NL, ld = d.ld;
  const int64_t T = nblocks_factor(N);
  const int64_t t = blockIdx.x;
  if (t == 0 && threadIdx.x == 0) *d.status = INT_MAX;
  if (t >= T * (T + 1) / 2) return;
  int I, J;
  tri_index(t, I, J);
  const Hyp& h = d.hf;
  const int i = threadIdx.x & 63;
  const int64_t gi = (int64_t)I * NB + i;
  double* __restrict__ A = d.A;
  for (int jj = threadIdx.x >> 6; jj < NB; jj += 4) {
    const int64_t gj = (int64_t)J * NB + jj;
    double v;
    if (gj > gi) {
      v = 0.0;
    } else if (gi < N) {
      v = k_entry(h, d.X, NL, gi, gj);
    } else if (gi == N && gj < N) {
      // residual y - m (gp:133 SF; gp:419-421 MF): lofi rows use mean_L, hifi mean_H
      const double m = (h.kind == 1 && gj < NL) ? h.meanL : h.meanH;
      v = d.y[gj] - m;
    } else {
      v = (gi == gj) ? 1.0 : 0.0;
    }
    A[gj * ld + gi] = v;
  }
}

// ---------------------------------------------------------------------------
// Diagonal block kb: Cholesky of the 64x64 tile and the explicit inverse of its
// factor, blocked in 16x16 sub-blocks so the serial part is four 16-step chains:
//   for each 16-column sub-block: (a) wave 0 factors the 16x16 diagonal block
//   (lane r owns row r in registers, column broadcasts by v_readlane) and inverts
//   it (lane c solves column c); (b) the sub-panel below is multiplied by that
//   inverse; (c) the trailing sub-matrix is updated -- (b) and (c) by all 256
//   threads. Then Linv's off-diagonal 16x16 blocks follow by block substitution.
// Rows >= N (the augmented row and padding) get pivot 1; a non-positive pivot
// on a real row is recorded in *status (LAPACK potrf's INFO, which NumPy turns
// into LinAlgError, gp:254 / gp:529) and replaced by 1 to keep the batch finite.
// ---------------------------------------------------------------------------
constexpr int SP = NB + 1;   // padded row stride of the row-major LDS tiles
constexpr int DB = 16;       // sub-block
constexpr int DP = DB + 1;

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Broadcast lane k of each 16-lane DPP row to the whole row (row_newbcast:k, gfx90a+):
// one v_mov_b64 with a 64-bit DPP source. The DPP control must be an immediate: the
// switch folds away once the callers' fully unrolled loops make k a constant.
// (s_nop 1: a DPP source written by the previous VALU instruction needs two wait
// states, which the compiler does not count for inline assembly.)
template <int K>
__device__ __forceinline__ double bcast16_(double v) {
  double r;
  asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "i"(K));
  return r;
}
// acc + (lane k's src) * mul (NEG: - ...), one v_fmac_f64 whose first source is the
// row_newbcast:k DPP operand: a pivot chain's rank-1 update step, or a substitution
// step, without a separate broadcast (fused multiply-add: the same rounding as
// acc - b * mul written out)
template <int K, bool NEG>
__device__ __forceinline__ double fmac_bcast16_(double acc, double src, double mul) {
  if (NEG)
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "i"(K));
  else
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc) : "v"(src), "v"(mul), "i"(K));
  return acc;
}
#define MFGP_BCAST16_CASES(F) \
  F(0) F(1) F(2) F(3) F(4) F(5) F(6) F(7) F(8) F(9) F(10) F(11) F(12) F(13) F(14)
__device__ __forceinline__ double bcast16(double v, int k) {
  switch (k) {
#define C_(K) case K: return bcast16_<K>(v);
    MFGP_BCAST16_CASES(C_)
#undef C_
    default: return bcast16_<15>(v);
  }
}
template <bool NEG>
__device__ __forceinline__ double fmac_bcast16(double acc, double src, double mul, int k) {
  switch (k) {
#define C_(K) case K: return fmac_bcast16_<K, NEG>(acc, src, mul);
    MFGP_BCAST16_CASES(C_)
#undef C_
    default: return fmac_bcast16_<15, NEG>(acc, src, mul);
  }
}

// 16x16 f64 MFMA block product on LDS operands: acc (+/-)= A[16xK] * B[Kx16] with
// A[i][k] = A[i*ars + k*acs], B[k][j] = B[k*brs + j*bcs].
template <bool NEG>
__device__ __forceinline__ d4 mfma16(const double* __restrict__ A, int ars, int acs, const double* __restrict__ B,
                                     int brs, int bcs, int K, d4 acc, int lane) {
  const int r = lane & 15, q = lane >> 4;
  for (int k0 = 0; k0 < K; k0 += 4) {
    double a = A[r * ars + (k0 + q) * acs];
    if (NEG) a = -a;
    acc = mfma(a, B[(k0 + q) * brs + r * bcs], acc);
  }
  return acc;
}

// S: 64x64 row-major (stride SP), lower triangle = the matrix. On exit S = L
// (zeros above the diagonal) and R = L^-1 (row-major, zeros above).
__device__ void factor_invert_64(double* __restrict__ S, double* __restrict__ R,
                                 double* __restrict__ U, int64_t g0, int64_t N, int* status) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r16 = lane & 15, q16 = lane >> 4;
  for (int kk = 0; kk < NB / DB; ++kk) {
    const int o = kk * DB;
    if (w == 0) {
      // (a) factor the 16x16 diagonal block in registers: lane r holds row o+(r&15)
      //     (the four 16-lane DPP rows of the wave hold identical copies); column
      //     values are broadcast inside each DPP row with row_newbcast, so no
      //     SGPR/LDS round trip sits on the pivot chain. LAPACK dpotf2 order:
      //     pivot = sqrt(a_jj), column scaled by 1/pivot.
      double d[DB];
#pragma unroll
      for (int c = 0; c < DB; ++c) d[c] = S[(o + r16) * SP + o + c];
      double rdiag = 1.0;
      int fail = INT_MAX;
#pragma unroll
      for (int j = 0; j < DB; ++j) {
        double p = bcast16(d[j], j);
        const int64_t g = g0 + o + j;
        const bool pad = g >= N;
        const bool bad = !pad && !(p > 0.0);
        fail = bad ? min(fail, (int)(g + 1)) : fail;
        p = (pad || bad) ? 1.0 : p;
        const double rs = rsqrt(p);
        const double l = (r16 >= j) ? (r16 == j ? p : d[j]) * rs : 0.0;
        rdiag = (r16 == j) ? rs : rdiag;
        d[j] = l;
        // d[k] -= l_r l_k for every row r: rows r > j are the update; rows r < j have
        // l_r = 0; row j's columns k > j are above the diagonal (never read: the
        // store below and the substitution read columns <= the row)
#pragma unroll
        for (int k = j + 1; k < DB; ++k) d[k] = fmac_bcast16<true>(d[k], l, l, k);
      }
      if (fail != INT_MAX && lane == 0) atomicMin(status, fail);
      if (lane < DB) {
#pragma unroll
        for (int c = 0; c < DB; ++c) S[(o + lane) * SP + o + c] = (c <= lane) ? d[c] : 0.0;
      }
      // inverse of the 16x16 factor: lane c solves column c = r16 by forward
      // substitution; L[i][m] is register m of DPP-row lane i.
      double x[DB];
#pragma unroll
      for (int i = 0; i < DB; ++i) {
        double s0 = (i == r16) ? 1.0 : 0.0, s1 = 0.0;
#pragma unroll
        for (int m = 0; m < i; ++m) {   // s -= L[i][m] x[m]
          if (m & 1) s1 = fmac_bcast16<true>(s1, d[m], x[m], i);
          else s0 = fmac_bcast16<true>(s0, d[m], x[m], i);
        }
        x[i] = (s0 + s1) * bcast16(rdiag, i);
      }
      // column c of Dinv (zero above the diagonal) into R's diagonal block
      if (lane < DB) {
#pragma unroll
        for (int i = 0; i < DB; ++i) R[(o + i) * SP + o + lane] = x[i];
      }
    } else if (kk == 0) {
      // the other waves meanwhile: R's blocks above the diagonal are zero
      for (int e = tid - 64; e < 6 * DB * DB; e += NT - 64) {
        const int b = e >> 8, i = (e >> 4) & 15, j = e & 15;   // blocks (0,1..3), (1,2..3), (2,3)
        const int I = b < 3 ? 0 : (b < 5 ? 1 : 2), J = b < 3 ? b + 1 : (b < 5 ? b - 1 : 3);
        R[(I * DB + i) * SP + J * DB + j] = 0.0;
      }
    }
    __syncthreads();
    STAMP(2 + 3 * kk);
    const int nrest = NB / DB - 1 - kk;   // 16-row blocks below the diagonal block
    // (b) sub-panel P = A_sub * Dinv^T, one 16x16 block per wave (MFMA)
    if (w < nrest) {
      const int R0 = o + DB + DB * w;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = mfma16<false>(S + R0 * SP + o, SP, 1, R + o * SP + o, 1, SP, DB, acc, lane);   // B[k][j] = Dinv[j][k]
#pragma unroll
      for (int v = 0; v < 4; ++v) S[(R0 + q16 + 4 * v) * SP + o + r16] = acc[v];
    }
    __syncthreads();
    STAMP(3 + 3 * kk);
    // (c) trailing update of the lower 16x16 blocks of rows/cols [o+16, 64) (MFMA)
    for (int t = w; t < nrest * (nrest + 1) / 2; t += NT / 64) {
      int bi = 0;
      while ((bi + 1) * (bi + 2) / 2 <= t) ++bi;
      const int bj = t - bi * (bi + 1) / 2;
      const int R0 = o + DB + DB * bi, C0 = o + DB + DB * bj;
      d4 acc;
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[v] = S[(R0 + q16 + 4 * v) * SP + C0 + r16];
      acc = mfma16<true>(S + R0 * SP + o, SP, 1, S + C0 * SP + o, 1, SP, DB, acc, lane);
#pragma unroll
      for (int v = 0; v < 4; ++v) S[(R0 + q16 + 4 * v) * SP + C0 + r16] = acc[v];
    }
    __syncthreads();
    STAMP(4 + 3 * kk);
  }
  // Linv: the diagonal blocks are in R (and the blocks above them zero); block rows
  // I = 1..3 by substitution:
  //   Linv_IJ = -Dinv_I * sum_{m=J}^{I-1} L_Im Linv_mJ      (MFMA, wave w -> J = w)
  STAMP(14);
  for (int I = 1; I < NB / DB; ++I) {
    if (w < I) {
      const int J = w;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
      acc = mfma16<false>(S + (I * DB) * SP + J * DB, SP, 1, R + (J * DB) * SP + J * DB, SP, 1, (I - J) * DB, acc,
                          lane);
      double* Uj = U + J * DB * DP;
#pragma unroll
      for (int v = 0; v < 4; ++v) Uj[(q16 + 4 * v) * DP + r16] = acc[v];
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      d4 acc2 = {0.0, 0.0, 0.0, 0.0};
      acc2 = mfma16<true>(R + (I * DB) * SP + I * DB, SP, 1, Uj, DP, 1, DB, acc2, lane);   // Dinv_I
#pragma unroll
      for (int v = 0; v < 4; ++v) R[(I * DB + q16 + 4 * v) * SP + J * DB + r16] = acc2[v];
    }
    __syncthreads();
    STAMP(14 + I);
  }
}

__global__ __launch_bounds__(NT) void k_potrf_diag(const GPDesc* __restrict__ descs, int kb) {
  const GPDesc& d = descs[blockIdx.x];
  const int64_t N = d.N, ld = d.ld;
  if (kb >= nblocks_factor(N)) return;
  __shared__ double sh[2 * NB * SP + (NB / DB - 1) * DB * DP];
  double* const S = sh;
  double* const R = sh + NB * SP;
  double* const U = R + NB * SP;
  const int tid = threadIdx.x;
  const int64_t o = (int64_t)kb * NB;
  double* __restrict__ A = d.A;
  STAMP(0);
  {
    // unconditional loads (the upper part of the tile is masked afterwards) keep
    // all 16 loads per thread in flight
    double v[NB * NB / NT];
#pragma unroll
    for (int t = 0; t < NB * NB / NT; ++t) {
      const int e = tid + t * NT, i = e & 63, j = e >> 6;
      v[t] = A[(o + j) * ld + o + i];
    }
#pragma unroll
    for (int t = 0; t < NB * NB / NT; ++t) {
      const int e = tid + t * NT, i = e & 63, j = e >> 6;
      S[i * SP + j] = (j <= i) ? v[t] : 0.0;
    }
  }
  __syncthreads();
  STAMP(1);
  factor_invert_64(S, R, U, o, N, d.status);
  double* __restrict__ Li = d.Linv + (int64_t)kb * TILE;
#pragma unroll 4
  for (int e = tid; e < NB * NB; e += NT) {
    const int i = e & 63, j = e >> 6;   // column-major: consecutive threads -> consecutive rows
    A[(o + j) * ld + o + i] = S[i * SP + j];
    Li[j * NB + i] = R[i * SP + j];
  }
  STAMP(18);
}

// Panel: L_ik = A_ik * Linv_kk^T for every row block i > kb.
__global__ __launch_bounds__(NT) void k_panel(const GPDesc* __restrict__ descs, int kb) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t nb = nblocks_factor(d.N);
  const int64_t ib = kb + 1 + (int64_t)blockIdx.x;
  if (ib >= nb) return;
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  load_tile_cm(As, d.A, d.ld, ib * NB, (int64_t)kb * NB, tid);
  load_tile_cm(Bs, d.Linv + (int64_t)kb * TILE, NB, 0, 0, tid);  // Bs[m][j] = Linv[j][m]
  __syncthreads();
  Acc acc;
  acc_zero(acc);
  tile_mma<false>(As, Bs, acc, wm, wn, lane);
  const int r = lane & 15, q = lane >> 4;
  double* __restrict__ A = d.A;
  const int64_t ld = d.ld;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = acc_row(wm, mt, q, v), col = acc_col(wn, nt, r);
        A[((int64_t)kb * NB + col) * ld + ib * NB + row] = acc.c[mt][nt][v];
      }
}

// Trailing update: A_ij -= L_ik L_jk^T for kb < j <= i (lower tiles only).
// Trailing tiles t0, t0+1, ... of step kb (t0 = 1 skips tile (kb+1, kb+1), which
// the look-ahead diagonal kernel updates itself).
__global__ __launch_bounds__(NT) void k_syrk(const GPDesc* __restrict__ descs, int kb, int t0) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t nb = nblocks_factor(d.N);
  const int64_t T = nb - kb - 1;
  const int64_t t = blockIdx.x + (int64_t)t0;
  if (T <= 0 || t >= T * (T + 1) / 2) return;
  int ii, jj;
  tri_index(t, ii, jj);
  const int64_t ib = kb + 1 + ii, jb = kb + 1 + jj;
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int r = lane & 15, q = lane >> 4;
  const int64_t ld = d.ld;
  double* __restrict__ A = d.A;
  load_tile_cm(As, A, ld, ib * NB, (int64_t)kb * NB, tid);
  load_tile_cm(Bs, A, ld, jb * NB, (int64_t)kb * NB, tid);
  Acc acc;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = acc_row(wm, mt, q, v), col = acc_col(wn, nt, r);
        acc.c[mt][nt][v] = A[(jb * NB + col) * ld + ib * NB + row];
      }
  __syncthreads();
  tile_mma<true>(As, Bs, acc, wm, wn, lane);
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = acc_row(wm, mt, q, v), col = acc_col(wn, nt, r);
        A[(jb * NB + col) * ld + ib * NB + row] = acc.c[mt][nt][v];
      }
}

// Trailing update over nk consecutive 64-column steps kb0 .. kb0 + nk - 1 at once
// (two-level blocking): A_ij -= sum_k L_ik L_jk^T for the lower tiles with jmin <=
// j <= min(i, jmax). The accumulator stays in registers across the nk steps and
// the MFMA sequence is k_syrk's, step after step, so the result is bit-equal to nk
// k_syrk launches; the tile is read and written once instead of nk times, and
// the next step's two operand tiles load while this step's MFMAs run.
__global__ __launch_bounds__(NT) void k_syrk_blk(const GPDesc* __restrict__ descs, int kb0, int nk, int jmin,
                                                 int jmax) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t nb = nblocks_factor(d.N);
  if (kb0 >= nb) return;
  const int64_t jm = jmax < nb - 1 ? jmax : nb - 1;
  if (jmin > jm) return;
  // tile t: column j (from jmin), row i >= j
  int64_t t = blockIdx.x, ib = -1, jb = -1;
  if (jm == nb - 1) {   // a triangle
    const int64_t T = nb - jmin;
    if (t >= T * (T + 1) / 2) return;
    int ii, jj;
    tri_index(t, ii, jj);
    ib = jmin + ii;
    jb = jmin + jj;
  } else {              // a few columns
    for (int64_t j = jmin; j <= jm; ++j) {
      if (t < nb - j) {
        ib = j + t;
        jb = j;
        break;
      }
      t -= nb - j;
    }
    if (ib < 0) return;
  }
  const int kn = (int)(kb0 + nk <= nb ? nk : nb - kb0);
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int r = lane & 15, q = lane >> 4;
  const int64_t ld = d.ld;
  double* __restrict__ A = d.A;
  TileRegs ra, rb;
  tile_fetch(ra, A + (int64_t)kb0 * NB * ld + ib * NB, ld, tid);
  tile_fetch(rb, A + (int64_t)kb0 * NB * ld + jb * NB, ld, tid);
  Acc acc;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = acc_row(wm, mt, q, v), col = acc_col(wn, nt, r);
        acc.c[mt][nt][v] = A[(jb * NB + col) * ld + ib * NB + row];
      }
  for (int s = 0; s < kn; ++s) {
    if (s > 0) __syncthreads();   // the previous step's LDS reads are done
    tile_put_k(As, ra, tid);
    tile_put_k(Bs, rb, tid);
    __syncthreads();
    if (s + 1 < kn) {
      const int64_t kc = (int64_t)(kb0 + s + 1) * NB;
      tile_fetch(ra, A + kc * ld + ib * NB, ld, tid);
      tile_fetch(rb, A + kc * ld + jb * NB, ld, tid);
    }
    tile_mma<true>(As, Bs, acc, wm, wn, lane);
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = acc_row(wm, mt, q, v), col = acc_col(wn, nt, r);
        A[(jb * NB + col) * ld + ib * NB + row] = acc.c[mt][nt][v];
      }
}

// ---------------------------------------------------------------------------
// Fused predict. One workgroup (256 threads, 4 waves; two workgroups per CU) =
// one GP x 64 grid cells. For each 128-row block I of the training set
// (sequential, left-looking):
//   acc  = psi_I^T                          (exp in registers, gp:139 / gp:426-429)
//   acc -= sum_{J<I} L_IJ V_J               (f64 MFMA over 16-deep K steps)
//   V_I  = L_II^-1 acc                      (two 64-row halves, 64-wide inverses:
//          V_top = Linv_a acc_top;  V_bot = Linv_b (acc_bot - L_ba V_top))
//   var_part += colsum(V_I o V_I);  mu_part += V_I^T z_I
// then mu = m + mu_part (gp:142-143 / gp:432), var = k** - var_part (diag of
// gp:146 / gp:435-436). z = L^-1 (y - m) is read from zv (row N of the
// augmented factor, extracted by k_extract_z). Every V block is stored: V stays
// resident in HBM for the incremental predicts (k_vstream) that follow appends.
//
// Staging: global_load_lds_dwordx4 (LDS-DMA) into a 3-stage ring of 16-deep K
// steps (16 KB of L + 8 KB of V per stage) with two steps in flight, a counted
// vmcnt and one raw s_barrier per step (no __syncthreads in the loop: its fence
// would drain the DMA). The XOR swizzles of the LDS images are applied on the
// global source addresses (the DMA writes lane-linear). All LDS lives in one
// array (hipcc vmcnt trap). The V panels of earlier row blocks are re-read from
// HBM N/256 times -- the 128-row blocks halve that traffic against 64-row ones;
// the second workgroup on the CU hides each one's psi / diagonal phases.
// ---------------------------------------------------------------------------
constexpr int KS = 16;                   // K depth of one pipeline step
constexpr int NSTAGE = 3;
constexpr int STAGE = KS * PW + KS * PBM;   // doubles per stage: As [KS][128] + Bs [KS][64]
constexpr int GLDS_PER_STEP = (KS + KS * PBM / 128) / (PNT / 64);   // per wave: 4 (L) + 2 (V)

// Buffer-descriptor LDS-DMA (buffer_load_dwordx4 ... lds): the lane part of the
// source offset is a VGPR fixed for the whole kernel, the row/step part an SGPR,
// so one DMA costs an s_mov to M0 and the load -- no per-row address VALU.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const double* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(bytes > 0x7fffffff ? 0x7fffffff : bytes), 0x00020000);
}

__device__ __forceinline__ void dma_buf(__amdgpu_buffer_rsrc_t rs, double* dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr)dst, 16, voff, soff, 0, 0);
}
// the same with the sc1 cache policy (aux 16): served by L2, never by a possibly
// stale line of this CU's L1 -- for bytes another workgroup stored in this launch
__device__ __forceinline__ void dma_buf_sc1(__amdgpu_buffer_rsrc_t rs, double* dst, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_vptr)dst, 16, voff, soff, 0, 16);
}


// Main-loop accumulator: wave wm owns rows wm*32.. x all 64 cells.
struct AccP {
  d4 c[2][4];
};
// Diagonal-step accumulator: wave owns 16 rows of a 64-row half x 64 cells.
struct AccH {
  d4 c[4];
};

// acc += A[32 rows of this wave][KS] * B[KS][64]  (acc holds -psi + sum L V)
__device__ __forceinline__ void main_mma(const double* __restrict__ As, const double* __restrict__ Bs, AccP& acc,
                                         int wm, int lane) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < KS; k0 += 4) {
    const int k = k0 + q;
    double a[2], b[4];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) a[mt] = As[swzp(k, wm * 32 + mt * 16 + r)];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) b[nt] = Bs[swz(k, nt * 16 + r)];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc.c[mt][nt] = mfma(a[mt], b[nt], acc.c[mt][nt]);
  }
}

// A fragments of a column-major 64x64 block (A[i][k] = G[k*lda + i]) for the 16
// rows p16.. of this wave, all 16 K steps: frag[t] = A[p16 + r][4t + q].
__device__ __forceinline__ void load_afrag(double* frag, const double* __restrict__ G, int64_t lda, int p16,
                                           int lane) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int t = 0; t < 16; ++t) frag[t] = gp(G)[(int64_t)(4 * t + q) * lda + p16 + r];
}

// acc (+/-)= A[16 x 4*nt4] (fragments) * img[rows rb..][64 cells]; nt4 K steps
template <bool NEG>
__device__ __forceinline__ void half_mma(const double* frag, const double* __restrict__ img, int rb, AccH& acc,
                                         int nt4, int lane) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    if (t < nt4) {
      const double a = NEG ? -frag[t] : frag[t];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc.c[nt] = mfma(a, img[swz(rb + 4 * t + q, nt * 16 + r)], acc.c[nt]);
    }
  }
}

// Fused np.amax / np.argmax of a GP's variance (simulator.py:672, 842, 1014 and
// the argmax of compute_sample_points, sim:352). Every cell tile publishes its
// (max, first argmax) from its epilogue; the last tile to arrive reduces them.
// The hand-off avoids device-scope fences (a release fence per workgroup would
// write back the XCD's L2 each time): the partial is stored with an agent-scope
// atomic store (write-through), drained with s_waitcnt, then the arrival counter
// is bumped; the last arriver reads the partials with agent-scope atomic loads
// and resets the counter for the next launch. Called by wave 0 of the tile's
// workgroup, lane l holding cell c0 + l (valid if inside the grid).
__device__ __forceinline__ void argmax_pair(double& bv, int64_t& bi, double ov, int64_t oi) {
  if (ov > bv || (ov == bv && oi < bi)) {
    bv = ov;
    bi = oi;
  }
}

__device__ void var_argmax_tile(const GPDesc& d, double v, int64_t c, bool valid, int64_t tile) {
  const int lane = threadIdx.x & 63;
  double bv = valid ? v : -__builtin_inf();
  int64_t bi = valid ? c : INT64_MAX;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) argmax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  const int64_t ntiles = ntiles_grid(d.M);
  unsigned* cnt = reinterpret_cast<unsigned*>(d.tred);   // tred = [counter | (max, argmax) per tile]
  double* part = d.tred + 1;
  unsigned old = 0;
  if (lane == 0) {
    __hip_atomic_store(part + 2 * tile, bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part + 2 * tile + 1, (double)bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  old = __shfl(old, 0);
  if (old != (unsigned)(ntiles - 1)) return;
  bv = -__builtin_inf();
  bi = INT64_MAX;
  for (int64_t t = lane; t < ntiles; t += 64)
    argmax_pair(bv, bi, __hip_atomic_load(part + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                (int64_t)__hip_atomic_load(part + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) argmax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  if (lane == 0) {
    if (d.vmax) *d.vmax = bv;
    if (d.vargmax) *d.vargmax = bi;
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ __launch_bounds__(PNT, 2) void k_predict(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t M = d.M;
  const int64_t c0 = (int64_t)blockIdx.x * PBM;
  if (c0 >= M) return;
  // ring: stage s at lds[s*STAGE] = As [KS][128] then Bs [KS][64]; the diagonal
  // step reuses the ring as the [128][64] image of acc / V (64 KB <= 72 KB).
  __shared__ double lds[NSTAGE * STAGE + PRB];
  double* const zs = lds + NSTAGE * STAGE;
  double* const img = lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave id (uniform)
  const int r = lane & 15, q = lane >> 4;
  const int p16 = w * 16;   // diagonal-step rows of this wave inside a 64-row half
  const Hyp& h = d.hp;
  const int64_t N = d.N, NL = d.NL, ld = d.ld;
  const int64_t nrb = prow_blocks(N);
  const int64_t nbf = nblocks_factor(N);
  const double* __restrict__ X = d.X;
  const double* __restrict__ Amat = d.A;
  double* __restrict__ Vt = d.V + (int64_t)blockIdx.x * d.vld * PBM;   // resident V tile
  double vsum[4] = {0.0, 0.0, 0.0, 0.0}, msum[4] = {0.0, 0.0, 0.0, 0.0};
  // DMA plan of one K step (kc = first factor column / V row of the step):
  //  L image [KS][128]: wave w moves rows k = w + 4j (j < 4), all of parity w&1;
  //    src = A[(kc + k)*ld + base + ((2*lane) ^ sw)]
  //  V image [KS][64]:  wave w moves row pairs p = w + 4j (j < 2), rows 2p + (lane>>5);
  //    src = Vt[(kc + 2p + (lane>>5))*64 + (((lane&31)*2) ^ ((lane>>5)<<4))]
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(Amat, (int64_t)8 * ld * ld);
  const __amdgpu_buffer_rsrc_t rsV = make_rsrc(Vt, (int64_t)8 * d.vld * PBM);
  const unsigned voffA = (unsigned)(8 * ((2 * lane) ^ ((w & 1) << 4)));
  const unsigned voffV =
      (unsigned)(8 * ((lane >> 5) * PBM + (((lane & 31) * 2) ^ ((lane >> 5) << 4))));
  auto dma_step = [&](double* st, int64_t base_, int64_t kc) {
#pragma unroll
    for (int j = 0; j < KS / 4; ++j) {
      const int k = w + 4 * j;
      dma_buf(rsA, st + k * PW, voffA, (unsigned)(8 * ((kc + k) * ld + base_)));
    }
#pragma unroll
    for (int j = 0; j < KS / 8; ++j) {
      const int pp = w + 4 * j;
      dma_buf(rsV, st + KS * PW + 2 * pp * PBM, voffV, (unsigned)(8 * (kc + 2 * pp) * PBM));
    }
  };

  for (int64_t I = 0; I < nrb; ++I) {
    const int64_t base = I * PRB;
    const int nk = (int)(base / KS);   // K steps: all columns left of the block
    // prologue: steps 0 and 1 in flight while psi is generated
#pragma unroll
    for (int s0 = 0; s0 < 2; ++s0) {
      if (s0 < nk) dma_step(lds + s0 * STAGE, base, (int64_t)s0 * KS);
    }
    AccP acc;
    {
      // this lane's four grid cells (columns nt*16 + r), scaled by the length scales
      double cLx[4], cLy[4], cHx[4], cHy[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        int64_t c = c0 + nt * 16 + r;
        if (c >= M) c = M - 1;
        const double gx = d.grid[2 * c], gy = d.grid[2 * c + 1];
        cLx[nt] = div_(gx, h.lL);
        cLy[nt] = div_(gy, h.lL);
        cHx[nt] = div_(gx, h.lH);
        cHy[nt] = div_(gy, h.lH);
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int64_t g = base + w * 32 + mt * 16 + q + 4 * v;
          double pv[4] = {0.0, 0.0, 0.0, 0.0};
          if (g < N) {
            const double tx = X[2 * g], ty = X[2 * g + 1];
            const double tLx = div_(tx, h.lL), tLy = div_(ty, h.lL);
            if (h.kind == 0) {
#pragma unroll
              for (int nt = 0; nt < 4; ++nt) pv[nt] = se_scaled(cLx[nt], cLy[nt], tLx, tLy, h.sL);
            } else if (g < NL) {
#pragma unroll
              for (int nt = 0; nt < 4; ++nt) pv[nt] = h.rho * se_scaled(cLx[nt], cLy[nt], tLx, tLy, h.sL);
            } else {
              const double tHx = div_(tx, h.lH), tHy = div_(ty, h.lH);
#pragma unroll
              for (int nt = 0; nt < 4; ++nt) {
#pragma clang fp contract(off)
                pv[nt] = h.rho2 * se_scaled(cLx[nt], cLy[nt], tLx, tLy, h.sL) +
                         se_scaled(cHx[nt], cHy[nt], tHx, tHy, h.sH);
              }
            }
          }
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) acc.c[mt][nt][v] = -pv[nt];   // acc = -psi + sum L V
        }
    }
    double frag[16];
    if (nk > 0) {
      // step 0 landed (step 1 may still be in flight)
      if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GLDS_PER_STEP) : "memory");
      else vm_wait_all();
      __builtin_amdgcn_s_barrier();
    }
    // acc += L_I,<I V_<I over 16-deep steps; steps s+1, s+2 in flight during step s
    for (int s = 0; s < nk; ++s) {
      const double* cur = lds + (s % NSTAGE) * STAGE;
      if (s + 2 < nk) dma_step(lds + ((s + 2) % NSTAGE) * STAGE, base, (int64_t)(s + 2) * KS);
      main_mma(cur, cur + KS * PW, acc, w, lane);
      if (s + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(GLDS_PER_STEP) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // ---- diagonal block: V_I = L_II^-1 (psi - L V), two 64-row halves ----
    const int64_t fa = 2 * I, fb = 2 * I + 1;       // 64-blocks of the factor
    const bool has_b = fb < nbf;                    // bottom half holds real rows
    load_afrag(frag, d.Linv + fa * TILE, NB, p16, lane);   // Linv_a
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int v = 0; v < 4; ++v) img[swz(w * 32 + mt * 16 + q + 4 * v, nt * 16 + r)] = -acc.c[mt][nt][v];
    if (tid < PRB) {
      const int64_t g = base + tid;
      zs[tid] = (g < N) ? d.zv[g] : 0.0;
    }
    __syncthreads();
    // V_top = Linv_a * T_top (Linv_a lower triangular: rows p16.. need K < p16 + 16)
    AccH vh;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) vh.c[nt] = d4{0.0, 0.0, 0.0, 0.0};
    half_mma<false>(frag, img, 0, vh, (p16 + 16) / 4, lane);
    if (has_b) load_afrag(frag, Amat + fa * NB * ld + fb * NB, ld, p16, lane);   // L_ba
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = p16 + q + 4 * v, col = nt * 16 + r;
        const double val = vh.c[nt][v];
        gp(Vt)[(base + row) * PBM + col] = val;
        if (base + row < N) {
          vsum[nt] += val * val;
          msum[nt] += val * zs[row];
        }
      }
    __syncthreads();   // every wave is done reading T_top
    if (has_b) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int v = 0; v < 4; ++v) img[swz(p16 + q + 4 * v, nt * 16 + r)] = vh.c[nt][v];
      __syncthreads();
      // T_bot -= L_ba V_top   (each wave: its own 16 rows of the bottom half)
      AccH th;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int v = 0; v < 4; ++v) th.c[nt][v] = img[swz(64 + p16 + q + 4 * v, nt * 16 + r)];
      half_mma<true>(frag, img, 0, th, 16, lane);
      load_afrag(frag, d.Linv + fb * TILE, NB, p16, lane);   // Linv_b
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int v = 0; v < 4; ++v) img[swz(64 + p16 + q + 4 * v, nt * 16 + r)] = th.c[nt][v];
      __syncthreads();
      // V_bot = Linv_b T_bot
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) vh.c[nt] = d4{0.0, 0.0, 0.0, 0.0};
      half_mma<false>(frag, img, 64, vh, (p16 + 16) / 4, lane);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = 64 + p16 + q + 4 * v, col = nt * 16 + r;
          const double val = vh.c[nt][v];
          gp(Vt)[(base + row) * PBM + col] = val;
          if (base + row < N) {
            vsum[nt] += val * val;
            msum[nt] += val * zs[row];
          }
        }
    }
    vm_wait_all();      // V_I stores complete before any later DMA reads them
    __syncthreads();    // and before the next prologue overwrites the LDS images
  }
  // reduce over the 4 row groups of the wave (lanes r, r+16, r+32, r+48), then
  // over the 4 waves (LDS, reusing the ring)
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    vsum[nt] += __shfl_xor(vsum[nt], 16);
    vsum[nt] += __shfl_xor(vsum[nt], 32);
    msum[nt] += __shfl_xor(msum[nt], 16);
    msum[nt] += __shfl_xor(msum[nt], 32);
  }
  double* red = lds;   // [2][4][PBM]
  if (q == 0) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      red[(0 * 4 + w) * PBM + nt * 16 + r] = vsum[nt];
      red[(1 * 4 + w) * PBM + nt * 16 + r] = msum[nt];
    }
  }
  __syncthreads();
  if (tid < PBM) {
    const int64_t c = c0 + tid;
    const double vs = (red[0 * PBM + tid] + red[1 * PBM + tid]) + (red[2 * PBM + tid] + red[3 * PBM + tid]);
    const double ms = (red[4 * PBM + tid] + red[5 * PBM + tid]) + (red[6 * PBM + tid] + red[7 * PBM + tid]);
    const double vc = h.kss - vs;
    if (c < M) {
      d.mu[c] = ms + h.meanH;
      d.var[c] = vc;
      if (d.rmu) {
        d.rmu[c] = ms + h.meanH;
        d.rvar[c] = vc;
      }
    }
    if (d.vmax || d.vargmax) var_argmax_tile(d, vc, c, c < M, blockIdx.x);
  }
}

// z = L^-1 (y - m) out of row N of the augmented factor into zv (after the
// full factor; the incremental kernels extend zv themselves).
__global__ __launch_bounds__(NT) void k_extract_z(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t j = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (j < d.N) d.zv[j] = d.A[j * d.ld + d.N];
}

// ---------------------------------------------------------------------------
// Incremental append. The reference refactors from
// scratch on every updt / updt_hifi (gp:257-268, gp:531-542 -> gp:254 / gp:529);
// the factor of the leading rows does not change, so appending rows [n0, N)
// (k = N - n0 <= KINC hifi rows) to a factor current for rows [0, n0) is the
// bordered Cholesky step
//   L21^T = L11^-1 K12,   L22 = chol(K22 - L21 L21^T),   z2 = L22^-1 (r2 - L21 z1)
// plus the new rows of the diagonal-block inverses. L21^T is a set of V columns:
// when every new point is a grid cell (the simulator samples only grid cells,
// sim:705 / sim:875) and V = L11^-1 psi^T is resident for rows < n0, column c of
// L21^T is V[:, cell(c)] -- psi(cell, X) and K(X, x_new) are the same numbers,
// same operation order (k_entry vs k_predict's psi). One launch (k_inc_stream,
// below): producer workgroups over 128-row chunks find the cells, gather the V
// columns into rows n0.. of A and sum their chunk's L21 L21^T, L21 z1 (MFMA); the
// last producer to arrive sums the partials and computes L22, z2 and the new
// Linv rows. Off the grid (or without a resident V) it solves L21^T itself by
// blocked forward substitution (one workgroup, f64 MFMA; slower, but general).
// ---------------------------------------------------------------------------
#ifndef MFGP_INC_WAVES
#define MFGP_INC_WAVES 4   // k_inc_stream waves per SIMD (occupancy; 5 measured 1-5 % slower)
#endif
constexpr int FCH = FUSED_CHUNK;           // rows of L21 per producer workgroup
constexpr int ISZ = KINC * KINC + KINC;    // partial sums per chunk: L21 L21^T | L21 z1
// iscr layout: [0] = 1 if the new points were found on the grid with V resident
// (k_append), [ISC0 + chunk * ISZ ...] = the producers' partials
constexpr int ISC0 = 1 + KINC;

// Data handed between workgroups of ONE launch (k_inc_stream) goes through
// write-through stores and L2-bypassing loads (relaxed, agent scope); each
// producer drains its stores (s_waitcnt) before it signals. No fence: a
// __threadfence writes the whole L2 back. XW = false: plain accesses (the
// consumers are later launches).
template <bool XW>
__device__ __forceinline__ double ldx(const double* p) {
  if constexpr (XW) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool XW>
__device__ __forceinline__ void stx(double* p, double v) {
  if constexpr (XW) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// A workgroup barrier that orders LDS only: this wave's LDS accesses complete, then
// s_barrier. Loads in flight stay in flight (__syncthreads' workgroup fence waits for
// them); for LDS data exchanged between the waves of one workgroup.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// 16-byte write-through store (global_store_dwordx4 ... sc1): a whole line per wave
// instruction where 8 lanes cover it, and no dirty line left in the XCD's L2 for the
// launch's end to write back (MI355X_MICROARCH.md: 16-B sc1 stores cost as plain ones)
__device__ __forceinline__ void st16_wt(double* p, dv2 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// The consumer's side of a hand-off. Every byte handed between workgroups of one
// launch is stored write-through (sc1, drained before the flag) and loaded with
// device-scope (sc1) loads that L2 does not serve from a possibly stale line, or
// read plain only when no workgroup of that XCD can have cached the line earlier
// in the launch (L2 is invalidated at kernel start); the consumer issues its
// loads after it saw the flag (no speculation). No acquire: an agent-scope
// acquire after each wait (its L2 invalidate) cost the lattice step 105 -> 172 us
// per launch at B = 8, and even one per wait on the polling lane 8 % (97.0k vs
// 89.2k GP-updates/s, round 5): DESIGN 2.2. tests/test_codeobj.py checks the
// emitted polls (sc1 loads, completed before the branch that leaves the spin).
__device__ __forceinline__ void publish(unsigned* f, unsigned v) {
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Wait (thread 0, the workgroup joins at the barrier) until *f == v. Bounded:
// after ~1 s the kernel records a synchronisation failure in *status (reported
// by the host) and goes on, so a lost signal can never hang the device.
constexpr int SYNC_FAIL = INT_MIN;
__device__ void wait_flag(const GPDesc& d, const unsigned* f, unsigned v) {
  if (threadIdx.x == 0) {
    int it = 0;
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != v) {
      __builtin_amdgcn_s_sleep(MFGP_SPIN_SLEEP);
      if (++it == (1 << 22)) {
        atomicMin(d.status, SYNC_FAIL);
        break;
      }
    }
  }
  __syncthreads();
}

// Wait (wave 0; the workgroup joins at the barrier) until the compact rows of
// this append are stored: every producer chunk's flag holds this launch's epoch,
// or sync[1] does (raised by the last producer to arrive, or by the finish when
// it solved L21 itself). Bounded like wait_flag.
__device__ void wait_l21(const GPDesc& d) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int it = 0;
    while (true) {
      bool mine = true;
      for (int c = lane; c < d.nprod; c += 64)
        mine = mine && __hip_atomic_load(d.pflag + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == d.epoch;
      const bool any = __hip_atomic_load(d.sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == d.epoch;
      if (any || __ballot(!mine) == 0) break;
      __builtin_amdgcn_s_sleep(MFGP_SPIN_SLEEP);
      if (++it == (1 << 22)) {
        if (lane == 0) atomicMin(d.status, SYNC_FAIL);
        break;
      }
    }
  }
  __syncthreads();
}

// Coordinates / observation of training row `row`: rows landing in this launch
// ([N - k_new, N), device source) are read from the source itself.
__device__ __forceinline__ const double* row_pt(const GPDesc& d, int64_t row) {
  const int64_t at = d.N - d.k_new;
  if (row >= at && d.srcX) return d.srcX + 2 * (row - at);
  if (row >= at && d.rows_inline) return d.rows_xy + 2 * (row - at);
  return d.X + 2 * row;
}
__device__ __forceinline__ double row_obs(const GPDesc& d, int64_t row) {
  const int64_t at = d.N - d.k_new;
  if (row >= at && d.srcY) return d.srcY[row - at];
  if (row >= at && d.rows_inline) return d.rows_y[row - at];
  return d.y[row];
}

// Identity padding for the 64-row blocks [ablk, nbf) entered for the first time,
// columns [c_lo, c_hi) (the full predict reads whole blocks: padding rows must
// stay finite), and, with `linv`, their Linv blocks.
// Rows [skip_lo, skip_hi) are left out (the caller stores them itself).
template <bool XW = false>
__device__ void inc_init_blocks(const GPDesc& d, int64_t c_lo, int64_t c_hi, bool linv, int64_t skip_lo = 0,
                                int64_t skip_hi = 0) {
  const int64_t nbf = nblocks_factor(d.N);
  const int tid = threadIdx.x, nthr = blockDim.x;
  for (int64_t bb = d.ablk; bb < nbf; ++bb) {
    const int64_t c1 = c_hi < (bb + 1) * NB ? c_hi : (bb + 1) * NB;
    if (c1 > c_lo) {
      for (int64_t e = tid; e < (c1 - c_lo) * NB; e += nthr) {
        const int64_t col = c_lo + (e >> 6);
        const int64_t row = bb * NB + (e & 63);
        if (row < skip_lo || row >= skip_hi) stx<XW>(&d.A[col * d.ld + row], (col == row) ? 1.0 : 0.0);
      }
    }
    if (linv)
      for (int e = tid; e < TILE; e += nthr) d.Linv[bb * TILE + e] = ((e & 63) == (e >> 6)) ? 1.0 : 0.0;
  }
}

// The compact bordered row j, entry r, for the cell workgroups' MFMA A operand:
// fp64 V: L21[r][j] for r < k, z1[j] at r = k, zeros; fp32 V (VT = float, the
// rows stored as floats over the same area): L21[r][j] for r < k, z1[j] at
// r = ZROW (the f32 stream sums the mean out of that fixed row), zeros.
constexpr int ZROW = KINC - 1;
template <bool XW, class VT>
__device__ __forceinline__ void store_l21c(double* l21c, int64_t j, int r, int k, double a, double z) {
  if constexpr (sizeof(VT) == 8) {
    stx<XW>(&l21c[j * KINC + r], r < k ? a : (r == k ? z : 0.0));
  } else {
    float* p = reinterpret_cast<float*>(l21c) + j * KINC + r;
    const float v = (float)(r < k ? a : (r == ZROW ? z : 0.0));
    if constexpr (XW) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
  }
}

// The resident V of this GP in the precision VT (fp64 d.V, fp32 d.Vf).
template <class VT>
__device__ __forceinline__ const VT* vres_ptr(const GPDesc& d) {
  if constexpr (sizeof(VT) == 8) return d.V;
  else return d.Vf;
}

// Partial L21 L21^T and L21 z1 over rows [j_lo, j_hi) into red[w][ISZ] (one slot per
// wave). Lane (r, q) holds L21[r][j], j = 4s + q, eight 4-row steps in flight per
// wave. With `cell`, L21[r][.] is gathered from the V column of the grid cell and
// written to row n0 + r of A; otherwise it is read from there. VT: the precision
// of the resident V (an fp32 V's entries are widened: L21 is then the factor of K
// perturbed by their rounding, |dL21| <= 2^-24 |L21|).
template <int NW, bool XW, bool FROMV, class VT>
__device__ void inc_schur_partial(const GPDesc& d, const int* cell, int64_t j_lo, int64_t j_hi,
                                  double (*red)[ISZ]) {
  // descriptor fields in registers: the write-through stores below would make the
  // compiler reload them (and drain every load) before each store
  const int64_t n0 = d.n0, ld = d.ld;
  const int k = (int)(d.N - n0);
  double* const A = d.A;
  double* const l21c = d.l21c;
  const double* const zv = d.zv;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  d4 sacc = {0.0, 0.0, 0.0, 0.0}, uacc = {0.0, 0.0, 0.0, 0.0};
  constexpr int IU = 8;
  const int cr = (FROMV && r < k) ? cell[r] : 0;
  const VT* vsrc = FROMV ? vres_ptr<VT>(d) + (int64_t)(cr / PBM) * d.vld * PBM + (cr % PBM) : nullptr;
  const double* src = A + n0 + (r < k ? r : 0);
  const int64_t sstride = FROMV ? PBM : ld;
  const int64_t s_lo = j_lo >> 2, s_hi = (j_hi + 3) >> 2;   // j_lo is a multiple of 4
  for (int64_t s0 = s_lo + w; s0 < s_hi; s0 += NW * IU) {
    double a[IU], zz[IU];
#pragma unroll
    for (int u = 0; u < IU; ++u) {
      const int64_t j = 4 * (s0 + NW * u) + q;
      const bool ok = j < j_hi;
      const int64_t jj = ok ? j : j_lo;
      a[u] = FROMV ? (double)gp(vsrc)[jj * sstride] : ldx<XW>(src + jj * sstride);
      zz[u] = gp(zv)[jj];
    }
#pragma unroll
    for (int u = 0; u < IU; ++u) {
      const int64_t j = 4 * (s0 + NW * u) + q;
      const bool ok = j < j_hi;
      a[u] = (ok && r < k) ? a[u] : 0.0;
      zz[u] = ok ? zz[u] : 0.0;
      if (FROMV && r < k && ok) stx<XW>(&A[j * ld + n0 + r], a[u]);
      // compact rows for the cell tiles: L21 | z1 | zeros
      if (ok) store_l21c<XW, VT>(l21c, j, r, k, a[u], zz[u]);
      sacc = mfma(a[u], a[u], sacc);
      uacc = mfma(a[u], zz[u], uacc);
    }
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    red[w][(q + 4 * v) * KINC + r] = sacc[v];
    if (r == 0) red[w][KINC * KINC + q + 4 * v] = uacc[v];
  }
}

// cell[c] = first grid index equal to new point c (INT_MAX if none); all NTHR
// threads of the workgroup take part, SB grid loads in flight per thread.
template <int NTHR>
__device__ void find_cells(const GPDesc& d, const double* px, const double* py, int* cell) {
  const int tid = threadIdx.x;
  const GLOBAL dv2* g2 = reinterpret_cast<const GLOBAL dv2*>(gp(d.grid));
  constexpr int SB = 8;
  for (int64_t e0 = tid; e0 < d.M; e0 += (int64_t)NTHR * SB) {
    dv2 gxy[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int64_t e = e0 + (int64_t)u * NTHR;
      gxy[u] = g2[e < d.M ? e : 0];
    }
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int64_t e = e0 + (int64_t)u * NTHR;
      bool hit = false;
#pragma unroll
      for (int c = 0; c < KINC; ++c) hit = hit || (gxy[u].x == px[c] && gxy[u].y == py[c]);
      if (hit && e < d.M) {
#pragma unroll
        for (int c = 0; c < KINC; ++c)
          if (gxy[u].x == px[c] && gxy[u].y == py[c]) atomicMin(&cell[c], (int)e);
      }
    }
  }
}

// Index of grid point (px, py) from the lattice structure: the rounded axis
// estimate and its neighbours, checked for exact equality (INT_MAX if none).
// The axes are strictly monotone, so an exact match is the only one.
__device__ int lattice_cell(const GPDesc& d, double px, double py) {
  const GridLattice& L = d.lat;
  if (L.nx <= 0 || !(px == px) || !(py == py)) return INT_MAX;
  const GLOBAL dv2* g2 = reinterpret_cast<const GLOBAL dv2*>(gp(d.grid));
  const int ix = (int)rint(fmin(fmax((px - L.x0) * L.xinv, 0.0), (double)(L.nx - 1)));
  const int iy = (int)rint(fmin(fmax((py - L.y0) * L.yinv, 0.0), (double)(L.ny - 1)));
  int64_t e[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int cx = ix + t / 3 - 1, cy = iy + t % 3 - 1;
    e[t] = (cx >= 0 && cx < L.nx && cy >= 0 && cy < L.ny) ? cx * L.sx + cy * L.sy : -1;
  }
  dv2 g[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) g[t] = g2[e[t] >= 0 ? e[t] : 0];
  int hit = INT_MAX;
#pragma unroll
  for (int t = 0; t < 9; ++t)
    if (e[t] >= 0 && g[t].x == px && g[t].y == py) hit = (int)e[t];
  return hit;
}

// End of a gathering producer chunk: its compact rows (and L21 rows in A) are
// drained and announced in pflag[chunk] (the cell workgroups wait for these),
// then the chunk's partials (red, summed over the waves) are stored for the finish.
__device__ __forceinline__ bool inc_chunk_done(const GPDesc& d, int64_t chunk, double (*red)[ISZ]) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) publish(d.pflag + chunk, d.epoch);
  FSTAMP(39);   // latest producer past its gather
  double* __restrict__ part = d.iscr + ISC0 + chunk * ISZ;
  for (int e = threadIdx.x; e < ISZ; e += NT) {
    double acc = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) acc += red[w][e];
    stx<true>(part + e, acc);
  }
  return true;
}

// Fast path of a producer chunk (at most FUSED_CHUNK rows) on a lattice grid: each
// wave estimates the new points' cells itself (lane r < k: point r, the rounded
// axis estimate), gathers its rows of L21 from those V columns and checks the
// estimates against the grid coordinates in the same round trip. Every wave
// checks the same points, so the verdict is uniform; on a miss nothing has been
// stored and the caller takes the general path. Otherwise as inc_schur_partial
// (FROMV): L21 rows into A and the compact rows, partials into red, and the
// chunk's identity padding of newly entered blocks (rows [n0, N) excepted: they
// are the L21 stores, so no barrier orders the two).
template <class VT>
__device__ __forceinline__ bool inc_gather_fast(const GPDesc& d, int64_t j_lo, int64_t j_hi, double (*red)[ISZ]) {
  constexpr int NW = NT / 64, IU = 8;
  static_assert(4 * NW * IU >= FUSED_CHUNK, "one round of loads covers a chunk");
  const int64_t n0 = d.n0, ld = d.ld, N = d.N;
  const int k = (int)(N - n0);
  double* const A = d.A;
  double* const l21c = d.l21c;
  const double* const zv = d.zv;
  const GridLattice L = d.lat;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const double* p = row_pt(d, n0 + (r < k ? r : 0));
  const double px = p[0], py = p[1];
  const int ix = (int)rint(fmin(fmax((px - L.x0) * L.xinv, 0.0), (double)(L.nx - 1)));
  const int iy = (int)rint(fmin(fmax((py - L.y0) * L.yinv, 0.0), (double)(L.ny - 1)));
  const int64_t cr = (px == px && py == py) ? ix * L.sx + iy * L.sy : 0;
  const dv2 g = reinterpret_cast<const GLOBAL dv2*>(gp(d.grid))[cr];
  const VT* src = vres_ptr<VT>(d) + (cr / PBM) * d.vld * PBM + (cr % PBM);
  double a[IU], zz[IU];
#pragma unroll
  for (int u = 0; u < IU; ++u) {
    const int64_t j = j_lo + 4 * (w + NW * u) + q;
    const int64_t jj = j < j_hi ? j : j_lo;
    a[u] = (double)gp(src)[jj * PBM];
    zz[u] = gp(zv)[jj];
  }
  const bool miss = r < k && !(g.x == px && g.y == py);
  if (__ballot(miss) != 0) return false;
  inc_init_blocks<true>(d, j_lo, j_hi, false, n0, N);
  d4 sacc = {0.0, 0.0, 0.0, 0.0}, uacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int u = 0; u < IU; ++u) {
    const int64_t j = j_lo + 4 * (w + NW * u) + q;
    const bool ok = j < j_hi;
    a[u] = (ok && r < k) ? a[u] : 0.0;
    zz[u] = ok ? zz[u] : 0.0;
    if (r < k && ok) stx<true>(&A[j * ld + n0 + r], a[u]);
    if (ok) store_l21c<true, VT>(l21c, j, r, k, a[u], zz[u]);
    sacc = mfma(a[u], a[u], sacc);
    uacc = mfma(a[u], zz[u], uacc);
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    red[w][(q + 4 * v) * KINC + r] = sacc[v];
    if (r == 0) red[w][KINC * KINC + q + 4 * v] = uacc[v];
  }
  return true;
}

// One producer chunk: land device-resident new rows (chunk 0), find the new
// points' grid cells, gather their V columns into rows n0.. of A for rows
// [chunk * ch, +ch) and store the chunk's partials. Returns false when L21 is not
// a set of V columns (off the grid / no resident V): the finish solves for it.
// All NTHR threads take part; `cell` and `red` are in LDS.
// Test build only (tests/test_codeobj.py): MFGP_NOINLINE_PRODUCE outlines the
// producer, the shape that once stalled k_inc_stream for seconds; the test checks
// that such a build is caught (a call inside the kernel) and the product one is not.
#ifdef MFGP_NOINLINE_PRODUCE
#define MFGP_PRODUCE_INLINE __attribute__((noinline))
#else
#define MFGP_PRODUCE_INLINE __forceinline__
#endif
template <class VT>
__device__ MFGP_PRODUCE_INLINE bool inc_produce(const GPDesc& d, int64_t chunk, int64_t ch, int* cell,
                                                double (*red)[ISZ]) {
  constexpr int NTHR = NT;
  constexpr bool XW = true;
  const int64_t n0 = d.n0, N = d.N;
  const int k = (int)(N - n0);
  const int tid = threadIdx.x;
  const int64_t kn = d.k_new, at = N - kn;   // rows [at, N) arrive from srcX / srcY
  if (chunk == 0 && kn > 0 && (d.srcX || d.rows_inline)) {
    // consumers are later launches (this one reads the sources: row_pt / row_obs)
    for (int64_t e = tid; e < 3 * kn; e += NTHR) {
      if (e < 2 * kn) const_cast<double*>(d.X)[2 * at + e] = row_pt(d, at + e / 2)[e % 2];
      else const_cast<double*>(d.y)[at + e - 2 * kn] = row_obs(d, at + e - 2 * kn);
    }
  }
  const bool try_v = n0 > 0 && d.vres >= n0 && vres_ptr<VT>(d) != nullptr && d.M > 0;
  if (!try_v) {
    if (chunk == 0 && tid == 0) stx<XW>(d.iscr, 0.0);
    return false;
  }
  const int64_t j_lo = chunk * ch;
  const int64_t j_hi = j_lo + ch < n0 ? j_lo + ch : n0;
  if (d.lat.nx > 0 && j_lo < n0 && ch <= FUSED_CHUNK && inc_gather_fast<VT>(d, j_lo, j_hi, red)) {
    if (chunk == 0 && tid == 0) stx<XW>(d.iscr, 1.0);
    return inc_chunk_done(d, chunk, red);
  }
  if (tid < KINC) cell[tid] = INT_MAX;
  __syncthreads();
  // lattice grids: a few probes per point; otherwise (or for a point off the
  // lattice) every thread scans the grid
  if (tid < k) {
    const double* p = row_pt(d, n0 + tid);
    cell[tid] = lattice_cell(d, p[0], p[1]);
  }
  __syncthreads();
  bool found = true;
  for (int c = 0; c < k; ++c) found = found && cell[c] != INT_MAX;
  if (!found) {
    double px[KINC], py[KINC];
#pragma unroll
    for (int c = 0; c < KINC; ++c) {
      const double* p = row_pt(d, n0 + (c < k ? c : 0));
      px[c] = c < k ? p[0] : __builtin_nan("");
      py[c] = c < k ? p[1] : __builtin_nan("");
    }
    __syncthreads();
    if (tid < KINC) cell[tid] = INT_MAX;
    __syncthreads();
    find_cells<NTHR>(d, px, py, cell);
    __syncthreads();
  }
  if (XW) FSTAMP(38);   // latest producer with its cells
  bool use_v = true;
  for (int c = 0; c < k; ++c) use_v = use_v && cell[c] != INT_MAX;
  if (chunk == 0 && tid == 0) stx<XW>(d.iscr, use_v ? 1.0 : 0.0);
  if (!use_v || j_lo >= n0) return use_v;   // off the grid: the finish solves
  inc_init_blocks<XW>(d, j_lo, j_hi, false);   // this chunk's columns of newly entered blocks
  __syncthreads();
  inc_schur_partial<NTHR / 64, XW, true, VT>(d, cell, j_lo, j_hi, red);
  return inc_chunk_done(d, chunk, red);
}

// LDS of the finish step (doubles; 256 threads):
//   phase 1 (partials / L21 solve, L22):  red [0,1088) ssum [1088,1360) K22s [1360,1616) Ts [1616,2640)
//   phase 2 (new Linv rows):              Ln [0,1024) Ps [1024,2048) Lb [2048,3056)
//   both:                                 L22s [3056,3312)
// (26.5 KB: LDS would fit five workgroups of k_inc_stream per CU; its 128 VGPRs allow four)
constexpr int FIN_LDS = 3312;
constexpr int LBW = 16;   // Linv_OO columns staged per pass (63 rows x 16 = 1008 doubles)

// The finish of a bordered append for one GP (one workgroup of NT threads): sum
// the producers' partials (chunks of `ch` rows) or solve L21 (off the grid),
// L22 = chol(K22 - L21 L21^T), z2, then the new rows of the diagonal-block
// inverses. FUSED (inside k_inc_stream): signals `sync[1]` once L21 is in A (when
// this step solved it) and `sync[2]` once L22 / z2 are, with the hand-off
// accesses of ldx / stx.
template <bool FUSED, class VT>
__device__ __forceinline__ void inc_finish(const GPDesc& d, double* sm, int64_t ch) {
  const int64_t n0 = d.n0, N = d.N, ld = d.ld, NL = d.NL;
  const int k = (int)(N - n0);
  const Hyp& h = d.hf;
  double* __restrict__ A = d.A;
  const double* __restrict__ X = d.X;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  double(*red)[ISZ] = reinterpret_cast<double(*)[ISZ]>(sm);
  double* ssum = sm + 1088;
  double* K22s = sm + 1360;   // K22 (+ noise + jitter on the diagonal), row-major
  double* Ts = sm + 1616;     // T_I image [64][16]
  double* Ln = sm;            // new rows of L inside the current block, [i][m]
  double* Ps = sm + 1024;     // L_WO Linv_OO of the current block, [i][c]
  double* Lb = sm + 2048;     // Linv_OO columns [cb, cb + LBW), [m][c - cb]
  double* L22s = sm + 3056;   // L22, row-major
  const int64_t bb0 = n0 / NB;
  const int nO0 = (int)(n0 - bb0 * NB);   // old rows in block bb0
  STAMP(20);
  // write-through: with status_host the launch's last cell group reads it (drained
  // with the L22 record before sync[2])
  if (tid == 0) __hip_atomic_store(d.status, INT_MAX, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  {
    // one K22 entry per thread (gp:523-529 via k_entry)
    const int a = tid / KINC, b = tid % KINC;
    K22s[tid] = (a < k && b <= a) ? k_entry_pts(h, NL, n0 + a, row_pt(d, n0 + a), n0 + b, row_pt(d, n0 + b)) : 0.0;
  }
  const bool gathered = n0 > 0 && ldx<FUSED>(d.iscr) != 0.0;
  inc_init_blocks<FUSED>(d, gathered ? n0 : 0, nblocks_factor(N) * NB, true);
  __syncthreads();
  STAMP(21);
  if (gathered) {
    const int64_t nch = (n0 + ch - 1) / ch;
    for (int e = tid; e < ISZ; e += NT) {
      // chunk partials in a fixed order; eight loads in flight per thread
      double acc = 0.0;
      for (int64_t c0 = 0; c0 < nch; c0 += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = (c0 + u < nch) ? ldx<FUSED>(d.iscr + ISC0 + (c0 + u) * ISZ + e) : 0.0;
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
      }
      ssum[e] = acc;
    }
  } else {
    // L21^T = L11^-1 K12, left-looking: T_I = K12_I - sum_{J<I} L_IJ W_J;  W_I = Linv_II T_I
    const int64_t nb0 = (n0 + NB - 1) / NB;
    for (int64_t I = 0; I < nb0; ++I) {
      const int64_t i0 = I * NB + w * 16;   // this wave's 16 rows
      d4 acc;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t row = i0 + q + 4 * v;
        acc[v] = (row < n0 && r < k) ? k_entry_pts(h, NL, row, X + 2 * row, n0 + r, row_pt(d, n0 + r)) : 0.0;
      }
      for (int64_t J = 0; J < I; ++J) {
#pragma unroll 4
        for (int t = 0; t < NB / 4; ++t) {
          const int64_t kc = J * NB + 4 * t + q;
          const double a = A[kc * ld + i0 + r];                                // L[i0 + r][kc]
          const double b = (r < k) ? ldx<FUSED>(&A[kc * ld + n0 + r]) : 0.0;   // W[kc][r]
          acc = mfma(-a, b, acc);
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) Ts[(w * 16 + q + 4 * v) * KINC + r] = acc[v];
      __syncthreads();
      const double* __restrict__ Li = d.Linv + I * TILE;
      d4 o = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
      for (int t = 0; t < NB / 4; ++t) {
        const int m = 4 * t + q;
        o = mfma(Li[m * NB + w * 16 + r], Ts[m * KINC + r], o);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t row = i0 + q + 4 * v;
        if (row < n0 && r < k) stx<FUSED>(&A[row * ld + n0 + r], o[v]);
      }
      if (FUSED) drain_stores();
      __syncthreads();   // W_I visible to every wave; Ts free
    }
    inc_schur_partial<NT / 64, FUSED, false, VT>(d, nullptr, 0, n0, red);
    if (FUSED) drain_stores();   // the compact rows, before sync[1]
    __syncthreads();
    for (int e = tid; e < ISZ; e += NT) ssum[e] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
    if (FUSED && tid == 0) publish(d.sync + 1, d.epoch);   // L21 is in A
  }
  __syncthreads();
  STAMP(22);
  // L22 = chol(K22 - L21 L21^T) and z2, wave 0 (LAPACK dpotf2 order, as in
  // factor_invert_64; lane r holds row r, DPP row broadcasts)
  if (w == 0) {
    double dd[KINC];
#pragma unroll
    for (int c = 0; c < KINC; ++c) {
      double v = (r == c) ? 1.0 : 0.0;
      if (r < k && c < k) v = K22s[r * KINC + c] - ssum[r * KINC + c];
      dd[c] = v;
    }
    const double yr = (r < k) ? row_obs(d, n0 + r) : 0.0;
    double rdiag = 1.0;
    int fail = INT_MAX;
#pragma unroll
    for (int j = 0; j < KINC; ++j) {
      double p = bcast16(dd[j], j);
      const bool pad = j >= k;
      const bool bad = !pad && !(p > 0.0);
      fail = bad ? min(fail, (int)(n0 + j + 1)) : fail;
      p = (pad || bad) ? 1.0 : p;
      const double rs = rsqrt(p);
      const double l = (r > j) ? dd[j] * rs : (r == j ? p * rs : 0.0);
      rdiag = (r == j) ? rs : rdiag;
      dd[j] = l;
      const double lu = (r > j) ? l : 0.0;
#pragma unroll
      for (int kk = j + 1; kk < KINC; ++kk) dd[kk] -= lu * bcast16(l, kk);
    }
    // z2 = L22^-1 (r2 - L21 z1), r2 = y - m_H (new rows are hifi; gp:133 / gp:421)
    double x = 0.0;
    if (r < k) x = (yr - h.meanH) - ssum[KINC * KINC + r];
#pragma unroll
    for (int j = 0; j < KINC; ++j) {
      if (r == j) x *= rdiag;
      const double zj = bcast16(x, j);
      if (r > j) x -= dd[j] * zj;
    }
    if (lane < k) {
#pragma unroll
      for (int c = 0; c < KINC; ++c) {
        L22s[lane * KINC + c] = (c <= lane) ? dd[c] : 0.0;
        if (c <= lane) stx<FUSED>(&A[(n0 + c) * ld + n0 + lane], dd[c]);
        // the record the cell workgroups read (no line of it is read before sync[2])
        stx<FUSED>(&d.l22r[lane * KINC + c], (c <= lane) ? dd[c] : 0.0);
      }
      stx<FUSED>(&d.zv[n0 + lane], x);
      stx<FUSED>(&d.l22r[KINC * KINC + lane], x);
    }
    if (fail != INT_MAX && lane == 0) atomicMin(d.status, fail);
    // the step's positive-definiteness verdict as soon as it is known (a mapped host
    // word: the eager append returns here while the posterior is still computed)
    if (FUSED && d.pd_host && lane == 0) __hip_atomic_store(d.pd_host, fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (FUSED) {
      drain_stores();
      if (lane == 0) publish(d.sync + 2, d.epoch);   // L22 and z2 are in A / zv
      WTRACE(3);
      if (FUSED) FSTAMP(32);
    }
  }
  __syncthreads();
  STAMP(23);
  // new rows' old-column part of block bb0 (L21 entries, in A)
  for (int e = tid; e < k * NB; e += NT) {
    const int i = e >> 6, m = e & 63;
    if (m < nO0) Ln[i * NB + m] = ldx<FUSED>(&A[(bb0 * NB + m) * ld + n0 + i]);
  }
  __syncthreads();
  STAMP(24);
  // new rows of the diagonal-block inverses. In block bb, with old rows O and new
  // rows W (a triangular inverse's rows do not depend on later rows):
  //   Linv_WO = -L_WW^-1 (L_WO Linv_OO),   Linv_WW = L_WW^-1
  // thread c: column c of the new rows, by forward substitution over the <= 16 new rows
  for (int64_t bb = bb0; bb * NB < N; ++bb) {
    double* __restrict__ Li = d.Linv + bb * TILE;
    const int64_t r0 = n0 > bb * NB ? n0 : bb * NB;
    const int64_t r1 = N < (bb + 1) * NB ? N : (bb + 1) * NB;
    const int nO = (int)(r0 - bb * NB), nW = (int)(r1 - r0);
    const int a0 = (int)(r0 - n0);   // first new row of this block, as a row of L22
    // L22 part of the new rows (columns n0.. of this block)
    for (int e = tid; e < nW * NB; e += NT) {
      const int i = e >> 6, m = e & 63;
      const int64_t col = bb * NB + m;
      if (col >= n0) {
        const int b = (int)(col - n0);
        Ln[i * NB + m] = (b <= a0 + i) ? L22s[(a0 + i) * KINC + b] : 0.0;
      } else if (bb != bb0) {
        Ln[i * NB + m] = ldx<FUSED>(&A[col * ld + r0 + i]);
      }
    }
    __syncthreads();
    // P = L_WO Linv_OO: element (i, c) per thread, Linv_OO lower triangular (its
    // upper part is stored as zeros), so the sum runs over all old rows m;
    // Linv_OO is staged through LDS LBW columns at a time
    for (int cb = 0; cb < nO; cb += LBW) {
      for (int e = tid; e < nO * LBW; e += NT) {
        const int c = e / nO, m = e - c * nO;   // consecutive threads: consecutive rows of one column
        Lb[m * LBW + c] = (cb + c < NB) ? Li[(cb + c) * NB + m] : 0.0;
      }
      __syncthreads();
      for (int e = tid; e < nW * LBW; e += NT) {
        const int i = e / LBW, c = e % LBW;
        double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
        int m = 0;
        for (; m + 4 <= nO; m += 4) {
          p0 += Ln[i * NB + m] * Lb[m * LBW + c];
          p1 += Ln[i * NB + m + 1] * Lb[(m + 1) * LBW + c];
          p2 += Ln[i * NB + m + 2] * Lb[(m + 2) * LBW + c];
          p3 += Ln[i * NB + m + 3] * Lb[(m + 3) * LBW + c];
        }
        for (; m < nO; ++m) p0 += Ln[i * NB + m] * Lb[m * LBW + c];
        Ps[i * NB + cb + c] = (p0 + p1) + (p2 + p3);
      }
      __syncthreads();
    }
    if (tid < NB) {
      const int c = tid;
      double xs[KINC];
#pragma unroll
      for (int i = 0; i < KINC; ++i) {
        xs[i] = 0.0;
        if (i < nW) {
          double t = (c < nO) ? -Ps[i * NB + c] : ((c == nO + i) ? 1.0 : 0.0);
#pragma unroll
          for (int i2 = 0; i2 < i; ++i2) t -= Ln[i * NB + nO + i2] * xs[i2];
          xs[i] = t / Ln[i * NB + nO + i];
          Li[c * NB + nO + i] = xs[i];
        }
      }
    }
    __syncthreads();
  }
  STAMP(25);
}

// ---------------------------------------------------------------------------
// Incremental predict: V is resident for rows < n0 and the factor has k = N - n0
// <= KINC new rows (k = 0: nothing appended since the last predict).
//   T      = psi_new^T - L21 V_old      (16 x n0 by n0 x 32 per wave, f64 MFMA)
//   V_new  = L22^-1 T                   -> rows [n0, N) of the resident V
//   var    = k** - colsum(V o V),  mu = m + V^T z   over all N rows
// V_old is read once: the kernel is HBM-bound. A workgroup covers 128 cells (two
// 64-cell V tiles) and each of its waves owns 32 cells over ALL n0 rows, so the
// stream needs no LDS and no barrier and a workgroup streams once per launch:
// at the headline size every cell workgroup is resident at once (one round, no
// tile-to-tile transitions, whose startup and epilogue round trips under full
// load left half the chip idle in the middle of the launch).
// Lane (r, q) of a wave: cells 2r, 2r + 1 of the wave's 32 (one 16-byte load per
// row), rows 4s + q of row step s; MFMA B operand = the cells' values, A operand =
// L21c[row][r] (rows r < k of L21, z1 at r = k, zeros above), so MFMA output row
// a is T (seeded with -psi_new) and row k is V_old^T z1. A ring of WS_S stages of
// WS_U row steps keeps WS_S - 1 stages of loads in flight while one is consumed.
// ---------------------------------------------------------------------------
constexpr int WS_CELLS = 32;            // cells per wave
constexpr int WS_WG = 4 * WS_CELLS;     // cells per workgroup (two V tiles; ntiles_wg)
// LDS of a cell workgroup (doubles): L22 (row-major) | z2 | new rows' (x, y) |
// cells' (x, y) | the row splits' partials (R = 4: 3 slots of 12 x 64)
constexpr int VS_LDS = KINC * KINC + KINC + 2 * KINC + 2 * WS_WG + 3 * 12 * 64;
static_assert(WS_WG == 2 * PBM, "a cell workgroup is two V tiles");
#ifndef MFGP_WS_U
#define MFGP_WS_U 2
#endif
#ifndef MFGP_WS_S
#define MFGP_WS_S 4
#endif
constexpr int WS_U = MFGP_WS_U, WS_S = MFGP_WS_S;
static_assert(WS_S >= 2, "a ring of at least two stages");

// psi of grid cell (gx, gy) against new training row g at (tx, ty): SF k, MF
// [rho k_L | rho^2 k_L + k_H] by the row's fidelity (gp:426-429), in the
// reference's operation order (as k_predict's psi)
__device__ __forceinline__ double psi_new(const Hyp& h, int64_t NL, int64_t g, double gx, double gy, double tx,
                                          double ty) {
#pragma clang fp contract(off)
  const double cLx = div_(gx, h.lL), cLy = div_(gy, h.lL);
  const double tLx = div_(tx, h.lL), tLy = div_(ty, h.lL);
  if (h.kind == 0) return se_scaled(cLx, cLy, tLx, tLy, h.sL);
  if (g < NL) return h.rho * se_scaled(cLx, cLy, tLx, tLy, h.sL);
  return h.rho2 * se_scaled(cLx, cLy, tLx, tLy, h.sL) +
         se_scaled(div_(gx, h.lH), div_(gy, h.lH), div_(tx, h.lH), div_(ty, h.lH), h.sH);
}

// MODE 0: k = 0 (no MFMA; V^T z by VALU). MODE 1: MFMA on L21 read from A (row
// stride ld, lanes r >= k masked), V^T z by VALU (k = KINC, or the compact rows
// are not for these rows). MODE 2: MFMA on the compact rows, V^T z1 = row k.
// Row steps per stage by mode: the rare modes carry z (and mask) registers and
// take one step per stage to stay inside the occupancy's register budget.
template <int MODE>
constexpr int ws_u() { return MODE == 2 ? WS_U : (MODE == 1 ? 1 : 2); }
template <int MODE>
constexpr int ws_s() { return MODE == 2 ? WS_S : (MODE == 1 ? 4 : 3); }

template <int MODE>
struct WsStage {
  dv2 v[ws_u<MODE>()];
  double a[ws_u<MODE>()], z[ws_u<MODE>()];
};

template <int MODE>
struct WsSrc {
  const GLOBAL dv2* vb;       // this lane's cells, row 0
  const GLOBAL double* ab;    // A operand, row 0 (MODE >= 1)
  int64_t astride;
  const GLOBAL double* zb;    // z, row 0 (MODE <= 1)
  int64_t n0;                 // end of this wave's row range
  int64_t j_lo;               // start of it (a multiple of 8)
};

// Rows j0 + 4u (u < WS_U) of this lane; GUARD clamps rows >= n0 to row 0.
template <int MODE, bool GUARD>
__device__ __forceinline__ void ws_load(WsStage<MODE>& s, const WsSrc<MODE>& src, int64_t j0) {
#pragma unroll
  for (int u = 0; u < ws_u<MODE>(); ++u) {
    const int64_t j = j0 + 4 * u;
    const int64_t jj = (!GUARD || j < src.n0) ? j : 0;   // clamped, loads stay unconditional
    // V is read once per update and is far larger than the Infinity Cache
    s.v[u] = __builtin_nontemporal_load(src.vb + jj * (PBM / 2));
    if (MODE >= 1) s.a[u] = src.ab[jj * src.astride];
    if (MODE <= 1) s.z[u] = src.zb[jj];
  }
}

// MODE 0 (the re-predict of an unchanged model) sums each cell's rows in four
// classes, (row mod 64) / 16, combined as ((0 + 1) + (2 + 3)) at the end: the
// order of k_predict's four waves, so a second predict() returns the same bits.
template <int MODE, bool GUARD>
__device__ __forceinline__ void ws_use(WsStage<MODE>& s, int64_t j0, int64_t n0, bool arow, d4* acc, double* vs,
                                       double* ms) {
  const int cls = MODE == 0 ? (int)((j0 & 63) >> 4) : 0;   // uniform: j0 = 4t + q
#pragma unroll
  for (int u = 0; u < ws_u<MODE>(); ++u) {
    if (GUARD && j0 + 4 * u >= n0) {
      s.v[u] = dv2{0.0, 0.0};
      s.a[u] = 0.0;
      s.z[u] = 0.0;
    }
    if (MODE == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c == cls) {   // explicit fma: k_predict's contracted a += x * y
          vs[2 * c] = __builtin_fma(s.v[u].x, s.v[u].x, vs[2 * c]);
          vs[2 * c + 1] = __builtin_fma(s.v[u].y, s.v[u].y, vs[2 * c + 1]);
          ms[2 * c] = __builtin_fma(s.v[u].x, s.z[u], ms[2 * c]);
          ms[2 * c + 1] = __builtin_fma(s.v[u].y, s.z[u], ms[2 * c + 1]);
        }
      continue;
    }
    vs[0] += s.v[u].x * s.v[u].x;
    vs[1] += s.v[u].y * s.v[u].y;
    if (MODE <= 1) {
      ms[0] += s.z[u] * s.v[u].x;
      ms[1] += s.z[u] * s.v[u].y;
    }
    if (MODE >= 1) {
      const double a = (MODE == 1 && !arow) ? 0.0 : s.a[u];
      acc[0] = mfma(a, s.v[u].x, acc[0]);
      acc[1] = mfma(a, s.v[u].y, acc[1]);
    }
  }
}

// The epilogue's L22 record, fetched during the stream: the sync[2] flag is read
// halfway (fused launches), the record itself at three quarters if the flag was
// up, so the epilogue skips both round trips (the finish publishes long before).
struct WsPrefetch {
  const unsigned* flag;   // null: nothing to prefetch
  unsigned epoch;
  const double* rec;      // KINC * KINC + KINC doubles
  unsigned fval;
  double r0, r1;          // rec[tid], rec[tid + NT] (tid + NT < record size)
  bool have;
};

__device__ __forceinline__ void ws_prefetch(WsPrefetch& pf, int64_t t, int64_t T) {
  if (!pf.flag) return;
  const int tid = threadIdx.x;
  if (t == T / 2) pf.fval = __hip_atomic_load(pf.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t == (3 * T) / 4) {
    pf.have = pf.fval == pf.epoch;
    if (pf.have) {
      // plain loads: no line of the record is read in this launch before sync[2]
      pf.r0 = pf.rec[tid];
      pf.r1 = tid + NT < KINC * KINC + KINC ? pf.rec[tid + NT] : 0.0;
    }
  }
}

// The row range [j_lo, n0) of this lane's cells: full stages pipelined, the
// ragged last stage guarded.
template <int MODE>
__device__ __forceinline__ void ws_stream(const WsSrc<MODE>& src, int q0, bool arow, d4* acc, double* vs,
                                          double* ms, WsPrefetch& pf) {
  constexpr int64_t RS = 4 * ws_u<MODE>();   // rows per stage
  constexpr int SS = ws_s<MODE>();           // stages in the ring
  const int64_t n0 = src.n0;
  const int64_t q = src.j_lo + q0;           // this lane's first row
  const int64_t T = (n0 - src.j_lo) / RS;    // full stages
  WsStage<MODE> st[SS];
#pragma unroll
  for (int s = 0; s < SS - 1; ++s)
    if (s < T) ws_load<MODE, false>(st[s], src, s * RS + q);
  int64_t t = 0;
  // steady state (sched_barrier keeps each stage's loads ahead of the use after it)
  for (; t + 2 * SS - 1 <= T; t += SS) {
    // the workgroups of a CU stream at unequal rates (the memory pipe favours the
    // oldest waves: 195 / 250 / 309 / 339 us for the four slots of a CU, measured),
    // so priority falls as a wave advances and the waves of a CU finish closer
    // together (3 stays with the producers and the finish, which the streams wait for)
    if (t >= (2 * T) / 3) __builtin_amdgcn_s_setprio(0);
    else if (t >= T / 3) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int s = 0; s < SS; ++s) ws_prefetch(pf, t + s, T);
#pragma unroll
    for (int s = 0; s < SS; ++s) {
      ws_load<MODE, false>(st[(s + SS - 1) % SS], src, (t + s + SS - 1) * RS + q);
      __builtin_amdgcn_sched_barrier(0);
      ws_use<MODE, false>(st[s], (t + s) * RS + q, n0, arow, acc, vs, ms);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // drain: fewer than 2 SS - 1 full stages left
#pragma unroll
  for (int s = 0; s < 2 * SS - 2; ++s) {
    if (t + s >= T) break;
    if (t + s + SS - 1 < T) ws_load<MODE, false>(st[(s + SS - 1) % SS], src, (t + s + SS - 1) * RS + q);
    ws_use<MODE, false>(st[s % SS], (t + s) * RS + q, n0, arow, acc, vs, ms);
  }
  if (src.j_lo + T * RS < n0) {
    const int64_t j0 = T * RS + q;
    ws_load<MODE, true>(st[0], src, j0);
    ws_use<MODE, true>(st[0], j0, n0, arow, acc, vs, ms);
  }
}

// Arrival of one wave's cell group (slot) of the launch, with its (max, first
// argmax) of var when the fused var max / argmax is asked for. The last group of
// the launch to arrive reduces the partials and, with status_host, copies the
// GP's status word into the mapped host word (every status write of the launch
// -- the finish's, a wait's timeout -- is drained before its group counts in).
// Write-through partials, a drain and a relaxed counter: no fence (a release
// fence writes the whole L2 back).
__device__ void var_argmax_group(const GPDesc& d, double bv, int64_t bi, int64_t slot, int64_t nslots) {
  const int lane = threadIdx.x & 63;
  const bool red = d.vmax || d.vargmax;
  unsigned* cnt = reinterpret_cast<unsigned*>(d.tred);   // tred = [counter | (max, argmax) per group]
  double* part = d.tred + 1;
  if (red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) argmax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  }
  unsigned old = 0;
  if (lane == 0) {
    if (red) {
      __hip_atomic_store(part + 2 * slot, bv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(part + 2 * slot + 1, (double)bi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  old = __shfl(old, 0);
  if (old != (unsigned)(nslots - 1)) return;
  if (red) {
    bv = -__builtin_inf();
    bi = INT64_MAX;
    for (int64_t t = lane; t < nslots; t += 64)
      argmax_pair(bv, bi, __hip_atomic_load(part + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                  (int64_t)__hip_atomic_load(part + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) argmax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  }
  if (lane == 0) {
    if (d.vmax) *d.vmax = bv;
    if (d.vargmax) *d.vargmax = bi;
    if (d.status_host) *d.status_host = __hip_atomic_load(d.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Value of register `v` of lane `src` (all lanes take part).
__device__ __forceinline__ double lane_get(double v, int src) { return __shfl(v, src); }

// One workgroup of the one-pass predict: 128 / R cells, R = d.rsplit row splits.
// Wave w owns cell group w % (4 / R) (32 cells) over row split w / (4 / R); with
// R > 1 (small batches, so that the chip still holds ~4 workgroups per CU) the
// splits' partial sums meet in LDS, added in split order. FUSED (inside
// k_inc_stream): the compact rows are read once sync[1] is signalled, L22 / z2
// once sync[2] is.
template <bool FUSED>
__device__ __forceinline__ void vstream_wg(const GPDesc& d, int64_t wgt, double* sm) {
  const int64_t M = d.M;
  const int64_t n0 = d.n0, N = d.N, ld = d.ld;
  const int k = (int)(N - n0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int R = d.rsplit;                   // 1, 2 or 4 (uniform)
  const int ncg = 4 / R;                    // cell groups per workgroup
  const int cpw = WS_CELLS * ncg;           // cells per workgroup
  const int si = w / ncg;                   // this wave's row split
  const int64_t cg = wgt * cpw + WS_CELLS * (w % ncg);   // first grid cell of this wave
  const int64_t vt = cg / PBM;              // its V tile
  const int cw = (int)(cg % PBM);           // and first cell inside it
  const bool live = cg < M;                 // a ragged last workgroup may hold empty groups
  double* __restrict__ Vt = d.V + vt * d.vld * PBM;
  const Hyp& h = d.hp;
  double* L22 = sm;                          // L22 (row-major) | z2
  double* Xn = sm + KINC * KINC + KINC;      // new rows' (x, y)
  double* Gc = Xn + 2 * KINC;                // the workgroup's cells' (x, y)
  const int64_t c0 = cg + 2 * r;             // this lane's cells c0, c0 + 1
  d4 acc[2];
  acc[0] = d4{0.0, 0.0, 0.0, 0.0};
  acc[1] = d4{0.0, 0.0, 0.0, 0.0};
  double vs[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, ms[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const bool mma = k > 0;
  const bool zrow = mma && k < KINC && d.l21c_ok;
  for (int e = tid; !FUSED && mma && e < KINC * KINC + KINC; e += NT) {
    // L22 | z2 (written by an earlier launch): the record of the append that
    // wrote the compact rows, else A / zv
    double v = 0.0;
    if (e < KINC * KINC) {
      const int ra = e / KINC, cb = e % KINC;
      if (ra < k && cb <= ra) v = d.l21c_ok ? d.l22r[e] : d.A[(n0 + cb) * ld + n0 + ra];
    } else if (e - KINC * KINC < k) {
      v = d.l21c_ok ? d.l22r[e] : d.zv[n0 + e - KINC * KINC];
    }
    L22[e] = v;
  }
  if (mma) {
    // the psi_new inputs through LDS (one 16-byte load per thread: the producers'
    // round trips at the start of the launch run beside this traffic)
    if (tid < cpw) {
      const int64_t cc = wgt * cpw + tid < M ? wgt * cpw + tid : M - 1;
      reinterpret_cast<dv2*>(Gc)[tid] = *reinterpret_cast<const GLOBAL dv2*>(gp(d.grid) + 2 * cc);
    } else if (tid >= NT - KINC) {
      const int a = tid - (NT - KINC);
      const double* p = row_pt(d, n0 + (a < k ? a : 0));
      Xn[2 * a] = p[0];
      Xn[2 * a + 1] = p[1];
    }
    __syncthreads();
  }
  if (live && mma && si == 0) {
    {
      // T = psi_new^T - L21 V_old: the accumulators start at -psi_new (MFMA output
      // row q + 4v of lane (r, q), cells c0 + x), so the epilogue has no exps left
      const int e0 = (int)(c0 - wgt * cpw);
      const double g0x = Gc[2 * e0], g0y = Gc[2 * e0 + 1], g1x = Gc[2 * e0 + 2], g1y = Gc[2 * e0 + 3];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int a = q + 4 * v;
        if (a < k) {
          const double tx = Xn[2 * a], ty = Xn[2 * a + 1];
          acc[0][v] = -psi_new(h, d.NL, n0 + a, g0x, g0y, tx, ty);
          acc[1][v] = -psi_new(h, d.NL, n0 + a, g1x, g1y, tx, ty);
        }
      }
    }
  }
  if (FUSED && mma) wait_l21(d);   // the compact rows of this append (all waves)
  WsPrefetch pf{(FUSED && mma) ? d.sync + 2 : nullptr, d.epoch, d.l22r, 0u, 0.0, 0.0, false};
  if (FUSED) WTRACE(1);
  // this wave's rows: split si of [0, n0) at multiples of 8 rows; a re-predict
  // (k = 0) streams all rows in split 0 (the exact summation order of k_predict)
  int64_t j_lo = 0, j_hi = n0;
  if (R > 1) {
    if (!mma) {
      j_hi = si == 0 ? n0 : 0;
    } else {
      j_lo = (si * n0 / R) & ~(int64_t)7;
      j_hi = si == R - 1 ? n0 : ((si + 1) * n0 / R) & ~(int64_t)7;
    }
  }
  if (live && j_hi > j_lo) {
    const GLOBAL dv2* vb = reinterpret_cast<const GLOBAL dv2*>(gp(Vt)) + (cw >> 1) + r;
    if (zrow) {
      const WsSrc<2> src{vb, gp(d.l21c) + r, KINC, nullptr, j_hi, j_lo};
      ws_stream<2>(src, q, true, acc, vs, ms, pf);
    } else if (mma) {
      const WsSrc<1> src{vb, gp(d.A) + n0 + (r < k ? r : 0), ld, gp(d.zv), j_hi, j_lo};
      ws_stream<1>(src, q, r < k, acc, vs, ms, pf);
    } else {
      const WsSrc<0> src{vb, nullptr, 0, gp(d.zv), j_hi, j_lo};
      ws_stream<0>(src, q, false, acc, vs, ms, pf);
    }
  }
  if (R > 1 && mma) {
    // the row splits' partials meet in LDS (lane-for-lane, before the lane
    // reductions), added to split 0's in split order
    double* part = Gc + 2 * WS_WG;   // [(R - 1) * ncg slots][12][64]
    if (si > 0) {
      double* pp = part + ((si - 1) * ncg + w % ncg) * 12 * 64 + lane;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        pp[v * 64] = acc[0][v];
        pp[(4 + v) * 64] = acc[1][v];
      }
      pp[8 * 64] = vs[0];
      pp[9 * 64] = vs[1];
      pp[10 * 64] = ms[0];
      pp[11 * 64] = ms[1];
    }
    __syncthreads();
    if (si == 0) {
      for (int sj = 1; sj < R; ++sj) {
        const double* pp = part + ((sj - 1) * ncg + w % ncg) * 12 * 64 + lane;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          acc[0][v] += pp[v * 64];
          acc[1][v] += pp[(4 + v) * 64];
        }
        vs[0] += pp[8 * 64];
        vs[1] += pp[9 * 64];
        ms[0] += pp[10 * 64];
        ms[1] += pp[11 * 64];
      }
    }
  }
  // colsums over the lanes' row residues q (and, for k = 0, the four row classes)
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    if (e >= 2 && mma) break;
    vs[e] += __shfl_xor(vs[e], 16);
    vs[e] += __shfl_xor(vs[e], 32);
    ms[e] += __shfl_xor(ms[e], 16);
    ms[e] += __shfl_xor(ms[e], 32);
  }
  if (!mma) {
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      vs[x] = (vs[x] + vs[2 + x]) + (vs[4 + x] + vs[6 + x]);
      ms[x] = (ms[x] + ms[2 + x]) + (ms[4 + x] + ms[6 + x]);
    }
  }
  if (FUSED) WTRACE(2);
  // L22 / z2 (sync[2]): from the stream's prefetch if every wave had it, else now
  const bool pre = (FUSED && mma) ? __syncthreads_and(pf.have) != 0 : false;
  if (pre) {
    for (int e = tid, i = 0; e < KINC * KINC + KINC; e += NT, ++i) {
      const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
      L22[e] = use ? (i == 0 ? pf.r0 : pf.r1) : 0.0;
    }
  }
  if (FUSED && mma && !pre) {
    // the workgroup's waves end their streams together
    if (tid == 0) {
      int it = 0;
      while (__hip_atomic_load(d.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != d.epoch) {
        __builtin_amdgcn_s_sleep(MFGP_SPIN_SLEEP);
        if (++it == (1 << 22)) {
          atomicMin(d.status, SYNC_FAIL);
          break;
        }
      }
    }
    __syncthreads();
    // plain loads: no line of the record is read in this launch before sync[2]
    // (an L2 miss for the first workgroup of an XCD, hits for the others)
    for (int e = tid; e < KINC * KINC + KINC; e += NT) {
      const double v = d.l22r[e];
      const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
      L22[e] = use ? v : 0.0;
    }
  }
  __syncthreads();
  if (FUSED) WTRACE(3);
  // epilogue: lane (r, x) with x = q < 2 finishes cell c0 + x. Row a of T for that
  // cell sits in acc[x][a / 4] of lane (r, a % 4).
  const int x = q & 1;
  const int64_t c = c0 + x;
  double vsum = x ? vs[1] : vs[0];
  double msum = x ? ms[1] : ms[0];
  if (mma) {
    if (zrow) {
      const double m0 = lane_get(acc[0][k / 4], r + 16 * (k % 4));
      const double m1 = lane_get(acc[1][k / 4], r + 16 * (k % 4));
      msum += x ? m1 : m0;
    }
    double vn[KINC];
#pragma unroll
    for (int a = 0; a < KINC; ++a) {
      vn[a] = 0.0;
      if (a < k) {
        const double t0 = lane_get(acc[0][a / 4], r + 16 * (a % 4));
        const double t1 = lane_get(acc[1][a / 4], r + 16 * (a % 4));
        double t = -(x ? t1 : t0);   // psi_new - L21 V_old
#pragma unroll
        for (int b = 0; b < a; ++b) t -= L22[a * KINC + b] * vn[b];
        vn[a] = t / L22[a * KINC + a];
        vsum += vn[a] * vn[a];
        msum += vn[a] * L22[KINC * KINC + a];
      }
    }
    if (live && si == 0 && q < 2 && c < M) {
#pragma unroll
      for (int a = 0; a < KINC; ++a)
        if (a < k) {
          gp(Vt)[(n0 + a) * PBM + cw + 2 * r + x] = vn[a];
        }
    }
  }
  const double vc = h.kss - vsum;
  const bool valid = live && si == 0 && q < 2 && c < M;
  if (valid) {
    d.mu[c] = msum + h.meanH;
    d.var[c] = vc;
    if (d.rmu) {
      d.rmu[c] = msum + h.meanH;
      d.rvar[c] = vc;
    }
  }
  if ((d.vmax || d.vargmax || d.status_host) && cg < M && si == 0)
    var_argmax_group(d, valid ? vc : -__builtin_inf(), valid ? c : INT64_MAX, cg / WS_CELLS,
                     (M + WS_CELLS - 1) / WS_CELLS);
  if (FUSED) WTRACE(4);
}

// ---------------------------------------------------------------------------
// One-pass predict over an fp32 V (MFGP_F32 models, BASELINE configs[4]): the
// same algorithm as vstream_wg, with V stored in fp32 -- half the bytes of the
// HBM-bound stream. Everything but V stays fp64: the factor, z, L21 (widened
// from the V gather), L22, the epilogue's solve for V_new, and both reductions
// (var = k** - colsum(V o V) and mu = m + V^T z accumulate in f64).
// Lane (r, q) of a wave: cells 4r .. 4r + 3 of the wave's 64 (one 64-cell V
// tile; one 16-byte load per row), rows 4s + q of row step s. T = psi_new^T -
// L21 V_old on the exact f32 MFMA (v_mfma_f32_16x16x4_f32), one per cell slot
// x: A = the compact rows (fp32: L21 rows 0..k-1, z1 in row ZROW), B = the
// slot's V entries; output lane (r, g) register v = row 4g + v, cell 4r + x.
// Row ZROW (lanes g = 3, register 3) is V_old^T z1: it is added into f64 and
// cleared once per pass of the stage ring, so no f32 sum runs over more than 32
// rows. T itself accumulates in f32 over all n0 rows (its error is divided by
// L22 >= sqrt(noise_H) in V_new). No row splits: 256 cells per workgroup.
// ---------------------------------------------------------------------------
constexpr int WF_CELLS = 64;            // cells per wave (one V tile)
constexpr int WF_WG = 4 * WF_CELLS;     // cells per workgroup (ntiles_wg(M, 1, 1))
constexpr int WF_LDS = KINC * KINC + KINC + 2 * KINC + 2 * WF_WG;
static_assert(WF_LDS <= FIN_LDS, "one LDS image serves every role");
static_assert(WF_WG == NT, "one thread per cell of the workgroup stages the psi inputs");
#ifndef MFGP_WF_S
#define MFGP_WF_S 4
#endif

// MODE as ws_*: 0 = k = 0 (VALU mean over z), 1 = A operand from A (widened
// to f32 per load; VALU mean), 2 = compact rows (mean from row ZROW).
template <int MODE>
constexpr int wf_u() { return 2; }
template <int MODE>
constexpr int wf_s() { return MODE == 2 ? MFGP_WF_S : 3; }

template <int MODE>
struct WfStage {
  f4 v[wf_u<MODE>()];
  float a[wf_u<MODE>()];
  double z[wf_u<MODE>()];
};

struct WfSrc {
  const GLOBAL f4* vb;        // this lane's cells, row 0
  const GLOBAL float* af;     // MODE 2: compact rows, this lane's entry of row 0
  const GLOBAL double* ad;    // MODE 1: A, row n0 + r of column 0
  int64_t astride;
  const GLOBAL double* zb;    // z, row 0 (MODE <= 1)
  int64_t n0;
};

template <int MODE, bool GUARD>
__device__ __forceinline__ void wf_load(WfStage<MODE>& s, const WfSrc& src, int64_t j0) {
#pragma unroll
  for (int u = 0; u < wf_u<MODE>(); ++u) {
    const int64_t j = j0 + 4 * u;
    const int64_t jj = (!GUARD || j < src.n0) ? j : 0;
    s.v[u] = __builtin_nontemporal_load(src.vb + jj * (PBM / 4));
    if (MODE == 2) s.a[u] = src.af[jj * KINC];
    if (MODE == 1) s.a[u] = (float)src.ad[jj * src.astride];
    if (MODE <= 1) s.z[u] = src.zb[jj];
  }
}

template <int MODE, bool GUARD>
__device__ __forceinline__ void wf_use(WfStage<MODE>& s, int64_t j0, int64_t n0, bool arow, f4* acc, double* vs,
                                       double* ms) {
#pragma unroll
  for (int u = 0; u < wf_u<MODE>(); ++u) {
    if (GUARD && j0 + 4 * u >= n0) {
      s.v[u] = f4{0.f, 0.f, 0.f, 0.f};
      s.a[u] = 0.f;
      s.z[u] = 0.0;
    }
    double vx[4];
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      vx[x] = (double)s.v[u][x];
      vs[x] = __builtin_fma(vx[x], vx[x], vs[x]);
      if (MODE <= 1) ms[x] = __builtin_fma(vx[x], s.z[u], ms[x]);
    }
    if (MODE >= 1) {
      const float a = (MODE == 1 && !arow) ? 0.f : s.a[u];
#pragma unroll
      for (int x = 0; x < 4; ++x) acc[x] = mfma(a, s.v[u][x], acc[x]);
    }
  }
}

// Row ZROW of the accumulators (lanes g = 3, register 3) into the f64 mean sums.
__device__ __forceinline__ void wf_flush_zrow(f4* acc, double* ms, bool zl) {
  static_assert(ZROW == 15, "row 15 = lane group 3, register 3");
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    const float t = acc[x][3];
    ms[x] += zl ? (double)t : 0.0;
    acc[x][3] = zl ? 0.f : t;
  }
}

template <int MODE>
__device__ __forceinline__ void wf_stream(const WfSrc& src, int q0, bool arow, f4* acc, double* vs, double* ms,
                                          WsPrefetch& pf) {
  constexpr int64_t RS = 4 * wf_u<MODE>();
  constexpr int SS = wf_s<MODE>();
  const int64_t n0 = src.n0;
  const int64_t q = q0;
  const int64_t T = n0 / RS;
  const bool zl = q0 == 3;
  WfStage<MODE> st[SS];
#pragma unroll
  for (int s = 0; s < SS - 1; ++s)
    if (s < T) wf_load<MODE, false>(st[s], src, s * RS + q);
  int64_t t = 0;
  for (; t + 2 * SS - 1 <= T; t += SS) {
    // as ws_stream: priority falls as a wave advances
    if (t >= (2 * T) / 3) __builtin_amdgcn_s_setprio(0);
    else if (t >= T / 3) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(2);
#pragma unroll
    for (int s = 0; s < SS; ++s) ws_prefetch(pf, t + s, T);
#pragma unroll
    for (int s = 0; s < SS; ++s) {
      wf_load<MODE, false>(st[(s + SS - 1) % SS], src, (t + s + SS - 1) * RS + q);
      __builtin_amdgcn_sched_barrier(0);
      wf_use<MODE, false>(st[s], (t + s) * RS + q, n0, arow, acc, vs, ms);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (MODE == 2) wf_flush_zrow(acc, ms, zl);
  }
#pragma unroll
  for (int s = 0; s < 2 * SS - 2; ++s) {
    if (t + s >= T) break;
    if (t + s + SS - 1 < T) wf_load<MODE, false>(st[(s + SS - 1) % SS], src, (t + s + SS - 1) * RS + q);
    wf_use<MODE, false>(st[s % SS], (t + s) * RS + q, n0, arow, acc, vs, ms);
  }
  if (T * RS < n0) {
    const int64_t j0 = T * RS + q;
    wf_load<MODE, true>(st[0], src, j0);
    wf_use<MODE, true>(st[0], j0, n0, arow, acc, vs, ms);
  }
  if (MODE == 2) wf_flush_zrow(acc, ms, zl);
}

// Pick element x of a per-slot quadruple (x uniform per lane).
__device__ __forceinline__ double pick4(double a0, double a1, double a2, double a3, int x) {
  return x == 0 ? a0 : (x == 1 ? a1 : (x == 2 ? a2 : a3));
}

// One workgroup of the fp32 one-pass predict: 256 cells, wave w owns cells
// [wgt * 256 + 64 w, +64) over all n0 rows. FUSED as vstream_wg.
template <bool FUSED>
__device__ __forceinline__ void vstream_wg_f32(const GPDesc& d, int64_t wgt, double* sm) {
  const int64_t M = d.M;
  const int64_t n0 = d.n0, N = d.N, ld = d.ld;
  const int k = (int)(N - n0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int64_t cg = wgt * WF_WG + WF_CELLS * w;   // first grid cell of this wave = its V tile's
  const bool live = cg < M;
  float* __restrict__ Vt = d.Vf + (cg / PBM) * d.vld * PBM;
  const Hyp& h = d.hp;
  double* L22 = sm;                          // L22 (row-major) | z2
  double* Xn = sm + KINC * KINC + KINC;      // new rows' (x, y)
  double* Gc = Xn + 2 * KINC;                // the workgroup's cells' (x, y)
  f4 acc[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) acc[x] = f4{0.f, 0.f, 0.f, 0.f};
  double vs[4] = {0.0, 0.0, 0.0, 0.0}, ms[4] = {0.0, 0.0, 0.0, 0.0};
  const bool mma = k > 0;
  const bool zrow = mma && k < KINC && d.l21c_ok;
  for (int e = tid; !FUSED && mma && e < KINC * KINC + KINC; e += NT) {
    double v = 0.0;
    if (e < KINC * KINC) {
      const int ra = e / KINC, cb = e % KINC;
      if (ra < k && cb <= ra) v = d.l21c_ok ? d.l22r[e] : d.A[(n0 + cb) * ld + n0 + ra];
    } else if (e - KINC * KINC < k) {
      v = d.l21c_ok ? d.l22r[e] : d.zv[n0 + e - KINC * KINC];
    }
    L22[e] = v;
  }
  if (mma) {
    {
      const int64_t cc = wgt * WF_WG + tid < M ? wgt * WF_WG + tid : M - 1;
      reinterpret_cast<dv2*>(Gc)[tid] = *reinterpret_cast<const GLOBAL dv2*>(gp(d.grid) + 2 * cc);
    }
    if (tid < KINC) {
      const double* p = row_pt(d, n0 + (tid < k ? tid : 0));
      Xn[2 * tid] = p[0];
      Xn[2 * tid + 1] = p[1];
    }
    __syncthreads();
  }
  if (live && mma) {
    // the accumulators start at -psi_new (row 4q + v of cell 4r + x), in f32
    const int e0 = WF_CELLS * w + 4 * r;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int a = 4 * q + v;
      if (a < k) {
        const double tx = Xn[2 * a], ty = Xn[2 * a + 1];
#pragma unroll
        for (int x = 0; x < 4; ++x)
          acc[x][v] = (float)(-psi_new(h, d.NL, n0 + a, Gc[2 * (e0 + x)], Gc[2 * (e0 + x) + 1], tx, ty));
      }
    }
  }
  if (FUSED && mma) wait_l21(d);
  WsPrefetch pf{(FUSED && mma) ? d.sync + 2 : nullptr, d.epoch, d.l22r, 0u, 0.0, 0.0, false};
  if (live && n0 > 0) {
    const GLOBAL f4* vb = reinterpret_cast<const GLOBAL f4*>(gp(Vt)) + r;
    if (zrow) {
      const WfSrc src{vb, reinterpret_cast<const GLOBAL float*>(gp(d.l21c)) + r, nullptr, 0, nullptr, n0};
      wf_stream<2>(src, q, true, acc, vs, ms, pf);
    } else if (mma) {
      const WfSrc src{vb, nullptr, gp(d.A) + n0 + (r < k ? r : 0), ld, gp(d.zv), n0};
      wf_stream<1>(src, q, r < k, acc, vs, ms, pf);
    } else {
      const WfSrc src{vb, nullptr, nullptr, 0, gp(d.zv), n0};
      wf_stream<0>(src, q, false, acc, vs, ms, pf);
    }
  }
  // colsums over the lanes' row residues q
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    vs[x] += __shfl_xor(vs[x], 16);
    vs[x] += __shfl_xor(vs[x], 32);
    ms[x] += __shfl_xor(ms[x], 16);
    ms[x] += __shfl_xor(ms[x], 32);
  }
  const bool pre = (FUSED && mma) ? __syncthreads_and(pf.have) != 0 : false;
  if (pre) {
    for (int e = tid, i = 0; e < KINC * KINC + KINC; e += NT, ++i) {
      const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
      L22[e] = use ? (i == 0 ? pf.r0 : pf.r1) : 0.0;
    }
  }
  if (FUSED && mma && !pre) {
    if (tid == 0) {
      int it = 0;
      while (__hip_atomic_load(d.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != d.epoch) {
        __builtin_amdgcn_s_sleep(MFGP_SPIN_SLEEP);
        if (++it == (1 << 22)) {
          atomicMin(d.status, SYNC_FAIL);
          break;
        }
      }
    }
    __syncthreads();
    for (int e = tid; e < KINC * KINC + KINC; e += NT) {
      const double v = d.l22r[e];
      const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
      L22[e] = use ? v : 0.0;
    }
  }
  __syncthreads();
  // epilogue: lane (r, q) finishes cell cg + 4r + q (slot x = q). Row a of T for
  // slot x sits in acc[x][a % 4] of lane (r, a / 4).
  const int x = q;
  const int64_t c = cg + 4 * r + x;
  double vsum = pick4(vs[0], vs[1], vs[2], vs[3], x);
  double msum = pick4(ms[0], ms[1], ms[2], ms[3], x);
  if (mma) {
    double vn[KINC];
#pragma unroll
    for (int a = 0; a < KINC; ++a) {
      vn[a] = 0.0;
      if (a < k) {
        const int src = r + 16 * (a / 4);
        const double t0 = (double)__shfl(acc[0][a % 4], src);
        const double t1 = (double)__shfl(acc[1][a % 4], src);
        const double t2 = (double)__shfl(acc[2][a % 4], src);
        const double t3 = (double)__shfl(acc[3][a % 4], src);
        double t = -pick4(t0, t1, t2, t3, x);   // psi_new - L21 V_old
#pragma unroll
        for (int b = 0; b < a; ++b) t -= L22[a * KINC + b] * vn[b];
        vn[a] = t / L22[a * KINC + a];
        vsum += vn[a] * vn[a];
        msum += vn[a] * L22[KINC * KINC + a];
      }
    }
    if (live && c < M) {
#pragma unroll
      for (int a = 0; a < KINC; ++a)
        if (a < k) gp(Vt)[(n0 + a) * PBM + 4 * r + x] = (float)vn[a];
    }
  }
  const double vc = h.kss - vsum;
  const bool valid = live && c < M;
  if (valid) {
    d.mu[c] = msum + h.meanH;
    d.var[c] = vc;
    if (d.rmu) {
      d.rmu[c] = msum + h.meanH;
      d.rvar[c] = vc;
    }
  }
  if ((d.vmax || d.vargmax || d.status_host) && live)
    var_argmax_group(d, valid ? vc : -__builtin_inf(), valid ? c : INT64_MAX, cg / WF_CELLS,
                     (M + WF_CELLS - 1) / WF_CELLS);
}

// Cells per one-pass-predict workgroup of descriptor d.
template <class VT>
__device__ __forceinline__ int64_t wg_cells(const GPDesc& d) {
  if constexpr (sizeof(VT) == 8) return WS_WG / d.rsplit;
  else return WF_WG;
}

template <class VT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_INC_WAVES, MFGP_INC_WAVES))) void k_vstream(
    const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  if ((int64_t)blockIdx.x * wg_cells<VT>(d) >= d.M) return;
  if (d.gate && *d.gate == 0) return;
  __shared__ double sm[VS_LDS > WF_LDS ? VS_LDS : WF_LDS];
  if constexpr (sizeof(VT) == 8) vstream_wg<false>(d, blockIdx.x, sm);
  else vstream_wg_f32<false>(d, blockIdx.x, sm);
}

// ---------------------------------------------------------------------------
// The bordered append (k_inc_stream). Grid (GPs, roles); per GP, roles < nprod
// are producers (inc_produce on FCH-row chunks of L21):
//   producers : gather L21 into A and their partials, drain, count arrivals
//               (sync[0]); the last one signals sync[1] (L21 complete, when
//               gathered), runs inc_finish (signals sync[1] itself when it
//               solves L21, then sync[2] once L22 / z2 are stored) and resets
//               sync[0] for the next launch.
// With d.tiles the same launch also runs the one-pass predict: roles >= nprod
// stream the 128-cell workgroups (vstream_wg<true>), waiting for sync[1] before
// the first L21 load and for sync[2] before the L22 solve of the epilogue. x = GP,
// so the linear dispatch order is every GP's producer 0, then producer 1, ...,
// then the cell workgroups round-robin over the GPs: producers are dispatched
// before any workgroup that waits for them and are therefore resident (no
// deadlock); the waits are bounded anyway. The flags hold the launch's epoch
// (host counter, never 0), so they need no reset. Without tiles nothing waits.
// Four workgroups per CU (128 VGPRs; 26.5 KB of LDS): at the headline size
// (8 GPs: 128 producers + 1024 cell workgroups) 1024 are resident at once and
// the last 128 cell workgroups take the producers' slots as they finish (9-15 us).
//
// Why the in-kernel hand-off is safe (gfx950: 8 XCDs, each with its own L2;
// per-CU L1; kernel boundaries write back and invalidate both):
//  * Forward progress. The dispatcher hands workgroups to the XCDs round-robin
//    in linear order (x = GP fastest, then role) and each XCD dispatches its
//    share in that order. Every producer has a lower linear id than every cell
//    workgroup, so on each XCD all its producers are dispatched before any of its
//    cell workgroups, and producers wait for nothing (the last arriver's finish
//    included). Producers therefore always run to completion even when they do
//    not all fit at once (configs[4]: 32 GPs x 64 producers = 2048 > 1024 slots),
//    and the cells waiting for them are released. The waits are bounded anyway
//    (~1 s, then MFGP_ERR_DEVICE via *status), and tests/test_codeobj.py checks
//    the code has no out-of-line calls (an outlined producer stalled it once).
//  * Visibility. Everything a producer hands over (L21 rows in A, the compact
//    rows, chunk partials, L22 record, z2) is stored with agent-scope atomic
//    stores (global_store ... sc1: written through the XCD's L2 to memory), then
//    drained (s_waitcnt vmcnt(0): the stores are acknowledged), and only then is
//    the flag stored (sc1). A consumer reads the flag with an agent-scope load
//    (sc1: not served from a stale L2 line). Data behind the flag is then read
//    either with sc1 loads (ldx<true>) or with plain loads of lines that no
//    workgroup of the launch reads before the flag is up (compact rows only after
//    every chunk's flag, the L22 record only after sync[2]); such a line cannot
//    be in this XCD's L2 or this CU's L1 (both invalidated at the kernel
//    boundary, never filled since), so the plain load fetches the written data.
//  * Cost. A release (buffer_wbl2 sc1) writes back the whole L2 -- +80 us per
//    step when 2048 workgroups did it -- and an acquire adds a buffer_inv sc1;
//    the construction above needs neither, at the price of the two rules: drain
//    before the flag, and no early read of a handed-over line.
// ---------------------------------------------------------------------------
// Producer role `role` < nprod of a fused append launch (k_inc_stream, k_inc_lat):
// gather its chunk of L21 and the partials, drain, count the arrival (sync[0]);
// the last one signals sync[1] (L21 complete, when gathered), runs inc_finish
// (which signals sync[1] itself when it solves L21, then sync[2]) and resets
// sync[0] for the next launch.
// `cell` [KINC] and `last` are LDS words of the caller's.
template <class VT>
__device__ __forceinline__ void inc_producer_role(const GPDesc& d, int64_t role, double* sm, int* cell,
                                                  unsigned& last) {
  const int64_t np = d.nprod;
  if (role == 0) FSTAMP(30);
  __builtin_amdgcn_s_setprio(3);   // producers and the finish before the cell streams
  const bool gathered = inc_produce<VT>(d, role, FCH, cell, reinterpret_cast<double(*)[ISZ]>(sm));
  FSTAMP(40);   // latest producer done storing (before the drain)
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(d.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (old == (unsigned)(np - 1)) ? 1u : 0u;
    if (last) {
      __hip_atomic_store(d.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (gathered) publish(d.sync + 1, d.epoch);   // every chunk of L21 is in A
    }
  }
  FSTAMP(31);   // latest producer arrival
  __syncthreads();
  WTRACE(1);
  if (last) inc_finish<true, VT>(d, sm, FCH);
  if (last) WTRACE(2);   // the hand-off accesses: tiles may stream concurrently
  WTRACE(4);
}

template <class VT>
__device__ __forceinline__ void inc_stream_wg(const GPDesc& d) {
  const int k = (int)(d.N - d.n0);
  if (k <= 0 || k > KINC) return;   // the host guarantees 0 < k <= KINC
  if (d.gate && *d.gate == 0) return;
  static_assert(VS_LDS <= FIN_LDS, "one LDS image serves every role");
  __shared__ double sm[FIN_LDS];
  WTRACE(0);
  const int64_t np = d.nprod, role = blockIdx.y;
  if (role >= np) {
    const int64_t wgt = role - np;
    if (d.tiles && wgt * wg_cells<VT>(d) < d.M) {
      if constexpr (sizeof(VT) == 8) vstream_wg<true>(d, wgt, sm);
      else vstream_wg_f32<true>(d, wgt, sm);
    }
    return;
  }
  __shared__ int cell[KINC];
  __shared__ unsigned last;
  inc_producer_role<VT>(d, role, sm, cell, last);
}

template <class VT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_INC_WAVES, MFGP_INC_WAVES))) void k_inc_stream(
    const GPDesc* __restrict__ descs) {
  inc_stream_wg<VT>(descs[blockIdx.x]);
}

// One GP, descriptor by value (kernarg segment: no upload copy before the launch).
template <class VT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_INC_WAVES, MFGP_INC_WAVES))) void k_inc_stream1(
    const GPDesc d) {
  inc_stream_wg<VT>(d);
}

// A batch of <= DESC_ARG_MAX GPs with the descriptors as the kernel argument
// (k_inc_lat_arg's reason: no per-step upload through the copy engine); the
// kernarg segment is indexed directly, a dynamic index into the by-value
// parameter would copy it to scratch.
template <class VT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_INC_WAVES, MFGP_INC_WAVES))) void k_inc_stream_arg(
    const DescArg a) {
  (void)a;
  const GPDesc* descs = (const GPDesc*)__builtin_amdgcn_kernarg_segment_ptr();
  inc_stream_wg<VT>(descs[blockIdx.x]);
}

#include "mfgp_lattice.inl"

// MFGP_F32 full predict: k_predict computed V in fp64 into the scratch d.V (the
// left-looking solve re-reads its own earlier rows, so it runs in fp64); rows
// [0, N) of every tile are rounded into the resident fp32 V. One workgroup per
// tile, 16-byte loads / 8-byte stores along the rows.
__global__ __launch_bounds__(NT) void k_vnarrow(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t t = blockIdx.x;
  if (t >= ntiles_grid(d.M)) return;
  const GLOBAL dv2* src = reinterpret_cast<const GLOBAL dv2*>(gp(d.V) + t * d.vld * PBM);
  GLOBAL float* dst = gp(d.Vf) + t * d.vld * PBM;
  const int64_t n2 = d.N * (PBM / 2);
  for (int64_t e = threadIdx.x; e < n2; e += NT) {
    const dv2 v = __builtin_nontemporal_load(src + e);
    typedef float fv2 __attribute__((ext_vector_type(2)));
    *reinterpret_cast<GLOBAL fv2*>(dst + 2 * e) = fv2{(float)v.x, (float)v.y};
  }
}

// One iteration of compute_sample_points (simulator.py:344-370) on the device:
// the cell of maximal posterior variance (its first occurrence, np.argmax) is
// appended as hifi row N - 1 with its posterior mean as the observation
// (sim:352-366), unless the maximal variance is at or below the threshold or
// max_points rows were chosen -- then the loop is over: *gate = 0 and every
// gated kernel after it is a no-op. state[1] counts the chosen points.
__global__ void k_choi_select(const GPDesc* __restrict__ descs, double threshold, double* __restrict__ points,
                              int64_t max_points) {
  const GPDesc& d = descs[0];
  if (threadIdx.x != 0 || *d.gate == 0) return;
  int64_t* cnt = reinterpret_cast<int64_t*>(d.gate) + 1;
  const double vmax = *d.vmax;
  const int64_t j = *d.vargmax;
  if (!(vmax > threshold) || *cnt >= max_points || j < 0 || j >= d.M) {
    *d.gate = 0;
    return;
  }
  const int64_t row = d.N - 1;
  const double gx = d.grid[2 * j], gy = d.grid[2 * j + 1];
  const_cast<double*>(d.X)[2 * row] = gx;
  const_cast<double*>(d.X)[2 * row + 1] = gy;
  const_cast<double*>(d.y)[row] = d.mu[j];
  points[2 * *cnt] = gx;
  points[2 * *cnt + 1] = gy;
  *cnt += 1;
}

// The batched form (mfgp_batch_sample_points): thread b decides for model b of the
// batch from its fused (max, argmax) -- stop at its threshold or its point budget
// (state[b] = {gate, count}), else take the argmax cell and its posterior mean as the
// next hifi row, staged in xn / yn at the model's place pos[b] among the batch
// step's members (its device-source rows), and record it in pts[b][count].
__global__ void k_choi_select_batch(int count, const int* __restrict__ pos, int64_t* __restrict__ state,
                                    const double* __restrict__ thr,
                                    const double* __restrict__ vmax, const int64_t* __restrict__ vargmax,
                                    const double* __restrict__ mu, const int64_t* __restrict__ moff,
                                    const double* const* __restrict__ grids, const int64_t* __restrict__ Ms,
                                    double* __restrict__ xn, double* __restrict__ yn, double* __restrict__ pts,
                                    int64_t max_points) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= count) return;
  int64_t* st = state + 2 * b;
  if (st[0] == 0) return;
  const double v = vmax[b];
  const int64_t j = vargmax[b], cnt = st[1];
  if (!(v > thr[b]) || cnt >= max_points || j < 0 || j >= Ms[b]) {
    st[0] = 0;
    return;
  }
  const double gx = grids[b][2 * j], gy = grids[b][2 * j + 1];
  const int p = pos[b];
  xn[2 * p] = gx;
  xn[2 * p + 1] = gy;
  yn[p] = mu[moff[b] + j];
  pts[2 * (b * max_points + cnt)] = gx;
  pts[2 * (b * max_points + cnt) + 1] = gy;
  st[1] = cnt + 1;
}

// Append the batch's new (device-resident) rows to every model's training set:
// one launch for the whole batch instead of two copies per model (full-refactor
// path; k_inc_l21 lands the rows of the bordered appends itself).
__global__ __launch_bounds__(64) void k_append(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.x];
  const int64_t kn = d.k_new;
  if (kn <= 0 || !d.srcX) return;
  double* X = const_cast<double*>(d.X);
  double* y = const_cast<double*>(d.y);
  const int64_t at = d.N - kn;
  for (int64_t e = threadIdx.x; e < 3 * kn; e += 64) {
    if (e < 2 * kn) X[2 * at + e] = d.srcX[e];
    else y[at + e - 2 * kn] = d.srcY[e - 2 * kn];
  }
}

// ---------------------------------------------------------------------------
#ifdef MFGP_STAMPS
hipError_t set_stamps(long long* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)); }
#endif
hipError_t launch_append(const GPDesc* d, int count, hipStream_t s) {
  hipLaunchKernelGGL(k_append, dim3(count), dim3(64), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_assemble(const GPDesc* d, int count, int64_t max_tiles, hipStream_t s) {
  hipLaunchKernelGGL(k_assemble, dim3((unsigned)max_tiles, count), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_potrf_diag(const GPDesc* d, int count, int kb, hipStream_t s) {
  hipLaunchKernelGGL(k_potrf_diag, dim3(count), dim3(NT), 0, s, d, kb);
  return hipGetLastError();
}
hipError_t launch_panel(const GPDesc* d, int count, int kb, int64_t max_below, hipStream_t s) {
  hipLaunchKernelGGL(k_panel, dim3((unsigned)max_below, count), dim3(NT), 0, s, d, kb);
  return hipGetLastError();
}
hipError_t launch_syrk(const GPDesc* d, int count, int kb, int64_t max_tri, int t0, hipStream_t s) {
  hipLaunchKernelGGL(k_syrk, dim3((unsigned)max_tri, count), dim3(NT), 0, s, d, kb, t0);
  return hipGetLastError();
}
hipError_t launch_syrk_blk(const GPDesc* d, int count, int kb0, int nk, int jmin, int jmax, int64_t max_tiles,
                           hipStream_t s) {
  if (max_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_syrk_blk, dim3((unsigned)max_tiles, count), dim3(NT), 0, s, d, kb0, nk, jmin, jmax);
  return hipGetLastError();
}
hipError_t launch_predict(const GPDesc* d, int count, int64_t max_ctiles, hipStream_t s) {
  hipLaunchKernelGGL(k_predict, dim3((unsigned)max_ctiles, count), dim3(PNT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_extract_z(const GPDesc* d, int count, int64_t max_n, hipStream_t s) {
  if (max_n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_extract_z, dim3((unsigned)((max_n + NT - 1) / NT), count), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_inc_factor(const GPDesc* d, int count, int64_t max_nprod, int vf32, hipStream_t s) {
  if (vf32) hipLaunchKernelGGL(k_inc_stream<float>, dim3(count, (unsigned)max_nprod), dim3(NT), 0, s, d);
  else hipLaunchKernelGGL(k_inc_stream<double>, dim3(count, (unsigned)max_nprod), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_choi_select_batch(int count, const int* pos, int64_t* state, const double* thr, const double* vmax,
                                    const int64_t* vargmax, const double* mu, const int64_t* moff,
                                    const double* const* grids, const int64_t* Ms, double* xn, double* yn,
                                    double* pts, int64_t max_points, hipStream_t s) {
  hipLaunchKernelGGL(k_choi_select_batch, dim3((count + 63) / 64), dim3(64), 0, s, count, pos, state, thr, vmax, vargmax,
                     mu, moff, grids, Ms, xn, yn, pts, max_points);
  return hipGetLastError();
}
hipError_t launch_choi_select(const GPDesc* d, double threshold, double* points, int64_t max_points,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_choi_select, dim3(1), dim3(64), 0, s, d, threshold, points, max_points);
  return hipGetLastError();
}
hipError_t launch_inc_stream(const GPDesc* d, int count, int64_t max_blocks, int vf32, hipStream_t s) {
  if (vf32) hipLaunchKernelGGL(k_inc_stream<float>, dim3(count, (unsigned)max_blocks), dim3(NT), 0, s, d);
  else hipLaunchKernelGGL(k_inc_stream<double>, dim3(count, (unsigned)max_blocks), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_inc_stream_arg(const GPDesc* h, int count, int64_t max_blocks, int vf32, hipStream_t s) {
  if (count < 1 || count > DESC_ARG_MAX) return hipErrorInvalidValue;
  DescArg a;
  std::memcpy(a.d, h, sizeof(GPDesc) * count);
  if (vf32) hipLaunchKernelGGL(k_inc_stream_arg<float>, dim3(count, (unsigned)max_blocks), dim3(NT), 0, s, a);
  else hipLaunchKernelGGL(k_inc_stream_arg<double>, dim3(count, (unsigned)max_blocks), dim3(NT), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_inc_stream1(const GPDesc& d, int64_t blocks, int vf32, hipStream_t s) {
  if (vf32) hipLaunchKernelGGL(k_inc_stream1<float>, dim3(1, (unsigned)blocks), dim3(NT), 0, s, d);
  else hipLaunchKernelGGL(k_inc_stream1<double>, dim3(1, (unsigned)blocks), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_vstream(const GPDesc* d, int count, int64_t max_ctiles, int vf32, hipStream_t s) {
  if (vf32) hipLaunchKernelGGL(k_vstream<float>, dim3((unsigned)max_ctiles, count), dim3(NT), 0, s, d);
  else hipLaunchKernelGGL(k_vstream<double>, dim3((unsigned)max_ctiles, count), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_inc_lat(const GPDesc* d, int count, int64_t max_blocks, int ka, int vf32, bool g1, hipStream_t s) {
  const dim3 g(count, (unsigned)max_blocks);
  if (g1) {
    if (ka == 8 && vf32) hipLaunchKernelGGL((k_inc_lat<8, float, true>), g, dim3(NT), 0, s, d);
    else if (ka == 8) hipLaunchKernelGGL((k_inc_lat<8, double, true>), g, dim3(NT), 0, s, d);
    else if (vf32) hipLaunchKernelGGL((k_inc_lat<16, float, true>), g, dim3(NT), 0, s, d);
    else hipLaunchKernelGGL((k_inc_lat<16, double, true>), g, dim3(NT), 0, s, d);
  } else {
    if (ka == 8 && vf32) hipLaunchKernelGGL((k_inc_lat<8, float, false>), g, dim3(NT), 0, s, d);
    else if (ka == 8) hipLaunchKernelGGL((k_inc_lat<8, double, false>), g, dim3(NT), 0, s, d);
    else if (vf32) hipLaunchKernelGGL((k_inc_lat<16, float, false>), g, dim3(NT), 0, s, d);
    else hipLaunchKernelGGL((k_inc_lat<16, double, false>), g, dim3(NT), 0, s, d);
  }
  return hipGetLastError();
}
hipError_t launch_inc_lat_arg(const GPDesc* h, int count, int64_t max_blocks, int ka, int vf32, bool g1,
                              hipStream_t s) {
  if (count < 1 || count > DESC_ARG_MAX) return hipErrorInvalidValue;
  DescArg a;
  std::memcpy(a.d, h, sizeof(GPDesc) * count);
  const dim3 g(count, (unsigned)max_blocks);
  if (g1) {
    if (ka == 8 && vf32) hipLaunchKernelGGL((k_inc_lat_arg<8, float, true>), g, dim3(NT), 0, s, a);
    else if (ka == 8) hipLaunchKernelGGL((k_inc_lat_arg<8, double, true>), g, dim3(NT), 0, s, a);
    else if (vf32) hipLaunchKernelGGL((k_inc_lat_arg<16, float, true>), g, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((k_inc_lat_arg<16, double, true>), g, dim3(NT), 0, s, a);
  } else {
    if (ka == 8 && vf32) hipLaunchKernelGGL((k_inc_lat_arg<8, float, false>), g, dim3(NT), 0, s, a);
    else if (ka == 8) hipLaunchKernelGGL((k_inc_lat_arg<8, double, false>), g, dim3(NT), 0, s, a);
    else if (vf32) hipLaunchKernelGGL((k_inc_lat_arg<16, float, false>), g, dim3(NT), 0, s, a);
    else hipLaunchKernelGGL((k_inc_lat_arg<16, double, false>), g, dim3(NT), 0, s, a);
  }
  return hipGetLastError();
}
hipError_t launch_lat_gemm2(const GPDesc* d, int count, int64_t max_tiles, int ka, int vf32, hipStream_t s) {
  const dim3 g(count, (unsigned)max_tiles);
  if (ka == 8 && vf32) hipLaunchKernelGGL((k_lat_gemm2<8, float>), g, dim3(G2NT), 0, s, d);
  else if (ka == 8) hipLaunchKernelGGL((k_lat_gemm2<8, double>), g, dim3(G2NT), 0, s, d);
  else if (vf32) hipLaunchKernelGGL((k_lat_gemm2<16, float>), g, dim3(G2NT), 0, s, d);
  else hipLaunchKernelGGL((k_lat_gemm2<16, double>), g, dim3(G2NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_lat_gemm2_arg(const GPDesc* h, int count, int64_t max_tiles, int ka, int vf32, hipStream_t s) {
  if (count < 1 || count > DESC_ARG_MAX) return hipErrorInvalidValue;
  DescArg a;
  std::memcpy(a.d, h, sizeof(GPDesc) * count);
  const dim3 g(count, (unsigned)max_tiles);
  if (ka == 8 && vf32) hipLaunchKernelGGL((k_lat_gemm2_arg<8, float>), g, dim3(G2NT), 0, s, a);
  else if (ka == 8) hipLaunchKernelGGL((k_lat_gemm2_arg<8, double>), g, dim3(G2NT), 0, s, a);
  else if (vf32) hipLaunchKernelGGL((k_lat_gemm2_arg<16, float>), g, dim3(G2NT), 0, s, a);
  else hipLaunchKernelGGL((k_lat_gemm2_arg<16, double>), g, dim3(G2NT), 0, s, a);
  return hipGetLastError();
}
hipError_t launch_lat_axes(const GPDesc* d, int count, int64_t max_tabw, hipStream_t s) {
  hipLaunchKernelGGL(k_lat_axes, dim3((unsigned)((4 * (max_tabw + 1) + 3) / 4), count), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_lat_tables(const GPDesc* d, int count, int64_t max_rows, hipStream_t s) {
  if (max_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_lat_tables, dim3((unsigned)((max_rows + 3) / 4), count), dim3(NT), 0, s, d);
  return hipGetLastError();
}
hipError_t launch_vnarrow(const GPDesc* d, int count, int64_t max_tiles, hipStream_t s) {
  if (max_tiles <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_vnarrow, dim3((unsigned)max_tiles, count), dim3(NT), 0, s, d);
  return hipGetLastError();
}

}  // namespace mfgp
