// Negative log-marginal likelihood and its gradient for gfx950 (MI355X), fp64.
//
// Reference: likelihood (gaussian_process.py:81-106 SF, 344-385 MF), minimised by
// train (gp:108-119 / 388-399) with autograd's value_and_grad and L-BFGS-B:
//   NLML = 1/2 r^T K^-1 r + sum_i log L_ii + N/2 log(2 pi),   r = y - m(hyp)
// Its gradient is analytic here:
//   dNLML/dh = 1/2 tr((K^-1 - a a^T) dK/dh) + a^T dr/dh,     a = K^-1 r
// The factor is the library's (k_assemble .. k_extract_z on a scratch model with
// the given hyperparameters). Then:
//   k_nlml_value  sum log L_ii and |z|^2 (z = L^-1 r, so r^T K^-1 r = |z|^2)
//   k_trinv       X = L^-1, block column per workgroup, left-looking, f64 MFMA
//   k_kinv        K^-1 = X^T X, lower 64x64 tiles, f64 MFMA
//   k_alpha       a = X^T z
//   k_nlml_grad   per lower tile: W = K^-1 - a a^T times every dK/dh (the SE
//                 kernel's derivatives in the reference's operation order), reduced
// The mean terms a^T dr/dh are O(N) and summed on the host.
#include <hip/hip_runtime.h>

#include "mfgp_device.h"
#include "mfgp_internal.h"

namespace mfgp {

constexpr int NHYP = 9;

__global__ __launch_bounds__(NT) void k_nlml_value(const GPDesc* __restrict__ descs, double* __restrict__ out) {
  const GPDesc& d = descs[blockIdx.x];
  const int64_t N = d.N, ld = d.ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  __shared__ double red[2][NT / 64];
  double sl = 0.0, sz = 0.0;
  for (int64_t i = tid; i < N; i += NT) {
    sl += log(d.A[i * ld + i]);
    const double z = d.zv[i];
    sz += z * z;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sl += __shfl_xor(sl, off);
    sz += __shfl_xor(sz, off);
  }
  if (lane == 0) {
    red[0][w] = sl;
    red[1][w] = sz;
  }
  __syncthreads();
  if (tid == 0) {
    out[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    out[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// Ts[swz(k, i)] = G[(c0 + i) * ld + r0 + k]: a 64x64 tile read along its columns'
// rows (k contiguous in memory), i.e. the k-major image of the tile's transpose;
// rows r0 + k >= nrows read as 0.
__device__ __forceinline__ void load_tile_rm(double* __restrict__ Ts, const double* __restrict__ G, int64_t ld,
                                             int64_t r0, int64_t c0, int64_t nrows, int tid) {
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int i = p * 8 + (tid >> 5);
    const int k = (tid & 31) * 2;
    const dv2 v = *reinterpret_cast<const GLOBAL dv2*>(gp(G) + (c0 + i) * ld + r0 + k);
    Ts[swz(k, i)] = (r0 + k < nrows) ? v.x : 0.0;
    Ts[swz(k + 1, i)] = (r0 + k + 1 < nrows) ? v.y : 0.0;
  }
}

__device__ __forceinline__ void store_acc_cm(const Acc& acc, double* __restrict__ G, int64_t ld, int64_t r0,
                                             int64_t c0, double scale, int wm, int wn, int lane) {
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        G[(c0 + acc_col(wn, nt, r)) * ld + r0 + acc_row(wm, mt, q, v)] = scale * acc.c[mt][nt][v];
}

// X = L^-1 (lower, block rows/columns of 64). Block column J per workgroup:
//   X_JJ = Linv_JJ;   X_IJ = Linv_II * (-(sum_{K=J}^{I-1} L_IK X_KJ))  for I > J.
__global__ __launch_bounds__(NT) void k_trinv(const GPDesc* __restrict__ descs, double* __restrict__ Xi) {
  const GPDesc& d = descs[0];
  const int64_t ld = d.ld, nbr = nblocks_rows(d.N);
  const int64_t J = blockIdx.x;
  if (J >= nbr) return;
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  for (int64_t I = J; I < nbr; ++I) {
    Acc acc;
    acc_zero(acc);
    for (int64_t K = J; K < I; ++K) {
      load_tile_cm(As, d.A, ld, I * NB, K * NB, tid);          // As[k][i] = L_IK[i][k]
      load_tile_rm(Bs, Xi, ld, K * NB, J * NB, ld, tid);       // Bs[k][j] = X_KJ[k][j]
      __syncthreads();
      tile_mma<true>(As, Bs, acc, wm, wn, lane);               // acc -= L_IK X_KJ
      __syncthreads();
    }
    load_tile_cm(As, d.Linv + I * TILE, NB, 0, 0, tid);        // As[k][i] = Linv_II[i][k]
    if (I == J) {
      for (int e = tid; e < TILE; e += NT) {
        const int i = e & 63, k = e >> 6;
        Bs[swz(k, i)] = (i == k) ? 1.0 : 0.0;                  // X_JJ = Linv_JJ * I
      }
    } else {
      // Bs[k][j] = T[k][j] from the accumulator (row k = acc row, column j = acc col)
      const int r = lane & 15, q = lane >> 4;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int v = 0; v < 4; ++v) Bs[swz(acc_row(wm, mt, q, v), acc_col(wn, nt, r))] = acc.c[mt][nt][v];
    }
    __syncthreads();
    Acc o;
    acc_zero(o);
    tile_mma<false>(As, Bs, o, wm, wn, lane);
    store_acc_cm(o, Xi, ld, I * NB, J * NB, 1.0, wm, wn, lane);
    __threadfence_block();
    __syncthreads();
  }
}

// The same for a batch (grid (block columns, GPs)): F = L^-1 of the n0 leading
// factor rows into each GP's resident F, stored by 64-column blocks, each block's
// rows contiguous (fblk_off: the lattice step streams a block's rows i >= 64 jb as
// one contiguous range; k_inc_lat then appends its rows). Within block J the tile
// X_KJ is a row-major 64 x 64 tile with row stride 64.
__global__ __launch_bounds__(NT) void k_trinv_f(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t ld = d.ld, nbr = nblocks_rows(d.n0);
  const int64_t J = blockIdx.x;
  if (J >= nbr || !d.lat_fbuild) return;
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int r = lane & 15, q = lane >> 4;
  // block J as a row-major matrix of absolute rows, row stride 64
  double* Xt = d.F + fblk_off(J, ld) - 64 * J * NB;
  for (int64_t I = J; I < nbr; ++I) {
    Acc acc;
    acc_zero(acc);
    for (int64_t K = J; K < I; ++K) {
      load_tile_cm(As, d.A, ld, I * NB, K * NB, tid);          // As[k][i] = L_IK[i][k]
      load_tile_cm(Bs, Xt, NB, 0, K * NB, tid);                // Bs[k][j] = X_KJ[k][j] (row-major block)
      __syncthreads();
      tile_mma<true>(As, Bs, acc, wm, wn, lane);               // acc -= L_IK X_KJ
      __syncthreads();
    }
    load_tile_cm(As, d.Linv + I * TILE, NB, 0, 0, tid);        // As[k][i] = Linv_II[i][k]
    if (I == J) {
      for (int e = tid; e < TILE; e += NT) {
        const int i = e & 63, k = e >> 6;
        Bs[swz(k, i)] = (i == k) ? 1.0 : 0.0;
      }
    } else {
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
          for (int v = 0; v < 4; ++v) Bs[swz(acc_row(wm, mt, q, v), acc_col(wn, nt, r))] = acc.c[mt][nt][v];
    }
    __syncthreads();
    Acc o;
    acc_zero(o);
    tile_mma<false>(As, Bs, o, wm, wn, lane);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          Xt[(I * NB + acc_row(wm, mt, q, v)) * NB + acc_col(wn, nt, r)] = o.c[mt][nt][v];
    __threadfence_block();
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// F = L^-1 of the n0 leading factor rows by recursive doubling (the lattice
// step's F; replaces the block-column k_trinv_f, whose first workgroup ran the
// whole column's chain of ~n0^2 / 8192 tile products, 1.9 ms for 8 GPs at the
// headline). With L = [A 0; B C] over a group of 2h blocks of 64,
//   L^-1 = [A^-1 0; -C^-1 B A^-1  C^-1],
// so once every h-block diagonal group is inverted (level l - 1), level l (h =
// 2^l) finishes the 2h-block groups in two launches of independent 64x64 output
// tiles: T = B A^-1 (T_ij = sum_{k >= j} B_ik F11_kj), then F21 = -C^-1 T
// (sum_{k <= i} F22_ik T_kj). Level 0's diagonal tiles are the factor's Linv
// blocks. The top level's products are 16 deep at n0 = 2048 instead of 528.
// Tiles of F are row-major 64 x 64 (fblk_off), T is a row-major scratch per GP.
// ---------------------------------------------------------------------------
// Level -1: the diagonal tiles F_JJ = Linv_JJ (row-major in F, column-major in Linv).
__global__ __launch_bounds__(NT) void k_trinv_diag(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t J = blockIdx.x;
  if (!d.lat_fbuild || J >= nblocks_rows(d.n0)) return;
  const double* Li = d.Linv + J * TILE;
  double* Ft = d.F + fblk_off(J, d.ld);
  for (int e = threadIdx.x; e < TILE; e += NT) {
    const int r = e >> 6, c = e & 63;
    Ft[e] = Li[c * NB + r];
  }
}

// Level l, phase 0 (T = B F11) or 1 (F21 = -F22 T). Grid (groups x h x h tiles, GPs).
template <int PHASE>
__global__ __launch_bounds__(NT) void k_trinv_lvl(const GPDesc* __restrict__ descs, int h, double* __restrict__ tscr,
                                                  int64_t tstride) {
  const GPDesc& d = descs[blockIdx.y];
  if (!d.lat_fbuild) return;
  const int64_t nbr = nblocks_rows(d.n0), ld = d.ld;
  const int64_t hh = (int64_t)h * h;
  const int64_t grp = blockIdx.x / hh, rem = blockIdx.x % hh;
  const int i = (int)(rem / h), j = (int)(rem % h);
  const int64_t s = grp * 2 * h;                   // first block of the group
  const int64_t h2 = nbr - s - h < h ? nbr - s - h : h;   // blocks in its second half
  if (i >= h2) return;
  double* const T = tscr + blockIdx.y * tstride + (grp * hh + (int64_t)i * h + j) * TILE;
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int r = lane & 15, q = lane >> 4;
  // operand tiles of product t: phase 0: A = B_ik (L, column-major), B = F11_kj
  // (row-major), k = j + t; phase 1: A = F22_ik (row-major), B = T_kj, k = t
  const int k0 = PHASE == 0 ? j : 0, k1 = PHASE == 0 ? h : i + 1;
  auto a_src = [&](int k) -> const double* {
    if (PHASE == 0) return d.A + (s + k) * NB * ld + (s + h + i) * NB;   // column-major tile, leading dim ld
    return d.F + fblk_off(s + h + k, ld) + (int64_t)(i - k) * TILE;      // F22_ik: block column s+h+k, row s+h+i
  };
  auto b_src = [&](int k) -> const double* {
    if (PHASE == 0) return d.F + fblk_off(s + j, ld) + (int64_t)(k - j) * TILE;   // F11_kj
    return tscr + blockIdx.y * tstride + (grp * hh + (int64_t)k * h + j) * TILE;  // T_kj
  };
  Acc acc;
  acc_zero(acc);
  TileRegs ra, rb;
  if (k0 < k1) {
    tile_fetch(ra, a_src(k0), PHASE == 0 ? ld : NB, tid);
    tile_fetch(rb, b_src(k0), NB, tid);
  }
  for (int k = k0; k < k1; ++k) {
    __syncthreads();   // the previous product's LDS reads are done
    if (PHASE == 0) tile_put_k(As, ra, tid);   // column-major B_ik: memory rows are its columns -> As[k][i] = B[i][k]
    else tile_put_t(As, ra, tid);              // row-major F22_ik: As[k][i] = F[i][k]
    tile_put_k(Bs, rb, tid);                   // row-major right operand: Bs[k][j] = X[k][j]
    __syncthreads();
    if (k + 1 < k1) {                          // the next product's tiles in flight during this one
      tile_fetch(ra, a_src(k + 1), PHASE == 0 ? ld : NB, tid);
      tile_fetch(rb, b_src(k + 1), NB, tid);
    }
    tile_mma<PHASE == 1>(As, Bs, acc, wm, wn, lane);
  }
  double* const out = PHASE == 0 ? T : d.F + fblk_off(s + j, ld) + (int64_t)(h + i - j) * TILE;   // F21_ij
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int v = 0; v < 4; ++v) out[acc_row(wm, mt, q, v) * NB + acc_col(wn, nt, r)] = acc.c[mt][nt][v];
}

// K^-1 = X^T X over the real rows (k < N): tile (I, J), I >= J, sums K >= I.
__global__ __launch_bounds__(NT) void k_kinv(const GPDesc* __restrict__ descs, const double* __restrict__ Xi,
                                             double* __restrict__ Kv) {
  const GPDesc& d = descs[0];
  const int64_t ld = d.ld, N = d.N, nbr = nblocks_rows(N);
  int I, J;
  tri_index(blockIdx.x, I, J);
  if (I >= nbr) return;
  __shared__ double As[TILE], Bs[TILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  Acc acc;
  acc_zero(acc);
  for (int64_t K = I; K < nbr; ++K) {
    load_tile_rm(As, Xi, ld, K * NB, (int64_t)I * NB, N, tid);   // As[k][i] = X_KI[k][i]
    load_tile_rm(Bs, Xi, ld, K * NB, (int64_t)J * NB, N, tid);   // Bs[k][j] = X_KJ[k][j]
    __syncthreads();
    tile_mma<false>(As, Bs, acc, wm, wn, lane);
    __syncthreads();
  }
  store_acc_cm(acc, Kv, ld, (int64_t)I * NB, (int64_t)J * NB, 1.0, wm, wn, lane);
}

// a = X^T z over the real rows: a_j = sum_{k >= j, k < N} X[k][j] z_k.
__global__ __launch_bounds__(NT) void k_alpha(const GPDesc* __restrict__ descs, const double* __restrict__ Xi,
                                              double* __restrict__ alpha) {
  const GPDesc& d = descs[0];
  const int64_t ld = d.ld, N = d.N;
  const int64_t j = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= N) return;
  double s = 0.0;
  for (int64_t k = j + lane; k < N; k += 64) s += Xi[j * ld + k] * d.zv[k];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) alpha[j] = s;
}

// 1/2 sum_ij W_ij dK_ij/dh over the lower triangle (off-diagonal pairs twice).
// SF hyp [m, s, l, sn]; MF hyp [mL, sL, lL, mH, sH, lH, rho, snL, snH] (log-scaled).
__global__ __launch_bounds__(NT) void k_nlml_grad(const GPDesc* __restrict__ descs, const double* __restrict__ Kv,
                                                  const double* __restrict__ alpha, double* __restrict__ part) {
#pragma clang fp contract(off)
  const GPDesc& d = descs[0];
  const int64_t ld = d.ld, N = d.N, NL = d.NL, nbr = nblocks_rows(N);
  const Hyp& h = d.hf;
  int I, J;
  tri_index(blockIdx.x, I, J);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  double g[NHYP];
#pragma unroll
  for (int p = 0; p < NHYP; ++p) g[p] = 0.0;
  if (I < nbr) {
    for (int e = tid; e < TILE; e += NT) {
      const int i = e & 63, j = e >> 6;
      const int64_t gi = (int64_t)I * NB + i, gj = (int64_t)J * NB + j;
      if (gi >= N || gj >= N || gj > gi) continue;
      const double W = Kv[gj * ld + gi] - alpha[gi] * alpha[gj];
      const double wt = (gi == gj) ? 0.5 * W : W;   // 1/2 * (2 for the symmetric pair, 1 on the diagonal)
      const double xi = d.X[2 * gi], yi = d.X[2 * gi + 1], xj = d.X[2 * gj], yj = d.X[2 * gj + 1];
      const double dxL = div_(xi, h.lL) - div_(xj, h.lL), dyL = div_(yi, h.lL) - div_(yj, h.lL);
      const double rL2 = dxL * dxL + dyL * dyL;
      const double EL = h.sL * exp(-0.5 * rL2);
      if (h.kind == 0) {
        g[1] += wt * EL;
        g[2] += wt * (EL * rL2);
        if (gi == gj) g[3] += wt * h.noiseL;
      } else {
        const bool li = gi < NL, lj = gj < NL;
        const double cL = (li && lj) ? 1.0 : ((!li && !lj) ? h.rho2 : h.rho);
        const double dr = (li && lj) ? 0.0 : ((!li && !lj) ? 2.0 * h.rho2 : h.rho);
        g[1] += wt * (cL * EL);
        g[2] += wt * (cL * EL * rL2);
        g[6] += wt * (dr * EL);
        if (!li && !lj) {
          const double dxH = div_(xi, h.lH) - div_(xj, h.lH), dyH = div_(yi, h.lH) - div_(yj, h.lH);
          const double rH2 = dxH * dxH + dyH * dyH;
          const double EH = h.sH * exp(-0.5 * rH2);
          g[4] += wt * EH;
          g[5] += wt * (EH * rH2);
        }
        if (gi == gj) {
          if (li) g[7] += wt * h.noiseL;
          else g[8] += wt * h.noiseH;
        }
      }
    }
  }
  __shared__ double red[NT / 64][NHYP];
#pragma unroll
  for (int p = 0; p < NHYP; ++p) {
    double v = g[p];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0) red[w][p] = v;
  }
  __syncthreads();
  if (tid < NHYP) part[(int64_t)blockIdx.x * NHYP + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

hipError_t launch_trinv_f(const GPDesc* d, int count, int64_t max_nbr, double* tscr, int64_t tstride, hipStream_t s) {
  if (max_nbr <= 0 || count <= 0) return hipSuccess;
  if (!tscr) {   // (no scratch: the block-column form)
    hipLaunchKernelGGL(k_trinv_f, dim3((unsigned)max_nbr, count), dim3(NT), 0, s, d);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_trinv_diag, dim3((unsigned)max_nbr, count), dim3(NT), 0, s, d);
  for (int64_t h = 1; h < max_nbr; h *= 2) {
    const int64_t groups = (max_nbr + 2 * h - 1) / (2 * h);
    const dim3 grid((unsigned)(groups * h * h), count);
    hipLaunchKernelGGL(k_trinv_lvl<0>, grid, dim3(NT), 0, s, d, (int)h, tscr, tstride);
    hipLaunchKernelGGL(k_trinv_lvl<1>, grid, dim3(NT), 0, s, d, (int)h, tscr, tstride);
  }
  return hipGetLastError();
}
// doubles of T scratch per GP for recursive doubling over nbr blocks: the largest
// level's groups x h x h tiles
int64_t trinv_scratch(int64_t nbr) {
  int64_t m = 0;
  for (int64_t h = 1; h < nbr; h *= 2) m = std::max(m, (nbr + 2 * h - 1) / (2 * h) * h * h);
  return m * TILE;
}
hipError_t launch_nlml_value(const GPDesc* d, int count, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_nlml_value, dim3(count), dim3(NT), 0, s, d, out);
  return hipGetLastError();
}

hipError_t launch_nlml_grad(const GPDesc* d, int64_t N, double* Xi, double* Kv, double* alpha, double* part,
                            hipStream_t s) {
  const int64_t nbr = nblocks_rows(N);
  if (nbr <= 0) return hipSuccess;
  const int64_t ntri = nbr * (nbr + 1) / 2;
  hipLaunchKernelGGL(k_trinv, dim3((unsigned)nbr), dim3(NT), 0, s, d, Xi);
  hipLaunchKernelGGL(k_kinv, dim3((unsigned)ntri), dim3(NT), 0, s, d, Xi, Kv);
  hipLaunchKernelGGL(k_alpha, dim3((unsigned)((N + NT / 64 - 1) / (NT / 64))), dim3(NT), 0, s, d, Xi, alpha);
  hipLaunchKernelGGL(k_nlml_grad, dim3((unsigned)ntri), dim3(NT), 0, s, d, Kv, alpha, part);
  return hipGetLastError();
}

int64_t nlml_partials(int64_t N) {
  const int64_t nbr = nblocks_rows(N);
  return nbr * (nbr + 1) / 2 * NHYP;
}

}  // namespace mfgp
