// Voronoi-cell reductions over the grid for gfx950 (MI355X), fp64.
//
// Reference (MSU-dcypherlab/mfgp-coverage, simulator.py): after every posterior
// update the planners reduce the grid cell by cell over the bounded Voronoi
// partition of the agents (voronoi_bounded, sim:154-191):
//   compute_centroids (sim:231-283): sum of mu, mu*x, mu*y over the cell's points
//   compute_max_var   (sim:286-323): max and first argmax of var in the cell
//   compute_loss      (sim:194-228): mean of |x - seed|^2 * f over the cell
// Membership is the reference's in_polygon (sim:105-124), matplotlib's
// Path.contains_points with radius 0: the crossing-number test below, the same
// comparison in the same arithmetic (no FMA contraction), so points on a cell
// boundary land in the same cells as in the reference (tests/golden/cells_*).
//
// k_cell_partial: grid (point tiles, cells); one thread per point per cell.
// k_cell_final:   one workgroup per cell sums the tile partials in tile order.
// A batch of partitions (the lockstep simulations of coverage.py: every seed's
// loss and Lloyd partitions, sim:895-904) is one launch: cell i reads the field
// w / var of its own seed, w + field[i] * M (field = null: every cell reads w).
//
// k_post_copy: the resident posterior of an unchanged model (a batch member that
// appended no rows) copied into the batch's outputs with its var max / first
// argmax -- the step's predict for a model whose state did not change.
#include <climits>
#include <cstdint>
#include <hip/hip_runtime.h>

#include "mfgp_internal.h"

namespace mfgp {

constexpr int CNT = 256;           // threads per workgroup (one point each)
constexpr int CMAXV = 256;         // polygon vertices held in LDS per cell
constexpr int CPART = 8;           // partial record: count, sw, swx, swy, sl, vmax, argmax, pad

// in_polygon of one point against the closed polygon (vx, vy)[0..nv): matplotlib's
// point_in_path crossing rule -- an edge whose end points straddle the point's y
// (yflag = vy >= ty) toggles the parity when
// ((vty1 - ty) * (vtx0 - vtx1) >= (vtx1 - tx) * (vty0 - vty1)) == yflag1.
__device__ __forceinline__ bool in_cell(const double* __restrict__ vx, const double* __restrict__ vy, int nv,
                                        double tx, double ty) {
#pragma clang fp contract(off)
  bool inside = false;
  double x0 = vx[0], y0 = vy[0];
  bool f0 = y0 >= ty;
  for (int e = 1; e <= nv; ++e) {
    const int k = e < nv ? e : 0;
    const double x1 = vx[k], y1 = vy[k];
    const bool f1 = y1 >= ty;
    if (f0 != f1) {
      const double lhs = (y1 - ty) * (x0 - x1);
      const double rhs = (x1 - tx) * (y0 - y1);
      if ((lhs >= rhs) == f1) inside = !inside;
    }
    f0 = f1;
    x0 = x1;
    y0 = y1;
  }
  return inside;
}

__device__ __forceinline__ void amax_pair(double& bv, int64_t& bi, double ov, int64_t oi) {
  if (ov > bv || (ov == bv && oi < bi)) {
    bv = ov;
    bi = oi;
  }
}

__global__ __launch_bounds__(CNT) void k_cell_partial(const double* __restrict__ grid, int64_t M,
                                                      const double* __restrict__ verts,
                                                      const int* __restrict__ vstart,
                                                      const double* __restrict__ seeds,
                                                      const double* __restrict__ w, const double* __restrict__ f,
                                                      const double* __restrict__ var,
                                                      const int* __restrict__ field, double* __restrict__ part,
                                                      int64_t ntiles) {
  const int cell = blockIdx.y;
  if (field) {   // this cell's seed's fields
    const int64_t fo = (int64_t)field[cell] * M;
    if (w) w += fo;
    if (var) var += fo;
  }
  const int64_t tile = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __shared__ double vx[CMAXV], vy[CMAXV];
  __shared__ double red[CNT / 64][CPART];
  const int v0 = vstart[cell];
  const int nv = min(vstart[cell + 1] - v0, CMAXV);
  for (int i = tid; i < nv; i += CNT) {
    vx[i] = verts[2 * (v0 + i)];
    vy[i] = verts[2 * (v0 + i) + 1];
  }
  __syncthreads();
  const double sx = seeds[2 * cell], sy = seeds[2 * cell + 1];
  const int64_t e = tile * CNT + tid;
  double cnt = 0.0, sw = 0.0, swx = 0.0, swy = 0.0, sl = 0.0;
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  if (e < M && nv >= 3) {
    const double x = grid[2 * e], y = grid[2 * e + 1];
    if (in_cell(vx, vy, nv, x, y)) {
#pragma clang fp contract(off)
      cnt = 1.0;
      if (w) {
        const double we = w[e];
        sw = we;
        swx = we * x;   // weighted_points = weights * in_points (sim:265)
        swy = we * y;
      }
      if (f) {
        const double dx = x - sx, dy = y - sy;
        sl = (dx * dx + dy * dy) * f[e];   // distances * f_val (sim:216-217)
      }
      if (var) {
        bv = var[e];
        bi = e;
      }
    }
  }
  // workgroup sums (fixed tree order) and (max, first argmax)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    cnt += __shfl_xor(cnt, off);
    sw += __shfl_xor(sw, off);
    swx += __shfl_xor(swx, off);
    swy += __shfl_xor(swy, off);
    sl += __shfl_xor(sl, off);
    amax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  }
  if (lane == 0) {
    red[wv][0] = cnt;
    red[wv][1] = sw;
    red[wv][2] = swx;
    red[wv][3] = swy;
    red[wv][4] = sl;
    red[wv][5] = bv;
    red[wv][6] = (double)bi;
  }
  __syncthreads();
  if (tid == 0) {
    double* p = part + ((int64_t)cell * ntiles + tile) * CPART;
    for (int j = 0; j < 5; ++j) p[j] = (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]);
    double mv = red[0][5];
    int64_t mi = (int64_t)red[0][6];
    for (int k = 1; k < CNT / 64; ++k) amax_pair(mv, mi, red[k][5], (int64_t)red[k][6]);
    p[5] = mv;
    p[6] = (double)mi;
  }
}

// out[cell] = {count, sum w, sum w*x, sum w*y, sum d^2 f, max var}, argmax[cell]
// (-1 if the cell holds no point); tile partials summed in tile order.
__global__ __launch_bounds__(64) void k_cell_final(const double* __restrict__ part, int64_t ntiles,
                                                  double* __restrict__ out, int64_t* __restrict__ argmax) {
  const int cell = blockIdx.x;
  const int lane = threadIdx.x;
  double acc[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  // lane-strided tiles, then a fixed tree: deterministic for a given tile count
  for (int64_t t = lane; t < ntiles; t += 64) {
    const double* p = part + ((int64_t)cell * ntiles + t) * CPART;
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[j] += p[j];
    amax_pair(bv, bi, p[5], (int64_t)p[6]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[j] += __shfl_xor(acc[j], off);
    amax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 5; ++j) out[cell * 6 + j] = acc[j];
    out[cell * 6 + 5] = bv;
    argmax[cell] = (bi == INT64_MAX) ? -1 : bi;
  }
}

hipError_t launch_cell_reduce(const double* grid, int64_t M, const double* verts, const int* vstart, int ncells,
                              const double* seeds, const double* w, const double* f, const double* var,
                              const int* field, double* part, double* out, int64_t* argmax, hipStream_t s) {
  const int64_t ntiles = (M + CNT - 1) / CNT;
  if (ntiles <= 0 || ncells <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_cell_partial, dim3((unsigned)ntiles, ncells), dim3(CNT), 0, s, grid, M, verts, vstart, seeds,
                     w, f, var, field, part, ntiles);
  hipLaunchKernelGGL(k_cell_final, dim3(ncells), dim3(64), 0, s, part, ntiles, out, argmax);
  return hipGetLastError();
}

int64_t cell_partial_doubles(int64_t M, int ncells) { return (int64_t)ncells * ((M + CNT - 1) / CNT) * CPART; }

// One workgroup per model: 16-byte loads and stores of mu / var (M even and the
// buffers 16-byte aligned, else one double at a time), the running (max, first
// argmax) of var per thread, then a wave reduction and one across the 16 waves.
constexpr int PCT = 1024;
__global__ __launch_bounds__(PCT) void k_post_copy(PostArg a) {
  const PostCopy& p = a.p[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t M = p.M;
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  const bool vec = (M % 2 == 0) && ((((uintptr_t)p.smu) | ((uintptr_t)p.svar) | ((uintptr_t)p.mu) |
                                     ((uintptr_t)p.var)) % 16 == 0);
  if (vec) {
    const double2* sm = reinterpret_cast<const double2*>(p.smu);
    const double2* sv = reinterpret_cast<const double2*>(p.svar);
    double2* dm = reinterpret_cast<double2*>(p.mu);
    double2* dv = reinterpret_cast<double2*>(p.var);
    for (int64_t i = tid; i < M / 2; i += PCT) {
      const double2 m2 = sm[i], v2 = sv[i];
      dm[i] = m2;
      dv[i] = v2;
      amax_pair(bv, bi, v2.x, 2 * i);
      amax_pair(bv, bi, v2.y, 2 * i + 1);
    }
  } else {
    for (int64_t i = tid; i < M; i += PCT) {
      const double v = p.svar[i];
      p.mu[i] = p.smu[i];
      p.var[i] = v;
      amax_pair(bv, bi, v, i);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) amax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
  __shared__ double rv[PCT / 64];
  __shared__ int64_t ri[PCT / 64];
  if (lane == 0) {
    rv[wv] = bv;
    ri[wv] = bi;
  }
  __syncthreads();
  if (tid == 0) {
    for (int k = 1; k < PCT / 64; ++k) amax_pair(bv, bi, rv[k], ri[k]);
    if (p.vmax) p.vmax[0] = bv;
    if (p.vargmax) p.vargmax[0] = bi;
  }
}

hipError_t launch_post_copy(const PostCopy* h, int count, hipStream_t s) {
  for (int i0 = 0; i0 < count; i0 += POST_MAX) {
    PostArg a{};
    const int n = count - i0 < POST_MAX ? count - i0 : POST_MAX;
    for (int i = 0; i < n; ++i) a.p[i] = h[i0 + i];
    hipLaunchKernelGGL(k_post_copy, dim3(n), dim3(PCT), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace mfgp
