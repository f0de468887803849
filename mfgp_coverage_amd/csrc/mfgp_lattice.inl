// Lattice-separable incremental step (k_inc_lat). Included by mfgp_kernels.hip
// after the bordered-append section (it reuses inc_produce / inc_finish, the
// hand-off primitives and var_argmax_group).
//
// The one-pass predict (k_inc_stream) reads the resident V = L^-1 psi^T once per
// update: 8 n0 M bytes, HBM-bound. On a lattice grid the same update needs no V
// pass. With w = L11^-T L21^T = K11^-1 K12 (n0 x k),
//   L21 V_old(c) = L21 L11^-1 psi_old(c)^T = w^T psi_old(c)^T
// and the SE kernel factorises over the two axes of a lattice cell c = (ix, iy):
//   psi(c, j) = c_j exp(-(x_ix - x_j)^2 / 2l^2) exp(-(y_iy - y_j)^2 / 2l^2)
// (MF: two such terms for a hifi row, rho^2 s_L k_L + s_H k_H; gp:426-429). So
//   T~[a, ix, iy] = sum_j (w_aj c_j Ex[j][ix]) Ey[j][iy]
// is a GEMM of (a, ix) rows by iy columns over the n0 (+ n_H) terms: 2 k M n_t
// flop on f64 MFMA instead of a V stream, and then per cell
//   T = psi_new - T~,  v_new = L22^-1 T,  var = var_old - |v_new|^2,
//   mu = mu_old + v_new^T z2                                  (bordered update)
// with var_old / mu_old the model's resident posterior of the n0 leading rows.
// w comes from the explicit inverse F = L^-1 (resident, lower triangular, stored
// row-major):
// w = F11^T L21^T, one parallel pass over F's lower triangle (HBM-bound, 8 n0^2/2
// bytes); F's new rows are -L22^-1 w^T and L22^-1, so F grows with the factor.
// The new rows of V (v_new) are still stored, so the V-stream path stays valid.
//
// Numerics: T = psi_new - w^T psi_old is formed from w, whose size grows with the
// conditioning of K; the host takes this path only when kss / (noise + jitter)
// <= LAT_RMAX (errors <= 1e-7 in the parity metric up to
// 1e4, 7e-5 at the reference's anti_two_corners ratio 6e6, which stays on the
// V stream), and refreshes var / mu from V after LAT_MAXD consecutive steps.
//
// One launch per batch, grid (GPs, roles); per GP the roles are
//   [0, nprod)                 producers + finish, exactly as k_inc_stream's
//   [nprod, nprod + nwu)       w units (64 rows of w x LAT_WCH rows of F, top
//                              block first): wait for the compact rows of their
//                              rows, then w[j][a] = sum_{i >= j} F[i][j] L21c[i][a]
//                              on MFMA; the block's last unit adds the chunks,
//                              write-through + drain + wflag[jb] = epoch; then a
//                              share of the new rows' separable tables
//   [.., + tiles * ksplit)     GEMM tiles: 64 (a, ix) rows x 64 iy columns, the
//                              term blocks in descending order (the order w
//                              becomes ready), split ksplit ways over the terms;
//                              the last split to arrive reduces the partials and
//                              runs the cell epilogue, F's new rows and the fused
//                              var max / argmax
// Every role waits only for roles with a lower linear id (x = GP fastest), so
// the dispatch-order argument of k_inc_stream holds; waits are bounded.
// ---------------------------------------------------------------------------
constexpr int LKS = 16;                   // term rows (j) per pipeline stage
#ifndef MFGP_LAT_NST
#define MFGP_LAT_NST 3
#endif
constexpr int LNST = MFGP_LAT_NST;        // stages in the LDS ring
constexpr int LBS = LKS * 64;             // Bs: Ey rows [LKS][64 iy], swizzled (swz)
constexpr int LWS = LKS * KINC;           // Ws: w rows [LKS][16 a]
constexpr int LXS = LKS * 16;             // Xs: Ex rows [LKS][16 ix of the tile]
constexpr int LSTG = LBS + LWS + LXS;      // doubles per stage
constexpr int LAT_EPI = 272 + 256 + 32 + 2 * 16 * (8 + 64);   // epilogue: L22, z2 | L22^-1 | new rows | their factors (later: a w block)
static_assert(2 * 16 * (8 + 64) >= 64 * KINC, "a w block fits the factors' place");
constexpr int LAT_RING = LNST * LSTG + LNST * 32;       // the ring | its flag words
constexpr int LAT_LDS = LAT_RING > LAT_EPI ? LAT_RING : LAT_EPI;   // 37.6 KB: four workgroups per CU
static_assert(LAT_LDS >= FIN_LDS, "the ring also holds the finish's LDS image");

static_assert(LNST > 3 || LAT_LDS + 16 <= 5120, "four workgroups per CU (40 KB of LDS each)");
constexpr int LAT_PART = 4 * 32 * 64;     // doubles of one split-K partial tile (4 waves x 32 acc x 64 lanes)

// The term blocks of split sp of S: every S-th block from the top (jb = nwb - 1
// - sp - m S, m = 0, 1, ..), so every split starts at the blocks whose w is ready
// first and all of them move down together as w becomes ready. Blocks jb >= jh
// have L and H parts (8 stages of 16 rows), blocks below jh the L part only (4).
__device__ __forceinline__ int64_t lat_nblk(int64_t from, int64_t S) { return from >= 0 ? from / S + 1 : 0; }
__device__ __forceinline__ void lat_stage(int64_t t, int64_t nwb, int64_t jh, int64_t sp, int64_t S, int64_t& jb,
                                          int& part, int64_t& j0) {
  const int64_t top = nwb - 1 - sp;
  const int64_t nh = top >= jh ? (top - jh) / S + 1 : 0;   // this split's blocks with H parts
  int64_t m;
  if (t < 8 * nh) {
    m = t / 8;
    part = (int)((t % 8) / 4);
  } else {
    t -= 8 * nh;
    m = nh + t / 4;
    part = 0;
  }
  jb = top - m * S;
  j0 = 64 * jb + 16 * (t % 4);
}
__device__ __forceinline__ int64_t lat_nstages(int64_t nwb, int64_t jh, int64_t sp, int64_t S) {
  const int64_t top = nwb - 1 - sp;
  const int64_t nb = lat_nblk(top, S);
  const int64_t nh = top >= jh ? (top - jh) / S + 1 : 0;
  return 8 * nh + 4 * (nb - nh);
}
__device__ __forceinline__ int64_t lat_jh(const GPDesc& d) {
  const int64_t nwb = d.nwb;
  if (d.hp.kind == 0) return nwb;
  return d.NL / 64 < nwb ? d.NL / 64 : nwb;
}

// Separable table entry (t: 0 = c_L ex_L, 1 = ey_L, 2 = c_H ex_H, 3 = ey_H) of
// training row `row` at (px, py) for lattice axis index `col`: the factor of
// psi(cell, row) along one axis, each in the SE kernel's operation order
// (x / l - x' / l, squared, exp(-0.5 *)); zero past the axis and for the H
// tables of lofi rows / SF models.
__device__ double lat_tab_value(const GPDesc& d, int t, int64_t row, int64_t col, double px, double py) {
#pragma clang fp contract(off)
  const Hyp& h = d.hp;
  const GridLattice& L = d.lat;
  const bool isx = (t & 1) == 0;
  if (col >= (isx ? L.nx : L.ny)) return 0.0;
  const bool hterm = t >= 2;
  if (hterm && (h.kind == 0 || row < d.NL)) return 0.0;
  const double l = hterm ? h.lH : h.lL;
  const double ax = isx ? d.grid[2 * (col * L.sx)] : d.grid[2 * (col * L.sy) + 1];
  const double dx = div_(ax, l) - div_(isx ? px : py, l);
  const double e = exp(-0.5 * (dx * dx));
  if (!isx) return e;
  const double c = hterm ? h.sH : (h.kind == 0 ? h.sL : (row < d.NL ? h.rho * h.sL : h.rho2 * h.sL));
  return c * e;
}

// Rows [lo, n0) of the compact rows are stored: every producer chunk from lo / FCH
// on holds this launch's epoch, or sync[1] does. Wave 0 polls; bounded.
__device__ void wait_l21_from(const GPDesc& d, int64_t lo) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int it = 0;
    while (true) {
      bool mine = true;
      for (int64_t c = lo / FCH + lane; c < d.nprod; c += 64)
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

// Spin (this wave) until *f == v; bounded like wait_flag.
__device__ __forceinline__ void spin_wave(const GPDesc& d, const unsigned* f, unsigned v) {
  int it = 0;
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != v) {
    __builtin_amdgcn_s_sleep(MFGP_SPIN_SLEEP);
    if (++it == (1 << 22)) {
      if ((threadIdx.x & 63) == 0) atomicMin(d.status, SYNC_FAIL);
      break;
    }
  }
}

template <class VT>
__device__ __forceinline__ double l21c_at(const double* l21c, int64_t i, int a) {
  if constexpr (sizeof(VT) == 8) return gp(l21c)[i * KINC + a];
  else return (double)gp(reinterpret_cast<const float*>(l21c))[i * KINC + a];
}

// w unit u (in role order: column blocks from the top, chunks of LAT_WCH rows
// within a block): its block jb, chunk c, the block's first unit u0 and units nc.
__device__ __forceinline__ void lat_wunit(int64_t n0, int64_t nwb, int64_t u, int64_t& jb, int64_t& c,
                                          int64_t& u0, int64_t& nc) {
  u0 = 0;
  for (jb = nwb - 1; jb > 0; --jb) {
    nc = lat_wunits_block(n0, jb);
    if (u < u0 + nc) break;
    u0 += nc;
  }
  nc = lat_wunits_block(n0, jb);
  c = u - u0;
}

// L22^-1 (rows / columns >= k zero) into Li [16][16] from the L22 record (sync[2]
// must have been seen; plain loads: no line of the record is read in this launch
// before that flag). L22 is scratch [16][16 | 16].
__device__ __forceinline__ void lat_l22inv(const GPDesc& d, int k, double* L22, double* Li) {
  const int tid = threadIdx.x;
  for (int e = tid; e < KINC * KINC; e += NT) {
    const double v = d.l22r[e];
    L22[e] = (e / KINC < k && e % KINC <= e / KINC) ? v : 0.0;
  }
  __syncthreads();
  if (tid < KINC) {
    // column c of L22^-1 by forward substitution
    const int c = tid;
    double x[KINC];
#pragma unroll
    for (int i = 0; i < KINC; ++i) {
      double t = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int b = 0; b < i; ++b) t -= L22[i * KINC + b] * x[b];
      x[i] = (i < k && i >= c) ? t / L22[i * KINC + i] : 0.0;
      Li[i * KINC + c] = x[i];
    }
  }
  __syncthreads();
}

// One w unit: columns j = 64 jb + [0, 64) of w = F11^T L21^T, rows i of chunk c
// of [64 jb, n0) -- F's lower triangle below the block. Each wave takes 32 of
// every 128 rows and all 64 columns: lane (r, q) loads F[i][64 jb + 16 cb + r]
// (four 128-byte lines per load, F row-major) for cb = 0..3 and the compact row
// entry L21c[i][r] once for all four (MFMA A = L21c, B = F), so 80 VGPRs hold
// 16 KB of F per wave in flight. The waves' sums meet in LDS in wave order. A
// block of one chunk stores w itself; otherwise each chunk stores its partial
// and the last of the block to arrive adds them in chunk order. Either way the
// block's flag is raised once w is stored; then the same workgroup writes F's
// new rows for the block, -L22^-1 w^T (and the top block's unit L22^-1).
template <class VT>
__device__ __forceinline__ void lat_wblock(const GPDesc& d, int64_t u, double* sm) {
  const int64_t n0 = d.n0, ld = d.ld;
  int64_t jb, c, u0, nc;
  lat_wunit(n0, d.nwb, u, jb, c, u0, nc);
  const int64_t i_lo = 64 * jb + LAT_WCH * c;
  const int64_t i_hi = i_lo + LAT_WCH < n0 ? i_lo + LAT_WCH : n0;
  const double* const l21c = d.l21c;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  WTRACE(0);
  // a share of the new rows' separable tables (read from the next launch on)
  const int k = (int)(d.N - n0);
  const int64_t tabw = d.tabw, tstride = (d.ld) * tabw;
  const int64_t tot = 4 * (int64_t)k * tabw;
  const int64_t per = (tot + d.nwu - 1) / d.nwu, e0 = u * per;
  const int64_t e1 = e0 + per < tot ? e0 + per : tot;
  for (int64_t e = e0 + tid; e < e1; e += NT) {
    const int t = (int)(e / (k * tabw));
    const int64_t rem = e % (k * tabw);
    const int a = (int)(rem / tabw);
    const int64_t col = rem % tabw;
    const double* p = row_pt(d, n0 + a);
    // written through: the GEMM tiles' epilogues read them in this launch (after
    // the w flags, which follow the drain below)
    stx<true>(&d.tab[t * tstride + (n0 + a) * tabw + col], lat_tab_value(d, t, n0 + a, col, p[0], p[1]));
  }
  wait_l21_from(d, i_lo);
  WTRACE(1);
  const GLOBAL double* Fr = gp(d.F) + 64 * jb + r;   // F[i][64 jb + 16 cb + r] at Fr[i * ld + 16 cb]
  d4 acc[4];
#pragma unroll
  for (int x = 0; x < 4; ++x) acc[x] = d4{0.0, 0.0, 0.0, 0.0};
#ifndef MFGP_DIAG_LATNOW
  constexpr int RG = 8;   // 4-row groups per wave per batch (128 rows per batch)
  for (int64_t i0 = i_lo + 32 * w; i0 < i_hi; i0 += 128) {
    double f[RG][4], a[RG];
#pragma unroll
    for (int x = 0; x < RG; ++x) {
      const int64_t i = i0 + 4 * x + q;
      const int64_t ii = i < i_hi ? i : i_lo;
      // F is read once per step and would evict the GEMM tiles' tables from L2
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) f[x][cb] = __builtin_nontemporal_load(Fr + ii * ld + 16 * cb);
      a[x] = l21c_at<VT>(l21c, ii, r);
    }
#pragma unroll
    for (int x = 0; x < RG; ++x) {
      const int64_t i = i0 + 4 * x + q;
      const double av = i < i_hi ? a[x] : 0.0;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[cb] = mfma(av, f[x][cb], acc[cb]);
    }
  }
#endif
  WTRACE(3);
  // the waves' sums in wave order: lane (r, g) register v of acc[cb] is w row
  // a = g + 4 v, column jl = 16 cb + r; Wb [64 jl][16 a] after the sum
  double* const red = sm;             // [4 w][4 cb][4 v][64 lanes]
  double* const Wb = sm;              // [64][16], once the sums are read
  double* const L22 = Wb + 64 * KINC;  // [16][16]
  double* const Li = L22 + KINC * KINC;
  static_assert(4096 <= LAT_LDS, "the w unit's LDS fits");
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int v = 0; v < 4; ++v) red[((w * 4 + cb) * 4 + v) * 64 + lane] = acc[cb][v];
  __syncthreads();
  double* const wv = d.wv;
  // thread tid sums outputs e = tid + 256 m: (jl, a) = (e >> 4, e & 15)
  double own[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int e = tid + NT * m, jl = e >> 4, a = e & 15;
    const int cb = jl >> 4, rr = jl & 15, v = a >> 2, g = a & 3;
    const int o = (cb * 4 + v) * 64 + 16 * g + rr;
    own[m] = (red[o] + red[1024 + o]) + (red[2048 + o] + red[3072 + o]);
  }
  __syncthreads();
  if (nc == 1) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int e = tid + NT * m;
      stx<true>(&wv[64 * jb * KINC + e], own[m]);
      Wb[e] = own[m];
    }
  } else {
    double* part = d.wpart + (u0 + c) * 1024;
#pragma unroll
    for (int m = 0; m < 4; ++m) stx<true>(part + tid + NT * m, own[m]);
    drain_stores();
    __syncthreads();
    unsigned& wlast = *reinterpret_cast<unsigned*>(sm + LAT_LDS + 10);
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(d.wcnt + jb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      wlast = old == (unsigned)(nc - 1) ? 1u : 0u;
      if (wlast) __hip_atomic_store(d.wcnt + jb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!wlast) return;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int e = tid + NT * m;
      double t = 0.0;
      for (int64_t cc = 0; cc < nc; ++cc) t += ldx<true>(d.wpart + (u0 + cc) * 1024 + e);
      stx<true>(&wv[64 * jb * KINC + e], t);
      Wb[e] = t;
    }
  }
  drain_stores();
  __syncthreads();
  if (tid == 0) publish(d.wflag + jb, d.epoch);
  WTRACE(2);
  // F's new rows for this block: F[n0 + a][j] = -sum_{b <= a} L22^-1[a][b] w[j][b]
  wait_flag(d, d.sync + 2, d.epoch);
  lat_l22inv(d, k, L22, Li);
  for (int e = tid; e < 64 * k; e += NT) {
    const int a = e >> 6, jl = e & 63;
    const int64_t j = 64 * jb + jl;
    if (j >= n0) continue;
    double t = 0.0;
    for (int b = 0; b <= a; ++b) t -= Li[a * KINC + b] * Wb[jl * KINC + b];
    d.F[(n0 + a) * ld + j] = t;   // F row-major
  }
  if (jb == d.nwb - 1)
    for (int e = tid; e < k * k; e += NT) {
      const int a = e / k, b = e % k;
      if (b <= a) d.F[(n0 + a) * ld + n0 + b] = Li[a * KINC + b];
    }
}

// Geometry of one GEMM tile, and its buffer-descriptor LDS-DMA plan (as
// k_predict's: the lane part of each source offset is a VGPR fixed for the
// kernel, the row part an SGPR).
struct LatGeo {
  __amdgpu_buffer_rsrc_t rtab, rw;   // the four tables; w
  int64_t tstride, tabw;
  int64_t nwb, jh, sp, S;
  int64_t ix0, iy0;
  unsigned vB, vW, vX;               // lane byte offsets: Bs, Ws, Xs
};

// Issue the DMAs of stage st into `slot` (waves 1..3; wave 0 only loads the w
// flags, so its vmcnt never waits for a flag's memory round trip behind a table
// load, nor theirs for a flag): Bs = 16 Ey rows x 64 iy (8 two-row DMAs, waves
// 1 and 2, swizzled as swz), Ws = 16 w rows and Xs = 16 Ex rows x 16 ix (wave 3,
// two 8-row DMAs each).
__device__ __forceinline__ void lat_issue(const LatGeo& G, int64_t st, double* slot, int w) {
  int64_t jb, j0;
  int part;
  lat_stage(st, G.nwb, G.jh, G.sp, G.S, jb, part, j0);
  const int64_t tx = (2 * part) * G.tstride, ty = tx + G.tstride;
  if (w < 3) {
    const int p0 = 4 * (w - 1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = p0 + u;
      dma_buf(G.rtab, slot + 2 * p * 64, G.vB, (unsigned)(8 * (ty + (j0 + 2 * p) * G.tabw + G.iy0)));
    }
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      dma_buf(G.rw, slot + LBS + 8 * h * KINC, G.vW, (unsigned)(8 * (j0 + 8 * h) * KINC));
      dma_buf(G.rtab, slot + LBS + LWS + 8 * h * 16, G.vX, (unsigned)(8 * (tx + (j0 + 8 * h) * G.tabw + G.ix0)));
    }
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 4], then the raw barrier (no
// fence: the stage's data is the DMA's, complete once vmcnt says so)
__device__ __forceinline__ void vm_wait_bar(int n) {
  switch (n) {
#define VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")\n\ts_barrier" ::: "memory"); break;
    VMW(0) VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12)
#undef VMW
    default: asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory"); break;
  }
}

// acc += A B over one stage: A[(a, ix)][j] = w[j][a] * Ex[j][ix] (formed from the
// Ws / Xs rows), B[j][iy] = Ey[j][iy]. Wave w: rows 32 w + 16 m + r (m = 0, 1), all
// 64 columns (blocks n = 0..3): per 4-row k-step 7 LDS reads, 2 products and 8
// MFMAs. The reads of two k-steps are issued ahead of their MFMAs.
template <int KA>
__device__ __forceinline__ void lat_compute(const double* slot, d4 (&acc)[2][4], int r, int q, int ar, int ixl0,
                                            int ixl1) {
  const double* Bs = slot;
  const double* Ws = slot + LBS;
  const double* Xs = slot + LBS + LWS;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    double wa[2], x0[2], x1[2], b[2][4];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 4 * (2 * hh + e) + q;
      wa[e] = Ws[j * KINC + ar];
      x0[e] = Xs[j * 16 + ixl0];
      x1[e] = Xs[j * 16 + ixl1];
#pragma unroll
      for (int n = 0; n < 4; ++n) b[e][n] = Bs[swz(j, 16 * n + r)];
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const double a0 = wa[e] * x0[e];
      const double a1 = wa[e] * x1[e];
#ifdef MFGP_DIAG_LATNOMMA   // diagnostic build: the loop without its MFMAs (timing only)
      acc[0][0][0] += a0 + b[e][0];
      acc[1][1][0] += a1 + b[e][1];
      continue;
#endif
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        acc[0][n] = mfma(a0, b[e][n], acc[0][n]);
        acc[1][n] = mfma(a1, b[e][n], acc[1][n]);
      }
    }
  }
}

// One GEMM tile (split s of ksplit): 128 (a, ix) rows x 64 iy columns, i.e.
// (128 / KA) x 64 cells; and, for the last split to arrive, the cell epilogue,
// F's new rows for its column blocks and the fused var max / argmax partials.
template <int KA, class VT>
__device__ __forceinline__ void lat_gemm(const GPDesc& d, int64_t tile, int64_t s, double* sm) {
  constexpr int IXPT = 128 / KA;   // lattice columns x per tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const GridLattice lat = d.lat;
  const int64_t ntiy = (lat.ny + 63) / 64;
  const int64_t tix = tile / ntiy, tiy = tile % ntiy;
  const int S = d.ksplit;
  LatGeo G;
  G.tabw = d.tabw;
  G.tstride = d.ld * d.tabw;
  G.rtab = make_rsrc(d.tab, (int64_t)8 * 4 * G.tstride);
  G.rw = make_rsrc(d.wv, (int64_t)8 * d.ld * KINC);
  G.vB = (unsigned)(8 * ((lane >> 5) * G.tabw + (((lane & 31) * 2) ^ ((lane >> 5) << 4))));
  G.vW = (unsigned)(8 * ((lane >> 3) * KINC + 2 * (lane & 7)));
  G.vX = (unsigned)(8 * ((lane >> 3) * G.tabw + 2 * (lane & 7)));
  G.nwb = d.nwb;
  G.jh = lat_jh(d);
  G.ix0 = tix * IXPT;
  G.iy0 = tiy * 64;
  G.sp = s;
  G.S = S;
  const int64_t lo = 0, hi = lat_nstages(G.nwb, G.jh, s, S);
  WTRACE(0);
  // this lane's A rows: a = row % KA, lattice column ixl = row / KA (rows 32 w + 16 m + r)
  const int ar = KA == 8 ? (r & 7) : r;
  const int ixl0 = KA == 8 ? 4 * w + (r >> 3) : 2 * w;
  const int ixl1 = KA == 8 ? 4 * w + 2 + (r >> 3) : 2 * w + 1;
  d4 acc[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = d4{0.0, 0.0, 0.0, 0.0};
  // w's readiness: wave 0 loads the flag word of each stage's block into LDS (an
  // agent-scope 4-byte LDS-DMA) two iterations before that stage's DMAs are
  // issued; waves 2 and 3, which stage the w rows, check it there after the
  // barrier (an LDS read, not a memory round trip) and spin on memory only if it
  // was not yet set. Wave 0 issues nothing else, so the flags' round trips never
  // sit in front of a table load in any wave's vmcnt order.
  // (descriptor fields the loop and the epilogue use, in registers: the raw
  // barriers' memory clobbers and the global stores would make the compiler reload
  // them from the descriptor, a scalar-memory round trip each time)
  const unsigned epoch = d.epoch;
  const unsigned* const wflag = d.wflag;
  const int cnt = w == 0 ? 1 : 4;   // vector-memory ops per issued stage
  unsigned* const fl = reinterpret_cast<unsigned*>(sm + LNST * LSTG);   // [LNST][64]
  const __amdgpu_buffer_rsrc_t rfl = make_rsrc(reinterpret_cast<const double*>(d.wflag),
                                               (int64_t)4 * (d.nwb + 1));
  auto blk = [&](int64_t st) {
    int64_t jb, j0;
    int part;
    lat_stage(st < hi ? st : hi - 1, G.nwb, G.jh, G.sp, G.S, jb, part, j0);
    return jb;
  };
  auto issue = [&](int64_t st, int64_t fst) {   // stage st's DMAs (waves 1..3), flag of stage fst (wave 0)
    if (w == 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rfl, (lds_vptr)(fl + ((fst - lo) % LNST) * 64), 4, 0u,
                                               (unsigned)(4 * blk(fst)), 0, 16 /* sc1: agent scope */);
#ifndef MFGP_DIAG_LATNODMA   // diagnostic build: no table / w DMAs (timing only)
    else
      lat_issue(G, st, sm + ((st - lo) % LNST) * LSTG, w);
#endif
  };
  constexpr int D = LNST - 1;   // stages in flight ahead of the one consumed
  static_assert(D * 4 <= 12, "vm_wait_bar covers the outstanding ops");
#ifdef MFGP_DIAG_LATNOWAIT   // diagnostic build: the GEMM does not wait for w (timing only)
  auto spin_wave = [](const GPDesc&, const unsigned*, unsigned) {};
#endif
  if (lo < hi) {
    if (w == 3)
      for (int64_t st = lo; st < lo + D && st < hi; ++st) spin_wave(d, wflag + blk(st), epoch);
    WTRACE(1);
    for (int64_t st = lo; st < lo + D && st < hi; ++st) issue(st, st + D);
    // iteration t: stage t sits in slot (t - lo) % LNST, issued D iterations ago
    // with the flag of stage t + D, and followed by the ops of the stages after it
    for (int64_t t = lo; t < hi; ++t) {
      const int64_t after = (hi - 1 - t) < (D - 1) ? (hi - 1 - t) : (D - 1);
      vm_wait_bar((int)after * cnt);
      if (t + D < hi) {
        if (w == 3 && fl[((t + D - lo) % LNST) * 64] != epoch) spin_wave(d, wflag + blk(t + D), epoch);
        issue(t + D, t + 2 * D);
      }
#ifndef MFGP_DIAG_LATNOCOMP   // diagnostic build: the pipeline without its compute (timing only)
      lat_compute<KA>(sm + ((t - lo) % LNST) * LSTG, acc, r, q, ar, ixl0, ixl1);
#endif
    }
  }
  vm_wait_all();
  __syncthreads();
  WTRACE(2);
  // the L22 record's flag (sync[2], raised by the finish long before any K loop
  // ends): read with the partial stores, so the reducer rarely waits for it
  unsigned& l22_seen = *reinterpret_cast<unsigned*>(sm + LAT_LDS + 11);
  if (tid == 0)
    l22_seen = __hip_atomic_load(d.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch ? 1u : 0u;
  // split-K: partials through memory, the last split reduces them in split order
  if (S > 1) {
    unsigned& lat_last = *reinterpret_cast<unsigned*>(sm + LAT_LDS + 9);
    double* part = d.gpart + (tile * S + s) * LAT_PART + (int64_t)w * 32 * 64 + lane;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int v = 0; v < 4; ++v) stx<true>(part + ((m * 4 + n) * 4 + v) * 64, acc[m][n][v]);
    drain_stores();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(d.gcnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lat_last = old == (unsigned)(S - 1) ? 1u : 0u;
      if (lat_last) __hip_atomic_store(d.gcnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!lat_last) return;
    // every split's partial (this one's too) from memory, added in split order
    // (p0 + p1) + p2 ...: the same bits whichever split arrives last
    const double* p0 = d.gpart + tile * S * LAT_PART + (int64_t)w * 32 * 64 + lane;
    for (int s2 = 0; s2 < S; ++s2) {
      double x[32];
#pragma unroll
      for (int e = 0; e < 32; ++e) x[e] = ldx<true>(p0 + s2 * LAT_PART + e * 64);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const double xv = x[(m * 4 + n) * 4 + v];
            acc[m][n][v] = s2 == 0 ? xv : acc[m][n][v] + xv;
          }
    }
  }
  if (!l22_seen) wait_flag(d, d.sync + 2, epoch);
  WTRACE(3);
  // ---- epilogue (LDS: the ring is dead) ----
  const int64_t n0 = d.n0;
  const int k = (int)(d.N - n0);
  constexpr int FW = IXPT + 64;
  constexpr int NBP = KA == 8 ? 2 : 1;      // 16-column blocks per cell pass
  constexpr int TW = 16 * NBP;              // Ts row width
  double* const L22 = sm;                   // [16][16] | z2 [16]
  double* const Li = L22 + KINC * KINC + KINC;   // L22^-1 [16][16]
  // psi(cell, new row a) = c_L exL[a][ix] eyL[a][iy] + c_H exH[a][ix] eyH[a][iy]:
  // the new rows' separable tables (written through by the w units before their
  // flags) for the tile's IXPT x 64 cells, [2 kinds][KA][IXPT | 64]
  double* const Fn = Li + KINC * KINC;
  double* const Ts = Fn + 2 * KA * FW;      // one cell pass of T: [4 waves][16 rows][TW]
  static_assert(KINC * KINC + KINC + KINC * KINC + 2 * 8 * (16 + 64) + 4 * 16 * 32 <= LAT_LDS &&
                    KINC * KINC + KINC + KINC * KINC + 2 * 16 * (8 + 64) + 4 * 16 * 16 <= LAT_LDS,
                "the epilogue's LDS fits the ring's");
  __syncthreads();   // the ring's last reads are done
  {
    // plain loads: no line of the record or of the new rows' tables is read in
    // this launch before sync[2] / the w flags
    for (int e = tid; e < KINC * KINC + KINC; e += NT) {
      const double v = d.l22r[e];
      const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
      L22[e] = use ? v : 0.0;
    }
    const int64_t tstride = d.ld * d.tabw, tabw = d.tabw;
    for (int e = tid; e < 2 * KA * FW; e += NT) {
      const int kind2 = e / (KA * FW), rem = e % (KA * FW);
      const int a = rem / FW, col = rem % FW;
      const bool isx = col < IXPT;
      const int t = 2 * kind2 + (isx ? 0 : 1);
      const int64_t idx = isx ? G.ix0 + col : G.iy0 + (col - IXPT);
      Fn[e] = a < k ? d.tab[t * tstride + (n0 + a) * tabw + idx] : 0.0;
    }
  }
  __syncthreads();
  if (tid < KINC) {
    // column c of L22^-1 by forward substitution
    const int c = tid;
    double x[KINC];
#pragma unroll
    for (int i = 0; i < KINC; ++i) {
      double t = (i == c) ? 1.0 : 0.0;
#pragma unroll
      for (int b = 0; b < i; ++b) t -= L22[i * KINC + b] * x[b];
      x[i] = (i < k && i >= c) ? t / L22[i * KINC + i] : 0.0;
      Li[i * KINC + c] = x[i];
    }
  }
  WTRACE(5);
  // ---- cells: one pass per (m, group of NBP column blocks); the waves put
  // their blocks' T into Ts (row rho = g + 4 v of block (m, n) is, for KA = 8,
  // lattice column h = rho / 8 of the wave's pair and new row a = rho % 8; for
  // KA = 16 new row a = rho), then thread tid finishes one cell: source wave
  // cw = tid / 64, (h, column) from the rest. ----
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  VT* const Vr = const_cast<VT*>(vres_ptr<VT>(d));
  const int64_t vld = d.vld;
  double* const omu = d.mu;
  double* const ovar = d.var;
  double* const rmu = d.rmu;
  double* const rvar = d.rvar;
  const double* const rmu_in = d.rmu_in;
  const double* const rvar_in = d.rvar_in;
  const int cw = tid >> 6, cl = tid & 63;
  const int ch = KA == 8 ? cl >> 5 : 0;
  const int cyl = KA == 8 ? cl & 31 : cl & 15;
  const bool cact = KA == 8 || cl < 16;
  constexpr int NPASS = 2 * (4 / NBP);
  auto cell_of = [&](int p, int64_t& ix, int64_t& iy) {
    const int m = p / (4 / NBP), nf = NBP * (p % (4 / NBP));
    ix = G.ix0 + (KA == 8 ? 4 * cw + 2 * m + ch : 2 * cw + m);
    iy = G.iy0 + 16 * nf + cyl;
  };
  auto cell_ok = [&](int64_t ix, int64_t iy) { return cact && ix < lat.nx && iy < lat.ny; };
  // the old posterior of this thread's cell of the next pass, one pass ahead
  double ov = 0.0, om = 0.0;
  {
    int64_t ix, iy;
    cell_of(0, ix, iy);
    if (cell_ok(ix, iy)) {
      const int64_t c = ix * lat.sx + iy * lat.sy;
      ov = rvar_in[c];
      om = rmu_in[c];
    }
  }
#pragma unroll
  for (int p = 0; p < NPASS; ++p) {
    const int m = p / (4 / NBP), nf = NBP * (p % (4 / NBP));
    __syncthreads();   // the previous pass's Ts reads (and Li) are done
#pragma unroll
    for (int nb = 0; nb < NBP; ++nb)
#pragma unroll
      for (int v = 0; v < 4; ++v) Ts[(w * 16 + q + 4 * v) * TW + 16 * nb + r] = acc[m][nf + nb][v];
    __syncthreads();
    int64_t ix, iy;
    cell_of(p, ix, iy);
    const double cov = ov, com = om;
    if (p + 1 < NPASS) {
      int64_t ix2, iy2;
      cell_of(p + 1, ix2, iy2);
      if (cell_ok(ix2, iy2)) {
        const int64_t c2 = ix2 * lat.sx + iy2 * lat.sy;
        ov = rvar_in[c2];
        om = rmu_in[c2];
      }
    }
    if (!cell_ok(ix, iy)) continue;
    const int64_t c = ix * lat.sx + iy * lat.sy;
    const int ixc = (int)(ix - G.ix0), iyc = IXPT + (int)(iy - G.iy0);
    const double* const Tc = Ts + (cw * 16 + (KA == 8 ? 8 * ch : 0)) * TW + cyl;
    VT* const vt = Vr + (c / PBM) * vld * PBM + (c % PBM);
    double vn[KA];
    double vs = 0.0, ms = 0.0;
#pragma unroll
    for (int a = 0; a < KA; ++a) {
      vn[a] = 0.0;
      if (a < k) {
        const double* fL = Fn + a * FW;
        const double* fH = Fn + (KA + a) * FW;
        const double pn = fL[ixc] * fL[iyc] + fH[ixc] * fH[iyc];
        double t = pn - Tc[a * TW];
#pragma unroll
        for (int b = 0; b < a; ++b) t -= L22[a * KINC + b] * vn[b];
        vn[a] = t * Li[a * KINC + a];   // 1 / L22[a][a]
        vs += vn[a] * vn[a];
        ms += vn[a] * L22[KINC * KINC + a];
        vt[(n0 + a) * PBM] = (VT)vn[a];
      }
    }
    const double vc = cov - vs;
    const double mc = com + ms;
    omu[c] = mc;
    ovar[c] = vc;
    if (rmu) {
      rmu[c] = mc;
      rvar[c] = vc;
    }
    argmax_pair(bv, bi, vc, c);
  }
  const int64_t tiles = d.lat_tiles;
  WTRACE(6);
  if (d.vmax || d.vargmax || d.status_host)
    var_argmax_group(d, bv, bi, tile * 4 + w, tiles * 4);
  WTRACE(4);
}

template <int KA, class VT>
__device__ __forceinline__ void inc_lat_wg(const GPDesc& d) {
  const int k = (int)(d.N - d.n0);
  if (k <= 0 || k > KINC) return;   // the host guarantees 0 < k <= KINC
  if (d.gate && *d.gate == 0) return;
  // ONE LDS object for every role: a second __shared__ variable would make the
  // compiler's waitcnt pass treat every LDS read as aliasing the ring's LDS-DMA
  // writes and drain vmcnt before it (no pipelining)
  __shared__ double sm[LAT_LDS + 16];
  const int64_t np = d.nprod, role = blockIdx.y;
  if (role < np) {
    inc_producer_role<VT>(d, role, sm, reinterpret_cast<int*>(sm + LAT_LDS),
                          *reinterpret_cast<unsigned*>(sm + LAT_LDS + 8));
    return;
  }
  if (role < np + d.nwu) {
    lat_wblock<VT>(d, role - np, sm);
    return;
  }
#ifdef MFGP_DIAG_LATNOGEMM   // diagnostic build: producers and w only (timing only)
  return;
#endif
  const int64_t g = role - np - d.nwu;
  if (g >= (int64_t)d.lat_tiles * d.ksplit) return;
  const int64_t tile = g % d.lat_tiles, s = g / d.lat_tiles;
  lat_gemm<KA, VT>(d, tile, s, sm);
}

// KA = 8 (appends of k <= 8 rows) or 16 (k <= 16): one kernel each, so each
// carries only its own epilogue's registers
template <int KA, class VT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_INC_WAVES, MFGP_INC_WAVES))) void k_inc_lat(
    const GPDesc* __restrict__ descs) {
  inc_lat_wg<KA, VT>(descs[blockIdx.x]);
}

// The separable tables of rows [tab_lo, n0) (full-path refresh; the step itself
// appends its new rows). Grid (GPs, row chunks of 4 rows x 4 tables x tabw).
__global__ __launch_bounds__(NT) void k_lat_tables(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  const int64_t lo = d.tab_lo, hi = d.n0, tabw = d.tabw, tstride = d.ld * tabw;
  const int64_t r0 = lo + 4 * (int64_t)blockIdx.x;
  if (r0 >= hi) return;
  for (int64_t e = threadIdx.x; e < 4 * 4 * tabw; e += NT) {
    const int64_t row = r0 + e / (4 * tabw);
    const int t = (int)((e / tabw) % 4);
    const int64_t col = e % tabw;
    if (row >= hi) continue;
    d.tab[t * tstride + row * tabw + col] = lat_tab_value(d, t, row, col, d.X[2 * row], d.X[2 * row + 1]);
  }
}
