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
// w comes from the explicit inverse F = L^-1 (resident, lower triangular):
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
//   [nprod, nprod + nwb)       w blocks (64 rows of w each, top block first):
//                              wait for the compact rows of their rows, then
//                              w[j][a] = sum_{i >= j} F[i][j] L21c[i][a] on MFMA,
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
constexpr int LXS = LKS * 8;              // Xs: Ex rows [LKS][8 ix of the tile]
constexpr int LSTG = LBS + LWS + LXS;      // doubles per stage
constexpr int LAT_TS = 65;                // row stride of the epilogue's T~ image [64][65]
constexpr int LAT_LDS = LNST * LSTG + LNST * 32 + 272 + 256 + 32;   // ring + flag words | epilogue: 37.6 KB
static_assert(LAT_LDS >= FIN_LDS, "the ring also holds the finish's LDS image");
static_assert(64 * LAT_TS + 272 + 256 + 32 <= LAT_LDS, "the epilogue image fits");
static_assert(LNST > 3 || LAT_LDS + 16 <= 5120, "four workgroups per CU (40 KB of LDS each)");
constexpr int LAT_PART = 4 * 16 * 64;     // doubles of one split-K partial tile (4 waves x 16 acc x 64 lanes)

// Stage s of the descending term order: blocks jb >= jh have L and H parts (8
// stages of 16 rows), blocks below jh the L part only (4 stages).
__device__ __forceinline__ void lat_stage(int64_t s, int64_t nwb, int64_t jh, int64_t& jb, int& part, int64_t& j0) {
  const int64_t nh = (nwb - jh) * 8;
  if (s < nh) {
    jb = nwb - 1 - s / 8;
    part = (int)((s % 8) / 4);
    j0 = 64 * jb + 16 * (s % 4);
  } else {
    s -= nh;
    jb = jh - 1 - s / 4;
    part = 0;
    j0 = 64 * jb + 16 * (s % 4);
  }
}
__device__ __forceinline__ int64_t lat_nstages(int64_t nwb, int64_t jh) { return (nwb - jh) * 8 + jh * 4; }
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

// One 64-row block jb of w = F11^T L21^T (+ row k: F^T z1, unused): wave w owns
// columns j = 64 jb + 16 w + r, lanes sum over rows i in [64 jb, n0) -- F's lower
// triangle below the block -- with two MFMAs per 8 rows (B = F[i][j] as one
// 16-byte load of rows 2q, 2q + 1; A = the compact rows L21c[i][a]). Four
// accumulators keep four MFMA chains in flight.
template <class VT>
__device__ __forceinline__ void lat_wblock(const GPDesc& d, int64_t jb) {
  const int64_t n0 = d.n0, ld = d.ld, i_lo = 64 * jb;
  const double* const l21c = d.l21c;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  WTRACE(0);
  wait_l21_from(d, i_lo);
  WTRACE(1);
  const int64_t j = i_lo + 16 * w + r;
  const GLOBAL dv2* Fc = reinterpret_cast<const GLOBAL dv2*>(gp(d.F) + j * ld);
  d4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = d4{0.0, 0.0, 0.0, 0.0};
  constexpr int IU = 8;
  for (int64_t i0 = i_lo; i0 < n0; i0 += 8 * IU) {
    dv2 f[IU];
    double a0[IU], a1[IU];
#pragma unroll
    for (int u = 0; u < IU; ++u) {
      const int64_t i = i0 + 8 * u + 2 * q;
      const int64_t ii = i < n0 ? i : i_lo;
      // F is read once per step and would evict the GEMM tiles' tables from L2
      f[u] = __builtin_nontemporal_load(Fc + (ii >> 1));
      a0[u] = l21c_at<VT>(l21c, ii, r);
      a1[u] = l21c_at<VT>(l21c, ii + 1 < n0 ? ii + 1 : ii, r);
    }
#pragma unroll
    for (int u = 0; u < IU; ++u) {
      const int64_t i = i0 + 8 * u + 2 * q;
      const double x0 = i < n0 ? a0[u] : 0.0;
      const double x1 = i + 1 < n0 ? a1[u] : 0.0;
      acc[(u & 1) * 2] = mfma(x0, f[u].x, acc[(u & 1) * 2]);
      acc[(u & 1) * 2 + 1] = mfma(x1, f[u].y, acc[(u & 1) * 2 + 1]);
    }
  }
  // lane (r, g) register v: row a = g + 4v of column j
  double* const wv = d.wv;
#pragma unroll
  for (int v = 0; v < 4; ++v)
    stx<true>(&wv[j * KINC + q + 4 * v], (acc[0][v] + acc[1][v]) + (acc[2][v] + acc[3][v]));
  drain_stores();
  __syncthreads();
  if (tid == 0) publish(d.wflag + jb, d.epoch);
  WTRACE(2);
  // a share of the new rows' separable tables (read from the next launch on)
  const int k = (int)(d.N - n0);
  const int64_t tabw = d.tabw, tstride = (d.ld) * tabw;
  const int64_t tot = 4 * (int64_t)k * tabw;
  const int64_t per = (tot + d.nwb - 1) / d.nwb, e0 = (d.nwb - 1 - jb) * per;
  const int64_t e1 = e0 + per < tot ? e0 + per : tot;
  for (int64_t e = e0 + tid; e < e1; e += NT) {
    const int t = (int)(e / (k * tabw));
    const int64_t rem = e % (k * tabw);
    const int a = (int)(rem / tabw);
    const int64_t col = rem % tabw;
    const double* p = row_pt(d, n0 + a);
    d.tab[t * tstride + (n0 + a) * tabw + col] = lat_tab_value(d, t, n0 + a, col, p[0], p[1]);
  }
}

// Geometry of one GEMM tile, and its buffer-descriptor LDS-DMA plan (as
// k_predict's: the lane part of each source offset is a VGPR fixed for the
// kernel, the row part an SGPR).
struct LatGeo {
  __amdgpu_buffer_rsrc_t rtab, rw;   // the four tables; w
  int64_t tstride, tabw;
  int64_t nwb, jh;
  int64_t ix0, iy0;
  unsigned vB, vW, vX;               // lane byte offsets: Bs, Ws, Xs
};

// Issue the DMAs of stage st into `slot` (waves 1..3; wave 0 only loads the w
// flags, so its vmcnt never waits for a flag's memory round trip behind a table
// load, nor theirs for a flag): Bs = 16 Ey rows x 64 iy (8 two-row DMAs:
// waves 1, 2 three each, wave 3 two, swizzled as swz), Ws = 16 w rows (waves 2,
// 3: 8 rows each), Xs = 16 Ex rows x 8 ix (wave 1).
__device__ __forceinline__ void lat_issue(const LatGeo& G, int64_t st, double* slot, int w) {
  int64_t jb, j0;
  int part;
  lat_stage(st, G.nwb, G.jh, jb, part, j0);
  const int64_t tx = (2 * part) * G.tstride, ty = tx + G.tstride;
  const int p0 = w == 1 ? 0 : (w == 2 ? 3 : 6), np = w == 3 ? 2 : 3;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    if (u < np) {
      const int p = p0 + u;
      dma_buf(G.rtab, slot + 2 * p * 64, G.vB, (unsigned)(8 * (ty + (j0 + 2 * p) * G.tabw + G.iy0)));
    }
  }
  if (w >= 2) dma_buf(G.rw, slot + LBS + 8 * (w - 2) * KINC, G.vW, (unsigned)(8 * (j0 + 8 * (w - 2)) * KINC));
  else dma_buf(G.rtab, slot + LBS + LWS, G.vX, (unsigned)(8 * (tx + j0 * G.tabw + G.ix0)));
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
// Ws / Xs rows), B[j][iy] = Ey[j][iy]. Wave (wm, wn): rows 32 wm.., columns 32 wn..
template <int KA>
__device__ __forceinline__ void lat_compute(const double* slot, d4 (&acc)[2][2], int wn, int r, int q, int ar,
                                            int ixl0, int ixl1) {
  const double* Bs = slot;
  const double* Ws = slot + LBS;
  const double* Xs = slot + LBS + LWS;
  // every operand of the stage first (20 LDS reads in flight), then the MFMAs:
  // the reads return in order, so the first k-step's MFMAs start after 5 of them
  double wa[LKS / 4], x0[LKS / 4], x1[LKS / 4], b0[LKS / 4], b1[LKS / 4];
#pragma unroll
  for (int ks = 0; ks < LKS / 4; ++ks) {
    const int j = 4 * ks + q;
    wa[ks] = Ws[j * KINC + ar];
    x0[ks] = Xs[j * 8 + ixl0];
    x1[ks] = Xs[j * 8 + ixl1];
    b0[ks] = Bs[swz(j, 32 * wn + r)];
    b1[ks] = Bs[swz(j, 32 * wn + 16 + r)];
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs
#pragma unroll
  for (int ks = 0; ks < LKS / 4; ++ks) {
    const double a0 = wa[ks] * x0[ks];
    const double a1 = wa[ks] * x1[ks];
#ifdef MFGP_DIAG_LATNOMMA   // diagnostic build: the loop without its MFMAs (timing only)
    acc[0][0][0] += a0 + b0[ks];
    acc[1][1][0] += a1 + b1[ks];
    continue;
#endif
    acc[0][0] = mfma(a0, b0[ks], acc[0][0]);
    acc[0][1] = mfma(a0, b1[ks], acc[0][1]);
    acc[1][0] = mfma(a1, b0[ks], acc[1][0]);
    acc[1][1] = mfma(a1, b1[ks], acc[1][1]);
  }
}

// One GEMM tile (split s of ksplit) and, for the last split to arrive, the cell
// epilogue of its (64 / KA) x 64 cells, F's new rows for its column blocks and
// the fused var max / argmax partials.
template <int KA, class VT>
__device__ __forceinline__ void lat_gemm(const GPDesc& d, int64_t tile, int64_t s, double* sm) {
  constexpr int IXPT = 64 / KA;   // lattice columns x per tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
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
  G.vX = (unsigned)(8 * ((lane >> 2) * G.tabw + 2 * (lane & 3)));
  G.nwb = d.nwb;
  G.jh = lat_jh(d);
  G.ix0 = tix * IXPT;
  G.iy0 = tiy * 64;
  const int64_t ns = lat_nstages(G.nwb, G.jh);
  const int64_t lo = ns * s / S, hi = ns * (s + 1) / S;
  WTRACE(0);
  // this lane's A rows: a = row % KA, lattice column ixl = row / KA (rows 32 wm + 16 m + r)
  const int ar = KA == 8 ? (r & 7) : r;
  const int ixl0 = KA == 8 ? 4 * wm + (r >> 3) : 2 * wm;
  const int ixl1 = KA == 8 ? 4 * wm + 2 + (r >> 3) : 2 * wm + 1;
  d4 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[m][n] = d4{0.0, 0.0, 0.0, 0.0};
  // w's readiness: wave 0 loads the flag word of each stage's block into LDS (an
  // agent-scope 4-byte LDS-DMA) two iterations before that stage's DMAs are
  // issued; waves 2 and 3, which stage the w rows, check it there after the
  // barrier (an LDS read, not a memory round trip) and spin on memory only if it
  // was not yet set. Wave 0 issues nothing else, so the flags' round trips never
  // sit in front of a table load in any wave's vmcnt order.
  const int cnt = w == 0 ? 1 : (w == 3 ? 3 : 4);   // vector-memory ops per issued stage
  unsigned* const fl = reinterpret_cast<unsigned*>(sm + LNST * LSTG);   // [LNST][64]
  const __amdgpu_buffer_rsrc_t rfl = make_rsrc(reinterpret_cast<const double*>(d.wflag),
                                               (int64_t)4 * (d.nwb + 1));
  auto blk = [&](int64_t st) {
    int64_t jb, j0;
    int part;
    lat_stage(st < hi ? st : hi - 1, G.nwb, G.jh, jb, part, j0);
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
  if (lo < hi) {
    if (w >= 2)
      for (int64_t st = lo; st < lo + D && st < hi; ++st) spin_wave(d, d.wflag + blk(st), d.epoch);
    WTRACE(1);
    for (int64_t st = lo; st < lo + D && st < hi; ++st) issue(st, st + D);
    // iteration t: stage t sits in slot (t - lo) % LNST, issued D iterations ago
    // with the flag of stage t + D, and followed by the ops of the stages after it
    for (int64_t t = lo; t < hi; ++t) {
      const int64_t after = (hi - 1 - t) < (D - 1) ? (hi - 1 - t) : (D - 1);
      vm_wait_bar((int)after * cnt);
      if (t + D < hi) {
        if (w >= 2 && fl[((t + D - lo) % LNST) * 64] != d.epoch) spin_wave(d, d.wflag + blk(t + D), d.epoch);
        issue(t + D, t + 2 * D);
      }
#ifndef MFGP_DIAG_LATNOCOMP   // diagnostic build: the pipeline without its compute (timing only)
      lat_compute<KA>(sm + ((t - lo) % LNST) * LSTG, acc, wn, r, q, ar, ixl0, ixl1);
#endif
      if (t == (lo + hi) / 2) WTRACE(5);
    }
  }
  vm_wait_all();
  __syncthreads();
  WTRACE(2);
  // split-K: partials through memory, the last split reduces them in split order
  if (S > 1) {
    unsigned& lat_last = *reinterpret_cast<unsigned*>(sm + LAT_LDS + 9);
    double* part = d.gpart + (tile * S + s) * LAT_PART + (int64_t)w * 16 * 64 + lane;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int v = 0; v < 4; ++v) stx<true>(part + ((m * 2 + n) * 4 + v) * 64, acc[m][n][v]);
    drain_stores();
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(d.gcnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lat_last = old == (unsigned)(S - 1) ? 1u : 0u;
      if (lat_last) __hip_atomic_store(d.gcnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!lat_last) return;
    d4 tot[2][2];
    for (int s2 = 0; s2 < S; ++s2) {
      const double* p2 = d.gpart + (tile * S + s2) * LAT_PART + (int64_t)w * 16 * 64 + lane;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const double x = (s2 == s) ? acc[m][n][v] : ldx<true>(p2 + ((m * 2 + n) * 4 + v) * 64);
            tot[m][n][v] = s2 == 0 ? x : tot[m][n][v] + x;
          }
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) acc[m][n] = tot[m][n];
  }
  // ---- epilogue: T~ to LDS, L22 / z2 (sync[2]), the new rows, L22^-1 ----
  const int64_t n0 = d.n0, ld = d.ld;
  const int k = (int)(d.N - n0);
  const Hyp& h = d.hp;
  double* Ts = sm;                               // T~ [64 rows (a, ixl)][LAT_TS], column = iy - iy0
  double* L22 = sm + 64 * LAT_TS;                // [16][16] | z2 [16]
  double* Li = L22 + KINC * KINC + KINC;         // L22^-1 [16][16]
  double* Xn = Li + KINC * KINC;                 // new rows (x, y)
  __syncthreads();   // the ring's last reads are done (split-K: nothing of it is live)
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) Ts[(32 * wm + 16 * m + q + 4 * v) * LAT_TS + 32 * wn + 16 * n + r] = acc[m][n][v];
  wait_flag(d, d.sync + 2, d.epoch);
  WTRACE(3);
  for (int e = tid; e < KINC * KINC + KINC; e += NT) {
    // plain loads: no line of the record is read in this launch before sync[2]
    const double v = d.l22r[e];
    const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
    L22[e] = use ? v : 0.0;
  }
  if (tid >= NT - KINC) {
    const int a = tid - (NT - KINC);
    const double* p = row_pt(d, n0 + (a < k ? a : 0));
    Xn[2 * a] = p[0];
    Xn[2 * a + 1] = p[1];
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
  // ---- cells: thread u of the tile's (64 / KA) x 64 cells (iy fastest) ----
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  VT* const Vr = const_cast<VT*>(vres_ptr<VT>(d));
  const GLOBAL double* grid = gp(d.grid);
  for (int u = tid; u < IXPT * 64; u += NT) {
    const int ixl = u >> 6, iyl = u & 63;
    const int64_t ix = G.ix0 + ixl, iy = G.iy0 + iyl;
    if (ix >= lat.nx || iy >= lat.ny) continue;
    const int64_t c = ix * lat.sx + iy * lat.sy;
    const double gx = grid[2 * c], gy = grid[2 * c + 1];
    const double* tt = Ts + (KA * ixl) * LAT_TS + iyl;   // T~ of row a at tt[a * LAT_TS]
    double vn[KA];
    double vs = 0.0, ms = 0.0;
#pragma unroll
    for (int a = 0; a < KA; ++a) {
      vn[a] = 0.0;
      if (a < k) {
        double t = psi_new(h, d.NL, n0 + a, gx, gy, Xn[2 * a], Xn[2 * a + 1]) - tt[a * LAT_TS];
#pragma unroll
        for (int b = 0; b < a; ++b) t -= L22[a * KINC + b] * vn[b];
        vn[a] = t / L22[a * KINC + a];
        vs += vn[a] * vn[a];
        ms += vn[a] * L22[KINC * KINC + a];
      }
    }
    const double vc = d.rvar_in[c] - vs;
    const double mc = d.rmu_in[c] + ms;
    VT* vt = Vr + (c / PBM) * d.vld * PBM + (c % PBM);
#pragma unroll
    for (int a = 0; a < KA; ++a)
      if (a < k) vt[(n0 + a) * PBM] = (VT)vn[a];
    d.mu[c] = mc;
    d.var[c] = vc;
    if (d.rmu) {
      d.rmu[c] = mc;
      d.rvar[c] = vc;
    }
    argmax_pair(bv, bi, vc, c);
  }
  // ---- F's new rows: -L22^-1 w^T for this tile's column blocks, L22^-1 (tile 0) ----
  const int64_t tiles = d.lat_tiles;
  for (int64_t jb = tile; jb < d.nwb; jb += tiles) {
    wait_flag(d, d.wflag + jb, d.epoch);
    for (int e = tid; e < 64 * k; e += NT) {
      const int a = e >> 6;
      const int64_t j = 64 * jb + (e & 63);
      if (j >= n0) continue;
      double t = 0.0;
      for (int b = 0; b <= a; ++b) t -= Li[a * KINC + b] * d.wv[j * KINC + b];
      d.F[j * ld + n0 + a] = t;
    }
  }
  if (tile == 0)
    for (int e = tid; e < k * k; e += NT) {
      const int a = e / k, b = e % k;
      if (b <= a) d.F[(n0 + b) * ld + n0 + a] = Li[a * KINC + b];
    }
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
  if (role < np + d.nwb) {
    lat_wblock<VT>(d, d.nwb - 1 - (role - np));
    return;
  }
  const int64_t g = role - np - d.nwb;
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
