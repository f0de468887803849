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
//   [nprod, nprod + nwu)       w units (a pair of 64-column blocks of F, the
//                              top block and the bottom one, x a row part):
//                              wait for the compact rows, then
//                              w[j][a] = sum_{i >= j} F[i][j] L21c[i][a] on
//                              MFMA; store w (or a partial: the last row part
//                              adds them), count it into ldone; then F's new rows
//                              and a share of the new rows' separable tables
//   [.., + nzu)                Z units: wait for all of w, sum w c ex per lattice
//                              row (the GEMM's A rows)
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

// Axis table entry (t as lat_tab_value, no coefficient) of lattice axis value p
// against axis column col: the factor lat_tab_value gives a training row whose
// coordinate is that axis value, bit for bit (same operations, same operands).
__device__ double lat_axis_value(const GPDesc& d, int t, int64_t p, int64_t col) {
#pragma clang fp contract(off)
  const Hyp& h = d.hp;
  const GridLattice& L = d.lat;
  const bool isx = (t & 1) == 0;
  const int64_t n = isx ? L.nx : L.ny;
  if (col >= n || p >= n) return 0.0;
  if (t >= 2 && h.kind == 0) return 0.0;
  const double l = t >= 2 ? h.lH : h.lL;
  const double ax = isx ? d.grid[2 * (col * L.sx)] : d.grid[2 * (col * L.sy) + 1];
  const double ap = isx ? d.grid[2 * (p * L.sx)] : d.grid[2 * (p * L.sy) + 1];
  const double dx = div_(ax, l) - div_(ap, l);
  return exp(-0.5 * (dx * dx));
}

// Lattice indices of a point: px | (py << 16) when both coordinates are axis
// values (exact equality; the rounded estimate and its neighbours), else -1.
__device__ int lattice_xy(const GPDesc& d, double px, double py) {
  const GridLattice& L = d.lat;
  if (L.nx <= 0 || !(px == px) || !(py == py)) return -1;
  const int ex = (int)rint(fmin(fmax((px - L.x0) * L.xinv, 0.0), (double)(L.nx - 1)));
  const int ey = (int)rint(fmin(fmax((py - L.y0) * L.yinv, 0.0), (double)(L.ny - 1)));
  int hx = -1, hy = -1;
  for (int t = -1; t <= 1; ++t) {
    const int cx = ex + t, cy = ey + t;
    if (cx >= 0 && cx < L.nx && d.grid[2 * (cx * L.sx)] == px) hx = cx;
    if (cy >= 0 && cy < L.ny && d.grid[2 * (cy * L.sy) + 1] == py) hy = cy;
  }
  return (hx >= 0 && hy >= 0) ? (hx | (hy << 16)) : -1;
}

// Phase hand-off: every unit of a phase counts its arrival (relaxed fetch_add,
// after draining its stores); the last of the n resets the count for the next
// launch and raises the phase flag (c[1] = epoch). Waiters poll that one word.
__device__ __forceinline__ void arrive_phase(unsigned* c, unsigned epoch, int64_t n) {
  const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old == (unsigned)(n - 1)) {
    __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish(c + 1, epoch);
  }
}
// Wait (thread 0 polls, the workgroup joins at the barrier) for a phase flag.
__device__ __forceinline__ void wait_phase(const GPDesc& d, const unsigned* c, unsigned epoch) {
  wait_flag(d, c + 1, epoch);
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

// L22^-1 (rows / columns >= k zero) into Li [16][16] from the L22 record (sync[2]
// must have been seen; L2-served loads: the finish stored it in this launch).
// L22 is scratch [16][16 | 16].
__device__ __forceinline__ void lat_l22inv(const GPDesc& d, int k, double* L22, double* Li) {
  const int tid = threadIdx.x;
  for (int e = tid; e < KINC * KINC; e += NT) {
    const double v = ldx<true>(d.l22r + e);
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

// Compact row i, entry a (written by the producers in this launch: an L2-served
// load of the agent scope, never a possibly stale L1 line).
template <class VT>
__device__ __forceinline__ double l21c_ld(const double* l21c, int64_t i, int a) {
  if constexpr (sizeof(VT) == 8) {
    return __hip_atomic_load(gp(l21c) + i * KINC + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    return (double)__hip_atomic_load(gp(reinterpret_cast<const float*>(l21c)) + i * KINC + a, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
  }
}

#ifndef MFGP_W_DEPTH_F
#define MFGP_W_DEPTH_F 10
#endif
#ifndef MFGP_W_DEPTH
#define MFGP_W_DEPTH 6
#endif
// The w units' share of F: F's lower triangle as one stream of 16-row steps,
// block jb's rows [64 jb, n0) in nb(jb) = ceil(n0 / 16) - 4 jb steps, the blocks
// in pair order 0, nwb - 1, 1, nwb - 2, ... (a pair's steps add up to the same K2
// = 2 ceil(n0 / 16) - 4 (nwb - 1) whichever pair; a share then spans few blocks);
// unit u of U takes the steps [u S / U, (u + 1) S / U) of the S in all. So every
// unit streams the same bytes whatever n0 and the unit count (a unit per block
// pair left 1 in 17 CUs with two units at B = 8, and the stream ran at the slower
// CUs' rate). A block's steps spread over units u_first .. u_last of it; each
// stores a partial of the block's w at slot u + (its position) of the GP's partials.
__device__ __forceinline__ int64_t wst_first(int64_t C, int64_t nwb, int64_t jb) {
  const int64_t K2 = 2 * C - 4 * (nwb - 1);
  return 2 * jb < nwb ? jb * K2 : (nwb - 1 - jb) * K2 + C - 4 * (nwb - 1 - jb);
}
__device__ __forceinline__ int64_t wst_start(int64_t u, int64_t S, int64_t U) { return u * S / U; }
__device__ __forceinline__ int64_t wst_unit(int64_t s, int64_t S, int64_t U) { return ((s + 1) * U - 1) / S; }
// block jb's position in the pair order (its partials: slots u + position, distinct
// since a position's units start where the previous position's end)
__device__ __forceinline__ int64_t wst_pos(int64_t nwb, int64_t jb) {
  return 2 * jb < nwb ? 2 * jb : 2 * (nwb - 1 - jb) + 1;
}

// One w unit: w = F11^T L21^T, w[j][a] = sum_{i >= j} F[i][j] L21c[i][a], over the
// unit's steps. Per step, wave w takes rows 4 w + q: lane (r, q) loads L21c[i][r]
// (the MFMA A operand, a = r) and F[i][32 hh + 2 r + c] for hh, c = 0, 1 (B; two
// 16-byte loads: 16 lanes cover a 512-byte row). Four steps in flight per wave in
// registers. At the end of a block's steps the waves' sums meet in LDS in wave
// order and the partial is stored (no wait: stores only, the stream goes on);
// after the stream each of the unit's blocks counts its partial in, and whoever
// counts a block in last adds its partials in slot order (the same bits whoever it
// is), stores the block of w, counts it into ldone[0] (the Z units wait for all
// nwb blocks) and writes F's new rows for its columns, -L22^-1 w^T (the top
// block's also the L22^-1 entries).
template <int KA, class VT>
__device__ __forceinline__ void lat_wblock(const GPDesc& d, int64_t u, double* sm) {
  // steps in flight per wave: the loop is latency-bound (each step waits for loads
  // issued DEPTH - 1 steps earlier), so fp32 F, whose raw 16-byte rows take half the
  // registers of the widened pairs, keeps more in flight
  constexpr int DEPTH = sizeof(VT) == 4 ? MFGP_W_DEPTH_F : MFGP_W_DEPTH;
  // M4: appends of k <= 8 rows (KA = 8) take the 4x4x4 f64 MFMA (v_mfma_f64_4x4x4_4b:
  // four 4 x 4 blocks, K = 4), whose blocks hold exactly the k <= 8 live rows a of w
  // in two instructions (a = r' + 4 t) where the 16x16x4 form's 16-row A operand
  // left half its rows zero; and on gfx950 it issues 1.64x the 16x16x4 form's
  // multiply-adds per cycle (tools/probe_mfma4.hip): the w units' MFMA time / 3.3.
  // Lane l = 16 q + 4 blk + r' (q: the K row, as before): A = L21c[i][r' + 4 t],
  // B = the lane's F value s, C lane 16 i + 4 blk + j = w[col_s(4 blk + j)][i + 4 t]
  constexpr bool M4 = KA == 8;
  constexpr int NA = M4 ? 2 : 1;   // A values per lane and step
  // a step's F in registers: two widened pairs (fp64 F) or the raw four floats (fp32)
  struct FRow {
    dv2 v[sizeof(VT) == 4 ? 1 : 2];
  };
  struct ARow {
    double v[NA];
  };
  const int64_t n0 = d.n0, ld = d.ld;
  const int nwb = d.nwb;
  const int64_t U = d.nwu;
  const double* const l21c = d.l21c;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const unsigned epoch = d.epoch;
  WTRACE(0);
  const int k = (int)(d.N - n0);
  // a share of the new rows' separable tables and lattice indices: read by the
  // GEMM's cells (in this launch, G1; after it, lat_g2) and by later steps. With
  // the GEMM as a second launch they are stored after the unit's F stream, off the
  // stream's start (two dependent round trips: the rows' coordinates, then the grid)
  auto tables_share = [&]() {
    const int64_t tabw = d.tabw, tstride = (d.ld) * tabw;
    const int64_t tot = 4 * (int64_t)k * tabw;
    const int64_t per = (tot + U - 1) / U, e0 = u * per;
    const int64_t e1 = e0 + per < tot ? e0 + per : tot;
    for (int64_t e = e0 + tid; e < e1; e += NT) {
      const int t = (int)(e / (k * tabw));
      const int64_t rem = e % (k * tabw);
      const int a = (int)(rem / tabw);
      const int64_t col = rem % tabw;
      const double* pt = row_pt(d, n0 + a);
      // written through: the GEMM tiles' epilogues read them in this launch (G1)
      stx<true>(&d.tab[t * tstride + (n0 + a) * tabw + col], lat_tab_value(d, t, n0 + a, col, pt[0], pt[1]));
    }
    if (u == 0 && tid < k) {
      const double* pt = row_pt(d, n0 + tid);
      d.lidx[n0 + tid] = lattice_xy(d, pt[0], pt[1]);
    }
  };
  if (!d.lat_g2) tables_share();
  const int64_t C = (n0 + 15) / 16;
  const int64_t K2 = 2 * C - 4 * (nwb - 1);
  const int64_t S = (nwb / 2) * K2 + (nwb & 1) * (C - 4 * (nwb / 2));
  const int64_t s0 = wst_start(u, S, U), s1 = wst_start(u + 1, S, U);
  const int64_t T = s1 - s0;
  // the unit's first step: pair p0, its first (odd0 = 0: block p0) or second block
  // (nwb - 1 - p0), step st0 of it
  const int64_t p0 = s0 / K2;
  const int64_t rem0 = s0 - p0 * K2;
  const bool odd0 = rem0 >= C - 4 * p0;
  const int64_t jb0 = odd0 ? nwb - 1 - p0 : p0;
  const int64_t st0 = odd0 ? rem0 - (C - 4 * p0) : rem0;
  // LDS: red [4 w][2 acc][4 v][64] (one 32-column half at a time) | the unit's
  // blocks [<= LAT_NWB_MAX] | their last-arrival marks | w of a block [64 jl][16 a]
  // | L22 | Li
  double* const red = sm;
  int* const segs = reinterpret_cast<int*>(sm + 2048);
  int* const lastm = segs + LAT_NWB_MAX;
  double* const Wh = sm + 2048 + LAT_NWB_MAX;
  double* const L22 = Wh + 64 * KINC;
  double* const Li = L22 + KINC * KINC + KINC;
  static_assert(LAT_NWB_MAX <= NT, "one thread per block of the unit counts it in");
  static_assert(2048 + LAT_NWB_MAX + 64 * KINC + 2 * KINC * KINC + KINC <= LAT_LDS, "the w unit's LDS fits");
  // a cursor over the steps: block jb, step st of its nb, in pair p (second block: odd)
  struct Cur {
    int64_t jb, st, nb, p;
    bool odd;
  };
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
  const Cur cur0{jb0, st0, C - 4 * jb0, p0, odd0};
  // lane (r, q) loads columns 32 hh + 2 r, 2 r + 1 (hh = 0, 1) of its row with two
  // 16-byte loads: MFMA 2 hh + 0 takes the even columns, 2 hh + 1 the odd ones. A
  // row past n0 (the block's last step) reloads row n0 - 1 (finite) and is masked.
  auto row_of = [&](const Cur& c) { return 64 * c.jb + 16 * c.st + 4 * w + q; };
  auto load_f = [&](const Cur& c, FRow& f) {
    const int64_t i = row_of(c);
    const int64_t ii = i < n0 ? i : n0 - 1;
    // plain loads: F stays in the memory-side cache across steps where it fits
    // (tools/probe_wloop.hip: 2 units per CU, plain 25 us vs non-temporal 26-30 us)
    if constexpr (sizeof(VT) == 4) {
      // MFGP_F32: F streamed in fp32 (half the bytes), widened for the f64 MFMA; one
      // 16-byte load per lane: columns 4 r .. 4 r + 3 (acc[j] then holds column 4 r + j;
      // seg_done stores by that map)
      // (kept as raw bits in a dv2 slot: widened at compute)
      f.v[0] = *reinterpret_cast<const GLOBAL dv2*>(gp(d.Ff) + fblk_off(c.jb, ld) + (ii - 64 * c.jb) * 64 + 4 * r);
    } else {
      const GLOBAL dv2* Fr =
          reinterpret_cast<const GLOBAL dv2*>(gp(d.F) + fblk_off(c.jb, ld) + (ii - 64 * c.jb) * 64 + 2 * r);
      f.v[0] = Fr[0];
      f.v[sizeof(VT) == 4 ? 0 : 1] = Fr[16];
    }
  };
  // The A operand L21[r][i]. When every new point is the lattice cell its rounded
  // axis estimate names (the producers' fast-path test, inc_gather_fast; every wave
  // tests the same points, so the verdict is uniform), L21[r][.] is the V column
  // of that cell, read here straight from the resident V (rows < n0: not written
  // in this launch): the F stream starts at once instead of after the producers'
  // compact rows (~9 us). Otherwise the compact rows, after the producers' flags.
  // the rows a of w this lane's A values carry: r (16x16x4), r' + 4 t (M4)
  const int ar0 = M4 ? (lane & 3) : r;
  const VT* asrc[NA];
  int64_t astr;
  bool selfg;
  {
    const GridLattice L = d.lat;
    int64_t cr[NA];
    bool miss = false;
#pragma unroll
    for (int t = 0; t < NA; ++t) {
      const int a = ar0 + 4 * t;
      const double* p = row_pt(d, n0 + (a < k ? a : 0));
      const double px = p[0], py = p[1];
      const int ix = (int)rint(fmin(fmax((px - L.x0) * L.xinv, 0.0), (double)(L.nx - 1)));
      const int iy = (int)rint(fmin(fmax((py - L.y0) * L.yinv, 0.0), (double)(L.ny - 1)));
      cr[t] = (px == px && py == py) ? ix * L.sx + iy * L.sy : 0;
      const dv2 g = reinterpret_cast<const GLOBAL dv2*>(gp(d.grid))[cr[t]];
      miss = miss || (a < k && !(g.x == px && g.y == py));
    }
    selfg = d.lat_selfg && L.nx > 0 && d.vres >= n0 && vres_ptr<VT>(d) != nullptr && __ballot(miss) == 0;
    // (lanes whose row a >= k carry no point: they read row 0's element, the same
    // line, so the compact rows' unused part costs no traffic; their MFMA input is zeroed)
#pragma unroll
    for (int t = 0; t < NA; ++t) {
      const int a = ar0 + 4 * t;
      asrc[t] = selfg ? vres_ptr<VT>(d) + (cr[t] / PBM) * d.vld * PBM + (cr[t] % PBM)
                      : reinterpret_cast<const VT*>(l21c) + (a < k ? a : 0);
    }
    astr = selfg ? (int64_t)PBM : (int64_t)KINC;
  }
  auto load_a = [&](const Cur& c, ARow& a) {
    const int64_t i = row_of(c);
    // L2-served (the compact rows were stored in this launch)
#pragma unroll
    for (int t = 0; t < NA; ++t)
      a.v[t] = (double)__hip_atomic_load(gp(asrc[t]) + (i < n0 ? i : n0 - 1) * astr, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  };
  // 16x16x4: acc[2 hh + c] (lane (n, g) register v: w[col 32 hh + 2 n + c][a = g + 4 v]);
  // M4: acc4[s][t] (lane 16 i + 4 blk + j: w[col_s(4 blk + j)][a = i + 4 t])
  d4 acc[M4 ? 1 : 4];
  double acc4[M4 ? 4 : 1][NA];
#pragma unroll
  for (int c = 0; c < (M4 ? 1 : 4); ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int c = 0; c < (M4 ? 4 : 1); ++c)
#pragma unroll
    for (int t = 0; t < NA; ++t) acc4[c][t] = 0.0;
  // (columns a >= k of w are never read: zero)
  auto compute = [&](const FRow& fr, const ARow& a, bool live) {
    dv2 f[2];
    if constexpr (sizeof(VT) == 4) {
      const f4 fq = __builtin_bit_cast(f4, fr.v[0]);   // columns 4 r .. 4 r + 3, widened
      f[0] = dv2{(double)fq.x, (double)fq.y};
      f[1] = dv2{(double)fq.z, (double)fq.w};
    } else {
      f[0] = fr.v[0];
      f[1] = fr.v[sizeof(VT) == 4 ? 0 : 1];
    }
    if constexpr (M4) {
      // F value s = 2 hh + c of the lane: column 32 hh + 2 r + c (fp64), 4 r + s (fp32)
#pragma unroll
      for (int t = 0; t < NA; ++t) {
        const double av = (live && ar0 + 4 * t < k) ? a.v[t] : 0.0;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          acc4[2 * hh][t] = mfma4(av, f[hh].x, acc4[2 * hh][t]);
          acc4[2 * hh + 1][t] = mfma4(av, f[hh].y, acc4[2 * hh + 1][t]);
        }
      }
    } else {
      const double av = (live && r < k) ? a.v[0] : 0.0;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        acc[2 * hh] = mfma(av, f[hh].x, acc[2 * hh]);
        acc[2 * hh + 1] = mfma(av, f[hh].y, acc[2 * hh + 1]);
      }
    }
  };
  int nseg = 0;
  // the end of block jb's steps in this unit: the waves' sums in wave order (one
  // 32-column half at a time), stored as the unit's partial of the block. Its
  // barriers wait for the LDS accesses only (lds_barrier: __syncthreads' fence would
  // wait for every load in flight). A block that ends inside the unit's stream keeps
  // its partial in registers (own_s) until the stream is done: its write-through
  // stores sit in the same in-order vmcnt queue as the F loads, and the loop's waits
  // for the loads behind them waited for their write acknowledgements too (the units
  // whose share spans two blocks streamed ~2.2 us longer)
  double own_s[4] = {0.0, 0.0, 0.0, 0.0};
  int64_t jb_s = -1;
  auto store_part = [&](const double (&own)[4], int64_t jb) {
    double* const part = d.wpart + (u + wst_pos(nwb, jb)) * 1024;
    if constexpr (sizeof(VT) == 4) {
      // (the fp32 F's lanes: own[2 hh + m2] is column 4 (jp >> 1) + 2 hh + (jp & 1), row a)
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const int x = tid + NT * (m & 1), jp = x >> 4, a = x & 15, hh = m >> 1;
        stx<true>(part + (((jp >> 1) << 2) | (hh << 1) | (jp & 1)) * 16 + a, own[m]);
      }
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m) stx<true>(part + tid + NT * m, own[m]);
    }
  };
  auto seg_done = [&](int64_t jb, bool defer) {
    // thread tid: outputs e = tid + 256 m, (jl, a) = (e >> 4, e & 15), jl = 32 hh +
    // jh; lane (rr, g) register v of acc[2 hh + c] is w row a = g + 4 v, column
    // jh = 2 rr + c
    double own[4];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      if constexpr (M4) {
        // half hh: the lane's F values s = 2 hh + c; red [4 w][c][t][64]
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int t = 0; t < NA; ++t) red[w * 256 + (c * 2 + t) * 64 + lane] = acc4[2 * hh + c][t];
        lds_barrier();
#pragma unroll
        for (int m2 = 0; m2 < 2; ++m2) {
          // output (local column jh of the half, row a): the lane 16 (a & 3) + (jh >> 1)
          // (r = 4 blk + j = jh >> 1), value c = jh & 1, t = a >> 2
          const int e = tid + NT * m2, jh = e >> 4, a = e & 15;
          const int o = ((jh & 1) * 2 + ((a >> 2) & 1)) * 64 + 16 * (a & 3) + (jh >> 1);
          own[2 * hh + m2] = a < 8 ? (red[o] + red[256 + o]) + (red[512 + o] + red[768 + o]) : 0.0;
        }
        lds_barrier();
      } else {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int v = 0; v < 4; ++v) red[w * 512 + (c * 4 + v) * 64 + lane] = acc[2 * hh + c][v];
        lds_barrier();
#pragma unroll
        for (int m2 = 0; m2 < 2; ++m2) {
          const int e = tid + NT * m2, jh = e >> 4, a = e & 15;
          const int o = ((jh & 1) * 4 + (a >> 2)) * 64 + 16 * (a & 3) + (jh >> 1);
          own[2 * hh + m2] = (red[o] + red[512 + o]) + (red[1024 + o] + red[1536 + o]);
        }
        lds_barrier();
      }
    }
#pragma unroll
    for (int c = 0; c < (M4 ? 1 : 4); ++c) acc[c] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int c = 0; c < (M4 ? 4 : 1); ++c)
#pragma unroll
      for (int t = 0; t < NA; ++t) acc4[c][t] = 0.0;
    // own[2 hh + m2] is output e = 512 hh + tid + 256 m2 of the block
    if (defer && jb_s < 0) {
#pragma unroll
      for (int m = 0; m < 4; ++m) own_s[m] = own[m];
      jb_s = jb;
    } else {
      store_part(own, jb);
    }
    if (tid == 0) segs[nseg] = (int)jb;
    ++nseg;
  };
  // the pipeline: step t's loads go out with step t - DEPTH + 1's MFMAs. Loads
  // past the unit's last step reload its last step (unused): a branch around a
  // load would make the compiler's wait for the current step also wait for the
  // loads behind it.
  FRow fb[DEPTH];
  ARow ab[DEPTH];
  Cur cl = cur0;   // the next step to load (clamped to the last)
  int64_t tl = 0;
  auto next_load = [&]() {
    if (tl + 1 < T) {
      adv(cl);
      ++tl;
    }
  };
  if (!selfg) {
    // the unit's lowest row: its first step's, or (spanning more blocks) at most
    // pair p0 + 1's first block's first
    const int64_t lo = 64 * jb0 + 16 * st0;
    const int64_t lo2 = st0 + T > C - 4 * jb0 ? 64 * (p0 + 1) : lo;
    wait_l21_from(d, lo < lo2 ? lo : lo2);
  }
  WTRACE(1);
  // the first DEPTH - 1 steps' loads in the loop's own order (F, then L21c, per
  // step): the compiler's waits in the loop then count DEPTH - 1 steps in flight
  // (issuing their F loads before the wait for the compact rows: within noise at
  // B = 8, 89.3k vs 88.9k GP-updates/s, and 128 spilled VGPRs at KA = 16)
#pragma unroll
  for (int b = 0; b + 1 < DEPTH; ++b) {
    load_f(cl, fb[b]);
    load_a(cl, ab[b]);
    next_load();
  }
  Cur cc = cur0;   // the step being computed
  // (whole groups of DEPTH steps, no exits in between: an exit path makes the
  // compiler's waits at the loop head drain every load in flight; the buffers by
  // compile-time index: registers)
  for (int64_t t0 = 0; t0 < T; t0 += DEPTH) {
#pragma unroll
    for (int b = 0; b < DEPTH; ++b) {
      const int64_t t = t0 + b;
      // issue step t + DEPTH - 1 (into the buffer step t - 1 used), then compute
      // step t (steps past T: the last step's rows again, masked)
      load_f(cl, fb[(b + DEPTH - 1) % DEPTH]);
      load_a(cl, ab[(b + DEPTH - 1) % DEPTH]);
      next_load();
      compute(fb[b], ab[b], t < T && row_of(cc) < n0);
      if (t < T) {
        if (cc.st + 1 == cc.nb || t + 1 == T) seg_done(cc.jb, t + 1 < T);
        if (t + 1 < T) adv(cc);
      }
    }
  }
  if (jb_s >= 0) store_part(own_s, jb_s);   // (the stream is done: no load behind it)
  WTRACE(3);
  // count the unit's partials in (one arrival per block, all at once)
  drain_stores();
  __syncthreads();
  if (tid < nseg) {
    const int64_t jb = segs[tid];
    const unsigned old = __hip_atomic_fetch_add(d.wcnt + jb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t f = wst_first(C, nwb, jb);
    const int64_t ncon = wst_unit(f + C - 4 * jb - 1, S, U) - wst_unit(f, S, U) + 1;
    const bool last = old == (unsigned)(ncon - 1);
    if (last) __hip_atomic_store(d.wcnt + jb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lastm[tid] = last ? 1 : 0;
  }
  __syncthreads();
  // the blocks this unit counted in last, in a row (thread 0: a handful)
  if (tid == 0) {
    int nl = 0;
    for (int g = 0; g < nseg; ++g)
      if (lastm[g]) segs[nl++] = segs[g];
    lastm[0] = nl;
  }
  __syncthreads();
  const int nlast = lastm[0];
  if (nlast == 0) {
    if (d.lat_g2) tables_share();
    return;
  }
  // the blocks' w: every contributor's partial in slot order (the same bits whoever
  // is last), stored, then counted into ldone[0] together (one lane each; the Z
  // units wait for all nwb blocks)
  for (int g = 0; g < nlast; ++g) {
    const int64_t jb = segs[g];
    const int64_t f = wst_first(C, nwb, jb);
    const int64_t ua = wst_unit(f, S, U), ub = wst_unit(f + C - 4 * jb - 1, S, U);
    const double* const p0p = d.wpart + (ua + wst_pos(nwb, jb)) * 1024;
    const int R = (int)(ub - ua + 1);
    double own[4];
    for (int r0 = 0; r0 < R; r0 += 4) {   // four partials' loads in flight at a time
      double x[4][4];
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int m = 0; m < 4; ++m) x[rr][m] = r0 + rr < R ? ldx<true>(p0p + (r0 + rr) * 1024 + tid + NT * m) : 0.0;
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int m = 0; m < 4; ++m)
          if (r0 + rr < R) own[m] = (r0 + rr == 0) ? x[rr][m] : own[m] + x[rr][m];
    }
    double* const wv = d.wv + 64 * jb * KINC;
#pragma unroll
    for (int m = 0; m < 4; ++m) stx<true>(wv + tid + NT * m, own[m]);
  }
  drain_stores();
  __syncthreads();
  // each block's own flag (the Z units poll all nwb of them: no count of the blocks'
  // arrivals on one word in between, one round trip fewer on the step's chain)
  if (tid < nlast) publish(d.wflag + segs[tid], epoch);
  WTRACE(2);
  // F's new rows for the blocks (read from the next launch on): F[n0 + a][j] =
  // -sum_{b <= a} L22^-1[a][b] w[j][b], w reloaded (this workgroup stored it)
  wait_flag(d, d.sync + 2, epoch);
  lat_l22inv(d, k, L22, Li);
  for (int g = 0; g < nlast; ++g) {
    const int64_t jb = segs[g];
    const double* const wv = d.wv + 64 * jb * KINC;
#pragma unroll
    for (int m = 0; m < 4; ++m) Wh[tid + NT * m] = ldx<true>(wv + tid + NT * m);
    __syncthreads();
    for (int e = tid; e < 64 * k; e += NT) {
      const int a = e >> 6, jl = e & 63;
      const int64_t j = 64 * jb + jl;
      if (j >= n0) continue;
      double t = 0.0;
      for (int bb = 0; bb <= a; ++bb) t -= Li[a * KINC + bb] * Wh[jl * KINC + bb];
      if constexpr (sizeof(VT) == 4) d.Ff[fblk_off(jb, ld) + (n0 + a - 64 * jb) * 64 + jl] = (float)t;
      else d.F[fblk_off(jb, ld) + (n0 + a - 64 * jb) * 64 + jl] = t;
    }
    if (jb == nwb - 1)
      for (int e = tid; e < k * k; e += NT) {
        const int a = e / k, bb = e % k;
        const int64_t j = n0 + bb, jb2 = j / 64;
        if (bb <= a) {
          if constexpr (sizeof(VT) == 4) d.Ff[fblk_off(jb2, ld) + (n0 + a - 64 * jb2) * 64 + j % 64] = (float)Li[a * KINC + bb];
          else d.F[fblk_off(jb2, ld) + (n0 + a - 64 * jb2) * 64 + j % 64] = Li[a * KINC + bb];
        }
      }
    __syncthreads();   // Wh is reused by the next block
  }
  if (d.lat_g2) tables_share();
}

// Wait (wave 0 polls, the workgroup joins at the barrier) until flags f[0, n)
// all hold the epoch; bounded like wait_flag.
__device__ void wait_flags_all(const GPDesc& d, const unsigned* f, int64_t n, unsigned epoch) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int it = 0;
    while (true) {
      bool mine = true;
      for (int64_t i = lane; i < n; i += 64)
        mine = mine && __hip_atomic_load(f + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
      if (__ballot(!mine) == 0) break;
      __builtin_amdgcn_s_sleep(MFGP_SPIN_SLEEP);
      if (++it == (1 << 22)) {
        if (lane == 0) atomicMin(d.status, SYNC_FAIL);
        break;
      }
    }
  }
  __syncthreads();
}

// Exclusive prefix over the workgroup of NV per-thread counts (in thread order),
// and the totals. scr: 4 * NV ints of LDS.
template <int NV>
__device__ __forceinline__ void block_scan(int (&v)[NV], int (&tot)[NV], int* scr) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int inc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) inc[i] = v[i];
#pragma unroll
  for (int off = 1; off < 64; off <<= 1)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int o = __shfl_up(inc[i], off);
      if (lane >= off) inc[i] += o;
    }
  __syncthreads();   // scr is free
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < NV; ++i) scr[w * NV + i] = inc[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    int before = 0, all = 0;
#pragma unroll
    for (int ww = 0; ww < NT / 64; ++ww) {
      const int x = scr[ww * NV + i];
      before += ww < w ? x : 0;
      all += x;
    }
    v[i] = before + inc[i] - v[i];
    tot[i] = all;
  }
}

// One Z unit: part `part`, lattice y-rows q in [c zq, c zq + zq) (zq = 2 NT /
// tabw), and every virtual (off-lattice) row v of the part with v % units == c.
// Rows j of the part on the lattice at (px, py):
//   Z[part][py][ix][a] = sum_j w[j][a] c_j ex(px, ix)          (axis table ex)
// and a virtual row j: Z[part][zq8 + v][ix][a] = w[j][a] (c_j ex_j(ix)) (its own
// table row). Thread (ql, ix) owns rows q = c zq + ql and c zq + zq / 2 + ql,
// column ix, all a. Rows are scanned in batches of ZR NT in row order (members
// bucketed by row q, stable), so each sum runs in row order. The axis-table
// loads of the first members go out before the wait for w. Ends with the rows
// stored (write-through, drain) and zflag[zu] = epoch.
constexpr int ZR = 8;      // rows per thread per scan batch
template <int KA>
__device__ __forceinline__ void lat_zunit(const GPDesc& d, int64_t zu, double* sm) {
  // members per row q per load batch: at KA = 8, 8 (two batches for the headline's
  // ~16 members per row) rather than 16, whose axis values held 64 VGPRs and made
  // the kernel spill 16 (2 now); the same FMAs in the same order, 0.5-2 % faster
  // (tools/ab_variants.sh zmb8 zmb12, round 4)
#ifndef MFGP_ZST
#define MFGP_ZST 6   // member-list Z units: members staged per row in LDS before the w wait
#endif
#ifndef MFGP_ZMB8
#define MFGP_ZMB8 8
#endif
  constexpr int ZMB = KA == 8 ? MFGP_ZMB8 : 6;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Hyp& h = d.hp;
  const int P = h.kind == 0 ? 1 : 2;
  const int64_t tabw = d.tabw;   // 64, 128 or 256 (host)
  const int ZQ = d.zq;           // 2 NT / tabw (<= 8)
  const int ZH = ZQ / 2;         // rows q per thread group
  const int64_t nu = d.nzu / P;
  const int part = (int)(zu / nu);
  const int64_t c = zu % nu;
  const int64_t ny = d.lat.ny;
  const int64_t n0 = d.n0, NL = d.NL;
  const int64_t j_lo = part == 1 ? NL : 0;
  const int ql = __builtin_amdgcn_readfirstlane((int)(tid / tabw));
  const int64_t ix = tid % tabw;
  const int64_t zq8 = (ny + ZKS - 1) / ZKS * ZKS;
  const int64_t zrows = d.zrows, tstride = d.ld * tabw;
  const unsigned epoch = d.epoch;
  const double* const wv = d.wv;
  const int* const lidx = d.lidx;
  double* const zb = d.zb;
  int* const zvl = d.zvl + part * (zrows + 1);
  const double* const axr = d.axt + (2 * part) * (tabw + 1) * tabw + ix;   // ex(p, ix) at axr[p * tabw]
  const double cL = h.kind == 0 ? h.sL : h.rho * h.sL, cLH = h.rho2 * h.sL;
  auto coef = [&](int64_t j) { return part == 1 ? h.sH : (j < NL ? cL : cLH); };
  // LDS: members [2048] (row), their px [2048], this unit's virtual rows [2048],
  // the waves' coefficient batches [4][2][ZMB][KA], scan scratch
  int* const mrow = reinterpret_cast<int*>(sm);
  int* const mpx = mrow + ZR * NT;
  int* const vrow = mpx + ZR * NT;
  double* const cw = sm + 3 * ZR * NT / 2 + w * 2 * ZMB * KA;
  int* const scr = reinterpret_cast<int*>(sm + 3 * ZR * NT / 2 + 4 * 2 * ZMB * KA);
  static_assert(3 * ZR * NT / 2 + 4 * 2 * ZMB * KA + 24 <= LAT_LDS, "the Z unit's LDS fits");
  WTRACE(0);
  double acc[2][KA];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int a = 0; a < KA; ++a) acc[hh][a] = 0.0;
  int64_t vbase = 0;   // virtual rows of the part before this batch
  bool waited = false;
  auto wait_w = [&]() {
    if (!waited) {
      WTRACE(1);
      wait_flags_all(d, d.wflag, d.nwb, epoch);   // w of every block
      WTRACE(3);
      waited = true;
    }
  };
  for (int64_t b0 = j_lo; b0 < n0; b0 += ZR * NT) {
    // per-thread counts of members of rows c zq + 0..7 (4-bit fields: <= ZR each)
    // and of virtual rows; no dynamically indexed arrays (they would live in scratch)
    int li[ZR];
    unsigned pk = 0;
    int nvirt = 0;
#pragma unroll
    for (int e = 0; e < ZR; ++e) {
      const int64_t j = b0 + (int64_t)tid * ZR + e;
      li[e] = j < n0 ? lidx[j] : -2;
      if (li[e] >= 0) {
        const int64_t b = (int64_t)(li[e] >> 16) - c * ZQ;
        if (b >= 0 && b < ZQ) pk += 1u << (4 * b);
      } else if (li[e] == -1) {
        nvirt += 1;
      }
    }
    int cnt[9], tot[9];
#pragma unroll
    for (int b = 0; b < 8; ++b) cnt[b] = (int)((pk >> (4 * b)) & 15u);
    cnt[8] = nvirt;
    block_scan<9>(cnt, tot, scr);
    int base[8];
    base[0] = 0;
#pragma unroll
    for (int b = 1; b < 8; ++b) base[b] = base[b - 1] + tot[b - 1];
    // this unit's first virtual row at or after vbase
    const int64_t vfirst = vbase + ((c - vbase % nu) % nu + nu) % nu;
    unsigned run = 0;   // members placed so far per bucket (4-bit fields)
    int vrun = 0;
#pragma unroll
    for (int e = 0; e < ZR; ++e) {
      const int64_t j = b0 + (int64_t)tid * ZR + e;
      if (li[e] >= 0) {
        const int64_t b = (int64_t)(li[e] >> 16) - c * ZQ;
        if (b >= 0 && b < ZQ) {
          int pos = 0;
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (i == b) pos = base[i] + cnt[i] + (int)((run >> (4 * i)) & 15u);
          run += 1u << (4 * b);
          mrow[pos] = (int)j;
          mpx[pos] = li[e] & 0xffff;
        }
      } else if (li[e] == -1) {
        const int64_t v = vbase + cnt[8] + vrun++;
        if (v % nu == c) vrow[(v - vfirst) / nu] = (int)j;
      }
    }
    __syncthreads();
    // members of this thread group's two rows, ZMB of each at a time: ex(px, ix)
    // for each (before the first wait for w), the coefficients w[j][a] c_j into the
    // wave's LDS, then the FMAs (row order)
    int lo[2] = {0, 0}, nm_all[2] = {0, 0};
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int b = ql + hh * ZH;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (i == b) {
          lo[hh] = base[i];
          nm_all[hh] = (c * ZQ + b < ny) ? tot[i] : 0;
        }
    }
    const int mmax = nm_all[0] > nm_all[1] ? nm_all[0] : nm_all[1];
    double ex[2][ZMB];
    auto load_ex = [&](int m0) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int m = 0; m < ZMB; ++m)
          ex[hh][m] = m0 + m < nm_all[hh] ? axr[(int64_t)mpx[lo[hh] + m0 + m] * tabw] : 0.0;
    };
    load_ex(0);
    wait_w();   // every wave (a barrier): members or not
    for (int m0 = 0; m0 < mmax; m0 += ZMB) {
      if (m0 > 0) load_ex(m0);
      {
        // all of the batch's coefficient loads in flight, then into LDS
        constexpr int NE = (2 * ZMB * KA + 63) / 64;
        double v[NE];
#pragma unroll
        for (int i = 0; i < NE; ++i) {
          const int e = lane + 64 * i;
          const int hh = e / (ZMB * KA), m = (e / KA) % ZMB, a = e % KA;
          v[i] = 0.0;
          // (selects, not a dynamic index into lo / nm_all: those would live in scratch)
          if (e < 2 * ZMB * KA && m0 + m < (hh ? nm_all[1] : nm_all[0])) {
            const int64_t j = mrow[(hh ? lo[1] : lo[0]) + m0 + m];
            v[i] = ldx<true>(&wv[j * KINC + a]) * coef(j);   // L2-served: stored in this launch
          }
        }
#pragma unroll
        for (int i = 0; i < NE; ++i)
          if (lane + 64 * i < 2 * ZMB * KA) cw[lane + 64 * i] = v[i];
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int m = 0; m < ZMB; ++m)
          if (m0 + m < nm_all[hh]) {
#pragma unroll
            for (int a = 0; a < KA; ++a) acc[hh][a] = __builtin_fma(cw[(hh * ZMB + m) * KA + a], ex[hh][m], acc[hh][a]);
          }
    }
    WTRACE(4);
    // this unit's virtual rows of the batch: Z row = w[j][a] (c_j ex_j(ix)), group ql == 0
    const int64_t nvb = tot[8];
    const int64_t nmine = vfirst < vbase + nvb ? (vbase + nvb - 1 - vfirst) / nu + 1 : 0;
    if (ql == 0)
      for (int64_t i = 0; i < nmine; ++i) {
        const int64_t v = vfirst + i * nu;
        const int64_t j = vrow[i];
        const double e = d.tab[(2 * part) * tstride + j * tabw + ix];
        double* zr = zb + ((part * zrows + zq8 + v) * tabw + ix) * KA;
#pragma unroll
        for (int a = 0; a < KA; ++a) stx<true>(zr + a, ldx<true>(&wv[j * KINC + a]) * e);
        if (ix == 0) __hip_atomic_store(zvl + 1 + v, (int)j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    vbase += nvb;
    __syncthreads();   // the lists are reused by the next batch
  }
  // the part's last virtual stage: rows [nv, round_up(nv, ZKS)) are zero (their
  // table row: the part's first row, any finite row)
  const int64_t nv = vbase, nv8 = (nv + ZKS - 1) / ZKS * ZKS;
  if (ql == 0)
    for (int64_t v = nv + ((c - nv % nu) % nu + nu) % nu; v < nv8; v += nu) {
      double* zr = zb + ((part * zrows + zq8 + v) * tabw + ix) * KA;
#pragma unroll
      for (int a = 0; a < KA; ++a) stx<true>(zr + a, 0.0);
      if (ix == 0) __hip_atomic_store(zvl + 1 + v, (int)j_lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  if (c == 0 && tid == 0) __hip_atomic_store(zvl, (int)nv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  WTRACE(5);
  // the rows through LDS, so that every store instruction writes 512 contiguous
  // bytes (write-through stores of scattered 8-byte pieces cost ~10 us here)
  double* const zst = sm;   // [ZH][tabw][KA] (the lists are dead)
  static_assert(4096 + 16 <= LAT_LDS, "the Z rows' staging fits");
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    __syncthreads();
#pragma unroll
    for (int a = 0; a < KA; ++a) zst[(ql * tabw + ix) * KA + a] = acc[hh][a];
    __syncthreads();
    const int64_t q0 = c * ZQ + hh * ZH;   // rows q0 .. q0 + ZH - 1, contiguous in zb
    const int64_t nrow = ny - q0 < ZH ? ny - q0 : ZH;
    double* const zr = zb + (part * zrows + q0) * tabw * KA;
    if (d.lat_g2) {
      // read by the next launch (k_lat_gemm2): no drain, no flags; written through (16 B
      // a lane), so the launch's end has no dirty Z lines to write back
      for (int64_t e = tid; e < nrow * tabw * KA / 2; e += NT) st16_wt(zr + 2 * e, dv2{zst[2 * e], zst[2 * e + 1]});
    } else {
      for (int64_t e = tid; e < nrow * tabw * KA / 2; e += NT) st16_wt(zr + 2 * e, dv2{zst[2 * e], zst[2 * e + 1]});
    }
  }
  if (d.lat_g2) {
    WTRACE(6);
    WTRACE(2);
    return;
  }
  drain_stores();
  __syncthreads();
  WTRACE(6);
  // this unit's rows are stored (the GEMM stages over them wait for this flag),
  // then the count of all Z units (the virtual stages wait for that)
  if (tid == 0) {
    publish(d.zflag + zu, epoch);
    arrive_phase(d.ldone + 2, epoch, d.nzu);
  }
  WTRACE(2);
}

// A Z unit reading the member lists of the part's scan unit (lat_zcsr: the scan
// units are the launch's first roles, before the producers): its rows' members are
// contiguous in the CSR, so the unit reads only them instead of bucketing every
// row of the part (at configs[4]'s 8,184 rows and 256 units per GP that scan was
// most of the Z phase). The sums, their order and everything after them are
// lat_zunit's: the same bits.
template <int KA>
__device__ __forceinline__ void lat_zunit_csr(const GPDesc& d, int64_t zu, double* sm) {
  constexpr int ZMB = KA == 8 ? MFGP_ZMB8 : 6;   // members per row q per load batch
  const int tid = threadIdx.x;
  const Hyp& h = d.hp;
  const int P = h.kind == 0 ? 1 : 2;
  const int64_t tabw = d.tabw;
  const int ZQ = d.zq;
  const int ZH = ZQ / 2;
  const int64_t nu = d.nzu / P;
  const int part = (int)(zu / nu);
  const int64_t c = zu % nu;
  const int64_t ny = d.lat.ny;
  const int64_t NL = d.NL;
  const int ql = __builtin_amdgcn_readfirstlane((int)(tid / tabw));
  const int64_t ix = tid % tabw;
  const int64_t zq8 = (ny + ZKS - 1) / ZKS * ZKS;
  const int64_t zrows = d.zrows, tstride = d.ld * tabw;
  const unsigned epoch = d.epoch;
  const double* const wv = d.wv;
  double* const zb = d.zb;
  const int* const zvl = d.zvl + part * (zrows + 1);
  const double* const axr = d.axt + (2 * part) * (tabw + 1) * tabw + ix;   // ex(p, ix) at axr[p * tabw]
  const double cL = h.kind == 0 ? h.sL : h.rho * h.sL, cLH = h.rho2 * h.sL;
  auto coef = [&](int64_t j) { return part == 1 ? h.sH : (j < NL ? cL : cLH); };
  // LDS: the unit's members in chunks of ZCH (their rows' lists are contiguous in the
  // CSR): training row j and axis column px, then (after the w wait) the c w rows;
  // then the stash: each row's members ZMB .. ZMB + ZST - 1 of the first chunk, their
  // axis rows ex(px, .) DMA'd before the w wait (MFGP_ZST; tabw a multiple of 128),
  // so that a row of up to ZMB + ZST members loads nothing after the wait
  constexpr int ZST = KA == 8 ? MFGP_ZST : 0;
  constexpr int ZCH = ZST > 0 ? 128 : 256;
  int* const mj = reinterpret_cast<int*>(sm);        // [ZCH]
  int* const mpx = mj + ZCH;                          // [ZCH]
  double* const cws = sm + ZCH;                       // [ZCH][KA]
  double* const stash = cws + ZCH * KA;               // [ZQ rows][ZST][tabw] = [2 NT][ZST]
  static_assert(ZCH + ZCH * KA + 2 * NT * ZST <= LAT_LDS, "the Z unit's LDS fits");
  const bool use_st = ZST > 0 && tabw % 128 == 0 && ZQ * tabw == 2 * NT;
  WTRACE(0);
  // the part's lists (the scan unit was dispatched before any producer)
  wait_flag(d, d.zflag + d.nzu + part, epoch);
  const unsigned* const off = d.csr + (int64_t)part * (tabw + 1 + d.ld);
  const unsigned* const mem = off + tabw + 1;
  auto ldu = [](const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  // the unit's rows c ZQ .. c ZQ + ZQ - 1 (those below ny): members [u_lo, u_hi)
  const int64_t qa = c * ZQ, qb = qa + ZQ < ny ? qa + ZQ : ny;
  const int u_lo = qa < ny ? (int)ldu(off + qa) : 0;
  const int u_hi = qa < ny ? (int)ldu(off + qb) : 0;
  int lo[2] = {0, 0}, nm[2] = {0, 0};   // this thread group's two rows, relative to u_lo
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int64_t q = c * ZQ + ql + hh * ZH;
    if (q < ny) {
      lo[hh] = (int)ldu(off + q) - u_lo;
      nm[hh] = (int)ldu(off + q + 1) - u_lo - lo[hh];
    }
  }
  WTRACE(1);
  double acc[2][KA];
#pragma unroll
  for (int hh = 0; hh < 2; ++hh)
#pragma unroll
    for (int a = 0; a < KA; ++a) acc[hh][a] = 0.0;
  bool waited = false;
  for (int c0 = 0; c0 < u_hi - u_lo; c0 += ZCH) {
    const int cn = u_hi - u_lo - c0 < ZCH ? u_hi - u_lo - c0 : ZCH;
    __syncthreads();   // (the previous chunk is summed)
    for (int e = tid; e < cn; e += NT) {
      const unsigned pk = ldu(mem + u_lo + c0 + e);
      mj[e] = (int)(pk & 0xffffu);
      mpx[e] = (int)(pk >> 16);
    }
    __syncthreads();
    // this thread's members in the chunk, per row: [b0, b1) relative to the chunk
    int b0[2], b1[2];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      b0[hh] = lo[hh] - c0 > 0 ? lo[hh] - c0 : 0;
      const int e1 = lo[hh] + nm[hh] - c0;
      b1[hh] = e1 < cn ? e1 : cn;
      if (b1[hh] < b0[hh]) b1[hh] = b0[hh];
    }
    const int mmax = (b1[0] - b0[0]) > (b1[1] - b0[1]) ? (b1[0] - b0[0]) : (b1[1] - b0[1]);
    double ex[2][ZMB];
    auto load_ex = [&](int m0) {
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int m = 0; m < ZMB; ++m) {
          const int e = b0[hh] + m0 + m;
          ex[hh][m] = e < b1[hh] ? axr[(int64_t)mpx[e] * tabw] : 0.0;
        }
    };
    load_ex(0);
    if (use_st && c0 == 0) {
      // the stash: one LDS-DMA per (row, slot, 128 columns), 16 bytes a lane (the wave
      // takes instructions w, w + 4, ...); no registers held across the wait
      const int NHf = (int)(tabw / 128);
      const int lane = tid & 63, wv4 = tid >> 6;
      const double* const axb = d.axt + (2 * part) * (tabw + 1) * tabw;
      for (int pi = wv4; pi < ZQ * ZST * NHf; pi += NT / 64) {
        const int r = pi / (ZST * NHf), sl = (pi / NHf) % ZST, hf = pi % NHf;
        const int64_t q = qa + r;
        if (q >= ny) continue;
        const int e = (int)ldu(off + q) - u_lo + ZMB + sl;   // the member (chunk 0)
        if (e >= (int)ldu(off + q + 1) - u_lo || e >= cn) continue;
        const double* src = axb + (int64_t)mpx[e] * tabw + hf * 128 + 2 * lane;
        __builtin_amdgcn_global_load_lds((const GLOBAL void*)src, (lds_vptr)(stash + ((int64_t)r * ZST + sl) * tabw + hf * 128),
                                         16, 0, 0);
      }
    }
    if (!waited) {
      wait_flags_all(d, d.wflag, d.nwb, epoch);   // w of every block (every wave: a barrier)
      WTRACE(3);
      waited = true;
    }
    // the chunk's c w rows into LDS, one element per thread at a time (all in flight)
    {
      constexpr int NE = (ZCH * KA + NT - 1) / NT;
      double v[NE];
#pragma unroll
      for (int i2 = 0; i2 < NE; ++i2) {
        const int e = tid + NT * i2, m = e / KA, a = e % KA;
        v[i2] = 0.0;
        if (m < cn) {
          const int64_t j = mj[m];
          v[i2] = ldx<true>(&wv[j * KINC + a]) * coef(j);   // L2-served: stored in this launch
        }
      }
      __syncthreads();   // (every thread has read mj: cws may be written)
#pragma unroll
      for (int i2 = 0; i2 < NE; ++i2)
        if (tid + NT * i2 < ZCH * KA) cws[tid + NT * i2] = v[i2];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the stash's DMAs: every wave's, at the barrier)
      __syncthreads();
    }
    // the members in order: batch 0 (registers), then the stash (ZST), then batches
    // of ZMB from memory -- the same FMAs in the same order as without the stash
    for (int m0 = 0; m0 < mmax;) {
      const bool st = use_st && c0 == 0 && m0 == ZMB;
      if (st) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
#pragma unroll
          for (int m = 0; m < ZMB; ++m)
            ex[hh][m] = m < ZST && b0[hh] + m0 + m < b1[hh] ? stash[((ql + hh * ZH) * ZST + m) * tabw + ix] : 0.0;
      } else if (m0 > 0) {
        load_ex(m0);
      }
      const int mn = st ? ZST : ZMB;
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int m = 0; m < ZMB; ++m) {
          const int e = b0[hh] + m0 + m;
          if (m < mn && e < b1[hh]) {
#pragma unroll
            for (int a = 0; a < KA; ++a) acc[hh][a] = __builtin_fma(cws[e * KA + a], ex[hh][m], acc[hh][a]);
          }
        }
      m0 += mn;
    }
  }
  if (!waited) {
    wait_flags_all(d, d.wflag, d.nwb, epoch);   // (a unit without members still waits: its virtual rows need w)
    WTRACE(3);
  }
  WTRACE(4);
  // this unit's virtual rows (v = c, c + nu, ...; the padding rows up to ZKS: zero):
  // Z row = w[j][a] (c_j ex_j(ix)), group ql == 0
  {
    const int64_t nv = (int64_t)__hip_atomic_load(zvl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t nv8 = (nv + ZKS - 1) / ZKS * ZKS;
    if (ql == 0)
      for (int64_t v = c; v < nv8; v += nu) {
        double* zr = zb + ((part * zrows + zq8 + v) * tabw + ix) * KA;
        if (v < nv) {
          const int64_t j = __hip_atomic_load(zvl + 1 + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const double e = d.tab[(2 * part) * tstride + j * tabw + ix];
#pragma unroll
          for (int a = 0; a < KA; ++a) stx<true>(zr + a, ldx<true>(&wv[j * KINC + a]) * e);
        } else {
#pragma unroll
          for (int a = 0; a < KA; ++a) stx<true>(zr + a, 0.0);
        }
      }
  }
  WTRACE(5);
  // the rows through LDS (512 contiguous bytes per store), as lat_zunit
  double* const zst = sm;   // [ZH][tabw][KA]
  static_assert(4096 + 16 <= LAT_LDS, "the Z rows' staging fits");
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    __syncthreads();
#pragma unroll
    for (int a = 0; a < KA; ++a) zst[(ql * tabw + ix) * KA + a] = acc[hh][a];
    __syncthreads();
    const int64_t q0 = c * ZQ + hh * ZH;
    const int64_t nrow = ny - q0 < ZH ? ny - q0 : ZH;
    double* const zr = zb + (part * zrows + q0) * tabw * KA;
    if (d.lat_g2) {
      for (int64_t e = tid; e < nrow * tabw * KA / 2; e += NT) st16_wt(zr + 2 * e, dv2{zst[2 * e], zst[2 * e + 1]});
    } else {
      for (int64_t e = tid; e < nrow * tabw * KA / 2; e += NT) st16_wt(zr + 2 * e, dv2{zst[2 * e], zst[2 * e + 1]});
    }
  }
  if (d.lat_g2) {
    WTRACE(6);
    WTRACE(2);
    return;
  }
  drain_stores();
  __syncthreads();
  WTRACE(6);
  if (tid == 0) {
    publish(d.zflag + zu, epoch);
    arrive_phase(d.ldone + 2, epoch, d.nzu);
  }
  WTRACE(2);
}

// The scan unit of a part (lat_zcsr: the launch's first roles): lists the part's
// training rows j < n0 on the lattice by lattice y-row q, in row order within each
// q -- the order in which a Z unit sums them -- as CSR in d.csr (offsets [ny + 1],
// then the members (px << 16) | j), and its off-lattice ("virtual") rows in row
// order in zvl (count, rows, padded to ZKS with the part's first row) as the Z units
// list them. Nothing here needs w: the units finish while the w units stream F. A stable counting
// sort: the buckets' sizes (LDS atomics), their offsets (a wave scan), then the
// rows in chunks of NT in row order, each row's place = its bucket's running
// offset + the same bucket's rows in the chunk's earlier waves + its rank among
// its wave's lanes of that bucket (nine ballots). Write-through stores: the Z units
// of the same launch read the lists.
constexpr int SCAN_B = 264;   // buckets held: ny <= 256 lattice rows + the virtual one
// (flag: where the unit publishes that its lists are stored; every output is stored
// write-through, so the Z units of this launch may read them after the flag)
__device__ __forceinline__ void lat_scan(const GPDesc& d, int part, double* sm, unsigned* flag) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int64_t j_lo = part == 1 ? d.NL : 0;
  const int n = (int)(d.n0 - j_lo);
  const int ny = d.lat.ny;            // <= 256 (the host's bound)
  int* const run = reinterpret_cast<int*>(sm);  // [SCAN_B] the buckets' next places
  int* const wc = run + SCAN_B;                 // [NT / 64][SCAN_B] this chunk's counts
  int* const vbase = wc + (NT / 64) * SCAN_B;   // the virtual bucket's first place
  static_assert(((1 + NT / 64) * SCAN_B + 2) / 2 <= LAT_LDS, "the scan unit's LDS fits");
  const int* const lidx = d.lidx + j_lo;
  auto bucket = [&](int li) { return li >= 0 ? (li >> 16) : ny; };
  for (int b = tid; b < (1 + NT / 64) * SCAN_B; b += NT) run[b] = 0;
  __syncthreads();
  constexpr int SU = 8;   // rows loaded ahead per thread
  for (int e0 = 0; e0 < n; e0 += SU * NT) {
    int li[SU];
#pragma unroll
    for (int u = 0; u < SU; ++u) {
      const int e = e0 + u * NT + tid;
      li[u] = e < n ? lidx[e] : -2;
    }
#pragma unroll
    for (int u = 0; u < SU; ++u)
      if (li[u] != -2) __hip_atomic_fetch_add(run + bucket(li[u]), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __syncthreads();
  unsigned* const off = d.csr + (int64_t)part * (d.tabw + 1 + d.ld);
  unsigned* const mem = off + d.tabw + 1;
  auto st_u = [](unsigned* p, unsigned v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto st_i = [](int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  if (wv == 0) {   // exclusive offsets of buckets 0 .. ny (ny: the virtual rows)
    int base = 0;
    for (int s0 = 0; s0 <= ny; s0 += 64) {
      const int b = s0 + lane;
      const int v = b <= ny ? run[b] : 0;
      int x = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
      }
      if (b <= ny) {
        run[b] = base + x - v;
        st_u(off + b, (unsigned)(base + x - v));
        if (b == ny) *vbase = base + x - v;
      }
      base += __shfl(x, 63);
    }
  }
  __syncthreads();
  int* const zvl = d.zvl + (int64_t)part * (d.zrows + 1);
  const int vb = *vbase;
  for (int c0 = 0; c0 < n; c0 += NT) {
    const int e = c0 + tid;
    const bool valid = e < n;
    const int li = valid ? lidx[e] : 0;
    const int b = bucket(li);
    unsigned long long mask = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 9; ++bit) {
      const unsigned long long bb = __ballot((b >> bit) & 1);
      mask &= ((b >> bit) & 1) ? bb : ~bb;
    }
    const int rank = __popcll(mask & ((1ull << lane) - 1ull));
    if (valid && rank == 0) wc[wv * SCAN_B + b] = __popcll(mask);
    __syncthreads();
    if (valid) {
      int pos = run[b] + rank;
      for (int w2 = 0; w2 < wv; ++w2) pos += wc[w2 * SCAN_B + b];
      const int j = (int)j_lo + e;
      if (b < ny) st_u(mem + pos, ((unsigned)(li & 0xffff) << 16) | (unsigned)j);
      else st_i(zvl + 1 + pos - vb, j);
    }
    __syncthreads();
    for (int bb = tid; bb <= ny; bb += NT) {
      int t = 0;
#pragma unroll
      for (int w2 = 0; w2 < NT / 64; ++w2) {
        t += wc[w2 * SCAN_B + bb];
        wc[w2 * SCAN_B + bb] = 0;
      }
      run[bb] += t;
    }
    __syncthreads();
  }
  const int nv = n - vb, nv8 = (nv + ZKS - 1) / ZKS * ZKS;
  for (int v = nv + tid; v < nv8; v += NT) st_i(zvl + 1 + v, (int)j_lo);
  if (tid == 0) st_i(zvl, nv);
  drain_stores();
  __syncthreads();
  if (tid == 0) publish(flag, d.epoch);   // the lists and places are stored
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

// acc += A B over one stage of ZKS = 8 K rows: A[(a, ix)][k] = Z rows (As, [8][128],
// swizzled by (k & 1) << 4), B[k][iy] = axis-table / table rows (Bs, [8][64], swz).
// Wave w: rows 32 w + 16 m + r (m = 0, 1), all 64 columns: per 4-row k-step 6 LDS
// reads and 8 MFMAs, the reads of both k-steps ahead of the MFMAs.
__device__ __forceinline__ void lat_zcompute(const double* slot, d4 (&acc)[2][4], int w, int r, int q) {
  const double* As = slot;
  const double* Bs = slot + ZKS * 128;
  double a[2][2], b[2][4];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int k = 4 * e + q;
#pragma unroll
    for (int m = 0; m < 2; ++m) a[e][m] = As[k * 128 + ((32 * w + 16 * m + r) ^ ((k & 1) << 4))];
#pragma unroll
    for (int n = 0; n < 4; ++n) b[e][n] = Bs[swz(k, 16 * n + r)];
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead of the MFMAs
#pragma unroll
  for (int e = 0; e < 2; ++e) {
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      acc[0][n] = mfma(a[e][0], b[e][n], acc[0][n]);
      acc[1][n] = mfma(a[e][1], b[e][n], acc[1][n]);
    }
  }
}

// The sum of SS split-K partials (in split order) of the accumulator blocks
// (m, nf + nb): all SS x NBE d4 loads in flight at once (L2-served: the splits
// stored them in this launch). NBE = 1: only block nf + half (the other is zero).
template <int SS, int NBP, int NBE>
__device__ __forceinline__ void lat_psum(const double* p0, int m, int nf, int half, d4 (&tv)[NBP]) {
  d4 x[SS][NBE];
#pragma unroll
  for (int s2 = 0; s2 < SS; ++s2)
#pragma unroll
    for (int e = 0; e < NBE; ++e) {
      const int n = nf + (NBE == NBP ? e : half);
#pragma unroll
      for (int v = 0; v < 4; ++v) x[s2][e][v] = ldx<true>(p0 + s2 * LAT_PART + ((m * 4 + n) * 4 + v) * 64);
    }
#pragma unroll
  for (int e = 0; e < NBE; ++e) {
    d4 t = x[0][e];
#pragma unroll
    for (int s2 = 1; s2 < SS; ++s2) t = t + x[s2][e];
    if constexpr (NBE == NBP) {
      tv[e] = t;
    } else {
#pragma unroll
      for (int nb = 0; nb < NBP; ++nb) tv[nb] = nb == half ? t : d4{0.0, 0.0, 0.0, 0.0};
    }
  }
}

// The epilogue's inputs of GEMM tile `tile`: the L22 record and the new rows'
// separable tables for the tile's cells (L2-served loads: both were written in
// this launch, before the L22 flag that the tile saw at its start). The GEMM
// issues them before it stores its split-K partial, so that they arrive while
// the tile's splits meet.
template <int KA>
struct LatEpiIn {
  static constexpr int IXPT = 128 / KA;
  static constexpr int FW = IXPT + 64;
  static constexpr int NR = (KINC * KINC + KINC + NT - 1) / NT;
  static constexpr int NF = (2 * KA * FW + NT - 1) / NT;
  double rv[NR], fv[NF];
};
template <int KA>
__device__ __forceinline__ void lat_epi_load(const GPDesc& d, int64_t tile, LatEpiIn<KA>& in) {
  using E = LatEpiIn<KA>;
  const int tid = threadIdx.x;
  const int64_t ntiy = (d.lat.ny + 63) / 64;
  const int64_t ix0 = (tile / ntiy) * E::IXPT, iy0 = (tile % ntiy) * 64;
  const int64_t n0 = d.n0;
  const int k = (int)(d.N - n0);
#pragma unroll
  for (int i = 0; i < E::NR; ++i) {
    const int e = tid + NT * i;
    in.rv[i] = e < KINC * KINC + KINC ? ldx<true>(d.l22r + e) : 0.0;
  }
  const int64_t tstride = d.ld * d.tabw, tabw = d.tabw;
#pragma unroll
  for (int i = 0; i < E::NF; ++i) {
    const int e = tid + NT * i;
    const int kind2 = e / (KA * E::FW), rem = e % (KA * E::FW);
    const int a = rem / E::FW, col = rem % E::FW;
    const bool isx = col < E::IXPT;
    const int t = 2 * kind2 + (isx ? 0 : 1);
    const int64_t idx = isx ? ix0 + col : iy0 + (col - E::IXPT);
    in.fv[i] = (e < 2 * KA * E::FW && a < k) ? ldx<true>(&d.tab[t * tstride + (n0 + a) * tabw + idx]) : 0.0;
  }
}

// The cells of GEMM tile `tile` (the share of split s of S, DESIGN.md section
// 2.4): T = psi_new - T~ from the accumulators (SPLIT = false, S = 1) or from the
// splits' stored partials (SPLIT = true; the caller waited until all are stored),
// v_new = L22^-1 T, var = var_old - |v_new|^2, mu = mu_old + v_new^T z2, the new V
// rows, and the fused var max / argmax. A separate function per SPLIT, so that the
// accumulators are dead here once a split has stored them.
template <int KA, class VT, bool SPLIT>
__device__ __forceinline__ void lat_epi(const GPDesc& d, int64_t tile, int64_t s, double* sm, const d4 (&acc)[2][4],
                                        const LatEpiIn<KA>& in) {
  constexpr int IXPT = 128 / KA;   // lattice columns x per tile
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 15, q = lane >> 4;
  const GridLattice lat = d.lat;
  const int64_t ntiy = (lat.ny + 63) / 64;
  const int64_t tix = tile / ntiy, tiy = tile % ntiy;
  const int S = d.ksplit;
  const int64_t ix0 = tix * IXPT, iy0 = tiy * 64;
  const unsigned epoch = d.epoch;
  const int64_t n0 = d.n0;
  const int k = (int)(d.N - n0);
  const int64_t tiles = d.lat_tiles;
  const double* p0 = d.gpart + tile * S * LAT_PART + (int64_t)w * 32 * 64 + lane;
  (void)epoch;
  WTRACE(3);
  // ---- epilogue (LDS: the ring is dead) ----
  constexpr int FW = IXPT + 64;
  constexpr int NBP = KA == 8 ? 2 : 1;      // 16-column blocks per cell pass
  constexpr int TW = 16 * NBP;              // Ts row width
  constexpr int NPASS = 2 * (4 / NBP);      // cell passes of the whole tile
  double* const L22 = sm;                   // [16][16] | z2 [16]
  double* const Li = L22 + KINC * KINC + KINC;   // L22^-1 [16][16]
  // psi(cell, new row a) = c_L exL[a][ix] eyL[a][iy] + c_H exH[a][ix] eyH[a][iy]:
  // the new rows' separable tables (written through by the w units before their
  // w halves counted in) for the tile's IXPT x 64 cells, [2 kinds][KA][IXPT | 64]
  double* const Fn = Li + KINC * KINC;
  double* const Ts = Fn + 2 * KA * FW;      // one cell pass of T: [4 waves][16 rows][TW]
  double* const amx = Ts + 4 * 16 * TW;     // the waves' (max, argmax) of var
  static_assert(KINC * KINC + KINC + KINC * KINC + 2 * 8 * (16 + 64) + 4 * 16 * 32 + 8 <= LAT_LDS &&
                    KINC * KINC + KINC + KINC * KINC + 2 * 16 * (8 + 64) + 4 * 16 * 16 + 8 <= LAT_LDS,
                "the epilogue's LDS fits the ring's");
  // this split's share: passes p = s, s + S, ... (S <= NPASS), or half of pass
  // s / 2 (S = 2 NPASS: one of the pass's two 16-column blocks, KA = 8)
  const int npass_mine = S <= NPASS ? (int)((NPASS - 1 - s) / S + 1) : 1;
  const int half = S <= NPASS ? -1 : (int)(s & 1);
  auto pass_of = [&](int i) { return S <= NPASS ? (int)(s + (int64_t)i * S) : (int)(s >> 1); };
  const GridLattice latc = lat;
  const int cw = tid >> 6, cl = tid & 63;
  const int ch = KA == 8 ? cl >> 5 : 0;
  const int cyl = KA == 8 ? cl & 31 : cl & 15;
  // (half >= 0: only the cells of 16-column block `half` of the pass, cyl >> 4)
  const bool cact = (KA == 8 || cl < 16) && (half < 0 || (cyl >> 4) == half);
  auto cell_of = [&](int p, int64_t& ix, int64_t& iy) {
    const int m = p / (4 / NBP), nf = NBP * (p % (4 / NBP));
    ix = ix0 + (KA == 8 ? 4 * cw + 2 * m + ch : 2 * cw + m);
    iy = iy0 + 16 * nf + cyl;
  };
  auto cell_ok = [&](int64_t ix, int64_t iy) { return cact && ix < latc.nx && iy < latc.ny; };
  const double* const rmu_in = d.rmu_in;
  const double* const rvar_in = d.rvar_in;
  // the old posterior of this thread's cell in each of its passes (resident
  // from the previous step: plain loads)
  // (S = 1: the first pass's only; the passes prefetch one ahead, registers are short)
  // (S > 1: each pass loads its cell's with its partials, in one round trip)
  double ov0 = 0.0, om0 = 0.0;
  if constexpr (!SPLIT) {
    int64_t ix, iy;
    cell_of(0, ix, iy);
    if (cell_ok(ix, iy)) {
      const int64_t c = ix * latc.sx + iy * latc.sy;
      ov0 = rvar_in[c];
      om0 = rmu_in[c];
    }
  }
  {
    // the record and the new rows' tables (lat_epi_load, issued by the caller)
    using E = LatEpiIn<KA>;
    constexpr int NR = E::NR, NF = E::NF;
    const double(&rv)[NR] = in.rv;
    const double(&fv)[NF] = in.fv;
    __syncthreads();   // the ring's last reads are done
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int e = tid + NT * i;
      const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
      if (e < KINC * KINC + KINC) L22[e] = use ? rv[i] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < NF; ++i)
      if (tid + NT * i < 2 * KA * FW) Fn[tid + NT * i] = fv[i];
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
  // ---- cells: per pass (m, group of NBP column blocks) the waves put their
  // blocks' T into Ts (row rho = g + 4 v of block (m, n) is, for KA = 8, lattice
  // column h = rho / 8 of the wave's pair and new row a = rho % 8; for KA = 16 new
  // row a = rho), then thread tid finishes one cell: source wave cw = tid / 64,
  // (h, column) from the rest. ----
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  VT* const Vr = const_cast<VT*>(vres_ptr<VT>(d));
  const int64_t vld = d.vld;
  double* const omu = d.mu;
  double* const ovar = d.var;
  double* const rmu = d.rmu;
  double* const rvar = d.rvar;
  // one pass: T of blocks (m, nf .. nf + NBP) into Ts, then this thread's cell
  auto do_pass = [&](int p, const d4 (&tv)[NBP], double cov, double com) {
    int64_t ix, iy;
    cell_of(p, ix, iy);
    const bool ok = cell_ok(ix, iy);
    const int64_t c = ix * latc.sx + iy * latc.sy;
    __syncthreads();   // the previous pass's Ts reads (and Li) are done
#pragma unroll
    for (int nb = 0; nb < NBP; ++nb)
#pragma unroll
      for (int v = 0; v < 4; ++v) Ts[(w * 16 + q + 4 * v) * TW + 16 * nb + r] = tv[nb][v];
    __syncthreads();
    if (!ok) return;
    const int ixc = (int)(ix - ix0), iyc = IXPT + (int)(iy - iy0);
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
  };
  if constexpr (!SPLIT) {
    // every pass is this workgroup's; T is in the accumulators (compile-time blocks)
    double ov = ov0, om = om0;
#pragma unroll
    for (int i = 0; i < NPASS; ++i) {
      const int m = i / (4 / NBP), nf = NBP * (i % (4 / NBP));
      d4 tv[NBP];
#pragma unroll
      for (int nb = 0; nb < NBP; ++nb) tv[nb] = acc[m][nf + nb];
      const double cov = ov, com = om;
      if (i + 1 < NPASS) {
        int64_t ix, iy;
        cell_of(i + 1, ix, iy);
        if (cell_ok(ix, iy)) {
          const int64_t c = ix * latc.sx + iy * latc.sy;
          ov = rvar_in[c];
          om = rmu_in[c];
        }
      }
      do_pass(i, tv, cov, com);
    }
  } else {
    for (int i = 0; i < npass_mine; ++i) {
      const int p = pass_of(i);
      const int m = p / (4 / NBP), nf = NBP * (p % (4 / NBP));
      double cov = 0.0, com = 0.0;
      {
        int64_t ix, iy;
        cell_of(p, ix, iy);
        if (cell_ok(ix, iy)) {
          const int64_t c = ix * latc.sx + iy * latc.sy;
          cov = rvar_in[c];
          com = rmu_in[c];
        }
      }
      // the splits' partials of blocks (m, nf .. nf + NBP), added in split order
      d4 tv[NBP];
      if (S == 2) lat_psum<2, NBP, NBP>(p0, m, nf, half, tv);
      else if (S == 4) lat_psum<4, NBP, NBP>(p0, m, nf, half, tv);
      else lat_psum<8, NBP, (NBP == 2 ? 1 : NBP)>(p0, m, nf, half, tv);
      do_pass(p, tv, cov, com);
    }
  }
  WTRACE(6);
  if (d.vmax || d.vargmax || d.status_host) {
    // the waves' (max, argmax) meet in LDS; wave 0 counts the workgroup in
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) argmax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
    int64_t* const ami = reinterpret_cast<int64_t*>(amx);
    if (lane == 0) {
      amx[2 * w] = bv;
      ami[2 * w + 1] = bi;
    }
    __syncthreads();
    if (w == 0) {
      bv = amx[0];
      bi = ami[1];
#pragma unroll
      for (int ww = 1; ww < 4; ++ww) argmax_pair(bv, bi, amx[2 * ww], ami[2 * ww + 1]);
      var_argmax_group(d, bv, bi, tile * S + s, tiles * S);
    }
  }
  WTRACE(4);
}

// One GEMM tile (split s of ksplit): 128 (a, ix) rows x 64 iy columns, i.e.
// (128 / KA) x 64 cells, over the K rows of both parts: first every part's
// lattice y-rows q < round_up(ny, ZKS) (A = Z rows, B = axis-table rows ey(q,
// iy)), then every part's virtual rows (A = Z rows, B = the row's own table row
// ey_j(iy)). Split s takes stages s, s + S, ... of each of the two lists. A wave
// waits, before its DMA of an axis stage, only for the Z unit that stores its two
// rows of it (zflag), so the K loop starts on the first Z units' rows while the
// others are still at work; the virtual stages (rows of every Z unit) wait for
// all of Z.
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
  const int64_t tabw = d.tabw, zrows = d.zrows, tstride = d.ld * tabw;
  const int64_t ix0 = tix * IXPT, iy0 = tiy * 64;
  const int P = d.hp.kind == 0 ? 1 : 2;
  const int64_t zq8 = (lat.ny + ZKS - 1) / ZKS * ZKS;
  const int ZQ = d.zq;
  const int64_t nu = d.nzu / P;   // Z units per part
  const unsigned epoch = d.epoch;
  const int* const zvl = d.zvl;
  WTRACE(0);
  // the L22 record (raised by the finish long before: the tile waits for Z units
  // and w anyway), so that the epilogue's loads can go out with the K loop's end
  wait_flag(d, d.sync + 2, epoch);
  const __amdgpu_buffer_rsrc_t rZ = make_rsrc(d.zb, (int64_t)8 * P * zrows * tabw * KA);
  const __amdgpu_buffer_rsrc_t rAx = make_rsrc(d.axt, (int64_t)8 * 4 * (tabw + 1) * tabw);
  const __amdgpu_buffer_rsrc_t rTab = make_rsrc(d.tab, (int64_t)8 * 4 * tstride);
  // lane byte offsets: A rows 2 w + h (swizzle by row parity h), B row pair w
  const unsigned vA0 = (unsigned)(8 * (2 * lane)), vA1 = (unsigned)(8 * ((2 * lane) ^ 16));
  const unsigned vBc = (unsigned)(8 * (((lane & 31) * 2) ^ ((lane >> 5) << 4)));
  const unsigned vB = vBc + (unsigned)(8 * (lane >> 5) * tabw);
  // stage lists: NA axis stages (part-major), then the virtual stages of part 0
  // and of part 1 (nv8[pt] / ZKS each, known once all of Z is stored)
  const int64_t npa = zq8 / ZKS, NA = P * npa;
  int64_t nvs[2] = {0, 0};
  auto issue = [&](int64_t g, bool virt, int64_t slot_t) {   // stage g's DMAs: 3 per wave
    int pt;
    int64_t q0;
    if (!virt) {
      pt = g < npa ? 0 : 1;
      q0 = (g - pt * npa) * ZKS;
      // the Z unit that stores this wave's rows q0 + 2 w, + 1 (padding rows past
      // ny: nobody's; zero since allocation)
      const int64_t zc = (q0 + 2 * w) / ZQ;
      if (zc < nu) spin_wave(d, d.zflag + pt * nu + zc, epoch);
    } else {
      pt = g < nvs[0] ? 0 : 1;
      q0 = zq8 + (g - (pt ? nvs[0] : 0)) * ZKS;
    }
    double* slot = sm + (slot_t % LNST) * LSTG;
    const int64_t ar = (pt * zrows + q0 + 2 * w) * tabw + ix0;
    // the Z rows were stored in this launch: L2-served (sc1) DMA loads
    dma_buf_sc1(rZ, slot + (2 * w) * 128, vA0, (unsigned)(8 * ar * KA));
    dma_buf_sc1(rZ, slot + (2 * w + 1) * 128, vA1, (unsigned)(8 * (ar + tabw) * KA));
    double* bdst = slot + ZKS * 128 + 2 * w * 64;
    if (!virt) {
      dma_buf(rAx, bdst, vB, (unsigned)(8 * (((2 * pt + 1) * (tabw + 1) + q0 + 2 * w) * tabw + iy0)));
    } else {
      // virtual rows: each half-wave its own training row's table row
      const int* vl = zvl + pt * (zrows + 1) + 1 + (q0 - zq8) + 2 * w;
      const int64_t ja = __hip_atomic_load(vl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t jb = __hip_atomic_load(vl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned vv = vBc + (unsigned)(8 * ((lane >> 5) ? jb : ja) * tabw);
      dma_buf(rTab, bdst, vv, (unsigned)(8 * ((2 * pt + 1) * tstride + iy0)));
    }
  };
  d4 acc[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = d4{0.0, 0.0, 0.0, 0.0};
  constexpr int D = LNST - 1;   // stages in flight ahead of the one consumed
  constexpr int CNT = 3;        // vector-memory ops per issued stage (every wave)
  static_assert(D * CNT <= 12, "vm_wait_bar covers the outstanding ops");
  // one pipelined pass over this split's stages of a list (stage t: list index
  // s + t S); the ring slot runs on across the two passes
  int64_t slot0 = 0;
  auto pass = [&](int64_t nlist, bool virt) {
    const int64_t hi = s < nlist ? (nlist - s + S - 1) / S : 0;
    for (int64_t t = 0; t < D && t < hi; ++t) issue(s + t * S, virt, slot0 + t);
    if (!virt) WTRACE(1);   // the first stages' Z units seen
    for (int64_t t = 0; t < hi; ++t) {
      const int64_t after = (hi - 1 - t) < (D - 1) ? (hi - 1 - t) : (D - 1);
      vm_wait_bar((int)after * CNT);
      lat_zcompute(sm + ((slot0 + t) % LNST) * LSTG, acc, w, r, q);
      // the next DMA after this stage's MFMAs: its wait for a Z unit never holds
      // up a stage that is already here
      if (t + D < hi) issue(s + (t + D) * S, virt, slot0 + t + D);
    }
    slot0 += hi;
  };
  pass(NA, false);
  // the virtual stages: every Z unit of the GP stored its rows and counts
  wait_phase(d, d.ldone + 2, epoch);
  for (int pt = 0; pt < P; ++pt) {
    const int64_t nv = __hip_atomic_load(zvl + pt * (zrows + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    nvs[pt] = (nv + ZKS - 1) / ZKS;
  }
  if (nvs[0] + nvs[1] > 0) {
    __syncthreads();   // the ring's last reads of the axis pass are done
    pass(nvs[0] + nvs[1], true);
  }
  vm_wait_all();
  __syncthreads();
  WTRACE(2);
  // the epilogue's inputs: in flight with the split-K partial's stores and the
  // splits' meeting (issued behind the stores: the accumulators are then free)
  LatEpiIn<KA> ein;
  // ---- split-K: every split stores its partial; the tile's splits meet (the
  // last to arrive raises the tile's flag), then split s sums the partials of
  // ITS share of the tile in split order ((p0 + p1) + p2 ...: the same bits
  // whichever split computes them) and finishes those cells. The splits of a
  // tile wait only for each other: the host keeps every GEMM workgroup of the
  // launch resident together (tiles x S <= the chip's slots) when S > 1.
  const int64_t tiles = d.lat_tiles;
  if (S > 1) {
    double* part = d.gpart + (tile * S + s) * LAT_PART + (int64_t)w * 32 * 64 + lane;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int v = 0; v < 4; ++v) stx<true>(part + ((m * 4 + n) * 4 + v) * 64, acc[m][n][v]);
    lat_epi_load<KA>(d, tile, ein);
    drain_stores();
    __syncthreads();
    if (tid == 0) {
      unsigned* const cnt = d.gcnt + tile;
      const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == (unsigned)(S - 1)) {
        __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        publish(d.gcnt + tiles + tile, epoch);
      }
    }
    wait_flag(d, d.gcnt + tiles + tile, epoch);   // every split's partial is stored
  } else {
    lat_epi_load<KA>(d, tile, ein);
  }
  if (S > 1) lat_epi<KA, VT, true>(d, tile, s, sm, acc, ein);
  else lat_epi<KA, VT, false>(d, tile, s, sm, acc, ein);
}

// G1: the GEMM tiles are roles of this launch (the one-launch form, MFGP_LAT_GEMM2=0);
// without them (the default, k_lat_gemm2 follows) the kernel carries no GEMM code,
// which cuts its spilled VGPRs from 58 to 16 (KA = 8)
template <int KA, class VT, bool G1>
__device__ __forceinline__ void inc_lat_wg(const GPDesc& d) {
  const int k = (int)(d.N - d.n0);
  if (k <= 0 || k > KINC) return;   // the host guarantees 0 < k <= KINC
  if (d.gate && *d.gate == 0) return;
  // ONE LDS object for every role: a second __shared__ variable would make the
  // compiler's waitcnt pass treat every LDS read as aliasing the ring's LDS-DMA
  // writes and drain vmcnt before it (no pipelining)
  __shared__ double sm[LAT_LDS + 16];
  const int64_t np = d.nprod;
  int64_t role = blockIdx.y;
  if (d.lat_zcsr) {
    // the scan units first (they wait for nothing), then the usual roles
    const int P = d.hp.kind == 0 ? 1 : 2;
    if (role < P) {
      lat_scan(d, (int)role, sm, d.zflag + d.nzu + role);
      return;
    }
    role -= P;
  }
  if (role < np) {
    WTRACE(0);
    inc_producer_role<VT>(d, role, sm, reinterpret_cast<int*>(sm + LAT_LDS),
                          *reinterpret_cast<unsigned*>(sm + LAT_LDS + 8));
    return;
  }
  if (role < np + d.nwu) {
    lat_wblock<KA, VT>(d, role - np, sm);
    return;
  }
  if (role < np + d.nwu + d.nzu) {
    // (the member-list form at KA = 8 only: at 16 its registers spilled the kernel)
    if constexpr (KA == 8) {
      if (d.lat_zcsr) lat_zunit_csr<KA>(d, role - np - d.nwu, sm);
      else lat_zunit<KA>(d, role - np - d.nwu, sm);
    } else {
      lat_zunit<KA>(d, role - np - d.nwu, sm);
    }
    return;
  }
  if constexpr (G1) {
    const int64_t g = role - np - d.nwu - d.nzu;
    if (d.lat_g2 || g >= (int64_t)d.lat_tiles * d.ksplit) return;
    const int64_t tile = g % d.lat_tiles, s = g / d.lat_tiles;
    lat_gemm<KA, VT>(d, tile, s, sm);
  }
}

// KA = 8 (appends of k <= 8 rows) or 16 (k <= 16): one kernel each, so each
// carries only its own epilogue's registers. Four workgroups per CU (<= 128
// VGPRs, LAT_LDS): the roles' dispatch-order argument and the split-K tiles'
// co-residency (tiles x S <= 2 per CU) rest on it (tests/test_codeobj.py).
// MFGP_LAT_WAVES: a diagnostic override (8: a forced-spill build for that test).
#ifndef MFGP_LAT_WAVES
#define MFGP_LAT_WAVES MFGP_INC_WAVES
#endif
template <int KA, class VT, bool G1>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_LAT_WAVES, MFGP_LAT_WAVES))) void k_inc_lat(
    const GPDesc* __restrict__ descs) {
  inc_lat_wg<KA, VT, G1>(descs[blockIdx.x]);
}

// The same step with the batch's descriptors as a by-value kernel argument (up
// to DESC_ARG_MAX of them, 9 KB): a step that needs no other kernel takes no
// per-step upload of its descriptor array. That upload is a host-to-device copy
// on the copy engine, and its hand-off back to the compute queue put ~16 us of
// idle stream time between consecutive steps (kernel trace: k_inc_lat ->
// k_inc_lat gaps of 21 us under rocprofv3).
template <int KA, class VT, bool G1>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(MFGP_LAT_WAVES, MFGP_LAT_WAVES))) void k_inc_lat_arg(
    const DescArg a) {
  // index the kernarg segment itself: a dynamic index into the by-value argument
  // would copy all 9 KB of it to scratch
  (void)a;
  const GPDesc* descs = (const GPDesc*)__builtin_amdgcn_kernarg_segment_ptr();
  inc_lat_wg<KA, VT, G1>(descs[blockIdx.x]);
}

// ---------------------------------------------------------------------------
// The lattice step's GEMM and cells as a second launch (k_lat_gemm2, the default):
// one 1024-thread workgroup per 64 (a, ix) x 64 iy tile, its K rows split four
// ways over four groups of four waves -- split s takes the stages s, s + 4, ... of
// each list, the order of the in-launch split-K at S = 4 -- and the splits' sums
// meeting in LDS in split order, ((p0 + p1) + p2) + p3, then one cell per thread.
// So no split-K partial goes through memory (64 KB stored and re-read per split
// tile in the one-launch form: 66 MB per step at B = 8) and no hand-off flag is
// polled: the kernel boundary orders the Z rows, the L22 record, the new rows'
// tables and w after the first launch (producers, w units, Z units).
// Measured at the headline (B = 8, per-workgroup traces, tools/trace_lat.py): the
// one-launch form ended at 99-104 us, ~40 us after its last Z unit (K loop under
// the Z units' flags, the split-K meeting through memory, the cells); the two
// launches end at ~80 us: the first at ~58, this one ~2 us later and ~20 us long
// (K loop ~16 us, the splits' meeting ~1.5, the cells ~2).
// ---------------------------------------------------------------------------
constexpr int G2S = 4;                          // K splits per workgroup
constexpr int G2NT = 64 * 4 * G2S;              // threads per workgroup
constexpr int G2R = 64;                         // (a, ix) rows per tile
constexpr int G2STG = ZKS * G2R + ZKS * 64;     // doubles per stage: A [8][64] | B [8][64]
#ifndef MFGP_G2NST
#define MFGP_G2NST 4
#endif
constexpr int G2NST = MFGP_G2NST;               // stages in each split's ring
constexpr int G2RING = G2S * G2NST * G2STG;     // the four rings
constexpr int G2PARTS = (G2S - 1) * G2R * 64;  // splits 1..3's sums [3][64][64] (in the rings' place)
static_assert(G2PARTS <= G2RING, "splits 1..3's sums fit the rings' place");
constexpr int G2EPI = KINC * KINC + KINC + KINC * KINC + 2 * 16 * (4 + 64) + 2 * 16;
constexpr int G2LDS = G2RING + G2EPI;           // 149 KB
static_assert(2 * 8 * (8 + 64) <= 2 * 16 * (4 + 64), "both KA's tables fit");

template <int KA, class VT>
__device__ __forceinline__ void lat_gemm2(const GPDesc& d, int64_t tile) {
  constexpr int IXPT = G2R / KA;   // lattice columns x per tile
  constexpr int FW = IXPT + 64;
  const int k = (int)(d.N - d.n0);
  if (k <= 0 || k > KINC) return;
  if (d.gate && *d.gate == 0) return;
  if (tile >= d.lat_tiles) return;   // (the grid is the batch's largest)
  __shared__ double sm[G2LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wg = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int s = wg >> 2, w = wg & 3;   // split, wave in the split
  const int r = lane & 15, q = lane >> 4;
  const GridLattice lat = d.lat;
  const int64_t ntiy = (lat.ny + 63) / 64;
  const int64_t tix = tile / ntiy, tiy = tile % ntiy;
  const int64_t ix0 = tix * IXPT, iy0 = tiy * 64;
  const int64_t tabw = d.tabw, zrows = d.zrows, tstride = d.ld * tabw;
  const int P = d.hp.kind == 0 ? 1 : 2;
  const int64_t zq8 = (lat.ny + ZKS - 1) / ZKS * ZKS;
  const int64_t n0 = d.n0;
  double* const L22 = sm + G2RING;                 // [16][16] | z2 [16]
  double* const Li = L22 + KINC * KINC + KINC;     // L22^-1 [16][16]
  double* const Fn = Li + KINC * KINC;             // new rows' tables [2][KA][FW]
  double* const amx = Fn + 2 * 16 * (4 + 64);      // the waves' (max, argmax)
  WTRACE2(0);
  // the cells' inputs (written by the first launch): L22 | z2, the new rows' tables,
  // then L22^-1 by forward substitution (16 threads). (Issuing the K loop's first
  // stages before these loads, their latencies overlapped: 92.1-92.7k vs 92.9-93.1k
  // GP-updates/s without, alternating runs on one box, round 4 -- within noise)
  auto prologue = [&]() {
  for (int e = tid; e < KINC * KINC + KINC; e += G2NT) {
    const bool use = e < KINC * KINC ? (e / KINC < k && e % KINC <= e / KINC) : (e - KINC * KINC < k);
    L22[e] = use ? d.l22r[e] : 0.0;
  }
  for (int e = tid; e < 2 * KA * FW; e += G2NT) {
    const int kind2 = e / (KA * FW), rem = e % (KA * FW);
    const int a = rem / FW, col = rem % FW;
    const bool isx = col < IXPT;
    const int t = 2 * kind2 + (isx ? 0 : 1);
    const int64_t idx = isx ? ix0 + col : iy0 + (col - IXPT);
    Fn[e] = a < k ? d.tab[t * tstride + (n0 + a) * tabw + idx] : 0.0;
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
  };
  // ---- the K loop: split s, wave w: tile rows 16 w + r, all 64 columns ----
  // Each split streams its stages through its own LDS ring (buffer_load ... lds,
  // G2NST stages, one s_barrier per stage for the whole workgroup: the four splits
  // run in lockstep, a split past its own stages idles). Loading the MFMA operands
  // straight into registers instead (no ring, no barriers) was not faster (K loop
  // 18.3 vs 15.8 us at B = 8): the loop runs at ~34 TF of the ~45 TF a bare f64
  // MFMA loop reaches with four waves per SIMD.
  const __amdgpu_buffer_rsrc_t rZ = make_rsrc(d.zb, (int64_t)8 * P * zrows * tabw * KA);
  const __amdgpu_buffer_rsrc_t rAx = make_rsrc(d.axt, (int64_t)8 * 4 * (tabw + 1) * tabw);
  const __amdgpu_buffer_rsrc_t rTab = make_rsrc(d.tab, (int64_t)8 * 4 * tstride);
  // lane offsets of a stage's DMAs (one instruction moves two 64-double rows: lanes
  // 0-31 row 2 w, 32-63 row 2 w + 1): A rows swizzled by ((row & 3) << 4), B rows
  // by ((row & 1) << 4) (swz)
  const int kr = 2 * w + (lane >> 5);
  const unsigned vA = (unsigned)(8 * (((lane & 31) * 2) ^ ((kr & 3) << 4)) + 8 * (lane >> 5) * tabw * KA);
  const unsigned vBc = (unsigned)(8 * (((lane & 31) * 2) ^ ((lane >> 5) << 4)));
  const unsigned vB = vBc + (unsigned)(8 * (lane >> 5) * tabw);
  const int64_t npa = zq8 / ZKS, NA = P * npa;
  int64_t nvs[2] = {0, 0};
  for (int pt = 0; pt < P; ++pt) nvs[pt] = (d.zvl[pt * (zrows + 1)] + ZKS - 1) / ZKS;
  double* const ring = sm + s * G2NST * G2STG;
  auto issue = [&](int64_t g, bool virt, int64_t slot_t) {   // list entry g: 2 DMAs per wave
    int pt;
    int64_t q0;
    if (!virt) {
      pt = g < npa ? 0 : 1;
      q0 = (g - pt * npa) * ZKS;
    } else {
      pt = g < nvs[0] ? 0 : 1;
      q0 = zq8 + (g - (pt ? nvs[0] : 0)) * ZKS;
    }
    double* slot = ring + (slot_t % G2NST) * G2STG;
    dma_buf(rZ, slot + (2 * w) * G2R, vA, (unsigned)(8 * ((pt * zrows + q0 + 2 * w) * tabw + ix0) * KA));
    double* bdst = slot + ZKS * G2R + 2 * w * 64;
    if (!virt) {
      dma_buf(rAx, bdst, vB, (unsigned)(8 * (((2 * pt + 1) * (tabw + 1) + q0 + 2 * w) * tabw + iy0)));
    } else {
      // virtual rows: each half-wave its own training row's table row
      const int* vl = d.zvl + pt * (zrows + 1) + 1 + (q0 - zq8) + 2 * w;
      const int64_t j = (lane >> 5) ? vl[1] : vl[0];
      dma_buf(rTab, bdst, vBc + (unsigned)(8 * j * tabw), (unsigned)(8 * ((2 * pt + 1) * tstride + iy0)));
    }
  };
  d4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};
  constexpr int D = G2NST - 1;   // stages in flight ahead of the one consumed
  constexpr int CNT = 2;         // DMAs per issued stage (every wave)
  static_assert((D - 1) * CNT <= 12, "vm_wait_bar covers the outstanding DMAs");
  int64_t slot0 = 0;
  auto prime = [&](int64_t nlist, bool virt) {   // the pass's first D stages
    const int64_t hi = s < nlist ? (nlist - s + G2S - 1) / G2S : 0;
    for (int64_t t = 0; t < D && t < hi; ++t) issue(s + t * G2S, virt, slot0 + t);
  };
  auto pass = [&](int64_t nlist, bool virt, bool primed) {
    const int64_t hi = s < nlist ? (nlist - s + G2S - 1) / G2S : 0;   // this split's stages
    const int64_t him = (nlist + G2S - 1) / G2S;                      // split 0's: the most
    if (!primed) prime(nlist, virt);
    for (int64_t t = 0; t < him; ++t) {
      // this wave's DMA groups issued for stages after t
      const int64_t last = hi < t + D ? hi : t + D;
      const int64_t after = last > t + 1 ? last - (t + 1) : 0;
      vm_wait_bar((int)after * CNT);
      if (t < hi) {
        const double* slot = ring + ((slot0 + t) % G2NST) * G2STG;
        const double* As = slot;
        const double* Bs = slot + ZKS * G2R;
        double a[2], b[2][4];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int kk = 4 * e + q;
          a[e] = As[kk * G2R + ((16 * w + r) ^ ((kk & 3) << 4))];
#pragma unroll
          for (int n = 0; n < 4; ++n) b[e][n] = Bs[swz(kk, 16 * n + r)];
        }
        __builtin_amdgcn_sched_barrier(0);   // the reads ahead of the MFMAs
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int n = 0; n < 4; ++n) acc[n] = mfma(a[e], b[e][n], acc[n]);
        if (t + D < hi) issue(s + (t + D) * G2S, virt, slot0 + t + D);
      }
    }
    slot0 += him;
  };
  prologue();
  // the cells' resident posterior (the previous step's), loaded before the K loop so
  // that the epilogue does not wait a round trip for it
  double pcov = 0.0, pcom = 0.0;
  if (tid < IXPT * 64) {
    const int64_t ix = ix0 + (tid >> 6), iy = iy0 + (tid & 63);
    if (ix < lat.nx && iy < lat.ny) {
      const int64_t c = ix * lat.sx + iy * lat.sy;
      pcov = d.rvar_in[c];
      pcom = d.rmu_in[c];
    }
  }
  pass(NA, false, false);
  if (nvs[0] + nvs[1] > 0) {
    __syncthreads();   // the ring's last reads of the axis pass are done
    pass(nvs[0] + nvs[1], true, false);
  }
  vm_wait_all();
  __syncthreads();   // every ring read is done: the rings become the splits' sums
  WTRACE2(2);
  // ---- the splits meet: 1..3 store their sums, split 0 adds them in split order ----
  // element (16 w + q + 4 v, 16 n + r) of split s's tile is acc[n][v] of its lane
  double* const Tt = sm;   // the tile's T~ [64][64] (split 1's place, then the sum)
  if (s > 0) {
    double* const P_ = sm + (s - 1) * G2R * 64;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) P_[(16 * w + q + 4 * v) * 64 + 16 * n + r] = acc[n][v];
  }
  __syncthreads();
  if (s == 0) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int o = (16 * w + q + 4 * v) * 64 + 16 * n + r;
        double t = acc[n][v] + sm[o];
        t = t + sm[G2R * 64 + o];
        t = t + sm[2 * G2R * 64 + o];
        Tt[o] = t;
      }
  }
  __syncthreads();
  WTRACE2(3);
  // ---- cells: thread t < IXPT x 64 finishes cell (ix0 + t / 64, iy0 + t % 64) ----
  double bv = -__builtin_inf();
  int64_t bi = INT64_MAX;
  if (tid < IXPT * 64) {
    const int ixl = tid >> 6, iyl = tid & 63;
    const int64_t ix = ix0 + ixl, iy = iy0 + iyl;
    if (ix < lat.nx && iy < lat.ny) {
      const int64_t c = ix * lat.sx + iy * lat.sy;
      const double cov = pcov, com = pcom;
      VT* const vt = const_cast<VT*>(vres_ptr<VT>(d)) + (c / PBM) * d.vld * PBM + (c % PBM);
      const double* const Tc = Tt + (ixl * KA) * 64 + iyl;
      const int iyc = IXPT + iyl;
      double vn[KA];
      double vs = 0.0, ms = 0.0;
#pragma unroll
      for (int a = 0; a < KA; ++a) {
        vn[a] = 0.0;
        if (a < k) {
          const double* fL = Fn + a * FW;
          const double* fH = Fn + (KA + a) * FW;
          const double pn = fL[ixl] * fL[iyc] + fH[ixl] * fH[iyc];
          double t = pn - Tc[a * 64];
#pragma unroll
          for (int b = 0; b < a; ++b) t -= L22[a * KINC + b] * vn[b];
          vn[a] = t * Li[a * KINC + a];   // 1 / L22[a][a]
          vs += vn[a] * vn[a];
          ms += vn[a] * L22[KINC * KINC + a];
          __hip_atomic_store(vt + (n0 + a) * PBM, (VT)vn[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      const double vc = cov - vs;
      const double mc = com + ms;
      // write-through stores (sc1): the launch leaves no dirty L2 lines for its end
      // to write back (MI355X_MICROARCH.md: a release writes back the XCD L2s)
      __hip_atomic_store(d.mu + c, mc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(d.var + c, vc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (d.rmu) {
        __hip_atomic_store(d.rmu + c, mc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(d.rvar + c, vc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      argmax_pair(bv, bi, vc, c);
    }
  }
  WTRACE2(6);
  if (d.vmax || d.vargmax || d.status_host) {
    // the waves' (max, argmax) meet in LDS in wave order; wave 0 counts the tile in
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) argmax_pair(bv, bi, __shfl_xor(bv, off), __shfl_xor(bi, off));
    int64_t* const ami = reinterpret_cast<int64_t*>(amx);
    if (lane == 0) {
      amx[2 * wg] = bv;
      ami[2 * wg + 1] = bi;
    }
    __syncthreads();
    if (wg == 0) {
      bv = amx[0];
      bi = ami[1];
      for (int ww = 1; ww < G2NT / 64; ++ww) argmax_pair(bv, bi, amx[2 * ww], ami[2 * ww + 1]);
      var_argmax_group(d, bv, bi, tile, d.lat_tiles);
    }
  }
  WTRACE2(4);
}

template <int KA, class VT>
__global__ __launch_bounds__(G2NT) void k_lat_gemm2(const GPDesc* __restrict__ descs) {
  lat_gemm2<KA, VT>(descs[blockIdx.x], blockIdx.y);
}
template <int KA, class VT>
__global__ __launch_bounds__(G2NT) void k_lat_gemm2_arg(const DescArg a) {
  (void)a;
  const GPDesc* descs = (const GPDesc*)__builtin_amdgcn_kernarg_segment_ptr();
  lat_gemm2<KA, VT>(descs[blockIdx.x], blockIdx.y);
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
  if (threadIdx.x < 4 && r0 + threadIdx.x < hi) {
    const int64_t row = r0 + threadIdx.x;
    d.lidx[row] = lattice_xy(d, d.X[2 * row], d.X[2 * row + 1]);
  }
}

// The axis tables of GPs with lat_axbuild: axt[t][p][col] for p, col < tabw (row
// tabw: zeros). Grid (GPs, 4 tables x (tabw + 1) rows / 4 rows per workgroup).
__global__ __launch_bounds__(NT) void k_lat_axes(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  if (!d.lat_axbuild) return;
  const int64_t tabw = d.tabw, rows = 4 * (tabw + 1);
  for (int64_t e = threadIdx.x; e < 4 * tabw; e += NT) {
    const int64_t rr = 4 * (int64_t)blockIdx.x + e / tabw, col = e % tabw;
    if (rr >= rows) continue;
    const int t = (int)(rr / (tabw + 1));
    const int64_t p = rr % (tabw + 1);
    d.axt[rr * tabw + col] = p < tabw ? lat_axis_value(d, t, p, col) : 0.0;
  }
}

// MFGP_F32: Ff = (float) F over F's storage, for the GPs whose F was just built
__global__ __launch_bounds__(NT) void k_narrow_f(const GPDesc* __restrict__ descs) {
  const GPDesc& d = descs[blockIdx.y];
  if (!d.lat_fbuild || !d.Ff || !d.vf32) return;
  const int64_t n = fblk_size(d.ld);
  for (int64_t e = ((int64_t)blockIdx.x * NT + threadIdx.x) * 2; e < n; e += (int64_t)gridDim.x * NT * 2) {
    if (e + 1 < n) {
      const dv2 v = *reinterpret_cast<const GLOBAL dv2*>(gp(d.F) + e);
      *reinterpret_cast<GLOBAL fv2*>(gp(d.Ff) + e) = fv2{(float)v.x, (float)v.y};
    } else {
      d.Ff[e] = (float)d.F[e];
    }
  }
}

hipError_t launch_narrow_f(const GPDesc* d, int count, int64_t max_elems, hipStream_t s) {
  if (count < 1 || max_elems <= 0) return hipSuccess;
  const int64_t wgs = std::min<int64_t>(1024, (max_elems / 2 + NT - 1) / NT);
  hipLaunchKernelGGL(k_narrow_f, dim3((unsigned)wgs, count), dim3(NT), 0, s, d);
  return hipGetLastError();
}
