// C ABI of libmfgp_hip.so (declared in include/mfgp_hip.h).
//
// Host-side state management for the GP posterior engine: contexts (one HIP
// stream + workspace each), models (device-resident training set, factor and
// grid), the batched update+predict driver, timing and error reporting.
// Mirrors the reference methods cited in include/mfgp_hip.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mfgp_hip.h"
#include "mfgp_internal.h"

using namespace mfgp;

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess) return set_err(MFGP_ERR_DEVICE, "%s: %s (%s:%d)", #expr,         \
                                         hipGetErrorString(e_), __FILE__, __LINE__);       \
  } while (0)

// The context's device for the duration of one entry point, the caller's restored on
// every return path (an entry point that set the device and left it
// changed torch.cuda.current_device() in a multi-GPU process). dev < 0: no change.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (dev < 0 || hipGetDevice(&prev) != hipSuccess) {
      prev = -1;
      return;
    }
    if (prev == dev || hipSetDevice(dev) != hipSuccess) prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

constexpr int RING = 64;       // descriptor upload slots
constexpr int MAXB = 256;      // GPs per launch
constexpr int64_t MAX_FULL_CAP = 16319;   // largest training capacity the full predict serves (ld <= 16383)
constexpr size_t F32_SCRATCH = size_t(16) << 30;   // bytes of fp64 V scratch for MFGP_F32 full predicts
// lattice-separable step (k_inc_lat): taken when kss / (smallest noise + jitter)
// <= LAT_RMAX (its error grows with the conditioning of K),
// and for at most LAT_MAXD consecutive steps before var / mu are recomputed from V
constexpr double LAT_RMAX = 1e4;
constexpr int LAT_MAXD = 256;
// planner counters (mfgp_ctx_planner_stats): model runs, bordered appends, V-stream
// predicts, lattice steps (of them by value / with k_lat_gemm2), full factors, full
// predicts; then the batched planner's host time (us) before, in and after its loop
constexpr int PLAN_NSTATS = 11;

struct EvPair {
  hipEvent_t a, b;
  int kind;  // 0 predict, 1 factor
};

}  // namespace

struct mfgp_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  // descriptor ring
  GPDesc* h_ring = nullptr;  // pinned [RING][MAXB]
  GPDesc* d_ring = nullptr;  // device [RING][MAXB]
  hipEvent_t ring_ev[RING];
  bool ring_used[RING];
  int ring_pos = 0;
  // workspace (V scratch + device outputs for host-pointer calls)
  double* ws = nullptr;
  size_t ws_bytes = 0;
  // timing: 0 off, 1 predict + factor launches, 2 predict launches only
  int timing = 0;
  int64_t timing_stride = 1, timing_seq = 0;   // bracket every stride-th eligible launch
  std::vector<EvPair> pending;
  std::vector<hipEvent_t> pool;
  double t_predict = 0.0, t_factor = 0.0;
  int64_t n_predict = 0, n_factor = 0;
  // deferred status words of ASYNC batches, with the model each belongs to (a
  // failed factor is dropped from its model at mfgp_ctx_synchronize)
  struct AsyncStatus {
    mfgp_model* m;
    int* dev;      // the model's status word (device)
    int* host;     // its mapped host copy written by the launch (k_inc_stream1), or null: copy dev
  };
  std::vector<AsyncStatus> async_status;
  // fp64 scratch in which the full predicts of MFGP_F32 models compute V
  // (k_predict re-reads its own rows), then rounded into their fp32 V
  double* vscr = nullptr;
  size_t vscr_bytes = 0;
  int f32_group = 1;          // full predicts per k_predict launch that share vscr
  // incremental append / predict (bordered Cholesky + resident V); off = always
  // refactor and recompute V from scratch, as the reference does
  bool incremental = true;
  bool fused = true;          // bordered append + one-pass predict in one launch (k_inc_stream)
  bool deferred = false;      // mfgp_append stages rows for a later (fused) bordered append
  bool lattice = true;        // lattice-separable appends (k_inc_lat) where they apply
  int lat_ksplit = 0;         // split-K of its GEMM tiles (0: chosen per launch; MFGP_LAT_KSPLIT, diagnostics)
  int lat_wu = 0;             // w units of a launch, all GPs (0: two per CU; MFGP_LAT_WU, diagnostics)
  int lat_selfg = -1;         // w units read L21 from V themselves (-1: for one GP; MFGP_LAT_SELFG, diagnostics)
  int lat_gemm2 = -1;         // the step's GEMM and cells as a second launch (k_lat_gemm2): -1 where its
                              // tiles fill the chip once or twice, 1 always, 0 never (in-launch split-K
                              // tiles); MFGP_LAT_GEMM2, diagnostics and tests
  bool trinv_columns = false;  // F by the block-column k_trinv_f instead of recursive doubling (MFGP_TRINV_COLUMNS)
  int factor_depth = 4;        // 64-column steps per trailing-update pass of the factor (MFGP_FACTOR_DEPTH; 1: one-level)
  bool lat_force = false;     // take it for small batches too (mfgp_ctx_set_lattice(2): tests)
  // launches of this context may run concurrently with other contexts' (several
  // streams on one GPU, mfgp_ctx_set_concurrent): no launch may rely on all of its
  // workgroups being resident at once -- the lattice step's GEMM runs as the second
  // launch (k_lat_gemm2, no cross-workgroup waits) instead of in-launch split-K tiles
  bool concurrent = false;
  int rsplit_force = 0;       // one-pass predict row splits per cell group (0: the host's rule)
  int lat_zcsr = 1;           // the Z units read member lists built by one scan unit per part
                              // instead of bucketing every row themselves (MFGP_LAT_ZCSR=0: off)
  int64_t spin_us = 2000;     // host polling of mapped status words before a synchronise (MFGP_SPIN_US; 0: off)
  // the eager append of one GP (spec_append_predict) returns at the step's L22
  // verdict, published by the launch as soon as it is known, instead of at the
  // launch's end: the caller's host work until its next call (the simulator's
  // grid check, the predict's argument handling) overlaps the posterior
  // (MFGP_EARLY_PD=0: wait for the launch's end)
  bool early_pd = true;
  bool early_running = false;  // such a launch may still run: the next entry point settles it first
  bool desc_arg = true;       // a batch step that is one k_inc_lat / k_inc_stream launch passes its
                              // descriptors by value
                              // (MFGP_DESC_ARG=0: upload them, diagnostics)
  // pinned host staging of the status words
  int* h_status = nullptr;
  size_t h_status_n = 0;

  int ncu = 256;              // compute units (hipDeviceProp multiProcessorCount)
  // the path counters of the planners' loops (mfgp_sample_points,
  // mfgp_batch_sample_points), moved here from the models when each loop ends:
  // which step form the Choi iterations took (mfgp_ctx_planner_stats)
  int64_t plan_stats[PLAN_NSTATS] = {0};
};

struct mfgp_model {
  mfgp_ctx* ctx = nullptr;
  int* gate_dev = nullptr;  // device gate of every step of this model (the planners' loops: 0 = skip)
  int kind = MFGP_SF;
  int dtype = MFGP_F64;     // precision of the resident V (MFGP_F32: fp32 storage and stream)
  int nhyp = 4;
  double hyp[9] = {0};
  double jitter = 1e-8;
  // training set (device)
  int64_t NL = 0, NH = 0, cap = 0;
  double* X = nullptr;  // [cap,2]
  double* y = nullptr;  // [cap]
  // factor (device)
  int64_t ld = 0;
  double* A = nullptr;     // [ld,ld]
  double* Linv = nullptr;  // [ld/NB][TILE]
  double* zv = nullptr;     // [cap] z = L^-1 (y - m)
  double* iscr = nullptr;   // incremental-append scratch (inc_scratch_doubles(cap))
  int* status = nullptr;
  int* status_host = nullptr;       // mapped pinned words the single-GP fused launch publishes into:
                                    // [0] its status (last act), [1] the L22 verdict (pd_host)
  int* status_host_dev = nullptr;   // its device address
  bool factored = false;
  int64_t factor_N = -1;    // rows [0, factor_N) of A / Linv / zv hold the current factor
  int64_t ablk = 0;         // 64-row blocks of A / Linv initialised (assembled or padded)
  double factor_hyp[9] = {0};
  double factor_jitter = 0.0;
  // grid (device)
  int64_t M = 0, Mcap = 0;
  double* grid = nullptr;
  GridLattice lat{};        // lattice structure of the grid (nx == 0: none)
  // resident V = L^-1 psi^T [vtiles][vld][PBM] (double, or float for MFGP_F32);
  // rows [0, v_n) valid for the current factor and grid
  void* V = nullptr;
  int64_t vld = 0, vtiles = 0, v_n = 0;
  double* tred = nullptr;     // [vtiles][2] per-tile (max, argmax) of var, then the tiles' arrival counter
  int64_t tred_n = 0;         // doubles of tred
  unsigned* sync = nullptr;   // k_inc_stream hand-off words {arrivals, L21 ready, L22 ready} (zeroed)
  unsigned epoch = 0;         // last k_inc_stream epoch of this model
  // the compact bordered rows in iscr (inc_l21c_offset) hold rows [l21c_n0, l21c_N)
  // bordered onto l21c_n0 factor rows (-1: none)
  int64_t l21c_n0 = -1, l21c_N = -1;
  // speculative predict: an (eager) append that follows the pattern append ->
  // predict runs the bordered append and the one-pass predict as one launch and
  // keeps mu | var in `spec_out` (mapped pinned, [2][M]) for the predict that
  // follows; any change to the model drops them
  double* spec_out = nullptr;
  double* spec_out_dev = nullptr;
  int64_t spec_cap = 0;
  bool spec_valid = false;
  // spec_out's trailer [2 cap] = (max var, its first argmax) holds the fused var
  // max / argmax of the launch that wrote spec_out (the eager append's): the
  // drop-in's np.amax / np.argmax of the covariance read it instead of rescanning
  bool spec_max = false;
  bool pred_since_append = false;   // a predict came after the last append
  // path counters (mfgp_model_stats)
  int64_t n_full_factor = 0, n_inc_factor = 0, n_full_predict = 0, n_vstream = 0, n_lattice = 0;
  int64_t n_lattice_arg = 0;   // lattice steps launched with their descriptors by value (k_inc_lat_arg)
  int64_t n_lattice_g2 = 0;    // lattice steps whose GEMM and cells ran as a second launch (k_lat_gemm2)
  int64_t n_post_copy = 0;     // batch predicts served from the resident posterior (k_post_copy: nothing appended)
  int64_t n_early_pd = 0;      // eager appends that returned at the launch's published L22 verdict
  unsigned* csr = nullptr;     // the scan units' member lists (csr_bytes; mfgp_internal.h)
  int64_t csr_n = 0;           // (bytes)
  // state generation: a new factor from scratch, a new grid or new hyperparameters
  // start a new one (the resident posterior, F and the tables belong to one)
  uint64_t gen = 1;
  // resident posterior: two buffers [mu | var] of M each, written by every predict
  // (incremental mode); buffer b holds the posterior of the res_n[b] leading rows
  double* res = nullptr;
  int64_t res_M = 0;
  int64_t res_n[2] = {-1, -1};
  uint64_t res_gen[2] = {0, 0};
  int res_depth[2] = {0, 0};   // lattice steps since var / mu were computed from V
  uint64_t res_tick[2] = {0, 0}, tick = 0;
  // lattice-separable step state (allocated on first use)
  double* F = nullptr;        // explicit L^-1 [F_ld][F_ld], rows [0, F_n) current for generation F_gen
  float* Ff = nullptr;        // MFGP_F32: F in fp32 (the rows the lattice steps stream and extend)
  int64_t F_ld = 0, F_n = 0;
  uint64_t F_gen = 0;
  double* tab = nullptr;      // separable tables [4][tab_ld][tabw], rows [0, tab_n)
  int64_t tab_ld = 0, tabw = 0, tab_n = 0;
  uint64_t tab_gen = 0;
  double* wv = nullptr;       // w [wv_ld][KINC]
  int64_t wv_ld = 0;
  unsigned* wflag = nullptr;  // [wv_ld / 64 + 2]
  unsigned* wcnt = nullptr;   // [wv_ld / 64 + 2]
  double* wpart = nullptr;    // [LAT_WU_MAX + wv_ld / 64 + 1][1024]
  double* gpart = nullptr;    // split-K partials
  size_t gpart_n = 0;
  unsigned* gcnt = nullptr;   // per GEMM tile
  int64_t gcnt_n = 0;
  int* lidx = nullptr;        // lattice indices per training row [tab_ld], rows [0, tab_n) (with the tables)
  double* axt = nullptr;      // axis tables [4][tabw + 1][tabw], current for generation axt_gen
  int64_t axt_w = 0;
  uint64_t axt_gen = 0;
  double* zb = nullptr;       // Z rows [P][zrows][tabw][zb_ka]
  int64_t zb_rows = 0, zb_w = 0;
  int zb_ka = 0;
  unsigned* zflag = nullptr;  // [zflag_n]
  int64_t zflag_n = 0;
  unsigned* ldone = nullptr;  // [4] lattice phase hand-offs (arrivals | flag, twice)
  int* zvl = nullptr;         // [2][zb_rows + 1]
};

namespace {

Hyp derive_hyp(int kind, const double* hyp, double jitter) {
  Hyp h{};
  h.kind = kind;
  h.jitter = jitter;
  if (kind == MFGP_SF) {
    // [mu, s^2, L, noise]  (gp:75-76, gp:132, gp:248-249)
    h.sL = std::exp(hyp[1]);
    h.lL = std::exp(hyp[2]);
    h.sH = h.sL;
    h.lH = h.lL;
    h.rho = 1.0;
    h.rho2 = 1.0;
    h.noiseL = h.noiseH = std::exp(hyp[3]);
    h.meanL = h.meanH = std::exp(hyp[0]);
    h.kss = h.sL;  // kernel(X*,X*) diagonal = s * exp(0)
  } else {
    // [mu_lo, s^2_lo, L_lo, mu_hi, s^2_hi, L_hi, rho, noise_lo, noise_hi]  (gp:510-514, 414-416)
    h.sL = std::exp(hyp[1]);
    h.lL = std::exp(hyp[2]);
    h.sH = std::exp(hyp[4]);
    h.lH = std::exp(hyp[5]);
    h.rho = std::exp(hyp[6]);
    h.rho2 = h.rho * h.rho;
    h.noiseL = std::exp(hyp[7]);
    h.noiseH = std::exp(hyp[8]);
    h.meanL = std::exp(hyp[0]);
    h.meanH = h.rho * h.meanL + std::exp(hyp[3]);
    h.kss = h.rho2 * h.sL + h.sH;  // gp:435-436 diagonal
  }
  return h;
}

int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

hipEvent_t ev_get(mfgp_ctx* c) {
  if (!c->pool.empty()) {
    hipEvent_t e = c->pool.back();
    c->pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

int ev_begin(mfgp_ctx* c, EvPair& p, int kind) {
  p.a = p.b = nullptr;
  if (!c->timing || (c->timing == 2 && kind != 0)) return MFGP_OK;
  if (c->timing_seq++ % c->timing_stride != 0) return MFGP_OK;
  p.a = ev_get(c);
  p.b = ev_get(c);
  p.kind = kind;
  HIP_TRY(hipEventRecord(p.a, c->stream));
  return MFGP_OK;
}

int ev_end(mfgp_ctx* c, EvPair& p) {
  if (!p.a) return MFGP_OK;
  HIP_TRY(hipEventRecord(p.b, c->stream));
  c->pending.push_back(p);
  return MFGP_OK;
}

int drain_timing(mfgp_ctx* c) {
  for (auto& p : c->pending) {
    HIP_TRY(hipEventSynchronize(p.b));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
    if (p.kind == 0) {
      c->t_predict += ms;
      c->n_predict += 1;
    } else {
      c->t_factor += ms;
      c->n_factor += 1;
    }
    c->pool.push_back(p.a);
    c->pool.push_back(p.b);
  }
  c->pending.clear();
  return MFGP_OK;
}

int ensure_h_status(mfgp_ctx* c, size_t n) {
  if (n <= c->h_status_n) return MFGP_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->h_status) HIP_TRY(hipHostFree(c->h_status));
  c->h_status = nullptr;
  c->h_status_n = 0;
  const size_t want = std::max<size_t>(n, 64);
  HIP_TRY(hipHostMalloc(&c->h_status, sizeof(int) * want, hipHostMallocDefault));
  c->h_status_n = want;
  return MFGP_OK;
}

int ensure_ws(mfgp_ctx* c, size_t bytes) {
  if (bytes <= c->ws_bytes) return MFGP_OK;
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t want = std::max(bytes, c->ws_bytes + c->ws_bytes / 2);
  if (c->ws) HIP_TRY(hipFree(c->ws));
  c->ws = nullptr;
  c->ws_bytes = 0;
  HIP_TRY(hipMalloc(&c->ws, want));
  c->ws_bytes = want;
  return MFGP_OK;
}

// Grow the training capacity of m to hold `need` rows. Keeps X / y and, when
// the factor is current for some rows, A / Linv / zv too (copied into the new
// leading dimension), so a growing GP stays on the incremental path.
int ensure_cap(mfgp_model* m, int64_t need) {
  if (need <= m->cap && m->A) return MFGP_OK;
  mfgp_ctx* c = m->ctx;
  int64_t cap = std::max<int64_t>({need, m->cap + m->cap / 2, 63});
  // the full predict (k_predict) addresses A through a 32-bit buffer descriptor:
  // ld <= 16383, i.e. a capacity of at most MAX_FULL_CAP rows; 1.5x growth stops there
  if (cap > MAX_FULL_CAP && need <= MAX_FULL_CAP) cap = MAX_FULL_CAP;
  int64_t ld = round_up(cap + 1, NB);
  cap = ld - 1;
  double *X = nullptr, *y = nullptr, *A = nullptr, *Li = nullptr, *zv = nullptr, *isc = nullptr;
  HIP_TRY(hipStreamSynchronize(c->stream));
  HIP_TRY(hipMalloc(&X, sizeof(double) * 2 * cap));
  HIP_TRY(hipMalloc(&y, sizeof(double) * cap));
  HIP_TRY(hipMalloc(&zv, sizeof(double) * cap));
  HIP_TRY(hipMalloc(&isc, sizeof(double) * inc_scratch_doubles(cap)));
  // producer ready flags start below every epoch (epochs are never 0)
  HIP_TRY(hipMemsetAsync(isc + inc_pflag_offset(cap), 0, sizeof(unsigned) * inc_pflag_count(cap), c->stream));
  HIP_TRY(hipMalloc(&A, sizeof(double) * ld * ld));
  HIP_TRY(hipMalloc(&Li, sizeof(double) * (ld / NB) * TILE));
  const int64_t n = m->NL + m->NH;
  if (n > 0) {
    HIP_TRY(hipMemcpyAsync(X, m->X, sizeof(double) * 2 * n, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(y, m->y, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
  }
  const bool keep = m->A && m->factored && m->ablk > 0;
  if (keep) {
    HIP_TRY(hipMemcpy2DAsync(A, sizeof(double) * ld, m->A, sizeof(double) * m->ld, sizeof(double) * m->ld, m->ld,
                             hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(Li, m->Linv, sizeof(double) * (m->ld / NB) * TILE, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(zv, m->zv, sizeof(double) * m->cap, hipMemcpyDeviceToDevice, c->stream));
  }
  // the lattice step's F and tables move to the new leading dimension too
  double *F = nullptr, *tab = nullptr;
  float* Ff = nullptr;
  int* lidx = nullptr;
  if (keep && m->F && m->F_n > 0) {
    HIP_TRY(hipMalloc(&F, sizeof(double) * fblk_size(ld)));
    HIP_TRY(hipMemsetAsync(F, 0, sizeof(double) * fblk_size(ld), c->stream));
    for (int64_t jb = 0; 64 * jb < m->F_n; ++jb)   // each column block's rows [64 jb, F_n)
      HIP_TRY(hipMemcpyAsync(F + fblk_off(jb, ld), m->F + fblk_off(jb, m->F_ld),
                             sizeof(double) * 64 * (m->F_n - 64 * jb), hipMemcpyDeviceToDevice, c->stream));
    if (m->Ff) {   // (MFGP_F32: the rows past the build live in Ff only)
      HIP_TRY(hipMalloc(&Ff, sizeof(float) * fblk_size(ld)));
      HIP_TRY(hipMemsetAsync(Ff, 0, sizeof(float) * fblk_size(ld), c->stream));
      for (int64_t jb = 0; 64 * jb < m->F_n; ++jb)
        HIP_TRY(hipMemcpyAsync(Ff + fblk_off(jb, ld), m->Ff + fblk_off(jb, m->F_ld),
                               sizeof(float) * 64 * (m->F_n - 64 * jb), hipMemcpyDeviceToDevice, c->stream));
    }
  }
  if (m->tab && m->tab_n > 0) {
    HIP_TRY(hipMalloc(&tab, sizeof(double) * 4 * ld * m->tabw));
    HIP_TRY(hipMemsetAsync(tab, 0, sizeof(double) * 4 * ld * m->tabw, c->stream));
    for (int t = 0; t < 4; ++t)
      HIP_TRY(hipMemcpyAsync(tab + (size_t)t * ld * m->tabw, m->tab + (size_t)t * m->tab_ld * m->tabw,
                             sizeof(double) * m->tab_n * m->tabw, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMalloc(&lidx, sizeof(int) * ld));
    HIP_TRY(hipMemcpyAsync(lidx, m->lidx, sizeof(int) * m->tab_n, hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (m->F) HIP_TRY(hipFree(m->F));
  if (m->Ff) HIP_TRY(hipFree(m->Ff));
  if (m->tab) HIP_TRY(hipFree(m->tab));
  if (m->lidx) HIP_TRY(hipFree(m->lidx));
  m->lidx = lidx;
  m->F = F;
  m->Ff = Ff;
  m->F_ld = F ? ld : 0;
  if (!F) m->F_n = 0;
  m->tab = tab;
  m->tab_ld = tab ? ld : 0;
  if (!tab) m->tab_n = 0;
  if (m->X) HIP_TRY(hipFree(m->X));
  if (m->y) HIP_TRY(hipFree(m->y));
  if (m->A) HIP_TRY(hipFree(m->A));
  if (m->Linv) HIP_TRY(hipFree(m->Linv));
  if (m->zv) HIP_TRY(hipFree(m->zv));
  if (m->iscr) HIP_TRY(hipFree(m->iscr));
  m->iscr = isc;
  m->l21c_N = -1;
  m->X = X;
  m->y = y;
  m->A = A;
  m->Linv = Li;
  m->zv = zv;
  m->cap = cap;
  m->ld = ld;
  if (!keep) {
    m->factored = false;
    m->ablk = 0;
    m->v_n = 0;
  }
  return MFGP_OK;
}

// Resident V for the current capacity and grid (contents kept when it fits).
size_t v_elem(const mfgp_model* m) { return m->dtype == MFGP_F32 ? sizeof(float) : sizeof(double); }

int ensure_v(mfgp_model* m) {
  const int64_t vld = round_up(m->cap, PRB);
  const int64_t tiles = ntiles_grid(m->M);
  if (m->V && m->vld == vld && m->vtiles >= tiles) return MFGP_OK;
  hipStream_t s = m->ctx->stream;
  const size_t es = v_elem(m);
  void* V = nullptr;
  HIP_TRY(hipMalloc(&V, es * (size_t)tiles * vld * PBM));
  if (m->V && m->v_n > 0 && m->vtiles >= tiles && m->vld >= m->v_n) {
    // capacity grew: move the valid rows of every tile to the new row stride
    HIP_TRY(hipMemcpy2DAsync(V, es * vld * PBM, m->V, es * m->vld * PBM, es * m->v_n * PBM, tiles,
                             hipMemcpyDeviceToDevice, s));
  } else {
    m->v_n = 0;
  }
  HIP_TRY(hipStreamSynchronize(s));
  if (m->V) HIP_TRY(hipFree(m->V));
  m->V = V;
  m->vld = vld;
  if (tiles > m->vtiles || !m->tred) {
    // [arrival counter | (max, argmax) per 64-cell tile (k_predict) or per 32-cell
    // wave group (one-pass predicts)]; the counter is zero between launches (the
    // last arriver of each launch resets it)
    if (m->tred) HIP_TRY(hipFree(m->tred));
    m->tred = nullptr;
    HIP_TRY(hipMalloc(&m->tred, sizeof(double) * (4 * tiles + 1)));
    HIP_TRY(hipMemsetAsync(m->tred, 0, sizeof(double) * (4 * tiles + 1), s));
    HIP_TRY(hipStreamSynchronize(s));
    m->tred_n = 4 * tiles + 1;
  }
  m->vtiles = tiles;
  return MFGP_OK;
}

int check_model(const mfgp_model* m) {
  if (!m || !m->ctx) return set_err(MFGP_ERR_ARG, "null model");
  return MFGP_OK;
}

GPDesc* acquire_slot(mfgp_ctx* c, int& slot, int& rc) {
  slot = c->ring_pos;
  c->ring_pos = (c->ring_pos + 1) % RING;
  rc = MFGP_OK;
  if (c->ring_used[slot]) {
    hipError_t e = hipEventSynchronize(c->ring_ev[slot]);
    if (e != hipSuccess) {
      rc = set_err(MFGP_ERR_DEVICE, "hipEventSynchronize: %s", hipGetErrorString(e));
      return nullptr;
    }
  }
  return c->h_ring + (size_t)slot * MAXB;
}

int upload_slot(mfgp_ctx* c, int slot, int count, const GPDesc** dptr) {
  HIP_TRY(hipMemcpyAsync(c->d_ring + (size_t)slot * MAXB, c->h_ring + (size_t)slot * MAXB,
                         sizeof(GPDesc) * count, hipMemcpyHostToDevice, c->stream));
  *dptr = c->d_ring + (size_t)slot * MAXB;
  return MFGP_OK;
}

int release_slot(mfgp_ctx* c, int slot) {
  HIP_TRY(hipEventRecord(c->ring_ev[slot], c->stream));
  c->ring_used[slot] = true;
  return MFGP_OK;
}
// A slot whose descriptors went into a launch by value (kernel argument: copied at
// the launch call) and were never uploaded: nothing on the stream reads it, so it
// needs no event (one hipEventRecord less per step: the drop-in step's host time).
void release_slot_unread(mfgp_ctx* c, int slot) { c->ring_used[slot] = false; }

constexpr int STATUS_UNSET = INT_MIN + 1;   // status_host before the launch writes it

// An eager append that returned at its L22 verdict (mfgp_ctx::early_pd) may still
// run: every entry point waits for it, and takes its status, before it reads or
// reuses anything the launch touches.
int settle(mfgp_ctx* c) { return (c && c->early_running) ? mfgp_ctx_synchronize(c) : MFGP_OK; }

void fill_desc(GPDesc& d, mfgp_model* m) {
  d.X = m->X;
  d.y = m->y;
  d.A = m->A;
  d.Linv = m->Linv;
  d.grid = m->grid;
  d.lat = m->lat;
  d.V = m->dtype == MFGP_F64 ? static_cast<double*>(m->V) : nullptr;
  d.Vf = m->dtype == MFGP_F32 ? static_cast<float*>(m->V) : nullptr;
  d.vf32 = m->dtype == MFGP_F32 ? 1 : 0;
  d.zv = m->zv;
  d.iscr = m->iscr;
  d.l21c = m->iscr ? m->iscr + inc_l21c_offset(m->cap) : nullptr;
  d.l22r = m->iscr ? m->iscr + inc_l22r_offset(m->cap) : nullptr;
  d.pflag = m->iscr ? reinterpret_cast<unsigned*>(m->iscr + inc_pflag_offset(m->cap)) : nullptr;
  d.mu = nullptr;
  d.var = nullptr;
  d.vmax = nullptr;
  d.vargmax = nullptr;
  d.tred = m->tred;
  d.gate = m->gate_dev;
  d.status = m->status;
  d.status_host = nullptr;
  d.pd_host = nullptr;
  d.srcX = nullptr;
  d.srcY = nullptr;
  d.k_new = 0;
  d.rows_inline = 0;
  d.sync = nullptr;
  d.epoch = 0;
  d.nprod = 0;
  d.tiles = 0;
  d.l21c_ok = 0;
  d.rsplit = 1;
  d.ld = m->ld;
  d.N = m->NL + m->NH;
  d.NL = m->NL;
  d.M = m->M;
  d.vld = m->vld;
  d.n0 = 0;
  d.vres = 0;
  d.ablk = m->ablk;
  d.F = nullptr;
  d.Ff = nullptr;
  d.tab = nullptr;
  d.wv = nullptr;
  d.wflag = nullptr;
  d.gpart = nullptr;
  d.gcnt = nullptr;
  d.rmu_in = nullptr;
  d.rvar_in = nullptr;
  d.rmu = nullptr;
  d.rvar = nullptr;
  d.tabw = 0;
  d.tab_lo = 0;
  d.ka = 8;
  d.ksplit = 1;
  d.lat_tiles = 0;
  d.nwb = 0;
  d.lat_fbuild = 0;
  d.nwu = 0;
  d.wpart = nullptr;
  d.wcnt = nullptr;
  d.lat_selfg = 0;
  d.lat_g2 = 0;
  d.lat_zcsr = 0;
  d.csr = nullptr;
  d.hf = derive_hyp(m->kind, m->hyp, m->jitter);
  d.hp = d.hf;
}

// A model's status word to check at the next mfgp_ctx_synchronize. One entry per
// model: every entry of a model would read the same device word (its value after
// the model's last launch), so repeated ASYNC steps add no copies to the sync. A
// model's entry that the one-GP fused launch publishes into mapped memory
// (host != null) is replaced by the device word when a later step does not.
void add_async_status(mfgp_ctx* c, mfgp_model* m) {
  for (auto& a : c->async_status)
    if (a.m == m) {
      a.host = nullptr;   // (a later launch of this model may not publish: read the word)
      return;
    }
  c->async_status.push_back({m, m->status, nullptr});
}

// ---- resident posterior (two buffers, tagged with the rows and generation) ----
int ensure_res(mfgp_model* m) {
  if (m->res && m->res_M >= m->M) return MFGP_OK;
  HIP_TRY(hipStreamSynchronize(m->ctx->stream));
  if (m->res) HIP_TRY(hipFree(m->res));
  m->res = nullptr;
  m->res_M = 0;
  m->res_n[0] = m->res_n[1] = -1;
  HIP_TRY(hipMalloc(&m->res, sizeof(double) * 4 * (size_t)m->M));
  m->res_M = m->M;
  return MFGP_OK;
}
double* res_mu(mfgp_model* m, int b) { return m->res + (size_t)b * 2 * m->res_M; }
double* res_var(mfgp_model* m, int b) { return m->res + (size_t)b * 2 * m->res_M + m->res_M; }
// the buffer holding the posterior of the n leading rows (-1: none)
int res_find(const mfgp_model* m, int64_t n) {
  for (int b = 0; b < 2; ++b)
    if (m->res && m->res_n[b] == n && m->res_gen[b] == m->gen) return b;
  return -1;
}
// the buffer a predict writes: not `keep`, else the least recently written
int res_out(const mfgp_model* m, int keep) {
  if (keep >= 0) return 1 - keep;
  return m->res_tick[0] <= m->res_tick[1] ? 0 : 1;
}
void res_tag(mfgp_model* m, int b, int64_t n, int depth) {
  m->res_n[b] = n;
  m->res_gen[b] = m->gen;
  m->res_depth[b] = depth;
  m->res_tick[b] = ++m->tick;
}
// Point a predict descriptor's resident outputs at a buffer (incremental mode);
// returns the buffer (-1: none). Tag it once the launch is enqueued.
int set_res_out(mfgp_model* m, GPDesc& d, int keep) {
  if (!m->ctx->incremental || m->M <= 0 || ensure_res(m) != MFGP_OK) return -1;
  const int b = res_out(m, keep);
  d.rmu = res_mu(m, b);
  d.rvar = res_var(m, b);
  return b;
}

// ---- lattice-separable step ----
bool lat_cond_ok(const mfgp_model* m) {
  const Hyp h = derive_hyp(m->kind, m->hyp, m->jitter);
  const double noise = (m->kind == MFGP_SF ? h.noiseL : std::min(h.noiseL, h.noiseH)) + h.jitter;
  return noise > 0.0 && h.kss / noise <= LAT_RMAX;
}
int64_t lat_tabw(const mfgp_model* m) { return round_up(std::max<int64_t>(m->lat.nx, m->lat.ny), 64); }
int64_t lat_tiles(const mfgp_model* m, int ka) {
  return ((m->lat.nx + 128 / ka - 1) / (128 / ka)) * ((m->lat.ny + 63) / 64);
}
// k_lat_gemm2's tiles: 64 (a, ix) rows x 64 iy columns
int64_t lat_tiles2(const mfgp_model* m, int ka) {
  return ((m->lat.nx + 64 / ka - 1) / (64 / ka)) * ((m->lat.ny + 63) / 64);
}
// Z units of the lattice-axis form: parts x ceil(ny / zq), zq lattice y-rows each
// (two per thread group of tabw threads)
int lat_zq(const mfgp_model* m) { return (int)(2 * NT / lat_tabw(m)); }
int64_t lat_nzu(const mfgp_model* m) {
  return (m->kind == MFGP_SF ? 1 : 2) * ((m->lat.ny + lat_zq(m) - 1) / lat_zq(m));
}
// Can the bordered append of rows [n0, N) and its predict take k_inc_lat?
bool lat_eligible(const mfgp_model* m, int64_t n0) {
  const int64_t k = m->NL + m->NH - n0;
  if (!m->ctx->lattice || m->lat.nx <= 0 || m->M <= 0 || k < 1 || k > KINC || n0 < 1) return false;
  if (lat_tabw(m) > NT) return false;   // a Z unit's thread per lattice column
  if ((n0 + 63) / 64 > LAT_NWB_MAX) return false;   // a w unit's blocks
  if (!lat_cond_ok(m)) return false;
  const int b = res_find(m, n0);
  return b >= 0 && m->res_depth[b] < LAT_MAXD;
}
// F, the tables, w and the flags at the model's leading dimension (contents kept
// across capacity growth: ensure_cap moves them)
// Small buffers that every GEMM workgroup of the lattice step reads (the axis
// tables, the member lists): whole 2 MiB units, so that they sit in one large page
hipError_t hip_malloc_2m(void** p, size_t bytes) {
  const size_t unit = size_t(2) << 20;
  return hipMalloc(p, (bytes + unit - 1) / unit * unit);
}

int ensure_lat(mfgp_model* m, int64_t tiles, int ksplit, int ka, int64_t nzu) {
  hipStream_t s = m->ctx->stream;
  const int64_t ld = m->ld, tabw = lat_tabw(m);
  const bool ff = m->dtype == MFGP_F32;   // (F streamed in fp32: DESIGN.md section 2.3)
  if (!m->F || m->F_ld != ld || (ff && !m->Ff)) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->F) HIP_TRY(hipFree(m->F));
    if (m->Ff) HIP_TRY(hipFree(m->Ff));
    m->F = nullptr;
    m->Ff = nullptr;
    HIP_TRY(hipMalloc(&m->F, sizeof(double) * fblk_size(ld)));
    HIP_TRY(hipMemsetAsync(m->F, 0, sizeof(double) * fblk_size(ld), s));   // F's upper triangle stays zero
    if (ff) {
      HIP_TRY(hipMalloc(&m->Ff, sizeof(float) * fblk_size(ld)));
      HIP_TRY(hipMemsetAsync(m->Ff, 0, sizeof(float) * fblk_size(ld), s));
    }
    m->F_ld = ld;
    m->F_n = 0;
  }
  if (!m->tab || m->tab_ld != ld || m->tabw != tabw) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->tab) HIP_TRY(hipFree(m->tab));
    m->tab = nullptr;
    HIP_TRY(hipMalloc(&m->tab, sizeof(double) * 4 * ld * tabw));
    HIP_TRY(hipMemsetAsync(m->tab, 0, sizeof(double) * 4 * ld * tabw, s));
    if (m->lidx) HIP_TRY(hipFree(m->lidx));
    m->lidx = nullptr;
    HIP_TRY(hipMalloc(&m->lidx, sizeof(int) * ld));
    m->tab_ld = ld;
    m->tabw = tabw;
    m->tab_n = 0;
  }
  if (!m->wv || m->wv_ld != ld) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->wv) HIP_TRY(hipFree(m->wv));
    if (m->wflag) HIP_TRY(hipFree(m->wflag));
    if (m->wcnt) HIP_TRY(hipFree(m->wcnt));
    if (m->wpart) HIP_TRY(hipFree(m->wpart));
    m->wv = nullptr;
    m->wflag = nullptr;
    m->wcnt = nullptr;
    m->wpart = nullptr;
    HIP_TRY(hipMalloc(&m->wv, sizeof(double) * ld * KINC));
    HIP_TRY(hipMemsetAsync(m->wv, 0, sizeof(double) * ld * KINC, s));
    HIP_TRY(hipMalloc(&m->wflag, sizeof(unsigned) * (ld / 64 + 2)));
    HIP_TRY(hipMemsetAsync(m->wflag, 0, sizeof(unsigned) * (ld / 64 + 2), s));   // below every epoch
    HIP_TRY(hipMalloc(&m->wcnt, sizeof(unsigned) * 2 * (ld / 64 + 2)));
    HIP_TRY(hipMemsetAsync(m->wcnt, 0, sizeof(unsigned) * 2 * (ld / 64 + 2), s));
    HIP_TRY(hipMalloc(&m->wpart, sizeof(double) * 1024 * (LAT_WU_MAX + ld / 64 + 1)));
    m->wv_ld = ld;
  }
  if (m->gcnt_n != tiles) {
    // [tiles] arrival counters of the splits | [tiles] flags (the epoch once all arrived)
    HIP_TRY(hipStreamSynchronize(s));
    if (m->gcnt) HIP_TRY(hipFree(m->gcnt));
    m->gcnt = nullptr;
    HIP_TRY(hipMalloc(&m->gcnt, sizeof(unsigned) * 2 * tiles));
    HIP_TRY(hipMemsetAsync(m->gcnt, 0, sizeof(unsigned) * 2 * tiles, s));   // flags below every epoch
    m->gcnt_n = tiles;
  }
  // the fused var max / argmax: one (max, argmax) slot per GEMM workgroup
  if (m->tred && 2 * tiles * ksplit + 1 > m->tred_n) {
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipFree(m->tred));
    m->tred = nullptr;
    const int64_t nd = 2 * tiles * ksplit + 1;
    HIP_TRY(hipMalloc(&m->tred, sizeof(double) * nd));
    HIP_TRY(hipMemsetAsync(m->tred, 0, sizeof(double) * nd, s));
    m->tred_n = nd;
  }
  if (!m->axt || m->axt_w != tabw) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->axt) HIP_TRY(hipFree(m->axt));
    m->axt = nullptr;
    HIP_TRY(hip_malloc_2m(reinterpret_cast<void**>(&m->axt), sizeof(double) * 4 * (tabw + 1) * tabw));
    m->axt_w = tabw;
    m->axt_gen = UINT64_MAX;   // build before use
  }
  // Z rows: per part the lattice y-rows (padded to ZKS), then one per training row
  // that could lie off the lattice; zeros where never written (padding rows)
  const int64_t zrows = round_up(m->lat.ny, ZKS) + ld;
  if (!m->zb || m->zb_rows != zrows || m->zb_w != tabw || m->zb_ka < ka) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->zb) HIP_TRY(hipFree(m->zb));
    if (m->zvl) HIP_TRY(hipFree(m->zvl));
    m->zb = nullptr;
    m->zvl = nullptr;
    const size_t zn = (size_t)2 * zrows * tabw * ka;
    HIP_TRY(hipMalloc(&m->zb, sizeof(double) * zn));
    HIP_TRY(hipMemsetAsync(m->zb, 0, sizeof(double) * zn, s));
    HIP_TRY(hipMalloc(&m->zvl, sizeof(int) * 2 * (zrows + 1)));
    HIP_TRY(hipMemsetAsync(m->zvl, 0, sizeof(int) * 2 * (zrows + 1), s));
    m->zb_rows = zrows;
    m->zb_w = tabw;
    m->zb_ka = ka;
  }
  if (m->csr_n < csr_bytes(tabw, ld)) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->csr) HIP_TRY(hipFree(m->csr));
    m->csr = nullptr;
    m->csr_n = csr_bytes(tabw, ld);
    HIP_TRY(hip_malloc_2m(reinterpret_cast<void**>(&m->csr), m->csr_n));
  }
  if (!m->ldone) {
    HIP_TRY(hipMalloc(&m->ldone, sizeof(unsigned) * 4));
    HIP_TRY(hipMemsetAsync(m->ldone, 0, sizeof(unsigned) * 4, s));   // no arrivals; flags below every epoch
  }
  if (m->zflag_n < nzu + 2) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->zflag) HIP_TRY(hipFree(m->zflag));
    m->zflag = nullptr;
    HIP_TRY(hipMalloc(&m->zflag, sizeof(unsigned) * (nzu + 2)));
    HIP_TRY(hipMemsetAsync(m->zflag, 0, sizeof(unsigned) * (nzu + 2), s));   // below every epoch
    m->zflag_n = (nzu + 2);
  }
  const size_t need = ksplit > 1 ? (size_t)tiles * ksplit * 8192 : 0;   // LAT_PART doubles per split tile
  if (need > m->gpart_n) {
    HIP_TRY(hipStreamSynchronize(s));
    if (m->gpart) HIP_TRY(hipFree(m->gpart));
    m->gpart = nullptr;
    HIP_TRY(hipMalloc(&m->gpart, sizeof(double) * need));
    m->gpart_n = need;
  }
  return MFGP_OK;
}
void free_lat(mfgp_model* m) {
  if (m->csr) (void)hipFree(m->csr);
  if (m->F) (void)hipFree(m->F);
  if (m->Ff) (void)hipFree(m->Ff);
  if (m->tab) (void)hipFree(m->tab);
  if (m->wv) (void)hipFree(m->wv);
  if (m->wflag) (void)hipFree(m->wflag);
  if (m->wcnt) (void)hipFree(m->wcnt);
  if (m->wpart) (void)hipFree(m->wpart);
  if (m->gpart) (void)hipFree(m->gpart);
  if (m->gcnt) (void)hipFree(m->gcnt);
  if (m->res) (void)hipFree(m->res);
  if (m->lidx) (void)hipFree(m->lidx);
  if (m->axt) (void)hipFree(m->axt);
  if (m->zb) (void)hipFree(m->zb);
  if (m->zflag) (void)hipFree(m->zflag);
  if (m->ldone) (void)hipFree(m->ldone);
  if (m->zvl) (void)hipFree(m->zvl);
}

// Enqueue assembly + blocked Cholesky for `count` models (descriptors already uploaded).
int enqueue_factor(mfgp_ctx* c, const GPDesc* dd, const GPDesc* hd, int count) {
  int64_t max_nb = 0, max_tiles = 0;
  for (int i = 0; i < count; ++i) {
    const int64_t nb = nblocks_factor(hd[i].N);
    max_nb = std::max(max_nb, nb);
    max_tiles = std::max(max_tiles, nb * (nb + 1) / 2);
  }
  EvPair ev{};
  int rc = ev_begin(c, ev, 1);
  if (rc) return rc;
  HIP_TRY(launch_assemble(dd, count, max_tiles, c->stream));
  // Blocked right-looking Cholesky, per 64-column step: diagonal factor +
  // inverse (k_potrf_diag), panel (k_panel), trailing update. Two-level: the
  // steps of a group of FD (c->factor_depth) update only the group's own columns
  // (k_syrk_blk, one step deep), and the rest of the trailing matrix takes the
  // group's FD steps in one pass (k_syrk_blk, FD deep) -- bit-equal to the
  // one-level order, each trailing tile read and written once per group.
  const int FD = std::max(1, c->factor_depth);
  hipStream_t cs = c->stream;
  for (int64_t K0 = 0; K0 < max_nb; K0 += FD) {
    const int64_t K1 = std::min<int64_t>(K0 + FD, max_nb);
    for (int64_t kb = K0; kb < K1; ++kb) {
      HIP_TRY(launch_potrf_diag(dd, count, (int)kb, cs));
      const int64_t below = max_nb - kb - 1;
      if (below <= 0) continue;
      HIP_TRY(launch_panel(dd, count, (int)kb, below, cs));
      const int64_t jmax = std::min<int64_t>(K0 + FD - 1, max_nb - 1);
      if (FD == 1) {
        HIP_TRY(launch_syrk(dd, count, (int)kb, below * (below + 1) / 2, 0, cs));
      } else if (jmax >= kb + 1) {
        int64_t tiles = 0;
        for (int64_t j = kb + 1; j <= jmax; ++j) tiles += max_nb - j;
        HIP_TRY(launch_syrk_blk(dd, count, (int)kb, 1, (int)(kb + 1), (int)jmax, tiles, cs));
      }
    }
    const int64_t jmin = K0 + FD;
    if (FD > 1 && jmin < max_nb) {
      const int64_t T = max_nb - jmin;
      HIP_TRY(launch_syrk_blk(dd, count, (int)K0, (int)(K1 - K0), (int)jmin, INT32_MAX, T * (T + 1) / 2, cs));
    }
  }
  int64_t max_n = 0;
  for (int i = 0; i < count; ++i) max_n = std::max(max_n, hd[i].N);
  HIP_TRY(launch_extract_z(dd, count, max_n, c->stream));
  return ev_end(c, ev);
}

int enqueue_inc_factor(mfgp_ctx* c, const GPDesc* dd, const GPDesc* hd, int count) {
  int64_t max_np = 0;
  for (int i = 0; i < count; ++i) max_np = std::max<int64_t>(max_np, hd[i].nprod);
  EvPair ev{};
  int rc = ev_begin(c, ev, 1);
  if (rc) return rc;
  HIP_TRY(launch_inc_factor(dd, count, max_np, hd[0].vf32, c->stream));
  return ev_end(c, ev);
}

int enqueue_vstream(mfgp_ctx* c, const GPDesc* dd, const GPDesc* hd, int count) {
  int64_t max_ct = 0;
  for (int i = 0; i < count; ++i) max_ct = std::max(max_ct, ntiles_wg(hd[i].M, hd[i].rsplit, hd[i].vf32));
  if (max_ct == 0) return MFGP_OK;
  EvPair ev{};
  int rc = ev_begin(c, ev, 0);
  if (rc) return rc;
  HIP_TRY(launch_vstream(dd, count, max_ct, hd[0].vf32, c->stream));
  return ev_end(c, ev);
}

// fp64 V bytes of a full predict of descriptor d (k_predict's image of V).
size_t v64_bytes(const GPDesc& d) { return sizeof(double) * (size_t)ntiles_grid(d.M) * d.vld * PBM; }

// MFGP_F32 full predicts compute V in fp64 scratch (k_predict's left-looking
// solve re-reads its own rows) and round it into the resident fp32 V
// (k_vnarrow): point the descriptors at slots of the context's scratch, as many
// GPs per launch as F32_SCRATCH holds (at least one). Call before the upload.
int assign_predict_scratch(mfgp_ctx* c, GPDesc* hd, int count) {
  if (count <= 0 || !hd[0].vf32) return MFGP_OK;
  size_t per = 0;
  for (int i = 0; i < count; ++i) per = std::max(per, v64_bytes(hd[i]));
  per = (per + 255) / 256 * 256;
  if (per == 0) return MFGP_OK;
  int g = (int)std::max<size_t>(1, std::min<size_t>((size_t)count, F32_SCRATCH / per));
  if (per * g > c->vscr_bytes) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->vscr) HIP_TRY(hipFree(c->vscr));
    c->vscr = nullptr;
    c->vscr_bytes = 0;
    // at most half of the free HBM (the resident state of the models comes first);
    // mfgp_ctx_trim gives the scratch back
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && per * g > fr / 2)
      g = (int)std::max<size_t>(1, std::min<size_t>((size_t)g, fr / 2 / per));
    HIP_TRY(hipMalloc(&c->vscr, per * g));
    c->vscr_bytes = per * g;
  }
  c->f32_group = g;
  for (int i = 0; i < count; ++i) hd[i].V = c->vscr + (per / sizeof(double)) * (i % g);
  return MFGP_OK;
}

int enqueue_predict(mfgp_ctx* c, const GPDesc* dd, const GPDesc* hd, int count) {
  int64_t max_ct = 0;
  for (int i = 0; i < count; ++i) {
    max_ct = std::max(max_ct, ntiles_grid(hd[i].M));
    // k_predict addresses A through a 32-bit buffer descriptor: 8 * ld^2 < 2^31
    if (hd[i].ld > MAX_FULL_CAP + 64)
      return set_err(MFGP_ERR_ARG,
                     "the full predict supports a training capacity of at most %lld rows (this model's is %lld, N = %lld)",
                     (long long)MAX_FULL_CAP, (long long)(hd[i].ld - 1), (long long)hd[i].N);
  }
  if (max_ct == 0) return MFGP_OK;
  EvPair ev{};
  int rc = ev_begin(c, ev, 0);
  if (rc) return rc;
  if (!hd[0].vf32) {
    HIP_TRY(launch_predict(dd, count, max_ct, c->stream));
  } else {
    // groups sharing the scratch run one after the other (stream order)
    const int g = c->f32_group;
    for (int g0 = 0; g0 < count; g0 += g) {
      const int gn = std::min(g, count - g0);
      HIP_TRY(launch_predict(dd + g0, gn, max_ct, c->stream));
      HIP_TRY(launch_vnarrow(dd + g0, gn, max_ct, c->stream));
    }
  }
  return ev_end(c, ev);
}

int status_error(int st) {
  if (st == INT_MIN)   // wait_flag gave up (mfgp_kernels.hip): a hand-off inside k_inc_stream never arrived
    return set_err(MFGP_ERR_DEVICE, "device synchronisation timeout in the fused append+predict launch");
  return set_err(MFGP_ERR_NOT_PD, "Matrix is not positive definite (leading minor of order %d)", st);
}

int read_status(mfgp_model* m) {
  mfgp_ctx* c = m->ctx;
  int rc = ensure_h_status(c, 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->h_status, m->status, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const int st = c->h_status[0];
  if (st != INT_MAX) return status_error(st);
  return MFGP_OK;
}

bool is_device_ptr(const void* p);

// The model's mapped pinned result buffer [2][M] (spec_out): host-bound predict
// outputs are written there by the kernels over the bus and kept, so that the
// predicts of an unchanged model return them (the same bits, no launch).
// Result buffers handed over by mfgp_predict_view come back here (process-wide:
// a view may outlive its model and context); ensure_spec_out takes one of at least
// the size it needs before it allocates. Bounded: beyond VIEW_POOL_MAX the
// returned buffer is freed.
struct ViewBuf {
  double* host;
  int64_t cap;   // doubles per half ([2][cap]), then the trailer (max var, argmax) at [2 cap]
  int has_max;   // the trailer holds the fused max / argmax of the var half
};
std::mutex g_view_mu;
std::vector<ViewBuf> g_view_pool;
constexpr size_t VIEW_POOL_MAX = 8;
// bytes of T scratch the recursive-doubling F build may hold in the workspace
constexpr int64_t TRINV_WS_MAX = int64_t(2) << 30;

int ensure_spec_out(mfgp_model* m) {
  if (m->spec_out && m->spec_cap >= m->M) return MFGP_OK;
  mfgp_ctx* c = m->ctx;
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (m->spec_out) HIP_TRY(hipHostFree(m->spec_out));
  m->spec_out = nullptr;
  m->spec_out_dev = nullptr;
  m->spec_cap = 0;
  m->spec_valid = false;
  m->spec_max = false;
  {
    // best fit: the smallest pooled buffer that holds M (a small model does not take
    // the large buffer another model just returned)
    std::lock_guard<std::mutex> g(g_view_mu);
    size_t best = g_view_pool.size();
    for (size_t i = 0; i < g_view_pool.size(); ++i)
      if (g_view_pool[i].cap >= m->M && (best == g_view_pool.size() || g_view_pool[i].cap < g_view_pool[best].cap))
        best = i;
    if (best < g_view_pool.size()) {
      // (the pool's buffers are laid out [2][cap]: mu at 0, var at cap)
      m->spec_out = g_view_pool[best].host;
      m->spec_cap = g_view_pool[best].cap;
      g_view_pool.erase(g_view_pool.begin() + (long)best);
    }
  }
  if (m->spec_out) {
    void* dev = nullptr;
    HIP_TRY(hipHostGetDevicePointer(&dev, m->spec_out, 0));
    m->spec_out_dev = static_cast<double*>(dev);
    return MFGP_OK;
  }
  // portable: a pooled buffer may serve a model of a context on another device
  HIP_TRY(hipHostMalloc(&m->spec_out, sizeof(double) * (2 * (size_t)m->M + 2),
                        hipHostMallocMapped | hipHostMallocPortable));
  void* dev = nullptr;
  HIP_TRY(hipHostGetDevicePointer(&dev, m->spec_out, 0));
  m->spec_out_dev = static_cast<double*>(dev);
  m->spec_cap = m->M;
  return MFGP_OK;
}

// Where the predict kernels write mu / var: the caller's buffers when both are
// device memory, else the model's result buffer (model_out_done copies it out).
int model_out(mfgp_model* m, double* mu, double* var, double*& kmu, double*& kvar, bool& host) {
  host = !(is_device_ptr(mu) && is_device_ptr(var));
  if (!host) {
    kmu = mu;
    kvar = var;
    return MFGP_OK;
  }
  int rc = ensure_spec_out(m);
  if (rc) return rc;
  m->spec_max = false;   // (this predict computes no fused max into the trailer)
  kmu = m->spec_out_dev;
  kvar = m->spec_out_dev + m->spec_cap;
  return MFGP_OK;
}

void model_out_done(mfgp_model* m, double* mu, double* var, bool host) {
  if (!host) return;
  if (mu != m->spec_out) std::memcpy(mu, m->spec_out, sizeof(double) * m->M);
  if (var != m->spec_out + m->spec_cap) std::memcpy(var, m->spec_out + m->spec_cap, sizeof(double) * m->M);
  m->spec_valid = true;
}

int ensure_sync(mfgp_model* m) {
  if (m->sync) return MFGP_OK;
  HIP_TRY(hipMalloc(&m->sync, 4 * sizeof(unsigned)));
  HIP_TRY(hipMemsetAsync(m->sync, 0, 4 * sizeof(unsigned), m->ctx->stream));
  return MFGP_OK;
}

// Bordered appends and their one-pass predicts in one k_inc_stream launch.
int enqueue_inc_stream(mfgp_ctx* c, const GPDesc* dd, const GPDesc* hd, int count) {
  int64_t max_blocks = 0;
  for (int i = 0; i < count; ++i)
    max_blocks = std::max(max_blocks, hd[i].nprod + ntiles_wg(hd[i].M, hd[i].rsplit, hd[i].vf32));
  EvPair ev{};
  int rc = ev_begin(c, ev, 0);
  if (rc) return rc;
  HIP_TRY(launch_inc_stream(dd, count, max_blocks, hd[0].vf32, c->stream));
  return ev_end(c, ev);
}

// Lattice-separable appends + predicts (k_inc_lat), after the explicit inverses
// and the separable tables they need (k_trinv_f / k_lat_tables: only when a model
// enters the mode with a new factor, grid or hyperparameters).
int enqueue_inc_lat(mfgp_ctx* c, const GPDesc* dd, const GPDesc* hd, int count) {
  int64_t max_blocks = 0, max_nbr = 0, max_rows = 0, max_axw = 0, max_tiles = 0;
  for (int i = 0; i < count; ++i) {
    max_blocks = std::max<int64_t>(max_blocks, hd[i].nprod + hd[i].nwu + hd[i].nzu + (hd[i].lat_zcsr ? 2 : 0) +
                                                   (hd[i].lat_g2 ? 0 : (int64_t)hd[i].lat_tiles * hd[i].ksplit));
    max_tiles = std::max<int64_t>(max_tiles, hd[i].lat_tiles);
    if (hd[i].lat_fbuild) max_nbr = std::max(max_nbr, nblocks_rows(hd[i].n0));
    max_rows = std::max(max_rows, hd[i].n0 - hd[i].tab_lo);
    if (hd[i].lat_axbuild) max_axw = std::max(max_axw, hd[i].tabw);
  }
  // the builds a new factor / grid / hyperparameters need, timed as factor work
  // (mfgp_ctx_get_timing's factor counters)
  EvPair evb{};
  if (max_nbr > 0 || max_rows > 0 || max_axw > 0) {
    int rc = ev_begin(c, evb, 1);
    if (rc) return rc;
  }
  if (max_nbr > 0) {
    // recursive doubling needs a T scratch per GP (8 MB at n0 = 2048); MFGP_TRINV_COLUMNS=1:
    // the block-column form (diagnostics)
    const int64_t tstride = trinv_scratch(max_nbr);
    double* tscr = nullptr;
    // the scratch is bounded (TRINV_WS_MAX, and half the free HBM): a batch that needs
    // more runs in GP chunks (configs[4]: 32 GPs x 128 MiB at N = 8192 -> chunks of 8)
    int chunk = count;
    if (!c->trinv_columns) {
      size_t free_b = 0, total_b = 0;
      int64_t budget = TRINV_WS_MAX;
      if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
        budget = std::min<int64_t>(budget, (int64_t)((free_b + c->ws_bytes) / 2));
      const int64_t per_gp = (int64_t)sizeof(double) * tstride;
      chunk = (int)std::max<int64_t>(1, std::min<int64_t>(count, budget / std::max<int64_t>(per_gp, 1)));
      int rc = ensure_ws(c, sizeof(double) * (size_t)(tstride * chunk));
      if (rc) return rc;
      tscr = c->ws;
    }
    for (int i0 = 0; i0 < count; i0 += chunk)
      HIP_TRY(launch_trinv_f(dd + i0, std::min(chunk, count - i0), max_nbr, tscr, tstride, c->stream));
    // MFGP_F32: the copy the lattice step streams, rounded once per build
    if (hd[0].vf32) {
      int64_t max_el = 0;
      for (int i = 0; i < count; ++i)
        if (hd[i].lat_fbuild) max_el = std::max<int64_t>(max_el, fblk_size(hd[i].ld));
      HIP_TRY(launch_narrow_f(dd, count, max_el, c->stream));
    }
  }
  if (max_rows > 0) HIP_TRY(launch_lat_tables(dd, count, max_rows, c->stream));
  if (max_axw > 0) HIP_TRY(launch_lat_axes(dd, count, max_axw, c->stream));
  {
    int rc = ev_end(c, evb);
    if (rc) return rc;
  }
  EvPair ev{};
  int rc = ev_begin(c, ev, 0);
  if (rc) return rc;
  HIP_TRY(launch_inc_lat(dd, count, max_blocks, hd[0].ka, hd[0].vf32, !hd[0].lat_g2, c->stream));
  if (hd[0].lat_g2) HIP_TRY(launch_lat_gemm2(dd, count, max_tiles, hd[0].ka, hd[0].vf32, c->stream));
  return ev_end(c, ev);
}

// A batch step that is one launch takes its host descriptors by value
// (k_inc_stream_arg, k_inc_lat_arg). The lattice step alone (k_inc_lat_arg):
// for a batch step that needs nothing else on the device -- no F / table / axis
// builds, no other appends or predicts -- so the descriptor array is not uploaded.
bool desc_arg_ok(const mfgp_ctx* c, const GPDesc* hd, int count) {
  if (!c->desc_arg || count < 1 || count > DESC_ARG_MAX) return false;
  for (int i = 0; i < count; ++i)
    if (hd[i].lat_fbuild || hd[i].n0 > hd[i].tab_lo || hd[i].lat_axbuild) return false;
  return true;
}

int enqueue_inc_stream_arg(mfgp_ctx* c, const GPDesc* hd, int count) {
  int64_t max_blocks = 0;
  for (int i = 0; i < count; ++i)
    max_blocks = std::max(max_blocks, hd[i].nprod + ntiles_wg(hd[i].M, hd[i].rsplit, hd[i].vf32));
  EvPair ev{};
  int rc = ev_begin(c, ev, 0);
  if (rc) return rc;
  HIP_TRY(launch_inc_stream_arg(hd, count, max_blocks, hd[0].vf32, c->stream));
  return ev_end(c, ev);
}

int enqueue_inc_lat_arg(mfgp_ctx* c, const GPDesc* hd, int count) {
  int64_t max_blocks = 0, max_tiles = 0;
  for (int i = 0; i < count; ++i) {
    max_blocks = std::max<int64_t>(max_blocks, hd[i].nprod + hd[i].nwu + hd[i].nzu + (hd[i].lat_zcsr ? 2 : 0) +
                                                   (hd[i].lat_g2 ? 0 : (int64_t)hd[i].lat_tiles * hd[i].ksplit));
    max_tiles = std::max<int64_t>(max_tiles, hd[i].lat_tiles);
  }
  EvPair ev{};
  int rc = ev_begin(c, ev, 0);
  if (rc) return rc;
  HIP_TRY(launch_inc_lat_arg(hd, count, max_blocks, hd[0].ka, hd[0].vf32, !hd[0].lat_g2, c->stream));
  if (hd[0].lat_g2) HIP_TRY(launch_lat_gemm2_arg(hd, count, max_tiles, hd[0].ka, hd[0].vf32, c->stream));
  return ev_end(c, ev);
}

// Row splits of the one-pass predict for a launch over these descriptors: 128-cell
// workgroups while they fill the chip (~4 per CU), else 64 or 32 cells with the
// rows split 2 or 4 ways (the drop-in simulator predicts one GP at a time).
void set_rsplit(const mfgp_ctx* c, GPDesc* hd, int count) {
  if (count > 0 && hd[0].vf32) {   // the fp32 stream has no row splits
    for (int i = 0; i < count; ++i) hd[i].rsplit = 1;
    return;
  }
  int64_t w1 = 0;
  for (int i = 0; i < count; ++i) w1 += ntiles_wg(hd[i].M);
  int R = (w1 >= 3 * c->ncu) ? 1 : (2 * w1 >= 3 * c->ncu ? 2 : 4);
  if (c->rsplit_force > 0) R = c->rsplit_force;   // (diagnostics: MFGP_RSPLIT)
  for (int i = 0; i < count; ++i) hd[i].rsplit = R;
}

bool hyp_same(const mfgp_model* m) {
  return m->factor_jitter == m->jitter && std::memcmp(m->factor_hyp, m->hyp, sizeof(m->hyp)) == 0;
}

bool factor_current(const mfgp_model* m) {
  return m->factored && m->factor_N == m->NL + m->NH && hyp_same(m);
}

// Rows [factor_N, N) can be appended to the current factor (k_inc_factor).
bool can_inc_factor(const mfgp_model* m) {
  const int64_t N = m->NL + m->NH;
  return m->ctx->incremental && m->factored && hyp_same(m) && m->factor_N < N && N - m->factor_N <= KINC;
}

// Predict by one pass over the resident V (k_vstream): V valid for rows < v_n,
// at most KINC factor rows beyond it (the factor must be current).
bool can_vstream(const mfgp_model* m) {
  const int64_t N = m->NL + m->NH;
  return m->ctx->incremental && m->M > 0 && m->V && m->vtiles >= ntiles_grid(m->M) && m->v_n <= N &&
         N - m->v_n <= KINC;
}

void mark_full_factor(mfgp_model* m) {
  m->n_full_factor += 1;
  m->gen += 1;   // a factor from scratch: new rounding of everything derived from it
  m->factored = true;
  m->factor_N = m->NL + m->NH;
  std::memcpy(m->factor_hyp, m->hyp, sizeof(m->hyp));
  m->factor_jitter = m->jitter;
  m->ablk = std::max(m->ablk, nblocks_factor(m->factor_N));
  m->v_n = 0;   // V belonged to the previous factor
  m->l21c_N = -1;
}

void mark_inc_factor(mfgp_model* m) {
  m->n_inc_factor += 1;
  m->factor_N = m->NL + m->NH;
  m->ablk = std::max(m->ablk, nblocks_factor(m->factor_N));
}

// Descriptor of a bordered append of rows [factor_N, N) (k_inc_stream; the
// caller sets tiles = 1 and the predict outputs to stream the cells too).
int fill_inc_desc(GPDesc& d, mfgp_model* m) {
  int rc = ensure_sync(m);
  if (rc) return rc;
  fill_desc(d, m);
  d.n0 = m->factor_N;
  d.vres = m->V ? m->v_n : 0;
  d.sync = m->sync;
  if (++m->epoch == 0) m->epoch = 1;
  d.epoch = m->epoch;
  d.nprod = (int)fused_producers(d.n0);
  d.l21c_ok = 1;   // the producers write the compact rows for (n0, N)
  m->l21c_n0 = d.n0;
  m->l21c_N = d.N;
  return MFGP_OK;
}

// One-pass predict over the V rows [0, v_n): the compact rows serve it when the
// last bordered append wrote them for exactly these rows.
void set_vstream_rows(GPDesc& d, const mfgp_model* m) {
  d.n0 = m->v_n;
  d.l21c_ok = (m->l21c_n0 == m->v_n && m->l21c_N == m->NL + m->NH) ? 1 : 0;
}

// Factor one model now (synchronous, status checked).
int factor_one(mfgp_model* m) {
  mfgp_ctx* c = m->ctx;
  int rc = ensure_cap(m, m->NL + m->NH);
  if (rc) return rc;
  int slot;
  GPDesc* hd = acquire_slot(c, slot, rc);
  if (!hd) return rc;
  fill_desc(hd[0], m);
  const GPDesc* dd = nullptr;
  if ((rc = upload_slot(c, slot, 1, &dd))) return rc;
  if ((rc = enqueue_factor(c, dd, hd, 1))) return rc;
  if ((rc = release_slot(c, slot))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  mark_full_factor(m);
  rc = read_status(m);
  m->factored = (rc == MFGP_OK);
  return rc;
}

// Bring the factor up to date for all N rows: bordered append of the rows
// beyond factor_N when possible, else a full refactor (synchronous).
int update_factor(mfgp_model* m) {
  if (factor_current(m)) return MFGP_OK;
  if (!can_inc_factor(m)) return factor_one(m);
  mfgp_ctx* c = m->ctx;
  int rc, slot;
  GPDesc* hd = acquire_slot(c, slot, rc);
  if (!hd) return rc;
  if ((rc = fill_inc_desc(hd[0], m))) return rc;
  const GPDesc* dd = nullptr;
  if ((rc = upload_slot(c, slot, 1, &dd))) return rc;
  if ((rc = enqueue_inc_factor(c, dd, hd, 1))) return rc;
  if ((rc = release_slot(c, slot))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  mark_inc_factor(m);
  rc = read_status(m);
  m->factored = (rc == MFGP_OK);
  return rc;
}

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice;
}

int copy_rows(mfgp_model* m, int64_t at, const double* X, const double* y, int64_t k) {
  if (k <= 0) return MFGP_OK;
  if (!X || !y) return set_err(MFGP_ERR_ARG, "null data pointer with k=%lld", (long long)k);
  HIP_TRY(hipMemcpyAsync(m->X + 2 * at, X, sizeof(double) * 2 * k, hipMemcpyDefault, m->ctx->stream));
  HIP_TRY(hipMemcpyAsync(m->y + at, y, sizeof(double) * k, hipMemcpyDefault, m->ctx->stream));
  return MFGP_OK;
}

}  // namespace

extern "C" {

const char* mfgp_last_error(void) { return g_err.c_str(); }

#ifdef MFGP_STAMPS
// diagnostic builds only (tools/): device buffer for the kernels' phase stamps
int mfgp_debug_set_stamps(void* p) {
  HIP_TRY(set_stamps((long long*)p));
  return MFGP_OK;
}
#endif
const char* mfgp_version(void) { return "mfgp_hip 0.3 gfx950 f64 f32v"; }

int mfgp_ctx_create(int device, mfgp_ctx** out) {
  const DeviceGuard dg_(device);
  if (!out) return set_err(MFGP_ERR_ARG, "null out");
  *out = nullptr;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return set_err(MFGP_ERR_ARG, "device %d out of range (%d devices)", device, n);
  mfgp_ctx* c = new mfgp_ctx();
  c->device = device;
  HIP_TRY(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
      c->ncu = ncu;
  }
  c->stream = c->own;
  if (const char* e = std::getenv("MFGP_DESC_ARG")) c->desc_arg = std::atoi(e) != 0;
  if (const char* e = std::getenv("MFGP_SPIN_US")) c->spin_us = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("MFGP_EARLY_PD")) c->early_pd = std::atoi(e) != 0;
  if (const char* e = std::getenv("MFGP_LAT_ZCSR")) c->lat_zcsr = std::atoi(e) != 0 ? 1 : 0;
  if (const char* e = std::getenv("MFGP_RSPLIT")) {
    const int r = std::atoi(e);
    c->rsplit_force = (r == 1 || r == 2 || r == 4) ? r : 0;
  }
  if (const char* e = std::getenv("MFGP_LAT_KSPLIT")) c->lat_ksplit = std::max(0, std::min(8, std::atoi(e)));
  if (const char* e = std::getenv("MFGP_LAT_WU")) c->lat_wu = std::max(0, std::atoi(e));
  if (const char* e = std::getenv("MFGP_LAT_SELFG")) c->lat_selfg = std::atoi(e) != 0;
  if (const char* e = std::getenv("MFGP_LAT_GEMM2")) c->lat_gemm2 = std::atoi(e) != 0 ? 1 : 0;
  if (const char* e = std::getenv("MFGP_TRINV_COLUMNS")) c->trinv_columns = std::atoi(e) != 0;
  if (const char* e = std::getenv("MFGP_FACTOR_DEPTH")) c->factor_depth = std::max(1, std::min(16, std::atoi(e)));
  // A/B runs: MFGP_LATTICE = 0 (V stream only), 1 (default), 2 (lattice without the size gate)
  if (const char* e = std::getenv("MFGP_LATTICE")) {
    const int v = std::atoi(e);
    c->lattice = v != 0;
    c->lat_force = v == 2;
  }
  HIP_TRY(hipHostMalloc(&c->h_ring, sizeof(GPDesc) * RING * MAXB, hipHostMallocDefault));
  HIP_TRY(hipMalloc(&c->d_ring, sizeof(GPDesc) * RING * MAXB));
  for (int i = 0; i < RING; ++i) {
    HIP_TRY(hipEventCreateWithFlags(&c->ring_ev[i], hipEventDisableTiming));
    c->ring_used[i] = false;
  }
  *out = c;
  return MFGP_OK;
}

void mfgp_ctx_destroy(mfgp_ctx* c) {
  const DeviceGuard dg_(c ? c->device : -1);
  (void)settle(c);
  if (!c) return;
  (void)hipStreamSynchronize(c->stream);
  (void)drain_timing(c);
  for (auto e : c->pool) (void)hipEventDestroy(e);
  for (int i = 0; i < RING; ++i) (void)hipEventDestroy(c->ring_ev[i]);
  if (c->ws) (void)hipFree(c->ws);
  if (c->vscr) (void)hipFree(c->vscr);
  if (c->d_ring) (void)hipFree(c->d_ring);
  if (c->h_status) (void)hipHostFree(c->h_status);
  if (c->h_ring) (void)hipHostFree(c->h_ring);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

int mfgp_ctx_trim(mfgp_ctx* c) {
  const DeviceGuard dg_(c ? c->device : -1);
  if (const int rc_ = settle(c)) return rc_;
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (c->vscr) HIP_TRY(hipFree(c->vscr));
  c->vscr = nullptr;
  c->vscr_bytes = 0;
  if (c->ws) HIP_TRY(hipFree(c->ws));
  c->ws = nullptr;
  c->ws_bytes = 0;
  return MFGP_OK;
}

int mfgp_ctx_set_stream(mfgp_ctx* c, void* s) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->stream = s ? (hipStream_t)s : c->own;
  return MFGP_OK;
}

void* mfgp_ctx_get_stream(mfgp_ctx* c) { return c ? (void*)c->stream : nullptr; }

int mfgp_ctx_synchronize(mfgp_ctx* c) {
  const DeviceGuard dg_(c ? c->device : -1);
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  c->early_running = false;
  int rc = ensure_h_status(c, c->async_status.size());
  if (rc) return rc;
  // the status words come back through pinned memory with the stream's last copies
  // (or straight from the mapped word the launch itself published them into)
  bool all_mapped = !c->async_status.empty();
  for (size_t i = 0; i < c->async_status.size(); ++i)
    if (!c->async_status[i].host) {
      all_mapped = false;
      HIP_TRY(hipMemcpyAsync(c->h_status + i, c->async_status[i].dev, sizeof(int), hipMemcpyDeviceToHost,
                             c->stream));
    }
  if (all_mapped && c->spin_us > 0) {
    // launches that publish their status into mapped host memory as their last act
    // (the one-GP fused step: the drop-in simulator's updt_hifi): poll those words
    // first, so that the stream synchronisation below starts when the kernel is
    // about to end and returns within its active-wait phase instead of sleeping
    // through the kernel and waking late (the outputs are visible only after it)
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < c->async_status.size(); ++i) {
      const volatile int* w = reinterpret_cast<const volatile int*>(c->async_status[i].host);
      while (*w == STATUS_UNSET) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(c->spin_us)) break;
      }
    }
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (size_t i = 0; i < c->async_status.size(); ++i) {
    const auto& as = c->async_status[i];
    if (as.host) {
      c->h_status[i] = *reinterpret_cast<volatile int*>(as.host);
      if (c->h_status[i] == STATUS_UNSET)   // not published (cannot happen with cell tiles): read the word
        HIP_TRY(hipMemcpy(c->h_status + i, as.dev, sizeof(int), hipMemcpyDeviceToHost));
    }
  }
  for (size_t i = 0; i < c->async_status.size(); ++i) {
    const int st = c->h_status[i];
    if (st == INT_MAX) continue;
    // a failed factor leaves its model without one: the next use refactors (and
    // raises again), instead of serving the failed factor and its V
    mfgp_model* m = c->async_status[i].m;
    m->factored = false;
    m->v_n = 0;
    m->l21c_N = -1;
    m->spec_valid = false;
    if (rc == MFGP_OK) rc = status_error(st);
  }
  c->async_status.clear();
  return rc;
}

int mfgp_ctx_set_incremental(mfgp_ctx* c, int enable) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->incremental = enable != 0;
  return MFGP_OK;
}

int mfgp_ctx_set_fused(mfgp_ctx* c, int enable) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->fused = enable != 0;
  return MFGP_OK;
}

int mfgp_ctx_set_deferred_appends(mfgp_ctx* c, int enable) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->deferred = enable != 0;
  return MFGP_OK;
}

int mfgp_ctx_set_lattice(mfgp_ctx* c, int enable) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->lattice = enable != 0;
  c->lat_force = enable == 2;
  return MFGP_OK;
}

int mfgp_ctx_set_concurrent(mfgp_ctx* c, int enable) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->concurrent = enable != 0;
  return MFGP_OK;
}

int mfgp_ctx_enable_timing(mfgp_ctx* c, int enable) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  c->timing = (enable == 2) ? 2 : (enable != 0 ? 1 : 0);
  return MFGP_OK;
}

int mfgp_ctx_set_timing_stride(mfgp_ctx* c, int64_t stride) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  if (stride < 1) return set_err(MFGP_ERR_ARG, "timing stride must be >= 1");
  c->timing_stride = stride;
  c->timing_seq = 0;
  return MFGP_OK;
}

int mfgp_ctx_get_timing(mfgp_ctx* c, double* pm, int64_t* pn, double* fm, int64_t* fn) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  int rc = drain_timing(c);
  if (rc) return rc;
  if (pm) *pm = c->t_predict;
  if (pn) *pn = c->n_predict;
  if (fm) *fm = c->t_factor;
  if (fn) *fn = c->n_factor;
  return MFGP_OK;
}

int mfgp_ctx_reset_timing(mfgp_ctx* c) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  int rc = drain_timing(c);
  c->t_predict = c->t_factor = 0.0;
  c->n_predict = c->n_factor = 0;
  return rc;
}

int mfgp_model_create(mfgp_ctx* c, int kind, int dtype, const double* hyp, int nhyp, double jitter,
                      mfgp_model** out) {
  const DeviceGuard dg_(c ? c->device : -1);
  if (const int rc_ = settle(c)) return rc_;
  if (!c || !out) return set_err(MFGP_ERR_ARG, "null ctx/out");
  *out = nullptr;
  if (kind != MFGP_SF && kind != MFGP_MF) return set_err(MFGP_ERR_ARG, "kind must be MFGP_SF or MFGP_MF");
  if (dtype != MFGP_F64 && dtype != MFGP_F32) return set_err(MFGP_ERR_ARG, "dtype must be MFGP_F64 or MFGP_F32");
  const int want = kind == MFGP_SF ? 4 : 9;
  if (!hyp || nhyp != want)
    return set_err(MFGP_ERR_ARG, "Hyperparameters must be of length 4 (single-fidelity) or 9 (multi-fidelity)");
  mfgp_model* m = new mfgp_model();
  m->ctx = c;
  m->kind = kind;
  m->dtype = dtype;
  m->nhyp = nhyp;
  std::memcpy(m->hyp, hyp, sizeof(double) * nhyp);
  m->jitter = jitter;
  HIP_TRY(hipMalloc(&m->status, sizeof(int)));
  {
    // "no failure" until a step writes it: a step whose kernels all skip (a gated
    // model of mfgp_batch_sample_points) must not read an uninitialised word
    const int ok = INT_MAX;
    HIP_TRY(hipMemcpy(m->status, &ok, sizeof(int), hipMemcpyHostToDevice));
  }
  int rc = ensure_cap(m, 63);
  if (rc) {
    mfgp_model_destroy(m);
    return rc;
  }
  *out = m;
  return MFGP_OK;
}

void mfgp_model_destroy(mfgp_model* m) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  (void)settle(m ? m->ctx : nullptr);
  if (!m) return;
  if (m->ctx) {
    (void)hipStreamSynchronize(m->ctx->stream);
    // an ASYNC batch's status word of this model dies with it (the work is done)
    auto& as = m->ctx->async_status;
    as.erase(std::remove_if(as.begin(), as.end(), [m](const mfgp_ctx::AsyncStatus& e) { return e.m == m; }),
             as.end());
  }
  if (m->spec_out) (void)hipHostFree(m->spec_out);
  if (m->status_host) (void)hipHostFree(m->status_host);
  if (m->X) (void)hipFree(m->X);
  if (m->y) (void)hipFree(m->y);
  if (m->A) (void)hipFree(m->A);
  if (m->Linv) (void)hipFree(m->Linv);
  if (m->zv) (void)hipFree(m->zv);
  if (m->iscr) (void)hipFree(m->iscr);
  if (m->status) (void)hipFree(m->status);
  if (m->grid) (void)hipFree(m->grid);
  if (m->V) (void)hipFree(m->V);
  if (m->tred) (void)hipFree(m->tred);
  if (m->sync) (void)hipFree(m->sync);
  free_lat(m);
  delete m;
}

int mfgp_ctx_planner_stats(mfgp_ctx* c, int64_t* out, int n, int reset) {
  if (!c || (n > 0 && !out)) return set_err(MFGP_ERR_ARG, "null ctx/out");
  if (const int rc_ = settle(c)) return rc_;   // (a running early-return launch first)
  for (int i = 0; i < n && i < PLAN_NSTATS; ++i) out[i] = c->plan_stats[i];
  if (reset)
    for (int64_t& v : c->plan_stats) v = 0;
  return MFGP_OK;
}

int mfgp_clone(const mfgp_model* src, mfgp_model** out) {
  const DeviceGuard dg_(src ? src->ctx->device : -1);
  if (const int rc_ = settle(src ? src->ctx : nullptr)) return rc_;
  int rc = check_model(src);
  if (rc) return rc;
  if (!out) return set_err(MFGP_ERR_ARG, "null out");
  mfgp_ctx* c = src->ctx;
  mfgp_model* m = nullptr;
  if ((rc = mfgp_model_create(c, src->kind, src->dtype, src->hyp, src->nhyp, src->jitter, &m))) return rc;
  if ((rc = ensure_cap(m, src->cap))) {
    mfgp_model_destroy(m);
    return rc;
  }
  // same capacity => same ld: the factor copies verbatim
  const int64_t n = src->NL + src->NH;
  m->NL = src->NL;
  m->NH = src->NH;
  if (n > 0) {
    HIP_TRY(hipMemcpyAsync(m->X, src->X, sizeof(double) * 2 * n, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(m->y, src->y, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream));
  }
  if (src->factored && src->ld == m->ld) {
    HIP_TRY(hipMemcpyAsync(m->A, src->A, sizeof(double) * src->ld * src->ld, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(m->Linv, src->Linv, sizeof(double) * (src->ld / NB) * TILE, hipMemcpyDeviceToDevice,
                           c->stream));
    HIP_TRY(hipMemcpyAsync(m->zv, src->zv, sizeof(double) * src->cap, hipMemcpyDeviceToDevice, c->stream));
    m->factored = true;
    m->factor_N = src->factor_N;
    m->ablk = src->ablk;
    std::memcpy(m->factor_hyp, src->factor_hyp, sizeof(m->factor_hyp));
    m->factor_jitter = src->factor_jitter;
  }
  if (src->M > 0) {
    HIP_TRY(hipMalloc(&m->grid, sizeof(double) * 2 * src->M));
    HIP_TRY(hipMemcpyAsync(m->grid, src->grid, sizeof(double) * 2 * src->M, hipMemcpyDeviceToDevice, c->stream));
    m->M = m->Mcap = src->M;
    m->lat = src->lat;
    // resident V (a deepcopy'd model keeps appending to the copy, sim:339)
    if (m->factored && src->V && src->v_n > 0 && src->vld == round_up(m->cap, PRB)) {
      if ((rc = ensure_v(m))) return rc;
      HIP_TRY(hipMemcpyAsync(m->V, src->V, v_elem(src) * (size_t)src->vtiles * src->vld * PBM,
                             hipMemcpyDeviceToDevice, c->stream));
      m->v_n = src->v_n;
    }
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  *out = m;
  return MFGP_OK;
}

int mfgp_model_set_hyp(mfgp_model* m, const double* hyp, int nhyp, double jitter) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if (!hyp || nhyp != m->nhyp)
    return set_err(MFGP_ERR_ARG, "Hyperparameters must be of length 4 (single-fidelity) or 9 (multi-fidelity)");
  if (jitter != m->jitter || std::memcmp(hyp, m->hyp, sizeof(double) * nhyp) != 0) {
    m->spec_valid = false;
    m->gen += 1;
  }
  std::memcpy(m->hyp, hyp, sizeof(double) * nhyp);
  m->jitter = jitter;
  return MFGP_OK;
}

// Is the grid a lattice of two strictly monotone axes, one coordinate constant
// along runs of consecutive cells (meshgrid order, either way round)?
GridLattice detect_lattice(const double* g, int64_t M) {
  GridLattice L{};
  if (M < 1 || M > INT_MAX) return L;
  auto monotone = [](const double* v, int64_t n, int64_t stride) {
    if (n < 2) return v[0] == v[0];
    const bool up = v[stride] > v[0];
    for (int64_t i = 1; i < n; ++i) {
      const double a = v[(i - 1) * stride], b = v[i * stride];
      if (!(up ? b > a : b < a)) return false;
    }
    return true;
  };
  for (int s = 0; s < 2; ++s) {       // s = the coordinate constant along a run
    const int f = 1 - s;
    int64_t run = 1;
    while (run < M && g[2 * run + s] == g[s]) ++run;
    if (M % run) continue;
    bool ok = true;
    for (int64_t i = 0; i < M && ok; ++i)
      ok = g[2 * i + s] == g[2 * (i - i % run) + s] && g[2 * i + f] == g[2 * (i % run) + f];
    const int64_t ns = M / run;
    if (!ok || !monotone(g + s, ns, 2 * run) || !monotone(g + f, run, 2)) continue;
    // slow axis: values g[2 j run + s], stride run; fast axis: g[2 j + f], stride 1
    const int64_t xn = s == 0 ? ns : run, xst = s == 0 ? run : 1;
    const int64_t yn = s == 0 ? run : ns, yst = s == 0 ? 1 : run;
    const double x0 = g[0], x1 = g[2 * (xn - 1) * xst];
    const double y0 = g[1], y1 = g[2 * (yn - 1) * yst + 1];
    L.nx = (int)xn;
    L.ny = (int)yn;
    L.sx = xst;
    L.sy = yst;
    L.x0 = x0;
    L.y0 = y0;
    L.xinv = xn > 1 ? (double)(xn - 1) / (x1 - x0) : 0.0;
    L.yinv = yn > 1 ? (double)(yn - 1) / (y1 - y0) : 0.0;
    return L;
  }
  return L;
}

int mfgp_set_grid(mfgp_model* m, const double* xs, int64_t M) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if (M < 0 || (M > 0 && !xs)) return set_err(MFGP_ERR_ARG, "bad grid");
  mfgp_ctx* c = m->ctx;
  m->v_n = 0;   // V columns belong to the previous grid
  m->spec_valid = false;
  m->gen += 1;
  if (M > m->Mcap) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (m->grid) HIP_TRY(hipFree(m->grid));
    m->grid = nullptr;
    HIP_TRY(hipMalloc(&m->grid, sizeof(double) * 2 * M));
    m->Mcap = M;
  }
  m->M = M;
  if (M > 0) HIP_TRY(hipMemcpyAsync(m->grid, xs, sizeof(double) * 2 * M, hipMemcpyDefault, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  m->lat = GridLattice{};
  if (M > 0) {
    std::vector<double> h(2 * (size_t)M);
    HIP_TRY(hipMemcpy(h.data(), m->grid, sizeof(double) * 2 * M, hipMemcpyDeviceToHost));
    m->lat = detect_lattice(h.data(), M);
  }
  return MFGP_OK;
}

int mfgp_set_data(mfgp_model* m, const double* XL, const double* yL, int64_t NL, const double* XH,
                  const double* yH, int64_t NH) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if (NL < 0 || NH < 0) return set_err(MFGP_ERR_ARG, "negative sizes");
  if (m->kind == MFGP_SF && NL != 0) return set_err(MFGP_ERR_ARG, "SF model takes its data in the H slots");
  m->spec_valid = false;
  if ((rc = ensure_cap(m, NL + NH))) return rc;
  m->NL = NL;
  m->NH = NH;
  if ((rc = copy_rows(m, 0, XL, yL, NL))) return rc;
  if ((rc = copy_rows(m, NL, XH, yH, NH))) return rc;
  m->factored = false;
  return factor_one(m);
}

int spec_append_predict(mfgp_model* m, const double* X, const double* y, int64_t k);

int mfgp_append(mfgp_model* m, const double* X, const double* y, int64_t k) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if (k < 0) return set_err(MFGP_ERR_ARG, "negative k");
  m->spec_valid = false;
  const bool spec = m->pred_since_append;   // the last append was followed by a predict
  m->pred_since_append = false;
  const int64_t n = m->NL + m->NH;
  if ((rc = ensure_cap(m, n + k))) return rc;
  if (k > 0 && (!X || !y)) return set_err(MFGP_ERR_ARG, "null data pointer with k=%lld", (long long)k);
  m->NH += k;
  if (!m->ctx->incremental) m->factored = false;   // reference behaviour: refactor from scratch
  const bool staged = m->ctx->deferred && can_inc_factor(m);   // the next factor user runs the append
  const bool sp = !staged && spec && m->ctx->fused && k > 0 && m->M > 0 && can_inc_factor(m) && m->V &&
                  m->v_n == m->factor_N && m->vtiles >= ntiles_grid(m->M);
  m->NH -= k;
  // the speculative step carries the rows in its launch (batch_run appends them)
  if (sp) return spec_append_predict(m, X, y, k);
  if ((rc = copy_rows(m, n, X, y, k))) return rc;
  m->NH += k;
  if (staged) return MFGP_OK;
  return update_factor(m);
}

int mfgp_truncate(mfgp_model* m, int64_t n_keep_hifi) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if (n_keep_hifi != m->NH) m->spec_valid = false;
  if (n_keep_hifi < 0 || n_keep_hifi > m->NH) return set_err(MFGP_ERR_ARG, "bad truncate size");
  if (n_keep_hifi != m->NH) {
    m->NH = n_keep_hifi;
    // the factor, z and V of the leading rows do not depend on later rows
    const int64_t N = m->NL + m->NH;
    if (m->factored && m->factor_N > N) m->factor_N = N;
    m->v_n = std::min(m->v_n, N);
    m->F_n = std::min(m->F_n, N);
    m->tab_n = std::min(m->tab_n, N);
    for (int b = 0; b < 2; ++b)
      if (m->res_n[b] > N) m->res_n[b] = -1;   // the posterior of rows that are gone
  }
  return MFGP_OK;
}

int mfgp_batch_truncate(mfgp_model** models, int count, int64_t n_keep_hifi) {
  const DeviceGuard dg_((models && count > 0 && models[0]) ? models[0]->ctx->device : -1);
  if (const int rc_ = settle((models && count > 0 && models[0]) ? models[0]->ctx : nullptr)) return rc_;
  if (count < 0 || (count > 0 && !models)) return set_err(MFGP_ERR_ARG, "bad batch");
  for (int i = 0; i < count; ++i) {
    const int rc = mfgp_truncate(models[i], n_keep_hifi);
    if (rc) return rc;
  }
  return MFGP_OK;
}

static int batch_run(mfgp_model** models, int count, const double* X, const double* y, const int64_t* k,
                     double* mu, double* var, double* vmax, int64_t* vargmax, int flags, bool do_factor,
                     bool do_predict, const int64_t* out_offs = nullptr, const int* vidx = nullptr);

// The speculative form of an eager append (mfgp_append): the bordered append and
// the one-pass predict as one launch, synchronised (a non-PD step is reported
// here, as by update_factor), with mu | var kept for the next predict.
int spec_append_predict(mfgp_model* m, const double* X, const double* y, int64_t k) {
  mfgp_ctx* c = m->ctx;
  int rc = settle(c);
  if (rc == MFGP_OK) rc = ensure_spec_out(m);
  if (rc) return rc;
  if (m->status_host) reinterpret_cast<volatile int*>(m->status_host)[1] = STATUS_UNSET;
  // (the fused var max / argmax into the buffer's trailer: the launch's last cell
  // group reduces the groups' partials for the status word anyway)
  double* tr = m->spec_out_dev + 2 * m->spec_cap;
  m->spec_max = false;
  rc = batch_run(&m, 1, X, y, &k, m->spec_out_dev, m->spec_out_dev + m->spec_cap, tr,
                 reinterpret_cast<int64_t*>(tr + 1), MFGP_ASYNC, true, true);
  if (rc == MFGP_OK) m->spec_max = true;
  if (rc == MFGP_OK && c->early_pd && c->spin_us > 0 && m->status_host && c->async_status.size() == 1 &&
      c->async_status[0].host == m->status_host) {
    // the launch publishes the L22 verdict of the step (the only status its
    // factor can fail with) into the model's second mapped word: a positive
    // definite step returns now, and the next entry point settles the launch
    // (its outputs, hang guards) before anything reads or reuses its buffers
    const volatile int* w = reinterpret_cast<const volatile int*>(m->status_host) + 1;
    const auto t0 = std::chrono::steady_clock::now();
    while (*w == STATUS_UNSET) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(c->spin_us)) break;
    }
    if (*w == INT_MAX) {
      c->early_running = true;
      m->spec_valid = true;
      m->n_early_pd += 1;
      return MFGP_OK;
    }
  }
  if (rc == MFGP_OK) rc = mfgp_ctx_synchronize(c);
  if (rc != MFGP_OK) {
    m->factored = false;   // a failed step leaves no usable factor
    return rc;
  }
  m->spec_valid = true;
  return MFGP_OK;
}

static int predict_view(mfgp_model* m, double** mu, double** var, void** view, int* running) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  int rc = check_model(m);
  if (rc) return rc;
  if (!mu || !var || !view) return set_err(MFGP_ERR_ARG, "null output");
  *mu = *var = nullptr;
  *view = nullptr;
  if (running) *running = 0;
  if (running && m->ctx->early_running && m->spec_valid && m->spec_out && m->M > 0 && factor_current(m)) {
    // the result of the eager append still being computed into the buffer handed
    // over here: the caller wraps it, then settles (mfgp_ctx_synchronize) before it
    // reads it or lets anyone else
    *running = 1;
    m->pred_since_append = true;
  } else {
    if ((rc = settle(m->ctx))) return rc;
    if (m->M == 0) return mfgp_predict(m, nullptr, nullptr);
    if ((rc = ensure_spec_out(m))) return rc;
    // the predict's host outputs are the result buffer itself: no copy
    if ((rc = mfgp_predict(m, m->spec_out, m->spec_out + m->spec_cap))) return rc;
  }
  ViewBuf* v = new ViewBuf{m->spec_out, m->spec_cap, m->spec_max ? 1 : 0};
  *mu = m->spec_out;
  *var = m->spec_out + m->spec_cap;
  *view = v;
  // the buffer is the caller's now: the model's next host-bound predict takes another
  m->spec_out = nullptr;
  m->spec_out_dev = nullptr;
  m->spec_cap = 0;
  m->spec_valid = false;
  m->spec_max = false;
  return MFGP_OK;
}

int mfgp_view_max(const void* view, double* vmax, int64_t* argmax, int* valid) {
  if (!view || !vmax || !argmax || !valid) return set_err(MFGP_ERR_ARG, "null view/output");
  const ViewBuf* v = static_cast<const ViewBuf*>(view);
  *valid = v->has_max;
  if (v->has_max) {
    *vmax = v->host[2 * v->cap];
    std::memcpy(argmax, v->host + 2 * v->cap + 1, sizeof(int64_t));
  }
  return MFGP_OK;
}

int mfgp_predict_view(mfgp_model* m, double** mu, double** var, void** view) {
  return predict_view(m, mu, var, view, nullptr);
}

int mfgp_predict_view_running(mfgp_model* m, double** mu, double** var, void** view, int* running) {
  if (!running) return set_err(MFGP_ERR_ARG, "null output");
  return predict_view(m, mu, var, view, running);
}

int mfgp_release_view(void* view) {
  if (!view) return MFGP_OK;
  ViewBuf* v = static_cast<ViewBuf*>(view);
  bool keep = false;
  {
    std::lock_guard<std::mutex> g(g_view_mu);
    if (g_view_pool.size() < VIEW_POOL_MAX) {
      g_view_pool.push_back(*v);
      keep = true;
    }
  }
  if (!keep) (void)hipHostFree(v->host);
  delete v;
  return MFGP_OK;
}

int mfgp_predict(mfgp_model* m, double* mu, double* var) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  mfgp_ctx* c = m->ctx;
  if (m->M > 0 && (!mu || !var)) return set_err(MFGP_ERR_ARG, "null output");
  m->pred_since_append = true;
  if (m->spec_valid && factor_current(m)) {   // kept from the last predict or the append (spec_append_predict)
    const size_t b = sizeof(double) * (size_t)m->M;
    if (is_device_ptr(mu) && is_device_ptr(var)) {
      HIP_TRY(hipMemcpyAsync(mu, m->spec_out_dev, b, hipMemcpyDeviceToDevice, c->stream));
      HIP_TRY(hipMemcpyAsync(var, m->spec_out_dev + m->spec_cap, b, hipMemcpyDeviceToDevice, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
    } else {
      if (mu != m->spec_out) std::memcpy(mu, m->spec_out, b);
      if (var != m->spec_out + m->spec_cap) std::memcpy(var, m->spec_out + m->spec_cap, b);
    }
    return MFGP_OK;
  }
  if (m->M > 0 && !factor_current(m) && can_inc_factor(m)) {
    // a staged (deferred) append: the bordered append and the one-pass predict
    // as one launch when V is resident (the batched path for one model)
    double *kmu = nullptr, *kvar = nullptr;
    bool host = false;
    if ((rc = model_out(m, mu, var, kmu, kvar, host))) return rc;
    rc = batch_run(&m, 1, nullptr, nullptr, nullptr, kmu, kvar, nullptr, nullptr, MFGP_ASYNC, true, true);
    if (rc == MFGP_OK) rc = mfgp_ctx_synchronize(c);
    if (rc == MFGP_OK) model_out_done(m, mu, var, host);
    if (rc != MFGP_OK) m->factored = false;   // a failed step leaves no usable factor
    return rc;
  }
  if ((rc = update_factor(m))) return rc;
  if (m->M == 0) return MFGP_OK;
  if ((rc = ensure_v(m))) return rc;
  double *kmu = nullptr, *kvar = nullptr;
  bool host = false;
  if ((rc = model_out(m, mu, var, kmu, kvar, host))) return rc;
  int slot;
  GPDesc* hd = acquire_slot(c, slot, rc);
  if (!hd) return rc;
  fill_desc(hd[0], m);
  hd[0].mu = kmu;
  hd[0].var = kvar;
  const int rb = set_res_out(m, hd[0], -1);
  const bool vst = can_vstream(m);
  set_vstream_rows(hd[0], m);
  set_rsplit(c, hd, 1);
  if (!vst && (rc = assign_predict_scratch(c, hd, 1))) return rc;
  const GPDesc* dd = nullptr;
  if ((rc = upload_slot(c, slot, 1, &dd))) return rc;
  if ((rc = vst ? enqueue_vstream(c, dd, hd, 1) : enqueue_predict(c, dd, hd, 1))) return rc;
  (vst ? m->n_vstream : m->n_full_predict) += 1;
  m->v_n = m->NL + m->NH;
  if (rb >= 0) res_tag(m, rb, m->v_n, 0);
  if ((rc = release_slot(c, slot))) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  model_out_done(m, mu, var, host);
  return MFGP_OK;
}

int64_t mfgp_model_n(const mfgp_model* m) { return m ? m->NL + m->NH : -1; }

int mfgp_model_stats(const mfgp_model* m, int64_t* out, int n) {
  if (!m || !out) return set_err(MFGP_ERR_ARG, "null model/out");
  if (const int rc_ = settle(m->ctx)) return rc_;
  // off-lattice training rows the last lattice step's Z units found (lidx = -1,
  // the step's "virtual" K rows): the counts they published, read back from the
  // device (both parts; an MF hifi row off the lattice counts in each)
  int64_t virt = 0;
  if (n > 9 && m->zvl && m->n_lattice > 0) {
    int nv[2] = {0, 0};
    HIP_TRY(hipStreamSynchronize(m->ctx->stream));
    HIP_TRY(hipMemcpy(&nv[0], m->zvl, sizeof(int), hipMemcpyDeviceToHost));
    if (m->kind == MFGP_MF) HIP_TRY(hipMemcpy(&nv[1], m->zvl + m->zb_rows + 1, sizeof(int), hipMemcpyDeviceToHost));
    virt = (int64_t)nv[0] + nv[1];
  }
  const int64_t v[14] = {m->factored ? m->factor_N : -1, m->v_n, m->n_full_factor, m->n_inc_factor,
                         m->n_full_predict, m->n_vstream, m->lat.nx, m->lat.ny, m->n_lattice, virt,
                         m->n_lattice_arg, m->n_lattice_g2, m->n_post_copy, m->n_early_pd};
  for (int i = 0; i < n && i < 14; ++i) out[i] = v[i];
  return MFGP_OK;
}
int64_t mfgp_model_nl(const mfgp_model* m) { return m ? m->NL : -1; }
int64_t mfgp_model_m(const mfgp_model* m) { return m ? m->M : -1; }

int mfgp_get_factor(mfgp_model* m, double* L_out) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if ((rc = update_factor(m))) return rc;
  const int64_t N = m->NL + m->NH;
  if (N == 0) return MFGP_OK;
  std::vector<double> cm((size_t)m->ld * N);
  HIP_TRY(hipMemcpyAsync(cm.data(), m->A, sizeof(double) * m->ld * N, hipMemcpyDeviceToHost, m->ctx->stream));
  HIP_TRY(hipStreamSynchronize(m->ctx->stream));
  for (int64_t i = 0; i < N; ++i)
    for (int64_t j = 0; j < N; ++j) L_out[i * N + j] = (j <= i) ? cm[(size_t)j * m->ld + i] : 0.0;
  return MFGP_OK;
}

// Shared driver of the batched entry points: append (optional), factor
// (do_factor) and predict (do_predict) `count` models with one set of launches
// per kind: bordered appends (k_inc_factor) and full refactors side by side,
// then one-pass predicts over the resident V (k_vstream) and full predicts.
// out_offs / vidx (or null): each model's offset into mu / var and index into
// vmax / vargmax, when `models` is a subset of the caller's batch (the models left
// after the unchanged ones took k_post_copy)
static int batch_run(mfgp_model** models, int count, const double* X, const double* y, const int64_t* k,
                     double* mu, double* var, double* vmax, int64_t* vargmax, int flags, bool do_factor,
                     bool do_predict, const int64_t* out_offs, const int* vidx) {
  if (!models || count <= 0) return set_err(MFGP_ERR_ARG, "empty batch");
  mfgp_ctx* c = models[0]->ctx;
  int rc = MFGP_OK;
  for (int i = 0; i < count; ++i) {
    if ((rc = check_model(models[i]))) return rc;
    if (models[i]->ctx != c) return set_err(MFGP_ERR_ARG, "batch models must share one context");
    if (models[i]->dtype != models[0]->dtype)
      return set_err(MFGP_ERR_ARG, "batch models must share one dtype (MFGP_F64 or MFGP_F32)");
    if (k && k[i] < 0) return set_err(MFGP_ERR_ARG, "negative k");
    if (!do_factor && !factor_current(models[i]))
      return set_err(MFGP_ERR_ARG, "model %d has no current factor (call mfgp_batch_append_factor first)", i);
  }
  if (do_predict && (!mu || !var)) return set_err(MFGP_ERR_ARG, "null output");
  // Members that append nothing to a current factor whose posterior is resident
  // for its rows (the lockstep simulations: seeds whose agents all exploited this
  // iteration, sim:872-891) are unchanged: their predict is the resident posterior,
  // copied into the outputs with its var max / argmax (k_post_copy, one launch),
  // and the batch step runs over the others -- so a ragged batch keeps its one
  // fused (or lattice) launch instead of falling back to streaming V for all.
  bool any_unchanged = false;   // (cheap test first: the pointer queries cost ~1 us each)
  for (int i = 0; i < count && !any_unchanged; ++i) any_unchanged = !(k && X && y) || k[i] == 0;
  if (any_unchanged && do_factor && do_predict && !out_offs && c->incremental && is_device_ptr(mu) &&
      is_device_ptr(var)) {
    const bool rows_given = k && X && y;
    std::vector<PostCopy> pc;
    std::vector<mfgp_model*> rest;
    std::vector<int64_t> rest_k, rest_off;
    std::vector<int> rest_vidx;
    int64_t oo = 0;
    for (int i = 0; i < count; ++i) {
      mfgp_model* m = models[i];
      const int64_t ki = rows_given ? k[i] : 0;
      const int64_t n = m->NL + m->NH;
      const int b = (ki == 0 && m->M > 0 && factor_current(m) && m->v_n == n) ? res_find(m, n) : -1;
      if (b >= 0) {
        pc.push_back({res_mu(m, b), res_var(m, b), mu + oo, var + oo, vmax ? vmax + i : nullptr,
                      vargmax ? vargmax + i : nullptr, m->M});
        m->n_post_copy += 1;
      } else {
        rest.push_back(m);
        rest_k.push_back(ki);
        rest_off.push_back(oo);
        rest_vidx.push_back(i);
      }
      oo += m->M;
    }
    if (!pc.empty()) {
      HIP_TRY(launch_post_copy(pc.data(), (int)pc.size(), c->stream));
      if (rest.empty()) return (flags & MFGP_ASYNC) ? MFGP_OK : mfgp_ctx_synchronize(c);
      // (the rows of the unchanged members are none: the others' rows stay contiguous)
      return batch_run(rest.data(), (int)rest.size(), X, y, rest_k.data(), mu, var, vmax, vargmax, flags, do_factor,
                       do_predict, rest_off.data(), rest_vidx.data());
    }
  }
  for (int i = 0; i < count; ++i) models[i]->spec_valid = false;
  // append new rows: device-resident sources are copied by one k_append launch
  // per sub-batch (below); host sources by plain copies here
  const bool has_new = do_factor && k && X && y;
  const bool dev_src = has_new && is_device_ptr(X) && is_device_ptr(y);
  std::vector<int64_t> src_off(count, 0), out_off(count, 0);
  int64_t off = 0, oo = 0;
  for (int i = 0; i < count; ++i) {
    mfgp_model* m = models[i];
    out_off[i] = out_offs ? out_offs[i] : oo;
    oo += m->M;
    if (!do_factor) continue;
    const int64_t ki = has_new ? k[i] : 0;
    const int64_t n = m->NL + m->NH;
    if ((rc = ensure_cap(m, n + ki))) return rc;
    src_off[i] = off;
    // host rows: the bordered appends carry them in their descriptors (rows_inline,
    // landed by the producers); the others are copied below, before their launches
    if (ki > 0) m->NH += ki;
    off += ki;
    if (!c->incremental) m->factored = false;   // reference behaviour: refactor every update
  }
  std::vector<mfgp_model*> order, porder;
  std::vector<int64_t> oo_ord;
  std::vector<int> res_b, res_depth;
  constexpr int CB = MAXB / 2;   // one descriptor slot per sub-batch: [factor order | predict order]
  for (int b0 = 0; b0 < count; b0 += CB) {
    const int nb = std::min(CB, count - b0);
    if (do_predict) {
      for (int i = 0; i < nb; ++i)
        if (models[b0 + i]->M > 0 && (rc = ensure_v(models[b0 + i]))) return rc;
    }
    int slot;
    GPDesc* hd = acquire_slot(c, slot, rc);
    if (!hd) return rc;
    // factor descriptors, ordered [bordered appends | full refactors | current]:
    // the factor kernels run over their contiguous sub-ranges (k_inc_l21 lands
    // the device-resident rows of the bordered appends, k_append those of the
    // full refactors)
    int ninc = 0, nfull = 0;
    order.clear();
    if (do_factor) {
      for (int i = 0; i < nb; ++i)
        if (!factor_current(models[b0 + i]) && can_inc_factor(models[b0 + i])) order.push_back(models[b0 + i]);
      ninc = (int)order.size();
      for (int i = 0; i < nb; ++i)
        if (!factor_current(models[b0 + i]) && !can_inc_factor(models[b0 + i])) order.push_back(models[b0 + i]);
      nfull = (int)order.size() - ninc;
      for (int i = 0; i < nb; ++i)
        if (factor_current(models[b0 + i])) order.push_back(models[b0 + i]);
      for (int i = 0; i < nb; ++i) {
        mfgp_model* m = order[i];
        if (i < ninc) {
          if ((rc = fill_inc_desc(hd[i], m))) return rc;
        } else {
          fill_desc(hd[i], m);
        }
        const int mi = (int)(std::find(models + b0, models + b0 + nb, m) - models);
        const int64_t ki = has_new ? k[mi] : 0;
        if (ki <= 0) continue;
        if (dev_src) {
          hd[i].srcX = X + 2 * src_off[mi];
          hd[i].srcY = y + src_off[mi];
          hd[i].k_new = ki;
        } else if (i < ninc && ki <= KINC) {
          std::memcpy(hd[i].rows_xy, X + 2 * src_off[mi], sizeof(double) * 2 * ki);
          std::memcpy(hd[i].rows_y, y + src_off[mi], sizeof(double) * ki);
          hd[i].rows_inline = 1;
          hd[i].k_new = ki;
        } else if ((rc = copy_rows(m, m->NL + m->NH - ki, X + 2 * src_off[mi], y + src_off[mi], ki))) {
          return rc;
        }
      }
      for (int i = 0; i < ninc + nfull; ++i) {   // host bookkeeping of the factors enqueued below
        if (i < ninc) mark_inc_factor(order[i]);
        else mark_full_factor(order[i]);
        add_async_status(c, order[i]);
      }
    }
    // predict descriptors (state after the factor step), ordered
    // [one-pass predicts over resident V | full predicts]
    int nv = 0, np = 0;
    if (do_predict) {
      porder.clear();
      oo_ord.clear();
      for (int pass = 0; pass < 2; ++pass)
        for (int i = 0; i < nb; ++i) {
          mfgp_model* m = models[b0 + i];
          if (m->M == 0 || can_vstream(m) != (pass == 0)) continue;
          porder.push_back(m);
          oo_ord.push_back(out_off[b0 + i]);
        }
      np = (int)porder.size();
      while (nv < np && can_vstream(porder[nv])) ++nv;
      res_b.assign(np, -1);
      for (int i = 0; i < np; ++i) {
        GPDesc& pd = hd[nb + i];
        fill_desc(pd, porder[i]);
        res_b[i] = set_res_out(porder[i], pd, -1);
        if (i < nv) set_vstream_rows(pd, porder[i]);
        pd.mu = mu + oo_ord[i];
        pd.var = var + oo_ord[i];
        int64_t mi = std::find(models + b0, models + b0 + nb, porder[i]) - models;
        if (vidx) mi = vidx[mi];
        if (vmax) pd.vmax = vmax + mi;
        if (vargmax) pd.vargmax = vargmax + mi;
      }
    }
    // bordered appends whose one-pass predicts follow from the same rows (V
    // resident up to the old factor) run as one k_inc_stream launch: their
    // factor descriptors take the predict outputs and the hand-off state
    bool fuse = c->fused && ninc > 0 && ninc == nv;
    for (int i = 0; fuse && i < ninc; ++i) fuse = order[i] == porder[i] && hd[i].n0 == porder[i]->v_n;
    if (fuse) {
      for (int i = 0; i < ninc; ++i) {
        GPDesc& fd = hd[i];
        const GPDesc& pd = hd[nb + i];
        fd.mu = pd.mu;
        fd.var = pd.var;
        fd.vmax = pd.vmax;
        fd.vargmax = pd.vargmax;
        fd.rmu = pd.rmu;
        fd.rvar = pd.rvar;
        fd.tiles = 1;
      }
    }
    // lattice grids, well-conditioned K and a resident posterior of the old rows:
    // the separable step (k_inc_lat) instead of the V stream
    bool lat = fuse;
    for (int i = 0; lat && i < ninc; ++i) lat = lat_eligible(order[i], hd[i].n0);
    res_depth.assign(ninc, 0);
    int ka = 8;
    int64_t tiles_sum = 0, nst_min = INT64_MAX;
    bool g2 = false;
    if (lat) {
      for (int i = 0; i < ninc; ++i) {
        if (order[i]->NL + order[i]->NH - hd[i].n0 > 8) ka = 16;
      }
      // the GEMM as a second launch (k_lat_gemm2: no split-K partials through memory,
      // no hand-off flags) where its tiles fill the chip once or twice: at the
      // headline (B = 8, 256 tiles) 80 vs 100 us per step; a batch of many more tiles
      // (configs[4]: 4096) keeps the in-launch tiles, whose GEMM overlaps the other
      // GPs' F streams (2.35 vs 3.05 ms per step), and so does one GP (52 vs 57 us)
      {
        int64_t t2 = 0;
        for (int i = 0; i < ninc; ++i) t2 += lat_tiles2(order[i], ka);
        g2 = c->lat_gemm2 > 0 || (c->lat_gemm2 < 0 && t2 >= c->ncu && t2 <= 2 * (int64_t)c->ncu);
        // (split-K tiles of one launch wait for each other: they need the whole chip)
        if (c->concurrent) g2 = true;
      }
      for (int i = 0; i < ninc; ++i) {
        const mfgp_model* m = order[i];
        tiles_sum += g2 ? lat_tiles2(m, ka) : lat_tiles(m, ka);
        // K stages of the axis rows (virtual rows add more)
        const int64_t nst = (m->kind == MFGP_SF ? 1 : 2) * (round_up(m->lat.ny, ZKS) / ZKS);
        nst_min = std::min(nst_min, nst);
      }
      // the lattice step has a fixed cost (its chain of dependent phases) plus the F
      // stream and the GEMM (~0.8 us per million n0^2); the V stream reads 8 n0 M
      // bytes per GP (~5.5 TB/s) -- measured at 128x128, N = 2048 (us per step, V
      // stream / lattice with the second-launch GEMM, round 3): B = 8 345 / 80; B = 1
      // 60 / 57 back to back; in the drop-in step (one GP, the eager append returning
      // at the L22 verdict, round 5: tools/bench_dropin.py) 93.2 / 88.3-90.3 us, so
      // the fixed cost is priced at 50 and one GP from n0 ~ 1700 (at M = 16384) takes
      // the lattice; configs[4] (32 GPs, 256x256, N = 8192, fp32 V) 11.2 / 2.4 ms
      double vs_us = 10.0, lat_us = 50.0;
      for (int i = 0; i < ninc; ++i) {
        const mfgp_model* m = order[i];
        const double n0 = (double)hd[i].n0, es = m->dtype == MFGP_F32 ? 4.0 : 8.0;
        vs_us += (double)m->M * n0 * es / 5.5e6;
        lat_us += 0.81 * n0 * n0 / 1.0e6;
      }
      if (lat_us >= vs_us && !c->lat_force) lat = false;
    }
    if (lat) {
      // split-K so that the GEMM tiles fill the chip about twice, >= 4 stages each
      // (the second-launch GEMM splits K inside its workgroups: S = 1 here)
      int S = (int)std::min<int64_t>(8, std::max<int64_t>(1, (2 * c->ncu + tiles_sum - 1) / tiles_sum));
      if (g2) S = 1;
      // (split s takes every S-th stage: at least 4 each)
      S = (int)std::max<int64_t>(1, std::min<int64_t>(S, nst_min / 4));
      if (c->lat_ksplit > 0) S = (int)std::max<int64_t>(1, std::min<int64_t>(c->lat_ksplit, nst_min));
      // a power of two (the splits share the tile's cell passes), and with S > 1 every
      // GEMM workgroup of the launch resident at once (the splits of a tile wait for
      // each other): tiles x S within two workgroups per CU
      {
        int p2 = 1;
        while (2 * p2 <= S) p2 *= 2;
        S = p2;
        while (S > 1 && tiles_sum * S > 2 * (int64_t)c->ncu) S /= 2;
      }
      // w units: two per CU over the launch (equal shares of the F stream: with an
      // uneven count the CUs holding one more unit set the stream's pace; two per CU
      // keep twice the loads in flight: tools/probe_wloop.hip, B = 8: 25 vs 30 us),
      // each GP's count by its F steps
      // and at least ~8 steps each: a block's partials are summed by one unit, four
      // partials per round trip (one GP at 128x128, N = 2048: 512 units 57.1 us per
      // launch, 256 units 52.4, 128 units 52.7; tools/sweep_lat_b1.sh)
      int64_t wsteps_sum = 0;
      for (int i = 0; i < ninc; ++i) wsteps_sum += lat_wsteps(hd[i].n0);
      // ... and for a large batch about 512 steps each, up to eight units per CU (more
      // loads queued: configs[4], 32 GPs at N = 8192, 2.86 ms per step with 512 units,
      // 2.41 with 2048; the headline keeps 512: 384 and 448 were slower)
      int64_t wu_total = std::max<int64_t>(c->ncu / 2, wsteps_sum / 8);
      if (wu_total > 2 * c->ncu)
        wu_total = std::max<int64_t>(2 * c->ncu, std::min<int64_t>(8 * c->ncu, wsteps_sum / 512));
      if (c->lat_wu > 0) wu_total = c->lat_wu;
      // w units that gather L21 from V themselves start the F stream at once; each
      // row's gather is repeated in every block column it meets (~2x F's bytes in
      // cache lines), which a batch's concurrent streams pay for (B = 8: 101.7 vs
      // 99.5 us) and one GP does not (57.1 vs 60.3 us)
      const int selfg = c->lat_selfg >= 0 ? c->lat_selfg : (ninc == 1 ? 1 : 0);
      for (int i = 0; i < ninc; ++i) {
        mfgp_model* m = order[i];
        GPDesc& fd = hd[i];
        const int64_t tiles = g2 ? lat_tiles2(m, ka) : lat_tiles(m, ka);
        const int64_t nzu = lat_nzu(m);
        if ((rc = ensure_lat(m, tiles, S, ka, nzu))) return rc;
        const int bin = res_find(m, fd.n0);
        fd.rmu_in = res_mu(m, bin);
        fd.rvar_in = res_var(m, bin);
        fd.rmu = res_mu(m, 1 - bin);
        fd.rvar = res_var(m, 1 - bin);
        res_b[i] = 1 - bin;
        res_depth[i] = m->res_depth[bin] + 1;
        fd.F = m->F;
        fd.Ff = m->Ff;
        fd.tab = m->tab;
        fd.tabw = m->tabw;
        fd.wv = m->wv;
        fd.wflag = m->wflag;
        fd.gpart = m->gpart;
        fd.gcnt = m->gcnt;
        fd.ka = ka;
        fd.ksplit = S;
        fd.lat_tiles = (int)tiles;
        fd.nwb = (int)((fd.n0 + 63) / 64);
        {
          const int64_t st = lat_wsteps(fd.n0);
          const int64_t u = (wu_total * st + wsteps_sum / 2) / wsteps_sum;
          fd.nwu = (int)std::max<int64_t>(1, std::min<int64_t>({u, (int64_t)LAT_WU_MAX, st}));
        }
        fd.wpart = m->wpart;
        fd.wcnt = m->wcnt;
        fd.lat_fbuild = (m->F_gen == m->gen && m->F_n >= fd.n0) ? 0 : 1;
        fd.lidx = m->lidx;
        fd.axt = m->axt;
        fd.zb = m->zb;
        fd.zrows = m->zb_rows;
        fd.zflag = m->zflag;
        fd.ldone = m->ldone;
        fd.zvl = m->zvl;
        fd.nzu = (int)nzu;
        fd.zq = lat_zq(m);
        fd.lat_axbuild = m->axt_gen == m->gen ? 0 : 1;
        fd.lat_selfg = selfg;
        fd.lat_g2 = g2 ? 1 : 0;
        // Z units reading the scan units' member lists (every lattice row count the scan
        // units bucket, rows and lattice indices within 16 bits)
        // -- by default (the bucketing Z units scan every row of their part; with the
        // lists: headline 93.2k -> 95.3k GP-updates/s, configs[4] 17.8k -> 19.3k)
        const bool zc = c->lat_zcsr != 0;
        (void)nzu;
        fd.lat_zcsr = (zc && ka == 8 && m->lat.ny <= 256 && m->ld <= 65535) ? 1 : 0;
        fd.csr = m->csr;
        fd.tab_lo = (m->tab_gen == m->gen) ? std::min(m->tab_n, fd.n0) : 0;
      }
    }
    if (nv > 0) {
      set_rsplit(c, hd + nb, nv);
      for (int i = 0; fuse && i < ninc; ++i) hd[i].rsplit = hd[nb].rsplit;
    }
    if (np > nv && (rc = assign_predict_scratch(c, hd + nb + nv, np - nv))) return rc;
    // one GP, append + one-pass predict fused, nothing else: launch with the
    // descriptor by value (no upload) and the status published into a mapped word
    // (the lattice step of one GP publishes its status the same way)
    const bool single = fuse && nb == 1 && ninc == 1 && np == 1 && nv == 1;
    if (single) {
      mfgp_model* m = order[0];
      if (!m->status_host) {
        HIP_TRY(hipHostMalloc(&m->status_host, 2 * sizeof(int), hipHostMallocMapped));
        void* dev = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dev, m->status_host, 0));
        m->status_host_dev = static_cast<int*>(dev);
      }
      *reinterpret_cast<volatile int*>(m->status_host) = STATUS_UNSET;
      reinterpret_cast<volatile int*>(m->status_host)[1] = STATUS_UNSET;
      hd[0].status_host = m->status_host_dev;
      hd[0].pd_host = m->status_host_dev + 1;
      for (auto it = c->async_status.rbegin(); it != c->async_status.rend(); ++it)
        if (it->m == m) {
          it->host = m->status_host;
          break;
        }
    }
    if (single && !lat) {
      mfgp_model* m = order[0];
      EvPair ev{};
      if ((rc = ev_begin(c, ev, 0))) return rc;
      HIP_TRY(launch_inc_stream1(hd[0], hd[0].nprod + ntiles_wg(hd[0].M, hd[0].rsplit, hd[0].vf32), hd[0].vf32,
                                 c->stream));
      if ((rc = ev_end(c, ev))) return rc;
      release_slot_unread(c, slot);
      m->v_n = m->NL + m->NH;
      m->n_vstream += 1;
      if (res_b[0] >= 0) res_tag(m, res_b[0], m->v_n, 0);
      continue;
    }
    bool lat_arg = false, by_value = false;
    if (do_factor && lat && nfull == 0 && ninc == nb && np == nv && desc_arg_ok(c, hd, ninc)) {
      // the whole step is one k_inc_lat launch: its descriptors go by value
      if ((rc = enqueue_inc_lat_arg(c, hd, ninc))) return rc;
      lat_arg = by_value = true;
    } else if (do_factor && fuse && !lat && nfull == 0 && ninc == nb && np == nv && c->desc_arg &&
               ninc <= DESC_ARG_MAX) {
      // the whole step is one k_inc_stream launch (append + one-pass predict)
      if ((rc = enqueue_inc_stream_arg(c, hd, ninc))) return rc;
      by_value = true;
    } else {
    const GPDesc* dd = nullptr;
    if ((rc = upload_slot(c, slot, nb + np, &dd))) return rc;
    if (do_factor) {
      if (dev_src && nfull > 0) HIP_TRY(launch_append(dd + ninc, nfull, c->stream));
      if (ninc > 0 && (rc = lat ? enqueue_inc_lat(c, dd, hd, ninc)
                                : (fuse ? enqueue_inc_stream(c, dd, hd, ninc) : enqueue_inc_factor(c, dd, hd, ninc))))
        return rc;
      if (nfull > 0 && (rc = enqueue_factor(c, dd + ninc, hd + ninc, nfull))) return rc;
    }
    if (nv > 0 && !fuse && (rc = enqueue_vstream(c, dd + nb, hd + nb, nv))) return rc;
    if (np > nv && (rc = enqueue_predict(c, dd + nb + nv, hd + nb + nv, np - nv))) return rc;
    }
    if (by_value) {
      release_slot_unread(c, slot);
    } else if ((rc = release_slot(c, slot))) {
      return rc;
    }
    for (int i = 0; i < np; ++i) {
      mfgp_model* m = porder[i];
      m->v_n = m->NL + m->NH;
      (i < nv ? m->n_vstream : m->n_full_predict) += 1;
      if (res_b[i] >= 0) res_tag(m, res_b[i], m->v_n, (lat && i < ninc) ? res_depth[i] : 0);
      if (lat && i < ninc) {
        m->n_lattice += 1;
        if (lat_arg) m->n_lattice_arg += 1;
        if (g2) m->n_lattice_g2 += 1;
        m->F_n = m->v_n;   // F's new rows and the new rows' tables came with the step
        m->F_gen = m->gen;
        m->tab_n = m->v_n;
        m->tab_gen = m->gen;
        m->axt_gen = m->gen;
      }
    }
  }
  if (flags & MFGP_ASYNC) return MFGP_OK;
  return mfgp_ctx_synchronize(c);
}

// The planners work on the caller's model itself instead of a deep copy (sim:339):
// the rows they append lie past the model's own, and the factor, z, V, F and the
// tables of the leading rows do not depend on later rows, so truncating back to the
// model's rows restores it. What the loop overwrites that a truncate does not bring
// back is saved and restored: the resident posterior (both ping-pong buffers and
// their tags: the lattice steps write them), the kept result's validity, the path
// counters (the loop's steps go to the context's planner counters instead). A copy
// of A, V and F (~320 MB per model at 128 x 128, N = 2048) and the allocations it
// took cost more than the whole loop (profiles/r06a_choi: ~36 of 44 ms for 8 seeds).
struct PlanSave {
  int64_t NH0 = 0;
  double* res = nullptr;   // device copy of m->res ([2][2][res_M]), or null
  int64_t res_n[2];
  uint64_t res_gen[2], res_tick[2], tick;
  int res_depth[2];
  bool spec_valid, spec_max, pred_since_append;
  int64_t cnt[9];
};
static void plan_counters(const mfgp_model* m, int64_t (&v)[9]) {
  const int64_t x[9] = {m->n_full_factor, m->n_inc_factor, m->n_full_predict, m->n_vstream, m->n_lattice,
                        m->n_lattice_arg, m->n_lattice_g2, m->n_post_copy, m->n_early_pd};
  for (int i = 0; i < 9; ++i) v[i] = x[i];
}
// doubles of device room plan_enter needs for m's resident posterior
static size_t plan_res_doubles(const mfgp_model* m) { return m->res ? 4 * (size_t)m->res_M : 0; }
// save what the loop may overwrite; `room` (plan_res_doubles) receives the posterior
static int plan_enter(mfgp_model* m, PlanSave& s, double* room) {
  s.NH0 = m->NH;
  s.res = (m->res && room) ? room : nullptr;
  if (s.res) HIP_TRY(hipMemcpyAsync(s.res, m->res, sizeof(double) * 4 * m->res_M, hipMemcpyDeviceToDevice, m->ctx->stream));
  for (int b = 0; b < 2; ++b) {
    s.res_n[b] = m->res_n[b];
    s.res_gen[b] = m->res_gen[b];
    s.res_tick[b] = m->res_tick[b];
    s.res_depth[b] = m->res_depth[b];
  }
  s.tick = m->tick;
  s.spec_valid = m->spec_valid;
  s.spec_max = m->spec_max;
  s.pred_since_append = m->pred_since_append;
  plan_counters(m, s.cnt);
  return MFGP_OK;
}
// back to the model's own rows and state (also after a failed loop: the error is
// the caller's to return); the loop's path counters go to the context's
static int plan_leave(mfgp_model* m, const PlanSave& s) {
  m->gate_dev = nullptr;
  int64_t now[9];
  plan_counters(m, now);
  int64_t* p = m->ctx->plan_stats;
  p[0] += 1;
  p[1] += now[1] - s.cnt[1];
  p[2] += now[3] - s.cnt[3];
  p[3] += now[4] - s.cnt[4];
  p[4] += now[5] - s.cnt[5];
  p[5] += now[6] - s.cnt[6];
  p[6] += now[0] - s.cnt[0];
  p[7] += now[2] - s.cnt[2];
  m->n_full_factor = s.cnt[0];
  m->n_inc_factor = s.cnt[1];
  m->n_full_predict = s.cnt[2];
  m->n_vstream = s.cnt[3];
  m->n_lattice = s.cnt[4];
  m->n_lattice_arg = s.cnt[5];
  m->n_lattice_g2 = s.cnt[6];
  m->n_post_copy = s.cnt[7];
  m->n_early_pd = s.cnt[8];
  m->NH = s.NH0;
  const int64_t N = m->NL + m->NH;
  if (m->factored && m->factor_N > N) m->factor_N = N;
  m->v_n = std::min(m->v_n, N);
  m->F_n = std::min(m->F_n, N);
  m->tab_n = std::min(m->tab_n, N);
  m->l21c_N = -1;   // (the compact rows in iscr are the loop's now)
  if (s.res && m->res) {
    HIP_TRY(hipMemcpyAsync(m->res, s.res, sizeof(double) * 4 * m->res_M, hipMemcpyDeviceToDevice, m->ctx->stream));
    for (int b = 0; b < 2; ++b) {
      m->res_n[b] = s.res_n[b];
      m->res_gen[b] = s.res_gen[b];
      m->res_tick[b] = s.res_tick[b];
      m->res_depth[b] = s.res_depth[b];
    }
    m->tick = std::max(m->tick, s.tick);
  } else {
    for (int b = 0; b < 2; ++b)
      if (m->res_n[b] > N) m->res_n[b] = -1;
  }
  // the kept result of the model's last predict: spec_out is not written by the loop
  m->spec_valid = s.spec_valid && factor_current(m);
  m->spec_max = s.spec_max && m->spec_valid;
  m->pred_since_append = s.pred_since_append;
  return MFGP_OK;
}

// compute_sample_points (simulator.py:326-374) as a device loop. Each iteration
// is k_choi_select (argmax cell + its mean -> new hifi row, or stop), a 1-row
// bordered append and a one-pass predict with the fused argmax, all gated by a
// device flag, so chunks of iterations are enqueued without a host round trip;
// the host reads the flag once per chunk and truncates the rows that a stopped
// loop did not append (the leading rows' factor and V stay valid).
int mfgp_sample_points(mfgp_model* model, double threshold, int64_t max_points, double* points, int64_t* count) {
  const DeviceGuard dg_(model ? model->ctx->device : -1);
  if (const int rc_ = settle(model ? model->ctx : nullptr)) return rc_;
  int rc = check_model(model);
  if (rc) return rc;
  if (!count || (max_points > 0 && !points)) return set_err(MFGP_ERR_ARG, "null output");
  if (max_points < 0) return set_err(MFGP_ERR_ARG, "negative max_points");
  if (model->M <= 0) return set_err(MFGP_ERR_ARG, "no grid: call mfgp_set_grid first");
  *count = 0;
  mfgp_ctx* c = model->ctx;
  if (!c->incremental) return set_err(MFGP_ERR_ARG, "mfgp_sample_points needs incremental updates enabled");
  if ((rc = update_factor(model))) return rc;
  // the reference works on a deep copy (sim:339); here on the model itself, brought
  // back to its own rows and state at the end (plan_enter / plan_leave)
  mfgp_model* t = model;
  const int64_t M = t->M;
  // workspace: mu, var [M] | vmax | vargmax | state {gate, count} | points [max_points][2] |
  // the saved resident posterior
  const size_t npt = 2 * (size_t)std::max<int64_t>(max_points, 1);
  const size_t nd = 2 * (size_t)M + 4 + npt + plan_res_doubles(t);
  if ((rc = ensure_ws(c, sizeof(double) * nd))) return rc;
  double* mu_s = c->ws;
  double* var_s = mu_s + M;
  double* vmax = var_s + M;
  int64_t* vargmax = reinterpret_cast<int64_t*>(vmax + 1);
  int64_t* state = vargmax + 1;
  double* pts = reinterpret_cast<double*>(state + 2);
  int* gate = reinterpret_cast<int*>(state);
  PlanSave sv;
  if ((rc = plan_enter(t, sv, pts + npt))) return rc;
  auto fail = [&](int code) {
    (void)plan_leave(t, sv);
    return code;
  };
  // initial posterior (sim:340-342)
  if ((rc = batch_run(&t, 1, nullptr, nullptr, nullptr, mu_s, var_s, vmax, vargmax, 0, false, true))) return fail(rc);
  const int64_t st0[2] = {1, 0};
  if (hipMemcpyAsync(state, st0, sizeof(st0), hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return fail(set_err(MFGP_ERR_DEVICE, "state upload failed"));
  const int64_t NH0 = t->NH;
  int64_t done = 0;
  bool active = true;
  constexpr int64_t CH = 32;   // iterations per chunk (two descriptors each)
  while (active && done < max_points) {
    const int64_t C = std::min<int64_t>(CH, max_points - done);
    const int64_t N = t->NL + t->NH;
    if ((rc = ensure_cap(t, N + C)) || (rc = ensure_v(t))) return fail(rc);
    if (!factor_current(t)) return fail(set_err(MFGP_ERR_DEVICE, "sample_points: factor lost on growth"));
    int slot;
    GPDesc* hd = acquire_slot(c, slot, rc);
    if (!hd) return fail(rc);
    for (int64_t it = 0; it < C; ++it) {
      t->NH += 1;   // assume the iteration runs; truncated below if the loop stopped
      GPDesc& fd = hd[2 * it];
      if ((rc = fill_inc_desc(fd, t))) return fail(rc);
      fd.mu = mu_s;
      fd.vmax = vmax;
      fd.vargmax = vargmax;
      fd.gate = gate;
      if (c->fused) {   // the iteration's append and predict in one launch
        fd.var = var_s;
        fd.tiles = 1;
      }
      mark_inc_factor(t);
      GPDesc& pd = hd[2 * it + 1];
      fill_desc(pd, t);
      set_vstream_rows(pd, t);
      pd.mu = mu_s;
      pd.var = var_s;
      pd.vmax = vmax;
      pd.vargmax = vargmax;
      pd.gate = gate;
      t->v_n = t->NL + t->NH;
    }
    set_rsplit(c, hd + 1, 1);
    for (int64_t i = 0; i < 2 * C; ++i) hd[i].rsplit = hd[1].rsplit;
    const GPDesc* dd = nullptr;
    if ((rc = upload_slot(c, slot, (int)(2 * C), &dd))) return fail(rc);
    const int vf = t->dtype == MFGP_F32 ? 1 : 0;
    for (int64_t it = 0; it < C; ++it) {
      const bool ok = hipSuccess == launch_choi_select(dd + 2 * it, threshold, pts, max_points, c->stream) &&
                      (c->fused ? hipSuccess == launch_inc_stream(dd + 2 * it, 1,
                                                                   hd[2 * it].nprod + ntiles_wg(M, hd[2 * it].rsplit, vf),
                                                                   vf, c->stream)
                                : (hipSuccess == launch_inc_factor(dd + 2 * it, 1, hd[2 * it].nprod, vf, c->stream) &&
                                   hipSuccess == launch_vstream(dd + 2 * it + 1, 1, ntiles_wg(M, hd[2 * it + 1].rsplit, vf),
                                                                vf, c->stream)));
      if (!ok) return fail(set_err(MFGP_ERR_DEVICE, "sample_points: launch failed"));
    }
    if ((rc = release_slot(c, slot))) return fail(rc);
    int64_t st[2] = {0, 0};
    if (hipMemcpyAsync(st, state, sizeof(st), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess)
      return fail(set_err(MFGP_ERR_DEVICE, "sample_points: state read failed"));
    active = (int)st[0] != 0;
    const int64_t ran = st[1] - done;
    done = st[1];
    if (ran < C) {
      // the loop stopped inside this chunk: drop the rows it did not append
      if ((rc = mfgp_truncate(t, NH0 + done))) return fail(rc);
    }
    if ((rc = read_status(t))) return fail(rc);
  }
  if (done > 0 && hipMemcpy(points, pts, sizeof(double) * 2 * done, hipMemcpyDefault) != hipSuccess)
    return fail(set_err(MFGP_ERR_DEVICE, "sample_points: copy out failed"));
  *count = done;
  if ((rc = plan_leave(t, sv))) return rc;
  return mfgp_ctx_synchronize(c);   // (the posterior's restore copy: ws is reused by the next call)
}

// compute_sample_points for a batch of models (the Choi planner's sample-set
// selection of many seeds, sim:326-374) stepped together: per iteration ONE
// k_choi_select_batch (every model's decision from its fused max / argmax) and ONE
// batched append + predict of every model's chosen row through the general batch
// step -- the lattice step where the batch takes it (its kernels and the V stream's
// honour each model's device gate, so a model past its threshold skips the rest of
// the chunk) -- with one host synchronisation per CH iterations. Each model works on
// its own rows past its own (sim:339's deep copy: plan_enter / plan_leave bring it
// back); the chosen points are the single-model loop's, up to the rounding of the
// batch step (ties decided by it).
int mfgp_batch_sample_points(mfgp_model** models, int count, const double* thresholds, int64_t max_points,
                             double* points, int64_t* counts) {
  const auto tp0 = std::chrono::steady_clock::now();
  const DeviceGuard dg_((models && count > 0 && models[0]) ? models[0]->ctx->device : -1);
  if (const int rc_ = settle((models && count > 0 && models[0]) ? models[0]->ctx : nullptr)) return rc_;
  if (count <= 0 || !models || !thresholds || !counts || (max_points > 0 && !points))
    return set_err(MFGP_ERR_ARG, "bad batch_sample_points arguments");
  if (max_points < 0) return set_err(MFGP_ERR_ARG, "negative max_points");
  mfgp_ctx* c = models[0]->ctx;
  if (!c->incremental) return set_err(MFGP_ERR_ARG, "mfgp_batch_sample_points needs incremental updates enabled");
  int rc = MFGP_OK;
  for (int b = 0; b < count; ++b) {
    if ((rc = check_model(models[b]))) return rc;
    if (models[b]->ctx != c) return set_err(MFGP_ERR_ARG, "batch models must share one context");
    if (models[b]->dtype != models[0]->dtype) return set_err(MFGP_ERR_ARG, "batch models must share one dtype");
    if (models[b]->M <= 0) return set_err(MFGP_ERR_ARG, "model %d: no grid (call mfgp_set_grid first)", b);
    for (int b2 = 0; b2 < b; ++b2)
      if (models[b2] == models[b]) return set_err(MFGP_ERR_ARG, "model %d appears twice in the batch", b);
    counts[b] = 0;
  }
  for (int b = 0; b < count; ++b)
    if ((rc = update_factor(models[b]))) return rc;
  mfgp_model* const* t = models;
  // device state: mu, var [sum M] | vmax [B] | vargmax [B] | state [B][2] | thr [B] | moff [B] |
  // Ms [B] | grids [B] | xn [B][2] | yn [B] | pos [B] | points [B][max_points][2] | the models'
  // saved resident posteriors
  std::vector<int64_t> moff(count), Ms(count);
  int64_t Mtot = 0;
  size_t nres = 0;
  for (int b = 0; b < count; ++b) {
    moff[b] = Mtot;
    Ms[b] = t[b]->M;
    Mtot += t[b]->M;
    nres += plan_res_doubles(t[b]);
  }
  const int64_t P = std::max<int64_t>(max_points, 1);
  // one 8-byte slot per entry (pos's ints take a slot each); the offsets below are
  // the only description of the layout, and the allocation is their end
  const size_t B_ = (size_t)count;
  const size_t o_mu = 0, o_var = o_mu + (size_t)Mtot, o_vmax = o_var + (size_t)Mtot, o_varg = o_vmax + B_;
  const size_t o_state = o_varg + B_, o_thr = o_state + 2 * B_, o_moff = o_thr + B_, o_Ms = o_moff + B_;
  const size_t o_grids = o_Ms + B_, o_xn = o_grids + B_, o_yn = o_xn + 2 * B_, o_pos = o_yn + B_;
  const size_t o_pts = o_pos + B_, o_res = o_pts + 2 * B_ * (size_t)P, nd = o_res + nres;
  double* ws = nullptr;
  if (hipMalloc(&ws, sizeof(double) * nd) != hipSuccess)
    return set_err(MFGP_ERR_DEVICE, "batch_sample_points: out of memory");
  std::vector<PlanSave> sv(count);
  int entered = 0;
  auto fail = [&](int code) {
    for (int b = 0; b < entered; ++b) (void)plan_leave(t[b], sv[b]);
    (void)hipStreamSynchronize(c->stream);   // (the restore copies read ws)
    (void)hipFree(ws);
    return code;
  };
  for (size_t b = 0, off = o_res; b < B_; off += plan_res_doubles(t[b]), ++b) {
    if ((rc = plan_enter(t[b], sv[b], ws + off))) return fail(rc);
    ++entered;
  }
  double* mu = ws + o_mu;
  double* var = ws + o_var;
  double* vmax = ws + o_vmax;
  int64_t* vargmax = reinterpret_cast<int64_t*>(ws + o_varg);
  int64_t* state = reinterpret_cast<int64_t*>(ws + o_state);
  double* thr = ws + o_thr;
  int64_t* moff_d = reinterpret_cast<int64_t*>(ws + o_moff);
  int64_t* Ms_d = reinterpret_cast<int64_t*>(ws + o_Ms);
  const double** grids_d = reinterpret_cast<const double**>(ws + o_grids);
  double* xn = ws + o_xn;
  double* yn = ws + o_yn;
  int* pos_d = reinterpret_cast<int*>(ws + o_pos);
  double* pts = ws + o_pts;
  std::vector<int64_t> st(2 * count);
  std::vector<const double*> grids(count);
  for (int b = 0; b < count; ++b) {
    st[2 * b] = 1;
    st[2 * b + 1] = 0;
    grids[b] = t[b]->grid;
  }
  hipStream_t s = c->stream;
  if (hipMemcpyAsync(state, st.data(), sizeof(int64_t) * 2 * count, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(thr, thresholds, sizeof(double) * count, hipMemcpyDefault, s) != hipSuccess ||
      hipMemcpyAsync(moff_d, moff.data(), sizeof(int64_t) * count, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(Ms_d, Ms.data(), sizeof(int64_t) * count, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(grids_d, grids.data(), sizeof(double*) * count, hipMemcpyHostToDevice, s) != hipSuccess)
    return fail(set_err(MFGP_ERR_DEVICE, "batch_sample_points: state upload failed"));
  // the initial posteriors and their max / argmax (sim:340-342)
  if ((rc = batch_run(const_cast<mfgp_model**>(t), count, nullptr, nullptr, nullptr, mu, var, vmax, vargmax, 0,
                      false, true)))
    return fail(rc);
  for (int b = 0; b < count; ++b) t[b]->gate_dev = reinterpret_cast<int*>(state + 2 * b);
  // the models still running (the batch step's members; a stopped one leaves at the
  // next chunk boundary), their offsets into mu / var and indices into vmax
  std::vector<int> live(count);
  for (int b = 0; b < count; ++b) live[b] = b;
  constexpr int64_t CH = 32;
  int64_t it_done = 0;
  const auto tp1 = std::chrono::steady_clock::now();
  while (!live.empty() && it_done < max_points) {
    const int64_t C = std::min<int64_t>(CH, max_points - it_done);
    // the live models are the batch step's members, in batch order: their rows at
    // their member places (pos), their outputs at their own offsets / indices
    std::vector<mfgp_model*> lm;
    std::vector<int64_t> lk, loff;
    std::vector<int> lvi, pos(count, -1);
    for (int b : live) {
      pos[b] = (int)lm.size();
      lm.push_back(t[b]);
      lk.push_back(1);
      loff.push_back(moff[b]);
      lvi.push_back(b);
    }
    if (hipMemcpyAsync(pos_d, pos.data(), sizeof(int) * count, hipMemcpyHostToDevice, s) != hipSuccess)
      return fail(set_err(MFGP_ERR_DEVICE, "batch_sample_points: upload failed"));
    for (int64_t it = 0; it < C; ++it) {
      if (launch_choi_select_batch(count, pos_d, state, thr, vmax, vargmax, mu, moff_d, grids_d, Ms_d, xn, yn, pts,
                                   max_points, s) != hipSuccess)
        return fail(set_err(MFGP_ERR_DEVICE, "batch_sample_points: launch failed"));
      if ((int)lm.size() == count)
        rc = batch_run(lm.data(), count, xn, yn, lk.data(), mu, var, vmax, vargmax, MFGP_ASYNC, true, true);
      else
        rc = batch_run(lm.data(), (int)lm.size(), xn, yn, lk.data(), mu, var, vmax, vargmax, MFGP_ASYNC, true, true,
                       loff.data(), lvi.data());
      if (rc) return fail(rc);
    }
    it_done += C;
    if (hipMemcpyAsync(st.data(), state, sizeof(int64_t) * 2 * count, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return fail(set_err(MFGP_ERR_DEVICE, "batch_sample_points: state read failed"));
    for (int b : live)
      if ((rc = read_status(t[b]))) return fail(rc);
    std::vector<int> keep;
    for (int b : live)
      if ((int)st[2 * b] != 0) keep.push_back(b);
    live.swap(keep);
  }
  const auto tp2 = std::chrono::steady_clock::now();
  for (int b = 0; b < count; ++b) {
    counts[b] = st[2 * b + 1];
    if (counts[b] > 0 && hipMemcpy(points + 2 * (size_t)b * (size_t)P, pts + 2 * (size_t)b * (size_t)P,
                                   sizeof(double) * 2 * counts[b], hipMemcpyDefault) != hipSuccess)
      return fail(set_err(MFGP_ERR_DEVICE, "batch_sample_points: copy out failed"));
  }
  for (int b = 0; b < count; ++b) (void)plan_leave(t[b], sv[b]);
  entered = 0;
  const bool sync_ok = hipStreamSynchronize(s) == hipSuccess;   // (the restore copies read ws)
  (void)hipFree(ws);
  const auto tp3 = std::chrono::steady_clock::now();
  auto us = [](std::chrono::steady_clock::duration dt) {
    return (int64_t)std::chrono::duration_cast<std::chrono::microseconds>(dt).count();
  };
  c->plan_stats[8] += us(tp1 - tp0);
  c->plan_stats[9] += us(tp2 - tp1);
  c->plan_stats[10] += us(tp3 - tp2);
  return sync_ok ? MFGP_OK : set_err(MFGP_ERR_DEVICE, "batch_sample_points: restore failed");
}

// Voronoi-cell reductions (simulator.py:194-323) on the device. Inputs may be
// host or device memory (host ones are staged through the context workspace);
// outputs likewise. Synchronous. field (host, [ncells]) or null: cell i reads
// w / var of seed field[i] ([nfield][M] each; the lockstep simulations' batch).
static int cell_reduce_impl(mfgp_ctx* c, const double* grid, int64_t M, int ncells, const int* vstart,
                            const double* verts, const double* seeds, const int* field, int nfield, const double* w,
                            const double* f, const double* var, double* out, int64_t* argmax) {
  if (!c) return set_err(MFGP_ERR_ARG, "null ctx");
  if (M < 0 || ncells < 0 || (M > 0 && !grid) || (ncells > 0 && (!vstart || !verts || !seeds || !out || !argmax)))
    return set_err(MFGP_ERR_ARG, "bad cell_reduce arguments");
  if (field && nfield < 1) return set_err(MFGP_ERR_ARG, "nfield must be >= 1");
  if (M == 0 || ncells == 0) {
    for (int i = 0; i < ncells; ++i) {
      for (int j = 0; j < 6; ++j) out[6 * i + j] = (j == 5) ? -HUGE_VAL : 0.0;
      argmax[i] = -1;
    }
    return MFGP_OK;
  }
  // vertex counts (the offsets must be readable on the host)
  if (is_device_ptr(vstart)) return set_err(MFGP_ERR_ARG, "vstart must be host memory");
  if (field && is_device_ptr(field)) return set_err(MFGP_ERR_ARG, "field must be host memory");
  if (vstart[0] != 0) return set_err(MFGP_ERR_ARG, "vstart[0] must be 0");
  for (int i = 0; i < ncells; ++i) {
    if (vstart[i + 1] - vstart[i] > 256 || vstart[i + 1] < vstart[i])
      return set_err(MFGP_ERR_ARG, "cell %d: bad vertex count", i);
    if (field && (field[i] < 0 || field[i] >= nfield)) return set_err(MFGP_ERR_ARG, "cell %d: field out of range", i);
  }
  const int64_t nf = field ? nfield : 1;
  const int64_t nv = vstart[ncells];
  const int64_t npart = cell_partial_doubles(M, ncells);
  // workspace layout (doubles): grid 2M | w nf M | f M | var nf M | verts 2nv | seeds 2n | part | out 6n |
  // argmax n | vstart | field; an input already in device memory is read in place and
  // takes no room (the lockstep driver's w / var at configs[4] scale had
  // kept ~32 MB of workspace that was never written)
  auto host_n = [](const double* p, int64_t n) -> int64_t { return (p && !is_device_ptr(p)) ? n : 0; };
  const int64_t off_g = 0, off_w = off_g + host_n(grid, 2 * M), off_f = off_w + host_n(w, nf * M);
  const int64_t off_v = off_f + host_n(f, M), off_vx = off_v + host_n(var, nf * M);
  const int64_t off_s = off_vx + 2 * nv, off_p = off_s + 2 * ncells, off_o = off_p + npart;
  const int64_t off_a = off_o + 6 * ncells, off_i = off_a + ncells, off_fd = off_i + (ncells + 2) / 2 + 1;
  const int64_t total = off_fd + (ncells + 1) / 2 + 1;
  int rc = ensure_ws(c, sizeof(double) * total);
  if (rc) return rc;
  double* ws = c->ws;
  hipStream_t s = c->stream;
  auto stage = [&](const double* p, int64_t n, int64_t off) -> const double* {
    if (!p) return nullptr;
    if (is_device_ptr(p)) return p;
    if (hipMemcpyAsync(ws + off, p, sizeof(double) * n, hipMemcpyHostToDevice, s) != hipSuccess) return nullptr;
    return ws + off;
  };
  const double* dg = stage(grid, 2 * M, off_g);
  const double* dw = stage(w, nf * M, off_w);
  const double* df = stage(f, M, off_f);
  const double* dv = stage(var, nf * M, off_v);
  const double* dx = stage(verts, 2 * nv, off_vx);
  const double* ds = stage(seeds, 2 * ncells, off_s);
  if (!dg || !dx || !ds || (w && !dw) || (f && !df) || (var && !dv))
    return set_err(MFGP_ERR_DEVICE, "cell_reduce: staging failed");
  int* dvs = reinterpret_cast<int*>(ws + off_i);
  HIP_TRY(hipMemcpyAsync(dvs, vstart, sizeof(int) * (ncells + 1), hipMemcpyHostToDevice, s));
  int* dfd = nullptr;
  if (field) {
    dfd = reinterpret_cast<int*>(ws + off_fd);
    HIP_TRY(hipMemcpyAsync(dfd, field, sizeof(int) * ncells, hipMemcpyHostToDevice, s));
  }
  const bool dev_out = is_device_ptr(out) && is_device_ptr(argmax);
  double* o = dev_out ? out : ws + off_o;
  int64_t* a = dev_out ? argmax : reinterpret_cast<int64_t*>(ws + off_a);
  HIP_TRY(launch_cell_reduce(dg, M, dx, dvs, ncells, ds, dw, df, dv, dfd, ws + off_p, o, a, s));
  if (!dev_out) {
    HIP_TRY(hipMemcpyAsync(out, o, sizeof(double) * 6 * ncells, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(argmax, a, sizeof(int64_t) * ncells, hipMemcpyDeviceToHost, s));
  }
  HIP_TRY(hipStreamSynchronize(s));
  return MFGP_OK;
}

int mfgp_cell_reduce(mfgp_ctx* c, const double* grid, int64_t M, int ncells, const int* vstart, const double* verts,
                     const double* seeds, const double* w, const double* f, const double* var, double* out,
                     int64_t* argmax) {
  const DeviceGuard dg_(c ? c->device : -1);
  if (const int rc_ = settle(c)) return rc_;
  return cell_reduce_impl(c, grid, M, ncells, vstart, verts, seeds, nullptr, 1, w, f, var, out, argmax);
}

int mfgp_batch_cell_reduce(mfgp_ctx* c, const double* grid, int64_t M, int ncells, const int* vstart,
                           const double* verts, const double* seeds, const int* field, int nfield, const double* w,
                           const double* f, const double* var, double* out, int64_t* argmax) {
  const DeviceGuard dg_(c ? c->device : -1);
  if (const int rc_ = settle(c)) return rc_;
  if (!field) return set_err(MFGP_ERR_ARG, "null field");
  return cell_reduce_impl(c, grid, M, ncells, vstart, verts, seeds, field, nfield, w, f, var, out, argmax);
}

// likelihood (gp:81-106 / gp:344-385) and its analytic gradient on the device,
// for the model's data under the given hyperparameters (the model is unchanged).
int mfgp_nlml(mfgp_model* m, const double* hyp, int nhyp, double* nlml, double* grad) {
  const DeviceGuard dg_(m ? m->ctx->device : -1);
  if (const int rc_ = settle(m ? m->ctx : nullptr)) return rc_;
  int rc = check_model(m);
  if (rc) return rc;
  if (!hyp || nhyp != m->nhyp)
    return set_err(MFGP_ERR_ARG, "Hyperparameters must be of length 4 (single-fidelity) or 9 (multi-fidelity)");
  if (!nlml) return set_err(MFGP_ERR_ARG, "null output");
  mfgp_ctx* c = m->ctx;
  const int64_t N = m->NL + m->NH;
  if (N == 0) {   // empty data: every term is an empty sum
    *nlml = 0.0;
    if (grad)
      for (int p = 0; p < nhyp; ++p) grad[p] = 0.0;
    return MFGP_OK;
  }
  mfgp_model* t = nullptr;   // scratch factor of K(hyp)
  if ((rc = mfgp_model_create(c, m->kind, MFGP_F64, hyp, nhyp, m->jitter, &t))) return rc;
  double *Xi = nullptr, *Kv = nullptr, *al = nullptr, *part = nullptr, *val = nullptr;
  auto done = [&](int code) {
    if (Xi) (void)hipFree(Xi);
    if (Kv) (void)hipFree(Kv);
    if (al) (void)hipFree(al);
    if (part) (void)hipFree(part);
    if (val) (void)hipFree(val);
    mfgp_model_destroy(t);
    return code;
  };
  if ((rc = ensure_cap(t, N))) return done(rc);
  HIP_TRY(hipMemcpyAsync(t->X, m->X, sizeof(double) * 2 * N, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(t->y, m->y, sizeof(double) * N, hipMemcpyDeviceToDevice, c->stream));
  t->NL = m->NL;
  t->NH = m->NH;
  if ((rc = factor_one(t))) return done(rc);   // LinAlgError as the reference's cholesky (gp:101 / 380)
  int slot;
  GPDesc* hd = acquire_slot(c, slot, rc);
  if (!hd) return done(rc);
  fill_desc(hd[0], t);
  const GPDesc* dd = nullptr;
  if ((rc = upload_slot(c, slot, 1, &dd))) return done(rc);
  if (hipMalloc(&val, sizeof(double) * 2) != hipSuccess) return done(set_err(MFGP_ERR_DEVICE, "alloc"));
  if (launch_nlml_value(dd, 1, val, c->stream) != hipSuccess) return done(set_err(MFGP_ERR_DEVICE, "launch"));
  const int64_t ld = t->ld, np = nlml_partials(N);
  if (grad) {
    if (hipMalloc(&Xi, sizeof(double) * ld * ld) != hipSuccess || hipMalloc(&Kv, sizeof(double) * ld * ld) != hipSuccess ||
        hipMalloc(&al, sizeof(double) * ld) != hipSuccess || hipMalloc(&part, sizeof(double) * np) != hipSuccess)
      return done(set_err(MFGP_ERR_DEVICE, "nlml: out of device memory"));
    if (launch_nlml_grad(dd, N, Xi, Kv, al, part, c->stream) != hipSuccess)
      return done(set_err(MFGP_ERR_DEVICE, "nlml: launch failed"));
  }
  if ((rc = release_slot(c, slot))) return done(rc);
  double v[2] = {0.0, 0.0};
  std::vector<double> hp, ha;
  HIP_TRY(hipMemcpyAsync(v, val, sizeof(v), hipMemcpyDeviceToHost, c->stream));
  if (grad) {
    hp.resize(np);
    ha.resize(N);
    HIP_TRY(hipMemcpyAsync(hp.data(), part, sizeof(double) * np, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(ha.data(), al, sizeof(double) * N, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  // NLML = 1/2 r^T K^-1 r + sum log L_ii + N/2 log(2 pi)   (gp:104-105 / gp:383-384)
  *nlml = 0.5 * v[1] + v[0] + 0.5 * std::log(2.0 * M_PI) * (double)N;
  if (grad) {
    for (int p = 0; p < nhyp; ++p) grad[p] = 0.0;
    const int64_t ntiles = np / 9;
    double g9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t tt = 0; tt < ntiles; ++tt)
      for (int p = 0; p < 9; ++p) g9[p] += hp[tt * 9 + p];
    // mean terms a^T dr/dh (r = y - m(hyp), gp:89-90 / gp:415-424)
    const Hyp h = derive_hyp(m->kind, hyp, m->jitter);
    double sa_lo = 0.0, sa_hi = 0.0;
    for (int64_t i = 0; i < N; ++i) (i < m->NL ? sa_lo : sa_hi) += ha[i];
    if (m->kind == MFGP_SF) {
      grad[0] = -h.meanL * (sa_lo + sa_hi);
      grad[1] = g9[1];
      grad[2] = g9[2];
      grad[3] = g9[3];
    } else {
      for (int p = 0; p < 9; ++p) grad[p] = g9[p];
      grad[0] += -h.meanL * sa_lo - h.rho * h.meanL * sa_hi;
      grad[3] += -std::exp(hyp[3]) * sa_hi;
      grad[6] += -h.rho * h.meanL * sa_hi;
    }
  }
  return done(MFGP_OK);
}

int mfgp_batch_append_predict(mfgp_model** models, int count, const double* X, const double* y, const int64_t* k,
                              double* mu, double* var, int flags) {
  const DeviceGuard dg_((models && count > 0 && models[0]) ? models[0]->ctx->device : -1);
  if (const int rc_ = settle((models && count > 0 && models[0]) ? models[0]->ctx : nullptr)) return rc_;
  return batch_run(models, count, X, y, k, mu, var, nullptr, nullptr, flags, true, true);
}

int mfgp_batch_append_predict_ex(mfgp_model** models, int count, const double* X, const double* y,
                                 const int64_t* k, double* mu, double* var, double* var_max, int64_t* var_argmax,
                                 int flags) {
  const DeviceGuard dg_((models && count > 0 && models[0]) ? models[0]->ctx->device : -1);
  if (const int rc_ = settle((models && count > 0 && models[0]) ? models[0]->ctx : nullptr)) return rc_;
  if ((var_max && !is_device_ptr(var_max)) || (var_argmax && !is_device_ptr(var_argmax)))
    return set_err(MFGP_ERR_ARG, "var_max / var_argmax must be device memory");
  return batch_run(models, count, X, y, k, mu, var, var_max, var_argmax, flags, true, true);
}

int mfgp_batch_append_factor(mfgp_model** models, int count, const double* X, const double* y, const int64_t* k,
                             int flags) {
  const DeviceGuard dg_((models && count > 0 && models[0]) ? models[0]->ctx->device : -1);
  if (const int rc_ = settle((models && count > 0 && models[0]) ? models[0]->ctx : nullptr)) return rc_;
  return batch_run(models, count, X, y, k, nullptr, nullptr, nullptr, nullptr, flags, true, false);
}

int mfgp_batch_predict(mfgp_model** models, int count, double* mu, double* var, int flags) {
  const DeviceGuard dg_((models && count > 0 && models[0]) ? models[0]->ctx->device : -1);
  if (const int rc_ = settle((models && count > 0 && models[0]) ? models[0]->ctx : nullptr)) return rc_;
  return batch_run(models, count, nullptr, nullptr, nullptr, mu, var, nullptr, nullptr, flags, false, true);
}

}  // extern "C"
