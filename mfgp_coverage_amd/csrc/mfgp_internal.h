// Internal types shared by the HIP kernels (mfgp_kernels.hip) and the C ABI
// (mfgp_capi.hip). Not part of the public interface (include/mfgp_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfgp {

constexpr int NB = 64;    // row block of the factor and of V = L^-1 psi^T
constexpr int BM = 64;    // grid cells per predict workgroup
constexpr int NT = 256;   // threads per workgroup (4 waves of 64)
constexpr int TILE = NB * NB;
constexpr int PRB = 128;  // predict: training rows per left-looking block
constexpr int PBM = 64;   // predict: grid cells per workgroup
constexpr int PNT = 256;  // predict: threads per workgroup (4 waves; two workgroups per CU)
constexpr int KINC = 16;  // incremental append: at most this many new rows per launch
constexpr int FUSED_CHUNK = 128; // rows of L21 per k_inc_stream producer workgroup
// iscr: [0] gathered flag | per-chunk partials | (at inc_l21c_offset, 128-byte
// aligned) the compact bordered rows L21c [cap][KINC]: row j holds L21[0..k)[j],
// then z1[j] at k (k < KINC), then zeros -- the cell tiles' MFMA A operand
constexpr int64_t inc_l21c_offset(int64_t cap) {
  return ((1 + KINC + ((cap + FUSED_CHUNK - 1) / FUSED_CHUNK) * (KINC * KINC + KINC)) + 15) / 16 * 16;
}
// then (128-byte aligned) the L22 record: L22 row-major [KINC][KINC] | z2 [KINC]
constexpr int64_t inc_l22r_offset(int64_t cap) { return (inc_l21c_offset(cap) + cap * KINC + 15) / 16 * 16; }
// then the producers' ready flags (k_inc_stream): one unsigned per FUSED_CHUNK-row
// chunk, holding the epoch of the launch whose compact rows of that chunk are stored
constexpr int64_t inc_pflag_offset(int64_t cap) { return inc_l22r_offset(cap) + KINC * KINC + KINC; }
constexpr int64_t inc_pflag_count(int64_t cap) { return (cap + FUSED_CHUNK - 1) / FUSED_CHUNK; }
constexpr int64_t inc_scratch_doubles(int64_t cap) { return inc_pflag_offset(cap) + (inc_pflag_count(cap) + 1) / 2; }
// k_inc_stream producers for a factor current for n0 rows (at least one: the finish)
inline int64_t fused_producers(int64_t n0) { return n0 > 0 ? (n0 + FUSED_CHUNK - 1) / FUSED_CHUNK : 1; }

// Hyperparameters in linear scale, derived on the host from the log-scaled
// vectors of simulator.py:53-56 / 83-84. SF uses the *L fields only.
struct Hyp {
  int kind;            // 0 = SF, 1 = MF
  int pad_;
  double sL, lL;       // output scale and length scale of k_L (SF: k)
  double sH, lH;       // k_H (MF only)
  double rho, rho2;    // AR(1) scale and rho*rho (gp:414, "rho ** 2")
  double noiseL, noiseH;
  double meanL, meanH; // prior means (gp:132 SF; gp:415-416 MF)
  double jitter;       // gp:42 / gp:298
  double kss;          // prior variance k**(x,x) (gp:146, gp:435-436)
};

// One GP of a batch. Device pointers; sizes in elements.
// A grid that is a lattice of two strictly monotone axes (cell e = ix*sx + iy*sy
// holds (xax[ix], yax[iy])), found by the host at set_grid; nx == 0 = not one.
// Lets the append kernel locate a grid point with a few probes instead of a scan.
struct GridLattice {
  int nx, ny;
  int64_t sx, sy;
  double x0, xinv, y0, yinv;   // index estimate: rint((x - x0) * xinv)
};

struct GPDesc {
  const double* X;     // [N,2] training coords: lofi rows [0,NL), hifi rows [NL,N)
  const double* y;     // [N]
  double* A;           // [ld,ld] column-major; lower triangle = L after the factor
  double* Linv;        // [nb][NB*NB] column-major inverses of the diagonal blocks of L
  const double* grid;  // [M,2]
  double* V;           // resident V = L^-1 psi^T: [ceil(M/PBM)][vld][PBM] (tile, row, cell); for an
                       // MFGP_F32 model: the fp64 scratch a full predict computes V in (k_predict)
  float* Vf;           // MFGP_F32 model: the resident V stored in fp32, same layout (null for F64)
  double* zv;          // [N] z = L^-1 (y - m)
  double* iscr;        // incremental append scratch: [0] = rows gathered from V, then per-chunk partial sums
  double* l21c;        // compact bordered rows [cap][KINC] inside iscr (inc_l21c_offset)
  double* l22r;        // L22 (row-major) | z2 of the last bordered append, inside iscr (inc_l22r_offset)
  double* mu;          // [M]
  double* var;         // [M]
  double* vmax;        // fused np.amax(var) (or null)
  int64_t* vargmax;    // fused first argmax of var (or null)
  double* tred;        // [1 + 2 ceil(M/PBM)]: tiles' arrival counter, then per-tile (max, argmax) of var
  int* gate;           // device loop gate (null = always run); 0 makes the gated kernels no-ops
  int* status;         // INT_MAX = ok, else 1 + first non-positive pivot row
  int* status_host;    // k_inc_stream with cell tiles: the launch's last cell group copies *status here
                       // (mapped pinned host word: the host reads it without a copy), or null
  int* pd_host;        // the fused step's L22 verdict (INT_MAX = positive definite, else the
                       // status value), published as soon as the finish knows it, or null
  const double* srcX;  // device rows to append at row N - k_new (k_append), or null
  const double* srcY;
  int64_t k_new;
  int rows_inline;     // 1: the k_new rows are rows_xy / rows_y below (a host append, k_new <= KINC)
  int pad_rows;
  double rows_xy[2 * KINC];
  double rows_y[KINC];
  int64_t ld, N, NL, M;
  int64_t vld;         // rows per V tile (>= prow_blocks(N) * PRB)
  int64_t n0;          // incremental kernels: rows [n0, N) are new (factor / V rows valid below n0)
  int64_t vres;        // k_inc_factor: rows of V valid for the current factor (0 = none)
  int64_t ablk;        // k_inc_factor: 64-row blocks of A / Linv already initialised
  GridLattice lat;     // lattice structure of `grid` (nx == 0: none)
  unsigned* sync;      // k_inc_stream hand-off: {producer arrivals, L21 ready, L22 / z2 ready}
  unsigned* pflag;     // k_inc_stream: per producer chunk, the epoch once its compact rows are stored (in iscr)
  unsigned epoch;      // k_inc_stream: value of this launch's ready flags (never 0)
  int nprod;           // k_inc_stream: producer workgroups ahead of the cell tiles
  int tiles;           // k_inc_stream: 1 = the launch also streams the cell tiles (one-pass predict)
  int l21c_ok;         // one-pass predict: l21c holds the rows [n0, N) bordered onto V's n0 rows
  int rsplit;          // one-pass predict: row splits per cell group (1, 2, 4; 128 / rsplit cells per workgroup)
  int vf32;            // 1 = the resident V is Vf (fp32; the one-pass predict streams 256 cells per workgroup)
  // lattice-separable step (k_inc_lat, mfgp_lattice.inl)
  float* Ff;           // MFGP_F32 models: F rounded to fp32 (the same layout), the copy the w units
                       // stream and extend (k_trinv_f still builds F in fp64; k_narrow_f rounds it)
  double* F;           // explicit L^-1, lower triangle in 64-column blocks: block jb holds rows
                       // [64 jb, ld) x 64 columns contiguously (F[i][j] at fblk_off(j / 64, ld) +
                       // (i - 64 (j / 64)) * 64 + j % 64); zeros above the diagonal
  double* tab;         // separable tables [4][ld][tabw]: c_L(j) ex_L, ey_L, c_H(j) ex_H, ey_H per training row j
  double* wv;          // w = L11^-T L21^T, [ld][KINC] (row j: w[j][0..KINC))
  unsigned* wflag;     // per 64-row block of w: the epoch of the launch that stored it
  double* gpart;       // split-K partial tiles [lat_tiles][ksplit][LAT_PART]
  unsigned* gcnt;      // per GEMM tile: arrivals of its splits (zero between launches)
  const double* rmu_in;   // resident posterior (mean, variance) of the n0 leading rows, [M]
  const double* rvar_in;
  double* rmu;         // resident posterior out [M]: every predict kernel writes it when non-null
  double* rvar;
  int64_t tabw;        // row width of the tables (a multiple of 64, >= nx, ny)
  int64_t tab_lo;      // k_lat_tables: rows [tab_lo, n0) are filled
  int ka;              // rows (new points) of a cell group in the GEMM: 8 (k <= 8) or 16
  int ksplit;          // split-K factor of the GEMM tiles
  int lat_tiles;       // GEMM tiles per GP: ceil(nx / (64 / ka)) * ceil(ny / 64)
  int nwb;             // 64-row blocks of w: ceil(n0 / 64)
  int lat_fbuild;      // k_trinv_f: 1 = compute F for the n0 factor rows
  int nwu;             // w units of the GP: each an equal share of F's 16-row steps (lat_wsteps)
  double* wpart;       // the units' partial w blocks [nwu + nwb][64 x 16] (unit u, block at position o of the pair order: slot u + o)
  unsigned* wcnt;      // per 64-column block: arrivals of its units' partials (zero between launches)
  // lattice-axis form of the step (every term on the lattice's own axis values)
  double* axt;         // axis tables [4][tabw + 1][tabw]: exp(-(a_p - a_col)^2 / 2 l^2) of the grid's
                       // axis values, x then y, L then H lengthscale; row tabw: zeros
  int* lidx;           // per training row: its lattice indices px | (py << 16), or -1 off the lattice
  double* zb;          // Z rows [P][zrows][tabw][ka]: per part and lattice y-row q (then per
                       // off-lattice "virtual" row), sum over the rows j on it of w[j][a] c_j ex_j(ix)
  int64_t zrows;       // Z rows per part: round_up(ny, ZKS) + ld (room for every row off the lattice)
  unsigned* zflag;     // per Z unit: the epoch once its rows are stored
  unsigned* ldone;     // [4]: w blocks stored (arrivals, zero between launches) | epoch once all are |
                       // Z units stored (arrivals) | epoch once all are
  int* zvl;            // per part [zrows + 1]: the count of virtual rows, then their training rows
  int nzu;             // Z units per GP: parts x ceil(ny / zq)
  int zq;              // lattice y-rows per Z unit (2 NT / tabw)
  int lat_axbuild;     // k_lat_axes: 1 = build axt (new grid or hyperparameters)
  int lat_selfg;       // k_inc_lat: 1 = the w units gather L21 from V themselves (lattice cells)
  int lat_g2;          // 1 = the GEMM and cells run as a second launch (k_lat_gemm2; lat_tiles are
                       // its 64-row tiles), k_inc_lat has no GEMM roles
  int lat_zcsr;        // 1 = one scan unit per part (the launch's first roles) lists the members by
                       // lattice row in csr, and the Z units read their rows' lists (lat_zunit_csr)
  unsigned* csr;       // member lists, per part [tabw + 1 + ld]: offsets by lattice y-row [ny + 1],
                       // then the members (px << 16) | j in row order, rows ascending (csr_bytes)
  Hyp hf;              // hyperparameters of the factorisation (updt_info time)
  Hyp hp;              // hyperparameters of predict (predict time)
};

// lattice step: w is computed by units that each stream an equal share of F's
// lower triangle, taken as one sequence of 16-row steps (block jb: ceil(n0 / 16) -
// 4 jb steps, block after block); at most LAT_WU_MAX units per GP, and n0 within
// LAT_NWB_MAX blocks of 64 columns
constexpr int LAT_WU_MAX = 512;
constexpr int LAT_NWB_MAX = 256;
constexpr int ZKS = 8;   // lattice-axis GEMM: K rows per pipeline stage (Z / axis-table rows)
// F's column block jb starts at fblk_off(jb, ld): blocks b < jb hold ld - 64 b rows of 64
inline __host__ __device__ int64_t fblk_off(int64_t jb, int64_t ld) { return 64 * jb * ld - 2048 * jb * (jb - 1); }
inline __host__ __device__ int64_t fblk_size(int64_t ld) { return fblk_off(ld / 64, ld); }
inline __host__ __device__ int64_t lat_wsteps(int64_t n0) {
  const int64_t C = (n0 + 15) / 16, nwb = (n0 + 63) / 64;
  return nwb * C - 2 * nwb * (nwb - 1);
}
inline __host__ __device__ int64_t nblocks_factor(int64_t N) { return (N + 1 + NB - 1) / NB; }
inline __host__ __device__ int64_t nblocks_rows(int64_t N) { return (N + NB - 1) / NB; }
inline __host__ __device__ int64_t ntiles_grid(int64_t M) { return (M + PBM - 1) / PBM; }
// one-pass predict workgroups: 128 / rsplit cells (32 per wave and row split); an
// fp32 V: 256 cells (64 per wave, no row splits)
inline __host__ __device__ int64_t ntiles_wg(int64_t M, int rsplit = 1, int vf32 = 0) {
  const int64_t c = vf32 ? 4 * PBM : 2 * PBM / rsplit;
  return (M + c - 1) / c;
}
inline __host__ __device__ int64_t prow_blocks(int64_t N) { return (N + PRB - 1) / PRB; }

// Launchers (mfgp_kernels.hip). `d` points to `count` descriptors in device memory.
hipError_t launch_append(const GPDesc* d, int count, hipStream_t s);
hipError_t launch_assemble(const GPDesc* d, int count, int64_t max_tiles, hipStream_t s);
hipError_t launch_potrf_diag(const GPDesc* d, int count, int kb, hipStream_t s);
hipError_t launch_panel(const GPDesc* d, int count, int kb, int64_t max_below, hipStream_t s);
hipError_t launch_syrk(const GPDesc* d, int count, int kb, int64_t max_tri, int t0, hipStream_t s);
hipError_t launch_syrk_blk(const GPDesc* d, int count, int kb0, int nk, int jmin, int jmax, int64_t max_tiles,
                           hipStream_t s);
hipError_t launch_predict(const GPDesc* d, int count, int64_t max_ctiles, hipStream_t s);
#ifdef MFGP_STAMPS
hipError_t set_stamps(long long* p);
#endif
hipError_t launch_extract_z(const GPDesc* d, int count, int64_t max_n, hipStream_t s);
// bordered append (k_inc_stream without cell tiles); max_nprod = max over GPs of nprod
// vf32: the batch's models store V in fp32 (GPDesc::Vf); a batch is of one V precision
hipError_t launch_inc_factor(const GPDesc* d, int count, int64_t max_nprod, int vf32, hipStream_t s);
// Descriptors of a batch passed by value as the kernel argument (k_inc_stream_arg,
// k_inc_lat_arg): a batch step that is one launch then uploads nothing
constexpr int DESC_ARG_MAX = 8;
struct DescArg {
  GPDesc d[DESC_ARG_MAX];
};
// bordered append + one-pass predict in one launch; max_blocks = max over GPs of nprod + cell tiles
hipError_t launch_inc_stream(const GPDesc* d, int count, int64_t max_blocks, int vf32, hipStream_t s);
// the same for ONE GP with its descriptor passed by value (kernel argument): no
// descriptor upload, and with rows_inline no row copies either
hipError_t launch_inc_stream1(const GPDesc& d, int64_t blocks, int vf32, hipStream_t s);
// the same for count <= DESC_ARG_MAX GPs from host descriptors passed by value
hipError_t launch_inc_stream_arg(const GPDesc* h, int count, int64_t max_blocks, int vf32, hipStream_t s);
// The member lists of the scan units (GPDesc::csr, per model): [2 parts][tabw + 1 + ld]
// unsigned (the offsets by lattice y-row, then the members)
__host__ __device__ inline int64_t csr_bytes(int64_t tabw, int64_t ld) { return 4 * 2 * (tabw + 1 + ld); }
// MFGP_F32 models whose F was just built (lat_fbuild): Ff = (float) F over F's storage
hipError_t launch_narrow_f(const GPDesc* d, int count, int64_t max_elems, hipStream_t s);
// the second launch of a lattice step (lat_g2): its GEMM and cells, max_tiles =
// max over GPs of lat_tiles
hipError_t launch_lat_gemm2(const GPDesc* d, int count, int64_t max_tiles, int ka, int vf32, hipStream_t s);
hipError_t launch_lat_gemm2_arg(const GPDesc* h, int count, int64_t max_tiles, int ka, int vf32, hipStream_t s);
// lattice-separable append + predict (k_inc_lat); max_blocks = max over GPs of
// nprod + nwu + lat_tiles * ksplit
// g1: the GEMM tiles are roles of this launch (else k_lat_gemm2 follows: lat_g2)
hipError_t launch_inc_lat(const GPDesc* d, int count, int64_t max_blocks, int ka, int vf32, bool g1, hipStream_t s);
// the same with the `count` <= DESC_ARG_MAX host descriptors `h` passed by value as
// the kernel argument (DescArg: no device copy of the descriptor array)
hipError_t launch_inc_lat_arg(const GPDesc* h, int count, int64_t max_blocks, int ka, int vf32, bool g1,
                              hipStream_t s);
// separable tables and lattice indices of rows [tab_lo, n0); max_rows = max over GPs of n0 - tab_lo
hipError_t launch_lat_tables(const GPDesc* d, int count, int64_t max_rows, hipStream_t s);
// axis tables (GPs with lat_axbuild); max_tabw = max over GPs of tabw
hipError_t launch_lat_axes(const GPDesc* d, int count, int64_t max_tabw, hipStream_t s);
// F = L^-1 of the n0 factor rows (block column per workgroup); max_nbr = max nblocks_rows(n0)
// F = L^-1 for the lattice step: recursive doubling with tscr (trinv_scratch(max_nbr)
// doubles per GP, tstride apart), or the block-column form without scratch
hipError_t launch_trinv_f(const GPDesc* d, int count, int64_t max_nbr, double* tscr, int64_t tstride, hipStream_t s);
int64_t trinv_scratch(int64_t nbr);
hipError_t launch_vstream(const GPDesc* d, int count, int64_t max_ctiles, int vf32, hipStream_t s);
// MFGP_F32 full predict: round the fp64 V that k_predict wrote into d.V (rows [0, N)
// of every tile) into the resident fp32 V (d.Vf)
hipError_t launch_vnarrow(const GPDesc* d, int count, int64_t max_tiles, hipStream_t s);
// field: null, or per cell the seed whose w / var it reads (w + field[cell] * M)
hipError_t launch_cell_reduce(const double* grid, int64_t M, const double* verts, const int* vstart, int ncells,
                              const double* seeds, const double* w, const double* f, const double* var,
                              const int* field, double* part, double* out, int64_t* argmax, hipStream_t s);
int64_t cell_partial_doubles(int64_t M, int ncells);
// the resident posterior of an unchanged model into a batch's outputs (k_post_copy):
// mu / var [M] copied from smu / svar, *vmax = max var, *vargmax = its first cell
struct PostCopy {
  const double* smu;
  const double* svar;
  double* mu;
  double* var;
  double* vmax;        // or null
  int64_t* vargmax;    // or null
  int64_t M;
};
constexpr int POST_MAX = 32;   // models per k_post_copy launch (descriptors by value)
struct PostArg {
  PostCopy p[POST_MAX];
};
hipError_t launch_post_copy(const PostCopy* h, int count, hipStream_t s);
hipError_t launch_nlml_value(const GPDesc* d, int count, double* out, hipStream_t s);
hipError_t launch_nlml_grad(const GPDesc* d, int64_t N, double* Xi, double* Kv, double* alpha, double* part,
                            hipStream_t s);
int64_t nlml_partials(int64_t N);
hipError_t launch_choi_select(const GPDesc* d, double threshold, double* points, int64_t max_points,
                              hipStream_t s);
hipError_t launch_choi_select_batch(int count, const int* pos, int64_t* state, const double* thr, const double* vmax,
                                    const int64_t* vargmax, const double* mu, const int64_t* moff,
                                    const double* const* grids, const int64_t* Ms, double* xn, double* yn,
                                    double* pts, int64_t max_points, hipStream_t s);

}  // namespace mfgp
