/*
 * mfgp_hip.h -- C ABI of the MI355X GP posterior engine (libmfgp_hip.so).
 *
 * Drop-in boundary for the hot path of MSU-dcypherlab/mfgp-coverage: the
 * reference has no FFI layer, its boundary is the Python class API of
 * gaussian_process.py (imported at simulator.py:25). Each entry point below
 * replaces one reference method; the Python mirror
 * (mfgp_coverage_amd/gaussian_process.py) binds them with ctypes
 * (see INTEGRATION.md).
 *
 * Conventions
 *   - plain pointers and sizes; no torch / HIP types in the signatures
 *     (streams are passed as void*, i.e. a hipStream_t).
 *   - coordinates are row-major [n,2] float64, values [n] float64.
 *   - every data pointer may be host or device memory (detected with
 *     hipPointerGetAttributes); inputs are borrowed for the call and copied,
 *     outputs are written into caller buffers.
 *   - return 0 on success, else an MFGP_ERR_* code; mfgp_last_error() gives a
 *     thread-local message.
 */
#ifndef MFGP_HIP_H
#define MFGP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFGP_OK 0
#define MFGP_ERR_NOT_PD 1   /* Cholesky pivot <= 0: numpy.linalg.LinAlgError (gp:254, gp:529) */
#define MFGP_ERR_ARG 2      /* bad argument: TypeError/ValueError (simulator.py:366, 652)     */
#define MFGP_ERR_DEVICE 3   /* HIP runtime error: RuntimeError                                */

#define MFGP_SF 0           /* SFGP, gaussian_process.py:23-268, hyp [mu, s2, L, noise]              */
#define MFGP_MF 1           /* MFGP, gaussian_process.py:271-578, hyp [mu_lo,s2_lo,L_lo,mu_hi,s2_hi,
                               L_hi,rho,noise_lo,noise_hi] (all log-scaled, simulator.py:53-56)     */
#define MFGP_F64 0
#define MFGP_F32 1          /* BASELINE configs[4]: the resident V = L^-1 psi^T stored and streamed
                               in fp32, and the lattice step's F = L^-1 streamed in fp32 (built in
                               fp64, rounded once per build); factor, solves and reductions fp64.
                               Tolerance vs the fp64 oracle: oracle/gp_oracle.py parity_errors_f32
                               (F32_TOL = 1e-4) */

#define MFGP_ASYNC 1        /* batch flag: do not synchronise; status via mfgp_ctx_synchronize */

typedef struct mfgp_ctx mfgp_ctx;
typedef struct mfgp_model mfgp_model;

/* One context per host thread: owns a HIP stream and a scratch workspace. */
int mfgp_ctx_create(int device, mfgp_ctx** out);
void mfgp_ctx_destroy(mfgp_ctx* ctx);
/* Give back the context's scratch (the fp64 V scratch of MFGP_F32 full predicts,
 * up to 16 GB, and the workspace) after synchronising; the next call that needs
 * it allocates it again. Models keep their resident state. */
int mfgp_ctx_trim(mfgp_ctx* ctx);
/* Launch on a caller stream (hipStream_t) instead of the context's own. NULL restores it. */
int mfgp_ctx_set_stream(mfgp_ctx* ctx, void* hip_stream);
void* mfgp_ctx_get_stream(mfgp_ctx* ctx);
/* Wait for all work; returns MFGP_ERR_NOT_PD if an ASYNC batch hit a non-PD factor. */
int mfgp_ctx_synchronize(mfgp_ctx* ctx);
/* Incremental updates (default on): an append of k <= 16 rows to a current
 * factor is a bordered Cholesky step (L21 = K21 L11^-T, L22 = chol(K22 - L21 L21^T))
 * instead of the reference's full refactor (gp:254 / gp:529), and predict keeps
 * V = L^-1 psi^T resident so that it streams V once instead of recomputing it.
 * Results agree with the full path to rounding. 0 = refactor and recompute V
 * on every update, as the reference does. */
int mfgp_ctx_set_incremental(mfgp_ctx* ctx, int enable);
/* With incremental updates: run a batch's bordered appends and the one-pass
 * predicts that follow them as ONE launch (k_inc_stream: the append's producer
 * workgroups hand L21 / L22 to the cell tiles inside the kernel). Default on;
 * 0 = two launches (k_inc_stream for the append alone, then k_vstream). Same
 * numbers either way. */
int mfgp_ctx_set_fused(mfgp_ctx* ctx, int enable);
/* Deferred appends (default 0): mfgp_append of rows that a bordered append can
 * take only stages them; the next call that needs the factor runs the append --
 * mfgp_predict as one launch with the one-pass predict (the single-model form of
 * the batched path). A non-positive-definite append is then reported by that
 * call instead of by mfgp_append (the reference raises in updt / updt_hifi,
 * gp:254 / gp:529). */
int mfgp_ctx_set_deferred_appends(mfgp_ctx* ctx, int enable);
/* Lattice-separable appends (default on): when the grid is a lattice, kss /
 * (smallest noise + jitter) <= 1e4 and the model holds the posterior of the old
 * rows, a bordered append + predict of k <= 16 rows runs as k_inc_lat: w =
 * K11^-1 K12 from the resident explicit inverse L^-1, then the SE kernel's
 * separability over the two lattice axes turns L21 V_old into Z rows (per lattice
 * y-row, the sum of w c ex over the training rows on it) times axis-table rows,
 * a GEMM over 2 ny terms (f64 MFMA; a training row off the lattice adds one term)
 * -- no pass over V -- and var / mu are updated from the previous posterior.
 * Batches whose V stream is estimated cheaper (one GP at the headline size) keep
 * it; 2 = take the lattice step for them too (tests). 0 = always the V stream
 * (k_inc_stream). Same numbers to rounding. */
int mfgp_ctx_set_lattice(mfgp_ctx* ctx, int enable);
/* Declare that this context's launches may run concurrently with launches of
 * other contexts on the same GPU (several streams stepping independent batches
 * side by side, e.g. a rank's seeds as four sub-batches). Default 0. With it no
 * launch relies on all of its workgroups being resident at once: the lattice
 * step always runs its GEMM as the second launch (k_lat_gemm2) rather than as
 * split-K tiles that wait for each other inside the first. Every other
 * cross-workgroup wait in the library is on a workgroup with a lower linear id,
 * dispatched (and so resident) before its waiter, which stays safe when other
 * kernels share the GPU. */
int mfgp_ctx_set_concurrent(mfgp_ctx* ctx, int enable);
/* Kernel timing with HIP events on the launch stream: enable = 1 times every
 * predict-kernel launch (fused predict or one-pass incremental predict) and
 * every factor stage; 2 times the predict launches only (each event pair is a
 * few microseconds of stream time); 0 = off. */
int mfgp_ctx_enable_timing(mfgp_ctx* ctx, int enable);
/* Bracket only every stride-th eligible launch with events (default 1), so a
 * timed run samples kernel durations without paying the events on every step. */
int mfgp_ctx_set_timing_stride(mfgp_ctx* ctx, int64_t stride);
/* Sum of predict-kernel durations (ms) and launch count since the last reset;
 * also the same for the factor stage (assemble + blocked Cholesky). */
int mfgp_ctx_get_timing(mfgp_ctx* ctx, double* predict_ms, int64_t* predict_launches,
                        double* factor_ms, int64_t* factor_calls);
int mfgp_ctx_reset_timing(mfgp_ctx* ctx);
/* Path counters of the planners' loops (mfgp_sample_points,
 * mfgp_batch_sample_points: each model's appended rows, dropped at the end) since
 * the last reset: out[0..n) = {model runs, bordered appends, one-pass predicts (V stream or
 * lattice step), lattice steps, of them launched with their descriptors by
 * value, of them with the GEMM and cells as a second launch, full refactors, full
 * predicts, then the batched planner's host time in microseconds before, in and
 * after its iteration loop}; n <= 11. reset != 0 zeroes them after the read. Which
 * step form the Choi iterations took and where their time went (tools/bench_planner.py). */
int mfgp_ctx_planner_stats(mfgp_ctx* ctx, int64_t* out, int n, int reset);

/* SFGP.__init__ (gp:28-64) / MFGP.__init__ (gp:276-327) with the caller's
 * hyperparameters (the simulator overwrites .hyp right after construction,
 * simulator.py:72-73, 99-100). nhyp = 4 (SF) or 9 (MF). jitter = 1e-8 in the
 * reference (gp:42, gp:298). */
int mfgp_model_create(mfgp_ctx* ctx, int kind, int dtype, const double* hyp, int nhyp,
                      double jitter, mfgp_model** out);
void mfgp_model_destroy(mfgp_model* m);
/* copy.deepcopy(model) (simulator.py:339). */
int mfgp_clone(const mfgp_model* src, mfgp_model** out);
/* Writes to .hyp / .jitter; they take effect at the next factorisation. */
int mfgp_model_set_hyp(mfgp_model* m, const double* hyp, int nhyp, double jitter);

/* The grid X* of predict(X_star) (gp:121 / gp:401), [M,2]. Cached on the device. */
int mfgp_set_grid(mfgp_model* m, const double* xstar, int64_t M);

/* updt_info (gp:229-255 / gp:493-529): replace the training set and refactor.
 * SF uses only the H slots (XL/yL must be NULL/0). Returns MFGP_ERR_NOT_PD like
 * np.linalg.cholesky raising LinAlgError. */
int mfgp_set_data(mfgp_model* m, const double* XL, const double* yL, int64_t NL,
                  const double* XH, const double* yH, int64_t NH);

/* updt (gp:257-268) / updt_hifi (gp:531-542): append k >= 0 rows and refactor.
 * When the previous append was followed by a predict (the simulator's step), the
 * append also runs the one-pass predict in the same launch and keeps the result
 * for the next mfgp_predict; a non-PD step is still reported here. That launch
 * publishes the step's positive-definiteness verdict as soon as it has it, and
 * mfgp_append returns then, while the launch computes the posterior: the next
 * entry point called on the context waits for the launch first (and reports a
 * failure of its later phases, e.g. a hand-off wait's timeout), so the caller's
 * host work in between overlaps it (MFGP_EARLY_PD=0: return at the launch's end). */
int mfgp_append(mfgp_model* m, const double* X, const double* y, int64_t k);

/* predict (gp:121-148 / gp:401-438): posterior mean and the diagonal of the
 * posterior covariance at every grid cell (the only part the callers use,
 * simulator.py:301, 341, 672, 685, 842, 855, 1014). mu, var: [M], host or
 * device memory. Results for host buffers are kept with the model: predicts of
 * an unchanged model return them again (the same bits, no launch). */
int mfgp_predict(mfgp_model* m, double* mu, double* var);
/* mfgp_predict without the host copy (the drop-in predict's path): the result is
 * left in the model's mapped pinned result buffer, which is handed over to the
 * caller -- *mu, *var point into it (writable, [M] each) until
 * mfgp_release_view(*view); the model takes another buffer from a process-wide
 * pool for its next host-bound predict, so a predict of an unchanged model after
 * a view recomputes. M = 0: *mu = *var = *view = NULL. */
int mfgp_predict_view(mfgp_model* m, double** mu, double** var, void** view);
/* mfgp_predict_view that may hand over the buffer of an eager append's launch
 * still computing into it (mfgp_append above): then *running = 1 and the caller
 * must call mfgp_ctx_synchronize before it reads the buffer or gives it to anyone
 * (the drop-in predict wraps the arrays meanwhile); else *running = 0 and it is
 * mfgp_predict_view. */
int mfgp_predict_view_running(mfgp_model* m, double** mu, double** var, void** view, int* running);
/* Return a buffer handed over by mfgp_predict_view (any thread, any time, also
 * after its model or context is destroyed). */
int mfgp_release_view(void* view);
/* The fused np.amax / np.argmax of a handed-over buffer's variance (the eager
 * append's launch reduces them beside its status word): *valid = 1 and the max
 * and its first cell when the launch that wrote the buffer computed them, else
 * *valid = 0 (a predict without an append before it). Read after the buffer is
 * ready (mfgp_predict_view_running: after mfgp_ctx_synchronize). */
int mfgp_view_max(const void* view, double* vmax, int64_t* argmax, int* valid);

/* Sizes and state readers (the Python mirror's .X/.L attributes). */
int64_t mfgp_model_n(const mfgp_model* m);      /* N = NL + NH */
int64_t mfgp_model_nl(const mfgp_model* m);
int64_t mfgp_model_m(const mfgp_model* m);
/* Path introspection (tests / benchmarks): out[0..n) = {factor rows (-1 = none),
 * resident V rows, full refactors, bordered appends, full predicts, one-pass
 * predicts (V stream or lattice step), grid lattice axes nx, ny (0 = the grid is
 * not a lattice: appends locate new points by a scan), lattice steps, off-lattice
 * training rows of the last lattice step (read back from the device; synchronises
 * the context's stream; only when n > 9), lattice steps launched with their
 * descriptors as the kernel argument, lattice steps whose GEMM and cells ran as a
 * second launch (k_lat_gemm2 or k_lat_gemm3), batch predicts served from the
 * resident posterior because the model appended nothing (k_post_copy), eager
 * appends of one GP that returned at the launch's published L22 verdict
 * (mfgp_append above)}; n <= 14. */
int mfgp_model_stats(const mfgp_model* m, int64_t* out, int n);
/* Copy the lower Cholesky factor L [N,N] (row-major, zeros above the diagonal). */
int mfgp_get_factor(mfgp_model* m, double* L_out);

/* Batched update + predict over `count` independent GPs (Monte-Carlo seeds):
 * for model i append k[i] rows (rows of X/y, concatenated in model order),
 * refactor, and predict into mu + i*M_i, var + i*M_i (concatenated in model
 * order). One set of launches serves the whole batch. flags: MFGP_ASYNC. */
int mfgp_batch_append_predict(mfgp_model** models, int count, const double* X, const double* y,
                              const int64_t* k, double* mu, double* var, int flags);
/* A member with k[i] = 0 whose factor and resident posterior are current (it
 * was predicted before and nothing changed) is not recomputed: its outputs are its
 * resident posterior (the same bits as its last predict), copied by one launch for
 * all such members (device outputs; mfgp_model_stats counts them), and the step
 * runs over the others. */
/* mfgp_batch_append_predict plus fused reductions of each model's variance:
 * var_max[i] = np.amax of the posterior covariance (its largest diagonal entry,
 * simulator.py:672, 842, 1014) and var_argmax[i] = the first cell attaining it
 * (the argmax of compute_sample_points, sim:352). Either may be NULL; both are
 * device memory, written in stream order (no host round trip). */
int mfgp_batch_append_predict_ex(mfgp_model** models, int count, const double* X, const double* y,
                                 const int64_t* k, double* mu, double* var, double* var_max,
                                 int64_t* var_argmax, int flags);
/* The two halves of mfgp_batch_append_predict (append + refactor only; predict
 * from the current factors only). mfgp_batch_predict needs a current factor. */
int mfgp_batch_append_factor(mfgp_model** models, int count, const double* X, const double* y,
                             const int64_t* k, int flags);
int mfgp_batch_predict(mfgp_model** models, int count, double* mu, double* var, int flags);
/* compute_sample_points (simulator.py:326-374), the Choi planner's sample-set
 * selection, on the device: on a copy of `model` (the model is unchanged),
 * repeatedly append the grid cell of maximal posterior variance (first argmax)
 * with its posterior mean as the observation, until the maximal variance is
 * <= threshold or max_points points were chosen. points: [max_points, 2], host
 * or device; *count = points chosen. Each iteration is a 1-row bordered append
 * and a one-pass predict; the loop runs in chunks on the device (one host
 * synchronisation per 32 iterations). Needs the grid set and incremental
 * updates enabled. */
int mfgp_sample_points(mfgp_model* model, double threshold, int64_t max_points, double* points, int64_t* count);
/* mfgp_sample_points for `count` models stepped together (the Choi planner of many
 * Monte-Carlo seeds, sim:326-374 once per seed): per iteration one decision launch
 * for all models and one batched 1-row append + predict (the lattice step where
 * the batch takes it); each model stops at its own thresholds[b] (host or device)
 * or after max_points points, and is unchanged (each works on a copy). points:
 * [count][max_points][2], host or device; counts[b] = points chosen for model b.
 * The models share one context and dtype and need their grids set. */
int mfgp_batch_sample_points(mfgp_model** models, int count, const double* thresholds, int64_t max_points,
                             double* points, int64_t* counts);
/* Keep only the first n_keep_hifi hifi rows (no refactor; benchmark reset). */
int mfgp_truncate(mfgp_model* m, int64_t n_keep_hifi);
/* mfgp_truncate of count models with one call (the benchmark's per-step reset). */
int mfgp_batch_truncate(mfgp_model** models, int count, int64_t n_keep_hifi);

/* likelihood (gp:81-106 SF / gp:344-385 MF): the negative log-marginal
 * likelihood of the model's training data under the log-scaled hyperparameters
 * `hyp` (nhyp = 4 or 9; the model's own .hyp and factor are unchanged), and,
 * if grad != NULL, its gradient with respect to hyp ([nhyp]; the reference uses
 * autograd for it in train, gp:108-119 / 388-399). MFGP_ERR_NOT_PD as the
 * reference's cholesky raising LinAlgError. */
int mfgp_nlml(mfgp_model* m, const double* hyp, int nhyp, double* nlml, double* grad);

/* Voronoi-cell reductions over the grid (simulator.py:194-323). Cell i is the
 * closed polygon verts[vstart[i] .. vstart[i+1]) ([.,2], vertices of the
 * caller's bounded Voronoi region, sim:154-191; at most 256 per cell) with seed
 * seeds[i]. A grid point belongs to every cell whose polygon contains it by the
 * reference's in_polygon test (sim:105-124: matplotlib's crossing rule,
 * reproduced exactly). Per cell, out[6i .. 6i+6) = {points, sum w, sum w*x,
 * sum w*y, sum |x - seed|^2 * f, max var} and argmax[i] = first grid index of
 * the max var (-1 if the cell is empty). w (compute_centroids' mu, sim:231-283),
 * f (compute_loss' truth, sim:194-228) and var (compute_max_var, sim:286-323)
 * may each be NULL. Arrays may be host or device memory except vstart (host).
 * Synchronous. */
int mfgp_cell_reduce(mfgp_ctx* ctx, const double* grid, int64_t M, int ncells, const int* vstart,
                     const double* verts, const double* seeds, const double* w, const double* f,
                     const double* var, double* out, int64_t* argmax);

/* mfgp_cell_reduce over the partitions of several seeds in one launch (the
 * lockstep simulations of a seed batch, mfgp_coverage_amd/coverage.py: every
 * seed's loss partition of its agents and Lloyd partition of its centroids,
 * simulator.py:895-904). Cell i reads the fields of seed field[i]: w + field[i]*M
 * and var + field[i]*M (w and var are [nfield][M], e.g. the batch's posterior
 * means / variances as mfgp_batch_append_predict wrote them); f [M] is shared.
 * field and vstart are host memory. Same per-cell outputs as mfgp_cell_reduce
 * (bit for bit: a cell's reduction does not depend on the other cells).
 * Synchronous. */
int mfgp_batch_cell_reduce(mfgp_ctx* ctx, const double* grid, int64_t M, int ncells, const int* vstart,
                           const double* verts, const double* seeds, const int* field, int nfield,
                           const double* w, const double* f, const double* var, double* out, int64_t* argmax);

const char* mfgp_last_error(void);
const char* mfgp_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MFGP_HIP_H */
