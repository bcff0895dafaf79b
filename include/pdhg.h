/*
 * pdhg.h — C ABI of the MI355X-native PDHG iteration for Hamilton–Jacobi
 * optimal-control PDEs (drop-in for the hot path of
 * TingweiMeng/PDHG-optimal-control, jaxsrc/).
 *
 * Plain C types only: host pointers + sizes, an opaque context that owns all
 * device (HBM) memory.  Bound from Python with ctypes by
 * pdhg-optimal-control_amd/pdhg_amd/_native.py; any other FFI (cffi, a C++
 * caller) can bind the same symbols.  See INTEGRATION.md.
 *
 * Reference interfaces replaced (file:line in jaxsrc/):
 *   pdhg_create              problem setup done by solve_HJ            run_example.py:157-191
 *                            + set_up_example_fns / compute_Dxx_fft_fv set_fns.py:52-166, utils/utils_precond.py:42-71
 *   pdhg_set_state/get_state the (phi, rho, alp) arrays passed between the jitted updates
 *                                                                       utils/utils_pdhg_solver.py:48-50, 96-98 (returns)
 *   pdhg_update_primal       update_primal_1d / update_primal_2d      update_fns_in_pdhg.py:135-147
 *                            (+ phi_bar = 2 phi' - phi and err1 sums,  utils/utils_pdhg_solver.py:55, 58)
 *   pdhg_update_dual         update_dual_alternative (<= rho_alp_iters update_fns_in_pdhg.py:167-180
 *                            calls of update_dual_oneiter :150-165)
 *   pdhg_iterate             the body of PDHG_solver_oneiter's loop    utils/utils_pdhg_solver.py:51-88
 *                            (primal, extrapolation, dual, err1/err2, convergence and NaN stop tests)
 *
 * Return convention: every function returns PDHG_OK (0) or a negative
 * pdhg_status; pdhg_last_error() gives the message (thread-local).
 * Threading: a context is single-caller.  It drives one GPU on its own HIP
 * stream (every entry point makes the context's device current first).  Multi-GPU:
 * either one process per GPU with a t-slab / x-slab context each and the caller's
 * communicator (pdhg_create_slab, pdhg_create_xslab; pdhg_amd/slab.py over RCCL), or
 * one host thread over a device list (pdhg_create_multi).  See DESIGN.md §7.
 */
#ifndef PDHG_MI355X_H
#define PDHG_MI355X_H

#ifdef __cplusplus
extern "C" {
#endif

#define PDHG_ABI_VERSION 1

typedef enum pdhg_status {
  PDHG_OK = 0,
  PDHG_ERR_ARG = -1,          /* bad argument (null pointer, size, value)            */
  PDHG_ERR_UNSUPPORTED = -2,  /* (egno, ndim, bc) or size combination not supported  */
  PDHG_ERR_HIP = -3,          /* HIP runtime error (message has the HIP error string) */
  PDHG_ERR_STATE = -4,        /* call order / state error (e.g. dual before primal)   */
  PDHG_ERR_NOMEM = -5         /* device allocation failed                             */
} pdhg_status;

/* Problem description: one PDHG time window of T unknown time rows
 * (T = time_step_per_PDHG - 1, utils/utils_pdhg_solver.py:121-137).
 * Mirrors the static arguments of the reference's jitted updates. */
typedef struct pdhg_problem {
  int egno;          /* example 1, 2 or 3                          set_fns.py:52            */
  int ndim;          /* 1 or 2                                                              */
  int bc_x, bc_y;    /* 0 periodic, 1 Neumann (egno 3: bc_x = 1)   run_example.py:229-240   */
  int nx, ny;        /* grid; ny = 1 when ndim == 1                                         */
  int T;             /* unknown time rows: phi is [T+1, nx(,ny)], rho / alp are [T, ...]    */
  int precision;     /* 4 = fp32 (default, bench), 8 = fp64 (tight parity)                  */
  int rho_alp_iters; /* max dual sub-iterations per outer iteration (reference: 10)         */
  int reserved0;
  double dx, dy, dt;
  double epsl;       /* viscosity epsilon                                                   */
  double c_on_rho;   /* c in R_T += c/dt                           update_fns_in_pdhg.py:80 */
  double C, pow_, Ct;/* preconditioner; pow_ and Ct are honoured in 1-D only, as the
                        reference (update_fns_in_pdhg.py:146)                              */
  const double* xs;  /* [nx] grid x coordinates (x_arr[0,:,0(,0)])                         */
  const double* ys;  /* [ny] grid y coordinates (x_arr[0,0,:,1]); NULL when ndim == 1      */
} pdhg_problem;

typedef struct pdhg_stats {
  int iters_run;     /* outer iterations executed by this call (incl. the stopping one)     */
  int status;        /* 0 = ran all n_iters, 1 = converged (err1<eps && err2<eps), 2 = NaN  */
  int inner_last;    /* dual sub-iterations of the last executed outer iteration            */
  int inner_total;   /* dual sub-iterations summed over this call                            */
  double err1;       /* primal error ||phi'-phi||/||phi|| of the last executed iteration     */
  double err2;       /* dual error (utils/utils_pdhg_solver.py:60-68)                         */
  double err_inner;  /* last dual sub-iteration error (update_fns_in_pdhg.py:162-164)        */
  double rho_min, rho_max; /* not computed (NaN) unless requested; reserved                 */
  int nan_seen;      /* a NaN appeared in phi' or rho' during this call                        */
  int first_nan_iter; /* iteration of this call (1-based) whose phi' or rho' first held a NaN; 0: none */
} pdhg_stats;

typedef struct pdhg_ctx pdhg_ctx;

const char* pdhg_last_error(void);
int pdhg_abi_version(void);

/* Number of HIP devices visible (0 when no GPU / no driver). */
int pdhg_device_count(int* count);

/* Allocates all device buffers for the window.  device = HIP ordinal. */
int pdhg_create(const pdhg_problem* prob, int device, pdhg_ctx** out);
int pdhg_destroy(pdhg_ctx* ctx);

/* State in the reference layout, float64 host arrays (C order):
 *   phi [T+1][nx][ny], rho [T][nx][ny],
 *   alp: n_alp arrays (2 in 1-D, 4 in 2-D) each [T][nx][ny][n_ctrl]
 *        (n_ctrl = 1 in 1-D and for egno 3, 2 otherwise), passed as one
 *        contiguous [n_alp][T][nx][ny][n_ctrl] block.
 * Only the live control components are stored on the device:
 * set_state fails with PDHG_ERR_UNSUPPORTED if a dead component is non-zero;
 * get_state writes zeros there.  A null array is not transferred: set_state overwrites the given parts of the
 * current state and keeps the device's values of the others (window marching re-seeds phi alone when rho / alp
 * are the ones the device holds); it resets the iteration / stop bookkeeping either way. */
int pdhg_set_state(pdhg_ctx* ctx, const double* phi, const double* rho, const double* alp);
int pdhg_get_state(pdhg_ctx* ctx, double* phi, double* rho, double* alp);
int pdhg_get_phi_bar(pdhg_ctx* ctx, double* phi_bar);   /* [T+1][nx][ny] */
/* Rows [row0, row0 + nrows) of the state in the reference layouts (a window of 3.4e9 points per array, C3's and
 * C4's, does not fit a host copy): phi / phi_bar rows of [T+1] -> [nrows][nx][ny], rho rows of [T] -> [nrows][nx][ny],
 * alp -> [n_alp][nrows][nx][ny][n_ctrl] (dead components zero).  Null pointers are skipped; rho / alp need
 * row0 + nrows <= T.  Same values as the matching rows of pdhg_get_state / pdhg_get_phi_bar. */
int pdhg_get_rows(pdhg_ctx* ctx, int row0, int nrows, double* phi, double* phi_bar, double* rho, double* alp);
/* phi_bar input of the drop-in dual update (update_dual_oneiter's first argument). */
int pdhg_set_phi_bar(pdhg_ctx* ctx, const double* phi_bar);

/* The reference's PDHG_multi_step initial state for a window
 * (utils/utils_pdhg_solver.py:123-137): every phi row = g, rho = c_on_rho,
 * alp = 0.  g: [nx][ny] host float64.  Built on the device (HBM-resident). */
int pdhg_init_state(pdhg_ctx* ctx, const double* g);

/* One primal update: phi <- phi + tau * H1^{-1}(cont_residual(rho, alp));
 * also forms phi_bar = 2 phi' - phi and the err1 sums. */
int pdhg_update_primal(pdhg_ctx* ctx, double tau);

/* update_dual_alternative: up to rho_alp_iters sub-iterations with early exit
 * at err < eps; *inner_used receives the sub-iterations executed. */
int pdhg_update_dual(pdhg_ctx* ctx, double sigma, double eps, int rho_alp_iters, int* inner_used);

/* Errors of the last primal+dual pair (err1, err2) as utils_pdhg_solver.py:58-68. */
int pdhg_errors(pdhg_ctx* ctx, double* err1, double* err2);

/* Error of the last dual sub-iteration (update_fns_in_pdhg.py:162-164), the value
 * update_dual_oneiter returns as its third output. */
int pdhg_inner_error(pdhg_ctx* ctx, double* err);

/* Up to n_iters outer iterations on the device with the reference's stop
 * rules (converged, then NaN).  tau = stepsz/1.5, sigma = stepsz*1.5
 * (utils_pdhg_solver.py:44-46).  No host synchronisation per iteration. */
int pdhg_iterate(pdhg_ctx* ctx, int n_iters, double tau, double sigma, double eps, int rho_alp_iters,
                 pdhg_stats* out);

/* Stop rules of pdhg_iterate (default: both on, as the reference).  Benchmarks may turn the NaN
 * stop off so a diverging configuration still executes exactly n_iters iterations. */
int pdhg_set_stop_rules(pdhg_ctx* ctx, int stop_on_converge, int stop_on_nan);

/* Blocks until the context's stream is idle. */
int pdhg_synchronize(pdhg_ctx* ctx);

/* Device bytes held by the context. */
int pdhg_device_bytes(pdhg_ctx* ctx, unsigned long long* bytes);

/* Which kernel variant a context selected (no reference counterpart; tests and benches assert the fast
 * paths engaged): "fused_residual" 1/0 (the dual sweep forms the next residual, k_dual_lds_2d FR; fp32 and
 * fp64 -- fp64 on 128-column strips with 4-row residual tasks, 2-row tasks at ny = 8192; fp32 ny = 8192 on 4-row
 * tasks),
 * "fast_rows" 1/0 (fp32 8/4-row y-transform kernels), "fast_dual" (-1 generic, 0 row-per-thread,
 * RX rows through LDS), "dual_ypl" (y per lane of the LDS dual: 4, or 2 for fp64 with PDHG_DUAL_YPL=2;
 * 0 without it), "fast_xt" (0 generic, 1 single-role, 2 warp-specialised, 3 row-batched,
 * 4 row-batched with LDS-DMA staging x-transform, 5 its half-real form at nx = 8192), "half_real", "fourstep", "fs16" (1-D nx = 65536 as
 * 16 x 4096, fp32 and fp64), "fs_wide", "glb_line", "thomas_chunk" (1-D t-solve in chunks: 32 rows per wave
 * fp32, 16 rows per half-wave fp64), "rows_rw", "res_threads", "upd_threads",
 * "row_threads" (threads of the generic row kernels), "res64" 1/0 (fp64 residual and update through the
 * 4-row fast kernels, ny = 2048 / 4096), "contig_fail" (large arrays of an fp32 2-D context that fell back
 * from a physically contiguous allocation to hipMalloc; environment PDHG_ALLOC=contig|none overrides the
 * contiguous-for-fp32-2-D default), "dual64" 1/0 (fp64 contexts: the row-per-thread time-marching dual
 * k_dual_fast_2d<EGNO, double>, or with nx % 8 == 0 and T >= 3 the LDS-row sweep k_dual_lds_2d<EGNO, 8, .., double>;
 * default on where ny % 256 == 0, environment PDHG_DUAL64=0 selects the generic per-point kernel), "f64_xt" 1/0 (fp64
 * nx = 512 ... 8192: k_precond_xt_f64_2d; PDHG_XT64=0 the generic kernel), "ip_rows" 1/0 (fp64 ny = 8192: row pairs in
 * one padded line), "upd8192" 1/0 (fp64 ny = 8192 with half-real x blocks: the 2-row fast update), "tc_spec" 1/0
 * (fp64 C3 shape, windows of >= 100 rows: the residual spectrum in task order), "t1_xt64" 1/0 (fp64 one-row windows at a power-of-two nx in
 * 512..4096: the carry-free k_precond_x_t1_2d<..., double>; PDHG_T1_XT=0 off), "graph" 1/0 (pdhg_iterate replays
 * windows of iterations from a captured HIP graph; default on, environment PDHG_GRAPH=0 launches every
 * iteration eagerly), "graph_window" (iterations per replayed graph). */
int pdhg_path_info(pdhg_ctx* ctx, const char* key, int* value);

/* Per-launch kernel timing for the benchmark: HIP events recorded on the
 * context's stream around every launch of the named kernel class
 * ("dual", "precond_fwd", "precond_bwd", "residual", "update") while
 * enabled.  Returns the accumulated milliseconds and launch count. */
int pdhg_profile_enable(pdhg_ctx* ctx, int enable);
int pdhg_profile_query(pdhg_ctx* ctx, const char* kernel_class, double* total_ms, int* launches);

/* Algorithmic HBM bytes of one outer iteration for k dual
 * sub-iterations, and of one launch of the named kernel class. */
int pdhg_algorithmic_bytes(pdhg_ctx* ctx, int k, const char* kernel_class, double* bytes);

/* ---------------- t-slab decomposition (multi-GPU) ----------------
 * New capability: the reference (JAX, single device, README.md:6) has no distributed path.  A window's
 * T_total unknown time rows are split into contiguous slabs, one context (one GPU) each; a slab context
 * owns rows [j0, j0 + p->T) (its phi arrays hold p->T + 1 rows: row 0 is global phi row j0).  The
 * caller moves planes between slabs (RCCL; pdhg_amd/slab.py) and runs one outer iteration of
 * utils_pdhg_solver.py:51-88 as:
 *   plane_out(0, rho row 0) -> [to the previous slab] || residual(1)     (halo overlapped with interior rows)
 *   -> plane_in(0, next slab's rho row 0) -> residual(2) -> forward(tau) -> plane_out(2, [D, S1])
 *   -> [allgather] -> fixup(allDS, allGS, rank, n) -> backward(tau, sums) -> [allreduce sums]
 *   -> primal_finalize(sums) -> plane_out(1, phi_bar row T) -> [to the next slab]
 *      || dual(sigma, k, 0, sums, 1)                                        (halo overlapped with interior rows)
 *   -> plane_in(1, previous slab's phi_bar row T) -> dual(sigma, k, 0, sums, 2) -> [allreduce]
 *   -> dual_finalize(eps, 0, sums) -> per further sub-iteration s: dual(sigma, k, s, sums, 3) -> [allreduce]
 *   -> dual_finalize(eps, s, sums) -> outer(k, sums) -> [allreduce when k > 1] -> outer_finalize(eps, k, sums).
 * Neighbour-exchange form (pdhg_amd.slab default): instead of the allgather of full [D, S1] planes,
 * classify the modes once (pdhg_slab_long_modes: long-range where some slab's gain G >= delta, a few
 * thousand low frequencies), then per iteration send D to the next slab and S1 to the previous one
 * (point to point), allgather only plane_out(3) = [D, S1] of the long-range modes, and call
 * fixup_nb(D from the previous slab, S1 from the next, allLong, allGS, rank, n).  The terms dropped for
 * the other modes are below delta relative (oracle/slab_oracle.py thomas_slabs_neighbour).
 * `parts` bit 0 = the rows that do not read a halo plane, bit 1 = the row that does (residual: the last
 * row unless this is the window's last slab; dual: row 0 unless it is the first slab, then the sums).
 * The Thomas recurrences are affine in the carries entering a slab (oracle/slab_oracle.py): D = the
 * zero-carry forward sweep's last row, S1 = sum P'_k b0_k; allGS: every slab's [G, S2]
 * (pdhg_slab_carry_gain, iteration-invariant, gather once).  Planes are device pointers in the context's
 * precision (float for p->precision 4, double for 8; D/S1 and G/S2 are pairs of spectral planes, see
 * pdhg_slab_plane_size); sums are device vectors of 16 doubles.
 * All calls enqueue on the context's stream (pdhg_set_stream to share the caller's).
 * ndim 2.  fp32: a power-of-two ny in [256, 8192] (the residual's halo-row split runs the fast row kernels).
 * fp64 (the reference's arithmetic, jaxsrc/update_fns_in_pdhg.py:10): any ny; ny = 2048 / 4096 split the halo row
 * off with the 4-row kernels, other ny run the generic row kernels over the whole slab after the halo.  Any nx
 * the single context supports: the fast DHT x kernels (fp32), the fp64 nx = 4096 kernel and its half-real
 * nx = 8192 form (kernels_xt_f64.hpp), or the generic runtime-radix kernel (other nx, and egno 3's bc (1,0) DCT
 * along x, jaxsrc/utils/utils_precond.py:159-174). */
int pdhg_create_slab(const pdhg_problem* p, int j0, int T_total, int device, pdhg_ctx** out);
int pdhg_set_stream(pdhg_ctx* ctx, void* hip_stream);
int pdhg_slab_plane_size(pdhg_ctx* ctx, unsigned long long* spatial, unsigned long long* spectral);
int pdhg_slab_begin(pdhg_ctx* ctx);                                       /* reset the device loop control */
int pdhg_slab_carry_gain(pdhg_ctx* ctx, void* GS_out);                    /* [G, S2], 2 spectral planes */
int pdhg_slab_residual(pdhg_ctx* ctx, int parts);                          /* residual + y-DHT of rows */
int pdhg_slab_forward(pdhg_ctx* ctx, double tau);                          /* x-DHT + forward sweep, [D, S1] */
int pdhg_slab_fixup(pdhg_ctx* ctx, const void* all_DS, const void* all_GS, int rank, int nranks);
int pdhg_slab_long_modes(pdhg_ctx* ctx, const void* all_GS, int nranks, double delta, int* K);
int pdhg_slab_fixup_nb(pdhg_ctx* ctx, const void* D_left, const void* S1_right, const void* all_long,
                       const void* all_GS, int rank, int nranks);
int pdhg_slab_backward(pdhg_ctx* ctx, double tau, double* sums);           /* backward + inverse + update */
int pdhg_slab_primal_finalize(pdhg_ctx* ctx, const double* sums);
int pdhg_slab_dual(pdhg_ctx* ctx, double sigma, int rho_alp_iters, int sub, double* sums, int parts);
int pdhg_slab_dual_finalize(pdhg_ctx* ctx, double eps, int sub, const double* sums);
int pdhg_slab_outer(pdhg_ctx* ctx, int rho_alp_iters, double* sums);
int pdhg_slab_outer_finalize(pdhg_ctx* ctx, double eps, int rho_alp_iters, const double* sums);
int pdhg_slab_plane_out(pdhg_ctx* ctx, int which, void* dst); /* 0 rho row 0, 1 phi_bar row T, 2 [D, S1],
                                                                 3 [D, S1] of the long-range modes */
int pdhg_slab_plane_in(pdhg_ctx* ctx, int which, const void* src); /* 0 rho halo, 1 phi_bar row 0 */
int pdhg_slab_status(pdhg_ctx* ctx, pdhg_stats* st);
/* Partitioned carry exchange (pdhg_amd.slab default): the column blocks are split into nparts parts so the
 * neighbour planes of part q travel while part q+1 sweeps forward and part q-1 sweeps backward:
 *   per part: forward_part -> carry_out_part(DS) -> [D -> next slab, S1 -> previous slab, modes part_modes]
 *   plane_out(3) -> [allgather long-range modes]
 *   per part: [wait for its planes] -> fixup_nb_part -> backward_part;   then update(tau, sums).
 * forward_part(q, n) over all q equals slab_forward; backward_part over all q + update equals slab_backward. */
int pdhg_slab_part_modes(pdhg_ctx* ctx, int part, int nparts, unsigned long long* m0, unsigned long long* m1);
int pdhg_slab_forward_part(pdhg_ctx* ctx, double tau, int part, int nparts);
int pdhg_slab_carry_out_part(pdhg_ctx* ctx, void* dst, int part, int nparts);   /* [D, S1] planes, modes of part */
int pdhg_slab_fixup_nb_part(pdhg_ctx* ctx, const void* D_left, const void* S1_right, const void* all_long,
                            const void* all_GS, int rank, int nranks, int part, int nparts);
int pdhg_slab_backward_part(pdhg_ctx* ctx, double tau, int part, int nparts);
int pdhg_slab_update(pdhg_ctx* ctx, double tau, double* sums);            /* inverse y + update + sums */

/* ---------------- x-slab decomposition (multi-GPU for T = 1 marching windows) -----------
 * New capability (the reference has no distributed path).  The reference's default marches windows of
 * T = time_step_per_PDHG - 1 = 1 rows (run_example.py:425, utils_pdhg_solver.py:121-206), which a t-slab
 * cannot split; an x-slab splits the GLOBAL grid's nx rows into nranks contiguous slabs of nloc = nx/nranks
 * rows (a multiple of 8), one context per GPU.  `p` describes the global problem (nx, xs global).  The
 * context's spatial arrays are local: nx_local = nloc + 16 rows, row i = global row (x0 - xl0 + i) mod nx,
 * live rows [xl0, xl0 + nloc) (xl0 = 8); pdhg_set_state / get_state / init_state take and return arrays of
 * that shape (ghost and padding rows filled from the global arrays by periodic wrap).  One outer iteration
 * of utils_pdhg_solver.py:51-88:
 *   halo_out(0, buf) -> [allgather] -> halo_in(0, left's, right's) -> residual -> wire(0, send)
 *   -> [all-to-all] -> wire(1, recv) -> precond -> wire(2, send) -> [all-to-all] -> wire(3, recv)
 *   -> update(tau, sums) -> halo_out(1, buf) -> [allgather] || [allreduce sums] -> slab_primal_finalize(sums)
 *   -> halo_in(1, left's, right's) -> slab_dual(sigma, k, s, sums, 3) -> [allreduce] -> slab_dual_finalize ...
 *   -> slab_outer -> [allreduce when k > 1] -> slab_outer_finalize   (the t-slab phase functions).
 * halo_out: [2][nq][T][ny] (nq = 1 + live controls for which 0 = rho/alp of the current set, 1 for
 * which 1 = phi_bar rows 1..T); side 0 = the first live row (to the left neighbour), side 1 = the last.
 * halo_in takes the left neighbour's and the right neighbour's halo_out buffers (periodic ring).
 * wire: [nranks][T][nb/nranks][nloc][B] elements (pdhg_xslab_sizes), chunk q = for / from rank q; stage 0
 * packs the y-transformed rows, 1 unpacks the received rows into whole x lines, 2 packs the
 * preconditioned lines, 3 unpacks them back into rows.  Halo and wire elements are in the context's precision
 * (float for p->precision 4, double for 8 = the reference's arithmetic).  ndim 2, bc (0,0) or egno 3's (1,0) (the
 * outer slabs' outer ghost rows replicate their edge row), (ny/B) % nranks == 0; fp32: a power-of-two ny in
 * [256, 8192]; fp64: ny = 2048 or 4096 (the fp64 4-row row kernels) and nx != 8192. */
int pdhg_create_xslab(const pdhg_problem* p, int rank, int nranks, int device, pdhg_ctx** out);
int pdhg_xslab_layout(pdhg_ctx* ctx, int* x0, int* nloc, int* nx_local, int* xl0);
int pdhg_xslab_sizes(pdhg_ctx* ctx, unsigned long long* wire, unsigned long long* halo_state,
                     unsigned long long* halo_phibar);                     /* element counts */
int pdhg_xslab_halo_out(pdhg_ctx* ctx, int which, void* dst);
int pdhg_xslab_halo_in(pdhg_ctx* ctx, int which, const void* from_left, const void* from_right);
int pdhg_xslab_residual(pdhg_ctx* ctx);                                    /* residual + y-DHT, local rows */
int pdhg_xslab_wire(pdhg_ctx* ctx, int stage, void* buf);
int pdhg_xslab_precond(pdhg_ctx* ctx);                                     /* x-DHT, Thomas, inverse x-DHT */
int pdhg_xslab_update(pdhg_ctx* ctx, double tau, double* sums);            /* inverse y-DHT + update + sums */

/* ---------------- multi-device context (create over a device list) ----------------
 * Replaces the single-device pdhg_create of the drop-in for callers that bring no communicator: one host
 * thread drives ndev t-slab contexts (pdhg_create_slab, one per listed device; a device may repeat) through
 * the choreography above, with planes moved device to device by hipMemcpyPeerAsync (xGMI) and the stop-test
 * sums folded in slab order on the first device, so a C / Go / Java caller gets the multi-GPU window without
 * re-implementing pdhg_amd/slab.py or linking RCCL.  The window's rows [0, p->T) are split near-equally
 * (the first T % ndev slabs get one more row).  State arrays are the WHOLE window in the reference layouts
 * (as pdhg_set_state / pdhg_get_state).  Same support as the t-slab (fp32 or fp64, ndim 2, bc (0,0) or egno 3's
 * (1,0)).  The stop-test sums are gathered on the first device, folded in slab order and copied back; with
 * PDHG_MULTI_PEER_FOLD=1 (and peer access between every device pair) each device folds them from its peers'
 * buffers instead (opt-in until validated on separate devices).
 * Keys of pdhg_multi_info: "ndev", "long_modes", "rows:<i>" (rows of slab i), "peer_fold". */
typedef struct pdhg_multi pdhg_multi;
int pdhg_create_multi(const pdhg_problem* p, const int* devices, int ndev, pdhg_multi** out);
int pdhg_multi_destroy(pdhg_multi* m);
int pdhg_multi_set_state(pdhg_multi* m, const double* phi, const double* rho, const double* alp);
int pdhg_multi_get_state(pdhg_multi* m, double* phi, double* rho, double* alp);
int pdhg_multi_init_state(pdhg_multi* m, const double* g);        /* pdhg_init_state on every slab */
int pdhg_multi_iterate(pdhg_multi* m, int n_iters, double tau, double sigma, double eps, int rho_alp_iters,
                       pdhg_stats* out);                          /* utils_pdhg_solver.py:51-88 on all slabs */
int pdhg_multi_set_stop_rules(pdhg_multi* m, int stop_on_converge, int stop_on_nan);
int pdhg_multi_synchronize(pdhg_multi* m);
int pdhg_multi_info(pdhg_multi* m, const char* key, int* value);   /* + "parts", "device:<i>" */
/* Per-phase timing of the choreography (events on slab 0's main stream, cross-slab waits included) while
 * enabled; phases "residual", "forward", "backward", "allreduce", "dual", "outer", "step". */
int pdhg_multi_profile(pdhg_multi* m, int enable);
int pdhg_multi_phase_ms(pdhg_multi* m, const char* phase, double* total_ms, int* steps);

/* Identity of the built library: a hash of the sources it was compiled from (build() compares it with
 * the tree and rebuilds on a mismatch, so a stale libpdhg.so is never what the tests load). */
const char* pdhg_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* PDHG_MI355X_H */
