/*
 * cfd.h — C ABI of the MI355X-native pressure-projection hot path of
 * TSultanov/cfd-demo (src/model.rs).  Plain C types only: an opaque handle,
 * POD structs, float/uint8 pointers and sizes.  No torch or HIP types cross
 * this boundary.
 *
 * Each entry point replaces one method of the reference's `Model`
 * (/root/reference/src/model.rs); the citation is given per function.  The
 * reference has no FFI of its own; INTEGRATION.md shows the Rust `extern "C"`
 * block and wrapper a maintainer would add to keep src/app.rs unchanged.
 *
 * Conventions
 *   - return 0 on success, a negative cfd_status on failure; cfd_last_error()
 *     returns a thread-local message for the last failure on this thread.
 *   - a handle is thread-affine (the reference moves Model into one worker
 *     thread, model.rs:1287); calls on one handle must not race.
 *   - host buffers are caller-owned; sizes follow the reference's flat
 *     row-major layout (model.rs:161-214):
 *        u: (nx+1)*ny   v: nx*(ny+1)   p, rhs, p_prime: nx*ny
 *     For a sharded model (cfd_create_sharded) every host buffer covers the
 *     rank's slab only: pressure rows [j0, j1) (cfd_get_slab), u rows
 *     [j0, j1), v rows [j0, j1] (the shared face row j1 is held by both
 *     neighbouring ranks).
 *   - the precondition nx % 8 == 0 of the reference's 8-lane loops
 *     (model.rs:541, 402-403) is enforced: other shapes return CFD_EINVAL.
 *   - cfd_update / cfd_update_n are asynchronous: they enqueue the step on the
 *     model's HIP stream and return.  Reading calls (snapshot, state,
 *     residuals) synchronise.
 */
#ifndef CFD_H
#define CFD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CFD_ABI_VERSION 1

typedef enum {
    CFD_OK = 0,
    CFD_EINVAL = -1,   /* bad argument or unsupported shape (nx % 8 != 0, ...) */
    CFD_EHIP = -2,     /* HIP runtime error (no device, out of memory, launch) */
    CFD_ERCCL = -3,    /* RCCL error (sharded models only) */
    CFD_ESTATE = -4,   /* call not valid in the model's current state */
    CFD_ENONFINITE = -5, /* a finished step left NaN/Inf in u or v (failure detection;
                            the reference has none): cfd_update refuses to step on
                            and cfd_get_residuals reports it (filling *out all the
                            same) until cfd_set_state injects a new state */
    CFD_ETIMEOUT = -6, /* a persistent Jacobi solve (k_jacobi_persist: CFD_PERSIST=1,
                          or slabs with CFD_PERSIST_SHARDED=1) or the resident
                          tolerance-mode solve (k_jacobi_resident: small single-domain
                          grids by default) waited past its deadline
                          (CFD_PERSIST_DEADLINE_US, default 10 s).  For the persistent
                          solve that is a fault (it completes with any number of its
                          workgroups resident); the resident solve needs all its
                          workgroups co-resident, so co-tenant kernels that hold CUs for
                          seconds can cause it.  Self-recovering since r5: the model
                          checkpoints its state (device copies) before the first
                          cfd_update_n / cfd_pressure_solve / cfd_piso_step after a
                          synchronisation whenever such a solve may run; the call that
                          detects the timeout (a synchronising call, or the next
                          cfd_update_n on a single domain) restores that checkpoint,
                          re-runs every call since with one launch per block, and
                          returns CFD_ETIMEOUT with the state VALID (that detecting
                          cfd_update_n itself enqueued nothing).  Slabs tell each
                          other through the step all-reduce and recover at the same
                          synchronisation.  Solves run per launch from then on;
                          cfd_get_recoveries counts these.  CFD_CKPT=0 disables the
                          checkpoint: the state is then invalid until cfd_set_state */
} cfd_status;

typedef struct cfd_model cfd_model;

/* Grid + optional Cylinder (model.rs:119-139).  dx = lx/nx and dy = ly/ny
 * are derived exactly as src/app.rs:37-38 does. */
typedef struct {
    uint64_t nx, ny;
    float lx, ly;
    int32_t has_cylinder;
    float cylinder_x, cylinder_y, cylinder_radius;
} cfd_grid;

/* SimulationParams (model.rs:13-21) + this build's knobs.  Reference
 * behaviour is jacobi_iters 50, corrector_passes 20, tol_enabled 1,
 * p_tol 1e-4, bc_kind CFD_BC_CHANNEL. */
enum { CFD_SCHEME_FIRST_ORDER = 0, CFD_SCHEME_SECOND_ORDER = 1 };
enum { CFD_INLET_UNIFORM = 0, CFD_INLET_PARABOLIC = 1 };
/* Pressure solver of each solve piso_step runs (model.rs:684, :710).
 * JACOBI is the reference's (model.rs:734-824).  SOR and MULTIGRID are the
 * solvers of the reference's JavaScript variant (index.html:741-774 and
 * :775-795 + :1344-1470): p' restarts from 0 each solve, arithmetic in double
 * with f32 storage as in the script; SOR is swept red-black (omega 1.7,
 * jacobi_iters iterations, early exit at p_tol); MULTIGRID runs 3 V-cycles and
 * reports max |A p' - rhs|.  Both run on sharded models too (>= 16 interior
 * rows and halo depth >= 2 per slab), bit-identical to the unsharded solve.
 * SOR, fixed count (tol_enabled 0): deep ghosts -- an hg-row p' exchange
 * every hg/2 iterations, the iterations between recomputing shrinking ghost
 * bands; with the tolerance on, a 2-row exchange and an all-reduced residual
 * per iteration (checked one iteration behind).  MULTIGRID: the fine levels
 * whose every slab boundary divides by 2^(l+1) (>= 16 rows per slab there)
 * are partitioned -- each rank smooths, forms residuals and restricts only
 * its rows, with 8-row ghost exchanges per level -- and the coarser levels
 * are gathered and solved whole on every rank. */
enum { CFD_SOLVER_JACOBI = 0, CFD_SOLVER_SOR = 1, CFD_SOLVER_MULTIGRID = 2 };
enum { CFD_BC_CHANNEL = 0, CFD_BC_CAVITY = 1 };
typedef struct {
    float dt;
    float viscosity;
    float target_inlet_velocity;   /* channel: inlet U; cavity: lid U */
    int32_t velocity_scheme;
    int32_t inlet_profile;
    int32_t pressure_solver;
    int32_t jacobi_iters;          /* sweeps per pressure solve (model.rs:737) */
    int32_t corrector_passes;      /* extra correction passes (model.rs:696) */
    int32_t tol_enabled;           /* early exits at p_tol (model.rs:816, 721) */
    float p_tol;
    int32_t bc_kind;
} cfd_params;

/* Residuals (model.rs:23-32). step_time_s is device time of the last step
 * measured with HIP events. */
typedef struct {
    uint64_t simulation_step;
    float simulation_time;
    float dt;
    float p, u, v;
    double step_time_s;
    uint32_t piso_substeps;
    uint64_t jacobi_sweeps_total;
} cfd_residuals;

/* Full persistent state: enough to resume bit-exactly.
 * Any pointer may be NULL to skip that field. */
typedef struct {
    float *u, *v, *p, *u_star, *v_star, *p_prime, *rhs;
    float dt;
    float simulation_time;
    uint64_t simulation_step;
    float last_p_residual, last_u_residual, last_v_residual;
    uint64_t jacobi_sweeps_total;
} cfd_state;

/* SimulationParams::default() (model.rs:44-55) + reference knob values. */
void cfd_default_params(cfd_params *out);
/* default_grid() (src/app.rs:32-53): 800 x 264, 30 x 10, cylinder r 0.75. */
void cfd_default_grid(cfd_grid *out);

/* Model::new (model.rs:219-299) on HIP device `device_ordinal`. */
int cfd_create(const cfd_grid *grid, const cfd_params *params, int device_ordinal,
               cfd_model **out);

/* 1D row-slab decomposition over n_ranks processes (one per GPU).  Rank 0
 * calls cfd_rccl_unique_id and distributes the 128 bytes out of band
 * (bench.py uses torch.distributed).  Results are bitwise identical to the
 * single-GPU model: the path has no sums across ranks, only halo copies and
 * exact maxima. */
int cfd_rccl_unique_id(void *out_128_bytes);
int cfd_create_sharded(const cfd_grid *grid, const cfd_params *params, int device_ordinal,
                       int n_ranks, int rank, const void *rccl_unique_id, cfd_model **out);
/* Testing stand-in for the RCCL communicator: n_ranks slabs inside ONE
 * process (one host thread per slab, any devices, several may share a GPU);
 * halo exchanges become device-to-device copies between the members and the
 * max all-reduce a host fold.  Kernels and row plans are those of the RCCL
 * path; only the transport differs.  Destroy the hub after its members. */
void *cfd_local_hub_create(int n_ranks);
void cfd_local_hub_destroy(void *hub);
int cfd_create_sharded_local(const cfd_grid *grid, const cfd_params *params, int device_ordinal,
                             int n_ranks, int rank, void *hub, cfd_model **out);
/* HIP devices visible to this process (bench.py's launched ranks check that
 * there is one per rank before creating anything). */
int cfd_device_count(int *n_out);
/* Ranks the model's transport reports: ncclCommCount of the RCCL
 * communicator, the LocalHub's size, or 1 for an unsharded model. */
int cfd_get_comm_size(const cfd_model *m, int *n_out);
/* Global pressure rows [j0, j1) held by this model (0, ny for cfd_create). */
int cfd_get_slab(const cfd_model *m, uint64_t *j0, uint64_t *j1);

/* Model::update (model.rs:304-379): one time step, asynchronous. */
int cfd_update(cfd_model *m);
/* n consecutive Model::update calls, enqueued without host round trips. */
int cfd_update_n(cfd_model *m, int n);
/* piso_step (model.rs:529-730) with an explicit dt_sub; no u_old copy, no
 * residual/CFL bookkeeping. */
int cfd_piso_step(cfd_model *m, float dt_sub);
/* jacobi_pressure (model.rs:734-824) on the current rhs and p_prime.
 * Synchronous; writes the returned max |dp'| to *residual_out (may be NULL). */
int cfd_pressure_solve(cfd_model *m, float *residual_out);

/* Single phases of piso_step, for known-answer tests. */
enum {
    CFD_PHASE_U_PREDICTOR = 0,   /* model.rs:538-580   */
    CFD_PHASE_V_PREDICTOR = 1,   /* model.rs:586-670   */
    CFD_PHASE_DIVERGENCE = 2,    /* model.rs:1406-1440 */
    CFD_PHASE_CORRECTOR = 3,     /* model.rs:1334-1404 */
    CFD_PHASE_BOUNDARY = 4,      /* model.rs:826-875   */
};
int cfd_run_phase(cfd_model *m, int phase, float dt_sub);

/* set_parameters (model.rs:1250-1257). */
int cfd_set_params(cfd_model *m, const cfd_params *params);
/* get_snapshot (model.rs:1259-1267): copies u, v, p (NULL skips) and dt. */
int cfd_get_snapshot(cfd_model *m, float *u, float *v, float *p, float *dt_out);
/* get_residuals (model.rs:1269-1280). */
int cfd_get_residuals(cfd_model *m, cfd_residuals *out);
/* Whole state, for fixtures and checkpoint/resume. */
int cfd_get_state(cfd_model *m, cfd_state *st);
int cfd_set_state(cfd_model *m, const cfd_state *st);
/* Obstacle masks as built by Model::new (u8, u and v layouts). */
int cfd_get_masks(cfd_model *m, uint8_t *mask_u, uint8_t *mask_v);

/* Wait for all work enqueued on the model's stream. */
int cfd_synchronize(cfd_model *m);
/* Last Jacobi kernel duration in ms averaged over the sweeps of the most
 * recent cfd_profile_sweeps() call; measured with HIP events on the
 * model's stream. */
int cfd_profile_sweeps(cfd_model *m, int n_sweeps, double *avg_ms_out);

/* Event timing of the pressure solves and whole steps inside cfd_update:
 * cfd_timing_begin starts recording, cfd_timing_end synchronises and returns
 * the summed solve time, sweeps timed, summed step time and steps timed. */
int cfd_timing_begin(cfd_model *m);
int cfd_timing_end(cfd_model *m, double *solve_ms, uint64_t *sweeps, double *step_ms,
                   uint64_t *steps);
/* Per-phase timing inside the timing window (off by default: every event
 * record costs the step a few microseconds): with on != 0, the following
 * cfd_timing_begin/end windows also time each step's predictor + first
 * divergence phase (model.rs:538-676) and its corrector / fused finish
 * (model.rs:693, 728, 333-377); cfd_timing_phase_ms returns the sums of the
 * last window (0 when a phase was not timed). */
int cfd_timing_phases(cfd_model *m, int on);
int cfd_timing_phase_ms(const cfd_model *m, double *predict_ms, double *finish_ms);
/* Sharded models over RCCL, same windows: the summed duration of every halo
 * exchange group and all-reduce on the stream it runs on (waiting for the
 * peer included), and how many there were.  (new; per-rank exchange time) */
int cfd_timing_exchange_ms(const cfd_model *m, double *exchange_ms, uint64_t *exchanges);
/* p' halo depth (rows exchanged per RCCL round) of a sharded model. */
int cfd_get_halo_depth(const cfd_model *m);
/* Jacobi kernel configuration chosen at creation: division form proven exact
 * for this grid's divisors (0 IEEE, 1 reciprocal multiply, 2 FMA-corrected)
 * and sweeps per launch (1 when the tolerance is on). */
int cfd_get_kernel_config(const cfd_model *m, int *fastdiv, int *temporal);
/* The Jacobi kernel a solve launches: kind 0 single sweep (k_jacobi), 1
 * register-march temporal blocking (k_jacobi_tb), 3 / 4 the
 * prefetch-pipelined march with 4 / 2 columns per lane (k_jacobi_pipe), 5 the
 * LDS row march (k_jacobi_lds; with the tolerance on its speculative form), 6
 * the tolerance-mode solve of a small grid as one resident launch
 * (k_jacobi_resident, default up to 2^21 cells; CFD_RESIDENT=0/1 forces), and
 * its instantiated name as rocprofv3 reports it (NUL-terminated, truncated to
 * name_len). */
int cfd_get_jacobi_kernel(const cfd_model *m, int *kind, char *name, size_t name_len);

/* Blocks of 8 sweeps the model's last fixed-count solve ran inside ONE
 * persistent launch (k_jacobi_persist; 0: none, every block its own launch).
 * Blocks after them (shorter ones of an uneven split) are k_jacobi_lds
 * launches of their own. */
int cfd_get_persist_blocks(const cfd_model *m, int *blocks);
/* Blocks of persistent solves that a workgroup ran for a neighbour tile whose
 * owner had not claimed them (k_jacobi_persist stealing; 0 when every owner
 * was resident), summed over the model's life.  Synchronises.  (new) */
int cfd_get_persist_steals(cfd_model *m, uint64_t *steals);
/* 8-sweep blocks run in the SUMS form -- (h + v) / dx^2 for h / dx^2 +
 * v / dy^2, one instruction per column pair and sweep fewer, taken only where
 * a guard proves it bitwise: persistent-solve blocks per tile
 * (k_jacobi_persist's per-task guard), summed over the model's life.
 * Synchronises.  (new; diagnostics) */
int cfd_get_persist_sums(cfd_model *m, uint64_t *blocks);
/* Collective calls this (sharded) model has enqueued: halo-exchange groups
 * and all-reduces, summed over its life (0 unsharded).  (new; diagnostics) */
int cfd_get_comm_calls(const cfd_model *m, uint64_t *n);
/* Solve timeouts this model recovered from by itself (CFD_ETIMEOUT). */
int cfd_get_recoveries(const cfd_model *m, uint64_t *n);
/* Tolerance-mode solves this model enqueued as one resident launch
 * (k_jacobi_resident, see cfd_get_jacobi_kernel kind 6); diagnostics. */
int cfd_get_resident_solves(const cfd_model *m, uint64_t *solves);
/* The tile geometry of the model's 8-sweep kind-5 Jacobi launch over its
 * first block's rows (persist != 0: the persistent form's): the dynamic LDS
 * pad in bytes (24 KiB caps a CU at 3 four-wave workgroups on cache-resident
 * slabs), the workgroups per CU the round is sized for, the wave columns and
 * the wave segments per column.  (new; diagnostics) */
int cfd_get_jacobi_geometry(const cfd_model *m, int persist, int *lds_pad, int *wgs_per_cu,
                            int *wave_cols, int *segments);

/* Host-only slab plan used by cfd_create_sharded (no device needed; the
 * multi-rank CPU tests drive the same plan):
 *   cfd_plan_slab  — global pressure rows [j0, j1) of `rank`;
 *   cfd_plan_sweep — local rows [lo, hi) that sweep `it` of an `iters`-sweep
 *                    solve recomputes with halo depth d, and whether d rows
 *                    of p' are exchanged after it;
 *   cfd_plan_halo  — ghost geometry of a field (kind 0 u, 1 v, 2 p'):
 *                    out6 = {send, recv, rows} with rank-1, then with rank+1,
 *                    in local rows. */
int cfd_plan_slab(uint64_t ny, int n_ranks, int rank, uint64_t *j0, uint64_t *j1);
int cfd_plan_sweep(int j0, int nyl, int ny, int halo_depth, int it, int iters, int *lo, int *hi,
                   int *exchange);
int cfd_plan_halo(int kind, int nyl, int depth, int rank, int n_ranks, int *out6);
/* The overlapped exchange block: out6 = the two bands the
 * p' exchange sends ({lo, hi} to rank-1, then to rank+1; empty without a
 * neighbour) and the interior {lo, hi} computed while it travels; returns 1
 * when the block splits, 0 when the slab is too thin (run it whole). */
int cfd_plan_overlap(int nyl, int halo_depth, int rank, int n_ranks, int lo, int hi, int *out6);
/* Temporally blocked form of cfd_plan_sweep: the launch starting at sweep
 * `it` runs *T <= t_max sweeps and stores its last sweep on local rows
 * [out_lo, out_hi); halo_depth <= 0 means unsharded. */
int cfd_plan_block(int j0, int nyl, int ny, int halo_depth, int it, int t_max, int iters, int *T,
                   int *out_lo, int *out_hi, int *exchange);

/* Visualisation modes of App (src/app.rs:505-509 VisualizationMode). */
typedef enum { CFD_VIS_PRESSURE = 0, CFD_VIS_VELOCITY = 1, CFD_VIS_VORTICITY = 2 } cfd_vis_mode;

/* Device-side equivalent of the image App::update_simulation_view builds
 * from a snapshot (src/app.rs:235-403): derive the mode's scalar field
 * (p; cell-centred |velocity|; interior vorticity, 0 elsewhere), its min/max
 * (NaN ignored) and the RGBA8 image (r = (norm*255) as u8, g = 0,
 * b = ((1-norm)*255) as u8, a = 255; cells whose centre is within the
 * cylinder radius, `<=`, grey 128), all on the device; only nx*ny*4 bytes
 * are copied into rgba (row-major, x fastest; NULL skips the image).
 * min_max_out (2 floats, may be NULL) gets the field's min and max before
 * the reference's 1e-6 range widening.  Sharded: the rank's slab rows, with
 * min/max reduced over all ranks (collective: every rank must call). */
int cfd_render(cfd_model *m, int mode, uint8_t *rgba, float *min_max_out);
/* The mode's derived scalar field itself (nx*ny f32; slab rows when sharded). */
int cfd_derive_field(cfd_model *m, int mode, float *out, float *min_max_out);

/* The grid and parameters the model runs with (NULL skips either). */
int cfd_get_config(const cfd_model *m, cfd_grid *grid, cfd_params *params);

/* ---- Model::run (model.rs:1282-1332): the asynchronous host runtime ----
 * cfd_run_start hands the model to a worker thread that loops exactly as the
 * reference's (model.rs:1287-1325): drain the queued commands in order
 * (Stop, SetParams, GetSnapshot — at most one snapshot per drain —, Pause,
 * Resume; model.rs:57-63), then either run one cfd_update and queue its
 * residuals, or wait 16 ms while paused.  Until cfd_run_stop returns, only
 * cfd_run_* calls may touch the model.  Any thread may call cfd_run_*.
 * Difference: Stop ends the worker (the reference's Stop only leaves the
 * command loop, model.rs:1296); cfd_run_stop joins it, frees the runner and
 * leaves the model to the caller. */
typedef struct cfd_runner cfd_runner;
int cfd_run_start(cfd_model *m, cfd_runner **out);             /* Model::run        :1282 */
int cfd_run_stop(cfd_runner *r);                               /* handle.stop()     :72   */
int cfd_run_pause(cfd_runner *r);                              /* handle.pause()    :110  */
int cfd_run_resume(cfd_runner *r);                             /* handle.resume()   :114  */
int cfd_run_set_params(cfd_runner *r, const cfd_params *p);    /* handle.set_params :104  */
int cfd_run_request_snapshot(cfd_runner *r);                   /* request_snapshot  :100  */
/* get_last_available_snapshot (:76-86): the newest snapshot published since
 * the previous call (slab sizes as cfd_get_snapshot; NULL skips a field);
 * *available = 0 when there is none. */
int cfd_run_last_snapshot(cfd_runner *r, float *u, float *v, float *p, float *dt_out,
                          int *paused_out, int *available);
/* get_new_log_messages (:88-98): up to `max` queued residual records, oldest
 * first; *n_out = records copied. */
int cfd_run_new_residuals(cfd_runner *r, cfd_residuals *out, int max, int *n_out);
/* 0 while the worker is healthy, else the first failing status of a call it
 * made (it then stops stepping and waits for Stop); msg gets the message. */
int cfd_run_status(cfd_runner *r, char *msg, size_t msg_len);
/* Steps the worker has completed. */
uint64_t cfd_run_steps(cfd_runner *r);

/* ---- the adaptive quadtree mesher (src/quad_mesh, src/utils/intersection.rs) ----
 * f64 throughout, as the reference.  Polygon construction, the geometry
 * predicates and the tesselation are host code; Mesh::from_quad_tree
 * (mesh.rs:51-227: leaf filtering, the O(n^2) face-neighbour search, the
 * cell/edge intersections) runs on the GPU.  Geometry calls return 0 / a
 * negative cfd_status like every entry point; the reference's PolygonError
 * comes back through *poly_error. */
typedef struct { double x, y; } cfd_point;                    /* point.rs */
typedef struct { cfd_point center; double half_width, half_height; } cfd_aabb;   /* aabb.rs */
enum { CFD_POLY_OK = 0, CFD_POLY_NOT_ENOUGH_VERTICES = 1, CFD_POLY_SELF_INTERSECTING = 2,
       CFD_POLY_INVALID_HOLE = 3 };                          /* PolygonError polygon.rs:12-16 */
typedef struct cfd_polygon cfd_polygon;
typedef struct cfd_quadtree cfd_quadtree;
typedef struct cfd_mesh cfd_mesh;

/* Polygon::new (polygon.rs:19-40): *out is NULL when *poly_error != 0. */
int cfd_polygon_new(const cfd_point *vertex_buffer, size_t n_points, const uint64_t *vertices,
                    size_t n_vertices, cfd_polygon **out, int *poly_error);
int cfd_polygon_new_rect(double x, double y, double w, double h, cfd_polygon **out); /* :42-53 */
int cfd_polygon_new_regular(cfd_point center, double radius, size_t n, double start_angle,
                            cfd_polygon **out);                                  /* new_polygon :55-67 */
/* add_hole (:69-79): on success the polygon takes ownership of `hole`. */
int cfd_polygon_add_hole(cfd_polygon *p, cfd_polygon *hole, int *poly_error);
/* contains_point (:81-103), intersects_aabb (:105-117), edges_intersect_aabb
 * (:119-133): *result 0 / 1. */
int cfd_polygon_contains_point(const cfd_polygon *p, cfd_point pt, int *result);
int cfd_polygon_intersects_aabb(const cfd_polygon *p, const cfd_aabb *box, int *result);
int cfd_polygon_edges_intersect_aabb(const cfd_polygon *p, const cfd_aabb *box, int *result);
int cfd_polygon_bounding_box(const cfd_polygon *p, cfd_aabb *out);               /* :150-178 */
int cfd_polygon_bounding_square(const cfd_polygon *p, cfd_aabb *out);            /* :180-184 */
/* edges (:186-196), reference quirk kept: edge k joins vertex_buffer[v_k] and
 * vertex_buffer[(v_k + 1) % n_vertices]; out gets 2 points per edge. */
int cfd_polygon_edges(const cfd_polygon *p, cfd_point *out, size_t max_edges, size_t *n_edges);
void cfd_polygon_destroy(cfd_polygon *p);

/* utils/intersection.rs: do_intersect (:20-38), line_segment_intersection
 * (:41-63; *found 0 for None), intersect_quad_edge (:68-129) for
 * quad = Quad::new_rect(center, hw, hh) (quad.rs:24-35; up to 8 points). */
int cfd_geom_do_intersect(cfd_point p, cfd_point q, cfd_point a, cfd_point b, int *result);
int cfd_geom_segment_intersection(cfd_point p, cfd_point q, cfd_point a, cfd_point b,
                                  cfd_point *out, int *found);
int cfd_geom_intersect_quad_edge(cfd_point center, double hw, double hh, cfd_point p1,
                                 cfd_point p2, cfd_point *out8, int *n);

/* tesselate (quad_tree.rs:17-100).  Nodes in depth-first pre-order; children
 * (4 per node, quadrant order of :43-91) as node indices, -1 for a leaf. */
int cfd_tesselate(const cfd_polygon *p, double feature_size, double max_cell_size,
                  cfd_quadtree **out);
int cfd_quadtree_size(const cfd_quadtree *t, uint64_t *n_nodes, uint64_t *n_leaves);
int cfd_quadtree_nodes(const cfd_quadtree *t, cfd_aabb *boxes, int64_t *children4);
void cfd_quadtree_destroy(cfd_quadtree *t);

/* Mesh::from_quad_tree (mesh.rs:51-227) on HIP device `device`.  Arrays as the
 * reference's SoA Mesh; neighbour lists of each cell in ascending cell order. */
enum { CFD_FACE_EAST = 0, CFD_FACE_WEST = 1, CFD_FACE_NORTH = 2, CFD_FACE_SOUTH = 3 };
int cfd_mesh_from_quadtree(const cfd_quadtree *t, const cfd_polygon *p, int device,
                           cfd_mesh **out);
/* sizes[0] cells, [1..4] neighbour index counts (east, west, north, south),
 * [5] intersection points. */
int cfd_mesh_sizes(const cfd_mesh *m, uint64_t *sizes6);
int cfd_mesh_cells(const cfd_mesh *m, double *cx, double *cy, double *hw, double *hh);
/* ranges: 2 x u64 (start, end) per cell. */
int cfd_mesh_neighbors(const cfd_mesh *m, int face, uint64_t *ranges, uint64_t *indexes);
int cfd_mesh_intersections(const cfd_mesh *m, uint64_t *ranges, cfd_point *points);
int cfd_mesh_full_bounding_box(const cfd_mesh *m, cfd_aabb *out);               /* :294-338 */
/* device time of the last cfd_mesh_from_quadtree's kernels (HIP events) */
int cfd_mesh_build_ms(const cfd_mesh *m, double *ms);
void cfd_mesh_destroy(cfd_mesh *m);

const char *cfd_last_error(void);
int cfd_abi_version(void);
void cfd_destroy(cfd_model *m);

#ifdef __cplusplus
}
#endif
#endif /* CFD_H */
