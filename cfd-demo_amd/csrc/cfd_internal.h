// cfd_internal.h — device-side data layout and kernel launch interface of the
// MI355X pressure-projection path.  Shared by cfd_kernels.hip (device code)
// and cfd_model.hip (host runtime behind include/cfd.h).
//
// Layout in HBM (one slab per GPU; a single-GPU model is the 1-slab case):
//   every field is row-major with x fastest and the reference's pitches
//   (u: nx+1, v: nx, p/rhs/p': nx — model.rs:161-214), so the reference's
//   flat wrap-around reads (U(nx+1,j) == U(0,j+1)) are plain loads here.
//   "local row" lj = global row j - j0.  Base pointers point at local row 0;
//   ghost rows sit at negative lj and at lj >= nyl:
//     u, u_old, u_star : rows [-G, nyl+G)        (G = 2)
//     v, v_old, v_star : rows [-G, nyl+1+G)      (v row nyl is the face shared
//                                                 with the rank above)
//     p                : rows [0, nyl)
//     rhs, p' (x2)     : rows [-HG, nyl+HG)      (HG = halo depth >= 1; deep-halo
//                                                 sweeps recompute ghost rows)
//   mask_u rows [0,nyl), mask_v rows [0,nyl] (u8, same pitches).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cfd.h"

namespace cfd {

constexpr int kGhostUV = 2;
constexpr int kMaxSweeps = 4096;   // per pressure solve
constexpr int kMaxPasses = 64;     // corrector passes + 1

// Residual maxima are published with atomicMax on f32 bits.  Device-scope
// atomics on ONE address serialise at the memory side (~10 ns each, measured:
// 6,000 per launch cost 54 us), so every maximum is spread over kResSlots
// addresses kResStride words apart and folded by its reader (fold_res /
// read_res).  Sweep k of a solve owns slots err_slots[(k*kResSlots + s)*kResStride];
// the 4 step maxima own red_slots likewise.  Slots are zero between uses.
constexpr int kResSlots = 32;
constexpr int kResStride = 16;
// persistent-solve words (k_jacobi_persist), one 64-B line each: line 0 [1]
// the abort flag, [2] the blocks stolen so far, [3] the blocks run in the
// SUMS form so far; then one line per tile: [0] its done flag, [1] its claim
// counter, [2..5] / [6..9] its waves' max |p'| stored in its last even / odd
// block
constexpr int kPersistFlagStride = 16;
// head lines: 0 = the persistent solve's words ([1] abort, [2] steals, [3]
// SUMS blocks); 2 = the resident solve's top barrier counter, 4 = its exit
// ticket, 5-12 its group counters, 13-20 its group generations
// (cfd_jacobi_resident.hip)
constexpr int kPersistHeadLines = 21;
// flag = epoch << kPersistBlockBits | blocks done: room for every block of the
// longest solve (kMaxSweeps / 8 = 512), epochs below 2^(32 - bits)
constexpr int kPersistBlockBits = 10;
static_assert((1 << kPersistBlockBits) > kMaxSweeps / 8, "persistent flag layout");
constexpr int kPersistMaxGroups = 16384;   // tiles (wave columns x row groups)
constexpr size_t kPersistWords = (size_t)(kPersistMaxGroups + kPersistHeadLines) * kPersistFlagStride;
// slot sets: kMaxSweeps per-sweep residual sets, then red (4), vis (2), 10
// spare; then the persistent solve's words
constexpr size_t kSlotWords = (size_t)(kMaxSweeps + 16) * kResSlots * kResStride + kPersistWords;

// Device-resident control block: every data-dependent decision of
// Model::update lives here so a whole step can be enqueued (or replayed as a
// hipGraph) with no host round trip.
struct Ctl {
    float dt;               // Model::dt (model.rs:170)
    float time;             // simulation_time
    uint32_t step;          // simulation_step
    float inlet;            // current_inlet_velocity (set at step start)
    int32_t cur;            // which p' buffer holds the current p'
    uint32_t n_exec_last;   // sweeps executed by the last solve
    float last_p;           // last_pressure_residual
    float res_u, res_v;     // last_u_residual / last_v_residual
    uint32_t red[7];        // step maxima as f32 bits: |du|, |dv|, |u|, |v|; red[6]: a
                            // persistent solve of some slab timed out (r5, all-reduced so
                            // every rank recovers); red[5]: the last
                            // solve's residual (all-reduced with the maxima on slabs); red[4]:
                            // non-finite flag (1: some new u/v value is NaN or +-Inf)
    uint32_t nonfinite_step;   // sticky: simulation_step after the first step whose
                               // velocities were not all finite (0 = never)
    uint32_t vis[2];        // render: max key, max ~key of the derived field (cfd_render.hip)
    uint32_t done;          // (unused since r6: the last-workgroup folds were removed; keeps the layout)
    uint64_t sweeps_total;
    // speculative temporal blocking with the tolerance on (k_spec_check):
    // spec_stop: a launch of this solve converged (later launches skip);
    // spec_launch / spec_redo: that launch and the stages its re-run keeps
    // (0: none, it converged on its last stage); spec_launches: launches run
    // (the finalize's buffer flips).  All 0 between solves.
    int32_t spec_stop, spec_redo, spec_launch, spec_launches;
    uint32_t spec_done;     // (unused since r6; keeps the layout)
    int32_t go[kMaxPasses + 1];      // go[p]: pass p of the corrector loop runs
    uint32_t err[kMaxSweeps];        // per-sweep max |p'new - p'| as f32 bits
};

// Scalars every kernel needs; passed by value as a kernel argument.
struct Geom {
    int32_t nx, ny;       // global pressure cells
    int32_t j0, nyl;      // global row of local row 0; owned rows
    int32_t hg;           // p' halo depth
    float dx, dy, nu, ly;
    float target_inlet;
    int32_t scheme, profile, bc_kind;
    int32_t tol_enabled;
    float p_tol;
    int32_t jacobi_iters;
    // Jacobi divisors exactly as model.rs:740-746 forms them, their rounded
    // reciprocals, and the division mode proven exact for all three
    // (0: IEEE `/`, 1: x * (1/c), 2: x * (1/c) + one FMA correction step);
    // see verify_division() in cfd_model.hip.
    float dx_sq, dy_sq, denom;
    float r_dx_sq, r_dy_sq, r_denom;
    int32_t fastdiv;
    int32_t tb_rows;      // fixed output rows per wave segment (0: balanced by tb_bpc)
    int32_t tb_bpc;       // target k_jacobi_tb blocks per CU (balanced segmentation)
    int32_t n_cu;         // compute units of the device
    int32_t tb_kind;      // 1: k_jacobi_tb (T <= 4); prefetch pipeline (T <= 8) with
                          // 3: 4 columns per lane, 4: 2 columns per lane; 5: the
                          // 2-column march with its rhs window in LDS
    int32_t xcd_remap;    // renumber blocks so each XCD gets contiguous tiles (xcd_block)
    // reciprocals of dx, dy, dx*dx, dy*dy; sp_pow2 = 1 when all four spacings
    // are exact powers of two (then sdiv multiplies, bit-identically)
    float r_dx, r_dy, r_dxx, r_dyy;
    int32_t sp_pow2;
    int32_t pred_div;     // predictors + divergence: 2: one row march (k_predict_march, both
                          // schemes), 1: fused 2-row tile (k_predict_div, first order),
                          // 0: separate launches; where the fused forms apply
    int32_t res_div;      // r4: the resident solve's division mode: fastdiv, or 3 (FMA-corrected
                          // above 2^-96, IEEE below; proven like the others) where fastdiv is 0
};

struct Fields {
    float *u, *v, *u_old, *v_old, *u_star, *v_star;   // at local row 0
    float *p, *rhs;
    float *pp[2];                                      // p' ping-pong
    const uint8_t *mask_u, *mask_v;
    const int32_t *obs;       // (i, j_global) pairs, cells touching this slab
    uint32_t *err_slots;      // spread per-sweep residual maxima (kResSlots per sweep)
    uint32_t *red_slots;      // spread step maxima (4 x kResSlots)
    uint32_t *vis_slots;      // spread render min/max keys (2 x kResSlots)
    int32_t n_obs;
    int32_t any_pmask;   // some predictor mask bit (bit 0) is set in this slab's masks
    size_t u_alloc, v_alloc;  // floats in the u/v allocations (incl. ghosts)
    float *u_alloc_base, *v_alloc_base, *u_old_base, *v_old_base, *u_star_base, *v_star_base;
    Ctl *ctl;
    // host-mapped word (pinned, zero-copy) mirroring Ctl::nonfinite_step, so the
    // host can see a blown-up run without synchronising the stream
    uint32_t *host_nonfinite;
    // host-mapped word the step finalize sets to Ctl::step (sharded models):
    // the RCCL watchdog's evidence of forward progress
    uint32_t *host_progress;
    uint32_t *persist;   // kPersistWords words after the slot sets (see kPersistFlagStride)
};

// ---- launchers (cfd_kernels.hip) ----
// pass < 0 means "not inside the corrector loop" (always runs).
void launch_step_begin(const Geom &g, const Fields &f, int copy, hipStream_t s);
void launch_copy_star(const Geom &g, const Fields &f, int pass, hipStream_t s);
// k_copy_star + k_divergence of a corrector pass in one launch (same values).
void launch_copy_star_div(const Geom &g, const Fields &f, int pass, float dt_override,
                          hipStream_t s);
void launch_u_predictor(const Geom &g, const Fields &f, float dt_override, hipStream_t s);
void launch_v_predictor(const Geom &g, const Fields &f, float dt_override, hipStream_t s);
// u and v predictors in one pass (same results as the two launches above).
void launch_predict(const Geom &g, const Fields &f, float dt_override, hipStream_t s);
// first-order predictors + divergence in one row march (k_predict_div), when
// predict_div_fused(): replaces launch_predict + the step's first divergence
bool predict_div_fused(const Geom &g, const Fields &f);
void launch_predict_div(const Geom &g, const Fields &f, float dt_override, hipStream_t s);
// both schemes' predictors + divergence in one row march (cfd_predict_march.hip),
// when predict_march_ok(): replaces launch_predict + the step's first divergence
bool predict_march_ok(const Geom &g, const Fields &f);
// set_inlet: also set Ctl::inlet from Ctl::step (k_step_begin's ramp,
// model.rs:311-316) — the step's k_step_begin is then not launched
// [row_lo, row_hi): the divergence rows the launch forms (>= 4 rows; default
// all owned rows) — a sharded step runs rows [2, nyl-2), which read no u/v
// ghost row, while the ghost exchange is in flight
void launch_predict_march(const Geom &g, const Fields &f, float dt_override, hipStream_t s,
                          bool set_inlet = false, int row_lo = 0, int row_hi = -1);
void launch_divergence(const Geom &g, const Fields &f, int pass, float dt_override,
                       hipStream_t s);
// One Jacobi sweep over local rows [row_lo, row_hi) (may reach into ghosts).
// res: publish this sweep's residual (always with the tolerance on; only the
// last sweep of a fixed-count solve needs it).
void launch_jacobi_sweep(const Geom &g, const Fields &f, int pass, int it, int row_lo,
                         int row_hi, int res, hipStream_t s);
// T consecutive Jacobi sweeps in one launch (temporal blocking, tolerance
// off): the final sweep's rows [out_lo, out_hi) are stored; sweep `it` of the
// block is the first.  T <= kMaxTemporal.
// `par` = launches of this solve before this one (selects the source buffer:
// buffers flip once per launch).
void launch_jacobi_block(const Geom &g, const Fields &f, int pass, int it, int par, int T,
                         int out_lo, int out_hi, int res, hipStream_t s);
// nblk consecutive 8-sweep kind-5 blocks (no residual) in ONE persistent
// launch whose workgroups hand rows to their neighbours through flags
// (k_jacobi_persist); res_it >= 0: the last block is the solve's last and
// publishes sweep res_it's residual; returns false (nothing launched) where
// the one-round geometry does not apply
bool launch_jacobi_persist(const Geom &g, const Fields &f, int pass, int par0, int nblk,
                           int out_lo, int out_hi, uint32_t epoch, int res_it, hipStream_t s);
// The tile geometry of the T = 8 kind-5 launch over rows [out_lo, out_hi)
// (persist: the persistent form's): dynamic LDS pad, workgroups per CU the
// round is sized for, wave columns, wave segments per column
// (cfd_jacobi_lds8.hip).
void lds_geometry8(const Geom &g, int out_lo, int out_hi, bool persist, int *pad, int *occ, int *nwc,
                   int *nseg);
// The block kernels behind it: k_jacobi_tb (T <= 4, cfd_jacobi_tb1.hip) and
// the prefetch-pipelined march with 4 or 2 columns per lane (T <= 8,
// cfd_jacobi_pipe4.hip / cfd_jacobi_pipe2.hip).
// res_slots: the slot set the last sweep's residual goes to, or null.
void launch_tb1(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                int out_hi, uint32_t *res_slots, hipStream_t s);
void launch_pipe4(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                  int out_hi, uint32_t *res_slots, hipStream_t s);
void launch_pipe2(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                  int out_hi, uint32_t *res_slots, hipStream_t s);
// kind 5: the same march with its rhs window in LDS (cfd_jacobi_lds.hip, T <= 8);
// mode 2 / 3: the speculative launch / its re-run (launch_jacobi_spec)
bool launch_lds_persist8(const Geom &g, const Fields &f, int pass, int par0, int nblk, int out_lo,
                         int out_hi, uint32_t epoch, uint32_t *rs, hipStream_t s);
// lag (r5, speculative solves on one domain): mode 2 -- the previous launch's
// sweep count, whose early-exit check this launch makes (0: none); mode 3 --
// the solve's last launch's, checked by the re-run (see k_jacobi_lds)
void launch_lds(const Geom &g, const Fields &f, int T, int pass, int it, int par, int out_lo,
                int out_hi, uint32_t *res_slots, hipStream_t s, int mode = 0, int lag = 0);
// Speculative temporal blocking for the tolerance mode (model.rs:748-819):
// the launch starting at sweep `it` runs T sweeps (kind 5) and publishes
// every sweep's residual; k_spec_check folds them, finds the first sweep
// below p_tol and, when it is not the launch's last, schedules the re-run
// (launch_jacobi_redo) of that launch with exactly that many sweeps from its
// untouched source buffer.  Later launches of the solve return at once.
// lag > 0 (one domain, the default since r6; CFD_SPEC_LAG=0 turns it off): no k_spec_check launches -- each launch checks the
// previous one (lag = its sweep count) and the re-run checks the last one
// (launch_jacobi_redo's last_*); see spec_lag_first.
void launch_jacobi_spec(const Geom &g, const Fields &f, int pass, int it, int par, int T,
                        int out_lo, int out_hi, hipStream_t s, int lag = 0);
void launch_spec_check(const Geom &g, const Fields &f, int pass, int it, int T, int par,
                       hipStream_t s);
// The whole tolerance-mode solve of a single-domain grid in one launch
// (cfd_jacobi_resident.hip); false: no tile plan fits (nothing launched).
// fin: its last workgroup also runs k_finalize_solve's body (exact_flips 2).
bool launch_jacobi_resident(const Geom &g, const Fields &f, int pass, int iters, int fin,
                            int check_break, hipStream_t s);
bool jacobi_resident_geometry(const Geom &g, int *br, int *bc, int *tiles, int *wgs);
// slabs (r5): after the re-run, the converged launch's result moved to the
// buffer the host counts n launches ahead (k_spec_align; nyl * nx % 4 == 0)
void launch_spec_align(const Geom &g, const Fields &f, int pass, int n, hipStream_t s);
void launch_jacobi_redo(const Geom &g, const Fields &f, int pass, int out_lo, int out_hi,
                        hipStream_t s, int last_it = 0, int last_par = 0, int last_T = 0);
// dst[q] = max(dst[q], slots of q) for q < n, then zero those slots (before
// an all-reduce of dst reads it).
void launch_fold_slots(uint32_t *dst, uint32_t *slots, int n, hipStream_t s);
// Visualisation (cfd_render.hip, src/app.rs:235-403): derived field of `mode`
// into `out` (may be null) with its min/max keys into 2 spread sets; then the
// RGBA8 image from the folded keys (field null: re-derive on the fly).
void launch_vis_field(const Geom &g, const Fields &f, int mode, float *out, uint32_t *slots,
                      hipStream_t s);
void launch_vis_color(const Geom &g, const Fields &f, int mode, const float *field, uint32_t *px,
                      const uint32_t *keys, int has_cyl, float cx, float cy, float radius,
                      hipStream_t s);
// Exhaustive check over all 2^32 f32 inputs x of x/c against the two fast
// forms; writes mismatch counts {mode1, mode2} to dev_counts (2 x u64).
void launch_verify_division(float c, float r, unsigned long long *dev_counts, hipStream_t s);
// flips = launches of a fixed-count solve (ignored with the tolerance on,
// where each executed sweep is one launch).  exact_flips: flip the current
// p' buffer exactly `flips` times regardless of the tolerance (solvers that
// work in place: SOR, multigrid); 2: Ctl::spec_launches times (speculative
// solve), and reset the speculative state.
void launch_finalize_solve(const Geom &g, const Fields &f, int pass, int iters, int check_break,
                           int flips, hipStream_t s, int exact_flips = 0);

// ---- alternative pressure solvers (cfd_solvers.hip; index.html) ----
// Double-precision constants of one grid level: dx2 = dx*dx, dy2 = dy*dy,
// denom = 2/dx2 + 2/dy2 exactly as the script forms them, their reciprocals,
// and fast = 1 when all three divisors are powers of two (x / c == x * (1/c)
// bit for bit for every double x).
struct SorConst {
    double dx2, dy2, denom;
    double r_dx2, r_dy2, r_denom;
    int32_t fast;
};
// One multigrid level: solution ping-pong buffers a/b (level 0: the model's
// current / other p' buffer), right-hand side, residual scratch, size and the
// level's constants (spacing 2^l times the model's, index.html:1458).
struct MgLevel {
    // biased to global row 0: element (i, j) of the level is a[j * nx + i]
    // for every stored row j in [ys, ye)
    float *a, *b, *rhs, *r;
    int32_t nx, ny;        // the level's global size
    double dx2, dy2, denom;
    double r_dx2, r_dy2, r_denom;
    int32_t fast;
    int32_t ys, ye;        // stored rows (a slab's rows + ghost rows; 0, ny unsharded)
    int32_t lo, hi;        // rows a launch outputs (set per launch; 0, ny unsharded)
};
constexpr int kMgMaxLevels = 40;
void launch_sor_color(float *pp, const float *rhs, int nx, int ny, const SorConst &k, int color,
                      Ctl *ctl, uint32_t *err_slots, int pass, int it, int tol, float p_tol, int res,
                      hipStream_t s);
// One whole red-black iteration per launch (k_sor_march) over the local
// interior rows [row_lo, row_hi) of a slab starting at global row j0 (p' and
// rhs rows readable in [lo_clamp, hi_clamp]), ping-pong between pa / pb from
// ctl->cur (iteration `it` reads buffer (cur + it) & 1; it = 0 reads nothing:
// p' starts at 0), when sor_fused_ok(nx, row_hi - row_lo).
bool sor_fused_ok(int nx, int nrows);
void launch_sor_fused(float *pa, float *pb, const float *rhs, int nx, int ny, const SorConst &k,
                      Ctl *ctl, uint32_t *err_slots, int pass, int it, int tol, float p_tol, int res,
                      int row_lo, int row_hi, int j0, int lo_clamp, int hi_clamp, hipStream_t s);
void launch_fill_zero(float *p, size_t n, const Ctl *ctl, int pass, hipStream_t s);
void launch_mg_smooth(const MgLevel &L, const float *src, float *dst, const Ctl *ctl, int pass,
                      hipStream_t s);
// Five smoothing sweeps src -> dst in one launch (temporal blocking: one
// wave per register window, or the LDS block form with CFD_MG_SMOOTH=1).
void launch_mg_smooth5(const MgLevel &L, const float *src, float *dst, const Ctl *ctl, int pass,
                       hipStream_t s);
// The wave-window form is selected (then the up-leg fuses its prolong-add
// into the smoothing: launch_mg_prolong_smooth5 reads src + prolongate(e)).
bool mg_smooth_wave_form();
void launch_mg_prolong_smooth5(const MgLevel &Cl, const float *e, const MgLevel &L, const float *src,
                               float *dst, const Ctl *ctl, int pass, hipStream_t s);
// ... and the down-leg forms the residual of its smoothed field in the same
// launch (launch_mg_smooth5_residual: dst and L.r).
void launch_mg_smooth5_residual(const MgLevel &L, const float *src, float *dst, const Ctl *ctl,
                                int pass, hipStream_t s);
void launch_mg_residual(const MgLevel &L, const float *p, const Ctl *ctl, int pass, hipStream_t s);
void launch_mg_restrict(const MgLevel &F, const MgLevel &Cl, const Ctl *ctl, int pass, hipStream_t s);
void launch_mg_prolong_add(const MgLevel &Cl, const float *e, const MgLevel &F, float *p,
                           const Ctl *ctl, int pass, hipStream_t s);
// fast: the hierarchy's division form (uniform: 2^l scaling keeps powers of two)
void launch_mg_tail(const MgLevel *dev_levels, int s_level, int coarsest, float *a0, float *b0,
                    int fast, const Ctl *ctl, int pass, hipStream_t s);
void launch_mg_final_residual(const MgLevel &L, const float *p, uint32_t *slots, const Ctl *ctl,
                              int pass, hipStream_t s);
void launch_corrector(const Geom &g, const Fields &f, int pass, float dt_override,
                      hipStream_t s);
void launch_boundary(const Geom &g, const Fields &f, hipStream_t s);
// The corrector finish: the 16-row band march where the fields allow float4
// access (nx % 4 == 0, 16-byte aligned arrays), else the scalar form.
void launch_correct_finish(const Geom &g, const Fields &f, float dt_override, hipStream_t s);
void launch_step_reduce(const Geom &g, const Fields &f, hipStream_t s);
// The corrector of pass `pass` and, when pass+1 exists (has_next) and the
// device's go flag says it runs, pass+1's head (u* <- u, v* <- v,
// divergence) in one launch (k_correct_head4, single domain; every pass of the
// loop uses it: the passes alternate the u* / v* arrays, and u / v are
// written only when the loop ends); correct_head_ok: its alignment and
// CFD_CORR_HEAD knob.
bool correct_head_ok(const Geom &g, const Fields &f);
void launch_correct_head(const Geom &g, const Fields &f, int pass, float dt_override, bool has_next,
                         hipStream_t s);
void launch_step_finalize(const Geom &g, const Fields &f, hipStream_t s);
// Slabs with persistent runs (r5): copy this rank's abort word (persist[1],
// a persistent solve timed out) into Ctl::red[6] before the step all-reduce
void launch_abort_to_red(const Fields &f, hipStream_t s);
// ... and, after its all-reduce outside a step, back into this rank's abort
// flag and host word (as the step finalize does)
void launch_abort_from_red(const Fields &f, hipStream_t s);

// Jacobi kernel geometry (exported for the roofline bookkeeping in bench).
constexpr int kJacRowsPerWave = 16;
constexpr int kMaxTemporal = 8;     // sweeps per temporally blocked launch (kind 3; 4 otherwise)
constexpr int kTbRowsPerWave = 32;  // output rows per wave segment (TB kernel)
constexpr int kJacWavesPerBlock = 4;

}  // namespace cfd
