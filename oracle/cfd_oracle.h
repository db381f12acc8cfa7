/*
 * cfd_oracle.h — CPU restatement of cfd-demo's pressure-projection hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing under oracle/ is part of the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it,
 * and only as the checker (or as the timed CPU baseline).
 *
 * PARITY UNPINNED: the reference (Rust, nightly portable_simd, 393 crates) cannot
 * be built in this image (no cargo/rustc) and its own tests never touch
 * src/model.rs, so no golden vector from the reference exists.  This scalar C
 * restatement is cross-checked bit-for-bit against an independent numpy
 * restatement (oracle/np_model.py) written from the same reading of
 * /root/reference/src/model.rs; see DESIGN.md "Oracle".
 *
 * Every function cites the reference lines it restates.
 */
#ifndef CFD_ORACLE_H
#define CFD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_model orc_model;

/* Grid + SimulationParams (model.rs:13-21, 44-55, 119-139) plus the build's
 * extension knobs (reference values in comments). */
typedef struct {
    uint64_t nx, ny;
    float lx, ly;
    int32_t has_cylinder;
    float cx, cy, radius;
} orc_grid;

typedef struct {
    float dt;                     /* 0.005   */
    float viscosity;              /* 1e-6    */
    float target_inlet_velocity;  /* 1.0     */
    int32_t scheme;               /* 0 FirstOrder, 1 SecondOrder */
    int32_t inlet_profile;        /* 0 Uniform, 1 Parabolic      */
    int32_t pressure_solver;      /* 0 Jacobi (only variant)     */
    int32_t jacobi_iters;         /* 50      (model.rs:737)      */
    int32_t corrector_passes;     /* 20      (model.rs:696)      */
    int32_t tol_enabled;          /* 1                           */
    float p_tol;                  /* 1e-4    (model.rs:736, 721) */
    int32_t bc_kind;              /* 0 channel (reference), 1 cavity (build-defined) */
} orc_params;

orc_model *orc_create(const orc_grid *g, const orc_params *p);
void orc_destroy(orc_model *m);
void orc_set_params(orc_model *m, const orc_params *p);

/* Model::update (model.rs:304-379). */
void orc_update(orc_model *m);
/* piso_step (model.rs:529-730). */
void orc_piso_step(orc_model *m, float dt_sub);
/* Individual phases, for known-answer tests. */
void orc_u_predictor(orc_model *m, float dt_sub);            /* model.rs:538-580 */
void orc_v_predictor(orc_model *m, float dt_sub);            /* model.rs:586-670 */
void orc_divergence(orc_model *m, float dt_sub);             /* model.rs:1406-1440 */
float orc_jacobi_pressure(orc_model *m);                     /* model.rs:734-824 */
void orc_corrector(orc_model *m, float dt_sub);              /* model.rs:1334-1404 */
void orc_boundary_conditions(orc_model *m);                  /* model.rs:826-875 */
float orc_auto_dt(const orc_model *m);                       /* model.rs:877-889 */
/* The solve piso_step runs (model.rs:684, :710) for params.pressure_solver:
 * 0 Jacobi (model.rs:734-824), 1 red-black SOR, 2 multigrid (the JavaScript
 * variant's solvers, cfd_oracle_solvers.c).  SOR counts one sweep per
 * iteration, multigrid one per solve. */
float orc_pressure_solve(orc_model *m);

/* cfd_oracle_solvers.c — the JavaScript variant's solvers on raw arrays
 * (index.html:741-795, 1344-1470; double arithmetic, f32 storage). */
float orc_sor_solve(float *pp, const float *rhs, size_t nx, size_t ny, float dx, float dy,
                    int iters, int tol_enabled, float p_tol, int *done);
float orc_mg_solve(float *pp, const float *rhs, int nx, int ny, float dx, float dy);
void orc_mg_smooth(float *p, const float *rhs, int nx, int ny, double dx, double dy,
                   int iterations);
void orc_mg_restrict(const float *fine, int nx_f, int ny_f, float *coarse, int nx_c, int ny_c);
void orc_mg_prolongate(const float *coarse, int nx_c, int ny_c, float *fine, int nx_f, int ny_f);
void orc_mg_vcycle(float *p, const float *rhs, int nx, int ny, double dx, double dy);
float orc_mg_residual(const float *p, const float *rhs, int nx, int ny, double dx, double dy);

/* Threads for the row loops of the Model::update path (default 1, the
 * reference's single worker thread, model.rs:1287).  n > 1 is the labelled
 * all-core CPU baseline of SURVEY §8(d): rows split across OpenMP threads,
 * per-thread maxima folded afterwards; every result is bit-identical to the
 * 1-thread run (no sums change order, maxima are order-independent). */
void orc_set_threads(int n);
int orc_get_threads(void);

/* Raw field access. Field ids: */
enum { ORC_U = 0, ORC_V, ORC_P, ORC_U_OLD, ORC_V_OLD, ORC_U_STAR, ORC_V_STAR,
       ORC_RHS, ORC_PP, ORC_PPN, ORC_NFIELDS };
float *orc_field(orc_model *m, int which);
size_t orc_field_len(const orc_model *m, int which);
const uint8_t *orc_mask(const orc_model *m, int which_uv);   /* 0 u, 1 v */

typedef struct {
    uint64_t step;
    float time, dt, p, u, v;
    float current_inlet_velocity;
    uint64_t jacobi_sweeps_total;
} orc_scalars;
void orc_get_scalars(const orc_model *m, orc_scalars *s);
void orc_set_scalars(orc_model *m, const orc_scalars *s);

#ifdef __cplusplus
}
#endif
#endif
