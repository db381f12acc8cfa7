/*
 * cfd_oracle.c — scalar C restatement of /root/reference/src/model.rs (the
 * Model::update hot path).  TEST INFRASTRUCTURE ONLY (see cfd_oracle.h):
 * never linked into the product library, never on the product path.
 *
 * PARITY UNPINNED (no reference build, no reference golden vectors); pinned
 * instead by bitwise agreement with the independent numpy restatement
 * oracle/np_model.py.
 *
 * Build with -ffp-contract=off and WITHOUT -ffast-math: Rust never contracts
 * a*b+c into an FMA and divides with IEEE f32 division, so every expression
 * below is evaluated in exactly the reference's order with one rounding per
 * operation.
 *
 * The reference processes rows in 8-lane std::simd chunks (LANES = 8,
 * model.rs:11).  Where the chunking changes the arithmetic (which columns feed
 * the Jacobi residual, the corrector tail's association, the zeroed lane of
 * the second-order v predictor) this file reproduces the chunk structure;
 * elsewhere lane k of chunk i is simply element i+k and the loops are
 * written per element.  Flat row-major arrays are indexed exactly as the
 * reference indexes them, so its wrap-around reads across row ends
 * (e.g. u[(nx+1) + j*(nx+1)] == U(0, j+1)) happen here too.
 */
#include "cfd_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define LANES 8 /* model.rs:11 */

/* Row-loop threads (orc_set_threads); 1 = the reference's single thread. */
static int g_threads = 1;
void orc_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
int orc_get_threads(void) { return g_threads; }
static inline int thread_id(void) {
#ifdef _OPENMP
    return omp_get_thread_num();
#else
    return 0;
#endif
}

struct orc_model {
    size_t nx, ny;
    float lx, ly, dx, dy;
    float dt, nu;
    size_t simulation_step, ramp_up_steps;
    float current_inlet_velocity, target_inlet_velocity;
    int scheme, profile, solver;
    int jacobi_iters, corrector_passes, tol_enabled, bc_kind;
    float p_tol;
    float *f[ORC_NFIELDS];
    size_t len[ORC_NFIELDS];
    uint8_t *mask_u, *mask_v;
    size_t *obs_i, *obs_j, n_obs;
    float last_pressure_residual, last_u_residual, last_v_residual;
    float simulation_time;
    uint64_t sweeps_total;
};

#define U_(m) ((m)->f[ORC_U])
#define V_(m) ((m)->f[ORC_V])

/* ---------------------------------------------------------------- init */

/* Model::new (model.rs:219-299): zero fields, obstacle masks from cell
 * centres with strict distance < radius (model.rs:236-260). */
orc_model *orc_create(const orc_grid *g, const orc_params *p) {
    orc_model *m = (orc_model *)calloc(1, sizeof(orc_model));
    size_t nx = (size_t)g->nx, ny = (size_t)g->ny;
    m->nx = nx;
    m->ny = ny;
    m->lx = g->lx;
    m->ly = g->ly;
    m->dx = g->lx / (float)nx; /* app.rs:37 */
    m->dy = g->ly / (float)ny; /* app.rs:38 */
    size_t size_u = (nx + 1) * ny, size_v = nx * (ny + 1), size_p = nx * ny;
    const size_t lens[ORC_NFIELDS] = {size_u, size_v, size_p, size_u, size_v,
                                      size_u, size_v, size_p, size_p, size_p};
    for (int k = 0; k < ORC_NFIELDS; ++k) {
        m->len[k] = lens[k];
        m->f[k] = (float *)calloc(lens[k] + 16, sizeof(float));
    }
    m->mask_u = (uint8_t *)calloc(size_u + 16, 1);
    m->mask_v = (uint8_t *)calloc(size_v + 16, 1);
    m->obs_i = (size_t *)calloc(size_p + 1, sizeof(size_t));
    m->obs_j = (size_t *)calloc(size_p + 1, sizeof(size_t));
    if (g->has_cylinder) {
        for (size_t j = 0; j < ny; ++j) {
            for (size_t i = 0; i < nx; ++i) {
                float x = ((float)i + 0.5f) * m->dx;
                float y = ((float)j + 0.5f) * m->dy;
                float ddx = x - g->cx;
                float ddy = y - g->cy;
                float distance = sqrtf(ddx * ddx + ddy * ddy);
                if (distance < g->radius) {
                    if (i > 0) m->mask_u[i + j * (nx + 1)] = 1;
                    if (i < nx) m->mask_u[(i + 1) + j * (nx + 1)] = 1;
                    if (j > 0) m->mask_v[i + j * nx] = 1;
                    if (j < ny) m->mask_v[i + (j + 1) * nx] = 1;
                    m->obs_i[m->n_obs] = i;
                    m->obs_j[m->n_obs] = j;
                    m->n_obs++;
                }
            }
        }
    }
    m->simulation_step = 0;
    m->ramp_up_steps = 100; /* model.rs:269 */
    m->current_inlet_velocity = 0.0f;
    orc_set_params(m, p);
    m->dt = p->dt;
    return m;
}

void orc_destroy(orc_model *m) {
    if (!m) return;
    for (int k = 0; k < ORC_NFIELDS; ++k) free(m->f[k]);
    free(m->mask_u);
    free(m->mask_v);
    free(m->obs_i);
    free(m->obs_j);
    free(m);
}

/* set_parameters (model.rs:1250-1257) + build knobs. */
void orc_set_params(orc_model *m, const orc_params *p) {
    m->nu = p->viscosity;
    m->dt = p->dt;
    m->target_inlet_velocity = p->target_inlet_velocity;
    m->scheme = p->scheme;
    m->solver = p->pressure_solver;
    m->profile = p->inlet_profile;
    m->jacobi_iters = p->jacobi_iters;
    m->corrector_passes = p->corrector_passes;
    m->tol_enabled = p->tol_enabled;
    m->p_tol = p->p_tol;
    m->bc_kind = p->bc_kind;
}

/* ------------------------------------------------- u predictor helpers */

/* get_v_north / get_v_south (model.rs:1056-1069): NOT averaged. */
static inline float get_v_north(const orc_model *m, size_t i, size_t j) {
    return V_(m)[i + (j + 1) * m->nx];
}
static inline float get_v_south(const orc_model *m, size_t i, size_t j) {
    return V_(m)[i + j * m->nx];
}
/* get_v_north_scalar / get_v_south_scalar (model.rs:983-989, 1028-1034). */
static inline float get_v_north_scalar(const orc_model *m, size_t i, size_t j) {
    size_t nx = m->nx;
    size_t idx_v_nw = i > 0 ? (i - 1) + (j + 1) * nx : 0;
    size_t idx_v_n = i + (j + 1) * nx;
    return 0.5f * (V_(m)[idx_v_nw] + V_(m)[idx_v_n]);
}
static inline float get_v_south_scalar(const orc_model *m, size_t i, size_t j) {
    size_t nx = m->nx;
    size_t idx_v_s = i > 0 ? (i - 1) + j * nx : 0;
    size_t idx_v = i + j * nx;
    return 0.5f * (V_(m)[idx_v_s] + V_(m)[idx_v]);
}

/* u_face_e_first_order (model.rs:893-908) */
static inline float u_face_e_fo(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx;
    float ul = u[i + j * (nx + 1)], ur = u[(i + 1) + j * (nx + 1)];
    float avg = (ul + ur) * 0.5f;
    return avg >= 0.0f ? ul : ur;
}
/* u_face_w_first_order (model.rs:929-941) */
static inline float u_face_w_fo(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx;
    float uc = u[i + j * (nx + 1)], uw = u[(i - 1) + j * (nx + 1)];
    float avg = (uw + uc) * 0.5f;
    return avg >= 0.0f ? uw : uc;
}
/* u_face_n_first_order (model.rs:966-981) */
static inline float u_face_n_fo(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx;
    float vn = get_v_north(m, i, j);
    return vn >= 0.0f ? u[i + j * (nx + 1)] : u[i + (j + 1) * (nx + 1)];
}
/* u_face_s_first_order (model.rs:1011-1026) */
static inline float u_face_s_fo(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx;
    float vs = get_v_south(m, i, j);
    return vs >= 0.0f ? u[i + (j - 1) * (nx + 1)] : u[i + j * (nx + 1)];
}
/* u_face_e_second_order (model.rs:911-926) */
static inline float u_face_e_so(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx, len = m->len[ORC_U];
    size_t idx = i + j * (nx + 1);
    size_t idx_e = (i + 1) + j * (nx + 1);
    if (u[idx] >= 0.0f) {
        if (i > 1) return 1.5f * u[idx] - 0.5f * u[idx - 1];
        return u[idx];
    } else if ((idx_e + 1) < len && i < nx - 1) {
        return 1.5f * u[idx_e] - 0.5f * u[idx_e + 1];
    }
    return u[idx_e];
}
/* u_face_w_second_order (model.rs:944-963) */
static inline float u_face_w_so(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx;
    size_t idx = i + j * (nx + 1);
    size_t idx_w = (i - 1) + j * (nx + 1);
    size_t idx_e = (i + 1) + j * (nx + 1);
    if (u[idx_w] >= 0.0f) {
        if (i > 2) return 1.5f * u[idx_w] - 0.5f * u[(i - 2) + j * (nx + 1)];
        return u[idx_w];
    }
    if (i < nx) return 1.5f * u[idx] - 0.5f * u[idx_e];
    return u[idx];
}
/* u_face_n_second_order (model.rs:992-1008) */
static inline float u_face_n_so(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx, ny = m->ny, len = m->len[ORC_U];
    size_t idx = i + j * (nx + 1);
    size_t idx_n = i + (j + 1) * (nx + 1);
    float vn = get_v_north_scalar(m, i, j);
    if (vn >= 0.0f) {
        if (j > 1) return 1.5f * u[idx] - 0.5f * u[i + (j - 1) * (nx + 1)];
        return u[idx];
    } else if ((i + (j + 2) * (nx + 1)) < len && j < ny - 1) {
        return 1.5f * u[idx_n] - 0.5f * u[i + (j + 2) * (nx + 1)];
    }
    return u[idx_n];
}
/* u_face_s_second_order (model.rs:1037-1053) */
static inline float u_face_s_so(const orc_model *m, size_t i, size_t j) {
    const float *u = U_(m);
    size_t nx = m->nx, ny = m->ny;
    size_t idx = i + j * (nx + 1);
    size_t idx_s = i + (j - 1) * (nx + 1);
    float vs = get_v_south_scalar(m, i, j);
    if (vs >= 0.0f) {
        if (j > 1) return 1.5f * u[idx_s] - 0.5f * u[i + (j - 2) * (nx + 1)];
        return u[idx_s];
    } else if (j < ny) {
        return 1.5f * u[idx] - 0.5f * u[i + (j + 1) * (nx + 1)];
    }
    return u[idx];
}

/* compute_ustar body for one lane (model.rs:382-436). */
static inline void compute_ustar_1(orc_model *m, float dt_sub, size_t i, size_t j,
                                   float v_n, float v_s, float u_n, float u_s,
                                   float u_e, float u_w) {
    const float *u = U_(m);
    size_t nx = m->nx;
    float dx = m->dx, dy = m->dy, nu = m->nu;
    size_t idx = i + j * (nx + 1);
    float f_e = u_e * u_e;
    float f_w = u_w * u_w;
    float f_n = v_n * u_n;
    float f_s = v_s * u_s;
    float convective = (f_e - f_w) / dx + (f_n - f_s) / dy;
    float uc = u[idx];
    float ue = u[(i + 1) + j * (nx + 1)];
    float uw = u[(i - 1) + j * (nx + 1)];
    float us = u[i + (j - 1) * (nx + 1)];
    float un = u[i + (j + 1) * (nx + 1)];
    float laplace = (ue - 2.0f * uc + uw) / (dx * dx) + (un - 2.0f * uc + us) / (dy * dy);
    float u_star = uc + dt_sub * (-convective + nu * laplace);
    if (m->mask_u[idx] == 1) u_star = 0.0f;
    m->f[ORC_U_STAR][idx] = u_star;
}

/* u predictor loops (model.rs:538-580): rows 1..ny-1 (exclusive), faces
 * (1..nx).step_by(8) -> with nx % 8 == 0 the lanes cover faces 1..=nx. */
void orc_u_predictor(orc_model *m, float dt_sub) {
    size_t nx = m->nx, ny = m->ny;
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (size_t j = 1; j < ny - 1; ++j) {
        for (size_t i = 1; i < nx; i += LANES) {
            for (size_t k = 0; k < LANES; ++k) {
                size_t ii = i + k;
                float vn = get_v_north(m, ii, j);
                float vs = get_v_south(m, ii, j);
                float un, us, ue, uw;
                if (m->scheme == 0) {
                    un = u_face_n_fo(m, ii, j);
                    us = u_face_s_fo(m, ii, j);
                    ue = u_face_e_fo(m, ii, j);
                    uw = u_face_w_fo(m, ii, j);
                } else {
                    un = u_face_n_so(m, ii, j);
                    us = u_face_s_so(m, ii, j);
                    ue = u_face_e_so(m, ii, j);
                    uw = u_face_w_so(m, ii, j);
                }
                compute_ustar_1(m, dt_sub, ii, j, vn, vs, un, us, ue, uw);
            }
        }
    }
}

/* ------------------------------------------------- v predictor helpers */

/* v_face_e_first_order(_scalar) (model.rs:1073-1095) */
static inline float v_face_e_fo(const orc_model *m, size_t i, size_t j) {
    size_t nx = m->nx, idx = i + j * nx;
    float u_e = U_(m)[(i + 1) + j * (nx + 1)];
    return u_e >= 0.0f ? V_(m)[idx] : V_(m)[idx + 1];
}
/* v_face_w_first_order(_scalar) (model.rs:1116-1142) */
static inline float v_face_w_fo(const orc_model *m, size_t i, size_t j) {
    size_t nx = m->nx, idx = i + j * nx;
    float u_w = U_(m)[i + j * (nx + 1)];
    return u_w >= 0.0f ? V_(m)[idx - 1] : V_(m)[idx];
}
/* v_face_n_first_order(_scalar) (model.rs:1163-1185) */
static inline float v_face_n_fo(const orc_model *m, size_t i, size_t j) {
    size_t nx = m->nx, idx = i + j * nx, idx_n = i + (j + 1) * nx;
    float avg = 0.5f * (V_(m)[idx] + V_(m)[idx_n]);
    return avg >= 0.0f ? V_(m)[idx] : V_(m)[idx_n];
}
/* v_face_s_first_order(_scalar) (model.rs:1207-1229) */
static inline float v_face_s_fo(const orc_model *m, size_t i, size_t j) {
    size_t nx = m->nx, idx = i + j * nx, idx_s = i + (j - 1) * nx;
    float avg = 0.5f * (V_(m)[idx_s] + V_(m)[idx]);
    return avg >= 0.0f ? V_(m)[idx_s] : V_(m)[idx];
}
/* v_face_e_second_order (model.rs:1098-1113) */
static inline float v_face_e_so(const orc_model *m, size_t i, size_t j) {
    const float *v = V_(m);
    size_t nx = m->nx, idx = i + j * nx, len = m->len[ORC_V];
    float u_e = U_(m)[(i + 1) + j * (nx + 1)];
    if (u_e >= 0.0f) {
        if (i > 0) return 1.5f * v[idx] - 0.5f * v[idx - 1];
        return v[idx];
    } else if ((idx + 2) < len && i < nx - 2) {
        return 1.5f * v[idx + 1] - 0.5f * v[idx + 2];
    }
    return v[idx + 1];
}
/* v_face_w_second_order (model.rs:1145-1160) */
static inline float v_face_w_so(const orc_model *m, size_t i, size_t j) {
    const float *v = V_(m);
    size_t nx = m->nx, idx = i + j * nx;
    float u_w = U_(m)[i + j * (nx + 1)];
    if (u_w >= 0.0f) {
        if (i > 1) return 1.5f * v[idx - 1] - 0.5f * v[idx - 2];
        return v[idx - 1];
    } else if (i < nx - 1) {
        return 1.5f * v[idx] - 0.5f * v[idx + 1];
    }
    return v[idx];
}
/* v_face_n_second_order (model.rs:1188-1204) */
static inline float v_face_n_so(const orc_model *m, size_t i, size_t j) {
    const float *v = V_(m);
    size_t nx = m->nx, ny = m->ny, idx = i + j * nx, idx_n = i + (j + 1) * nx;
    size_t len = m->len[ORC_V];
    float avg = 0.5f * (v[idx] + v[idx_n]);
    if (avg >= 0.0f) {
        if (j > 1) return 1.5f * v[idx] - 0.5f * v[i + (j - 1) * nx];
        return v[idx];
    } else if ((i + (j + 2) * nx) < len && j < ny - 1) {
        return 1.5f * v[idx_n] - 0.5f * v[i + (j + 2) * nx];
    }
    return v[idx_n];
}
/* v_face_s_second_order (model.rs:1232-1248) */
static inline float v_face_s_so(const orc_model *m, size_t i, size_t j) {
    const float *v = V_(m);
    size_t nx = m->nx, ny = m->ny, idx = i + j * nx, idx_s = i + (j - 1) * nx;
    float avg = 0.5f * (v[idx_s] + v[idx]);
    if (avg >= 0.0f) {
        if (j > 1) return 1.5f * v[idx_s] - 0.5f * v[i + (j - 2) * nx];
        return v[idx_s];
    } else if (j < ny) {
        return 1.5f * v[idx] - 0.5f * v[i + (j + 1) * nx];
    }
    return v[idx];
}

/* compute_vstar body for one lane (model.rs:439-521; the scalar branch
 * :464-494 and the SIMD branch :498-520 evaluate the same expression; a
 * masked face is 0 in both). */
static inline void compute_vstar_1(orc_model *m, float dt_sub, size_t i, size_t j,
                                   float u_e, float u_w, float v_n, float v_s,
                                   float v_e, float v_w) {
    const float *v = V_(m);
    size_t nx = m->nx, idx = i + j * nx;
    float dx = m->dx, dy = m->dy;
    if (m->mask_v[idx] == 1) {
        m->f[ORC_V_STAR][idx] = 0.0f;
        return;
    }
    float f_e = u_e * v_e;
    float f_w = u_w * v_w;
    float f_n = v_n * v_n;
    float f_s = v_s * v_s;
    float convective = (f_e - f_w) / dx + (f_n - f_s) / dy;
    float v_val = v[idx];
    float v_e_val = v[(i + 1) + j * nx];
    float v_w_val = v[(i - 1) + j * nx];
    float v_n_val = v[i + (j + 1) * nx];
    float v_s_val = v[i + (j - 1) * nx];
    float laplace = (v_e_val - 2.0f * v_val + v_w_val) / (dx * dx) +
                    (v_n_val - 2.0f * v_val + v_s_val) / (dy * dy);
    m->f[ORC_V_STAR][idx] = v_val + dt_sub * (-convective + m->nu * laplace);
}

/* v predictor loops (model.rs:586-670): rows 1..ny (exclusive), columns
 * (1..nx-1).step_by(8); the last chunk (i + 8 > nx - 1) covers columns
 * i..nx-1 inclusive through the scalar branch of compute_vstar.  In the
 * SecondOrder loop the lane for column nx-1 is never filled (break at
 * i + k >= nx - 1, :648-650) so all six of its inputs stay 0.0. */
void orc_v_predictor(orc_model *m, float dt_sub) {
    size_t nx = m->nx, ny = m->ny;
    const float *u = U_(m);
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (size_t j = 1; j < ny; ++j) {
        for (size_t i = 1; i < nx - 1; i += LANES) {
            int last = (i + LANES > nx - 1);
            size_t nlanes = last ? (nx - i) : LANES;
            float ue[LANES] = {0}, uw[LANES] = {0}, vn[LANES] = {0}, vs[LANES] = {0},
                  ve[LANES] = {0}, vw[LANES] = {0};
            for (size_t k = 0; k < nlanes; ++k) {
                size_t ii = i + k;
                if (m->scheme == 1 && ii >= nx - 1) break;
                ue[k] = u[(ii + 1) + j * (nx + 1)];
                uw[k] = u[ii + j * (nx + 1)];
                if (m->scheme == 0) {
                    vn[k] = v_face_n_fo(m, ii, j);
                    vs[k] = v_face_s_fo(m, ii, j);
                    ve[k] = v_face_e_fo(m, ii, j);
                    vw[k] = v_face_w_fo(m, ii, j);
                } else {
                    vn[k] = v_face_n_so(m, ii, j);
                    vs[k] = v_face_s_so(m, ii, j);
                    ve[k] = v_face_e_so(m, ii, j);
                    vw[k] = v_face_w_so(m, ii, j);
                }
            }
            for (size_t k = 0; k < nlanes; ++k)
                compute_vstar_1(m, dt_sub, i + k, j, ue[k], uw[k], vn[k], vs[k], ve[k], vw[k]);
        }
    }
}

/* ---------------------------------------------------------- divergence */

/* recompute_divergence (model.rs:1406-1440), all nx*ny cells. */
void orc_divergence(orc_model *m, float dt_sub) {
    size_t nx = m->nx, ny = m->ny;
    const float *us = m->f[ORC_U_STAR], *vs = m->f[ORC_V_STAR];
    float *rhs = m->f[ORC_RHS];
    float dx = m->dx, dy = m->dy;
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (size_t j = 0; j < ny; ++j) {
        for (size_t i = 0; i < nx; ++i) {
            float u_e = us[(i + 1) + j * (nx + 1)];
            float u_w = us[i + j * (nx + 1)];
            float v_n = vs[i + (j + 1) * nx];
            float v_s = vs[i + j * nx];
            rhs[i + j * nx] = ((u_e - u_w) / dx + (v_n - v_s) / dy) / dt_sub;
        }
    }
}

/* --------------------------------------------------------------- Jacobi */

/* jacobi_pressure (model.rs:734-824).  The residual is taken only over the
 * SIMD chunks (columns 1..=nx-8 when nx % 8 == 0): the scalar tail chunk
 * (:755-772) never updates max_error.  Per chunk the reference keeps
 * max_error = max(max_error, reduce_max(|new - center|)) with reduce_max
 * ignoring NaN lanes and `error > max_error` false for NaN; that is exactly a
 * running `if (e > max_error) max_error = e` over the chunk columns, which is
 * how it is written here (and lets the compiler vectorise the row loop like
 * the reference's 8-lane SIMD).  p' is warm-started (never zeroed). */
static inline float jac_point(const float *pp, const float *rhs, size_t idx, size_t nx,
                              float dx_sq, float dy_sq, float denom, float omega, float om1) {
    float right = pp[idx + 1];
    float left = pp[idx - 1];
    float top = pp[idx + nx];
    float bot = pp[idx - nx];
    float center = pp[idx];
    float horizontal = (right + left) / dx_sq;
    float vertical = (top + bot) / dy_sq;
    float p_update = (horizontal + vertical - rhs[idx]) / denom;
    return omega * p_update + om1 * center;
}

float orc_jacobi_pressure(orc_model *m) {
    size_t nx = m->nx, ny = m->ny;
    float dx = m->dx, dy = m->dy;
    const float jacobi_omega = 0.75f;
    float max_error = 0.0f;
    const float dx_sq = dx * dx;
    const float dy_sq = dy * dy;
    const float om1 = 1.0f - jacobi_omega;
    const float denom = 2.0f / (dx * dx) + 2.0f / (dy * dy);
    const float *rhs = m->f[ORC_RHS];
    /* columns covered by full 8-lane chunks: i in [1, simd_end) */
    size_t simd_end = 1;
    while (simd_end + LANES <= nx - 1) simd_end += LANES;
    /* per-column running maxima (element-wise, so the row loop vectorises),
     * one set per thread; the max over all of them is order-independent */
    const int nt = g_threads;
    const size_t cstride = nx + 8;
    float *colmax = (float *)malloc((size_t)nt * cstride * sizeof(float));
    for (int iter = 0; iter < m->jacobi_iters; ++iter) {
        const float *pp = m->f[ORC_PP];
        float *ppn = m->f[ORC_PPN];
#pragma omp parallel num_threads(nt)
        {
            float *cm = colmax + (size_t)thread_id() * cstride;
            for (size_t i = 0; i < nx; ++i) cm[i] = 0.0f;
#pragma omp for schedule(static)
            for (size_t j = 1; j < ny - 1; ++j) {
                const size_t row = j * nx;
                for (size_t i = 1; i < simd_end; ++i) {
                    float nv = jac_point(pp, rhs, row + i, nx, dx_sq, dy_sq, denom, jacobi_omega, om1);
                    ppn[row + i] = nv;
                    float e = fabsf(nv - pp[row + i]);
                    cm[i] = e > cm[i] ? e : cm[i];
                }
                for (size_t i = simd_end; i < nx; ++i)   /* scalar tail, no residual */
                    ppn[row + i] = jac_point(pp, rhs, row + i, nx, dx_sq, dy_sq, denom, jacobi_omega, om1);
            }
        }
        max_error = 0.0f;
        for (int t = 0; t < nt; ++t) {
            const float *cm = colmax + (size_t)t * cstride;
            for (size_t i = 1; i < simd_end; ++i) max_error = cm[i] > max_error ? cm[i] : max_error;
        }
        /* std::mem::swap (model.rs:805) */
        float *tmp = m->f[ORC_PP];
        m->f[ORC_PP] = m->f[ORC_PPN];
        m->f[ORC_PPN] = tmp;
        float *p = m->f[ORC_PP];
        /* p' boundary conditions, in the reference's order (model.rs:807-815) */
        for (size_t i = 0; i < nx; ++i) {
            p[i] = p[i + nx];
            p[i + (ny - 1) * nx] = p[i + (ny - 2) * nx];
        }
        for (size_t j = 0; j < ny; ++j) {
            p[j * nx] = p[1 + j * nx];
            p[(nx - 1) + j * nx] = 0.0f;
        }
        m->sweeps_total++;
        if (m->tol_enabled && max_error < m->p_tol) break; /* :816 */
    }
    free(colmax);
    m->last_pressure_residual = max_error;
    return max_error;
}

/* ----------------------------------------------------------- corrector */

/* apply_corrector (model.rs:1334-1404). */
void orc_corrector(orc_model *m, float dt_sub) {
    size_t nx = m->nx, ny = m->ny;
    float dx = m->dx, dy = m->dy;
    float *u = U_(m), *v = V_(m), *p = m->f[ORC_P];
    const float *us = m->f[ORC_U_STAR], *vs = m->f[ORC_V_STAR], *pp = m->f[ORC_PP];
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (size_t j = 0; j < ny; ++j) {
        for (size_t i = 1; i < nx; i += LANES) {
            if (i + LANES > nx) {
                /* scalar tail (:1338-1346): dt * (pr - pl) / dx associates as
                 * (dt * (pr - pl)) / dx */
                for (size_t k = 0; k < nx - i; ++k) {
                    size_t idx = i + k + j * (nx + 1);
                    float p_right = pp[i + k + j * nx];
                    float p_left = pp[(i - 1) + k + j * nx];
                    u[idx] = us[idx] - dt_sub * (p_right - p_left) / dx;
                }
                continue;
            }
            for (size_t k = 0; k < LANES; ++k) {
                size_t idx = i + k + j * (nx + 1);
                float p_right = pp[i + k + j * nx];
                float p_left = pp[(i - 1) + k + j * nx];
                float correction = dt_sub * ((p_right - p_left) / dx);
                u[idx] = us[idx] - correction;
            }
        }
    }
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (size_t j = 1; j < ny; ++j) {
        for (size_t i = 0; i < nx; i += LANES) {
            size_t nl = (i + LANES > nx) ? (nx - i) : LANES;
            for (size_t k = 0; k < nl; ++k) {
                size_t idx = i + k + j * nx;
                float p_top = pp[idx];
                float p_bottom = pp[i + k + (j - 1) * nx];
                if (nl == LANES) {
                    float correction = dt_sub * ((p_top - p_bottom) / dy);
                    v[idx] = vs[idx] - correction;
                } else {
                    v[idx] = vs[idx] - dt_sub * (p_top - p_bottom) / dy;
                }
            }
        }
    }
#pragma omp parallel for schedule(static) num_threads(g_threads)
    for (size_t k = 0; k < nx * ny; ++k) p[k] += pp[k];
}

/* ------------------------------------------------------------------ BCs */

/* apply_boundary_conditions (model.rs:826-875).  bc_kind 1 (lid-driven
 * cavity) is build-defined: side walls and bottom no-slip,
 * lid row ny-1 moves at the ramped inlet velocity on faces 1..nx-1. */
void orc_boundary_conditions(orc_model *m) {
    size_t nx = m->nx, ny = m->ny;
    float dy = m->dy;
    float *u = U_(m), *v = V_(m);
    if (m->bc_kind == 0) {
        for (size_t j = 0; j < ny; ++j) {
            size_t idx = j * (nx + 1);
            float y = ((float)j + 0.5f) * dy;
            float inlet_val;
            if (m->profile == 0) {
                inlet_val = m->current_inlet_velocity;
            } else {
                float center = m->ly / 2.0f;
                float radius = m->ly / 2.0f;
                float t = (y - center) / radius;
                float val = m->current_inlet_velocity * (1.0f - t * t);
                inlet_val = val < 0.0f ? 0.0f : val;
            }
            u[idx] = inlet_val;
        }
        for (size_t j = 0; j < ny; ++j) u[nx + j * (nx + 1)] = u[(nx - 1) + j * (nx + 1)];
        for (size_t i = 0; i < nx + 1; ++i) {
            u[i] = 0.0f;
            u[i + (ny - 1) * (nx + 1)] = 0.0f;
        }
    } else {
        for (size_t j = 0; j < ny; ++j) {
            u[j * (nx + 1)] = 0.0f;
            u[nx + j * (nx + 1)] = 0.0f;
        }
        for (size_t i = 0; i < nx + 1; ++i) {
            u[i] = 0.0f;
            u[i + (ny - 1) * (nx + 1)] = (i > 0 && i < nx) ? m->current_inlet_velocity : 0.0f;
        }
    }
    for (size_t i = 0; i < nx; ++i) {
        v[i] = 0.0f;
        v[i + ny * nx] = 0.0f;
    }
    for (size_t k = 0; k < m->n_obs; ++k) {
        size_t i = m->obs_i[k], j = m->obs_j[k];
        u[i + j * (nx + 1)] = 0.0f;
        v[i + j * nx] = 0.0f;
    }
}

/* compute_automatic_time_step (model.rs:877-889). */
float orc_auto_dt(const orc_model *m) {
    float max_u = 0.0f, max_v = 0.0f;
    /* maxima over NaN-free values are order-independent: threads are exact */
#pragma omp parallel for schedule(static) num_threads(g_threads) reduction(max : max_u)
    for (size_t k = 0; k < m->len[ORC_U]; ++k) max_u = fmaxf(max_u, fabsf(U_(m)[k]));
#pragma omp parallel for schedule(static) num_threads(g_threads) reduction(max : max_v)
    for (size_t k = 0; k < m->len[ORC_V]; ++k) max_v = fmaxf(max_v, fabsf(V_(m)[k]));
    float max_vel = fmaxf(max_u, max_v);
    if (max_vel == 0.0f) return m->dt;
    const float cfl = 0.2f;
    float dt_cfl = cfl * fminf(m->dx, m->dy) / max_vel;
    return fminf(dt_cfl, m->dt);
}

/* The solve piso_step runs at model.rs:684 / :710 for the selected solver. */
float orc_pressure_solve(orc_model *m) {
    if (m->solver == 1) {
        int n = 0;
        float r = orc_sor_solve(m->f[ORC_PP], m->f[ORC_RHS], m->nx, m->ny, m->dx, m->dy,
                                m->jacobi_iters, m->tol_enabled, m->p_tol, &n);
        m->sweeps_total += (uint64_t)n;
        m->last_pressure_residual = r;
        return r;
    }
    if (m->solver == 2) {
        float r = orc_mg_solve(m->f[ORC_PP], m->f[ORC_RHS], (int)m->nx, (int)m->ny, m->dx, m->dy);
        m->sweeps_total += 1;
        m->last_pressure_residual = r;
        return r;
    }
    return orc_jacobi_pressure(m);
}

/* ---------------------------------------------------------------- step */

/* piso_step (model.rs:529-730). */
void orc_piso_step(orc_model *m, float dt_sub) {
    orc_u_predictor(m, dt_sub);
    orc_v_predictor(m, dt_sub);
    orc_divergence(m, dt_sub);
    m->last_pressure_residual = orc_pressure_solve(m);
    orc_corrector(m, dt_sub);
    for (int pass = 0; pass < m->corrector_passes; ++pass) {
        memcpy(m->f[ORC_U_STAR], U_(m), m->len[ORC_U] * sizeof(float));
        memcpy(m->f[ORC_V_STAR], V_(m), m->len[ORC_V] * sizeof(float));
        orc_divergence(m, dt_sub);
        m->last_pressure_residual = orc_pressure_solve(m);
        orc_corrector(m, dt_sub);
        if (m->tol_enabled && m->last_pressure_residual < m->p_tol) break; /* :721 */
    }
    orc_boundary_conditions(m);
}

/* Model::update (model.rs:304-379). */
void orc_update(orc_model *m) {
    memcpy(m->f[ORC_U_OLD], U_(m), m->len[ORC_U] * sizeof(float));
    memcpy(m->f[ORC_V_OLD], V_(m), m->len[ORC_V] * sizeof(float));
    if (m->simulation_step < m->ramp_up_steps) {
        m->current_inlet_velocity =
            ((float)m->simulation_step / (float)m->ramp_up_steps) * m->target_inlet_velocity;
    } else {
        m->current_inlet_velocity = m->target_inlet_velocity;
    }
    float dt_sub = m->dt / 1.0f; /* substep_count = 1 (model.rs:267, 317) */
    orc_piso_step(m, dt_sub);
    float ru = 0.0f, rv = 0.0f;
#pragma omp parallel for schedule(static) num_threads(g_threads) reduction(max : ru)
    for (size_t k = 0; k < m->len[ORC_U]; ++k)
        ru = fmaxf(ru, fabsf(U_(m)[k] - m->f[ORC_U_OLD][k]));
#pragma omp parallel for schedule(static) num_threads(g_threads) reduction(max : rv)
    for (size_t k = 0; k < m->len[ORC_V]; ++k)
        rv = fmaxf(rv, fabsf(V_(m)[k] - m->f[ORC_V_OLD][k]));
    m->last_u_residual = ru;
    m->last_v_residual = rv;
    m->simulation_step += 1;
    m->simulation_time += m->dt;
    float previous_dt = m->dt;
    float new_dt = orc_auto_dt(m);
    m->dt = (new_dt > previous_dt) ? fminf(new_dt, previous_dt * 1.1f) : new_dt;
}

/* --------------------------------------------------------------- access */

float *orc_field(orc_model *m, int which) { return m->f[which]; }
size_t orc_field_len(const orc_model *m, int which) { return m->len[which]; }
const uint8_t *orc_mask(const orc_model *m, int which_uv) {
    return which_uv == 0 ? m->mask_u : m->mask_v;
}

void orc_get_scalars(const orc_model *m, orc_scalars *s) {
    s->step = m->simulation_step;
    s->time = m->simulation_time;
    s->dt = m->dt;
    s->p = m->last_pressure_residual;
    s->u = m->last_u_residual;
    s->v = m->last_v_residual;
    s->current_inlet_velocity = m->current_inlet_velocity;
    s->jacobi_sweeps_total = m->sweeps_total;
}

void orc_set_scalars(orc_model *m, const orc_scalars *s) {
    m->simulation_step = (size_t)s->step;
    m->simulation_time = s->time;
    m->dt = s->dt;
    m->last_pressure_residual = s->p;
    m->last_u_residual = s->u;
    m->last_v_residual = s->v;
    m->current_inlet_velocity = s->current_inlet_velocity;
    m->sweeps_total = s->jacobi_sweeps_total;
}
