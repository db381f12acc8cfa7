/*
 * cfd_oracle_solvers.c — CPU restatement of the alternative pressure solvers
 * of the reference's JavaScript variant (/root/reference/index.html): SOR
 * (:741-774) and the multigrid V-cycle (:775-795, :1344-1470).  TEST
 * INFRASTRUCTURE ONLY (see cfd_oracle.h): never linked into the product.
 *
 * The Rust model declares only PressureSolver::Jacobi (model.rs:148-152);
 * SURVEY.md §8(f) row 3 adds these two as selectable solvers of the same
 * Model::update step (cfd_params.pressure_solver 1 and 2).
 *
 * Arithmetic: JavaScript numbers are IEEE doubles while the script's arrays
 * are Float32Array, so every expression here is evaluated in double, in the
 * script's order (left-associative, no contraction: build with
 * -ffp-contract=off), and rounded to f32 exactly where the script stores into
 * an array.  dx, dy are the model's f32 spacings widened to double.
 *
 * Pinning: the multigrid functions are checked bit for bit against the
 * script's own mgSmooth / mgRestrict / mgProlongate / mgVcycle and its
 * multigrid branch, executed by node on the same inputs
 * (tests/golden/make_js_golden.py -> tests/golden/js_mg_*.npz).  The SOR
 * restatement cannot be pinned that way: the script sweeps
 * lexicographically (a sequential dependency chain no GPU reproduces); this
 * file, like the GPU, sweeps red-black with the script's per-cell formula,
 * and is cross-checked against an independent numpy restatement
 * (tests/test_oracle_solvers.py).
 */
#include "cfd_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------- SOR */

/* One color of red-black SOR: cells (i + j) % 2 == color of the interior
 * i = 1..nx-2, j = 1..ny-2, each with the script's update (index.html:
 * 751-758; omega 1.7, denom = 2/dx2 + 2/dy2 from :181-183). */
static void sor_color(float *pp, const float *rhs, size_t nx, size_t ny, double dx, double dy,
                      double denom, int color, double *max_error) {
    const double omega = 1.7;
    for (size_t j = 1; j + 1 < ny; ++j) {
        for (size_t i = 1 + ((j + 1 + (size_t)color) & 1); i + 1 < nx; i += 2) {
            size_t idx = i + j * nx;
            double p_old = (double)pp[idx];
            double p_update = (((double)pp[idx + 1] + (double)pp[idx - 1]) / (dx * dx) +
                               ((double)pp[idx + nx] + (double)pp[idx - nx]) / (dy * dy) -
                               (double)rhs[idx]) / denom;
            pp[idx] = (float)((1.0 - omega) * p_old + omega * p_update);
            double error = fabs((double)pp[idx] - p_old);
            if (error > *max_error) *max_error = error;
        }
    }
}

/* index.html:741-774 in red-black order: p' = 0, up to `iters` iterations of
 * {red, black, p' BCs (:761-770)}, stop once the iteration's max |dp'|
 * (rounded to f32) is below p_tol when tol_enabled.  Returns that residual;
 * *done = iterations run. */
float orc_sor_solve(float *pp, const float *rhs, size_t nx, size_t ny, float dxf, float dyf,
                    int iters, int tol_enabled, float p_tol, int *done) {
    double dx = (double)dxf, dy = (double)dyf;
    double dx2 = dx * dx, dy2 = dy * dy;
    double denom = 2.0 / dx2 + 2.0 / dy2;
    memset(pp, 0, nx * ny * sizeof(float)); /* :743 */
    float final_res = 0.0f;
    int n = 0;
    for (int iter = 0; iter < iters; ++iter) {
        double max_error = 0.0;
        sor_color(pp, rhs, nx, ny, dx, dy, denom, 0, &max_error);
        sor_color(pp, rhs, nx, ny, dx, dy, denom, 1, &max_error);
        for (size_t i = 0; i < nx; ++i) { /* :762-765 */
            pp[i] = pp[i + nx];
            pp[i + (ny - 1) * nx] = pp[i + (ny - 2) * nx];
        }
        for (size_t j = 0; j < ny; ++j) { /* :767-770 */
            pp[j * nx] = pp[1 + j * nx];
            pp[nx - 1 + j * nx] = 0.0f;
        }
        ++n;
        final_res = (float)max_error;
        if (tol_enabled && final_res < p_tol) break; /* :772 */
    }
    if (done) *done = n;
    return final_res;
}

/* ------------------------------------------------------------- multigrid */

/* mgSmooth (index.html:1347-1369): `iterations` plain Jacobi sweeps of the
 * interior; boundary cells keep their values. */
void orc_mg_smooth(float *p, const float *rhs, int nx, int ny, double dx, double dy,
                   int iterations) {
    float *p_new = (float *)calloc((size_t)nx * ny + 1, sizeof(float));
    const double denom_local = 2.0 / (dx * dx) + 2.0 / (dy * dy);
    for (int it = 0; it < iterations; ++it) {
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i) {
                size_t idx = (size_t)i + (size_t)j * nx;
                double p_e = p[idx + 1], p_w = p[idx - 1];
                double p_n = p[idx + nx], p_s = p[idx - nx];
                p_new[idx] = (float)(((p_e + p_w) / (dx * dx) + (p_n + p_s) / (dy * dy) -
                                      (double)rhs[idx]) / denom_local);
            }
        for (int j = 1; j < ny - 1; ++j)
            for (int i = 1; i < nx - 1; ++i)
                p[(size_t)i + (size_t)j * nx] = p_new[(size_t)i + (size_t)j * nx];
    }
    free(p_new);
}

/* mgRestrict (index.html:1372-1395): full weighting of the interior, then
 * injection on the rows and (overwriting the corners) the columns. */
void orc_mg_restrict(const float *fine, int nx_f, int ny_f, float *coarse, int nx_c, int ny_c) {
    memset(coarse, 0, (size_t)nx_c * ny_c * sizeof(float));
    for (int j = 1; j < ny_c - 1; ++j)
        for (int i = 1; i < nx_c - 1; ++i) {
            size_t fi = 2 * (size_t)i, fj = 2 * (size_t)j, w = (size_t)nx_f;
            double sum = (double)fine[fi + fj * w] +
                         0.5 * ((double)fine[(fi - 1) + fj * w] + (double)fine[(fi + 1) + fj * w] +
                                (double)fine[fi + (fj - 1) * w] + (double)fine[fi + (fj + 1) * w]) +
                         0.25 * ((double)fine[(fi - 1) + (fj - 1) * w] +
                                 (double)fine[(fi - 1) + (fj + 1) * w] +
                                 (double)fine[(fi + 1) + (fj - 1) * w] +
                                 (double)fine[(fi + 1) + (fj + 1) * w]);
            coarse[(size_t)i + (size_t)j * nx_c] = (float)(sum / 4.0);
        }
    for (int i = 0; i < nx_c; ++i) {
        coarse[i] = fine[2 * (size_t)i];
        coarse[(size_t)i + (size_t)(ny_c - 1) * nx_c] =
            fine[2 * (size_t)i + (size_t)(ny_f - 1) * nx_f];
    }
    for (int j = 0; j < ny_c; ++j) {
        coarse[(size_t)j * nx_c] = fine[(size_t)(2 * j) * nx_f];
        coarse[(size_t)(nx_c - 1) + (size_t)j * nx_c] =
            fine[(size_t)(nx_f - 1) + (size_t)(2 * j) * nx_f];
    }
}

/* mgProlongate (index.html:1398-1421): bilinear, weights a, b in {0, 0.5}. */
void orc_mg_prolongate(const float *coarse, int nx_c, int ny_c, float *fine, int nx_f, int ny_f) {
    for (int j = 0; j < ny_f; ++j) {
        double y_coarse = j / 2.0;
        int j0 = (int)floor(y_coarse);
        int j1 = j0 + 1 < ny_c - 1 ? j0 + 1 : ny_c - 1;
        double b = y_coarse - j0;
        for (int i = 0; i < nx_f; ++i) {
            double x_coarse = i / 2.0;
            int i0 = (int)floor(x_coarse);
            int i1 = i0 + 1 < nx_c - 1 ? i0 + 1 : nx_c - 1;
            double a = x_coarse - i0;
            fine[(size_t)i + (size_t)j * nx_f] =
                (float)((1 - a) * (1 - b) * (double)coarse[(size_t)i0 + (size_t)j0 * nx_c] +
                        a * (1 - b) * (double)coarse[(size_t)i1 + (size_t)j0 * nx_c] +
                        (1 - a) * b * (double)coarse[(size_t)i0 + (size_t)j1 * nx_c] +
                        a * b * (double)coarse[(size_t)i1 + (size_t)j1 * nx_c]);
        }
    }
}

/* mgVcycle (index.html:1424-1470), recursive as in the script. */
void orc_mg_vcycle(float *p, const float *rhs, int nx, int ny, double dx, double dy) {
    const double denom_local = 2.0 / (dx * dx) + 2.0 / (dy * dy);
    orc_mg_smooth(p, rhs, nx, ny, dx, dy, 5);
    float *r = (float *)calloc((size_t)nx * ny + 1, sizeof(float));
    for (int j = 1; j < ny - 1; ++j)
        for (int i = 1; i < nx - 1; ++i) {
            size_t idx = (size_t)i + (size_t)j * nx;
            double p_e = p[idx + 1], p_w = p[idx - 1], p_n = p[idx + nx], p_s = p[idx - nx];
            double ap = (p_e + p_w) / (dx * dx) + (p_n + p_s) / (dy * dy) -
                        denom_local * (double)p[idx];
            r[idx] = (float)((double)rhs[idx] - ap);
        }
    if (nx <= 4 || ny <= 4) {
        orc_mg_smooth(p, rhs, nx, ny, dx, dy, 10);
        free(r);
        return;
    }
    int nx_c = (nx + 1) / 2, ny_c = (ny + 1) / 2;
    float *r_c = (float *)calloc((size_t)nx_c * ny_c + 1, sizeof(float));
    float *e_c = (float *)calloc((size_t)nx_c * ny_c + 1, sizeof(float));
    float *e_f = (float *)calloc((size_t)nx * ny + 1, sizeof(float));
    orc_mg_restrict(r, nx, ny, r_c, nx_c, ny_c);
    orc_mg_vcycle(e_c, r_c, nx_c, ny_c, 2 * dx, 2 * dy);
    orc_mg_prolongate(e_c, nx_c, ny_c, e_f, nx, ny);
    for (size_t k = 0; k < (size_t)nx * ny; ++k) p[k] = (float)((double)p[k] + (double)e_f[k]);
    orc_mg_smooth(p, rhs, nx, ny, dx, dy, 5);
    free(r);
    free(r_c);
    free(e_c);
    free(e_f);
}

/* Final residual of the multigrid branch (index.html:783-795): max |A p - rhs|
 * over the interior, NaN ignored (`>` is false for NaN), rounded to f32. */
float orc_mg_residual(const float *p, const float *rhs, int nx, int ny, double dx, double dy) {
    const double denom_local = 2.0 / (dx * dx) + 2.0 / (dy * dy);
    double max_error = 0.0;
    for (int j = 1; j < ny - 1; ++j)
        for (int i = 1; i < nx - 1; ++i) {
            size_t idx = (size_t)i + (size_t)j * nx;
            double r = ((double)p[idx + 1] + (double)p[idx - 1]) / (dx * dx) +
                       ((double)p[idx + nx] + (double)p[idx - nx]) / (dy * dy) -
                       denom_local * (double)p[idx] - (double)rhs[idx];
            if (fabs(r) > max_error) max_error = fabs(r);
        }
    return (float)max_error;
}

/* The multigrid branch of the script's pressure correction (index.html:
 * 775-795): p' = 0, 3 V-cycles, then the residual; no p' boundary conditions
 * afterwards, as in the script. */
float orc_mg_solve(float *pp, const float *rhs, int nx, int ny, float dxf, float dyf) {
    double dx = (double)dxf, dy = (double)dyf;
    memset(pp, 0, (size_t)nx * ny * sizeof(float));
    for (int cycle = 0; cycle < 3; ++cycle) orc_mg_vcycle(pp, rhs, nx, ny, dx, dy);
    return orc_mg_residual(pp, rhs, nx, ny, dx, dy);
}
