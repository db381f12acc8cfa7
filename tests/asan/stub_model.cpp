// stub_model.cpp — CPU stand-in for the device side of include/cfd.h, used
// only by the sanitizer build of the host code (tests/asan).  It implements
// the entry points the native runtime (cfd_runtime.cpp) and the mesher's host
// code (cfd_mesh.hip) call, with host memory and a step counter, so the
// runtime's threads, queues and snapshot slots run under ASan/UBSan without a
// GPU.  Test infrastructure: never linked into libcfd_amd.so.
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cfd.h"

struct cfd_model {
    cfd_grid grid;
    cfd_params params;
    std::vector<float> u, v, p;
    uint64_t step = 0;
    int fail_after = -1;   // cfd_update fails (CFD_EHIP) from this step on
};

namespace {
thread_local std::string g_err;
int fail(int code, const char *m) {
    g_err = m;
    return code;
}
}  // namespace

extern "C" {

void cfdrt_set_error(const char *msg) { g_err = msg ? msg : ""; }
const char *cfd_last_error(void) { return g_err.c_str(); }

int cfdrt_check_params(const cfd_model *m, const cfd_params *p) {
    if (!m || !p) return fail(CFD_EINVAL, "null");
    if (p->jacobi_iters < 0 || p->jacobi_iters > 4096) return fail(CFD_EINVAL, "jacobi_iters out of range");
    return 0;
}

// stub-only constructor (not in cfd.h)
cfd_model *stub_model_create(uint64_t nx, uint64_t ny, int fail_after) {
    cfd_model *m = new cfd_model();
    m->grid = cfd_grid{nx, ny, 1.0f, 1.0f, 0, 0.f, 0.f, 0.f};
    std::memset(&m->params, 0, sizeof(m->params));
    m->params.jacobi_iters = 50;
    m->u.assign((nx + 1) * ny, 0.f);
    m->v.assign(nx * (ny + 1), 0.f);
    m->p.assign(nx * ny, 0.f);
    m->fail_after = fail_after;
    return m;
}
void stub_model_destroy(cfd_model *m) { delete m; }

int cfd_get_slab(const cfd_model *m, uint64_t *j0, uint64_t *j1) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (j0) *j0 = 0;
    if (j1) *j1 = m->grid.ny;
    return 0;
}

int cfd_get_config(const cfd_model *m, cfd_grid *g, cfd_params *p) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (g) *g = m->grid;
    if (p) *p = m->params;
    return 0;
}

int cfd_update(cfd_model *m) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (m->fail_after >= 0 && m->step >= (uint64_t)m->fail_after) return fail(CFD_EHIP, "stub failure");
    std::this_thread::sleep_for(std::chrono::microseconds(200));
    ++m->step;
    for (size_t k = 0; k < m->u.size(); k += 7) m->u[k] += 1.0f;
    return 0;
}

int cfd_get_residuals(cfd_model *m, cfd_residuals *out) {
    if (!m || !out) return fail(CFD_EINVAL, "null argument");
    std::memset(out, 0, sizeof(*out));
    out->simulation_step = m->step;
    out->dt = 0.005f;
    out->piso_substeps = 1;
    return 0;
}

int cfd_get_snapshot(cfd_model *m, float *u, float *v, float *p, float *dt_out) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (u) std::memcpy(u, m->u.data(), m->u.size() * 4);
    if (v) std::memcpy(v, m->v.data(), m->v.size() * 4);
    if (p) std::memcpy(p, m->p.data(), m->p.size() * 4);
    if (dt_out) *dt_out = 0.005f;
    return 0;
}

int cfd_set_params(cfd_model *m, const cfd_params *p) {
    int rc = cfdrt_check_params(m, p);
    if (rc) return rc;
    m->params = *p;
    return 0;
}

}  // extern "C"

extern "C" void cfd_default_params(cfd_params *o) {   // model.rs:44-55 defaults (as cfd_model.hip)
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->dt = 0.005f;
    o->viscosity = 0.000001f;
    o->target_inlet_velocity = 1.0f;
    o->jacobi_iters = 50;
    o->corrector_passes = 20;
    o->tol_enabled = 1;
    o->p_tol = 1e-4f;
}
