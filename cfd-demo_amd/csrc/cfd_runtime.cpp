// cfd_runtime.cpp — Model::run (/root/reference/src/model.rs:1282-1332) as a
// native host runtime over the C ABI: a worker thread owns the model and, per
// loop iteration, drains the command queue (Stop, SetParams, GetSnapshot,
// Pause, Resume — model.rs:57-63, 1291-1315) and then either steps the model
// and publishes its residuals (:1317-1320) or sleeps 16 ms while paused
// (:1322).  The mpsc channels of the reference become a mutex-guarded command
// deque, a latest-snapshot slot (get_last_available_snapshot drains the
// channel and keeps only the newest, :76-86, so only the newest is kept) and a
// residual deque (get_new_log_messages, :88-98).
//
// Only the public C ABI is used here (cfd_update, cfd_get_residuals,
// cfd_get_snapshot, cfd_set_params), from the worker thread alone, which
// keeps the handle's one-thread rule (include/cfd.h).  Host C++ only: no
// device code in this file.
//
// Deliberate difference: the reference's Command::Stop only breaks out of the
// command loop (model.rs:1296) and its thread ends when a send fails after the
// handle is dropped (:1304, :1319); here Stop ends the worker, and
// cfd_run_stop joins it and hands the model back to the caller.
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cfd.h"

extern "C" void cfdrt_set_error(const char *msg);   // cfd_model.hip (internal)
extern "C" int cfdrt_check_params(const cfd_model *m, const cfd_params *p);   // ditto

namespace {

enum CmdKind { CMD_STOP, CMD_PARAMS, CMD_SNAPSHOT, CMD_PAUSE, CMD_RESUME };

struct Cmd {
    CmdKind kind;
    cfd_params params;
};

constexpr size_t kMaxQueuedResiduals = size_t(1) << 20;   // oldest dropped beyond this

}  // namespace

struct cfd_runner {
    cfd_model *model = nullptr;
    size_t n_u = 0, n_v = 0, n_p = 0;
    std::thread worker;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Cmd> cmds;
    std::deque<cfd_residuals> residuals;
    // snapshot slot: the newest snapshot not yet taken
    std::vector<float> snap_u, snap_v, snap_p;
    float snap_dt = 0.f;
    int snap_paused = 0;
    bool snap_ready = false;
    int status = 0;            // first failing cfd_* status of the worker
    std::string error;
    uint64_t steps = 0;

    void run();
};

void cfd_runner::run() {
    bool paused = false;
    std::vector<float> u(n_u), v(n_v), p(n_p);
    for (;;) {
        std::deque<Cmd> batch;
        {
            std::lock_guard<std::mutex> lk(mu);
            batch.swap(cmds);
        }
        bool stop = false, snapshot_sent = false;
        for (const Cmd &c : batch) {   // model.rs:1294-1315, in order
            if (c.kind == CMD_STOP) {
                stop = true;
                break;
            }
            int rc = 0;
            if (c.kind == CMD_PARAMS) {
                rc = cfd_set_params(model, &c.params);
            } else if (c.kind == CMD_SNAPSHOT && !snapshot_sent) {
                float dt = 0.f;
                rc = cfd_get_snapshot(model, u.data(), v.data(), p.data(), &dt);
                if (!rc) {
                    std::lock_guard<std::mutex> lk(mu);
                    snap_u.swap(u);
                    snap_v.swap(v);
                    snap_p.swap(p);
                    if (u.size() != n_u) {
                        u.assign(n_u, 0.f);
                        v.assign(n_v, 0.f);
                        p.assign(n_p, 0.f);
                    }
                    snap_dt = dt;
                    snap_paused = paused ? 1 : 0;
                    snap_ready = true;
                }
                snapshot_sent = true;
            } else if (c.kind == CMD_PAUSE) {
                paused = true;
            } else if (c.kind == CMD_RESUME) {
                paused = false;
            }
            if (rc) {
                std::lock_guard<std::mutex> lk(mu);
                if (!status) {
                    status = rc;
                    error = cfd_last_error();
                }
            }
        }
        if (stop) return;
        bool failed;
        {
            std::lock_guard<std::mutex> lk(mu);
            failed = status != 0;
        }
        if (!paused && !failed) {   // model.rs:1317-1320
            cfd_residuals r;
            int rc = cfd_update(model);
            if (!rc) rc = cfd_get_residuals(model, &r);
            std::lock_guard<std::mutex> lk(mu);
            if (rc) {
                status = rc;
                error = cfd_last_error();
            } else {
                residuals.push_back(r);
                if (residuals.size() > kMaxQueuedResiduals) residuals.pop_front();
                ++steps;
            }
        } else {                    // model.rs:1322 (or a failed model: wait for Stop)
            std::unique_lock<std::mutex> lk(mu);
            cv.wait_for(lk, std::chrono::milliseconds(16), [&] { return !cmds.empty(); });
        }
    }
}

namespace {

int run_fail(int code, const char *msg) {
    cfdrt_set_error(msg);   // the thread's cfd_last_error() (cfd_model.hip)
    return code;
}

int post(cfd_runner *r, Cmd c) {
    if (!r) return run_fail(CFD_EINVAL, "null runner");
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->cmds.push_back(c);
    }
    r->cv.notify_one();
    return 0;
}

}  // namespace

extern "C" {

int cfd_run_start(cfd_model *m, cfd_runner **out) {
    if (!m || !out) return run_fail(CFD_EINVAL, "null model or out");
    uint64_t j0 = 0, j1 = 0;
    int rc = cfd_get_slab(m, &j0, &j1);
    if (rc) return rc;
    cfd_residuals probe;
    rc = cfd_get_residuals(m, &probe);   // fails loudly on a broken model / device
    if (rc) return rc;
    cfd_runner *r = new cfd_runner();
    r->model = m;
    // snapshot sizes: the model's slab in the reference layout (include/cfd.h)
    cfd_grid g;
    rc = cfd_get_config(m, &g, nullptr);
    if (rc) {
        delete r;
        return rc;
    }
    const uint64_t nyl = j1 - j0;
    const uint64_t nx = g.nx;
    r->n_u = (size_t)((nx + 1) * nyl);
    r->n_v = (size_t)(nx * (nyl + 1));
    r->n_p = (size_t)(nx * nyl);
    r->worker = std::thread([r] { r->run(); });
    *out = r;
    return 0;
}

int cfd_run_stop(cfd_runner *r) {
    if (!r) return run_fail(CFD_EINVAL, "null runner");
    Cmd c{};
    c.kind = CMD_STOP;
    post(r, c);
    if (r->worker.joinable()) r->worker.join();
    delete r;
    return 0;
}

int cfd_run_pause(cfd_runner *r) {
    Cmd c{};
    c.kind = CMD_PAUSE;
    return post(r, c);
}

int cfd_run_resume(cfd_runner *r) {
    Cmd c{};
    c.kind = CMD_RESUME;
    return post(r, c);
}

int cfd_run_set_params(cfd_runner *r, const cfd_params *p) {
    if (!r || !p) return run_fail(CFD_EINVAL, "null runner or params");
    // the reference's set_parameters cannot fail (model.rs:1250-1257): reject
    // what cfd_set_params would reject here, before the worker sees it
    if (int rc = cfdrt_check_params(r->model, p)) return rc;
    Cmd c{};
    c.kind = CMD_PARAMS;
    c.params = *p;
    return post(r, c);
}

int cfd_run_request_snapshot(cfd_runner *r) {
    Cmd c{};
    c.kind = CMD_SNAPSHOT;
    return post(r, c);
}

int cfd_run_last_snapshot(cfd_runner *r, float *u, float *v, float *p, float *dt_out,
                          int *paused_out, int *available) {
    if (!r || !available) return run_fail(CFD_EINVAL, "null runner or available");
    std::lock_guard<std::mutex> lk(r->mu);
    *available = r->snap_ready ? 1 : 0;
    if (!r->snap_ready) return 0;
    if (u) std::memcpy(u, r->snap_u.data(), r->n_u * 4);
    if (v) std::memcpy(v, r->snap_v.data(), r->n_v * 4);
    if (p) std::memcpy(p, r->snap_p.data(), r->n_p * 4);
    if (dt_out) *dt_out = r->snap_dt;
    if (paused_out) *paused_out = r->snap_paused;
    r->snap_ready = false;
    return 0;
}

int cfd_run_new_residuals(cfd_runner *r, cfd_residuals *out, int max, int *n_out) {
    if (!r || !n_out || (max > 0 && !out)) return run_fail(CFD_EINVAL, "bad arguments");
    std::lock_guard<std::mutex> lk(r->mu);
    int n = 0;
    while (n < max && !r->residuals.empty()) {
        out[n++] = r->residuals.front();
        r->residuals.pop_front();
    }
    *n_out = n;
    return 0;
}

int cfd_run_status(cfd_runner *r, char *msg, size_t msg_len) {
    if (!r) return run_fail(CFD_EINVAL, "null runner");
    std::lock_guard<std::mutex> lk(r->mu);
    if (msg && msg_len) {
        std::strncpy(msg, r->error.c_str(), msg_len - 1);
        msg[msg_len - 1] = '\0';
    }
    return r->status;
}

uint64_t cfd_run_steps(cfd_runner *r) {
    if (!r) return 0;
    std::lock_guard<std::mutex> lk(r->mu);
    return r->steps;
}

}  // extern "C"
