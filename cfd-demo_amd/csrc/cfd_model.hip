// cfd_model.hip — host runtime behind include/cfd.h.
//
// One cfd_model owns one slab of the grid on one GPU: its HBM fields, a HIP
// stream, the device control block (cfd::Ctl) and, for sharded models, an RCCL
// communicator with the two neighbouring ranks.  Model::update
// (/root/reference/src/model.rs:304-379) becomes a fixed sequence of kernel
// launches on that stream; the data-dependent control flow of the reference
// (Jacobi early exit :816, corrector-loop break :721, CFL dt :368-377) is
// decided on the device from Ctl, so a step is enqueued without any host
// round trip.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cmath>
#include <initializer_list>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstring>
#include <string>
#include <functional>
#include <vector>

#include "../../include/cfd.h"
#include "cfd_internal.h"
#include "slab_plan.h"

using namespace cfd;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(CFD_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

#define RCCL_TRY(expr)                                                                     \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess)                                                             \
            return fail(CFD_ERCCL, std::string(#expr) + ": " + ncclGetErrorString(r_));    \
    } while (0)

// An operation on the model's communicator.  Should a call return
// ncclInProgress (a non-blocking communicator), settle() waits, under the
// RCCL deadline, until the communicator's state leaves ncclInProgress.
#define RCCL_OP(expr)                                                                      \
    do {                                                                                   \
        int rc_ = settle((expr), #expr);                                                   \
        if (rc_) return rc_;                                                               \
    } while (0)

const float kNaN = std::nanf("");

size_t round4(size_t n) { return (n + 3) & ~size_t(3); }

// In-process stand-in for the RCCL communicator (testing only): n slabs in
// one process, each driven by its own host thread, possibly all on one GPU.
// Halo exchanges become device-to-device copies between the members' buffers
// and the max all-reduce a host fold, each fenced by host barriers.  Every
// kernel and every row range the sharded path launches is unchanged, so a
// 1-GPU box can check the whole decomposition against the single-domain
// oracle (tests/test_gpu_sharded.py).
struct LocalHub {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    std::vector<cfd_model *> members;
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t my = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != my; });
        }
    }
};

// Fields that travel between slabs.
enum FieldId { FLD_U = 0, FLD_V, FLD_PP0, FLD_PP1, FLD_RHS };

}  // namespace

// One per device: the last persistent Jacobi launch of this process on it.
// Opt-in serialization (CFD_PERSIST_GATE=1): the r3 launch needed the whole
// GPU, two at once could each hold part of it and wait for the rest; the
// ticketed r4 launch (k_jacobi_persist) runs beside anything.
struct PersistGate {
    std::mutex mu;
    hipEvent_t ev = nullptr;
    hipStream_t last = nullptr;   // the stream of the device's last persistent launch
};
static PersistGate &persist_gate(int device) {
    static PersistGate gates[64];
    return gates[device & 63];
}

struct cfd_model {
    int device = 0;
    hipStream_t stream = nullptr;
    // sharded fixed-count solves: the boundary bands and their p' exchange run
    // on cstream while the interior runs on stream (SURVEY.md §8(e) overlap)
    hipStream_t cstream = nullptr;
    hipEvent_t ev_ov0 = nullptr, ev_ov1 = nullptr, ev_rhs = nullptr, ev_uv = nullptr;
    static constexpr bool overlap = true;
    cfd_grid grid{};
    cfd_params params{};
    Geom g{};
    Fields f{};
    // allocations
    float *u_all = nullptr, *v_all = nullptr, *uo_all = nullptr, *vo_all = nullptr;
    float *us_all = nullptr, *vs_all = nullptr;
    float *p = nullptr, *rhs = nullptr, *pp_all[2] = {nullptr, nullptr};
    uint8_t *mask_u = nullptr, *mask_v = nullptr;
    int32_t *obs = nullptr;
    Ctl *ctl = nullptr;
    uint32_t *slots = nullptr;   // spread residual maxima (cfd_internal.h kResSlots)
    float *vis_buf = nullptr;    // render output (nx*nyl words), allocated on first use
    uint32_t *h_nonfinite = nullptr;   // pinned host word the device sets (Fields::host_nonfinite)
    // sharded tolerance mode: per-sweep residuals copied to pinned host words,
    // each with its completion event (kLag ring, see enqueue_solve_host_driven)
    static constexpr int kResRing = 8;
    uint32_t *h_res = nullptr;
    hipEvent_t ev_res[kResRing] = {};
    double rccl_timeout_s = 300.0;      // CFD_RCCL_TIMEOUT_S
    std::vector<uint8_t> h_mask_u, h_mask_v;
    std::vector<uint8_t> dmask_u, dmask_v;   // staging for the async mask upload
    // sharding
    int n_ranks = 1, rank = 0;
    uint64_t j0 = 0, j1 = 0;
    ncclComm_t comm = nullptr;
    LocalHub *hub = nullptr;   // testing stand-in for comm
    int host_cur = 0;   // mirror of ctl->cur, valid when the tolerance is off
    // SOR: one fused launch per red-black iteration (k_sor_march) where it
    // applies; CFD_SOR_FUSED=0 keeps the two color passes in place
    bool sor_fused = [] {
        const char *e = getenv("CFD_SOR_FUSED");
        return !(e && atoi(e) == 0);
    }();
    // p' ghost rows deeper than 1 are stale (a host-driven tolerance solve or
    // cfd_profile_sweeps refreshed only one row per sweep): the next deep-halo
    // fixed-count solve re-exchanges hg rows before its first sweep
    bool pp_ghosts_shallow = false;
    int t_max = kMaxTemporal;   // sweeps per temporally blocked launch (CFD_TEMPORAL)
    // timing
    hipEvent_t ev_step0 = nullptr, ev_step1 = nullptr, ev_prof0 = nullptr, ev_prof1 = nullptr;
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> solve_events;
    // per-phase events (cfd_timing_phases): [0] predictors + first
    // divergence, [1] the corrector / finish, [2] the RCCL halo exchanges and
    // all-reduces (each on the stream it runs on, waiting for the peer
    // included), summed at cfd_timing_end
    bool timing_phases = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> phase_events[3];
    double phase_ms[3] = {0.0, 0.0, 0.0};
    uint64_t phase_count[3] = {0, 0, 0};
    hipEvent_t phase_mark(int ph, bool end, hipStream_t st = nullptr) {
        if (!(timing && timing_phases)) return nullptr;
        hipEvent_t e = take_event();
        (void)hipEventRecord(e, st ? st : stream);
        if (end) phase_events[ph].back().second = e;
        else phase_events[ph].emplace_back(e, nullptr);
        return e;
    }
    size_t ev_next = 0;
    uint64_t timed_sweeps = 0, timed_steps = 0, timed_launches = 0;
    double timed_step_ms = 0.0;
    bool stepped = false;
    // multigrid hierarchy (cfd_solvers.hip), built on the first multigrid solve
    std::vector<MgLevel> mg;     // level table; level 0's a/b are the p' buffers of the solve
    MgLevel *mg_dev = nullptr;   // device copy for k_mg_tail
    float *mg_pool = nullptr;
    int mg_tail = 0;             // first level handled inside the single-workgroup tail

    bool sharded() const { return n_ranks > 1; }
    size_t u_rows_alloc() const { return (size_t)g.nyl + 2 * kGhostUV; }
    size_t v_rows_alloc() const { return (size_t)g.nyl + 1 + 2 * kGhostUV; }

    hipEvent_t take_event() {
        if (ev_next == ev_pool.size()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            ev_pool.push_back(e);
        }
        return ev_pool[ev_next++];
    }

    // ---------------------------------------------------------------- halos
    float *field_ptr(int id) {
        switch (id) {
        case FLD_U: return f.u;
        case FLD_V: return f.v;
        case FLD_PP0: return f.pp[0];
        case FLD_PP1: return f.pp[1];
        default: return f.rhs;
        }
    }
    size_t field_pitch(int id) const { return id == FLD_U ? (size_t)g.nx + 1 : (size_t)g.nx; }

    // Ghost-row exchange of one field with both neighbours (geometry from
    // plan_halo): one RCCL group of at most two sends and two receives.
    uint64_t comm_calls = 0;   // halo groups + all-reduces enqueued (cfd_get_comm_calls)
    int exchange(int id, int kind, int depth, hipStream_t st = nullptr) {
        if (!sharded()) return 0;
        ++comm_calls;
        if (!st) st = stream;
        if (hub) return exchange_local(id, kind, depth, st);
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        phase_mark(2, false, st);
        RCCL_TRY(ncclGroupStart());
        int rc = exchange_ops(id, kind, depth, st);
        RCCL_OP(ncclGroupEnd());
        phase_mark(2, true, st);
        return rc;
    }

    // The sends and receives of one field's ghost exchange (inside a group).
    int exchange_ops(int id, int kind, int depth, hipStream_t st) {
        float *base = field_ptr(id);
        const size_t pitch = field_pitch(id);
        int h[6];
        plan_halo(kind, g.nyl, depth, rank, n_ranks, h);
        if (h[2] > 0) {
            RCCL_OP(ncclSend(base + (long)h[0] * (long)pitch, (size_t)h[2] * pitch, ncclFloat,
                              rank - 1, comm, st));
            RCCL_OP(ncclRecv(base + (long)h[1] * (long)pitch, (size_t)h[2] * pitch, ncclFloat,
                              rank - 1, comm, st));
        }
        if (h[5] > 0) {
            RCCL_OP(ncclSend(base + (long)h[3] * (long)pitch, (size_t)h[5] * pitch, ncclFloat,
                              rank + 1, comm, st));
            RCCL_OP(ncclRecv(base + (long)h[4] * (long)pitch, (size_t)h[5] * pitch, ncclFloat,
                              rank + 1, comm, st));
        }
        return 0;
    }

    // LocalHub form: copy the neighbours' send rows straight into our ghosts.
    int exchange_local(int id, int kind, int depth, hipStream_t st) {
        HIP_TRY(hipStreamSynchronize(st));
        hub->barrier();   // every member's rows are final
        float *base = field_ptr(id);
        const size_t pitch = field_pitch(id);
        int h[6];
        plan_halo(kind, g.nyl, depth, rank, n_ranks, h);
        for (int side = 0; side < 2; ++side) {
            const int rows = h[3 * side + 2];
            if (rows == 0) continue;
            cfd_model *peer = hub->members[side == 0 ? rank - 1 : rank + 1];
            int ph[6];
            plan_halo(kind, peer->g.nyl, depth, peer->rank, n_ranks, ph);
            const int psend = side == 0 ? ph[3] : ph[0];   // peer's rows facing us
            HIP_TRY(hipMemcpyAsync(base + (long)h[3 * side + 1] * (long)pitch,
                                   peer->field_ptr(id) + (long)psend * (long)pitch,
                                   (size_t)rows * pitch * 4, hipMemcpyDeviceToDevice, st));
        }
        HIP_TRY(hipStreamSynchronize(st));
        hub->barrier();   // nobody overwrites rows a peer is still copying
        return 0;
    }

    // u/v ghost rows before the predictors: both fields in
    // ONE RCCL group (one launch latency over xGMI instead of two).
    int exchange_uv(hipStream_t st = nullptr) {
        if (!sharded()) return 0;
        ++comm_calls;
        if (!st) st = stream;
        if (hub) {
            int rc = exchange_local(FLD_U, HALO_U, 2, st);
            if (rc) return rc;
            return exchange_local(FLD_V, HALO_V, 2, st);
        }
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        phase_mark(2, false, st);
        RCCL_TRY(ncclGroupStart());
        int rc = exchange_ops(FLD_U, HALO_U, 2, st);
        if (!rc) rc = exchange_ops(FLD_V, HALO_V, 2, st);
        RCCL_OP(ncclGroupEnd());
        phase_mark(2, true, st);
        return rc;
    }

    // p' halo: `rows` owned boundary rows of buffer `buf` each way.
    int exchange_pp(int buf, int rows, hipStream_t st = nullptr) {
        return exchange(buf ? FLD_PP1 : FLD_PP0, HALO_PP, rows, st);
    }

    // rhs ghosts `rhs_rows` deep and p' buffer `buf`'s `pp_rows` deep in ONE
    // RCCL group (one collective call: the speculative slab solve's first block)
    int exchange_rhs_pp(int rhs_rows, int buf, int pp_rows) {
        if (!sharded()) return 0;
        ++comm_calls;
        const int pid = buf ? FLD_PP1 : FLD_PP0;
        if (hub) {
            int rc = exchange_local(FLD_RHS, HALO_PP, rhs_rows, stream);
            if (rc) return rc;
            return exchange_local(pid, HALO_PP, pp_rows, stream);
        }
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        phase_mark(2, false, stream);
        RCCL_TRY(ncclGroupStart());
        int rc = exchange_ops(FLD_RHS, HALO_PP, rhs_rows, stream);
        if (!rc) rc = exchange_ops(pid, HALO_PP, pp_rows, stream);
        RCCL_OP(ncclGroupEnd());
        phase_mark(2, true, stream);
        return rc;
    }

    int allreduce_max_u32(uint32_t *dev, size_t n) {
        if (!sharded()) return 0;
        ++comm_calls;
        if (hub) {
            std::vector<uint32_t> acc(n, 0u), mine(n);
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();
            const size_t off = (size_t)(dev - (uint32_t *)f.ctl);   // same slot in every member
            for (cfd_model *peer : hub->members) {
                HIP_TRY(hipMemcpy(mine.data(), (uint32_t *)peer->f.ctl + off, n * 4,
                                  hipMemcpyDeviceToHost));
                for (size_t k = 0; k < n; ++k) acc[k] = std::max(acc[k], mine[k]);
            }
            hub->barrier();
            HIP_TRY(hipMemcpy(dev, acc.data(), n * 4, hipMemcpyHostToDevice));
            return 0;
        }
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        phase_mark(2, false);
        RCCL_OP(ncclAllReduce(dev, dev, n, ncclUint32, ncclMax, comm, stream));
        phase_mark(2, true);
        return 0;
    }

    // Resolve the result of a call on the (non-blocking) communicator: poll
    // its asynchronous state while it is ncclInProgress, up to the deadline.
    int settle(ncclResult_t r, const char *what) {
        if (r == ncclSuccess) return 0;
        if (r == ncclInProgress && comm) {
            const auto t0 = std::chrono::steady_clock::now();
            for (;;) {
                ncclResult_t st = ncclInProgress;
                r = ncclCommGetAsyncError(comm, &st);
                if (r == ncclSuccess) r = st;
                if (r != ncclInProgress) break;
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >
                    rccl_timeout_s) {
                    ncclCommAbort(comm);
                    comm = nullptr;
                    comm_aborted = true;
                    return fail(CFD_ERCCL, std::string(what) + ": still in progress after " +
                                               std::to_string((int)rccl_timeout_s) +
                                               " s; the communicator was aborted");
                }
                std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
            if (r == ncclSuccess) return 0;
        }
        return fail(CFD_ERCCL, std::string(what) + ": " + ncclGetErrorString(r));
    }

    // Wait for the stream (ev == nullptr) or for one event, with the RCCL
    // communicator watched: a peer that failed (ncclCommGetAsyncError) or made
    // no progress for CFD_RCCL_TIMEOUT_S seconds aborts the communicator and
    // fails with CFD_ERCCL instead of blocking forever.
    int wait_done(hipEvent_t ev) {
        if (!comm) {
            HIP_TRY(ev ? hipEventSynchronize(ev) : hipStreamSynchronize(stream));
            return 0;
        }
        // the deadline runs from the last forward progress the host saw (a
        // finished step: the device mirrors Ctl::step into h_nonfinite[1]),
        // not from the start of the wait, so a long healthy queue never trips it
        auto t0 = std::chrono::steady_clock::now();
        uint32_t seen = *(volatile uint32_t *)(h_nonfinite + 1);
        for (int spin = 0;; ++spin) {
            const hipError_t q = ev ? hipEventQuery(ev) : hipStreamQuery(stream);
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady)
                return fail(CFD_EHIP, std::string("stream/event query: ") + hipGetErrorString(q));
            const uint32_t now_step = *(volatile uint32_t *)(h_nonfinite + 1);
            if (now_step != seen) {
                seen = now_step;
                t0 = std::chrono::steady_clock::now();
            }
            ncclResult_t ar = ncclSuccess;
            const ncclResult_t r = ncclCommGetAsyncError(comm, &ar);
            const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            if (r != ncclSuccess || ar != ncclSuccess || el > rccl_timeout_s) {
                const std::string why = (r != ncclSuccess || ar != ncclSuccess)
                                            ? std::string("RCCL asynchronous error: ") +
                                                  ncclGetErrorString(r != ncclSuccess ? r : ar)
                                            : "RCCL exchange made no progress for " +
                                                  std::to_string((int)rccl_timeout_s) + " s";
                ncclCommAbort(comm);
                comm = nullptr;
                comm_aborted = true;
                return fail(CFD_ERCCL, why + " (rank " + std::to_string(rank) +
                                           "); the communicator was aborted");
            }
            if (spin < 256)
                std::this_thread::yield();
            else
                std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    bool comm_aborted = false;

    // -------------------------------------------------------------- solve
    // jacobi_pressure (model.rs:734-824).  Unsharded: one launch per sweep
    // over global rows 1..=ny-2, early exit decided on the device.  Sharded
    // (tolerance off): halo depth hg, p' exchanged every hg sweeps; between
    // exchanges each sweep also recomputes a shrinking band of ghost rows, so
    // results equal the single-domain sweep bit for bit.
    // ------------------------------------------- alternative solvers (index.html)
    static bool exact_pow2(double c) {
        int e;
        return c > 0.0 && std::isfinite(c) && std::frexp(c, &e) == 0.5 && std::isnormal(1.0 / c);
    }

    // The script's constants for spacing (dx, dy) (index.html:181-183, 1349).
    static void level_consts(double dx, double dy, double *dx2, double *dy2, double *denom,
                             double *r, int32_t *fast) {
        *dx2 = dx * dx;
        *dy2 = dy * dy;
        *denom = 2.0 / (dx * dx) + 2.0 / (dy * dy);
        r[0] = 1.0 / *dx2;
        r[1] = 1.0 / *dy2;
        r[2] = 1.0 / *denom;
        *fast = exact_pow2(*dx2) && exact_pow2(*dy2) && exact_pow2(*denom) ? 1 : 0;
        if (const char *e = getenv("CFD_FASTDIV"))
            if (atoi(e) == 0) *fast = 0;
    }

    void begin_solve_timing(int pass, hipEvent_t *e0) {
        *e0 = nullptr;
        if (timing && pass <= 0) {
            *e0 = take_event();
            (void)hipEventRecord(*e0, stream);
        }
    }
    void end_solve_timing(hipEvent_t e0, uint64_t sweeps, uint64_t launches) {
        if (!e0) return;
        hipEvent_t e1 = take_event();
        (void)hipEventRecord(e1, stream);
        solve_events.emplace_back(e0, e1);
        timed_sweeps += sweeps;
        timed_launches += launches;
    }

    SorConst sor_consts() const {
        SorConst k;
        double r[3];
        level_consts((double)g.dx, (double)g.dy, &k.dx2, &k.dy2, &k.denom, r, &k.fast);
        k.r_dx2 = r[0];
        k.r_dy2 = r[1];
        k.r_denom = r[2];
        return k;
    }

    // SOR on a slab (k_sor_march over the owned interior rows): each
    // iteration reads 2 p' ghost rows per side (the red rows just outside the
    // slab are recomputed from them) and 1 rhs ghost row, so the written
    // buffer's 2 boundary rows go to the neighbours after every iteration.
    // Fixed count: only the last iteration's residual is all-reduced.  With
    // the tolerance on (residual_out != null, the host-driven corrector loop)
    // every iteration's is, and the host checks them one iteration behind
    // the launches, as the sharded Jacobi does (model.rs:816 / index.html:772).
    int enqueue_sor_sharded(const SorConst &k, int pass, float *residual_out, hipEvent_t e0) {
        const int iters = params.jacobi_iters;
        const int lo = std::max(0, 1 - (int)j0), hi = std::min(g.nyl, (int)g.ny - 1 - (int)j0);
        if (iters < 1 || g.hg < 2 || !sor_fused_ok(g.nx, hi - lo))
            return fail(CFD_EINVAL, "sharded SOR needs >= 1 iteration, halo depth >= 2 and >= 16 "
                                    "interior rows per slab");
        const bool tol = g.tol_enabled != 0;
        float res_local = 0.f;
        if (tol && !residual_out) residual_out = &res_local;
        if (!tol) return enqueue_sor_sharded_deep(k, pass, e0);
        int rc = exchange(FLD_RHS, HALO_PP, 1);
        if (rc) return rc;
        int n = iters, checked = 0;
        bool done = false;
        auto converged = [&](int it, bool *yes) -> int {
            int rc2 = wait_done(ev_res[it % kResRing]);
            if (rc2) return rc2;
            float e;
            std::memcpy(&e, (const void *)&h_res[it % kResRing], 4);
            *yes = e < params.p_tol;
            return 0;
        };
        for (int it = 0; it < iters && !done; ++it) {
            const int res = tol || it == iters - 1;
            launch_sor_fused(f.pp[0], f.pp[1], f.rhs, g.nx, g.ny, k, f.ctl, f.err_slots, pass, it,
                             tol, g.p_tol, res, lo, hi, (int)j0, -g.hg, g.nyl + g.hg - 1, stream);
            if (res) {
                launch_fold_slots(f.ctl->err + it, f.err_slots + (size_t)it * kResSlots * kResStride,
                                  1, stream);
                rc = allreduce_max_u32(f.ctl->err + it, 1);
                if (rc) return rc;
            }
            rc = exchange_pp((host_cur + it + 1) & 1, 2);
            if (rc) return rc;
            if (!tol) continue;
            HIP_TRY(hipMemcpyAsync(&h_res[it % kResRing], f.ctl->err + it, 4, hipMemcpyDeviceToHost,
                                   stream));
            HIP_TRY(hipEventRecord(ev_res[it % kResRing], stream));
            while (checked <= it - 1 && !done) {
                bool yes = false;
                rc = converged(checked, &yes);
                if (rc) return rc;
                if (yes) {
                    n = checked + 1;
                    done = true;
                }
                ++checked;
            }
        }
        while (tol && !done && checked < iters) {
            bool yes = false;
            rc = converged(checked, &yes);
            if (rc) return rc;
            if (yes) {
                n = checked + 1;
                done = true;
            }
            ++checked;
        }
        end_solve_timing(e0, (uint64_t)n, (uint64_t)n);
        // with the tolerance on the finalize recounts n from the (identical)
        // all-reduced residuals and flips the buffer n times
        launch_finalize_solve(g, f, tol ? -1 : pass, iters, !tol && pass >= 1 ? 1 : 0, iters,
                              stream);
        HIP_TRY(hipGetLastError());
        host_cur = (host_cur + (tol ? n : iters)) & 1;
        pp_ghosts_shallow = true;
        if (tol) {
            float r = 0.f;
            HIP_TRY(hipMemcpyAsync(&r, &f.ctl->last_p, 4, hipMemcpyDeviceToHost, stream));
            rc = wait_done(nullptr);
            if (rc) return rc;
            *residual_out = r;
        }
        return 0;
    }

    // Fixed-count SOR on a slab with deep ghosts: an iteration's output rows
    // [a, b) read p' rows [a-2, b+2) and rhs rows [a-1, b+1), so after an
    // exchange of hg p' rows (and hg rhs rows once per solve) the next
    // K = hg/2 iterations can each recompute a band of ghost rows two rows
    // narrower than the one before, and p' crosses the link once every K
    // iterations instead of after every one.  Iteration 0 reads no p' (the
    // solve starts from 0).  Every ghost row is computed from the same values
    // as its owner computes it, so the result is bitwise the single domain's.
    int enqueue_sor_sharded_deep(const SorConst &k, int pass, hipEvent_t e0) {
        const int iters = params.jacobi_iters;
        const int glo = 1 - (int)j0, ghi = (int)g.ny - 1 - (int)j0;   // global rows 1..ny-2
        const int K = std::max(1, g.hg / 2);
        int rc = exchange(FLD_RHS, HALO_PP, g.hg);
        if (rc) return rc;
        for (int it = 0; it < iters; ++it) {
            const int d = it % K;
            const int a = std::max(glo, -g.hg + 2 * (d + 1));
            const int b = std::min(ghi, g.nyl + g.hg - 2 * (d + 1));
            const int res = it == iters - 1;
            launch_sor_fused(f.pp[0], f.pp[1], f.rhs, g.nx, g.ny, k, f.ctl, f.err_slots, pass, it,
                             0, g.p_tol, res, a, b, (int)j0, -g.hg, g.nyl + g.hg - 1, stream);
            if (res) {
                launch_fold_slots(f.ctl->err + it, f.err_slots + (size_t)it * kResSlots * kResStride,
                                  1, stream);
                rc = allreduce_max_u32(f.ctl->err + it, 1);
                if (rc) return rc;
            }
            if (d == K - 1 && it + 1 < iters) {
                rc = exchange_pp((host_cur + it + 1) & 1, g.hg);
                if (rc) return rc;
            }
        }
        // the corrector reads p' ghost rows -1 and nyl (the shared v faces):
        // a last iteration that recomputed no ghost row (d == K-1) is
        // followed by a full exchange; otherwise its recomputed band covers
        // both, and only the deeper ghosts are stale
        const bool last_bare = iters > 0 && (iters - 1) % K == K - 1;
        if (last_bare) {
            rc = exchange_pp((host_cur + iters) & 1, g.hg);
            if (rc) return rc;
        }
        end_solve_timing(e0, (uint64_t)iters, (uint64_t)iters);
        launch_finalize_solve(g, f, pass, iters, pass >= 1 ? 1 : 0, iters, stream);
        HIP_TRY(hipGetLastError());
        host_cur = (host_cur + iters) & 1;
        pp_ghosts_shallow = !last_bare;
        return 0;
    }

    // SOR (index.html:741-774) swept red-black: fused iterations ping-pong
    // (sor_fused), else two color passes in place on the current p'.
    int enqueue_sor(int pass) {
        const int iters = params.jacobi_iters;
        hipEvent_t e0;
        begin_solve_timing(pass, &e0);
        const SorConst k = sor_consts();
        if (sharded()) return enqueue_sor_sharded(k, pass, nullptr, e0);
        if (iters > 0 && sor_fused && sor_fused_ok(g.nx, g.ny - 2)) {
            // one launch per iteration, ping-pong from the device's current
            // buffer; the finalize flips it once per executed iteration
            for (int it = 0; it < iters; ++it)
                launch_sor_fused(f.pp[0], f.pp[1], f.rhs, g.nx, g.ny, k, f.ctl, f.err_slots, pass,
                                 it, g.tol_enabled, g.p_tol, g.tol_enabled || it == iters - 1, 1,
                                 g.ny - 1, 0, -g.hg, g.nyl + g.hg - 1, stream);
            end_solve_timing(e0, (uint64_t)iters, (uint64_t)iters);
            launch_finalize_solve(g, f, pass, iters, pass >= 1 ? 1 : 0, iters, stream);
            if (!g.tol_enabled) host_cur = (host_cur + iters) & 1;
            HIP_TRY(hipGetLastError());
            return 0;
        }
        float *pp = f.pp[host_cur];
        launch_fill_zero(pp, (size_t)g.nx * g.ny, f.ctl, pass, stream);
        for (int it = 0; it < iters; ++it) {
            const int res = g.tol_enabled || it == iters - 1;
            for (int color = 0; color < 2; ++color)
                launch_sor_color(pp, f.rhs, g.nx, g.ny, k, color, f.ctl, f.err_slots, pass, it,
                                 g.tol_enabled, g.p_tol, res, stream);
        }
        end_solve_timing(e0, (uint64_t)iters, 2 * (uint64_t)iters + 1);
        launch_finalize_solve(g, f, pass, iters, pass >= 1 ? 1 : 0, 0, stream, 1);
        HIP_TRY(hipGetLastError());
        return 0;
    }

    // Level table of mgVcycle's recursion: sizes floor((n+1)/2) down to the
    // first level with nx <= 4 or ny <= 4 (index.html:1444-1451), spacing
    // doubling per level (:1458).
    //
    // Sharded models partition the fine levels too (mg_P levels; see
    // enqueue_mg_partitioned): level l of rank r owns global rows
    // [J0 / 2^l, J1 / 2^l) of its slab [J0, J1) and stores kMgGhost ghost
    // rows each side.  A level is partitioned when every rank's boundary is
    // divisible by 2^(l+1) (the restriction maps owned rows onto owned rows),
    // every slab keeps >= 2 kMgGhost rows there, and the level lies above the
    // single-workgroup tail; the coarser levels are gathered whole to every
    // rank.  Every level pointer is biased to global row 0.
    static constexpr int kMgGhost = 8;   // >= 7: 5 sweeps + residual + the restriction's row
    int mg_P = 0;
    bool mg_part_env = [] {
        const char *e = getenv("CFD_MG_PARTITION");
        return !(e && atoi(e) == 0);
    }();
    // owned rows of level l for `rank` (partitioned levels)
    void mg_rows(int l, int r, int *j0o, int *j1o) const {
        uint64_t a, b;
        plan_slab(g.ny, n_ranks, r, &a, &b);
        *j0o = (int)(a >> l);
        *j1o = r == n_ranks - 1 ? mg[l].ny : (int)(b >> l);
    }
    int mg_partition_levels(const std::vector<std::pair<int, int>> &dims, int tail) const {
        if (!sharded() || !mg_part_env || !mg_smooth_wave_form()) return 0;
        if (const char *e = getenv("CFD_MG_TB"))
            if (atoi(e) == 0) return 0;
        int P = 0;
        for (int l = 0; l < tail && l + 1 < (int)dims.size(); ++l) {
            bool ok = true;
            for (int r = 0; r < n_ranks && ok; ++r) {
                uint64_t a, b;
                plan_slab(g.ny, n_ranks, r, &a, &b);
                const uint64_t m = 1ull << (l + 1);
                const int j0l = (int)(a >> l);
                const int j1l = r == n_ranks - 1 ? dims[l].second : (int)(b >> l);
                ok = a % m == 0 && j1l - j0l >= 2 * kMgGhost;
            }
            if (!ok) break;
            P = l + 1;
        }
        return P;
    }

    int mg_build() {
        if (!mg.empty()) return 0;
        std::vector<std::pair<int, int>> dims{{g.nx, g.ny}};
        while (!(dims.back().first <= 4 || dims.back().second <= 4)) {
            if ((int)dims.size() >= kMgMaxLevels) return fail(CFD_EINVAL, "multigrid: too many levels");
            dims.push_back({(dims.back().first + 1) / 2, (dims.back().second + 1) / 2});
        }
        const int nl = (int)dims.size();
        // levels of at most CFD_MG_TAIL cells (default 64 x 64) run inside k_mg_tail
        long thr = 4096;
        if (const char *e = getenv("CFD_MG_TAIL")) thr = atol(e);
        mg_tail = nl - 1;
        for (int l = 0; l < nl; ++l)
            if ((long)dims[l].first * dims[l].second <= thr) {
                mg_tail = l;
                break;
            }
        mg_P = mg_partition_levels(dims, mg_tail);
        mg.resize(nl);
        for (int l = 0; l < nl; ++l) {
            std::memset(&mg[l], 0, sizeof(MgLevel));
            mg[l].nx = dims[l].first;
            mg[l].ny = dims[l].second;
            mg[l].ys = 0;
            mg[l].ye = mg[l].ny;
            if (l < mg_P) {
                int a, b;
                mg_rows(l, rank, &a, &b);
                mg[l].ys = std::max(0, a - kMgGhost);
                mg[l].ye = std::min(mg[l].ny, b + kMgGhost);
            }
        }
        // level 0: the residual; a sharded model also keeps its own solution
        // buffers and rhs (the gathered whole grid when no level partitions:
        // every rank then solves the whole grid redundantly, see enqueue_mg)
        auto rows_of = [&](int l) { return (size_t)(mg[l].ye - mg[l].ys); };
        size_t total = (sharded() ? 4 : 1) * round4((size_t)g.nx * rows_of(0));
        for (int l = 1; l < nl; ++l) total += 4 * round4((size_t)dims[l].first * rows_of(l));
        HIP_TRY(hipMalloc((void **)&mg_pool, total * 4));
        HIP_TRY(hipMemsetAsync(mg_pool, 0, total * 4, stream));
        float *cur = mg_pool;
        for (int l = 0; l < nl; ++l) {
            MgLevel &L = mg[l];
            const size_t n = (size_t)L.nx * rows_of(l);
            const long bias = (long)L.ys * L.nx;   // pointers address global rows
            auto take = [&]() {
                float *p0 = cur - bias;
                cur += round4(n);
                return p0;
            };
            if (l == 0 && !sharded()) {
                L.rhs = f.rhs;
                L.r = take();
            } else {
                L.a = take();
                L.b = take();
                L.rhs = take();
                L.r = take();
            }
            const double scale = std::ldexp(1.0, l);   // 2*dx per recursion, exact
            double r[3];
            level_consts((double)g.dx * scale, (double)g.dy * scale, &L.dx2, &L.dy2, &L.denom, r,
                         &L.fast);
            L.r_dx2 = r[0];
            L.r_dy2 = r[1];
            L.r_denom = r[2];
            L.lo = L.ys;
            L.hi = L.ye;
        }
        HIP_TRY(hipMalloc((void **)&mg_dev, sizeof(MgLevel) * nl));
        HIP_TRY(hipMemcpy(mg_dev, mg.data(), sizeof(MgLevel) * nl, hipMemcpyHostToDevice));
        return 0;
    }

    // The multigrid branch (index.html:775-795): p' = 0, 3 V-cycles on the
    // current p' buffer, residual max |A p' - rhs| into the solve's slot set.
    // Sharded multigrid: the V-cycle's coarse levels shrink below one row per
    // slab, so every rank gathers the whole rhs (point-to-point all-gather),
    // solves the whole grid redundantly with the single-domain kernels — the
    // same arithmetic on the same data, so every rank holds the single-domain
    // result bit for bit — and keeps its slab's rows plus hg ghost rows of it.
    int gather_rhs() {
        float *full = mg[0].rhs;
        const size_t nx = (size_t)g.nx;
        if (hub) {
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();   // every member's rhs is final
            for (cfd_model *peer : hub->members)
                HIP_TRY(hipMemcpyAsync(full + (size_t)peer->j0 * nx, peer->f.rhs,
                                       (size_t)peer->g.nyl * nx * 4, hipMemcpyDeviceToDevice, stream));
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();   // nobody overwrites an rhs a peer is still copying
            return 0;
        }
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        HIP_TRY(hipMemcpyAsync(full + (size_t)j0 * nx, f.rhs, (size_t)g.nyl * nx * 4,
                               hipMemcpyDeviceToDevice, stream));
        RCCL_TRY(ncclGroupStart());
        for (int r = 0; r < n_ranks; ++r) {
            if (r == rank) continue;
            uint64_t a, b;
            plan_slab(g.ny, n_ranks, r, &a, &b);
            RCCL_OP(ncclSend(f.rhs, (size_t)g.nyl * nx, ncclFloat, r, comm, stream));
            RCCL_OP(ncclRecv(full + a * nx, (size_t)(b - a) * nx, ncclFloat, r, comm, stream));
        }
        RCCL_OP(ncclGroupEnd());
        return 0;
    }

    // ---- multigrid on slabs with partitioned fine levels (mg_P > 0) ----
    // Ghost rows of level arrays with both neighbours (which: 0 a, 1 b, 2 rhs):
    // rows [J0-d, J0) come from rank-1's owned rows, [J1, J1+d) from rank+1's,
    // every item in one RCCL group (LocalHub: device copies from the peers).
    struct MgX {
        int l, which, depth;
    };
    static float *mg_arr(const MgLevel &L, int which) {
        return which == 0 ? L.a : which == 1 ? L.b : L.rhs;
    }
    int mg_exchange(std::initializer_list<MgX> items) {
        if (hub) {
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();   // every member's rows are final
            for (const MgX &x : items) {
                const size_t nx = (size_t)mg[x.l].nx, d = (size_t)x.depth;
                int j0, j1;
                mg_rows(x.l, rank, &j0, &j1);
                float *mine = mg_arr(mg[x.l], x.which);
                if (rank > 0) {
                    const float *peer = mg_arr(hub->members[rank - 1]->mg[x.l], x.which);
                    HIP_TRY(hipMemcpyAsync(mine + (j0 - (long)d) * nx, peer + (j0 - (long)d) * nx,
                                           d * nx * 4, hipMemcpyDeviceToDevice, stream));
                }
                if (rank < n_ranks - 1) {
                    const float *peer = mg_arr(hub->members[rank + 1]->mg[x.l], x.which);
                    HIP_TRY(hipMemcpyAsync(mine + (long)j1 * nx, peer + (long)j1 * nx, d * nx * 4,
                                           hipMemcpyDeviceToDevice, stream));
                }
            }
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();   // nobody overwrites rows a peer is still copying
            return 0;
        }
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        RCCL_TRY(ncclGroupStart());
        for (const MgX &x : items) {
            const size_t nx = (size_t)mg[x.l].nx, n = (size_t)x.depth * nx;
            int j0, j1;
            mg_rows(x.l, rank, &j0, &j1);
            float *a = mg_arr(mg[x.l], x.which);
            if (rank > 0) {
                RCCL_OP(ncclSend(a + (long)j0 * nx, n, ncclFloat, rank - 1, comm, stream));
                RCCL_OP(ncclRecv(a + (long)(j0 - x.depth) * nx, n, ncclFloat, rank - 1, comm, stream));
            }
            if (rank < n_ranks - 1) {
                RCCL_OP(ncclSend(a + (long)(j1 - x.depth) * nx, n, ncclFloat, rank + 1, comm, stream));
                RCCL_OP(ncclRecv(a + (long)j1 * nx, n, ncclFloat, rank + 1, comm, stream));
            }
        }
        RCCL_OP(ncclGroupEnd());
        return 0;
    }
    // every rank's owned rows of the (whole, not partitioned) level l's rhs
    int mg_allgather_rhs(int l) {
        const size_t nx = (size_t)mg[l].nx;
        int j0, j1;
        mg_rows(l, rank, &j0, &j1);
        if (hub) {
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();
            for (int r = 0; r < n_ranks; ++r) {
                if (r == rank) continue;
                int a, b;
                mg_rows(l, r, &a, &b);
                HIP_TRY(hipMemcpyAsync(mg[l].rhs + (long)a * nx, hub->members[r]->mg[l].rhs + (long)a * nx,
                                       (size_t)(b - a) * nx * 4, hipMemcpyDeviceToDevice, stream));
            }
            HIP_TRY(hipStreamSynchronize(stream));
            hub->barrier();
            return 0;
        }
        if (!comm) return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
        RCCL_TRY(ncclGroupStart());
        for (int r = 0; r < n_ranks; ++r) {
            if (r == rank) continue;
            int a, b;
            mg_rows(l, r, &a, &b);
            RCCL_OP(ncclSend(mg[l].rhs + (long)j0 * nx, (size_t)(j1 - j0) * nx, ncclFloat, r, comm, stream));
            RCCL_OP(ncclRecv(mg[l].rhs + (long)a * nx, (size_t)(b - a) * nx, ncclFloat, r, comm, stream));
        }
        RCCL_OP(ncclGroupEnd());
        return 0;
    }

    // The V-cycles (index.html:1444-1470) with levels 0..P-1 partitioned:
    // down  each rank smooths (5 sweeps) and forms the residual over its rows
    //       plus the row below (the restriction reads it), restricts onto its
    //       coarse rows and exchanges that level's rhs ghosts; level P is
    //       gathered whole (all-gather of the restricted rhs rows);
    // coarse levels P..Lc run whole on every rank with the single-domain
    //       kernels and the tail (identical arithmetic on identical data);
    // up    each rank exchanges its pre-smoothed field's 5 ghost rows (and
    //       the coarse correction's 3), prolong-adds and smooths its rows.
    // Every level-l row is computed from the same values as in the
    // single-domain solve, so the result is bitwise the same; the whole grid
    // is touched only on the small gathered levels.
    int enqueue_mg_partitioned(int pass, float *residual_out, hipEvent_t e0) {
        const int lc = (int)mg.size() - 1, P = mg_P;
        int J0[kMgMaxLevels + 1], J1[kMgMaxLevels + 1];
        for (int l = 0; l <= P; ++l) mg_rows(l, rank, &J0[l], &J1[l]);
        auto lvl = [&](int l, int lo, int hi) {
            MgLevel L = mg[l];
            L.lo = lo;
            L.hi = hi;
            return L;
        };
        // (the allocation of a level array is rounded up to 4 floats)
        auto zero = [&](const MgLevel &L) {
            launch_fill_zero(L.a + (long)L.ys * L.nx, round4((size_t)(L.ye - L.ys) * L.nx), f.ctl, pass,
                             stream);
        };
        const size_t nx = (size_t)g.nx;
        int launches = 1;
        // level 0: the slab's rhs rows and their ghosts; p' = 0 (index.html:777)
        HIP_TRY(hipMemcpyAsync(mg[0].rhs + (long)J0[0] * nx, f.rhs, (size_t)g.nyl * nx * 4,
                               hipMemcpyDeviceToDevice, stream));
        zero(mg[0]);
        int rc = mg_exchange({{0, 2, kMgGhost}});
        if (rc) return rc;
        for (int cycle = 0; cycle < 3; ++cycle) {
            if (cycle > 0) {   // the last up-leg wrote level 0's rows only
                rc = mg_exchange({{0, 0, kMgGhost}});
                if (rc) return rc;
            }
            for (int l = 0; l < P; ++l) {
                const MgLevel L = lvl(l, std::max(0, J0[l] - 1), J1[l]);
                launch_mg_smooth5_residual(L, L.a, L.b, f.ctl, pass, stream);
                const MgLevel Cl = lvl(l + 1, J0[l + 1], J1[l + 1]);
                if (l + 1 < P) {
                    zero(Cl);
                    launch_mg_restrict(L, Cl, f.ctl, pass, stream);
                    rc = mg_exchange({{l + 1, 2, kMgGhost}});
                } else {
                    zero(Cl);
                    launch_mg_restrict(L, Cl, f.ctl, pass, stream);
                    rc = mg_allgather_rhs(P);
                }
                if (rc) return rc;
                launches += 3;
            }
            for (int l = P; l < mg_tail; ++l) {   // whole levels
                const MgLevel L = mg[l];
                launch_mg_smooth5_residual(L, L.a, L.b, f.ctl, pass, stream);
                launch_mg_restrict(L, mg[l + 1], f.ctl, pass, stream);
                launches += 2;
            }
            launch_mg_tail(mg_dev, mg_tail, lc, mg[mg_tail].a, mg[mg_tail].b, mg[0].fast, f.ctl, pass,
                           stream);
            ++launches;
            for (int l = mg_tail - 1; l >= P; --l) {
                const MgLevel L = mg[l], Cl = mg[l + 1];
                launch_mg_prolong_smooth5(Cl, l + 1 == lc ? Cl.b : Cl.a, L, L.b, L.a, f.ctl, pass, stream);
                ++launches;
            }
            for (int l = P - 1; l >= 0; --l) {
                if (l + 1 < P)
                    rc = mg_exchange({{l, 1, kSmT5}, {l + 1, 0, 3}});
                else
                    rc = mg_exchange({{l, 1, kSmT5}});
                if (rc) return rc;
                const MgLevel L = lvl(l, J0[l], J1[l]);
                const MgLevel Cl = l + 1 < P ? lvl(l + 1, J0[l + 1], J1[l + 1]) : mg[l + 1];
                launch_mg_prolong_smooth5(Cl, l + 1 == lc ? Cl.b : Cl.a, L, L.b, L.a, f.ctl, pass, stream);
                ++launches;
            }
        }
        // the slab's p' (and, by exchange, its deep ghosts), then the residual
        // max |A p' - rhs| over the slab's interior rows, all-reduced
        HIP_TRY(hipMemcpyAsync(f.pp[host_cur], mg[0].a + (long)J0[0] * nx, (size_t)g.nyl * nx * 4,
                               hipMemcpyDeviceToDevice, stream));
        rc = exchange_pp(host_cur, g.hg);
        if (rc) return rc;
        pp_ghosts_shallow = false;
        const MgLevel L0 = lvl(0, J0[0], J1[0]);
        launch_mg_final_residual(L0, f.pp[host_cur] - (long)J0[0] * nx, f.err_slots, f.ctl, pass, stream);
        launch_fold_slots(f.ctl->err, f.err_slots, 1, stream);
        rc = allreduce_max_u32(f.ctl->err, 1);
        if (rc) return rc;
        end_solve_timing(e0, 1, (uint64_t)launches + 1);
        launch_finalize_solve(g, f, pass, 1, pass >= 1 ? 1 : 0, 0, stream, 1);
        HIP_TRY(hipGetLastError());
        if (residual_out) {
            float r = 0.f;
            HIP_TRY(hipMemcpyAsync(&r, &f.ctl->last_p, 4, hipMemcpyDeviceToHost, stream));
            rc = wait_done(nullptr);
            if (rc) return rc;
            *residual_out = r;
        }
        return 0;
    }
    static constexpr int kSmT5 = 5;   // the smoothing window's halo (5 sweeps)

    int enqueue_mg(int pass, float *residual_out = nullptr) {
        int rc = mg_build();
        if (rc) return rc;
        hipEvent_t e0;
        begin_solve_timing(pass, &e0);
        if (sharded() && mg_P > 0) return enqueue_mg_partitioned(pass, residual_out, e0);
        if (sharded()) {
            rc = gather_rhs();
            if (rc) return rc;
        }
        const int lc = (int)mg.size() - 1;
        auto lvl = [&](int l) {
            MgLevel L = mg[l];
            if (l == 0 && !sharded()) {
                L.a = f.pp[host_cur];
                L.b = f.pp[host_cur ^ 1];
            }
            return L;
        };
        const MgLevel L0 = lvl(0);
        launch_fill_zero(L0.a, (size_t)g.nx * g.ny, f.ctl, pass, stream);
        // 5 smooths x -> y: one temporally blocked launch, or 5 single sweeps
        // ping-ponging x/y (CFD_MG_TB=0; the result lands in y either way)
        const char *tbe = getenv("CFD_MG_TB");
        const bool tb = !(tbe && atoi(tbe) == 0);
        int launches = 1;
        auto smooth5 = [&](const MgLevel &L, float *x, float *y) {
            if (tb) {
                launch_mg_smooth5(L, x, y, f.ctl, pass, stream);
                launches += 1;
            } else {
                for (int t = 0; t < 5; ++t)
                    launch_mg_smooth(L, t & 1 ? y : x, t & 1 ? x : y, f.ctl, pass, stream);
                launches += 5;
            }
        };
        for (int cycle = 0; cycle < 3; ++cycle) {
            for (int l = 0; l < mg_tail; ++l) {   // down: 5 smooths a->b, residual, restrict
                const MgLevel L = lvl(l);
                if (tb && mg_smooth_wave_form()) {
                    // the residual is formed by the smoothing launch itself
                    launch_mg_smooth5_residual(L, L.a, L.b, f.ctl, pass, stream);
                    launches += 1;
                } else {
                    smooth5(L, L.a, L.b);
                    launch_mg_residual(L, L.b, f.ctl, pass, stream);
                    launches += 1;
                }
                launch_mg_restrict(L, lvl(l + 1), f.ctl, pass, stream);
                launches += 1;
            }
            launch_mg_tail(mg_dev, mg_tail, lc, L0.a, L0.b, L0.fast, f.ctl, pass, stream);
            ++launches;
            for (int l = mg_tail - 1; l >= 0; --l) {   // up: prolong-add into b, 5 smooths b->a
                const MgLevel L = lvl(l), Cl = lvl(l + 1);
                const float *e = l + 1 == lc ? Cl.b : Cl.a;
                if (tb && mg_smooth_wave_form()) {
                    // the prolong-add happens as the smoothing loads its window
                    launch_mg_prolong_smooth5(Cl, e, L, L.b, L.a, f.ctl, pass, stream);
                    launches += 1;
                    continue;
                }
                launch_mg_prolong_add(Cl, e, L, L.b, f.ctl, pass, stream);
                smooth5(L, L.b, L.a);
                launches += 1;
            }
        }
        launch_mg_final_residual(L0, L0.a, f.err_slots, f.ctl, pass, stream);
        if (sharded()) {
            // the slab's rows and its hg ghost rows (inside the grid) of the
            // whole-grid solution: the deep ghosts are exact afterwards
            const int lo = std::max(-g.hg, -(int)j0), hi = std::min(g.nyl + g.hg, g.ny - (int)j0);
            HIP_TRY(hipMemcpyAsync(f.pp[host_cur] + (long)lo * g.nx, L0.a + ((long)j0 + lo) * g.nx,
                                   (size_t)(hi - lo) * g.nx * 4, hipMemcpyDeviceToDevice, stream));
            pp_ghosts_shallow = false;
        }
        end_solve_timing(e0, 1, (uint64_t)launches + 1);
        launch_finalize_solve(g, f, pass, 1, pass >= 1 ? 1 : 0, 0, stream, 1);
        HIP_TRY(hipGetLastError());
        if (residual_out) {
            float r = 0.f;
            HIP_TRY(hipMemcpyAsync(&r, &f.ctl->last_p, 4, hipMemcpyDeviceToHost, stream));
            rc = wait_done(nullptr);
            if (rc) return rc;
            *residual_out = r;
        }
        return 0;
    }

    // nblk >= 2 eight-sweep blocks on rows [lo, hi) in one persistent launch
    // (k_jacobi_persist); *done = false when it does not apply.  Persistent
    // launches of this process on one device never overlap (each needs every
    // workgroup resident): each waits for the device's previous one, whichever
    // model ran it.
    int launch_persist(int pass, int par0, int nblk, int lo, int hi, int res_it, bool *done) {
        *done = false;
        if (nblk < 2 || !persist_env || capturing || g.tb_kind != 5) return 0;
        if (persist_epoch + 1 >= (1u << (32 - kPersistBlockBits))) {
            // epochs wrap: clear the flags (stream-ordered) and restart
            HIP_TRY(hipMemsetAsync(f.persist, 0, kPersistWords * 4, stream));
            persist_epoch = 0;
        }
        PersistGate &gate = persist_gate(device);
        std::lock_guard<std::mutex> lk(gate.mu);
        // a stream orders its own launches; with CFD_PERSIST_GATE=1, after
        // another model's stream ran the device's last persistent launch, this
        // one waits for everything that stream has enqueued so far.  Off by
        // default since r4: the ticketed launch completes beside any other
        // kernel (k_jacobi_persist), so the gate is no longer needed for
        // correctness
        if (persist_gate_env && gate.last && gate.last != stream) {
            hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
            (void)hipStreamIsCapturing(gate.last, &cs);
            if (cs == hipStreamCaptureStatusNone) {
                if (!gate.ev) HIP_TRY(hipEventCreateWithFlags(&gate.ev, hipEventDisableTiming));
                HIP_TRY(hipEventRecord(gate.ev, gate.last));
                HIP_TRY(hipStreamWaitEvent(stream, gate.ev, 0));
            }
        }
        if (!launch_jacobi_persist(g, f, pass, par0, nblk, lo, hi, persist_epoch + 1, res_it, stream))
            return 0;
        last_abort_resident = false;
        gate.last = stream;
        ++persist_epoch;
        *done = true;
        return 0;
    }

    int enqueue_solve(int pass) {
        if (params.pressure_solver == CFD_SOLVER_SOR) return enqueue_sor(pass);
        if (params.pressure_solver == CFD_SOLVER_MULTIGRID) return enqueue_mg(pass);
        const int iters = params.jacobi_iters;
        const int lo_g = 1 - (int)j0, hi_g = (int)g.ny - 1 - (int)j0;   // global rows 1..ny-2
        bool evt = timing && pass <= 0;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (evt) {
            e0 = take_event();
            e1 = take_event();
            HIP_TRY(hipEventRecord(e0, stream));
        }
        const bool spec = spec_mode();
        const int tmax = g.tol_enabled ? 1 : t_max;
        int launches = 0;   // buffers flip once per launch
        bool resident = false;   // the resident launch also finalizes the solve
        if (!sharded()) {
            // (never under hipGraph capture: its workgroups must be resident
            // at once, and the device gate orders only eager launches)
            if (spec && resident_mode() && !capturing) {
                // the whole solve in one launch, the early exit decided on the
                // device; in-process resident / persistent launches of
                // different models on one device are ordered (all its
                // workgroups must be resident at once)
                PersistGate &gate = persist_gate(device);
                std::lock_guard<std::mutex> lk(gate.mu);
                if (gate.last && gate.last != stream) {
                    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
                    (void)hipStreamIsCapturing(gate.last, &cs);
                    if (cs == hipStreamCaptureStatusNone) {
                        if (!gate.ev) HIP_TRY(hipEventCreateWithFlags(&gate.ev, hipEventDisableTiming));
                        HIP_TRY(hipEventRecord(gate.ev, gate.last));
                        HIP_TRY(hipStreamWaitEvent(stream, gate.ev, 0));
                    }
                }
                resident = launch_jacobi_resident(g, f, pass, iters, 1, pass >= 1 ? 1 : 0, stream);
                if (resident) {
                    ++resident_solves;
                    last_abort_resident = true;
                    gate.last = stream;
                    // launches the per-launch path would count (host_cur is
                    // not tracked with the tolerance on; Ctl::spec_launches is)
                    for (int it = 0; it < iters;) {
                        int T, lo, hi, exch;
                        plan_block((int)j0, g.nyl, g.ny, 0, it, kMaxTemporal, iters, &T, &lo, &hi, &exch);
                        it += T;
                        ++launches;
                    }
                }
            }
            if (resident) {
            } else if (spec) {
                // the tolerance mode, temporally blocked (speculative): each
                // launch runs kSpecT sweeps with every sweep's residual, a check
                // finds the reference's early exit (model.rs:816), and the
                // converged launch is re-run with exactly its sweeps
                // the check (r6 default, spec_lag_first): each launch checks
                // the previous one and the re-run checks the last;
                // CFD_SPEC_LAG=0: a one-workgroup k_spec_check launch after
                // every launch
                const bool lag = spec_lag_env;
                int prev_T = 0, last_it = 0;
                for (int it = 0; it < iters;) {
                    int T, lo, hi, exch;
                    plan_block((int)j0, g.nyl, g.ny, 0, it, kMaxTemporal, iters, &T, &lo, &hi, &exch);
                    launch_jacobi_spec(g, f, pass, it, launches, T, lo, hi, stream, lag ? prev_T : 0);
                    if (!lag) launch_spec_check(g, f, pass, it, T, launches, stream);
                    prev_T = T;
                    last_it = it;
                    it += T;
                    ++launches;
                }
                if (iters > 0)
                    launch_jacobi_redo(g, f, pass, lo_g, hi_g, stream, last_it, launches - 1,
                                       lag ? prev_T : 0);
            } else if (tmax <= 1) {
                for (int it = 0; it < iters; ++it)
                    launch_jacobi_sweep(g, f, pass, it, lo_g, hi_g,
                                        g.tol_enabled || it == iters - 1, stream);
                launches = iters;
            } else {
                int it = 0;
                last_persist_blocks = 0;
                if (persist_env && persist_req > 0 && !capturing && tmax == 8 && g.tb_kind == 5) {
                    // the leading run of full 8-sweep blocks as one persistent
                    // launch, the solve's last block (which publishes the
                    // residual) included when it is a full block too
                    int nblk = 0, res_it = -1;
                    for (int k = 0; k < iters;) {
                        int T, lo, hi, exch;
                        plan_block((int)j0, g.nyl, g.ny, 0, k, tmax, iters, &T, &lo, &hi, &exch);
                        if (T != 8) break;
                        if (k + T >= iters) res_it = iters - 1;
                        k += T;
                        ++nblk;
                    }
                    bool done = false;
                    int rc = launch_persist(pass, launches, nblk, lo_g, hi_g, res_it, &done);
                    if (rc) return rc;
                    if (done) {
                        last_persist_blocks = nblk;
                        it = 8 * nblk;
                        launches = nblk;
                    }
                }
                for (; it < iters;) {
                    int T, lo, hi, exch;
                    plan_block((int)j0, g.nyl, g.ny, 0, it, tmax, iters, &T, &lo, &hi, &exch);
                    launch_jacobi_block(g, f, pass, it, launches, T, lo, hi, it + T == iters,
                                        stream);
                    it += T;
                    ++launches;
                }
            }
            if (evt) HIP_TRY(hipEventRecord(e1, stream));   // sweeps only
        } else if (g.tol_enabled && spec_slab_ok()) {
            const int n = enqueue_spec_slabs(pass, evt ? e1 : nullptr);
            if (n < 0) return n;
            if (evt) {
                solve_events.emplace_back(e0, e1);
                timed_sweeps += (uint64_t)iters;
                timed_launches += (uint64_t)n;
            }
            return 0;
        } else {
            // the deep-halo sweeps recompute ghost rows, which read rhs there.
            // Overlapped (r2): the rhs exchange runs on cstream while the first
            // launch's interior rows, whose T sweeps read no rhs ghost row
            // (the march for output rows [a, b) loads rhs rows [a-T, b+T)),
            // run on stream; the edge rows follow once the ghosts are in.
            last_persist_blocks = 0;
            const bool rhs_ovl = overlap && tmax > 1 && !pp_ghosts_shallow && iters > 0;
            bool rhs_pending = false;
            // whatever path leaves this block, stream waits for the rhs exchange
            // on cstream (so a sync of stream also covers that RCCL group)
            struct JoinRhs {
                cfd_model *m;
                bool *pending;
                ~JoinRhs() {
                    if (*pending) (void)hipStreamWaitEvent(m->stream, m->ev_rhs, 0);
                }
            } join_rhs{this, &rhs_pending};
            int rc0;
            if (rhs_ovl) {
                HIP_TRY(hipEventRecord(ev_ov0, stream));   // rhs written
                HIP_TRY(hipStreamWaitEvent(cstream, ev_ov0, 0));
                rc0 = exchange(FLD_RHS, HALO_PP, g.hg, cstream);
                if (rc0) return rc0;
                HIP_TRY(hipEventRecord(ev_rhs, cstream));
                rhs_pending = true;
            } else {
                rc0 = exchange(FLD_RHS, HALO_PP, g.hg);
                if (rc0) return rc0;
            }
            if (pp_ghosts_shallow) {   // sweep 0 reads p' ghosts hg rows deep
                rc0 = exchange_pp(host_cur, g.hg);
                if (rc0) return rc0;
                pp_ghosts_shallow = false;
            }
            for (int it = 0; it < iters;) {
                int T, lo, hi, exch;
                plan_block(g.j0, g.nyl, g.ny, g.hg, it, tmax, iters, &T, &lo, &hi, &exch);
                const int res = it + T == iters;
                if (rhs_pending) {
                    rhs_pending = false;
                    // the kernel's march loads rhs rows [a-T, b+T) (prefetch
                    // included), so no loaded row is an exchanged ghost row
                    const int a = std::max(lo, T), b = std::min(hi, g.nyl - T);
                    const bool split = a < b && !exch;
                    if (split) launch_jacobi_block(g, f, pass, it, launches, T, a, b, res, stream);
                    HIP_TRY(hipStreamWaitEvent(stream, ev_rhs, 0));
                    if (split) {
                        if (lo < a) launch_jacobi_block(g, f, pass, it, launches, T, lo, a, res, stream);
                        if (b < hi) launch_jacobi_block(g, f, pass, it, launches, T, b, hi, res, stream);
                        it += T;
                        ++launches;
                        continue;
                    }
                }
                // Overlap: the block before an exchange first
                // computes the hg-row bands the exchange sends, on cstream, which
                // then runs the exchange, while the interior rows run on stream.
                // Ghost rows need no compute here: the exchange replaces them.
                int ov[6];
                const bool ovl = overlap && exch && tmax > 1 &&
                                 plan_overlap(g.nyl, g.hg, rank, n_ranks, lo, hi, ov);
                if (ovl) {
                    HIP_TRY(hipEventRecord(ev_ov0, stream));
                    HIP_TRY(hipStreamWaitEvent(cstream, ev_ov0, 0));
                    for (int b = 0; b < 2; ++b)   // empty bands launch nothing
                        launch_jacobi_block(g, f, pass, it, launches, T, ov[2 * b], ov[2 * b + 1], res,
                                            cstream);
                    launch_jacobi_block(g, f, pass, it, launches, T, ov[4], ov[5], res, stream);
                    int rc = exchange_pp((host_cur + launches + 1) & 1, g.hg, cstream);
                    if (rc) return rc;
                    HIP_TRY(hipEventRecord(ev_ov1, cstream));
                    HIP_TRY(hipStreamWaitEvent(stream, ev_ov1, 0));
                } else if (tmax == 1) {
                    launch_jacobi_sweep(g, f, pass, it, lo, hi, res, stream);
                } else {
                    // a run of 8-sweep blocks between two exchanges as one
                    // persistent launch over the first block's rows: later
                    // blocks recompute ghost rows past their valid band too,
                    // which only feed ghost rows and are replaced by the next
                    // exchange (owned rows stay inside every block's band)
                    int nrun = 0;
                    if (T == 8 && tmax == 8 && !exch && !res && persist_sharded_env)
                        for (int k = it; k < iters;) {
                            int T2, lo2, hi2, ex2;
                            plan_block(g.j0, g.nyl, g.ny, g.hg, k, tmax, iters, &T2, &lo2, &hi2, &ex2);
                            if (T2 != 8 || ex2 || k + T2 == iters) break;
                            k += T2;
                            ++nrun;
                        }
                    bool done = false;
                    if (nrun >= 2) {
                        int rc = launch_persist(pass, launches, nrun, lo, hi, -1, &done);
                        if (rc) return rc;
                    }
                    if (done) {
                        it += 8 * nrun;
                        launches += nrun;
                        last_persist_blocks += nrun;
                        continue;
                    }
                    launch_jacobi_block(g, f, pass, it, launches, T, lo, hi, res, stream);
                }
                it += T;
                ++launches;
                if (exch && !ovl) {
                    int rc = exchange_pp((host_cur + launches) & 1, g.hg);
                    if (rc) return rc;
                }
            }
            const int last = iters > 0 ? iters - 1 : 0;
            if (!merge_res_allreduce) {
                launch_fold_slots(f.ctl->err + last,
                                  f.err_slots + (size_t)last * kResSlots * kResStride, 1, stream);
                int rc = allreduce_max_u32(f.ctl->err + last, 1);
                if (rc) return rc;
            }
            if (evt) HIP_TRY(hipEventRecord(e1, stream));   // sweeps + halo rounds
        }
        if (resident) {
            // k_jacobi_resident's last workgroup finalized the solve
        } else {
            launch_finalize_solve(g, f, pass, iters, pass >= 1 ? 1 : 0, launches, stream,
                                  spec ? 2 : 0);
        }
        HIP_TRY(hipGetLastError());
        if (evt) {
            solve_events.emplace_back(e0, e1);
            timed_sweeps += (uint64_t)iters;
            timed_launches += (uint64_t)launches;
        }
        host_cur = (host_cur + launches) & 1;
        return 0;
    }

    // Sharded with the tolerance on: the reference's early exit (model.rs:816)
    // needs the all-reduced residual of every sweep.  Sweep k's residual is
    // copied to a pinned host word behind its all-reduce; the host enqueues
    // sweep k+1 (kernel, residual fold, all-reduce, 1-row p' exchange) BEFORE
    // it waits for sweep k's word, so the GPU and the xGMI link never idle on
    // the host's decision (one-sweep-lagged convergence).  When sweep k has
    // converged, sweep k+1 is already queued: its kernel reads sweep k's
    // all-reduced residual on the device and returns without writing
    // (k_jacobi's early exit), so p' and the sweep count are the reference's;
    // only its all-reduce and exchange of an untouched buffer run in vain.
    int enqueue_solve_host_driven(float *residual_out) {
        if (params.pressure_solver == CFD_SOLVER_SOR) {
            hipEvent_t e0;
            begin_solve_timing(-1, &e0);
            return enqueue_sor_sharded(sor_consts(), -1, residual_out, e0);
        }
        if (params.pressure_solver == CFD_SOLVER_MULTIGRID) {
            float r = 0.f;
            return enqueue_mg(-1, residual_out ? residual_out : &r);
        }
        const int iters = params.jacobi_iters;
        const int lo = std::max(0, 1 - (int)j0), hi = std::min(g.nyl, (int)g.ny - 1 - (int)j0);
        constexpr int kLag = 1;
        static_assert(kLag < kResRing, "lag ring");
        int n = iters;   // sweeps the reference executes
        auto converged = [&](int k, bool *yes) -> int {
            int rc = wait_done(ev_res[k % kResRing]);
            if (rc) return rc;
            float e;
            std::memcpy(&e, (const void *)&h_res[k % kResRing], 4);
            *yes = e < params.p_tol;
            return 0;
        };
        int checked = 0;   // sweeps whose residual the host has read
        bool done = false;
        for (int it = 0; it < iters && !done; ++it) {
            launch_jacobi_sweep(g, f, -1, it, lo, hi, 1, stream);
            launch_fold_slots(f.ctl->err + it, f.err_slots + (size_t)it * kResSlots * kResStride, 1,
                              stream);
            int rc = allreduce_max_u32(f.ctl->err + it, 1);
            if (rc) return rc;
            rc = exchange_pp((host_cur + it + 1) & 1, 1);
            if (rc) return rc;
            HIP_TRY(hipMemcpyAsync(&h_res[it % kResRing], f.ctl->err + it, 4, hipMemcpyDeviceToHost,
                                   stream));
            HIP_TRY(hipEventRecord(ev_res[it % kResRing], stream));
            while (checked <= it - kLag && !done) {
                bool yes = false;
                rc = converged(checked, &yes);
                if (rc) return rc;
                if (yes) {
                    n = checked + 1;
                    done = true;
                }
                ++checked;
            }
        }
        while (!done && checked < iters) {
            bool yes = false;
            int rc = converged(checked, &yes);
            if (rc) return rc;
            if (yes) {
                n = checked + 1;
                done = true;
            }
            ++checked;
        }
        if (iters == 0) n = 0;
        // the device finalize recomputes n from the (identical) all-reduced slots
        launch_finalize_solve(g, f, -1, iters, 0, n, stream);
        HIP_TRY(hipGetLastError());
        host_cur = (host_cur + n) & 1;
        pp_ghosts_shallow = true;
        float res = 0.f;
        HIP_TRY(hipMemcpyAsync(&res, &f.ctl->last_p, 4, hipMemcpyDeviceToHost, stream));
        int rc = wait_done(nullptr);
        if (rc) return rc;
        if (residual_out) *residual_out = res;
        return 0;
    }

    bool host_driven() const { return sharded() && params.tol_enabled && !spec_slab_ok(); }
    // r5: the tolerance-mode Jacobi solve on slabs as speculative T-sweep
    // blocks (enqueue_solve): per block one T-row p' exchange, one speculative
    // launch publishing every sweep's residual, one all-reduce of the block's
    // T residuals and the device-side check -- instead of a launch, a fold,
    // an all-reduce, an exchange and a host read per sweep.  The default
    // since r6 (the host-side stop below): the default_grid() channel on 2
    // RCCL ranks (loopback) 102.3 -> 33.5 ms per step, 2,102 -> 569
    // collective calls (profiles/r6/prof_r6e/tolbench_*.log), bitwise;
    // CFD_SPEC_SLABS=0 keeps the host-driven per-sweep loop.
    bool spec_slab_env = [] {
        const char *e = getenv("CFD_SPEC_SLABS");
        return !(e && atoi(e) == 0);
    }();
    bool spec_slab_ok() const {
        // (k_spec_align moves float4s from pp + hg * nx: 16-B aligned rows)
        return sharded() && spec_env && spec_slab_env && params.pressure_solver == CFD_SOLVER_JACOBI &&
               g.hg >= 2 && g.nyl >= 2 * kMaxTemporal && ((size_t)g.nyl * g.nx) % 4 == 0 &&
               ((size_t)g.hg * g.nx) % 4 == 0;
    }
    // r6: the host's view of the speculative blocks.  After its all-reduce a
    // block's T residuals -- the same values on every rank -- are copied to
    // pinned host words; the host reads block 0 at once (from rest a solve
    // usually ends in its first sweeps) and every later block one block
    // behind, and enqueues no block (and, in enqueue_piso, no corrector pass)
    // past the one where the solve has ended.  Every rank reads the same
    // values, so every rank stops at the same block and the collective
    // sequences stay matched; the device's own check (k_spec_check, the
    // go flags) stays authoritative for the bits.  So a solve's collectives
    // track its convergence (r5 enqueued all blocks of all 20 passes:
    // 1,014 calls against the host-driven loop's 30, GPUTEST_r05).
    static constexpr int kSpecRing = 4;
    uint32_t *h_spec = nullptr;               // kSpecRing x kMaxTemporal pinned words
    hipEvent_t ev_spec[kSpecRing] = {};
    bool spec_converged = false;              // the last speculative slab solve ended early
    int enqueue_spec_slabs(int pass, hipEvent_t e1) {
        const int iters = params.jacobi_iters;
        const int Tm = std::min(kMaxTemporal, g.hg);
        const int lo = std::max(0, 1 - (int)j0), hi = std::min(g.nyl, (int)g.ny - 1 - (int)j0);
        const int nb = iters > 0 ? (iters + Tm - 1) / Tm : 0;
        int it = 0, launches = 0, checked = 0, rc = 0;
        int blk_T[kSpecRing] = {};
        bool stop = false;
        // reads block `checked`'s all-reduced residuals (waits for them)
        auto check_next = [&]() -> int {
            const int slot = checked % kSpecRing;
            int rc2 = wait_done(ev_spec[slot]);
            if (rc2) return rc2;
            for (int k = 0; k < blk_T[slot] && !stop; ++k) {
                float e;
                std::memcpy(&e, (const void *)&h_spec[slot * kMaxTemporal + k], 4);
                stop = e < params.p_tol;   // model.rs:816 (NaN: no exit)
            }
            ++checked;
            return 0;
        };
        for (int b = 0; b < nb && !stop; ++b) {
            const int T = iters / nb + (b < iters % nb ? 1 : 0);   // even split, no short tail
            // the block's source, T rows deep; every block reads rhs rows T
            // deep into the ghosts: the first block's exchange carries them
            rc = b == 0 ? exchange_rhs_pp(g.hg, (host_cur + launches) & 1, T)
                        : exchange_pp((host_cur + launches) & 1, T);
            if (rc) return rc;
            launch_jacobi_spec(g, f, pass, it, launches, T, lo, hi, stream);
            launch_fold_slots(f.ctl->err + it, f.err_slots + (size_t)it * kResSlots * kResStride, T,
                              stream);
            rc = allreduce_max_u32(f.ctl->err + it, (size_t)T);   // every rank decides alike
            if (rc) return rc;
            launch_spec_check(g, f, pass, it, T, launches, stream);
            const int slot = b % kSpecRing;
            HIP_TRY(hipMemcpyAsync(&h_spec[slot * kMaxTemporal], f.ctl->err + it, 4 * (size_t)T,
                                   hipMemcpyDeviceToHost, stream));
            HIP_TRY(hipEventRecord(ev_spec[slot], stream));
            blk_T[slot] = T;
            it += T;
            ++launches;
            while (!stop && checked <= (b == 0 ? 0 : b - 1)) {
                rc = check_next();
                if (rc) return rc;
            }
        }
        // the pass loop's break (pass >= 1 with a pass after it) needs the
        // solve's outcome: the last blocks too
        const bool need = pass >= 1 && pass < params.corrector_passes;
        while (need && !stop && checked < launches) {
            rc = check_next();
            if (rc) return rc;
        }
        spec_converged = stop;
        if (iters > 0) {
            launch_jacobi_redo(g, f, pass, lo, hi, stream);
            launch_spec_align(g, f, pass, launches, stream);
            // the corrector reads one p' ghost row of the result (the re-run
            // and the alignment wrote owned rows only)
            rc = exchange_pp((host_cur + launches) & 1, 1);
            if (rc) return rc;
        }
        if (e1) HIP_TRY(hipEventRecord(e1, stream));
        launch_finalize_solve(g, f, pass, iters, pass >= 1 ? 1 : 0, launches, stream, 3);
        HIP_TRY(hipGetLastError());
        host_cur = (host_cur + launches) & 1;
        pp_ghosts_shallow = true;   // the converged block's re-run: ghosts stale
        return launches;
    }

    // Persistent fixed-count solve (k_jacobi_persist); CFD_PERSIST=0 opts out
    // everywhere.  Each launch gets a new flag epoch from the host (flags start
    // at 0).  Single domain: opt-in (CFD_PERSIST=1) since r4 -- the per-launch
    // march with the guarded SUMS form is faster there (profiles/r4); slabs
    // keep the persistent runs between exchanges (CFD_PERSIST_SHARDED).
    int persist_req = [] {
        const char *e = getenv("CFD_PERSIST");
        return e ? atoi(e) : -1;
    }();
    bool persist_env = persist_req != 0;
    // (the solve's last, residual-publishing block runs inside the persistent
    // launch too)
    // slabs: the blocks between two p' exchanges as one persistent launch,
    // opt-in (CFD_PERSIST_SHARDED=1).  r5 same-geometry A/B (the rank slabs'
    // owned rows + 2 x 32 ghost rows, the 24 KiB pad they get; medians of 3,
    // profiles/r5/prof_r5b/slab_*.log): per launch 5.08 / 5.30 / 5.18 us per
    // sweep against persistent 5.42 / 5.72 / 5.44 on the 4096^2, 8192 x 2112
    // and 16384 x 1088 shapes, so every slab of the weak-scaling series runs
    // one launch per 8-sweep block between its exchanges
    bool persist_sharded_env = [] {
        const char *e = getenv("CFD_PERSIST_SHARDED");
        return e && atoi(e) != 0;
    }();
    // serialize persistent launches of different models on one device
    // (CFD_PERSIST_GATE=1; see launch_persist)
    bool persist_gate_env = [] {
        const char *e = getenv("CFD_PERSIST_GATE");
        return e && atoi(e) != 0;
    }();
    uint32_t persist_epoch = 0;
    int last_persist_blocks = 0;   // cfd_get_persist_blocks
    bool capturing = false;   // inside update_graph's capture: no persistent launch

    // Speculative temporal blocking for the tolerance mode (single domain,
    // Jacobi, kind-5 kernels at any field size); CFD_SPEC=0
    // keeps one launch per sweep with the per-sweep early exit.
    bool spec_env = [] {
        const char *e = getenv("CFD_SPEC");
        return !(e && atoi(e) == 0);
    }();
    // the lagged early-exit check (r5, spec_lag_first): the default since r6
    // -- C3 in the reference's control flow 10.81 -> 10.50 ms per step (best
    // of 3, medians 10.85 -> 10.53; profiles/r6/prof_r6d/ab_speclag.log);
    // CFD_SPEC_LAG=0 keeps a k_spec_check launch after every speculative launch
    bool spec_lag_env = [] {
        const char *e = getenv("CFD_SPEC_LAG");
        return !(e && atoi(e) == 0);
    }();
    bool spec_mode() const {
        return spec_env && !sharded() && g.tol_enabled &&
               params.pressure_solver == CFD_SOLVER_JACOBI;
    }
    // The tolerance-mode solve of a small grid as ONE resident launch
    // (k_jacobi_resident, cfd_jacobi_resident.hip): CFD_RESIDENT=1 on any
    // grid, 0 never; default on up to kResidentAutoCells cells, where the
    // per-launch row march is latency-bound.  Off after a timeout.
    static constexpr long kResidentAutoCells = 1l << 21;
    int resident_env = [] {
        const char *e = getenv("CFD_RESIDENT");
        return e ? atoi(e) : -1;
    }();
    bool resident_off = false;
    uint64_t resident_solves = 0;   // resident launches enqueued (cfd_get_resident_solves)
    bool resident_mode() const {
        if (resident_env == 0 || resident_off || !spec_mode()) return false;
        if (resident_env < 0 && (long)g.nx * g.ny > kResidentAutoCells) return false;
        int br, bc, nt, wg;
        if (!jacobi_resident_geometry(g, &br, &bc, &nt, &wg)) return false;
        // by default one tile per workgroup (C2's 1024^2 needs 2-3 per
        // workgroup and ran 3.65 -> 7.07 ms per step resident,
        // profiles/r4/ab_c2_r4j.log)
        return resident_env > 0 || nt <= wg;
    }

    // u* <- u, v* <- v and the divergence at the head of a corrector pass
    // (model.rs:698-704): one fused launch (CFD_COPY_DIV=0: the two launches)
    bool copy_div_env = [] {
        const char *e = getenv("CFD_COPY_DIV");
        return !(e && atoi(e) == 0);
    }();
    void pass_head(int pass, float dt_override) {
        if (copy_div_env) {
            launch_copy_star_div(g, f, pass, dt_override, stream);
        } else {
            launch_copy_star(g, f, pass, stream);
            launch_divergence(g, f, pass, dt_override, stream);
        }
    }

    // piso_step (model.rs:529-730).
    // finish = inside update() with no extra corrector passes: the corrector,
    // the boundaries and the step reductions run as one fused pass.
    int enqueue_piso(float dt_override, bool finish = false) {
        // K1-K3: the fused march when it applies, else predictors + divergence
        const bool march = predict_march_ok(g, f);
        const bool fused = march || predict_div_fused(g, f);
        phase_mark(0, false);
        if (march && finish && uv_async) {
            // rows [2, nyl-2) read u rows >= 0 and <= nyl-1 and v rows <= nyl;
            // the edge rows (4-row launches overlapping the interior ones:
            // identical values) follow the ghost exchange
            launch_predict_march(g, f, dt_override, stream, true, 2, g.nyl - 2);
            HIP_TRY(hipStreamWaitEvent(stream, ev_uv, 0));
            launch_predict_march(g, f, dt_override, stream, false, 0, 4);
            launch_predict_march(g, f, dt_override, stream, false, g.nyl - 4, g.nyl);
        } else if (march)
            launch_predict_march(g, f, dt_override, stream, finish && step_begin_folded);
        else if (fused)
            launch_predict_div(g, f, dt_override, stream);
        else
            launch_predict(g, f, dt_override, stream);
        auto first_divergence = [&](int pass) {
            if (!fused) launch_divergence(g, f, pass, dt_override, stream);
            phase_mark(0, true);
        };
        if (finish) {
            first_divergence(host_driven() ? -1 : 0);
            // a fixed-count step on slabs needs the solve's residual only for
            // reporting: it rides the step-end all-reduce (Ctl::red[5]) instead
            // of an all-reduce of its own
            merge_res_allreduce = sharded() && !host_driven();
            int rc = host_driven() ? enqueue_solve_host_driven(nullptr) : enqueue_solve(0);
            merge_res_allreduce = false;
            if (rc) return rc;
            phase_mark(1, false);
            launch_correct_finish(g, f, dt_override, stream);
            phase_mark(1, true);
            HIP_TRY(hipGetLastError());
            return 0;
        }
        if (!host_driven()) {
            first_divergence(0);
            int rc = enqueue_solve(0);
            if (rc) return rc;
            // single domain: each corrector that a further pass follows also
            // does that pass's head, as the device's go flag decides
            // (k_correct_head4; every pass, the last included, runs it: the
            // passes alternate the u* / v* arrays)
            const int passes = params.corrector_passes;
            const bool fuse = !sharded() && passes >= 1 && correct_head_ok(g, f);
            auto corrector = [&](int pass) {
                if (fuse)
                    launch_correct_head(g, f, pass, dt_override, pass < passes, stream);
                else
                    launch_corrector(g, f, pass, dt_override, stream);
            };
            corrector(0);
            const bool spec_slabs = sharded() && g.tol_enabled && spec_slab_ok();
            for (int pass = 1; pass <= passes; ++pass) {
                if (!fuse) pass_head(pass, dt_override);
                rc = enqueue_solve(pass);
                if (rc) return rc;
                corrector(pass);
                // slabs: the host knows where the loop ends (enqueue_spec_slabs)
                // and enqueues no pass the device would skip (model.rs:721-723)
                if (spec_slabs && spec_converged) break;
            }
        } else {
            first_divergence(-1);
            float res = 0.f;
            int rc = enqueue_solve_host_driven(&res);
            if (rc) return rc;
            launch_corrector(g, f, -1, dt_override, stream);
            for (int pass = 1; pass <= params.corrector_passes; ++pass) {
                pass_head(-1, dt_override);
                rc = enqueue_solve_host_driven(&res);
                if (rc) return rc;
                launch_corrector(g, f, -1, dt_override, stream);
                if (res < params.p_tol) break;
            }
        }
        launch_boundary(g, f, stream);
        HIP_TRY(hipGetLastError());
        return 0;
    }

    // Model::update (model.rs:304-379).
    // rec_step: record the step's GPU time for cfd_get_residuals (the last
    // step of a cfd_update_n batch only: every event record on the stream
    // costs the step a few microseconds of dispatch)
    bool step_begin_folded = false;   // this step's (enqueue_update)
    // fixed-count steps on slabs: the solve residual rides the step all-reduce
    bool merge_res_allreduce = false;
    bool uv_async = false;   // this step's u/v exchange runs on cstream (enqueue_update)
    int enqueue_update(bool rec_step = true) {
        if (rec_step) HIP_TRY(hipEventRecord(ev_step0, stream));
        const bool fused = params.corrector_passes == 0;
        // one launch less where the predictor march can carry the work: it
        // sets the inlet ramp (all k_step_begin does when nothing is copied)
        step_begin_folded = fused && predict_march_ok(g, f);
        if (!step_begin_folded) launch_step_begin(g, f, fused ? 0 : 1, stream);
        // slabs: the u/v ghost exchange runs on cstream while the predictor
        // march forms the rows that read no ghost (enqueue_piso)
        uv_async = sharded() && overlap && fused && step_begin_folded && g.nyl >= 8;
        int rc;
        if (uv_async) {
            HIP_TRY(hipEventRecord(ev_ov0, stream));   // u, v final (last step's finish)
            HIP_TRY(hipStreamWaitEvent(cstream, ev_ov0, 0));
            rc = exchange_uv(cstream);
            if (rc) return rc;
            HIP_TRY(hipEventRecord(ev_uv, cstream));
        } else {
            rc = exchange_uv();
        }
        if (rc) return rc;
        rc = enqueue_piso(kNaN, fused);
        if (rc) return rc;
        if (!fused) launch_step_reduce(g, f, stream);
        if (sharded()) launch_fold_slots(f.ctl->red, f.red_slots, 4, stream);
        // slabs with persistent runs: a rank whose persistent solve timed out
        // tells every rank through the step all-reduce (red[6])
        if (sharded() && persist_env && persist_sharded_env) launch_abort_to_red(f, stream);
        rc = allreduce_max_u32(f.ctl->red, 7);   // maxima, non-finite flag, solve residual, abort
        if (rc) return rc;
        launch_step_finalize(g, f, stream);
        HIP_TRY(hipGetLastError());
        if (rec_step) HIP_TRY(hipEventRecord(ev_step1, stream));
        if (timing) timed_steps++;
        if (rec_step) stepped = true;   // ev_step0 / ev_step1 hold a step
        return 0;
    }
    std::vector<hipEvent_t> step_events;

    // ------------------------------------------------------------ hipGraph
    // The launch sequence of a step is the same every step for an unsharded
    // Jacobi model: every data-dependent choice (buffers, early exits, pass
    // gating, dt) is read from Ctl on the device, so kernel arguments never
    // change.  cfd_update_n then captures graph_steps steps once and replays
    // the instantiated graph.  Dropped when the parameters
    // change; not used while solve timing is on (its events are per solve).
    // Opt-in (CFD_GRAPH=1): measured 1.2486 vs 1.2507 ms per step at 4096^2
    // (r2, tools/graph_ab.py) — the inter-kernel gaps are not launch overhead.
    hipGraphExec_t step_graph = nullptr;
    int graph_cur_delta = 0;   // host_cur advance of one replay
    int graph_steps = 4;
    bool graph_enabled = [] {
        const char *e = getenv("CFD_GRAPH");
        return e && atoi(e) != 0;
    }();
    bool graph_ok() const {
        return graph_enabled && !sharded() && !timing &&
               params.pressure_solver == CFD_SOLVER_JACOBI;
    }
    void drop_graph() {
        if (step_graph) (void)hipGraphExecDestroy(step_graph);
        step_graph = nullptr;
    }
    int update_graph(int n) {
        if (!step_graph) {
            const int hc0 = host_cur;
            HIP_TRY(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
            int rc = 0;
            capturing = true;
            for (int k = 0; k < graph_steps && !rc; ++k) rc = enqueue_update(false);
            capturing = false;
            hipGraph_t graph = nullptr;
            const hipError_t ce = hipStreamEndCapture(stream, &graph);
            if (rc || ce != hipSuccess) {
                if (graph) (void)hipGraphDestroy(graph);
                host_cur = hc0;
                return rc ? rc : fail(CFD_EHIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(ce));
            }
            const hipError_t ie = hipGraphInstantiate(&step_graph, graph, nullptr, nullptr, 0);
            (void)hipGraphDestroy(graph);
            if (ie != hipSuccess) {
                step_graph = nullptr;
                host_cur = hc0;
                return fail(CFD_EHIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(ie));
            }
            graph_cur_delta = (host_cur - hc0) & 1;
            host_cur = hc0;   // captured, not executed
        }
        int k = 0;
        for (; k + graph_steps <= n - 1; k += graph_steps) {   // the last step stays out: it
            HIP_TRY(hipGraphLaunch(step_graph, stream));       // records the step time
            host_cur = (host_cur + graph_cur_delta) & 1;
        }
        for (; k < n; ++k) {
            int rc = enqueue_update(k == n - 1);
            if (rc) return rc;
        }
        return 0;
    }

    // Slabs with persistent runs, entry points outside Model::update
    // (cfd_piso_step, cfd_pressure_solve): a rank whose persistent solve timed
    // out tells every rank through an all-reduce of the abort word, so every
    // rank recovers at its next synchronisation and replays the same calls
    // (inside a step the step all-reduce carries it, enqueue_update)
    int abort_allreduce() {
        if (!(sharded() && persist_env && persist_sharded_env)) return 0;
        launch_abort_to_red(f, stream);
        int rc = allreduce_max_u32(f.ctl->red + 6, 1);
        if (rc) return rc;
        launch_abort_from_red(f, stream);
        HIP_TRY(hipGetLastError());
        return 0;
    }

    int sync() {
        HIP_TRY(hipSetDevice(device));
        int rc = wait_done(nullptr);
        if (rc) return rc;
        rc = persist_timeout_check(true);
        if (rc) return rc;
        ck_commit();   // everything enqueued so far is final: no replay needed
        return 0;
    }
    // A persistent (k_jacobi_persist) or resident (k_jacobi_resident) solve
    // that gave up waiting left an invalid p' and every step after it
    // computed from it.  r5: the model recovers by itself -- it restores the
    // checkpoint it took before the first entry since its last
    // synchronisation (ck_begin) and re-runs those entries with one launch
    // per block -- and reports the fault once (CFD_ETIMEOUT; the state is
    // valid when it returns).  Solves run per launch from then on.
    // at_sync: the stream has drained (slabs detect only there, so every rank
    // re-runs the same entries)
    int persist_timeout_check(bool at_sync) {
        if (!h_nonfinite || !*(volatile uint32_t *)(h_nonfinite + 2)) return 0;
        if (!at_sync && sharded()) return 0;
        const char *which = last_abort_resident ? "resident tolerance-mode" : "persistent";
        HIP_TRY(hipStreamSynchronize(stream));
        if (cstream) HIP_TRY(hipStreamSynchronize(cstream));
        *(volatile uint32_t *)(h_nonfinite + 2) = 0u;
        persist_env = false;
        resident_off = true;
        if (ck_open) {
            const size_t n_entries = ck_replay.size();
            int rc = recover();
            if (rc) return rc;
            return fail(CFD_ETIMEOUT, std::string(which) + " Jacobi solve timed out waiting for a "
                                      "workgroup; recovered: the state was restored from the "
                                      "model's checkpoint and " + std::to_string(n_entries) +
                                      " call(s) re-run with one launch per block (the state is "
                                      "valid); per-launch solves from now on");
        }
        clear_abort_words();
        return fail(CFD_ETIMEOUT, std::string(which) + " Jacobi solve timed out waiting for a "
                                  "workgroup (no checkpoint was open); its result is invalid; "
                                  "per-launch solves from now on");
    }

    // ---- self-recovery checkpoint (r5) ---------------------------------
    // Taken (stream-ordered device copies) at the first cfd_update_n /
    // cfd_pressure_solve / cfd_piso_step after a synchronisation, when the
    // model may run a persistent or resident solve; the entries enqueued
    // since are kept as replays.  A synchronisation that finds no fault
    // commits (drops) them.
    struct CkSeg {
        void *ptr;
        size_t bytes;
    };
    std::vector<CkSeg> ck_segs;   // u, v, u_old, v_old, u*, v*, p, rhs, p' x2, Ctl
    char *ck_pool = nullptr;
    size_t ck_bytes = 0;
    bool ck_open = false;
    int ck_host_cur = 0;
    bool ck_shallow = false;
    std::vector<std::function<int()>> ck_replay;
    uint64_t recoveries = 0;   // cfd_get_recoveries
    bool last_abort_resident = false;
    bool ckpt_env = [] {   // CFD_CKPT=0: no checkpoint (a timeout then invalidates the state)
        const char *e = getenv("CFD_CKPT");
        return !(e && atoi(e) == 0);
    }();
    bool ckpt_needed() const {
        if (!ckpt_env || params.pressure_solver != CFD_SOLVER_JACOBI) return false;
        if (persist_env && (sharded() ? persist_sharded_env : persist_req > 0)) return true;
        return resident_mode();
    }
    int ck_begin() {
        if (ck_open || !ckpt_needed()) return 0;
        if (!ck_pool) {
            size_t tot = 0;
            for (const CkSeg &sg : ck_segs) tot += (sg.bytes + 255) & ~(size_t)255;
            HIP_TRY(hipMalloc((void **)&ck_pool, tot));
            ck_bytes = tot;
        }
        size_t off = 0;
        for (const CkSeg &sg : ck_segs) {
            HIP_TRY(hipMemcpyAsync(ck_pool + off, sg.ptr, sg.bytes, hipMemcpyDeviceToDevice, stream));
            off += (sg.bytes + 255) & ~(size_t)255;
        }
        ck_host_cur = host_cur;
        ck_shallow = pp_ghosts_shallow;
        ck_replay.clear();
        ck_open = true;
        return 0;
    }
    void ck_record(std::function<int()> fn) {
        if (ck_open) ck_replay.push_back(std::move(fn));
    }
    void ck_commit() {
        ck_open = false;
        ck_replay.clear();
    }
    // the abort word and the resident solve's barrier lines (its counters,
    // generations and exit ticket stay where an aborted launch left them)
    int clear_abort_words() {
        HIP_TRY(hipMemset(f.persist, 0, (size_t)kPersistHeadLines * kPersistFlagStride * 4));
        return 0;
    }
    int recover() {
        size_t off = 0;
        for (const CkSeg &sg : ck_segs) {
            HIP_TRY(hipMemcpy(sg.ptr, ck_pool + off, sg.bytes, hipMemcpyDeviceToDevice));
            off += (sg.bytes + 255) & ~(size_t)255;
        }
        // residual slot sets are zero between solves; an aborted solve may
        // have left some behind
        HIP_TRY(hipMemset(f.err_slots, 0, (size_t)kMaxSweeps * kResSlots * kResStride * 4));
        int rc = clear_abort_words();
        if (rc) return rc;
        *(volatile uint32_t *)h_nonfinite = 0u;
        host_cur = ck_host_cur;
        pp_ghosts_shallow = ck_shallow;
        ++recoveries;
        std::vector<std::function<int()>> replay;
        replay.swap(ck_replay);
        ck_open = false;
        const bool tm = timing;
        timing = false;   // the re-run is not a measurement
        for (auto &fn : replay) {
            rc = fn();
            if (rc) break;
        }
        timing = tm;
        if (rc) return rc;
        rc = wait_done(nullptr);
        if (rc) return rc;
        if (*(volatile uint32_t *)(h_nonfinite + 2))   // per-launch solves cannot time out
            return fail(CFD_ETIMEOUT, "the re-run after a solve timeout timed out");
        return 0;
    }

    int read_ctl(Ctl *out) {
        int rc = sync();
        if (rc) return rc;
        HIP_TRY(hipMemcpy(out, f.ctl, offsetof(Ctl, go), hipMemcpyDeviceToHost));
        return 0;
    }

    void destroy() {
        {   // the persistent-launch gate must not keep this model's stream
            PersistGate &gate = persist_gate(device);
            std::lock_guard<std::mutex> lk(gate.mu);
            if (gate.last == stream) gate.last = nullptr;
        }
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        if (comm) ncclCommDestroy(comm);
        comm = nullptr;
        for (hipEvent_t e : ev_res)
            if (e) (void)hipEventDestroy(e);
        if (h_res) (void)hipHostFree(h_res);
        for (hipEvent_t e : ev_spec)
            if (e) (void)hipEventDestroy(e);
        if (h_spec) (void)hipHostFree(h_spec);
        for (void *ptr : {(void *)u_all, (void *)v_all, (void *)uo_all, (void *)vo_all,
                          (void *)us_all, (void *)vs_all, (void *)p, (void *)rhs,
                          (void *)pp_all[0], (void *)pp_all[1], (void *)mask_u, (void *)mask_v,
                          (void *)obs, (void *)ctl, (void *)slots, (void *)vis_buf,
                          (void *)mg_pool, (void *)mg_dev})
            if (ptr) (void)hipFree(ptr);
        if (h_nonfinite) (void)hipHostFree(h_nonfinite);
        if (ck_pool) (void)hipFree(ck_pool);
        drop_graph();
        for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
        if (ev_step0) (void)hipEventDestroy(ev_step0);
        if (ev_step1) (void)hipEventDestroy(ev_step1);
        if (ev_prof0) (void)hipEventDestroy(ev_prof0);
        if (ev_prof1) (void)hipEventDestroy(ev_prof1);
        if (stream) (void)hipStreamDestroy(stream);
        if (cstream) (void)hipStreamDestroy(cstream);
        if (ev_ov0) (void)hipEventDestroy(ev_ov0);
        if (ev_ov1) (void)hipEventDestroy(ev_ov1);
        if (ev_rhs) (void)hipEventDestroy(ev_rhs);
        if (ev_uv) (void)hipEventDestroy(ev_uv);
    }
};

namespace {

int validate(const cfd_grid *grid, const cfd_params *p) {
    if (!grid || !p) return fail(CFD_EINVAL, "null grid or params");
    if (grid->nx < 16 || grid->nx % 8 != 0)
        return fail(CFD_EINVAL, "nx must be a multiple of 8 and >= 16 (model.rs:541 precondition)");
    if (grid->ny < 4) return fail(CFD_EINVAL, "ny must be >= 4");
    if ((grid->nx + 1) * grid->ny > (1ull << 31))
        return fail(CFD_EINVAL, "grid too large for 32-bit row indexing");
    if (!(grid->lx > 0.f) || !(grid->ly > 0.f)) return fail(CFD_EINVAL, "lx, ly must be > 0");
    if (p->jacobi_iters < 0 || p->jacobi_iters > kMaxSweeps)
        return fail(CFD_EINVAL, "jacobi_iters out of range [0, 4096]");
    if (p->corrector_passes < 0 || p->corrector_passes > kMaxPasses - 1)
        return fail(CFD_EINVAL, "corrector_passes out of range [0, 63]");
    if (p->velocity_scheme != 0 && p->velocity_scheme != 1)
        return fail(CFD_EINVAL, "velocity_scheme must be 0 or 1");
    if (p->inlet_profile != 0 && p->inlet_profile != 1)
        return fail(CFD_EINVAL, "inlet_profile must be 0 or 1");
    if (p->pressure_solver < CFD_SOLVER_JACOBI || p->pressure_solver > CFD_SOLVER_MULTIGRID)
        return fail(CFD_EINVAL, "pressure_solver must be 0 (Jacobi), 1 (SOR) or 2 (multigrid)");
    if (p->bc_kind != 0 && p->bc_kind != 1) return fail(CFD_EINVAL, "bc_kind must be 0 or 1");
    return 0;
}

// Sharded SOR (enqueue_sor_sharded) needs >= 1 iteration, halo depth >= 2
// and >= 16 interior rows in the slab.  Checked wherever the solver can be
// chosen (create, cfd_set_params, cfd_run_set_params), so a step never fails
// half-way through with u*, v* and rhs already written.
int validate_sharded(const cfd_model *m, const cfd_params *p) {
    if (m->n_ranks <= 1 || p->pressure_solver != CFD_SOLVER_SOR) return 0;
    const int lo = std::max(0, 1 - (int)m->j0);
    const int hi = std::min((int)(m->j1 - m->j0), (int)m->grid.ny - 1 - (int)m->j0);
    if (p->jacobi_iters < 1 || m->g.hg < 2 || !sor_fused_ok((int)m->grid.nx, hi - lo))
        return fail(CFD_EINVAL, "sharded SOR needs >= 1 iteration, halo depth >= 2 and >= 16 "
                                "interior rows per slab (rank " + std::to_string(m->rank) + " has " +
                                    std::to_string(hi - lo) + ", halo depth " +
                                    std::to_string(m->g.hg) + ")");
    return 0;
}

void apply_params(cfd_model *m, const cfd_params *p) {
    m->params = *p;
    m->g.nu = p->viscosity;
    m->g.target_inlet = p->target_inlet_velocity;
    m->g.scheme = p->velocity_scheme;
    m->g.profile = p->inlet_profile;
    m->g.bc_kind = p->bc_kind;
    m->g.tol_enabled = p->tol_enabled ? 1 : 0;
    m->g.p_tol = p->p_tol;
    m->g.jacobi_iters = p->jacobi_iters;
}

// Pick the cheapest division form that is bit-identical to IEEE `/` for ALL
// 2^32 f32 inputs, for each of the three Jacobi divisors, by exhaustive
// check on the device (a few ms; cached per divisor value).  x * RN(1/c) is
// exact e.g. for the power-of-two divisors of the 2^k cavity grids; the
// FMA-corrected form covers most other divisors; anything else keeps IEEE
// division.  CFD_FASTDIV=0 forces IEEE, CFD_FASTDIV=2 prefers the FMA-corrected form.
std::mutex g_div_mu;
std::vector<std::pair<uint32_t, int>> g_div_cache;   // divisor bits -> ok mask (bit0 m1, bit1 m2)

int division_ok_mask(hipStream_t s, float c, float r, int *mask) {
    uint32_t bits;
    std::memcpy(&bits, &c, 4);
    {
        std::lock_guard<std::mutex> lk(g_div_mu);
        for (auto &e : g_div_cache)
            if (e.first == bits) {
                *mask = e.second;
                return 0;
            }
    }
    unsigned long long *d = nullptr, h[3] = {0, 0, 0};
    HIP_TRY(hipMalloc((void **)&d, 24));
    HIP_TRY(hipMemsetAsync(d, 0, 24, s));
    launch_verify_division(c, r, d, s);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(h, d, 24, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipFree(d));
    *mask = (h[0] == 0 ? 1 : 0) | (h[1] == 0 ? 2 : 0) | (h[2] == 0 ? 4 : 0);
    std::lock_guard<std::mutex> lk(g_div_mu);
    g_div_cache.emplace_back(bits, *mask);
    return 0;
}

int choose_division(hipStream_t s, Geom &g) {
    g.fastdiv = 0;
    g.res_div = 0;
    const char *env = getenv("CFD_FASTDIV");
    if (env && atoi(env) == 0) return 0;
    int m1, m2, m3;
    int rc;
    if ((rc = division_ok_mask(s, g.dx_sq, g.r_dx_sq, &m1)) ||
        (rc = division_ok_mask(s, g.dy_sq, g.r_dy_sq, &m2)) ||
        (rc = division_ok_mask(s, g.denom, g.r_denom, &m3)))
        return rc;
    const int all = m1 & m2 & m3;
    g.fastdiv = (all & 1) ? 1 : (all & 2) ? 2 : 0;
    if (env && atoi(env) == 2 && (all & 2)) g.fastdiv = 2;   // test hook: prefer mode 2
    // the resident solve also has the guarded FMA form (3), opt-in
    // (CFD_RESIDENT_DIV=3): its per-division branch measured slower than
    // IEEE division on the reference default (3.87 vs 3.57 ms per step,
    // profiles/r4/ab_refdef_r4t.log)
    const char *rd = getenv("CFD_RESIDENT_DIV");
    g.res_div = g.fastdiv != 0 ? g.fastdiv : (rd && atoi(rd) == 3 && (all & 4)) ? 3 : 0;
    return 0;
}

// Model::new (model.rs:219-299), restricted to rows [j0, j1) of the slab.
int build_model(cfd_model *m, const cfd_grid *grid, const cfd_params *p, int device, int hg) {
    m->device = device;
    m->grid = *grid;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&m->cstream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&m->ev_ov0, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&m->ev_ov1, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&m->ev_rhs, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&m->ev_uv, hipEventDisableTiming));
    HIP_TRY(hipEventCreate(&m->ev_step0));
    HIP_TRY(hipEventCreate(&m->ev_step1));
    HIP_TRY(hipEventCreate(&m->ev_prof0));
    HIP_TRY(hipEventCreate(&m->ev_prof1));
    const int nx = (int)grid->nx, ny = (int)grid->ny;
    Geom &g = m->g;
    g.nx = nx;
    g.ny = ny;
    g.j0 = (int)m->j0;
    g.nyl = (int)(m->j1 - m->j0);
    g.hg = hg;
    // the kernels address a field slab with 32-bit byte offsets
    if ((uint64_t)(g.nyl + 2 * hg + 2 * kGhostUV + 1) * (uint64_t)(nx + 1) * 4u >= (1ull << 31))
        return fail(CFD_EINVAL, "slab too large for 32-bit buffer offsets (2 GiB per field)");
    g.dx = grid->lx / (float)grid->nx;   // src/app.rs:37
    g.dy = grid->ly / (float)grid->ny;   // src/app.rs:38
    g.ly = grid->ly;
    apply_params(m, p);
    // Jacobi divisors exactly as jacobi_pressure forms them (model.rs:740-746)
    g.dx_sq = g.dx * g.dx;
    g.dy_sq = g.dy * g.dy;
    g.denom = 2.0f / (g.dx * g.dx) + 2.0f / (g.dy * g.dy);
    g.r_dx_sq = 1.0f / g.dx_sq;
    g.r_dy_sq = 1.0f / g.dy_sq;
    g.r_denom = 1.0f / g.denom;
    {
        // spacings that are exact powers of two: division == reciprocal multiply
        auto pow2f = [](float c) {
            int e;
            return c > 0.0f && std::isfinite(c) && std::frexp(c, &e) == 0.5f &&
                   std::isnormal(1.0f / c);
        };
        g.r_dx = 1.0f / g.dx;
        g.r_dy = 1.0f / g.dy;
        g.r_dxx = 1.0f / (g.dx * g.dx);
        g.r_dyy = 1.0f / (g.dy * g.dy);
        g.sp_pow2 = pow2f(g.dx) && pow2f(g.dy) && pow2f(g.dx * g.dx) && pow2f(g.dy * g.dy) ? 1 : 0;
        if (const char *e = getenv("CFD_FASTDIV"))
            if (atoi(e) == 0) g.sp_pow2 = 0;
    }
    {
        int rc0 = choose_division(m->stream, g);
        if (rc0) return rc0;
    }
    // kind 4 (prefetch-pipelined march, 2 columns per lane) at T = 4 is the
    // fastest measured geometry on the bench workload (tools/tune_tb.py, r1:
    // 8.45 us/sweep vs 11.05 for kind 1 and 11.3 for kind 3 at its best T)
    // Default Jacobi march (measured at 4096^2 on developed fields, r2:
    // profiles/r2/tune_r2b_kind5.log, ab_lds_*.log): with the proven-exact
    // reciprocal multiply, kind 5 (rhs window in LDS, DPP-folded sums) at
    // T = 8 sweeps per launch, one round of balanced segments, progress-ordered
    // issue priority and lighter boundary-row segments, 5.1-5.4 us per sweep
    // (box to box), against 7.75 for kind 4 at T = 8 and 9.04 at T = 4; under IEEE (or FMA-corrected)
    // division the march is VALU-bound and kind 4 at T = 4 stays (r1: 6144^2
    // 7.3e11 vs 6.1e11 cell-updates/s at T = 8).  Single domain and slabs alike.
    g.tb_kind = g.fastdiv == 1 ? 5 : 4;
    g.pred_div = 2;
    if (const char *e = getenv("CFD_PRED_DIV")) g.pred_div = std::min(std::max(atoi(e), 0), 2);
    if (const char *kv = getenv("CFD_TB_KIND")) {
        const int k = atoi(kv);
        g.tb_kind = (k == 3 || k == 4 || k == 5) ? k : 1;
    }
    // the pipelined kernels (kinds 3/4) park masked lanes at a far voffset
    // that must not wrap past 2^32 when the row offset is added: slabs up to
    // 1 GiB per field (kind 5 bases its descriptors at each wave's rows)
    if (g.tb_kind != 5 && (uint64_t)(g.nyl + 2 * g.hg) * (uint64_t)nx * 4u > (1ull << 30))
        g.tb_kind = 1;
    m->t_max = g.tb_kind == 3 ? 6 : 4;
    {
        // kind 4 past the 256 MB Infinity Cache: 8 sweeps per launch halve the
        // HBM traffic (8192^2: 2.33e12 vs 1.38e12 cell-updates/s, r1)
        const uint64_t jac_ws = 3ull * (uint64_t)(g.nyl + 2 * g.hg) * (uint64_t)nx * 4u;
        if (g.tb_kind == 4 && g.fastdiv == 1 && m->n_ranks == 1 && jac_ws > (256ull << 20))
            m->t_max = 8;
        if (g.tb_kind == 5) m->t_max = 8;
    }
    if (const char *tv = getenv("CFD_TEMPORAL")) m->t_max = std::max(1, atoi(tv));
    m->t_max = std::min(m->t_max, g.tb_kind == 1 ? 4 : kMaxTemporal);
    // output rows per wave segment: 24 for kind 4 (12-slot unrolled march);
    // kind 5 sizes its segments to one round of resident waves (tb_rows 0,
    // cfd_jacobi_lds.hip lds_segments; 4096^2: ~38 rows, fixed 40 rows gave
    // 6.42 us/sweep, 32 gave 6.50, 24 gave 6.68)
    g.tb_rows = g.tb_kind == 5 ? 0 : 24;
    if (const char *rv = getenv("CFD_TB_ROWS")) g.tb_rows = std::max(4, std::min(1024, atoi(rv)));
    g.tb_bpc = 3;
    if (const char *bv = getenv("CFD_TB_BPC")) {   // balanced segmentation instead
        g.tb_bpc = std::max(1, std::min(16, atoi(bv)));
        g.tb_rows = 0;
    }
    g.xcd_remap = 1;
    if (const char *xv = getenv("CFD_XCD_REMAP")) g.xcd_remap = atoi(xv) ? 1 : 0;
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess ||
            ncu <= 0)
            ncu = 256;
        g.n_cu = ncu;
    }


    const size_t W = (size_t)nx + 1, nyl = (size_t)g.nyl;
    const size_t u_alloc = round4(m->u_rows_alloc() * W);
    const size_t v_alloc = round4(m->v_rows_alloc() * (size_t)nx);
    const size_t p_n = nyl * nx;
    const size_t pp_n = (nyl + 2 * (size_t)hg) * nx;
    auto zalloc = [&](void **ptr, size_t bytes) -> int {
        HIP_TRY(hipMalloc(ptr, bytes));
        HIP_TRY(hipMemsetAsync(*ptr, 0, bytes, m->stream));
        return 0;
    };
    int rc = 0;
    if ((rc = zalloc((void **)&m->u_all, u_alloc * 4)) || (rc = zalloc((void **)&m->v_all, v_alloc * 4)) ||
        (rc = zalloc((void **)&m->uo_all, u_alloc * 4)) || (rc = zalloc((void **)&m->vo_all, v_alloc * 4)) ||
        (rc = zalloc((void **)&m->us_all, u_alloc * 4)) || (rc = zalloc((void **)&m->vs_all, v_alloc * 4)) ||
        (rc = zalloc((void **)&m->p, p_n * 4)) || (rc = zalloc((void **)&m->rhs, pp_n * 4)) ||
        (rc = zalloc((void **)&m->pp_all[0], pp_n * 4)) || (rc = zalloc((void **)&m->pp_all[1], pp_n * 4)) ||
        (rc = zalloc((void **)&m->mask_u, nyl * W + 16)) || (rc = zalloc((void **)&m->mask_v, (nyl + 1) * nx + 16)) ||
        (rc = zalloc((void **)&m->ctl, sizeof(Ctl))) ||
        (rc = zalloc((void **)&m->slots, kSlotWords * 4)))
        return rc;
    // the self-recovery checkpoint's segments (cfd_model::ck_begin)
    m->ck_segs = {{m->u_all, u_alloc * 4}, {m->v_all, v_alloc * 4}, {m->uo_all, u_alloc * 4},
                  {m->vo_all, v_alloc * 4}, {m->us_all, u_alloc * 4}, {m->vs_all, v_alloc * 4},
                  {m->p, p_n * 4},         {m->rhs, pp_n * 4},        {m->pp_all[0], pp_n * 4},
                  {m->pp_all[1], pp_n * 4}, {m->ctl, sizeof(Ctl)}};
    // word 0: first non-finite step; word 1: last finished step (watchdog)
    // [0] non-finite step, [1] progress (sharded), [2] persistent-solve timeout
    HIP_TRY(hipHostMalloc((void **)&m->h_nonfinite, 16, hipHostMallocMapped | hipHostMallocCoherent));
    *(volatile uint32_t *)m->h_nonfinite = 0u;
    *(volatile uint32_t *)(m->h_nonfinite + 1) = 0u;
    *(volatile uint32_t *)(m->h_nonfinite + 2) = 0u;
    HIP_TRY(hipHostMalloc((void **)&m->h_res, 4 * cfd_model::kResRing, hipHostMallocDefault));
    for (hipEvent_t &e : m->ev_res) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc((void **)&m->h_spec, 4 * cfd_model::kSpecRing * kMaxTemporal, hipHostMallocDefault));
    for (hipEvent_t &e : m->ev_spec) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    if (const char *to = getenv("CFD_RCCL_TIMEOUT_S")) m->rccl_timeout_s = std::max(1.0, atof(to));

    // obstacle masks and cell list from cell centres (model.rs:235-260)
    std::vector<uint8_t> mu(nyl * W, 0), mv((nyl + 1) * nx, 0);
    std::vector<int32_t> obs;
    if (grid->has_cylinder) {
        for (int j = 0; j < ny; ++j) {
            for (int i = 0; i < nx; ++i) {
                const float x = ((float)i + 0.5f) * g.dx;
                const float y = ((float)j + 0.5f) * g.dy;
                const float ddx = x - grid->cylinder_x;
                const float ddy = y - grid->cylinder_y;
                const float distance = std::sqrt(ddx * ddx + ddy * ddy);
                if (!(distance < grid->cylinder_radius)) continue;
                const long lj = (long)j - (long)m->j0;
                if (lj >= 0 && lj < (long)nyl) {
                    if (i > 0) mu[lj * W + i] = 1;
                    if (i < nx) mu[lj * W + i + 1] = 1;
                }
                if (j > 0 && lj >= 0 && lj <= (long)nyl) mv[lj * nx + i] = 1;
                if (j < ny && lj + 1 >= 0 && lj + 1 <= (long)nyl) mv[(lj + 1) * nx + i] = 1;
                if (lj >= 0 && lj <= (long)nyl) {
                    obs.push_back(i);
                    obs.push_back(j);
                }
            }
        }
    }
    m->h_mask_u = mu;
    m->h_mask_v = mv;
    // device masks: bit 0 = predictor mask (model.rs:235-260), bit 1 = face
    // zeroed by the obstacle loop of apply_boundary_conditions (:866-874)
    std::vector<uint8_t> dmu(mu), dmv(mv);
    for (size_t k = 0; k < obs.size(); k += 2) {
        const long oi = obs[k], lj = (long)obs[k + 1] - (long)m->j0;
        if (lj >= 0 && lj < (long)nyl) dmu[lj * W + oi] |= 2;
        if (lj >= 0 && lj <= (long)nyl) dmv[lj * nx + oi] |= 2;
    }
    m->dmask_u = std::move(dmu);
    m->dmask_v = std::move(dmv);
    HIP_TRY(hipMemcpyAsync(m->mask_u, m->dmask_u.data(), m->dmask_u.size(), hipMemcpyHostToDevice,
                           m->stream));
    HIP_TRY(hipMemcpyAsync(m->mask_v, m->dmask_v.data(), m->dmask_v.size(), hipMemcpyHostToDevice,
                           m->stream));
    if (!obs.empty()) {
        HIP_TRY(hipMalloc((void **)&m->obs, obs.size() * 4));
        HIP_TRY(hipMemcpyAsync(m->obs, obs.data(), obs.size() * 4, hipMemcpyHostToDevice, m->stream));
    }

    Fields &f = m->f;
    const size_t uoff = (size_t)kGhostUV * W, voff = (size_t)kGhostUV * nx;
    f.u_alloc_base = m->u_all;
    f.v_alloc_base = m->v_all;
    f.u_old_base = m->uo_all;
    f.v_old_base = m->vo_all;
    f.u_star_base = m->us_all;
    f.v_star_base = m->vs_all;
    f.u_alloc = u_alloc;
    f.v_alloc = v_alloc;
    f.u = m->u_all + uoff;
    f.v = m->v_all + voff;
    f.u_old = m->uo_all + uoff;
    f.v_old = m->vo_all + voff;
    f.u_star = m->us_all + uoff;
    f.v_star = m->vs_all + voff;
    f.p = m->p;
    f.rhs = m->rhs + (size_t)hg * nx;   // hg ghost rows each side (sharded solves)
    f.pp[0] = m->pp_all[0] + (size_t)hg * nx;
    f.pp[1] = m->pp_all[1] + (size_t)hg * nx;
    f.mask_u = m->mask_u;
    f.mask_v = m->mask_v;
    f.obs = m->obs;
    f.n_obs = (int32_t)(obs.size() / 2);
    // without an obstacle in reach the masks are all zero and the predictors
    // skip their mask loads (a slab can hold mask rows of a cylinder whose
    // cells lie just outside it, so n_obs alone does not decide this)
    f.any_pmask = 0;
    for (uint8_t b : m->h_mask_u) f.any_pmask |= b & 1;
    for (uint8_t b : m->h_mask_v) f.any_pmask |= b & 1;
    f.ctl = m->ctl;
    {
        void *dp = nullptr;
        HIP_TRY(hipHostGetDevicePointer(&dp, m->h_nonfinite, 0));
        f.host_nonfinite = (uint32_t *)dp;
        f.host_progress = m->n_ranks > 1 ? (uint32_t *)dp + 1 : nullptr;
    }
    f.err_slots = m->slots;
    f.red_slots = m->slots + (size_t)kMaxSweeps * kResSlots * kResStride;
    f.vis_slots = f.red_slots + (size_t)4 * kResSlots * kResStride;
    f.persist = m->slots + (size_t)(kMaxSweeps + 16) * kResSlots * kResStride;

    Ctl c0;
    std::memset(&c0, 0, sizeof(c0));
    c0.dt = p->dt;
    c0.go[0] = 1;
    HIP_TRY(hipMemcpyAsync(m->ctl, &c0, sizeof(Ctl), hipMemcpyHostToDevice, m->stream));
    HIP_TRY(hipStreamSynchronize(m->stream));
    return 0;
}

// Communicator creation with a deadline.  ncclCommInitRank blocks in its
// bootstrap until every rank has arrived, and RCCL's non-blocking config does
// not change that (measured: ncclCommInitRankConfig with blocking = 0 did not
// return while the peer was missing).  So the blocking call runs on a helper
// thread and the caller waits at most CFD_RCCL_TIMEOUT_S: a rank that never
// arrives makes cfd_create_sharded fail with CFD_ERCCL instead of hanging.
// The stuck bootstrap is abandoned (the detached thread stays blocked; should
// a late peer still complete it, the thread aborts that communicator itself).
struct CommInitJob {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false, abandoned = false;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclSuccess;
    hipError_t he = hipSuccess;
};

int comm_init(cfd_model *m, const ncclUniqueId &id, int n_ranks, int rank) {
    auto job = std::make_shared<CommInitJob>();
    const int device = m->device;
    std::thread([job, id, n_ranks, rank, device] {
        ncclComm_t c = nullptr;
        ncclResult_t r = ncclInternalError;
        const hipError_t he = hipSetDevice(device);
        if (he == hipSuccess) r = ncclCommInitRank(&c, n_ranks, id, rank);
        std::lock_guard<std::mutex> lk(job->mu);
        if (job->abandoned) {
            if (r == ncclSuccess && c) ncclCommAbort(c);
            return;
        }
        job->comm = c;
        job->r = r;
        job->he = he;
        job->done = true;
        job->cv.notify_all();
    }).detach();
    std::unique_lock<std::mutex> lk(job->mu);
    const auto limit = std::chrono::duration<double>(m->rccl_timeout_s);
    if (!job->cv.wait_for(lk, limit, [&] { return job->done; })) {
        job->abandoned = true;
        return fail(CFD_ERCCL, "ncclCommInitRank: rank " + std::to_string(rank) + " of " +
                                   std::to_string(n_ranks) + ": not every rank joined within " +
                                   std::to_string((int)m->rccl_timeout_s) +
                                   " s (CFD_RCCL_TIMEOUT_S); creation abandoned");
    }
    if (job->he != hipSuccess)
        return fail(CFD_EHIP, std::string("hipSetDevice (RCCL init thread): ") + hipGetErrorString(job->he));
    if (job->r != ncclSuccess)
        return fail(CFD_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(job->r));
    m->comm = job->comm;
    return 0;
}

int create_common(const cfd_grid *grid, const cfd_params *params, int device, int n_ranks, int rank,
                  const void *uid, LocalHub *hub, cfd_model **out) {
    if (!out) return fail(CFD_EINVAL, "null out");
    *out = nullptr;
    int rc = validate(grid, params);
    if (rc) return rc;
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(CFD_EINVAL, "bad rank/n_ranks");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(CFD_EHIP, "no HIP device available");
    if (device < 0 || device >= ndev) return fail(CFD_EINVAL, "device ordinal out of range");
    cfd_model *m = new cfd_model();
    m->n_ranks = n_ranks;
    m->rank = rank;
    plan_slab(grid->ny, n_ranks, rank, &m->j0, &m->j1);
    int hg = 1;
    if (n_ranks > 1) {
        // Deep halos: one RCCL round every hg sweeps (a round over xGMI is
        // latency-bound, ~20-30 us) against ~hg/nyl redundant ghost-row
        // compute; default hg = nyl/32 clamped to [8, 32] (32 at the bench's
        // 1024-2048-row slabs: 7 rounds per 200-sweep step, ~3 % extra rows).
        // The floor 8 (r6; 4 before) lets the tolerance mode's speculative
        // blocks run 8 sweeps per exchange on thin slabs too (the default
        // channel on 2 ranks: 13 blocks of 4 per solve -> 7 of 8)
        uint64_t min_rows = grid->ny / (uint64_t)n_ranks;
        const char *env = getenv("CFD_HALO_DEPTH");
        hg = env ? atoi(env)
                 : (int)std::max<uint64_t>(kMaxTemporal, std::min<uint64_t>(32, min_rows / 32));
        if (hg < 1) hg = 1;
        if ((uint64_t)hg + 2 > min_rows) hg = (int)(min_rows > 3 ? min_rows - 2 : 1);
        if (min_rows < 4) {
            delete m;
            return fail(CFD_EINVAL, "each slab needs at least 4 rows");
        }
    }
    rc = build_model(m, grid, params, device, hg);
    if (!rc) rc = validate_sharded(m, params);
    if (!rc && n_ranks > 1 && hub) {
        if (hub->n != n_ranks) {
            rc = fail(CFD_EINVAL, "local hub size != n_ranks");
        } else {
            std::lock_guard<std::mutex> lk(hub->mu);
            hub->members[rank] = m;
            m->hub = hub;
        }
    } else if (!rc && n_ranks > 1) {
        ncclUniqueId id;
        std::memcpy(&id, uid, sizeof(id));
        rc = comm_init(m, id, n_ranks, rank);
    }
    if (rc) {
        m->destroy();
        delete m;
        return rc;
    }
    *out = m;
    return 0;
}

}  // namespace

// =============================================================== C ABI

extern "C" {

const char *cfd_last_error(void) { return g_last_error.c_str(); }
// internal (not in cfd.h): lets the host runtime (cfd_runtime.cpp) report
// through the same thread-local message
void cfdrt_set_error(const char *msg) { g_last_error = msg ? msg : ""; }
// internal: the host-only checks cfd_set_params makes, for cfd_run_set_params
// to reject bad parameters synchronously (reads only the immutable grid)
int cfdrt_check_params(const cfd_model *m, const cfd_params *p) {
    if (!m) return fail(CFD_EINVAL, "null model");
    int rc = validate(&m->grid, p);
    if (rc) return rc;
    return validate_sharded(m, p);
}

int cfd_get_config(const cfd_model *m, cfd_grid *grid, cfd_params *params) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (grid) *grid = m->grid;
    if (params) *params = m->params;
    return 0;
}
int cfd_abi_version(void) { return CFD_ABI_VERSION; }

void cfd_default_params(cfd_params *o) {
    if (!o) return;
    o->dt = 0.005f;                  // model.rs:47
    o->viscosity = 0.000001f;        // model.rs:48
    o->target_inlet_velocity = 1.0f; // model.rs:49
    o->velocity_scheme = CFD_SCHEME_FIRST_ORDER;
    o->inlet_profile = CFD_INLET_UNIFORM;
    o->pressure_solver = CFD_SOLVER_JACOBI;
    o->jacobi_iters = 50;            // model.rs:737
    o->corrector_passes = 20;        // model.rs:696
    o->tol_enabled = 1;
    o->p_tol = 1e-4f;                // model.rs:736, 721
    o->bc_kind = CFD_BC_CHANNEL;
}

void cfd_default_grid(cfd_grid *o) {
    if (!o) return;
    o->nx = 800;                     // src/app.rs:34
    o->ny = 264;
    o->lx = 30.0f;
    o->ly = 10.0f;
    o->has_cylinder = 1;
    o->cylinder_x = 30.0f / 4.0f;    // src/app.rs:47
    o->cylinder_y = 10.0f / 2.0f;
    o->cylinder_radius = 0.75f;
}

int cfd_create(const cfd_grid *grid, const cfd_params *params, int device_ordinal, cfd_model **out) {
    return create_common(grid, params, device_ordinal, 1, 0, nullptr, nullptr, out);
}

int cfd_rccl_unique_id(void *out) {
    if (!out) return fail(CFD_EINVAL, "null out");
    ncclUniqueId id;
    RCCL_TRY(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

int cfd_create_sharded(const cfd_grid *grid, const cfd_params *params, int device_ordinal,
                       int n_ranks, int rank, const void *uid, cfd_model **out) {
    if (n_ranks > 1 && !uid) return fail(CFD_EINVAL, "null rccl unique id");
    return create_common(grid, params, device_ordinal, n_ranks, rank, uid, nullptr, out);
}

void *cfd_local_hub_create(int n_ranks) {
    if (n_ranks < 1) return nullptr;
    LocalHub *h = new LocalHub();
    h->n = n_ranks;
    h->members.assign(n_ranks, nullptr);
    return h;
}

void cfd_local_hub_destroy(void *hub) { delete static_cast<LocalHub *>(hub); }

int cfd_create_sharded_local(const cfd_grid *grid, const cfd_params *params, int device_ordinal,
                             int n_ranks, int rank, void *hub, cfd_model **out) {
    if (!hub) return fail(CFD_EINVAL, "null local hub");
    return create_common(grid, params, device_ordinal, n_ranks, rank, nullptr,
                         static_cast<LocalHub *>(hub), out);
}

int cfd_device_count(int *n_out) {
    if (!n_out) return fail(CFD_EINVAL, "null out");
    *n_out = 0;
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess && e != hipErrorNoDevice)
        return fail(CFD_EHIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    *n_out = e == hipSuccess ? n : 0;
    return 0;
}

int cfd_get_comm_size(const cfd_model *m, int *n_out) {
    if (!m || !n_out) return fail(CFD_EINVAL, "null model or out");
    if (m->hub) {
        *n_out = m->hub->n;
    } else if (m->comm) {
        int n = 0;
        RCCL_TRY(ncclCommCount(m->comm, &n));
        *n_out = n;
    } else if (m->n_ranks > 1) {
        return fail(CFD_ERCCL, "the RCCL communicator was aborted after an earlier failure");
    } else {
        *n_out = 1;
    }
    return 0;
}

int cfd_get_slab(const cfd_model *m, uint64_t *j0, uint64_t *j1) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (j0) *j0 = m->j0;
    if (j1) *j1 = m->j1;
    return 0;
}

int cfd_update(cfd_model *m) { return cfd_update_n(m, 1); }

int cfd_update_n(cfd_model *m, int n) {
    if (!m) return fail(CFD_EINVAL, "null model");
    HIP_TRY(hipSetDevice(m->device));
    // a solve timeout first (its junk steps may have raised the non-finite
    // flag too): recovered from the checkpoint, reported once
    if (int rc = m->persist_timeout_check(false)) return rc;
    // failure detection: a step the device has already finished left a NaN or
    // Inf in u/v (zero-copy word, no stream synchronisation)
    if (const uint32_t bad = *(volatile uint32_t *)m->h_nonfinite)
        return fail(CFD_ENONFINITE, "non-finite velocity (NaN/Inf) after step " + std::to_string(bad) +
                                        "; cfd_set_state clears it");
    if (n <= 0) return 0;
    if (int rc = m->ck_begin()) return rc;
    m->ck_record([m, n]() {
        for (int k = 0; k < n; ++k)
            if (int rc = m->enqueue_update(k == n - 1)) return rc;
        return 0;
    });
    // solve timing: one event pair around the whole batch for the step time
    if (m->timing) {
        hipEvent_t e0 = m->take_event();
        HIP_TRY(hipEventRecord(e0, m->stream));
        m->step_events.push_back(e0);
    }
    int rc = 0;
    if (m->graph_ok()) {
        rc = m->update_graph(n);
    } else {
        for (int k = 0; k < n && !rc; ++k) rc = m->enqueue_update(k == n - 1);
    }
    if (m->timing) {
        hipEvent_t e1 = m->take_event();
        HIP_TRY(hipEventRecord(e1, m->stream));
        m->step_events.push_back(e1);
    }
    return rc;
}

int cfd_piso_step(cfd_model *m, float dt_sub) {
    if (!m) return fail(CFD_EINVAL, "null model");
    HIP_TRY(hipSetDevice(m->device));
    if (int rc = m->ck_begin()) return rc;
    auto run = [m, dt_sub]() {
        int rc = m->exchange_uv();
        if (!rc) rc = m->enqueue_piso(dt_sub);
        return rc ? rc : m->abort_allreduce();
    };
    m->ck_record(run);
    return run();
}

int cfd_pressure_solve(cfd_model *m, float *residual_out) {
    if (!m) return fail(CFD_EINVAL, "null model");
    HIP_TRY(hipSetDevice(m->device));
    int rc;
    if (m->host_driven()) {
        return m->enqueue_solve_host_driven(residual_out);
    }
    if ((rc = m->ck_begin())) return rc;
    auto run = [m]() {
        int rc2 = m->enqueue_solve(-1);
        return rc2 ? rc2 : m->abort_allreduce();
    };
    m->ck_record(run);
    rc = run();
    if (rc) return rc;
    Ctl c;
    rc = m->read_ctl(&c);
    if (rc) return rc;
    if (residual_out) *residual_out = c.last_p;
    return 0;
}

int cfd_run_phase(cfd_model *m, int phase, float dt_sub) {
    if (!m) return fail(CFD_EINVAL, "null model");
    HIP_TRY(hipSetDevice(m->device));
    switch (phase) {
    case CFD_PHASE_U_PREDICTOR: {
        int rc = m->exchange_uv();
        if (rc) return rc;
        launch_u_predictor(m->g, m->f, dt_sub, m->stream);
        break;
    }
    case CFD_PHASE_V_PREDICTOR: {
        int rc = m->exchange_uv();
        if (rc) return rc;
        launch_v_predictor(m->g, m->f, dt_sub, m->stream);
        break;
    }
    case CFD_PHASE_DIVERGENCE: launch_divergence(m->g, m->f, -1, dt_sub, m->stream); break;
    case CFD_PHASE_CORRECTOR: launch_corrector(m->g, m->f, -1, dt_sub, m->stream); break;
    case CFD_PHASE_BOUNDARY: launch_boundary(m->g, m->f, m->stream); break;
    default: return fail(CFD_EINVAL, "unknown phase");
    }
    HIP_TRY(hipGetLastError());
    return m->sync();
}

int cfd_set_params(cfd_model *m, const cfd_params *p) {
    if (!m) return fail(CFD_EINVAL, "null model");
    int rc = validate(&m->grid, p);
    if (rc) return rc;
    rc = validate_sharded(m, p);
    if (rc) return rc;
    rc = m->sync();
    if (rc) return rc;
    m->drop_graph();   // kernel arguments follow the parameters
    {
        // host mirror of the current p' buffer (the tolerance-driven Jacobi
        // solve flips it on the device); fixed-count and in-place solves use it
        Ctl c;
        rc = m->read_ctl(&c);
        if (rc) return rc;
        m->host_cur = c.cur;
    }
    apply_params(m, p);
    // set_parameters overwrites dt (model.rs:1252)
    HIP_TRY(hipMemcpy(&m->ctl->dt, &p->dt, 4, hipMemcpyHostToDevice));
    return 0;
}

int cfd_get_snapshot(cfd_model *m, float *u, float *v, float *p, float *dt_out) {
    if (!m) return fail(CFD_EINVAL, "null model");
    int rc = m->sync();
    if (rc) return rc;
    const size_t W = (size_t)m->g.nx + 1, nx = (size_t)m->g.nx, nyl = (size_t)m->g.nyl;
    if (u) HIP_TRY(hipMemcpy(u, m->f.u, nyl * W * 4, hipMemcpyDeviceToHost));
    if (v) HIP_TRY(hipMemcpy(v, m->f.v, (nyl + 1) * nx * 4, hipMemcpyDeviceToHost));
    if (p) HIP_TRY(hipMemcpy(p, m->f.p, nyl * nx * 4, hipMemcpyDeviceToHost));
    if (dt_out) HIP_TRY(hipMemcpy(dt_out, &m->ctl->dt, 4, hipMemcpyDeviceToHost));
    return 0;
}

namespace {

float decode_key(uint32_t k, bool is_min) {   // inverse of ord_key (cfd_render.hip)
    if (is_min) {
        if (!k) return INFINITY;
        k = ~k;
    } else if (!k) {
        return -INFINITY;
    }
    const uint32_t b = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
    float x;
    std::memcpy(&x, &b, 4);
    return x;
}

// cfd_render / cfd_derive_field: field or image of `mode` for the model's
// slab, min/max reduced over ranks, one D2H copy of nx*nyl words.
int render_common(cfd_model *m, int mode, bool field, void *host_out, float *min_max_out) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (mode < CFD_VIS_PRESSURE || mode > CFD_VIS_VORTICITY)
        return fail(CFD_EINVAL, "unknown visualisation mode");
    HIP_TRY(hipSetDevice(m->device));
    const size_t n = (size_t)m->g.nx * (size_t)m->g.nyl;
    if (!m->vis_buf) HIP_TRY(hipMalloc((void **)&m->vis_buf, n * 4));
    if (mode == CFD_VIS_VORTICITY) {   // reads u/v one row above the slab
        int rc = m->exchange_uv();
        if (rc) return rc;
    }
    Fields &f = m->f;
    launch_vis_field(m->g, f, mode, field ? m->vis_buf : nullptr, f.vis_slots, m->stream);
    launch_fold_slots(f.ctl->vis, f.vis_slots, 2, m->stream);
    int rc = m->allreduce_max_u32(f.ctl->vis, 2);
    if (rc) return rc;
    const cfd_grid &gr = m->grid;
    if (!field && host_out)
        launch_vis_color(m->g, f, mode, nullptr, (uint32_t *)m->vis_buf, f.ctl->vis,
                         gr.has_cylinder, gr.cylinder_x, gr.cylinder_y, gr.cylinder_radius,
                         m->stream);
    HIP_TRY(hipGetLastError());
    uint32_t keys[2] = {0u, 0u};
    HIP_TRY(hipMemcpyAsync(keys, f.ctl->vis, 8, hipMemcpyDeviceToHost, m->stream));
    HIP_TRY(hipMemsetAsync(f.ctl->vis, 0, 8, m->stream));
    if (host_out) HIP_TRY(hipMemcpyAsync(host_out, m->vis_buf, n * 4, hipMemcpyDeviceToHost, m->stream));
    if (int rc2 = m->wait_done(nullptr)) return rc2;
    if (min_max_out) {
        min_max_out[0] = decode_key(keys[1], true);
        min_max_out[1] = decode_key(keys[0], false);
    }
    return 0;
}

}  // namespace

int cfd_render(cfd_model *m, int mode, uint8_t *rgba, float *min_max_out) {
    return render_common(m, mode, false, rgba, min_max_out);
}

int cfd_derive_field(cfd_model *m, int mode, float *out, float *min_max_out) {
    return render_common(m, mode, true, out, min_max_out);
}

int cfd_get_residuals(cfd_model *m, cfd_residuals *out) {
    if (!m || !out) return fail(CFD_EINVAL, "null argument");
    Ctl c;
    int rc = m->read_ctl(&c);
    if (rc) return rc;
    out->simulation_step = c.step;
    out->simulation_time = c.time;
    out->dt = c.dt;
    out->p = c.last_p;
    out->u = c.res_u;
    out->v = c.res_v;
    out->piso_substeps = 1;   // substep_count (model.rs:267)
    out->jacobi_sweeps_total = c.sweeps_total;
    float ms = 0.f;
    if (m->stepped && hipEventElapsedTime(&ms, m->ev_step0, m->ev_step1) == hipSuccess)
        out->step_time_s = ms * 1e-3;
    else
        out->step_time_s = 0.0;
    if (c.nonfinite_step)   // *out is filled all the same
        return fail(CFD_ENONFINITE, "non-finite velocity (NaN/Inf) after step " +
                                        std::to_string(c.nonfinite_step));
    return 0;
}

int cfd_get_state(cfd_model *m, cfd_state *st) {
    if (!m || !st) return fail(CFD_EINVAL, "null argument");
    Ctl c;
    int rc = m->read_ctl(&c);
    if (rc) return rc;
    const size_t W = (size_t)m->g.nx + 1, nx = (size_t)m->g.nx, nyl = (size_t)m->g.nyl;
    if (st->u) HIP_TRY(hipMemcpy(st->u, m->f.u, nyl * W * 4, hipMemcpyDeviceToHost));
    if (st->v) HIP_TRY(hipMemcpy(st->v, m->f.v, (nyl + 1) * nx * 4, hipMemcpyDeviceToHost));
    if (st->p) HIP_TRY(hipMemcpy(st->p, m->f.p, nyl * nx * 4, hipMemcpyDeviceToHost));
    if (st->u_star) HIP_TRY(hipMemcpy(st->u_star, m->f.u_star, nyl * W * 4, hipMemcpyDeviceToHost));
    if (st->v_star) HIP_TRY(hipMemcpy(st->v_star, m->f.v_star, (nyl + 1) * nx * 4, hipMemcpyDeviceToHost));
    if (st->p_prime) HIP_TRY(hipMemcpy(st->p_prime, m->f.pp[c.cur], nyl * nx * 4, hipMemcpyDeviceToHost));
    if (st->rhs) HIP_TRY(hipMemcpy(st->rhs, m->f.rhs, nyl * nx * 4, hipMemcpyDeviceToHost));
    st->dt = c.dt;
    st->simulation_time = c.time;
    st->simulation_step = c.step;
    st->last_p_residual = c.last_p;
    st->last_u_residual = c.res_u;
    st->last_v_residual = c.res_v;
    st->jacobi_sweeps_total = c.sweeps_total;
    return 0;
}

int cfd_set_state(cfd_model *m, const cfd_state *st) {
    if (!m || !st) return fail(CFD_EINVAL, "null argument");
    Ctl c;
    int rc = m->read_ctl(&c);
    if (rc) return rc;
    const size_t W = (size_t)m->g.nx + 1, nx = (size_t)m->g.nx, nyl = (size_t)m->g.nyl;
    if (st->u) HIP_TRY(hipMemcpy(m->f.u, st->u, nyl * W * 4, hipMemcpyHostToDevice));
    if (st->v) HIP_TRY(hipMemcpy(m->f.v, st->v, (nyl + 1) * nx * 4, hipMemcpyHostToDevice));
    if (st->p) HIP_TRY(hipMemcpy(m->f.p, st->p, nyl * nx * 4, hipMemcpyHostToDevice));
    if (st->u_star) HIP_TRY(hipMemcpy(m->f.u_star, st->u_star, nyl * W * 4, hipMemcpyHostToDevice));
    if (st->v_star) HIP_TRY(hipMemcpy(m->f.v_star, st->v_star, (nyl + 1) * nx * 4, hipMemcpyHostToDevice));
    if (st->p_prime) HIP_TRY(hipMemcpy(m->f.pp[c.cur], st->p_prime, nyl * nx * 4, hipMemcpyHostToDevice));
    if (st->rhs) HIP_TRY(hipMemcpy(m->f.rhs, st->rhs, nyl * nx * 4, hipMemcpyHostToDevice));
    c.dt = st->dt;
    c.time = st->simulation_time;
    c.step = (uint32_t)st->simulation_step;
    c.last_p = st->last_p_residual;
    c.res_u = st->last_u_residual;
    c.res_v = st->last_v_residual;
    c.sweeps_total = st->jacobi_sweeps_total;
    c.nonfinite_step = 0;   // a new state: failure detection starts over
    c.red[4] = 0;
    c.red[6] = 0;           // and an old solve timeout with it
    rc = m->clear_abort_words();
    if (rc) return rc;
    HIP_TRY(hipMemcpy(m->f.ctl, &c, offsetof(Ctl, go), hipMemcpyHostToDevice));
    *(volatile uint32_t *)m->h_nonfinite = 0u;
    m->host_cur = c.cur;
    // ghosts of the injected slab
    rc = m->exchange_uv();
    if (rc) return rc;
    rc = m->exchange_pp(c.cur, m->g.hg);
    if (rc) return rc;
    return m->sync();
}

int cfd_get_masks(cfd_model *m, uint8_t *mask_u, uint8_t *mask_v) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (mask_u) std::memcpy(mask_u, m->h_mask_u.data(), m->h_mask_u.size());
    if (mask_v) std::memcpy(mask_v, m->h_mask_v.data(), m->h_mask_v.size());
    return 0;
}

int cfd_synchronize(cfd_model *m) {
    if (!m) return fail(CFD_EINVAL, "null model");
    return m->sync();
}

int cfd_profile_sweeps(cfd_model *m, int n_sweeps, double *avg_ms_out) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (n_sweeps < 1 || n_sweeps > kMaxSweeps) return fail(CFD_EINVAL, "n_sweeps out of range");
    HIP_TRY(hipSetDevice(m->device));
    const int lo = std::max(0, 1 - (int)m->j0), hi = std::min(m->g.nyl, (int)m->g.ny - 1 - (int)m->j0);
    hipEvent_t a = m->ev_prof0, b = m->ev_prof1;
    Geom g = m->g;
    g.tol_enabled = 0;
    HIP_TRY(hipEventRecord(a, m->stream));
    for (int it = 0; it < n_sweeps; ++it)
        launch_jacobi_sweep(g, m->f, -1, it, lo, hi, it == n_sweeps - 1, m->stream);
    HIP_TRY(hipEventRecord(b, m->stream));
    launch_finalize_solve(g, m->f, -1, n_sweeps, 0, n_sweeps, m->stream);
    HIP_TRY(hipGetLastError());
    m->host_cur = (m->host_cur + n_sweeps) & 1;
    m->pp_ghosts_shallow = m->sharded();   // owned rows only were swept
    int rc = m->sync();
    if (rc) return rc;
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, a, b));
    if (avg_ms_out) *avg_ms_out = ms / n_sweeps;
    return 0;
}

// Timing of the pressure solves inside cfd_update (HIP events on the model's
// stream): enable, run steps, then read the totals.
int cfd_timing_begin(cfd_model *m) {
    if (!m) return fail(CFD_EINVAL, "null model");
    int rc = m->sync();
    if (rc) return rc;
    m->timing = true;
    m->ev_next = 0;
    m->solve_events.clear();
    m->step_events.clear();
    for (auto &pe : m->phase_events) pe.clear();
    m->timed_sweeps = 0;
    m->timed_launches = 0;
    m->timed_steps = 0;
    return 0;
}

int cfd_timing_end(cfd_model *m, double *solve_ms, uint64_t *sweeps, double *step_ms, uint64_t *steps) {
    if (!m) return fail(CFD_EINVAL, "null model");
    int rc = m->sync();
    if (rc) return rc;
    double s_ms = 0.0, t_ms = 0.0;
    for (auto &pr : m->solve_events) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
        s_ms += ms;
    }
    for (size_t k = 0; k + 1 < m->step_events.size(); k += 2) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, m->step_events[k], m->step_events[k + 1]));
        t_ms += ms;
    }
    for (int ph = 0; ph < 3; ++ph) {
        m->phase_ms[ph] = 0.0;
        m->phase_count[ph] = 0;
        for (auto &pr : m->phase_events[ph]) {
            float ms = 0.f;
            if (!pr.second) continue;
            HIP_TRY(hipEventElapsedTime(&ms, pr.first, pr.second));
            m->phase_ms[ph] += ms;
            ++m->phase_count[ph];
        }
        m->phase_events[ph].clear();
    }
    if (solve_ms) *solve_ms = s_ms;
    if (sweeps) *sweeps = m->timed_sweeps;
    if (step_ms) *step_ms = t_ms;
    if (steps) *steps = m->timed_steps;
    m->timing = false;
    m->ev_next = 0;
    m->solve_events.clear();
    m->step_events.clear();
    return 0;
}

int cfd_timing_phases(cfd_model *m, int on) {
    if (!m) return fail(CFD_EINVAL, "null model");
    m->timing_phases = on != 0;
    return 0;
}

int cfd_timing_phase_ms(const cfd_model *m, double *predict_ms, double *finish_ms) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (predict_ms) *predict_ms = m->phase_ms[0];
    if (finish_ms) *finish_ms = m->phase_ms[1];
    return 0;
}

int cfd_timing_exchange_ms(const cfd_model *m, double *exchange_ms, uint64_t *exchanges) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (exchange_ms) *exchange_ms = m->phase_ms[2];
    if (exchanges) *exchanges = m->phase_count[2];
    return 0;
}

int cfd_get_halo_depth(const cfd_model *m) { return m ? m->g.hg : 0; }

int cfd_get_kernel_config(const cfd_model *m, int *fastdiv, int *temporal) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (fastdiv) *fastdiv = m->g.fastdiv;
    if (temporal) *temporal = m->spec_mode() ? kMaxTemporal : m->g.tol_enabled ? 1 : m->t_max;
    return 0;
}

int cfd_get_jacobi_kernel(const cfd_model *m, int *kind, char *name, size_t name_len) {
    if (!m) return fail(CFD_EINVAL, "null model");
    const bool spec = m->spec_mode();
    const bool resident = m->resident_mode();
    const int T = spec ? kMaxTemporal : m->g.tol_enabled ? 1 : m->t_max;
    const int k = resident ? 6 : spec ? 5 : T <= 1 ? 0 : m->g.tb_kind;
    if (kind) *kind = k;
    if (name && name_len) {
        char buf[96];
        if (resident)
            snprintf(buf, sizeof buf, "k_jacobi_resident<%d>", m->g.res_div);
        else if (spec)
            snprintf(buf, sizeof buf, "k_jacobi_lds<%d, %d, 2>", T, m->g.fastdiv);
        else if (k == 0)
            snprintf(buf, sizeof buf, "k_jacobi<%d, %d>", kJacRowsPerWave, m->g.fastdiv);
        else if (k == 1)
            snprintf(buf, sizeof buf, "k_jacobi_tb<%d, %d>", T, m->g.fastdiv);
        else if (k == 5)
            snprintf(buf, sizeof buf, "k_jacobi_lds<%d, %d, 0>", T, m->g.fastdiv);
        else
            snprintf(buf, sizeof buf, "k_jacobi_pipe<%d, %d, %d>", T, m->g.fastdiv, k == 3 ? 4 : 2);
        snprintf(name, name_len, "%s", buf);
    }
    return 0;
}

int cfd_get_jacobi_geometry(const cfd_model *m, int persist, int *lds_pad, int *wgs_per_cu,
                            int *wave_cols, int *segments) {
    if (!m) return fail(CFD_EINVAL, "null model");
    if (hipSetDevice(m->device) != hipSuccess) return fail(CFD_EHIP, "hipSetDevice");
    // the rows of the solve's first 8-sweep block (a slab's owned rows plus
    // the ghost rows that block recomputes)
    int T, lo, hi, exch;
    plan_block((int)m->j0, m->g.nyl, m->g.ny, m->sharded() ? m->g.hg : 0, 0, 8,
               std::max(8, m->params.jacobi_iters), &T, &lo, &hi, &exch);
    if (!m->sharded()) lo = 1 - (int)m->j0, hi = (int)m->g.ny - 1 - (int)m->j0;
    int pad = 0, occ = 0, nwc = 0, nseg = 0;
    lds_geometry8(m->g, lo, hi, persist != 0, &pad, &occ, &nwc, &nseg);
    if (lds_pad) *lds_pad = pad;
    if (wgs_per_cu) *wgs_per_cu = occ;
    if (wave_cols) *wave_cols = nwc;
    if (segments) *segments = nseg;
    return 0;
}

int cfd_get_persist_steals(cfd_model *m, uint64_t *steals) {
    if (!m || !steals) return fail(CFD_EINVAL, "null argument");
    int rc = m->sync();
    if (rc) return rc;
    uint32_t v = 0;
    HIP_TRY(hipMemcpy(&v, m->f.persist + 2, 4, hipMemcpyDeviceToHost));
    *steals = v;
    return 0;
}

int cfd_get_persist_sums(cfd_model *m, uint64_t *blocks) {
    if (!m || !blocks) return fail(CFD_EINVAL, "null argument");
    int rc = m->sync();
    if (rc) return rc;
    uint32_t v = 0;
    HIP_TRY(hipMemcpy(&v, m->f.persist + 3, 4, hipMemcpyDeviceToHost));
    *blocks = v;   // persistent blocks run in the SUMS form
    return 0;
}

int cfd_get_comm_calls(const cfd_model *m, uint64_t *n) {
    if (!m || !n) return fail(CFD_EINVAL, "null argument");
    *n = m->comm_calls;
    return 0;
}

int cfd_get_recoveries(const cfd_model *m, uint64_t *n) {
    if (!m || !n) return fail(CFD_EINVAL, "null argument");
    *n = m->recoveries;
    return 0;
}

int cfd_get_resident_solves(const cfd_model *m, uint64_t *solves) {
    if (!m || !solves) return fail(CFD_EINVAL, "null argument");
    *solves = m->resident_solves;
    return 0;
}

int cfd_get_persist_blocks(const cfd_model *m, int *blocks) {
    if (!m || !blocks) return fail(CFD_EINVAL, "null argument");
    *blocks = m->last_persist_blocks;
    return 0;
}

// ---- host-only slab plan (no device needed) ----
int cfd_plan_slab(uint64_t ny, int n_ranks, int rank, uint64_t *j0, uint64_t *j1) {
    if (n_ranks < 1 || rank < 0 || rank >= n_ranks || !j0 || !j1)
        return fail(CFD_EINVAL, "bad plan_slab arguments");
    plan_slab(ny, n_ranks, rank, j0, j1);
    return 0;
}

int cfd_plan_sweep(int j0, int nyl, int ny, int halo_depth, int it, int iters, int *lo, int *hi,
                   int *exchange) {
    if (halo_depth < 1 || !lo || !hi || !exchange) return fail(CFD_EINVAL, "bad plan_sweep arguments");
    plan_sweep(j0, nyl, ny, halo_depth, it, iters, lo, hi, exchange);
    return 0;
}

int cfd_plan_block(int j0, int nyl, int ny, int halo_depth, int it, int t_max, int iters, int *T,
                   int *out_lo, int *out_hi, int *exchange) {
    if (t_max < 1 || !T || !out_lo || !out_hi || !exchange)
        return fail(CFD_EINVAL, "bad plan_block arguments");
    plan_block(j0, nyl, ny, halo_depth, it, t_max, iters, T, out_lo, out_hi, exchange);
    return 0;
}

int cfd_plan_overlap(int nyl, int halo_depth, int rank, int n_ranks, int lo, int hi, int *out6) {
    if (!out6 || n_ranks < 1 || rank < 0 || rank >= n_ranks) return fail(CFD_EINVAL, "bad plan_overlap arguments");
    return plan_overlap(nyl, halo_depth, rank, n_ranks, lo, hi, out6);
}

int cfd_plan_halo(int kind, int nyl, int depth, int rank, int n_ranks, int *out6) {
    if (kind < 0 || kind > 2 || !out6) return fail(CFD_EINVAL, "bad plan_halo arguments");
    plan_halo(kind, nyl, depth, rank, n_ranks, out6);
    return 0;
}

void cfd_destroy(cfd_model *m) {
    if (!m) return;
    m->destroy();
    delete m;
}

}  // extern "C"
