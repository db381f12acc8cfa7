"""cfdamd — host-side mirror of cfd-demo's `Model` interface
(/root/reference/src/model.rs) over the MI355X C ABI (include/cfd.h).

Names, defaults and argument meaning follow the reference:

    SimulationParams / VelocityScheme / InletProfile / PressureSolver  model.rs:13-21, 44-55, 141-159
    Grid / Cylinder                                                  model.rs:119-139
    Model.new / update / set_parameters / get_snapshot /
    get_residuals / run                                              model.rs:219, 304, 1250-1332
    SimulationControlHandle (stop, pause, resume, set_params,
    request_snapshot, get_last_available_snapshot,
    get_new_log_messages)                                            model.rs:57-117

Every call goes to the HIP library; there is no CPU fallback.  Fields are
returned as float32 numpy arrays in the reference's flat layout.
"""
from __future__ import annotations

import ctypes as C
import enum
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from . import _lib
from ._lib import (CFD_ENONFINITE, CfdError, CfdGrid, CfdParams, CfdResiduals, CfdState, check,
                   load)

__all__ = [
    "VelocityScheme", "InletProfile", "PressureSolver", "BoundaryKind", "Cylinder", "Grid",
    "SimulationParams", "Residuals", "SimSnapshot", "Model", "SimulationControlHandle",
    "CfdError", "default_grid", "cavity_grid", "rccl_unique_id", "device_count", "load", "LocalHub",
    "VisualizationMode", "CFD_ENONFINITE",
]


class VelocityScheme(enum.IntEnum):          # model.rs:141-146
    FirstOrder = 0
    SecondOrder = 1


class InletProfile(enum.IntEnum):            # model.rs:154-159
    Uniform = 0
    Parabolic = 1


class PressureSolver(enum.IntEnum):          # model.rs:148-152
    Jacobi = 0
    # the JavaScript variant's solvers (index.html:741-774, 775-795, 1344-1470)
    Sor = 1
    Multigrid = 2


class VisualizationMode(enum.IntEnum):       # app.rs:505-509
    Pressure = 0
    Velocity = 1
    Vorticity = 2


class BoundaryKind(enum.IntEnum):            # build-defined
    Channel = 0
    Cavity = 1


@dataclass
class Cylinder:                              # model.rs:133-139
    center_x: float
    center_y: float
    radius: float


@dataclass
class Grid:                                  # model.rs:119-131
    nx: int
    ny: int
    lx: float
    ly: float
    obstacle: Optional[Cylinder] = None

    @property
    def dx(self) -> float:
        return float(np.float32(self.lx) / np.float32(self.nx))

    @property
    def dy(self) -> float:
        return float(np.float32(self.ly) / np.float32(self.ny))

    def _c(self) -> CfdGrid:
        o = self.obstacle
        return CfdGrid(self.nx, self.ny, self.lx, self.ly, 1 if o else 0,
                       o.center_x if o else 0.0, o.center_y if o else 0.0,
                       o.radius if o else 0.0)


def default_grid() -> Grid:
    """src/app.rs:32-53."""
    lx, ly = 30.0, 10.0
    return Grid(800, 264, lx, ly, Cylinder(lx / 4.0, ly / 2.0, 0.75))


def assemble_slabs(slabs, nx: int) -> dict:
    """Global flat fields from the states of the row slabs of one grid:
    `slabs` = [(j0, j1, state)] in rank order (state as Model.get_state()
    returns it).  Owned rows are concatenated; v and v* take the shared face
    row j1 of each slab from the slab above (both compute it, bit-identically:
    raises ValueError when they differ)."""
    out = {}
    for f in ("u", "p", "p_prime", "u_star", "rhs"):
        out[f] = np.concatenate([s[f] for (_, _, s) in slabs])
    for f in ("v", "v_star"):
        parts = []
        for k, (j0, j1, s) in enumerate(slabs):
            rows = s[f].reshape(j1 - j0 + 1, nx)
            last = k == len(slabs) - 1
            parts.append(rows if last else rows[:-1])
            if not last:
                nxt = slabs[k + 1][2][f].reshape(-1, nx)[0]
                if not np.array_equal(rows[-1].view(np.uint32), nxt.view(np.uint32)):
                    raise ValueError(f"{f}: shared face row {j1} differs between slabs {k} and {k + 1}")
        out[f] = np.concatenate(parts).ravel()
    return out


def cavity_grid(nx: int, ny: Optional[int] = None) -> Grid:
    """Build-defined lid-driven cavity: unit height, dx = dy."""
    ny = nx if ny is None else ny
    return Grid(nx, ny, float(nx) / float(ny), 1.0, None)


@dataclass
class SimulationParams:                      # model.rs:13-21, defaults :44-55
    dt: float = 0.005
    viscosity: float = 0.000001
    target_inlet_velocity: float = 1.0
    velocity_scheme: VelocityScheme = VelocityScheme.FirstOrder
    inlet_profile: InletProfile = InletProfile.Uniform
    pressure_solver: PressureSolver = PressureSolver.Jacobi
    # build knobs; reference behaviour by default
    jacobi_iters: int = 50                   # model.rs:737
    corrector_passes: int = 20               # model.rs:696
    tol_enabled: bool = True                 # model.rs:816, 721
    p_tol: float = 1e-4                      # model.rs:736
    bc_kind: BoundaryKind = BoundaryKind.Channel

    def _c(self) -> CfdParams:
        return CfdParams(self.dt, self.viscosity, self.target_inlet_velocity,
                         int(self.velocity_scheme), int(self.inlet_profile),
                         int(self.pressure_solver), self.jacobi_iters, self.corrector_passes,
                         1 if self.tol_enabled else 0, self.p_tol, int(self.bc_kind))

    @staticmethod
    def cavity(reynolds: float, iters: int, lid: float = 1.0, **kw) -> "SimulationParams":
        """Lid-driven cavity, nu = U L / Re with L = 1."""
        return SimulationParams(viscosity=lid * 1.0 / reynolds, target_inlet_velocity=lid,
                                jacobi_iters=iters, bc_kind=BoundaryKind.Cavity, **kw)


@dataclass
class Residuals:                             # model.rs:23-32
    simulation_step: int
    simulation_time: float
    dt: float
    p: float
    u: float
    v: float
    step_time: float                         # seconds (device time, HIP events)
    piso_substeps: int
    jacobi_sweeps_total: int = 0


@dataclass
class SimSnapshot:                           # model.rs:36-42
    p: np.ndarray
    u: np.ndarray
    v: np.ndarray
    dt: float
    paused: bool = False


class LocalHub:
    """In-process stand-in for the RCCL communicator (testing): slabs of one
    grid driven by threads of this process (cfd_local_hub_create)."""

    def __init__(self, n_ranks: int):
        self.handle = load().cfd_local_hub_create(n_ranks)
        self.n_ranks = n_ranks

    def close(self):
        if self.handle:
            load().cfd_local_hub_destroy(self.handle)
            self.handle = None


def device_count() -> int:
    """HIP devices visible to this process (cfd_device_count)."""
    n = C.c_int()
    check("cfd_device_count", load().cfd_device_count(C.byref(n)))
    return int(n.value)


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    check("cfd_rccl_unique_id", load().cfd_rccl_unique_id(buf))
    return buf.raw


def _fp(a: Optional[np.ndarray]):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(C.POINTER(C.c_float))


class Model:
    """`Model` (model.rs:166-214) with its fields resident in HBM."""

    def __init__(self, grid: Grid, params: SimulationParams, device: int = 0, *,
                 n_ranks: int = 1, rank: int = 0, unique_id: Optional[bytes] = None,
                 local_hub: Optional["LocalHub"] = None):
        L = load()
        self.grid = grid
        self.params = params
        self._runner = None   # live SimulationControlHandle: it owns the handle
        self._h = C.c_void_p()
        g, p = grid._c(), params._c()
        if n_ranks == 1:
            check("cfd_create", L.cfd_create(C.byref(g), C.byref(p), device, C.byref(self._h)))
        elif local_hub is not None:
            check("cfd_create_sharded_local",
                  L.cfd_create_sharded_local(C.byref(g), C.byref(p), device, n_ranks, rank,
                                             local_hub.handle, C.byref(self._h)))
        else:
            check("cfd_create_sharded",
                  L.cfd_create_sharded(C.byref(g), C.byref(p), device, n_ranks, rank,
                                       unique_id, C.byref(self._h)))
        j0, j1 = C.c_uint64(), C.c_uint64()
        check("cfd_get_slab", L.cfd_get_slab(self._h, C.byref(j0), C.byref(j1)))
        self.j0, self.j1 = int(j0.value), int(j1.value)
        self.n_ranks, self.rank = n_ranks, rank

    @classmethod
    def new(cls, grid: Grid, params: SimulationParams, device: int = 0) -> "Model":
        return cls(grid, params, device)

    # ---------------------------------------------------------------- sizes
    @property
    def nyl(self) -> int:
        return self.j1 - self.j0

    def _sizes(self):
        nx, nyl = self.grid.nx, self.nyl
        return (nx + 1) * nyl, nx * (nyl + 1), nx * nyl

    # ----------------------------------------------------------------- step
    def update(self) -> None:
        """Model::update (model.rs:304-379); asynchronous."""
        check("cfd_update", load().cfd_update(self._hh()))

    def update_n(self, n: int) -> None:
        check("cfd_update_n", load().cfd_update_n(self._hh(), n))

    def piso_step(self, dt_sub: float) -> None:
        check("cfd_piso_step", load().cfd_piso_step(self._hh(), dt_sub))

    def jacobi_pressure(self) -> float:
        """jacobi_pressure (model.rs:734-824) on the current rhs / p'."""
        r = C.c_float()
        check("cfd_pressure_solve", load().cfd_pressure_solve(self._hh(), C.byref(r)))
        return float(r.value)

    def pressure_solve(self) -> float:
        """One solve of the selected pressure solver (params.pressure_solver) on
        the current rhs; returns its residual."""
        return self.jacobi_pressure()

    def run_phase(self, phase: int, dt_sub: float) -> None:
        check("cfd_run_phase", load().cfd_run_phase(self._hh(), phase, dt_sub))

    def synchronize(self) -> None:
        check("cfd_synchronize", load().cfd_synchronize(self._hh()))

    # --------------------------------------------------------------- params
    def set_parameters(self, params: SimulationParams) -> None:
        """set_parameters (model.rs:1250-1257)."""
        p = params._c()
        check("cfd_set_params", load().cfd_set_params(self._hh(), C.byref(p)))
        self.params = params

    # ---------------------------------------------------------------- reads
    def get_snapshot(self) -> SimSnapshot:
        """get_snapshot (model.rs:1259-1267)."""
        su, sv, sp = self._sizes()
        u, v, p = (np.empty(n, np.float32) for n in (su, sv, sp))
        dt = C.c_float()
        check("cfd_get_snapshot",
              load().cfd_get_snapshot(self._hh(), _fp(u), _fp(v), _fp(p), C.byref(dt)))
        return SimSnapshot(p=p, u=u, v=v, dt=float(dt.value))

    def get_residuals(self) -> Residuals:
        """get_residuals (model.rs:1269-1280)."""
        r = CfdResiduals()
        check("cfd_get_residuals", load().cfd_get_residuals(self._hh(), C.byref(r)))
        return Residuals(int(r.simulation_step), float(r.simulation_time), float(r.dt),
                         float(r.p), float(r.u), float(r.v), float(r.step_time_s),
                         int(r.piso_substeps), int(r.jacobi_sweeps_total))

    def get_state(self) -> dict:
        su, sv, sp = self._sizes()
        arrs = {k: np.empty(n, np.float32) for k, n in
                (("u", su), ("v", sv), ("p", sp), ("u_star", su), ("v_star", sv),
                 ("p_prime", sp), ("rhs", sp))}
        st = CfdState(*(_fp(arrs[k]) for k in ("u", "v", "p", "u_star", "v_star", "p_prime",
                                               "rhs")))
        check("cfd_get_state", load().cfd_get_state(self._hh(), C.byref(st)))
        arrs.update(dt=np.float32(st.dt), simulation_time=np.float32(st.simulation_time),
                    simulation_step=int(st.simulation_step),
                    last_p_residual=np.float32(st.last_p_residual),
                    last_u_residual=np.float32(st.last_u_residual),
                    last_v_residual=np.float32(st.last_v_residual),
                    jacobi_sweeps_total=int(st.jacobi_sweeps_total))
        return arrs

    def set_state(self, **kw) -> None:
        """Inject fields/scalars (any subset); others keep their values."""
        cur = self.get_state()
        arrs = {}
        for k in ("u", "v", "p", "u_star", "v_star", "p_prime", "rhs"):
            a = kw.get(k, cur[k])
            arrs[k] = np.ascontiguousarray(a, dtype=np.float32)
            if arrs[k].size != cur[k].size:
                raise ValueError(f"{k}: expected {cur[k].size} values, got {arrs[k].size}")
        st = CfdState(*(_fp(arrs[k]) for k in ("u", "v", "p", "u_star", "v_star", "p_prime",
                                               "rhs")))
        st.dt = float(kw.get("dt", cur["dt"]))
        st.simulation_time = float(kw.get("simulation_time", cur["simulation_time"]))
        st.simulation_step = int(kw.get("simulation_step", cur["simulation_step"]))
        st.last_p_residual = float(kw.get("last_p_residual", cur["last_p_residual"]))
        st.last_u_residual = float(kw.get("last_u_residual", cur["last_u_residual"]))
        st.last_v_residual = float(kw.get("last_v_residual", cur["last_v_residual"]))
        st.jacobi_sweeps_total = int(kw.get("jacobi_sweeps_total", cur["jacobi_sweeps_total"]))
        check("cfd_set_state", load().cfd_set_state(self._hh(), C.byref(st)))

    def get_masks(self):
        su, sv, _ = self._sizes()
        mu, mv = np.empty(su, np.uint8), np.empty(sv, np.uint8)
        check("cfd_get_masks", load().cfd_get_masks(
            self._hh(), mu.ctypes.data_as(C.POINTER(C.c_uint8)),
            mv.ctypes.data_as(C.POINTER(C.c_uint8))))
        return mu, mv

    # --------------------------------------------------------------- timing
    def profile_sweeps(self, n: int) -> float:
        ms = C.c_double()
        check("cfd_profile_sweeps", load().cfd_profile_sweeps(self._hh(), n, C.byref(ms)))
        return float(ms.value)

    def timing_begin(self) -> None:
        check("cfd_timing_begin", load().cfd_timing_begin(self._hh()))

    def timing_end(self):
        a, b, c, d = C.c_double(), C.c_uint64(), C.c_double(), C.c_uint64()
        check("cfd_timing_end", load().cfd_timing_end(self._hh(), C.byref(a), C.byref(b),
                                                      C.byref(c), C.byref(d)))
        return {"solve_ms": a.value, "sweeps": int(b.value), "step_ms": c.value,
                "steps": int(d.value)}

    def timing_phases(self, on: bool = True) -> None:
        """Also time the predictor and finish phases in timing windows."""
        check("cfd_timing_phases", load().cfd_timing_phases(self._hh(), 1 if on else 0))

    def timing_phase_ms(self) -> dict:
        a, b = C.c_double(), C.c_double()
        check("cfd_timing_phase_ms",
              load().cfd_timing_phase_ms(self._hh(), C.byref(a), C.byref(b)))
        return {"predict_ms": a.value, "finish_ms": b.value}

    def timing_exchange_ms(self) -> dict:
        """RCCL exchange groups + all-reduces of the last timing window with
        phases on (sharded models over RCCL; 0 otherwise)."""
        a, n = C.c_double(), C.c_uint64()
        check("cfd_timing_exchange_ms",
              load().cfd_timing_exchange_ms(self._hh(), C.byref(a), C.byref(n)))
        return {"exchange_ms": a.value, "exchanges": int(n.value)}

    @property
    def kernel_config(self) -> dict:
        fd, tb = C.c_int(), C.c_int()
        check("cfd_get_kernel_config",
              load().cfd_get_kernel_config(self._hh(), C.byref(fd), C.byref(tb)))
        return {"fastdiv": fd.value, "temporal": tb.value}

    # -------------------------------------------------------- visualisation
    def render(self, mode: "VisualizationMode" = VisualizationMode.Pressure):
        """The image App::update_simulation_view builds (app.rs:235-403),
        derived on the device: returns (rgba uint8 (nyl, nx, 4), (min, max))."""
        img = np.empty((self.nyl, self.grid.nx, 4), np.uint8)
        mm = np.empty(2, np.float32)
        check("cfd_render", load().cfd_render(
            self._hh(), int(mode), img.ctypes.data_as(C.POINTER(C.c_uint8)), _fp(mm)))
        return img, (float(mm[0]), float(mm[1]))

    def derive_field(self, mode: "VisualizationMode"):
        """The mode's scalar field (nyl, nx) f32 and its (min, max)."""
        out = np.empty((self.nyl, self.grid.nx), np.float32)
        mm = np.empty(2, np.float32)
        check("cfd_derive_field", load().cfd_derive_field(self._hh(), int(mode), _fp(out), _fp(mm)))
        return out, (float(mm[0]), float(mm[1]))

    def launches_per_solve(self) -> int:
        """Jacobi launches of one fixed-count solve, from the same host plan
        (cfd_plan_block) the runtime follows."""
        tmax = self.kernel_config["temporal"]
        iters = self.params.jacobi_iters
        hg = self.halo_depth if self.n_ranks > 1 else 0
        T, lo, hi, ex = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        it = n = 0
        while it < iters:
            check("cfd_plan_block", load().cfd_plan_block(
                self.j0, self.nyl, self.grid.ny, hg, it, tmax, iters, C.byref(T), C.byref(lo),
                C.byref(hi), C.byref(ex)))
            it += T.value
            n += 1
        return n

    @property
    def jacobi_kernel(self) -> dict:
        """Kind and rocprofv3 name of the kernel the solve launches (include/cfd.h:
        5 the LDS row march, 6 the resident tolerance-mode solve, ...)."""
        kind, name = C.c_int(), C.create_string_buffer(96)
        check("cfd_get_jacobi_kernel",
              load().cfd_get_jacobi_kernel(self._hh(), C.byref(kind), name, 96))
        return {"kind": kind.value, "name": name.value.decode()}

    def jacobi_geometry(self, persist: bool = True) -> dict:
        """Tile geometry of the 8-sweep kind-5 launch (cfd_get_jacobi_geometry):
        LDS pad bytes, workgroups per CU of the round, wave columns, segments."""
        v = [C.c_int32() for _ in range(4)]
        check("cfd_get_jacobi_geometry",
              load().cfd_get_jacobi_geometry(self._hh(), int(bool(persist)), *(C.byref(x) for x in v)))
        return dict(lds_pad=v[0].value, wgs_per_cu=v[1].value, wave_cols=v[2].value,
                    segments=v[3].value)

    @property
    def persist_steals(self) -> int:
        """Persistent-solve blocks run by a workgroup other than the tile's
        owner (cfd_get_persist_steals; 0 when every owner was resident)."""
        n = C.c_uint64()
        check("cfd_get_persist_steals", load().cfd_get_persist_steals(self._hh(), C.byref(n)))
        return int(n.value)

    @property
    def persist_sums(self) -> int:
        """Persistent-solve blocks run in the guarded SUMS form
        (cfd_get_persist_sums)."""
        n = C.c_uint64()
        check("cfd_get_persist_sums", load().cfd_get_persist_sums(self._hh(), C.byref(n)))
        return int(n.value)

    @property
    def comm_calls(self) -> int:
        """Halo-exchange groups + all-reduces enqueued (cfd_get_comm_calls)."""
        n = C.c_uint64()
        check("cfd_get_comm_calls", load().cfd_get_comm_calls(self._hh(), C.byref(n)))
        return int(n.value)

    @property
    def recoveries(self) -> int:
        """Solve timeouts the model recovered from by itself: checkpoint
        restored, calls since re-run per launch (cfd_get_recoveries)."""
        n = C.c_uint64()
        check("cfd_get_recoveries", load().cfd_get_recoveries(self._hh(), C.byref(n)))
        return int(n.value)

    @property
    def resident_solves(self) -> int:
        """Tolerance-mode solves enqueued as one resident launch
        (k_jacobi_resident; cfd_get_resident_solves)."""
        n = C.c_uint64()
        check("cfd_get_resident_solves", load().cfd_get_resident_solves(self._hh(), C.byref(n)))
        return int(n.value)

    @property
    def persist_blocks(self) -> int:
        """8-sweep blocks the last fixed-count solve ran in one persistent
        launch (k_jacobi_persist); 0 when every block had its own launch."""
        n = C.c_int()
        check("cfd_get_persist_blocks", load().cfd_get_persist_blocks(self._hh(), C.byref(n)))
        return n.value

    @property
    def comm_size(self) -> int:
        """Ranks the transport reports (ncclCommCount; LocalHub size; 1)."""
        n = C.c_int()
        check("cfd_get_comm_size", load().cfd_get_comm_size(self._hh(), C.byref(n)))
        return int(n.value)

    @property
    def halo_depth(self) -> int:
        return int(load().cfd_get_halo_depth(self._hh()))

    # ------------------------------------------------------------------ run
    def run(self) -> "SimulationControlHandle":
        """Model::run (model.rs:1282-1332): a worker thread owns the model and
        steps it while draining commands."""
        return SimulationControlHandle(self)

    def _hh(self):
        """The native handle for a direct call: refused while Model.run()'s
        worker owns it (include/cfd.h: only cfd_run_* until cfd_run_stop)."""
        if self._runner is not None:
            raise CfdError("Model", -4, "the model is owned by a running SimulationControlHandle; "
                                        "stop() it first")
        return self._h

    def close(self) -> None:
        r = getattr(self, "_runner", None)
        if r is not None:
            r.stop()   # the worker must let go of the handle before it is freed
        if getattr(self, "_h", None) and self._h.value:
            load().cfd_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SimulationControlHandle:
    """model.rs:65-117 over the native runtime (cfd_run_*, csrc/cfd_runtime.cpp):
    a C++ worker thread owns the model and steps it while draining the
    commands sent here; snapshots and residual records come back through it."""

    def __init__(self, model: Model):
        self._model = model
        self._r = C.c_void_p()
        check("cfd_run_start", load().cfd_run_start(model._hh(), C.byref(self._r)))
        model._runner = self

    def _live(self):
        if not self._r.value:
            raise CfdError("cfd_run", -4, "runner stopped")
        return self._r

    def stop(self):
        """Stop and join the worker; the model is usable again afterwards."""
        if self._r.value:
            check("cfd_run_stop", load().cfd_run_stop(self._r))
            self._r = C.c_void_p()
            if self._model._runner is self:
                self._model._runner = None

    def join(self, timeout=None):
        self.stop()

    def status(self):
        buf = C.create_string_buffer(256)
        rc = load().cfd_run_status(self._live(), buf, 256)
        return rc, buf.value.decode()

    @property
    def steps(self) -> int:
        return int(load().cfd_run_steps(self._live()))

    def get_last_available_snapshot(self) -> Optional[SimSnapshot]:
        su, sv, sp = self._model._sizes()
        u, v, p = (np.empty(n, np.float32) for n in (su, sv, sp))
        dt, paused, avail = C.c_float(), C.c_int(), C.c_int()
        check("cfd_run_last_snapshot", load().cfd_run_last_snapshot(
            self._live(), _fp(u), _fp(v), _fp(p), C.byref(dt), C.byref(paused), C.byref(avail)))
        if not avail.value:
            return None
        return SimSnapshot(p=p, u=u, v=v, dt=float(dt.value), paused=bool(paused.value))

    def get_new_log_messages(self) -> List[Residuals]:
        out: List[Residuals] = []
        buf = (CfdResiduals * 256)()
        n = C.c_int()
        while True:
            check("cfd_run_new_residuals",
                  load().cfd_run_new_residuals(self._live(), buf, 256, C.byref(n)))
            for r in buf[:n.value]:
                out.append(Residuals(int(r.simulation_step), float(r.simulation_time),
                                     float(r.dt), float(r.p), float(r.u), float(r.v),
                                     float(r.step_time_s), int(r.piso_substeps),
                                     int(r.jacobi_sweeps_total)))
            if n.value < 256:
                return out

    def request_snapshot(self):
        check("cfd_run_request_snapshot", load().cfd_run_request_snapshot(self._live()))

    def set_params(self, params: SimulationParams):
        p = params._c()
        check("cfd_run_set_params", load().cfd_run_set_params(self._live(), C.byref(p)))
        self._model.params = params

    def pause(self):
        check("cfd_run_pause", load().cfd_run_pause(self._live()))

    def resume(self):
        check("cfd_run_resume", load().cfd_run_resume(self._live()))

    def __del__(self):
        try:
            self.stop()
        except Exception:
            pass
