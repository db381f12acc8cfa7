"""Independent numpy restatement of cfd-demo's Model::update hot path.

TEST INFRASTRUCTURE ONLY — never imported by the product package.  It exists
to pin the C restatement (oracle/cfd_oracle.c): the two were written
separately (this one vectorised over flat index arrays, that one as scalar
loops mirroring the reference's chunked loops) and must agree bit-for-bit.
PARITY UNPINNED against the reference itself: the Rust crate cannot be built
in this image (see DESIGN.md "Oracle").

All arithmetic is float32 with one rounding per numpy ufunc (numpy never
fuses multiply-add), matching Rust's f32 semantics.  Citations are
/root/reference/src/model.rs line numbers.
"""
from __future__ import annotations

import numpy as np

F = np.float32
ZERO = F(0.0)
HALF = F(0.5)
ONE_HALF = F(1.5)
TWO = F(2.0)


def _ld(a: np.ndarray, idx: np.ndarray) -> np.ndarray:
    """Gather a[idx] with out-of-range indices clamped.  Clamped lanes only
    ever feed the *untaken* side of an np.where, mirroring a branch the
    reference does not execute."""
    return a[np.clip(idx, 0, a.size - 1)]


class NpModel:
    """Mirror of `Model` (model.rs:166-214), flat row-major f32 fields."""

    def __init__(self, nx, ny, lx, ly, cylinder=None, dt=0.005, viscosity=1e-6,
                 target_inlet_velocity=1.0, scheme=0, inlet_profile=0,
                 jacobi_iters=50, corrector_passes=20, tol_enabled=True,
                 p_tol=1e-4, bc_kind=0):
        assert nx % 8 == 0
        self.nx, self.ny = nx, ny
        self.lx, self.ly = F(lx), F(ly)
        self.dx = F(self.lx / F(nx))
        self.dy = F(self.ly / F(ny))
        self.dt = F(dt)
        self.nu = F(viscosity)
        self.target = F(target_inlet_velocity)
        self.scheme = scheme
        self.profile = inlet_profile
        self.jacobi_iters = jacobi_iters
        self.corrector_passes = corrector_passes
        self.tol_enabled = bool(tol_enabled)
        self.p_tol = F(p_tol)
        self.bc_kind = bc_kind
        su, sv, sp = (nx + 1) * ny, nx * (ny + 1), nx * ny
        z = lambda n: np.zeros(n, dtype=F)
        self.u, self.v, self.p = z(su), z(sv), z(sp)
        self.u_old, self.v_old = z(su), z(sv)
        self.u_star, self.v_star = z(su), z(sv)
        self.rhs, self.pp, self.ppn = z(sp), z(sp), z(sp)
        self.mask_u = np.zeros(su, dtype=np.uint8)
        self.mask_v = np.zeros(sv, dtype=np.uint8)
        self.obstacle = []
        if cylinder is not None:  # model.rs:235-260
            cx, cy, r = (F(c) for c in cylinder)
            jj, ii = np.meshgrid(np.arange(ny), np.arange(nx), indexing="ij")
            x = (ii.astype(F) + HALF) * self.dx
            y = (jj.astype(F) + HALF) * self.dy
            ddx, ddy = x - cx, y - cy
            dist = np.sqrt(ddx * ddx + ddy * ddy)
            inside = dist < r
            ci, cj = ii[inside], jj[inside]
            self.mask_u[(ci + cj * (nx + 1))[ci > 0]] = 1
            self.mask_u[((ci + 1) + cj * (nx + 1))[ci < nx]] = 1
            self.mask_v[(ci + cj * nx)[cj > 0]] = 1
            self.mask_v[(ci + (cj + 1) * nx)[cj < ny]] = 1
            # row-major (j outer, i inner) order as the reference pushes them
            order = np.lexsort((ci, cj))
            self.obstacle = list(zip(ci[order].tolist(), cj[order].tolist()))
        self.step = 0
        self.time = F(0.0)
        self.inlet = F(0.0)
        self.res_p = F(0.0)
        self.res_u = F(0.0)
        self.res_v = F(0.0)
        self.sweeps = 0

    # ------------------------------------------------------------ predictors
    def u_predictor(self, dt):
        """u* on rows 1..=ny-2, faces 1..=nx (model.rs:538-580, 381-436)."""
        nx, ny = self.nx, self.ny
        u, v = self.u, self.v
        W = nx + 1
        J, I = np.meshgrid(np.arange(1, ny - 1), np.arange(1, nx + 1), indexing="ij")
        I, J = I.ravel(), J.ravel()
        c = I + J * W
        uc, ue1, uw1 = u[c], u[c + 1], u[c - 1]
        un1, us1 = u[c + W], u[c - W]
        vn = v[I + (J + 1) * nx]           # get_v_north, not averaged
        vs = v[I + J * nx]                 # get_v_south
        if self.scheme == 0:
            ue = np.where((uc + ue1) * HALF >= ZERO, uc, ue1)
            uw = np.where((uw1 + uc) * HALF >= ZERO, uw1, uc)
            un = np.where(vn >= ZERO, uc, un1)
            us = np.where(vs >= ZERO, us1, uc)
        else:
            # east face (model.rs:911-926)
            e_pos = np.where(I > 1, ONE_HALF * uc - HALF * _ld(u, c - 1), uc)
            e_neg = np.where(I < nx - 1, ONE_HALF * ue1 - HALF * _ld(u, c + 2), ue1)
            ue = np.where(uc >= ZERO, e_pos, e_neg)
            # west face (model.rs:944-963)
            w_pos = np.where(I > 2, ONE_HALF * uw1 - HALF * _ld(u, c - 2), uw1)
            w_neg = np.where(I < nx, ONE_HALF * uc - HALF * ue1, uc)
            uw = np.where(uw1 >= ZERO, w_pos, w_neg)
            # north face (model.rs:992-1008): decision on averaged v
            vnb = HALF * (v[(I - 1) + (J + 1) * nx] + v[I + (J + 1) * nx])
            n_pos = np.where(J > 1, ONE_HALF * uc - HALF * _ld(u, c - W), uc)
            n_neg = np.where(J <= ny - 3, ONE_HALF * un1 - HALF * _ld(u, c + 2 * W), un1)
            un = np.where(vnb >= ZERO, n_pos, n_neg)
            # south face (model.rs:1037-1053)
            vsb = HALF * (v[(I - 1) + J * nx] + v[I + J * nx])
            s_pos = np.where(J > 1, ONE_HALF * us1 - HALF * _ld(u, c - 2 * W), us1)
            s_neg = ONE_HALF * uc - HALF * un1
            us = np.where(vsb >= ZERO, s_pos, s_neg)
        dx, dy, nu = self.dx, self.dy, self.nu
        conv = (ue * ue - uw * uw) / dx + (vn * un - vs * us) / dy
        lap = (ue1 - TWO * uc + uw1) / (dx * dx) + (un1 - TWO * uc + us1) / (dy * dy)
        us_new = uc + dt * (-conv + nu * lap)
        us_new = np.where(self.mask_u[c] == 1, ZERO, us_new)
        self.u_star[c] = us_new

    def v_predictor(self, dt):
        """v* on rows 1..=ny-1, cols 1..=nx-1 (model.rs:586-670, 438-521)."""
        nx, ny = self.nx, self.ny
        u, v = self.u, self.v
        W = nx + 1
        J, I = np.meshgrid(np.arange(1, ny), np.arange(1, nx), indexing="ij")
        I, J = I.ravel(), J.ravel()
        c = I + J * nx
        vc, ve1, vw1, vn1, vs1 = v[c], v[c + 1], v[c - 1], v[c + nx], v[c - nx]
        uE = u[(I + 1) + J * W]
        uW = u[I + J * W]
        if self.scheme == 0:
            ve = np.where(uE >= ZERO, vc, ve1)
            vw = np.where(uW >= ZERO, vw1, vc)
            vn = np.where(HALF * (vc + vn1) >= ZERO, vc, vn1)
            vs = np.where(HALF * (vs1 + vc) >= ZERO, vs1, vc)
        else:
            e_pos = np.where(I > 0, ONE_HALF * vc - HALF * vw1, vc)
            e_neg = np.where(I < nx - 2, ONE_HALF * ve1 - HALF * _ld(v, c + 2), ve1)
            ve = np.where(uE >= ZERO, e_pos, e_neg)
            w_pos = np.where(I > 1, ONE_HALF * vw1 - HALF * _ld(v, c - 2), vw1)
            w_neg = np.where(I < nx - 1, ONE_HALF * vc - HALF * ve1, vc)
            vw = np.where(uW >= ZERO, w_pos, w_neg)
            n_pos = np.where(J > 1, ONE_HALF * vc - HALF * _ld(v, c - nx), vc)
            n_neg = np.where(J <= ny - 2, ONE_HALF * vn1 - HALF * _ld(v, c + 2 * nx), vn1)
            vn = np.where(HALF * (vc + vn1) >= ZERO, n_pos, n_neg)
            s_pos = np.where(J > 1, ONE_HALF * vs1 - HALF * _ld(v, c - 2 * nx), vs1)
            s_neg = ONE_HALF * vc - HALF * vn1
            vs = np.where(HALF * (vs1 + vc) >= ZERO, s_pos, s_neg)
            # column nx-1: the lane is never filled (model.rs:647-650)
            last = I == nx - 1
            uE = np.where(last, ZERO, uE)
            uW = np.where(last, ZERO, uW)
            ve = np.where(last, ZERO, ve)
            vw = np.where(last, ZERO, vw)
            vn = np.where(last, ZERO, vn)
            vs = np.where(last, ZERO, vs)
        dx, dy, nu = self.dx, self.dy, self.nu
        conv = (uE * ve - uW * vw) / dx + (vn * vn - vs * vs) / dy
        lap = (ve1 - TWO * vc + vw1) / (dx * dx) + (vn1 - TWO * vc + vs1) / (dy * dy)
        out = vc + dt * (-conv + nu * lap)
        out = np.where(self.mask_v[c] == 1, ZERO, out)
        self.v_star[c] = out

    # ------------------------------------------------------------ pressure
    def divergence(self, dt):
        """model.rs:1406-1440."""
        nx, ny = self.nx, self.ny
        us = self.u_star.reshape(ny, nx + 1)
        vs = self.v_star.reshape(ny + 1, nx)
        rhs = ((us[:, 1:] - us[:, :-1]) / self.dx + (vs[1:, :] - vs[:-1, :]) / self.dy) / dt
        self.rhs[:] = rhs.ravel()

    def jacobi(self):
        """Weighted Jacobi, omega 0.75 (model.rs:734-824)."""
        nx, ny = self.nx, self.ny
        dx2, dy2 = self.dx * self.dx, self.dy * self.dy
        omega = F(0.75)
        om1 = F(1.0) - omega
        denom = TWO / (self.dx * self.dx) + TWO / (self.dy * self.dy)
        J, I = np.meshgrid(np.arange(1, ny - 1), np.arange(1, nx), indexing="ij")
        c = (I + J * nx).ravel()
        # residual columns: full 8-lane chunks only (1..=nx-8)
        res_cols = (I.ravel() <= nx - 8)
        rhs = self.rhs[c]
        err = F(0.0)
        for _ in range(self.jacobi_iters):
            P = self.pp
            new = omega * (((P[c + 1] + P[c - 1]) / dx2 + (P[c + nx] + P[c - nx]) / dy2 - rhs)
                           / denom) + om1 * P[c]
            e = np.abs(new - P[c])[res_cols]
            err = F(np.fmax.reduce(e, initial=F(0.0))) if e.size else F(0.0)
            self.ppn[c] = new
            self.pp, self.ppn = self.ppn, self.pp
            P = self.pp.reshape(ny, nx)
            P[0, :] = P[1, :]
            P[ny - 1, :] = P[ny - 2, :]
            P[:, 0] = P[:, 1]
            P[:, nx - 1] = ZERO
            self.sweeps += 1
            if self.tol_enabled and err < self.p_tol:
                break
        self.res_p = err
        return err

    def corrector(self, dt):
        """model.rs:1334-1404 (tail columns nx-7..nx-1 associate (dt*dp)/dx)."""
        nx, ny = self.nx, self.ny
        P = self.pp.reshape(ny, nx)
        U = self.u.reshape(ny, nx + 1)
        Us = self.u_star.reshape(ny, nx + 1)
        dp = P[:, 1:] - P[:, :-1]                     # cols 1..nx-1
        body = Us[:, 1:nx] - dt * (dp / self.dx)
        tail = Us[:, 1:nx] - (dt * dp) / self.dx
        cols = np.arange(1, nx)
        U[:, 1:nx] = np.where(cols[None, :] >= nx - 7, tail, body)
        V = self.v.reshape(ny + 1, nx)
        Vs = self.v_star.reshape(ny + 1, nx)
        V[1:ny, :] = Vs[1:ny, :] - dt * ((P[1:, :] - P[:-1, :]) / self.dy)
        self.p += self.pp

    def boundary(self):
        """model.rs:826-875 (channel); bc_kind 1 = build-defined cavity."""
        nx, ny = self.nx, self.ny
        U = self.u.reshape(ny, nx + 1)
        V = self.v.reshape(ny + 1, nx)
        if self.bc_kind == 0:
            if self.profile == 0:
                U[:, 0] = self.inlet
            else:
                y = (np.arange(ny).astype(F) + HALF) * self.dy
                center = self.ly / TWO
                radius = self.ly / TWO
                t = (y - center) / radius
                val = self.inlet * (F(1.0) - t * t)
                U[:, 0] = np.where(val < ZERO, ZERO, val)
            U[:, nx] = U[:, nx - 1]
            U[0, :] = ZERO
            U[ny - 1, :] = ZERO
        else:
            U[:, 0] = ZERO
            U[:, nx] = ZERO
            U[0, :] = ZERO
            U[ny - 1, :] = ZERO
            U[ny - 1, 1:nx] = self.inlet
        V[0, :] = ZERO
        V[ny, :] = ZERO
        for (i, j) in self.obstacle:
            U[j, i] = ZERO
            V[j, i] = ZERO

    # ----------------------------------------------------------------- step
    def piso_step(self, dt):
        self.u_predictor(dt)
        self.v_predictor(dt)
        self.divergence(dt)
        self.jacobi()
        self.corrector(dt)
        for _ in range(self.corrector_passes):
            self.u_star[:] = self.u
            self.v_star[:] = self.v
            self.divergence(dt)
            self.jacobi()
            self.corrector(dt)
            if self.tol_enabled and self.res_p < self.p_tol:
                break
        self.boundary()

    def update(self):
        """model.rs:304-379."""
        self.u_old[:] = self.u
        self.v_old[:] = self.v
        if self.step < 100:
            self.inlet = F(F(self.step) / F(100.0)) * self.target
        else:
            self.inlet = self.target
        dt = self.dt
        self.piso_step(dt)
        self.res_u = F(np.fmax.reduce(np.abs(self.u - self.u_old), initial=F(0.0)))
        self.res_v = F(np.fmax.reduce(np.abs(self.v - self.v_old), initial=F(0.0)))
        self.step += 1
        self.time = F(self.time + self.dt)
        mu = np.fmax.reduce(np.abs(self.u), initial=F(0.0))
        mv = np.fmax.reduce(np.abs(self.v), initial=F(0.0))
        mvel = F(max(mu, mv))
        if mvel == ZERO:
            new_dt = self.dt
        else:
            new_dt = F(min(F(F(0.2) * F(min(self.dx, self.dy))) / mvel, self.dt))
        self.dt = new_dt
