"""numpy restatement of the reference's visualisation (src/app.rs:235-403,
App::update_simulation_view): the derived scalar field of each
VisualizationMode (app.rs:505-509), its min/max and the RGB ramp with the
obstacle overlay.

TEST INFRASTRUCTURE ONLY (checker for cfd_render / cfd_derive_field): never
imported by the product package.  f32 throughout, one IEEE operation per
Rust operation (numpy does not contract), correctly rounded sqrt/division.
PARITY UNPINNED against the reference itself (no Rust toolchain here, and
the reference has no rendering fixtures): this follows the source text.
"""
import numpy as np

F = np.float32
PRESSURE, VELOCITY, VORTICITY = 0, 1, 2


def derive(mode, u, v, p, nx, ny, dx, dy):
    """The mode's scalar field, shape (ny, nx) (app.rs:237-245, 282-305, 339-360)."""
    u = np.asarray(u, F).reshape(ny, nx + 1)
    v = np.asarray(v, F).reshape(ny + 1, nx)
    if mode == PRESSURE:
        return np.asarray(p, F).reshape(ny, nx).copy()
    if mode == VELOCITY:                                   # app.rs:290-303
        u_cell = F(0.5) * (u[:, :-1] + u[:, 1:])
        v_cell = F(0.5) * (v[:-1, :] + v[1:, :])
        return np.sqrt(u_cell * u_cell + v_cell * v_cell)
    vort = np.zeros((ny, nx), F)                           # app.rs:343-360
    if ny > 2 and nx > 2:
        i = slice(1, nx - 1)
        ip = slice(2, nx)
        j, jp = slice(1, ny - 1), slice(2, ny)
        u_bottom = F(0.5) * (u[j, i] + u[j, ip])
        u_top = F(0.5) * (u[jp, i] + u[jp, ip])
        du_dy = (u_top - u_bottom) / F(dy)
        v_left = F(0.5) * (v[j, i] + v[jp, i])
        v_right = F(0.5) * (v[j, ip] + v[jp, ip])
        dv_dx = (v_right - v_left) / F(dx)
        vort[j, i] = dv_dx - du_dy
    return vort


def min_max(field):
    """`if x < min_val` / `if x > max_val` scans from +inf / -inf: NaN ignored."""
    a = np.asarray(field, F).ravel()
    a = a[~np.isnan(a)]
    if a.size == 0:
        return F(np.inf), F(-np.inf)
    return F(a.min()), F(a.max())


def sat_u8(x):
    """Rust `f as u8`: saturating, NaN -> 0, truncation toward zero."""
    x = np.asarray(x, F)
    out = np.zeros(x.shape, np.uint8)
    ok = x > 0
    out[ok] = np.minimum(np.trunc(x[ok]), F(255)).astype(np.uint8)
    return out


def render(mode, u, v, p, nx, ny, dx, dy, cylinder=None):
    """RGBA8 image (ny, nx, 4) and (min, max) before the 1e-6 widening."""
    field = derive(mode, u, v, p, nx, ny, dx, dy)
    mn, mx = min_max(field)
    lo, hi = mn, mx
    if abs(F(hi - lo)) < F(1e-6):                          # app.rs:252-254
        hi = F(lo + F(1.0))
    norm = (field - lo) / F(hi - lo)
    img = np.zeros((ny, nx, 4), np.uint8)
    img[..., 0] = sat_u8(norm * F(255.0))
    img[..., 2] = sat_u8((F(1.0) - norm) * F(255.0))
    img[..., 3] = 255
    if cylinder is not None:                               # app.rs:262-277
        cx, cy, r = (F(c) for c in cylinder)
        x = (np.arange(nx, dtype=F) + F(0.5)) * F(dx)
        y = (np.arange(ny, dtype=F) + F(0.5)) * F(dy)
        ddx = (x - cx)[None, :]
        ddy = (y - cy)[:, None]
        inside = np.sqrt(ddx * ddx + ddy * ddy) <= r
        img[inside] = (128, 128, 128, 255)
    return img, (mn, mx)
