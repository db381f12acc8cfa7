"""CPU: the numpy restatement of the reference's visualisation
(oracle/render.py, src/app.rs:235-403) on hand-computed cases — the checker
cfd_render is held to on the GPU (tests/test_gpu_render.py)."""
import numpy as np

from render import PRESSURE, VELOCITY, VORTICITY, derive, min_max, render, sat_u8

F = np.float32


def test_sat_u8_is_rusts_saturating_cast():
    x = np.array([np.nan, -1.0, -0.0, 0.0, 0.99, 1.0, 254.99, 255.0, 300.0, np.inf, -np.inf], F)
    assert sat_u8(x).tolist() == [0, 0, 0, 0, 0, 1, 254, 255, 255, 255, 0]


def test_pressure_ramp_hand_computed():
    nx, ny = 2, 2
    p = np.array([0.0, 1.0, 2.0, 3.0], F)
    u = np.zeros(ny * (nx + 1), F)
    v = np.zeros((ny + 1) * nx, F)
    img, (mn, mx) = render(PRESSURE, u, v, p, nx, ny, 1.0, 1.0)
    assert (mn, mx) == (0.0, 3.0)
    # norm = 0, 1/3, 2/3, 1 -> r = (norm*255) as u8, b = ((1-norm)*255) as u8; in f32
    # 1 - 0.33333334 = 0.6666666 and 0.6666666 * 255 = 169.99998, truncated to 169
    assert img[..., 0].ravel().tolist() == [0, 85, 170, 255]
    assert img[..., 2].ravel().tolist() == [255, 169, 84, 0]
    assert (img[..., 1] == 0).all() and (img[..., 3] == 255).all()


def test_constant_field_widens_range_and_nan_is_ignored():
    nx, ny = 4, 2
    p = np.full(nx * ny, 2.5, F)
    p[3] = np.nan
    img, (mn, mx) = render(PRESSURE, np.zeros(ny * (nx + 1), F), np.zeros((ny + 1) * nx, F), p,
                           nx, ny, 1.0, 1.0)
    assert (mn, mx) == (2.5, 2.5)
    # range widened to 1: norm 0 everywhere -> (0, 0, 255); NaN -> norm NaN -> (0, 0, 0)
    flat = img.reshape(-1, 4)
    assert flat[0].tolist() == [0, 0, 255, 255] and flat[3].tolist() == [0, 0, 0, 255]
    assert min_max(np.full(3, np.nan, F)) == (np.inf, -np.inf)


def test_velocity_and_vorticity_hand_computed():
    nx, ny = 3, 3
    # u = y (face rows), v = 0: |vel| = cell-centred u, vorticity = -du/dy on interior
    u = np.repeat(np.arange(ny, dtype=F), nx + 1)
    v = np.zeros((ny + 1) * nx, F)
    mag = derive(VELOCITY, u, v, None, nx, ny, 0.5, 0.5)
    assert np.array_equal(mag, np.repeat(np.arange(ny, dtype=F), nx).reshape(ny, nx))
    w = derive(VORTICITY, u, v, None, nx, ny, 0.5, 0.5)
    want = np.zeros((ny, nx), F)
    want[1, 1] = -(F(2.0) - F(1.0)) / F(0.5)
    assert np.array_equal(w, want)


def test_obstacle_overlay_uses_inclusive_radius():
    nx, ny = 4, 4
    p = np.arange(16, dtype=F)
    # cell centres at 0.5, 1.5, ...; radius exactly the distance to the 4 centre cells
    r = float(np.sqrt(F(0.5) * F(0.5) + F(0.5) * F(0.5)))
    img, _ = render(PRESSURE, np.zeros(20, F), np.zeros(20, F), p, nx, ny, 1.0, 1.0,
                    cylinder=(2.0, 2.0, r))
    grey = (img[..., :3] == 128).all(-1)
    assert grey.sum() == 4 and grey[1:3, 1:3].all()
