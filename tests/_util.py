"""Shared helpers for the test-suite (test infrastructure only)."""
import numpy as np

STATE_FIELDS = ("u", "v", "p", "u_star", "v_star", "p_prime")


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).ravel()


def assert_bitwise(name, got, want, nan_equal=False):
    """Every f32 word identical.  nan_equal: any NaN matches any NaN (the
    sign/payload of a NaN produced by arithmetic is the hardware's default
    NaN, not part of the reference's semantics)."""
    assert np.shape(got) == np.shape(want), f"{name}: shape {np.shape(got)} != {np.shape(want)}"
    g, w = bits(got), bits(want)
    ne = g != w
    if nan_equal:
        ne &= ~(np.isnan(g.view(np.float32)) & np.isnan(w.view(np.float32)))
    bad = np.nonzero(ne)[0]
    if bad.size:
        k = bad[0]
        raise AssertionError(
            f"{name}: {bad.size}/{g.size} words differ; first at {k}: got "
            f"{np.float32(got.ravel()[k])!r} want {np.float32(want.ravel()[k])!r}")


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    n = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (n if n > 0 else 1.0))
