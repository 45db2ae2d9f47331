"""The hull support cells (collide_x.h hull_support_cells / hull_cell; the step kernel's
support search over a hull scans only its direction cell's candidate vertices): on CPU, through
the host builder exported by the narrow-phase harness (tools/libxcheck.so, xcheck_cells), for
random directions - spread over the sphere and concentrated at cell edges and cube corners - the
first maximal vertex of the fp32 scan over ALL vertices is a candidate of the direction's cell,
and so is every vertex tied with it, so the candidate scan returns the same vertex; and the
exact (fp64) maximiser is a candidate too."""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

LIB = Path(__file__).resolve().parents[1] / "tools" / "libxcheck.so"


def _lib():
    if not LIB.exists():
        pytest.skip("tools/libxcheck.so not built (__graft_entry__.build)")
    lib = C.CDLL(str(LIB))
    lib.xcheck_cells.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    return lib


def hull_cell(d, G):
    """collide_x.h hull_cell, restated (fp32 like the kernel)."""
    d = np.asarray(d, np.float32)
    e = np.abs(d)
    if e[0] >= e[1] and e[0] >= e[2]:
        ax, mj, a, b = 0, d[0], d[1], d[2]
    elif e[1] >= e[2]:
        ax, mj, a, b = 1, d[1], d[2], d[0]
    else:
        ax, mj, a, b = 2, d[2], d[0], d[1]
    inv = np.float32(1.0) / np.float32(abs(mj))
    hg = np.float32(0.5 * G)
    ia = int(min(max(np.float32(a * inv + np.float32(1.0)) * hg, 0.0), G - 1.0))
    ib = int(min(max(np.float32(b * inv + np.float32(1.0)) * hg, 0.0), G - 1.0))
    return ((2 * ax + (1 if mj < 0 else 0)) * G + ia) * G + ib


def _hulls(dp):
    from helpers import capsule_points
    out = []
    for r, hl in ((0.0085, 0.006), (0.01, 0.0), (0.006, 0.012)):
        _, v = dp.mjcf.convex_hull_collider(capsule_points(r, hl))
        out.append(v)
    rng = np.random.RandomState(3)
    p = rng.normal(size=(200, 3)) * (0.02, 0.01, 0.005)
    out.append(dp.mjcf.convex_hull_collider(p)[1][:64])
    cube = np.array([[x, y, z] for x in (-1, 1) for y in (-1, 1) for z in (-1, 1)], float) * 0.01
    out.append(cube)
    return out


def _dirs(rng, n):
    d = rng.normal(size=(n, 3))
    # cell edges and cube edges / corners: ratios at exact cell boundaries, axis-aligned, ties
    k = rng.randint(0, 5, size=(n // 2, 3)) / 2.0 - 1.0
    e = k * rng.choice([1.0, -1.0], size=(n // 2, 3)) + rng.normal(size=(n // 2, 3)) * 1e-7 * rng.randint(0, 2, (n // 2, 1))
    return np.concatenate([d, e]).astype(np.float32)


def test_support_cells_keep_the_support(dp):
    lib = _lib()
    G = lib.xcheck_cell_grid()
    rng = np.random.RandomState(0)
    for v in _hulls(dp):
        v32 = np.asarray(v, np.float32)
        n = len(v32)
        cells = np.zeros(6 * G * G, np.uint64)
        assert lib.xcheck_cells(np.ascontiguousarray(v32.astype(np.float64)).ctypes.data, n, cells.ctypes.data) == 6 * G * G
        sizes = [bin(int(c)).count("1") for c in cells]
        assert min(sizes) >= 1
        for d in _dirs(rng, 4000):
            if not d.any():
                continue
            m = int(cells[hull_cell(d, G)])
            p32 = (np.float32(d[2]) * v32[:, 2] + (np.float32(d[1]) * v32[:, 1] + np.float32(d[0]) * v32[:, 0])).astype(np.float32)
            best = p32.max()
            for i in np.nonzero(p32 == best)[0]:  # the fp32 maximiser and every vertex tied with it
                assert (m >> int(i)) & 1, (d, i, bin(m))
            i64 = int(np.argmax(v32.astype(np.float64) @ d.astype(np.float64)))
            assert (m >> i64) & 1, (d, i64)
        print(f"{n} vertices: candidates per cell mean {np.mean(sizes):.1f} max {max(sizes)}")
