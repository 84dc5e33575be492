"""CPU check of the rewrite behind the coefs=2 sweep's clusters (csrc/tfp_scan.hip, CellCache
c_lo/c_hi): a group's max2 points cut only at gaps wider than dgap = floor(2 tol 1e6) - 3
micro-units, and each cluster searched by its first and last point, hit exactly the frames that
one of the points hits, for every frame window the reference builds at that tolerance:
[fmt6(q2 - tol), fmt6(q2 + tol)] (src/fp_handler.c:339-347, "%f" = oracle fmt6). Brute force over
random and adversarial point sets and windows; no GPU.
"""
import math

import numpy as np
import pytest

import oracle_py as oracle


def _clusters(pts, dgap):
    out = []
    for v in pts:
        if out and v - out[-1][1] <= dgap:
            out[-1][1] = v
        else:
            out.append([v, v])
    return out


def _window(q2, tol):
    return oracle.fmt6(q2 - tol), oracle.fmt6(q2 + tol)


@pytest.mark.parametrize("tol", [0.0, 0.000004, 0.0005, 0.001, 0.0105, 0.1, 0.3, 0.45])
def test_clusters_hit_exactly_what_points_hit(tol):
    rng = np.random.default_rng(int(tol * 1e6) + 11)
    dgap = max(0, math.floor(2 * tol * 1e6) - 3)
    w = 2 * tol * 1e6
    checked = 0
    for trial in range(60):
        n = int(rng.integers(1, 40))
        base = int(rng.integers(-40_000_000, 40_000_000))
        # gaps around dgap (and around the window width), duplicates and wide gaps
        choices = [0, 1, max(dgap - 1, 0), dgap, dgap + 1, dgap + 2, dgap + 3, int(w), int(w) + 1, 2 * dgap + 5,
                   int(rng.integers(0, 3 * dgap + 10))]
        gaps = [choices[int(rng.integers(len(choices)))] for _ in range(n - 1)]
        pts = np.cumsum([base] + gaps).tolist()
        cl = _clusters(pts, dgap)
        lo, hi = pts[0] - int(w) - 20, pts[-1] + int(w) + 20
        xs = set(rng.integers(lo, hi + 1, 300).tolist())
        for v in pts:  # windows whose ends sit at the points
            for d in range(-3, 4):
                xs.add(v + int(w / 2) + d)
                xs.add(v - int(w / 2) + d)
        for x in xs:
            for frac in (0.0, 0.3, 0.5, 0.8):
                q2 = (x + frac) / 1e6
                L2, U2 = _window(q2, tol)
                assert U2 - L2 >= dgap  # the sweep checks this per batch (else it searches the points)
                by_points = any(L2 <= v <= U2 for v in pts)
                by_clusters = any(L2 <= c[1] and U2 >= c[0] for c in cl)
                assert by_points == by_clusters, (tol, pts, cl, q2, L2, U2)
                checked += 1
    assert checked > 10000
