"""The oracle's array-wise survival pieces against the literal loops they restate (CPU).

``oracle.moeva_oracle.fast_non_dominated_sort`` computes pymoo's fast-non-dominated-sort
DISCOVERY order array-wise (front k+1 ordered by the position of each member's last
dominator in front k, then by index); the survival oracle's last-front selection and niching
depend on that order, and the GPU survival is bit-exact against the oracle.  Here it is
pinned to pymoo 0.4.2.2's literal double loop (restated below from the published algorithm:
pymoo/util/nds/fast_non_dominated_sort.py + NonDominatedSorting.do's n_stop_if_ranked cut)
on integer objectives with many ties and long dominance chains.  The one-direction
vectorised get_ref_dirs_from_points and niching()'s blocked key draws are pinned likewise."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import moeva_oracle as mo  # noqa: E402


def literal_fast_nds(F, n_stop_if_ranked):
    """pymoo fast_non_dominated_sort (the i < j double loop, is_dominating lists) followed by
    NonDominatedSorting.do's n_stop_if_ranked truncation."""
    M = mo.domination_matrix(F)
    n = M.shape[0]
    is_dom = [[] for _ in range(n)]
    n_dominated = np.zeros(n, dtype=int)
    fronts, cur, n_ranked = [], [], 0
    for i in range(n):
        for j in range(i + 1, n):
            rel = M[i, j]
            if rel == 1:
                is_dom[i].append(j)
                n_dominated[j] += 1
            elif rel == -1:
                is_dom[j].append(i)
                n_dominated[i] += 1
        if n_dominated[i] == 0:
            cur.append(i)
            n_ranked += 1
    fronts.append(cur)
    while n_ranked < n:
        nxt = []
        for i in cur:
            for j in is_dom[i]:
                n_dominated[j] -= 1
                if n_dominated[j] == 0:
                    nxt.append(j)
                    n_ranked += 1
        fronts.append(nxt)
        cur = nxt
    out, nr = [], 0
    for f in fronts:
        out.append(np.asarray(f, dtype=np.int64))
        nr += len(f)
        if nr >= n_stop_if_ranked:
            break
    return out


@pytest.mark.parametrize("seed", range(12))
def test_fast_nds_equals_literal_loop(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 90))
    hi = int(rng.integers(2, 6))  # few distinct values: ties and equal rows
    F = rng.integers(0, hi, size=(n, 3)).astype(np.float64)
    if seed % 3 == 0:  # a long dominance chain on top
        F[: n // 2] = np.arange(n // 2)[:, None] + rng.integers(0, 2, size=(n // 2, 3))
    for stop in (1, n // 3 + 1, n):
        got, rank = mo.fast_non_dominated_sort(F, stop)
        ref = literal_fast_nds(F, stop)
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            np.testing.assert_array_equal(a, b)  # the exact order inside every front
        for k, f in enumerate(got):
            assert np.all(rank[f] == k)


@pytest.mark.parametrize("seed", range(4))
def test_ref_dirs_one_direction_equals_loop(seed):
    rng = np.random.default_rng(100 + seed)
    pts = rng.dirichlet(np.ones(3), size=40)
    pts[::7] *= 1e-7  # near the origin: the |dot| <= 1e-6 branch
    pts[3] = [0.9, -0.2, 0.3]  # a negative coordinate: the clip-and-renormalise branch
    asp = np.array([[1.0, 1.0, 1.0]]) / 3.0
    np.testing.assert_array_equal(mo.ref_dirs_from_points(pts, asp, 0.05),
                                  mo._ref_dirs_from_points_loop(pts, asp, 0.05))


@pytest.mark.parametrize("seed", range(6))
def test_niching_key_blocks_do_not_change_survivors(seed, monkeypatch):
    rng = np.random.default_rng(200 + seed)
    L, R = int(rng.integers(20, 120)), int(rng.integers(3, 30))
    niche_of = rng.integers(0, R, size=L)
    dist = rng.integers(0, 4, size=L).astype(np.float64)  # ties in the min distance
    count = rng.integers(0, 3, size=R)
    n_rem = int(rng.integers(1, L))
    ref = None
    for kb in (1, 3, 8, 64):
        monkeypatch.setattr(mo, "NICHE_KEY_BLOCK", kb)
        got = mo.niching(n_rem, count, niche_of, dist, 7, 5 + seed)
        assert len(set(got.tolist())) == n_rem  # distinct survivors
        if ref is None:
            ref = got
        np.testing.assert_array_equal(got, ref)
