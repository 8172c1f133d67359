"""The near-tie analysis of tests/dtw_neartie.py on CPU (no GPU): the cheapest path through a
DTW result's own token entries is that result's optimal path (margin 0), and entries moved off
the optimum cost more."""
import numpy as np

from oracle import dtw as odtw
from tests.dtw_neartie import _anchors, anchored_path


def test_anchored_path_reproduces_the_optimum():
    rng = np.random.default_rng(0)
    for _ in range(20):
        rows, cols = rng.integers(3, 12), rng.integers(20, 80)
        x = rng.standard_normal((rows, cols)).astype(np.float32)
        ti, tj = odtw.dtw(x)
        a = _anchors(ti, tj, 0)
        p = anchored_path(x, [t // 2 for t in a])
        assert p is not None
        opt = float(x[ti, tj].astype(np.float64).sum())
        got = float(x[p[0], p[1]].astype(np.float64).sum())
        assert abs(got - opt) <= 1e-4 * max(1.0, abs(opt)), (got, opt)
        # moving one entry cannot make the path cheaper than the optimum
        if len(a) > 1:
            b = list(a)
            k = int(rng.integers(0, len(b)))
            lo = b[k - 1] if k > 0 else 0
            hi = b[k + 1] if k + 1 < len(b) else 2 * (cols - 1)
            b[k] = int(rng.integers(lo // 2, hi // 2 + 1)) * 2
            q = anchored_path(x, [t // 2 for t in b])
            if q is not None:
                assert float(x[q[0], q[1]].astype(np.float64).sum()) >= opt - 1e-4 * max(1.0, abs(opt))


def test_anchored_path_rejects_non_monotone_entries():
    x = np.zeros((3, 10), np.float32)
    assert anchored_path(x, [5, 3]) is None
    assert anchored_path(x, [2]) is None          # wrong row count
