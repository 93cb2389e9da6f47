"""CPU restatement of the pruned exact 5-NN of k_sdf_front (csrc/anr_sdf.hip) checked
against brute force: Morton-ordered cells of 64 vertices with bounding boxes, cells visited by box
distance from the ray's middle sample, a cell skipped when its fp32 box bound exceeds every lane's
5th-best d^2, lexicographic (d^2, index) insertion. The claim under test: the result equals the K
smallest (d^2, index) pairs (pytorch3d knn_points' heap result, index order on ties) exactly, with
d^2 = (dx*dx + dy*dy) + dz*dz in fp32 and no margin on the bound. The GPU kernel itself is checked by
tests/test_gpu_sdf.py (goldens G6/G7, the 600-duplicate tie test)."""
import numpy as np

K = 5
CELL = 64


def _d2(p, v):
    d = (p[:, None, :] - v[None, :, :]).astype(np.float32)
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def _box_d2(p, lo, hi):
    d = np.where(p < lo, p - lo, np.where(p > hi, p - hi, np.float32(0))).astype(np.float32)
    return (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]


def _cells(v):
    mn, mx = v.min(0), v.max(0)
    q = np.clip(((v - mn) * (np.float32(63.99) / (mx - mn))).astype(np.int64), 0, 63)
    code = np.zeros(len(v), np.int64)
    for b in range(6):
        for c in range(3):
            code |= ((q[:, c] >> b) & 1) << (3 * b + c)
    order = np.argsort((code << 13) | np.arange(len(v)), kind='stable')
    cells = [order[i:i + CELL] for i in range(0, len(v), CELL)]
    return cells, np.array([v[c].min(0) for c in cells]), np.array([v[c].max(0) for c in cells])


def _pruned_knn(P, v, cells, lo, hi):
    """One 'wave' = the rows of P; returns (d2, idx) of the K best per row and the cells visited."""
    best_d = np.full((len(P), K), np.inf, np.float32)
    best_i = np.zeros((len(P), K), np.int64)
    pm = P[len(P) // 2]
    order = np.argsort([_box_d2(pm, lo[c], hi[c]) for c in range(len(cells))], kind='stable')
    visited = 0
    for c in order:
        if not np.any(_box_d2(P, lo[c], hi[c]) <= best_d[:, K - 1]):
            continue
        visited += 1
        idx = cells[c]
        d = _d2(P, v[idx])
        for r in range(len(P)):  # lexicographic (d2, index) merge
            cand = list(zip(best_d[r], best_i[r])) + list(zip(d[r], idx))
            cand = [x for x in cand if np.isfinite(x[0])]
            cand.sort(key=lambda x: (x[0], x[1]))
            cand = cand[:K]
            for k in range(K):
                best_d[r, k], best_i[r, k] = cand[k] if k < len(cand) else (np.inf, 0)
    return best_d, best_i, visited


def test_pruned_knn_equals_bruteforce_with_ties():
    rng = np.random.Generator(np.random.PCG64(17))
    n = 640
    u = rng.standard_normal((n, 3))
    v = (u / np.linalg.norm(u, axis=1, keepdims=True) * [0.25, 0.85, 0.15]).astype(np.float32)
    dup = rng.choice(n // 2, 120, replace=False)
    v[n // 2 + rng.choice(n // 2, 120, replace=False)] = v[dup]  # exact d^2 ties
    cells, lo, hi = _cells(v)
    visited_total = 0
    for ray in range(12):
        o = np.array([0.0, 0.0, 3.0], np.float32)
        t = (rng.uniform(-1, 1, 3) * [0.3, 0.9, 0.2]).astype(np.float32)
        dirn = (t - o) / np.linalg.norm(t - o)
        z = np.linspace(2.5, 3.5, 64, dtype=np.float32)
        P = (o[None] + dirn[None] * z[:, None]).astype(np.float32)
        bd, bi, visited = _pruned_knn(P, v, cells, lo, hi)
        visited_total += visited
        d = _d2(P, v)
        ref = np.lexsort((np.broadcast_to(np.arange(n), d.shape), d), axis=1)[:, :K]
        assert np.array_equal(bi, ref)
        assert np.array_equal(bd, np.take_along_axis(d, ref, 1))
    assert visited_total < 12 * len(cells)  # the bound prunes


def test_box_bound_never_exceeds_member_distance():
    """The monotonicity argument for a margin-free bound, on adversarial fp32 inputs."""
    rng = np.random.Generator(np.random.PCG64(3))
    v = (rng.standard_normal((4096, 3)) * 10.0 ** rng.integers(-6, 2, (4096, 1))).astype(np.float32)
    P = (rng.standard_normal((256, 3)) * 10.0 ** rng.integers(-6, 2, (256, 1))).astype(np.float32)
    for c in range(0, 4096, 64):
        m = v[c:c + 64]
        b = _box_d2(P, m.min(0), m.max(0))
        assert np.all(b[:, None] <= _d2(P, m))
