"""CPU checks of the ISS / cloud-resolution restatement (oracle/or_keypoints.cpp) itself
(SURVEY 8(f) F3).  Parity vs real PCL/Eigen is unpinned (no PCL anywhere in this pipeline, no
reference tests for this path); these pin the restatement by independent arithmetic:

* Eigen 3.2.0 SelfAdjointEigenSolver<Matrix3d>: eigenvalues within 1e-14 (relative to the
  largest) of LAPACK's (numpy.linalg.eigvalsh) on random symmetric matrices, exact on diagonal,
  zero, repeated and rank-1 matrices;
* computeCloudResolution: per-point terms bit-identical to an exhaustive numpy FLANN-order
  kNN (sequential float L2_Simple, float sqrt), the mean equal to a Python sequential double
  loop; duplicates give 0-length terms, a single point gives 0;
* ISS: every keypoint is a candidate (third > 0) and a local maximum of the third eigenvalue
  within the non-max radius with >= min_neighbors neighbours (checked by numpy), and every
  non-keypoint candidate fails one of those; third values equal a numpy restatement of the
  scatter matrix (sequential double sums in FLANN order) fed to the same solver.
"""
import numpy as np
import pytest

import oracle_lib as O


def _flann_d2(P, Q):
    dx = Q[:, None, 0] - P[None, :, 0]
    dy = Q[:, None, 1] - P[None, :, 1]
    dz = Q[:, None, 2] - P[None, :, 2]
    return ((np.float32(0) + dx * dx) + dy * dy) + dz * dz


def test_eigen_random_vs_lapack():
    rng = np.random.default_rng(1)
    A = rng.normal(size=(4000, 3, 3)) * rng.uniform(1e-6, 1e3, size=(4000, 1, 1))
    A = A + A.transpose(0, 2, 1)
    ev = O.eigen_selfadjoint3(A)
    ref = np.linalg.eigvalsh(A)
    scale = np.abs(ref).max(axis=1, keepdims=True)
    assert np.all(np.abs(ev - ref) <= 1e-14 * scale)
    assert np.all(np.diff(ev, axis=1) >= 0)  # ascending


def test_eigen_vectors_random_vs_lapack():
    """The eigenvector half (Householder Q x Givens rotations) used by SHOT's LRF: orthonormal,
    A v = lambda v, equal to LAPACK's up to sign where the spectrum is separated, and the
    values bit-identical to the values-only path (the vectors never feed back)."""
    rng = np.random.default_rng(5)
    A = rng.normal(size=(3000, 3, 3)) * rng.uniform(1e-6, 1e3, size=(3000, 1, 1))
    A = A + A.transpose(0, 2, 1)
    ev, vec = O.eigen_selfadjoint3_vectors(A)
    assert np.array_equal(ev, O.eigen_selfadjoint3(A))
    scale = np.abs(ev).max(axis=1)
    for i in range(len(A)):
        V = vec[i].T   # columns = eigenvectors
        assert np.allclose(V.T @ V, np.eye(3), atol=1e-13)
        assert np.allclose(A[i] @ V, V * ev[i], atol=1e-12 * scale[i])
    w, U = np.linalg.eigh(A)
    gap = np.minimum(np.diff(w, axis=2 - 1)[:, 0], np.diff(w, axis=1)[:, 1]) / scale
    sep = gap > 1e-3
    for i in np.nonzero(sep)[0][:500]:
        for k in range(3):
            assert abs(abs(np.dot(vec[i, k], U[i][:, k])) - 1.0) < 1e-9


def test_eigen_vectors_special_matrices():
    ev, vec = O.eigen_selfadjoint3_vectors(np.array([np.diag([3.0, 1.0, 2.0]), np.eye(3) * 5.0]))
    assert np.array_equal(ev[0], [1.0, 2.0, 3.0])
    assert np.array_equal(np.abs(vec[0]), [[0, 1, 0], [0, 0, 1], [1, 0, 0]])
    assert np.array_equal(vec[1], np.eye(3))


def test_eigen_special_matrices():
    M = np.array([np.diag([3.0, 1.0, 2.0]), np.zeros((3, 3)), np.eye(3) * 5.0,
                  [[1.0, 1.0, 0.0], [1.0, 1.0, 0.0], [0.0, 0.0, 0.0]]])
    ev = O.eigen_selfadjoint3(M)
    assert np.array_equal(ev[0], [1.0, 2.0, 3.0])
    assert np.array_equal(ev[1], [0.0, 0.0, 0.0])
    assert np.array_equal(ev[2], [5.0, 5.0, 5.0])
    assert np.allclose(ev[3], [0.0, 0.0, 2.0], atol=1e-15)


def test_eigen_scatter_of_a_plane_has_zero_smallest():
    # points on z = 0: the scatter matrix has an exact zero row/column
    rng = np.random.default_rng(2)
    p = rng.random((50, 3))
    p[:, 2] = 0.0
    d = p - p[0]
    C = d.T @ d
    ev = O.eigen_selfadjoint3(C[None])
    assert ev[0, 0] == 0.0 and ev[0, 1] > 0


def _resolution_numpy(x, y, z):
    P = np.stack([x, y, z], 1).astype(np.float32)
    fin = np.isfinite(P).all(1)
    Pf = P[fin]
    terms = np.full(len(x), np.nan, np.float32)
    if len(Pf) >= 2:
        d = np.sort(_flann_d2(Pf, Pf), axis=1)[:, 1]
        terms[np.nonzero(fin)[0]] = np.sqrt(d).astype(np.float32)
    acc, cnt = 0.0, 0
    for t in terms:
        if not np.isnan(t):
            acc += float(t)
            cnt += 1
    return (acc / cnt if cnt else 0.0), terms


@pytest.mark.parametrize("case", ["uniform", "surface", "duplicates", "nan", "outliers", "single", "two"])
def test_resolution_exact(case):
    rng = np.random.default_rng(3)
    n = 2500
    x, y, z = rng.random((3, n)).astype(np.float32)
    if case == "surface":
        z = (0.05 * np.sin(4 * x) * np.cos(3 * y)).astype(np.float32)
    elif case == "duplicates":
        x[100:200], y[100:200], z[100:200] = x[:100], y[:100], z[:100]
    elif case == "nan":
        x[::7] = np.nan
        y[3::11] = np.inf
    elif case == "outliers":
        x[:5] += np.float32(50.0) * np.arange(1, 6, dtype=np.float32)
    elif case == "single":
        x, y, z = x[:1], y[:1], z[:1]
    elif case == "two":
        x, y, z = x[:2], y[:2], z[:2]
    res, terms = O.cloud_resolution(x, y, z)
    ref, rterms = _resolution_numpy(x, y, z)
    assert np.array_equal(np.isnan(terms), np.isnan(rterms))
    ok = ~np.isnan(rterms)
    assert np.array_equal(terms[ok].view(np.uint32), rterms[ok].view(np.uint32))
    assert res == ref


def _iss_numpy_checks(x, y, z, sal, nm, kp, third, min_nb=5):
    P = np.stack([x, y, z], 1).astype(np.float32)
    n = len(P)
    rr = np.float32(nm * nm)
    d = _flann_d2(P, P)
    is_kp = np.zeros(n, bool)
    is_kp[kp] = True
    for i in range(n):
        nb = np.nonzero(d[i] < rr)[0]
        expect = third[i] > 0 and len(nb) >= min_nb and not np.any(third[nb] > third[i])
        assert expect == is_kp[i], i
    # third: sequential double scatter in FLANN order, then the restated solver
    rs = np.float32(sal * sal)
    for i in range(0, n, 7):
        nb = np.nonzero(d[i] < rs)[0]
        nb = nb[np.lexsort((nb, d[i, nb]))]
        cov = np.zeros(9)
        if len(nb) >= min_nb:
            c = P[i].astype(np.float64)
            for j in nb:
                q = P[j].astype(np.float64) - c
                for a in range(3):
                    for b in range(3):
                        cov[a * 3 + b] += q[a] * q[b]
        e3, e2, e1 = O.eigen_selfadjoint3(cov.reshape(1, 3, 3))[0]
        t = 0.0
        if np.isfinite([e1, e2, e3]).all() and e3 >= 0:
            with np.errstate(divide="ignore", invalid="ignore"):
                if e2 / e1 < 0.975 and e3 / e2 < 0.975:
                    t = e3
        assert third[i] == t, i


def test_iss_surface():
    rng = np.random.default_rng(4)
    n = 1500
    u, v = rng.random((2, n)).astype(np.float32)
    w = (0.15 * np.sin(5 * u) * np.cos(4 * v)).astype(np.float32)
    res, _ = O.cloud_resolution(u, v, w)
    kp, third = O.iss_keypoints(u, v, w, 6 * res, 4 * res)
    assert 0 < len(kp) < n and np.all(np.diff(kp) > 0)
    _iss_numpy_checks(u, v, w, 6 * res, 4 * res, kp, third)


def test_iss_plane_has_no_keypoints():
    rng = np.random.default_rng(5)
    u, v = rng.random((2, 800)).astype(np.float32)
    w = np.zeros_like(u)
    res, _ = O.cloud_resolution(u, v, w)
    kp, third = O.iss_keypoints(u, v, w, 6 * res, 4 * res)
    assert len(kp) == 0 and np.all(third == 0)


def test_iss_rejected_parameters():
    x = np.zeros(3, np.float32)
    kp, third = O.iss_keypoints(x, x, x, 0.0, 0.1)
    assert len(kp) == 0


def _corner_scene(n, seed):
    rng = np.random.default_rng(seed)
    m = n // 4
    pts = []
    for axis in range(3):
        p = rng.random((m, 3)).astype(np.float32) * 0.3
        p[:, axis] = 0.0
        pts.append(p)
    u, v = rng.random((2, n - 3 * m)).astype(np.float32) * 0.6
    w = (0.01 * np.sin(40 * u) * np.cos(30 * v)).astype(np.float32) - 0.05
    pts.append(np.stack([u, v, w], 1))
    P = np.concatenate(pts).astype(np.float32) + rng.normal(0, 1e-4, (n, 3)).astype(np.float32)
    return P[:, 0].copy(), P[:, 1].copy(), P[:, 2].copy()


def test_harris3d_response_nms_and_snap():
    """Harris3D restatement (keypoints.h:150-162, 365-395) against numpy: the response formula
    in float32 over FLANN-ordered neighbours' normals (sampled points), the suppression rule on
    every point, and the snap of every corner to its nearest cloud point."""
    x, y, z = _corner_scene(3000, 6)
    r = 0.03  # a denser ball than the reference's 0.01 on this small scene
    kp, resp, corners = O.harris3d(x, y, z, radius=r)
    nx, ny, nz, _ = O.normals(x, y, z, r)
    P = np.stack([x, y, z], 1)
    d = _flann_d2(P, P)
    rr = np.float32(r * r)
    f32 = np.float32
    for i in range(0, len(x), 11):
        nb = np.nonzero(d[i] < rr)[0]
        nb = nb[np.lexsort((nb, d[i, nb]))]
        s = [f32(0)] * 6
        cnt = 0
        for j in nb:
            if not np.isfinite(nx[j]):
                continue
            a, b, c = nx[j], ny[j], nz[j]
            s = [s[0] + a * a, s[1] + b * a, s[2] + c * a, s[3] + b * b, s[4] + c * b, s[5] + c * c]
            cnt += 1
        c0, c1, c2, c5, c6, c7 = [v / f32(cnt) for v in s] if cnt else [f32(0)] * 6
        tr = c0 + c5 + c7
        want = f32(0)
        if tr != 0:
            det = c0 * c5 * c7 + f32(2) * c1 * c2 * c6 - c2 * c2 * c5 - c1 * c1 * c7 - c6 * c6 * c0
            want = f32(0.04) + det - f32(0.04) * tr * tr
        assert np.float32(resp[i]).view(np.uint32) == np.float32(want).view(np.uint32), i
    # suppression: corners = points with resp >= 1e-6 and no larger neighbour, in index order
    is_max = [bool(resp[i] >= np.float32(1e-6) and not np.any(resp[d[i] < rr] > resp[i])) for i in range(len(x))]
    assert len(corners) == sum(is_max)
    # snap: nearest cloud point of each refined corner, kept when d2 < 1e-4
    snapped = []
    for c in corners:
        dc = _flann_d2(P, c[None, :].astype(np.float32))[0]
        j = int(np.lexsort((np.arange(len(x)), dc))[0])
        if float(dc[j]) < 1e-4:
            snapped.append(j)
    assert np.array_equal(kp, np.asarray(snapped, np.int32))
