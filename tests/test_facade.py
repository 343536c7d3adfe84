"""The C++ PCL-compatible facade (include/pfx_pcl.hpp): tests/cpp/facade_driver.cpp writes the
reference's NARF + Features<T> flow (keypoints.h:199-231, features.h:175-196, tools.h:22-32) against
it.  CPU: the driver compiles and links against libpfx.so.  GPU: its outputs equal the Python
C-ABI path (itself bit-exact against the oracle) on a reference cloud."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "facade_driver.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "build", "facade_driver")
PCD = os.path.join(ROOT, "tests", "golden", "clouds", "indoor_source.pcd")
PCD_T = os.path.join(ROOT, "tests", "golden", "clouds", "indoor_target.pcd")


def build_driver():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    lib = os.path.join(ROOT, "pcl_feature_extraction_amd")
    cmd = ["g++", "-std=c++14", "-O2", "-Wall", "-Wextra", "-Werror", "-pthread", "-I", os.path.join(ROOT, "include"), SRC,
           "-L", lib, "-lpfx", f"-Wl,-rpath,{lib}", "-o", EXE]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return EXE


def test_facade_compiles_and_links():
    exe = build_driver()
    assert os.access(exe, os.X_OK)


@pytest.mark.gpu
def test_facade_matches_c_abi(ctx, tmp_path):
    from parity import bits_equal
    from pcl_feature_extraction_amd.pcd import read_pcd
    exe = build_driver()
    r = subprocess.run([exe, PCD, str(tmp_path), PCD_T], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    c = read_pcd(PCD)
    x, y, z = c.x, c.y, c.z
    kp = np.fromfile(tmp_path / "keypoints.i32", np.int32)
    assert np.array_equal(kp, np.asarray(ctx.narf_keypoints(x, y, z), np.int32))
    nrm = np.fromfile(tmp_path / "normals.f32", np.float32).reshape(-1, 8)
    want = np.stack(ctx.normals(x, y, z, 0.05))
    got = nrm[:, [0, 1, 2, 4]].T
    # raw bits, NaN rows included (PCL's quiet_NaN for points without a normal)
    assert bits_equal(got, want)
    rows = kp[kp < len(x)]
    fp = np.fromfile(tmp_path / "fpfh.f32", np.float32).reshape(-1, 33)
    wf = ctx.fpfh(x, y, z, want[0], want[1], want[2], x[rows], y[rows], z[rows], 0.08)
    assert fp.shape == wf.shape
    assert bits_equal(fp, wf)
    sd = np.fromfile(tmp_path / "shot.f32", np.float32).reshape(-1, 352)
    wd, _ = ctx.shot(x, y, z, want[0], want[1], want[2], x[rows], y[rows], z[rows], 0.08)
    assert sd.shape == wd.shape
    assert bits_equal(sd, wd)

    # features.h:224-273 run verbatim against the facade (two threads, KdTreeFLANN<FPFHSignature33>)
    tf = np.fromfile(tmp_path / "fpfh_target.f32", np.float32).reshape(-1, 33)
    corr = np.fromfile(tmp_path / "corr.i32", np.int32).reshape(-1, 2)
    q, m = ctx.correspondences(fp, tf)
    assert np.array_equal(corr[:, 0], q) and np.array_equal(corr[:, 1], m)
    import oracle_lib as O
    oq, om = O.correspondences(fp, tf)
    assert np.array_equal(q, oq) and np.array_equal(m, om) and len(q) > 0

    # keypoints.h:177-189 (ISS branch) verbatim against the facade
    res = np.fromfile(tmp_path / "resolution.f64", np.float64)[0]
    ores, _ = O.cloud_resolution(x, y, z)
    assert res == ores
    okp, _ = O.iss_keypoints(x, y, z, 6 * ores, 4 * ores)
    ixyz = np.fromfile(tmp_path / "iss_xyz.f32", np.float32).reshape(-1, 3)
    assert len(okp) > 0 and np.array_equal(ixyz, np.stack([x[okp], y[okp], z[okp]], 1))

    # keypoints.h:150-176 (Harris3D / Harris6D) + getKeypointsCloud through the facade
    rgb = np.ascontiguousarray(c.fields["rgb"]).view(np.uint32)
    for six in (False, True):
        tag = "harris6d" if six else "harris3d"
        if six:
            hk, resp, cor, _ = ctx.harris6d_keypoints(x, y, z, rgb, details=True)
        else:
            hk, resp, cor = ctx.harris3d_keypoints(x, y, z, details=True)
        hxyz = np.fromfile(tmp_path / f"{tag}_xyz.f32", np.float32).reshape(-1, 3)
        assert len(hk) > 0 and np.array_equal(hxyz, np.stack([x[hk], y[hk], z[hk]], 1))
        hc = np.fromfile(tmp_path / f"{tag}_corners.f32", np.float32).reshape(-1, 4)
        assert np.array_equal(hc[:, :3].view(np.uint32), cor.view(np.uint32))
        # PCL's output intensity: the response of each corner's own point (refine=False: the
        # corners are those points)
        if six:
            _, _, c0, _ = ctx.harris6d_keypoints(x, y, z, rgb, refine=False, details=True)
        else:
            _, _, c0 = ctx.harris3d_keypoints(x, y, z, refine=False, details=True)
        rb = resp.view(np.uint32)
        by_xyz = {}
        for i, p in enumerate(np.stack([x, y, z], 1).tolist()):
            by_xyz.setdefault(tuple(p), set()).add(int(rb[i]))  # duplicates: any of their responses
        assert len(c0) == len(hc)
        assert all(int(b) in by_xyz[tuple(p)] for p, b in zip(c0.tolist(), hc[:, 3].view(np.uint32)))

    # features.h:282-297 (filterCorrespondences) through the facade
    sk = np.fromfile(tmp_path / "src_kp_xyz.f32", np.float32).reshape(-1, 3)
    tk = np.fromfile(tmp_path / "tgt_kp_xyz.f32", np.float32).reshape(-1, 3)
    keep, T = ctx.ransac_rejector(sk, tk, q, m)
    filt = np.fromfile(tmp_path / "filtered.i32", np.int32).reshape(-1, 2)
    assert np.array_equal(filt, np.stack([q[keep], m[keep]], 1))
    Tf = np.fromfile(tmp_path / "transformation.f32", np.float32).reshape(4, 4)
    assert np.array_equal(Tf.view(np.uint32), np.asarray(T, np.float32).view(np.uint32))
