"""The C-ABI multi-GPU scan batch (include/pfx.h pfx_batch_*, csrc/pfx_batch.hip; SURVEY 8(e),
configs[4]): one process, G devices, RCCL communicator from ncclCommInitAll, per-device two-stream
pipeline, descriptor gather to the first device.  tests/cpp/batch_driver.cpp is the C++ host that
replaces the reference's per-scan loop (evaluation.cpp:272-852) with it.

CPU: the driver compiles and links.  GPU (one device on the test box): the 8 configs[4] scans
(seeds 100-107, 200k points each) through the batch -- from Python and from the C++ driver -- equal
the per-scan C-ABI entry points (pfx_narf_keypoints, pfx_normals, pfx_fpfh) bit for bit."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "batch_driver.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "build", "batch_driver")
N_SCAN = 200_000
SEEDS = [100 + i for i in range(8)]


def build_driver():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    lib = os.path.join(ROOT, "pcl_feature_extraction_amd")
    cmd = ["g++", "-std=c++14", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"), SRC,
           "-L", lib, "-lpfx", f"-Wl,-rpath,{lib}", "-o", EXE]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return EXE


def test_batch_driver_compiles_and_links():
    exe = build_driver()
    assert os.access(exe, os.X_OK)


def _bits(a):  # raw bits, NaN rows included (PCL's quiet_NaN on every side)
    return np.ascontiguousarray(np.asarray(a, np.float32)).view(np.uint32)


@pytest.fixture(scope="module")
def clouds():
    from pcl_feature_extraction_amd.synth import synth_room
    return [tuple(np.ascontiguousarray(a) for a in synth_room(N_SCAN, s)[:3]) for s in SEEDS]


@pytest.fixture(scope="module")
def per_scan(clouds):
    """Each scan through the per-scan host C-ABI on one context (the reference's loop body)."""
    from pcl_feature_extraction_amd import Context
    out = []
    with Context(0) as c:
        for x, y, z in clouds:
            kp = np.asarray(c.narf_keypoints(x, y, z), np.int32)
            rows = kp[(kp >= 0) & (kp < len(x))]
            nx, ny, nz, _ = c.normals(x, y, z, 0.05)
            d = c.fpfh(x, y, z, nx, ny, nz, x[rows], y[rows], z[rows], 0.08)
            out.append((d, rows))
    return out


@pytest.mark.gpu
def test_batch_equals_per_scan_c_abi(clouds, per_scan):
    from pcl_feature_extraction_amd import Batch
    with Batch([0]) as b:
        got = b.narf_fpfh(clouds)
        again = b.narf_fpfh(clouds[:3])  # slots reused, fewer scans
    assert len(got) == len(SEEDS)
    for s, ((d, i), (wd, wi)) in enumerate(zip(got, per_scan)):
        assert len(i) > 0, s
        assert np.array_equal(i, wi), s
        assert np.array_equal(_bits(d), _bits(wd)), s
    for s, (d, i) in enumerate(again):
        assert np.array_equal(i, per_scan[s][1]) and np.array_equal(_bits(d), _bits(per_scan[s][0])), s


@pytest.mark.gpu
def test_cpp_batch_driver_equals_per_scan_c_abi(clouds, per_scan, tmp_path):
    exe = build_driver()
    files = []
    for s, (x, y, z) in enumerate(clouds):
        f = tmp_path / f"scan{s}.f32"
        np.concatenate([x, y, z]).astype(np.float32).tofile(f)
        files.append(str(f))
    r = subprocess.run([exe, str(tmp_path), "0", *files], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rows = np.fromfile(tmp_path / "rows.i64", np.int64)
    desc = np.fromfile(tmp_path / "desc.f32", np.float32).reshape(-1, 33)
    idx = np.fromfile(tmp_path / "idx.i32", np.int32)
    assert rows.tolist() == [len(i) for _, i in per_scan]
    o = 0
    for s, (wd, wi) in enumerate(per_scan):
        k = int(rows[s])
        assert np.array_equal(idx[o:o + k], wi), s
        assert np.array_equal(_bits(desc[o:o + k]), _bits(wd)), s
        o += k


@pytest.mark.gpu
def test_batch_rejects_bad_arguments():
    from pcl_feature_extraction_amd import Batch, PfxError
    with pytest.raises(PfxError):
        Batch([0, 0])  # a device listed twice
    with pytest.raises(PfxError):
        Batch([64])  # no such device
    with Batch([0]) as b:
        x = np.zeros(10, np.float32)
        with pytest.raises(PfxError):
            b.narf_fpfh([(x, x, x)], normal_radius=-1.0)
        assert b.narf_fpfh([]) == []
