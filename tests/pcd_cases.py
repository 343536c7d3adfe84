"""PCD files for the loader tests (pcl::io::loadPCDFile<PointXYZRGB>, evaluation.cpp:226-235):
ascii as pcl::io::savePCDFile writes it (evaluation.cpp:258), and binary with other field
orders, extra and 1-byte fields (unaligned x y z), comments and NaN points."""
import numpy as np


def cloud(n, seed):
    r = np.random.default_rng(seed)
    x, y, z = (r.normal(0, 2, n).astype(np.float32) for _ in range(3))
    x[::17] = np.nan  # non-dense cloud
    return x, y, z


def write_ascii(path, x, y, z):
    n = len(x)
    rgb = np.arange(n, dtype=np.uint32) * 2654435761 % (1 << 24)
    with open(path, "w") as f:
        f.write("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgb\nSIZE 4 4 4 4\n"
                "TYPE F F F U\nCOUNT 1 1 1 1\n" f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 1 2 3 1 0 0 0\nPOINTS {n}\n"
                "DATA ascii\n")
        for i in range(n):
            f.write(f"{x[i]:.9g} {y[i]:.9g} {z[i]:.9g} {rgb[i]}\n")


def write_binary_mixed(path, x, y, z):
    """FIELDS intensity(u8) label(u16) z y curvature x : x y z at unaligned byte offsets."""
    n = len(x)
    dt = np.dtype([("intensity", "u1"), ("label", "<u2"), ("z", "<f4"), ("y", "<f4"), ("curvature", "<f4"),
                   ("x", "<f4")])
    rec = np.zeros(n, dt)
    rec["x"], rec["y"], rec["z"] = x, y, z
    rec["intensity"] = np.arange(n) % 251
    rec["label"] = np.arange(n) % 60000
    with open(path, "wb") as f:
        f.write(("# comment line\nVERSION 0.7\nFIELDS intensity label z y curvature x\nSIZE 1 2 4 4 4 4\n"
                 "TYPE U U F F F F\nCOUNT 1 1 1 1 1 1\n" f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\n"
                 f"POINTS {n}\nDATA binary\n").encode())
        f.write(rec.tobytes())
