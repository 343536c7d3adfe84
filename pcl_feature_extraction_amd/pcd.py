"""PCD v0.7 reader/writer for the clouds on the reference's path.

The reference loads clouds with ``pcl::io::loadPCDFile<PointXYZRGB>`` (evaluation.cpp:226-235).
The repo's clouds (reference data/{indoor,underwater}/*.pcd) are
``FIELDS x y z rgb``, ``SIZE 4``, ``TYPE F``, ``DATA binary``, followed by zero padding up to
``4096 + 16*N`` bytes (PCL 1.7 ``writeBinary`` page stretch).  This reader handles ``binary``
and ``ascii`` data with arbitrary float/int fields and returns structure-of-arrays numpy views,
the layout the HIP path consumes (xyz SoA, float32).
"""
from __future__ import annotations

import dataclasses
from typing import Dict

import numpy as np

_TYPES = {("F", 4): np.float32, ("F", 8): np.float64, ("I", 1): np.int8, ("I", 2): np.int16,
          ("I", 4): np.int32, ("U", 1): np.uint8, ("U", 2): np.uint16, ("U", 4): np.uint32}


@dataclasses.dataclass
class PointCloud:
    """Unorganised cloud as SoA arrays (``x``, ``y``, ``z`` float32 contiguous) + extra fields."""
    x: np.ndarray
    y: np.ndarray
    z: np.ndarray
    fields: Dict[str, np.ndarray]
    width: int
    height: int
    viewpoint: tuple  # (tx, ty, tz, qw, qx, qy, qz) as in the PCD header

    @property
    def n(self) -> int:
        return int(self.x.shape[0])

    @property
    def sensor_origin(self):
        return tuple(float(v) for v in self.viewpoint[:3])

    @property
    def is_dense(self) -> bool:
        return bool(np.isfinite(self.x).all() and np.isfinite(self.y).all()
                    and np.isfinite(self.z).all())


def read_pcd(path: str) -> PointCloud:
    with open(path, "rb") as f:
        raw = f.read()
    header = {}
    pos = 0
    while True:
        end = raw.index(b"\n", pos)
        line = raw[pos:end].decode("ascii", "replace").strip()
        pos = end + 1
        if not line or line.startswith("#"):
            continue
        key, _, val = line.partition(" ")
        header[key.upper()] = val.split()
        if key.upper() == "DATA":
            break
    fields = header["FIELDS"]
    sizes = [int(s) for s in header["SIZE"]]
    types = header["TYPE"]
    counts = [int(c) for c in header.get("COUNT", ["1"] * len(fields))]
    width = int(header["WIDTH"][0])
    height = int(header.get("HEIGHT", ["1"])[0])
    npts = int(header.get("POINTS", [str(width * height)])[0])
    vp = tuple(float(v) for v in header.get("VIEWPOINT", ["0", "0", "0", "1", "0", "0", "0"]))
    dt = np.dtype([(name, _TYPES[(t, s)], (c,)) if c > 1 else (name, _TYPES[(t, s)])
                   for name, s, t, c in zip(fields, sizes, types, counts)])
    mode = header["DATA"][0].lower()
    if mode == "binary":
        need = dt.itemsize * npts
        if len(raw) - pos < need:
            raise ValueError(f"{path}: truncated binary PCD ({len(raw) - pos} < {need} bytes)")
        rec = np.frombuffer(raw, dtype=dt, count=npts, offset=pos)
    elif mode == "ascii":
        vals = np.array(raw[pos:].decode("ascii").split(), dtype=np.float64)
        ncol = sum(counts)
        vals = vals[: npts * ncol].reshape(npts, ncol)
        rec = np.zeros(npts, dtype=dt)
        col = 0
        for name, c in zip(fields, counts):
            rec[name] = vals[:, col] if c == 1 else vals[:, col:col + c]
            col += c
    else:
        raise ValueError(f"{path}: unsupported PCD DATA mode {mode!r} (binary/ascii only)")
    out = {name: np.ascontiguousarray(rec[name]) for name in fields}
    x = out.pop("x").astype(np.float32, copy=False)
    y = out.pop("y").astype(np.float32, copy=False)
    z = out.pop("z").astype(np.float32, copy=False)
    return PointCloud(np.ascontiguousarray(x), np.ascontiguousarray(y), np.ascontiguousarray(z),
                      out, width, height, vp)


def write_pcd(path: str, x, y, z, rgb=None) -> None:
    """Binary ``x y z rgb`` PCD (the layout of the reference's data files)."""
    n = len(x)
    rec = np.zeros(n, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgb", "<f4")])
    rec["x"], rec["y"], rec["z"] = x, y, z
    if rgb is not None:
        rec["rgb"] = np.asarray(rgb, dtype=np.uint32).view(np.float32)
    head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z rgb\n"
            "SIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\n"
            f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA binary\n")
    with open(path, "wb") as f:
        f.write(head.encode("ascii"))
        f.write(rec.tobytes())
