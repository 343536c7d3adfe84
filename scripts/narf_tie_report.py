"""NARF greedy-selection tie report (test infrastructure, CPU only).

NarfKeypoint::compute orders the non-maximum-suppression survivors with a non-stable std::sort on
strength (PCL 1.7 narf_keypoint.cpp; restated in oracle/or_narf.cpp keypoints() and on the host
side of pfx_narf.hip), then accepts them greedily unless one already accepted lies closer than
min_distance_between_interest_points * support_size (md).  The order of equal-strength survivors
is implementation-defined (libstdc++'s introsort pivots changed across GCC releases; the reference
was built with an Indigo-era GCC), so "keypoint indices bit-exact" would depend on the toolchain
exactly when two tied survivors lie closer than md: equal strengths sort next to each other, and
swapping two adjacent survivors more than md apart changes neither decision (each depends only on
the survivors accepted before it), so any permutation of a tie group whose members are pairwise
>= md apart gives the same keypoints.

For each cloud: the survivors (the oracle's interest image, the NMS rule of keypoints()), the tie
groups among them, and the tied pairs closer than md (the ones that could move a keypoint).

usage: python scripts/narf_tie_report.py [--seeds 2 100 101 102]   (1M-point configs[2] scans)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle_lib as O  # noqa: E402


def survivors(interest, min_interest):
    """(pixel index, strength) of the NMS survivors, raster order (or_narf.cpp keypoints())."""
    h, w = interest.shape
    iv = interest
    ok = ~(iv < min_interest)  # (PCL's `if (interest_value < min_interest_value) continue`: NaN passes)
    is_max = ok.copy()
    pad = np.pad(iv, 1, constant_values=0.0)
    out = np.pad(np.zeros((h, w), bool), 1, constant_values=True)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx == 0 and dy == 0:
                continue
            nb = pad[1 + dy:1 + dy + h, 1 + dx:1 + dx + w]
            # a neighbour in the image whose interest is not <= iv (NaN on either side) breaks it;
            # neighbours outside the image are skipped
            is_max &= (nb <= iv) | out[1 + dy:1 + dy + h, 1 + dx:1 + dx + w]
    idx = np.flatnonzero(is_max.ravel())
    return idx, iv.ravel()[idx]


def tie_report(x, y, z, name):
    p = dict(O.NARF_DEFAULT)
    kp, dbg = O.narf_keypoints(x, y, z, debug=True)
    ri = O.range_image_planar(x, y, z)
    idx, s = survivors(dbg["interest"], p["min_interest_value"])
    pts = ri.reshape(-1, 4)[idx, :3].astype(np.float64)
    md = p["min_distance_between_interest_points"] * p["support_size"]
    groups, close = 0, []
    vals, inv, counts = np.unique(s, return_inverse=True, return_counts=True)
    for g in np.flatnonzero(counts > 1):
        members = np.flatnonzero(inv == g)
        groups += 1
        for a in range(len(members)):
            for b in range(a + 1, len(members)):
                d = float(np.linalg.norm(pts[members[a]] - pts[members[b]]))
                if d < md:
                    close.append({"pixels": [int(idx[members[a]]), int(idx[members[b]])], "strength": float(vals[g]),
                                  "distance": round(d, 6)})
    # sensitivity: the greedy selection with every tie group in ascending and in descending raster
    # order (the two extremes an unstable sort can produce); accepted survivors that differ
    md2 = np.float32(md) * np.float32(md)
    p32 = pts.astype(np.float32)

    def greedy(tie_sign):
        order = np.lexsort((tie_sign * idx, -s))
        acc = []
        for i in order:
            ok = True
            for j in acc:
                d = p32[i] - p32[j]
                if d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]) < md2:
                    ok = False
                    break
            if ok:
                acc.append(i)
        return set(int(idx[i]) for i in acc)
    a, b = greedy(1), greedy(-1)
    return {"cloud": name, "points": int(len(x)), "keypoints": int(len(kp)), "survivors": int(len(idx)),
            "tie_groups": groups, "tied_survivors": int(counts[counts > 1].sum()), "tied_pairs_closer_than_md": close,
            "md": md, "order_independent": not close,
            "keypoints_moved_by_tie_order": len(a ^ b) // 2 if len(a) == len(b) else sorted(a ^ b)}


def reference_clouds():
    from pcl_feature_extraction_amd.pcd import read_pcd
    d = os.path.join(ROOT, "tests", "golden", "clouds")
    for name in ("indoor_source", "indoor_target", "underwater_source", "underwater_target"):
        c = read_pcd(os.path.join(d, name + ".pcd"))
        yield name, c.x, c.y, c.z


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="*", default=[2, 100, 101, 102])
    args = ap.parse_args()
    rows = [tie_report(x, y, z, name) for name, x, y, z in reference_clouds()]
    from pcl_feature_extraction_amd.synth import synth_room
    for seed in args.seeds:
        x, y, z, _ = synth_room(1_000_000, seed)
        rows.append(tie_report(x, y, z, f"synth_room(1M, seed {seed})"))
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
