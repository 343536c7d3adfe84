"""Which SURVEY A.5 / A.6 statements the NARF keypoint set hinges on (VERDICT r04 #2c; test
infrastructure, CPU only): the oracle's restatement (oracle/or_narf.cpp, the reading the GPU path
is bit-exact against) vs the same restatement with ONE medium / low confidence statement swapped
for its most plausible other reading (orc_narf_set_alt bits, listed in or_narf.cpp).  For each
reading: keypoints lost / new per cloud (the reference's four clouds, and with --seeds the
configs[2] 1M-point rooms).  A statement whose alternative moves no keypoint does not matter for
parity on these clouds; one that moves many is where an unpinned restatement is most exposed.

usage: python scripts/narf_alt_report.py [--seeds 2] [--json out.jsonl]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import oracle_lib as O  # noqa: E402
from narf_tie_report import reference_clouds  # noqa: E402

ALTS = [
    (1 << 0, "A.5.1", "local plane from every pixel of the 5x5 window, 9 closest (restated: step 2, 4 closest)"),
    (1 << 1, "A.5.3", "score update: 3x3 mean including the centre pixel (restated: the 8 neighbours)"),
    (1 << 2, "A.5.3", "score update without the early return below minimum_border_probability"),
    (1 << 3, "A.5.4", "shadow pass reads un-updated opposite scores (restated: in place, raster order)"),
    (1 << 4, "A.5.7", "principal-curvature magnitude lambda_max (restated: sqrt(lambda_max))"),
    (1 << 5, "A.5.7", "curvature beams skip veil/shadow pixels (restated: a beam ends there)"),
    (1 << 6, "A.6", "region grow accepts within 2 px AND within R (restated: OR)"),
    (1 << 7, "A.6", "positive score = scs for pixel distance <= 2 (restated: < 2)"),
    (1 << 8, "A.6", "negative score not squared (restated: squared)"),
    (1 << 9, "A.6", "direction angle from atan2(v_y, v_x) (restated: acos(v_x))"),
    (1 << 10, "A.6", "histogram cell lrint without floorf (restated: lrint(floorf(.)))"),
    (1 << 11, "A.6", "interest = negative x max(h_i h_j nd), no sqrt (restated: sqrt)"),
]


def set_alt(mask):
    O.lib().orc_narf_set_alt(ctypes.c_int(mask))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="*", default=[])
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    clouds = list(reference_clouds())
    if args.seeds:
        from pcl_feature_extraction_amd.synth import synth_room
        for seed in args.seeds:
            x, y, z, _ = synth_room(1_000_000, seed)
            clouds.append((f"room_seed{seed}", x, y, z))
    set_alt(0)
    base = {name: set(O.narf_keypoints(x, y, z).tolist()) for name, x, y, z in clouds}
    rows = []
    print("%-6s %-92s %s" % ("stmt", "alternative reading", "  ".join("%s (%d kp)" % (n, len(base[n])) for n in base)))
    for bitv, stmt, what in ALTS:
        set_alt(bitv)
        cells, row = [], {"bit": bitv, "statement": stmt, "reading": what, "clouds": {}}
        for name, x, y, z in clouds:
            k = set(O.narf_keypoints(x, y, z).tolist())
            lost, new = len(base[name] - k), len(k - base[name])
            row["clouds"][name] = {"keypoints": len(k), "lost": lost, "new": new}
            cells.append("-%d/+%d" % (lost, new))
        rows.append(row)
        print("%-6s %-92s %s" % (stmt, what, "  ".join("%18s" % c for c in cells)), flush=True)
    set_alt(0)
    if args.json:
        with open(args.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
