"""NARF greedy-selection ties: NarfKeypoint orders its NMS survivors with a
non-stable std::sort on strength, so keypoints depend on the sort's (toolchain-defined) order of
equal strengths exactly when two tied survivors lie closer than md = 0.05 m
(scripts/narf_tie_report.py).  On the reference's own clouds no two survivors tie, so their
keypoint indices do not depend on the libstdc++ the reference (or this build) was compiled with;
the configs[2] synthetic rooms do have such ties (profiles/r05_narf_tie_report.jsonl: 4-7 of ~85
keypoints move between the two extreme tie orders) -- stated at the boundary (include/pfx.h)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import narf_tie_report as T  # noqa: E402


def test_reference_clouds_have_no_consequential_ties():
    for name, x, y, z in T.reference_clouds():
        r = T.tie_report(x, y, z, name)
        assert r["survivors"] > 0 and r["keypoints"] > 0, name
        assert r["order_independent"], (name, r["tied_pairs_closer_than_md"])
        assert r["keypoints_moved_by_tie_order"] == 0, name


def test_tie_sensitivity_detects_a_planted_tie():
    """The report's machinery on a hand-made interest image: two adjacent equal maxima (a tie
    closer than md) are found, and the extreme tie orders accept different survivors."""
    h, w = 8, 8
    iv = np.zeros((h, w), np.float32)
    iv[3, 3] = iv[3, 4] = 0.9     # tied, adjacent: both survive NMS (equal neighbours do not suppress)
    iv[6, 6] = 0.7
    idx, s = T.survivors(iv, 0.45)
    assert sorted(idx.tolist()) == [3 * w + 3, 3 * w + 4, 6 * w + 6]
    assert np.count_nonzero(s == np.float32(0.9)) == 2


def test_alternative_readings_selector_restores_the_restatement():
    """scripts/narf_alt_report.py's selector (orc_narf_set_alt): an alternative reading moves the
    keypoints of a reference cloud, and mask 0 gives the documented restatement back bit for bit
    (the reading the GPU path is compared against everywhere else)."""
    import ctypes
    import oracle_lib as O
    name, x, y, z = [c for c in T.reference_clouds() if c[0] == "underwater_source"][0]
    base = O.narf_keypoints(x, y, z)
    try:
        O.lib().orc_narf_set_alt(ctypes.c_int(1 << 8))  # A.6 negative score not squared
        alt = O.narf_keypoints(x, y, z)
    finally:
        O.lib().orc_narf_set_alt(ctypes.c_int(0))
    assert not np.array_equal(alt, base)
    assert np.array_equal(O.narf_keypoints(x, y, z), base)
