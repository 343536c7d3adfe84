"""List-buffer capacity guards.  A compact (16-bit) list reserves (k + 1) / 2
32-bit words of the list buffer; its write guard must count those words, not k: with k, a list
whose words end within k / 2 words of the buffer's end was silently left unwritten while the
reservation cursor stayed inside the buffer, so neither the deferred build's gate nor the
readback asked for a rebuild.

The first list buffer of a fresh context is sized by PFX_LIST_WORDS around the slot demand of a
default build of the same cloud (the demand moves by a few arena tails from run to run, so a
spread of sizes puts the build's last reservations at, just inside and just past the buffer's
end); every size must give the default build's normals bit for bit -- from the deferred compact
build when it fits, from the exact rebuild when it does not."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def test_list_buffer_edge_sizes_are_exact():
    from pcl_feature_extraction_amd import Context
    from pcl_feature_extraction_amd.synth import synth_room

    x, y, z, _ = synth_room(200_000, 5)
    r = 0.05
    with Context(0) as c:
        ref = c.normals(x, y, z, r)
    old = os.environ.get("PFX_LIST_WORDS")
    fitted = reran = 0

    def run(words):
        nonlocal fitted, reran
        os.environ["PFX_LIST_WORDS"] = str(max(256, int(words)))
        with Context(0) as c:
            out = c.normals(x, y, z, r)
            slots = c.stat("normals_slots")
            if c.stat("normals_speculative_reruns"):
                reran += 1
            else:
                fitted += 1
                assert slots <= c.stat("normals_list_words")
        for a, b in zip(ref, out):
            assert np.array_equal(_bits(a), _bits(b)), f"list buffer of {words} words"
        return slots

    try:
        # a fresh context's first build with room to spare: its reservation total (list words +
        # tile padding + the arena tails of every workgroup that reserved, 16384 words at a time)
        s0 = run(1 << 29)
        assert s0 > 0
        for words in (s0 // 4, s0 // 2, s0 - 40000, s0 - 4096, s0 - 300, s0 - 9, s0 - 1, s0, s0 + 1, s0 + 2,
                      s0 + 7, s0 + 64, s0 + 300, s0 + 1024, s0 + 4096):
            run(words)
    finally:
        if old is None:
            os.environ.pop("PFX_LIST_WORDS", None)
        else:
            os.environ["PFX_LIST_WORDS"] = old
    # both paths taken: builds that fit the sized buffer and builds that had to be redone
    assert fitted > 0 and reran > 0
