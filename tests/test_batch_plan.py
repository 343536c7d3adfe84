"""The C-ABI batch's host-side plan (pfx_batch_plan, csrc/pfx_batch.hip; SURVEY 8(e), configs[4]):
the round-robin deal of the scans over G devices and the scan-order layout of the gathered
descriptor rows, which pfx_batch_narf_fpfh follows.  No device work: runs on CPU for G = 1, 2, 3,
8 (the G > 1 RCCL send/recv group itself needs several GPUs).

Bar: the deal equals the Python ranks' (dist.owned_scans: scan s on rank s % G), a simulated
gather that puts every device's blocks at the plan's offsets reproduces the scans' rows in scan
order exactly, and invalid counts are rejected."""
import numpy as np
import pytest

from pcl_feature_extraction_amd.api import batch_plan
from pcl_feature_extraction_amd.dist import owned_scans
from pcl_feature_extraction_amd import PfxError


@pytest.mark.parametrize("G", [1, 2, 3, 8])
@pytest.mark.parametrize("n_scans", [0, 1, 5, 8, 17])
def test_plan_deal_and_gather_layout(G, n_scans):
    rng = np.random.default_rng(G * 100 + n_scans)
    rows = rng.integers(0, 40, n_scans)
    if n_scans > 2:
        rows[1] = 0  # a scan without keypoints
    dev, slot, off = batch_plan(n_scans, G, rows)
    # the deal: device d owns exactly dist.owned_scans(n, G, d), in slot order
    for d in range(G):
        mine = [s for s in range(n_scans) if dev[s] == d]
        assert mine == owned_scans(n_scans, G, d)
        assert [int(slot[s]) for s in mine] == list(range(len(mine)))
    # the layout: offsets are the scan-order prefix sums
    assert off[0] == 0 and np.array_equal(np.diff(off), rows)
    # simulated gather: each device's blocks (rows tagged with their scan) placed at the offsets
    blocks = {s: np.full((int(rows[s]), 2), s, np.int64) for s in range(n_scans)}
    for s in range(n_scans):
        blocks[s][:, 1] = np.arange(rows[s])
    out = np.full((int(off[-1]), 2), -1, np.int64)
    for d in range(G):
        for s in owned_scans(n_scans, G, d):
            out[off[s]:off[s + 1]] = blocks[s]
    want = np.concatenate([blocks[s] for s in range(n_scans)]) if n_scans else np.zeros((0, 2), np.int64)
    assert np.array_equal(out, want)


def test_plan_without_rows_and_invalid_counts():
    dev, slot, off = batch_plan(8, 3)
    assert dev.tolist() == [0, 1, 2, 0, 1, 2, 0, 1] and slot.tolist() == [0, 0, 0, 1, 1, 1, 2, 2]
    assert off.tolist() == [0] * 9
    with pytest.raises(PfxError):
        batch_plan(4, 0)
    with pytest.raises(PfxError):
        batch_plan(-1, 2)
    with pytest.raises(PfxError):
        batch_plan(2, 2, [3, -1])


def test_plan_rejects_short_rows_and_negative_counts():
    """rows_per_scan must hold n_scans entries (the C side reads that many), and any
    n_scans < 0 is PfxError, not a numpy error."""
    with pytest.raises(PfxError):
        batch_plan(4, 2, [1, 2, 3])
    with pytest.raises(PfxError):
        batch_plan(2, 2, [1, 2, 3])
    with pytest.raises(PfxError):
        batch_plan(-5, 2)
    dev, slot, off = batch_plan(3, 2, [1, 2, 3])
    assert off.tolist() == [0, 1, 3, 6]
