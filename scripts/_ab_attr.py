"""A/B helper: runs bench.py with one OverlappedNarfFpfh attribute overridden.
usage: python scripts/_ab_attr.py name=value -- <bench args>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
name, val = sys.argv[1].split("=")
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[3:]
import pcl_feature_extraction_amd.pipeline as P  # noqa: E402
init = P.OverlappedNarfFpfh.__init__


def patched(self, *a, **k):
    init(self, *a, **k)
    setattr(self, name, type(getattr(self, name))(eval(val)))


P.OverlappedNarfFpfh.__init__ = patched
import bench  # noqa: E402
bench.main()
