"""bwtmi -- MI355X-native engine behind the `bwt.py` surface of wyim-pgl/bwt-algorithm.

Python keeps the reference's names; the work runs in libbwtmi.so (HIP kernels
for gfx950 + exact native post-processing).  See DESIGN.md.
"""
from .records import TandemRepeat, Job, RepeatList
from .motif import MotifUtils, RepeatAlignmentSummary
from .core import BWTCore
from .tiers import Tier1STRFinder, Tier2LCPFinder, Tier3LongReadFinder
from .finder import TandemRepeatFinder

__all__ = ["TandemRepeat", "Job", "RepeatList", "MotifUtils", "RepeatAlignmentSummary", "BWTCore",
           "Tier1STRFinder", "Tier2LCPFinder", "Tier3LongReadFinder", "TandemRepeatFinder", "main"]


def main(argv=None):
    from .cli import main as _main
    return _main(argv)
