#!/usr/bin/env python3
"""Drop-in for the reference's `bwt.py` (CLI and module names), backed by the
MI355X-native engine in bwtmi / libbwtmi.so:

    python bwt.py REF.fa [-o repeat.tab] [--format strfinder|bed|vcf|trf_table|trf_dat] ...
    from bwt import TandemRepeatFinder, BWTCore, MotifUtils, Tier2LCPFinder
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bwtmi import (BWTCore, MotifUtils, TandemRepeat, TandemRepeatFinder, Tier1STRFinder,  # noqa: E402,F401
                   Tier2LCPFinder, Tier3LongReadFinder)
from bwtmi.cli import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
