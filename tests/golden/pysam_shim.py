"""A ``pysam`` stand-in module for running the reference script in THIS container.

Test infrastructure only (used by make_golden.py to generate fixtures).  It maps
the two pysam classes the reference touches (DuplexUMIConsensusReads.py:3,
:1372, :1476, :1494) onto the host package's record class and BAM codec.
"""
import sys
import types

from duplexumiconsensusreads_amd import bam, records


def install():
    mod = types.ModuleType("pysam")
    mod.AlignedSegment = records.AlignedSegment
    mod.AlignmentFile = bam.AlignmentFile
    sys.modules["pysam"] = mod
    return mod
