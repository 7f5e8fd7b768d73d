"""Host side of the per-family hot path: the reference's ``main`` loop body
(DuplexUMIConsensusReads.py:1544-1594) with the six ``make_consensus_read``
calls per family replaced by ONE batched backend call per batch of families.

Host keeps (exactly as the reference does them, same order):
  check_family_UMIs / check_family_rnames   :100-128  (sys.exit on mismatch)
  split_family                              :132-154
  check_number_reads (random.sample)        :157-188  (RNG order preserved)
Backend (HIP library, or the C oracle in tests) does:
  remove_clipping / mask / trim_3prime_N    :191-325
  4x single-strand + 2x duplex consensus    :1291-1386
Host then formats records (writer.py) and mate fields (:1390-1419).

Failure semantics: if the reference would raise on a family (status codes in
include/dcr.h), ``FamilyResult.crash`` names the exception type; the CLI
re-raises it at that family, after writing everything before it, as the
reference would.
"""
from __future__ import annotations

import dataclasses
import random as _random
from typing import Callable, List, Optional

import numpy as np

from . import writer
from duplexumiconsensusreads_amd.batch import OutArrays, pack_families
from duplexumiconsensusreads_amd.params import ConsensusParams

STATUS_NAME = {1: "IndexError", 2: "TypeError", 3: "ValueError", 4: "OverflowError", 5: "exit"}
UPSTREAM, PREP = 6, 0x10       # include/dcr.h DCR_ST_UPSTREAM, DCR_ST_PREP


class FamilyExit(Exception):
    """The reference prints an error and calls sys.exit(1) for this family."""


def reference_exception(name: str) -> Exception:
    """The exception the reference raises for a record status (include/dcr.h
    DCR_ST_*): IndexError / TypeError / ValueError / OverflowError, or the
    sys.exit(1) of most_likely_nucleotide on an invalid nucleotide (:582-585)."""
    if name == "exit":
        return FamilyExit("ERROR: invalid nucleotide found in the reads")
    return {"IndexError": IndexError, "TypeError": TypeError, "ValueError": ValueError,
            "OverflowError": OverflowError}[name](f"reference would raise {name} here")


@dataclasses.dataclass
class FamilyResult:
    code: str
    reads: list                       # the family as read (input order)
    subs: Optional[list] = None       # 4 downsampled subfamilies, or None if filtered
    crash: Optional[str] = None       # exception type the reference raises
    ss: Optional[list] = None         # 4 single-strand records
    ds: Optional[list] = None         # 2 duplex records (mate fields fixed)

    @property
    def filtered(self):
        return self.subs is None and self.crash is None


def check_family(reads, code):
    """check_family_UMIs (:100-113) and check_family_rnames (:116-128)."""
    umi1 = reads[0].get_tag("RX")
    parts = umi1.split("-")
    if len(parts) < 2:
        raise IndexError("list index out of range")       # :108 on an RX without '-'
    umi2 = "-".join([parts[1], parts[0]])
    for r in reads:
        if r.get_tag("RX") != umi1 and r.get_tag("RX") != umi2:
            raise FamilyExit(f"ERROR: family {code} has different UMI tags. \n Please check output file "
                             "of previous step of the pipeline (fgbio GroupReadsByUmi)")
    rname = reads[0].reference_id
    for r in reads[1:]:
        if r.reference_id != rname:
            raise FamilyExit(f"ERROR: family {code} has difference rnames (e.g. chromosome numbers). \n "
                             "Please check output file of previous step of the pipeline (fgbio GroupReadsByUmi)")


def split_family(reads):
    """split_family (:132-154): by strand x read1/read2 flags."""
    out = [[], [], [], []]
    for r in reads:
        if not r.is_reverse and r.is_read1:
            out[0].append(r)
        elif not r.is_reverse and r.is_read2:
            out[1].append(r)
        elif r.is_reverse and r.is_read1:
            out[2].append(r)
        elif r.is_reverse and r.is_read2:
            out[3].append(r)
    return out


def check_number_reads(split, min_reads, max_reads, rng=_random):
    """check_number_reads (:157-188), same RNG call sequence."""
    for idx, sub in enumerate(split):
        if len(sub) < min_reads:
            return None
        elif len(sub) > max_reads:
            split[idx] = rng.sample(split[idx], max_reads)
    return split


def prepare_family(reads, params: ConsensusParams, rng=_random) -> FamilyResult:
    code = reads[0].get_tag("MI").split("/")[0]
    check_family(reads, code)
    subs = check_number_reads(split_family(reads), params.min_reads, params.max_reads, rng)
    return FamilyResult(code=code, reads=reads, subs=subs)


Backend = Callable[[object, ConsensusParams], tuple]


def run_batch(results: List[FamilyResult], params: ConsensusParams, backend: Backend):
    """Run the hot path for every non-filtered family in ``results`` (in place)."""
    todo = [r for r in results if r.subs is not None and r.crash is None]
    if not todo:
        return results
    packed = pack_families([r.subs for r in todo])
    ss, ds, info = backend(packed, params)
    finish_batch(todo, packed, ss, ds, info)
    return results


def finish_batch(todo, packed, ss: OutArrays, ds: OutArrays, info):
    """Resolve statuses in the reference's execution order and build records."""
    for f, fam in enumerate(todo):
        crash = None
        for k in range(4):                             # preprocess_family (:1272-1283): the first
            st = int(ss.status[4 * f + k])             # subfamily with a failing read (DCR_ST_PREP | s)
            if st & PREP:
                crash = STATUS_NAME[st & 15]
                break
        if crash is None:
            for k in range(4):                         # single-strand calls in order
                st = int(ss.status[4 * f + k])
                if st and st != UPSTREAM:
                    crash = STATUS_NAME[st]
                    break
        if crash is None:
            for j in range(2):
                st = int(ds.status[2 * f + j])
                if st and st != UPSTREAM:
                    crash = STATUS_NAME[st]
                    break
        if crash is not None:
            fam.crash = crash
            continue
        ss_recs = [writer.single_strand_record(ss.record(4 * f + k, packed.ss_col_off), fam.subs[k])
                   for k in range(4)]
        d0 = writer.duplex_record(ds.record(2 * f, packed.ds_col_off), ss_recs[0], ss_recs[1])
        d1 = writer.duplex_record(ds.record(2 * f + 1, packed.ds_col_off), ss_recs[2], ss_recs[3])
        fam.ss = ss_recs
        fam.ds = writer.fix_paired_end_fields(d0, d1)
