"""Command line drop-in for the reference script's ``main``
(DuplexUMIConsensusReads.py:1426-1650): same flags (``parse_args`` :10-91),
same output files, same summary lines, same record order.

What changes is the middle of the loop.  The reference calls
``make_consensus_read`` six times per family (:1560-1588); here complete
families are collected into batches and each batch is ONE ``dcr_run_batch``
call on the GPU (``pipeline.run_batch``), then drained in input order.  The
host keeps the per-read filters (``pass_filters`` :1135-1181), MI grouping
(``add_read_to_family`` :1185-1217), the family checks and the seeded
downsampling (``pipeline.prepare_family``), so the RNG call sequence is the
reference's.

Failure semantics follow the reference: records of every family before a
failing one are written, then the reference's exception (or ``sys.exit(1)``
with its message) is raised at that family.
"""
from __future__ import annotations

import argparse
import random
import sys
from typing import List, Optional

from . import bam, pipeline
from .params import ConsensusParams

SPLIT_NAMES = {0: "A1", 1: "B2", 2: "B1", 3: "A2"}      # split_dict (:1511)


def parse_args(argv):
    """The reference's flags (:10-91), names and defaults unchanged."""
    ap = argparse.ArgumentParser(description="call consensus reads from paired-end, Duplex-UMI reads, "
                                             "preserving mapping information")
    ap.add_argument("-i", "--input_file", required=True, type=str)
    ap.add_argument("-o", "--output_file", required=False, default=None, type=str)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-q", "--min_map_quality", required=False, default=20, type=int)
    ap.add_argument("--min_base_quality", required=False, default=20, type=int)
    ap.add_argument("--min_reads", required=False, default=1, type=int)
    ap.add_argument("--max_reads", required=False, default=100, type=int)
    ap.add_argument("--max_base_quality", required=False, default=60, type=int)
    ap.add_argument("--base_quality_shift", required=False, default=0, type=int)
    ap.add_argument("--error_rate_post_labeling", required=False, default=0, type=int)
    ap.add_argument("--error_rate_pre_labeling", required=False, default=0, type=int)
    ap.add_argument("--deletion_score", required=False, default=30, type=int)
    ap.add_argument("--no_insertion_score", required=False, default=30, type=int)
    # not a reference flag: families per device call (does not change any output)
    ap.add_argument("--batch_families", required=False, default=65536, type=int, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


class ReadFormatExit(SystemExit):
    """``pass_filters`` prints an error and calls sys.exit(1) (:1148-1165)."""


def pass_filters(read, map_q_threshold: int) -> bool:
    """``pass_filters`` (:1135-1181): format checks (exit), then the flag /
    MAPQ filters."""
    if not read.has_tag("MI"):
        print("ERROR: family code tag (MI) not found in file")
        raise ReadFormatExit(1)
    if not read.has_tag("RX"):
        print("ERROR: family code tag (RX) not found in file")
        raise ReadFormatExit(1)
    cs = read.cigarstring
    if cs is None:                        # `x in None` (:1158) on a read without CIGAR
        raise TypeError("argument of type 'NoneType' is not iterable")
    if any(x in cs for x in ("P", "N", "B", "*")):
        print("ERROR: unexpected symbols (P, N, B, *) were found in CIGAR strings.")
        raise ReadFormatExit(1)
    if any(op == 4 for op, _ in read.cigartuples[1:-1]):
        print("ERROR: softclips (S) found in the middle of the read.")
        raise ReadFormatExit(1)
    return (read.is_paired and read.is_proper_pair and not read.is_unmapped and not read.mate_is_unmapped
            and not read.is_supplementary and not read.is_qcfail and read.mapping_quality >= map_q_threshold)


def family_code_of(read) -> str:
    return read.get_tag("MI").split("/")[0]       # :1204, :1209


class _Run:
    """One pass over the input: counters, the pending batch, the writers."""

    def __init__(self, params: ConsensusParams, backend, batch_families: int, consensusbam, unprocessedbam,
                 verbose: bool, rng):
        self.params, self.backend, self.batch_families = params, backend, batch_families
        self.consensusbam, self.unprocessedbam = consensusbam, unprocessedbam
        self.verbose, self.rng = verbose, rng
        self.pending: List[pipeline.FamilyResult] = []
        self.processed = 0
        self.excluded = 0

    def family_done(self, family):
        """preprocess_family (:1226-1287) for one completed family.  Filtered
        families go to the side file at once, as the reference writes them
        (:1536-1540); the rest wait for their batch."""
        code = family_code_of(family[0])
        try:
            res = pipeline.prepare_family(family, self.params, self.rng)
        except pipeline.FamilyExit as e:
            self.drain()
            print(str(e))
            raise SystemExit(1)
        except Exception:
            self.drain()
            raise
        if res.subs is None:
            self.excluded += 1
            for r in family:
                self.unprocessedbam.write(r)
            return
        res.code = code
        self.processed += 1
        self.pending.append(res)
        if len(self.pending) >= self.batch_families:
            self.drain()

    def drain(self):
        """Run the pending batch on the device and write its records in input
        order; stop at the first family the reference would fail on."""
        if not self.pending:
            return
        todo, self.pending = self.pending, []
        pipeline.run_batch(todo, self.params, self.backend)
        for fam in todo:
            if fam.crash is not None:
                exc = pipeline.reference_exception(fam.crash)
                if isinstance(exc, pipeline.FamilyExit):
                    print(str(exc))
                    raise SystemExit(1)
                raise exc
            if self.verbose:
                for idx in range(4):
                    print("Single-strand consensus for subfamily", fam.code, SPLIT_NAMES[idx], "in progress")
                print("Double-strand consensus for family", fam.code, "in progress")
            for rec in fam.ds:
                self.consensusbam.write(rec)
            if self.verbose:
                print("Consensus reads for family", fam.code, "have been sucessfully written \n")


def default_backend(device: int = 0):
    """The HIP library on ``device`` (fails loudly without it: no CPU fallback)."""
    from . import _lib
    ctx = _lib.Context(ConsensusParams(), device=device)
    return _lib.backend(ctx)


def main(argv: Optional[list] = None, backend=None, rng=random) -> int:
    """``main`` (:1426-1650).  ``backend`` defaults to the HIP library."""
    args = parse_args(sys.argv[1:] if argv is None else argv)
    params = ConsensusParams.from_args(args)
    try:
        inbam = bam.AlignmentFile(args.input_file, "rb")
        if args.verbose:
            print(args.input_file, "has been read.")
    except Exception:
        print("ERROR: input file not found. \n Please specify file name of a valid .bam file. "
              "Include the format in the file name.")
        raise SystemExit(1)
    if args.output_file is None:
        consensus_filename = "%s_cons.bam" % args.input_file[:-4]
    elif args.output_file.endswith(".bam"):
        consensus_filename = args.output_file
    else:
        print("ERROR: output file is not specified in the right format. \n Please specify the file name of a "
              "valid .bam file. Include the format in the file name.")
        raise SystemExit(1)
    if backend is None:
        backend = default_backend()
    consensusbam = bam.AlignmentFile(consensus_filename, "wb", template=inbam)
    excludedbam = bam.AlignmentFile("%s_filteredreads.bam" % consensus_filename[:-4], "wb", template=inbam)
    unprocessedbam = bam.AlignmentFile("%s_filteredfamilies.bam" % consensus_filename[:-4], "wb", template=inbam)

    run = _Run(params, backend, max(1, args.batch_families), consensusbam, unprocessedbam, args.verbose, rng)
    passed_reads = excluded_reads = 0
    family: Optional[list] = None
    code = None
    try:
        for read in inbam:
            try:
                ok = pass_filters(read, params.min_map_quality)
            except BaseException:
                run.drain()
                raise
            if not ok:
                excluded_reads += 1
                excludedbam.write(read)
                continue
            passed_reads += 1
            if family is None:                         # add_read_to_family (:1202-1217)
                family, code = [read], family_code_of(read)
            elif family_code_of(read) == code:
                family.append(read)
            else:
                run.family_done(family)
                family, code = [read], family_code_of(read)
        if family is None:
            # the reference calls preprocess_family(None, None) here (:1597) -> TypeError
            run.drain()
            raise TypeError("'NoneType' object is not iterable")
        run.family_done(family)
        run.drain()
        if args.verbose:
            print("\n Input file has been completely read \n")
        tot_r = passed_reads + excluded_reads
        tot_f = run.processed + run.excluded
        print("\n A total of %d reads (%.2f %%) passed the initial quality filters." %
              (passed_reads, passed_reads / tot_r * 100))
        print("\n A total of %d reads (%.2f %%) were filtered out." % (excluded_reads, excluded_reads / tot_r * 100))
        print("\n A total of %d families (%.2f %%) were successfully processed to generate a consensus read." %
              (run.processed, run.processed / tot_f * 100))
        print("\n A total of %d families (%.2f %%) were filtered out due to not enough reads to generate a "
              "consensus read." % (run.excluded, run.excluded / tot_f * 100))
    finally:
        excludedbam.close()
        unprocessedbam.close()
        consensusbam.close()
        inbam.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
