"""Command line drop-in for the reference script's ``main``
(DuplexUMIConsensusReads.py:1426-1650): same flags (``parse_args`` :10-91),
same output files, same stdout, same record order.

The per-record work runs natively (libdcr_io.so, include/dcr_io.h):

* the ingest reads the BAM (threaded BGZF inflate), applies ``pass_filters``
  (:1135-1181), groups MI runs (:1185-1217), checks and splits families and
  downsamples with CPython's MT19937 (:100-188), and packs whole batches of
  families into pinned host memory;
* the device runs the six ``make_consensus_read`` calls of every family of a
  batch (:1560-1582) in one asynchronous submit (stream.DeviceStream);
* the writer formats the duplex records (:1352-1419) and deflates BGZF
  blocks on a worker pool; excluded reads and filtered families are copied
  through as stored.

Batches are pipelined: a thread ingests batch k+1 while the device runs batch
k and the main thread writes batch k-1.

Failure semantics follow the reference: everything the reference writes
before it stops (consensus records of earlier families; side-file records up
to the failing family, ``dcr_host_batch.tab_*_cut``) is written, then its
exception, or its message and ``sys.exit(1)``, is raised at that family.
"""
from __future__ import annotations

import argparse
import contextlib
from concurrent.futures import ThreadPoolExecutor
import ctypes
import io
import os
import queue
import random
import shutil
import socket
import subprocess
import sys
import threading
import time
from typing import Optional

import numpy as np

from . import native_io
from .params import ConsensusParams

SPLIT_NAMES = {0: "A1", 1: "B2", 2: "B1", 3: "A2"}      # split_dict (:1511)
EQX_LINE = 'Symbols "x" and "=" were found in CIGAR strings and were changed to "M"'   # :375
STAGE_LINES = ("\t\t * Reconstruct alignment in progress", "\t\t * Call consensus in progress",
               "\t\t * Adjust consensus fields in progress")                            # :1318-1341
BADCHAR_LINE = ("\n ERROR: input values to nucleotide/INDEL list in function call_consensus() and subfunction "
                "most_likely_nucleotide() are different than the allowed ones. \n Please check documentation")


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
    # not reference flags: batching and codec knobs (they do not change any record)
    ap.add_argument("--batch_reads", required=False, default=int(os.environ.get("DCR_BATCH_READS", 1 << 19)), type=int,
                    help=argparse.SUPPRESS)   # DCR_BATCH_READS: A/B runs of the bench, which calls main() without flags
    ap.add_argument("--threads", required=False, default=0, type=int, help=argparse.SUPPRESS)
    ap.add_argument("--compression_level", required=False, default=6, type=int, help=argparse.SUPPRESS)
    ap.add_argument("--device", required=False, default=0, type=int, help=argparse.SUPPRESS)
    # one process per GPU over ranges of whole families (sharded mode below)
    ap.add_argument("--gpus", required=False, default=1, type=int, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


class ReferenceExit(SystemExit):
    """The reference prints an error and calls sys.exit(1)."""


def badchar_column(hb, f: int, k: int, min_base_quality: int):
    """The column most_likely_nucleotide prints before exiting on an invalid
    letter (:582-585), for single-strand consensus k of processed family f.

    Error reporting only (the device already decided the outcome): the reads
    are preprocessed as :191-325 do and laid out as reconstruct_alignment
    (:458-545) does until the first column holding a letter outside
    A T C G N a t c g n + -."""
    a = hb.a
    allowed = set("ATCGNatcgn+-")
    pos, cig, seq = [], [], []
    for r in range(int(a["sub_off"][4 * f + k]), int(a["sub_off"][4 * f + k + 1])):
        o, n = int(a["seq_off"][r]), int(a["seq_len"][r])
        s = a["bases"][o:o + n].tobytes().decode("latin-1")
        q = a["quals"][o:o + n]
        c0 = int(a["cig_off"][r])
        ops, s5, s3, inseq = [], 0, 0, False
        for w in a["cigar"][c0:c0 + int(a["cig_n"][r])]:
            op, ln = int(w) & 15, int(w) >> 4
            if op == 4:
                if not inseq:
                    s5 = ln
                else:
                    s3 = ln
            elif op != 5:
                inseq = True
                ops.append((op, ln))
        keep = slice(s5, -s3) if s3 else slice(s5, None)
        s, q = s[keep], q[keep]
        s = "".join("N" if qq < min_base_quality else ch for ch, qq in zip(s, q))
        tn = len(s) - len(s.rstrip("N"))
        s = s[:len(s) - tn]
        exp = [0 if op in (7, 8) else op for op, ln in ops for _ in range(ln)]
        pos.append(int(a["read_pos"][r]))
        cig.append(exp[:len(exp) - tn])
        seq.append(s)
    lo, hi = min(pos), max(p + len(s) for p, s in zip(pos, seq))
    ic, iz = [0] * len(pos), [0] * len(pos)
    for p in range(lo, hi):
        cur = [c[i] if i < len(c) else 99 for c, i in zip(cig, ic)]
        col = []
        if 1 in cur:
            for r, op in enumerate(cur):
                if op == 1:
                    col.append(seq[r][iz[r]].lower())
                    ic[r] += 1
                    iz[r] += 1
                else:
                    col.append("+")
        else:
            for r in range(len(pos)):
                if p < pos[r] or iz[r] >= len(seq[r]):
                    col.append("N")
                elif cig[r][ic[r]] == 2:
                    col.append("-")
                    ic[r] += 1
                else:
                    col.append(seq[r][iz[r]])
                    ic[r] += 1
                    iz[r] += 1
        if any(ch not in allowed for ch in col):
            return np.array(col)
    return None


_BACKENDS = {}        # device -> DeviceStream kept for later runs in this process


def default_backend(params: ConsensusParams, device: int = 0):
    """The HIP library on ``device`` (fails loudly without it: no CPU fallback).

    The context (stream, workspace, slots) and its pinned host batches are
    made once per process and device and reused by later ``main`` calls (a
    service that converts many BAMs, or the bench's repeated passes), as a
    caching host allocator would: the first call pays the allocation."""
    from . import _lib
    from .stream import DeviceStream
    if os.environ.get("DCR_BACKEND_CACHE") == "0":        # A/B runs: a fresh context per call
        return DeviceStream(_lib.Context(params, device=device), owns_ctx=True)
    be = _BACKENDS.get(device)
    if be is None or be.closed:
        ctx = _lib.Context(params, device=device)
        be = DeviceStream(ctx, owns_ctx=True, persistent=True)
        _BACKENDS[device] = be
        if len(_BACKENDS) == 1:
            import atexit
            atexit.register(_close_backends)
    elif be.ctx.params != params:
        be.ctx.set_params(params)
    return be


def _close_backends():
    for be in _BACKENDS.values():
        be.close(final=True)
    _BACKENDS.clear()
    if _INFLATERS:
        native_io.set_inflate_hook(None)
        for inf, _ in _INFLATERS.values():
            inf.close()
        _INFLATERS.clear()


_INFLATERS = {}       # device -> (_lib.Inflater, its hook), kept for later runs in this process


def gpu_inflate(device: int = 0):
    """BGZF inflate on ``device`` for the ingests this process opens from now
    on (include/dcr_inflate.h; the native ingest hands each chunk's members to
    the device inflater and takes its chunk buffers page-locked from it).
    One inflater per process and device, kept like the backend.

    On by default, DCR_GPU_INFLATE=0 keeps the host inflate pool.  The
    ingest streams the input's members to the device in spans launched ahead
    of the reader: measured whole-node on C2 it beats the host
    pool at input levels 1 and 6 (profiles/r03m).  A member is still ~4 ms of
    serial decode on one wavefront, so the per-chunk launches tried first
    lost (profiles/r03g, r03h)."""
    if os.environ.get("DCR_GPU_INFLATE") == "0":
        if native_io._HOOK is not None:
            native_io.set_inflate_hook(None)
        return None
    got = _INFLATERS.get(device)
    if got is None:
        from . import _lib
        inf = _lib.Inflater(device)
        got = (inf, inf.hook())
        _INFLATERS[device] = got
        if len(_INFLATERS) == 1 and not _BACKENDS:
            import atexit
            atexit.register(_close_backends)
    native_io.set_inflate_hook(got[1])
    return got[0]


def _as_backend(backend, params, device=0):
    if backend is None:
        return default_backend(params, device)
    if hasattr(backend, "submit"):
        return backend
    from .stream import CallBackend
    return CallBackend(backend, params)


def _raise_reference(kind: str, msg: str = ""):
    if kind == "exit":
        raise ReferenceExit(1)
    exc = {"IndexError": IndexError, "TypeError": TypeError, "ValueError": ValueError,
           "OverflowError": OverflowError, "AttributeError": AttributeError}.get(kind)
    if kind == "UnicodeEncodeError":
        raise UnicodeEncodeError("ascii", "", 0, 1, "ordinal not in range(128)")
    raise (exc or RuntimeError)(msg or f"reference would raise {kind} here")


class _Driver:
    def __init__(self, args, params, backend, ing, cons, excl, unproc):
        self.args, self.params, self.backend = args, params, backend
        self.ing, self.cons, self.excl, self.unproc = ing, cons, excl, unproc
        self.verbose = args.verbose
        # per-stage busy seconds and totals (bench.py --e2e reports them)
        self.trace = None          # optional [(stage, t0, t1)] (bench.py)
        self.ends_at_eof = True    # False for a sharded range that stops before the end
        self.stats = {"batches": 0, "consensus_records": 0, "consensus_bases": 0, "ingest_s": 0.0,
                      "submit_s": 0.0, "wait_s": 0.0, "write_s": 0.0, "idle_s": 0.0}

    # -- stdout of one batch, in the reference's order --------------------------
    def _prints(self, hb, fail_f, kind, which, last_batch):
        a = hb.a
        F = hb.n_fam
        eqx = a["fam_eqx"][:4 * F]
        if not self.verbose and fail_f >= F and not eqx.any():
            return
        if not self.verbose:
            # only the =/X lines (:374-375), per processed family in order
            nz = np.nonzero(eqx.reshape(F, 4).any(axis=1))[0] if F else []
            for f in nz:
                if f > fail_f:
                    break
                for k in range(4):
                    if f == fail_f and not self._ss_started(k, kind, which):
                        break
                    for _ in range(int(eqx[4 * f + k])):
                        print(EQX_LINE)
            return
        max_reads = self.params.max_reads
        n_tab = hb.s.n_tab
        for t in range(n_tab):
            kind_t, p = int(a["tab_kind"][t]), int(a["tab_proc"][t])
            code = hb.name(a["tab_code"][t])
            sampled = int(a["tab_sampled"][t])
            for k in range(4):                                              # :183-186
                if sampled >> k & 1:
                    print("Family", code, "subfamily", SPLIT_NAMES[k], "has been randomly downsampled to",
                          max_reads, "reads to form consensus read")
            if kind_t == native_io.FAM_FILTERED:
                print("Not enough reads in family", code, "to form consensus reads \n")       # :180
                continue
            failing = p == fail_f
            self._trim_prints(hb, p, kind if failing else None, which if failing else None)
            if failing and which >= 8:
                return
            for k in range(4):
                if failing and which == k and kind == "TypeError":
                    print("Single-strand consensus for subfamily", code, SPLIT_NAMES[k], "in progress")
                    return
                print("Single-strand consensus for subfamily", code, SPLIT_NAMES[k], "in progress")   # :1566-1567
                for _ in range(int(eqx[4 * p + k])):
                    print(EQX_LINE)
                if failing and which == k:
                    self._stage_prints(kind)
                    return
                for line in STAGE_LINES:
                    print(line)
            print("Double-strand consensus for family", code, "in progress")                    # :1578-1579
            for j in range(2):
                if failing and which == 4 + j and kind != "UnicodeEncodeError":
                    self._stage_prints(kind)
                    return
                for line in STAGE_LINES:
                    print(line)
                if failing and which == 4 + j:
                    return
            # the family the input's end completes (a range that ends early
            # completes its last family on the next family's first read)
            is_last = last_batch and t == n_tab - 1 and self.ends_at_eof
            print("Consensus reads for family", code,
                  "have been sucessfully writen \n" if is_last else "have been sucessfully written \n")  # :1597, :1631

    @staticmethod
    def _ss_started(k, kind, which):
        """Were subfamily k's =/X lines printed before the failure?"""
        if which >= 8:
            return False
        if which >= 4 or k < which:
            return True
        return k == which and kind != "TypeError"

    @staticmethod
    def _stage_prints(kind):
        """Stage lines printed before a consensus call fails (:1318-1341)."""
        n = {"exit": 2, "TypeError": 0}.get(kind, 3)
        for line in STAGE_LINES[:n]:
            print(line)

    def _trim_prints(self, hb, p, kind, which):
        """Verbose '3-prime N trimming' lines (:306-310): one per trailing 'N'
        after clip removal and masking, printing the masked sequence."""
        a = hb.a
        mb = self.params.min_base_quality
        r0, r1 = int(a["sub_off"][4 * p]), int(a["sub_off"][4 * p + 4])
        for r in range(r0, r1):
            o, n = int(a["seq_off"][r]), int(a["seq_len"][r])
            if n == 0:
                return
            cig = a["cigar"][int(a["cig_off"][r]):int(a["cig_off"][r]) + int(a["cig_n"][r])]
            s5 = s3 = 0
            inseq = False
            for c in cig:
                op, ln = int(c) & 15, int(c) >> 4
                if op == 4:
                    if not inseq:
                        s5 = ln
                    else:
                        s3 = ln
                elif op != 5:
                    inseq = True
            seq = a["bases"][o + s5:o + n - s3].copy()
            q = a["quals"][o + s5:o + n - s3]
            seq[q < mb] = ord("N")
            text = seq.tobytes().decode("latin-1")
            tn = len(text) - len(text.rstrip("N"))
            for _ in range(tn):
                print("3-prime N trimming has been performed on read", text)

    # -- one batch --------------------------------------------------------------
    def finish(self, hb, handle, last_batch):
        t0 = time.perf_counter()
        res = self.backend.result(handle)
        t1 = time.perf_counter()
        if self.trace is not None:
            self.trace.append(("wait", t0, t1))
        F = hb.n_fam
        st = self.stats
        if getattr(self.backend, "device_writer", False):
            # records formatted and compressed on the device (dcr_submit_write)
            nz = np.flatnonzero(res.fam_fail)
            fail_f = int(nz[0]) if len(nz) else F
            kind, which = None, -1
            if fail_f < F:
                code = int(res.fam_fail[fail_f])
                kind, which = native_io.FAIL_NAMES.get(code & 0xff), code >> 8
            self._prints(hb, fail_f, kind, which, last_batch)
            if fail_f == F:
                self.cons.put_blocks(res.bgzf, res.record_bytes)
            elif fail_f:
                self.cons.write(res.record_bytes_of(fail_f))
            lens = res.ds_len[:2 * fail_f]
        else:
            ss, ds, rstat = res
            fail_f, kind, which = native_io.first_failure(hb, ss, ds, F, rstat)
            self._prints(hb, fail_f, kind, which, last_batch)
            self.cons.write_consensus(hb, ss, ds, fail_f)
            lens = np.ctypeslib.as_array(ctypes.cast(ds.len, ctypes.POINTER(ctypes.c_int32)), (2 * F,))[:2 * fail_f] \
                if F else np.zeros(0, np.int32)
        st["batches"] += 1
        st["consensus_records"] += 2 * fail_f
        st["consensus_bases"] += int(lens.sum())
        st["wait_s"] += t1 - t0
        if fail_f < F:
            t = int(np.nonzero(hb.a["tab_proc"][:hb.s.n_tab] == fail_f)[0][0])
            exc_cut, filt_cut = int(hb.a["tab_exc_cut"][t]), int(hb.a["tab_filt_cut"][t])
        else:
            exc_cut, filt_cut = hb.s.n_side_exc, hb.s.n_side_filt
        self.excl.write(hb.a["side_exc"][:exc_cut])
        self.unproc.write(hb.a["side_filt"][:filt_cut])
        st["write_s"] += time.perf_counter() - t1
        if self.trace is not None:
            self.trace.append(("write", t1, time.perf_counter()))
        if fail_f < F:
            if kind == "exit":
                col = badchar_column(hb, fail_f, which, self.params.min_base_quality) if which < 4 else None
                if col is not None:
                    print("nucleotides = ", col)
                print(BADCHAR_LINE)
            _raise_reference(kind)
        if hb.end_kind == native_io.END_ERROR:
            ek, msg = hb.error()
            if ek == "exit":
                print(msg)
            _raise_reference(ek, msg)

    def run(self, batch_reads):
        """Ingest thread -> device -> writer, in input order."""
        n_buf = 4                       # filling, queued, on the device, being written
        free = queue.Queue()
        t0 = time.perf_counter()
        batches = [self.backend.host_batch(batch_reads) for _ in range(n_buf)]
        for hb in batches:
            free.put(hb)
        self.stats["alloc_s"] = time.perf_counter() - t0
        ready = queue.Queue()
        stop = threading.Event()

        first = [True]

        def ingest():
            try:
                while not stop.is_set():
                    hb = free.get()
                    if hb is None:
                        return
                    t0 = time.perf_counter()
                    if first[0] and hb.s.cap_reads >= (1 << 18):
                        # the first batch at an eighth of the capacities: the
                        # device starts on it while the rest of the pipeline
                        # fills (batch boundaries never change the outputs); a
                        # family too large for it takes the full batch
                        first[0] = False
                        caps = (hb.s.cap_fam, hb.s.cap_tab, hb.s.cap_reads, hb.s.cap_cigar, hb.s.cap_bases)
                        hb.s.cap_fam, hb.s.cap_tab = caps[0] // 8, caps[1] // 8
                        hb.s.cap_reads, hb.s.cap_cigar, hb.s.cap_bases = caps[2] // 8, caps[3] // 8, caps[4] // 8
                        try:
                            self.ing.next(hb)
                        except native_io.IOError_ as e:
                            if "exceeds the batch capacities" not in str(e):
                                raise
                            (hb.s.cap_fam, hb.s.cap_tab, hb.s.cap_reads, hb.s.cap_cigar, hb.s.cap_bases) = caps
                            self.ing.next(hb)
                        finally:
                            (hb.s.cap_fam, hb.s.cap_tab, hb.s.cap_reads, hb.s.cap_cigar, hb.s.cap_bases) = caps
                    else:
                        first[0] = False
                        self.ing.next(hb)
                    t1 = time.perf_counter()
                    self.stats["ingest_s"] += t1 - t0
                    if self.trace is not None:
                        self.trace.append(("ingest", t0, t1))
                    ready.put(hb)
                    if hb.end_kind != native_io.END_FULL:
                        return
            except BaseException as e:      # surfaced in the main thread
                ready.put(e)

        th = threading.Thread(target=ingest, name="dcr-ingest", daemon=True)
        th.start()
        pending = None
        try:
            while True:
                t0 = time.perf_counter()
                hb = ready.get()
                self.stats["idle_s"] += time.perf_counter() - t0
                if isinstance(hb, BaseException):
                    raise hb
                t0 = time.perf_counter()
                handle = self.backend.submit(hb)
                t1 = time.perf_counter()
                self.stats["submit_s"] += t1 - t0
                if self.trace is not None:
                    self.trace.append(("submit", t0, t1))
                if pending is not None:
                    self.finish(*pending, last_batch=False)
                    free.put(pending[0])
                pending = (hb, handle)
                if hb.end_kind != native_io.END_FULL:
                    break
            self.finish(*pending, last_batch=True)
            pending = None
        finally:
            stop.set()
            free.put(None)
            th.join()
            t0 = time.perf_counter()
            self.backend.close()
            if hasattr(self.backend, "release"):
                self.backend.release(batches)
            self.stats["backend_close_s"] = time.perf_counter() - t0


def main(argv: Optional[list] = None, backend=None, rng=random, stats: Optional[dict] = None) -> int:
    """``main`` (:1426-1650).  ``backend`` defaults to the HIP library;
    ``stats`` (optional) receives per-stage times and output totals."""
    t_start = time.perf_counter()
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)
    params = ConsensusParams.from_args(args)
    group = _shard_group()
    if group is not None:
        return _main_sharded(args, params, backend, rng, stats, group)
    if args.gpus > 1:
        return _launch_ranks(argv, args.gpus)
    if backend is None:
        gpu_inflate(args.device)       # the GPU path reads its input through the device inflater too
    try:
        ing = native_io.Ingest(args.input_file, params.min_map_quality, params.min_reads, params.max_reads,
                               params.min_base_quality, args.threads)
        if args.verbose:
            print(args.input_file, "has been read.")
    except Exception:
        print("ERROR: input file not found. \n Please specify file name of a valid .bam file. "
              "Include the format in the file name.")
        raise ReferenceExit(1)
    if args.output_file is None:
        consensus_filename = "%s_cons.bam" % args.input_file[:-4]
    elif args.output_file.endswith(".bam"):
        consensus_filename = args.output_file
    else:
        print("ERROR: output file is not specified in the right format. \n Please specify the file name of a "
              "valid .bam file. Include the format in the file name.")
        raise ReferenceExit(1)
    be = _as_backend(backend, params, args.device)
    cons, excl, unproc = _open_writers(
        [consensus_filename, "%s_filteredreads.bam" % consensus_filename[:-4],
         "%s_filteredfamilies.bam" % consensus_filename[:-4]], ing.header, args, ing)
    ing.set_rng_state(rng.getstate())
    t_open = time.perf_counter()
    try:
        drv = _Driver(args, params, be, ing, cons, excl, unproc)
        if stats is not None and "trace" in stats:
            drv.trace = stats["trace"]
        try:
            drv.run(max(args.batch_reads, 1))
        finally:
            if stats is not None:
                stats.update(drv.stats)
                stats["open_s"] = t_open - t_start
                stats["run_s"] = time.perf_counter() - t_open
        c = ing.counters()
        if stats is not None:
            stats.update(c)
        if args.verbose:
            print("\n Input file has been completely read \n")
        _print_summary(c)
    finally:
        t_close = time.perf_counter()
        try:
            rng.setstate(ing.rng_state(rng.getstate()))
        finally:
            try:
                _close_all(excl.close, unproc.close, cons.close)
            finally:
                t_wclose = time.perf_counter()
                ing.close()
        if stats is not None:
            stats["close_s"] = time.perf_counter() - t_close
            stats["close_writers_s"] = t_wclose - t_close
    return 0


def _close_all(*closers):
    """Call every closer even when one raises; re-raise the first error."""
    err = None
    for fn in closers:
        try:
            fn()
        except BaseException as e:          # noqa: BLE001 - re-raised below
            if err is None:
                err = e
    if err is not None:
        raise err


def _open_writers(paths, header, args, ing=None):
    """BGZF writers for ``paths``; when one fails to open, the ones already
    open are closed (and ``ing`` with them) before the error propagates."""
    ws = []
    try:
        for p in paths:
            ws.append(native_io.BgzfWriter(p, header, args.compression_level, args.threads))
    except BaseException:
        _close_all(*(w.close for w in ws), *((ing.close,) if ing is not None else ()))
        raise
    return ws


def _print_summary(c):
    """The closing counts (:1642-1649)."""
    passed_reads, excluded_reads = c["passed"], c["excluded"]
    processed, excluded = c["processed"], c["filtered"]
    tot_r, tot_f = passed_reads + excluded_reads, processed + excluded
    print("\n A total of %d reads (%.2f %%) passed the initial quality filters." %
          (passed_reads, passed_reads / tot_r * 100))
    print("\n A total of %d reads (%.2f %%) were filtered out." % (excluded_reads, excluded_reads / tot_r * 100))
    print("\n A total of %d families (%.2f %%) were successfully processed to generate a consensus read." %
          (processed, processed / tot_f * 100))
    print("\n A total of %d families (%.2f %%) were filtered out due to not enough reads to generate a "
          "consensus read." % (excluded, excluded / tot_f * 100))


# -- sharded mode: one process per GPU over ranges of whole families ---------------
#
# ``--gpus N`` relaunches the CLI as N ranks (torch.distributed.run, gloo for
# the small control messages; no data-path collective).  Rank 0 finds N-1
# split points, each the first read of a family (native_io.split_points);
# every rank runs the ordinary pipeline over its range into part files, and
# rank 0 concatenates the parts in order under the header, prints the ranks'
# stdout in order and the summary.  The result is the single-process result:
#   * a family never straddles two ranks, and a range that ends early
#     completes its last family there, as the reference does when the next
#     family's first read arrives;
#   * random.sample draws: the (population, size) of every call depends only
#     on the data, so each rank's exact starting state is the state after
#     the calls of the ranks before it.  A rank's ingest asks for that state
#     at its first random.sample call and waits for the earlier ranks' calls
#     (their own passes, or host-only count passes started on demand:
#     _StateExchange); no rank runs twice, and an input that is never
#     downsampled neither counts nor waits;
#   * the first failing rank ends the output exactly as the reference stops:
#     its parts are already cut where the reference stops writing, later
#     ranks are dropped and its exception is raised.

_EXC = {c.__name__: c for c in (IndexError, TypeError, ValueError, OverflowError, AttributeError, KeyError,
                                 ZeroDivisionError, UnicodeEncodeError)}
_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _shard_group():
    """(dist, rank, world) when this process is a rank of the sharded CLI
    (DCR_SHARD=1, set by _launch_ranks, in a torch.distributed group of more
    than one process), else None.  torch is only imported in that case."""
    if os.environ.get("DCR_SHARD") != "1":
        return None
    import torch.distributed as dist
    if not dist.is_initialized():
        if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
            return None
        # gloo announces its connections on file descriptor 1: keep them out
        # of the CLI's stdout
        sys.stdout.flush()
        saved, null = os.dup(1), os.open(os.devnull, os.O_WRONLY)
        os.dup2(null, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            os.dup2(saved, 1)
            os.close(saved)
            os.close(null)
    if dist.get_world_size() <= 1:
        return None
    return dist, dist.get_rank(), dist.get_world_size()


def _rank_device(args, local):
    """--device + the local rank, wrapped over the visible GPUs (counting them
    does not initialise the GPU on this stack)."""
    try:
        import torch
        n = torch.cuda.device_count()
    except Exception:
        n = 0
    return args.device + (local % n if n else local)


def _launch_ranks(argv, n):
    """N ranks of this CLI, one per GPU, started before anything here touches a GPU."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    rest = []
    skip = False
    for a in argv:                       # drop --gpus N / --gpus=N
        if skip:
            skip = False
            continue
        if a == "--gpus":
            skip = True
            continue
        if a.startswith("--gpus="):
            continue
        rest.append(a)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "duplexumiconsensusreads_amd.cli", *rest]
    env = dict(os.environ, DCR_SHARD="1")
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def _run_range(args, params, backend, path, rng, rng_state, rng_range, parts, device, gate=None, header=b""):
    """The ordinary pipeline over one range of families into ``parts``;
    stdout, outcome, counters and random.sample calls in a dict.  ``gate``
    (optional): the ingest's state gate (native_io.Ingest.set_state_gate).
    ``header``: rank 0 writes the final files themselves, header first."""
    res = {"status": "ok", "exc_args": (), "calls": [], "counters": None, "stdout": "", "stats": {},
           "sizes": [0, 0, 0]}
    out = io.StringIO()
    if backend is None:
        gpu_inflate(device)
    ing = native_io.Ingest(path, params.min_map_quality, params.min_reads, params.max_reads,
                           params.min_base_quality, args.threads, rng_range[0], rng_range[1])
    be = _as_backend(backend, params, device)
    cons, excl, unproc = _open_writers(parts, header, args, ing)
    ing.set_rng_state(rng_state)
    if gate is not None:
        ing.set_state_gate(gate)
    drv = _Driver(args, params, be, ing, cons, excl, unproc)
    drv.ends_at_eof = rng_range[1] == -1
    try:
        with contextlib.redirect_stdout(out):
            drv.run(max(args.batch_reads, 1))
    except ReferenceExit as e:
        res["status"], res["exc_args"] = "exit", (e.code,)
    except tuple(_EXC.values()) as e:
        res["status"], res["exc_args"] = type(e).__name__, e.args
    except Exception as e:                  # not a reference outcome: reported as is
        res["status"], res["exc_args"] = "error", (repr(e),)
    finally:
        res["calls"] = ing.sample_calls()
        res["counters"] = ing.counters()
        res["stats"] = dict(drv.stats)
        res["stdout"] = out.getvalue()
        try:
            _close_all(excl.close, unproc.close, cons.close)
        finally:
            ing.close()
        res["sizes"] = [os.path.getsize(p) for p in parts]
    return res


def _count_calls(path, params, rng_range, threads, stop, batch_reads=1 << 19):
    """The (population, size) of every random.sample call of one range, by a
    host-only ingest (host inflate, no device work, batches discarded): the
    calls depend only on the data (family and subfamily sizes), not on the
    generator's state.  Returns None (nothing to publish: the rank's own pass
    publishes) unless the ingest reached the end of the range or stopped where
    the reference stops; a stop request also gives None.  Batches are sized as
    the CLI's (``--batch_reads``), so a family the CLI can hold fits here."""
    ing = native_io.Ingest(path, params.min_map_quality, params.min_reads, params.max_reads,
                           params.min_base_quality, threads, rng_range[0], rng_range[1], host_inflate=True)
    complete = False
    try:
        hb = native_io.HostBatch(reads=max(batch_reads, 1))
        while not stop.is_set():
            ing.next(hb)
            if hb.end_kind != native_io.END_FULL:
                complete = True              # END_EOF, or END_ERROR: the calls up to the reference's stop
                break
    except Exception:  # noqa: BLE001 - an unfinished count is not published
        complete = False
    finally:
        calls = ing.sample_calls()
        ing.close()
    return calls if complete else None


class _StateExchange:
    """Rerun-free random.sample states for the sharded CLI.

    Rank r's exact starting state is the state after every call of the ranks
    before it.  Each rank's ingest is gated (``gate``): a rank that reaches
    its first random.sample call asks for that state, and waits only then; a
    rank that never samples never waits (its output does not depend on the
    state).  The calls of rank q are published in the process group's store
    by whichever finishes first: rank q's own pass, or a host-only count
    pass over rank q's range (``_count_calls``) that rank q starts in a
    thread once any rank has asked.  Nothing is counted, and nothing waits,
    for an input that is never downsampled."""

    _seq = 0

    _FAILED = b"failed"

    def __init__(self, dist, rank, world, s0, path, params, rng_range, threads, batch_reads=1 << 19):
        from datetime import timedelta
        _StateExchange._seq += 1       # every rank opens its exchanges in the same order
        self.store = dist.distributed_c10d._get_default_store()
        self.pre = "dcr_shard/%d/" % _StateExchange._seq
        self.rank, self.world, self.s0 = rank, world, s0
        self.wait_timeout = timedelta(hours=6)
        self.lock = threading.Lock()
        self.published = False
        self.gated_state = None
        self.wait_s = 0.0
        self.counted = False
        self.stop = threading.Event()
        self.th = None
        if rng_range is not None and rank < world - 1:
            # only later ranks read this rank's calls
            self.th = threading.Thread(target=self._counter, args=(path, params, rng_range, threads, batch_reads),
                                       name="dcr-count", daemon=True)
            self.th.start()

    def publish(self, calls):
        """``calls``: this range's random.sample calls; None marks the rank as
        failed before it knew them (a later rank's gate then raises instead
        of waiting for calls that never come)."""
        with self.lock:
            if self.published:
                return
            self.published = True
        val = self._FAILED if calls is None else np.asarray(calls, np.int32).reshape(-1).tobytes()
        self.store.set(self.pre + "calls%d" % self.rank, val)

    def _counter(self, path, params, rng_range, threads, batch_reads):
        from datetime import timedelta
        while not self.stop.is_set():
            try:
                self.store.wait([self.pre + "need"], timedelta(milliseconds=200))
                break
            except Exception:  # noqa: BLE001 - the store's timeout
                continue
        if self.stop.is_set() or self.published:
            return
        self.counted = True
        calls = _count_calls(path, params, rng_range, threads, self.stop, batch_reads)
        if calls is not None and not self.stop.is_set():
            self.publish(calls)

    def gate(self):
        """The ingest's state gate: the state after ranks 0..rank-1's calls."""
        t0 = time.perf_counter()
        self.store.set(self.pre + "need", b"1")
        keys = [self.pre + "calls%d" % q for q in range(self.rank)]
        if keys:
            self.store.wait(keys, self.wait_timeout)
        state = self.s0
        for k in keys:
            val = self.store.get(k)
            if val == self._FAILED:
                raise RuntimeError("%s: an earlier rank failed before publishing its random.sample calls" % k)
            flat = np.frombuffer(val, np.int32)
            state = native_io.py_replay(state, [(int(flat[2 * i]), int(flat[2 * i + 1]))
                                                for i in range(len(flat) // 2)])
        self.gated_state = state
        self.wait_s += time.perf_counter() - t0
        return state

    def close(self):
        self.stop.set()
        if self.th is not None:
            self.th.join()


def _copy_range(src, dst_fd, n, dst_off):
    """Bytes [0, n) of the file ``src`` into ``dst_fd`` at ``dst_off``, in the
    kernel (copy_file_range: no user-space round trip; a reflink where the
    file system has one)."""
    with open(src, "rb") as f:
        fd, done = f.fileno(), 0
        while done < n:
            try:
                k = os.copy_file_range(fd, dst_fd, n - done, done, dst_off + done)
            except OSError:
                k = 0
            if k <= 0:                      # no copy_file_range here: pread / pwrite
                chunk = os.pread(fd, min(n - done, 64 << 20), done)
                if not chunk:
                    raise IOError(f"{src}: short part file")
                k = os.pwrite(dst_fd, chunk, dst_off + done)
            done += k


def _part_dir(finals):
    """Where ranks 1..N-1 write their parts: a memory-backed directory when
    there is one with room (DCR_PART_DIR overrides), else beside the output.
    A part is written once there during the pass and once into the final
    file at the merge, from memory (no second trip through the file system)."""
    d = os.environ.get("DCR_PART_DIR")
    if d:
        return d
    try:
        st = os.statvfs("/dev/shm")
        if st.f_bavail * st.f_frsize >= (16 << 30):
            return "/dev/shm"
    except OSError:
        pass
    return os.path.dirname(os.path.abspath(finals[0]))


def _write_part_at(part, final, n, off, threads=4, mapped=False):
    """``n`` bytes of ``part`` written into ``final`` at ``off`` by a few
    threads, the part mapped.  ``mapped``: the final file's range is already
    allocated (rank 0's posix_fallocate before the offsets are broadcast), so
    the range is mapped too and the slices are plain memory copies (page
    faults of one file proceed in parallel, buffered writes to it take the
    inode lock in turn: 200 MB in 0.075 s against 0.15 s by pwrite on ext4).
    Otherwise the slices are pwritten from the mapped part (page-cache writes
    from user memory run about twice the rate of copy_file_range between two
    files)."""
    import mmap
    if not n:
        return
    fd = os.open(final, os.O_RDWR if mapped else os.O_WRONLY)
    try:
        with open(part, "rb") as f:
            mm = mmap.mmap(f.fileno(), n, prot=mmap.PROT_READ)
        step = max(1 << 20, -(-n // threads))
        step = (step + 4095) & ~4095
        starts = range(0, n, step)
        # a mapping past the end of the file faults (SIGBUS): map only a range the file holds
        if mapped and os.fstat(fd).st_size >= off + n:
            a0 = off & ~(mmap.ALLOCATIONGRANULARITY - 1)
            dm = mmap.mmap(fd, off + n - a0, offset=a0)
            views = [np.frombuffer(dm, np.uint8)[off - a0:], np.frombuffer(mm, np.uint8)]
            try:
                def copy(a):
                    np.copyto(views[0][a:a + step], views[1][a:a + step])
                with ThreadPoolExecutor(threads) as ex:
                    list(ex.map(copy, starts))
            finally:
                views.clear()                # the arrays export the mappings: released before closing
                dm.close()
                mm.close()
            return
        try:
            view = memoryview(mm)

            def put(a):
                b = min(a + step, n)
                while a < b:
                    a += os.pwrite(fd, view[a:b], off + a)
            if n <= step:
                put(0)
            else:
                with ThreadPoolExecutor(threads) as ex:
                    list(ex.map(put, starts))
        finally:
            view.release()
            mm.close()
    finally:
        os.close(fd)


def _merge_parallel(dist, rank, finals, header, args, sizes, upto, parts):
    """The output files, each byte written once into them.  Rank 0 wrote its
    range straight into the final files (header, records, EOF); rank r > 0
    writes its part (without its EOF block) at rank 0's length minus its EOF
    plus the sizes of parts 1..r-1, an exclusive scan of the part sizes every
    rank holds (``sizes[r][k]``), all ranks at once, into ranges rank 0 has
    allocated (posix_fallocate) before it broadcasts the offsets; rank 0 then
    puts the BGZF EOF block at the end."""
    eof = len(_BGZF_EOF)
    if rank == 0:
        for k in range(3):
            if sizes[0][k] == 0:             # rank 0 never opened its writers: the header alone
                w = native_io.BgzfWriter(finals[k], header, args.compression_level, args.threads)
                w.close()
                sizes[0][k] = os.path.getsize(finals[k])

    def ends_of(s0):
        return [s0[k] - eof + sum(max(sizes[r][k] - eof, 0) for r in range(1, upto)) for k in range(3)]
    mapped = False
    if rank == 0 and upto > 1:
        # the finals' whole length allocated before any rank writes: the
        # ranks then copy into mapped ranges (no fault can meet a missing
        # block or the end of the file); a file system without fallocate
        # keeps the pwrite path
        mapped = True
        for k, e in enumerate(ends_of([sizes[0][j] for j in range(3)])):
            fd = os.open(finals[k], os.O_RDWR)
            try:
                start = sizes[0][k] - eof
                if e + eof > start:
                    os.posix_fallocate(fd, start, e + eof - start)
            except OSError:
                mapped = False
            finally:
                os.close(fd)
    obj = [[sizes[0][k] for k in range(3)], mapped]
    dist.broadcast_object_list(obj, src=0)
    s0, mapped = obj
    ends = ends_of(s0)
    for k in range(3):
        off = s0[k] - eof
        for r in range(1, upto):
            n = max(sizes[r][k] - eof, 0)
            if r == rank and n:
                _write_part_at(parts[k], finals[k], n, off, mapped=mapped)
            off += n
    if rank == 0:
        for k in range(3):
            fd = os.open(finals[k], os.O_WRONLY)
            try:
                os.pwrite(fd, _BGZF_EOF, ends[k])
                if os.fstat(fd).st_size != ends[k] + eof:   # already so when the finals were allocated
                    os.ftruncate(fd, ends[k] + eof)
            finally:
                os.close(fd)
    dist.barrier()


def _main_sharded(args, params, backend, rng, stats, group):
    dist, rank, world = group
    path = args.input_file
    try:
        header = native_io.bam_header(path)
        in_ok = True
    except Exception:
        in_ok = False
    if not in_ok:
        if rank == 0:
            print("ERROR: input file not found. \n Please specify file name of a valid .bam file. "
                  "Include the format in the file name.")
        raise ReferenceExit(1)
    if rank == 0 and args.verbose:
        print(path, "has been read.")
    if args.output_file is None:
        consensus_filename = "%s_cons.bam" % path[:-4]
    elif args.output_file.endswith(".bam"):
        consensus_filename = args.output_file
    else:
        if rank == 0:
            print("ERROR: output file is not specified in the right format. \n Please specify the file name of a "
                  "valid .bam file. Include the format in the file name.")
        raise ReferenceExit(1)
    finals = [consensus_filename, "%s_filteredreads.bam" % consensus_filename[:-4],
              "%s_filteredfamilies.bam" % consensus_filename[:-4]]
    obj = [native_io.split_points(path, world, params) if rank == 0 else None,
           rng.getstate() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    splits, s0 = obj
    pts = [0] + [v for v in splits if v != -1]
    ranges = [(pts[i], pts[i + 1] if i + 1 < len(pts) else -1) for i in range(len(pts))]
    mine = ranges[rank] if rank < len(ranges) else None
    # rank 0 writes the final files themselves; the others write parts that
    # the merge puts in place once their offsets are known
    if rank == 0:
        parts = list(finals)
    else:
        pd = _part_dir(finals)
        parts = [os.path.join(pd, "%s.%d.part%d" % (os.path.basename(f), os.getppid(), rank)) for f in finals]
    local = int(os.environ.get("LOCAL_RANK", rank))
    device = _rank_device(args, local) if backend is None else args.device
    empty = {"status": "ok", "exc_args": (), "calls": [], "counters": None, "stdout": "", "stats": {},
             "sizes": [0, 0, 0]}
    result, used, rounds = empty, None, 0
    xch = _StateExchange(dist, rank, world, s0, path, params, mine, args.threads, args.batch_reads)
    done = False
    try:
        if mine is not None:
            result = _run_range(args, params, backend, path, rng, s0, mine, parts, device,
                                gate=xch.gate if rank > 0 else None, header=header if rank == 0 else b"")
            used, rounds = (xch.gated_state or s0), 1
        done = True
    finally:
        # this rank's calls for the later ranks (if no count pass published
        # them first); a rank that raised before knowing them publishes the
        # failure marker, so no later rank's gate waits for them
        xch.publish(result["calls"] if done else None)
        xch.close()
    # a safety net only: with the gate, a rank sampled from its exact state
    while True:
        results = [None] * world
        dist.all_gather_object(results, result)
        # this rank's exact starting state: the calls of the (ok) ranks before it
        state, target = s0, None
        for r in range(rank):
            if results[r]["status"] != "ok":
                break
            state = native_io.py_replay(state, results[r]["calls"])
        else:
            target = state
        # a rank that never sampled does not depend on the state
        again = bool(mine is not None and target is not None and result["calls"] and target != used)
        flags = [None] * world
        dist.all_gather_object(flags, again)
        if not any(flags):
            break
        if again:
            result = _run_range(args, params, backend, path, rng, target, mine, parts, device,
                                header=header if rank == 0 else b"")
            used = target
            rounds += 1
    if stats is not None:
        stats.update(result["stats"])
        stats["shard_rounds"] = rounds
        stats["state_wait_s"] = xch.wait_s
        stats["count_pass"] = xch.counted
    # the first failing rank ends the output as the reference stops; later
    # ranks are dropped (every rank derives the same cut from the results)
    fail = next((r for r in range(world) if results[r]["status"] != "ok"), None)
    upto = min((fail + 1) if fail is not None else world, len(ranges))
    t_merge = time.perf_counter()
    _merge_parallel(dist, rank, finals, header, args, [list(results[r]["sizes"]) for r in range(world)], upto,
                    parts)
    if stats is not None:
        stats["merge_s"] = time.perf_counter() - t_merge
    if rank == 0:
        sys.stdout.write("".join(results[r]["stdout"] for r in range(upto)))
        state = s0
        for r in range(upto):
            state = native_io.py_replay(state, results[r]["calls"])
        if stats is not None:
            stats["ranks"] = [results[r]["stats"] for r in range(world)]
    if rank != 0:
        for p in parts:
            if os.path.exists(p):
                os.remove(p)
        return 0
    rng.setstate(state)
    if fail is None:
        tot = {}
        for r in range(min(world, len(ranges))):
            for k, v in (results[r]["counters"] or {}).items():
                tot[k] = tot.get(k, 0) + v
        if args.verbose:
            print("\n Input file has been completely read \n")
        _print_summary(tot)
        return 0
    st, ea = results[fail]["status"], results[fail]["exc_args"]
    if st == "exit":
        raise ReferenceExit(*ea)
    if st in _EXC:
        raise _EXC[st](*ea)
    raise RuntimeError(f"rank {fail}: {ea[0] if ea else st}")


if __name__ == "__main__":
    sys.exit(main())
