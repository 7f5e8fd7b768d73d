"""Benchmark: consensus bases/s of the duplex-consensus drop-in on MI355X,
whole node, plus the SSCS kernel's HBM roofline.

Workload (BASELINE.json configs[1]): per GPU a synthetic
duplex BAM of 10 M reads = 312,500 MI families x 4 subfamilies x 8 reads,
2x150 bp ``150M`` reads, no indels, qualities {Q37 .80, Q25 .12, Q12 .08}.

value: one step = one run of the CLI drop-in (cli.main, the reference's
``main`` DuplexUMIConsensusReads.py:1426-1650) over that BAM, from opening
the input to closing the three outputs: native ingest (BGZF inflate,
filters, grouping, downsampling, packing into pinned memory), asynchronous
device batches (H2D, kernels, D2H on side streams), native record writer and
BGZF deflate.  value = duplex consensus bases written by all ranks / the
slowest rank's time (SURVEY.md §8d metric (1)).  The per-stage busy times are
in config.stages.

roofline: the single-strand kernel k_consensus_fast<ss> on the same batch
with its inputs resident in HBM (K device-only passes, HIP events on the
context stream): SURVEY.md §8d algorithmic bytes / average launch / 8 TB/s.
config.device_resident holds that loop's consensus bases/s (kernels only).

cpu_baseline: the whole node on the CPU, like for like with value: the same
CLI over the same C2 BAM with the C restatement (oracle/, kind "port") as the
consensus backend on the host cores, host BGZF inflate and host record
writer / deflate (no GPU anywhere), timed from BAM open to output close; the
cores are the box's CPU quota (cgroup cpu.max).  Its ``kernels_only`` field
is the restatement alone on the packed batch (no BAM I/O).

--config C3 / C4 / C5 runs the other BASELINE.json shapes (per-GPU shards).
Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2]
(N > 1 is launched by torch.distributed.run, one process per GPU; every rank
owns its own shard of families: weak scaling, no data-path collective.  C4
at N > 1 deals one shared stream of N x 1,000 families to the ranks by LPT.)

N > 1 (the driver's scaling runs) times the drop-in's own multi-GPU mode by
default: ONE input BAM holding every rank's families (N x 312,500 on C2,
assembled from the ranks' BGZF pieces) through the sharded CLI (cli --gpus:
split points at family starts, one process per GPU over its range, parallel
part merge), every pass between barriers on all ranks; per-GPU work is fixed
("weak").  --independent times one private BAM per rank instead.
--sharded-input-of-rank0 splits rank 0's batch alone over the N ranks
(strong scaling of one 10 M-read input).  --in-level sets the input's BGZF
level (default 1; 6 is samtools' default).
"""
from __future__ import annotations

import argparse
import faulthandler
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

faulthandler.enable()     # a native crash prints the Python stacks to stderr

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "consensus bases/sec (whole node) + SSCS kernel HBM GB/s vs peak, 1/2/4/8 GPUs"

# families per GPU for each workload shape (weak scaling: every rank its own shard)
CONFIG_FAMILIES = {
    "C2": 312_500,     # 10 M reads: 4 subfamilies x 8 reads
    "C3": 400_000,     # ~12.5 M reads = C3's 100 M reads / 8 GPUs; Zipf(1.5) 1..100, 5% indels, 3% clips
    "C4": 1_000,       # 20 loci x 50 families, subfamilies log-uniform 100..1000 (--max_reads 1000)
    "C5": 200_000,     # one 4 M-read streaming chunk of the 1 B-read run: Poisson(4)+1
}
WORKLOAD = {
    "C2": "C2 (BASELINE.json configs[1]): 10M-read synthetic duplex BAM per GPU, 312,500 MI families x "
          "4 subfamilies x 8 reads, 2x150bp, no indels",
    "C3": "C3 shape (BASELINE.json configs[2]) per GPU: skewed subfamilies Zipf(1.5) on 1..100, 5% of reads with "
          "a 1-3 bp indel, 3% soft-clipped, 2x150bp",
    "C4": "C4 shape (BASELINE.json configs[3]): 20 loci x 50 families, subfamilies log-uniform 100..1000 reads "
          "(--max_reads 1000), 2x150bp",
    "C5": "C5 shape (BASELINE.json configs[4]): one 4M-read chunk, subfamilies Poisson(4)+1, 2x150bp",
}


def make_batch(config, families, seed, max_reads=1000):
    from duplexumiconsensusreads_amd import synth
    if config == "C2":
        return synth.packed_fixed_size(families, seed=seed)
    return synth.packed_config(synth.CONFIGS[config], families, seed=seed, max_reads=max_reads)


def shared_share(config, families, seed, rank, world):
    """C4 at N > 1 (the load-balance case): one shared stream
    of families x N families, cut into consecutive chunks and dealt to ranks
    by LPT on their read bases (shard.rank_share), so a few deep families do
    not pile onto one GPU.  Every rank plans from the stream's family sizes
    (cheap, identical on all ranks) and generates only its own families."""
    from duplexumiconsensusreads_amd import shard, synth
    cfg = synth.CONFIGS[config]
    total = families * world
    costs = (synth.config_family_reads(cfg, total, seed, max_reads=1000) * cfg.read_len).tolist()
    mine, loads = shard.rank_share(costs, rank, world)
    packed = synth.packed_config(cfg, total, seed=seed, max_reads=1000, keep=mine)
    mean = sum(loads) / world
    return packed, {"families": total, "rank_read_bases": loads,
                    "max_over_mean": (max(loads) / mean) if mean else None,
                    "split": "consecutive chunks of ~1/32 of a rank's share, dealt by LPT (shard.rank_share)"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def sscs_algorithmic_bytes(packed, padded=False):
    """sum_r(2 len_r + 4 n_cig_r + 4 + 1) + T*(2 + 4) + 16 per
    subfamily, T = max(pos_r + len_r) - min(pos_r) (:458-459, on the input
    reads' query lengths: 150 on C2).  ``padded``: T is the subfamily's output
    region instead (T rounded up to 16 columns, the bytes the kernel stores)."""
    per_read = 2 * packed.seq_len.astype(np.int64) + 4 * packed.cig_n.astype(np.int64) + 5
    reads_b = int(per_read.sum())
    n_sub = len(packed.ss_col_off) - 1
    if padded:
        cols = int(packed.ss_col_off[-1])
    else:
        so = packed.sub_off.astype(np.int64)
        pos = packed.read_pos.astype(np.int64)
        end = pos + packed.seq_len.astype(np.int64)
        nonempty = so[1:] > so[:-1]
        starts = so[:-1][nonempty]
        cols = int((np.maximum.reduceat(end, starts) - np.minimum.reduceat(pos, starts)).sum()) if len(starts) else 0
    return reads_b + 6 * cols + 16 * n_sub


def cpu_baseline(packed, reps):
    """The C restatement (oracle/dcr_oracle.c, test infrastructure used here
    only as the timed CPU leg) over the bench batch itself, multi-threaded
    over families.  The C2 batch takes ~1-2 s per pass on 16 threads, so the
    sample is the whole batch, repeated ``reps`` times (~10-30 thread-s)."""
    from duplexumiconsensusreads_amd.params import ConsensusParams
    from oracle import dcr_oracle_c
    threads = min(16, os.cpu_count() or 1)   # the GPU box's CPU share is 16
    dts, bases = [], 0
    for _ in range(reps):
        t0 = time.perf_counter()
        _, ds, _ = dcr_oracle_c.run(packed, ConsensusParams(), n_threads=threads, want_info=False)
        dts.append(time.perf_counter() - t0)
        bases = int(ds.len.sum())
        del ds
    dt = min(dts)
    return {"value": bases / dt, "unit": "consensus bases/s", "cores": threads, "kind": "port",
            "sample": f"the whole bench batch ({packed.n_fam} families, {packed.n_reads} reads), "
                      f"C restatement oracle/dcr_oracle.c on {threads} threads, kernels only (no BAM I/O), "
                      f"best of {reps}: {dt:.2f} s per pass"}


def cpu_cores():
    """(cores of the process's CPU quota or None, os.cpu_count()): the GPU box
    runs under a cgroup quota (cpu.max 1600000/100000 = 16 cores) on a host
    with many more CPUs."""
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return quota, os.cpu_count()


def cpu_baseline_whole_node(bam_path, params_args, workdir, reps, threads):
    """The CLI drop-in over the bench BAM with no GPU: the C restatement as
    the consensus backend (oracle/dcr_oracle_c.run on ``threads`` threads,
    test infrastructure used here only as the timed CPU leg), the native
    ingest's host inflate pool and the host record writer / BGZF deflate.
    Best of ``reps`` passes, each from BAM open to output close."""
    import contextlib
    import io
    import random
    from duplexumiconsensusreads_amd import cli, native_io
    from oracle import dcr_oracle_c

    def oracle(packed, params):
        return dcr_oracle_c.run(packed, params, n_threads=threads)

    hook = native_io._HOOK
    native_io.set_inflate_hook(None)            # the host inflate pool (no device inflater)
    dts, st = [], {}
    try:
        for i in range(reps):
            for f in os.listdir(workdir):
                if f.startswith("cpu"):
                    os.remove(os.path.join(workdir, f))
            st = {}
            random.seed(4)
            t0 = time.perf_counter()
            with contextlib.redirect_stdout(io.StringIO()):
                cli.main(["-i", bam_path, "-o", os.path.join(workdir, f"cpu{i}.bam"), *params_args],
                         backend=oracle, stats=st)
            dts.append(time.perf_counter() - t0)
    finally:
        native_io.set_inflate_hook(hook)
    dt = min(dts)
    return st.get("consensus_bases", 0) / dt, dt, st


def load_traffic(kernel, n_fam):
    """HBM bytes per launch of ``kernel`` from the committed PMC passes
    (tools/pmc_traffic.py -> profiles/traffic.json: FETCH_SIZE x2 + WRITE_SIZE,
    MI355X_MICROARCH.md §HBM), scaled to this batch when the profiled batch
    had a different family count; None when absent."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        k = t["kernels"][kernel]
        return k["hbm_bytes_per_launch"] * n_fam / t["families"], t
    except (OSError, KeyError, ValueError, ZeroDivisionError):
        return None, None


def device_resident(packed, params, local, steps, warmup):
    """K device-only passes over the batch resident in HBM (kernel timing)."""
    import torch
    from duplexumiconsensusreads_amd import _lib
    from duplexumiconsensusreads_amd.device import DeviceBatch
    db = DeviceBatch(packed, device=f"cuda:{local}")
    ctx = _lib.Context(params, device=local)
    ctx.reserve(db.batch_struct)
    torch.cuda.synchronize()
    for _ in range(warmup):
        ctx.run_device(db.batch_struct, db.ss_struct, db.ds_struct)
    ctx.sync()
    st_ss = db.out["ss"]["status"][:4 * packed.n_fam]
    st_ds = db.out["ds"]["status"][:2 * packed.n_fam]
    n_bad = int((st_ss != 0).sum().item() + (st_ds != 0).sum().item())
    bases = int(db.out["ds"]["len"].view(torch.int32)[:2 * packed.n_fam].sum().item())
    kms = {k: 0.0 for k in _lib.KERNELS}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.run_device(db.batch_struct, db.ss_struct, db.ds_struct)
        tm = ctx.last_kernel_timing()   # waits on this step's events only
        for k in kms:
            kms[k] += tm[k]
    ctx.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ctx.close()
    del db
    torch.cuda.empty_cache()
    return {k: v / steps for k, v in kms.items()}, bases, n_bad, dt / steps


def one_input_bam(path, packed, seed, level, rank, world, tdist):
    """ONE BAM of every rank's families (the sharded CLI's input at N > 1):
    each rank writes its records as BGZF blocks, rank 0 the header, and every
    rank copies its piece (EOF block dropped) to its offset in ``path`` (an
    exclusive scan of the piece sizes), as the CLI's parallel merge does."""
    from duplexumiconsensusreads_amd import cli, native_io, synth
    eof = len(cli._BGZF_EOF)
    piece = f"{path}.piece{rank}"
    synth.write_packed_bam(piece, packed, seed=seed, level=level, header=False)
    head = f"{path}.head"
    if rank == 0:
        w = native_io.BgzfWriter(head, synth.BamHeader_bytes(), level=level)
        w.close()
    sizes = [None] * world
    tdist.all_gather_object(sizes, os.path.getsize(piece) - eof)
    tdist.barrier()
    hl = os.path.getsize(head) - eof
    if rank == 0:
        with open(path, "wb") as f:
            f.truncate(hl + sum(sizes) + eof)
        fd = os.open(path, os.O_WRONLY)
        cli._copy_range(head, fd, hl, 0)
        os.pwrite(fd, cli._BGZF_EOF, hl + sum(sizes))
        os.close(fd)
    tdist.barrier()
    fd = os.open(path, os.O_WRONLY)
    cli._copy_range(piece, fd, sizes[rank], hl + sum(sizes[:rank]))
    os.close(fd)
    os.remove(piece)
    tdist.barrier()


def e2e_passes(path, params_args, device, steps, warmup, workdir):
    """W untimed + K timed CLI runs over the BAM at ``path``; returns
    (seconds of the K runs, stats of the last run)."""
    from duplexumiconsensusreads_amd import cli
    import contextlib
    import io

    def argv_of(i):
        # a fresh output name per pass (the previous pass's files deleted
        # outside the timed region): every pass writes new files, as a
        # first-time run does, never a rewrite of the last pass's outputs
        for f in os.listdir(workdir):
            if f.startswith("cons"):
                os.remove(os.path.join(workdir, f))
        out = os.path.join(workdir, f"cons{i}.bam")
        return ["-i", path, "-o", out, "--device", str(device), *params_args]

    import random
    cold = None
    for i in range(warmup):
        argv = argv_of(i)
        random.seed(4)                  # downsampling draws from random.seed(4)
        tw = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            cli.main(argv)
        cold = time.perf_counter() - tw if cold is None else cold
    stats = {}
    # the CLI keeps its device context and pinned host batches per process
    # (cli.default_backend): the warmup passes pay their allocation, timed
    # passes reuse them, as a long-running converter would
    dt = 0.0
    passes = []
    infl = cli._INFLATERS.get(device)
    if infl is not None:
        infl[0].totals(reset=True)
    cpu0 = os.times()                   # the process's user + system CPU seconds (every thread)
    for i in range(steps):
        argv = argv_of(warmup + i)
        stats = {"trace": []}
        random.seed(4)
        t_pass = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            cli.main(argv, stats=stats)
        dt_pass = time.perf_counter() - t_pass
        dt += dt_pass
        passes.append(round(dt_pass, 4))
    cpu1 = os.times()
    trace = stats.pop("trace")
    log("last pass timeline (ms from CLI start): " +
        " ".join(f"{k}[{(a - t_pass) * 1e3:.0f},{(b - t_pass) * 1e3:.0f}]" for k, a, b in trace))
    stats["first_pass_s"] = cold        # the cold first pass (allocations included)
    stats["passes_s"] = passes
    stats["host_cpu_s_per_pass"] = round(((cpu1.user - cpu0.user) + (cpu1.system - cpu0.system)) / max(steps, 1), 4)
    if infl is not None:                # BGZF inflate on the device (cli.gpu_inflate)
        t = infl[0].totals()
        stats["gpu_inflate"] = {"kernel_ms_per_pass": t["kernel_ms"] / max(steps, 1),
                                "launches_per_pass": t["runs"] / max(steps, 1),
                                "GBps_of_output_in_kernel": (t["bytes"] / (t["kernel_ms"] * 1e6)) if t["kernel_ms"] else None}
    else:
        stats["gpu_inflate"] = None
    return dt, stats


def e2e_passes_sharded(path, params_args, steps, warmup, workdir, tdist, rank):
    """--sharded: W untimed + K timed runs of the sharded CLI (cli.main with
    one rank per GPU over ranges of whole families of ONE input,
    cli._main_sharded) on all ranks at once; each pass is bracketed by
    barriers, its time is this rank's view of the slowest rank.  Returns
    (seconds of the K runs, this rank's stats of the last run)."""
    from duplexumiconsensusreads_amd import cli
    import contextlib
    import io
    os.environ["DCR_SHARD"] = "1"           # cli.main joins this process group (cli._shard_group)

    def one(i, stats):
        if rank == 0:
            for f in os.listdir(workdir):
                if f.startswith("cons"):
                    os.remove(os.path.join(workdir, f))
        out = os.path.join(workdir, f"cons{i}.bam")
        argv = ["-i", path, "-o", out, "--device", "0", *params_args]
        if tdist is not None:
            tdist.barrier()
        t = time.perf_counter()
        with contextlib.redirect_stdout(io.StringIO()):
            cli.main(argv, stats=stats)
        if tdist is not None:
            tdist.barrier()
        return time.perf_counter() - t

    for i in range(warmup):
        one(i, {})
    dt, passes, stats = 0.0, [], {}
    for i in range(steps):
        stats = {}
        d = one(warmup + i, stats)
        dt += d
        passes.append(round(d, 4))
    stats["passes_s"] = passes
    return dt, stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIG_FAMILIES),
                    help="workload shape (SURVEY.md §8d); C2 is the headline line, the others are "
                         "per-GPU shards of C3 / C4 / C5 reported for coverage")
    ap.add_argument("--families", type=int, default=None, help="families per GPU (C2: 312,500)")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-reps", type=int, default=2, help="passes of the CPU baseline over the batch")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--kernel-only", action="store_true", help="skip the whole-node CLI runs")
    ap.add_argument("--kernel-steps", type=int, default=10, help="device-resident passes for the roofline")
    ap.add_argument("--sharded", action="store_true",
                    help="the sharded CLI over ONE input (the default at N > 1; at N = 1 the plain CLI)")
    ap.add_argument("--independent", action="store_true",
                    help="N > 1: one private BAM per rank through the plain CLI (no sharding)")
    ap.add_argument("--sharded-input-of-rank0", action="store_true",
                    help="strong scaling: ONE input of rank 0's batch only, split over the N ranks")
    ap.add_argument("--in-level", type=int, default=1, help="BGZF compression level of the synthetic input BAM")
    ap.add_argument("--level6-passes", type=int, default=2,
                    help="single GPU: timed CLI passes over the same families written at BGZF level 6 "
                         "(reported beside the headline in config; 0 skips)")
    ap.add_argument("--max-reads", type=int, default=None,
                    help="--max_reads of the CLI runs (default: the reference's 100; C4: 1000, the whole deep "
                         "subfamilies).  Below a config's subfamily sizes the CLI downsamples (random.seed(4)); "
                         "the device-resident batch is then capped at the same size")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # ranks beyond the visible GPUs share them (the sharded CLI's rehearsal
    # on a one-GPU box); counting devices does not initialise the GPU
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    dist = world > 1
    # N > 1: the drop-in's own multi-GPU mode (one input, cli --gpus) unless --independent
    args.sharded = (args.sharded or args.sharded_input_of_rank0 or dist) and not args.independent
    one_input_of_all = args.sharded and not args.sharded_input_of_rank0
    dev = f"cuda:{local}"
    tdist = None
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if args.sharded:      # the sharded CLI's control messages (no data-path collective) ride on gloo
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device(dev))
    red_dev = None if args.sharded else dev
    from duplexumiconsensusreads_amd import _lib, shard, synth
    from duplexumiconsensusreads_amd.params import ConsensusParams

    t0 = time.perf_counter()
    families = args.families or CONFIG_FAMILIES[args.config]
    shared = None
    max_reads = args.max_reads if args.max_reads is not None else (1000 if args.config == "C4" else 100)
    bam_packed = None            # the BAM's families when the CLI downsamples them (C4 at --max-reads 100)
    if args.config == "C4" and dist:
        packed, shared = shared_share(args.config, families, args.seed, rank, world)
    else:
        packed = make_batch(args.config, families, args.seed + 1000 * rank, max_reads=min(max_reads, 1000))
        if args.config != "C2" and max_reads < 1000:
            bam_packed = make_batch(args.config, families, args.seed + 1000 * rank, max_reads=1000)
    log(f"[rank {rank}] generated {packed.n_reads} reads in {time.perf_counter() - t0:.1f} s")
    # C4 runs with --max_reads 1000 by default (the deep families whole)
    params = ConsensusParams(max_reads=max_reads)
    params_args = ["--max_reads", str(max_reads)] if max_reads != 100 else []

    # -- SSCS kernel roofline: device-resident passes ------------------------------
    kavg, dev_bases, n_bad, dev_step = device_resident(packed, params, local, args.kernel_steps, 2)
    log(f"[rank {rank}] device-resident step {dev_step * 1e3:.2f} ms")

    # -- whole node: the CLI over a BAM of the same families -------------------------
    workdir = None
    if args.sharded:         # one shared directory (rank 0's) for the one input and the outputs
        wd = [tempfile.mkdtemp(prefix="dcr_bench_sharded_", dir=os.environ.get("DCR_BENCH_DIR")) if rank == 0
              else None]
        if dist:
            tdist.broadcast_object_list(wd, src=0)
        workdir = wd[0]
    else:
        workdir = tempfile.mkdtemp(prefix=f"dcr_bench_r{rank}_", dir=os.environ.get("DCR_BENCH_DIR"))
    stats, e2e_s, level6, cpu_whole = {}, None, None, None
    try:
        if not args.kernel_only:
            bam_path = os.path.join(workdir, "in.bam")
            t0 = time.perf_counter()
            src = bam_packed if bam_packed is not None else packed
            if one_input_of_all and dist:
                one_input_bam(bam_path, src, args.seed + 1000 * rank, args.in_level, rank, world, tdist)
                log(f"[rank {rank}] one input of {world} ranks' families: {os.path.getsize(bam_path) / 1e6:.0f} MB "
                    f"BAM (level {args.in_level}) in {time.perf_counter() - t0:.1f} s")
            elif rank == 0 or not args.sharded:
                synth.write_packed_bam(bam_path, src, seed=args.seed + 1000 * rank, level=args.in_level)
                log(f"[rank {rank}] wrote {os.path.getsize(bam_path) / 1e6:.0f} MB BAM (level {args.in_level}) "
                    f"in {time.perf_counter() - t0:.1f} s")
            if dist:
                tdist.barrier()
            torch.cuda.synchronize()
            if args.sharded:
                e2e_s, stats = e2e_passes_sharded(bam_path, params_args, args.steps, args.warmup, workdir,
                                                  tdist if dist else None, rank)
            else:
                e2e_s, stats = e2e_passes(bam_path, params_args, local, args.steps, args.warmup, workdir)
            torch.cuda.synchronize()
            if dist:
                tdist.barrier()
            log(f"[rank {rank}] {args.steps} CLI passes in {e2e_s:.2f} s: "
                f"{ {k: v for k, v in stats.items() if k != 'ranks'} }")
            if not args.no_cpu and not dist and not args.sharded:
                quota, ncpu = cpu_cores()
                threads = int(quota) if quota else min(16, ncpu or 1)
                v, dt, st = cpu_baseline_whole_node(bam_path, params_args, workdir, args.cpu_reps, threads)
                cpu_whole = {"value": v, "pass_s": round(dt, 3), "threads": threads, "quota_cores": quota,
                             "host_cpus": ncpu, "consensus_bases": st.get("consensus_bases")}
                log(f"[rank {rank}] CPU whole node (oracle backend, host codecs): {v / 1e6:.1f} M consensus "
                    f"bases/s, {dt:.2f} s per pass")
            if args.level6_passes > 0 and not dist and not args.sharded and args.in_level != 6:
                # the same families from a level-6 input (a BAM as aligners
                # write it): more inflate work per byte, not the headline
                bam6 = os.path.join(workdir, "in6.bam")
                t0 = time.perf_counter()
                synth.write_packed_bam(bam6, src, seed=args.seed, level=6)
                log(f"[rank {rank}] wrote {os.path.getsize(bam6) / 1e6:.0f} MB BAM (level 6) in "
                    f"{time.perf_counter() - t0:.1f} s")
                os.remove(bam_path)
                torch.cuda.synchronize()
                s6, st6 = e2e_passes(bam6, params_args, local, args.level6_passes, 0, workdir)
                level6 = {"value": st6.get("consensus_bases", 0) * args.level6_passes / s6,
                          "unit": "consensus bases/s", "passes_s": st6.get("passes_s"),
                          "input_bytes": os.path.getsize(bam6)}
                log(f"[rank {rank}] level-6 input: {level6['value'] / 1e6:.1f} M consensus bases/s")
    finally:
        if rank == 0 or not args.sharded:
            shutil.rmtree(workdir, ignore_errors=True)

    e2e_bases = stats.get("consensus_bases", 0) * args.steps
    in_bases = int((bam_packed if bam_packed is not None else packed).seq_len.astype(np.int64).sum()) * args.steps
    if args.sharded and not one_input_of_all and rank != 0:
        in_bases = 0            # one input: rank 0's batch
    # per-rank busy time of the last CLI pass (whole pass, ingest thread, waits on the device)
    mine = {"rank": rank, "e2e_s_per_pass": (e2e_s or 0.0) / max(args.steps, 1),
            "device_resident_ms": dev_step * 1e3,
            **{k: round(v, 4) for k, v in stats.items()
               if k in ("ingest_s", "wait_s", "idle_s", "write_s", "run_s", "merge_s", "shard_rounds",
                        "consensus_bases")}}
    per_rank = [mine]
    if dist:
        per_rank = [None] * world
        tdist.all_gather_object(per_rank, mine)
    if dist:
        slowest = shard.max_over_ranks(e2e_s or 0.0, device=red_dev)
        dev_slowest = shard.max_over_ranks(dev_step, device=red_dev)
        e2e_bases, in_bases, dev_bases, n_bad = shard.sum_over_ranks([e2e_bases, in_bases, dev_bases, n_bad],
                                                                     device=red_dev)
    else:
        slowest, dev_slowest = e2e_s or 0.0, dev_step

    if rank == 0:
        alg = sscs_algorithmic_bytes(packed)
        alg_padded = sscs_algorithmic_bytes(packed, padded=True)
        if args.config == "C2":
            dom, dom_label = "k_consensus_fast<ss>", ("k_consensus_fast<false, false> + k_fast_rows (single-strand "
                                                      "consensus; the HIP-event slot spans both launches)")
            dom_ms = kavg[dom]
            # the slot's two launches: the kernel and its row expansion
            traffic, tsrc = load_traffic("k_consensus_fast<false, false>", packed.n_fam)
            rows_traffic, _ = load_traffic("k_fast_rows", packed.n_fam)
            if traffic is not None and rows_traffic is not None:
                traffic += rows_traffic
        else:
            dom_label = "single-strand stage (k_recmeta<ss> + k_consensus_fast<ss> + k_consensus_exact<ss> + k_consensus_general<ss>)"
            dom_ms = sum(kavg[k] for k in _lib.KERNELS[0:4])
            traffic, tsrc = None, None
        achieved = alg / (dom_ms / 1000.0) / 1e9
        if args.kernel_only:
            value, ms_step = dev_bases / dev_slowest, dev_slowest * 1e3
            value_kind = "device-resident kernels only (--kernel-only)"
        else:
            value, ms_step = e2e_bases / slowest, slowest * 1e3 / args.steps
            value_kind = "whole node: CLI from BAM open to output close"
        stage = {k: (round(v, 4) if isinstance(v, float) else v) for k, v in stats.items() if k.endswith("_s")}
        stage["gpu_inflate"] = stats.get("gpu_inflate")
        stage["host_cpu_s_per_pass"] = stats.get("host_cpu_s_per_pass")   # user + sys, every thread
        res = {
            "metric": METRIC, "value": value, "unit": "consensus bases/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong" if (args.sharded and not one_input_of_all) else "weak", "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": WORKLOAD[args.config] + (
                           (f"; ONE input of {world} x {packed.n_reads} reads (every rank's families) split over the "
                            f"{world} GPUs by the sharded CLI (cli --gpus {world})" if one_input_of_all else
                            f"; ONE input of {packed.n_reads} reads split over the {world} GPU(s) by the sharded CLI")
                           if args.sharded and dist else ""),
                       "value_is": value_kind, "input_bgzf_level": args.in_level, "max_reads": max_reads,
                       "whole_node_level6_input": level6,
                       "input_reads_per_gpu": (bam_packed if bam_packed is not None else packed).n_reads,
                       "families_per_gpu": packed.n_fam, "reads_per_gpu": packed.n_reads,
                       "input_bases_per_s": (in_bases / slowest) if slowest else None,
                       "consensus_records_per_pass": stats.get("consensus_records"),
                       "stages_s_last_pass": stage,
                       "device_resident": {"consensus_bases_per_s": dev_bases / dev_slowest,
                                           "ms_per_step": dev_slowest * 1e3, "kernel_ms": kavg,
                                           "records_not_ok": n_bad},
                       "single_strand_stage_GBps": alg / (sum(kavg[k] for k in _lib.KERNELS[0:4]) / 1e3) / 1e9,
                       "parallelism": (f"one input sharded x{world} by ranges of whole families (cli --gpus {world}), "
                                       "one process per GPU, parallel part merge, no data-path collective"
                                       if args.sharded else
                                       f"family-sharded x{world}, one process per GPU, no data-path collective"),
                       "per_rank": per_rank, "shared_stream": shared},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": dom_label,
                         "kernel_ms": dom_ms, "algorithmic_bytes_per_launch": alg,
                         "algorithmic_T": "max(pos + len) - min(pos) per subfamily (SURVEY §8d)",
                         "achieved_padded": alg_padded / (dom_ms / 1000.0) / 1e9,
                         "frac_padded": alg_padded / (dom_ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
                         "algorithmic_bytes_per_launch_padded": alg_padded,
                         "traffic_source": (f"profiles/traffic.json ({tsrc.get('source', '')})" if tsrc else None)},
        }
        if not args.no_cpu and world == 1:
            ko = cpu_baseline(packed, args.cpu_reps)
            if cpu_whole is not None:
                # like for like with value: the whole CLI pass on the CPU
                res["cpu_baseline"] = {
                    "value": cpu_whole["value"], "unit": "consensus bases/s",
                    "cores": cpu_whole["quota_cores"] or cpu_whole["threads"], "kind": "port",
                    "sample": (f"the whole-node CLI (cli.main, DuplexUMIConsensusReads.py:1426-1650) over the same "
                               f"{packed.n_reads}-read C2 BAM, best of {args.cpu_reps} passes "
                               f"({cpu_whole['pass_s']:.2f} s per pass): consensus by the C restatement "
                               f"oracle/dcr_oracle.c on {cpu_whole['threads']} threads, host BGZF inflate pool, "
                               f"host record writer and deflate; no GPU"),
                    "threads": cpu_whole["threads"], "quota_cores": cpu_whole["quota_cores"],
                    "host_cpus": cpu_whole["host_cpus"], "gpu_over_cpu": value / cpu_whole["value"],
                    "kernels_only": ko}
            else:
                res["cpu_baseline"] = ko
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
