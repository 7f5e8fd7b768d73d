"""Benchmark: consensus bases/s of the duplex-consensus hot path on MI355X.

Workload (BASELINE.json configs[1]): per GPU a synthetic
duplex batch of 10 M reads = 312,500 MI families x 4 subfamilies x 8 reads,
2x150 bp ``150M`` reads, no indels, qualities {Q37 .80, Q25 .12, Q12 .08}.
One step = the whole hot path over that batch with inputs resident in HBM:
1.25 M single-strand consensus records (k_recmeta<ss>, k_consensus_fast<ss>
and its exact pass, k_decide + k_consensus_general<ss>) and 625 k duplex
records (the same kernels <ds>), per-read preprocessing fused into them.
--config C3 / C4 / C5 runs the other BASELINE.json shapes (per-GPU shards).

value = duplex consensus bases emitted by all ranks per second (weak scaling:
each rank owns its own families, no data-path collective; max time over
ranks).  roofline = the single-strand kernel's algorithmic bytes
 / its HIP-event-timed average launch / 8 TB/s.
cpu_baseline = the C restatement (oracle/, kind "port") on a bounded sample
of the same workload on this host.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--families F]
(N > 1 is launched by torch.distributed.run, one process per GPU.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

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
    "C2": "C2 (BASELINE.json configs[1]): 10M-read synthetic duplex batch per GPU, 312,500 MI families x "
          "4 subfamilies x 8 reads, 2x150bp, no indels",
    "C3": "C3 shape (BASELINE.json configs[2]) per GPU: skewed subfamilies Zipf(1.5) on 1..100, 5% of reads with "
          "a 1-3 bp indel, 3% soft-clipped, 2x150bp",
    "C4": "C4 shape (BASELINE.json configs[3]): 20 loci x 50 families, subfamilies log-uniform 100..1000 reads "
          "(--max_reads 1000), 2x150bp",
    "C5": "C5 shape (BASELINE.json configs[4]): one 4M-read chunk, subfamilies Poisson(4)+1, 2x150bp",
}


def make_batch(config, families, seed):
    from duplexumiconsensusreads_amd import synth
    if config == "C2":
        return synth.packed_fixed_size(families, seed=seed)
    return synth.packed_config(synth.CONFIGS[config], families, seed=seed, max_reads=1000)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def sscs_algorithmic_bytes(packed):
    """sum_r(2 len_r + 4 n_cig_r + 4 + 1) + T*(2 + 4) + 16 per
    subfamily, with T the subfamily's alignment width (here T_ub == T: no
    clipping, no indels)."""
    per_read = 2 * packed.seq_len.astype(np.int64) + 4 * packed.cig_n.astype(np.int64) + 5
    reads_b = int(per_read.sum())
    cols = int(packed.ss_col_off[-1])
    n_sub = len(packed.ss_col_off) - 1
    return reads_b + 6 * cols + 16 * n_sub


def cpu_baseline(packed, reps):
    """The C restatement (oracle/dcr_oracle.c, test infrastructure used here
    only as the timed CPU leg) over the bench batch itself, multi-threaded
    over families.  The C2 batch takes ~1-2 s per pass on 16 threads, so the
    sample is the whole batch, repeated ``reps`` times (≈10-30 thread-s)."""
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
                      f"C restatement oracle/dcr_oracle.c on {threads} threads, best of {reps}: "
                      f"{dt:.2f} s per pass"}


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIG_FAMILIES),
                    help="workload shape (SURVEY.md §8d); C2 is the headline line, the others are "
                         "per-GPU shards of C3 / C4 / C5 reported for coverage")
    ap.add_argument("--families", type=int, default=None, help="families per GPU (C2: 312,500)")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-reps", type=int, default=2, help="passes of the CPU baseline over the batch")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    from duplexumiconsensusreads_amd import _lib
    from duplexumiconsensusreads_amd.device import DeviceBatch
    from duplexumiconsensusreads_amd.params import ConsensusParams

    t0 = time.perf_counter()
    families = args.families or CONFIG_FAMILIES[args.config]
    packed = make_batch(args.config, families, args.seed + 1000 * rank)
    log(f"[rank {rank}] generated {packed.n_reads} reads in {time.perf_counter() - t0:.1f} s")
    dev = f"cuda:{local}"
    db = DeviceBatch(packed, device=dev)
    # C4 runs with --max_reads 1000; the batch is already downsampled
    params = ConsensusParams(max_reads=1000) if args.config == "C4" else ConsensusParams()
    ctx = _lib.Context(params, device=local)
    ctx.reserve(db.batch_struct)
    torch.cuda.synchronize()

    for _ in range(args.warmup):
        ctx.run_device(db.batch_struct, db.ss_struct, db.ds_struct)
    ctx.sync()
    # correctness guard on the bench batch itself: every record must be OK
    st_ss = db.out["ss"]["status"][:4 * packed.n_fam]
    st_ds = db.out["ds"]["status"][:2 * packed.n_fam]
    n_bad = int((st_ss != 0).sum().item() + (st_ds != 0).sum().item())
    bases = int(db.out["ds"]["len"].view(torch.int32)[:2 * packed.n_fam].sum().item())

    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    kms = {k: 0.0 for k in _lib.KERNELS}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.run_device(db.batch_struct, db.ss_struct, db.ds_struct)
        tm = ctx.last_kernel_timing()   # waits on this step's events only
        for k in kms:
            kms[k] += tm[k]
    ctx.sync()
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        from duplexumiconsensusreads_amd import shard
        elapsed = shard.max_over_ranks(elapsed, device=dev)
        total_bases, n_bad = shard.sum_over_ranks([bases, n_bad], device=dev)
    else:
        total_bases = bases

    if rank == 0:
        ms_step = elapsed * 1000.0 / args.steps
        value = total_bases * args.steps / elapsed
        kavg = {k: v / args.steps for k, v in kms.items()}
        alg = sscs_algorithmic_bytes(packed)
        if args.config == "C2":
            dom, dom_label = "k_consensus_fast<ss>", "k_consensus_fast<false, false> (single-strand consensus)"
            dom_ms = kavg[dom]
            traffic, tsrc = load_traffic("k_consensus_fast<false, false>", packed.n_fam)
        else:
            # records split between the fast and general kernels: the whole single-strand stage
            dom_label = "single-strand stage (k_recmeta<ss> + k_consensus_fast<ss> + k_consensus_exact<ss> + k_consensus_general<ss>)"
            dom_ms = sum(kavg[k] for k in _lib.KERNELS[1:5])
            traffic, tsrc = None, None
        achieved = alg / (dom_ms / 1000.0) / 1e9
        res = {
            "metric": METRIC, "value": value, "unit": "consensus bases/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": WORKLOAD[args.config],
                       "families_per_gpu": packed.n_fam, "reads_per_gpu": packed.n_reads,
                       "input_bytes_per_gpu": packed.nbytes(),
                       "kernel_ms": kavg,
                       "single_strand_stage_GBps": alg / (sum(kavg[k] for k in _lib.KERNELS[1:5]) / 1e3) / 1e9,
                       "records_not_ok": n_bad,
                       "parallelism": f"family-sharded x{world}, no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": dom_label,
                         "kernel_ms": dom_ms, "algorithmic_bytes_per_launch": alg,
                         "traffic_source": (f"profiles/traffic.json ({tsrc.get('source', '')})" if tsrc else None)},
        }
        if not args.no_cpu and world == 1:
            del db
            res["cpu_baseline"] = cpu_baseline(packed, args.cpu_reps)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    ctx.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
