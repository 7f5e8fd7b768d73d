"""C5 at streaming scale: a >= 100 M-read BAM of
the C5 shape (subfamily sizes Poisson(4)+1, 2x150, 150M),
written at BGZF level 6 in pieces, then ``cli.main`` on one GPU with the
device record writer (thousands of chunk windows, batch-slot reuse, the
inflate stream's span ring, the ingest's per-process caches) and the same CLI
driven by the C oracle (oracle/dcr_oracle.c, test infrastructure: the
checker) on the same file.  stdout, the consensus base count and the
decompressed bytes of all three outputs must be identical (sha256 over a
streaming inflate of each).  One JSON line with the whole-node rate and the
comparison goes to stdout and to OUT.json.

    python3 tools/c5_stream.py [n_reads] [workdir] [out.json]
"""
import contextlib
import functools
import gzip
import hashlib
import io
import json
import os
import random
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from duplexumiconsensusreads_amd import cli, native_io, synth  # noqa: E402

SUFFIXES = (".bam", "_filteredreads.bam", "_filteredfamilies.bam")


def log(*a):
    print(*a, flush=True)


def write_input(path, n_reads, level=6, chunk_fam=200_000, seed=5):
    """Pieces of C5 families appended to one BAM (header, pieces without
    their EOF blocks, one EOF block); MI codes distinct across pieces."""
    eof = len(cli._BGZF_EOF)
    w = native_io.BgzfWriter(path, synth.BamHeader_bytes(), level=level)
    w.close()
    os.truncate(path, os.path.getsize(path) - eof)
    total, fam0, ci = 0, 0, 0
    t0 = time.perf_counter()
    with open(path, "ab") as out:
        while total < n_reads:
            packed = synth.packed_config(synth.CONFIGS["C5"], chunk_fam, seed=seed + ci)
            piece = path + ".piece"
            synth.write_packed_bam(piece, packed, seed=seed + ci, level=level, header=False, fam_id0=fam0)
            with open(piece, "rb") as f:
                data = f.read()
            out.write(data[:len(data) - eof])
            os.remove(piece)
            total += packed.n_reads
            fam0 += packed.n_fam
            ci += 1
            del packed, data
            if ci % 5 == 0:
                log(f"input: {total / 1e6:.1f} M reads, {fam0} families, {time.perf_counter() - t0:.0f} s")
        out.write(cli._BGZF_EOF)
    return total, fam0


def run_cli(inp, out, backend):
    buf, stats = io.StringIO(), {}
    rng = random.Random(4)
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(buf):
        rc = cli.main(["-i", inp, "-o", out], backend=backend, rng=rng, stats=stats)
    return rc, time.perf_counter() - t0, buf.getvalue(), stats, rng.getstate()


def digest(path, res, key):
    h, n = hashlib.sha256(), 0
    with gzip.open(path, "rb") as f:
        while True:
            b = f.read(32 << 20)
            if not b:
                break
            h.update(b)
            n += len(b)
    res[key] = (n, h.hexdigest())


def main():
    n_reads = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    wd = sys.argv[2] if len(sys.argv) > 2 else os.environ.get("DCR_BENCH_DIR", "/tmp")
    out_json = sys.argv[3] if len(sys.argv) > 3 else None
    os.makedirs(wd, exist_ok=True)
    inp = os.path.join(wd, "c5_stream.bam")
    t0 = time.perf_counter()
    reads, fams = write_input(inp, n_reads)
    t_in = time.perf_counter() - t0
    log(f"input written: {reads} reads, {fams} families, {os.path.getsize(inp) / 1e9:.2f} GB at level 6 in {t_in:.0f} s")
    out_gpu, out_cpu = os.path.join(wd, "c5_gpu.bam"), os.path.join(wd, "c5_cpu.bam")

    def ticker(label, stop):            # a line every 30 s on the real stderr (gpurun's hang watchdog;
        t = time.perf_counter()         # the CLI's stdout is being captured)
        while not stop.wait(30):
            print(f"{label}: {time.perf_counter() - t:.0f} s", file=sys.__stderr__, flush=True)

    # the oracle-backend CLI first: the host inflate pool (the GPU CLI below
    # installs the device inflater for the process)
    stop = threading.Event()
    threading.Thread(target=ticker, args=("oracle cli", stop), daemon=True).start()
    oracle = functools.partial(__import__("oracle.dcr_oracle_c", fromlist=["run"]).run, n_threads=16)
    rc_c, s_c, so_c, st_c, rng_c = run_cli(inp, out_cpu, oracle)
    stop.set()
    log(f"oracle cli: rc {rc_c}, {s_c:.1f} s")
    # the product path: backend None = the device context with the device
    # record writer and the GPU input inflate (cli.main)
    stop = threading.Event()
    threading.Thread(target=ticker, args=("gpu cli", stop), daemon=True).start()
    rc_g, s_g, so_g, st_g, rng_g = run_cli(inp, out_gpu, None)
    stop.set()
    log(f"gpu cli: rc {rc_g}, {s_g:.1f} s, {st_g.get('batches')} batches, "
        f"{st_g.get('consensus_bases', 0) / s_g / 1e6:.1f} M consensus bases/s")
    infl = cli._INFLATERS.get(0)
    gpu_infl = None
    if infl is not None:
        t = infl[0].totals()
        gpu_infl = {"kernel_ms": t["kernel_ms"], "launches": t["runs"]}
    dig = {}
    ths = [threading.Thread(target=digest, args=(o[:-4] + suf, dig, (side, suf)))
           for o, side in ((out_gpu, "gpu"), (out_cpu, "cpu")) for suf in SUFFIXES]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    same = {suf: dig[("gpu", suf)] == dig[("cpu", suf)] for suf in SUFFIXES}
    res = {"reads": reads, "families": fams, "input_level": 6, "input_bytes": os.path.getsize(inp),
           "gpu_cli_s": s_g, "oracle_cli_s": s_c, "batches": st_g.get("batches"),
           "consensus_records": st_g.get("consensus_records"), "consensus_bases": st_g.get("consensus_bases"),
           "whole_node_consensus_bases_per_s": st_g.get("consensus_bases", 0) / s_g,
           "input_reads_per_s": reads / s_g,
           "stdout_identical": so_g == so_c, "rng_state_identical": rng_g == rng_c,
           "consensus_bases_identical": st_g.get("consensus_bases") == st_c.get("consensus_bases"),
           "outputs_identical": same, "output_sizes_decompressed": {s: dig[("gpu", s)][0] for s in SUFFIXES},
           "stages_s": {k: round(v, 3) for k, v in st_g.items() if k.endswith("_s") and isinstance(v, float)},
           "gpu_inflate": gpu_infl}
    if not res["stdout_identical"]:
        a, b = so_g.splitlines(), so_c.splitlines()
        k = next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), min(len(a), len(b)))
        res["stdout_first_difference"] = {"line": k, "lines": [len(a), len(b)],
                                          "gpu": a[max(0, k - 2):k + 3], "oracle": b[max(0, k - 2):k + 3]}
    line = json.dumps(res)
    log(line)
    if out_json:
        with open(out_json, "w") as f:
            f.write(line + "\n")
    for p in (inp, out_gpu, out_cpu):
        for suf in ("",) if p == inp else SUFFIXES:
            q = p if p == inp else p[:-4] + suf
            if os.path.exists(q):
                os.remove(q)
    ok = all(same.values()) and res["stdout_identical"] and res["consensus_bases_identical"] and rc_g == rc_c == 0
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
