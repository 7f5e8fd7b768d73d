"""Device-bound streaming: the batches of a C5-shaped BAM ingested into
pinned host batches up front, then submitted back to back through the
two-slot DeviceStream (H2D on the copy stream, kernels + device writer on
the compute stream, D2H on the second copy stream) for several rounds, so a
rocprofv3 kernel + memory-copy trace shows whether the copies of one batch
hide under the kernels of the other (tools/overlap.py).
usage: python tools/stream_resident.py <workdir> [families] [batch_reads] [rounds]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from duplexumiconsensusreads_amd import _lib, native_io, synth  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams  # noqa: E402
from duplexumiconsensusreads_amd.stream import DeviceStream  # noqa: E402


def main():
    wd = sys.argv[1]
    fams = int(sys.argv[2]) if len(sys.argv) > 2 else 250_000
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    os.makedirs(wd, exist_ok=True)
    path = os.path.join(wd, "c5r.bam")
    packed = synth.packed_config(synth.CONFIGS["C5"], fams, seed=7)
    synth.write_packed_bam(path, packed, seed=7, level=1)
    del packed
    params = ConsensusParams()
    ctx = _lib.Context(params, device=0)
    ds = DeviceStream(ctx, owns_ctx=True)
    ing = native_io.Ingest(path, params.min_map_quality, params.min_reads, params.max_reads,
                           params.min_base_quality)
    hbs = []
    while True:
        hb = ds.host_batch(batch)
        ing.next(hb)
        hbs.append(hb)
        if hb.end_kind != native_io.END_FULL:
            break
    ing.close()
    bases = sum(int(hb.s.n_bases) for hb in hbs)
    print(f"{len(hbs)} batches, {sum(int(hb.s.n_reads) for hb in hbs)} reads", flush=True)
    for r in range(rounds):
        t = time.perf_counter()
        prev = None
        out_bytes = 0
        for hb in hbs:
            h = ds.submit(hb)
            if prev is not None:
                out_bytes += ds.result(prev).bgzf.nbytes
            prev = h
        out_bytes += ds.result(prev).bgzf.nbytes
        dt = time.perf_counter() - t
        print(f"round {r}: {dt * 1e3:.1f} ms, {bases / dt / 1e9:.2f} G input bases/s through H2D + kernels + "
              f"device writer + D2H ({out_bytes / 1e6:.0f} MB of BGZF out)", flush=True)
    ds.close()


if __name__ == "__main__":
    main()
