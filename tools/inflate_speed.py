"""Device BGZF inflate speed (csrc/dcr_inflate.hip) on a synthetic C2 BAM:
one launch over every member of the file (full occupancy), and launches of
the ingest's chunk size, kernel ms from HIP events; output checked against
the host inflate (zlib via bam.bgzf_stream).

    python3 tools/inflate_speed.py [families] [level] > out.json
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from duplexumiconsensusreads_amd import _lib, synth
    from duplexumiconsensusreads_amd.bam import bgzf_stream
    fams = int(sys.argv[1]) if len(sys.argv) > 1 else 312_500
    level = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    d = tempfile.mkdtemp()
    path = os.path.join(d, "in.bam")
    synth.write_packed_bam(path, synth.packed_fixed_size(fams, seed=2), seed=2, level=level)
    blob = np.fromfile(path, np.uint8)
    m, total = _lib.bgzf_members(blob.tobytes())
    inf = _lib.Inflater(0)
    res = {"families": fams, "level": level, "members": len(m), "compressed_bytes": int(blob.nbytes),
           "output_bytes": int(total)}
    rc, out = inf.run(blob, m, total)          # warm
    assert rc == 0, _lib.load().dcr_last_error()
    want = np.frombuffer(bgzf_stream(path), np.uint8)
    assert np.array_equal(out, want)
    t0 = time.perf_counter()
    rc, out = inf.run(blob, m, total)
    res["all_members_wall_ms"] = (time.perf_counter() - t0) * 1e3
    ms, n = inf.last()
    res["all_members_kernel_ms"] = ms
    res["all_members_GBps"] = total / ms / 1e6
    for per in (1024, 2560, 4096):
        ks, k0 = [], 0
        while k0 < len(m):
            sub = m[k0:k0 + per].copy()
            o0 = int(sub[0]["out_off"])
            sub["out_off"] -= o0
            nb = int(sub[-1]["out_off"] + sub[-1]["isize"])
            rc, _ = inf.run(blob, sub, nb)
            assert rc == 0
            ks.append(inf.last()[0])
            k0 += per
        res[f"chunks_of_{per}_kernel_ms_avg"] = float(np.mean(ks[:-1] if len(ks) > 1 else ks))
        res[f"chunks_of_{per}_GBps"] = float(total / sum(ks) / 1e6)
    # DINF_STAMP builds (DCR_LIB_PATH=.../libdcr_istamp.so): per-phase cycles per member
    import ctypes
    lib = _lib.load()
    if hasattr(lib, "dcr_inflater_stamps"):
        out = (ctypes.c_double * 16)()
        lib.dcr_inflater_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.dcr_inflater_stamps(inf.handle, out, 1)
        sub = m[:1024].copy()
        nb = int(sub[-1]["out_off"] + sub[-1]["isize"])
        inf.run(blob, sub, nb)
        if lib.dcr_inflater_stamps(inf.handle, out, 1) == 1:
            names = ["header_tables", "literal_tokens", "match_decode", "match_copy", "flush_write", "final"]
            n = len(sub)
            res["stamp_cycles_per_member"] = {k: out[i] / n for i, k in enumerate(names)}
            res["tokens_per_member"] = {"literal_pairs": out[9] / n, "literal_single": out[8] / n,
                                        "matches": out[10] / n, "match_bytes": out[11] / n,
                                        "loop_iterations": out[12] / n, "output": out[13] / n}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
