"""GPU deflate phase probe: k_deflate over a formatted consensus stream with
s_memtime phase stamps (dcr_deflate_probe, diagnostic entry of libdcr.so)."""
import ctypes
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, ".")
from duplexumiconsensusreads_amd import _lib, native_io, synth  # noqa: E402
from duplexumiconsensusreads_amd.params import ConsensusParams  # noqa: E402
from duplexumiconsensusreads_amd.stream import DeviceStream  # noqa: E402

PHASES = ["load+clear", "hash", "count+crc", "keys+rank", "trees(t0)", "codes", "bits", "scan(t0)", "emit",
          "frame(t0)", "assign", "header(t0)"]


def main():
    path = "/tmp/probe.bam"
    synth.write_packed_bam(path, synth.packed_fixed_size(16_384, seed=5), seed=5)
    ctx = _lib.Context(ConsensusParams(), device=0)
    ds = DeviceStream(ctx, device_writer=True)
    ing = native_io.Ingest(path)
    hb = native_io.HostBatch(reads=1 << 20)
    ing.next(hb)
    res = ds.result(ds.submit(hb))
    raw = res.record_bytes_of(hb.n_fam)
    if len(sys.argv) > 1:          # a sample of the record stream for host-side parse studies
        raw[:8 << 20].tofile(sys.argv[1])
    lib = _lib.load()
    fn = lib.dcr_deflate_probe
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    nb = (raw.nbytes + 0x7f80 - 1) // 0x7f80       # room for blocks of half the BGZF maximum
    slots = np.zeros(nb * 65536, np.uint8)
    sizes = np.zeros(nb, np.int64)
    for dbg in [0]:
        st = np.zeros(12, np.uint64)
        ms = ctypes.c_float()
        cb = ctypes.c_int64()
        for rep in range(3):
            st[:] = 0
            _lib._check(fn(ctx._ctx, raw.ctypes.data, raw.nbytes, st.ctypes.data, ctypes.byref(ms),
                           ctypes.byref(cb), slots.ctypes.data if rep == 0 else None,
                           sizes.ctypes.data if rep == 0 else None))
        # every member inflates (zlib, gzip framing) to its block of the input
        # (the library's block size may differ from 0xff00: members are consecutive)
        rb = raw.tobytes()
        at = 0
        for b in range(nb if not os.environ.get("DFL_NOVERIFY") else 0):
            if not sizes[b]:
                break
            mem = slots[b * 65536:b * 65536 + int(sizes[b])].tobytes()
            d = zlib.decompressobj(31)
            got = d.decompress(mem)
            assert d.eof and not d.unused_data and got == rb[at:at + len(got)], f"block {b} differs"
            at += len(got)
        if not os.environ.get("DFL_NOVERIFY"):      # ablation builds (invalid members): timing only
            assert at == len(rb), "members do not cover the stream"
            nb = b + 1 if sizes[b] else b
        import hashlib
        hsh = hashlib.sha1()
        for b in range(nb):
            hsh.update(slots[b * 65536:b * 65536 + int(sizes[b])].tobytes())
        print(f"verified {nb} members with zlib, {int(sizes.sum())} compressed bytes, sha1 {hsh.hexdigest()[:16]}")
        tot = st.sum()
        print(f"dbg={dbg}: {raw.nbytes / 1e6:.1f} MB -> {cb.value / 1e6:.1f} MB ({raw.nbytes / cb.value:.2f}x) in "
              f"{ms.value:.2f} ms = {raw.nbytes / ms.value / 1e6:.2f} GB/s")
        print("  " + "  ".join(f"{name} {100.0 * v / tot:.1f}%" for name, v in zip(PHASES, st)))


if __name__ == "__main__":
    main()
