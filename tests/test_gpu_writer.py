"""The device record writer (dcr_submit_write: outcome scan, record
formatting and BGZF deflate on the GPU) against the host writer
(csrc/dcr_format.cpp over the kernel outputs of dcr_submit) on the same
batches: the decompressed record stream must be byte-identical, every BGZF
block a valid member with the right CRC32 / ISIZE, and the per-family
outcomes equal to the host scan's; the members are the host emulation's
(dcr_deflate_emulate) byte for byte."""
import gzip
import struct
import zlib

import numpy as np
import pytest

from duplexumiconsensusreads_amd import native_io, synth
from duplexumiconsensusreads_amd.params import ConsensusParams

pytestmark = pytest.mark.gpu


def members(blob):
    """Split concatenated BGZF blocks; check each one; return the data."""
    out, p = [], 0
    while p < len(blob):
        assert blob[p:p + 4] == b"\x1f\x8b\x08\x04"
        bsize = struct.unpack_from("<H", blob, p + 16)[0] + 1
        crc, isize = struct.unpack_from("<II", blob, p + bsize - 8)
        data = zlib.decompress(blob[p + 18:p + bsize - 8], -15)
        assert len(data) == isize and zlib.crc32(data) == crc
        out.append(data)
        p += bsize
    return b"".join(out)


def batches(path, params, reads):
    ing = native_io.Ingest(path, params.min_map_quality, params.min_reads, params.max_reads,
                           params.min_base_quality)
    while True:
        hb = native_io.HostBatch(reads=reads, side_bytes=1 << 24)
        ing.next(hb)
        yield hb
        if hb.end_kind != native_io.END_FULL:
            break


@pytest.mark.parametrize("kind", ["c1", "indel_clip", "c2"])
def test_device_writer_matches_host_writer(tmp_path, kind):
    from duplexumiconsensusreads_amd import _lib
    from duplexumiconsensusreads_amd.stream import DeviceStream
    path = str(tmp_path / "in.bam")
    if kind == "c2":
        synth.write_packed_bam(path, synth.packed_fixed_size(20_000, seed=7), seed=7)
    else:
        cfg = synth.SynthConfig("t", 400, sub_size="poisson5", seed=9,
                                indel_frac=0.3 if kind == "indel_clip" else 0.0,
                                softclip_frac=0.3 if kind == "indel_clip" else 0.0)
        synth.write_config_bam(path, cfg)
    params = ConsensusParams()
    ctx = _lib.Context(params, device=0)
    dev = DeviceStream(ctx, device_writer=True)
    host = DeviceStream(ctx, device_writer=False)
    n_fam = 0
    for hb in batches(path, params, 50_000):
        F = hb.n_fam
        n_fam += F
        res = dev.result(dev.submit(hb))
        fetched = res.record_bytes_of(F).tobytes()     # before the slot is submitted again
        got = members(res.bgzf.tobytes())
        ss, ds, rs = host.result(host.submit(hb))
        f_host, kind_h, _ = native_io.first_failure(hb, ss, ds, F, rs)
        nz = np.flatnonzero(res.fam_fail)
        assert (int(nz[0]) if len(nz) else F) == f_host
        assert f_host == F, "synthetic inputs have no failing family"
        out = str(tmp_path / f"host_{n_fam}.bam")
        w = native_io.BgzfWriter(out, b"")
        w.write_consensus(hb, ss, ds, F)
        w.close()
        want = gzip.decompress(open(out, "rb").read())
        assert len(got) == res.record_bytes
        assert got == want
        assert fetched == want
        # the device deflate is the host emulation's algorithm, scheduled for
        # the GPU (dcr_deflate.h parse_dev, BitOut2): the same members, byte
        # for byte
        emu = b"".join(native_io.deflate_emulate(fetched[i:i + 0xff00]) for i in range(0, len(fetched), 0xff00))
        assert emu == res.bgzf.tobytes()
    assert n_fam > 0
    dev.close()
    host.close()
    ctx.close()
