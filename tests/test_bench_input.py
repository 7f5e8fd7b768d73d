"""bench.py at N > 1 times the sharded CLI over ONE input holding every
rank's families (bench.one_input_bam: each rank writes its records as BGZF
blocks, rank 0 the header, every rank copies its piece to its offset).  Two
gloo ranks on CPU: the assembled file is one valid BAM whose records are rank
0's then rank 1's, exactly as one writer over both batches gives them."""
import multiprocessing as mp
import os
import socket

from duplexumiconsensusreads_amd import bam, synth


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _rank(rank, world, port, path, q):
    import torch.distributed as dist

    import bench
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        packed = synth.packed_fixed_size(300 + 50 * rank, seed=2 + 1000 * rank)
        bench.one_input_bam(path, packed, 2 + 1000 * rank, 1, rank, world, dist)
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_one_input_of_two_ranks(tmp_path):
    path = str(tmp_path / "in.bam")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, path, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=300) for _ in ps)
    for p in ps:
        p.join(60)
    assert got == [(0, "ok"), (1, "ok")], got
    # the same records from one writer per rank batch, concatenated
    want = []
    for r in range(2):
        ref = str(tmp_path / f"ref{r}.bam")
        synth.write_packed_bam(ref, synth.packed_fixed_size(300 + 50 * r, seed=2 + 1000 * r), seed=2 + 1000 * r,
                               level=1)
        with bam.AlignmentFile(ref, "rb") as f:
            want += [x.to_dict() for x in f]
    with bam.AlignmentFile(path, "rb") as f:
        assert f.header.encode() == bam.AlignmentFile(str(tmp_path / "ref0.bam"), "rb").header.encode()
        recs = [x.to_dict() for x in f]
    assert len(recs) == 4 * 8 * 650
    assert recs == want
    assert open(path, "rb").read()[-28:] == bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    assert not [p for p in os.listdir(tmp_path) if ".piece" in p]
