"""The sharded CLI on the GPU: ``--gpus 2`` (two ranks launched through
torch.distributed.run, both on the box's one GPU here) against the
single-process CLI on the same input, as subprocesses: the three output
BAMs record for record and stdout must be identical."""
import os
import subprocess
import sys

import pytest

from duplexumiconsensusreads_amd import bam, synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.pop("DCR_SHARD", None)
    p = subprocess.run([sys.executable, "-m", "duplexumiconsensusreads_amd.cli", *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=240)
    return p.returncode, p.stdout


def _records(path):
    with bam.AlignmentFile(path, "rb") as f:
        return [r.to_dict() for r in f]


def test_gpu_sharded_cli_matches_single(tmp_path):
    path = str(tmp_path / "in.bam")
    cfg = synth.SynthConfig("t", 3000, sub_size="poisson5", seed=21, low_mapq_frac=0.1, indel_frac=0.1,
                            softclip_frac=0.1)
    synth.write_config_bam(path, cfg)
    one, many = str(tmp_path / "one.bam"), str(tmp_path / "many.bam")
    # no downsampling: the two runs are separate processes, and the CLI (like
    # the reference) draws from an unseeded random module (the seeded
    # downsampling case is tests/test_cli_shard.py)
    rc1, out1 = _run(["-i", path, "-o", one, "--min_reads", "3", "-v"])
    rc2, out2 = _run(["--gpus", "2", "-i", path, "-o", many, "--min_reads", "3", "-v"])
    assert rc1 == 0 and rc2 == 0
    if out2 != out1:
        l1, l2 = out1.splitlines(), out2.splitlines()
        i = next((k for k in range(min(len(l1), len(l2))) if l1[k] != l2[k]), min(len(l1), len(l2)))
        raise AssertionError(f"stdout differs at line {i} of {len(l1)} / {len(l2)}:\n"
                             f"single: {l1[max(0, i - 2):i + 3]}\nsharded: {l2[max(0, i - 2):i + 3]}")
    for s1, s2 in (("", ""), ("_filteredreads", "_filteredreads"), ("_filteredfamilies", "_filteredfamilies")):
        a, b = _records(one[:-4] + s1 + ".bam"), _records(many[:-4] + s2 + ".bam")
        assert len(a) == len(b) and a == b
    assert not [p for p in os.listdir(tmp_path) if ".part" in p]
