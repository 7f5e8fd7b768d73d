"""The span-stream protocol behind the GPU inflate (csrc/dcr_span_stream.h) on
the CPU, driven by the real ingest (csrc/dcr_ingest.cpp).

tests/native/stream_host.cpp runs the protocol with a host worker in the
device's role; tests/native/ingest_driver.cpp runs the ingest over a BAM to its
end and hashes every packed batch.  Checked here:

* BAMs of small BGZF blocks (0.5-4 KiB of data each, as BGZF allows) give the
  same batches through the stream as through the host pool.  Before the
  protocol advanced its `fetched` mark per span, a 64 MiB chunk of such
  members covered more than four spans and the fetch and the producer waited
  for each other for ever (round-3 advisor finding at dcr_inflate.hip:874);
* the same with every 2nd or 3rd chunk inflated by the host pool beside the
  stream (DCR_HOST_CHUNK_EVERY);
* the same under ThreadSanitizer and AddressSanitizer builds with 16 scanner
  and pack threads (the pool sizes of the one unexplained bench exit in round
  3): no race report (e.g. the stream's start offset read by the member
  scanner while the reader advanced it, dcr_ingest.cpp open_stream) and no
  heap error;
* the slot buffers are sized once by the protocol's start() on the opening
  thread: no buffer grows (a hipFree / hipHostMalloc on the device) on the
  producer thread while spans are in flight (``late_allocs`` 0, the round-3
  exit suspect of DESIGN.md §5).
"""
import os
import subprocess

import pytest

from duplexumiconsensusreads_amd import synth

from .bgzf_util import reblock

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BUILD = os.path.join(NATIVE, "_build")


@pytest.fixture(scope="module")
def drivers():
    subprocess.run(["make", "-s", "-C", NATIVE, "-j3"], check=True)
    return BUILD


@pytest.fixture(scope="module")
def bams(tmp_path_factory):
    d = tmp_path_factory.mktemp("stream")
    big = str(d / "c2.bam")
    packed = synth.packed_fixed_size(6000, sub_size=8, seed=11)          # 192 k reads, ~70 MB of records
    synth.write_packed_bam(big, packed, seed=11, level=1)
    small = str(d / "c2_small_blocks.bam")
    nblk = reblock(big, small, 512, 4096, seed=1)
    assert nblk > 20000                     # a 64 MiB chunk spans > kSlots spans of 4,096 members
    return big, small


def _run(exe, bam, hook, env_extra=None, timeout=300):
    env = dict(os.environ)
    env.update(env_extra or {})
    r = subprocess.run([exe, bam, str(hook)], capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    f = r.stdout.split()
    return dict(zip(f[0::2], f[1::2])), r.stderr


def _same(a, b):
    for k in ("batches", "end", "records", "passed", "excluded", "processed", "filtered", "hash"):
        assert a[k] == b[k], (k, a, b)


def test_small_blocks_through_the_stream_equal_the_host_pool(drivers, bams):
    big, small = bams
    exe = os.path.join(drivers, "ingest_driver")
    ref, _ = _run(exe, big, 0)
    host_small, _ = _run(exe, small, 0)
    _same(ref, host_small)
    for bam in (big, small):
        got, _ = _run(exe, bam, 1)
        assert got["hooked"] == "1" and got["streams"] == "1", got
        _same(ref, got)
        # the slots were sized at the stream's start: the producer never
        # grew (freed / re-allocated) a buffer while spans were in flight
        assert got["late_allocs"] == "0", got
    assert int(got["spans"]) >= 8                   # the small-block run went through many spans


@pytest.mark.parametrize("every", ["2", "3"])
def test_host_chunks_beside_the_stream_equal_the_host_pool(drivers, bams, every):
    """DCR_HOST_CHUNK_EVERY=k: every k-th chunk inflated by the host pool,
    its members skipped by the stream (spans end at the gap); the reader's
    chunking and the member scanner's replay of it must agree."""
    big, small = bams
    exe = os.path.join(drivers, "ingest_driver")
    ref, _ = _run(exe, big, 0)
    for bam in (big, small):
        got, _ = _run(exe, bam, 1, {"DCR_HOST_CHUNK_EVERY": every})
        assert got["hooked"] == "1" and got["streams"] == "1", got
        _same(ref, got)


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_stream_ingest_under_sanitizers_16_16_pools(drivers, bams, kind):
    big, small = bams
    ref, _ = _run(os.path.join(drivers, "ingest_driver"), big, 0)
    exe = os.path.join(drivers, f"ingest_driver_{kind}")
    env = {"DCR_SCAN_THREADS": "16", "DCR_PACK_THREADS": "16", "DCR_HOST_CHUNK_EVERY": "2",
           "TSAN_OPTIONS": "halt_on_error=1 exitcode=66", "ASAN_OPTIONS": "detect_leaks=0 exitcode=67"}
    for bam in (small, big):
        got, err = _run(exe, bam, 1, env, timeout=600)
        assert "WARNING: ThreadSanitizer" not in err and "ERROR: AddressSanitizer" not in err, err[-4000:]
        _same(ref, got)
        assert got["late_allocs"] == "0", got


# ---- round 3's protocol, for the one unexplained bench exit ------------------
# tests/native/Makefile (target r3) extracts round 3's ingest from this
# repository's history (git 205281c) and links it with r3_stream_host.cpp, a
# host restatement of round 3's span protocol (dcr_inflate.hip:797-1057 at
# that commit).  What each suspect does under it, on the CPU:
#   * a late member-scanner start (the start-offset race): the stream serves a
#     later member's bytes at offset 0, the header check fails and the open
#     returns "not a BAM file" at once -- a Python RuntimeError with a
#     traceback, not a silent exit;
#   * 16 scanner + 16 pack threads, several passes sharing one inflater: the
#     same batches as the host pool, no heap error under AddressSanitizer, and
#     ThreadSanitizer reports only the start-offset race;
#   * small BGZF blocks: the fetch/producer deadlock -- a hang, not an exit.
# None of the three ends a process silently within seconds
# (profiles/r03o/pool_ab_16_16_2_failed.log); DESIGN §5 records what remains.

def _git_has_round3():
    try:
        subprocess.run(["git", "-C", ROOT, "cat-file", "-e", "205281c:duplexumiconsensusreads_amd/csrc/dcr_ingest.cpp"],
                       check=True, capture_output=True)
        return True
    except (OSError, subprocess.CalledProcessError):
        return False


@pytest.fixture(scope="module")
def r3_drivers(drivers):
    # archaeology of round 3's build: several 600 s subprocess runs, opt-in
    # (DCR_TEST_ROUND3=1); they check old code from git history, not the
    # shipped ingest, which the tests above cover
    if os.environ.get("DCR_TEST_ROUND3") != "1":
        pytest.skip("round-3 archaeology tests are opt-in: DCR_TEST_ROUND3=1")
    if not _git_has_round3():
        pytest.skip("round 3's sources are not in this checkout's history")
    subprocess.run(["make", "-s", "-C", NATIVE, "-j3", "r3"], check=True)
    return BUILD


R3_POOLS = {"DCR_SCAN_THREADS": "16", "DCR_PACK_THREADS": "16", "ASAN_OPTIONS": "detect_leaks=0 exitcode=67",
            "TSAN_OPTIONS": "halt_on_error=0 exitcode=66"}


def _run_raw(exe, bam, env_extra, timeout):
    env = dict(os.environ)
    env.update(R3_POOLS)
    env.update(env_extra)
    return subprocess.run([exe, bam, "1"], capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.parametrize("kind", ["", "_asan"])
def test_round3_late_member_scan_is_a_clean_open_error(r3_drivers, bams, kind):
    big, _ = bams
    r = _run_raw(os.path.join(r3_drivers, "r3_driver" + kind), big, {"DCR_R3_LATE_MS": "100"}, 120)
    assert r.returncode == 4, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert r.stderr.strip() == "open: not a BAM file", r.stderr[-3000:]


def test_round3_16_16_pools_several_passes(r3_drivers, bams):
    big, _ = bams
    ref, _ = _run(os.path.join(r3_drivers, "ingest_driver"), big, 0)
    for kind in ("", "_asan"):
        r = _run_raw(os.path.join(r3_drivers, "r3_driver" + kind), big,
                     {"DCR_TEST_PASSES": "3", "DCR_R3_COPY_US": "200"}, 600)
        assert r.returncode == 0 and "ERROR: AddressSanitizer" not in r.stderr, (r.returncode, r.stderr[-3000:])
        lines = r.stdout.strip().splitlines()
        assert len(lines) == 3
        for ln in lines:
            f = ln.split()
            _same(ref, dict(zip(f[0::2], f[1::2])))
    # ThreadSanitizer: the start-offset race and nothing else
    r = _run_raw(os.path.join(r3_drivers, "r3_driver_tsan"), big, {"DCR_TEST_PASSES": "2"}, 600)
    reports = r.stderr.count("WARNING: ThreadSanitizer")
    assert reports >= 1 and r.stderr.count("Inflater::scan_members") >= reports, r.stderr[-4000:]


def test_round3_small_blocks_hang(r3_drivers, bams):
    _, small = bams
    with pytest.raises(subprocess.TimeoutExpired):
        _run_raw(os.path.join(r3_drivers, "r3_driver"), small, {}, 15)
