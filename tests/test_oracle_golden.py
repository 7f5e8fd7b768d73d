"""Pin the CPU oracle (oracle/dcr_oracle.py) + host record writer against the
golden vectors produced by running the reference script (tests/golden/)."""
import random

import numpy as np
import pytest

from .harness import writer
from oracle import dcr_oracle as O
from tests.golden_io import input_record, load_families, load_kats


def records_from_oracle(case_reads, res):
    """Oracle cores -> reference-identical records through the host writer."""
    by_name = {r["qname"]: input_record(r) for r in case_reads}
    ss_recs = []
    for k in range(4):
        sub = [by_name[r["qname"]] for r in res["subs"][k]]
        # the writer sees input reads as the reference does after preprocessing:
        # only mapq, MI, RX, flags and tid are read from them
        ss_recs.append(writer.single_strand_record(res["ss"][k], sub))
    ds = [writer.duplex_record(res["ds"][0], ss_recs[0], ss_recs[1]),
          writer.duplex_record(res["ds"][1], ss_recs[2], ss_recs[3])]
    ds = writer.fix_paired_end_fields(ds[0], ds[1])
    return ss_recs, ds


FAM = load_families()


@pytest.mark.parametrize("chunk", range(8))
def test_oracle_matches_reference_families(chunk):
    cases = FAM["cases"][chunk::8]
    n_ok = 0
    for case in cases:
        P = O.Params.from_dict(FAM["params"][case["params"]])
        exp = case["expect"]
        rng = random.Random(exp["seed"])
        try:
            res = O.process_family(case["reads"], P, rng)
        except O.RefCrash as e:
            assert exp["status"] in ("crash:" + e.kind, e.kind), (case["fam"], exp["status"], str(e))
            continue
        if res is None:
            assert exp["status"] == "filtered", case["fam"]
            continue
        assert exp["status"] == "ok", (case["fam"], exp["status"])
        ss, ds = records_from_oracle(case["reads"], res)
        for got, want in zip(ss, exp["ss"]):
            assert got.to_dict() == want, (case["fam"], "ss")
        for got, want in zip(ds, exp["ds"]):
            assert got.to_dict() == want, (case["fam"], "ds")
        assert [[r["qname"] for r in s] for s in res["subs"]] == exp["sub_reads"]
        n_ok += 1
    assert n_ok > 0


def test_kats():
    P = O.Params()
    for k in load_kats():
        if k["kind"] == "reconstruct":
            al, aq, mp = O.reconstruct(k["pos"], [[tuple(t) for t in c] for c in k["cigar"]],
                                       k["seq"], k["qual"])
            assert ["".join(r) for r in al] == k["aligned"], k["name"]
            assert [[v for v in row] for row in aq] == k["aligned_qual"], k["name"]
            assert mp == k["min_pos"]
        elif k["kind"] == "call":
            PP = O.Params.from_dict(FAM["params"][k["params"]])
            aq = [[v if isinstance(v, int) else v for v in row] for row in k["aligned_qual"]]
            cons, cq = O.call_consensus([list(r) for r in k["aligned"]], aq, PP)
            assert "".join(cons) == k["cons"], k["name"]
            assert cq == k["cons_qual"], k["name"]
        elif k["kind"] == "adjust":
            seq, qual, cig, pos = O.adjust(list(k["cons"]), k["cons_qual"], k["min_pos"])
            assert seq == k["seq"] and qual == k["qual"] and pos == k["pos"], k["name"]
            assert [list(t) for t in cig] == k["cigar"], k["name"]


def test_doc_figure_values():
    """docs/figs/reconstruct_alignment.png and adjustconsfields.png."""
    kats = {k["name"] + ":" + k["kind"]: k for k in load_kats()}
    rec = kats["doc_figure:reconstruct"]
    assert rec["aligned"] == ["AATTCaCGG", "AATTCaCGG", "NATTC+-GG", "NATTC+CGG"]
    adj = kats["doc_adjust_figure:adjust"]
    assert adj["pos"] == 11 and adj["seq"] == "AATTCGG" and adj["cigar"] == [[0, 5], [2, 1], [0, 2]]


def test_pairwise_sum_matches_numpy():
    rng = np.random.default_rng(0)
    for n in list(range(1, 300)) + [511, 1000, 2049, 3000]:
        a = rng.random(n) * 10.0 ** rng.integers(-5, 5, n)
        assert (0.0 + O.pairwise_sum(list(a))) / n == np.mean(a), n
        assert O.round_half_even_3(np.mean(a)) == np.round(np.mean(a), 3)
