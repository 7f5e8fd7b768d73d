"""Pin the C restatement (oracle/dcr_oracle.c) against the reference's golden
vectors through the host pipeline (pack -> backend -> statuses -> writer)."""
import random

import pytest

from .harness import pipeline
from duplexumiconsensusreads_amd.params import ConsensusParams
from oracle import dcr_oracle_c
from tests.golden_io import input_record, load_families

FAM = load_families()


def run_cases_with_backend(cases, params_name, backend):
    P = ConsensusParams.from_oracle_dict(FAM["params"][params_name])
    results, expects = [], []
    for case in cases:
        reads = [input_record(r) for r in case["reads"]]
        rng = random.Random(case["expect"]["seed"])
        try:
            res = pipeline.prepare_family(reads, P, rng)
        except pipeline.FamilyExit:
            res = pipeline.FamilyResult(code="?", reads=reads, crash="exit")
        except IndexError:
            res = pipeline.FamilyResult(code="?", reads=reads, crash="IndexError")
        results.append(res)
        expects.append(case["expect"])
    pipeline.run_batch(results, P, backend)
    return results, expects


def check_results(results, expects, cases):
    n_ok = 0
    for res, exp, case in zip(results, expects, cases):
        st = exp["status"]
        if st == "filtered":
            assert res.filtered, case["fam"]
        elif st.startswith("crash:") or st == "exit":
            want = st.split(":")[-1]
            assert res.crash == want, (case["fam"], res.crash, st)
        else:
            assert res.crash is None and not res.filtered, (case["fam"], res.crash)
            for got, want in zip(res.ss, exp["ss"]):
                assert got.to_dict() == want, (case["fam"], "ss", got.to_dict(), want)
            for got, want in zip(res.ds, exp["ds"]):
                assert got.to_dict() == want, (case["fam"], "ds")
            n_ok += 1
    return n_ok


@pytest.mark.parametrize("pname", sorted(FAM["params"]))
def test_c_oracle_matches_reference(pname):
    cases = [c for c in FAM["cases"] if c["params"] == pname]
    results, expects = run_cases_with_backend(cases, pname, dcr_oracle_c.run)
    n_ok = check_results(results, expects, cases)
    assert n_ok > 0 or pname == "pre1"


def test_c_oracle_threads_identical():
    cases = [c for c in FAM["cases"] if c["params"] == "default"][:300]
    r1, e1 = run_cases_with_backend(cases, "default", lambda pk, p: dcr_oracle_c.run(pk, p, n_threads=1))
    r4, e4 = run_cases_with_backend(cases, "default", lambda pk, p: dcr_oracle_c.run(pk, p, n_threads=4))
    for a, b in zip(r1, r4):
        assert a.crash == b.crash
        if a.ds:
            assert [x.to_dict() for x in a.ds] == [x.to_dict() for x in b.ds]
