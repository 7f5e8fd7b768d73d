"""Loading helpers for the committed golden fixtures (tests/golden/)."""
import gzip
import json
import os

from duplexumiconsensusreads_amd.records import AlignedSegment

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_families():
    with gzip.open(os.path.join(GOLDEN, "families.json.gz"), "rt") as f:
        return json.load(f)


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)


def load_e2e():
    with gzip.open(os.path.join(GOLDEN, "e2e_c1_small.json.gz"), "rt") as f:
        return json.load(f)


def input_record(d):
    r = AlignedSegment()
    r.query_name = d["qname"]
    r.flag = d["flag"]
    r.reference_id = d["tid"]
    r.reference_start = d["pos"]
    r.mapping_quality = d["mapq"]
    r.cigartuples = [tuple(x) for x in d["cigar"]]
    r.query_sequence = d["seq"]
    r.query_qualities = d["qual"]
    r.set_tags([("MI", d["MI"]), ("RX", d["RX"])])
    return r
