"""pysam-compatible alignment record used by the host side of the drop-in.

The reference drives everything through ``pysam.AlignedSegment``
(DuplexUMIConsensusReads.py:1372-1384 builds consensus records, :1135-1181 and
:191-325 read input records).  pysam is not installed in this image, so the
host ships a record class with the subset of pysam semantics the reference
relies on:

* ``mapping_quality`` setter truncates floats (pysam's Cython ``nb_int``
  conversion; the reference assigns ``np.mean(...)`` at :1377).
* ``query_sequence`` setter clears the qualities (pysam behaviour; the
  reference re-assigns qualities right after every sequence change, :247-251,
  :285-286, :317-318).
* ``set_tags`` infers BAM tag types the way pysam does (smallest integer type,
  'f' for floats, 'Z' for str, 'B' arrays for lists).  Float tags are stored as
  float32, so ``get_tag`` of an 'f' tag returns the float32-rounded value,
  exactly as a pysam record read back from its own bam1_t would.
"""
from __future__ import annotations

import array
import struct

CIGAR_CHARS = "MIDNSHP=XB"
_CIGAR_CODE = {c: i for i, c in enumerate(CIGAR_CHARS)}

# BAM flag bits (SAM spec 1.4)
FPAIRED, FPROPER, FUNMAP, FMUNMAP, FREVERSE, FMREVERSE = 1, 2, 4, 8, 16, 32
FREAD1, FREAD2, FSECONDARY, FQCFAIL, FDUP, FSUPPLEMENTARY = 64, 128, 256, 512, 1024, 2048


def _f32(x: float) -> float:
    return struct.unpack("<f", struct.pack("<f", x))[0]


def tag_typecode(value):
    """pysam's inference of a tag's BAM type code for an untyped value."""
    if isinstance(value, bool):
        value = int(value)
    if isinstance(value, int):
        if value < 0:
            if value >= -128:
                return "c"
            if value >= -32768:
                return "s"
            return "i"
        if value <= 255:
            return "C"
        if value <= 65535:
            return "S"
        return "I"
    if isinstance(value, float):
        return "f"
    if isinstance(value, (str, bytes)):
        return "Z"
    if isinstance(value, (list, tuple, array.array)):
        return "B"
    # numpy scalars
    try:
        import numpy as np
        if isinstance(value, np.integer):
            return tag_typecode(int(value))
        if isinstance(value, np.floating):
            return "f"
    except ImportError:  # pragma: no cover
        pass
    raise ValueError(f"cannot infer tag type for {type(value)!r}")


def array_subtype(values):
    """pysam's element type for an untyped list tag ('B' array)."""
    if isinstance(values, array.array):
        return {"b": "c", "B": "C", "h": "s", "H": "S", "i": "i", "I": "I",
                "l": "i", "L": "I", "f": "f", "d": "f"}[values.typecode]
    vals = list(values)
    if any(isinstance(v, float) for v in vals):
        return "f"
    if not vals:
        return "C"
    lo, hi = min(vals), max(vals)
    if lo < 0:
        if lo >= -128 and hi <= 127:
            return "c"
        if lo >= -32768 and hi <= 32767:
            return "s"
        return "i"
    if hi <= 255:
        return "C"
    if hi <= 65535:
        return "S"
    return "I"


_ARRAY_CODE = {"c": "b", "C": "B", "s": "h", "S": "H", "i": "i", "I": "I", "f": "f"}


def normalise_tag(value, typecode):
    """Value as it reads back from a bam1_t after pysam stored it."""
    if typecode == "f":
        return _f32(float(value))
    if typecode in "cCsSiI":
        return int(value)
    if typecode == "Z":
        return value.decode() if isinstance(value, bytes) else str(value)
    if typecode == "A":
        return str(value)
    if typecode == "B":
        sub = array_subtype(value)
        if sub == "f":
            return array.array("f", [float(v) for v in value])
        return array.array(_ARRAY_CODE[sub], [int(v) for v in value])
    raise ValueError(typecode)


class AlignedSegment:
    """Subset of ``pysam.AlignedSegment`` (see module docstring)."""

    __slots__ = ("query_name", "flag", "reference_id", "reference_start",
                 "_mapq", "_cigar", "_seq", "_qual", "next_reference_id",
                 "next_reference_start", "template_length", "_tags")

    def __init__(self, header=None):
        self.query_name = None
        self.flag = 0
        self.reference_id = -1
        self.reference_start = -1
        self._mapq = 255
        self._cigar = None
        self._seq = None
        self._qual = None
        self.next_reference_id = -1
        self.next_reference_start = -1
        self.template_length = 0
        self._tags = []   # list of [tag, typecode, value]

    # -- scalar fields -------------------------------------------------
    @property
    def mapping_quality(self):
        return self._mapq

    @mapping_quality.setter
    def mapping_quality(self, v):
        # pysam stores into an unsigned C field through nb_int: floats truncate
        self._mapq = int(v)

    # -- cigar ----------------------------------------------------------
    @property
    def cigartuples(self):
        if not self._cigar:
            return None
        return [tuple(x) for x in self._cigar]

    @cigartuples.setter
    def cigartuples(self, v):
        self._cigar = [(int(op), int(n)) for op, n in v] if v else None

    @property
    def cigarstring(self):
        if not self._cigar:
            return None
        return "".join(f"{n}{CIGAR_CHARS[op]}" for op, n in self._cigar)

    @cigarstring.setter
    def cigarstring(self, s):
        if s is None or s == "*":
            self._cigar = None
            return
        out, num = [], ""
        for ch in s:
            if ch.isdigit():
                num += ch
            else:
                out.append((_CIGAR_CODE[ch], int(num)))
                num = ""
        self._cigar = out

    @property
    def query_sequence(self):
        return self._seq

    @query_sequence.setter
    def query_sequence(self, s):
        self._seq = s if s else None
        self._qual = None      # pysam: setting the sequence invalidates qualities

    @property
    def query_qualities(self):
        # pysam returns None when the record holds no sequence (l_qseq == 0)
        return self._qual if self._seq else None

    @query_qualities.setter
    def query_qualities(self, q):
        if q is None:
            self._qual = None
        else:
            self._qual = array.array("B", [int(x) for x in q])

    @property
    def query_length(self):
        return len(self._seq) if self._seq else 0

    @property
    def query_alignment_length(self):
        """pysam: query length without soft clips."""
        n = self.query_length
        if self._cigar:
            for op, ln in self._cigar:
                if op == 4:
                    n -= ln
        return n

    @property
    def reference_length(self):
        if not self._cigar:
            return None
        return sum(n for op, n in self._cigar if op in (0, 2, 3, 7, 8))

    @property
    def reference_end(self):
        rl = self.reference_length
        return None if rl is None else self.reference_start + rl

    # -- flags ----------------------------------------------------------
    def _bit(b):  # noqa: N805
        return property(lambda self: bool(self.flag & b))

    is_paired = _bit(FPAIRED)
    is_proper_pair = _bit(FPROPER)
    is_unmapped = _bit(FUNMAP)
    mate_is_unmapped = _bit(FMUNMAP)
    is_reverse = _bit(FREVERSE)
    mate_is_reverse = _bit(FMREVERSE)
    is_read1 = _bit(FREAD1)
    is_read2 = _bit(FREAD2)
    is_secondary = _bit(FSECONDARY)
    is_qcfail = _bit(FQCFAIL)
    is_duplicate = _bit(FDUP)
    is_supplementary = _bit(FSUPPLEMENTARY)
    del _bit

    # -- tags -----------------------------------------------------------
    def get_tag(self, tag, with_value_type=False):
        for t, code, v in self._tags:
            if t == tag:
                return (v, code) if with_value_type else v
        raise KeyError(f"tag '{tag}' not present")

    def has_tag(self, tag):
        return any(t == tag for t, _, _ in self._tags)

    def get_tags(self, with_value_type=False):
        if with_value_type:
            return [(t, v, code) for t, code, v in self._tags]
        return [(t, v) for t, code, v in self._tags]

    def set_tags(self, tags):
        self._tags = []
        for item in tags or ():
            if len(item) == 3:
                t, v, code = item
            else:
                t, v = item
                code = tag_typecode(v)
            if code in "cCsSiI":
                code = tag_typecode(int(v))
            self._tags.append([t, code, normalise_tag(v, code)])

    def set_tag(self, tag, value, value_type=None):
        self._tags = [x for x in self._tags if x[0] != tag]
        if value is None:
            return
        code = value_type or tag_typecode(value)
        self._tags.append([tag, code, normalise_tag(value, code)])

    def __repr__(self):
        return (f"AlignedSegment({self.query_name}, flag={self.flag}, tid={self.reference_id}, "
                f"pos={self.reference_start}, mapq={self._mapq}, cigar={self.cigarstring}, "
                f"seq={self._seq})")

    def to_dict(self):
        """Decoded-record view used for parity comparisons."""
        tags = []
        for t, code, v in self._tags:
            if code == "B":
                tags.append([t, "B" + array_subtype(v), [float(x) if isinstance(v, array.array)
                                                         and v.typecode == "f" else int(x) for x in v]])
            else:
                tags.append([t, code, v])
        return {
            "qname": self.query_name, "flag": self.flag, "tid": self.reference_id,
            "pos": self.reference_start, "mapq": self._mapq, "cigar": self.cigarstring,
            "rnext": self.next_reference_id, "pnext": self.next_reference_start,
            "tlen": self.template_length, "seq": self._seq,
            "qual": list(self._qual) if self._qual is not None else None, "tags": tags,
        }
