"""Host model of the general kernel's insertion layout by events (test
infrastructure: tests/test_fil_model.py checks it against the oracle's
column-by-column reconstruct_alignment, DuplexUMIConsensusReads.py:430-547).

The reference walks every column t = 0..T-1 with every read; a column is an
insertion column when some read's current CIGAR op is I (:476-478).  Only reads
holding an I run can make one, and between insertion blocks every read
advances one op per column once started (:506-535), so:

phase A  (lane = read with an I run): the column where each I run becomes
         current follows from the number of normal columns since the read's
         start; blocks of insertion columns are found event by event
         (activations at the same column form one block, its length the longest
         of their runs) instead of column by column;
phase B  (lane = column): every read's element at column t from N(t), the
         number of normal columns before t: op index j = N(t) - N(s_r) (+ the I
         run's length once it is past), then the op and the base index at j.

Records outside its assumptions return None (the kernel keeps the
column-by-column layout for them): a read with more than one I run or more than
four runs, an I read whose bases run out before its I run ends, or a read with
fewer M + I ops than bases.
"""
from __future__ import annotations


def _runs(cig):
    return [(0 if o in (7, 8) else o, n) for o, n in cig]


def fil_layout(pos, cigars, seqs, quals):
    """(al, aq, min_pos) as oracle.reconstruct, or None when ineligible."""
    n = len(pos)
    runs = [_runs(c) for c in cigars]
    lens = [len(s) for s in seqs]
    min_pos = min(pos)
    T = max(p + ln for p, ln in zip(pos, lens)) - min_pos
    for r in range(n):
        if len(runs[r]) > 4:
            return None
        mi = sum(ln for o, ln in runs[r] if o in (0, 1))
        if mi < lens[r]:
            return None                    # ops exhausted while bases remain (an IndexError case)
        if sum(1 for o, _ in runs[r] if o == 1) > 1:
            return None
    s = [p - min_pos for p in pos]        # the column where the read starts (:506)
    # ---- phase A: I reads
    ird = {}
    for r in range(n):
        for k, (o, ln) in enumerate(runs[r]):
            if o == 1:
                a = sum(l2 for o2, l2 in runs[r][:k])             # M/D ops before the I run
                b = sum(l2 for o2, l2 in runs[r][:k] if o2 == 0)   # bases before it
                if b + ln > lens[r]:
                    return None                                   # bases run out in or before the run
                if b >= lens[r] and a > 0:
                    return None
                # every M/D op before the run is advanced with bases left
                # (b < len before each: the last M is base b - 1 < len)
                ird[r] = {"need": a, "L": ln, "is": b, "E": None}
    insflag = [0] * T
    t = 0
    pend = set(ird)
    while pend:
        cand = {r: (t if ird[r]["need"] == 0 else max(t, s[r]) + ird[r]["need"]) for r in pend}
        tn = min(cand.values())
        if tn >= T:
            break
        for r in pend:
            ird[r]["need"] -= max(0, tn - max(t, s[r])) if ird[r]["need"] > 0 else 0
        act = [r for r in pend if ird[r]["need"] == 0 and cand[r] == tn]
        B = max(ird[r]["L"] for r in act)
        for c in range(tn, min(T, tn + B)):
            insflag[c] = 1
        for r in act:
            ird[r]["E"] = tn
            pend.discard(r)
        t = tn + B
    # prefix counts of normal columns: N[t] = normal columns in [0, t)
    N = [0] * (T + 1)
    for c in range(T):
        N[c + 1] = N[c] + (0 if insflag[c] else 1)
    # ---- phase B
    al = [[] for _ in range(n)]
    aq = [[] for _ in range(n)]
    for r in range(n):
        info = ird.get(r)
        for c in range(T):
            if insflag[c]:
                if info is not None and info["E"] is not None and info["E"] <= c < info["E"] + info["L"]:
                    i = info["is"] + (c - info["E"])
                    al[r].append(seqs[r][i].lower())
                    aq[r].append(quals[r][i])
                else:
                    al[r].append("+")
                    aq[r].append("+")
                continue
            if c < s[r]:
                al[r].append("N")
                aq[r].append(2)
                continue
            j = N[c] - N[s[r]]
            if info is not None and info["E"] is not None and info["E"] < c:
                j += info["L"]
            # op at expanded index j, bases consumed before it
            acc = accis = 0
            op = -1
            isx = 0
            for o, ln in runs[r]:
                if op < 0 and j < acc + ln:
                    op = o
                    isx = accis + (j - acc if o in (0, 1) else 0)
                acc += ln
                if o in (0, 1):
                    accis += ln
            if op < 0:
                isx = accis
            if isx >= lens[r]:
                al[r].append("N")
                aq[r].append(2)
            elif op == 2:
                al[r].append("-")
                aq[r].append("-")
            elif op == 0:
                al[r].append(seqs[r][isx])
                aq[r].append(quals[r][isx])
            else:
                raise AssertionError(f"op {op} at a normal column (read {r}, column {c})")
    return al, aq, min_pos
