"""Checker utilities over oracle outputs — TEST INFRASTRUCTURE ONLY (see ``oracle/__init__``).

``perm_report`` classifies, pair by pair, how a ``perm_mat`` computed on the device relates to the
oracle's for the same inputs.  The reference picks matches by ``round(k * min(n1, n2))`` (half to
even, ``soft_topk.py:56-77``) among the Hungarian assignment of ``ds_mat`` ranked by ds_mat
(``ngm.py:444-449``), so two correct fp32 evaluations can differ in exactly three ways:

* ``select_tie``  : same Hungarian assignment, same match count, a different pick among matches
                    whose oracle ds_mat values are equal within ``tol`` (soft top-k saturates at
                    1.0: many exact ties, torch's argsort order among them is implementation
                    defined, quirk A.10(v));
* ``lsa_near_tie``: a different Hungarian assignment, same count, and the oracle's ds_mat values at
                    the picks equal those at the oracle's picks within ``tol`` (scipy's LSAP on
                    near-equal costs: a last-ulp difference of ds_mat moves the optimum);
* ``k_rounding``  : the counts differ by one because k * min(n1, n2) of the oracle lies within
                    ``k_tol * min(n1, n2)`` of a .5 rounding boundary (the k_prob parity tolerance
                    straddles it) and the two sides round to neighbouring integers.

Anything else is ``mismatch``.
"""
import numpy as np
import torch


def _half_even(x):
    return int(np.round(float(x)))          # numpy rounds half to even, like torch.round


def classify_pair(P, R, ds_ref, L=None, Lr=None, k=None, k_ref=None, m=None, tol=1e-5, k_tol=1e-4):
    """One pair: P / R = device / oracle perm_mat, ds_ref = oracle ds_mat, L / Lr = device /
    oracle Hungarian 0/1 matrices, k / k_ref = k_prob, m = min(n1, n2)."""
    if torch.equal(P, R):
        return "identical"
    cp, cr = int((P > 0).sum()), int((R > 0).sum())
    if cp == cr:
        a, b = ds_ref[P > 0], ds_ref[R > 0]
        if a.numel() and float((torch.sort(a).values - torch.sort(b).values).abs().max()) <= tol:
            if L is not None and Lr is not None and torch.equal(L, Lr):
                return "select_tie"
            return "lsa_near_tie"
        return "mismatch"
    if k is not None and abs(cp - cr) == 1 and m:
        x = float(k_ref) * m
        frac = x - np.floor(x)
        if abs(frac - 0.5) <= k_tol * m and _half_even(float(k) * m) != _half_even(x):
            return "k_rounding"
    return "mismatch"


def perm_report(res, ref, n1, n2, tol=1e-5, k_tol=1e-4):
    """Per-pair classification of ``res`` (device outputs, any device) against ``ref`` (oracle)
    -> dict with the class of every pair and the counts / fractions."""
    P, R = res["perm_mat"].detach().float().cpu(), ref["perm_mat"].detach().float().cpu()
    L = res["lsa"].detach().float().cpu() if "lsa" in res else None
    Lr = ref["lsa"].detach().float().cpu() if "lsa" in ref else None
    k, kr = res["k_prob"].detach().float().cpu(), ref["k_prob"].detach().float().cpu()
    ds = ref["ds_mat"].detach().float().cpu()
    cls = []
    for b in range(P.shape[0]):
        m = min(int(n1[b]), int(n2[b]))
        cls.append(classify_pair(P[b], R[b], ds[b], None if L is None else L[b], None if Lr is None else Lr[b],
                                 k[b], kr[b], m, tol, k_tol))
    B = len(cls)
    counts = {c: cls.count(c) for c in ("identical", "select_tie", "lsa_near_tie", "k_rounding", "mismatch")}
    return {"classes": cls, "counts": counts, "pairs": B,
            "identical_frac": counts["identical"] / max(B, 1),
            "tie_equivalent_frac": (counts["identical"] + counts["select_tie"] + counts["lsa_near_tie"]) / max(B, 1),
            "explained_frac": (B - counts["mismatch"]) / max(B, 1)}
