"""Checker utilities over oracle outputs — TEST INFRASTRUCTURE ONLY (see ``oracle/__init__``).

``perm_report`` classifies, pair by pair, how a ``perm_mat`` computed on the device relates to the
oracle's for the same inputs.  The reference picks matches by ``round(k * min(n1, n2))`` (half to
even, ``soft_topk.py:56-77``) among the Hungarian assignment of ``ds_mat`` ranked by ds_mat
(``ngm.py:444-449``), so two correct fp32 evaluations can differ in exactly three ways:

* ``select_tie``  : same Hungarian assignment (so its cost gap under the oracle's ds_mat is 0), same
                    match count, a different pick among matches whose oracle ds_mat values are
                    equal within ``tol`` (soft top-k saturates at 1.0: many exact ties, torch's
                    argsort order among them is implementation defined, quirk A.10(v));
* ``lsa_near_tie``: a different Hungarian assignment L whose total under the ORACLE's ds_mat is
                    within ``m * opt_eps`` (1e-6 per match) of the oracle assignment's -- L is an
                    optimum of the oracle's own costs up to rounding, as scipy's LSAP on near-equal
                    costs can return -- same count, and the oracle's ds_mat values at the picks
                    equal those at the oracle's picks within ``tol``;
* ``k_rounding``  : the counts differ by one because k * min(n1, n2) of the two sides round to
                    neighbouring integers while the two k_prob agree within ``k_tol`` (the k_prob
                    tolerance straddles a .5 rounding boundary).

A bf16-mode ds_mat deviates from the oracle's by some ``delta`` per entry, so for reduced-precision
results (``perm_report(..., reduced_precision=True)``; never for fp32) one more class is provable
rather than a tie:

* ``lsa_eps_opt`` : same match count, and the device's Hungarian assignment L is within
                    ``2 * m * delta`` of optimal under the ORACLE's ds_mat (for any assignment A,
                    |cost_dev(A) - cost_ref(A)| <= m * delta, so the device optimum can lose at
                    most 2 m delta against the oracle optimum); scipy's LSAP then legitimately
                    returns a different optimum of the perturbed costs.

Every class other than ``identical`` also requires the device's picks to be matches of its own
Hungarian assignment (P <= L) when L is given, and records the assignment gap (``pair_detail``).
Anything else is ``mismatch``.
"""
import numpy as np
import torch


def _half_even(x):
    return int(np.round(float(x)))          # numpy rounds half to even, like torch.round


OPT_EPS = 1e-6      # per-match slack of "optimal under the oracle's costs" (fp32 rounding of the sums)


def lsa_gap(ds_ref, L, Lr):
    """Oracle-optimal total minus the total of assignment L, both under the oracle's ds_mat (float64)."""
    return float(ds_ref[Lr > 0].double().sum() - ds_ref[L > 0].double().sum())


def classify_pair(P, R, ds_ref, L=None, Lr=None, k=None, k_ref=None, m=None, tol=1e-5, k_tol=1e-4, delta=None,
                  opt_eps=OPT_EPS):
    """One pair: P / R = device / oracle perm_mat, ds_ref = oracle ds_mat, L / Lr = device /
    oracle Hungarian 0/1 matrices, k / k_ref = k_prob, m = min(n1, n2), delta = max |device ds_mat -
    oracle ds_mat| of the pair."""
    if torch.equal(P, R):
        return "identical"
    have_lsa = L is not None and Lr is not None
    if have_lsa and bool(((P > 0) & ~(L > 0)).any()):
        return "mismatch"                      # a pick outside the device's own assignment
    cp, cr = int((P > 0).sum()), int((R > 0).sum())
    if cp == cr:
        a, b = ds_ref[P > 0], ds_ref[R > 0]
        picks_tie = bool(a.numel()) and float((torch.sort(a).values - torch.sort(b).values).abs().max()) <= tol
        if not have_lsa:
            return "select_tie" if picks_tie else "mismatch"      # unproven: no assignments given
        gap = lsa_gap(ds_ref, L, Lr)
        mm = m or int((Lr > 0).sum())
        if picks_tie and torch.equal(L, Lr):
            return "select_tie"
        if picks_tie and gap <= mm * opt_eps:
            return "lsa_near_tie"
        if delta is not None and mm and gap <= 2.0 * mm * float(delta) + mm * opt_eps:
            return "lsa_eps_opt"
        return "mismatch"
    if k is not None and abs(cp - cr) == 1 and m:
        if abs(float(k) - float(k_ref)) <= k_tol and _half_even(float(k) * m) != _half_even(float(k_ref) * m):
            return "k_rounding"
    return "mismatch"


def pair_detail(P, R, ds_ref, L=None, Lr=None, k=None, k_ref=None, m=None, delta=None):
    """Diagnostics of one differing pair: match counts, the device assignment's optimality gap under
    the oracle's ds_mat with the bounds it is judged against, and k * m of both sides."""
    d = {"count": int((P > 0).sum()), "count_ref": int((R > 0).sum())}
    if L is not None and Lr is not None:
        d["lsa_gap"] = lsa_gap(ds_ref, L, Lr)
        d["lsa_identical"] = bool(torch.equal(L, Lr))
        d["picks_in_own_assignment"] = not bool(((P > 0) & ~(L > 0)).any())
        if m:
            d["near_tie_bound"] = m * OPT_EPS
            if delta is not None:
                d["eps_opt_bound"] = 2.0 * m * float(delta) + m * OPT_EPS
    if k is not None and m:
        d["k_m"], d["k_ref_m"] = float(k) * m, float(k_ref) * m
    return d


def perm_report(res, ref, n1, n2, tol=1e-5, k_tol=1e-4, reduced_precision=False):
    """Per-pair classification of ``res`` (device outputs, any device) against ``ref`` (oracle)
    -> dict with the class of every pair and the counts / fractions.  ``reduced_precision``: the
    device ran a bf16 mode; its per-pair ds_mat deviation enables the ``lsa_eps_opt`` class."""
    P, R = res["perm_mat"].detach().float().cpu(), ref["perm_mat"].detach().float().cpu()
    L = res["lsa"].detach().float().cpu() if "lsa" in res else None
    Lr = ref["lsa"].detach().float().cpu() if "lsa" in ref else None
    k, kr = res["k_prob"].detach().float().cpu(), ref["k_prob"].detach().float().cpu()
    ds = ref["ds_mat"].detach().float().cpu()
    dsd = res["ds_mat"].detach().float().cpu()
    cls, deltas, detail = [], [], {}
    for b in range(P.shape[0]):
        m = min(int(n1[b]), int(n2[b]))
        delta = float((dsd[b] - ds[b]).abs().max())
        deltas.append(delta)
        # lsa_eps_opt is a reduced-precision class only: in fp32 a different assignment must
        # be a near-tie of the oracle's own costs (m * OPT_EPS), not merely within 2 m delta of optimal
        cls.append(classify_pair(P[b], R[b], ds[b], None if L is None else L[b], None if Lr is None else Lr[b],
                                 k[b], kr[b], m, tol, k_tol, delta if reduced_precision else None))
        if cls[-1] != "identical":
            detail[b] = pair_detail(P[b], R[b], ds[b], None if L is None else L[b], None if Lr is None else Lr[b],
                                    k[b], kr[b], m, delta)
            detail[b]["class"] = cls[-1]
    B = len(cls)
    counts = {c: cls.count(c) for c in ("identical", "select_tie", "lsa_near_tie", "lsa_eps_opt", "k_rounding",
                                        "mismatch")}
    return {"classes": cls, "counts": counts, "pairs": B,
            "identical_frac": counts["identical"] / max(B, 1),
            "tie_equivalent_frac": (counts["identical"] + counts["select_tie"] + counts["lsa_near_tie"]) / max(B, 1),
            "explained_frac": (B - counts["mismatch"]) / max(B, 1),
            "ds_mat_delta": deltas, "reduced_precision": bool(reduced_precision), "detail": detail}
