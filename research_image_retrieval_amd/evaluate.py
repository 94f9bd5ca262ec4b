"""Revisited-protocol mAP (host side, numpy) — restatement of the reference's
utils/evaluate.py:4-194, the consumer of the ranker's output.  It stays on the
host: it is O(#positives) per query, not the hot path.

Arithmetic follows the reference exactly (float64, same accumulation order),
so results are bit-identical; tests/golden pins that.  Two reference defects
are NOT reproduced (documented in DESIGN.md):
  * 'oxford5k'/'paris6k' unpack 4 values from a 2-value return (:157) and
    raise; here they print and return the mAP;
  * with truncated (li=True) lists a query whose positives all fall outside
    the list makes ``max(pos)`` raise (:104); here its AP and P@k are 0.
"""
import numpy as np


def compute_ap(ranks, nres):
    """Trapezoidal AP over the zero-based ranks of the positives (:4-34)."""
    ap = 0.0
    step = 1.0 / nres
    for j, r in enumerate(ranks):
        p0 = 1.0 if r == 0 else float(j) / r
        p1 = float(j + 1) / (r + 1)
        ap += (p0 + p1) * step / 2.0
    return ap


def _positions(ranks, i, wanted, li):
    if li:
        row = np.asarray(ranks[i])
    else:
        row = ranks[:, i]
    if len(wanted) == 0:
        return np.zeros(0, dtype=np.int64)
    return np.flatnonzero(np.isin(row, wanted))


def _shift_by_junk(pos, junk):
    """Each positive moves up by the number of junk items ranked before it."""
    if len(junk) == 0:
        return pos
    pos = pos.copy()
    return pos - np.searchsorted(junk, pos, side="left")


def compute_map(ranks, gnd, keeps=None, li=False):
    nq = len(gnd)
    aps = np.zeros(nq)
    m_ap = 0.0
    empty = 0
    if keeps:
        pr = np.zeros(len(keeps))
        prs = np.zeros((nq, len(keeps)))
    for i in range(nq):
        ok = np.array(gnd[i]["ok"])
        if ok.shape[0] == 0:
            aps[i] = float("+inf")
            if keeps:
                prs[i, :] = float("+inf")
            empty += 1
            continue
        junk = np.array(gnd[i]["junk"]) if "junk" in gnd[i] else np.empty(0)
        pos = _positions(ranks, i, ok, li)
        jpos = _positions(ranks, i, junk, li)
        pos = _shift_by_junk(pos, jpos)
        ap = compute_ap(pos, len(ok))
        m_ap += ap
        aps[i] = ap
        if keeps:
            pos1 = pos + 1
            for j, kap in enumerate(keeps):
                if len(pos1) == 0:
                    prs[i, j] = 0.0
                    continue
                kp = min(max(pos1), kap)
                prs[i, j] = (pos1 <= kp).sum() / kp
            pr += prs[i, :]
    m_ap = m_ap / (nq - empty)
    if keeps:
        return m_ap, aps, pr / (nq - empty), prs
    return m_ap, aps


def _protocol(gnd, ok_keys, junk_keys):
    out = []
    for g in gnd:
        out.append({"ok": np.concatenate([g[k] for k in ok_keys]),
                    "junk": np.concatenate([g[k] for k in junk_keys])})
    return out


def compute_map_and_print(dataset, featuretype, mode, ranks, gnd, kappas=(1, 5, 10), verbose=False, li=False):
    kappas = list(kappas)
    if dataset.startswith("oxford5k") or dataset.startswith("paris6k"):
        m, _aps = compute_map(ranks, gnd, li=li)
        print(">> {}: mAP {:.2f}".format(dataset, np.around(m * 100, decimals=2)))
        return np.around(m * 100, decimals=2)
    if not (dataset.startswith("roxford5k") or dataset.startswith("rparis6k")):
        raise ValueError(f"unknown dataset {dataset}")
    mapE, apsE, mprE, _ = compute_map(ranks, _protocol(gnd, ["easy"], ["junk", "hard"]), kappas, li=li)
    mapM, apsM, mprM, _ = compute_map(ranks, _protocol(gnd, ["easy", "hard"], ["junk"]), kappas, li=li)
    mapH, apsH, mprH, _ = compute_map(ranks, _protocol(gnd, ["hard"], ["junk", "easy"]), kappas, li=li)
    r = lambda v: np.around(v * 100, decimals=2)  # noqa: E731
    print(">> Test Dataset: {} *** Feature Type: {} >>".format(dataset, featuretype))
    print(">> mAP Eeay: {}, Medium: {}, Hard: {}".format(r(mapE), r(mapM), r(mapH)))
    print(">> mP@k{} Easy: {}, Medium: {}, Hard: {}".format(kappas, r(mprE), r(mprM), r(mprH)))
    if verbose:
        print(">> Query aps: >>\nEeay: {}\nMedium: {}\nHard: {}".format(r(apsE), r(apsM), r(apsH)))
    return r(mapE), r(mapM), r(mapH)
