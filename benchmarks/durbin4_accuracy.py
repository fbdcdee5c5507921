#!/usr/bin/env python3
"""Per-item accuracy of the three Durbin kernels against scipy's solve_toeplitz on the same r (the oracle,
features.py:226-228): durbin4_kernel (the default for 128 <= p <= 150), durbin8_kernel (lpc 'lattice8') and
the LDS Durbin (lpc 'lds'), on the golden sets and on the WSJ golden signals at orders 128, 130, 146, 149
(where durbin4 stops at an earlier phase than at p = 150).  For every set: quantiles of each kernel's a error
(max |a - a_ref| / max |a_ref| per item) and gg error (|gg - gg_ref| / gg_ref), of the ratio e4 / e8, and the
largest feature difference between the kernels.  One JSON line per set (the evidence behind the bars of
tests/test_gpu_parity.py::test_durbin4_matches_durbin8 and tests/test_durbin4_orders.py).

    python benchmarks/durbin4_accuracy.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch  # noqa: F401
    from conftest import load_golden
    from test_gpu_parity import run_gpu
    from oracle import fdlp_oracle as O
    cases = [("wsj", None), ("reverb", None), ("mel80", None), ("wsj", 128), ("wsj", 130), ("wsj", 146),
             ("wsj", 149)]
    for name, order in cases:
        meta, sig, ref, z = load_golden(name)
        if order is not None:
            meta = json.loads(json.dumps(meta))
            meta["opts"]["order"] = order
        runs = {k: run_gpu(meta, sig, z, debug=True, lpc=k) for k in ("auto", "lattice8", "lds")}
        nf = sum(runs["auto"][0].geometry(sig[u].size)[0] for u in meta["utts"])
        d = {k: pl.debug_fetch(nf, keys=("r", "a", "gg")) for k, (pl, _) in runs.items()}
        r = d["auto"]["r"].reshape(-1, d["auto"]["r"].shape[-1])
        p = d["auto"]["a"].shape[-1] - 1
        live = np.flatnonzero(r[:, 0] > 0)
        ea = {k: np.empty(live.size) for k in d}
        eg = {k: np.empty(live.size) for k in d}
        for n, i in enumerate(live):
            a_ref, gg_ref = O.lpc_from_autocorr(r[i], p)
            sc = np.abs(a_ref).max()
            for k in d:
                a = d[k]["a"].reshape(-1, p + 1)[i]
                g = d[k]["gg"].reshape(-1)[i]
                ea[k][n] = np.abs(a - a_ref).max() / sc
                eg[k][n] = abs(g - gg_ref) / abs(gg_ref)
        q = lambda x: {s: float(np.quantile(x, v)) for s, v in (("p50", 0.5), ("p99", 0.99), ("max", 1.0))}
        ratio = ea["auto"] / np.maximum(ea["lattice8"], 1e-300)
        feat = {}
        for k in ("lattice8", "lds"):
            feat[k] = max(float(np.nanmax(np.abs(runs["auto"][1][u][0] - runs[k][1][u][0]))) for u in meta["utts"])
        print(json.dumps(dict(set=name, order=p, items=int(live.size),
                              a_err={k: q(v) for k, v in ea.items()}, gg_err={k: q(v) for k, v in eg.items()},
                              a_ratio_4_over_8=q(ratio), frac_ratio_gt2=float(np.mean(ratio > 2)),
                              feature_maxdiff_vs_auto=feat)), flush=True)


if __name__ == "__main__":
    main()
