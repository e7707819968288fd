#!/usr/bin/env python3
"""Price trace_queue's per-batch work: least-squares fit of each 64-query batch's duration on
its wave-iteration counts (refill, node loop, leaf phases, triangle-deal chunks, traversal
calls), from the batch records tools/trace_tail.py writes (<out>_batches.npz, diagnostic build
`make wgt`).  Prints the per-iteration costs (us), the fit's R^2 and each term's share of the
summed batch time.

    python tools/batch_fit.py gpurun_out/r4_trace_tail3_batches.npz
"""
import argparse

import numpy as np

TERMS = ["const", "refill", "node", "leaf", "chunks", "calls"]


def fit(path):
    d = np.load(path)
    y = d["dur"].astype(float)
    X = np.stack([np.ones_like(y)] + [d[k].astype(float) for k in TERMS[1:]], 1)
    c = np.linalg.lstsq(X, y, rcond=None)[0]
    pred = X @ c
    r2 = 1.0 - ((y - pred) ** 2).sum() / ((y - y.mean()) ** 2).sum()
    share = (X * c).sum(0) / y.sum()
    return c, r2, share, X.mean(0), y.mean(), len(y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz", nargs="+")
    a = ap.parse_args()
    for p in a.npz:
        c, r2, share, mean, ymean, n = fit(p)
        print(f"{p}: {n} batches, mean {ymean:.2f} us, R^2 {r2:.3f}")
        print("  term      us/iter   mean/batch  share")
        for t, ci, mi, si in zip(TERMS, c, mean, share):
            print(f"  {t:8s} {ci:8.3f} {mi:11.2f} {si:7.3f}")


if __name__ == "__main__":
    main()
