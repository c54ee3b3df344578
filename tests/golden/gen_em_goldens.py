"""Generates tests/golden/em_goldens.npz from the REFERENCE implementation.

Run in the build container only (needs /root/reference):
    python -B tests/golden/gen_em_goldens.py

Imports /root/reference/src/ReadsCluster.py and calls its EMCluster
(ReadsCluster.py:221-277) on seeded synthetic feature matrices, re-seeding
numpy's global RNG with 2023 before every call (the per-window RNG contract,
SURVEY.md §8(a15)).  The final per-read likelihood comes from the reference's
own loglik (:104-122) on the returned (pi, theta, gamma).  Only the resulting
input/output arrays are committed; no reference code is copied.
"""
import os
import sys

import numpy as np

REF = "/root/reference/src"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "em_goldens.npz")


def make_matrix(rs, n, nf, n_clusters, noise, dup_frac=0.0):
    protos = rs.randint(0, 5, size=(n_clusters, nf))
    assign = rs.randint(0, n_clusters, size=n)
    X = protos[assign].copy()
    flip = rs.random_sample((n, nf)) < noise
    X[flip] = rs.randint(0, 5, size=int(flip.sum()))
    n_dup = int(dup_frac * n)
    if n_dup:
        X[n - n_dup:] = X[0]
    return X.astype(np.int64)


CASES = [
    # (n, nf, clusters, noise, dup_frac, seed)
    (6, 10, 2, 0.05, 0.0, 1),
    (6, 12, 1, 0.2, 0.0, 2),
    (8, 20, 2, 0.1, 0.5, 3),
    (10, 40, 3, 0.05, 0.0, 4),
    (16, 40, 2, 0.08, 0.0, 5),
    (16, 200, 2, 0.08, 0.0, 6),
    (16, 60, 2, 0.3, 0.0, 7),
    (16, 50, 3, 0.02, 0.5, 8),
    (20, 100, 4, 0.1, 0.0, 9),
    (24, 30, 2, 0.0, 0.0, 10),
    (32, 500, 2, 0.08, 0.0, 11),
    (32, 120, 3, 0.15, 0.25, 12),
    (32, 64, 1, 0.05, 0.0, 13),
    (40, 300, 4, 0.05, 0.0, 14),
    (48, 80, 2, 0.4, 0.0, 15),
    (64, 1000, 2, 0.08, 0.0, 16),
    (64, 200, 3, 0.1, 0.6, 17),
    (64, 3000, 2, 0.08, 0.0, 18),
    (64, 150, 5, 0.05, 0.0, 19),
    (12, 15, 2, 0.0, 0.9, 20),
    (64, 400, 2, 0.02, 0.9, 21),
    (9, 11, 2, 0.1, 0.0, 22),
]


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import ReadsCluster as RC  # reference module (this container only)

    arrays = {}
    for idx, (n, nf, nc, noise, dup, seed) in enumerate(CASES):
        rs = np.random.RandomState(1000 + seed)
        X = make_matrix(rs, n, nf, nc, noise, dup)
        np.random.seed(2023)
        K, _, Rclust, theta, gamma, pie, bics = RC.EMCluster(X, initselection=1)
        lik = RC.loglik(pie, theta, gamma, X)
        pre = f"c{idx:02d}_"
        arrays[pre + "X"] = X.astype(np.uint8)
        arrays[pre + "K"] = np.array(K)
        arrays[pre + "Rclust"] = np.asarray(Rclust)
        arrays[pre + "BICList"] = np.asarray(bics)
        arrays[pre + "gamma"] = gamma
        arrays[pre + "pi"] = np.asarray(pie)
        arrays[pre + "lik"] = lik
        arrays[pre + "theta_sum"] = np.asarray(theta).sum(axis=(1, 2))
        if nf <= 500:
            arrays[pre + "theta"] = np.asarray(theta)
        print(idx, n, nf, "K=", K, "BIC[:3]=", np.round(bics[:3], 3))
    # legacy RNG stream after seed(2023): the exponentials numpy's dirichlet consumes
    arrays["rng_2023_exp"] = np.random.RandomState(2023).standard_exponential(4096)
    arrays["n_cases"] = np.array(len(CASES))
    np.savez_compressed(OUT, **arrays)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
