"""Times the batched GPU EMCluster on config-3-like feature matrices
(64 reads x ~1600 columns, two haplotypes, 8% symbol noise)."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from svscope_amd.reads_cluster import em_cluster_batch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--windows", type=int, default=1024)
ap.add_argument("--reads", type=int, default=64)
ap.add_argument("--feat", type=int, default=1600)
ap.add_argument("--haps", type=int, default=2)
a = ap.parse_args()
rs = np.random.RandomState(3)
mats = []
for w in range(a.windows):
    protos = rs.randint(0, 5, size=(a.haps, a.feat))
    X = protos[rs.randint(0, a.haps, size=a.reads)]
    flip = rs.random_sample(X.shape) < 0.08
    X[flip] = rs.randint(0, 5, size=int(flip.sum()))
    mats.append(X.astype(np.uint8))
em_cluster_batch(mats[:4])  # warm up
timing = {}
t = time.time()
out = em_cluster_batch(mats, timing=timing)
wall = time.time() - t
print(json.dumps({"windows": a.windows, "reads": a.reads, "feat": a.feat, "wall_s": round(wall, 3),
                  "windows_per_s": round(a.windows / wall, 1), "timing": timing,
                  "K_hist": np.bincount([o["K"] for o in out]).tolist(),
                  "rng_used_mean": float(np.mean([o["rng_used"] for o in out]))}))
