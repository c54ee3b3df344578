"""Runs the kernel-variant oracle cases of tests/test_poa_gpu.py under one
environment N times in one process and counts the runs whose results differ
from the oracle (a nondeterministic failure shows as a rate, not a verdict).
  SVS_POA_STRIP_GLOBAL_POOL=1 SVS_POA_WPJ=4 python tools/repeat_variant_check.py 20"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers  # noqa: E402
from oracle.spoa_oracle import poa as oracle_poa  # noqa: E402
from svscope_amd import synth  # noqa: E402
from svscope_amd.poa import poa_batch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
cases = helpers.random_cases(31, 40, max_seqs=10, max_len=260, edits=20)
cases += [synth.make_window(w, 12, 1500)[0] for w in range(2)]
want = [oracle_poa(c, 1) for c in cases]
bad_runs = 0
for k in range(n):
    got = poa_batch(cases)
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    if bad:
        bad_runs += 1
        print("run", k, "mismatched cases", bad[:10], flush=True)
print("runs", n, "bad runs", bad_runs, flush=True)
