"""Stress check for an intermittent kernel-variant mismatch: alternates a
decision batch of config-3 windows (churns device memory, graph blocks and
caches on every CU) with the kernel-variant oracle cases of
tests/test_poa_gpu.py under the two environments that once failed, and
counts mismatches.  python tools/stress_variant.py ROUNDS"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import helpers  # noqa: E402
from oracle.spoa_oracle import poa as oracle_poa  # noqa: E402
from svscope_amd import synth  # noqa: E402
from svscope_amd.decision_maker import DecisionBatch  # noqa: E402
from svscope_amd.poa import poa_batch  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cases = helpers.random_cases(31, 40, max_seqs=10, max_len=260, edits=20)
cases += [synth.make_window(w, 12, 1500)[0] for w in range(2)]
want = [oracle_poa(c, 1) for c in cases]
wins = [synth.make_window(w, 64, 3000) for w in range(48)]
wins = [(w[4], w[0], w[1], w[2], w[3]) for w in wins]  # (TDRecord, sequenceList, ReadIDs, flank_5, flank_3)
envs = [{"SVS_POA_STRIP_GLOBAL_POOL": "1", "SVS_POA_WPJ": "4"},
        {"SVS_POA_VERIFY_GRAPH": "1", "SVS_POA_PRUNE_SLACK": "-0.3", "SVS_POA_WPJ": "2"},
        {}, {"SVS_POA_WPJ": "2"}]
bad = 0
for k in range(rounds):
    DecisionBatch(wins)
    for env in envs:
        old = {e: os.environ.get(e) for e in env}
        os.environ.update(env)
        try:
            got = poa_batch(cases)
        finally:
            for e, v in old.items():
                if v is None:
                    os.environ.pop(e, None)
                else:
                    os.environ[e] = v
        diff = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
        if diff:
            bad += 1
            print("round", k, "env", env, "mismatched cases", diff, flush=True)
    print("round", k, "done", flush=True)
print("rounds", rounds, "bad", bad, flush=True)
