"""The device sort's reuse walk (poa_fold.hip dfs_sort; DESIGN §4.2 "Sort
reuse") replayed on the host against spoa's full DFS topological order: for
every fold of a task, walking the previous order's segments (copying the ones
with no changed or done node, running the DFS from the other segments' roots,
then the new ids as roots) must give exactly the order the DFS gives
(tests/cpp/sort_walk_replay.cpp, linked with the CPU oracle; the device's own
planes are checked against the host graph under SVS_POA_VERIFY_GRAPH=1 in the
GPU tests)."""
import os
import random
import subprocess
import tempfile

import pytest

from tests import helpers

SRC = os.path.join(helpers.ROOT, "tests", "cpp", "sort_walk_replay.cpp")
ORACLE = os.path.join(helpers.ROOT, "oracle", "spoa_oracle.cpp")
BIN = os.path.join(helpers.ROOT, "tests", "build", "sort_walk_replay")


@pytest.fixture(scope="module")
def replay():
    newest = max(os.path.getmtime(SRC), os.path.getmtime(ORACLE))
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < newest:
        os.makedirs(os.path.dirname(BIN), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-o", BIN, SRC])
    return BIN


def run(replay, seqs, seed, trials):
    """(DFS examinations the walk ran, ranks it copied)"""
    fd, path = tempfile.mkstemp(suffix=".txt")
    with os.fdopen(fd, "w") as f:
        f.write("\n".join(seqs) + "\n")
    try:
        out = subprocess.run([replay, path, str(seed), str(trials)], capture_output=True, text=True, timeout=300)
    finally:
        os.unlink(path)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stderr + out.stdout
    f = out.stdout.split()
    return int(f[2]), int(f[5])


def test_walk_gives_the_dfs_order_on_synthetic_windows(replay):
    from svscope_amd import synth
    for w in range(3):
        win = synth.make_window(w, 24, 800)
        exams, copied = run(replay, win[0], w + 1, 4)  # the window, then 3 random thirds of it
        assert copied > exams  # most of each previous order is reused


def test_walk_gives_the_dfs_order_on_random_cases(replay):
    rnd = random.Random(5)
    n = 0
    for _ in range(60):
        seqs = [s for s in helpers.random_poa_case(rnd) if s]
        if len(seqs) < 2:
            continue
        run(replay, seqs, 1, 3)
        n += 1
    assert n >= 20
