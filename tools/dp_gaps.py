"""Where the DP stream waits: an SVS_POA_TRACE timeline (svs_poa_engine.cpp
PoaTrace) of the device-graph engine, per DP launch.

A group's DP launch can start when the previous DP launch on the stream has
ended and the group's own loop has come round: its previous launch's fold
chain (kern 10+g), the host's wait / fold / pack phases for that group, then
the new tasks' chains (kern 20+g).  For each DP launch this script takes the
latest of those ends as what the launch waited for, and sums the DP stream's
idle time by cause.  Also prints the mean length of each stage of the loop.

  python tools/dp_gaps.py trace.txt [TAIL_MS]

TAIL_MS: only the DP launches of the trace's last TAIL_MS (bench.py's timed
steps come after its warm-up batches in the same session).
"""
import collections
import json
import sys


def runs(path):
    cur = None
    for line in open(path):
        if line.startswith("# begin"):
            if cur:
                yield cur
            cur = {"host": [], "kern": []}
            continue
        p = line.split()
        if not p or cur is None:
            continue
        if p[0] == "host":
            cur["host"].append((p[1], int(p[2]), float(p[3]), float(p[4])))
        elif p[0] == "kern":
            cur["kern"].append((int(p[1]), float(p[2]), float(p[3])))
    if cur:
        yield cur


def analyse(r, tail_ms=None):
    dp = sorted([k for k in r["kern"] if k[0] < 10], key=lambda k: k[1])
    if tail_ms:
        dp = [k for k in dp if k[1] >= dp[-1][2] - tail_ms]
    if len(dp) < 3:
        return None
    by = collections.defaultdict(list)  # (kind, group) -> [(t0, t1)], kinds: fold chain, pre chain, host phases
    for g, a, b in r["kern"]:
        if 10 <= g < 20:
            by[("chain", g - 10)].append((a, b))
        elif 20 <= g < 30:
            by[("pre", g - 20)].append((a, b))
    for name, g, a, b in r["host"]:
        by[(name, g)].append((a, b))
    for v in by.values():
        v.sort()

    def last_end_before(kind, g, t):
        ends = [b for a, b in by.get((kind, g), []) if b <= t + 0.05]
        return max(ends) if ends else None

    idle = collections.Counter()
    stage = collections.defaultdict(list)
    prev_end_g = {}
    for i in range(1, len(dp)):
        g, s, e = dp[i]
        gap = s - dp[i - 1][2]
        ends = {"dp_stream": dp[i - 1][2]}
        for kind in ("chain", "wait", "fold", "pack", "pre"):
            t = last_end_before(kind, g, s)
            if t is not None and (g not in prev_end_g or t >= prev_end_g[g] - 0.05):
                ends[kind] = t
        cause = max(ends, key=lambda k: ends[k])
        if gap > 0.02:
            idle[cause] += gap
        if g in prev_end_g:
            p = prev_end_g[g]
            # the loop's stages after this group's previous DP launch
            chain = [x for x in by.get(("chain", g), []) if x[0] >= p - 0.05 and x[1] <= s + 0.05]
            if chain:
                stage["fold_chain_ms"].append(chain[0][1] - chain[0][0])
                stage["chain_end_after_dp_ms"].append(chain[0][1] - p)
            stage["loop_ms"].append(s - p)
            for kind in ("wait", "fold", "pack"):
                ph = [x for x in by.get((kind, g), []) if x[0] >= p - 0.05 and x[1] <= s + 0.05]
                if ph:
                    stage[kind + "_ms"].append(sum(b - a for a, b in ph))
        prev_end_g[g] = e
    # host phases of the scheduler thread (a long one holds up both groups)
    host = {}
    for name in sorted({h[0] for h in r["host"]}):
        d = [b - a for n, _, a, b in r["host"] if n == name]
        host[name] = {"n": len(d), "total_ms": round(sum(d), 1), "over_10ms": sum(1 for x in d if x > 10),
                      "over_10ms_total_ms": round(sum(x for x in d if x > 10), 1)}
    span = dp[-1][2] - dp[0][1]
    busy = sum(e - s for _, s, e in dp)
    return {"dp_launches": len(dp), "span_ms": round(span, 1), "dp_busy_frac": round(busy / span, 4),
            "dp_idle_ms_by_cause": {k: round(v, 1) for k, v in idle.most_common()},
            "mean_dp_ms": round(busy / len(dp), 2),
            "loop_stage_means_ms": {k: round(sum(v) / len(v), 2) for k, v in stage.items() if v},
            "host_phases": host}


if __name__ == "__main__":
    tail = float(sys.argv[2]) if len(sys.argv) > 2 else None
    out = [a for a in (analyse(r, tail) for r in runs(sys.argv[1])) if a]
    print(json.dumps(out[-1] if len(out) == 1 else out, indent=1))
