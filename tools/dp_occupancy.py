"""Resident DP waves over time, from an SVS_WG_TIMES dump (development build
of poa_strip.hip: one record per wave, start and end by s_memrealtime at
100 MHz, the job index, the launch's job table, WPJ and job count, the job's
rows and read length, and for wave 0 the strip rows the job computed).

    python tools/dp_occupancy.py DUMP [LAST_LAUNCHES] [SLOTS]

Launches are told apart by their job table (one per task group, so one per
DP stream) and stream order (a launch starts after the previous one on its
stream has ended).  Over the last LAST_LAUNCHES launches (the bench's timed
ones: its `poa_launches`) it prints the mean resident DP waves over the time
any DP launch runs, the share of that time spent at each occupancy level,
and per launch how long its waves kept the chip full: the time until its
resident waves fell below 90 % / 50 % of its peak, against its length.
SLOTS: the chip's DP wave slots (7 per SIMD x 1024 SIMDs = 7168).
"""
import collections
import json
import sys

import numpy as np


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    slots = int(sys.argv[3]) if len(sys.argv) > 3 else 7168
    a = np.fromfile(path, dtype=np.uint64).reshape(-1, 8)
    t0 = a[:, 0].astype(np.int64)
    t1 = a[:, 1].astype(np.int64)
    key = a[:, 3]
    launches = []
    for k in np.unique(key):
        idx = np.where(key == k)[0]
        idx = idx[np.argsort(t0[idx], kind="stable")]
        cur, cur_end = [], -1
        for i in idx:
            if cur and t0[i] > cur_end:
                launches.append(np.array(cur))
                cur, cur_end = [], -1
            cur.append(i)
            cur_end = max(cur_end, t1[i])
        if cur:
            launches.append(np.array(cur))
    launches.sort(key=lambda ix: t0[ix].min())
    if last:
        launches = launches[-last:]
    sel = np.concatenate(launches)
    # resident waves over time (s_memrealtime ticks: 10 ns, 1e5 per ms)
    ev = np.concatenate([np.stack([t0[sel], np.ones(len(sel), np.int64)], 1),
                         np.stack([t1[sel], -np.ones(len(sel), np.int64)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    times, d = ev[:, 0], ev[:, 1]
    level = np.cumsum(d)
    dt = np.diff(times)
    lv = level[:-1]
    busy = dt[lv > 0].sum()
    wave_ticks = (lv * dt).sum()
    bins = [0, 1, 0.25 * slots, 0.5 * slots, 0.75 * slots, 0.9 * slots, 1e12]
    hist = collections.OrderedDict()
    names = ["idle", "<25%", "25-50%", "50-75%", "75-90%", ">=90%"]
    for n, lo, hi in zip(names, bins[:-1], bins[1:]):
        m = (lv >= lo) & (lv < hi)
        if n == "idle":
            continue
        hist[n] = round(float(dt[m].sum() / busy), 4)
    per = []
    for ix in launches:
        s0, e1 = t0[ix].min(), t1[ix].max()
        evl = np.concatenate([np.stack([t0[ix], np.ones(len(ix), np.int64)], 1),
                              np.stack([t1[ix], -np.ones(len(ix), np.int64)], 1)])
        evl = evl[np.lexsort((evl[:, 1], evl[:, 0]))]
        lvl = np.cumsum(evl[:, 1])
        peak = lvl.max()
        ipk = int(np.argmax(lvl))
        after = np.arange(len(lvl)) > ipk

        def first_below(fr):
            w = np.where(after & (lvl < fr * peak))[0]
            return (evl[w[0], 0] - s0) if len(w) else (e1 - s0)

        waves = (t1[ix] - t0[ix])
        per.append({
            "ms": (e1 - s0) / 1e5, "waves": len(ix), "peak": int(peak),
            "full90_ms": first_below(0.9) / 1e5, "full50_ms": first_below(0.5) / 1e5,
            "fill": float(waves.sum() / (peak * (e1 - s0))),
            "wave_ms_mean": float(waves.mean() / 1e5), "wave_ms_max": float(waves.max() / 1e5),
        })
    P = {k: float(np.mean([p[k] for p in per])) for k in per[0]}
    # the launches' waves by start delay (after the launch's first wave) and
    # duration, in launch-relative ms; job order against duration (the engine
    # issues the longest expected job first)
    late, early_d, late_d, late_s, rank_corr, end_early, end_all = [], [], [], [], [], [], []
    for ix in launches:
        s0 = t0[ix].min()
        st = (t0[ix] - s0) / 1e5
        du = (t1[ix] - t0[ix]) / 1e5
        lt = st > 1.0
        late.append(lt.mean())
        early_d.append(np.percentile(du[~lt], [10, 50, 90, 100]))
        if lt.any():
            late_d.append(du[lt].mean())
            late_s.append(st[lt].mean())
        end_early.append((st + du)[~lt].max())
        end_all.append((st + du).max())
        job = (a[ix, 2] >> np.uint64(32)).astype(np.int64)
        if len(ix) > 8:
            rj = np.argsort(np.argsort(job)).astype(float)
            rd = np.argsort(np.argsort(-du)).astype(float)
            rank_corr.append(np.corrcoef(rj, rd)[0, 1])
    P["late_wave_share"] = float(np.mean(late))
    P["early_wave_ms_p10_p50_p90_max"] = [round(float(x), 2) for x in np.mean(early_d, axis=0)]
    P["late_wave_ms_mean"] = float(np.mean(late_d)) if late_d else 0.0
    P["late_wave_start_ms_mean"] = float(np.mean(late_s)) if late_s else 0.0
    P["last_early_wave_end_ms"] = float(np.mean(end_early))
    P["last_wave_end_ms"] = float(np.mean(end_all))
    P["job_order_vs_duration_rank_corr"] = float(np.mean(rank_corr)) if rank_corr else 0.0
    # resident waves of the launch itself and of all DP launches at 5 % steps
    # of each launch's length, averaged over launches
    own_prof, all_prof = [], []
    for ix in launches:
        s0, e1 = t0[ix].min(), t1[ix].max()
        pts = s0 + (np.arange(21) / 20.0 * (e1 - s0)).astype(np.int64)
        pts[-1] -= 1
        own_prof.append([int(((t0[ix] <= p) & (t1[ix] > p)).sum()) for p in pts])
        k = np.searchsorted(times, pts, side="right") - 1
        all_prof.append(level[np.clip(k, 0, len(level) - 1)])
    P["own_resident_at_5pct_steps"] = [int(x) for x in np.mean(own_prof, axis=0)]
    P["all_dp_resident_at_5pct_steps"] = [int(x) for x in np.mean(all_prof, axis=0)]
    # what predicts a job's duration (wave 0 of each job, which ends with the
    # traceback): rank correlations within each launch, averaged
    def rank(x):
        return np.argsort(np.argsort(x, kind="stable"), kind="stable").astype(float)

    pred = collections.defaultdict(list)
    for ix in launches:
        w0 = ix[(a[ix, 2] & np.uint64(0xFF)) == 0]
        if len(w0) < 16:
            continue
        du = (t1[w0] - t0[w0]).astype(float)
        V = a[w0, 4].astype(float)
        L = a[w0, 5].astype(float)
        rows = a[w0, 6].astype(float)
        job = (a[w0, 2] >> np.uint64(32)).astype(float)
        start = (t0[w0] - t0[ix].min()).astype(float)
        early = start < 1e5  # started within 1 ms of the launch
        feats = {"computed_strip_rows": rows, "sweep_rows": V * np.ceil((L + 1) / 64.0), "graph_rows": V,
                 "read_len": L, "minus_job_index": -job}
        for k, f in feats.items():
            m = early
            if m.sum() > 16 and np.std(f[m]) > 0:
                pred[k].append(np.corrcoef(rank(f[m]), rank(du[m]))[0, 1])
    P["duration_rank_corr_early_jobs"] = {k: round(float(np.mean(v)), 3) for k, v in pred.items()}
    # how much of the DP busy time two launches overlap
    iv = sorted((t0[ix].min(), t1[ix].max()) for ix in launches)
    ev2 = sorted([(s, 1) for s, _ in iv] + [(e, -1) for _, e in iv])
    lvl, last_t, acc = 0, None, collections.Counter()
    for tt, dd in ev2:
        if last_t is not None:
            acc[lvl] += tt - last_t
        lvl += dd
        last_t = tt
    tot = sum(v for k, v in acc.items() if k > 0)
    P["busy_share_by_concurrent_launches"] = {str(k): round(v / tot, 4) for k, v in sorted(acc.items()) if k > 0}
    out = {
        "records": int(len(a)), "launches": len(launches),
        "dp_busy_ms": float(busy / 1e5),
        "mean_resident_waves_over_busy": float(wave_ticks / busy),
        "mean_resident_over_slots": float(wave_ticks / busy / slots),
        "busy_time_share_by_occupancy": hist,
        "per_launch_means": P,
        "slots": slots,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
