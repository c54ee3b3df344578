"""Per-window somatic/germline decision, batched for the GPU.

``Decision(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, windowFlag='NormalOutput',
Tlabel='tumor', readcutoff=3, hcutoff=3, scutoff=0.05) -> list[10]`` keeps the
signature, gate, labelling and record format of
/root/reference/src/DecisionMaker.py:110-191:
  gate :134 -> MSAFeatureSelection :136 -> EMCluster if >= 10 features :137-138
  -> per-cluster somatic/germline test in ascending label order :145-154
  -> POA consensus per reported cluster :155-176 -> record :178-190.
``DecisionBatch(windows, ...)`` runs the same logic for many windows with one
batched GPU POA for all window MSAs, one batched GPU EM, and one batched GPU
POA for all cluster consensus sequences.
"""
import time

import numpy as np

from .data_scanner import SeqDecoder, msa_feature_selection_batch
from .poa import poa_batch
from .reads_cluster import em_cluster_batch


def _tag(read_id):
    return read_id.split("|")[0].split("_")[-1]


def DecisionBatch(windows, Tlabel="tumor", readcutoff=3, hcutoff=3, scutoff=0.05, context=None, stats=None):
    """windows: list of (TDRecord, sequenceList, ReadIDs, flank_5, flank_3[, windowFlag]).
    Returns the list of 10-field records, in input order."""
    t_start = time.perf_counter()
    phase = {}
    records = []
    gated = []
    for w, win in enumerate(windows):
        rec, seqs, ids, f5, f3 = win[:5]
        flag = win[5] if len(win) > 5 else "NormalOutput"
        chrom, start, end = rec.strip().split("\t")[0:3]
        records.append([chrom, start, end, "-", "-", 0, "-", "-", 0, flag])
        if len(ids):
            tags, counts = np.unique(np.array([_tag(x) for x in ids]), return_counts=True)
        else:
            tags, counts = np.array([]), np.array([])
        if len(seqs) > 3 and tags.shape[0] >= 2 and np.min(counts) >= 3:
            gated.append(w)
    if not gated:
        return records
    t0 = time.perf_counter()
    feats = msa_feature_selection_batch([(windows[w][1], windows[w][3], windows[w][4], np.asarray(windows[w][2]))
                                         for w in gated], hcutoff, scutoff, context=context, stats=stats)
    phase["msa_and_features_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    em_idx = [k for k, (_, feat, _) in enumerate(feats) if feat.shape[0] != 0 and feat.shape[1] >= 10]
    ems = em_cluster_batch([feats[k][1] for k in em_idx], context=context, timing=phase) if em_idx else []
    phase["em_total_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    # cluster labelling (ascending label order, DecisionMaker.py:145-154)
    plans = []
    jobs = []
    for k, em in zip(em_idx, ems):
        encoded, _, ids = feats[k]
        ids = np.asarray(ids)
        labels = em["Rclust"]
        som, germ = [], []
        for L in np.unique(labels):
            idx = np.where(labels == L)[0]
            types = np.unique([_tag(x) for x in ids[idx]])
            if types.shape[0] == 1 and types[0] == Tlabel and idx.shape[0] >= readcutoff:
                som.append(idx)
            elif idx.shape[0] >= readcutoff:
                germ.append(idx)
        entry = dict(w=gated[k], ids=ids, som=som, germ=germ, som_job=[], germ_job=[])
        for kind in ("som", "germ"):
            for idx in entry[kind]:
                rows = [SeqDecoder(r) for r in encoded[idx + 1]]
                if max(len(x) for x in rows) > 0:
                    entry[kind + "_job"].append(len(jobs))
                    jobs.append(rows)
                else:
                    entry[kind + "_job"].append(None)
        plans.append(entry)
    phase["labelling_s"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    cons = []
    if jobs:
        res = poa_batch(jobs, algorithm=1, genmsa=False, context=context, return_stats=stats is not None)
        if stats is not None:
            res, st = res
            stats.append(("consensus_poa", st))
        cons = [c for c, _ in res]
    phase["consensus_s"] = time.perf_counter() - t0
    for p in plans:
        som_seq = [cons[j] if j is not None else "-" for j in p["som_job"]]
        germ_seq = [cons[j] if j is not None else "-" for j in p["germ_job"]]
        if len(som_seq) > 0 and len(p["germ"]) > 0:
            r = records[p["w"]]
            r[3] = ";".join(som_seq)
            r[4] = ";".join(",".join(list(p["ids"][i])) for i in p["som"])
            r[5] = len(som_seq)
            r[6] = ";".join(germ_seq)
            r[7] = ";".join(",".join(list(p["ids"][i])) for i in p["germ"])
            r[8] = len(germ_seq)
            r[9] = r[9] + "|EMOutput"
    if stats is not None:
        phase["decision_total_s"] = time.perf_counter() - t_start
        stats.append(("phases", phase))
    return records


def Decision(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, windowFlag="NormalOutput", Tlabel="tumor",
             readcutoff=3, hcutoff=3, scutoff=0.05):
    return DecisionBatch([(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, windowFlag)], Tlabel, readcutoff,
                         hcutoff, scutoff)[0]
