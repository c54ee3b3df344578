"""ORACLE — test infrastructure only.  Never imported by the svscope_amd product.

Literal CPU restatement of the per-window decision logic, built on the CPU
POA oracle (spoa_oracle) and the numpy EM oracle (em_oracle):
  DataScanner.SeqEncoder / SeqDecoder     /root/reference/src/DataScanner.py:124-137
  DataScanner.CallMargin                  :146-165
  DataScanner.FindNonSameSite             :167-179
  DataScanner.MSAFeatureSelection         :181-220 (incl. the DEL-read id quirk :204)
  DecisionMaker.Decision                  /root/reference/src/DecisionMaker.py:110-191
  SomTDDetector.TDscope_npz               /root/reference/src/SomTDDetector.py:63-73
Pinned by tests/golden/decision_goldens.json (reference Decision run with this
package's POA oracle standing in for pyspoa; see gen_decision_goldens.py).
"""
import numpy as np

from . import em_oracle
from .spoa_oracle import poa

_ENC = {"A": 0, "T": 1, "C": 2, "G": 3, "-": 4}
_DEC = {0: "A", 1: "T", 2: "C", 3: "G", 4: "-"}


def seq_encoder(s):
    return np.array([_ENC[ch.upper()] for ch in s])


def seq_decoder(codes):
    return "".join(_DEC[c] for c in codes if c != 4)


def call_margin(msa, flank_5, flank_3):
    ex = msa[0]
    pool = []
    tmp = ""
    for i in range(len(ex)):
        if ex[i] != "-":
            tmp += ex[i]
            pool.append(i)
        if tmp == flank_5:
            break
    tmp = ""
    for i in range(len(ex) - 1, 0, -1):
        if ex[i] != "-":
            tmp = ex[i] + tmp
            pool.append(i)
        if tmp == flank_3:
            break
    return np.array(pool)


def find_non_same_site(M, cutoff=3):
    counts = np.zeros((5, M.shape[1]))
    for a in range(5):
        cols, cnt = np.unique(np.where(M == a)[1], return_counts=True)
        counts[a, cols] = cnt
    return np.where(np.sort(counts, axis=0)[-2] >= cutoff)[0]


def msa_feature_selection(seqs, flank_5, flank_3, read_ids, hcutoff=3, scutoff=0.05):
    read_ids = np.asarray(read_ids)
    lens = np.array([len(x) for x in seqs[1:]])
    dels = np.where(lens == 0)[0]
    if dels.shape[0] > 0:
        undel = np.setdiff1d(np.arange(len(read_ids)), dels)
        undel_ids = list(read_ids[undel])
        del_ids = list(read_ids[undel])  # reference quirk (DataScanner.py:204)
        _, unmsa = poa(seqs, 1)
        enc = [seq_encoder(r) for r in unmsa]
        width = len(enc[-1])
        read_ids = np.array(undel_ids + del_ids)
        encoded = np.array(enc + [[4] * width] * len(del_ids))
        msa = unmsa + [["-"] * width] * len(del_ids)
    else:
        _, msa = poa(seqs, 1)
        encoded = np.array([seq_encoder(r) for r in msa])
    pool = call_margin(msa, flank_5, flank_3)
    raw = encoded[1:, np.setdiff1d(np.arange(encoded.shape[1]), pool)]
    feat = raw[:, find_non_same_site(raw, cutoff=max([hcutoff, encoded.shape[0] * scutoff]))]
    return encoded, feat, read_ids


def _tag(x):
    return x.split("|")[0].split("_")[-1]


def decision(td_record, seqs, read_ids, flank_5, flank_3, window_flag="NormalOutput", tlabel="tumor",
             readcutoff=3, hcutoff=3, scutoff=0.05, em_result=None):
    chrom, start, end = td_record.strip().split("\t")[0:3]
    tags, tag_count = np.unique(np.array([_tag(x) for x in read_ids]), return_counts=True)
    record = [chrom, start, end, "-", "-", 0, "-", "-", 0, window_flag]
    if len(seqs) > 3 and tags.shape[0] >= 2 and np.min(tag_count) >= 3:
        encoded, feat, read_ids = msa_feature_selection(seqs, flank_5, flank_3, np.asarray(read_ids), hcutoff, scutoff)
        if feat.shape[0] != 0 and feat.shape[1] >= 10:
            em = em_result if em_result is not None else em_oracle.em_cluster(feat)
            labels = em["Rclust"]
            som_idx, som_seq, germ_idx, germ_seq = [], [], [], []
            for L in np.unique(labels):
                sub = np.array(read_ids)[np.where(labels == L)[0]]
                types = np.unique([_tag(x) for x in sub])
                idx = np.where(labels == L)[0]
                if types.shape[0] == 1 and types[0] == tlabel and sub.shape[0] >= readcutoff:
                    som_idx.append(idx)
                elif idx.shape[0] >= readcutoff:
                    germ_idx.append(idx)
            for idx in som_idx:
                rows = [seq_decoder(r) for r in encoded[idx + 1]]
                som_seq.append(poa(rows, 1)[0] if max(len(x) for x in rows) > 0 else "-")
            for idx in germ_idx:
                rows = [seq_decoder(r) for r in encoded[idx + 1]]
                germ_seq.append(poa(rows, 1)[0] if max(len(x) for x in rows) > 0 else "-")
            if len(som_seq) > 0 and len(germ_idx) > 0:
                ids = np.array(read_ids)
                record = [chrom, start, end, ";".join(som_seq),
                          ";".join(",".join(list(ids[i])) for i in som_idx), len(som_seq),
                          ";".join(germ_seq), ";".join(",".join(list(ids[i])) for i in germ_idx), len(germ_seq),
                          window_flag + "|EMOutput"]
    return record


def tdscope_npz(td_record, seqs, read_ids, flank_5, flank_3):
    return decision(td_record, seqs, read_ids, flank_5, flank_3)


def record_line(rec):
    return "\t".join(str(x) for x in rec)
