"""Per-window drivers with the reference signatures
(/root/reference/src/SomTDDetector.py:26-73).

``TDscope_npz(TDRecord, sequenceList, ReadIDs, flank_5, flank_3)`` -> Decision.
``TDscope(TDRecord, DataMaker, DataMaker2, DecisionMaker)`` keeps the DUP
corner re-scan branch (:41-58); DataMaker/DataMaker2 are the caller's
BAM readers (pysam, out of scope here) bound with functools.partial exactly as
SVscope.py:152-154 does, so both stay picklable.
``TDscope_npz_batch(rows)`` is the batched form used by localGraph_npz, and
``TDscope_batch(records, DataMaker, DataMaker2)`` the batched form of TDscope
used by localGraph (svscope_amd/data_maker.py holds the readers).
"""
import logging
import re
import time

import numpy as np

from .decision_maker import Decision, DecisionBatch, WindowFailed

log = logging.getLogger("svscope_amd")


def TDscope(TDRecord, DataMaker, DataMaker2, DecisionMaker):
    start_time = time.time()
    sequenceList, ReadIDs, flank_5, flank_3, TDRecord, flag = DataMaker(TDRecord)
    SVType = TDRecord.strip().split("\t")[3].split(",")[0]
    Record = DecisionMaker(TDRecord, sequenceList, ReadIDs, flank_5, flank_3, flag)
    if (Record[-1].split("|")[-1] != "EMOutput") and (SVType == "DUP"):
        reSCANDat = DataMaker2(TDRecord)
        sequenceList_5, ReadIDs_5, flank_5_5, flank_3_5, TDRecord, flag5 = reSCANDat[0]
        sequenceList_3, ReadIDs_3, flank_5_3, flank_3_3, TDRecord, flag3 = reSCANDat[1]
        Record5 = DecisionMaker(TDRecord, sequenceList_5, ReadIDs_5, flank_5_5, flank_3_5, flag5)
        if Record5[-1].split("|")[-1] == "EMOutput":
            Record = Record5
        else:
            Record3 = DecisionMaker(TDRecord, sequenceList_3, ReadIDs_3, flank_5_3, flank_3_3, flag3)
            if Record3[-1].split("|")[-1] == "EMOutput":
                Record = Record3
            elif len([x for x in np.setdiff1d(ReadIDs_5, ReadIDs) if re.search("_tumor", x)]) >= 3:
                Record[-1] = flag5
            elif len([x for x in np.setdiff1d(ReadIDs_3, ReadIDs) if re.search("_tumor", x)]) >= 3:
                Record[-1] = flag3
    log.info("pipeline for region %s finished Take %ss", TDRecord, time.time() - start_time)
    return Record


def _emoutput(rec):
    return rec[-1].split("|")[-1] == "EMOutput"


def TDscope_batch(TDRecords, DataMaker, DataMaker2, map_fn=map, context=None, Tlabel="tumor", readcutoff=3,
                  hcutoff=3, scutoff=0.05, bundles=None):
    """TDscope over many windows, each Decision round batched on the GPU.

    Same records as ``[TDscope(r, DataMaker, DataMaker2, Decision) for r in
    TDRecords]`` (SomTDDetector.py:26-61): DataMaker for every window
    (through ``map_fn``, e.g. a process pool's map, since it is BAM I/O),
    one DecisionBatch for all of them, then for the DUP windows without an
    EMOutput one DataMaker2 each, one DecisionBatch for their 5' corners, one
    for the 3' corners of those still without, and the flag rewrite of
    :55-58.  ``bundles``, if given, is the precomputed DataMaker output.

    A window past an engine limit in any of its Decision rounds fails alone:
    the other windows' records are completed, then one WindowFailed carries
    them (None for the failed windows) and the failed indices."""
    data = list(bundles) if bundles is not None else list(map_fn(DataMaker, TDRecords))
    kw = dict(Tlabel=Tlabel, readcutoff=readcutoff, hcutoff=hcutoff, scutoff=scutoff, context=context)
    failed = {}

    def batch(windows, owners):
        # one Decision round; a failed window's owner (an index into data) fails
        try:
            return DecisionBatch(windows, **kw)
        except WindowFailed as e:
            for j, why in e.failed.items():
                failed.setdefault(owners[j], why)
            return e.records

    # the window record's column 4 (IndexError on a 3-column record, as :39)
    sv_types = [d[4].strip().split("\t")[3].split(",")[0] for d in data]
    records = batch([(d[4], d[0], d[1], d[2], d[3], d[5]) for d in data], list(range(len(data))))
    dup = [i for i, rec in enumerate(records) if rec is not None and not _emoutput(rec) and sv_types[i] == "DUP"]
    if dup:
        rescans = list(map_fn(DataMaker2, [data[i][4] for i in dup]))
        rec5 = batch([tuple(r[0][k] for k in (4, 0, 1, 2, 3, 5)) for r in rescans], dup)
        left = [j for j in range(len(dup)) if rec5[j] is not None and not _emoutput(rec5[j])]
        rec3 = batch([tuple(rescans[j][1][k] for k in (4, 0, 1, 2, 3, 5)) for j in left], [dup[j] for j in left])
        rec3 = dict(zip(left, rec3))
        for j, i in enumerate(dup):
            if i in failed:
                continue
            c5, c3 = rescans[j]
            if _emoutput(rec5[j]):
                records[i] = rec5[j]
            elif _emoutput(rec3[j]):
                records[i] = rec3[j]
            elif len([x for x in np.setdiff1d(c5[1], data[i][1]) if re.search("_tumor", x)]) >= 3:
                records[i][-1] = c5[5]
            elif len([x for x in np.setdiff1d(c3[1], data[i][1]) if re.search("_tumor", x)]) >= 3:
                records[i][-1] = c3[5]
    if failed:
        for i in failed:
            records[i] = None
        raise WindowFailed(failed, records)
    return records


def TDscope_npz(TDRecord, sequenceList, ReadIDs, flank_5, flank_3):
    return Decision(TDRecord, sequenceList, ReadIDs, flank_5, flank_3)


def TDscope_npz_batch(rows, context=None, stats=None):
    """rows: [sequenceList, ReadIDs, flank_5, flank_3, TDRecord] bundle rows
    (SomTDDetector_AimDatFetch.py:118, read back at SVscope.py:212)."""
    return DecisionBatch([(r[4], list(r[0]), np.asarray(r[1]), r[2], r[3]) for r in rows], context=context,
                         stats=stats)
