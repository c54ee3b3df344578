"""Per-window drivers with the reference signatures
(/root/reference/src/SomTDDetector.py:26-73).

``TDscope_npz(TDRecord, sequenceList, ReadIDs, flank_5, flank_3)`` -> Decision.
``TDscope(TDRecord, DataMaker, DataMaker2, DecisionMaker)`` keeps the DUP
corner re-scan branch (:41-58); DataMaker/DataMaker2 are the caller's
BAM readers (pysam, out of scope here) bound with functools.partial exactly as
SVscope.py:152-154 does, so both stay picklable.
``TDscope_npz_batch(rows)`` is the batched form used by localGraph_npz.
"""
import logging
import re
import time

import numpy as np

from .decision_maker import Decision, DecisionBatch

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


def TDscope_npz(TDRecord, sequenceList, ReadIDs, flank_5, flank_3):
    return Decision(TDRecord, sequenceList, ReadIDs, flank_5, flank_3)


def TDscope_npz_batch(rows, context=None, stats=None):
    """rows: [sequenceList, ReadIDs, flank_5, flank_3, TDRecord] bundle rows
    (SomTDDetector_AimDatFetch.py:118, read back at SVscope.py:212)."""
    return DecisionBatch([(r[4], list(r[0]), np.asarray(r[1]), r[2], r[3]) for r in rows], context=context,
                         stats=stats)
