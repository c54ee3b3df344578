"""AlnFeature: the CPU tail after localGraph.

Turns Raw.bed into the somatic VCF, with the reference's functions, file
names and columns:

  OVLEN / windowInfo / background   /root/reference/src/DataScanner.py:413-481
  makeupDB / query_reads / spanchrRatio                          :328-410
  AlnFeature                        /root/reference/src/SVscope.py:241-339
  generate_vcfheader / bed2vcf      /root/reference/src/OutVCF.py:17-77

MisScore (the only arithmetic of any size here) runs on the GPU through
pairwise_compare.MisScorePipe.  Everything else is table work on the host.

Two hooks replace what this image cannot run:
  * ``readers.tabix(path)`` -> an object with ``fetch(chrom=None, start=None,
    end=None)`` yielding bed lines (pysam.TabixFile by default: pysam is not
    installed here, so the default fails loudly at the first window);
  * ``model``: the random forest, any object with ``predict_proba`` and
    ``predict`` over the ten feature columns.  The reference unpickles its
    model file (src/RandomForest.1218.WholeData8-2.FinalModel.joblib); this
    build never deserialises pickles, so the caller supplies the model object.
The BAM -> bed.gz step is bedtools | bgzip && tabix, run as the reference
runs it, only when the bed.gz files are missing.
"""
import functools
import logging
import os
import re
import sqlite3
import subprocess
import time
from concurrent.futures import ProcessPoolExecutor

import numpy as np

log = logging.getLogger("svscope_amd")


class PysamTabix:
    def tabix(self, path):
        import pysam  # absent in this image: raises here
        return pysam.TabixFile(path)


DEFAULT_READERS = PysamTabix()


# ------------------------------------------------------------- alignment DB
def makeupDB(bed_file, dbName, batchsize=500000, readers=None):
    """bed.gz alignments -> sqlite (DataScanner.py:328-389)."""
    readers = readers or DEFAULT_READERS
    conn = sqlite3.connect("%s.sqlite" % dbName)
    cur = conn.cursor()
    cur.execute("CREATE TABLE IF NOT EXISTS reads_length (read_id TEXT PRIMARY KEY, length INTEGER)")
    cur.execute("CREATE TABLE IF NOT EXISTS reads_alignment (id INTEGER PRIMARY KEY, read_id TEXT, chrom TEXT, "
                "start INTEGER, end INTEGER, mapQ INTEGER, strand TEXT, "
                "FOREIGN KEY (read_id) REFERENCES reads_length (read_id))")
    cur.execute("CREATE INDEX IF NOT EXISTS idx_read_id ON reads_alignment (read_id)")
    cur.execute("CREATE INDEX IF NOT EXISTS idx_read_id ON reads_length (read_id)")
    conn.commit()
    ins = "INSERT INTO reads_alignment (read_id, chrom, start, end, mapQ, strand) VALUES (?, ?, ?, ?, ?, ?)"
    for bedF in bed_file.split(","):
        batch = []
        for row in readers.tabix(bedF).fetch():
            f = row.split("\t")
            batch.append((f[3], f[0], int(f[1]), int(f[2]), f[4], f[5]))
            if len(batch) >= batchsize:
                cur.executemany(ins, batch)
                conn.commit()
                batch = []
        if batch:
            cur.executemany(ins, batch)
            conn.commit()
    cur.close()
    conn.close()
    return "%s.sqlite" % dbName


def query_reads(dbFile, read_id):
    conn = sqlite3.connect(dbFile)
    cur = conn.cursor()
    cur.execute("SELECT * FROM reads_alignment WHERE read_id = ?", (read_id,))
    out = cur.fetchall()
    cur.close()
    conn.close()
    return out


def spanchrRatio(readIDList, dbFile):
    """Fraction of reads whose alignments touch more than one chromosome
    (DataScanner.py:403-410)."""
    if not readIDList:
        raise ValueError("need at least one array to concatenate")  # np.vstack([]) in the reference
    chroms = {}
    for rid in readIDList:
        rows = query_reads(dbFile, rid.split("|")[-1])
        if not rows:
            # np.vstack of an empty result beside (n, 7) rows (or alone, then a
            # 7-column frame over a (1, 0) array) raises in the reference
            raise ValueError("read %s has no alignment in %s" % (rid, dbFile))
        for row in rows:
            chroms.setdefault(row[1], set()).add(row[2])
    return sum(1 for c in chroms.values() if len(c) != 1) / len(chroms)


# --------------------------------------------------------------- background
def OVLEN(window, start, end):
    """Overlap of an alignment with a window (DataScanner.py:413-425, its
    four cases; the remaining boundary cases give 0 as there)."""
    ws, we = (int(x) for x in window.strip().split("\t")[1:3])
    if start <= ws and end >= we:
        return we - ws
    if start > ws and end < we:
        return end - start
    if start > ws and end > we:
        return we - start
    if start < ws and end < we:
        return end - ws
    return 0


def windowInfo(window, bed_file, dbFile, mapQcutoff=5, showchromSpan=False, showmapQ=False, readers=None):
    """[window, COV, mapQRate(, chromSpan, read ids)] (DataScanner.py:427-467):
    per read the first chrom/strand, min start, max end, min mapQ."""
    readers = readers or DEFAULT_READERS
    chrom, start, end = window.strip().split("\t")[0:3]
    window_write = chrom + "_" + start + "_" + end
    wlen = int(end) - int(start)
    per_read = {}
    for bedfile in bed_file.split(","):
        for line in readers.tabix(bedfile).fetch(chrom, int(start), int(end)):
            f = line.strip().split("\t")[0:6]
            rid, s, e, mq = f[3], int(f[1]), int(f[2]), int(f[4])
            if rid in per_read:
                r = per_read[rid]
                per_read[rid] = [r[0], min(r[1], s), max(r[2], e), min(r[3], mq), r[4]]
            else:
                per_read[rid] = [f[0], s, e, mq, f[5]]
    if per_read:
        ids = sorted(per_read)  # groupby order
        cov = sum(OVLEN(window, per_read[r][1], per_read[r][2]) for r in ids) / wlen
        mapq_rate = sum(1 for r in ids if per_read[r][3] < mapQcutoff) / len(ids)
        if showchromSpan:
            return [window_write, cov, mapq_rate, spanchrRatio(ids, dbFile), ",".join(ids)]
        return [window_write, cov, mapq_rate]
    if showchromSpan:
        return [window_write, np.nan, np.nan, np.nan, ""]
    return [window_write, np.nan, np.nan]


def background(windowFile, bed_file, dbFile, showchromSpan=False, workthread=100, readers=None):
    """windowInfo over every window of a file (EMOutput rows only when
    showchromSpan), as a DataFrame (DataScanner.py:469-481)."""
    import pandas as pd
    with open(windowFile) as fh:
        windows = fh.readlines()
    if showchromSpan:
        windows = [x for x in windows if re.search(r"EMOutput", x)]
    fn = functools.partial(windowInfo, bed_file=bed_file, dbFile=dbFile, showchromSpan=showchromSpan,
                           readers=readers)
    if int(workthread) > 1:
        with ProcessPoolExecutor(max_workers=int(workthread)) as ex:
            bg = list(ex.map(fn, windows))
    else:
        bg = [fn(w) for w in windows]
    cols = ["window", "COV", "mapQRate"] + (["chromSpan", "TotalReadID"] if showchromSpan else [])
    return pd.DataFrame(bg, columns=cols)


# ------------------------------------------------------------------- VCF
def parse_fasta(fai):
    chromosomes = {}
    with open(fai) as fh:
        for line in fh:
            f = line.split("\t")
            chromosomes[f[0]] = f[1]
    return chromosomes


def generate_vcfheader(chromosomes, out_vcf, fasta):
    """OutVCF.py:17-36 (same lines, same order)."""
    info = ("##INFO=<ID=SVTYPE,Number=1,Type=String,Description=\"Type of structural variant\">\n"
            "##INFO=<ID=SVLEN,Number=1,Type=Integer,Description=\"Length of the SV\">\n"
            "##INFO=<ID=END,Number=1,Type=Integer,Description=\"End position of the SV\">\n"
            "##INFO=<ID=SUPPORT,Number=1,Type=Integer,Description=\"Number of reads supporting the structural "
            "variation\">\n"
            "##INFO=<ID=RNAMES,Number=.,Type=String,Description=\"Names of supporting reads\">\n"
            "##INFO=<ID=AF,Number=1,Type=Float,Description=\"Allele Frequency\">\n")
    with open(out_vcf, "w") as vcf:
        vcf.write("##fileformat=VCFv4.2\n##source=TDscope.1.0\n"
                  "##FILTER=<ID=PASS,Description=\"All filters passed\">\n")
        vcf.write("##fileDate=\"" + time.strftime("%Y/%m/%d %H:%M:%S", time.localtime()) + "\"\n")
        vcf.write("##reference=" + fasta + "\n")
        for chrom, length in chromosomes.items():
            vcf.write("##contig=<ID=" + chrom + ",length=" + length + ">\n")
        vcf.write("##ALT=<ID=INS,Description=\"Insertion\">\n##ALT=<ID=DEL,Description=\"Deletion\">\n")
        vcf.write("##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n")
        vcf.write(info)
    return out_vcf


def sv_type(svlen):
    """INS at SVLEN >= 50, DEL at <= -50, otherwise MisAlign (OutVCF.py:63-67)."""
    return "INS" if svlen >= 50 else ("DEL" if svlen <= -50 else "MisAlign")


def bed2vcf(input_bed1, input_bed2, input_bed3, out_vcf, TumorID, reference):
    """Raw.bed + Somatic.bed + RandomForestResult.tsv -> VCF (OutVCF.py:38-77)."""
    import pandas as pd
    raw = pd.read_csv(input_bed1, sep="\t", header=None).drop_duplicates()
    raw.index = raw[0] + "_" + raw[1].apply(str) + "-" + raw[2].apply(str)
    som = pd.read_csv(input_bed2, sep="\t", header=None).drop_duplicates()
    som.index = som[3]
    model = pd.read_csv(input_bed3, sep="\t", index_col=0)
    generate_vcfheader(parse_fasta("%s.fai" % reference), out_vcf, reference)
    with open(out_vcf, "a") as vcf:
        vcf.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t{}\n".format(TumorID))
        for w in model.index:
            r = list(raw.loc[w])
            s = list(som.loc[w])
            support = s[4].split(";")[0]
            svlen = int(s[-3])
            t = sv_type(svlen)
            info = "SVLEN={};SVTYPE={};END={};SUPPORT={};RNAMES={};AF={};ConfidenceSV={};DecisionSV={}".format(
                svlen, t, r[2], len(support.split(",")), support, s[-2], model.loc[w, "yprob"], model.loc[w, "y_hat"])
            vcf.write("\t".join([r[0], str(r[1]), "TDscope." + t + "." + w, ",".join(r[6].split(";")),
                                 ",".join(r[3].split(";")), ".", "PASS", info, "GT", "0/1\n"]))
    return out_vcf


# ------------------------------------------------------------- features
def _window_key(x):
    return "_".join(x.split("_")[:2]) + "-" + x.split("_")[-1]


def _read_names(cell):
    return [a.split("|")[-1] for a in ",".join(cell.split(";")).split(",")]


FEATURES = ["COV_Tumor", "mapQ_Tumor", "COV_Normal", "mapQ_Normal", "ABSMisScore", "chromSpan_Tumor",
            "chromSpan_Normal", "AdaptRatio_T", "AdaptRatio_N", "SupportReadSpanRatio"]


def feature_table(bg_T, bg_N, sv_T, sv_N, somatic, raw_path, db_tumor):
    """The random forest's ten features per reported window (SVscope.py:270-307):
    coverage and mapQ z-scores against the genome background, chromosome-span
    rates, the fraction of each sample's usable reads that the window's
    clusters adopted, |MisScore| and the support reads' chromosome-span rate."""
    import pandas as pd
    sv_T, sv_N = sv_T.copy(), sv_N.copy()
    for sv, bg in ((sv_T, bg_T.dropna()), (sv_N, bg_N.dropna())):
        sv["COV_Zscore"] = (sv["COV"] - np.mean(bg["COV"])) / np.std(bg["COV"])
        sv["mapQ_Zscore"] = (sv["mapQRate"] - np.mean(bg["mapQRate"])) / np.std(bg["mapQRate"])
    sv_T = sv_T.drop_duplicates()
    sv_N = sv_N.drop_duplicates()
    sv_T.index = sv_T["window"].apply(_window_key)
    sv_N.index = sv_N["window"].apply(_window_key)
    raw = pd.read_csv(raw_path, header=None, sep="\t")
    raw.columns = ["chrom", "start", "end", "SomSeq", "SomReads", "SomCount", "GermSeq", "GermReads", "GermCount",
                   "Label"]
    rf = raw.loc[raw["Label"] == "NormalOutput|EMOutput"].drop_duplicates().copy()
    rf["window"] = rf["chrom"] + "_" + rf["start"].apply(str) + "-" + rf["end"].apply(str)
    rf.index = rf["window"]
    wl = np.intersect1d(somatic.index, rf.index)
    pool = pd.concat([sv_T.loc[wl, ["window", "COV_Zscore", "mapQ_Zscore", "chromSpan"]],
                      sv_N.loc[wl, ["COV_Zscore", "mapQ_Zscore", "chromSpan"]],
                      rf.loc[wl, "SomReads"],
                      rf.loc[wl, "SomReads"].apply(_read_names) + rf.loc[wl, "GermReads"].apply(_read_names),
                      sv_T.loc[wl, "TotalReadID"].apply(lambda x: x.split(",")),
                      sv_T.loc[wl, "mapQRate"],
                      sv_N.loc[wl, "TotalReadID"].apply(lambda x: x.split(",")),
                      sv_N.loc[wl, "mapQRate"],
                      somatic.loc[wl, "ABSMisScore"]], axis=1)
    pool.columns = ["window", "COV_Tumor", "mapQ_Tumor", "chromSpan_Tumor", "COV_Normal", "mapQ_Normal",
                    "chromSpan_Normal", "SomReads", "AdaptReads", "TotalRead_T", "mapQRate_T", "TotalRead_N",
                    "mapQRate_N", "ABSMisScore"]

    def adapt(x, tot, rate):
        d = len(x[tot]) * (1 - x[rate])
        return np.intersect1d(x["AdaptReads"], x[tot]).shape[0] / d if d > 0 else 0

    pool["AdaptRatio_T"] = pool.apply(lambda x: adapt(x, "TotalRead_T", "mapQRate_T"), axis=1)
    pool["AdaptRatio_N"] = pool.apply(lambda x: adapt(x, "TotalRead_N", "mapQRate_N"), axis=1)
    pool["SupportReadSpanRatio"] = pool["SomReads"].apply(lambda x: spanchrRatio(_read_names(x), db_tumor))
    return pool


def merge_vcfs(savedir, out_vcf, tsid):
    """SVscope.py:321-338: header of out_vcf (INV/BND ALT lines before
    ##FORMAT), then its 'True' lines and InterALNSVs.vcf's records, sorted
    like sort -k1,1 -k2,2n."""
    from .local_graph import sort_lines
    merged = os.path.join(savedir, "%s.mergedSomatic.vcf" % "_".join(tsid))
    with open(out_vcf) as fh:
        lines = fh.readlines()
    body = [x for x in lines if "True" in x]
    inter = os.path.join(savedir, "InterALNSVs.vcf")
    if os.path.exists(inter):
        with open(inter) as fh:
            body += [x for x in fh if "#" not in x]
    with open(merged, "w") as out:
        for rec in (x for x in lines if "#" in x):
            if "##FORMAT" in rec:
                out.write("##ALT=<ID=INV,Description=\"Invasion\">\n##ALT=<ID=BND,Description=\"Translocation\">\n")
            out.write(rec)
        out.write("".join(line + "\n" for line in sort_lines([x.rstrip("\n") for x in body])))
    return merged


def AlnFeature(args, model, readers=None, context=None):
    """SVscope.py:241-339: alignment features, MisScore (GPU), the random
    forest and the VCFs.  Returns the merged VCF path; like the reference, it
    raises when fewer than two VCFs exist in savedir (its mergeVCF is unbound)."""
    from .pairwise_compare import MisScorePipe
    os.makedirs(args.savedir, exist_ok=True)
    tsid, nsid = args.TSampleID.split(","), args.NSampleID.split(",")
    tbed = ",".join(os.path.join(args.savedir, "%s.bed.gz" % t) for t in tsid)
    nbed = ",".join(os.path.join(args.savedir, "%s.bed.gz" % n) for n in nsid)
    for bams, beds in ((args.Tumorbam, tbed), (args.Normalbam, nbed)):
        if not os.path.exists(beds.split(",")[-1]):
            for bam, bed in zip(bams.split(","), beds.split(",")):
                subprocess.check_call("bedtools bamtobed -i {0} -cigar | bgzip > {1} && tabix {1}".format(bam, bed),
                                      shell=True)
    db_t = os.path.join(args.savedir, "Tumor") + ".sqlite"
    db_n = os.path.join(args.savedir, "Normal") + ".sqlite"
    if not os.path.exists(db_t):
        db_t = makeupDB(tbed, os.path.join(args.savedir, "Tumor"), readers=readers)
        db_n = makeupDB(nbed, os.path.join(args.savedir, "Normal"), readers=readers)
    th = int(args.thread)
    bg_T = background(args.genomeWindow, tbed, db_t, showchromSpan=False, workthread=th, readers=readers)
    bg_N = background(args.genomeWindow, nbed, db_n, showchromSpan=False, workthread=th, readers=readers)
    sv_T = background(args.rawBedFile, tbed, db_t, showchromSpan=True, workthread=th, readers=readers)
    sv_N = background(args.rawBedFile, nbed, db_n, showchromSpan=True, workthread=th, readers=readers)
    som = MisScorePipe(args.rawBedFile, context=context).drop_duplicates()
    som.index = som["chrom"] + "_" + som["start"].apply(str) + "-" + som["end"].apply(str)
    som["ABSMisScore"] = som["MisScore"].apply(np.abs)
    som_out = os.path.join(args.savedir, "%s.Somatic.bed" % args.TSampleID)
    som.to_csv(som_out, sep="\t", index=False, header=None)
    pool = feature_table(bg_T, bg_N, sv_T, sv_N, som, args.rawBedFile, db_t)
    X = pool[FEATURES]
    pool["yprob"] = model.predict_proba(X)[:, 1]
    pool["y_hat"] = model.predict(X)
    pool_out = os.path.join(args.savedir, "RandomForestResult.tsv")
    pool.to_csv(pool_out, sep="\t")
    out_vcf = os.path.join(args.savedir, "%s.vcf" % "_".join(tsid))
    bed2vcf(args.rawBedFile, som_out, pool_out, out_vcf, args.TSampleID, args.Reference)
    if len([x for x in os.listdir(args.savedir) if x.split(".")[-1] == "vcf"]) >= 2:
        return merge_vcfs(args.savedir, out_vcf, tsid)
    raise UnboundLocalError("local variable 'mergeVCF' referenced before assignment")
