"""Deterministic synthetic candidate windows.

Produces rows in the reference's localGraph_npz bundle format
``[sequenceList, ReadIDs, flank_5, flank_3, TDRecord]``
(/root/reference/src/SomTDDetector_AimDatFetch.py:107-123, consumed by
SVscope.py:209-220): sequenceList = [reference row] + reads (tumor reads
first, as DataMaker orders its BAM list), ReadIDs "<Sample>_<tag>|<qname>".

Window w uses RandomState(20250509 + w):
  * reference row: uniform ACGT, length R, flanks = first/last `offset` bp;
  * germline haplotype = reference; somatic haplotype = reference with a
    200-800 bp random insertion (even w) or a 100-600 bp deletion (odd w) at
    the centre;
  * N/2 normal reads (germline); N/2 tumor reads of which ceil(N/4) are
    somatic, the rest germline; every read spans flank+core+flank;
  * ONT-like error, 8 % per base: 3.5 % substitution, 2.5 % deletion, 2 %
    insertion (insertion rate doubled inside homopolymer runs, where the
    inserted base repeats the run); read i uses RandomState(seed*1000+i)
    (mod 2**32).
"""
import numpy as np

_ALPHA = np.frombuffer(b"ACGT", dtype=np.uint8)

CONFIGS = {
    1: dict(n_windows=1, n_reads=16, ref_len=2000),
    2: dict(n_windows=1000, n_reads=32, ref_len=2000),
    3: dict(n_windows=10000, n_reads=64, ref_len=3000),
}


def _mutate(hap, rs, p_sub=0.035, p_del=0.025, p_ins=0.02):
    n = hap.shape[0]
    u = rs.random_sample(n)
    keep = u >= p_del
    sub = keep & (u < p_del + p_sub)
    bases = hap.copy()
    if sub.any():
        bases[sub] = (bases[sub] + rs.randint(1, 4, size=int(sub.sum()))) % 4
    homo = np.zeros(n, dtype=bool)
    if n > 1:
        eq = hap[1:] == hap[:-1]
        homo[1:] |= eq
        homo[:-1] |= eq
    # mean insertion rate ~p_ins with homopolymer positions at 2x the others
    frac_h = homo.mean() if n else 0.0
    base_rate = p_ins / (1.0 + frac_h)
    rate = np.where(homo, 2 * base_rate, base_rate)
    ins = rs.random_sample(n) < rate
    ins_base = np.where(homo, bases, rs.randint(0, 4, size=n))
    counts = keep.astype(np.int64) + ins.astype(np.int64)
    out = np.empty(int(counts.sum()), dtype=np.int64)
    ends = np.cumsum(counts)
    starts = ends - counts
    out[starts[keep]] = bases[keep]
    ins_pos = np.where(ins)[0]
    out[ends[ins_pos] - 1] = ins_base[ins_pos]
    return out


def _mutated_len(hap, rs, p_sub=0.035, p_del=0.025, p_ins=0.02):
    """len(_mutate(hap, rs, ...)) with the same random draws, without building
    the read."""
    n = hap.shape[0]
    u = rs.random_sample(n)
    keep = u >= p_del
    n_sub = int((keep & (u < p_del + p_sub)).sum())
    if n_sub:
        rs.randint(1, 4, size=n_sub)
    homo = np.zeros(n, dtype=bool)
    if n > 1:
        eq = hap[1:] == hap[:-1]
        homo[1:] |= eq
        homo[:-1] |= eq
    frac_h = homo.mean() if n else 0.0
    base_rate = p_ins / (1.0 + frac_h)
    ins = rs.random_sample(n) < np.where(homo, 2 * base_rate, base_rate)
    return int(keep.sum()) + int(ins.sum())


def _to_str(codes):
    return _ALPHA[codes].tobytes().decode("ascii")


def make_window(w, n_reads, ref_len, offset=50, chrom="chrS", sample_t="T1", sample_n="N1", error=0.08,
                ins_range=(200, 801)):
    """One window; ``error`` scales the 8 % ONT profile (3.5/2.5/2 % sub/del/
    ins), ``ins_range`` the somatic insertion length (the defaults are §8(d)'s
    profile; other values give the harsher probes of tools/prune_probe.py)."""
    seed = (20250509 + w) % (2 ** 32)
    rs = np.random.RandomState(seed)
    ref = rs.randint(0, 4, size=ref_len)
    mid = ref_len // 2
    k = error / 0.08
    mut = {} if error == 0.08 else dict(p_sub=0.035 * k, p_del=0.025 * k, p_ins=0.02 * k)
    if w % 2 == 0:
        ins_len = int(rs.randint(*ins_range))
        som = np.concatenate([ref[:mid], rs.randint(0, 4, size=ins_len), ref[mid:]])
    else:
        del_len = int(rs.randint(100, 601))
        del_len = min(del_len, max(0, ref_len - 2 * offset - 2))
        a = mid - del_len // 2
        som = np.concatenate([ref[:a], ref[a + del_len:]])
    n_normal = n_reads // 2
    n_tumor = n_reads - n_normal
    n_som = min(n_tumor, -(-n_reads // 4))
    reads, ids = [], []
    for i in range(n_tumor):
        hap = som if i < n_som else ref
        rrs = np.random.RandomState((seed * 1000 + i) % (2 ** 32))
        reads.append(_to_str(_mutate(hap, rrs, **mut)))
        ids.append(f"{sample_t}_tumor|w{w}_r{i}")
    for i in range(n_tumor, n_reads):
        rrs = np.random.RandomState((seed * 1000 + i) % (2 ** 32))
        reads.append(_to_str(_mutate(ref, rrs, **mut)))
        ids.append(f"{sample_n}_normal|w{w}_r{i}")
    ref_s = _to_str(ref)
    record = f"{window_key(w, ref_len, offset, chrom)}\t{n_tumor}"
    return [[ref_s] + reads, np.array(ids), ref_s[:offset], ref_s[ref_len - offset:], record]


def window_lengths(w, n_reads, ref_len, offset=50):
    """[len(s) for s in make_window(w, n_reads, ref_len)[0]] at the default
    error profile, from the same random draws but without building the reads
    (about 2/3 of make_window's time; bench.py deals windows by these)."""
    seed = (20250509 + w) % (2 ** 32)
    rs = np.random.RandomState(seed)
    ref = rs.randint(0, 4, size=ref_len)
    mid = ref_len // 2
    if w % 2 == 0:
        ins_len = int(rs.randint(200, 801))
        som = np.concatenate([ref[:mid], rs.randint(0, 4, size=ins_len), ref[mid:]])
    else:
        del_len = min(int(rs.randint(100, 601)), max(0, ref_len - 2 * offset - 2))
        a = mid - del_len // 2
        som = np.concatenate([ref[:a], ref[a + del_len:]])
    n_tumor = n_reads - n_reads // 2
    n_som = min(n_tumor, -(-n_reads // 4))
    lens = [ref_len]
    for i in range(n_reads):
        hap = som if i < n_som else ref
        lens.append(_mutated_len(hap, np.random.RandomState((seed * 1000 + i) % (2 ** 32))))
    return lens


def window_key(w, ref_len, offset=50, chrom="chrS"):
    """chrom, start, end of window w's TDRecord, tab-separated: the first three
    fields of its Raw.bed record (what local_graph.window_key reads back)."""
    start = 1_000_000 + w * 10_000 + offset
    return f"{chrom}\t{start}\t{start + ref_len - 2 * offset}"


def make_windows(config=None, n_windows=None, n_reads=None, ref_len=None, start=0, offset=50):
    if config is not None:
        c = CONFIGS[config]
        n_windows = c["n_windows"] if n_windows is None else n_windows
        n_reads = c["n_reads"] if n_reads is None else n_reads
        ref_len = c["ref_len"] if ref_len is None else ref_len
    return [make_window(w, n_reads, ref_len, offset=offset) for w in range(start, start + n_windows)]


def save_npz(path, windows):
    """Writes a localGraph_npz bundle (object array under key 'DatSet')."""
    arr = np.empty(len(windows), dtype=object)
    for k, row in enumerate(windows):
        arr[k] = np.array(row, dtype=object)
    np.savez(path, DatSet=arr)
