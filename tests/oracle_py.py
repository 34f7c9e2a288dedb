"""ctypes binding of the CPU oracle (oracle/tfbs_oracle.c) plus a small driver that
replays find-tfbs's ``run`` (main.rs:234-393) over decoded inputs.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product package.
"""
import ctypes as C
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libtfbs_oracle.so")

_lib = None

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
u8p = C.POINTER(C.c_uint8)
intp = C.POINTER(C.c_int)


def build():
    subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(
            os.path.join(ORACLE_DIR, "tfbs_oracle.c")
        ):
            build()
        L = C.CDLL(ORACLE_SO)
        L.orc_to_nucleotide.argtypes = [C.c_uint8]
        L.orc_range_overlaps.argtypes = [C.c_uint64] * 4
        L.orc_merge_ranges.argtypes = [u64p, u64p, C.c_int, u64p, u64p]
        L.orc_parse_weight.argtypes = [C.c_char_p, i32p]
        L.orc_parse_threshold_file.argtypes = [C.c_char_p, C.c_float, i32p]
        L.orc_patterns_new.restype = C.c_void_p
        L.orc_patterns_free.argtypes = [C.c_void_p]
        L.orc_patterns_count.argtypes = [C.c_void_p]
        L.orc_pattern_info.argtypes = [C.c_void_p, C.c_int, intp, intp, intp, i32p, intp]
        L.orc_pattern_weights.argtypes = [C.c_void_p, C.c_int]
        L.orc_pattern_weights.restype = i32p
        L.orc_pattern_name.argtypes = [C.c_void_p, C.c_int]
        L.orc_pattern_name.restype = C.c_char_p
        L.orc_parse_pwm_files.argtypes = [C.c_char_p, C.c_char_p, C.c_float, C.c_char_p, C.c_int, C.c_void_p]
        L.orc_patterns_add.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int32, C.c_int, i32p,
                                       C.c_char_p]
        L.orc_reverse_complement.argtypes = [i32p, C.c_int, i32p]
        L.orc_patch_haplotype.argtypes = [C.c_uint64, C.c_uint64, C.c_int, u64p, u8p, intp, u8p, intp, u8p, u64p,
                                          C.c_int, u8p, u64p, C.c_int]
        L.orc_matches.argtypes = [i32p, C.c_int, C.c_int32, C.c_int, u8p, u64p, C.c_int, u64p, u64p, C.c_int]
        L.orc_counts_as_genotypes.argtypes = [u32p, u32p, C.c_int, u32p, C.c_char_p, C.c_size_t, C.c_char_p,
                                              C.c_size_t]
        L.orc_count_matches_by_sample.restype = C.c_void_p
        L.orc_count_matches_by_sample.argtypes = [C.c_int, C.c_int, u64p, u64p, C.POINTER(C.c_uint16), intp, intp,
                                                  u32p, C.c_int, intp, u64p, u64p]
        L.orc_keys_count.argtypes = [C.c_void_p]
        L.orc_keys_get.argtypes = [C.c_void_p, C.c_int, intp, u64p, u64p, intp, u32p, u32p]
        L.orc_keys_free.argtypes = [C.c_void_p]
        L.orc_job_new.restype = C.c_void_p
        L.orc_job_new.argtypes = [C.c_int, C.c_char_p, C.c_uint32]
        L.orc_job_free.argtypes = [C.c_void_p]
        L.orc_job_add_pattern.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int32, C.c_int, i32p,
                                          C.c_char_p]
        L.orc_job_add_patterns.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_job_add_bed.argtypes = [C.c_void_p, C.c_char_p, u64p, u64p, C.c_int]
        L.orc_job_ext.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, u64p, u64p]
        L.orc_region_begin.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_char_p, C.c_int]
        L.orc_region_add_record_gt.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_char_p, C.c_char_p, i32p]
        L.orc_region_add_record_carriers.argtypes = [C.c_void_p, C.c_uint64, C.c_char_p, C.c_char_p, u32p, C.c_int]
        L.orc_region_end.argtypes = [C.c_void_p]
        L.orc_job_rows.argtypes = [C.c_void_p]
        L.orc_job_rows.restype = C.c_char_p
        L.orc_job_clear_rows.argtypes = [C.c_void_p]
        L.orc_job_nkeys.argtypes = [C.c_void_p]
        L.orc_job_key.argtypes = [C.c_void_p, C.c_int, intp, u64p, u64p, intp, u32p, u32p]
        L.orc_job_stats.argtypes = [C.c_void_p, intp, intp, u64p]
        L.orc_job_set_scan_only.argtypes = [C.c_void_p, C.c_int]
        L.orc_job_phase_seconds.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        L.orc_job_digests.argtypes = [C.c_void_p, u64p, u64p, u64p]
        L.orc_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_xxh64.restype = C.c_uint64
        _lib = L
    return _lib


def arr(ctype, vals):
    vals = list(vals)
    return (ctype * max(1, len(vals)))(*vals)


NUC = "ACGTN"


def nucs(s):
    return [NUC.index(c) for c in s]


# --------------------------------------------------------------------------
# unit-level wrappers
# --------------------------------------------------------------------------
def patch_haplotype(rng, diffs, ref):
    """rng=(s,e); diffs=[(pos, 'REF', 'ALT')]; ref=[('A', pos)...] -> [(nuc, pos)] or int error."""
    L = lib()
    dpos = arr(C.c_uint64, [d[0] for d in diffs])
    dref = arr(C.c_uint8, [x for d in diffs for x in nucs(d[1])])
    dnref = arr(C.c_int, [len(d[1]) for d in diffs])
    dalt = arr(C.c_uint8, [x for d in diffs for x in nucs(d[2])])
    dnalt = arr(C.c_int, [len(d[2]) for d in diffs])
    rn = arr(C.c_uint8, [NUC.index(n) for n, _ in ref])
    rp = arr(C.c_uint64, [p for _, p in ref])
    cap = len(ref) + sum(len(d[2]) for d in diffs) + 4
    on = (C.c_uint8 * cap)()
    op = (C.c_uint64 * cap)()
    r = L.orc_patch_haplotype(rng[0], rng[1], len(diffs), dpos, dref, dnref, dalt, dnalt, rn, rp, len(ref), on, op,
                              cap)
    if r < 0:
        return r
    return [(NUC[on[i]], op[i]) for i in range(r)]


def matches(w5, min_score, hap, kind=0):
    """w5: list of [a,c,g,t,n] rows; hap=[('A', pos)...] -> [(start, end)]."""
    L = lib()
    flat = arr(C.c_int32, [x for row in w5 for x in row])
    n = len(hap)
    hn = arr(C.c_uint8, [NUC.index(c) for c, _ in hap])
    hp = arr(C.c_uint64, [p for _, p in hap])
    cap = n + 2
    os_ = (C.c_uint64 * cap)()
    oe = (C.c_uint64 * cap)()
    r = L.orc_matches(flat, len(w5), min_score, kind, hn, hp, n, os_, oe, cap)
    if r < 0:
        return r
    return [(os_[i], oe[i]) for i in range(r)]


def counts_as_genotypes(v1, v2):
    L = lib()
    n = len(v1)
    maf = C.c_uint32()
    info = C.create_string_buffer(64 + 16 * n)
    gts = C.create_string_buffer(64 + 24 * n)
    r = L.orc_counts_as_genotypes(arr(C.c_uint32, v1), arr(C.c_uint32, v2), n, C.byref(maf), info, len(info), gts,
                                  len(gts))
    if r != 1:
        return None
    return maf.value, info.value.decode(), gts.value.decode()


def count_matches_by_sample(nsamp, match_list, inner):
    """match_list: [((s,e), pid, [(sample, side)])]; inner: [(bed_idx, s, e)] ->
    {(bed_idx, (s,e), pid): (L, R)}"""
    L = lib()
    ids, off, cnt = [], [], []
    for (_, _), _, hs in match_list:
        off.append(len(ids))
        cnt.append(len(hs))
        ids.extend(2 * s + side for s, side in hs)
    k = L.orc_count_matches_by_sample(
        nsamp, len(match_list), arr(C.c_uint64, [m[0][0] for m in match_list]),
        arr(C.c_uint64, [m[0][1] for m in match_list]), arr(C.c_uint16, [m[1] for m in match_list]),
        arr(C.c_int, off), arr(C.c_int, cnt), arr(C.c_uint32, ids), len(inner),
        arr(C.c_int, [i[0] for i in inner]), arr(C.c_uint64, [i[1] for i in inner]),
        arr(C.c_uint64, [i[2] for i in inner]))
    out = {}
    try:
        for i in range(L.orc_keys_count(k)):
            b, s, e, pid = C.c_int(), C.c_uint64(), C.c_uint64(), C.c_int()
            l = (C.c_uint32 * max(1, nsamp))()
            r = (C.c_uint32 * max(1, nsamp))()
            L.orc_keys_get(k, i, C.byref(b), C.byref(s), C.byref(e), C.byref(pid), l, r)
            out[(b.value, (s.value, e.value), pid.value)] = (list(l[:nsamp]), list(r[:nsamp]))
    finally:
        L.orc_keys_free(k)
    return out


def merge_ranges(ranges):
    L = lib()
    n = len(ranges)
    os_ = (C.c_uint64 * max(1, n))()
    oe = (C.c_uint64 * max(1, n))()
    m = L.orc_merge_ranges(arr(C.c_uint64, [r[0] for r in ranges]), arr(C.c_uint64, [r[1] for r in ranges]), n, os_,
                           oe)
    return [(os_[i], oe[i]) for i in range(m)]


class Patterns:
    """Oracle pattern list (pattern.rs:37-87)."""

    def __init__(self):
        self.h = lib().orc_patterns_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_patterns_free(self.h)
            self.h = None

    @classmethod
    def from_files(cls, pwm_file, thr_dir, thr, names, add_reverse=True):
        p = cls()
        r = lib().orc_parse_pwm_files(pwm_file.encode(), thr_dir.encode(), thr, ",".join(names).encode(),
                                      1 if add_reverse else 0, p.h)
        if r < 0:
            raise RuntimeError("oracle parse_pwm_files failed: %d" % r)
        return p

    def add(self, kind, direction, pid, min_score, w5, name):
        flat = arr(C.c_int32, [x for row in w5 for x in row])
        lib().orc_patterns_add(self.h, kind, direction, pid, min_score, len(w5), flat, name.encode())

    def __len__(self):
        return lib().orc_patterns_count(self.h)

    def get(self, i):
        L = lib()
        k, d, pid, ln = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        ms = C.c_int32()
        L.orc_pattern_info(self.h, i, C.byref(k), C.byref(d), C.byref(pid), C.byref(ms), C.byref(ln))
        w = L.orc_pattern_weights(self.h, i)
        rows = [[w[j * 5 + c] for c in range(5)] for j in range(ln.value)]
        return {"kind": k.value, "direction": d.value, "pattern_id": pid.value, "min_score": ms.value,
                "weights": rows, "name": L.orc_pattern_name(self.h, i).decode()}

    def as_list(self):
        return [self.get(i) for i in range(len(self))]


class Job:
    """One oracle run over merged regions (main.rs:234-436, single worker thread)."""

    def __init__(self, nsamp, chrom, patterns, beds, min_maf=0):
        """patterns: list of dicts (Patterns.as_list()); beds: [(basename, [(s,e),...])]."""
        L = lib()
        self.L = L
        self.nsamp = nsamp
        self.h = L.orc_job_new(nsamp, chrom.encode(), min_maf)
        for p in patterns:
            flat = arr(C.c_int32, [x for row in p["weights"] for x in row])
            L.orc_job_add_pattern(self.h, p["kind"], p["direction"], p["pattern_id"], p["min_score"],
                                  len(p["weights"]), flat, p["name"].encode())
        self.bed_names = []
        for name, ranges in beds:
            self.bed_names.append(name)
            L.orc_job_add_bed(self.h, name.encode(), arr(C.c_uint64, [r[0] for r in ranges]),
                              arr(C.c_uint64, [r[1] for r in ranges]), len(ranges))

    def close(self):
        if self.h:
            self.L.orc_job_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def ext(self, s, e):
        es, ee = C.c_uint64(), C.c_uint64()
        r = self.L.orc_job_ext(self.h, s, e, C.byref(es), C.byref(ee))
        if r:
            raise RuntimeError("ext failed %d" % r)
        return es.value, ee.value

    def begin(self, s, e, ref_ascii):
        r = self.L.orc_region_begin(self.h, s, e, ref_ascii.encode(), len(ref_ascii))
        return r

    def add_record_gt(self, pos, n_alleles, ref, alt, gts):
        flat = arr(C.c_int32, [x for g in gts for x in g])
        return self.L.orc_region_add_record_gt(self.h, pos, n_alleles, ref.encode(), alt.encode(), flat)

    def add_record_carriers(self, pos, ref, alt, hap_ids):
        return self.L.orc_region_add_record_carriers(self.h, pos, ref.encode(), alt.encode(),
                                                     arr(C.c_uint32, hap_ids), len(hap_ids))

    def add_record_carriers_np(self, pos, ref, alt, hap_ids):
        """hap_ids: a contiguous numpy uint32 array (no per-id conversion)."""
        return self.L.orc_region_add_record_carriers(self.h, pos, ref.encode(), alt.encode(),
                                                     hap_ids.ctypes.data_as(u32p), len(hap_ids))

    def end(self):
        return self.L.orc_region_end(self.h)

    def rows(self):
        return self.L.orc_job_rows(self.h).decode()

    def keys(self):
        out = {}
        n = self.nsamp
        for i in range(self.L.orc_job_nkeys(self.h)):
            b, s, e, pid = C.c_int(), C.c_uint64(), C.c_uint64(), C.c_int()
            l = (C.c_uint32 * max(1, n))()
            r = (C.c_uint32 * max(1, n))()
            self.L.orc_job_key(self.h, i, C.byref(b), C.byref(s), C.byref(e), C.byref(pid), l, r)
            out[(self.bed_names[b.value], (s.value, e.value), pid.value)] = (list(l[:n]), list(r[:n]))
        return out

    def keys_np(self):
        """keys() with numpy uint32 vectors (large sample counts)."""
        import numpy as np
        out = {}
        n = self.nsamp
        for i in range(self.L.orc_job_nkeys(self.h)):
            b, s, e, pid = C.c_int(), C.c_uint64(), C.c_uint64(), C.c_int()
            l = np.zeros(max(1, n), dtype=np.uint32)
            r = np.zeros(max(1, n), dtype=np.uint32)
            self.L.orc_job_key(self.h, i, C.byref(b), C.byref(s), C.byref(e), C.byref(pid),
                               l.ctypes.data_as(u32p), r.ctypes.data_as(u32p))
            out[(self.bed_names[b.value], (s.value, e.value), pid.value)] = (l[:n], r[:n])
        return out

    def set_scan_only(self, on=True):
        """Skip count_matches_by_sample and the rows (the bench's scan-only CPU baseline)."""
        self.L.orc_job_set_scan_only(self.h, 1 if on else 0)

    def phase_seconds(self):
        """Wall seconds summed over regions: (load_diffs+patch, find_all_matches, keys+rows)."""
        out = (C.c_double * 3)()
        self.L.orc_job_phase_seconds(self.h, out)
        return tuple(out)

    def clear_rows(self):
        self.L.orc_job_clear_rows(self.h)

    def digests(self):
        """(keys, rows, n_rows) digests of the last region (orc_job_digests): the order-free
        sketch of its count_matches_by_sample map and XXH64 of its rows without POS (the
        rows since the last clear_rows)."""
        k, r, n = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self.L.orc_job_digests(self.h, C.byref(k), C.byref(r), C.byref(n))
        return k.value, r.value, n.value

    def stats(self):
        a, b, c = C.c_int(), C.c_int(), C.c_uint64()
        self.L.orc_job_stats(self.h, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value


# --------------------------------------------------------------------------
# run(): the reference CLI flow over test-data-style inputs (main.rs:234-393)
# --------------------------------------------------------------------------
def read_fai(path):
    idx = {}
    for line in open(path):
        f = line.rstrip("\n").split("\t")
        if len(f) >= 5:
            idx[f[0]] = (int(f[1]), int(f[2]), int(f[3]), int(f[4]))
    return idx


def fasta_fetch(fa, fai, chrom, start, stop):
    """bio::io::fasta::IndexedReader fetch(chrom, start, stop) + read (half-open, truncated at the end)."""
    ln, off, lb, lw = fai[chrom]
    stop = min(stop, ln)
    if start >= stop:
        return ""
    out = []
    with open(fa, "rb") as f:
        pos = start
        while pos < stop:
            line_no, col = divmod(pos, lb)
            f.seek(off + line_no * lw + col)
            take = min(lb - col, stop - pos)
            out.append(f.read(take).decode())
            pos += take
    return "".join(out)


def load_bed(path, chrom):
    """bed.rs:9-19"""
    out = []
    for line in open(path):
        line = line.rstrip("\n")
        if not line:
            continue
        f = line.split("\t")
        if f[0] == chrom:
            out.append((int(f[1]), int(f[2])))
    return out


def load_peak_files(bed_files, chrom, after_position):
    """bed.rs:25-47 -> (merged peaks, [(basename, peaks)])"""
    peak_map = {}
    for b in bed_files:
        if not os.path.exists(b):
            raise FileNotFoundError(b)
        peak_map[b] = [p for p in load_bed(b, chrom) if p[0] >= after_position]
    allr = [p for v in peak_map.values() for p in v]
    merged = merge_ranges(allr)
    merged.sort(key=lambda r: r[0])
    simple = {}
    for k, v in peak_map.items():
        simple[os.path.basename(k)] = v
    return merged, list(simple.items())


def run(chrom, records, bed_files, fasta, sample_names, wanted_samples, pwm_file, thr_dir, thr, names,
        forward_only=False, min_maf=0, after_position=0):
    """records: the decoded BCF (tests/golden/*.records.json); returns VCF text."""
    pats = Patterns.from_files(pwm_file, thr_dir, thr, names, add_reverse=not forward_only)
    plist = pats.as_list()
    assert len(plist) > 0
    merged, beds = load_peak_files(bed_files, chrom, after_position)
    if wanted_samples is None:
        sel = list(range(len(sample_names)))
    else:
        want = set(wanted_samples)
        sel = [i for i, s in enumerate(sample_names) if s in want]
    header = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT" + "".join(
        "\t" + sample_names[i] for i in sel) + "\n"
    job = Job(len(sel), chrom, plist, beds, min_maf)
    fai = read_fai(fasta + ".fai")
    out = [header]
    fake = 1
    for (s, e) in merged:
        es, ee = job.ext(s, e)
        ref = fasta_fetch(fasta, fai, chrom, es, ee + 1)
        r = job.begin(s, e, ref)
        if r:
            raise RuntimeError("region begin failed %d" % r)
        for rec in records:
            if rec["chrom"] != chrom:
                continue
            p0, rl = rec["pos0"], rec["rlen"]
            if not (p0 < ee + 1 and p0 + rl > es):  # htslib region overlap
                continue
            al = rec["alleles"]
            if len(al) < 2:
                raise RuntimeError("record with one allele")
            gts = [rec["gt"][i][:2] + [-2147483647] * (2 - len(rec["gt"][i][:2])) for i in sel]
            r = job.add_record_gt(p0, len(al), al[0], al[1], gts)
            if r:
                raise RuntimeError("add record failed %d" % r)
        r = job.end()
        if r:
            raise RuntimeError("region failed %d" % r)
    txt = job.rows()
    job.close()
    return "".join(out) + txt
