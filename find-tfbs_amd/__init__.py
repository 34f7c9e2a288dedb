"""find-tfbs_amd: MI355X-native drop-in for find-tfbs's per-haplotype TFBS scoring path.

This module mirrors the reference's Rust interface for that path (names,
argument meaning, error behaviour) over the C ABI of include/tfbs_amd.h:

  reference (find-tfbs v1.0.1)                    here
  ----------------------------------------------  ---------------------------------
  pattern.rs:13-16   parse_weight                 parse_weight
  pattern.rs:18-35   parse_threshold_file         parse_threshold_file
  pattern.rs:37-87   parse_pwm_files              parse_pwm_files -> PatternSet
  pattern.rs:141-171 matches                      matches / Scanner.matches (GPU)
  haplotype.rs:94    patch_haplotype              patch_haplotype
  haplotype.rs:77    load_haplotypes  \
  main.rs:94         find_all_matches  >          RegionBatch (+ Scanner.scan, GPU)
  main.rs:500        count_matches_by_sample /    RegionBatch.keys
  main.rs:439        counts_as_genotypes          counts_as_genotypes
  main.rs:415-429    row emission                 RegionBatch.rows

The reference panics where TfbsError is raised.  The scan always runs on a HIP
device; without one, Scanner() raises TfbsError(TFBS_E_NODEVICE).
"""
import ctypes as C
from collections import namedtuple

from . import _capi
from ._capi import TfbsError, check, lib, tfbs_pattern_desc  # noqa: F401

TFBS_OK = 0
TFBS_E_NODEVICE = -10
KIND_PWM, KIND_OTHER = 0, 1
DIR_P, DIR_N = 0, 1
NUCLEOTIDES = "ACGTN"  # types.rs:5-8, the weight index order

Range = namedtuple("Range", "start end")  # range.rs:4-8, inclusive
NucleotidePos = namedtuple("NucleotidePos", "nuc pos")  # types.rs:23-27 (nuc as 'A'..'N')
Diff = namedtuple("Diff", "pos reference alternative")  # types.rs:39-44 (strings)
HaplotypeId = namedtuple("HaplotypeId", "sample_id side")  # types.rs:66-70, side 0 Left / 1 Right
Match = namedtuple("Match", "range pattern_id haplotype_ids")  # types.rs:32-37


class Weight:
    """types.rs:103-114: four milli-log-odds weights, N forced to 0."""

    __slots__ = ("acgtn",)

    def __init__(self, a, c, g, t):
        self.acgtn = [a, c, g, t, 0]

    def __eq__(self, o):
        return isinstance(o, Weight) and self.acgtn == o.acgtn

    def __repr__(self):
        return "Weight(%r)" % (self.acgtn,)


class Pattern:
    """types.rs:86-90: PWM (kind 0) or OtherPattern (kind 1)."""

    def __init__(self, name, pattern_id, weights=None, min_score=0, direction=DIR_P, kind=KIND_PWM):
        self.name = name
        self.pattern_id = pattern_id
        self.weights = list(weights or [])
        self.min_score = min_score
        self.direction = direction
        self.kind = kind

    @classmethod
    def PWM(cls, weights, name, pattern_id, min_score, direction=DIR_P):
        return cls(name, pattern_id, weights, min_score, direction, KIND_PWM)

    @classmethod
    def OtherPattern(cls, name, pattern_id):
        return cls(name, pattern_id, [], 0, DIR_P, KIND_OTHER)

    def __len__(self):  # pattern_length (types.rs:92-101)
        return len(self.weights) if self.kind == KIND_PWM else 0

    def __eq__(self, o):
        return (isinstance(o, Pattern) and (self.name, self.pattern_id, self.weights, self.min_score,
                                             self.direction, self.kind) ==
                (o.name, o.pattern_id, o.weights, o.min_score, o.direction, o.kind))

    def __repr__(self):
        return "Pattern(%s id=%d L=%d min=%d dir=%s)" % (self.name, self.pattern_id, len(self), self.min_score,
                                                         "+-"[self.direction])


def _u(x):
    return x.encode() if isinstance(x, str) else x


def parse_weight(s):
    v = C.c_int32()
    check(lib().tfbs_parse_weight(_u(s), C.byref(v)))
    return v.value


def parse_threshold_file(filename, pwm_threshold):
    v = C.c_int32()
    r = check(lib().tfbs_parse_threshold_file(_u(filename), pwm_threshold, C.byref(v)))
    return v.value if r == 1 else None


class PatternSet:
    """An immutable tfbs_patterns handle (Vec<Pattern> of the reference)."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def from_patterns(cls, patterns):
        n = len(patterns)
        descs = (tfbs_pattern_desc * max(1, n))()
        keep = []
        for i, p in enumerate(patterns):
            flat = [x for w in p.weights for x in (w.acgtn if isinstance(w, Weight) else list(w)[:4] + [0])]
            arr = (C.c_int32 * max(1, len(flat)))(*flat)
            name = _u(p.name)
            keep.append((arr, name))
            descs[i] = tfbs_pattern_desc(p.pattern_id, p.direction, p.kind, len(p), arr, p.min_score, name)
        h = C.c_void_p()
        check(lib().tfbs_patterns_create(descs, n, C.byref(h)))
        return cls(h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().tfbs_patterns_destroy(self.h)
            self.h = None

    def __len__(self):
        return lib().tfbs_patterns_count(self.h)

    def __getitem__(self, i):
        d = tfbs_pattern_desc()
        check(lib().tfbs_patterns_get(self.h, i, C.byref(d)))
        ws = [Weight(*(d.weights[5 * j + c] for c in range(4))) for j in range(d.length)]
        return Pattern(d.name.decode(), d.pattern_id, ws, d.min_score, d.direction, d.kind)

    def to_list(self):
        return [self[i] for i in range(len(self))]

    def name_of(self, pattern_id):
        s = lib().tfbs_patterns_name_of(self.h, pattern_id)
        return s.decode() if s is not None else None

    @property
    def max_length(self):
        return lib().tfbs_patterns_max_length(self.h)

    def mfma_bound(self, i, window):
        """The matrix-core bound of pattern i on one window ("ACGTN" string of the pattern's
        length): dict(eligible, q8, t8, scale, c); bound = c + scale * q8 / 8, candidate iff q8 > t8."""
        codes = (C.c_uint8 * max(1, len(window)))(*["ACGTN".index(ch) for ch in window])
        out = _capi.tfbs_mfma_bound()
        check(lib().tfbs_patterns_mfma_bound(self.h, i, codes, C.byref(out)))
        return {n: getattr(out, n) for n, _ in out._fields_}

    def subset(self, keep_pattern_id):
        """A new PatternSet of the patterns whose pattern_id passes keep_pattern_id (both
        strands of a PWM share an id, so they stay together): a pattern shard of SURVEY.md
        8(e)'s region x PWM split.  Batches scanning it pass the whole set's max_length to
        RegionBatch(window_lmax=...) so their windows are the unsharded run's."""
        return PatternSet.from_patterns([p for p in self.to_list() if keep_pattern_id(p.pattern_id)])

    def plan_stats(self, tile_blocks=20, mfma=False):
        """Host-side summary of the device plan (octet/quad/generic/MFMA strands, tiles)."""
        st = _capi.tfbs_plan_stats()
        check(lib().tfbs_patterns_plan_stats(self.h, tile_blocks, 1 if mfma else 0, C.byref(st)))
        return {n: getattr(st, n) for n, _ in st._fields_}


def parse_pwm_files(pwm_file, threshold_dir, pwm_threshold, wanted_pwms, add_reverse_patterns=True):
    """pattern.rs:37-87.  Returns a PatternSet (index it or .to_list() for Pattern objects)."""
    h = C.c_void_p()
    check(lib().tfbs_patterns_from_files(_u(pwm_file), _u(threshold_dir), pwm_threshold,
                                         _u(",".join(wanted_pwms)), 1 if add_reverse_patterns else 0, C.byref(h)))
    return PatternSet(h)


def device_count():
    n = C.c_int()
    rc = lib().tfbs_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def _nuc_codes(hap):
    return [NUCLEOTIDES.index(n.nuc if isinstance(n, NucleotidePos) else n[0]) for n in hap]


def patch_haplotype(rng, diffs, ref_haplotype):
    """haplotype.rs:94-156 (host C++ in libtfbs_amd).  diffs: [Diff(pos, 'REF', 'ALT')]."""
    L = lib()
    nd = len(diffs)
    dref = [NUCLEOTIDES.index(c) for d in diffs for c in d.reference]
    dalt = [NUCLEOTIDES.index(c) for d in diffs for c in d.alternative]
    n = len(ref_haplotype)
    cap = n + sum(len(d.alternative) for d in diffs) + 8
    on = (C.c_uint8 * cap)()
    op = (C.c_uint64 * cap)()
    nout = C.c_size_t()
    check(L.tfbs_patch_haplotype(
        rng[0], rng[1], nd, (C.c_uint64 * max(1, nd))(*[d.pos for d in diffs]),
        (C.c_uint8 * max(1, len(dref)))(*dref), (C.c_uint32 * max(1, nd))(*[len(d.reference) for d in diffs]),
        (C.c_uint8 * max(1, len(dalt)))(*dalt), (C.c_uint32 * max(1, nd))(*[len(d.alternative) for d in diffs]),
        (C.c_uint8 * max(1, n))(*_nuc_codes(ref_haplotype)),
        (C.c_uint64 * max(1, n))(*[x[1] for x in ref_haplotype]), n, on, op, cap, C.byref(nout)))
    return [NucleotidePos(NUCLEOTIDES[on[i]], op[i]) for i in range(nout.value)]


def counts_as_genotypes(v1, v2, verbose=False):
    """main.rs:439-498 -> (distinct_counts, maf, freq0, freq1, freq2, genotypes) or None."""
    n = len(v1)
    maf = C.c_uint32()
    info = C.create_string_buffer(64 + 16 * n)
    gts = C.create_string_buffer(64 + 24 * n)
    r = check(lib().tfbs_counts_as_genotypes((C.c_uint32 * max(1, n))(*v1), (C.c_uint32 * max(1, n))(*v2), n,
                                             C.byref(maf), info, len(info), gts, len(gts)))
    if r != 1:
        return None
    s = info.value.decode()
    counts_part, freqs_part = s.split(";")
    counts = [int(x) for x in counts_part[len("COUNTS="):].split(",")]
    f0, f1, f2 = (int(x) for x in freqs_part[len("freqs="):].split("/"))
    return counts, maf.value, f0, f1, f2, gts.value.decode()


class Scanner:
    """A device context: the pattern tables resident on one GPU (one per host thread)."""

    def __init__(self, patterns, device=0):
        self.patterns = patterns if isinstance(patterns, PatternSet) else PatternSet.from_patterns(patterns)
        self.h = C.c_void_p()
        check(lib().tfbs_ctx_create(device, self.patterns.h, C.byref(self.h)))

    def close(self):
        if getattr(self, "h", None):
            lib().tfbs_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def matches_all(self, haplotype):
        """pattern.rs:141-171 for every pattern: list (per pattern, creation order) of [(start, end)]."""
        n = len(haplotype)
        nucs = (C.c_uint8 * max(1, n))(*_nuc_codes(haplotype))
        pos = (C.c_uint64 * max(1, n))(*[x[1] for x in haplotype])
        npat = len(self.patterns)
        counts = (C.c_uint32 * max(1, npat))()
        total = C.c_size_t()
        cap = 64
        while True:
            s = (C.c_uint64 * cap)()
            e = (C.c_uint64 * cap)()
            rc = lib().tfbs_matches(self.h, nucs, pos, n, counts, s, e, cap, C.byref(total))
            if rc == -1 and total.value > cap:
                cap = total.value
                continue
            check(rc)
            break
        out, k = [], 0
        for i in range(npat):
            out.append([(s[k + j], e[k + j]) for j in range(counts[i])])
            k += counts[i]
        return out

    def matches(self, pattern_index, haplotype, haplotype_ids=()):
        p = self.patterns[pattern_index]
        ids = tuple(haplotype_ids)
        return [Match(Range(a, b), p.pattern_id, ids) for a, b in self.matches_all(haplotype)[pattern_index]]

    def last_scan_ms(self):
        return lib().tfbs_ctx_last_scan_ms(self.h)


def matches(pattern, haplotype, haplotype_ids=(), verbose=False):
    """pattern.rs:141-171 for one Pattern on one haplotype (GPU; builds a one-pattern Scanner)."""
    sc = Scanner([pattern])
    try:
        return sc.matches(0, haplotype, haplotype_ids)
    finally:
        sc.close()


class RegionBatch:
    """load_haplotypes + find_all_matches + count_matches_by_sample over many merged regions."""

    VECTOR_END = -2147483647

    def __init__(self, patterns, n_samples, keep_membership=True, window_lmax=None, build_device=None):
        self.patterns = patterns
        self.n_samples = n_samples
        self.h = C.c_void_p()
        check(lib().tfbs_batch_create(patterns.h, n_samples, 1 if keep_membership else 0, C.byref(self.h)))
        self.beds = []
        if window_lmax is not None:  # a pattern shard: the whole set's windows (tfbs_batch_set_window_lmax)
            check(lib().tfbs_batch_set_window_lmax(self.h, window_lmax))
        if build_device is not None:  # haplotype grouping on a device (tfbs_batch_set_build_device)
            check(lib().tfbs_batch_set_build_device(self.h, build_device))

    def build_stats(self):
        """(regions grouped on the device, regions built on the host)."""
        d, h = C.c_uint64(), C.c_uint64()
        check(lib().tfbs_batch_build_stats(self.h, C.byref(d), C.byref(h)))
        return d.value, h.value

    def patch_stats(self):
        """Regions grouped on the device whose distinct groups the host patched."""
        p = C.c_uint64()
        check(lib().tfbs_batch_patch_stats(self.h, C.byref(p)))
        return p.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().tfbs_batch_destroy(self.h)
            self.h = None

    def add_bed(self, basename):
        self.beds.append(basename)
        return check(lib().tfbs_batch_add_bed(self.h, _u(basename)))

    def ext(self, start, end):
        es, ee = C.c_uint64(), C.c_uint64()
        check(lib().tfbs_batch_region_ext(self.h, start, end, C.byref(es), C.byref(ee)))
        return es.value, ee.value

    def begin(self, start, end, ref_ascii):
        check(lib().tfbs_batch_region_begin(self.h, start, end, _u(ref_ascii), len(ref_ascii)))

    def add_inner(self, bed, start, end):
        check(lib().tfbs_batch_region_add_inner(self.h, bed, start, end))

    def add_record_gt(self, pos, n_alleles, ref, alt, gts):
        flat = [x for g in gts for x in (list(g[:2]) + [self.VECTOR_END] * (2 - len(g[:2])))]
        check(lib().tfbs_batch_region_add_record_gt(self.h, pos, n_alleles, _u(ref), _u(alt),
                                                    (C.c_int32 * max(1, len(flat)))(*flat)))

    def add_record_carriers(self, pos, ref, alt, hap_ids):
        hap_ids = list(hap_ids)
        check(lib().tfbs_batch_region_add_record_carriers(self.h, pos, _u(ref), _u(alt),
                                                          (C.c_uint32 * max(1, len(hap_ids)))(*hap_ids),
                                                          len(hap_ids)))

    def end(self):
        check(lib().tfbs_batch_region_end(self.h))

    def synth_fill(self, seed, first, count, indel_pct=0):
        check(lib().tfbs_synth_fill_batch(self.h, seed, first, count, indel_pct))
        if "synthetic.bed" not in self.beds:  # registered by the library on first use
            self.beds.append("synthetic.bed")

    @property
    def num_regions(self):
        return lib().tfbs_batch_num_regions(self.h)

    @property
    def num_haplotypes(self):
        return lib().tfbs_batch_num_haplotypes(self.h)

    @property
    def num_windows(self):
        return lib().tfbs_batch_num_windows(self.h)

    @property
    def num_cell_ops(self):
        return lib().tfbs_batch_num_cell_ops(self.h)

    @property
    def num_effective_windows(self):
        return lib().tfbs_batch_num_effective_windows(self.h)

    @property
    def num_scan_windows(self):
        """Windows the scan executes (reference-window reuse skips SNV-only haplotypes'
        windows equal to the reference's)."""
        return lib().tfbs_batch_num_scan_windows(self.h)

    @property
    def num_scan_cell_ops(self):
        return lib().tfbs_batch_num_scan_cell_ops(self.h)

    @property
    def input_bytes(self):
        return lib().tfbs_batch_input_bytes(self.h)

    @property
    def output_bytes(self):
        return lib().tfbs_batch_output_bytes(self.h)

    def region_stats(self, r):
        a, b = C.c_uint32(), C.c_uint32()
        check(lib().tfbs_batch_region_stats(self.h, r, C.byref(a), C.byref(b)))
        return a.value, b.value

    def scan(self, scanner, upload=True, download=True, reduce=False, encode=False):
        """tfbs_scan; then either download the dense counts or (reduce=True) classify the
        keys on the GPU and fetch only what row emission needs (tfbs_batch_reduce), and
        (encode=True) encode every varying key's per-sample totals on the GPU
        (tfbs_batch_encode) so rows format from codes."""
        if upload:
            check(lib().tfbs_batch_upload(scanner.h, self.h))
        check(lib().tfbs_scan(scanner.h, self.h))
        if reduce or encode:
            check(lib().tfbs_batch_reduce(scanner.h, self.h))
            if encode:
                self.encode(scanner)
        elif download:
            check(lib().tfbs_batch_download(scanner.h, self.h))

    def encode(self, scanner, r0=0, r1=None, device_codes=False):
        """tfbs_batch_encode for regions [r0, r1) (after a reduced scan); device_codes: keep the
        per-sample codes on the GPU (for rows_bgzf)."""
        check(lib().tfbs_batch_encode_flags(scanner.h, self.h, r0, self.num_regions if r1 is None else r1,
                                            1 if device_codes else 0))

    def keys(self, region):
        """count_matches_by_sample for one region: {(bed, (s, e), pattern_id): (L, R)}."""
        L = lib()
        n = C.c_size_t()
        check(L.tfbs_batch_region_num_keys(self.h, region, C.byref(n)))
        out = {}
        ns = self.n_samples
        for k in range(n.value):
            bed, s, e, pid = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint16()
            l = (C.c_uint32 * max(1, ns))()
            r = (C.c_uint32 * max(1, ns))()
            check(L.tfbs_batch_region_key(self.h, region, k, C.byref(bed), C.byref(s), C.byref(e), C.byref(pid), l,
                                          r))
            out[(self.beds[bed.value], (s.value, e.value), pid.value)] = (list(l[:ns]), list(r[:ns]))
        return out

    def keys_np(self, region):
        """keys() with numpy uint32 vectors (large sample counts)."""
        import numpy as np
        L = lib()
        n = C.c_size_t()
        check(L.tfbs_batch_region_num_keys(self.h, region, C.byref(n)))
        out = {}
        ns = self.n_samples
        for k in range(n.value):
            bed, s, e, pid = C.c_uint32(), C.c_uint64(), C.c_uint64(), C.c_uint16()
            l = np.zeros(max(1, ns), dtype=np.uint32)
            r = np.zeros(max(1, ns), dtype=np.uint32)
            check(L.tfbs_batch_region_key(self.h, region, k, C.byref(bed), C.byref(s), C.byref(e), C.byref(pid),
                                          l.ctypes.data_as(_capi.u32p), r.ctypes.data_as(_capi.u32p)))
            out[(self.beds[bed.value], (s.value, e.value), pid.value)] = (l[:ns], r[:ns])
        return out

    def region_rows(self, region, chromosome, min_maf=0, fake_position=1):
        """Rows of one region (main.rs:415-429); returns (text, next fake_position)."""
        fp = C.c_uint32(fake_position)
        p = C.c_void_p()
        n = C.c_size_t()
        check(lib().tfbs_batch_region_rows(self.h, region, _u(chromosome), min_maf, C.byref(fp), C.byref(p),
                                           C.byref(n)))
        try:
            text = C.string_at(p, n.value).decode()
        finally:
            lib().tfbs_free(p)
        return text, fp.value

    def digest(self, region):
        """tfbs_batch_region_digest: the region's keys at the distinct-haplotype level."""
        d = C.c_uint64()
        check(lib().tfbs_batch_region_digest(self.h, region, C.byref(d)))
        return d.value

    def key_digest_sum(self, region):
        """tfbs_batch_region_key_digest_sum: order-free; pattern shards add up to the whole."""
        d = C.c_uint64()
        check(lib().tfbs_batch_region_key_digest_sum(self.h, region, C.byref(d)))
        return d.value

    def region_digests(self, r0=0, r1=None, min_maf=0, threads=16, keys=True, rows=True):
        """tfbs_batch_region_digests over regions [r0, r1): numpy uint64 arrays (keys, rows,
        n_rows) -- the canonical sketch of each region's count_matches_by_sample vectors and
        XXH64 of its rows without POS, comparable with the oracle's orc_job_digests (None for
        a digest not asked for)."""
        import numpy as np
        r1 = self.num_regions if r1 is None else r1
        n = max(1, r1 - r0)
        k, r, c = (np.zeros(n, dtype=np.uint64) for _ in range(3))
        p = C.POINTER(C.c_uint64)
        ptr = lambda a, on: a.ctypes.data_as(p) if on else None
        check(lib().tfbs_batch_region_digests(self.h, r0, r1, min_maf, threads, ptr(k, keys), ptr(r, rows),
                                              ptr(c, rows)))
        return (k[:r1 - r0] if keys else None), (r[:r1 - r0] if rows else None), (c[:r1 - r0] if rows else None)

    def input_digest(self, region):
        """tfbs_batch_region_input_digest: what the host prep packed for the region."""
        d = C.c_uint64()
        check(lib().tfbs_batch_region_input_digest(self.h, region, C.byref(d)))
        return d.value

    def format_rows(self, chromosome, min_maf=0, threads=1, r0=0, r1=None):
        """Format the rows of regions [r0, r1) on host threads and discard them: (rows, bytes)."""
        r, n = C.c_uint64(), C.c_uint64()
        check(lib().tfbs_batch_format_rows(self.h, _u(chromosome), min_maf, threads, r0,
                                           self.num_regions if r1 is None else r1, C.byref(r), C.byref(n)))
        return r.value, n.value

    def prep_seconds(self):
        """(generation CPU-s, build_region CPU-s, build + commit wall-s, fill wall-s) of synth_fill."""
        out = (C.c_double * 4)()
        check(lib().tfbs_batch_prep_seconds(self.h, out))
        return tuple(out)

    def rows_bgzf(self, scanner, chromosome, min_maf=0, fake_position=1, r0=0, r1=None, fd=None):
        """tfbs_batch_rows_bgzf: the rows of regions [r0, r1) as BGZF blocks built on the
        GPU (after encode over them), written to file descriptor fd; without fd they are
        returned.  Returns (bytes or bytes written, next fake_position, rows, text bytes)."""
        import os
        import tempfile
        fp = C.c_uint32(fake_position)
        nw, nr, nb = C.c_uint64(), C.c_uint64(), C.c_uint64()
        tmp = None
        if fd is None:
            tmp = tempfile.TemporaryFile()
            fd_ = tmp.fileno()
        else:
            fd_ = fd
        try:
            check(lib().tfbs_batch_rows_bgzf(scanner.h, self.h, r0, self.num_regions if r1 is None else r1,
                                             _u(chromosome), min_maf, C.byref(fp), fd_, C.byref(nw), C.byref(nr),
                                             C.byref(nb)))
            if tmp is not None:
                tmp.seek(0)
                out = tmp.read()
            else:
                out = nw.value
        finally:
            if tmp is not None:
                tmp.close()
        return out, fp.value, nr.value, nb.value

    def rows(self, chromosome, min_maf=0, fake_position=1):
        """Rows for every region (main.rs:415-429); returns (text, next fake_position)."""
        fp = C.c_uint32(fake_position)
        p = C.c_void_p()
        n = C.c_size_t()
        check(lib().tfbs_batch_rows(self.h, _u(chromosome), min_maf, C.byref(fp), C.byref(p), C.byref(n)))
        try:
            text = C.string_at(p, n.value).decode()
        finally:
            lib().tfbs_free(p)
        return text, fp.value


class SynthRegion:
    """A synthetic phased region."""

    def __init__(self, seed, index, n_samples, lmax, indel_pct=0):
        L = lib()
        self.h = C.c_void_p()
        check(L.tfbs_synth_region_make(seed, index, n_samples, lmax, indel_pct, C.byref(self.h)))
        ms, me, es = C.c_uint64(), C.c_uint64(), C.c_uint64()
        ref = C.c_char_p()
        nref, nrec = C.c_size_t(), C.c_size_t()
        L.tfbs_synth_region_info(self.h, C.byref(ms), C.byref(me), C.byref(es), C.byref(ref), C.byref(nref),
                                 C.byref(nrec))
        self.merged = (ms.value, me.value)
        self.ext_start = es.value
        self.ref = C.string_at(ref, nref.value).decode()
        self.records = []
        for i in range(nrec.value):
            pos = C.c_uint64()
            r, a = C.c_char_p(), C.c_char_p()
            car = C.POINTER(C.c_uint32)()
            n = C.c_size_t()
            L.tfbs_synth_region_record(self.h, i, C.byref(pos), C.byref(r), C.byref(a), C.byref(car), C.byref(n))
            self.records.append((pos.value, r.value.decode(), a.value.decode(), list(car[:n.value])))
        L.tfbs_synth_region_destroy(self.h)
        self.h = None


def synth_write_pwms(directory, n_pwms, length_config, seed):
    p = C.c_void_p()
    check(lib().tfbs_synth_write_pwms(_u(directory), n_pwms, length_config, seed, C.byref(p)))
    try:
        names = C.string_at(p).decode().split(",")
    finally:
        lib().tfbs_free(p)
    return names


def range_overlaps(a, b):
    """range.rs:18-21: asymmetric -- are b's endpoints inside a?"""
    return a[0] <= b[0] <= a[1] or a[0] <= b[1] <= a[1]


def select_inner_peaks(merged, beds):
    """main.rs:62-72: [(bed index, start, end)] of every bed range p with p.overlaps(merged)."""
    out = []
    for bi, (_, ranges) in enumerate(beds):
        for (s, e) in ranges:
            if range_overlaps((s, e), merged):
                out.append((bi, s, e))
    return out


def run(chromosome, bcf, bed_files, reference_genome_file, wanted_samples, pwm_file, pwm_threshold_directory,
        pwm_threshold, wanted_pwms, output_file, forward_only=False, run_tabix=False, min_maf=0, threads=1,
        after_position=0, verbose=False, device=0, regions_per_batch=0, devices=None):
    """main.rs:234-393 `run` with the reference's argument order; writes the BGZF VCF.
    devices: list of HIP devices; batch g of merged regions runs on devices[g % n] (same
    text for any list; a device may repeat)."""
    a = _capi.tfbs_run_args()
    keep = [_u(x) if x is not None else None for x in (chromosome, bcf, ",".join(bed_files), reference_genome_file,
                                                        wanted_samples, pwm_file, pwm_threshold_directory,
                                                        ",".join(wanted_pwms), output_file)]
    (a.chromosome, a.bcf, a.bed_files, a.reference, a.samples_file, a.pwm_file, a.pwm_threshold_dir, a.pwm_names,
     a.output) = keep
    a.pwm_threshold = pwm_threshold
    a.forward_only = 1 if forward_only else 0
    a.min_maf = min_maf
    a.threads = threads
    a.after_position = after_position
    a.tabix = 1 if run_tabix else 0
    a.verbose = 1 if verbose else 0
    a.device = device
    a.regions_per_batch = regions_per_batch
    dev = _u(",".join(str(int(d)) for d in devices)) if devices else None
    a.devices = dev
    check(lib().tfbs_run(C.byref(a)))


class BcfReader:
    """Streaming BCF2 reader (f2): IndexedReader::from_path + fetch + records (raw GT).
    fetch() with nondecreasing beg on one contig reads the file once."""

    def __init__(self, path):
        self.h = C.c_void_p()
        check(lib().tfbs_bcf_open(_u(path), C.byref(self.h)))
        n = lib().tfbs_bcf_num_samples(self.h)
        self.samples = [lib().tfbs_bcf_sample_name(self.h, i).decode() for i in range(n)]
        self.selected = list(range(n))
        self.indexed = bool(lib().tfbs_bcf_indexed(self.h))

    def select(self, idx):
        """Decode GT only for these sample indices, in this order."""
        idx = [int(i) for i in idx]
        arr = (C.c_size_t * max(1, len(idx)))(*idx)
        check(lib().tfbs_bcf_select(self.h, arr, len(idx)))
        self.selected = idx

    def set_carriers_mode(self, on=True):
        """Records keep load_diffs' carrier ids (and the ploidy check) instead of raw GT."""
        check(lib().tfbs_bcf_set_carriers_mode(self.h, 1 if on else 0))
        self.carriers_mode = bool(on)

    def __del__(self):
        if getattr(self, "h", None):
            lib().tfbs_bcf_close(self.h)
            self.h = None

    def fetch(self, chrom, beg, end):
        n = C.c_size_t()
        check(lib().tfbs_bcf_fetch(self.h, _u(chrom), beg, end, C.byref(n)))
        out = []
        ns = len(self.selected)
        for i in range(n.value):
            pos, rlen, na = C.c_uint64(), C.c_uint32(), C.c_uint32()
            ref, alt = C.c_char_p(), C.c_char_p()
            gt = _capi.i32p()
            check(lib().tfbs_bcf_record(self.h, i, C.byref(pos), C.byref(rlen), C.byref(na), C.byref(ref),
                                        C.byref(alt), C.byref(gt)))
            rec = {"pos0": pos.value, "rlen": rlen.value, "n_alleles": na.value, "ref": ref.value.decode(),
                   "alt": alt.value.decode() if alt.value is not None else None}
            if getattr(self, "carriers_mode", False):
                ids, nc, st = _capi.u32p(), C.c_size_t(), C.c_int()
                check(lib().tfbs_bcf_record_carriers(self.h, i, C.byref(ids), C.byref(nc), C.byref(st)))
                rec["carriers"] = [ids[k] for k in range(nc.value)]
                rec["gt_status"] = st.value
            else:
                rec["gt"] = [[gt[2 * s], gt[2 * s + 1]] for s in range(ns)]
            out.append(rec)
        return out


def fasta_fetch(path, chrom, start, stop):
    p = C.c_void_p()
    n = C.c_size_t()
    check(lib().tfbs_fasta_fetch(_u(path), _u(chrom), start, stop, C.byref(p), C.byref(n)))
    try:
        return C.string_at(p, n.value).decode()
    finally:
        lib().tfbs_free(p)


def bgzf_write(path, text, flushes=0):
    b = _u(text)
    check(lib().tfbs_bgzf_write_file(_u(path), b, len(b), flushes))


def bgzf_read(path):
    p = C.c_void_p()
    n = C.c_size_t()
    check(lib().tfbs_bgzf_read_file(_u(path), C.byref(p), C.byref(n)))
    try:
        return C.string_at(p, n.value).decode()
    finally:
        lib().tfbs_free(p)


def merge_ranges(ranges):
    n = len(ranges)
    os_, oe = (C.c_uint64 * max(1, n))(), (C.c_uint64 * max(1, n))()
    m = C.c_size_t()
    check(lib().tfbs_merge_ranges((C.c_uint64 * max(1, n))(*[r[0] for r in ranges]),
                                  (C.c_uint64 * max(1, n))(*[r[1] for r in ranges]), n, os_, oe, C.byref(m)))
    return [(os_[i], oe[i]) for i in range(m.value)]
