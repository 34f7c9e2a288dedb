"""ctypes declarations for libtfbs_amd.so (include/tfbs_amd.h).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) into
find-tfbs_amd/lib/.  Loading fails loudly if it is missing: there is no
Python or CPU fallback for the scan.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# TFBS_LIB overrides the in-tree build (e.g. a host-AddressSanitizer build of the same sources)
LIB_PATH = os.environ.get("TFBS_LIB") or os.path.join(HERE, "lib", "libtfbs_amd.so")

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i32p = C.POINTER(C.c_int32)
vp = C.c_void_p


class tfbs_pattern_desc(C.Structure):
    _fields_ = [
        ("pattern_id", C.c_uint16),
        ("direction", C.c_uint8),
        ("kind", C.c_uint8),
        ("length", C.c_uint32),
        ("weights", i32p),
        ("min_score", C.c_int32),
        ("name", C.c_char_p),
    ]


class tfbs_plan_stats(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("n_octet_strands", "n_quad_strands", "n_generic_strands",
                                           "n_fast_tiles", "n_fast_units", "n_generic_tiles",
                                           "max_tile_blocks")] + [("lut_bytes", C.c_uint64)] + \
        [(n, C.c_uint32) for n in ("n_mfma_strands", "n_mfma_tiles", "n_mfma_supers")]


class tfbs_mfma_bound(C.Structure):
    _fields_ = [("eligible", C.c_int32), ("q8", C.c_int64), ("t8", C.c_int64), ("scale", C.c_int64),
                ("c", C.c_int64)]


class tfbs_run_args(C.Structure):
    _fields_ = [
        ("chromosome", C.c_char_p), ("bcf", C.c_char_p), ("bed_files", C.c_char_p), ("reference", C.c_char_p),
        ("samples_file", C.c_char_p), ("pwm_file", C.c_char_p), ("pwm_threshold_dir", C.c_char_p),
        ("pwm_names", C.c_char_p), ("output", C.c_char_p), ("pwm_threshold", C.c_float), ("forward_only", C.c_int),
        ("min_maf", C.c_uint32), ("threads", C.c_uint32), ("after_position", C.c_uint64), ("tabix", C.c_int),
        ("verbose", C.c_int), ("device", C.c_int), ("regions_per_batch", C.c_uint32), ("devices", C.c_char_p),
    ]


# (name, restype, argtypes) for every symbol in include/tfbs_amd.h
SIGNATURES = [
    ("tfbs_strerror", C.c_char_p, [C.c_int]),
    ("tfbs_last_error", C.c_char_p, []),
    ("tfbs_version", C.c_char_p, []),
    ("tfbs_patterns_create", C.c_int, [C.POINTER(tfbs_pattern_desc), C.c_size_t, C.POINTER(vp)]),
    ("tfbs_patterns_from_files", C.c_int, [C.c_char_p, C.c_char_p, C.c_float, C.c_char_p, C.c_int, C.POINTER(vp)]),
    ("tfbs_patterns_count", C.c_size_t, [vp]),
    ("tfbs_patterns_get", C.c_int, [vp, C.c_size_t, C.POINTER(tfbs_pattern_desc)]),
    ("tfbs_patterns_name_of", C.c_char_p, [vp, C.c_uint16]),
    ("tfbs_patterns_max_length", C.c_uint32, [vp]),
    ("tfbs_patterns_destroy", None, [vp]),
    ("tfbs_patterns_plan_stats", C.c_int, [vp, C.c_uint32, C.c_int, C.POINTER(tfbs_plan_stats)]),
    ("tfbs_patterns_mfma_bound", C.c_int, [vp, C.c_size_t, C.POINTER(C.c_uint8), C.POINTER(tfbs_mfma_bound)]),
    ("tfbs_parse_weight", C.c_int, [C.c_char_p, i32p]),
    ("tfbs_parse_threshold_file", C.c_int, [C.c_char_p, C.c_float, i32p]),
    ("tfbs_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("tfbs_ctx_create", C.c_int, [C.c_int, vp, C.POINTER(vp)]),
    ("tfbs_ctx_destroy", None, [vp]),
    ("tfbs_ctx_sync", C.c_int, [vp]),
    ("tfbs_ctx_set_host_threads", C.c_int, [vp, C.c_uint32]),
    ("tfbs_ctx_last_scan_ms", C.c_float, [vp]),
    ("tfbs_ctx_last_scan_launches", C.c_int, [vp]),
    ("tfbs_ctx_last_mfma_ms", C.c_float, [vp]),
    ("tfbs_ctx_window_lists", C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_double)]),
    ("tfbs_ctx_scan_counters", C.c_int, [vp, C.POINTER(C.c_uint64)]),
    ("tfbs_matches", C.c_int, [vp, u8p, u64p, C.c_size_t, u32p, u64p, u64p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("tfbs_patch_haplotype", C.c_int, [C.c_uint64, C.c_uint64, C.c_size_t, u64p, u8p, u32p, u8p, u32p, u8p, u64p,
                                       C.c_size_t, u8p, u64p, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("tfbs_batch_create", C.c_int, [vp, C.c_uint32, C.c_int, C.POINTER(vp)]),
    ("tfbs_batch_destroy", None, [vp]),
    ("tfbs_batch_add_bed", C.c_int, [vp, C.c_char_p]),
    ("tfbs_batch_set_window_lmax", C.c_int, [vp, C.c_uint32]),
    ("tfbs_batch_set_build_device", C.c_int, [vp, C.c_int]),
    ("tfbs_batch_build_stats", C.c_int, [vp, u64p, u64p]),
    ("tfbs_batch_patch_stats", C.c_int, [vp, u64p]),
    ("tfbs_batch_region_ext", C.c_int, [vp, C.c_uint64, C.c_uint64, u64p, u64p]),
    ("tfbs_batch_region_begin", C.c_int, [vp, C.c_uint64, C.c_uint64, C.c_char_p, C.c_size_t]),
    ("tfbs_batch_region_add_inner", C.c_int, [vp, C.c_uint32, C.c_uint64, C.c_uint64]),
    ("tfbs_batch_region_add_record_gt", C.c_int, [vp, C.c_uint64, C.c_uint32, C.c_char_p, C.c_char_p, i32p]),
    ("tfbs_batch_region_add_record_carriers", C.c_int, [vp, C.c_uint64, C.c_char_p, C.c_char_p, u32p, C.c_size_t]),
    ("tfbs_batch_region_end", C.c_int, [vp]),
    ("tfbs_batch_num_regions", C.c_size_t, [vp]),
    ("tfbs_batch_num_haplotypes", C.c_size_t, [vp]),
    ("tfbs_batch_num_windows", C.c_uint64, [vp]),
    ("tfbs_batch_num_effective_windows", C.c_uint64, [vp]),
    ("tfbs_batch_num_cell_ops", C.c_uint64, [vp]),
    ("tfbs_batch_num_scan_windows", C.c_uint64, [vp]),
    ("tfbs_batch_num_scan_cell_ops", C.c_uint64, [vp]),
    ("tfbs_batch_input_bytes", C.c_uint64, [vp]),
    ("tfbs_batch_output_bytes", C.c_uint64, [vp]),
    ("tfbs_batch_upload", C.c_int, [vp, vp]),
    ("tfbs_scan", C.c_int, [vp, vp]),
    ("tfbs_batch_download", C.c_int, [vp, vp]),
    ("tfbs_batch_reduce", C.c_int, [vp, vp]),
    ("tfbs_batch_assemble", C.c_int, [vp, vp]),
    ("tfbs_batch_assemble_wait", C.c_int, [vp, vp]),
    ("tfbs_step", C.c_int, [vp, vp]),
    ("tfbs_ctx_last_assemble_ms", C.c_float, [vp]),
    ("tfbs_batch_encode", C.c_int, [vp, vp, C.c_size_t, C.c_size_t]),
    ("tfbs_batch_encode_flags", C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_int]),
    ("tfbs_ctx_rows_bgzf_seconds", C.c_int, [vp, C.POINTER(C.c_double)]),
    ("tfbs_batch_rows_bgzf", C.c_int, [vp, vp, C.c_size_t, C.c_size_t, C.c_char_p, C.c_uint32, u32p, C.c_int,
                                       u64p, u64p, u64p]),
    ("tfbs_batch_region_num_keys", C.c_int, [vp, C.c_size_t, C.POINTER(C.c_size_t)]),
    ("tfbs_batch_region_key", C.c_int, [vp, C.c_size_t, C.c_size_t, u32p, u64p, u64p, u16p, u32p, u32p]),
    ("tfbs_batch_rows", C.c_int, [vp, C.c_char_p, C.c_uint32, u32p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    ("tfbs_batch_region_rows", C.c_int, [vp, C.c_size_t, C.c_char_p, C.c_uint32, u32p, C.POINTER(C.c_void_p),
                                         C.POINTER(C.c_size_t)]),
    ("tfbs_batch_region_digest", C.c_int, [vp, C.c_size_t, u64p]),
    ("tfbs_batch_region_key_digest_sum", C.c_int, [vp, C.c_size_t, u64p]),
    ("tfbs_batch_region_input_digest", C.c_int, [vp, C.c_size_t, u64p]),
    ("tfbs_batch_region_digests", C.c_int, [vp, C.c_size_t, C.c_size_t, C.c_uint32, C.c_uint32, u64p, u64p, u64p]),
    ("tfbs_batch_region_stats", C.c_int, [vp, C.c_size_t, u32p, u32p]),
    ("tfbs_batch_format_rows", C.c_int, [vp, C.c_char_p, C.c_uint32, C.c_uint32, C.c_size_t, C.c_size_t, u64p,
                                         u64p]),
    ("tfbs_batch_prep_seconds", C.c_int, [vp, C.POINTER(C.c_double)]),
    ("tfbs_free", None, [C.c_void_p]),
    ("tfbs_counts_as_genotypes", C.c_int, [u32p, u32p, C.c_size_t, u32p, C.c_char_p, C.c_size_t, C.c_char_p,
                                           C.c_size_t]),
    ("tfbs_run", C.c_int, [C.c_void_p]),
    ("tfbs_bcf_open", C.c_int, [C.c_char_p, C.POINTER(vp)]),
    ("tfbs_inflate_raw", C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]),
    ("tfbs_bcf_close", None, [vp]),
    ("tfbs_bcf_select", C.c_int, [vp, C.POINTER(C.c_size_t), C.c_size_t]),
    ("tfbs_bcf_num_samples", C.c_size_t, [vp]),
    ("tfbs_bcf_indexed", C.c_int, [vp]),
    ("tfbs_bcf_sample_name", C.c_char_p, [vp, C.c_size_t]),
    ("tfbs_bcf_fetch", C.c_int, [vp, C.c_char_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_size_t)]),
    ("tfbs_bcf_set_carriers_mode", C.c_int, [vp, C.c_int]),
    ("tfbs_bcf_record_carriers", C.c_int, [vp, C.c_size_t, C.POINTER(u32p), C.POINTER(C.c_size_t), C.POINTER(C.c_int)]),
    ("tfbs_bcf_record", C.c_int, [vp, C.c_size_t, u64p, u32p, u32p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                  C.POINTER(i32p)]),
    ("tfbs_fasta_fetch", C.c_int, [C.c_char_p, C.c_char_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_void_p),
                                   C.POINTER(C.c_size_t)]),
    ("tfbs_bgzf_write_file", C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t, C.c_int]),
    ("tfbs_bgzf_read_file", C.c_int, [C.c_char_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]),
    ("tfbs_merge_ranges", C.c_int, [u64p, u64p, C.c_size_t, u64p, u64p, C.POINTER(C.c_size_t)]),
    ("tfbs_synth_write_pwms", C.c_int, [C.c_char_p, C.c_uint32, C.c_int, C.c_uint64, C.POINTER(C.c_void_p)]),
    ("tfbs_synth_region_make", C.c_int, [C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                         C.POINTER(vp)]),
    ("tfbs_synth_region_destroy", None, [vp]),
    ("tfbs_synth_region_info", None, [vp, u64p, u64p, u64p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                      C.POINTER(C.c_size_t)]),
    ("tfbs_synth_region_record", None, [vp, C.c_size_t, u64p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                        C.POINTER(u32p), C.POINTER(C.c_size_t)]),
    ("tfbs_synth_fill_batch", C.c_int, [vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]),
]

_lib = None


class TfbsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("%s (%d): %s" % (msg, code, _lib.tfbs_strerror(code).decode() if _lib else "?"))
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("find-tfbs_amd native library missing at %s: run `make` or "
                              "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if rc < 0:
        raise TfbsError(rc, lib().tfbs_last_error().decode(errors="replace"))
    return rc
