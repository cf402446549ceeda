"""ctypes binding of libngsep_amd.so (include/ngsep_gpu.h).

The library is the product: HIP kernels for gfx950 behind a C ABI.  Loading fails loudly
when the shared object is missing -- there is no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
ABI_VERSION = 12                                   # NGSEP_ABI_VERSION (include/ngsep_gpu.h)
DEFAULT_LIB_PATH = os.path.join(_HERE, "lib", "libngsep_amd.so")
# NGSEP_LIB_PATH: an A/B tuning build of the same ABI, for measurements only.  It is announced on stderr when taken, and
# bench.py records it in its line (config.lib_path), so no result can come from a swapped library silently.
LIB_PATH = os.environ.get("NGSEP_LIB_PATH") or DEFAULT_LIB_PATH
if LIB_PATH != DEFAULT_LIB_PATH:
    import sys
    print(f"ngsepcore_amd: NGSEP_LIB_PATH overrides the library: {LIB_PATH}", file=sys.stderr, flush=True)

NGSEP_OK = 0
NGSEP_E_INVALID = -1
NGSEP_E_IO = -2
NGSEP_E_FORMAT = -3
NGSEP_E_DEVICE = -4
NGSEP_E_UNSUPPORTED = -5


class NgsepParams(ctypes.Structure):
    _fields_ = [
        ("min_mq", ctypes.c_int32),
        ("max_alns_per_start", ctypes.c_int32),
        ("ignore5", ctypes.c_int32),
        ("ignore3", ctypes.c_int32),
        ("max_base_qs", ctypes.c_int32),
        ("min_quality", ctypes.c_int32),
        ("ploidy", ctypes.c_int32),
        ("process_nonunique", ctypes.c_int32),
        ("process_secondary", ctypes.c_int32),
        ("ignore_lowercase_ref", ctypes.c_int32),
        ("call_embedded", ctypes.c_int32),
        ("calc_strand_bias", ctypes.c_int32),
        ("print_sample_ploidy", ctypes.c_int32),
        ("het_rate_set", ctypes.c_int32),
        ("het_rate", ctypes.c_double),
        ("query_first", ctypes.c_int32),
        ("query_last", ctypes.c_int32),
        ("query_seq", ctypes.c_char * 256),
        ("sample_id", ctypes.c_char * 256),
        ("prune_candidates", ctypes.c_int32),
        ("dump_all_positions", ctypes.c_int32),
        ("window_positions", ctypes.c_int32),
        ("multisample", ctypes.c_int32),
        ("min_allele_depth_freq", ctypes.c_double),
        ("coverage_stats", ctypes.c_int32),
        ("max_coverage", ctypes.c_int32),
        ("relative_allele_counts", ctypes.c_int32),
        ("rac_min_rd", ctypes.c_int32),
        ("rac_min_bq", ctypes.c_int32),
        ("full_records", ctypes.c_int32),
        ("indel_passthrough", ctypes.c_int32),
    ]


P = ctypes.POINTER


class NgsepReadBatch(ctypes.Structure):
    _fields_ = [
        ("n_reads", ctypes.c_int64),
        ("seq_id", P(ctypes.c_int32)),
        ("first", P(ctypes.c_int32)),
        ("flags", P(ctypes.c_int32)),
        ("read_group", P(ctypes.c_int32)),
        ("cigar_off", P(ctypes.c_int64)),
        ("cigar_n", P(ctypes.c_int32)),
        ("cigar", P(ctypes.c_int32)),
        ("seq_off", P(ctypes.c_int64)),
        ("seq_len", P(ctypes.c_int32)),
        ("bases", ctypes.c_char_p),
        ("quals", ctypes.c_char_p),
        ("has_quals", P(ctypes.c_uint8)),
    ]


class NgsepSiteOut(ctypes.Structure):
    _fields_ = [
        ("seq_id", ctypes.c_int32),
        ("pos", ctypes.c_int32),
        ("ref", ctypes.c_int8),
        ("n_alleles", ctypes.c_int8),
        ("alt", ctypes.c_int8),
        ("third", ctypes.c_int8),
        ("genotype", ctypes.c_int8),
        ("strand_bias", ctypes.c_int8),
        ("gq", ctypes.c_int16),
        ("qual", ctypes.c_int16),
        ("is_call", ctypes.c_int8), ("pool", ctypes.c_uint8),
        ("dp", ctypes.c_int32),
        ("counts", ctypes.c_int32 * 4),
        ("strand_counts", (ctypes.c_int32 * 2) * 4),
        ("logc", ctypes.c_double * 10),
    ]


class NgsepPopSiteOut(ctypes.Structure):
    _fields_ = [
        ("seq_id", ctypes.c_int32),
        ("pos", ctypes.c_int32),
        ("n_alleles", ctypes.c_int8),
        ("alleles", ctypes.c_int8 * 4),
        ("multisnv_type", ctypes.c_int8),
        ("qual", ctypes.c_int16),
        ("pad", ctypes.c_int16),
    ]


class NgsepSampleCall(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int8),
        ("n_called", ctypes.c_int8),
        ("called", ctypes.c_int8 * 2),
        ("gq", ctypes.c_int16),
        ("total_cn", ctypes.c_int16),
        ("dp", ctypes.c_int32),
        ("counts", ctypes.c_int32 * 4),
        ("acn", ctypes.c_int16 * 4),
        ("pl", ctypes.c_int32 * 10),
    ]


class NgsepStats(ctypes.Structure):
    _fields_ = [
        ("alignments_in", ctypes.c_int64),
        ("alignments_admitted", ctypes.c_int64),
        ("positions_genotyped", ctypes.c_int64),
        ("candidates", ctypes.c_int64),
        ("sites_called", ctypes.c_int64),
        ("read_bases", ctypes.c_int64),
        ("slot_bytes", ctypes.c_int64),
        ("kernel_ms", ctypes.c_double),
        ("scan_ms", ctypes.c_double),
        ("genotype_ms", ctypes.c_double),
        ("tile_positions", ctypes.c_int32),
        ("tile_rows_max", ctypes.c_int32),
        ("slot_size", ctypes.c_int32),
        ("hard_sites", ctypes.c_int32),
        ("pile_bytes", ctypes.c_int64),
        ("exact_bound_passes", ctypes.c_int64),
        ("global_positions", ctypes.c_int64),
        ("n_tiles", ctypes.c_int64),
        ("layout_ms", ctypes.c_double),
        ("upload_ms", ctypes.c_double),
        ("carved_positions", ctypes.c_int64),
        ("other_allele_calls", ctypes.c_int64),
        ("realign_ms", ctypes.c_double),         # ABI 10
        ("realign_regions", ctypes.c_int64),
        ("keep_raw_ms", ctypes.c_double),
        ("region_setup_ms", ctypes.c_double),
        ("region_device_ms", ctypes.c_double),
        ("region_merge_ms", ctypes.c_double),
        ("window_wait_ms", ctypes.c_double),
        ("region_gather_ms", ctypes.c_double),
    ]


# exported symbols and their signatures (kept in sync with include/ngsep_gpu.h)
_CTX = ctypes.c_void_p
SIGNATURES = {
    "ngsep_abi_version": (ctypes.c_int, []),
    "ngsep_params_default": (None, [P(NgsepParams)]),
    "ngsep_open": (ctypes.c_int, [ctypes.c_int, P(NgsepParams), P(_CTX)]),
    "ngsep_close": (ctypes.c_int, [_CTX]),
    "ngsep_last_error": (ctypes.c_char_p, [_CTX]),
    "ngsep_get_stats": (ctypes.c_int, [_CTX, P(NgsepStats)]),
    "ngsep_device_count": (ctypes.c_int, []),
    "ngsep_set_reference": (ctypes.c_int, [_CTX, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64]),
    "ngsep_load_fasta": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_n_sequences": (ctypes.c_int, [_CTX]),
    "ngsep_sequence_name": (ctypes.c_char_p, [_CTX, ctypes.c_int]),
    "ngsep_process_alignments": (ctypes.c_int, [_CTX, P(NgsepReadBatch)]),
    "ngsep_notify_end": (ctypes.c_int, [_CTX]),
    "ngsep_fetch_sites": (ctypes.c_int, [_CTX, P(NgsepSiteOut), ctypes.c_int64, P(ctypes.c_int64)]),
    "ngsep_clear_sites": (ctypes.c_int, [_CTX]),
    "ngsep_write_vcf_header": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_append_vcf_records": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_format_site": (ctypes.c_int64, [_CTX, P(NgsepSiteOut), ctypes.c_char_p, ctypes.c_int64]),
    "ngsep_site_vcf_line": (ctypes.c_int64, [_CTX, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]),
    "ngsep_population_site_vcf_line": (ctypes.c_int64, [_CTX, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int64]),
    "ngsep_call_bam": (ctypes.c_int, [_CTX, ctypes.c_char_p, ctypes.c_char_p]),
    "ngsep_set_samples": (ctypes.c_int, [_CTX, ctypes.c_int32, P(ctypes.c_char_p), ctypes.c_int32, P(ctypes.c_int32),
                                         P(ctypes.c_int32)]),
    "ngsep_fetch_population_sites": (ctypes.c_int, [_CTX, P(NgsepPopSiteOut), P(NgsepSampleCall), ctypes.c_int64,
                                                    P(ctypes.c_int64)]),
    "ngsep_write_population_vcf": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_submit_staged": (ctypes.c_int, [_CTX]),
    "ngsep_collect_staged": (ctypes.c_int, [_CTX, P(ctypes.c_double)]),
    "ngsep_call_population_bams": (ctypes.c_int, [_CTX, P(ctypes.c_char_p), ctypes.c_int32, ctypes.c_char_p]),
    "ngsep_call_population_region_bams": (ctypes.c_int, [_CTX, P(ctypes.c_char_p), ctypes.c_int32, ctypes.c_char_p,
                                                          ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p]),
    "ngsep_bam_open": (ctypes.c_int, [_CTX, ctypes.c_char_p, P(ctypes.c_void_p)]),
    "ngsep_bam_next_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, P(NgsepReadBatch)]),
    "ngsep_bam_close": (ctypes.c_int, [ctypes.c_void_p]),
    "ngsep_bgzf_inflate": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                          ctypes.POINTER(ctypes.c_int64)]),
    "ngsep_fetch_carved_regions": (ctypes.c_int, [_CTX, P(ctypes.c_int32), P(ctypes.c_int64), P(ctypes.c_int64), ctypes.c_int64, P(ctypes.c_int64)]),
    "ngsep_clear_carved_regions": (ctypes.c_int, [_CTX]),
    "ngsep_bam_set_region": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64]),
    "ngsep_call_region_bam": (ctypes.c_int, [_CTX, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_char_p]),
    "ngsep_clean_cut": (ctypes.c_int, [_CTX, P(ctypes.c_char_p), ctypes.c_int32, ctypes.c_char_p, ctypes.c_int64, P(ctypes.c_int64),
                                       P(ctypes.c_int64)]),
    "ngsep_call_bam_multi": (ctypes.c_int, [P(_CTX), ctypes.c_int32, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int64]),
    "ngsep_call_population_bams_multi": (ctypes.c_int, [P(_CTX), ctypes.c_int32, P(ctypes.c_char_p), ctypes.c_int32,
                                                        ctypes.c_char_p, ctypes.c_int64]),
    "ngsep_plan_windows": (ctypes.c_int, [_CTX, P(ctypes.c_char_p), ctypes.c_int32, ctypes.c_int64, P(ctypes.c_int32),
                                          P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_int64), ctypes.c_int64,
                                          P(ctypes.c_int64)]),
    "ngsep_stage_alignments": (ctypes.c_int, [_CTX, P(NgsepReadBatch)]),
    "ngsep_stage_finish": (ctypes.c_int, [_CTX]),
    "ngsep_run_staged": (ctypes.c_int, [_CTX, P(ctypes.c_double)]),
    "ngsep_release_staged": (ctypes.c_int, [_CTX]),
    "ngsep_fetch_coverage": (ctypes.c_int, [_CTX, P(ctypes.c_int64), P(ctypes.c_int64), P(ctypes.c_int64),
                                            P(ctypes.c_int64)]),
    "ngsep_write_coverage": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_clear_coverage": (ctypes.c_int, [_CTX]),
    "ngsep_coverage_bam": (ctypes.c_int, [_CTX, ctypes.c_char_p, ctypes.c_char_p]),
    "ngsep_rac_bam": (ctypes.c_int, [_CTX, ctypes.c_char_p, ctypes.c_char_p]),
    "ngsep_set_known_variants": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_set_known_strs": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_fetch_rac": (ctypes.c_int, [_CTX, P(ctypes.c_double), P(ctypes.c_double), P(ctypes.c_double)]),
    "ngsep_write_rac": (ctypes.c_int, [_CTX, ctypes.c_char_p]),
    "ngsep_clear_rac": (ctypes.c_int, [_CTX]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Loads libngsep_amd.so; raises if it was not built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the MI355X HIP extension is required; there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.ngsep_abi_version() != ABI_VERSION:     # the structures above are this ABI's (include/ngsep_gpu.h)
        raise RuntimeError(f"{LIB_PATH} implements ABI {lib.ngsep_abi_version()}, this package ABI {ABI_VERSION}: rebuild it")
    _lib = lib
    return lib


class NgsepError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ngsep error {code}: {msg}")
        self.code = code
