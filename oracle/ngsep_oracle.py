"""ctypes wrapper of the CPU restatement (oracle/build/libngsep_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libngsep_oracle.so")
MAX_ALLELES = 16


class OracleParams(ctypes.Structure):
    _fields_ = [
        ("min_mq", ctypes.c_int32), ("max_alns_per_start", ctypes.c_int32), ("ignore5", ctypes.c_int32),
        ("ignore3", ctypes.c_int32), ("max_base_qs", ctypes.c_int32), ("min_quality", ctypes.c_int32),
        ("ploidy", ctypes.c_int32), ("process_nonunique", ctypes.c_int32), ("process_secondary", ctypes.c_int32),
        ("ignore_lowercase_ref", ctypes.c_int32), ("call_embedded", ctypes.c_int32),
        ("calc_strand_bias", ctypes.c_int32), ("print_sample_ploidy", ctypes.c_int32),
        ("het_rate_set", ctypes.c_int32), ("het_rate", ctypes.c_double), ("sample_id", ctypes.c_char_p),
        ("query_seq", ctypes.c_char_p), ("query_first", ctypes.c_int32), ("query_last", ctypes.c_int32),
        ("indel_passthrough", ctypes.c_int32), ("known_vcf", ctypes.c_char_p), ("known_strs", ctypes.c_char_p),
    ]


class OracleCounts(ctypes.Structure):
    _fields_ = [
        ("n_alleles", ctypes.c_int), ("f", ctypes.c_int), ("g", ctypes.c_int), ("max_base_qs", ctypes.c_int),
        ("total_count", ctypes.c_int), ("low_bq_count", ctypes.c_int),
        ("counts", ctypes.c_int * MAX_ALLELES), ("counts_strand", (ctypes.c_int * 2) * MAX_ALLELES),
        ("allele_error_log_probs", ctypes.c_double * MAX_ALLELES),
        ("logc", (ctypes.c_double * MAX_ALLELES) * MAX_ALLELES),
    ]


class OracleStats(ctypes.Structure):
    _fields_ = [("alignments_read", ctypes.c_int64), ("alignments_admitted", ctypes.c_int64),
                ("positions_genotyped", ctypes.c_int64), ("variants_called", ctypes.c_int64),
                ("seconds", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        l = ctypes.CDLL(LIB)
        l.ngo_params_default.argtypes = [ctypes.POINTER(OracleParams)]
        l.ngo_counts_init.argtypes = [ctypes.POINTER(OracleCounts), ctypes.c_int, ctypes.c_double, ctypes.c_int]
        l.ngo_counts_update.argtypes = [ctypes.POINTER(OracleCounts), ctypes.c_int, ctypes.c_int, ctypes.c_int]
        l.ngo_counts_posteriors.argtypes = [ctypes.POINTER(OracleCounts), ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
        l.ngo_phred.argtypes = [ctypes.c_double]
        l.ngo_java_round.restype = ctypes.c_int64
        l.ngo_java_round.argtypes = [ctypes.c_double]
        l.ngo_fisher_pvalue.restype = ctypes.c_double
        l.ngo_fisher_pvalue.argtypes = [ctypes.c_int] * 4
        l.ngo_table_error.restype = ctypes.c_double
        l.ngo_table_error.argtypes = [ctypes.c_int, ctypes.c_int]
        l.ngo_table_gt.restype = ctypes.c_double
        l.ngo_table_gt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
        l.ngo_run_ssvd.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                   ctypes.POINTER(OracleParams), ctypes.POINTER(OracleStats)]
        l.ngo_java_fmt2.argtypes = [ctypes.c_double, ctypes.c_char_p, ctypes.c_int]
        l.ngo_population_info.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        l.ngo_run_mvd.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(OracleParams),
                                  ctypes.c_double, ctypes.POINTER(OracleStats)]
        l.ngo_run_coverage.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64),
                                       ctypes.POINTER(OracleStats)]
        l.ngo_run_rac.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, ctypes.POINTER(OracleStats)]
        _lib = l
    return _lib


def params(**kw) -> OracleParams:
    p = OracleParams()
    lib().ngo_params_default(ctypes.byref(p))
    for k, v in kw.items():
        if isinstance(v, str):
            v = v.encode()
        setattr(p, k, v)
    if "het_rate" in kw:
        p.het_rate_set = 1
    return p


def run_ssvd(fasta: str, sam: str, out_vcf: str, dump: str | None = None, **kw) -> OracleStats:
    p = params(**kw)
    st = OracleStats()
    rc = lib().ngo_run_ssvd(fasta.encode(), sam.encode(), out_vcf.encode(), dump.encode() if dump else None,
                            ctypes.byref(p), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle failed rc={rc}")
    return st


def run_mvd(fasta: str, sam: str, out_vcf: str, min_adf: float = 0.0, **kw) -> OracleStats:
    """MultisampleVariantsDetector restatement (discovery/MultisampleVariantsDetector.java:421-693)."""
    p = params(**kw)
    st = OracleStats()
    rc = lib().ngo_run_mvd(fasta.encode(), sam.encode(), out_vcf.encode(), ctypes.byref(p), min_adf, ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle failed rc={rc}")
    return st


def java_fmt2(x: float) -> str:
    buf = ctypes.create_string_buffer(64)
    lib().ngo_java_fmt2(x, buf, 64)
    return buf.value.decode()


def population_info(calls, n_alleles: int) -> str:
    """calls: list of (n_called, [called0, called1], [acn0..acn3])."""
    n = len(calls)
    nc = (ctypes.c_int * max(n, 1))(*[c[0] for c in calls])
    cl = (ctypes.c_int * max(2 * n, 1))(*[x for c in calls for x in (list(c[1]) + [0, 0])[:2]])
    acn = (ctypes.c_int * max(4 * n, 1))(*[x for c in calls for x in (list(c[2]) + [0, 0, 0, 0])[:4]])
    buf = ctypes.create_string_buffer(256)
    lib().ngo_population_info(n, nc, cl, acn, n_alleles, buf, 256)
    return buf.value.decode()


class Counts:
    """CountsHelper restatement (CountsHelper.java:83-251)."""

    def __init__(self, n_alleles: int, het_proportion: float = 0.5, max_base_qs: int = 30):
        self.c = OracleCounts()
        lib().ngo_counts_init(ctypes.byref(self.c), n_alleles, het_proportion, max_base_qs)

    def update(self, allele_idx: int, q: int, negative: bool = False):
        lib().ngo_counts_update(ctypes.byref(self.c), allele_idx, q, int(negative))

    def logc(self, i: int, j: int) -> float:
        return self.c.logc[i][j]

    def posteriors(self, het_rate: float):
        n = self.c.n_alleles
        out = (ctypes.c_double * (n * n))()
        lib().ngo_counts_posteriors(ctypes.byref(self.c), het_rate, out)
        return [[out[i * n + j] for j in range(n)] for i in range(n)]


def run_coverage(fasta: str, sam: str, out_txt: str, min_mq: int = 20, max_coverage: int = 300):
    """CoverageStatisticsCalculator restatement (discovery/CoverageStatisticsCalculator.java:108-216).
    Returns (counts, counts_unique, high, high_unique, stats); counts[i] = positions whose pileup holds i
    alignments, i < max_coverage."""
    c = (ctypes.c_int64 * max_coverage)()
    u = (ctypes.c_int64 * max_coverage)()
    hi, hu = ctypes.c_int64(), ctypes.c_int64()
    st = OracleStats()
    rc = lib().ngo_run_coverage(fasta.encode(), sam.encode(), out_txt.encode(), min_mq, max_coverage, c, u,
                                ctypes.byref(hi), ctypes.byref(hu), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle failed rc={rc}")
    return list(c), list(u), hi.value, hu.value, st


def run_rac(fasta: str, sam: str, out_txt: str, min_rd: int = 10, max_rd: int = 1000, min_bq: int = 20,
            secondary: int = 0) -> OracleStats:
    """RelativeAlleleCountsCalculator restatement (discovery/RelativeAlleleCountsCalculator.java:183-331):
    printResults' text into out_txt."""
    st = OracleStats()
    rc = lib().ngo_run_rac(fasta.encode(), sam.encode(), out_txt.encode(), min_rd, max_rd, min_bq, secondary,
                           ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"oracle failed rc={rc}")
    return st
