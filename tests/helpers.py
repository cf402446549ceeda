"""Shared helpers for the parity tests: data generation, oracle runs, VCF comparison."""
from __future__ import annotations

import os

import ngsep_oracle
import pysynth

from ngsepcore_amd import GpuPileupSession, default_params

OPTION_MAP = {  # GPU ngsep_params field -> oracle params field (same meaning)
    "min_mq": "min_mq", "max_alns_per_start": "max_alns_per_start", "ignore5": "ignore5",
    "ignore3": "ignore3", "max_base_qs": "max_base_qs", "min_quality": "min_quality", "ploidy": "ploidy",
    "process_nonunique": "process_nonunique", "process_secondary": "process_secondary",
    "ignore_lowercase_ref": "ignore_lowercase_ref", "calc_strand_bias": "calc_strand_bias",
    "print_sample_ploidy": "print_sample_ploidy", "het_rate": "het_rate", "query_seq": "query_seq",
    "query_first": "query_first", "query_last": "query_last", "sample_id": "sample_id",
    "call_embedded": "call_embedded", "indel_passthrough": "indel_passthrough",
}


def gpu_params(**kw):
    p = default_params()
    for k, v in kw.items():
        if isinstance(v, str):
            v = v.encode()
        setattr(p, k, v)
        if k == "het_rate":
            p.het_rate_set = 1
    return p


def make_data(tmpdir, name="d", **synth_kw):
    syn = pysynth.Synth(**synth_kw)
    fa, sam, bam = syn.write(os.path.join(str(tmpdir), name))
    return syn, fa, sam, bam


def oracle_vcf(tmpdir, fa, sam, name="oracle", dump=False, **opts):
    out = os.path.join(str(tmpdir), name + ".vcf")
    dpath = os.path.join(str(tmpdir), name + ".dump") if dump else None
    st = ngsep_oracle.run_ssvd(fa, sam, out, dpath, **{OPTION_MAP[k]: v for k, v in opts.items()})
    return out, dpath, st


def gpu_vcf_bam(tmpdir, fa, bam, name="gpu", **opts):
    out = os.path.join(str(tmpdir), name + ".vcf")
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        s.processFile(bam, out)
        st = s.stats()
    return out, st


def vcf_records(path):
    return [l.rstrip("\n") for l in open(path) if not l.startswith("#")]


def diff_vcf(a_path, b_path, limit=10):
    a, b = open(a_path).read().splitlines(), open(b_path).read().splitlines()
    out = []
    if len(a) != len(b):
        out.append(f"line counts differ: {len(a)} vs {len(b)}")
    sa, sb = set(a), set(b)
    for l in a:
        if l not in sb:
            out.append("only oracle: " + l)
            if len(out) > limit:
                break
    for l in b:
        if l not in sa:
            out.append("only gpu:    " + l)
            if len(out) > 2 * limit:
                break
    if not out and a != b:   # same lines, different order or multiplicity
        i = next(k for k in range(min(len(a), len(b))) if a[k] != b[k])
        out.append(f"record order differs at line {i + 1}: {a[i]!r} vs {b[i]!r}")
    return out


def read_dump(path):
    """oracle per-position dump: seq, pos, ref, DP, counts, 10 log-conditionals (upper triangle)."""
    rows = {}
    for l in open(path):
        f = l.rstrip("\n").split("\t")
        rows[(f[0], int(f[1]))] = (int(f[3]), tuple(int(x) for x in f[4].split(",")), tuple(float(x) for x in f[5:15]))
    return rows


def oracle_params_from(opts):
    """GPU option names -> oracle parameter names (same meaning)."""
    return {OPTION_MAP[k]: v for k, v in opts.items()}
