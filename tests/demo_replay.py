"""Replay of the reference's own genotype fields through a caller (shared by the CPU and GPU suites).

tests/golden/reference_demo_pl.csv.gz holds every biallelic-SNV genotype field of the reference's output
VCF (training/yeastDemo_ann_q40_s_fi_I2_noREP_noCNV.vcf.gz, MultisampleVariantsDetector, 2 samples) whose
base counts are all REF/ALT: (n_ref, n_alt, ref, alt, PL, DP, GQ, GT).  The VCF carries no base
qualities; the fields consistent with every base at the Q30 cap (10,508) are
replayed here as pileups of 1-bp Q30 reads:

  * one site per distinct (n_ref, n_alt, ref, alt, DP) on contig "demo" (every 4th position);
  * sample S0 = the field: n_ref reads of the reference base, n_alt of the alternative at Q30 ('?'),
    and DP - n_ref - n_alt reads at Q2 ('#'), which CountsHelper counts in DP only (q <= 3,
    CountsHelper.java:210-216);
  * sample S1 = a carrier (20 Q30 reads of the alternative) so that the site is emitted whatever S0's
    genotype (MultisampleVariantsDetector.onPileup, :533);
  * all reads start at the site: the run uses maxAlnsPerStartPos 0 (no cap, AlignmentsPileupGenerator
    .processSameStartAlns :424).

The caller's S0 column (GT:PL:GQ:DP:BSDP) must reproduce the reference's field for every replayed key:
PL through CalledSNV's float log-conditionals and VCFFileWriter's Math.round, GQ through
CountsHelper.getPosteriorProbabilities + VariantDiscoverySNVQAlgorithm.genotypeSNV (:21-97).
"""
from __future__ import annotations

import csv
import gzip
import os

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURE = os.path.join(HERE, "reference_demo_pl.csv.gz")
SPACING = 4
CARRIER = 20


def rows():
    return list(csv.DictReader(gzip.open(FIXTURE, "rt")))


def keys(rs):
    """distinct replay keys in first-seen order"""
    seen, out = set(), []
    for r in rs:
        k = (int(r["n_ref"]), int(r["n_alt"]), int(r["ref_idx"]), int(r["alt_idx"]), int(r["dp"]))
        if k not in seen:
            seen.add(k)
            out.append(k)
    return out


def write(tmpdir, ks):
    """FASTA + coordinate-sorted SAM of the replay; returns (fasta, sam, {position: key})."""
    L = SPACING * (len(ks) + 2)
    ref = bytearray(b"A" * L)
    site = {}
    for i, k in enumerate(ks):
        p = SPACING * (i + 1)
        ref[p - 1] = ord("ACGT"[k[2]])
        site[p] = k
    fa = os.path.join(str(tmpdir), "demo.fa")
    with open(fa, "w") as f:
        f.write(">demo\n")
        for i in range(0, L, 80):
            f.write(ref[i:i + 80].decode() + "\n")
    sam = os.path.join(str(tmpdir), "demo.sam")
    n = 0
    with open(sam, "w") as f:
        f.write(f"@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:demo\tLN:{L}\n@RG\tID:S0\tSM:S0\n@RG\tID:S1\tSM:S1\n")
        for p in sorted(site):
            nr, na, ri, ai, dp = site[p]
            reads = ([("ACGT"[ri], "?", "S0")] * nr + [("ACGT"[ai], "?", "S0")] * na +
                     [("ACGT"[ri], "#", "S0")] * (dp - nr - na) + [("ACGT"[ai], "?", "S1")] * CARRIER)
            for base, q, rg in reads:
                f.write(f"r{n}\t0\tdemo\t{p}\t60\t1M\t*\t0\t0\t{base}\t{q}\tRG:Z:{rg}\n")
                n += 1
    return fa, sam, site


def parse_vcf(path):
    """{position: S0 field dict} of a population VCF (samples S0, S1)."""
    out = {}
    for line in open(path):
        if line.startswith("#"):
            continue
        fs = line.rstrip("\n").split("\t")
        fmt = fs[8].split(":")
        out[int(fs[1])] = dict(zip(fmt, fs[9].split(":")), REF=fs[3], ALT=fs[4])
    return out


def check(rs, site, got):
    """Compares the replayed S0 fields with the reference's fields that the all-Q30 model reproduces.
    Returns (fields checked, mismatches)."""
    by_key = {}
    for p, k in site.items():
        by_key[k] = got.get(p)
    checked, bad = 0, []
    for r in rs:
        k = (int(r["n_ref"]), int(r["n_alt"]), int(r["ref_idx"]), int(r["alt_idx"]), int(r["dp"]))
        g = by_key.get(k)
        if g is None:
            bad.append(("site not emitted", k))
            continue
        pl = f"{r['pl_rr']},{r['pl_ra']},{r['pl_aa']}"
        if g["PL"] != pl:
            continue        # real (non-Q30) base qualities: not reproducible without the reads
        checked += 1
        bsdp = [0, 0, 0, 0]
        bsdp[k[2]] += k[0]
        bsdp[k[3]] += k[1]
        want = {"GQ": r["gq"], "DP": r["dp"], "GT": r["gt"], "BSDP": ",".join(map(str, bsdp))}
        for f, v in want.items():
            if g.get(f) != v:
                bad.append((f, k, g.get(f), v))
    return checked, bad
