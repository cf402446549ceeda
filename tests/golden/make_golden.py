"""Regenerates the committed golden fixtures (run in the build container, not on the GPU box).

1. reference_demo_pl.csv.gz -- data extracted from the reference's own output file
   training/yeastDemo_ann_q40_s_fi_I2_noREP_noCNV.vcf.gz (an NGSEP VCF, 2 samples): every
   biallelic-SNV genotype field whose BSDP holds only REF/ALT base counts, as
   (n_ref, n_alt, ref_idx, alt_idx, PL0, PL1, PL2, DP, GQ, GT).  Needs /root/reference (read only).
2. <case>.vcf / <case>.dump.gz -- outputs of the oracle (CPU restatement) on seeded synthetic
   inputs (tools/synth), plus <case>.sam.md5 pinning the generator's output.  The GPU tests
   compare the HIP path with these files without running the oracle.

3. reference_strs.txt.gz -- data extracted from the reference's own input file training/Saccharomyces_cerevisiae_STRs.txt
   (TRF output over sacCer3): the first three fields of every line (sequence, first, last), the only fields
   SimpleGenomicRegionFileHandler.loadRegions reads for -knownSTRs, in file order with the file's separators.
   Needs /root/reference (read only): python tests/golden/make_golden.py --strs

Usage: python tests/golden/make_golden.py [--no-reference] [--strs]
"""
from __future__ import annotations

import gzip
import hashlib
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools", "synth")):
    if p not in sys.path:
        sys.path.insert(0, p)

REF_VCF = "/root/reference/training/yeastDemo_ann_q40_s_fi_I2_noREP_noCNV.vcf.gz"
REF_STRS = "/root/reference/training/Saccharomyces_cerevisiae_STRs.txt"


def str_fixture(path):
    """the (sequence, first, last) fields of the reference's STR file, space separated as there"""
    n = 0
    with open(REF_STRS) as f, gzip.GzipFile(path, "wb", mtime=0) as g:
        for line in f:
            fl = line.split()
            if len(fl) < 3:
                continue
            g.write((" ".join(fl[:3]) + "\n").encode())
            n += 1
    return n

# name -> (synth kwargs, oracle option kwargs); kept small so the oracle runs in seconds
CASES = {
    "c1_chrI_10x": (dict(genome=0, n_contigs=1, depth=10, seed=1), {}),
    "edge_2contigs_25x": (dict(genome=0, n_contigs=2, depth=25, seed=7, secondary_rate=0.01, lowmq_rate=0.01,
                               noqual_rate=0.005, softclip_rate=0.05, dup_rate=0.02, lower_frac=0.01,
                               quality_model=2, snv_rate=3e-3), {}),
    "edge_2contigs_25x_csb_ploidy1": (dict(genome=0, n_contigs=2, depth=25, seed=7, secondary_rate=0.01,
                                           lowmq_rate=0.01, noqual_rate=0.005, softclip_rate=0.05, dup_rate=0.02,
                                           lower_frac=0.01, quality_model=2, snv_rate=3e-3),
                                      {"calc_strand_bias": 1, "ploidy": 1, "min_quality": 20}),
}
# BASELINE.json configs at full size (the bench workloads): only the md5 and the record count of the oracle's
# VCF are committed (tests/golden/full_sizes.json); the GPU suite regenerates the data on the box and
# compares the HIP VCF byte for byte.  configs[1] = yeast 30x (seed 2), configs[2] = human chr20 30x
# (seed 3, per-contig streams: the bench's chr20 workload); configs[3] = human WGS 30x (seed 4): chr21, one of
# the contigs of the bench's shard 0 of 8 (bench.py --config wgs generates each contig exactly this way)
FULL_CASES = {
    "configs1_yeast_30x": dict(genome=0, depth=30, seed=2),
    "configs2_chr20_30x": dict(genome=1, contig_first=19, n_contigs=1, depth=30, seed=3, rng_per_contig=1),
    "configs3_wgs_chr21_30x": dict(genome=1, contig_first=20, n_contigs=1, depth=30, seed=4, rng_per_contig=1),
    # the other two sequences of the bench's shard 0 of 8 (chr1 + chr15 + chr21): the staged 3-sequence device run
    # of bench.py --config wgs is compared with all three (tests/test_gpu_wgs_shard.py)
    "configs3_wgs_chr15_30x": dict(genome=1, contig_first=14, n_contigs=1, depth=30, seed=4, rng_per_contig=1),
    "configs3_wgs_chr1_30x": dict(genome=1, contig_first=0, n_contigs=1, depth=30, seed=4, rng_per_contig=1),
}
# configs[4] at full size for one GPU's shard: MultisampleVariantsDetector on 200 synthetic yeast samples at 10x,
# chrIV (the bench's --config multisample workload); the oracle's population VCF md5 + record count
FULL_POP_CASES = {
    "configs4_chrIV_200x10x": dict(genome=0, depth=10.0, seed=5, n_samples=200, contig_first=3, n_contigs=1),
    # configs[4]'s shape with a 2 kb collapsed repeat where every sample is ~300x deep (tests/test_gpu_deep_population.py)
    "deep_repeat_200x10x": dict(genome=2, custom_len=16000, depth=10.0, seed=42, n_samples=200, snv_rate=3e-3,
                                hot_first=7001, hot_len=2000, hot_depth=290.0),
}
# CoverageStats (CoverageStatisticsCalculator) fixtures: synth case -> (min_mq, max_coverage)
COVERAGE_CASES = {"edge_2contigs_25x": (20, 300), "c1_chrI_10x": (20, 12)}
DUMP_CASE = ("dump_custom8k_30x", dict(genome=2, custom_len=8000, depth=30, seed=5, noqual_rate=0.01,
                                       softclip_rate=0.05, quality_model=2))


def reference_fixture(out_path: str) -> int:
    rows = []
    with gzip.open(REF_VCF, "rt") as f:
        for line in f:
            if line.startswith("#"):
                continue
            fs = line.rstrip("\n").split("\t")
            ref, alt = fs[3], fs[4]
            if len(ref) != 1 or len(alt) != 1 or ref not in "ACGT" or alt not in "ACGT":
                continue
            fmt = fs[8].split(":")
            ri, ai = "ACGT".index(ref), "ACGT".index(alt)
            for s in fs[9:]:
                d = dict(zip(fmt, s.split(":")))
                if "BSDP" not in d or "PL" not in d or "DP" not in d or "GQ" not in d:
                    continue
                b = [int(x) for x in d["BSDP"].split(",")]
                if sum(b) != b[ri] + b[ai]:
                    continue
                pl = d["PL"].split(",")
                rows.append(f"{b[ri]},{b[ai]},{ri},{ai},{pl[0]},{pl[1]},{pl[2]},{d['DP']},{d['GQ']},{d['GT']}\n")
    with gzip.GzipFile(out_path, "wb", mtime=0) as g:
        g.write(b"n_ref,n_alt,ref_idx,alt_idx,pl_rr,pl_ra,pl_aa,dp,gq,gt\n")
        g.write("".join(rows).encode())
    return len(rows)


def reference_population_fixture(out_path: str) -> int:
    """Biallelic SNV lines of the reference's population VCF: both samples' GT/ACN and the INFO
    fields DiversityStatistics produces (NS, AN, AFS, MAF; this older NGSEP does not print OH)."""
    rows = []
    with gzip.open(REF_VCF, "rt") as f:
        for line in f:
            if line.startswith("#"):
                continue
            fs = line.rstrip("\n").split("\t")
            ref, alt = fs[3], fs[4]
            if len(ref) != 1 or len(alt) != 1 or ref not in "ACGT" or alt not in "ACGT":
                continue
            info = dict(kv.split("=", 1) for kv in fs[7].split(";") if "=" in kv)
            if not all(k in info for k in ("NS", "AN", "AFS", "MAF")):
                continue
            fmt = fs[8].split(":")
            cols = []
            for smp in fs[9:]:
                d = dict(zip(fmt, smp.split(":")))
                cols += [d.get("GT", "."), d.get("ACN", ".").replace(",", "|")]
            rows.append(",".join(cols + [info["NS"], info["AN"], info["AFS"].replace(",", "|"), info["MAF"]]) + "\n")
    with gzip.GzipFile(out_path, "wb", mtime=0) as g:
        g.write(b"gt0,acn0,gt1,acn1,ns,an,afs,maf\n")
        g.write("".join(rows).encode())
    return len(rows)


def md5(path: str) -> str:
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def oracle_fixtures():
    import ngsep_oracle
    import pysynth
    with tempfile.TemporaryDirectory() as d:
        for name, (skw, opts) in CASES.items():
            syn = pysynth.Synth(**skw)
            fa, sam, _ = syn.write(os.path.join(d, name))
            syn.close()
            ngsep_oracle.run_ssvd(fa, sam, os.path.join(HERE, name + ".vcf"), **opts)
            open(os.path.join(HERE, name + ".sam.md5"), "w").write(md5(sam) + "\n")
            print(name, "ok")
        name, skw = DUMP_CASE
        syn = pysynth.Synth(**skw)
        fa, sam, _ = syn.write(os.path.join(d, name))
        syn.close()
        dump = os.path.join(d, name + ".dump")
        ngsep_oracle.run_ssvd(fa, sam, os.path.join(d, name + ".vcf"), dump)
        with open(dump, "rb") as f, gzip.GzipFile(os.path.join(HERE, name + ".dump.gz"), "wb", mtime=0) as g:
            g.write(f.read())
        open(os.path.join(HERE, name + ".sam.md5"), "w").write(md5(sam) + "\n")
        print(name, "ok")
        for name, (min_mq, max_cov) in COVERAGE_CASES.items():
            skw, _ = CASES[name]
            syn = pysynth.Synth(**skw)
            fa, sam, _ = syn.write(os.path.join(d, name))
            syn.close()
            ngsep_oracle.run_coverage(fa, sam, os.path.join(HERE, name + ".coverage.txt"), min_mq=min_mq,
                                      max_coverage=max_cov)
            print(name, "coverage ok")


def full_size_fixtures(names=None):
    """oracle VCF md5 + record count (+ SAM md5 pinning the generator) of the full-size configs"""
    import json
    import time
    import ngsep_oracle
    import pysynth
    path = os.path.join(HERE, "full_sizes.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("NGSEP_GOLDEN_TMP")) as d:
        for name, skw in FULL_CASES.items():
            if names and name not in names:
                continue
            t = time.time()
            syn = pysynth.Synth(**skw)
            fa, sam, _ = syn.write(os.path.join(d, name))
            syn.close()
            vcf = os.path.join(d, name + ".vcf")
            st = ngsep_oracle.run_ssvd(fa, sam, vcf)
            n = sum(1 for l in open(vcf) if not l.startswith("#"))
            out[name] = {"synth": skw, "sam_md5": md5(sam), "vcf_md5": md5(vcf), "vcf_records": n,
                         "positions_genotyped": st.positions_genotyped, "oracle_seconds": round(st.seconds, 1)}
            with gzip.GzipFile(os.path.join(HERE, name + ".vcf.gz"), "wb", mtime=0) as g:
                g.write(open(vcf, "rb").read())
            print(name, out[name], f"{time.time() - t:.0f}s", flush=True)
            for f in (fa, sam, vcf, os.path.join(d, name + ".bam"), os.path.join(d, name + ".bam.bai")):
                if os.path.exists(f):
                    os.remove(f)
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)


def full_size_population_fixtures(names=None):
    """oracle population VCF md5 + record count of the full-size multisample shard (tests/golden/full_sizes_pop.json)"""
    import json
    import time
    import ngsep_oracle
    import pysynth
    path = os.path.join(HERE, "full_sizes_pop.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    with tempfile.TemporaryDirectory(dir=os.environ.get("NGSEP_GOLDEN_TMP")) as d:
        for name, skw in FULL_POP_CASES.items():
            if names and name not in names:
                continue
            t = time.time()
            syn = pysynth.Synth(**skw)
            fa, sam, _ = syn.write(os.path.join(d, name))
            syn.close()
            vcf = os.path.join(d, name + ".vcf")
            st = ngsep_oracle.run_mvd(fa, sam, vcf, 0.0)
            n = sum(1 for l in open(vcf) if not l.startswith("#"))
            out[name] = {"synth": skw, "sam_md5": md5(sam), "vcf_md5": md5(vcf), "vcf_records": n,
                         "positions_genotyped": st.positions_genotyped, "oracle_seconds": round(st.seconds, 1)}
            with gzip.GzipFile(os.path.join(HERE, name + ".vcf.gz"), "wb", mtime=0) as g:
                g.write(open(vcf, "rb").read())
            print(name, out[name], f"{time.time() - t:.0f}s", flush=True)
            for f in os.listdir(d):
                os.remove(os.path.join(d, f))
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    if "--strs" in sys.argv:
        print("reference STR rows:", str_fixture(os.path.join(HERE, "reference_strs.txt.gz")))
        sys.exit(0)
    if "--full-pop" in sys.argv:
        full_size_population_fixtures([a for a in sys.argv[2:] if not a.startswith("-")] or None)
        sys.exit(0)
    if "--full" in sys.argv:
        full_size_fixtures([a for a in sys.argv[2:] if not a.startswith("-")] or None)
        sys.exit(0)
    if "--no-reference" not in sys.argv:
        n = reference_fixture(os.path.join(HERE, "reference_demo_pl.csv.gz"))
        print("reference fixture rows:", n)
        n = reference_population_fixture(os.path.join(HERE, "reference_demo_population.csv.gz"))
        print("reference population rows:", n)
    oracle_fixtures()
