"""-knownVariants (SingleSampleVariantsDetector.findSNVS :896-906,
SingleSampleVariantPileupListener.onPileup :158-176 / genotypeVariantSample :361-391,
VariantDiscoverySNVQAlgorithm.genotypeSNV :21-62): the GPU genotypes the input SNVs (a forced-site queue into
KP, no scan) and writes hom-ref / het / hom-alt / undecided records with the input ID and QUAL; the VCF must
equal the oracle's.  The input mixes the simulator's true SNVs, random reference sites, shared positions and
sites without reads."""
import os
import random

import pytest

import ngsep_oracle
import pysynth
from helpers import gpu_params
from ngsepcore_amd import GpuPileupSession, _lib


def _known_vcf(path, syn, fa_truth, seed, n_random=3000):
    """The truth SNVs (alternate kept) + random positions with random alternates, some sharing a position,
    some past the contigs' coverage; IDs and QUALs varied."""
    rng = random.Random(seed)
    contigs = syn.contigs()
    recs = []
    for l in open(fa_truth):
        if l.startswith("#"):
            continue
        f = l.rstrip("\n").split("\t")
        if len(f[3]) == 1 and len(f[4]) == 1:
            recs.append((f[0], int(f[1]), f[3], f[4]))
    for _ in range(n_random):
        name, seq = rng.choice(contigs)
        p = rng.randint(1, len(seq))
        ref = chr(seq[p - 1]).upper()
        if ref not in "ACGT":
            continue
        alt = rng.choice([b for b in "ACGT" if b != ref])
        recs.append((name, p, ref, alt))
        if rng.random() < 0.05:                                  # a second alternate at the same position
            recs.append((name, p, ref, rng.choice([b for b in "ACGT" if b not in (ref, alt)])))
    rng.shuffle(recs)
    with open(path, "w") as o:
        o.write("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        o.write(f"{contigs[0][0]}\t5\tref_only\tA\t.\t.\t.\t.\n")     # reference site: skipped
        for k, (n, p, r, a) in enumerate(recs):
            q = "." if k % 7 == 0 else str(k % 300 + 0.4)
            idv = "." if k % 5 == 0 else f"rs{k}"
            o.write(f"{n}\t{p}\t{idv}\t{r}\t{a}\t{q}\t.\t.\n")
    return len(recs)


@pytest.mark.gpu
@pytest.mark.parametrize("kw,opts", [
    (dict(genome=pysynth.YEAST, n_contigs=2, depth=20, seed=41, snv_rate=2e-3), {}),
    (dict(genome=pysynth.YEAST, n_contigs=2, depth=8, seed=42, snv_rate=3e-3, quality_model=2, noqual_rate=0.01),
     {"min_quality": 20, "ploidy": 1}),
    (dict(genome=pysynth.YEAST, n_contigs=1, contig_first=2, depth=25, seed=43, snv_rate=2e-3), {"window_positions": 25000}),
])
def test_known_variants_vcf_identical(tmp_path, kw, opts):
    syn = pysynth.Synth(**kw)
    base = os.path.join(str(tmp_path), "kv")
    fa, sam, bam = syn.write(base)
    known = os.path.join(str(tmp_path), "known.vcf")
    n = _known_vcf(known, syn, base + "_truth.vcf", kw["seed"])
    syn.close()
    oopts = {k: v for k, v in opts.items() if k != "window_positions"}
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, known_vcf=known, **oopts)
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        s.set_known_variants(known)
        s.processFile(bam, g)
    orec = [l for l in open(o) if not l.startswith("#")]
    grec = [l for l in open(g) if not l.startswith("#")]
    assert len(orec) > n // 2
    assert grec == orec
    gts = {l.split("\t")[9].split(":")[0] for l in grec}
    assert {"0/0", "0/1"} <= gts or {"0", "1"} <= gts


def _known_vcf_indels(path, syn, discovered_vcf, seed, n_random=400):
    """Input records for the indel realigner's fixed events: the INDEL / STR / SNV records a discovery run called
    (alternates kept), random deletions, insertions (one-base REF too), MNPs, two-ALT indels and alleles with N at
    random positions, some sharing a position with another record; INFO TYPE varied (STR sets the pileup's STR flag,
    UND / INDEL / EMBEDDED are kept as the record's type); IDs and QUALs varied."""
    rng = random.Random(seed)
    contigs = dict(syn.contigs())
    recs = []
    for l in open(discovered_vcf):
        if l.startswith("#"):
            continue
        f = l.rstrip("\n").split("\t")
        recs.append((f[0], int(f[1]), f[3], f[4], f[7] if "TYPE=" in f[7] else "."))
    names = list(contigs)
    for _ in range(n_random):
        name = rng.choice(names)
        seq = contigs[name]
        p = rng.randint(2, len(seq) - 20)
        ref = seq[p - 1:p + rng.randint(0, 6)].decode().upper()
        if "N" in ref:
            continue
        kind = rng.random()
        if kind < 0.3 and len(ref) > 1:
            alt = ref[0]
        elif kind < 0.55:
            alt = ref + "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 4)))
        elif kind < 0.7 and len(ref) > 1:
            alt = "".join(rng.choice("ACGT") for _ in range(len(ref)))
            if alt == ref:
                continue
        elif kind < 0.8:
            alt = ref + "A," + ref + "TT"
        elif kind < 0.85:
            alt = ref[0] + "N" * len(ref)
        else:
            alt = ref + "G"
        info = rng.choice([".", "TYPE=STR", "TYPE=INDEL", "TYPE=UND", "TYPE=EMBEDDED", "NS=3;TYPE=STR"])
        recs.append((name, p, ref, alt, info))
        if rng.random() < 0.1:                                     # an SNV at the same first position
            recs.append((name, p, ref[0], rng.choice([b for b in "ACGT" if b != ref[0]]), "."))
    rng.shuffle(recs)
    with open(path, "w") as o:
        o.write("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        for k, (n, p, r, a, i) in enumerate(recs):
            q = "." if k % 7 == 0 else str(k % 300 + 0.4)
            idv = "." if k % 5 == 0 else f"rs{k}"
            o.write(f"{n}\t{p}\t{idv}\t{r}\t{a}\t{q}\t.\t{i}\n")
    return len(recs)


@pytest.mark.gpu
@pytest.mark.parametrize("kw,opts", [
    (dict(genome=pysynth.YEAST, n_contigs=2, depth=20, seed=61, snv_rate=2e-3, indel_rate=4e-4), {}),
    (dict(genome=pysynth.YEAST, n_contigs=1, depth=10, seed=62, snv_rate=3e-3, indel_rate=6e-4, quality_model=2),
     {"min_quality": 20, "ploidy": 1}),
    (dict(genome=pysynth.YEAST, n_contigs=1, contig_first=2, depth=25, seed=63, snv_rate=2e-3, indel_rate=3e-4),
     {"window_positions": 25000}),
])
def test_known_indels_vcf_identical(tmp_path, kw, opts):
    """-knownVariants with indel / MNP inputs on data with indels: the realigner takes the records as its input
    variants (fixed events at their first positions, SingleSampleVariantsDetector.java:897-905; IndelRealigner
    PileupListener.intersectWithVariants :141-157), the known SNVs are genotyped from the realigned alignments and the
    other records by callIndel with the variant given (SingleSampleVariantPileupListener.genotypeVariantSample
    :361-391), every record written with the input's ID, QS and TYPE.  WHOLE VCF equal to the oracle's."""
    syn = pysynth.Synth(**kw)
    base = os.path.join(str(tmp_path), "ki")
    fa, sam, bam = syn.write(base)
    oopts = {k: v for k, v in opts.items() if k != "window_positions"}
    disc = os.path.join(str(tmp_path), "disc.vcf")
    ngsep_oracle.run_ssvd(fa, sam, disc, **oopts)
    known = os.path.join(str(tmp_path), "known.vcf")
    n = _known_vcf_indels(known, syn, disc, kw["seed"])
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, known_vcf=known, **oopts)
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        s.set_known_variants(known)
        s.processFile(bam, g)
        assert not s.carved_regions()
    orec = [l for l in open(o) if not l.startswith("#")]
    grec = [l for l in open(g) if not l.startswith("#")]
    assert len(orec) > n // 2
    assert sum(1 for l in orec if len(l.split("\t")[3]) > 1 or len(l.split("\t")[4]) > 1) > 50
    assert grec == orec


def test_known_variants_refused_types(tmp_path):
    """Multi-allelic SNVs and records that repeat an allele are refused (their genotyping is not in this build), not
    skipped; indels, MNPs and alleles with N are accepted (ABI 9)."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=5, seed=3)
    fa, _, _ = syn.write(os.path.join(str(tmp_path), "r"))
    name = syn.contigs()[0][0]
    syn.close()
    head = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n"
    s = GpuPileupSession(gpu_params())
    s.load_fasta(fa)
    for bad in (f"{name}\t10\t.\tA\tC,G\t.\t.\t.\n", f"{name}\t10\t.\tAC\tA,A\t.\t.\t.\n"):
        known = os.path.join(str(tmp_path), "bad.vcf")
        open(known, "w").write(head + bad)
        with pytest.raises(_lib.NgsepError) as e:
            s.set_known_variants(known)
        assert e.value.code == _lib.NGSEP_E_UNSUPPORTED
    good = os.path.join(str(tmp_path), "good.vcf")
    open(good, "w").write(head + f"{name}\t10\t.\tAC\tA\t.\t.\t.\n{name}\t20\t.\tAT\tGC\t.\t.\t.\n"
                          f"{name}\t30\t.\tA\tN\t.\t.\t.\n{name}\t40\t.\tA\tC\t.\t.\tSVTYPE=DEL\n")
    s.set_known_variants(good)
    s.close()


@pytest.mark.gpu
def test_cleared_known_variants_equal_fresh_discovery(tmp_path):
    """ngsep_set_known_variants(c, NULL) returns the session to discovery: the previous file's records stop being the
    realigner's input variants (no region opened, no event counted by ngsep_clean_cut), so the VCF equals a fresh
    session's -- after a cleared file and after a refused one."""
    kw = dict(genome=pysynth.YEAST, n_contigs=1, depth=15, seed=64, snv_rate=2e-3, indel_rate=4e-4)
    syn = pysynth.Synth(**kw)
    base = os.path.join(str(tmp_path), "kc")
    fa, sam, bam = syn.write(base)
    disc = os.path.join(str(tmp_path), "disc.vcf")
    ngsep_oracle.run_ssvd(fa, sam, disc)
    known = os.path.join(str(tmp_path), "known.vcf")
    _known_vcf_indels(known, syn, disc, kw["seed"])
    name = syn.contigs()[0][0]
    syn.close()
    bad = os.path.join(str(tmp_path), "bad.vcf")
    with open(bad, "w") as o:
        o.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n" + f"{name}\t10\t.\tA\tC,G\t.\t.\t.\n")
    fresh = os.path.join(str(tmp_path), "fresh.vcf")
    with GpuPileupSession(gpu_params()) as s:
        s.load_fasta(fa)
        s.processFile(bam, fresh)
    want = open(fresh).read()
    for second in (None, bad):
        out = os.path.join(str(tmp_path), "again.vcf")
        with GpuPileupSession(gpu_params()) as s:
            s.load_fasta(fa)
            s.set_known_variants(known)
            if second is None:
                s.set_known_variants(None)
            else:
                with pytest.raises(Exception):
                    s.set_known_variants(second)
            s.processFile(bam, out)
        assert open(out).read() == want
