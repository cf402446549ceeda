"""Ploidy >= 3: the pool algorithm (SingleSampleVariantPileupListener.discoverSNV's
pool branch :238-254, createSNVVariantPool :297-332, genotypeVariantPool :402-503) on the GPU (KT's
candidate test + k_posterior_pool) must write the oracle's VCF byte for byte: discovery with multi-allelic
sites kept or re-genotyped as biallelic, -knownVariants (genotypeVariantSample :361-391), streamed windows.
The pooled data carry SNVs at allele counts k/H over H donor haplotypes, some with two alternatives.
Parity against the reference itself is unpinned (no pool output ships with the reference); the shared
CountsHelper tables are pinned by tests/test_golden.py."""
import os

import pytest

import ngsep_oracle
import pool_data
import pysynth
from helpers import gpu_params
from ngsepcore_amd import GpuPileupSession


def _records(path):
    return [l for l in open(path) if not l.startswith("#")]


def _run_gpu(fa, bam, out, known=None, **opts):
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        if known:
            s.set_known_variants(known)
        s.processFile(bam, out)


@pytest.mark.gpu
@pytest.mark.parametrize("ploidy,opts,data", [
    (3, {}, dict(seed=11)),
    (4, {}, dict(seed=12, haplotypes=4)),
    (6, {"min_quality": 20}, dict(seed=13, haplotypes=12, depth=80)),
    (10, {"het_rate": 0.05}, dict(seed=14, haplotypes=10)),
    (64, {}, dict(seed=15, haplotypes=16, depth=120)),
    (4, {"window_positions": 9000, "max_base_qs": 25}, dict(seed=16)),
])
def test_pool_discovery_vcf_identical(tmp_path, ploidy, opts, data):
    fa, sam, bam = pool_data.write_pool(os.path.join(str(tmp_path), "pool"), **data)
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, ploidy=ploidy, **{k: v for k, v in opts.items() if k != "window_positions"})
    g = os.path.join(str(tmp_path), "g.vcf")
    _run_gpu(fa, bam, g, ploidy=ploidy, **opts)
    orec, grec = _records(o), _records(g)
    assert len(orec) > 50
    assert any("TYPE=MULTISNV" in l for l in orec) or ploidy >= 10
    assert grec == orec
    assert open(g).read() == open(o).read()


@pytest.mark.gpu
def test_pool_on_diploid_synth_vcf_identical(tmp_path):
    """The simulator's diploid genomes called as tetraploid pools (hom-alt and 0.5 heterozygous sites)."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=30, seed=17)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, ploidy=4)
    g = os.path.join(str(tmp_path), "g.vcf")
    _run_gpu(fa, bam, g, ploidy=4)
    assert len(_records(o)) > 100
    assert open(g).read() == open(o).read()


@pytest.mark.gpu
@pytest.mark.parametrize("ploidy", [3, 8])
def test_pool_known_variants_vcf_identical(tmp_path, ploidy):
    """-knownVariants with the pool algorithm: every input SNV genotyped (undecided below ploidy reads or
    below -minQuality), FORMAT with BSDP, the input's ID and QUAL."""
    fa, sam, bam = pool_data.write_pool(os.path.join(str(tmp_path), "pool"), seed=20 + ploidy)
    disc = os.path.join(str(tmp_path), "disc.vcf")
    ngsep_oracle.run_ssvd(fa, sam, disc, ploidy=ploidy)
    known = os.path.join(str(tmp_path), "known.vcf")
    seqs = [l[1:].strip() for l in open(fa) if l.startswith(">")]
    with open(known, "w") as k:
        k.write("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        n = 0
        for l in _records(disc):
            f = l.split("\t")
            for a in f[4].split(","):
                k.write(f"{f[0]}\t{f[1]}\tv{n}\t{f[3]}\t{a}\t{n % 90}\t.\t.\n")
                n += 1
        ref = {}
        name = None
        for l in open(fa):
            if l.startswith(">"):
                name = l[1:].strip()
                ref[name] = []
            else:
                ref[name].append(l.strip())
        for s in seqs:
            r = "".join(ref[s])
            for p in range(101, len(r), 997):                     # reference-only sites: hom-ref / undecided
                alt = "C" if r[p - 1] != "C" else "G"
                k.write(f"{s}\t{p}\tr{p}\t{r[p - 1]}\t{alt}\t.\t.\t.\n")
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, ploidy=ploidy, known_vcf=known)
    g = os.path.join(str(tmp_path), "g.vcf")
    _run_gpu(fa, bam, g, known=known, ploidy=ploidy)
    orec = _records(o)
    assert len(orec) > 100
    gts = {l.split("\t")[9].split(":")[0] for l in orec}
    assert {"0/0", "0/1"} <= gts
    assert _records(g) == orec


@pytest.mark.gpu
@pytest.mark.parametrize("ploidy,n_samples,opts", [
    (4, 6, {}),
    (3, 12, {"min_allele_depth_freq": 0.05}),
    (8, 4, {"min_quality": 20}),
])
def test_pool_population_vcf_identical(tmp_path, ploidy, n_samples, opts):
    """MultisampleVariantsDetector with -ploidy >= 3: every sample genotyped by genotypeVariantPool
    (genotypeVariantSample :368-371, setAllCounts, makeUndecided below 40), the multi-allelic shrink loop,
    the variant QS and INFO from the pool calls (KTM without the SNVQ bound + KPM's pool branch); one BAM
    holding every sample's read group, as ngsep_call_population_bams reads it."""
    from ngsepcore_amd import MultisampleVariantsDetector
    samples = [f"P{k:02d}" for k in range(n_samples)]
    fa, sam, bam = pool_data.write_pool(os.path.join(str(tmp_path), "pop"), seed=30 + ploidy, depth=25.0 * n_samples,
                                        haplotypes=ploidy, rg_samples=samples, length=30000)
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, opts.get("min_allele_depth_freq", 0.0), ploidy=ploidy,
                         **{k: v for k, v in opts.items() if k != "min_allele_depth_freq"})
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setNormalPloidy(ploidy)
    if "min_allele_depth_freq" in opts:
        d.setMinAlleleDepthFrequency(opts["min_allele_depth_freq"])
    if "min_quality" in opts:
        d.setMinQuality(opts["min_quality"])
    d.setOutFilename(os.path.join(str(tmp_path), "g.vcf"))
    d.run([bam])
    orec = _records(o)
    assert len(orec) > 30
    assert _records(d.outFilename) == orec


@pytest.mark.gpu
@pytest.mark.parametrize("ploidy,kw,opts", [
    (4, dict(depth=40, seed=81, indel_rate=6e-4, snv_rate=3e-3), {}),
    (3, dict(depth=30, seed=82, indel_rate=4e-4, snv_rate=3e-3), {"call_embedded": 1}),
    (6, dict(depth=50, seed=83, indel_rate=5e-4, snv_rate=2e-3, quality_model=2), {"window_positions": 40000, "min_quality": 20}),
])
def test_pool_indel_regions_vcf_identical(tmp_path, ploidy, kw, opts):
    """The indel realigner at ploidy >= 3 (its listener chain has no ploidy limit, SingleSampleVariantsDetector.java
    :919-925): the pool algorithm's indel branch over the realigner's spans (discoverIndel :275-296, createIndelVariantPool
    :333-338, genotypeVariantPool over the indel alleles :402-503), the pool SNV fallback and the realigned alignments'
    SNVs on the device (k_posterior_pool over the replayed columns).  WHOLE VCF equal to the oracle's."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, **kw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "pi"))
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, ploidy=ploidy, **{k: v for k, v in opts.items() if k != "window_positions"})
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params(ploidy=ploidy, **opts)) as s:
        s.load_fasta(fa)
        s.processFile(bam, g)
        assert s.carved_regions() == []
    orec, grec = _records(o), _records(g)
    assert sum(1 for l in orec if len(l.split("\t")[3]) > 1 or "," in l.split("\t")[4] or len(l.split("\t")[4]) > 1) > 5
    assert grec == orec


@pytest.mark.gpu
@pytest.mark.parametrize("ploidy", [4])
def test_pool_known_indels_vcf_identical(tmp_path, ploidy):
    """-knownVariants at ploidy >= 3 with indel / MNP inputs: genotypeVariantPool over each record's alleles
    (genotypeVariantSample :378-379), makeUndecided below -minQuality, the copy numbers genotypeVariantPool set -- except
    for a sequence's first record, which intersectVariantsCNVs recomputes from the counts (:969-991)."""
    from test_gpu_known import _known_vcf_indels
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=40, seed=84, indel_rate=5e-4, snv_rate=3e-3)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "pk"))
    disc = os.path.join(str(tmp_path), "disc.vcf")
    ngsep_oracle.run_ssvd(fa, sam, disc, ploidy=ploidy)
    known = os.path.join(str(tmp_path), "known.vcf")
    n = _known_vcf_indels(known, syn, disc, 84, n_random=300)
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, ploidy=ploidy, known_vcf=known)
    g = os.path.join(str(tmp_path), "g.vcf")
    _run_gpu(fa, bam, g, known=known, ploidy=ploidy)
    orec = _records(o)
    assert len(orec) > n // 2
    assert _records(g) == orec


@pytest.mark.gpu
def test_pool_population_indels_vcf_identical(tmp_path):
    """MultisampleVariantsDetector at ploidy 4 with the realigner: every sample's indel genotype by genotypeVariantPool
    (genotypeVariantSample :378-379, makeUndecided below 40), discoverPopulationIndel's shrink loop, KPM's pool branch over
    the regions' columns.  Population VCF equal to the oracle's (path A)."""
    from test_gpu_multisample import gpu_mvd, oracle_mvd, population
    from helpers import diff_vcf
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=50000, n_samples=8, depth=16, seed=85,
                                   indel_rate=5e-4, snv_rate=3e-3)
    o = oracle_mvd(tmp_path, fa, sam, 0.0, ploidy=4)
    assert sum(1 for l in _records(o) if "TYPE=INDEL" in l or "TYPE=STR" in l) > 3
    g, _ = gpu_mvd(tmp_path, syn, rgs, ploidy=4)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
