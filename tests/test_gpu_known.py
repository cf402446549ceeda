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


def test_known_variants_refused_types(tmp_path):
    """Indels and multi-allelic records are refused (their genotyping is not in this build), not skipped."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=5, seed=3)
    fa, _, _ = syn.write(os.path.join(str(tmp_path), "r"))
    name = syn.contigs()[0][0]
    syn.close()
    known = os.path.join(str(tmp_path), "bad.vcf")
    open(known, "w").write(f"#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n{name}\t10\t.\tAC\tA\t.\t.\t.\n")
    s = GpuPileupSession(gpu_params())
    s.load_fasta(fa)
    with pytest.raises(_lib.NgsepError) as e:
        s.set_known_variants(known)
    assert e.value.code == _lib.NGSEP_E_UNSUPPORTED
    s.close()
