"""GPU parity of the MultisampleVariantsDetector path (discovery/MultisampleVariantsDetector.java:421-693)
against the CPU restatement (oracle/ngsep_oracle.c ngo_run_mvd).

Bar: population VCF text identical (variant QS, INFO NS/AN/AFS/OH/MAF/TYPE, every sample's
GT:PL:GQ:DP:BSDP:ACN).  The per-sample fp64 log-likelihood sums follow the reference's read order
(read groups of a sample in HashSet order, pending-list order inside each), so PL/GQ agree exactly.
"""
import os

import pytest

from helpers import diff_vcf, gpu_params, oracle_params_from
import ngsep_oracle
import pysynth
from ngsepcore_amd import GpuPileupSession

pytestmark = pytest.mark.gpu


def population(tmp_path, **kw):
    syn = pysynth.Synth(**kw)
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "pop"))
    n = max(1, syn.params.n_samples)
    rgs = [(f"S{syn.params.sample_idx + k:03d}", f"S{syn.params.sample_idx + k:03d}") for k in range(n)]
    return syn, fa, sam, rgs


def oracle_mvd(tmp_path, fa, sam, min_adf=0.0, **opts):
    out = os.path.join(str(tmp_path), "oracle_mvd.vcf")
    ngsep_oracle.run_mvd(fa, sam, out, min_adf, **oracle_params_from(opts))
    return out


def gpu_mvd(tmp_path, syn, rgs, staged=False, **opts):
    out = os.path.join(str(tmp_path), "gpu_mvd.vcf")
    p = gpu_params(multisample=1, **opts)
    with GpuPileupSession(p) as s:
        s.set_samples(rgs)
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        if staged == "pipelined":
            # two passes in flight (ngsep_submit_staged x2, then collect x2): the second pass's result is written
            s.stage(syn.batch())
            s.stage_finish()
            s.submit_staged()
            s.submit_staged()
            s.collect_staged()
            s.collect_staged()
        elif staged:
            s.stage(syn.batch())
            s.stage_finish()
            s.run_staged()
        else:
            s.processAlignments(syn.batch())
            s.notifyEndOfAlignments()
        s.write_population_vcf(out)
        st = s.stats()
    return out, st


def n_records(path):
    return sum(1 for l in open(path) if not l.startswith("#"))


@pytest.mark.parametrize("kw,opts", [
    (dict(n_samples=20, depth=10, snv_rate=2e-3), {}),
    (dict(n_samples=48, depth=6, snv_rate=3e-3, quality_model=2), {}),
    (dict(n_samples=16, depth=12, snv_rate=3e-3, quality_model=2), {"min_allele_depth_freq": 0.02, "min_quality": 20}),
    (dict(n_samples=12, depth=15, snv_rate=2e-3), {"ploidy": 1, "het_rate": 0.01}),
    (dict(n_samples=10, depth=10, snv_rate=2e-3, lower_frac=0.01), {"ignore_lowercase_ref": 1, "max_base_qs": 25}),
])
def test_population_vcf_identical(tmp_path, kw, opts):
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=40000, seed=5, **kw)
    min_adf = opts.pop("min_allele_depth_freq", 0.0)
    o = oracle_mvd(tmp_path, fa, sam, min_adf, **opts)
    g, st = gpu_mvd(tmp_path, syn, rgs, min_allele_depth_freq=min_adf, **opts)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    assert n_records(o) > 20


def test_population_200_samples_staged(tmp_path):
    """C5 shape (200 samples at 10x) on a short contig, staged run path."""
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=8000, seed=6, n_samples=200,
                                   depth=10, snv_rate=3e-3)
    o = oracle_mvd(tmp_path, fa, sam)
    g, st = gpu_mvd(tmp_path, syn, rgs, staged=True)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    assert n_records(o) > 10
    assert st.hard_sites < st.positions_genotyped      # the per-sample bounds dropped positions
    g2, _ = gpu_mvd(tmp_path, syn, rgs, staged="pipelined")
    d = diff_vcf(o, g2)
    assert not d, "\n".join(d[:20])
    # every per-sample call through the whole-record list instead of the packed 32-B record
    os.environ["NGSEP_POP_ALL_BIG"] = "1"
    try:
        g3, _ = gpu_mvd(tmp_path, syn, rgs, staged="pipelined")
    finally:
        del os.environ["NGSEP_POP_ALL_BIG"]
    d = diff_vcf(o, g3)
    assert not d, "\n".join(d[:20])


def test_population_bams_path_b(tmp_path):
    """`MultisampleVariantsDetector -r REF -o OUT.vcf S000.bam ... S011.bam`: samples from the BAM
    headers, files merged in AlignmentsPileupGenerator's order (C++ path, ngsep_call_population_bams)."""
    import subprocess
    from ngsepcore_amd import MultisampleVariantsDetector
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=30000, seed=8, n_samples=12,
                                   depth=10, snv_rate=3e-3)
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    o = oracle_mvd(tmp_path, fa, sam)
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setOutFilename(os.path.join(str(tmp_path), "gpu_b.vcf"))
    d.run(bams[::-1])                       # file order does not change the merge (ties: equal spans)
    diff = diff_vcf(o, d.outFilename)
    assert not diff, "\n".join(diff[:20])
    # the streaming heap merge (files larger than one whole-file batch) == the parallel whole-file merge
    os.environ["NGSEP_POP_STREAM"] = "1"
    try:
        d.setOutFilename(os.path.join(str(tmp_path), "gpu_b_stream.vcf"))
        d.run(bams)
    finally:
        del os.environ["NGSEP_POP_STREAM"]
    diff = diff_vcf(o, d.outFilename)
    assert not diff, "\n".join(diff[:20])
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ngsepcore_amd", "lib", "ngsep-amd")
    out_cli = os.path.join(str(tmp_path), "cli.vcf")
    subprocess.run([cli, "MultisampleVariantsDetector", "-r", fa, "-o", out_cli] + bams, check=True)
    diff = diff_vcf(o, out_cli)
    assert not diff, "\n".join(diff[:20])


def test_reference_fields_replayed_on_gpu(tmp_path):
    """The reference's own genotype fields (training/yeastDemo_*.vcf.gz, the 10,508 all-Q30-consistent
    ones, tests/demo_replay.py) replayed as Q30 pileups through the HIP population path (KTM + KPM, BAM
    decoded in C++): GT, PL, GQ, DP and BSDP equal the reference's own output."""
    import demo_replay as R
    from ngsepcore_amd import MultisampleVariantsDetector
    rs = R.rows()
    fa, sam, site = R.write(tmp_path, R.keys(rs))
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "demo.bam"))
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setMaxAlnsPerStartPos(0)
    d.setOutFilename(os.path.join(str(tmp_path), "replay_gpu.vcf"))
    d.run([bam]).close()
    checked, bad = R.check(rs, site, R.parse_vcf(d.outFilename))
    assert not bad, bad[:10]
    assert checked == 10508


@pytest.mark.parametrize("kw,opts", [
    (dict(genome=pysynth.CUSTOM, custom_len=30000, seed=9, n_samples=16, depth=10, snv_rate=3e-3), {}),
    (dict(genome=pysynth.CUSTOM, custom_len=20000, seed=10, n_samples=12, depth=8, snv_rate=3e-3, quality_model=2),
     {"ploidy": 1, "het_rate": 0.01}),
    (dict(genome=pysynth.CUSTOM, custom_len=15000, seed=11, n_samples=8, depth=16, snv_rate=3e-3), {"ploidy": 4}),
])
def test_population_known_variants(tmp_path, kw, opts):
    """`MultisampleVariantsDetector -knownVariants` (MultisampleVariantsDetector.onPileup :539-551, genotypeVariant
    :664-693): every input SNV at a covered position genotyped in every sample and written with the input's ID,
    whatever its QS; population VCF identical to the oracle's through path B (sample BAMs) and the staged path."""
    from test_gpu_known import _known_vcf
    from ngsepcore_amd import MultisampleVariantsDetector
    syn, fa, sam, rgs = population(tmp_path, **kw)
    known = os.path.join(str(tmp_path), "known.vcf")
    _known_vcf(known, syn, os.path.join(str(tmp_path), "pop_truth.vcf"), kw["seed"], n_random=400)
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, 0.0, known_vcf=known, **oracle_params_from(opts))
    assert n_records(o) > 100
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    d = MultisampleVariantsDetector()
    for k, v in opts.items():
        setattr(d.params, k, v)
    if "het_rate" in opts:
        d.params.het_rate_set = 1
    d.setGenome(fa)
    d.setKnownVariantsFile(known)
    d.setOutFilename(os.path.join(str(tmp_path), "gpu_b.vcf"))
    d.run(bams).close()
    diff = diff_vcf(o, d.outFilename)
    assert not diff, "\n".join(diff[:20])


@pytest.mark.parametrize("kw,opts", [
    (dict(n_samples=12, depth=10, seed=21, indel_rate=3e-4, snv_rate=2e-3), {}),
    (dict(n_samples=16, depth=8, seed=22, indel_rate=5e-4, snv_rate=3e-3, quality_model=2), {"call_embedded": 1}),
    (dict(n_samples=10, depth=12, seed=23, indel_rate=4e-4, snv_rate=2e-3), {"ploidy": 1, "het_rate": 0.01}),
    (dict(n_samples=20, depth=6, seed=24, indel_rate=6e-4, snv_rate=3e-3), {"min_quality": 20, "min_allele_depth_freq": 0.02}),
])
def test_population_indels_vcf_identical(tmp_path, kw, opts):
    """MultisampleVariantsDetector with the indel realigner first in its chain (MultisampleVariantsDetector.java:449-450):
    population indel / STR records (discoverPopulationVariantWithSpan / discoverPopulationIndel :599-634, every sample
    genotyped by callIndel over the variant's alleles), the SNVs of the realigned alignments (KPM over the regions'
    columns), lastIndelEnd / embedded SNVs (:522-538).  The WHOLE population VCF equals the oracle's through path A
    (ngsep_process_alignments) and path B (one BAM per sample, files in sample order: the merge's ties go to the lower
    file index); no region is handed back.  Parity is against the oracle restatement only: the reference holds no
    population indel fixture (parity unpinned)."""
    from ngsepcore_amd import MultisampleVariantsDetector
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=60000, **kw)
    min_adf = opts.get("min_allele_depth_freq", 0.0)
    oopts = {k: v for k, v in opts.items() if k != "min_allele_depth_freq"}
    o = oracle_mvd(tmp_path, fa, sam, min_adf, **oopts)
    ro = [l for l in open(o) if not l.startswith("#")]
    assert sum(1 for l in ro if "TYPE=INDEL" in l or "TYPE=STR" in l) > 3
    g, st = gpu_mvd(tmp_path, syn, rgs, **opts)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    det = MultisampleVariantsDetector()
    for k, v in opts.items():
        setattr(det.params, k, v)
    if "het_rate" in opts:
        det.params.het_rate_set = 1
    det.setGenome(fa)
    det.setOutFilename(os.path.join(str(tmp_path), "gpu_b.vcf"))
    det.run(bams).close()
    d = diff_vcf(o, det.outFilename)
    assert not d, "\n".join(d[:20])


@pytest.mark.parametrize("kw,opts", [
    (dict(n_samples=12, depth=10, seed=31, indel_rate=4e-4, snv_rate=2e-3), {}),
    (dict(n_samples=10, depth=12, seed=32, indel_rate=5e-4, snv_rate=2e-3), {"ploidy": 1, "het_rate": 0.01}),
])
def test_population_known_indels(tmp_path, kw, opts):
    """`MultisampleVariantsDetector -knownVariants` with indel / MNP inputs on data with indels: the records are the
    realigner's input variants (MultisampleVariantsDetector.run :432-438), every input SNV is genotyped by KPM from
    the realigned columns and every other record in every sample by callIndel with the variant given
    (genotypeVariant :664-693); the WHOLE population VCF equals the oracle's, through path A and path B."""
    from test_gpu_known import _known_vcf_indels
    from ngsepcore_amd import MultisampleVariantsDetector
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=50000, **kw)
    disc = oracle_mvd(tmp_path, fa, sam, 0.0, **opts)
    known = os.path.join(str(tmp_path), "known.vcf")
    n = _known_vcf_indels(known, syn, disc, kw["seed"], n_random=150)
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, 0.0, known_vcf=known, **oracle_params_from(opts))
    ro = [l for l in open(o) if not l.startswith("#")]
    assert len(ro) > n // 2
    assert sum(1 for l in ro if len(l.split("\t")[3]) > 1 or len(l.split("\t")[4]) > 1) > 30
    g = os.path.join(str(tmp_path), "gpu_a.vcf")
    with GpuPileupSession(gpu_params(multisample=1, **opts)) as s:
        s.set_samples(rgs)
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        s.set_known_variants(known)
        s.processAlignments(syn.batch())
        s.notifyEndOfAlignments()
        s.write_population_vcf(g)
        assert not s.carved_regions()
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    det = MultisampleVariantsDetector()
    for k, v in opts.items():
        setattr(det.params, k, v)
    if "het_rate" in opts:
        det.params.het_rate_set = 1
    det.setGenome(fa)
    det.setKnownVariantsFile(known)
    det.setOutFilename(os.path.join(str(tmp_path), "gpu_b.vcf"))
    det.run(bams).close()
    d = diff_vcf(o, det.outFilename)
    assert not d, "\n".join(d[:20])


def test_population_read_groups_of_samples(tmp_path):
    """Samples with several read groups and reads of no sample (round 4's population layout: one stream per
    (sample, read-group rank), the reads of no sample in the last stream, pooled counts only).  The SAM header maps
    read groups S000-S009 two by two to samples P0-P4 (their calls in HashSet order of the group ids,
    PileupRecord.getAlleleCalls(span, readGroups) :104-111), S010 to P5, and lists no S011: its reads enter the
    pooled counts of every position but no sample."""
    syn, fa, sam, _ = population(tmp_path, genome=pysynth.CUSTOM, custom_len=30000, seed=9, n_samples=12,
                                 depth=8, snv_rate=3e-3)
    sm = {f"S{k:03d}": f"P{k // 2}" for k in range(10)}
    sm["S010"] = "P5"
    lines = []
    for l in open(sam):
        if l.startswith("@RG"):
            rid = l.split("\t")[1][3:]
            if rid not in sm:
                continue
            l = f"@RG\tID:{rid}\tSM:{sm[rid]}\n"
        lines.append(l)
    sam2 = os.path.join(str(tmp_path), "pop_rg.sam")
    with open(sam2, "w") as f:
        f.writelines(lines)
    rgs = [(f"S{k:03d}", sm.get(f"S{k:03d}")) for k in range(12)]
    o = oracle_mvd(tmp_path, fa, sam2)
    for staged in (False, True):
        g, st = gpu_mvd(tmp_path, syn, rgs, staged=staged)
        d = diff_vcf(o, g)
        assert not d, "\n".join(d[:20])
    assert n_records(o) > 10
    assert sum(1 for l in open(o) if l.startswith("#CHROM"))  # (header present)
    hdr = [l for l in open(o) if l.startswith("#CHROM")][0].rstrip("\n").split("\t")
    assert hdr[9:] == [f"P{k}" for k in range(6)]


@pytest.mark.parametrize("window", [5000, 12345])
def test_population_window_sizes(tmp_path, window):
    """Windows cut the population run's coordinate (each window's reads laid out again with a halo of the read span,
    KLM's sample tiles and KPM's gathers crossing window and halo boundaries): the VCF is the whole run's."""
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=40000, seed=11, n_samples=24, depth=8,
                                   snv_rate=3e-3)
    o = oracle_mvd(tmp_path, fa, sam)
    g, st = gpu_mvd(tmp_path, syn, rgs, window_positions=window)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    assert n_records(o) > 20


def test_population_sample_without_reads(tmp_path):
    """A sample of the header with no alignment at all (no stream in the population layout): every site genotypes
    it undecided with empty counts, as the reference does."""
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=20000, seed=12, n_samples=8, depth=10,
                                   snv_rate=3e-3)
    lines = open(sam).readlines()
    last_rg = max(i for i, l in enumerate(lines) if l.startswith("@RG"))
    lines.insert(last_rg + 1, "@RG\tID:SX00\tSM:S004a\n")     # sorts between S004 and S005
    sam2 = os.path.join(str(tmp_path), "pop_empty.sam")
    with open(sam2, "w") as f:
        f.writelines(lines)
    o = oracle_mvd(tmp_path, fa, sam2)
    g, st = gpu_mvd(tmp_path, syn, rgs + [("SX00", "S004a")])
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    assert n_records(o) > 10


def test_population_long_span_alignment(tmp_path):
    """One alignment with a 30 kb reference skip (CIGAR N) in a 100-sample population: the per-sample column bound
    KPM's gather is sized by is the true per-sample coverage (a sweep over the starts and ends), not the reads
    starting within the run's longest span -- which this one alignment would inflate past the kernel's columns and
    refuse.  Path B (one BAM, 100 read groups) == the oracle."""
    from ngsepcore_amd import MultisampleVariantsDetector
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=60000, seed=9, n_samples=100,
                                   depth=10, snv_rate=3e-3)
    name, seq = syn.contigs()[0]
    syn.close()
    seq = bytes(seq).decode().upper()
    p, gap = 5001, 30000
    bases = seq[p - 1:p - 1 + 60] + seq[p - 1 + 60 + gap:p - 1 + 120 + gap]
    rec = "\t".join(["longskip", "0", name, str(p), "60", f"60M{gap}N60M", "*", "0", "0", bases, "I" * 120,
                     "RG:Z:S000"]) + "\n"
    head, body = [], []
    for l in open(sam):
        (head if l.startswith("@") else body).append(l)
    k = next(i for i, l in enumerate(body) if int(l.split("\t")[3]) > p)
    body.insert(k, rec)
    sam2 = os.path.join(str(tmp_path), "long.sam")
    with open(sam2, "w") as f:
        f.writelines(head + body)
    bam = pysynth.sam_to_bam(sam2, os.path.join(str(tmp_path), "long.bam"))
    o = oracle_mvd(tmp_path, fa, sam2)
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setOutFilename(os.path.join(str(tmp_path), "gpu_long.vcf"))
    d.run([bam])
    diff = diff_vcf(o, d.outFilename)
    assert not diff, "\n".join(diff[:20])
    assert n_records(o) > 20
