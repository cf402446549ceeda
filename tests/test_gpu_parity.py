"""GPU parity: the HIP path (libngsep_amd.so) against the CPU restatement of the reference.

Bar (BASELINE.json north star): allele counts and depths bit-exact; genotype log-likelihoods
bit-exact here (same fp64 summation order as CountsHelper.updateCounts); VCF text identical.
GQ/QUAL come from pow/log10, where the device libm and glibc may differ by an ulp; the
VCF equality below shows they agree on these inputs (any difference would fail the test).
"""
import os

import pytest

from helpers import diff_vcf, gpu_params, gpu_vcf_bam, make_data, oracle_vcf, read_dump, vcf_records
import pysynth
from ngsepcore_amd import GpuPileupSession

pytestmark = pytest.mark.gpu


def test_c1_yeast_chrI_10x_vcf_identical(tmp_path):
    """configs[0]: yeast chrI, 10x, 150 bp (seed 1)."""
    _, fa, sam, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=1, depth=10, seed=1)
    o, _, ost = oracle_vcf(tmp_path, fa, sam)
    g, gst = gpu_vcf_bam(tmp_path, fa, bam)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d)
    assert gst.positions_genotyped == ost.positions_genotyped
    assert len(vcf_records(g)) > 100


@pytest.mark.parametrize("opts", [
    {},
    {"ignore_lowercase_ref": 1},
    {"max_alns_per_start": 2, "ignore5": 3, "ignore3": 2},
    {"ploidy": 1},
    {"calc_strand_bias": 1, "min_quality": 20},
    {"max_base_qs": 20, "het_rate": 0.01, "print_sample_ploidy": 1, "sample_id": "S000"},
    {"process_nonunique": 1, "min_mq": 10},
    {"process_secondary": 1},
    {"query_seq": "chrII", "query_first": 20000, "query_last": 150000},
])
def test_edge_cases_vcf_identical(tmp_path, opts):
    """Reader/admission edge cases: secondary and low-MAPQ records, missing qualities, soft clips,
    PCR duplicates, lower-case reference, N bases, triallelic sites (uniform quality model)."""
    _, fa, sam, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=2, contig_first=0, depth=25, seed=7,
                                secondary_rate=0.01, lowmq_rate=0.01, noqual_rate=0.005, softclip_rate=0.05,
                                dup_rate=0.02, lower_frac=0.01, quality_model=2, snv_rate=3e-3)
    o, _, _ = oracle_vcf(tmp_path, fa, sam, **opts)
    g, _ = gpu_vcf_bam(tmp_path, fa, bam, **opts)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d)


def test_every_position_tally_bitexact(tmp_path):
    """dump mode: DP, A/C/G/T counts and all 10 log-conditionals at every covered position."""
    _, fa, sam, bam = make_data(tmp_path, genome=pysynth.CUSTOM, custom_len=40000, depth=30, seed=5,
                                noqual_rate=0.01, softclip_rate=0.05, quality_model=2)
    _, dump, _ = oracle_vcf(tmp_path, fa, sam, dump=True)
    ref = read_dump(dump)
    with GpuPileupSession(gpu_params(dump_all_positions=1)) as s:
        s.load_fasta(fa)
        s.processFile(bam, os.path.join(str(tmp_path), "dump_gpu.vcf"))
    # processFile writes calls only; rerun through path A for the raw records
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=40000, depth=30, seed=5, noqual_rate=0.01,
                        softclip_rate=0.05, quality_model=2)
    with GpuPileupSession(gpu_params(dump_all_positions=1)) as s:
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        s.processAlignments(syn.batch())
        s.notifyEndOfAlignments()
        got = s.getCalledVariants()
    gmap = {(x.sequence, x.pos): x for x in got}
    assert len(gmap) == len(ref)
    for k, (dp, counts, logc) in ref.items():
        x = gmap[k]
        assert x.dp == dp, k
        assert tuple(x.counts) == counts, k
        assert tuple(x.logc) == logc, k   # bit-exact fp64


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden_cases():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("name", ["c1_chrI_10x", "edge_2contigs_25x", "edge_2contigs_25x_csb_ploidy1"])
def test_golden_vcf(tmp_path, name):
    """HIP path vs the committed oracle VCFs (tests/golden), no oracle run needed."""
    skw, opts = _golden_cases().CASES[name]
    syn = pysynth.Synth(**skw)
    fa, _, bam = syn.write(os.path.join(str(tmp_path), name))
    syn.close()
    g, _ = gpu_vcf_bam(tmp_path, fa, bam, **opts)
    d = diff_vcf(os.path.join(GOLDEN, name + ".vcf"), g)
    assert not d, "\n".join(d)


def test_golden_dump_bitexact(tmp_path):
    """DP, counts and the 10 fp64 log-conditionals at every covered position == committed dump."""
    import gzip
    name, skw = _golden_cases().DUMP_CASE
    ref = {}
    for l in gzip.open(os.path.join(GOLDEN, name + ".dump.gz"), "rt"):
        f = l.rstrip("\n").split("\t")
        ref[(f[0], int(f[1]))] = (int(f[3]), tuple(int(x) for x in f[4].split(",")), tuple(float(x) for x in f[5:15]))
    syn = pysynth.Synth(**skw)
    with GpuPileupSession(gpu_params(dump_all_positions=1)) as s:
        for n, seq in syn.contigs():
            s.set_reference(n, seq)
        s.processAlignments(syn.batch())
        s.notifyEndOfAlignments()
        got = {(x.sequence, x.pos): x for x in s.getCalledVariants()}
    syn.close()
    assert len(got) == len(ref)
    for k, (dp, counts, logc) in ref.items():
        x = got[k]
        assert (x.dp, tuple(x.counts), tuple(x.logc)) == (dp, counts, logc), k


@pytest.mark.parametrize("depth,snv_rate,het", [(30, 1e-3, 0.001), (6, 3e-3, 0.001), (12, 1e-2, 0.05), (40, 1e-3, 0.1)])
def test_pruning_is_exact(tmp_path, depth, snv_rate, het):
    """KT's candidate pruning + integer hom-ref bound return exactly the calls of genotyping every
    position (low depth and high error/heterozygosity put many candidates near the bound)."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=depth, seed=3, quality_model=2, snv_rate=snv_rate)
    res = []
    for prune in (1, 0):
        with GpuPileupSession(gpu_params(prune_candidates=prune, het_rate=het, min_quality=0)) as s:
            for name, seq in syn.contigs():
                s.set_reference(name, seq)
            s.processAlignments(syn.batch())
            s.notifyEndOfAlignments()
            res.append([(x.sequence, x.pos, x.gq, x.qual, tuple(x.logc)) for x in s.getCalledVariants()])
            if prune:
                st = s.stats()
    assert res[0] == res[1]
    assert len(res[0]) > 100
    assert st.hard_sites < st.candidates     # the bound dropped candidates


def test_scan_overflow_survivors(tmp_path):
    """Dense variants (1 in 10 positions) and -minQuality 0: more count-bound survivors per 2048-position KL tile
    than the workgroup gathers itself, so KG gathers the rest; calls equal genotyping every position."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=20, seed=13, quality_model=2, snv_rate=0.1)
    res = []
    for prune in (1, 0):
        with GpuPileupSession(gpu_params(prune_candidates=prune, min_quality=0)) as s:
            for name, seq in syn.contigs():
                s.set_reference(name, seq)
            s.processAlignments(syn.batch())
            s.notifyEndOfAlignments()
            res.append([(x.sequence, x.pos, x.gq, x.qual, tuple(x.counts), tuple(x.logc)) for x in s.getCalledVariants()])
            if prune:
                st = s.stats()
    assert res[0] == res[1] and len(res[0]) > 10000
    assert st.hard_sites > 128 * (st.global_positions // 2048) // 4     # survivors well past the tiles' own lists


def test_path_a_equals_path_b(tmp_path):
    """ngsep_process_alignments (JNI-style batches) == ngsep_call_bam (BAM decoded in C++)."""
    syn, fa, sam, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=2, depth=20, seed=9)
    g, _ = gpu_vcf_bam(tmp_path, fa, bam)
    with GpuPileupSession() as s:
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        s.processAlignments(syn.batch())
        s.notifyEndOfAlignments()
        out = os.path.join(str(tmp_path), "a.vcf")
        s.write_vcf(out)
    assert open(out).read() == open(g).read()


def test_staged_run_repeatable(tmp_path):
    """bench path: stage once, run several times -> identical calls each run."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=4, depth=30, seed=2)
    with GpuPileupSession() as s:
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        s.stage(syn.batch())
        s.stage_finish()
        runs = []
        for _ in range(3):
            s.run_staged()
            runs.append([(x.sequence, x.pos, x.gq) for x in s.getCalledVariants()])
        s.release_staged()
    assert runs[0] == runs[1] == runs[2] and len(runs[0]) > 100


def test_async_passes_identical(tmp_path):
    """ngsep_submit_staged / ngsep_collect_staged (two passes in flight) give every pass the same
    calls as a synchronous run, including when the first pass's record estimate is too small."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=20, seed=4, quality_model=2, snv_rate=3e-3)
    with GpuPileupSession(gpu_params(min_quality=0)) as s:
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        s.stage(syn.batch())
        s.stage_finish()
        s.run_staged()
        ref = [(x.sequence, x.pos, x.gq, x.qual, tuple(x.logc)) for x in s.getCalledVariants()]
        got = []
        s.submit_staged()
        for k in range(5):
            if k + 1 < 5:
                s.submit_staged()
            s.collect_staged()
            got.append([(x.sequence, x.pos, x.gq, x.qual, tuple(x.logc)) for x in s.getCalledVariants()])
    assert len(ref) > 1000
    for g in got:
        assert g == ref


@pytest.mark.parametrize("window", [0, 5000])
@pytest.mark.parametrize("depth,het", [(12, 0.05), (40, 0.1), (90, 0.001), (300, 0.001)])
def test_scan_depths(tmp_path, window, depth, het):
    """KL at several depths (above 255 covering reads the count bound is skipped) and window sizes (a window's
    halo and tile cuts): pruned calls == genotyping every position (KQ queues all, KG gathers, KP genotypes)."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=depth, seed=11, quality_model=2, snv_rate=3e-3)
    res = []
    for prune in (1, 0):
        with GpuPileupSession(gpu_params(prune_candidates=prune, het_rate=het, min_quality=0, window_positions=window)) as s:
            for name, seq in syn.contigs():
                s.set_reference(name, seq)
            s.processAlignments(syn.batch())
            s.notifyEndOfAlignments()
            res.append([(x.sequence, x.pos, x.gq, x.qual, tuple(x.counts), tuple(x.logc)) for x in s.getCalledVariants()])
    assert res[0] == res[1]
    assert len(res[0]) > 100


@pytest.mark.parametrize("window", [1024, 7000, 0])
def test_window_size_vcf_identical(tmp_path, window):
    """configs[0] data through windows of several sizes (each a separate device run with its halo): VCF
    identical to the oracle's."""
    _, fa, sam, bam = make_data(tmp_path, genome=pysynth.YEAST, n_contigs=1, depth=10, seed=1)
    o, _, _ = oracle_vcf(tmp_path, fa, sam)
    g, gst = gpu_vcf_bam(tmp_path, fa, bam, window_positions=window)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d)
    assert gst.tile_positions == 2048


def test_reference_fields_single_sample_dump(tmp_path):
    """The reference's genotype fields replayed as Q30 pileups (tests/demo_replay.py, sample S0 only)
    through the single-sample HIP path in dump mode (KT + KP, every covered position): DP, BSDP and the
    PL triple from the fp64 log-conditionals (float cast, Math.round) equal the reference's own output
    for all 10,508 all-Q30-consistent fields."""
    import math
    import numpy as np
    import demo_replay as R
    rs = R.rows()
    fa, sam, site = R.write(tmp_path, R.keys(rs))
    lines = [l for l in open(sam) if l.startswith("@") or not l.rstrip("\n").endswith("RG:Z:S1")]
    open(sam, "w").writelines(lines)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "demo_s0.bam"))
    with GpuPileupSession(gpu_params(dump_all_positions=1, max_alns_per_start=0)) as s:
        s.load_fasta(fa)
        s.processFileBatches(bam)
        got = {x.pos: x for x in s.getCalledVariants()}
    pl = lambda v: int(math.floor(-10.0 * float(np.float32(v)) + 0.5))
    checked = 0
    by_key = {k: got.get(p) for p, k in site.items()}
    for r in rs:
        nr, na, ri, ai, dp = (int(r["n_ref"]), int(r["n_alt"]), int(r["ref_idx"]), int(r["alt_idx"]), int(r["dp"]))
        x = by_key[(nr, na, ri, ai, dp)]
        assert x is not None and x.dp == dp
        bsdp = [0, 0, 0, 0]
        bsdp[ri] += nr
        bsdp[ai] += na
        assert x.counts == bsdp
        got_pl = (pl(x.log_conditional(ri, ri)), pl(x.log_conditional(ri, ai)), pl(x.log_conditional(ai, ai)))
        if got_pl == (int(r["pl_rr"]), int(r["pl_ra"]), int(r["pl_aa"])):
            checked += 1
    assert checked == 10508


def test_full_records_agree_with_default(tmp_path):
    """ngsep_params.full_records (ABI 5): the whole CountsHelper state per record.  The default records carry
    what CalledSNV keeps -- the (ref,ref), (ref,alt), (alt,alt) log-conditionals and the reference / alternative
    strand counts -- and must equal those entries of the whole records bit for bit; the VCF is the same."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=20, seed=71, snv_rate=3e-3)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "fr"))
    syn.close()
    runs = {}
    for full in (0, 1):
        out = os.path.join(str(tmp_path), f"fr{full}.vcf")
        with GpuPileupSession(gpu_params(full_records=full, calc_strand_bias=1)) as s:
            s.load_fasta(fa)
            s.processFileBatches(bam)
            runs[full] = s.getCalledVariants()
            s.write_vcf(out)
    lean, whole = runs[0], runs[1]
    assert len(lean) == len(whole) > 100
    n_multi = 0
    for a, b in zip(lean, whole):
        assert (a.sequence, a.pos, a.alleles, a.genotype, a.gq, a.qual, a.dp, a.counts, a.strand_bias) == \
               (b.sequence, b.pos, b.alleles, b.genotype, b.gq, b.qual, b.dp, b.counts, b.strand_bias)
        if len(a.alleles) == 2:
            ri, ai = "ACGT".index(a.alleles[0]), "ACGT".index(a.alleles[1])
            for i, j in ((ri, ri), (ri, ai), (ai, ai)):
                assert a.log_conditional(i, j) == b.log_conditional(i, j)
            for k in (ri, ai):
                assert a.strand_counts[k] == b.strand_counts[k]
        else:
            n_multi += 1
            assert a.logc == b.logc and a.strand_counts == b.strand_counts   # multi-allelic records are whole
    assert open(os.path.join(str(tmp_path), "fr0.vcf")).read() == open(os.path.join(str(tmp_path), "fr1.vcf")).read()
