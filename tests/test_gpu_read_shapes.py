"""Both detectors on the read shapes real BAMs carry (tests/read_shapes.py): paired-end flags with overlapping mates,
improper pairs, mates on another sequence or unmapped; mixed read lengths (75-250 bp and 5-20 kb reads); hard clips,
'=' / 'X' per-base CIGARs, 'N' reference skips and 'P' padding on the SNV path; duplicate / QC-fail / supplementary
records (kept, as the reference's filter keeps them), secondary and low-MAPQ ones (filtered), NH tags, SEQ '*',
repeated records.  The HIP VCF (BAM decoded in C++, ngsep_call_bam / ngsep_call_population_bams) equals the oracle's
(the SAM text) -- ReadAlignment.java:60-69, :747-871, :1180-1266; ReadAlignmentFileReader.java:219-306.

Also the layout cost of the mixed lengths: a 64-read group is padded to its longest read, so a
5-20 kb read pads its group's 63 other reads."""
import os

import pytest

from helpers import diff_vcf, gpu_params, gpu_vcf_bam, oracle_vcf
import ngsep_oracle
import pysynth
import read_shapes

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def single(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("shapes1"))
    sam, fa = os.path.join(d, "s.sam"), os.path.join(d, "s.fa")
    read_shapes.make_sam(sam, fa, seed=11, depth=20, lengths=(40000, 25000), indel_rate=3e-4)
    bam = pysynth.sam_to_bam(sam, os.path.join(d, "s.bam"))
    return d, fa, sam, bam


@pytest.mark.parametrize("opts", [
    {},
    {"calc_strand_bias": 1, "ignore5": 3, "ignore3": 2},
    {"max_alns_per_start": 2, "min_mq": 30, "max_base_qs": 25},
    {"ploidy": 1, "het_rate": 0.01},
])
def test_single_sample_read_shapes_vcf_identical(single, opts):
    d, fa, sam, bam = single
    tag = "_".join(f"{k}{v}" for k, v in sorted(opts.items())) or "default"
    o, _, _ = oracle_vcf(d, fa, sam, name="o_" + tag, **opts)
    g, st = gpu_vcf_bam(d, fa, bam, name="g_" + tag, **opts)
    diff = diff_vcf(o, g)
    assert not diff, "\n".join(diff[:20])
    assert sum(1 for l in open(o) if not l.startswith("#")) > 40


def test_single_sample_read_shapes_small_windows(single):
    """7 kb streamed windows: the 5-20 kb reads span several windows (halo = the longest span), the realigner regions
    included; the VCF is the whole run's"""
    d, fa, sam, bam = single
    o, _, _ = oracle_vcf(d, fa, sam, name="o_win")
    g, st = gpu_vcf_bam(d, fa, bam, name="g_win", window_positions=7000)
    diff = diff_vcf(o, g)
    assert not diff, "\n".join(diff[:20])


@pytest.mark.parametrize("opts", [{}, {"ploidy": 4}])
def test_population_read_shapes_vcf_identical(tmp_path, opts):
    """MultisampleVariantsDetector path B over one BAM of 10 read groups with the same shapes"""
    from ngsepcore_amd import MultisampleVariantsDetector
    d = str(tmp_path)
    sam, fa = os.path.join(d, "p.sam"), os.path.join(d, "p.fa")
    read_shapes.make_sam(sam, fa, seed=12, n_samples=10, depth=6, lengths=(30000, 15000), indel_rate=3e-4)
    bam = pysynth.sam_to_bam(sam, os.path.join(d, "p.bam"))
    o = os.path.join(d, "o.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, 0.0, **opts)
    assert sum(1 for l in open(o) if not l.startswith("#")) > 10
    det = MultisampleVariantsDetector()
    for k, v in opts.items():
        setattr(det.params, k, v)
    det.setGenome(fa)
    det.setOutFilename(os.path.join(d, "g.vcf"))
    det.run([bam]).close()
    diff = diff_vcf(o, det.outFilename)
    assert not diff, "\n".join(diff[:20])


def test_mixed_length_layout_cost(single):
    """The read-group layout's bytes against the reads' own bytes on the mixed-length set (reported in DESIGN.md
    section 2): group padding to the longest read is what the 5-20 kb reads cost."""
    d, fa, sam, bam = single
    g, st = gpu_vcf_bam(d, fa, bam, name="g_cost")
    ratio = st.pile_bytes / max(1, st.read_bases)
    print(f"layout bytes {st.pile_bytes}, read bases {st.read_bases}, ratio {ratio:.2f}")
    assert st.read_bases > 0 and ratio >= 1.0
