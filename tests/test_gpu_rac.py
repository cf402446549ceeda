"""RelativeAlleleCountsCalculator (discovery/RelativeAlleleCountsCalculator.java:183-331):
the GPU report (k_rac over the streamed windows' byte pile) against the oracle's restatement, byte for byte,
on BAM input and on path A batches.  The proportion sums are added per block (a different order than the
reference's running sum): the report prints them at 2 decimals, which this data does not move."""
import os

import pytest

import ngsep_oracle
import pysynth
from ngsepcore_amd import RelativeAlleleCountsCalculator, _lib, default_params, GpuPileupSession


def _data(tmp_path, **kw):
    syn = pysynth.Synth(**kw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "rac"))
    return syn, fa, sam, bam


@pytest.mark.gpu
@pytest.mark.parametrize("kw,opts", [
    (dict(genome=pysynth.YEAST, n_contigs=3, depth=20, seed=3, snv_rate=3e-3, indel_rate=1e-4), {}),
    (dict(genome=pysynth.YEAST, n_contigs=2, depth=12, seed=9, secondary_rate=0.02, noqual_rate=0.01, softclip_rate=0.05,
          quality_model=2, snv_rate=5e-3), dict(min_rd=5, min_bq=25, secondary=1)),
    (dict(genome=pysynth.YEAST, n_contigs=1, contig_first=0, depth=40, seed=4, dup_rate=0.05, indel_rate=3e-4), dict(max_rd=3)),
])
def test_rac_report_identical(tmp_path, kw, opts):
    syn, fa, sam, bam = _data(tmp_path, **kw)
    o = os.path.join(str(tmp_path), "o.txt")
    ngsep_oracle.run_rac(fa, sam, o, **opts)
    calc = RelativeAlleleCountsCalculator()
    calc.setGenome(fa)
    if "min_rd" in opts:
        calc.setMinRD(opts["min_rd"])
    if "min_bq" in opts:
        calc.setMinBaseQualityScore(opts["min_bq"])
    if "max_rd" in opts:
        calc.setMaxRD(opts["max_rd"])
    if opts.get("secondary"):
        calc.setSecondaryAlns(True)
    g = os.path.join(str(tmp_path), "g.txt")
    calc.runProcess(bam, g)
    assert open(g).read() == open(o).read()
    assert calc.moments[0] > 1000
    # path A (the caller's own reader) gives the same distributions; the generator's batch view is the
    # default reader's (no secondary records), so it is checked against the oracle without -s
    calc2 = RelativeAlleleCountsCalculator()
    for k in ("rac_min_rd", "rac_min_bq", "max_alns_per_start", "process_secondary"):
        setattr(calc2.params, k, getattr(calc.params, k))
    g2 = os.path.join(str(tmp_path), "g2.txt")
    calc2.processBatches([syn.batch()], contigs=syn.contigs(), out_path=g2)
    syn.close()
    if opts.get("secondary"):
        o = os.path.join(str(tmp_path), "o_nosec.txt")
        ngsep_oracle.run_rac(fa, sam, o, **dict(opts, secondary=0))
    assert open(g2).read() == open(o).read()


@pytest.mark.gpu
def test_rac_small_windows(tmp_path):
    """Streamed windows of 30000 positions: the distributions do not depend on the cut (and no genome: the
    sequences come from the BAM header, as the reference's optional -r allows)."""
    syn, fa, sam, bam = _data(tmp_path, genome=pysynth.YEAST, n_contigs=2, depth=15, seed=12, snv_rate=4e-3)
    syn.close()
    o = os.path.join(str(tmp_path), "o.txt")
    ngsep_oracle.run_rac(fa, sam, o)
    calc = RelativeAlleleCountsCalculator()
    calc.params.window_positions = 30000
    g = os.path.join(str(tmp_path), "g.txt")
    calc.runProcess(bam, g)
    assert open(g).read() == open(o).read()


def test_rac_params_checked():
    """minBQ outside [4, 30] cannot be decided from the pile's codes: refused, not approximated."""
    p = default_params()
    p.relative_allele_counts = 1
    p.rac_min_bq = 35
    with pytest.raises(_lib.NgsepError):
        GpuPileupSession(p)


def test_oracle_rac_kat(tmp_path):
    """Known answers of the restatement on a hand-made pileup: 12 reads over one 20-bp contig, 9 A and 3 C
    at position 5 (Q30), every other position all-reference: one pileup of proportion 0.25 and two alleles,
    the others proportion 0.0 and one allele."""
    ref = "ACGTAACCGGTTACGTACGT"
    fa = os.path.join(str(tmp_path), "k.fa")
    open(fa, "w").write(">k\n" + ref + "\n")
    sam = os.path.join(str(tmp_path), "k.sam")
    with open(sam, "w") as f:
        f.write("@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:k\tLN:20\n")
        for i in range(12):
            seq = list(ref)
            if i >= 9:
                seq[4] = "C"
            f.write(f"r{i}\t0\tk\t1\t60\t20M\t*\t0\t0\t{''.join(seq)}\t{'?' * 20}\n")
    out = os.path.join(str(tmp_path), "k.txt")
    st = ngsep_oracle.run_rac(fa, sam, out)
    txt = open(out).read().splitlines()
    assert st.positions_genotyped == 20
    assert txt[0] == "Distribution of allele proportions"
    assert txt[1] == "0.0\t19.0" and txt[26] == "0.25\t1.0"
    i = txt.index("Distribution of number of alleles")
    assert txt[i + 1] == "1\t19" and txt[i + 2] == "2\t1"
    assert "Count\t20" in txt and "Sum\t0.25" in txt
    assert not any(l.startswith("Distribution of allele proportions per sequence") for l in txt)   # 20 bp <= 100000
