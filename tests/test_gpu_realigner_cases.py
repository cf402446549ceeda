"""The product's realigner (ngsepcore_amd/csrc/realign.cpp through ngsep_call_bam / ngsep_call_population_bams) on the
region-logic pileups of tests/test_oracle_realigner_kat.py -- floating indels in homopolymer runs, two-length events,
deletions longer than their run, read ends drawn as mismatches or soft clips, -knownSTRs fixed events: the WHOLE VCF
equals the oracle's, whose region logic the independent Python restatement (tests/realigner_restatement.py) pins on the
same data.  Product == oracle == restatement on the code that decides which reads get rewritten."""
import os

import pytest

import ngsep_oracle
import pysynth
from helpers import diff_vcf, gpu_params
from ngsepcore_amd import GpuPileupSession, MultisampleVariantsDetector
from test_oracle_realigner_kat import write_case

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", list(range(12)))
def test_single_sample_cases_vcf_identical(tmp_path, seed):
    known = seed % 2 == 1
    fa, sam, _, _, _, strs = write_case(str(tmp_path), seed, known_strs=known)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "c.bam"))
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o, **({"known_strs": strs} if known else {}))
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params()) as s:
        s.load_fasta(fa)
        if known:
            s.set_known_strs(strs)
        s.processFile(bam, g)
        assert not s.carved_regions()
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    assert sum(1 for l in open(o) if "TYPE=INDEL" in l or "TYPE=STR" in l) > 3


@pytest.mark.parametrize("seed", list(range(100, 106)))
def test_population_cases_vcf_identical(tmp_path, seed):
    known = seed % 2 == 1
    fa, sam, _, _, _, strs = write_case(str(tmp_path), seed, n_samples=6, depth=8, known_strs=known)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "c.bam"))
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, 0.0, **({"known_strs": strs} if known else {}))
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    if known:
        d.setKnownSTRsFile(strs)
    d.setOutFilename(os.path.join(str(tmp_path), "g.vcf"))
    d.run([bam]).close()
    diff = diff_vcf(o, d.outFilename)
    assert not diff, "\n".join(diff[:20])
