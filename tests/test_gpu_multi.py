"""Several device contexts driven from ONE process through the C ABI (ngsep_call_bam_multi /
ngsep_call_population_bams_multi, ABI 11): one host thread and one context per device, windows cut by
ngsep_clean_cut taken from an in-process queue, records merged in (sequence, window) order.  The test box has one GPU,
so the contexts share device 0 -- two threads, two contexts, two sets of streams and pinned buffers running concurrently
on one card; the VCF must equal the one-context run byte for byte, for both detectors, on indel-bearing data (the
realigner decides where a cut may fall), with -knownVariants and in pass-through mode (whole sequences, carved regions
gathered on the first context)."""
import os

import pytest

import ngsep_oracle
import pysynth
from helpers import gpu_params
from ngsepcore_amd import GpuPileupSession, MultisampleVariantsDetector
from ngsepcore_amd.sharding import call_bam_multi, call_population_multi

pytestmark = pytest.mark.gpu


def _data(tmp_path, **kw):
    syn = pysynth.Synth(**kw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "m"))
    return syn, fa, sam, bam


@pytest.mark.parametrize("n_ctx,window", [(2, 25000), (3, 40000), (2, 0)])
def test_multi_context_single_sample_identical(tmp_path, n_ctx, window):
    syn, fa, sam, bam = _data(tmp_path, genome=pysynth.CUSTOM, custom_len=200000, seed=81, snv_rate=2e-3, indel_rate=5e-4,
                              depth=20)
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession(gpu_params()) as s:
        s.load_fasta(fa)
        s.processFile(bam, full)
    text = open(full).read()
    assert sum(1 for l in text.splitlines() if "TYPE=INDEL" in l or "TYPE=STR" in l) > 5
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o)
    assert text == open(o).read()
    got = call_bam_multi(fa, bam, os.path.join(str(tmp_path), "multi.vcf"), [0] * n_ctx, window=window)
    assert got == text
    assert not any(f.startswith("multi.vcf.part") for f in os.listdir(str(tmp_path)))


def test_multi_context_yeast_contigs_known_variants(tmp_path):
    """several sequences, -knownVariants on the first context only (the others take it)"""
    syn, fa, sam, bam = _data(tmp_path, genome=pysynth.YEAST, n_contigs=3, depth=12, seed=82, snv_rate=2e-3, indel_rate=3e-4)
    truth = os.path.join(str(tmp_path), "m_truth.vcf")
    syn.close()
    known = os.path.join(str(tmp_path), "known.vcf")
    with open(known, "w") as o:
        o.write("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\n")
        for l in open(truth):
            if not l.startswith("#"):
                f = l.split("\t")
                o.write("\t".join(f[:5] + [".", ".", "."]) + "\n")
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession(gpu_params()) as s:
        s.load_fasta(fa)
        s.set_known_variants(known)
        s.processFile(bam, full)
    got = call_bam_multi(fa, bam, os.path.join(str(tmp_path), "multi.vcf"), [0, 0], window=60000, known_vcf=known)
    assert got == open(full).read()
    assert len(got.splitlines()) > 100


def test_multi_context_passthrough_carved(tmp_path):
    syn, fa, sam, bam = _data(tmp_path, genome=pysynth.YEAST, n_contigs=3, depth=15, seed=83, indel_rate=3e-4)
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession(gpu_params(indel_passthrough=1)) as s:
        s.load_fasta(fa)
        s.processFile(bam, full)
        want = s.carved_regions()
    info = []
    got = call_bam_multi(fa, bam, os.path.join(str(tmp_path), "multi.vcf"), [0, 0], params=gpu_params(indel_passthrough=1),
                         window=20000, sessions_out=info)
    assert got == open(full).read()
    assert info[1] == want and len(want) > 3


@pytest.mark.parametrize("window", [25000, 0])
def test_multi_context_population_identical(tmp_path, window):
    syn, fa, sam, bam = _data(tmp_path, genome=pysynth.CUSTOM, custom_len=150000, seed=84, snv_rate=2e-3, indel_rate=5e-4,
                              n_samples=8, depth=6)
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    syn.close()
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setOutFilename(os.path.join(str(tmp_path), "full.vcf"))
    d.run(bams).close()
    want = open(d.outFilename).read()
    got = call_population_multi(fa, bams, os.path.join(str(tmp_path), "multi.vcf"), [0, 0], window=window)
    assert got == want
    assert sum(1 for l in want.splitlines() if "TYPE=INDEL" in l or "TYPE=STR" in l) > 3


def test_cli_devices_option(tmp_path):
    """`ngsep-amd SingleSampleVariantsDetector ... -devices 0,0 -window 30000` == the one-device CLI run"""
    import subprocess
    syn, fa, sam, bam = _data(tmp_path, genome=pysynth.CUSTOM, custom_len=120000, seed=85, snv_rate=2e-3, indel_rate=4e-4,
                              depth=15)
    syn.close()
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ngsepcore_amd", "lib", "ngsep-amd")
    one, two = os.path.join(str(tmp_path), "one"), os.path.join(str(tmp_path), "two")
    subprocess.run([cli, "SingleSampleVariantsDetector", "-i", bam, "-r", fa, "-o", one], check=True)
    subprocess.run([cli, "SingleSampleVariantsDetector", "-i", bam, "-r", fa, "-o", two, "-devices", "0,0", "-window", "30000"],
                   check=True)
    assert open(two + ".vcf").read() == open(one + ".vcf").read()
