"""BASELINE.json configs[1] (yeast 30x), configs[2] (human chr20 30x) and a configs[3] contig (human WGS 30x, chr21
of the bench's 8-GPU shard 0) at full size: the HIP VCF equals,
byte for byte, the oracle's VCF committed as tests/golden/<name>.vcf.gz (md5 and record count in
tests/golden/full_sizes.json, made by make_golden.py --full in the build container).  The data is
regenerated here from the same seeds; at 30x the scan's count bound drops ~98.6 % of the candidates, so
these runs put the pruning of whole genomes under the oracle's check."""
import gzip
import hashlib
import json
import os

import pytest

import pysynth
from ngsepcore_amd import GpuPileupSession

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = json.load(open(os.path.join(GOLDEN, "full_sizes.json")))


def _md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def _first_diff(got_path, name):
    want = gzip.open(os.path.join(GOLDEN, name + ".vcf.gz"), "rt").read().splitlines()
    got = open(got_path).read().splitlines()
    for k, (a, b) in enumerate(zip(want, got)):
        if a != b:
            return f"line {k + 1}: oracle {a!r} != gpu {b!r}"
    return f"line counts {len(want)} vs {len(got)}"


# chr1 (249 Mb) is compared in the staged shard-0 run only (tests/test_gpu_wgs_shard.py)
@pytest.mark.parametrize("name", sorted(n for n in CASES if n != "configs3_wgs_chr1_30x"))
def test_full_size_vcf_identical(tmp_path, name):
    case = CASES[name]
    syn = pysynth.Synth(**case["synth"])
    d = str(tmp_path)
    fa, bam = os.path.join(d, "g.fa"), os.path.join(d, "g.bam")
    pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
    pysynth.lib().ngs_synth_write_bam(syn.h, bam.encode())
    # path B: BAM on disk -> VCF (the drop-in for SingleSampleVariantsDetector)
    out = os.path.join(d, "b.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.processFile(bam, out)
        st = s.stats()
    assert st.positions_genotyped == case["positions_genotyped"]
    assert _md5(out) == case["vcf_md5"], _first_diff(out, name)
    # the bench's staged path over the same reads (resident layout, two passes in flight)
    out2 = os.path.join(d, "a.vcf")
    with GpuPileupSession() as s:
        for n, q in syn.contigs():
            s.set_reference(n, q)
        s.stage(syn.batch())
        s.stage_finish()
        s.submit_staged()
        s.submit_staged()
        s.collect_staged()
        s.collect_staged()
        s.write_vcf(out2)
    syn.close()
    assert _md5(out2) == case["vcf_md5"], _first_diff(out2, name)


POP_JSON = os.path.join(GOLDEN, "full_sizes_pop.json")
POP_CASES = json.load(open(POP_JSON)) if os.path.exists(POP_JSON) else {}


def _first_diff_pop(got_path, name):
    want = gzip.open(os.path.join(GOLDEN, name + ".vcf.gz"), "rt").read().splitlines()
    got = open(got_path).read().splitlines()
    for k, (a, b) in enumerate(zip(want, got)):
        if a != b:
            return f"line {k + 1}: oracle {a[:300]!r} != gpu {b[:300]!r}"
    return f"line counts {len(want)} vs {len(got)}"


@pytest.mark.parametrize("name", sorted(POP_CASES))
def test_full_size_population_vcf_identical(tmp_path, name):
    """configs[4] at one GPU's full shard (200 samples x 10x, chrIV): the population VCF of
    MultisampleVariantsDetector path B (200 sample BAMs) and of the bench's pipelined staged path equal the
    oracle's byte for byte."""
    from ngsepcore_amd import MultisampleVariantsDetector, default_params
    case = POP_CASES[name]
    syn = pysynth.Synth(**case["synth"])
    d = str(tmp_path)
    fa = os.path.join(d, "g.fa")
    pysynth.lib().ngs_synth_write_fasta(syn.h, fa.encode())
    bams = syn.write_sample_bams(os.path.join(d, "pop"))
    mvd = MultisampleVariantsDetector()
    mvd.setGenome(fa)
    mvd.setOutFilename(os.path.join(d, "b.vcf"))
    mvd.run(bams).close()
    assert _md5(mvd.outFilename) == case["vcf_md5"], _first_diff_pop(mvd.outFilename, name)
    for b in bams:
        os.remove(b)
    # the bench's path: staged population, two passes in flight
    p = default_params()
    p.multisample = 1
    out2 = os.path.join(d, "a.vcf")
    n = max(1, syn.params.n_samples)
    with GpuPileupSession(p) as s:
        s.set_samples([(f"S{k:03d}", f"S{k:03d}") for k in range(n)])
        for nm, q in syn.contigs():
            s.set_reference(nm, q)
        s.stage(syn.batch())
        s.stage_finish()
        s.submit_staged()
        s.submit_staged()
        s.collect_staged()
        s.collect_staged()
        s.write_population_vcf(out2)
    syn.close()
    assert _md5(out2) == case["vcf_md5"], _first_diff_pop(out2, name)
