"""GPU parity of CoverageStats (coverage.hip) against the oracle's CoverageStatisticsCalculator restatement
(discovery/CoverageStatisticsCalculator.java:108-216): the printed histograms must be identical (integer
work: bit-exact)."""
import os
import subprocess

import pytest

import coverage_kat
import ngsep_oracle
import pysynth
from ngsepcore_amd import CoverageStatisticsCalculator, GpuPileupSession, default_params

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def gpu_text(bam, out, fa=None, **setters):
    calc = CoverageStatisticsCalculator()
    if fa:
        calc.setGenome(fa)
    for k, v in setters.items():
        getattr(calc, k)(v)
    calc.processFile(bam, out)
    return open(out).read(), calc


@pytest.mark.parametrize("max_cov", [1024, 300, 3, 1])
def test_kat_identical(tmp_path, max_cov):
    """Indels, N skips longer than a tile, soft clips, secondary / low-MAPQ / unmapped records."""
    fa, sam = coverage_kat.write(tmp_path)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "kat.bam"))
    o = os.path.join(str(tmp_path), "o.txt")
    ngsep_oracle.run_coverage(fa, sam, o, max_coverage=max_cov)
    g, calc = gpu_text(bam, os.path.join(str(tmp_path), "g.txt"), fa, setMaxCoverage=max_cov)
    assert g == open(o).read()
    assert g == coverage_kat.text(*coverage_kat.expected(max_cov))


def test_kat_without_genome(tmp_path):
    """-r is optional for CoverageStats: sequences come from the BAM header."""
    fa, sam = coverage_kat.write(tmp_path)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "kat.bam"))
    g, _ = gpu_text(bam, os.path.join(str(tmp_path), "g.txt"))
    assert g == coverage_kat.text(*coverage_kat.expected(300))


@pytest.mark.parametrize("kw,min_mq,max_cov", [
    ({"depth": 10, "seed": 1}, 20, 300),
    ({"depth": 30, "seed": 7, "secondary_rate": 0.02, "lowmq_rate": 0.05, "dup_rate": 0.01, "softclip_rate": 0.05}, 20, 300),
    ({"depth": 30, "seed": 8, "secondary_rate": 0.02, "lowmq_rate": 0.05}, 4, 40),
    ({"depth": 60, "seed": 9, "dup_rate": 0.05}, 20, 50),
])
def test_yeast_identical(tmp_path, kw, min_mq, max_cov):
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, **kw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    o = os.path.join(str(tmp_path), "o.txt")
    _, _, _, _, ost = ngsep_oracle.run_coverage(fa, sam, o, min_mq=min_mq, max_coverage=max_cov)
    g, calc = gpu_text(bam, os.path.join(str(tmp_path), "g.txt"), fa, setMinMQ=min_mq, setMaxCoverage=max_cov)
    assert g == open(o).read()
    assert sum(calc.getCoverageCounts()) + calc.getHighCoverageCount() == ost.positions_genotyped


def test_path_a_batches_equal_path_b(tmp_path):
    """Reader-filtered batches through ngsep_process_alignments == the BAM path (no secondary / low MAPQ in
    the data, so the synthetic batch view's default reader filters change nothing)."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=20, seed=4, secondary_rate=0.0, lowmq_rate=0.0)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    a = CoverageStatisticsCalculator()
    a.processBatches([syn.batch()], contigs=syn.contigs())
    syn.close()
    b, _ = gpu_text(bam, os.path.join(str(tmp_path), "g.txt"), fa)
    assert a.printCoverageStats() == b
    o = os.path.join(str(tmp_path), "o.txt")
    ngsep_oracle.run_coverage(fa, sam, o)
    assert b == open(o).read()


def test_staged_runs_accumulate(tmp_path):
    """Staged entry points (bench): each run adds one pass of histograms; clear resets."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=10, seed=1)
    p = default_params()
    p.coverage_stats, p.process_secondary, p.max_alns_per_start = 1, 1, 100
    import ctypes
    with GpuPileupSession(p) as s:
        for name, seq in syn.contigs():
            s.set_reference(name, seq)
        s.stage(syn.batch())
        s.stage_finish()
        n = p.max_coverage
        outs = []
        for _ in range(3):
            s.run_staged()
            a = (ctypes.c_int64 * n)()
            s._check(s._lib.ngsep_fetch_coverage(s._ctx, a, None, None, None))
            outs.append(list(a))
        s.release_staged()
    syn.close()
    assert outs[1] == [2 * v for v in outs[0]] and outs[2] == [3 * v for v in outs[0]]
    assert sum(outs[0]) > 200000          # chrI 10x: ~230 kb covered


def test_cli(tmp_path):
    fa, sam = coverage_kat.write(tmp_path)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "kat.bam"))
    exe = os.path.join(ROOT, "ngsepcore_amd", "lib", "ngsep-amd")
    out = os.path.join(str(tmp_path), "cli.txt")
    subprocess.run([exe, "CoverageStats", "-i", bam, "-o", out, "-r", fa, "-minMQ", "20"], check=True, timeout=60)
    assert open(out).read() == coverage_kat.text(*coverage_kat.expected(300))
    r = subprocess.run([exe, "CoverageStats", "-i", bam], check=True, timeout=60, capture_output=True, text=True)
    assert r.stdout == coverage_kat.text(*coverage_kat.expected(300))


@pytest.mark.parametrize("name", ["c1_chrI_10x", "edge_2contigs_25x"])
def test_golden_coverage(tmp_path, name):
    """HIP path vs the committed oracle fixtures (tests/golden/*.coverage.txt), no oracle run needed."""
    import hashlib
    import importlib.util
    golden = os.path.join(ROOT, "tests", "golden")
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(golden, "make_golden.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    skw, _ = m.CASES[name]
    min_mq, max_cov = m.COVERAGE_CASES[name]
    syn = pysynth.Synth(**skw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), name))
    syn.close()
    assert hashlib.md5(open(sam, "rb").read()).hexdigest() == open(os.path.join(golden, name + ".sam.md5")).read().strip()
    g, _ = gpu_text(bam, os.path.join(str(tmp_path), "g.txt"), fa, setMinMQ=min_mq, setMaxCoverage=max_cov)
    assert g == open(os.path.join(golden, name + ".coverage.txt")).read()
