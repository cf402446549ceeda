"""CoverageStats restatement (oracle) pinned by hand-derived known answers, and the host-side contract of
the GPU entry points (no GPU needed).  The reference ships no test or fixture for
CoverageStatisticsCalculator, so beyond these KATs the restatement is parity unpinned."""
import ctypes
import os

import pytest

import coverage_kat
import ngsep_oracle
from ngsepcore_amd import CoverageStatisticsCalculator, NgsepError, _lib


@pytest.mark.parametrize("max_cov", [300, 3, 2, 1])
def test_oracle_coverage_kat(tmp_path, max_cov):
    fa, sam = coverage_kat.write(tmp_path)
    out = os.path.join(str(tmp_path), "o.txt")
    c, u, hi, hu, st = ngsep_oracle.run_coverage(fa, sam, out, max_coverage=max_cov)
    ec, eu, ehi, ehu = coverage_kat.expected(max_cov)
    c[0] = u[0] = 0
    assert (c, u, hi, hu) == (ec, eu, ehi, ehu)
    assert open(out).read() == coverage_kat.text(ec, eu, ehi, ehu)
    assert st.alignments_admitted == 8


def test_oracle_coverage_min_mq(tmp_path):
    """-minMQ decides isUnique (ReadAlignmentFileReader.isMultiple): r2 (MAPQ 10) becomes unique at 5."""
    fa, sam = coverage_kat.write(tmp_path)
    c10, u10, *_ = ngsep_oracle.run_coverage(fa, sam, os.path.join(str(tmp_path), "a.txt"), min_mq=10)
    c20, u20, *_ = ngsep_oracle.run_coverage(fa, sam, os.path.join(str(tmp_path), "b.txt"), min_mq=20)
    assert c10[1:] == c20[1:]
    assert sum(k * v for k, v in enumerate(u10)) == sum(k * v for k, v in enumerate(u20)) + 10


def test_oracle_same_start_cap_100(tmp_path):
    """processFile sets maxAlnsPerStartPos 100 (:112): 150 reads at one start -> depth 100."""
    fa = os.path.join(str(tmp_path), "r.fa")
    open(fa, "w").write(">c1\n" + "A" * 200 + "\n")
    sam = os.path.join(str(tmp_path), "a.sam")
    with open(sam, "w") as f:
        f.write("@SQ\tSN:c1\tLN:200\n")
        for k in range(150):
            f.write(f"q{k}\t0\tc1\t10\t60\t5M\t*\t0\t0\tAAAAA\tIIIII\n")
    c, u, hi, hu, st = ngsep_oracle.run_coverage(fa, sam, os.path.join(str(tmp_path), "o.txt"))
    assert c[100] == 5 and u[100] == 5 and sum(c[1:]) == 5
    assert st.alignments_admitted == 100


def test_coverage_options_validated():
    calc = CoverageStatisticsCalculator()
    p = calc.params
    assert (p.coverage_stats, p.process_secondary, p.max_alns_per_start, p.max_coverage) == (1, 1, 100, 300)
    p.max_coverage = 5000
    ctx = ctypes.c_void_p()
    lib = _lib.load()
    rc = lib.ngsep_open(0, ctypes.byref(p), ctypes.byref(ctx))
    assert rc == _lib.NGSEP_E_UNSUPPORTED
    lib.ngsep_close(ctx)


@pytest.mark.skipif(_lib.load().ngsep_device_count() > 0, reason="checks the no-GPU failure mode")
def test_coverage_without_device_fails_loudly(tmp_path):
    import pysynth
    fa, sam = coverage_kat.write(tmp_path)
    bam = pysynth.sam_to_bam(sam, os.path.join(str(tmp_path), "kat.bam"))
    calc = CoverageStatisticsCalculator()
    with pytest.raises(NgsepError) as e:
        calc.processFile(bam, os.path.join(str(tmp_path), "g.txt"))
    assert e.value.code == _lib.NGSEP_E_DEVICE
