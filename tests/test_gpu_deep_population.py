"""MultisampleVariantsDetector at any depth (MultisampleVariantsDetector.java:522-558 -> genotypeVariant :674-693 ->
PileupRecord.getAlleleCalls(span, readGroups) :104-111): the reference genotypes a population position whatever its
per-sample depth, so the HIP path refuses none.

* KLM's counting scan (k_scan_pop<true>) holds per-position byte counters; the tiles where some sample is deeper than
  kKlmCountMaxCov (127) take the exact-bound scan (k_scan_pop<false>), launched over those tiles only.
* KPM / k_stage_a gather each sample's column into LDS while (S + 1) x the per-sample coverage bound fits
  kPopGatherCap, into a device scratch otherwise (GCOL).

Bar: the population VCF text identical to the oracle's (oracle/ngsep_oracle.c ngo_run_mvd).
"""
import os

import pytest

from helpers import diff_vcf
import pysynth
from test_gpu_multisample import gpu_mvd, n_records, oracle_mvd, population

pytestmark = pytest.mark.gpu


def _with_env(name, fn):
    os.environ[name] = "1"
    try:
        return fn()
    finally:
        del os.environ[name]


def test_deep_population_every_tile_exact_scan(tmp_path):
    """8 samples at 150x each: every KLM tile is deeper than the counting scan's byte counters carry, so the whole run
    takes k_scan_pop<false>; staged, streamed and (NGSEP_POP_GCOL) scratch-column runs all equal the oracle."""
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=9000, seed=41, n_samples=8, depth=150,
                                   snv_rate=3e-3, quality_model=2)
    o = oracle_mvd(tmp_path, fa, sam)
    assert n_records(o) > 10
    for staged in (False, True):
        g, st = gpu_mvd(tmp_path, syn, rgs, staged=staged)
        d = diff_vcf(o, g)
        assert not d, "\n".join(d[:20])
    g, st = _with_env("NGSEP_POP_GCOL", lambda: gpu_mvd(tmp_path, syn, rgs, staged="pipelined"))
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    # one-stage KPM over every column, from the scratch too
    os.environ["NGSEP_KPM_ONE_STAGE"] = "1"
    try:
        g, st = _with_env("NGSEP_POP_GCOL", lambda: gpu_mvd(tmp_path, syn, rgs, staged=True))
    finally:
        del os.environ["NGSEP_KPM_ONE_STAGE"]
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])


def test_collapsed_repeat_200_samples(tmp_path):
    """configs[4]'s shape (200 samples at 10x) with a 2 kb collapsed repeat where every sample is ~300x deep (yeast rDNA,
    centromeres): the counting scan runs everywhere else, the exact-bound scan on the repeat's tiles, and KPM's columns
    ((S + 1) x ~300 codes, past the 40 KB of LDS a position's columns had) come from the scratch.  The oracle takes
    75 s here, so its VCF is the committed golden tests/golden/deep_repeat_200x10x.vcf.gz (md5 in full_sizes_pop.json,
    made by make_golden.py --full-pop; path B and the pipelined staged path are compared with it by
    test_gpu_full_size.py).  Here: path A streamed (ngsep_process_alignments) and the one-stage KPM."""
    import gzip
    import hashlib
    import json
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    case = json.load(open(os.path.join(golden, "full_sizes_pop.json")))["deep_repeat_200x10x"]
    syn = pysynth.Synth(**case["synth"])
    n = syn.params.n_samples
    rgs = [(f"S{k:03d}", f"S{k:03d}") for k in range(n)]
    want = gzip.open(os.path.join(golden, "deep_repeat_200x10x.vcf.gz"), "rb").read()
    assert hashlib.md5(want).hexdigest() == case["vcf_md5"]
    assert any(7001 <= int(l.split(b"\t")[1]) <= 9000 for l in want.splitlines() if not l.startswith(b"#"))
    for env in (None, "NGSEP_KPM_ONE_STAGE"):
        if env:
            os.environ[env] = "1"
        try:
            g, st = gpu_mvd(tmp_path, syn, rgs)
        finally:
            if env:
                del os.environ[env]
        got = open(g, "rb").read()
        if got != want:
            d = [f"line {k + 1}: {a[:200]!r} != {b[:200]!r}" for k, (a, b) in
                 enumerate(zip(want.splitlines(), got.splitlines())) if a != b]
            raise AssertionError((env, len(want.splitlines()), len(got.splitlines()), d[:5]))


def test_collapsed_repeat_pool_ploidy(tmp_path):
    """The pool algorithm (ploidy 4, KPM's pool branch walks its scratch column per frequency hypothesis) on a
    population with a collapsed repeat: identical to the oracle."""
    syn, fa, sam, rgs = population(tmp_path, genome=pysynth.CUSTOM, custom_len=8000, seed=43, n_samples=24, depth=10,
                                   snv_rate=3e-3, hot_first=3001, hot_len=1200, hot_depth=200)
    o = oracle_mvd(tmp_path, fa, sam, ploidy=4)
    assert n_records(o) > 10
    g, st = _with_env("NGSEP_POP_GCOL", lambda: gpu_mvd(tmp_path, syn, rgs, staged=True, ploidy=4))
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
    g, st = gpu_mvd(tmp_path, syn, rgs, ploidy=4)
    d = diff_vcf(o, g)
    assert not d, "\n".join(d[:20])
