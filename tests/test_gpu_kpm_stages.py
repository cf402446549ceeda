"""KPM's two stages (k_stage_a, then k_posterior_multi over the positions whose QS can pass) against the one-stage path
(NGSEP_KPM_ONE_STAGE=1, read once per process: run in a child process) and the oracle
(MultisampleVariantsDetector.onPileup :522-558 -- DESIGN.md section 3, "Two stages").

Cases: a small population; 100 samples at a high SNV rate, so that positions with more than 64 samples KLM could not
prove hom-ref exist (stage A passes them on whole); a low-coverage population, where many columns reach the exact bound
with one or two calls; het_rate 0.1 (the priors move the bound's thresholds).
"""
import os
import subprocess
import sys

import pytest

from helpers import diff_vcf, oracle_params_from
import ngsep_oracle
from test_gpu_multisample import gpu_mvd, n_records, population
import pysynth

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

CHILD = r"""
import json, os, sys
root = os.path.dirname({here!r})
for p in ({here!r}, root, os.path.join(root, "oracle"), os.path.join(root, "tools", "synth")):
    sys.path.insert(0, p)
import pysynth
from test_gpu_multisample import gpu_mvd, population
kw, opts, tmp = json.loads(sys.argv[1])
syn, fa, sam, rgs = population(tmp, genome=pysynth.CUSTOM, custom_len=40000, seed=9, **kw)
out, st = gpu_mvd(tmp, syn, rgs, **opts)
print(out)
"""


CASES = [
    (dict(n_samples=24, depth=10, snv_rate=2e-3), {}),
    (dict(n_samples=100, depth=8, snv_rate=8e-3), {}),
    (dict(n_samples=40, depth=3, snv_rate=3e-3), {}),
    (dict(n_samples=30, depth=10, snv_rate=3e-3), {"het_rate": 0.1}),
]


@pytest.mark.parametrize("kw,opts", CASES)
def test_two_stages_equal_one_stage_and_oracle(tmp_path, kw, opts):
    two_dir = tmp_path / "two"
    one_dir = tmp_path / "one"
    two_dir.mkdir()
    one_dir.mkdir()
    syn, fa, sam, rgs = population(two_dir, genome=pysynth.CUSTOM, custom_len=40000, seed=9, **kw)
    two, _ = gpu_mvd(two_dir, syn, rgs, **opts)
    import json
    env = dict(os.environ, NGSEP_KPM_ONE_STAGE="1")
    r = subprocess.run([sys.executable, "-c", CHILD.format(here=HERE), json.dumps([kw, opts, str(one_dir)])],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    one = r.stdout.strip().splitlines()[-1]
    d = diff_vcf(one, two)
    assert not d, "\n".join(d[:20])
    o = os.path.join(str(tmp_path), "oracle.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, 0.0, **oracle_params_from(opts))
    d = diff_vcf(o, two)
    assert not d, "\n".join(d[:20])
    assert n_records(o) > 10
