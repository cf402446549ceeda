"""BASELINE.json configs[3] at the bench's real device run: shard 0 of the 8-GPU contig split (chr1 + chr15 +
chr21, 397.7 M positions, 79.7 M reads) staged into ONE GpuPileupSession exactly as `bench.py --config wgs
--wgs-shards 8 --wgs-shard 0` does it (each synthetic contig's reads index its own sequence list and are shifted
to the session's ids; one device run whose read-group layout holds 12 G read bases), run as the bench's pipelined
passes (ngsep_submit_staged / ngsep_collect_staged, two in flight).  Each sequence's block of the VCF equals, byte
for byte, the oracle's VCF of that sequence (tests/golden/configs3_wgs_chr{1,15,21}_30x.vcf.gz, made by
make_golden.py --full; chr21 is last, so its reads sit > 11 GB into the layout).  Reference: per-sequence output of
SingleSampleVariantsDetector.findSNVS / saveSequenceVariants (SingleSampleVariantsDetector.java:896-968)."""
import ctypes
import gzip
import json
import os

import numpy as np
import pytest

import pysynth
from ngsepcore_amd import GpuPileupSession
from ngsepcore_amd.sharding import assign_contigs

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = json.load(open(os.path.join(GOLDEN, "full_sizes.json")))

HUMAN = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555), ("chr5", 181538259),
         ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636), ("chr9", 138394717), ("chr10", 133797422),
         ("chr11", 135086622), ("chr12", 133275309), ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189),
         ("chr16", 90338345), ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
         ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]


def _golden_records(name):
    with gzip.open(os.path.join(GOLDEN, name + ".vcf.gz"), "rt") as f:
        return [l for l in f if not l.startswith("#")]


def test_wgs_shard0_staged_run_equals_oracle(tmp_path):
    shard = assign_contigs(HUMAN, 8)[0]
    assert shard == ["chr1", "chr15", "chr21"] or sorted(shard) == ["chr1", "chr15", "chr21"]
    idx = [k for k, (n, _) in enumerate(HUMAN) if n in shard]
    out = os.path.join(str(tmp_path), "shard0.vcf")
    with GpuPileupSession() as s:
        positions = 0
        for k in idx:
            syn = pysynth.Synth(genome=pysynth.HUMAN, depth=30, seed=4, contig_first=k, n_contigs=1, rng_per_contig=1)
            base = len(s.sequence_names())
            for name, seq in syn.contigs():
                s.set_reference(name, seq)
            batch = syn.batch()
            if base:
                sid = np.ascontiguousarray(np.ctypeslib.as_array(batch.seq_id, shape=(batch.n_reads,)) + base, dtype=np.int32)
                batch.seq_id = sid.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            s.stage(batch)
            syn.close()
        s.stage_finish()
        st = s.stats()
        s.submit_staged()
        s.submit_staged()
        s.collect_staged()
        s.collect_staged()
        s.write_vcf(out)
    want_pos = sum(CASES[f"configs3_wgs_{HUMAN[k][0]}_30x"]["positions_genotyped"] for k in idx)
    assert st.positions_genotyped == want_pos
    got = {}
    with open(out) as f:
        for l in f:
            if not l.startswith("#"):
                got.setdefault(l.split("\t", 1)[0], []).append(l)
    assert sorted(got) == sorted(HUMAN[k][0] for k in idx)
    for k in idx:
        name = HUMAN[k][0]
        want = _golden_records(f"configs3_wgs_{name}_30x")
        g = got[name]
        assert len(g) == len(want) == CASES[f"configs3_wgs_{name}_30x"]["vcf_records"], name
        for a, b in zip(want, g):
            assert a == b, f"{name}: oracle {a!r} != gpu {b!r}"
