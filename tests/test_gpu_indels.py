"""Alignments with indels (first step): the device path carves the indel realigner's
reach out of its plan (ngsep_gpu.h ngsep_fetch_carved_regions) and calls every other position.

The reference runs IndelRealignerPileupListener (discovery/IndelRealignerPileupListener.java:85-526) before
the SNV listener; around an indel event it realigns every overlapping alignment and calls indels, so the
SNV calls there depend on it.  Away from the events it is a pass-through (:85-126) -- the oracle with
indel_passthrough=1 is then the reference, and the calls outside the carved regions must be identical.
Data: seeded donor indels of 1-10 bp (tools/synth indel_rate), reads with I/D CIGAR items across them."""
import os

import pytest

import ngsep_oracle
import pysynth
from ngsepcore_amd import GpuPileupSession, _lib, default_params
from helpers import gpu_params


def _carve_expected(syn):
    """[(seq, first, last)]: every admitted alignment with I/D carves [first - R, last + indel bases + R],
    R = largest span + 100, merged per sequence (reads here: no same-start overflow, default filters)."""
    b = syn.batch()
    names = [n for n, _ in syn.contigs()]
    lens = [len(s) for _, s in syn.contigs()]
    per = {}
    spans = {}
    for i in range(b.n_reads):
        co, cn = b.cigar_off[i], b.cigar_n[i]
        cig = [b.cigar[co + k] for k in range(cn)]
        last = b.first[i] + sum(c // 8 for c in cig if c & 1) - 1
        s = b.seq_id[i]
        spans[s] = max(spans.get(s, 0), last - b.first[i] + 1)
        ind = sum(c // 8 for c in cig if (c & 7) in (1, 2))
        if ind:
            per.setdefault(s, []).append((b.first[i], last + ind))
    out = []
    for s in sorted(per):
        R = spans[s] + 100
        iv = sorted((max(1, a - R), min(lens[s], z + R)) for a, z in per[s])
        merged = []
        for a, z in iv:
            if merged and a <= merged[-1][1] + 1:
                merged[-1][1] = max(merged[-1][1], z)
            else:
                merged.append([a, z])
        out += [(names[s], a, z) for a, z in merged]
    return out


def test_carved_regions_host_geometry():
    """The carve intervals (host side, before any device work) on path A batches; the device step then
    fails loudly here (no GPU), after the regions are recorded."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, contig_first=1, depth=12, seed=31, indel_rate=2e-4, dup_rate=0)
    s = GpuPileupSession(default_params())
    for n, q in syn.contigs():
        s.set_reference(n, q)
    rc = s._lib.ngsep_process_alignments(s._ctx, __import__("ctypes").byref(syn.batch()))
    if rc == _lib.NGSEP_OK:
        rc = s._lib.ngsep_notify_end(s._ctx)
    got = s.carved_regions()
    want = _carve_expected(syn)
    s.close()
    syn.close()
    assert rc in (_lib.NGSEP_OK, _lib.NGSEP_E_DEVICE)
    assert len(want) > 3
    assert got == want


def _outside(vcf, carved):
    by = {}
    for n, a, z in carved:
        by.setdefault(n, []).append((a, z))
    out = []
    for l in open(vcf):
        if l.startswith("#"):
            continue
        f = l.split("\t", 2)
        p = int(f[1])
        if not any(a <= p <= z for a, z in by.get(f[0], [])):
            out.append(l)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kw,win", [(dict(depth=25, seed=32, indel_rate=1e-4), 0),
                                    (dict(depth=15, seed=33, indel_rate=3e-4, quality_model=2, snv_rate=3e-3), 0),
                                    (dict(depth=25, seed=32, indel_rate=1e-4), 40000)])
def test_calls_outside_carved_regions_identical(tmp_path, kw, win):
    """win > 0: ngsep_call_bam streams windows of `win` positions while it reads (engine.cpp stream_advance):
    the carved regions, the calls and the genotyped-position count do not depend on the cut."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, **kw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "ind"))
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    ost = ngsep_oracle.run_ssvd(fa, sam, o, indel_passthrough=1)
    g = os.path.join(str(tmp_path), "g.vcf")
    p = gpu_params()
    if win:
        p.window_positions = win
    with GpuPileupSession(p) as s:
        s.load_fasta(fa)
        s.processFile(bam, g)
        carved = s.carved_regions()
        st = s.stats()
    assert len(carved) > 2
    if win:
        with GpuPileupSession(gpu_params()) as s:
            s.load_fasta(fa)
            s.processFile(bam, g + ".whole")
            assert s.carved_regions() == carved
        assert open(g).read() == open(g + ".whole").read()
    ro, rg = _outside(o, carved), _outside(g, carved)
    assert rg == [l for l in open(g) if not l.startswith("#")]      # no call inside a carved region
    assert ro == rg and len(rg) > 50
    # every covered position is either genotyped on the device or inside a carved region
    assert st.positions_genotyped + st.carved_positions == ost.positions_genotyped
