"""Alignments with indels.

Default (params.indel_passthrough = 0): the indel realigner's regions are replayed on the host (realign.cpp:
alignment edits, span calls, allele clusters, indel genotypes, the listener's span rules) and their span-1
columns genotyped on the device; the WHOLE VCF -- indel / STR records, SNVs of realigned alignments,
TYPE=EMBEDDED with -embeddedSNVs -- must equal the oracle's (oracle/ngsep_oracle_indel.inc).  Parity here is
against the oracle restatement only: the reference holds no indel fixture (parity unpinned).

Pass-through (indel_passthrough = 1, the ABI 5 behaviour): the device path carves the indel realigner's
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
    p = default_params()
    p.indel_passthrough = 1
    s = GpuPileupSession(p)
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
    p = gpu_params(indel_passthrough=1)
    if win:
        p.window_positions = win
    with GpuPileupSession(p) as s:
        s.load_fasta(fa)
        s.processFile(bam, g)
        carved = s.carved_regions()
        st = s.stats()
    assert len(carved) > 2
    if win:
        with GpuPileupSession(gpu_params(indel_passthrough=1)) as s:
            s.load_fasta(fa)
            s.processFile(bam, g + ".whole")
            assert s.carved_regions() == carved
        assert open(g).read() == open(g + ".whole").read()
    ro, rg = _outside(o, carved), _outside(g, carved)
    assert rg == [l for l in open(g) if not l.startswith("#")]      # no call inside a carved region
    assert ro == rg and len(rg) > 50
    # every covered position is either genotyped on the device or inside a carved region
    assert st.positions_genotyped + st.carved_positions == ost.positions_genotyped


def _records(vcf):
    return [l for l in open(vcf) if not l.startswith("#")]


@pytest.mark.gpu
@pytest.mark.parametrize("kw,opts", [
    (dict(depth=25, seed=32, indel_rate=1e-4), {}),
    (dict(depth=15, seed=33, indel_rate=3e-4, quality_model=2, snv_rate=3e-3), {}),
    (dict(depth=25, seed=32, indel_rate=1e-4), dict(window_positions=40000)),
    (dict(depth=30, seed=34, indel_rate=1e-3, snv_rate=2e-2, n_contigs=1), dict(call_embedded=1)),
    (dict(depth=20, seed=35, indel_rate=2e-4, quality_model=2), dict(min_quality=0, ploidy=1)),
])
def test_indel_regions_vcf_identical(tmp_path, kw, opts):
    """The realigner's regions called here: the WHOLE VCF equals the oracle's (indel / STR records, the
    realigned alignments' SNVs, embedded SNVs), no region is handed back, every covered position is genotyped;
    a window cut (window_positions) changes nothing."""
    syn = pysynth.Synth(genome=pysynth.YEAST, **{"n_contigs": 2, **kw})
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "ind"))
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    oopts = {k: v for k, v in opts.items() if k != "window_positions"}
    ost = ngsep_oracle.run_ssvd(fa, sam, o, **oopts)
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        s.processFile(bam, g)
        assert s.carved_regions() == []
        st = s.stats()
    ro, rg = _records(o), _records(g)
    n_indel = sum(1 for l in ro if "TYPE=INDEL" in l or "TYPE=STR" in l)
    assert n_indel > 3
    if opts.get("call_embedded"):
        assert any("TYPE=EMBEDDED" in l for l in ro)
    for a, b in zip(ro, rg):
        assert a == b, (a, b)
    assert len(ro) == len(rg)
    assert st.positions_genotyped == ost.positions_genotyped


def _str_file(path, syn, seed, around=()):
    """A -knownSTRs regions file: random regions (some pairs 0-6 bp apart, exercising mergeSTRs' gap and overlap
    rules), regions around the given positions (indel events), space- and tab-separated lines, and lines the reference
    skips (unknown sequence, unparsable numbers)."""
    import random
    names = [n for n, _ in syn.contigs()]
    seqs = [q for _, q in syn.contigs()]
    rnd = random.Random(seed)
    lines = []
    for _ in range(250):
        c = rnd.randrange(len(names))
        a = rnd.randrange(1, len(seqs[c]) - 60)
        b = a + rnd.randrange(0, 30)
        lines.append(f"{names[c]}\t{a}\t{b}")
        if rnd.random() < 0.4:
            g = rnd.randrange(0, 7)
            lines.append(f"{names[c]} {b + g} {b + g + rnd.randrange(1, 12)}")
        if rnd.random() < 0.1:      # 3-5 bp apart: mergeSTRs compares the reference suffix / prefix
            lines.append(f"{names[c]}\t{b + 4}\t{b + 4 + rnd.randrange(6, 15)}")
    for name, p in around:
        lines.append(f"{name}\t{p - rnd.randrange(0, 4)}\t{p + rnd.randrange(2, 12)}")
    lines += ["chrNotInGenome\t5\t10", "a line that does not parse", f"{names[0]}\tx\t5", f"{names[0]}\t7"]
    rnd.shuffle(lines)
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


@pytest.mark.gpu
@pytest.mark.parametrize("kw,opts", [
    (dict(depth=25, seed=32, indel_rate=1e-4), {}),
    (dict(depth=25, seed=36, indel_rate=3e-4, snv_rate=3e-3), dict(call_embedded=1)),
    (dict(depth=20, seed=37, indel_rate=2e-4, quality_model=2), dict(window_positions=40000)),
])
def test_known_strs_vcf_identical(tmp_path, kw, opts):
    """-knownSTRs (SingleSampleVariantsDetector.findSNVS :906-912): the input STRs become the indel realigner's input
    variants (IndelRealignerPileupListener.java:85-153), so every STR opens a realigned region; TYPE=STR records,
    embedded positions and lastIndelEnd follow the listener (:146-161, :264).  The WHOLE VCF equals the oracle's."""
    syn = pysynth.Synth(genome=pysynth.YEAST, **{"n_contigs": 2, **kw})
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "ind"))
    o0 = os.path.join(str(tmp_path), "o0.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o0)
    around = [(l.split("\t")[0], int(l.split("\t")[1])) for l in _records(o0) if "TYPE=INDEL" in l][::2]
    strs = os.path.join(str(tmp_path), "strs.txt")
    _str_file(strs, syn, kw["seed"], around)
    syn.close()
    o = os.path.join(str(tmp_path), "o.vcf")
    oopts = {k: v for k, v in opts.items() if k != "window_positions"}
    ost = ngsep_oracle.run_ssvd(fa, sam, o, known_strs=strs.encode(), **oopts)
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        s.set_known_strs(strs)
        s.processFile(bam, g)
        assert s.carved_regions() == []
        st = s.stats()
    ro, rg = _records(o), _records(g)
    assert sum(1 for l in ro if "TYPE=STR" in l) > 5
    assert ro != _records(o0)
    for a, b in zip(ro, rg):
        assert a == b, (a, b)
    assert len(ro) == len(rg)
    assert st.positions_genotyped == ost.positions_genotyped


def _reference_strs(tmp_path):
    """the reference's own -knownSTRs input (training/Saccharomyces_cerevisiae_STRs.txt: TRF regions over sacCer3, 14,063
    lines, overlapping and nested ones included), as committed in tests/golden/reference_strs.txt.gz (its sequence,
    first and last fields; tests/golden/make_golden.py --strs)"""
    import gzip
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_strs.txt.gz")
    path = os.path.join(str(tmp_path), "Saccharomyces_cerevisiae_STRs.txt")
    with gzip.open(src, "rb") as g, open(path, "wb") as f:
        f.write(g.read())
    return path


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [{}, dict(call_embedded=1)])
def test_reference_strs_vcf_identical(tmp_path, opts):
    """-knownSTRs with the reference's own STR file on a synthetic genome of sacCer3's names and lengths (chrI, chrII) with
    donor indels: makeNonRedundantSTRs over its regions, every merged STR a realigner input variant; the WHOLE VCF equals
    the oracle's through ngsep_call_bam.  (The regions are the reference's; the bases they cover are synthetic, so most
    are not repeats here -- the realigner and the listener treat them as input STRs all the same.)"""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=15, seed=41, indel_rate=3e-4, snv_rate=2e-3)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "yst"))
    syn.close()
    strs = _reference_strs(tmp_path)
    o = os.path.join(str(tmp_path), "o.vcf")
    ost = ngsep_oracle.run_ssvd(fa, sam, o, known_strs=strs.encode(), **opts)
    g = os.path.join(str(tmp_path), "g.vcf")
    with GpuPileupSession(gpu_params(**opts)) as s:
        s.load_fasta(fa)
        s.set_known_strs(strs)
        s.processFile(bam, g)
        assert s.carved_regions() == []
        st = s.stats()
    ro, rg = _records(o), _records(g)
    assert sum(1 for l in ro if "TYPE=STR" in l) > 10
    for a, b in zip(ro, rg):
        assert a == b, (a, b)
    assert len(ro) == len(rg)
    assert st.positions_genotyped == ost.positions_genotyped


@pytest.mark.gpu
@pytest.mark.parametrize("opts", [{}, dict(call_embedded=1)])
def test_reference_strs_population_vcf_identical(tmp_path, opts):
    """MultisampleVariantsDetector -knownSTRs (:439-446) with the reference's STR file: 12 samples on sacCer3's chrI
    with population indels; the WHOLE population VCF equals the oracle's (path B: one BAM per sample)."""
    from ngsepcore_amd import MultisampleVariantsDetector
    from helpers import diff_vcf
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=1, depth=8, seed=42, n_samples=12, indel_rate=4e-4, snv_rate=2e-3)
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "pop"))
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    syn.close()
    strs = _reference_strs(tmp_path)
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_mvd(fa, sam, o, 0.0, known_strs=strs.encode(), **opts)
    assert sum(1 for l in _records(o) if "TYPE=STR" in l) > 3
    d = MultisampleVariantsDetector()
    for k, v in opts.items():
        setattr(d.params, k, v)
    d.setGenome(fa)
    d.setKnownSTRsFile(strs)
    d.setOutFilename(os.path.join(str(tmp_path), "g.vcf"))
    d.run(bams).close()
    diff = diff_vcf(o, d.outFilename)
    assert not diff, "\n".join(diff[:20])
