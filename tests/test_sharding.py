"""Contig sharding (ngsepcore_amd/sharding.py) on CPU: world_size-2 gloo process group.

The per-sequence caller here is the oracle restricted to one sequence (-querySeq), standing in for the
GPU caller of each rank (gpu_contig_caller); what is tested is the assignment, the gather of record
blocks to rank 0 and the merge, which must reproduce the single-process VCF byte for byte."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import ngsep_oracle
import pysynth
from ngsepcore_amd.sharding import assign_contigs, call_sharded, merge_vcf, split_vcf


def test_assign_contigs_balanced_and_deterministic():
    contigs = [("chrI", 230218), ("chrII", 813184), ("chrIII", 316620), ("chrIV", 1531933), ("chrV", 576874)]
    a = assign_contigs(contigs, 2)
    assert sorted(sum(a, [])) == sorted(c for c, _ in contigs)
    assert a == assign_contigs(contigs, 2)
    loads = [sum(dict(contigs)[c] for c in part) for part in a]
    assert max(loads) - min(loads) <= max(l for _, l in contigs)
    assert assign_contigs(contigs, 8)[5:] == [[], [], []]


def test_split_merge_roundtrip():
    text = "##fileformat=VCFv4.2\n#CHROM\tPOS\n" + "b\t5\n" + "a\t1\n" + "a\t9\n"
    h, blocks = split_vcf(text)
    assert h.count("\n") == 2 and blocks == {"b": "b\t5\n", "a": "a\t1\na\t9\n"}
    assert merge_vcf(h, blocks, ["b", "a"]) == text
    with pytest.raises(ValueError):
        merge_vcf(h, blocks, ["a"])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fa, sam, contigs, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        def call(name):
            out = os.path.join(out_dir, f"r{rank}_{name}.vcf")
            ngsep_oracle.run_ssvd(fa, sam, out, query_seq=name)
            return open(out).read()
        call_sharded(contigs, call, os.path.join(out_dir, "merged.vcf"), dist)
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_vcf_identical(tmp_path):
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=8, seed=3)
    contigs = [(n, len(s)) for n, s in syn.contigs()]
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    ngsep_oracle.run_ssvd(fa, sam, full)
    mp.spawn(_worker, args=(2, _free_port(), fa, sam, contigs, str(tmp_path)), nprocs=2, join=True)
    merged = open(os.path.join(str(tmp_path), "merged.vcf")).read()
    assert merged == open(full).read()
    assert len(split_vcf(merged)[1]) == 3


@pytest.mark.gpu
def test_gpu_contig_caller_merge_identical(tmp_path):
    """The production per-sequence caller (libngsep_amd path B with -querySeq) merged in reference order
    == the whole-genome GPU VCF (single process: the rank-0 view of the sharded run)."""
    from ngsepcore_amd import GpuPileupSession
    from ngsepcore_amd.sharding import gpu_contig_caller
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=12, seed=6)
    contigs = [(n, len(s)) for n, s in syn.contigs()]
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.processFile(bam, full)
    merged = call_sharded(contigs, gpu_contig_caller(fa, bam), os.path.join(str(tmp_path), "m.vcf"))
    assert merged == open(full).read()


def test_bam_header_sequences(tmp_path):
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=4, depth=2, seed=3)
    _, _, bam = syn.write(os.path.join(str(tmp_path), "h"))
    from ngsepcore_amd.sharding import bam_header_sequences
    assert bam_header_sequences(bam) == [(n, len(s)) for n, s in syn.contigs()]
    syn.close()


def _reordered_sam(src, dst, order):
    """the same records with the @SQ lines in another order (sorted by the new reference order)"""
    head, recs = [], []
    for l in open(src):
        (head if l.startswith("@") else recs).append(l)
    sq = {l.split("\t")[1][3:]: l for l in head if l.startswith("@SQ")}
    other = [l for l in head if not l.startswith("@SQ")]
    rank = {n: k for k, n in enumerate(order)}
    recs.sort(key=lambda l: (rank[l.split("\t")[2]], int(l.split("\t")[3])))
    with open(dst, "w") as f:
        f.writelines(other[:1] + [sq[n] for n in order] + other[1:] + recs)
    return dst


def test_two_rank_sharded_bam_order_differs_from_fasta(tmp_path):
    """BAM header order != FASTA order: the single-process run writes the sequences in BAM order, and so
    does the merge when its order comes from the BAM header."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=8, seed=4)
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "d"))
    names = [n for n, _ in syn.contigs()]
    lens = dict((n, len(s)) for n, s in syn.contigs())
    syn.close()
    order = [names[2], names[0], names[1]]
    sam2 = _reordered_sam(sam, os.path.join(str(tmp_path), "re.sam"), order)
    bam2 = pysynth.sam_to_bam(sam2, os.path.join(str(tmp_path), "re.bam"))
    from ngsepcore_amd.sharding import bam_header_sequences
    contigs = bam_header_sequences(bam2)
    assert [n for n, _ in contigs] == order and dict(contigs) == lens
    full = os.path.join(str(tmp_path), "full.vcf")
    ngsep_oracle.run_ssvd(fa, sam2, full)
    mp.spawn(_worker, args=(2, _free_port(), fa, sam2, contigs, str(tmp_path)), nprocs=2, join=True)
    merged = open(os.path.join(str(tmp_path), "merged.vcf")).read()
    assert merged == open(full).read()
    assert [l.split("\t")[0] for l in merged.splitlines() if not l.startswith("#")][0] == order[0]


@pytest.mark.gpu
def test_gpu_region_calls_merged_equal_whole_file(tmp_path):
    """ngsep_call_region_bam over pieces of every sequence (BAI seeks), concatenated in order == the
    whole-file GPU VCF; and call_bam_sharded on a BAM whose header order differs from the FASTA's."""
    from ngsepcore_amd import GpuPileupSession
    from ngsepcore_amd.sharding import bam_header_sequences, call_bam_sharded
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=15, seed=8, softclip_rate=0.05)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.processFile(bam, full)
    header, body = "", []
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        for name, L in bam_header_sequences(bam):
            cuts = [1, L // 3, L // 3 + 1, 2 * L // 3, 2 * L // 3 + 1, L]
            for a, b in ((cuts[0], cuts[1]), (cuts[2], cuts[3]), (cuts[4], cuts[5])):
                out = os.path.join(str(tmp_path), f"{name}_{a}.vcf")
                s._check(s._lib.ngsep_call_region_bam(s._ctx, bam.encode(), name.encode(), a, b, out.encode()))
                t = open(out).read()
                header = header or "".join(l for l in t.splitlines(True) if l.startswith("#"))
                body += [l for l in t.splitlines(True) if not l.startswith("#")]
    assert header + "".join(body) == open(full).read()
    names = [n for n, _ in bam_header_sequences(bam)]
    sam2 = _reordered_sam(sam, os.path.join(str(tmp_path), "re.sam"), [names[1], names[2], names[0]])
    bam2 = pysynth.sam_to_bam(sam2, os.path.join(str(tmp_path), "re.bam"))
    full2 = os.path.join(str(tmp_path), "full2.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.processFile(bam2, full2)
    merged = call_bam_sharded(fa, bam2, os.path.join(str(tmp_path), "m2.vcf"))
    assert merged == open(full2).read()


def _mvd_worker(rank, world, port, fa, sam, contigs, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        def call(name):
            out = os.path.join(out_dir, f"m{rank}_{name}.vcf")
            ngsep_oracle.run_mvd(fa, sam, out, query_seq=name)
            return open(out).read()
        call_sharded(contigs, call, os.path.join(out_dir, "merged_mvd.vcf"), dist)
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_population_vcf_identical(tmp_path):
    """MultisampleVariantsDetector split by sequence over two gloo ranks (the oracle restricted to each
    sequence as the per-rank caller): merged population VCF == the single-process one."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=6, seed=9, n_samples=6, snv_rate=2e-3)
    contigs = [(n, len(s)) for n, s in syn.contigs()]
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "p"))
    syn.close()
    full = os.path.join(str(tmp_path), "full_mvd.vcf")
    ngsep_oracle.run_mvd(fa, sam, full)
    mp.spawn(_mvd_worker, args=(2, _free_port(), fa, sam, contigs, str(tmp_path)), nprocs=2, join=True)
    merged = open(os.path.join(str(tmp_path), "merged_mvd.vcf")).read()
    assert merged == open(full).read()
    assert len(split_vcf(merged)[1]) == 3


@pytest.mark.gpu
def test_gpu_population_sharded_identical(tmp_path):
    """call_population_sharded (per-sequence population calls over the per-sample BAMs' indexes) == the
    single-process MultisampleVariantsDetector VCF on the same BAMs."""
    from ngsepcore_amd import MultisampleVariantsDetector
    from ngsepcore_amd.sharding import call_population_sharded
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=8, seed=10, n_samples=12, snv_rate=2e-3)
    fa, _, _ = syn.write(os.path.join(str(tmp_path), "p"))
    bams = syn.write_sample_bams(os.path.join(str(tmp_path), "p"))
    syn.close()
    d = MultisampleVariantsDetector()
    d.setGenome(fa)
    d.setOutFilename(os.path.join(str(tmp_path), "whole.vcf"))
    d.run(bams).close()
    merged = call_population_sharded(fa, bams, os.path.join(str(tmp_path), "sharded.vcf"))
    assert merged == open(d.outFilename).read()
    assert sum(1 for l in merged.splitlines() if not l.startswith("#")) > 20


@pytest.mark.gpu
def test_gpu_sharded_known_variants_equal_whole_file(tmp_path):
    """-knownVariants through the sharded drivers (every rank genotypes its sequences' input variants): the
    merged single-sample and population VCFs equal the whole-file runs."""
    from test_gpu_known import _known_vcf
    from ngsepcore_amd import GpuPileupSession, MultisampleVariantsDetector
    from ngsepcore_amd.sharding import call_bam_sharded, call_population_sharded
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=12, seed=12)
    base = os.path.join(str(tmp_path), "d")
    fa, sam, bam = syn.write(base)
    known = os.path.join(str(tmp_path), "known.vcf")
    _known_vcf(known, syn, base + "_truth.vcf", 12, n_random=600)
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.set_known_variants(known)
        s.processFile(bam, full)
    merged = call_bam_sharded(fa, bam, os.path.join(str(tmp_path), "m.vcf"), known_vcf=known)
    assert merged == open(full).read()
    pop = pysynth.Synth(genome=pysynth.YEAST, n_contigs=2, depth=8, seed=13, n_samples=6)
    pfa, psam, _ = pop.write(os.path.join(str(tmp_path), "p"))
    bams = pop.write_sample_bams(os.path.join(str(tmp_path), "pop"))
    pknown = os.path.join(str(tmp_path), "pknown.vcf")
    _known_vcf(pknown, pop, os.path.join(str(tmp_path), "p_truth.vcf"), 13, n_random=300)
    pop.close()
    d = MultisampleVariantsDetector()
    d.setGenome(pfa)
    d.setKnownVariantsFile(pknown)
    d.setOutFilename(os.path.join(str(tmp_path), "pfull.vcf"))
    d.run(bams).close()
    pmerged = call_population_sharded(pfa, bams, os.path.join(str(tmp_path), "pm.vcf"), known_vcf=pknown)
    assert pmerged == open(d.outFilename).read()


def test_two_rank_sharded_indel_vcf_identical(tmp_path):
    """The sharded driver on data with indels (gloo, world size 2): every rank's per-sequence VCF carries its
    indel / STR records (the realigner runs inside each sequence), the merge == the whole-file VCF."""
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=10, seed=37, indel_rate=3e-4)
    contigs = [(n, len(s)) for n, s in syn.contigs()]
    fa, sam, _ = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    ngsep_oracle.run_ssvd(fa, sam, full)
    assert "TYPE=INDEL" in open(full).read()
    mp.spawn(_worker, args=(2, _free_port(), fa, sam, contigs, str(tmp_path)), nprocs=2, join=True)
    merged = open(os.path.join(str(tmp_path), "merged.vcf")).read()
    assert merged == open(full).read()


@pytest.mark.gpu
def test_gpu_contig_caller_indels_merge_identical(tmp_path):
    """The production per-sequence caller on data with indels: the merged VCF == the whole-file GPU VCF ==
    the oracle's (indel / STR records included; nothing is handed back as a carved region)."""
    from ngsepcore_amd import GpuPileupSession
    from ngsepcore_amd.sharding import gpu_contig_caller
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=15, seed=38, indel_rate=3e-4)
    contigs = [(n, len(s)) for n, s in syn.contigs()]
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        s.processFile(bam, full)
        assert s.carved_regions() == []
    o = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, o)
    assert open(full).read().split("#CHROM")[1] == open(o).read().split("#CHROM")[1]
    merged = call_sharded(contigs, gpu_contig_caller(fa, bam), os.path.join(str(tmp_path), "m.vcf"))
    assert merged == open(full).read()
    assert "TYPE=INDEL" in merged


def _carved_worker(rank, world, port, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from ngsepcore_amd.sharding import gather_carved
        local = [[("chrII", 500, 900), ("chrI", 10, 20)], [("chrIII", 5, 7), ("chrI", 1, 4)]][rank]
        got = gather_carved(local, ["chrI", "chrII", "chrIII"], dist)
        if rank == 0:
            with open(os.path.join(out_dir, "carved.txt"), "w") as f:
                f.write(repr(got))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_two_rank_carved_regions_gathered(tmp_path):
    """Pass-through mode: each rank's carved regions (ngsep_fetch_carved_regions) reach rank 0 in the BAM header's
    sequence order, then by position (sharding.gather_carved)."""
    mp.spawn(_carved_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    got = eval(open(os.path.join(str(tmp_path), "carved.txt")).read())
    assert got == [("chrI", 1, 4), ("chrI", 10, 20), ("chrII", 500, 900), ("chrIII", 5, 7)]


@pytest.mark.gpu
def test_gpu_sharded_passthrough_carved_bed(tmp_path):
    """call_bam_sharded in pass-through mode (indel_passthrough = 1): the merged VCF equals the whole-file run and
    <out>.carved.bed lists the same regions as the whole-file session (SingleSampleVariantsDetector.java:919-925 is
    the reference behaviour those regions stand in for)."""
    from ngsepcore_amd import GpuPileupSession
    from ngsepcore_amd.sharding import call_bam_sharded
    from helpers import gpu_params
    syn = pysynth.Synth(genome=pysynth.YEAST, n_contigs=3, depth=15, seed=39, indel_rate=3e-4)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    with GpuPileupSession(gpu_params(indel_passthrough=1)) as s:
        s.load_fasta(fa)
        s.processFile(bam, full)
        want = s.carved_regions()
    assert len(want) > 3
    out = os.path.join(str(tmp_path), "m.vcf")
    # (20 kb windows: pass-through mode must not cut a sequence -- its carve-out uses the run's longest span -- so the
    # driver falls back to whole sequences and neither the VCF nor the BED depends on the window size)
    for window in (4 << 20, 20000):
        merged = call_bam_sharded(fa, bam, out, params=gpu_params(indel_passthrough=1), window=window)
        assert merged == open(full).read()
        bed = [l.split("\t") for l in open(out + ".carved.bed").read().splitlines()]
        assert [(n, int(a) + 1, int(b)) for n, a, b in bed] == want


def _window_worker(rank, world, port, fa, sam, bam, contigs, out_dir, window, multi):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from ngsepcore_amd import GpuPileupSession
        from ngsepcore_amd.sharding import call_windows, clean_cut
        s = GpuPileupSession()                     # (the reference for ngsep_clean_cut: no device needed)
        s.load_fasta(fa)
        calls = []

        def region(name, first, last):
            out = os.path.join(out_dir, f"r{rank}_{name}_{first}.vcf")
            calls.append((name, first, last))
            if multi:
                ngsep_oracle.run_mvd(fa, sam, out, 0.0, query_seq=name, query_first=first, query_last=last)
            else:
                ngsep_oracle.run_ssvd(fa, sam, out, query_seq=name, query_first=first, query_last=last)
            return open(out).read()

        call_windows(contigs, region, lambda n, p: clean_cut(s, [bam], n, p), os.path.join(out_dir, "merged.vcf"), window, dist)
        with open(os.path.join(out_dir, f"calls{rank}.txt"), "w") as f:
            f.write(repr(calls))
        s.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("multi", [False, True])
def test_two_rank_window_sharding_one_contig(tmp_path, multi):
    """ONE contig split into exact windows (ngsep_clean_cut) taken by two gloo ranks from the shared queue, each window
    run as a region from its cut minus the lead (the oracle stands in for each rank's GPU caller): the merged VCF ==
    the whole-file VCF, on data with indels (the realigner's events decide where a cut may fall) -- for
    SingleSampleVariantsDetector and MultisampleVariantsDetector."""
    kw = dict(genome=pysynth.CUSTOM, custom_len=160000, seed=71, snv_rate=2e-3, indel_rate=5e-4)
    kw.update(dict(n_samples=6, depth=6) if multi else dict(depth=20))
    syn = pysynth.Synth(**kw)
    contigs = [(n, len(s)) for n, s in syn.contigs()]
    assert len(contigs) == 1
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "d"))
    syn.close()
    full = os.path.join(str(tmp_path), "full.vcf")
    if multi:
        ngsep_oracle.run_mvd(fa, sam, full, 0.0)
    else:
        ngsep_oracle.run_ssvd(fa, sam, full)
    text = open(full).read()
    assert sum(1 for l in text.splitlines() if "TYPE=INDEL" in l or "TYPE=STR" in l) > 5
    mp.spawn(_window_worker, args=(2, _free_port(), fa, sam, bam, contigs, str(tmp_path), 20000, multi), nprocs=2, join=True)
    merged = open(os.path.join(str(tmp_path), "merged.vcf")).read()
    assert merged == text
    import ast
    c0 = ast.literal_eval(open(os.path.join(str(tmp_path), "calls0.txt")).read())
    c1 = ast.literal_eval(open(os.path.join(str(tmp_path), "calls1.txt")).read())
    assert len(c0) >= 2 and len(c1) >= 2                 # both ranks took windows of the one contig


def test_clean_cut_properties(tmp_path):
    """ngsep_clean_cut: deterministic, never before pos, the sequence end + 1 past it, and no cut inside the reach of
    an alignment with an indel."""
    from ngsepcore_amd import GpuPileupSession
    from ngsepcore_amd.sharding import clean_cut
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=80000, seed=72, depth=15, indel_rate=2e-3)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "c"))
    name, seq = syn.contigs()[0]
    syn.close()
    ev = []
    for l in open(sam):
        if l.startswith("@"):
            continue
        f = l.split("\t")
        import re
        ops = re.findall(r"(\d+)([MIDNSHP=X])", f[5])
        span = sum(int(n) for n, o in ops if o in "MDN=X")
        ind = sum(int(n) for n, o in ops if o in "ID")
        if ind:
            ev.append((int(f[3]), int(f[3]) + span - 1 + ind))
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        prev = 0
        for pos in range(1, len(seq) + 2000, 7000):
            c, lead = clean_cut(s, [bam], name, pos)
            assert (c, lead) == clean_cut(s, [bam], name, pos)
            assert c >= pos and c <= len(seq) + 1 and lead > 0
            assert c >= prev or pos > prev
            if c <= len(seq):
                assert all(not (a - 150 <= c <= b + 150) for a, b in ev)
            prev = c


@pytest.mark.gpu
@pytest.mark.parametrize("multi", [False, True])
def test_gpu_window_caller_merge_identical(tmp_path, multi):
    """The production window path on the GPU (ngsep_clean_cut + ngsep_call_region_bam / ngsep_call_population_region_bams
    per window from its lead-in, the records inside the window kept), single process: the merged VCF == the whole-file
    GPU VCF on indel-bearing data with 25 kb windows."""
    from ngsepcore_amd import GpuPileupSession, MultisampleVariantsDetector
    from ngsepcore_amd.sharding import call_bam_sharded, call_population_sharded
    kw = dict(genome=pysynth.CUSTOM, custom_len=150000, seed=73, snv_rate=2e-3, indel_rate=5e-4)
    kw.update(dict(n_samples=6, depth=6) if multi else dict(depth=20))
    syn = pysynth.Synth(**kw)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "w"))
    full = os.path.join(str(tmp_path), "full.vcf")
    if multi:
        bams = syn.write_sample_bams(os.path.join(str(tmp_path), "pop"))
        d = MultisampleVariantsDetector()
        d.setGenome(fa)
        d.setOutFilename(full)
        d.run(bams).close()
        merged = call_population_sharded(fa, bams, os.path.join(str(tmp_path), "m.vcf"), window=25000)
    else:
        with GpuPileupSession() as s:
            s.load_fasta(fa)
            s.processFile(bam, full)
        merged = call_bam_sharded(fa, bam, os.path.join(str(tmp_path), "m.vcf"), window=25000)
    syn.close()
    text = open(full).read()
    assert sum(1 for l in text.splitlines() if "TYPE=INDEL" in l or "TYPE=STR" in l) > 5
    assert merged == text


def test_plan_windows_matches_python_plan(tmp_path):
    """ngsep_plan_windows (the windows ngsep_call_bam_multi's threads take from their in-process queue): every header
    sequence covered once, in order, contiguous, cut where ngsep_clean_cut cuts -- the same windows sharding.py's
    window_units(compute_cuts(...)) gives the multi-process driver; whole sequences at window 0 and in pass-through
    mode."""
    from ngsepcore_amd import GpuPileupSession
    from ngsepcore_amd.sharding import bam_header_sequences, clean_cut, compute_cuts, plan_windows, window_units
    from helpers import gpu_params
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=150000, seed=74, depth=12, indel_rate=5e-4)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "p"))
    syn.close()
    contigs = bam_header_sequences(bam)
    with GpuPileupSession() as s:
        s.load_fasta(fa)
        for window in (20000, 55555, 1 << 30):
            got = plan_windows(s, [bam], window)
            want = window_units(contigs, compute_cuts(contigs, window, lambda n, p: clean_cut(s, [bam], n, p)))
            assert got == [(n, a, b, lead) for n, _, a, b, lead in want]
            for (n, a, b, _), nxt in zip(got, got[1:] + [None]):
                if nxt is not None and nxt[0] == n:
                    assert nxt[1] == b + 1
            assert got[0][1] == 1 and got[-1][2] == contigs[-1][1]
        assert len(plan_windows(s, [bam], 20000)) >= 5
        assert plan_windows(s, [bam], 0) == [(n, 1, l, 0) for n, l in contigs]
    with GpuPileupSession(gpu_params(indel_passthrough=1)) as s:
        s.load_fasta(fa)
        assert plan_windows(s, [bam], 20000) == [(n, 1, l, 0) for n, l in contigs]


def test_multi_driver_fails_loudly_without_device(tmp_path):
    """ngsep_call_bam_multi on contexts without a HIP device: an error, no output and no CPU fallback."""
    import ctypes
    if __import__("torch").cuda.is_available():
        pytest.skip("a GPU is present")
    from ngsepcore_amd import GpuPileupSession, NgsepError
    from ngsepcore_amd.sharding import call_bam_multi
    syn = pysynth.Synth(genome=pysynth.CUSTOM, custom_len=20000, seed=75, depth=5)
    fa, sam, bam = syn.write(os.path.join(str(tmp_path), "n"))
    syn.close()
    out = os.path.join(str(tmp_path), "m.vcf")
    with pytest.raises(NgsepError):
        call_bam_multi(fa, bam, out, [0, 0], window=5000)
    with GpuPileupSession() as s:              # the same context twice is refused before any device work
        ctxs = (ctypes.c_void_p * 2)(s._ctx.value, s._ctx.value)
        assert s._lib.ngsep_call_bam_multi(ctxs, 2, bam.encode(), out.encode(), 5000) == -1
