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
