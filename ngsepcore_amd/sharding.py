"""Contig sharding across the GPUs of one node: one process per GPU, no collective on
the hot path.

Sequences are independent units of SingleSampleVariantsDetector: the reference writes each sequence's
calls sorted on onSequenceEnd (SingleSampleVariantsDetector.java:933-968, 1026-1032), so the VCF of a
whole run is the header followed by the per-sequence record blocks in reference order.  Each rank calls
the sequences assigned to it (largest first onto the least-loaded rank), the record blocks are gathered
to rank 0 once at the end (a host-side object gather over torch.distributed: nccl/RCCL on the GPU
node, gloo in the CPU tests) and rank 0 writes header + blocks in reference order -- byte-identical to
the single-process output.
"""
from __future__ import annotations

import gzip
import os
import struct
import tempfile
from typing import Callable, Dict, List, Optional, Sequence, Tuple


def bam_header_sequences(bam: str) -> List[Tuple[str, int]]:
    """(name, length) of every @SQ reference of a BAM header, in header order -- the order in which a
    single-process SingleSampleVariantsDetector run meets (and writes) the sequences of a sorted BAM."""
    with gzip.open(bam, "rb") as f:
        if f.read(4) != b"BAM\1":
            raise ValueError(f"{bam}: not a BAM file")
        (l_text,) = struct.unpack("<i", f.read(4))
        f.read(l_text)
        (n_ref,) = struct.unpack("<i", f.read(4))
        out = []
        for _ in range(n_ref):
            (l_name,) = struct.unpack("<i", f.read(4))
            name = f.read(l_name)[:-1].decode()
            (l_ref,) = struct.unpack("<i", f.read(4))
            out.append((name, l_ref))
        return out


def assign_contigs(contigs: Sequence[Tuple[str, int]], world: int) -> List[List[str]]:
    """Longest-processing-time assignment of (name, length) sequences to `world` ranks; ties go to the
    lowest rank, so every rank computes the same assignment."""
    if world < 1:
        raise ValueError("world size must be >= 1")
    load = [0] * world
    out: List[List[str]] = [[] for _ in range(world)]
    order = sorted(range(len(contigs)), key=lambda i: (-int(contigs[i][1]), i))
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(contigs[i][0])
        load[r] += int(contigs[i][1])
    return out


def split_vcf(text: str) -> Tuple[str, Dict[str, str]]:
    """VCF text -> (header, {sequence: its record lines})."""
    header, blocks = [], {}
    for line in text.splitlines(keepends=True):
        if line.startswith("#"):
            header.append(line)
        else:
            seq = line.split("\t", 1)[0]
            blocks[seq] = blocks.get(seq, "") + line
    return "".join(header), blocks


def merge_vcf(header: str, blocks: Dict[str, str], order: Sequence[str]) -> str:
    """Header + record blocks in reference order (sequences without calls contribute nothing)."""
    extra = set(blocks) - set(order)
    if extra:
        raise ValueError(f"records on sequences outside the reference: {sorted(extra)}")
    return header + "".join(blocks.get(s, "") for s in order)


def gather_blocks(local: Dict[str, str], dist=None) -> Optional[Dict[str, str]]:
    """Rank 0 receives every rank's {sequence: records}; other ranks get None.  Without a process group
    (single process) the local blocks are returned."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return dict(local)
    rank = dist.get_rank()
    got = [None] * dist.get_world_size() if rank == 0 else None
    dist.gather_object(local, got, dst=0)
    if rank != 0:
        return None
    merged: Dict[str, str] = {}
    for part in got:
        for seq, rec in part.items():
            if seq in merged:
                raise ValueError(f"sequence {seq} called on two ranks")
            merged[seq] = rec
    return merged


def call_sharded(contigs: Sequence[Tuple[str, int]], call_contig: Callable[[str], str], out_vcf: str,
                 dist=None) -> Optional[str]:
    """Runs `call_contig(name) -> VCF text of that sequence` for this rank's sequences and writes the
    merged VCF on rank 0 (returns its text there, None elsewhere).  `contigs` must be the alignment file's
    sequences in its header order (bam_header_sequences): records on any other sequence are an error."""
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    mine = assign_contigs(contigs, world)[rank]
    header = ""
    local: Dict[str, str] = {}
    for name in mine:
        h, blocks = split_vcf(call_contig(name))
        header = header or h
        local.update(blocks)
    # every rank may hold no calls; the header is the same on all ranks (options + reference)
    if world > 1:
        hs = [None] * world if rank == 0 else None
        dist.gather_object(header, hs, dst=0)
        if rank == 0:
            header = next((x for x in hs if x), "")
    merged = gather_blocks(local, dist)
    if merged is None:
        return None
    text = merge_vcf(header, merged, [c[0] for c in contigs])
    with open(out_vcf, "w") as f:
        f.write(text)
    return text


def gpu_contig_caller(fasta: str, bam: str, params=None, device: int = 0,
                      known_vcf: Optional[str] = None) -> Callable[[str], str]:
    """The production per-sequence caller: SingleSampleVariantsDetector.findSNVS restricted to one
    sequence on this rank's GPU through the BAI index (ngsep_call_region_bam: only that sequence's BGZF
    blocks are read; without an index the file is streamed up to the sequence).  One device context per
    rank, the reference loaded once."""
    from .discovery import GpuPileupSession

    lengths = dict(bam_header_sequences(bam))
    state = {}

    def call(name: str) -> str:
        if "s" not in state:
            state["s"] = GpuPileupSession(params, device)
            state["s"].load_fasta(fasta)
            if known_vcf:                          # -knownVariants: each rank genotypes its sequences' inputs
                state["s"].set_known_variants(known_vcf)
        s = state["s"]
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "c.vcf")
            s._check(s._lib.ngsep_call_region_bam(s._ctx, bam.encode(), name.encode(), 1, lengths[name], out.encode()))
            return open(out).read()

    def close():
        if "s" in state:
            state.pop("s").close()

    def carved():
        # the indel realigner's regions this rank handed back (pass-through mode, -knownVariants with indel reads)
        return state["s"].carved_regions() if "s" in state else []
    call.close = close
    call.carved = carved
    return call


def gather_carved(local: List[Tuple[str, int, int]], order: Sequence[str], dist=None) -> Optional[List[Tuple[str, int, int]]]:
    """Every rank's carved regions on rank 0 (None elsewhere), in the BAM header's sequence order."""
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        got = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
        dist.gather_object(local, got, dst=0)
        if dist.get_rank() != 0:
            return None
        allr = [r for part in got for r in part]
    else:
        allr = list(local)
    rank_of = {n: k for k, n in enumerate(order)}
    return sorted(allr, key=lambda r: (rank_of.get(r[0], len(order)), r[1], r[2]))


def call_bam_sharded(fasta: str, bam: str, out_vcf: str, params=None, dist=None, device: Optional[int] = None,
                     known_vcf: Optional[str] = None) -> Optional[str]:
    """SingleSampleVariantsDetector over the GPUs of one node: the BAM header's sequences split over the
    ranks (assign_contigs), each rank calling its own through the index on its GPU (device = local rank
    by default), the per-sequence blocks merged on rank 0 in header order."""
    contigs = bam_header_sequences(bam)
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    caller = gpu_contig_caller(fasta, bam, params, device, known_vcf)
    try:
        text = call_sharded(contigs, caller, out_vcf, dist)
        # the regions left to the caller's own indel path (ngsep_fetch_carved_regions), merged like the records and
        # written beside the VCF as the CLI does (<out>.carved.bed, 0-based half-open)
        regions = gather_carved(caller.carved(), [c[0] for c in contigs], dist)
        if regions:
            with open(out_vcf + ".carved.bed", "w") as f:
                for n, a, b in regions:
                    f.write(f"{n}\t{a - 1}\t{b}\n")
        return text
    finally:
        caller.close()


def gpu_population_caller(fasta: str, bams: Sequence[str], params=None, device: int = 0,
                          known_vcf: Optional[str] = None) -> Callable[[str], str]:
    """MultisampleVariantsDetector restricted to one sequence (-querySeq; every BAM read from that
    sequence's index chunks): the population VCF text of that sequence.  One device context per rank, the
    reference and the known variants loaded once (ngsep_call_population_region_bams reuses it)."""
    import ctypes
    from .discovery import GpuPileupSession, default_params

    lengths = dict(bam_header_sequences(bams[0]))
    arr = (ctypes.c_char_p * len(bams))(*[b.encode() for b in bams])
    state = {}

    def call(name: str) -> str:
        if "s" not in state:
            p = default_params()
            if params is not None:
                ctypes.pointer(p)[0] = params
            p.multisample = 1
            state["s"] = GpuPileupSession(p, device)
            state["s"].load_fasta(fasta)
            if known_vcf:                          # -knownVariants: each rank genotypes its sequences' inputs
                state["s"].set_known_variants(known_vcf)
        s = state["s"]
        with tempfile.TemporaryDirectory() as t:
            out = os.path.join(t, "p.vcf")
            s._check(s._lib.ngsep_call_population_region_bams(s._ctx, arr, len(bams), name.encode(), 1,
                                                                lengths.get(name, 1 << 31), out.encode()))
            return open(out).read()

    def close():
        if "s" in state:
            state.pop("s").close()
    call.close = close
    return call


def call_population_sharded(fasta: str, bams: Sequence[str], out_vcf: str, params=None, dist=None,
                            device: Optional[int] = None, known_vcf: Optional[str] = None) -> Optional[str]:
    """MultisampleVariantsDetector over the GPUs of one node (configs[4]): sequences split over the ranks,
    the population VCF blocks merged on rank 0 in the first BAM's header order (the multi-file merge meets
    the sequences in that order, AlignmentsPileupGenerator.java:268-289)."""
    contigs = bam_header_sequences(bams[0])
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    caller = gpu_population_caller(fasta, bams, params, device, known_vcf)
    try:
        return call_sharded(contigs, caller, out_vcf, dist)
    finally:
        caller.close()
