"""Contig and window sharding across the GPUs of one node: one process per GPU, no collective on
the hot path.

Sequences are independent units of SingleSampleVariantsDetector: the reference writes each sequence's
calls sorted on onSequenceEnd (SingleSampleVariantsDetector.java:933-968, 1026-1032), so the VCF of a
whole run is the header followed by the per-sequence record blocks in reference order.  Each rank calls
the sequences assigned to it (largest first onto the least-loaded rank), the record blocks are gathered
to rank 0 once at the end (a host-side object gather over torch.distributed: nccl/RCCL on the GPU
node, gloo in the CPU tests) and rank 0 writes header + blocks in reference order -- byte-identical to
the single-process output.

Window granularity (window > 0): every sequence is cut into windows of about `window` bp at boundaries the library
proves exact (ngsep_clean_cut: a position no indel-realigner event can reach, so the realigner and the listeners'
state there do not depend on what came before); the ranks take windows from a shared queue (a counter in the
process group's store), each window is called as a region (querySeq, AlignmentsPileupGenerator.java:242-254,310-322)
from its boundary minus the lead the cut reports, and only the records inside the window are kept.  The blocks of
(sequence, window) are merged on rank 0 in order: a single-contig BAM uses every GPU.
"""
from __future__ import annotations

import gzip
import os
import struct
import tempfile
import zlib
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


def window_starts(length: int, window: int) -> List[int]:
    """Nominal first positions of a sequence's windows (1, 1 + window, ...)."""
    return list(range(1, max(1, int(length)) + 1, max(1, int(window))))


def window_units(contigs: Sequence[Tuple[str, int]], cuts: Dict[Tuple[str, int], Tuple[int, int]]) -> List[Tuple[str, int, int, int, int]]:
    """(sequence, window index, first, last, lead) of every non-empty window: [first, last] between consecutive
    cuts (made monotone: a cut never moves before an earlier one), lead = the cut's lead-in."""
    out = []
    for name, length in contigs:
        ks = sorted(k for (n, k) in cuts if n == name)
        b = [1]
        leads = [0]
        for k in ks:
            if k == 0:
                continue
            c, lead = cuts[(name, k)]
            b.append(max(b[-1], min(int(c), int(length) + 1)))
            leads.append(int(lead))
        b.append(int(length) + 1)
        for i in range(len(b) - 1):
            if b[i] < b[i + 1]:
                out.append((name, i, b[i], b[i + 1] - 1, leads[i]))
    return out


def compute_cuts(contigs: Sequence[Tuple[str, int]], window: int, cut_fn: Callable[[str, int], Tuple[int, int]],
                 dist=None) -> Dict[Tuple[str, int], Tuple[int, int]]:
    """Every window boundary's (cut, lead) through cut_fn(sequence, nominal position) -- the boundaries split over
    the ranks and all-gathered, so every rank holds the same table."""
    todo = [(name, k, p) for name, length in contigs for k, p in enumerate(window_starts(length, window))]
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    mine = {}
    for i, (name, k, p) in enumerate(todo):
        if i % world != rank:
            continue
        mine[(name, k)] = (1, 0) if k == 0 else tuple(cut_fn(name, p))
    if world == 1:
        return mine
    parts = [None] * world
    dist.all_gather_object(parts, mine)
    out = {}
    for part in parts:
        out.update(part)
    return out


_queue_uses = [0]


def shared_queue(n: int, dist=None, tag: str = ""):
    """Unit indexes 0 .. n - 1 handed out to the ranks as they ask (a counter in the process group's store); with
    no store, rank r takes r, r + world, ...  The store key is the call's ordinal on this rank plus `tag` (the unit
    list's digest): ranks that disagree on either use different counters, so every unit is then called on several
    ranks and the merge refuses the duplicate windows, never mixing two queues."""
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    store = None
    if world > 1:
        try:
            store = dist.distributed_c10d._get_default_store()
        except Exception:
            store = None
    if store is None:
        yield from range(rank, n, world)
        return
    _queue_uses[0] += 1
    key = f"ngsep_queue_{_queue_uses[0]}_{tag}"
    while True:
        i = int(store.add(key, 1)) - 1
        if i >= n:
            return
        yield i


def keep_window(text: str, first: int, last: int) -> Tuple[str, str]:
    """(header, the records of text with first <= POS <= last)."""
    header, recs = [], []
    for line in text.splitlines(keepends=True):
        if line.startswith("#"):
            header.append(line)
            continue
        pos = int(line.split("\t", 2)[1])
        if first <= pos <= last:
            recs.append(line)
    return "".join(header), "".join(recs)


def call_windows(contigs: Sequence[Tuple[str, int]], call_region: Callable[[str, int, int], str],
                 cut_fn: Callable[[str, int], Tuple[int, int]], out_vcf: str, window: int, dist=None) -> Optional[str]:
    """Window-granular sharding: call_region(sequence, first, last) -> VCF text of that region run; the merged VCF
    on rank 0 (its text returned there, None elsewhere)."""
    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1
    rank = dist.get_rank() if dist is not None and dist.is_initialized() else 0
    units = window_units(contigs, compute_cuts(contigs, window, cut_fn, dist))
    header = ""
    local: Dict[Tuple[str, int], str] = {}
    tag = "%08x" % zlib.crc32(repr(units).encode())
    for i in shared_queue(len(units), dist, tag):
        name, k, first, last, lead = units[i]
        h, recs = keep_window(call_region(name, max(1, first - lead), last), first, last)
        header = header or h
        local[(name, k)] = recs
    if world > 1:
        hs = [None] * world if rank == 0 else None
        dist.gather_object(header, hs, dst=0)
        if rank == 0:
            header = next((x for x in hs if x), "")
        got = [None] * world if rank == 0 else None
        dist.gather_object(local, got, dst=0)
        if rank != 0:
            return None
        merged: Dict[Tuple[str, int], str] = {}
        for part in got:
            for key, rec in part.items():
                if key in merged:
                    raise ValueError(f"window {key} called on two ranks")
                merged[key] = rec
    else:
        merged = local
    if not header:                                    # (no window anywhere: the header of a one-position region run)
        header, _ = keep_window(call_region(contigs[0][0], 1, 1) if contigs else "", 1, 0)
    text = header + "".join(merged.get((u[0], u[1]), "") for u in units)
    with open(out_vcf, "w") as f:
        f.write(text)
    return text


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
        # the indel realigner's regions this rank handed back (pass-through mode)
        return state["s"].carved_regions() if "s" in state else []

    def region(name: str, first: int, last: int) -> str:
        session()
        s = state["s"]
        with tempfile.TemporaryDirectory() as d:
            out = os.path.join(d, "c.vcf")
            s._check(s._lib.ngsep_call_region_bam(s._ctx, bam.encode(), name.encode(), first, last, out.encode()))
            state["windows"] = state.get("windows", 0) + 1
            state["positions"] = state.get("positions", 0) + int(s.stats().positions_genotyped)
            return open(out).read()

    def cut(name: str, pos: int):
        session()
        return clean_cut(state["s"], [bam], name, pos)

    def session():
        if "s" not in state:
            state["s"] = GpuPileupSession(params, device)
            state["s"].load_fasta(fasta)
            if known_vcf:
                state["s"].set_known_variants(known_vcf)
    call.close = close
    call.carved = carved
    call.region = region
    call.cut = cut
    call.state = state
    return call


def clean_cut(session, bams: Sequence[str], name: str, pos: int) -> Tuple[int, int]:
    """ngsep_clean_cut through a session (its reference, and its input variants when set): (cut, lead)."""
    import ctypes
    arr = (ctypes.c_char_p * len(bams))(*[b.encode() for b in bams])
    cut, lead = ctypes.c_int64(0), ctypes.c_int64(0)
    session._check(session._lib.ngsep_clean_cut(session._ctx, arr, len(bams), name.encode(), int(pos), ctypes.byref(cut),
                                                ctypes.byref(lead)))
    return int(cut.value), int(lead.value)


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
                     known_vcf: Optional[str] = None, window: int = 4 << 20, work: Optional[dict] = None) -> Optional[str]:
    """SingleSampleVariantsDetector over the GPUs of one node (device = local rank by default): with window > 0
    (default 4 Mb) the sequences' exact windows from a shared queue (call_windows), else the BAM header's sequences
    split over the ranks (assign_contigs); each region called through the index on the rank's GPU, the blocks merged
    on rank 0 in header order."""
    contigs = bam_header_sequences(bam)
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    caller = gpu_contig_caller(fasta, bam, params, device, known_vcf)
    if params is not None and getattr(params, "indel_passthrough", 0):
        # pass-through mode carves [first - R, last + R] around every indel read with R from the run's own longest
        # span: a window's run would see a local R and re-carve its lead-in, so the carve-out (and the positions it
        # leaves uncalled) would depend on the cuts -- whole sequences only
        window = 0
    try:
        if window > 0:
            text = call_windows(contigs, caller.region, caller.cut, out_vcf, window, dist)
        else:
            text = call_sharded(contigs, caller, out_vcf, dist)
        # the regions left to the caller's own indel path (ngsep_fetch_carved_regions), merged like the records and
        # written beside the VCF as the CLI does (<out>.carved.bed, 0-based half-open)
        if work is not None:                       # (this rank's share: region runs and their genotyped positions)
            work["windows"] = caller.state.get("windows", 0)
            work["positions"] = caller.state.get("positions", 0)
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

    def region(name: str, first: int, last: int) -> str:
        session()
        s = state["s"]
        with tempfile.TemporaryDirectory() as t:
            out = os.path.join(t, "p.vcf")
            s._check(s._lib.ngsep_call_population_region_bams(s._ctx, arr, len(bams), name.encode(), first, last, out.encode()))
            return open(out).read()

    def cut(name: str, pos: int):
        session()
        return clean_cut(state["s"], bams, name, pos)

    def session():
        if "s" not in state:
            p = default_params()
            if params is not None:
                ctypes.pointer(p)[0] = params
            p.multisample = 1
            state["s"] = GpuPileupSession(p, device)
            state["s"].load_fasta(fasta)
            if known_vcf:
                state["s"].set_known_variants(known_vcf)
    call.close = close
    call.region = region
    call.cut = cut
    return call


def call_population_sharded(fasta: str, bams: Sequence[str], out_vcf: str, params=None, dist=None,
                            device: Optional[int] = None, known_vcf: Optional[str] = None, window: int = 4 << 20) -> Optional[str]:
    """MultisampleVariantsDetector over the GPUs of one node (configs[4]): exact windows from a shared queue
    (window > 0, default 4 Mb; call_windows) or whole sequences split over the ranks, the population VCF blocks
    merged on rank 0 in the first BAM's header order (the multi-file merge meets the sequences in that order,
    AlignmentsPileupGenerator.java:268-289)."""
    contigs = bam_header_sequences(bams[0])
    if device is None:
        device = int(os.environ.get("LOCAL_RANK", "0"))
    caller = gpu_population_caller(fasta, bams, params, device, known_vcf)
    try:
        if window > 0:
            return call_windows(contigs, caller.region, caller.cut, out_vcf, window, dist)
        return call_sharded(contigs, caller, out_vcf, dist)
    finally:
        caller.close()


# ------------------------------------------------------------------------------------------------------------------
# several devices from ONE process through the C ABI (ngsep_call_bam_multi / ngsep_call_population_bams_multi, ABI 11):
# one context per device, one host thread each, windows from an in-process queue -- what a Java/JNI caller gets
# ------------------------------------------------------------------------------------------------------------------
def plan_windows(session, bams: Sequence[str], window: int) -> List[Tuple[str, int, int, int]]:
    """ngsep_plan_windows: the (sequence, first, last, lead) windows the multi-device drivers run (host only)."""
    import ctypes
    arr = (ctypes.c_char_p * len(bams))(*[b.encode() for b in bams])
    n = ctypes.c_int64(0)
    session._check(session._lib.ngsep_plan_windows(session._ctx, arr, len(bams), int(window), None, None, None, None, 0,
                                                    ctypes.byref(n)))
    k = n.value
    sid = (ctypes.c_int32 * max(1, k))()
    first, last, lead = ((ctypes.c_int64 * max(1, k))() for _ in range(3))
    session._check(session._lib.ngsep_plan_windows(session._ctx, arr, len(bams), int(window), sid, first, last, lead, k,
                                                    ctypes.byref(n)))
    names = session.sequence_names()
    return [(names[sid[i]], int(first[i]), int(last[i]), int(lead[i])) for i in range(k)]


def _multi_sessions(fasta, devices, params, known_vcf, known_strs, multisample):
    import ctypes
    from .discovery import GpuPileupSession, default_params
    p = default_params()
    if params is not None:
        ctypes.pointer(p)[0] = params
    if multisample:
        p.multisample = 1
    sessions = [GpuPileupSession(p, int(d)) for d in devices]
    sessions[0].load_fasta(fasta)                     # (the other contexts take the first one's reference)
    if known_vcf:
        sessions[0].set_known_variants(known_vcf)
    if known_strs:
        sessions[0].set_known_strs(known_strs)
    return sessions


def call_bam_multi(fasta: str, bam: str, out_vcf: str, devices: Sequence[int], params=None, window: int = 4 << 20,
                   known_vcf: Optional[str] = None, known_strs: Optional[str] = None, sessions_out=None) -> str:
    """SingleSampleVariantsDetector over several devices of this process (ngsep_call_bam_multi): the VCF text."""
    import ctypes
    sessions = _multi_sessions(fasta, devices, params, known_vcf, known_strs, False)
    try:
        ctxs = (ctypes.c_void_p * len(sessions))(*[s._ctx.value for s in sessions])
        sessions[0]._check(sessions[0]._lib.ngsep_call_bam_multi(ctxs, len(sessions), bam.encode(), out_vcf.encode(), int(window)))
        if sessions_out is not None:
            sessions_out.append([s.stats() for s in sessions])
            sessions_out.append(sessions[0].carved_regions())
        return open(out_vcf).read()
    finally:
        for s in sessions:
            s.close()


def call_population_multi(fasta: str, bams: Sequence[str], out_vcf: str, devices: Sequence[int], params=None,
                          window: int = 4 << 20, known_vcf: Optional[str] = None, known_strs: Optional[str] = None) -> str:
    """MultisampleVariantsDetector over several devices of this process (ngsep_call_population_bams_multi)."""
    import ctypes
    sessions = _multi_sessions(fasta, devices, params, known_vcf, known_strs, True)
    try:
        ctxs = (ctypes.c_void_p * len(sessions))(*[s._ctx.value for s in sessions])
        arr = (ctypes.c_char_p * len(bams))(*[b.encode() for b in bams])
        sessions[0]._check(sessions[0]._lib.ngsep_call_population_bams_multi(ctxs, len(sessions), arr, len(bams),
                                                                           out_vcf.encode(), int(window)))
        return open(out_vcf).read()
    finally:
        for s in sessions:
            s.close()
