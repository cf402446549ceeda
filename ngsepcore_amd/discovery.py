"""Host-side mirror of NGSEP's SNV discovery interface, backed by libngsep_amd.so.

Names, option meanings and defaults follow the reference:
  * SingleSampleVariantsDetector  (src/ngsep/discovery/SingleSampleVariantsDetector.java:62-1082,
    options main/CommandsDescriptor.xml:565-703)
  * AlignmentsPileupGenerator.processAlignments / notifyEndOfAlignments
    (discovery/AlignmentsPileupGenerator.java:334-361,447-452) -> GpuPileupSession
  * SingleSampleVariantPileupListener.getCalledVariants (:139-141) -> GpuPileupSession.getCalledVariants
Errors surface as NgsepError (the reference throws IOException / IllegalArgumentException).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

from . import _lib
from ._lib import (NgsepError, NgsepParams, NgsepPopSiteOut, NgsepReadBatch, NgsepSampleCall, NgsepSiteOut,
                   NgsepStats)

BASES = "ACGT"


def default_params() -> NgsepParams:
    p = NgsepParams()
    _lib.load().ngsep_params_default(ctypes.byref(p))
    return p


@dataclass
class CalledSite:
    """One called variant (CalledSNV, triallelic CalledGenomicVariantImpl, or -- ploidy >= 3 -- the
    CalledGenomicVariantImpl of genotypeVariantPool: `called` holds its called alleles' indexes)."""
    sequence: str
    pos: int
    ref: str
    alleles: List[str]
    genotype: int
    gq: int
    qual: int
    dp: int
    counts: List[int]
    strand_counts: List[List[int]]
    logc: List[float]
    strand_bias: int
    is_call: bool
    called: List[int] = None
    vcf_line: str = None        # indel / STR records (ABI 6): the record's VCF line; embedded SNVs: TYPE=EMBEDDED
    embedded: bool = False

    def log_conditional(self, i: int, j: int) -> float:
        """SNVQ records: i, j are DNA indexes; pool records: indexes into `alleles`."""
        if i > j:
            i, j = j, i
        n = len(self.alleles) if self.called is not None else 4
        base = i * n - i * (i - 1) // 2
        return self.logc[base + j - i]


def java_string_hash(s: str) -> int:
    h = 0
    for ch in s.encode("utf-16-be").decode("utf-16-be"):
        h = (31 * h + ord(ch)) & 0xFFFFFFFF
    return h


def java_hashset_order(ids: Sequence[str]) -> List[int]:
    """Iteration order of a java.util.HashSet<String> filled with ids in order (Sample.readGroups,
    variants/Sample.java:36): buckets of the final table (16, doubled past 0.75 load), insertion order
    inside a bucket.  Returns indexes into ids."""
    cap = 16
    while len(ids) > cap * 3 // 4:
        cap *= 2
    def bucket(i):
        h = java_string_hash(ids[i])
        return (h ^ (h >> 16)) & (cap - 1)
    return sorted(range(len(ids)), key=lambda i: (bucket(i), i))


@dataclass
class PopulationSite:
    """One MultisampleVariantsDetector VCF line: the variant and one call per sample."""
    sequence: str
    pos: int
    alleles: List[str]
    qual: int
    multisnv_type: bool
    calls: List[NgsepSampleCall]
    embedded: bool = False               # TYPE=EMBEDDED (an SNV inside an indel / STR, -embeddedSNVs)
    vcf_line: Optional[str] = None       # an indel / STR record: its whole VCF line


class GpuPileupSession:
    """One device context: reference + alignment stream -> called SNVs.

    Mirrors the listener chain IndelRealigner -> SingleSampleVariantPileupListener ->
    SingleSampleVariantsDetector for SNV-only alignments (SingleSampleVariantsDetector.java:919-925).
    """

    def __init__(self, params: Optional[NgsepParams] = None, device: int = 0):
        self._lib = _lib.load()
        self._ctx = ctypes.c_void_p()
        p = params if params is not None else default_params()
        rc = self._lib.ngsep_open(device, ctypes.byref(p), ctypes.byref(self._ctx))
        self._check(rc)
        self.params = p

    # -- plumbing
    def _check(self, rc: int):
        if rc != _lib.NGSEP_OK:
            msg = self._lib.ngsep_last_error(self._ctx).decode() if self._ctx else "open failed"
            raise NgsepError(rc, msg)

    def close(self):
        if self._ctx:
            self._lib.ngsep_close(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- reference (ReferenceGenome with lower case kept)
    def load_fasta(self, path: str):
        self._check(self._lib.ngsep_load_fasta(self._ctx, path.encode()))

    def set_known_variants(self, vcf_path: Optional[str]):
        """-knownVariants (SingleSampleVariantsDetector.findSNVS :896-906): genotype these biallelic SNVs."""
        self._check(self._lib.ngsep_set_known_variants(self._ctx, vcf_path.encode() if vcf_path else None))

    def set_known_strs(self, path: Optional[str]):
        """-knownSTRs (SingleSampleVariantsDetector.findSNVS :906-912): input STRs for the indel realigner."""
        self._check(self._lib.ngsep_set_known_strs(self._ctx, path.encode() if path else None))

    def set_reference(self, name: str, bases: bytes):
        self._check(self._lib.ngsep_set_reference(self._ctx, name.encode(), bases, len(bases)))

    def sequence_names(self) -> List[str]:
        n = self._lib.ngsep_n_sequences(self._ctx)
        return [self._lib.ngsep_sequence_name(self._ctx, i).decode() for i in range(n)]

    # -- alignments (AlignmentsPileupGenerator)
    def processAlignments(self, batch: NgsepReadBatch):
        self._check(self._lib.ngsep_process_alignments(self._ctx, ctypes.byref(batch)))

    def notifyEndOfAlignments(self):
        self._check(self._lib.ngsep_notify_end(self._ctx))

    def processFile(self, bam_path: str, out_vcf: str):
        """SingleSampleVariantsDetector.findSNVS on a BAM file, VCF written to out_vcf."""
        self._check(self._lib.ngsep_call_bam(self._ctx, bam_path.encode(), out_vcf.encode()))

    def processFileBatches(self, bam_path: str, batch_reads: int = 1 << 20):
        """Path A fed by the C++ reader: the BAM's reader-filtered alignments in batches through
        processAlignments, then notifyEndOfAlignments (what a JNI host with its own reader does)."""
        b = ctypes.c_void_p()
        self._check(self._lib.ngsep_bam_open(self._ctx, bam_path.encode(), ctypes.byref(b)))
        try:
            batch = NgsepReadBatch()
            while True:
                self._check(self._lib.ngsep_bam_next_batch(b, batch_reads, ctypes.byref(batch)))
                if batch.n_reads == 0:
                    break
                self.processAlignments(batch)
        finally:
            self._lib.ngsep_bam_close(b)
        self.notifyEndOfAlignments()

    # -- staged runs (measurement)
    def stage(self, batch: NgsepReadBatch):
        self._check(self._lib.ngsep_stage_alignments(self._ctx, ctypes.byref(batch)))

    def stage_finish(self):
        self._check(self._lib.ngsep_stage_finish(self._ctx))

    def run_staged(self) -> float:
        ms = ctypes.c_double()
        self._check(self._lib.ngsep_run_staged(self._ctx, ctypes.byref(ms)))
        return ms.value

    def submit_staged(self):
        self._check(self._lib.ngsep_submit_staged(self._ctx))

    def collect_staged(self) -> float:
        ms = ctypes.c_double()
        self._check(self._lib.ngsep_collect_staged(self._ctx, ctypes.byref(ms)))
        return ms.value

    def release_staged(self):
        self._check(self._lib.ngsep_release_staged(self._ctx))

    # -- results
    def raw_sites(self) -> Sequence[NgsepSiteOut]:
        n = ctypes.c_int64()
        self._check(self._lib.ngsep_fetch_sites(self._ctx, None, 0, ctypes.byref(n)))
        arr = (NgsepSiteOut * max(n.value, 1))()
        self._check(self._lib.ngsep_fetch_sites(self._ctx, arr, n.value, ctypes.byref(n)))
        return arr[: n.value]

    def getCalledVariants(self) -> List[CalledSite]:
        names = self.sequence_names()
        out = []
        for i, s in enumerate(self.raw_sites()):
            if s.is_call & 8:                    # an indel / STR call (IndelRealignerPileupListener + callIndel)
                # the record's length first (cap 0), then the whole line: a multi-allelic STR's PL list grows
                # with the square of its allele count
                need = self._lib.ngsep_site_vcf_line(self._ctx, i, None, 0)
                if need < 0:
                    raise NgsepError(int(need), self._lib.ngsep_last_error(self._ctx).decode())
                buf = ctypes.create_string_buffer(int(need) + 1)
                self._lib.ngsep_site_vcf_line(self._ctx, i, buf, int(need) + 1)
                f = buf.value.decode().rstrip("\n").split("\t")
                gt = f[9].split(":")[0]
                out.append(CalledSite(
                    sequence=f[0], pos=int(f[1]), ref=f[3], alleles=[f[3]] + f[4].split(","),
                    genotype=-1, gq=int(f[9].split(":")[2]), qual=int(f[5]), dp=int(f[9].split(":")[3]),
                    counts=[int(x) for x in f[9].split(":")[4].split(",")], strand_counts=[], logc=[],
                    strand_bias=-1, is_call=True, called=[int(x) for x in gt.replace("|", "/").split("/")],
                    vcf_line=buf.value.decode()))
                continue
            alleles = [chr(s.ref)]
            called = None
            if s.pool:
                alleles += [BASES[k] for k in range(4) if (s.pool >> k) & 1 and BASES[k] != chr(s.ref)]
                called = [alleles.index(BASES[x]) for x in (s.alt, s.third) if x >= 0]
            else:
                if s.n_alleles >= 2:
                    alleles.append(BASES[s.alt])
                if s.n_alleles == 3:
                    alleles.append(BASES[s.third])
            out.append(CalledSite(
                sequence=names[s.seq_id] if 0 <= s.seq_id < len(names) else "?", pos=s.pos, ref=chr(s.ref),
                alleles=alleles, genotype=s.genotype, gq=s.gq, qual=s.qual, dp=s.dp, counts=list(s.counts),
                strand_counts=[list(x) for x in s.strand_counts], logc=list(s.logc),
                strand_bias=s.strand_bias, is_call=bool(s.is_call & 1), called=called, embedded=bool(s.is_call & 4)))
        return out

    def clear(self):
        self._check(self._lib.ngsep_clear_sites(self._ctx))

    def carved_regions(self):
        """Regions around indel-bearing alignments the device path did not call (the indel realigner's
        reach, ngsep_fetch_carved_regions): [(sequence, first, last)], 1-based inclusive."""
        n = ctypes.c_int64()
        self._check(self._lib.ngsep_fetch_carved_regions(self._ctx, None, None, None, 0, ctypes.byref(n)))
        k = max(n.value, 1)
        sid, a, b = (ctypes.c_int32 * k)(), (ctypes.c_int64 * k)(), (ctypes.c_int64 * k)()
        self._check(self._lib.ngsep_fetch_carved_regions(self._ctx, sid, a, b, n.value, ctypes.byref(n)))
        names = self.sequence_names()
        return [(names[sid[i]], a[i], b[i]) for i in range(n.value)]

    def format_site(self, s: NgsepSiteOut) -> str:
        buf = ctypes.create_string_buffer(4096)
        self._lib.ngsep_format_site(self._ctx, ctypes.byref(s), buf, 4096)
        return buf.value.decode()

    def write_vcf(self, path: str):
        self._check(self._lib.ngsep_write_vcf_header(self._ctx, path.encode()))
        self._check(self._lib.ngsep_append_vcf_records(self._ctx, path.encode()))

    # -- multisample (MultisampleVariantsDetector)
    def set_samples(self, read_groups: Sequence[tuple]):
        """read_groups: (read group id, sample id) per read-group index of the batches, as the BAM
        headers list them (MultisampleVariantsDetector.loadSamplesFromAlignmentHeaders, :499-523):
        samples are sorted by id, each sample's groups are visited in Java HashSet order."""
        samples = sorted({sm for _, sm in read_groups if sm is not None})
        sidx = {sm: i for i, sm in enumerate(samples)}
        rg_sample = [sidx[sm] if sm is not None else -1 for _, sm in read_groups]
        rg_rank = [0] * len(read_groups)
        for sm in samples:
            members = [g for g, (_, s2) in enumerate(read_groups) if s2 == sm]
            order = java_hashset_order([read_groups[g][0] for g in members])
            for rank, k in enumerate(order):
                rg_rank[members[k]] = rank
        self.samples = samples
        ids = (ctypes.c_char_p * max(len(samples), 1))(*[x.encode() for x in samples])
        gs = (ctypes.c_int32 * max(len(read_groups), 1))(*rg_sample)
        gr = (ctypes.c_int32 * max(len(read_groups), 1))(*rg_rank)
        self._check(self._lib.ngsep_set_samples(self._ctx, len(samples), ids, len(read_groups), gs, gr))

    def raw_population_sites(self):
        n = ctypes.c_int64()
        self._check(self._lib.ngsep_fetch_population_sites(self._ctx, None, None, 0, ctypes.byref(n)))
        S = len(self.samples)
        sites = (NgsepPopSiteOut * max(n.value, 1))()
        calls = (NgsepSampleCall * max(n.value * S, 1))()
        self._check(self._lib.ngsep_fetch_population_sites(self._ctx, sites, calls, n.value, ctypes.byref(n)))
        return sites[: n.value], calls[: n.value * S]

    def population_vcf_line(self, i: int) -> str:
        """the VCF line of population site i (ngsep_population_site_vcf_line, ABI 8)"""
        need = self._lib.ngsep_population_site_vcf_line(self._ctx, i, None, 0)
        if need < 0:
            raise NgsepError(int(need), self._lib.ngsep_last_error(self._ctx).decode())
        buf = ctypes.create_string_buffer(int(need) + 1)
        self._lib.ngsep_population_site_vcf_line(self._ctx, i, buf, int(need) + 1)
        return buf.value.decode()

    def getPopulationVariants(self) -> List[PopulationSite]:
        """the population records; an indel / STR record (multisnv_type 3: the realigner's regions, ABI 8) takes its
        alleles from its VCF line and carries that line in vcf_line (its per-sample calls are only there)"""
        names = self.sequence_names()
        sites, calls = self.raw_population_sites()
        S = len(self.samples)
        out = []
        for i, s in enumerate(sites):
            seq = names[s.seq_id] if 0 <= s.seq_id < len(names) else "?"
            if s.multisnv_type == 3:
                line = self.population_vcf_line(i)
                f = line.split("\t", 6)
                out.append(PopulationSite(sequence=seq, pos=s.pos, alleles=[f[3]] + ([] if f[4] == "." else f[4].split(",")),
                                          qual=s.qual, multisnv_type=False, calls=[], vcf_line=line))
                continue
            out.append(PopulationSite(
                sequence=seq, pos=s.pos,
                alleles=[BASES[s.alleles[k]] for k in range(s.n_alleles)], qual=s.qual,
                multisnv_type=s.multisnv_type == 1, calls=list(calls[i * S:(i + 1) * S]), embedded=s.multisnv_type == 2))
        return out

    def write_population_vcf(self, path: str):
        self._check(self._lib.ngsep_write_population_vcf(self._ctx, path.encode()))

    def stats(self) -> NgsepStats:
        st = NgsepStats()
        self._check(self._lib.ngsep_get_stats(self._ctx, ctypes.byref(st)))
        return st


class SingleSampleVariantsDetector:
    """Drop-in for ngsep.discovery.SingleSampleVariantsDetector (SNV path).

    Setter names follow the Java class; run() is SingleSampleVariantsDetector.run (:589-656)
    restricted to findSNVS (the SV/CNV analyses are off by default and out of scope).
    """

    DEF_MIN_QUALITY = 40
    DEF_MAX_BASE_QS = 30
    DEF_MIN_MQ = 20
    DEF_PLOIDY = 2
    DEF_MAX_ALNS_PER_START_POS = 5
    DEF_HETEROZYGOSITY_RATE_DIPLOID = 0.001

    def __init__(self):
        self.params = default_params()
        self.inputFile: Optional[str] = None
        self.genomeFile: Optional[str] = None
        self.outputPrefix: Optional[str] = None
        self.knownVariantsFile: Optional[str] = None
        self.knownSTRsFile: Optional[str] = None
        self.device = 0

    # setters (CommandsDescriptor reflective setters)
    def setKnownVariantsFile(self, v: str): self.knownVariantsFile = v
    def getKnownVariantsFile(self) -> Optional[str]: return self.knownVariantsFile
    def setKnownSTRsFile(self, v: str): self.knownSTRsFile = v                   # (:400-402)
    def getKnownSTRsFile(self) -> Optional[str]: return self.knownSTRsFile
    def setInputFile(self, v: str): self.inputFile = v
    def setGenome(self, v: str): self.genomeFile = v
    def setOutputPrefix(self, v: str): self.outputPrefix = v
    def setSampleId(self, v: str): self.params.sample_id = v.encode()
    def setNormalPloidy(self, v: int): self.params.ploidy = int(v)
    def setPrintSamplePloidy(self, v: bool): self.params.print_sample_ploidy = int(bool(v))
    def setMinMQ(self, v: int): self.params.min_mq = int(v)
    def setMaxAlnsPerStartPos(self, v: int): self.params.max_alns_per_start = int(v)
    def setProcessNonUniquePrimaryAlignments(self, v: bool): self.params.process_nonunique = int(bool(v))
    def setProcessSecondaryAlignments(self, v: bool): self.params.process_secondary = int(bool(v))
    def setBasesToIgnore5P(self, v: int): self.params.ignore5 = int(v)
    def setBasesToIgnore3P(self, v: int): self.params.ignore3 = int(v)
    def setHeterozygosityRate(self, v: float):
        self.params.het_rate = float(v)
        self.params.het_rate_set = 1
    def setMaxBaseQS(self, v: int): self.params.max_base_qs = int(v)
    def setMinQuality(self, v: int): self.params.min_quality = int(v)
    def setIgnoreLowerCaseRef(self, v: bool): self.params.ignore_lowercase_ref = int(bool(v))
    def setCallEmbeddedSNVs(self, v: bool): self.params.call_embedded = int(bool(v))
    def setCalcStrandBias(self, v: bool): self.params.calc_strand_bias = int(bool(v))
    def setQuerySeq(self, v: str): self.params.query_seq = v.encode()
    def setQueryFirst(self, v: int): self.params.query_first = int(v)
    def setQueryLast(self, v: int): self.params.query_last = int(v)

    _OPTIONS = {
        "-i": ("setInputFile", str), "-r": ("setGenome", str), "-o": ("setOutputPrefix", str),
        "-sampleId": ("setSampleId", str), "-ploidy": ("setNormalPloidy", int),
        "-minMQ": ("setMinMQ", int), "-maxAlnsPerStartPos": ("setMaxAlnsPerStartPos", int),
        "-ignore5": ("setBasesToIgnore5P", int), "-ignore3": ("setBasesToIgnore3P", int),
        "-h": ("setHeterozygosityRate", float), "-maxBaseQS": ("setMaxBaseQS", int),
        "-minQuality": ("setMinQuality", int), "-querySeq": ("setQuerySeq", str),
        "-first": ("setQueryFirst", int), "-last": ("setQueryLast", int),
        "-knownVariants": ("setKnownVariantsFile", str),
        "-knownSTRs": ("setKnownSTRsFile", str),
    }
    _FLAGS = {
        "-psp": "setPrintSamplePloidy", "-p": "setProcessNonUniquePrimaryAlignments",
        "-s": "setProcessSecondaryAlignments", "-ignoreLowerCaseRef": "setIgnoreLowerCaseRef",
        "-embeddedSNVs": "setCallEmbeddedSNVs", "-csb": "setCalcStrandBias",
    }

    @classmethod
    def main(cls, args: Sequence[str]) -> "SingleSampleVariantsDetector":
        inst = cls()
        i = 0
        args = list(args)
        while i < len(args):
            a = args[i]
            if a in cls._OPTIONS and i + 1 < len(args):
                name, typ = cls._OPTIONS[a]
                getattr(inst, name)(typ(args[i + 1]))
                i += 2
            elif a in cls._FLAGS:
                getattr(inst, cls._FLAGS[a])(True)
                i += 1
            else:
                raise ValueError(f"Unrecognized option {a}")
        inst.run()
        return inst

    def run(self):
        if self.inputFile is None:
            raise NgsepError(_lib.NGSEP_E_IO, "The input file with alignments is a required parameter")
        if self.genomeFile is None:
            raise NgsepError(_lib.NGSEP_E_IO, "The reference genome file is a required parameter")
        with GpuPileupSession(self.params, self.device) as s:
            s.load_fasta(self.genomeFile)
            if self.knownVariantsFile:
                s.set_known_variants(self.knownVariantsFile)
            elif self.knownSTRsFile:
                s.set_known_strs(self.knownSTRsFile)
            s.processFile(self.inputFile, (self.outputPrefix or "variants") + ".vcf")
            self.stats = s.stats()


class MultisampleVariantsDetector:
    """Drop-in for ngsep.discovery.MultisampleVariantsDetector (SNV path,
    discovery/MultisampleVariantsDetector.java:54-693; options main/CommandsDescriptor.xml).

    Alignments arrive through a GpuPileupSession in multisample mode; run() processes one batch
    stream whose read-group indexes refer to read_groups (e.g. a merged BAM of all samples)."""

    DEF_MIN_QUALITY = 40
    DEF_MIN_ALLELE_DEPTH_FREQUENCY = 0.0
    DEF_OUTPUT_FILE = "variants.vcf"

    def __init__(self):
        self.params = default_params()
        self.params.multisample = 1
        self.genomeFile: Optional[str] = None
        self.outFilename = self.DEF_OUTPUT_FILE
        self.device = 0

    def setGenome(self, v: str): self.genomeFile = v
    def setKnownVariantsFile(self, v: str): self.knownVariantsFile = v          # (:193-195)
    def setKnownSTRsFile(self, v: str): self.knownSTRsFile = v                  # (:439-446)
    def setCallEmbeddedSNVs(self, v: bool): self.params.call_embedded = int(bool(v))
    def setOutFilename(self, v: str): self.outFilename = v
    def setMinAlleleDepthFrequency(self, v: float): self.params.min_allele_depth_freq = float(v)
    def setHeterozygosityRate(self, v: float):
        self.params.het_rate = float(v)
        self.params.het_rate_set = 1
    def setMinQuality(self, v: int): self.params.min_quality = int(v)
    def setMaxBaseQS(self, v: int): self.params.max_base_qs = int(v)
    def setNormalPloidy(self, v: int): self.params.ploidy = int(v)
    def setPrintSamplePloidy(self, v: bool): self.params.print_sample_ploidy = int(bool(v))
    def setMinMQ(self, v: int): self.params.min_mq = int(v)
    def setMaxAlnsPerStartPos(self, v: int): self.params.max_alns_per_start = int(v)
    def setProcessNonUniquePrimaryAlignments(self, v: bool): self.params.process_nonunique = int(bool(v))
    def setProcessSecondaryAlignments(self, v: bool): self.params.process_secondary = int(bool(v))
    def setBasesToIgnore5P(self, v: int): self.params.ignore5 = int(v)
    def setBasesToIgnore3P(self, v: int): self.params.ignore3 = int(v)
    def setIgnoreLowerCaseRef(self, v: bool): self.params.ignore_lowercase_ref = int(bool(v))
    def setQuerySeq(self, v: str): self.params.query_seq = v.encode()
    def setQueryFirst(self, v: int): self.params.query_first = int(v)
    def setQueryLast(self, v: int): self.params.query_last = int(v)

    def run(self, input_files: Sequence[str]) -> GpuPileupSession:
        """MultisampleVariantsDetector.run (:421-459) on BAM files: samples from the headers,
        files merged in the generator's order, VCF written to outFilename."""
        if self.genomeFile is None:
            raise NgsepError(_lib.NGSEP_E_IO, "The reference genome file is a required parameter")
        s = GpuPileupSession(self.params, self.device)
        s.load_fasta(self.genomeFile)
        if getattr(self, "knownVariantsFile", None):
            s.set_known_variants(self.knownVariantsFile)
        elif getattr(self, "knownSTRsFile", None):          # (the realigner's input STRs when no input variants)
            s.set_known_strs(self.knownSTRsFile)
        arr = (ctypes.c_char_p * len(input_files))(*[f.encode() for f in input_files])
        s._check(s._lib.ngsep_call_population_bams(s._ctx, arr, len(input_files), self.outFilename.encode()))
        return s

    def session(self, read_groups: Sequence[tuple]) -> GpuPileupSession:
        s = GpuPileupSession(self.params, self.device)
        s.set_samples(read_groups)
        return s

    def run_batches(self, read_groups: Sequence[tuple], batches, contigs=None) -> GpuPileupSession:
        """AlignmentsPileupGenerator.processFiles over already merged batches, then the VCF."""
        s = self.session(read_groups)
        if contigs is not None:
            for name, seq in contigs:
                s.set_reference(name, seq)
        elif self.genomeFile is not None:
            s.load_fasta(self.genomeFile)
        else:
            raise NgsepError(_lib.NGSEP_E_IO, "The reference genome file is a required parameter")
        for b in batches:
            s.processAlignments(b)
        s.notifyEndOfAlignments()
        s.write_population_vcf(self.outFilename)
        return s


class CoverageStatisticsCalculator:
    """Drop-in for ngsep.discovery.CoverageStatisticsCalculator (discovery/CoverageStatisticsCalculator.java:
    31-216; command CoverageStats, main/CommandsDescriptor.xml:458-477): per-position numAlignments and
    numUniqueAlns histograms, the per-position loop on the GPU (coverage.hip)."""

    DEF_MIN_MQ_UNIQUE_ALIGNMENT = 20

    def __init__(self):
        self.params = default_params()
        self.params.coverage_stats = 1
        self.params.process_secondary = 1      # processFile (:108-114)
        self.params.max_alns_per_start = 100
        self.params.max_coverage = 300
        self.inputFile: Optional[str] = None
        self.outputFile: Optional[str] = None
        self.genomeFile: Optional[str] = None
        self.device = 0
        self.coverageCounts: List[int] = []
        self.coverageCountUniqueAlignments: List[int] = []
        self.highCoverageCount = 0
        self.highCoverageCountUniqueAlignments = 0

    def setInputFile(self, v: str): self.inputFile = v
    def setOutputFile(self, v: str): self.outputFile = v
    def setGenome(self, v: str): self.genomeFile = v
    def setMinMQ(self, v: int): self.params.min_mq = int(v)
    def getMinMQ(self) -> int: return self.params.min_mq
    def setMaxCoverage(self, v: int): self.params.max_coverage = int(v)
    def getMaxCoverage(self) -> int: return self.params.max_coverage
    def getCoverageCounts(self) -> List[int]: return self.coverageCounts
    def getHighCoverageCount(self) -> int: return self.highCoverageCount

    def getCoverageMaxCount(self) -> int:
        """Most frequent depth >= 1 (:200-208)."""
        m = 1
        for i in range(1, len(self.coverageCounts)):
            if self.coverageCounts[m] < self.coverageCounts[i]:
                m = i
        return m

    def _session(self) -> GpuPileupSession:
        s = GpuPileupSession(self.params, self.device)
        if self.genomeFile is not None:
            s.load_fasta(self.genomeFile)
        return s

    def _collect(self, s: GpuPileupSession):
        n = self.params.max_coverage
        a, u = (ctypes.c_int64 * n)(), (ctypes.c_int64 * n)()
        hi, hu = ctypes.c_int64(), ctypes.c_int64()
        s._check(s._lib.ngsep_fetch_coverage(s._ctx, a, u, ctypes.byref(hi), ctypes.byref(hu)))
        self.coverageCounts, self.coverageCountUniqueAlignments = list(a), list(u)
        self.highCoverageCount, self.highCoverageCountUniqueAlignments = hi.value, hu.value

    def run(self):
        if self.inputFile is None:
            raise NgsepError(_lib.NGSEP_E_IO, "The alignments input file is a required parameter")
        self.processFile(self.inputFile, self.outputFile)

    def processFile(self, inputFile: str, outputFile: Optional[str] = None):
        """processFile (:99-122): BAM -> histograms -> printCoverageStats (stdout when outputFile is None)."""
        with self._session() as s:
            s._check(s._lib.ngsep_coverage_bam(s._ctx, inputFile.encode(), (outputFile or "-").encode()))
            self._collect(s)

    def processBatches(self, batches, contigs=None):
        """Path A: reader-filtered alignment batches (the generator's input) -> histograms."""
        with self._session() as s:
            if contigs is not None:
                for name, seq in contigs:
                    s.set_reference(name, seq)
            for b in batches:
                s.processAlignments(b)
            s.notifyEndOfAlignments()
            self._collect(s)

    def printCoverageStats(self, out=None) -> str:
        lines = [f"{i}\t{self.coverageCounts[i]}\t{self.coverageCountUniqueAlignments[i]}"
                 for i in range(1, len(self.coverageCounts))]
        lines.append(f"More\t{self.highCoverageCount}\t{self.highCoverageCountUniqueAlignments}")
        txt = "\n".join(lines) + "\n"
        if out is not None:
            out.write(txt)
        return txt


class RelativeAlleleCountsCalculator:
    """Drop-in for ngsep.discovery.RelativeAlleleCountsCalculator (discovery/RelativeAlleleCountsCalculator.java:
    26-331; command RelativeAlleleCounts, main/CommandsDescriptor.xml): the distributions of the proportion of
    the second most frequent allele and of the number of alleles over the pileups, the per-position loop on the
    GPU (kernels.hip k_rac over the streamed windows' byte pile)."""

    DEF_MIN_RD = 10
    DEF_MAX_RD = 1000
    DEF_MIN_BASE_QUALITY_SCORE = 20

    def __init__(self):
        self.params = default_params()
        self.params.relative_allele_counts = 1
        self.params.rac_min_rd = self.DEF_MIN_RD
        self.params.rac_min_bq = self.DEF_MIN_BASE_QUALITY_SCORE
        self.params.max_alns_per_start = self.DEF_MAX_RD       # runProcess: generator.setMaxAlnsPerStartPos(maxRD)
        self.params.process_secondary = 0
        self.inputFile: Optional[str] = None
        self.outputFile: Optional[str] = None
        self.genomeFile: Optional[str] = None
        self.device = 0
        self.proportions: List[float] = []
        self.numAlleles: List[float] = []
        self.moments: List[float] = []

    def setInputFile(self, v: str): self.inputFile = v
    def setOutputFile(self, v: str): self.outputFile = v
    def setGenome(self, v: str): self.genomeFile = v
    def setMinRD(self, v: int): self.params.rac_min_rd = int(v)
    def getMinRD(self) -> int: return self.params.rac_min_rd
    def setMaxRD(self, v: int): self.params.max_alns_per_start = int(v)
    def getMaxRD(self) -> int: return self.params.max_alns_per_start
    def setMinBaseQualityScore(self, v: int): self.params.rac_min_bq = int(v)
    def getMinBaseQualityScore(self) -> int: return self.params.rac_min_bq
    def setSecondaryAlns(self, v: bool): self.params.process_secondary = 1 if v else 0
    def isSecondaryAlns(self) -> bool: return bool(self.params.process_secondary)

    def _session(self) -> GpuPileupSession:
        s = GpuPileupSession(self.params, self.device)
        if self.genomeFile is not None:
            s.load_fasta(self.genomeFile)
        return s

    def _collect(self, s: GpuPileupSession):
        p, n, m = (ctypes.c_double * 51)(), (ctypes.c_double * 10)(), (ctypes.c_double * 6)()
        s._check(s._lib.ngsep_fetch_rac(s._ctx, p, n, m))
        self.proportions, self.numAlleles, self.moments = list(p), list(n), list(m)

    def run(self):
        if self.inputFile is None:
            raise NgsepError(_lib.NGSEP_E_IO, "The alignments input file is a required parameter")
        self.runProcess(self.inputFile, self.outputFile or "-")

    def runProcess(self, filename: str, out_path: Optional[str] = None):
        """runProcess + printResults (:183-244): BAM -> distributions -> report text (out_path; None = no text)."""
        with self._session() as s:
            s._check(s._lib.ngsep_rac_bam(s._ctx, filename.encode(), out_path.encode() if out_path else None))
            self._collect(s)

    def processBatches(self, batches, contigs=None, out_path: Optional[str] = None):
        """Path A: reader-filtered alignment batches (the generator's input) -> distributions."""
        with self._session() as s:
            if contigs is not None:
                for name, seq in contigs:
                    s.set_reference(name, seq)
            for b in batches:
                s.processAlignments(b)
            s.notifyEndOfAlignments()
            self._collect(s)
            if out_path:
                s._check(s._lib.ngsep_write_rac(s._ctx, out_path.encode()))
