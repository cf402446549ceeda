"""ctypes wrapper of libngsep_synth.so: seeded synthetic genomes/reads.

Test and bench data infrastructure only.
"""
from __future__ import annotations

import ctypes
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(_HERE)))
from ngsepcore_amd._lib import NgsepReadBatch  # noqa: E402

LIB = os.path.join(_HERE, "build", "libngsep_synth.so")
YEAST, HUMAN, CUSTOM = 0, 1, 2


class SynthParams(ctypes.Structure):
    _fields_ = [
        ("genome", ctypes.c_int32), ("contig_first", ctypes.c_int32), ("n_contigs", ctypes.c_int32),
        ("custom_len", ctypes.c_int64), ("depth", ctypes.c_double), ("read_len", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("snv_rate", ctypes.c_double), ("dup_rate", ctypes.c_double),
        ("lower_frac", ctypes.c_double), ("n_frac", ctypes.c_double), ("sample_idx", ctypes.c_int32),
        ("quality_model", ctypes.c_int32), ("secondary_rate", ctypes.c_double), ("lowmq_rate", ctypes.c_double),
        ("noqual_rate", ctypes.c_double), ("softclip_rate", ctypes.c_double), ("n_samples", ctypes.c_int32),
        ("trunc_len", ctypes.c_int64), ("rng_per_contig", ctypes.c_int32), ("indel_rate", ctypes.c_double),
        ("hot_first", ctypes.c_int64), ("hot_len", ctypes.c_int64), ("hot_depth", ctypes.c_double),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        l = ctypes.CDLL(LIB)
        l.ngs_synth_default.argtypes = [ctypes.POINTER(SynthParams)]
        l.ngs_synth_create.restype = ctypes.c_void_p
        l.ngs_synth_create.argtypes = [ctypes.POINTER(SynthParams)]
        l.ngs_synth_free.argtypes = [ctypes.c_void_p]
        l.ngs_synth_n_contigs.argtypes = [ctypes.c_void_p]
        l.ngs_synth_contig_name.restype = ctypes.c_char_p
        l.ngs_synth_contig_name.argtypes = [ctypes.c_void_p, ctypes.c_int]
        l.ngs_synth_contig_len.restype = ctypes.c_int64
        l.ngs_synth_contig_len.argtypes = [ctypes.c_void_p, ctypes.c_int]
        l.ngs_synth_contig_seq.restype = ctypes.c_void_p
        l.ngs_synth_contig_seq.argtypes = [ctypes.c_void_p, ctypes.c_int]
        l.ngs_synth_n_reads.restype = ctypes.c_int64
        l.ngs_synth_n_reads.argtypes = [ctypes.c_void_p]
        l.ngs_synth_n_bases.restype = ctypes.c_int64
        l.ngs_synth_n_bases.argtypes = [ctypes.c_void_p]
        l.ngs_synth_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(NgsepReadBatch)]
        for f in ("ngs_synth_write_fasta", "ngs_synth_write_sam", "ngs_synth_write_bam", "ngs_synth_write_truth"):
            getattr(l, f).argtypes = [ctypes.c_void_p, ctypes.c_char_p]
        l.ngs_sam_to_bam.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        l.ngs_synth_write_bam_sample.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int]
        _lib = l
    return _lib


def sam_to_bam(sam: str, bam: str) -> str:
    rc = lib().ngs_sam_to_bam(sam.encode(), bam.encode())
    if rc != 0:
        raise IOError(f"sam_to_bam failed ({rc}) for {sam}")
    return bam


class Synth:
    def __init__(self, genome=YEAST, depth=30.0, seed=2, n_contigs=0, contig_first=0, custom_len=0, **kw):
        p = SynthParams()
        lib().ngs_synth_default(ctypes.byref(p))
        p.genome, p.depth, p.seed, p.n_contigs, p.contig_first, p.custom_len = genome, depth, seed, n_contigs, contig_first, custom_len
        for k, v in kw.items():
            setattr(p, k, v)
        self.params = p
        self.h = lib().ngs_synth_create(ctypes.byref(p))

    def close(self):
        if self.h:
            lib().ngs_synth_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def contigs(self):
        n = lib().ngs_synth_n_contigs(self.h)
        out = []
        for i in range(n):
            L = lib().ngs_synth_contig_len(self.h, i)
            seq = ctypes.string_at(lib().ngs_synth_contig_seq(self.h, i), L)
            out.append((lib().ngs_synth_contig_name(self.h, i).decode(), seq))
        return out

    @property
    def n_reads(self):
        return lib().ngs_synth_n_reads(self.h)

    @property
    def n_bases(self):
        return lib().ngs_synth_n_bases(self.h)

    def batch(self) -> NgsepReadBatch:
        b = NgsepReadBatch()
        lib().ngs_synth_batch(self.h, ctypes.byref(b))
        return b

    def write(self, prefix: str):
        l = lib()
        for f, suf in (("ngs_synth_write_fasta", ".fa"), ("ngs_synth_write_sam", ".sam"),
                       ("ngs_synth_write_bam", ".bam"), ("ngs_synth_write_truth", "_truth.vcf")):
            rc = getattr(l, f)(self.h, (prefix + suf).encode())
            if rc != 0:
                raise IOError(f"{f} failed for {prefix}{suf}")
        return prefix + ".fa", prefix + ".sam", prefix + ".bam"

    def write_sample_bams(self, prefix: str):
        """one BAM per sample of a population (n_samples > 1)"""
        out = []
        for k in range(max(1, self.params.n_samples)):
            path = f"{prefix}_S{self.params.sample_idx + k:03d}.bam"
            if lib().ngs_synth_write_bam_sample(self.h, path.encode(), k) != 0:
                raise IOError(f"write failed for {path}")
            out.append(path)
        return out
