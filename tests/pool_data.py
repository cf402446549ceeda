"""Seeded pooled-sample data for the ploidy >= 3 tests (SingleSampleVariantPileupListener.genotypeVariantPool,
:402-503): a reference, H donor haplotypes carrying SNVs at chosen allele counts k/H (some sites with two
alternative alleles), reads drawn uniformly from the haplotypes.  Test data infrastructure only.

Writes FASTA + coordinate-sorted SAM (the oracle's input) and the BAM + BAI the product reads (pysynth).
"""
from __future__ import annotations

import numpy as np

import pysynth

_B = np.frombuffer(b"ACGT", dtype=np.uint8)


def write_pool(prefix: str, length: int = 60000, haplotypes: int = 8, depth: float = 60.0, seed: int = 1,
               site_rate: float = 4e-3, multi_frac: float = 0.25, read_len: int = 150, n_contigs: int = 2,
               low_q_frac: float = 0.05, rg_samples=None):
    """rg_samples: None (one sample, no @RG) or a list of sample names; reads then get read groups
    (one per sample) round-robin, each sample its own haplotype pool -- the multisample case."""
    rng = np.random.default_rng(seed)
    fa, sam = prefix + ".fa", prefix + ".sam"
    contigs = []
    for c in range(n_contigs):
        ref = _B[rng.integers(0, 4, size=length)].copy()
        contigs.append((f"pool{c + 1}", ref))
    groups = rg_samples or [None]
    with open(fa, "w") as f:
        for name, ref in contigs:
            f.write(f">{name}\n")
            s = ref.tobytes().decode()
            for i in range(0, len(s), 80):
                f.write(s[i:i + 80] + "\n")
    recs = []
    for ci, (name, ref) in enumerate(contigs):
        for gi, sm in enumerate(groups):
            haps = np.tile(ref, (haplotypes, 1))
            sites = np.nonzero(rng.random(length) < site_rate)[0]
            for p in sites:
                r = int(np.nonzero(_B == ref[p])[0][0])
                alts = [a for a in range(4) if a != r]
                rng.shuffle(alts)
                k1 = int(rng.integers(1, haplotypes + 1))
                order = rng.permutation(haplotypes)
                haps[order[:k1], p] = _B[alts[0]]
                if rng.random() < multi_frac and k1 < haplotypes:
                    k2 = int(rng.integers(1, haplotypes - k1 + 1))
                    haps[order[k1:k1 + k2], p] = _B[alts[1]]
            n_reads = int(length * depth / read_len / len(groups))
            starts = np.sort(rng.integers(0, length - read_len + 1, size=n_reads))
            hsel = rng.integers(0, haplotypes, size=n_reads)
            neg = rng.random(n_reads) < 0.5
            for i in range(n_reads):
                s0 = int(starts[i])
                seq = haps[hsel[i], s0:s0 + read_len].copy()
                q = rng.integers(20, 41, size=read_len)
                low = rng.random(read_len) < low_q_frac
                q[low] = rng.integers(2, 8, size=int(low.sum()))
                err = rng.random(read_len) < 0.003
                if err.any():
                    seq[err] = _B[rng.integers(0, 4, size=int(err.sum()))]
                nmask = rng.random(read_len) < 0.002
                seq[nmask] = ord("N")
                recs.append((ci, s0 + 1, f"r{ci}_{gi}_{i}", 16 if neg[i] else 0, seq.tobytes().decode(),
                             (q + 33).astype(np.uint8).tobytes().decode(), sm))
    recs.sort(key=lambda r: (r[0], r[1]))
    with open(sam, "w") as f:
        f.write("@HD\tVN:1.6\tSO:coordinate\n")
        for name, ref in contigs:
            f.write(f"@SQ\tSN:{name}\tLN:{len(ref)}\n")
        for sm in groups:
            if sm is not None:
                f.write(f"@RG\tID:rg_{sm}\tSM:{sm}\n")
        for ci, pos, qn, flag, seq, qual, sm in recs:
            tag = f"\tRG:Z:rg_{sm}" if sm is not None else ""
            f.write(f"{qn}\t{flag}\t{contigs[ci][0]}\t{pos}\t60\t{len(seq)}M\t*\t0\t0\t{seq}\t{qual}{tag}\n")
    bam = pysynth.sam_to_bam(sam, prefix + ".bam")
    return fa, sam, bam
