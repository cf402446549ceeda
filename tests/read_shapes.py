"""Seeded SAM text with the read shapes real BAMs carry (test-data infrastructure, never imported by the product).

The tools/synth generator writes single-end, fixed-length M/I/D/S records; the reference's reader and pileup path take
much more (ReadAlignment.java:60-69 op codes, :747-871 updateAlleleCallsInfo, :1180-1266 setCigarString;
ReadAlignmentFileReader.java:219-306 loadAlignment / isMultiple / isSameAlignment).  This module writes, for one
sample or a population of read groups:

* paired-end fragments: flags 0x1 / 0x2 / 0x20 / 0x40 / 0x80 / 0x10, overlapping mates (fragments shorter than the two
  reads), improper pairs, mates on the other sequence (RNEXT), mates unmapped (0x8, the unmapped mate placed at its
  partner's position with flag 0x4 and CIGAR '*');
* mixed read lengths: 75-250 bp, plus a few 5-20 kb single-end reads;
* CIGAR styles: M, '=' / 'X' per base against the reference, hard clips (H, the bases absent from SEQ), soft clips,
  'N' reference skips (spliced reads), 'P' padding between M blocks, I / D from donor indels;
* reader corner cases: PCR-duplicate (0x400), QC-fail (0x200) and supplementary (0x800) records (all kept: the filter
  is unmapped + secondary + multiple, AlignmentsPileupGenerator.java:367-372), secondary (0x100), NH:i tags, MAPQ 0-60,
  a record repeated verbatim (isSameAlignment), SEQ '*' records, unmapped records without a position at the end.

The oracle (oracle/ngsep_oracle.c) reads the SAM; the HIP path reads the same records as BAM (tools/synth
ngs_sam_to_bam).  Deterministic in the seed.
"""
from __future__ import annotations

import numpy as np

BASES = "ACGT"


def _rand_seq(rng, n):
    return "".join(BASES[i] for i in rng.choice(4, size=n, p=[0.3, 0.2, 0.2, 0.3]))


class Donor:
    """One diploid individual: SNVs (shared positions across samples with per-sample genotypes) and small indels."""

    def __init__(self, ref: str, sites, rng):
        self.ref = ref
        self.hap = [dict(), dict()]          # 0-based ref position -> ("S", base) | ("I", bases) | ("D", length)
        for pos, kind, val, af in sites:
            for h in (0, 1):
                if rng.random() < af:
                    self.hap[h][pos] = (kind, val)

    def walk(self, h, start, nbases, rng, max_ref=None):
        """the read bases and the alignment ops (list of (op, len)) of a read of nbases starting at ref position start
        (0-based) on haplotype h; stops at the sequence end"""
        ev = self.hap[h]
        seq, ops = [], []

        def op(o, n):
            if n <= 0:
                return
            if ops and ops[-1][0] == o:
                ops[-1] = (o, ops[-1][1] + n)
            else:
                ops.append((o, n))
        p = start
        L = len(self.ref) if max_ref is None else min(len(self.ref), max_ref)
        while len(seq) < nbases and p < L:
            e = ev.get(p)
            if e and e[0] == "D" and seq and p + e[1] < L:
                op("D", e[1])
                p += e[1]
                continue
            b = self.ref[p].upper()
            if e and e[0] == "S":
                b = e[1]
            seq.append(b)
            op("M", 1)
            if e and e[0] == "I" and len(seq) + len(e[1]) < nbases:
                seq.extend(e[1])
                op("I", len(e[1]))
            p += 1
        return "".join(seq), ops, p - start


def make_sites(ref, rng, snv_rate, indel_rate):
    sites = []
    for pos in range(20, len(ref) - 20):
        u = rng.random()
        if u < snv_rate:
            rb = ref[pos].upper()
            alt = BASES[(BASES.index(rb) + 1 + int(rng.integers(3))) % 4]
            sites.append((pos, "S", alt, float(rng.uniform(0.1, 0.9))))
        elif u < snv_rate + indel_rate:
            if rng.random() < 0.5:
                sites.append((pos, "I", _rand_seq(rng, int(rng.integers(1, 6))), float(rng.uniform(0.1, 0.9))))
            else:
                sites.append((pos, "D", int(rng.integers(1, 6)), float(rng.uniform(0.1, 0.9))))
    # no two events within 8 bp (each read walk applies one per position)
    out, last = [], -100
    for s in sites:
        if s[0] - last > 8:
            out.append(s)
            last = s[0]
    return out


def _quals(rng, n):
    q = rng.choice([2, 8, 15, 22, 27, 30, 33, 35, 37, 40], size=n, p=[.02, .03, .05, .1, .1, .1, .15, .15, .2, .1])
    return "".join(chr(33 + int(x)) for x in q)


def _errors(seq, qual, rng):
    s = list(seq)
    for i, c in enumerate(s):
        q = ord(qual[i]) - 33
        if rng.random() < 10 ** (-q / 10) and c in BASES:
            s[i] = BASES[(BASES.index(c) + 1 + int(rng.integers(3))) % 4]
        if rng.random() < 0.001:
            s[i] = "N"
    return "".join(s)


def _cigar(ops):
    return "".join(f"{n}{o}" for o, n in ops)


def _eqx(ops, seq, ref, start):
    """M runs rewritten as '=' / 'X' per base against the reference"""
    out, rp, qp = [], start, 0

    def add(o, n):
        if out and out[-1][0] == o:
            out[-1] = (o, out[-1][1] + n)
        else:
            out.append((o, n))
    for o, n in ops:
        if o == "M":
            for k in range(n):
                add("=" if seq[qp + k] == ref[rp + k].upper() else "X", 1)
            rp += n
            qp += n
        elif o in "DN":
            add(o, n)
            rp += n
        elif o in "IS":
            add(o, n)
            qp += n
        else:
            add(o, n)
    return out


class Rec:
    __slots__ = ("name", "flag", "seq_name", "pos", "mapq", "cigar", "rnext", "pnext", "tlen", "seq", "qual", "tags")

    def line(self):
        return "\t".join([self.name, str(self.flag), self.seq_name, str(self.pos), str(self.mapq), self.cigar, self.rnext,
                          str(self.pnext), str(self.tlen), self.seq, self.qual] + self.tags) + "\n"


def _rec(name, flag, seq_name, pos, mapq, cigar, rnext, pnext, tlen, seq, qual, tags):
    r = Rec()
    r.name, r.flag, r.seq_name, r.pos, r.mapq, r.cigar = name, flag, seq_name, pos, mapq, cigar
    r.rnext, r.pnext, r.tlen, r.seq, r.qual, r.tags = rnext, pnext, tlen, seq, qual, tags
    return r


def _shape(rng, donor, h, ref, start, rlen, sname, styles):
    """one mapped read: (pos 1-based, cigar, seq, qual) with a CIGAR style drawn from styles"""
    u = rng.random()
    style = "M"
    acc = 0.0
    for name, pr in styles:
        acc += pr
        if u < acc:
            style = name
            break
    if style == "N":                        # a spliced read: two blocks across a reference skip
        a = int(rng.integers(20, max(21, rlen - 20)))
        gap = int(rng.integers(50, 600))
        s1, o1, span1 = donor.walk(h, start, a, rng)
        if start + span1 + gap + (rlen - len(s1)) >= len(ref):
            style = "M"
        else:
            s2, o2, _ = donor.walk(h, start + span1 + gap, rlen - len(s1), rng)
            if not s2 or o2[0][0] != "M" or o1[-1][0] != "M":
                style = "M"
            else:
                seq, ops = s1 + s2, o1 + [("N", gap)] + o2
    if style != "N":
        seq, ops, _ = donor.walk(h, start, rlen, rng)
    if not ops or ops[0][0] != "M" or ops[-1][0] != "M":
        return None
    qual = _quals(rng, len(seq))
    seq = _errors(seq, qual, rng)
    pos = start + 1
    if style == "EQX":
        ops = _eqx(ops, seq, ref, start)
    elif style == "P" and len(ops) >= 1 and ops[0][0] == "M" and ops[0][1] > 10:
        k = int(rng.integers(3, ops[0][1] - 3))
        ops = [("M", k), ("P", int(rng.integers(1, 3))), ("M", ops[0][1] - k)] + ops[1:]
    elif style in ("H", "S"):
        c5 = int(rng.integers(3, 16)) if rng.random() < 0.7 else 0
        c3 = int(rng.integers(3, 16)) if (rng.random() < 0.7 or c5 == 0) else 0
        ok = ops[0][1] > c5 + c3 + 2 if len(ops) == 1 else (ops[0][1] > c5 + 2 and ops[-1][1] > c3 + 2)
        if ok:
            ops = list(ops)
            if c5:
                ops[0] = ("M", ops[0][1] - c5)
                pos += c5
            if c3:
                ops[-1] = ("M", ops[-1][1] - c3)
            if style == "H":
                seq, qual = seq[c5:len(seq) - c3], qual[c5:len(qual) - c3]
                ops = ([("H", c5)] if c5 else []) + ops + ([("H", c3)] if c3 else [])
            else:
                ops = ([("S", c5)] if c5 else []) + ops + ([("S", c3)] if c3 else [])
    return pos, _cigar(ops), seq, qual


def make_sam(path, fa_path, seed=1, n_samples=1, depth=12.0, lengths=(40000, 25000), snv_rate=3e-3, indel_rate=2e-4,
             long_frac=0.01, styles=None):
    """Writes the FASTA and the SAM; returns the read-group ids (one per sample, S000 ...)."""
    rng = np.random.default_rng(seed)
    names = [f"chr{chr(65 + i)}" for i in range(len(lengths))]
    refs = []
    for L in lengths:
        s = list(_rand_seq(rng, L))
        for i in rng.choice(L, size=L // 200, replace=False):       # a few lower-case (soft-masked) bases
            s[i] = s[i].lower()
        refs.append("".join(s))
    with open(fa_path, "w") as f:
        for n, s in zip(names, refs):
            f.write(f">{n}\n")
            for i in range(0, len(s), 60):
                f.write(s[i:i + 60] + "\n")
    styles = styles or [("EQX", 0.12), ("H", 0.08), ("S", 0.06), ("N", 0.05), ("P", 0.02)]
    sites = [make_sites(r, rng, snv_rate, indel_rate) for r in refs]
    rgs = [f"S{k:03d}" for k in range(n_samples)]
    recs = [[] for _ in refs]                 # per sequence: (pos, order, Rec)
    unmapped_tail = []
    order = 0
    for si, sm in enumerate(rgs):
        donors = [Donor(refs[c], sites[c], rng) for c in range(len(refs))]
        for c, ref in enumerate(refs):
            L = len(ref)
            target = depth * L
            bases = 0
            fno = 0
            while bases < target:
                fno += 1
                name = f"{sm}_{names[c]}_f{fno}"
                h = int(rng.integers(2))
                mapq = int(rng.choice([60, 60, 60, 60, 42, 25, 15, 3, 0]))
                tags = [f"RG:Z:{sm}"]
                if rng.random() < 0.05:
                    tags.append(f"NH:i:{int(rng.choice([1, 1, 2, 3]))}")
                extra = 0
                u = rng.random()
                if rng.random() < 0.01:
                    extra |= 0x400
                if rng.random() < 0.005:
                    extra |= 0x200
                if u < long_frac:                                  # a long single-end read
                    rlen = int(rng.integers(5000, 20000))
                    start = int(rng.integers(0, max(1, L - rlen - 1)))
                    sh = _shape(rng, donors[c], h, ref, start, rlen, names[c], [])
                    if sh is None:
                        continue
                    pos, cig, seq, qual = sh
                    flag = (0x10 if rng.random() < 0.5 else 0) | extra
                    recs[c].append((pos, order, _rec(name, flag, names[c], pos, mapq, cig, "*", 0, 0, seq, qual, tags)))
                    order += 1
                    bases += len(seq)
                    continue
                if u < 0.25:                                       # single end, 75-250 bp
                    rlen = int(rng.integers(75, 251))
                    start = int(rng.integers(0, L - rlen - 1))
                    sh = _shape(rng, donors[c], h, ref, start, rlen, names[c], styles)
                    if sh is None:
                        continue
                    pos, cig, seq, qual = sh
                    flag = (0x10 if rng.random() < 0.5 else 0) | extra
                    if rng.random() < 0.02:
                        seq, qual = "*", "*"                       # SEQ '*' (readLength from the CIGAR)
                    recs[c].append((pos, order, _rec(name, flag, names[c], pos, mapq, cig, "*", 0, 0, seq, qual, tags)))
                    order += 1
                    bases += rlen
                    continue
                # a pair: R1 forward at the fragment start, R2 reverse ending at the fragment end (overlapping mates
                # when the fragment is shorter than both reads)
                r1 = int(rng.integers(75, 251))
                r2 = int(rng.integers(75, 251)) if rng.random() < 0.5 else r1
                frag = int(np.clip(rng.normal(300, 80), max(r1, r2) + 1, 700))
                start = int(rng.integers(0, L - frag - 1))
                a = _shape(rng, donors[c], h, ref, start, r1, names[c], styles)
                b = _shape(rng, donors[c], h, ref, start + frag - r2, r2, names[c], styles)
                if a is None or b is None:
                    continue
                proper = 0x2 if rng.random() < 0.93 else 0
                kind = rng.random()
                f1 = 0x1 | proper | 0x40 | 0x20 | extra
                f2 = 0x1 | proper | 0x80 | 0x10 | extra
                tlen = b[0] + r2 - a[0]
                if kind < 0.04:                                    # mate unmapped: placed at its partner's position
                    f1 = (f1 | 0x8) & ~0x22
                    recs[c].append((a[0], order, _rec(name, f1, names[c], a[0], mapq, a[1], "=", a[0], 0, a[2], a[3], tags)))
                    order += 1
                    f2u = 0x1 | 0x80 | 0x4 | (f2 & 0x600)
                    recs[c].append((a[0], order, _rec(name, f2u, names[c], a[0], 0, "*", "=", a[0], 0, b[2], b[3], tags)))
                    order += 1
                    bases += r1
                    continue
                rn1 = rn2 = "="
                if kind < 0.07 and len(refs) > 1:                  # the mate on the other sequence
                    rn1 = rn2 = names[(c + 1) % len(refs)]
                    tlen = 0
                    f1 &= ~0x2
                    f2 &= ~0x2
                recs[c].append((a[0], order, _rec(name, f1, names[c], a[0], mapq, a[1], rn1, b[0], tlen, a[2], a[3], tags)))
                order += 1
                recs[c].append((b[0], order, _rec(name, f2, names[c], b[0], mapq, b[1], rn2, a[0], -tlen, b[2], b[3], tags)))
                order += 1
                bases += r1 + r2
                if rng.random() < 0.01:                            # a supplementary record of R1's last part
                    k = max(20, r1 // 3)
                    cig = f"{r1 - k}H{k}M"
                    sp = a[0] + (r1 - k)
                    recs[c].append((sp, order, _rec(name, (f1 | 0x800) & ~0x20, names[c], sp, mapq, cig, "=", b[0], 0,
                                                    a[2][-k:] if a[2] != "*" and len(a[2]) == r1 else "*",
                                                    a[3][-k:] if len(a[3]) == r1 else "*", tags)))
                    order += 1
                if rng.random() < 0.01:                            # a secondary alignment
                    sp = int(rng.integers(0, L - r1 - 1))
                    recs[c].append((sp + 1, order, _rec(name, f1 | 0x100, names[c], sp + 1, 0, f"{r1}M", "*", 0, 0, a[2] if len(a[2]) == r1 else "*",
                                                        a[3] if len(a[3]) == r1 else "*", tags)))
                    order += 1
            if rng.random() < 0.5:
                unmapped_tail.append(_rec(f"{sm}_{names[c]}_u", 0x4, "*", 0, 0, "*", "*", 0, 0, _rand_seq(rng, 100),
                                          _quals(rng, 100), [f"RG:Z:{sm}"]))
    with open(path, "w") as f:
        f.write("@HD\tVN:1.6\tSO:coordinate\n")
        for n, s in zip(names, refs):
            f.write(f"@SQ\tSN:{n}\tLN:{len(s)}\n")
        for sm in rgs:
            f.write(f"@RG\tID:{sm}\tSM:{sm}\tPL:ILLUMINA\n")
        for c in range(len(refs)):
            rs = sorted(recs[c], key=lambda t: (t[0], t[1]))
            for k, (_, _, r) in enumerate(rs):
                line = r.line()
                f.write(line)
                if k % 997 == 5:                                   # a record repeated verbatim (isSameAlignment)
                    f.write(line)
        for r in unmapped_tail:
            f.write(r.line())
    return rgs


def shape_stats(sam_path):
    """counts of the shapes the file holds (the tests assert each is present)"""
    st = dict(paired=0, overlap=0, eqx=0, hard=0, skip=0, pad=0, long=0, dup=0, qcfail=0, supp=0, secondary=0,
              mate_other=0, mate_unmapped=0, seq_star=0, lengths=set())
    for l in open(sam_path):
        if l.startswith("@"):
            continue
        f = l.split("\t")
        flag, cig = int(f[1]), f[5]
        st["paired"] += bool(flag & 1)
        st["eqx"] += ("=" in cig or "X" in cig)
        st["hard"] += "H" in cig
        st["skip"] += "N" in cig
        st["pad"] += "P" in cig
        st["dup"] += bool(flag & 0x400)
        st["qcfail"] += bool(flag & 0x200)
        st["supp"] += bool(flag & 0x800)
        st["secondary"] += bool(flag & 0x100)
        st["mate_unmapped"] += bool(flag & 0x8)
        st["mate_other"] += f[6] not in ("=", "*")
        st["seq_star"] += f[9] == "*"
        if f[9] != "*":
            st["lengths"].add(len(f[9]))
            st["long"] += len(f[9]) >= 5000
        if (flag & 0x41) == 0x41 and f[6] == "=" and 0 < int(f[8]) < 2 * len(f[9]):
            st["overlap"] += 1
    return st
