"""Known-answer checks of the oracle's pool algorithm (ploidy >= 3): single-site pileups built by hand, the
expected VCF line computed here by an independent pure-Python restatement of
SingleSampleVariantPileupListener.discoverSNV's pool branch (:238-254), createSNVVariantPool (:297-332),
genotypeVariantPool (:402-503), CountsHelper.updateCounts / getPosteriorProbabilities(h, major)
(CountsHelper.java:147-185,209-251,451-495) and CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts
(:228-282).  No reference output carries pool calls, so these pin the C restatement against a second
reading of the Java, not against the reference itself (parity unpinned)."""
import math
import os
import random

import pytest

import ngsep_oracle

BASES = "ACGT"


def jround(x):
    return int(math.floor(x + 0.5))


def phred(p):
    if p == 0:
        return 255
    s = -10 * math.log10(p)
    return 255 if s > 255 else jround(s)


def gt_cache(f, q, j):
    af = f / 500.0
    e = 10 ** (-0.1 * q)
    if j == 0:
        return math.log10(1 - e)
    return math.log10(af * (1 - e) + (1 - af) * e / (j - 1))


def helper(alleles, calls, freq):
    """calculateCountsGTSNV: counts over `alleles` and the full log-conditional matrix"""
    n = len(alleles)
    f, g = jround(freq * 500), jround((1 - freq) * 500)
    counts = [0] * n
    L = [[0.0] * n for _ in range(n)]
    total = 0
    for base, q in calls:
        total += 1
        q = min(30, q)
        if q <= 3:
            continue
        if base not in alleles:
            continue
        idx = alleles.index(base)
        counts[idx] += 1
        err_n = -0.1 * q - math.log10(n - 1)
        for i in range(n):
            L[i][i] += gt_cache(f, q, 0) if i == idx else err_n
            for j in range(n):
                if i != j:
                    L[i][j] += gt_cache(f, q, n) if j == idx else (gt_cache(g, q, n) if i == idx else err_n)
    return counts, L, total


def posteriors(ev):
    m = max(ev)
    p = [0.0 if x - m < -20 else 10 ** (x - m) for x in ev]
    t = sum(p)
    return [x / t for x in p]


def pool_genotype(alleles, calls, P, h):
    freqs = []
    fr = 1.0 / P
    while fr < 0.51:
        freqs.append(fr)
        fr += 1.0 / P
    hs = [helper(alleles, calls, f) for f in freqs]
    counts, L0, total = hs[0]
    major = max(range(len(alleles)), key=lambda i: (counts[i], -i))
    if counts[major] < P:
        return None
    t_hom = L0[major][major] + math.log10(1 - h)
    max_het, min_hom, max_alt, max_fi = 0.0, 1.0, -1, 0
    for i in range(len(alleles)):
        if i == major:
            continue
        terms = posteriors([t_hom] + [hs[j][1][major][i] + math.log10(h) for j in range(len(freqs))])
        im = max(range(len(terms)), key=lambda k: (terms[k], -k))
        if im == 0:
            min_hom = min(min_hom, terms[0])
        elif max_alt == -1 or max_het < terms[im]:
            max_het, max_fi, max_alt = terms[im], im - 1, i
    if max_alt == -1:
        return dict(called=[major], gq=phred(1 - min_hom), L=L0, counts=counts, dp=total)
    L = hs[max_fi][1]
    n = len(alleles)
    ev = posteriors([L[major][j] + (math.log10(1 - h) if j == major else math.log10(h / (n - 1))) for j in range(n)])
    return dict(called=sorted([major, max_alt]), gq=phred(1 - ev[max_alt]), L=L, counts=counts, dp=total)


def acn_from_counts(called, counts, P):
    acn = [0] * len(counts)
    if called == [0]:
        acn[0] = P
        return acn
    rc = [max(1, counts[c]) for c in called]
    tr = sum(rc)
    tc = 0
    for c, r in zip(called, rc):
        acn[c] = max(1, jround(P * r / tr))
        tc += acn[c]
    if tc < P:
        acn[called[0]] += P - tc
    else:
        ex = tc - P
        for c in reversed(called):
            rm = min(ex, acn[c] - 1)
            acn[c] -= rm
            ex -= rm
    return acn


def expected_line(seq, pos, ref, calls, P, h, minq=40):
    c4 = [sum(1 for b, q in calls if b == x and min(30, q) > 3) for x in BASES]
    s = sum(c4)
    min_count = max(1, (0.5 / P) * s)
    alleles = [ref] + [BASES[i] for i in range(4) if c4[i] >= min_count and BASES[i] != ref]
    if len(alleles) < 2:
        return None
    r = pool_genotype(alleles, calls, P, h)
    multi = len(alleles) > 2
    if multi:
        if r is None or r["called"] == [0]:
            return None
        if not (len(r["called"]) == 2 and r["called"][0] != 0):
            alt = alleles[r["called"][-1]]
            alleles = [ref, alt]
            multi = False
            r = pool_genotype(alleles, calls, P, h)
    if r is None or r["called"] == [0] or minq > r["gq"]:
        return None
    n = len(alleles)
    c = r["called"]
    gt = f"{c[0]}/{c[0]}" if len(c) == 1 else f"{c[0]}/{c[1]}"
    pl = ",".join(str(jround(-10 * r["L"][i][j])) for j in range(n) for i in range(j + 1))
    acn = acn_from_counts(c, r["counts"], P)
    return (f"{seq}\t{pos}\t.\t{ref}\t{','.join(alleles[1:])}\t0\t.\t{'TYPE=MULTISNV' if multi else '.'}\t"
            f"GT:PL:GQ:DP:ADP:ACN\t{gt}:{pl}:{r['gq']}:{r['dp']}:{','.join(map(str, r['counts']))}:"
            f"{','.join(map(str, acn))}")


def write_site(tmp, mixture, seed):
    """reads of 60 bp over position 100 of a 300 bp contig; every other base is the reference at q 35"""
    rng = random.Random(seed)
    refseq = "".join(rng.choice(BASES) for _ in range(300))
    ref = refseq[99]
    calls = []
    for base, q in mixture:
        calls.append((ref if base == "R" else base, q))
    rng.shuffle(calls)
    fa, sam = os.path.join(tmp, "s.fa"), os.path.join(tmp, "s.sam")
    with open(fa, "w") as f:
        f.write(">c1\n" + refseq + "\n")
    rows = []
    for k, (b, q) in enumerate(calls):
        start = 100 - rng.randint(1, 60) + 1       # 1-based start, covers 100
        s = list(refseq[start - 1:start - 1 + 60])
        s[100 - start] = b
        qs = [35] * 60
        qs[100 - start] = q
        rows.append((start, f"r{k}", 16 if k % 3 == 0 else 0, "".join(s), "".join(chr(x + 33) for x in qs)))
    rows.sort(key=lambda r: r[0])
    with open(sam, "w") as f:
        f.write("@SQ\tSN:c1\tLN:300\n")
        for start, qn, flag, s, qs in rows:
            f.write(f"{qn}\t{flag}\tc1\t{start}\t60\t60M\t*\t0\t0\t{s}\t{qs}\n")
    return fa, sam, ref, calls


MIXTURES = [
    # (mixture of (allele, q); "R" = the reference, "X"/"Y"/"Z" = the others, "N"), ploidy, h
    ([("R", 30)] * 20 + [("X", 30)] * 20, 4, 1e-3),
    ([("R", 30)] * 30 + [("X", 25)] * 8, 4, 1e-3),
    ([("R", 30)] * 30 + [("X", 25)] * 8, 8, 1e-3),
    ([("R", 30)] * 10 + [("X", 30)] * 18 + [("Y", 28)] * 14, 3, 1e-3),      # multi-allelic, re-genotyped
    ([("X", 30)] * 25 + [("Y", 2)] * 4, 4, 1e-3),                            # homozygous alternative
    ([("R", 30)] * 2 + [("X", 30)] * 20 + [("Y", 28)] * 16, 4, 1e-3),        # multi-allelic kept (1/2)
    ([("R", 30)] * 12 + [("X", 30)] * 10 + [("Y", 20)] * 6 + [("Z", 12)] * 5 + [("N", 30)] * 3, 10, 0.01),
    ([("R", 35)] * 40 + [("X", 30)] * 6 + [("Y", 3)] * 5, 13, 1e-3),
    ([("R", 30)] * 5 + [("X", 30)] * 25 + [("Y", 30)] * 3, 4, 1e-3),
    ([("R", 35)] * 40 + [("X", 30)] * 3, 13, 1e-3),                          # no call
]


@pytest.mark.parametrize("k", range(len(MIXTURES)))
def test_pool_single_site_known_answer(tmp_path, k):
    mixture, P, h = MIXTURES[k]
    rng = random.Random(k)
    fa, sam, ref, calls = write_site(str(tmp_path), [], k)
    others = [b for b in BASES if b != ref]
    rng.shuffle(others)
    sub = {"R": ref, "X": others[0], "Y": others[1], "Z": others[2], "N": "N"}
    fa, sam, ref, calls = write_site(str(tmp_path), [(sub[a], q) for a, q in mixture], k)
    out = os.path.join(str(tmp_path), "o.vcf")
    ngsep_oracle.run_ssvd(fa, sam, out, ploidy=P, het_rate=h, het_rate_set=1)
    got = [l.rstrip("\n") for l in open(out) if not l.startswith("#")]
    exp = expected_line("c1", 100, ref, calls, P, h)
    assert got == ([exp] if exp else [])
    assert (exp is None) == (k == len(MIXTURES) - 1)
