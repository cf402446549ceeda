"""An independent pure-Python restatement of the reference's indel path, read from the Java (not from
ngsepcore_amd/csrc/realign.cpp nor oracle/ngsep_oracle_indel.inc): test infrastructure for
tests/test_oracle_indel_kat.py, which checks the C oracle's indel functions against it.

  CountsHelper.calculateCountsIndel / updateCountsIndel / calculateLogCond   discovery/CountsHelper.java:96-105,253-304,384-396
  CountsHelper caches (alleleFreqCache, logProbCacheGT, logProbCacheError)  discovery/CountsHelper.java:135-187
  CountsHelper.updateCounts (SNV counts of the clustering's het posteriors)  discovery/CountsHelper.java:209-251
  CountsHelper.getPosteriorProbabilities / calculatePosteriorProbabilities  discovery/CountsHelper.java:410-443,472-495
  LogMath.logSum                                                             math/LogMath.java:38-44
  VariantDiscoverySNVQAlgorithm.callIndel / getIndexesMaxGenotype            discovery/VariantDiscoverySNVQAlgorithm.java:223-361
  AlleleCallClustersBuilder.clusterAlleleCalls and helpers                  discovery/AlleleCallClustersBuilder.java:72-261
  HammingSequenceDistanceMeasure.makeHammingConsensus                        sequences/HammingSequenceDistanceMeasure.java:88-101
  CountsRankHelper.selectBest                                                math/CountsRankHelper.java:31-51
  CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts / makeUndecided variants/CalledGenomicVariantImpl.java:228-325
  SingleSampleVariantPileupListener.genotypeVariantSample (indel, ploidy<3)  discovery/SingleSampleVariantPileupListener.java:361-391
  VCFFileWriter.printGenotypeInfo (GT, PL, GQ, DP, ADP, ACN)                  vcf/VCFFileWriter.java:159-256
  ReadAlignment.moveIndelStart / realignStart / realignEnd                   alignments/ReadAlignment.java:1114-1153,1372-1469

Java semantics kept: Math.round (floor(x + 0.5)), (byte) casts of quality scores, int division, stable
Collections.sort over TreeMap order (CountsRankHelper), TreeSet string order (Python str order = Java
String.compareTo for ASCII)."""
from __future__ import annotations

import math

NUM_FREQ = 501                      # DEF_NUM_FREQUENCIES
MIN_BASE_QS = 3                     # DEF_MIN_BASE_QS
MAX_BASE_QS = 30                    # DEF_MAX_BASE_QS
LOG_ERR_INDEL = math.log10(0.0001)  # DEF_LOG_ERROR_PROB_INDEL
BASES = "ACGT"


def jround(x: float) -> int:
    return int(math.floor(x + 0.5))


def to_byte(v: int) -> int:
    v &= 0xFF
    return v - 256 if v > 127 else v


def phred(p: float) -> int:        # PhredScoreHelper.calculatePhredScore
    if p == 0:
        return 255
    s = -10 * math.log10(p)
    if s > 255:
        return 255
    return to_short(jround(s))


def to_short(v: int) -> int:
    v &= 0xFFFF
    return v - 65536 if v > 32767 else v


def prob(q: int) -> float:         # PhredScoreHelper.calculateProbability
    return 0.0 if q >= 255 else 10 ** (-0.1 * q)


# ---- the caches: m = DEF_MAX_BASE_QS + 1 quality rows (an index past them is Java's
# ArrayIndexOutOfBoundsException) ----
def cache_error(q: int, j: int) -> float:
    if q > MAX_BASE_QS:
        raise IndexError("logProbCacheError has 31 rows")
    e0 = -0.1 * q
    return e0 if j == 0 else e0 - math.log10(j - 1)


def cache_gt(f: int, q: int, j: int) -> float:
    if q > MAX_BASE_QS:
        raise IndexError("logProbCacheGT has 31 quality rows")
    af = f / (NUM_FREQ - 1)
    e = prob(q)
    s = 1 - e
    if j == 0:
        return math.log10(s)
    return math.log10(af * s + (1 - af) * e / (j - 1))


def allele_freq(f: int):
    af = f / (NUM_FREQ - 1)
    return math.log10(af), math.log10(1 - af)


def log_sum(a: float, b: float) -> float:
    if a - b > 20:
        return a
    if b - a > 20:
        return b
    return a + math.log10(1 + math.pow(10.0, b - a))


class Helper:
    """CountsHelper over a list of alleles (counts, strand counts omitted, log-conditionals n x n)."""

    def __init__(self, alleles, max_base_qs=MAX_BASE_QS, het_prop=0.5):
        self.alleles = list(alleles)
        n = len(alleles)
        self.counts = [0] * n
        self.L = [[0.0] * n for _ in range(n)]
        self.total = 0
        self.max_bqs = to_byte(max_base_qs) if to_byte(max_base_qs) > 0 else MAX_BASE_QS   # setMaxBaseQS if > 0
        self.het = het_prop

    # calculateLogCond (:384-396)
    def log_cond(self, allele: str, call: str, quals: str) -> float:
        lc = 0.0
        for i in range(len(allele)):
            q = to_byte(min(self.max_bqs, ord(quals[i]) - 33))
            if q < MIN_BASE_QS:
                continue
            lc += cache_gt(0, q, 0) if allele[i] == call[i] else cache_error(q, 4)
        return lc

    # updateCountsIndel (:253-304)
    def update_indel(self, call: str, quals: str):
        self.total += 1
        index = self.alleles.index(call) if call in self.alleles else -1
        f = jround(self.het * NUM_FREQ)
        n = len(self.alleles)
        lca = [0.0] * n
        best = -1
        for i, a in enumerate(self.alleles):
            if len(a) == len(call):
                lca[i] = max(LOG_ERR_INDEL, self.log_cond(a, call, quals))
                if lca[i] > LOG_ERR_INDEL and (best == -1 or lca[best] < lca[i]):
                    best = i
            else:
                lca[i] = LOG_ERR_INDEL
        if index >= 0 and best >= 0 and best != index:
            index = min(index, best)
        elif index < 0 and best >= 0:
            index = best
        if index >= 0:
            self.counts[index] += 1
        f0, f1 = allele_freq(f)
        for i in range(n):
            self.L[i][i] += lca[i]
            for j in range(n):
                if i == j:
                    continue
                if j == index:
                    self.L[i][j] += log_sum(f0 + lca[index], f1 + LOG_ERR_INDEL)
                elif i == index:
                    self.L[i][j] += log_sum(f1 + lca[index], f0 + LOG_ERR_INDEL)
                else:
                    self.L[i][j] += LOG_ERR_INDEL

    # updateCounts (:209-251), negative strand ignored
    def update_snv(self, allele: str, q: int):
        self.total += 1
        n = len(self.alleles)
        f = jround(self.het * (NUM_FREQ - 1))
        g = jround((1 - self.het) * (NUM_FREQ - 1))
        q = to_byte(q)
        if q <= MIN_BASE_QS:
            return
        if q > self.max_bqs:
            q = self.max_bqs
        if allele not in self.alleles:
            return
        idx = self.alleles.index(allele)
        self.counts[idx] += 1
        for i in range(n):
            self.L[i][i] += cache_gt(f, q, 0) if i == idx else cache_error(q, n)
            for j in range(n):
                if i != j:
                    if j == idx:
                        self.L[i][j] += cache_gt(f, q, n)
                    elif i == idx:
                        self.L[i][j] += cache_gt(g, q, n)
                    else:
                        self.L[i][j] += cache_error(q, n)

    # getPosteriorProbabilities (:410-443) + calculatePosteriorProbabilities (:472-495)
    def posteriors(self, het_rate: float):
        n = len(self.alleles)
        hetero = n * (n - 1)
        lph = math.log10(het_rate / hetero) if hetero else 0.0
        lpo = math.log10((1 - het_rate) / n)
        ev = []
        for i in range(n):
            ev.append(self.L[i][i] + lpo)
            for j in range(n):
                if i != j:
                    ev.append(self.L[i][j] + lph)
        log_max = 1.0
        for x in ev:
            if log_max > 0 or log_max < x:
                log_max = x
        tot = 0.0
        for k in range(len(ev)):
            ev[k] -= log_max
            ev[k] = 0.0 if ev[k] < -20 else math.pow(10.0, ev[k])
            tot += ev[k]
        ev = [x / tot for x in ev]
        post = [[0.0] * n for _ in range(n)]
        k = 0
        for i in range(n):
            post[i][i] = ev[k]
            k += 1
            for j in range(n):
                if i != j:
                    post[i][j] = ev[k]
                    k += 1
        return post


def indel_helper(alleles, calls, max_base_qs=MAX_BASE_QS):
    """calculateCountsIndel(alleles, calls, maxBaseQS, 0.5); calls = [(allele, quals)]"""
    h = Helper(alleles, max_base_qs, 0.5)
    for a, q in calls:
        h.update_indel(a, q)
    return h


def max_genotype(post, default=0):
    """getIndexesMaxGenotype (VariantDiscoverySNVQAlgorithm.java:223-243)"""
    n = len(post)
    if default < 0 or default >= n:
        default = 0
    idx = [default, default]
    pmax = post[default][default]
    for i in range(n):
        for j in range(i, n):
            g = post[i][j] + (post[j][i] if i != j else 0.0)
            if g > pmax + 0.01:
                pmax = g
                idx = [i, j]
    return idx


# ---- CalledGenomicVariantImpl ----
class Called:
    def __init__(self, n_alleles, called, total_cn=2):
        self.n = n_alleles
        self.called = list(called)
        self.gq = 0
        self.dp = 0
        self.report = None           # (counts, logs) over the variant's alleles
        self.total_cn = max(len(called), total_cn)   # setIndexesCalledAlleles: max(#called, getCopyNumber())
        self.acn = [0] * n_alleles
        self.update_cn(self.total_cn)

    def undecided(self):
        return len(self.called) == 0

    def homref(self):
        return len(self.called) == 1 and self.called[0] == 0

    # updateAllelesCopyNumberFromCounts (:228-282)
    def update_cn(self, total):
        self.total_cn = total
        self.acn = [0] * self.n
        if self.undecided():
            return
        if self.homref():
            self.acn[0] = total
            return
        nc = len(self.called)
        if total <= nc:
            for c in self.called:
                self.acn[c] = 1
            return
        if self.report is None:
            d = total // nc
            for c in self.called:
                self.acn[c] = d
            self.acn[self.called[0]] += total - d * nc
            return
        rc = [self.report[0][c] or 1 for c in self.called]
        tr = sum(rc)
        tc = 0
        for i, c in enumerate(self.called):
            self.acn[c] = max(1, to_short(jround(total * rc[i] / tr)))
            tc += self.acn[c]
        if tc < total:
            self.acn[self.called[0]] += total - tc
        else:
            ex = tc - total
            for c in reversed(self.called):
                if ex <= 0:
                    break
                rm = min(ex, self.acn[c] - 1)
                self.acn[c] -= rm
                ex -= rm

    def make_undecided(self):            # makeUndecided (:320-325)
        self.called = []
        self.gq = 0
        self.update_cn(self.total_cn)


def call_indel(alleles, h: Helper, het_rate, is_str, is_input_str, variant=None):
    """callIndel (VariantDiscoverySNVQAlgorithm.java:265-361).  variant=None: (variant alleles, type, qs, call) or
    None; variant given (its alleles = h.alleles): the Called over them"""
    counts = h.counts
    post = h.posteriors(het_rate)
    if h.total == 0:
        if variant is None:
            return None
        return Called(len(alleles), [])
    im = max_genotype(post, 0)
    if variant is None:
        hal = h.alleles
        al = [hal[0]]
        idx = [0]
        change = False
        if 0 < im[0] < len(hal):
            al.append(hal[im[0]])
            idx.append(im[0])
            change = change or len(hal[im[0]]) != len(hal[0])
        if im[1] > 0 and im[1] != im[0] and im[1] < len(hal):
            al.append(hal[im[1]])
            idx.append(im[1])
            change = change or len(hal[im[1]]) != len(hal[0])
            if len(al) == 3 and len(hal[im[1]]) != len(al[1]):
                change = True
        if not change and not is_input_str:
            return None
        qs = phred(post[0][0])
        report = ([counts[i] for i in idx], [[h.L[i][j] for j in idx] for i in idx])
        if im[1] != im[0]:
            called = [1, 2] if len(al) == 3 else [0, 1]
        else:
            called = [0] if im[0] == 0 else [1]
        c = Called(len(al), called)
    else:
        al = list(alleles)
        qs = None
        report = (list(counts), [row[:] for row in h.L])
        if im[0] > 100 or im[1] > 100:
            called = []
        elif im[1] != im[0]:
            called = [im[0], im[1]]
        else:
            called = [im[0]]
        c = Called(len(al), called)
    pmax = post[im[0]][im[1]] + (post[im[1]][im[0]] if im[0] != im[1] else 0.0)
    c.gq = phred(1 - pmax)
    c.dp = h.total
    c.report = report
    return (al, "STR" if is_str else "INDEL", qs, c)


def genotype_fields(c: Called, ploidy: int) -> str:
    """printGenotypeInfo (VCFFileWriter.java:159-256) for FORMAT GT:PL:GQ:DP:ADP:ACN"""
    if not c.called:
        gt = "./." if ploidy > 1 else "."
    elif len(c.called) == 1:
        gt = str(c.called[0]) + (f"/{c.called[0]}" if ploidy > 1 else "")
    else:
        gt = f"{c.called[0]}/{c.called[1]}"
    pl = []
    for j in range(c.n):
        for i in range(j + 1):
            pl.append(str(jround(-10 * c.report[1][i][j])) if c.report else "0")
    adp = ",".join(str(c.report[0][i]) if c.report else "0" for i in range(c.n))
    if c.total_cn == 0:
        acn = "."
    else:
        v = list(c.acn)
        if c.undecided():
            v[0] = c.total_cn
        acn = ",".join(str(x) for x in v)
    return f"{gt}:{','.join(pl)}:{c.gq}:{c.dp}:{adp}:{acn}"


def single_sample_indel(alleles, calls, het_rate, is_str, is_input_str, min_quality, ploidy, max_base_qs=MAX_BASE_QS):
    """discoverIndel at ploidy < 3 + discoverVariant's filters (SingleSampleVariantPileupListener.java:213-232,
    257-296) + updateAllelesCopyNumberFromCounts(ploidy): "REF\\tALT\\tQS\\tTYPE\\tGT:..." or None"""
    h = indel_helper(alleles, calls, max_base_qs)
    r = call_indel(alleles, h, het_rate, is_str, is_input_str)
    if r is None:
        return None
    al, typ, qs, c = r
    if c.undecided() or c.homref() or min_quality > c.gq:
        return None
    c.update_cn(ploidy)
    return f"{al[0]}\t{','.join(al[1:])}\t{qs}\t{typ}\t{genotype_fields(c, ploidy)}"


def population_sample_indel(alleles, calls, het_rate, ploidy, max_base_qs=MAX_BASE_QS):
    """genotypeVariantSample for an indel variant at ploidy < 3 with a fresh listener (minQuality 40)"""
    h = indel_helper(alleles, calls, max_base_qs)
    c = call_indel(alleles, h, het_rate, False, False, variant=alleles)
    if isinstance(c, tuple):
        c = c[3]
    c.update_cn(ploidy)
    if 40 > c.gq:
        c.make_undecided()
    return genotype_fields(c, ploidy)


def _normalize(ev):
    """CountsHelper.calculatePosteriorProbabilities (:472-495) on a list"""
    log_max = 1.0
    for x in ev:
        if log_max > 0 or log_max < x:
            log_max = x
    out = [0.0 if x - log_max < -20 else math.pow(10.0, x - log_max) for x in ev]
    tot = sum(out)
    return [x / tot for x in out]


def _first_max(v):
    """NumberArrays.getIndexMaximum: the first maximum"""
    k = 0
    for i in range(1, len(v)):
        if v[k] < v[i]:
            k = i
    return k


def pool_genotype_indel(alleles, calls, haplotypes, het_rate, max_base_qs=MAX_BASE_QS):
    """genotypeVariantPool (SingleSampleVariantPileupListener.java:402-503) over an indel variant: the Called, with the
    copy numbers setAllelesCopyNumber leaves (:480-498)"""
    n = len(alleles)
    step = 1.0 / haplotypes
    freqs, helpers = [], []
    freq = step
    while freq < 0.51:
        freqs.append(freq)
        hp = Helper(alleles, max_base_qs, freq)
        for a, q in calls:
            hp.update_indel(a, q)
        helpers.append(hp)
        freq += step
    helper = helpers[0]
    counts = helper.counts
    major = _first_max(counts)
    if counts[major] < haplotypes:
        c = Called(n, [], total_cn=0)            # new CalledGenomicVariantImpl(variant, new byte[0])
        c.update_cn(haplotypes)
        return c
    lph, lpo = math.log10(het_rate), math.log10(1 - het_rate)
    term_hom = helper.L[major][major] + lpo
    max_het, min_hom, max_freq_idx, max_freq, max_alt = 0.0, 1.0, 0, 0.0, -1
    for i in range(n):
        if i == major:
            continue
        terms = _normalize([term_hom] + [helpers[j].L[major][i] + lph for j in range(len(freqs))])
        k = _first_max(terms)
        if k == 0:
            min_hom = min(min_hom, terms[0])
        elif max_alt == -1 or max_het < terms[k]:
            max_het, max_freq_idx, max_freq, max_alt = terms[k], k - 1, freqs[k - 1], i
    called = sorted([major] + ([max_alt] if max_alt != -1 else []))
    c = Called(n, called, total_cn=0)
    c.dp = helper.total
    acn = [0] * n
    if max_alt == -1:
        c.gq = phred(1 - min_hom)
        acn[major] = haplotypes
    else:
        helper = helpers[max_freq_idx]
        # CountsHelper.getPosteriorProbabilities(h, idxMajorAllele) (CountsHelper.java:451-467)
        ev = _normalize([helper.L[major][j] + (lpo if j == major else math.log10(het_rate / (n - 1))) for j in range(n)])
        c.gq = phred(1 - ev[max_alt])
        alt_cn = to_short(jround(max_freq * haplotypes))
        if alt_cn == 0:
            alt_cn += 1
        elif alt_cn == haplotypes:
            alt_cn -= 1
        acn[max_alt] = alt_cn
        acn[major] = haplotypes - alt_cn
    c.total_cn = sum(acn)                        # setAllelesCopyNumber
    c.acn = acn
    c.report = (list(counts), [row[:] for row in helper.L])
    return c


def pool_sample_indel(alleles, calls, het_rate, ploidy, min_quality=40, max_base_qs=MAX_BASE_QS):
    """genotypeVariantSample at ploidy >= 3 for an indel variant (:378-379, makeUndecided below min_quality :388)"""
    c = pool_genotype_indel(alleles, calls, ploidy, het_rate, max_base_qs)
    if min_quality > c.gq:
        c.make_undecided()
    return genotype_fields(c, ploidy)


# ---- AlleleCallClustersBuilder ----
def select_best(items, mx):
    """CountsRankHelper.selectBest: counts in TreeMap (key) order, stable sort by count descending"""
    counts = {}
    for it in items:
        counts[it] = counts.get(it, 0) + 1
    keys = sorted(counts)
    keys = sorted(keys, key=lambda k: -counts[k])     # Python's sort is stable, as Collections.sort
    return keys[:mx]


def hamming_consensus(seqs):
    return "".join(select_best([s[i] for s in seqs], 1)[0] for i in range(len(seqs[0])))


def het_posteriors(calls, consensus, max_bqs):
    ans = []
    for i, c in enumerate(consensus):
        if c not in BASES:
            ans.append(0.0)
            continue
        if all(a[i] == c for a, _ in calls):
            ans.append(0.0)
            continue
        h = Helper(BASES)                                 # new CountsHelper(): ACGT, DEF_MAX_BASE_QS, 0.5
        for a, q in calls:
            h.update_snv(a[i], to_byte(min(max_bqs, ord(q[i]) - 33)))
        post = h.posteriors(0.001)
        ic = BASES.index(c)
        best = 0.0
        for k in range(4):
            hp = post[ic][k] + post[k][ic]
            if k != ic and hp > best:
                best = hp
        ans.append(best)
    return ans


def split_alleles(calls, consensus, max_bqs):
    hp = het_posteriors(calls, consensus, max_bqs)
    sites = [i for i, v in enumerate(hp) if v >= 0.51]
    if not sites:
        return {consensus}
    haps = ["".join(a[k] for k in sites) for a, _ in calls]
    m = len(sites)
    max_haps = min(10, m // 2 + 1) if m > 3 else 2
    sel = select_best(haps, max_haps)
    out = set()
    for hap in sel:
        seqs = [a for (a, _), h in zip(calls, haps) if h == hap]
        if seqs:
            out.add(hamming_consensus(seqs))
    return out


def cluster_alleles(calls, reference, max_base_qs=MAX_BASE_QS):
    """clusterAlleleCalls (:72-141): calls = [(allele, quals)]; returns [reference] + the others in TreeSet order"""
    by_len = {}
    for a, q in calls:
        by_len.setdefault(len(a), []).append((a, q))
    if len(by_len) >= 3:                               # filterLengthClusters (:147-157)
        min_count = 0.2 * len(calls)
        by_len = {l: v for l, v in by_len.items() if min_count <= len(v)}
    allele_set = set()
    mbq = to_byte(max_base_qs)
    for l, cl in by_len.items():
        sugg = {reference} if l == len(reference) else set()
        if len(cl) < 5 * len(sugg):
            length_alleles = sugg
        else:
            cons = hamming_consensus([a for a, _ in cl])
            sugg.add(cons)
            if l < 4 or len(cl) < 10:
                length_alleles = sugg
            else:
                length_alleles = split_alleles(cl, cons, mbq)
        allele_set |= length_alleles
    allele_set.add(reference)
    return [reference] + [a for a in sorted(allele_set) if a != reference]


# ---- ReadAlignment edits over (first, last, alignment codes len * 8 + op) ----
OPS = "HDIMPNSX"                                       # ALIGNMENT_CHAR_CODES: H0 D1 I2 M3 P4 N5 S6 X7
M, D, I = 3, 1, 2


def parse_cigar(s):
    out, n = [], 0
    for ch in s:
        if ch.isdigit():
            n = n * 10 + int(ch)
        else:
            out.append(n * 8 + OPS.index(ch))
            n = 0
    return out


def cigar_text(codes):
    return "".join(f"{c // 8}{OPS[c & 7]}" for c in codes)


def move_indel_start(first, aln, indel_ref_pos, new_pos):
    """moveIndelStart (:1114-1153): (moved, new codes)"""
    disp = new_pos - indel_ref_pos
    if disp == 0:
        return True, list(aln)
    new = [0] * len(aln)
    nxt = -1
    cur = first
    for i, v in enumerate(aln):
        ln, op = v // 8, v & 7
        if op in (D, I) and cur == indel_ref_pos + 1:
            if i == 0 or i == len(aln) - 1:
                return False, list(aln)
            ob, lb = aln[i - 1] & 7, aln[i - 1] // 8
            if not (ob & 2) or not (ob & 1) or lb <= -disp:
                return False, list(aln)
            oa, la = aln[i + 1] & 7, aln[i + 1] // 8
            if not (oa & 2) or not (oa & 1) or la <= disp:
                return False, list(aln)
            new[i - 1] = (lb + disp) * 8 + ob
            new[i] = v
            new[i + 1] = (la - disp) * 8 + oa
            nxt = i + 1
        elif i != nxt:
            new[i] = v
        if v & 1:
            cur += ln
    if nxt < 0:
        return False, list(aln)
    return True, new


def realign_start(first, last, aln, new_first, first_match, ref_pos_after, read_pos_after):
    """realignStart (:1372-1418): (first, last, codes); `last` is left as it was"""
    out = [first_match * 8 + M]
    nref = new_first + first_match
    ur = read_pos_after - first_match
    uf = ref_pos_after - nref
    if uf < 0 or ur < 0:
        return first, last, list(aln)                  # "Can not realign start": unchanged
    d = ur - uf
    if d == 0:
        if ur > 0:
            out.append(ur * 8 + M)
    elif d > 0:
        out.append(d * 8 + I)
        if uf > 0:
            out.append(uf * 8 + M)
    else:
        out.append(-d * 8 + D)
        if ur > 0:
            out.append(ur * 8 + M)
    cur, copy = 0, False
    for v in aln:
        ln, op = v // 8, v & 7
        if copy:
            out.append(v)
        if v & 2:
            if not copy and read_pos_after < cur + ln:
                copy = True
                out.append((cur + ln - read_pos_after) * 8 + op)
            cur += ln
    return new_first, last, out


def realign_end(first, last, aln, read_length, ref_pos_before, aln_pos_before, final_start, final_len):
    """realignEnd (:1427-1469): (first, last, codes)"""
    bp_end = read_length - aln_pos_before - 1
    out, cur, copy = [], 0, True
    for v in aln:
        ln, op = v // 8, v & 7
        if v & 2:
            if copy and aln_pos_before < cur + ln:
                diff = cur + ln - aln_pos_before - 1
                out.append((ln - diff) * 8 + op)
                copy = False
            cur += ln
        if copy:
            out.append(v)
    uf = final_start - ref_pos_before - 1
    ur = bp_end - final_len
    if uf < 0 or ur < 0:
        return first, last, list(aln)                  # "Can not realign end": unchanged
    d = ur - uf
    if d == 0:
        if ur > 0:
            out.append(ur * 8 + M)
    elif d > 0:
        out.append(d * 8 + I)
        if uf > 0:
            out.append(uf * 8 + M)
    else:
        out.append(-d * 8 + D)
        if ur > 0:
            out.append(ur * 8 + M)
    out.append(final_len * 8 + M)
    return first, final_start + final_len - 1, out
