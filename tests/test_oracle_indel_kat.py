"""The oracle's indel functions (oracle/ngsep_oracle_indel.inc, ngsep_oracle.c) against an independent pure-Python
restatement of the Java (tests/indel_restatement.py) on seeded random and hand-made inputs: CountsHelper's indel
counts and log-conditionals, AlleleCallClustersBuilder.clusterAlleleCalls, callIndel (single-sample discovery and the
population genotype of a given variant) and ReadAlignment's moveIndelStart / realignStart / realignEnd.

The GPU path's indel records equal the oracle's (tests/test_gpu_indels.py, test_gpu_multisample.py); these checks pin
the oracle with a second reading of the Java, so the two C++/C twins cannot share a misreading unseen.  No reference
output holds indel calls: beyond this, indel parity stays unpinned against the reference itself."""
import ctypes
import random

import pytest

import indel_restatement as R
import ngsep_oracle

CP = ctypes.c_char_p


def _lib():
    l = ngsep_oracle.lib()
    if not getattr(l, "_indel_kat", False):
        l.ngo_t_indel_counts.restype = ctypes.c_int
        l.ngo_t_indel_counts.argtypes = [ctypes.c_int, ctypes.POINTER(CP), ctypes.c_int, ctypes.POINTER(CP), ctypes.POINTER(CP),
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double)]
        l.ngo_t_cluster.restype = ctypes.c_int
        l.ngo_t_cluster.argtypes = [CP, ctypes.c_int, ctypes.POINTER(CP), ctypes.POINTER(CP), ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        l.ngo_t_call_indel.restype = ctypes.c_int
        l.ngo_t_call_indel.argtypes = [ctypes.c_int, ctypes.POINTER(CP), ctypes.c_int, ctypes.POINTER(CP), ctypes.POINTER(CP),
                                       ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_char_p, ctypes.c_int]
        l.ngo_t_genotype_indel_sample.restype = None
        l.ngo_t_genotype_indel_sample.argtypes = [ctypes.c_int, ctypes.POINTER(CP), ctypes.c_int, ctypes.POINTER(CP),
                                                  ctypes.POINTER(CP), ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                                  ctypes.c_char_p, ctypes.c_int]
        l.ngo_t_genotype_indel_sample_q.restype = None
        l.ngo_t_genotype_indel_sample_q.argtypes = [ctypes.c_int, ctypes.POINTER(CP), ctypes.c_int, ctypes.POINTER(CP),
                                                    ctypes.POINTER(CP), ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                                    ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        l.ngo_t_edit.restype = ctypes.c_int
        l.ngo_t_edit.argtypes = [ctypes.c_int, CP, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        l._indel_kat = True
    return l


def _arr(strs):
    a = (CP * max(1, len(strs)))()
    for i, s in enumerate(strs):
        a[i] = s.encode()
    return a


def _quals(rnd, n, lo=0, hi=30):
    return "".join(chr(33 + rnd.randint(lo, hi)) for _ in range(n))


def _mutate(rnd, s, rate):
    return "".join(rnd.choice("ACGT") if rnd.random() < rate else c for c in s)


def _pileup(rnd, ref, n_calls, n_haps=2, err=0.03):
    """span calls of a few haplotypes (indels change the length) with substitution errors and random qualities"""
    haps = [ref]
    for _ in range(n_haps - 1):
        k = rnd.randrange(1, len(ref))
        if rnd.random() < 0.5:
            haps.append(ref[:k] + "".join(rnd.choice("ACGT") for _ in range(rnd.randint(1, 6))) + ref[k:])
        else:
            haps.append(ref[:k] + ref[k + min(len(ref) - k - 1, rnd.randint(1, 4)):])
    calls = []
    for _ in range(n_calls):
        h = rnd.choice(haps)
        calls.append((_mutate(rnd, h, err), _quals(rnd, len(h), 2, 30)))
    return calls


@pytest.mark.parametrize("seed", range(40))
def test_indel_counts(seed):
    """calculateCountsIndel: counts exactly, log-conditionals to the last bits (same operation order)"""
    rnd = random.Random(1000 + seed)
    ref = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(2, 12)))
    calls = _pileup(rnd, ref, rnd.randint(1, 40), rnd.randint(1, 3), 0.05)
    alleles = R.cluster_alleles(calls, ref)
    alleles += [a for a in {c for c, _ in calls[:3]} if a not in alleles]   # calls matching no allele exactly
    mbq = rnd.choice([30, 20, 12, 0])
    h = R.indel_helper(alleles, calls, mbq)
    n = len(alleles)
    counts = (ctypes.c_int * n)()
    logc = (ctypes.c_double * (n * n))()
    t = _lib().ngo_t_indel_counts(n, _arr(alleles), len(calls), _arr([c for c, _ in calls]), _arr([q for _, q in calls]),
                                  mbq, counts, logc)
    assert t == h.total == len(calls)
    assert list(counts) == h.counts
    for i in range(n):
        for j in range(n):
            assert logc[i * n + j] == pytest.approx(h.L[i][j], rel=1e-13, abs=1e-13)


@pytest.mark.parametrize("seed", range(60))
def test_cluster_alleles(seed):
    """clusterAlleleCalls: the length clusters, their filter, consensus and the split of a long cluster at its
    heterozygous sites (het posteriors, haplotypes, CountsRankHelper order), the TreeSet order"""
    rnd = random.Random(2000 + seed)
    ref = "".join(rnd.choice("ACGT") for _ in range(rnd.choice([2, 3, 5, 8, 14])))
    calls = _pileup(rnd, ref, rnd.choice([3, 6, 9, 12, 25, 40]), rnd.randint(1, 4), rnd.choice([0.0, 0.02, 0.1]))
    if seed % 5 == 0:      # two same-length haplotypes of a long allele: the split at variant sites
        alt = _mutate(rnd, ref, 0.3)
        calls = [(rnd.choice([ref, alt]), _quals(rnd, len(ref), 20, 30)) for _ in range(30)]
    mbq = rnd.choice([30, 25])
    want = R.cluster_alleles(calls, ref, mbq)
    buf = ctypes.create_string_buffer(1 << 16)
    n = _lib().ngo_t_cluster(ref.encode(), len(calls), _arr([c for c, _ in calls]), _arr([q for _, q in calls]), mbq, buf, 1 << 16)
    got = buf.value.decode().split(",")
    assert n == len(want)
    assert got == want


def test_cluster_split_kat():
    """A hand-made long cluster: 12 calls of the reference's length from two haplotypes differing at 2 sites (Q30):
    split at the variant sites, both haplotypes are alleles; 6 calls (>= 5 x 1 suggested allele, < 10): the suggested
    reference and the consensus; 4 calls (< 5): the suggested reference alone"""
    ref = "ACGTACGTAC"
    h2 = "ACCTACGTTC"
    q = "?" * 10
    calls = [(ref, q)] * 6 + [(h2, q)] * 6
    assert R.cluster_alleles(calls, ref) == [ref, h2]
    calls6 = [(ref, q)] + [(h2, q)] * 5
    assert R.cluster_alleles(calls6, ref) == [ref, h2]       # consensus h2 (majority) + the suggested reference
    calls4 = [(ref, q), (h2, q), (h2, q), (h2, q)]
    assert R.cluster_alleles(calls4, ref) == [ref]
    buf = ctypes.create_string_buffer(4096)
    for cl in (calls, calls6, calls4):
        _lib().ngo_t_cluster(ref.encode(), len(cl), _arr([c for c, _ in cl]), _arr([x for _, x in cl]), 30, buf, 4096)
        assert buf.value.decode().split(",") == R.cluster_alleles(cl, ref)


@pytest.mark.parametrize("seed", range(60))
def test_call_indel(seed):
    """callIndel with variant == null + the listener's filters and copy numbers: the record's fields"""
    rnd = random.Random(3000 + seed)
    ref = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(2, 10)))
    calls = _pileup(rnd, ref, rnd.randint(1, 45), rnd.randint(1, 3), rnd.choice([0.0, 0.02]))
    alleles = R.cluster_alleles(calls, ref)
    het = rnd.choice([0.001, 0.01, 1e-6])
    is_str = rnd.random() < 0.3
    is_input = is_str and rnd.random() < 0.5
    minq = rnd.choice([40, 10, 0])
    ploidy = rnd.choice([2, 1])
    want = R.single_sample_indel(alleles, calls, het, is_str, is_input, minq, ploidy)
    buf = ctypes.create_string_buffer(1 << 16)
    ok = _lib().ngo_t_call_indel(len(alleles), _arr(alleles), len(calls), _arr([c for c, _ in calls]),
                                 _arr([q for _, q in calls]), 30, het, int(is_str), int(is_input), minq, ploidy, buf, 1 << 16)
    if want is None:
        assert ok == 0
        return
    assert ok == 1
    f = buf.value.decode().rstrip("\n").split("\t")
    got = f"{f[3]}\t{f[4]}\t{f[5]}\t{f[7].split('=')[1]}\t{f[9]}"
    assert got == want


def test_call_indel_kat():
    """Closed form: 10 calls of an insertion allele at Q30 against a 2-bp reference -- homozygous alternative,
    PL(ref/ref) = round(-10 * 10 * log10(1e-4)) = 400, PL(alt/alt) = 0"""
    ref, alt = "AC", "AGGC"
    calls = [(alt, "????")] * 10
    want = R.single_sample_indel([ref, alt], calls, 0.001, False, False, 40, 2)
    assert want.startswith("AC\tAGGC\t")
    fields = want.split("\t")[4].split(":")
    assert fields[0] == "1/1"
    pl = [int(x) for x in fields[1].split(",")]
    assert pl[0] == 400 and pl[2] == 0
    buf = ctypes.create_string_buffer(4096)
    assert _lib().ngo_t_call_indel(2, _arr([ref, alt]), 10, _arr([alt] * 10), _arr(["????"] * 10), 30, 0.001, 0, 0, 40, 2, buf, 4096)
    f = buf.value.decode().split("\t")
    assert f"{f[3]}\t{f[4]}\t{f[5]}\tINDEL\t{f[9].strip()}" == want


@pytest.mark.parametrize("seed", range(40))
def test_population_sample_indel(seed):
    """genotypeVariantSample over a given indel variant (MultisampleVariantsDetector.genotypeVariant's per-sample call):
    callIndel with the variant, copy numbers, makeUndecided below 40"""
    rnd = random.Random(4000 + seed)
    ref = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(2, 8)))
    calls = _pileup(rnd, ref, rnd.randint(0, 15), rnd.randint(1, 3), 0.02)
    alleles = R.cluster_alleles(_pileup(rnd, ref, 30, 3, 0.0), ref)
    het = rnd.choice([0.001, 0.01])
    ploidy = rnd.choice([2, 1])
    want = R.population_sample_indel(alleles, calls, het, ploidy)
    buf = ctypes.create_string_buffer(1 << 16)
    _lib().ngo_t_genotype_indel_sample(len(alleles), _arr(alleles), len(calls), _arr([c for c, _ in calls]),
                                       _arr([q for _, q in calls]), 30, het, ploidy, buf, 1 << 16)
    assert buf.value.decode() == want


def _edit(op, cigar, first, *a):
    buf = ctypes.create_string_buffer(1024)
    f, l = ctypes.c_int(), ctypes.c_int()
    args = list(a) + [0] * (4 - len(a))
    r = _lib().ngo_t_edit(op, cigar.encode(), first, *args, buf, 1024, ctypes.byref(f), ctypes.byref(l))
    return r, buf.value.decode(), f.value, l.value


def _random_cigar(rnd):
    items = [(rnd.randint(3, 40), "M")]
    for _ in range(rnd.randint(0, 3)):
        items.append((rnd.randint(1, 8), rnd.choice("ID")))
        items.append((rnd.randint(3, 40), "M"))
    if rnd.random() < 0.2:
        items.insert(0, (rnd.randint(1, 10), "S"))
    return "".join(f"{n}{o}" for n, o in items)


@pytest.mark.parametrize("seed", range(80))
def test_alignment_edits(seed):
    """moveIndelStart, realignStart and realignEnd on random alignments and arguments (including the refused moves and
    the 'can not realign' early returns): the new CIGAR, first and last"""
    rnd = random.Random(5000 + seed)
    cig = _random_cigar(rnd)
    first = rnd.randint(100, 1000)
    aln = R.parse_cigar(cig)
    span = sum(v // 8 for v in aln if v & 1)
    rlen = sum(v // 8 for v in aln if v & 2)
    last = first + span - 1
    # moveIndelStart at an event's key (the reference position before it) or anywhere
    keys, cur = [], first
    for v in aln:
        if (v & 7) in (1, 2):
            keys.append(cur - 1)
        if v & 1:
            cur += v // 8
    ip = rnd.choice(keys) if keys and rnd.random() < 0.8 else rnd.randint(first, last)
    np_ = ip + rnd.randint(-6, 6)
    ok, new = R.move_indel_start(first, aln, ip, np_)
    r, c, f, l = _edit(0, cig, first, ip, np_)
    assert (r == 1) == ok
    assert c == R.cigar_text(new) and f == first
    # realignStart(newAlnFirst, firstMatchLength, refPosAfter, alnReadPosAfter)
    fm = rnd.randint(1, 12)
    nf = first + rnd.randint(-8, 8)
    rpa = rnd.randint(first, last)
    apa = rnd.randint(fm, max(fm, rlen - 1))
    nf2, nl2, new = R.realign_start(first, last, aln, nf, fm, rpa, apa)
    r, c, f, l = _edit(1, cig, first, nf, fm, rpa, apa)
    assert (c, f, l) == (R.cigar_text(new), nf2, nl2)
    # realignEnd(refPosBefore, alnPosBefore, finalMatchRefStart, finalMatchLength)
    apb = rnd.randint(0, rlen - 2)
    fl = rnd.randint(1, max(1, rlen - apb - 1))
    rpb = rnd.randint(first, last)
    fms = rpb + rnd.randint(-3, 12)
    nf3, nl3, new = R.realign_end(first, last, aln, rlen, rpb, apb, fms, fl)
    r, c, f, l = _edit(2, cig, first, rpb, apb, fms, fl)
    assert (c, f, l) == (R.cigar_text(new), nf3, nl3)


def test_alignment_edit_kats():
    """Hand-made: a 2-bp deletion moved 3 bp left; a realigned start that becomes an insertion; a refused move past
    the preceding match"""
    assert R.move_indel_start(101, R.parse_cigar("20M2D30M"), 120, 117) == (True, R.parse_cigar("17M2D33M"))
    assert _edit(0, "20M2D30M", 101, 120, 117)[:2] == (1, "17M2D33M")
    assert R.move_indel_start(101, R.parse_cigar("20M2D30M"), 120, 99)[0] is False
    assert _edit(0, "20M2D30M", 101, 120, 99)[0] == 0
    # realignStart(newAlnFirst=103, firstMatchLength=5, refPosAfter=110, alnReadPosAfter=12): 7 read bp over 2 ref bp
    f, l, new = R.realign_start(101, 150, R.parse_cigar("50M"), 103, 5, 110, 12)
    assert (f, R.cigar_text(new)) == (103, "5M5I2M38M")
    assert _edit(1, "50M", 101, 103, 5, 110, 12)[1:3] == ("5M5I2M38M", 103)


@pytest.mark.parametrize("seed", range(40))
def test_pool_sample_indel(seed):
    """genotypeVariantPool over an indel variant (ploidy >= 3: SingleSampleVariantPileupListener.java:378-379, 402-503)
    and the given-variant callIndel at ploidy < 3 with -minQuality: the oracle's sample call against the restatement's
    (undecided below `ploidy` calls of the major allele, heterozygous at the best frequency hypothesis, the copy numbers
    setAllelesCopyNumber leaves, makeUndecided below min_quality)."""
    rnd = random.Random(9000 + seed)
    ref = "".join(rnd.choice("ACGT") for _ in range(rnd.randint(3, 9)))
    calls = _pileup(rnd, ref, rnd.choice([0, 2, 5, 12, 30, 60]), n_haps=rnd.choice([1, 2, 3]))
    alleles = R.cluster_alleles(calls, ref)
    if len(alleles) < 2:
        alleles = [ref, ref + "A"]
    ploidy = rnd.choice([1, 2, 3, 4, 6, 8])
    het = rnd.choice([0.001, 0.01, 0.1])
    minq = rnd.choice([0, 20, 40])
    out = ctypes.create_string_buffer(8192)
    _lib().ngo_t_genotype_indel_sample_q(len(alleles), _arr(alleles), len(calls), _arr([c for c, _ in calls]),
                                        _arr([q for _, q in calls]), 30, het, ploidy, minq, out, 8192)
    if ploidy >= 3:
        want = R.pool_sample_indel(alleles, calls, het, ploidy, minq)
    else:
        h = R.indel_helper(alleles, calls)
        c = R.call_indel(alleles, h, het, False, False, variant=alleles)
        if isinstance(c, tuple):
            c = c[3]
        c.update_cn(ploidy)
        if minq > c.gq:
            c.make_undecided()
        want = R.genotype_fields(c, ploidy)
    assert out.value.decode() == want
