"""The oracle (CPU restatement) against the reference's own test inputs and closed-form answers.

CountsHelperTest (test/ngsep/discovery/test/CountsHelperTest.java:12-87) feeds 990 'A' and 10 'C'
calls with quality char 'A' (Q32, capped to 30) for heterozygous proportions 0.01/0.25/0.5 and
prints logConditionalProbs; it has no asserts, so the expected values are the ones derived
analytically in SURVEY.md section 4 from CountsHelper.java:135-251.
"""
import math

import pytest

import ngsep_oracle as O

KAT = {  # het proportion -> ([0][0], [0][1], [1][0])
    0.01: (-30.43016665627752, -24.340953333429084, -1939.8516325470448),
    0.25: (-30.43016665627752, -129.988001885514, -596.4326307269221),
    0.5: (-30.43016665627752, -301.029995663977, -301.029995663977),
}


@pytest.mark.parametrize("hp", sorted(KAT))
def test_counts_helper_test_vectors(hp):
    c = O.Counts(2, hp, 30)
    q = min(30, ord("A") - 33)
    for i in range(1000):
        c.update(0 if i < 990 else 1, q)
    got = (c.logc(0, 0), c.logc(0, 1), c.logc(1, 0))
    for g, e in zip(got, KAT[hp]):
        assert g == pytest.approx(e, rel=1e-15, abs=1e-12)
    assert c.c.total_count == 1000 and c.c.counts[0] == 990 and c.c.counts[1] == 10


def test_bins_f_g():
    """CountsHelper.java:212-213: f=round(h*500), g=round((1-h)*500)."""
    for hp, f, g in ((0.01, 5, 495), (0.25, 125, 375), (0.5, 250, 250)):
        c = O.Counts(2, hp)
        assert (c.c.f, c.c.g) == (f, g)


def test_closed_form_all_q30_reference():
    """n reads, all Q30, all the reference allele A (4-allele SNV model, f=g=250):
    [A][A] = n*log10(1-1e-3), [A][x] = n*log10(0.5*(1-e)+0.5*e/3), [x][x] = n*(-3-log10 3)."""
    n = 17
    c = O.Counts(4, 0.5, 30)
    for _ in range(n):
        c.update(0, 30)
    e = 10 ** -3
    assert c.logc(0, 0) == pytest.approx(n * math.log10(1 - e), rel=1e-12)
    assert c.logc(0, 1) == pytest.approx(n * math.log10(0.5 * (1 - e) + 0.5 * e / 3), rel=1e-12)
    assert c.logc(2, 2) == pytest.approx(n * (-3 - math.log10(3)), rel=1e-12)
    assert c.logc(1, 3) == c.logc(2, 2)
    # PL of a hom-ref call would be [0, round(3.0132 n), round(34.771 n)] in phred units
    assert round(-10 * c.logc(0, 1) + 10 * c.logc(0, 0)) == round(3.0132 * n)


def test_low_quality_and_cap():
    c = O.Counts(4, 0.5, 20)
    c.update(0, 3)      # q <= 3: counted in total only (CountsHelper.java:214-216)
    c.update(-1, 25)    # N: total only
    c.update(1, 30)     # capped to maxBaseQS 20
    assert c.c.total_count == 3 and c.c.low_bq_count == 1 and c.c.counts[1] == 1
    assert c.logc(1, 1) == O.lib().ngo_table_gt(250, 20, 0)


def test_phred_and_java_round():
    lib = O.lib()
    assert lib.ngo_phred(0.0) == 255
    assert lib.ngo_phred(1.0) == 0
    assert lib.ngo_phred(1e-30) == 255
    assert lib.ngo_phred(-1e-17) == 0          # log10 of a negative is NaN -> Math.round -> 0
    assert lib.ngo_phred(10 ** -4.05) == 41    # 40.5 rounds up (ties toward +inf)
    assert lib.ngo_java_round(-2.5) == -2 and lib.ngo_java_round(2.5) == 3
    assert lib.ngo_java_round(0.49999999999999994) == 0


def test_posterior_homref():
    """A clean hom-ref pileup: P(ref/ref) dominates (VariantDiscoverySNVQAlgorithm.java:223-243)."""
    c = O.Counts(4, 0.5, 30)
    for _ in range(30):
        c.update(2, 30)
    post = c.posteriors(0.001)
    assert post[2][2] > 0.999
    assert sum(map(sum, post)) == pytest.approx(1.0)


def _one_tail(a, b, c, d):
    """FisherExactTest.java:65-98: reorder so a is the smallest cell, then sum the hypergeometric
    probabilities of the tables obtained by moving a->0 (exact, i.e. without the quick cut-off)."""
    if a > b:
        a, b, c, d = b, a, d, c
    if a > c:
        a, b, c, d = c, d, a, b
    total = 0.0
    while a >= 0 and d >= 0:
        n = a + b + c + d
        total += math.comb(a + b, a) * math.comb(c + d, c) / math.comb(n, a + c)
        a, b, c, d = a - 1, b + 1, c + 1, d - 1
    return total


@pytest.mark.parametrize("t", [(5, 5, 5, 5), (3, 1, 1, 3), (10, 0, 0, 10), (0, 7, 9, 2), (12, 3, 4, 20), (40, 2, 1, 38)])
def test_fisher_exact_one_tail(t):
    p = O.lib().ngo_fisher_pvalue(*t)
    # the quick mode stops once further terms cannot change two significant digits (:86-89)
    assert p == pytest.approx(_one_tail(*t), rel=1e-2)
    assert p == pytest.approx(O.lib().ngo_fisher_pvalue(t[1], t[0], t[3], t[2]), rel=1e-2)
