"""The oracle's indel realigner region logic and the listeners' span branches against an independent pure-Python
restatement of the Java (tests/realigner_restatement.py), on seeded synthetic pileups built here and on hand-made
ones.  The C oracle (oracle/ngsep_oracle_indel.inc) and the product (ngsepcore_amd/csrc/realign.cpp) restate the same
Java with the same decomposition; this second reading breaks that common mode for the code that decides which reads get
rewritten:

  * every pileup the realigner ran on: its reference span and STR / new-STR / embedded flags (onPileup,
    intersectWithVariants, conciliateIndels, analyzeIndels, lookForNewSTR, checkTandemRepeat, moveIndelStarts);
  * the span allele calls the listener then reads (PileupRecord.getAlleleCalls(span) over the edited alignments);
  * every alignment's final first / last / CIGAR / bases to ignore (moveIndelStart, processEndsOfAlignments with
    realignStart / realignEnd / trimming, calculateInsertedConsensusSequence, calculateDeletionConsensusLength);
  * the indel / STR records of SingleSampleVariantsDetector (discoverVariantWithSpan, lastIndelEnd) and of
    MultisampleVariantsDetector (discoverPopulationVariantWithSpan / discoverPopulationIndel, genotypeVariant).

The pileups: a random reference with planted homopolymer runs, indels inside the runs whose gap each read places at a
random equivalent offset (the realigner's votes and moves), indels elsewhere, two-length events (new STRs), reads whose
end falls inside an event drawn as mismatches or soft clips (processEndsOfAlignments' realignments and trims), and
-knownSTRs inputs (fixed events).  The oracle writes its trace with NGO_REALIGN_TRACE; the GPU path equals the oracle
on whole VCFs (tests/test_gpu_indels.py, test_gpu_multisample.py)."""
import os
import random

import pytest

import ngsep_oracle
import realigner_restatement as RR

BASES = "ACGT"
QCHARS = "#+5:?FFFFF"          # phred 2, 10, 20, 25, 30, 37 (quality-weighted towards high)


# ------------------------------------------------------------------------------------------------------------------
# synthetic pileups
# ------------------------------------------------------------------------------------------------------------------
class Event:
    """an indel on some haplotypes: ins (bases after anchor a) or del (k reference bases after anchor a); a run event
    floats: each read anchors it anywhere in [lo, hi] (equivalent alignments of the same haplotype)"""

    def __init__(self, kind, lo, hi, k, bases=""):
        self.kind, self.lo, self.hi, self.k, self.bases = kind, lo, hi, k, bases


def make_reference(rnd, length, n_runs):
    ref = [rnd.choice(BASES) for _ in range(length)]
    runs = []
    for j in range(n_runs):
        start = 150 + j * ((length - 300) // max(1, n_runs)) + rnd.randint(0, 40)
        b = rnd.choice(BASES)
        rl = rnd.randint(6, 12) if j % 3 else 3               # (every third run short: only the reads show a repeat)
        for i in range(rl):
            ref[start - 1 + i] = b
        # the run's neighbours differ from its base (a clean run)
        ref[start - 2] = rnd.choice([x for x in BASES if x != b])
        ref[start - 1 + rl] = rnd.choice([x for x in BASES if x != b])
        runs.append((start, start + rl - 1, b))
    return "".join(ref), runs


def make_events(rnd, ref, runs, n_random, multi_frac=0.3):
    """per event: a list of alleles (Event or None = reference) -> haplotypes pick among them"""
    sites = []
    for (r0, r1, b) in runs:
        alts = []
        if r1 - r0 + 1 <= 3:
            # a short run: insertions of one and two copies (two lengths; lookForNewSTR finds the repeat in a read)
            alts = [Event("ins", r0 - 1, r1, 1, b), Event("ins", r0 - 1, r1, 2, b * 2)]
        elif rnd.random() < 0.25:
            # a deletion longer than the run, anchored before it (a fixed event's window is shorter than it)
            alts = [Event("del", r0 - 1, r0 - 1, r1 - r0 + 1 + rnd.randint(1, 4))]
        else:
            for _ in range(2 if rnd.random() < multi_frac else 1):
                k = rnd.randint(1, 4)
                if rnd.random() < 0.5:
                    alts.append(Event("ins", r0 - 1, r1, k, b * k))
                else:
                    k = min(k, r1 - r0)
                    alts.append(Event("del", r0 - 1, r1 - k, k))
        sites.append(alts)
    used = {p for r0, r1, _ in runs for p in range(r0 - 20, r1 + 20)}
    for _ in range(n_random):
        a = rnd.randint(120, len(ref) - 150)
        if any(p in used for p in range(a - 30, a + 30)):
            continue
        used.update(range(a - 30, a + 30))
        if rnd.random() < 0.5:
            ev = Event("ins", a, a, 0, "".join(rnd.choice(BASES) for _ in range(rnd.randint(1, 9))))
            ev.k = len(ev.bases)
        else:
            ev = Event("del", a, a, rnd.randint(1, 12))
        sites.append([ev])
    return sites


def haplotype_window(ref, evs, lo, hi, rnd):
    """bases and reference positions (None: inserted) of ref[lo..hi] (1-based) with the events applied, each floating
    event anchored at a random allowed position"""
    anchors = {}
    dels = set()
    for e in evs:
        a = rnd.randint(e.lo, e.hi)
        if e.kind == "ins":
            anchors[a] = e.bases
        else:
            dels.update(range(a + 1, a + 1 + e.k))
    seq, rp = [], []
    if lo - 1 in anchors:
        pass                                                     # (an insertion before the window is not needed)
    for p in range(lo, hi + 1):
        if p not in dels:
            seq.append(ref[p - 1])
            rp.append(p)
        if p in anchors:
            for ch in anchors[p]:
                seq.append(ch)
                rp.append(None)
    return seq, rp


def cigar_of(rp):
    """CIGAR of a read's reference positions (M runs, I for None, D for gaps; a trailing insertion soft-clipped)"""
    ops = []

    def push(op, n):
        if ops and ops[-1][0] == op:
            ops[-1][1] += n
        else:
            ops.append([op, n])
    prev = None
    for x in rp:
        if x is None:
            push("I", 1)
            continue
        if prev is not None and x > prev + 1:
            push("D", x - prev - 1)
        push("M", 1)
        prev = x
    if ops[-1][0] == "I":
        ops[-1][0] = "S"
    return ops


def redraw_ends(rnd, ops, first):
    """an aligner's view of a read whose end falls near an event: the short piece on the far side of the first / last
    indel aligned as mismatches (M, contiguous) or soft-clipped.  Returns (ops, first)."""
    ind = [i for i, (o, _) in enumerate(ops) if o in "ID"]
    if not ind:
        return ops, first
    i = ind[0]
    if i == 1 and ops[0][0] == "M" and ops[0][1] < 45 and rnd.random() < 0.6:
        a = ops[0][1] + (ops[1][1] if ops[1][0] == "I" else 0)
        ref_start_next = first + ops[0][1] + (ops[1][1] if ops[1][0] == "D" else 0)
        if rnd.random() < 0.25:
            ops = [["S", a]] + ops[2:]
            first = ref_start_next
        elif ref_start_next - a >= 1:
            ops = [["M", a + ops[2][1]]] + ops[3:] if ops[2][0] == "M" else [["M", a]] + ops[2:]
            first = ref_start_next - a
        return ops, first
    j = ind[-1]
    if j == len(ops) - 2 and ops[-1][0] == "M" and ops[-1][1] < 45 and rnd.random() < 0.6:
        c = ops[-1][1] + (ops[j][1] if ops[j][0] == "I" else 0)
        if rnd.random() < 0.25:
            ops = ops[:j] + [["S", c]]
        else:
            ops = ops[:j] + [["M", c]]
            if len(ops) >= 2 and ops[-2][0] == "M":
                ops = ops[:-2] + [["M", ops[-2][1] + c]]
    return ops, first


def mutate(rnd, bases):
    out, quals = [], []
    for b in bases:
        qc = rnd.choice(QCHARS)
        q = ord(qc) - 33
        if rnd.random() < 10 ** (-q / 10.0) * 0.75:
            b = rnd.choice([x for x in BASES if x != b])
        out.append(b)
        quals.append(qc)
    return "".join(out), "".join(quals)


def write_case(tmp, seed, n_samples=1, depth=24, length=4000, read_len=100, n_runs=8, n_random=8, known_strs=False,
               n_contigs=1):
    """FASTA + coordinate-sorted SAM (+ the -knownSTRs file): returns (fa, sam, seqs, strs, samples)"""
    rnd = random.Random(seed)
    seqs, lines, strs = [], [], []
    header = ["@HD\tVN:1.6\tSO:coordinate"]
    samples = [f"S{k:03d}" for k in range(n_samples)]
    rid = 0
    for ci in range(n_contigs):
        name = f"chr{ci + 1}"
        ref, runs = make_reference(rnd, length, n_runs)
        seqs.append((name, ref))
        header.append(f"@SQ\tSN:{name}\tLN:{len(ref)}")
        sites = make_events(rnd, ref, runs, n_random)
        if known_strs:
            for (r0, r1, _) in runs:
                if rnd.random() < 0.7:
                    strs.append((name, r0, r1))
        recs = []
        for s in samples:
            # genotype per site: two haplotypes, each the reference or one of the site's alleles
            haps = [[], []]
            for alts in sites:
                g = rnd.random()
                for h in range(2):
                    if g < 0.35 or (g < 0.7 and h == 0):
                        haps[h].append(rnd.choice(alts))
            n_reads = depth * length // read_len
            for _ in range(n_reads):
                h = rnd.randrange(2)
                start = rnd.randint(1, length - read_len - 40)
                seq, rp = haplotype_window(ref, haps[h], start, min(length, start + read_len + 60), rnd)
                seq, rp = seq[:read_len], rp[:read_len]
                if rp[0] is None or len(seq) < read_len:
                    continue
                ops = cigar_of(rp)
                ops, first = redraw_ends(rnd, ops, rp[0])
                if ops[0][0] in "ID" or ops[-1][0] in "ID":
                    continue
                bases, quals = mutate(rnd, "".join(seq))
                cig = "".join(f"{n}{o}" for o, n in ops)
                flag = 16 if rnd.random() < 0.5 else 0
                recs.append((first, f"r{rid}\t{flag}\t{name}\t{first}\t60\t{cig}\t*\t0\t0\t{bases}\t{quals}\tRG:Z:{s}"))
                rid += 1
        recs.sort(key=lambda r: r[0])
        lines += [r[1] for r in recs]
    for s in samples:
        header.append(f"@RG\tID:{s}\tSM:{s}")
    fa = os.path.join(tmp, f"case{seed}.fa")
    with open(fa, "w") as f:
        for name, ref in seqs:
            f.write(f">{name}\n")
            for i in range(0, len(ref), 70):
                f.write(ref[i:i + 70] + "\n")
    sam = os.path.join(tmp, f"case{seed}.sam")
    with open(sam, "w") as f:
        f.write("\n".join(header + lines) + "\n")
    strs_path = None
    if known_strs:
        strs_path = os.path.join(tmp, f"case{seed}.strs")
        with open(strs_path, "w") as f:
            for n, a, b in strs:
                f.write(f"{n}\t{a}\t{b}\n")
    return fa, sam, seqs, strs, samples, strs_path


# ------------------------------------------------------------------------------------------------------------------
# the oracle's side
# ------------------------------------------------------------------------------------------------------------------
def oracle_run(tmp, fa, sam, multi, strs_path=None, **kw):
    out = os.path.join(tmp, "o.vcf")
    tr = os.path.join(tmp, "o.trace")
    os.environ["NGO_REALIGN_TRACE"] = tr
    try:
        if strs_path:
            kw["known_strs"] = strs_path
        if multi:
            ngsep_oracle.run_mvd(fa, sam, out, 0.0, **kw)
        else:
            ngsep_oracle.run_ssvd(fa, sam, out, **kw)
    finally:
        del os.environ["NGO_REALIGN_TRACE"]
    trace, alns = [], []
    for l in open(tr):
        l = l.rstrip("\n")
        (alns if l.startswith("A") else trace).append(l)
    alns.sort(key=lambda l: int(l.split("\t")[1]))
    recs = []
    for l in open(out):
        if l.startswith("#"):
            continue
        f = l.rstrip("\n").split("\t")
        info = dict(x.split("=", 1) for x in f[7].split(";") if "=" in x)
        if info.get("TYPE") not in ("INDEL", "STR"):
            continue
        recs.append("\t".join([f[0], f[1], f[3], f[4], f[5], info["TYPE"]] + f[9:]))
    return trace, alns, recs


def compare(tmp, seed, multi=False, known=False, **case_kw):
    fa, sam, seqs, strs, samples, strs_path = write_case(tmp, seed, n_samples=6 if multi else 1,
                                                         depth=8 if multi else 24, known_strs=known, **case_kw)
    o_trace, o_alns, o_recs = oracle_run(tmp, fa, sam, multi, strs_path)
    ev = {}
    p_trace, p_alns, p_recs = RR.run(sam, seqs, "population" if multi else "single",
                                     samples=[(s, [s]) for s in sorted(samples)] if multi else None,
                                     known_strs=strs if known else None, events=ev)
    assert len(p_trace) == len(o_trace)
    for i, (a, b) in enumerate(zip(p_trace, o_trace)):
        assert a == b, f"trace line {i}: restatement {a!r} oracle {b!r}"
    assert p_alns == o_alns
    assert p_recs == o_recs
    return ev, o_recs


SEEDS = list(range(24))


@pytest.mark.parametrize("seed", SEEDS)
def test_single_sample_region_logic(tmp_path, seed):
    """SingleSampleVariantsDetector: pileup spans/flags, span calls, final alignments and indel / STR records equal the
    restatement's on 24 seeded pileups (half of them with -knownSTRs inputs: the realigner's fixed events)"""
    ev, recs = compare(str(tmp_path), seed, multi=False, known=seed % 2 == 1)
    assert recs and ev["conciliate"] > 0


@pytest.mark.parametrize("seed", range(100, 108))
def test_population_region_logic(tmp_path, seed):
    """MultisampleVariantsDetector (6 samples): the same trace plus the population indel / STR records
    (discoverPopulationVariantWithSpan / discoverPopulationIndel, every sample's genotype)"""
    ev, recs = compare(str(tmp_path), seed, multi=True, known=seed % 2 == 1)
    assert recs


def test_branches_exercised(tmp_path):
    """The seeded cases together reach every branch of the region logic the KATs are about: votes moving indel starts
    (and moves refused), a new STR from the reference and from the reads, fixed events, processEndsOfAlignments'
    realigned starts / ends and trims.  realignStart / realignEnd's "Can not realign" returns are unreachable from
    processEndsOfAlignments (there unknownBpRef = eventLast - eventFirst - 1 >= 0 and unknownBpRead = eventLast - eventFirst
    + offset >= 1 for the start; unknownBpRef = deletion length >= 0 and unknownBpRead = max(offset, 0) for the end):
    the restatement counts them and they stay 0 (tests/test_oracle_indel_kat.py drives those returns directly)."""
    tot = {}
    for seed in range(8):
        d = os.path.join(str(tmp_path), str(seed))
        os.makedirs(d)
        ev, _ = compare(d, seed, multi=False, known=seed % 2 == 1)
        for k, v in ev.items():
            tot[k] = tot.get(k, 0) + v
    for k in ("conciliate", "move", "move_refused", "max_i_moved", "new_str_ref", "new_str_read", "fixed_event",
              "realign_start", "realign_end", "trim_start", "trim_end", "embedded"):
        assert tot.get(k, 0) > 0, (k, tot)
    assert tot.get("realign_start_fail", 0) == 0 and tot.get("realign_end_fail", 0) == 0


def test_hand_made_new_str_and_fixed_event(tmp_path):
    """Hand-made: a 10-base A run with reads carrying 1- and 2-base insertions of A at random offsets (two lengths:
    lookForNewSTR finds the run in the reference: span = run + 2, the STR flag and a new-STR record), then the same
    reads with the run given as -knownSTRs (a fixed event: no new STR, an input-STR record)."""
    rnd = random.Random(7)
    left = "".join(rnd.choice("CGT") for _ in range(300))
    right = "".join(rnd.choice("CGT") for _ in range(300))
    ref = left + "A" * 10 + right
    r0 = len(left) + 1
    lines = []
    rid = 0
    for k in range(40):
        ins = 1 + (k % 3 == 0)
        start = rnd.randint(200, r0 - 20)
        anchor = rnd.randint(r0 - 1, r0 + 9)
        seq = ref[start - 1:anchor] + "A" * ins + ref[anchor:anchor + 200]
        seq = seq[:120]
        m1 = anchor - start + 1
        cig = f"{m1}M{ins}I{120 - m1 - ins}M"
        lines.append((start, f"h{rid}\t0\tchrA\t{start}\t60\t{cig}\t*\t0\t0\t{seq}\t{'F' * 120}\tRG:Z:S000"))
        rid += 1
    for k in range(20):
        start = rnd.randint(200, r0 - 20)
        seq = ref[start - 1:start + 119]
        lines.append((start, f"h{rid}\t16\tchrA\t{start}\t60\t120M\t*\t0\t0\t{seq}\t{'F' * 120}\tRG:Z:S000"))
        rid += 1
    lines.sort(key=lambda x: x[0])
    fa = os.path.join(str(tmp_path), "h.fa")
    sam = os.path.join(str(tmp_path), "h.sam")
    with open(fa, "w") as f:
        f.write(">chrA\n" + ref + "\n")
    with open(sam, "w") as f:
        f.write(f"@HD\tVN:1.6\tSO:coordinate\n@SQ\tSN:chrA\tLN:{len(ref)}\n@RG\tID:S000\tSM:S000\n")
        f.write("\n".join(l for _, l in lines) + "\n")
    for known in (False, True):
        strs_path = None
        if known:
            strs_path = os.path.join(str(tmp_path), "h.strs")
            with open(strs_path, "w") as f:
                f.write(f"chrA\t{r0}\t{r0 + 9}\n")
        o_trace, o_alns, o_recs = oracle_run(str(tmp_path), fa, sam, False, strs_path)
        ev = {}
        p_trace, p_alns, p_recs = RR.run(sam, [("chrA", ref)], "single", known_strs=[("chrA", r0, r0 + 9)] if known else None,
                                         events=ev)
        assert p_trace == o_trace and p_alns == o_alns and p_recs == o_recs
        assert len(o_recs) == 1 and o_recs[0].split("\t")[5] == "STR"
        if known:
            assert ev.get("fixed_event", 0) > 0 and not ev.get("new_str_ref")
        else:
            assert ev.get("new_str_ref", 0) > 0
