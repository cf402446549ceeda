"""Hand-built SAM for the CoverageStats known-answer tests (shared by the CPU and GPU suites).

Expected histograms are derived by hand from CoverageStatisticsCalculator.processPileup
(discovery/CoverageStatisticsCalculator.java:177-190) over PileupRecord.addAlignment's [first, last]
overlap (PileupRecord.java:154-167) with the generator options of processFile (:108-114)."""
import os

REF = {"c1": "ACGT" * 2500, "c2": "A" * 100}    # c1 10,000 bp: reads cross the 4096-position tiles

RECORDS = [
    # name flag seq pos mapq cigar             seq            qual
    ("r1", 0, "c1", 5, 60, "10M", "ACGTACGTAC"),        # 5..14 unique
    ("r2", 0, "c1", 8, 10, "4M2D4M", "ACGTACGT"),       # 8..17, MAPQ 10 < minMQ and no NH -> not unique
    ("r3", 256, "c1", 8, 60, "3M", "TAC"),              # secondary: kept (processSecondaryAlignments), not unique
    ("r4", 4, "c1", 9, 60, "3M", "TAC"),                # unmapped: dropped by the reader
    ("r5", 0, "c1", 4090, 60, "5M", "ACGTA"),           # 4090..4094
    ("r6", 0, "c1", 4094, 60, "4M", "ACGT"),            # 4094..4097: crosses the first tile boundary
    ("r7", 16, "c1", 4100, 60, "10M6000N10M", "ACGTACGTACACGTACGTAC"),   # 4100..10119: spans > one tile
    ("r8", 0, "c2", 1, 60, "2S3M1I2M", "AAAAAAAA"),     # c2 1..5 (soft clip and insertion: no ref positions)
    ("r9", 16, "c2", 3, 60, "3M", "AAA"),               # c2 3..5
]


def write(tmpdir):
    fa = os.path.join(str(tmpdir), "kat.fa")
    with open(fa, "w") as f:
        for n, s in REF.items():
            f.write(f">{n}\n{s}\n")
    sam = os.path.join(str(tmpdir), "kat.sam")
    with open(sam, "w") as f:
        f.write("@HD\tVN:1.6\tSO:coordinate\n")
        for n, s in REF.items():
            f.write(f"@SQ\tSN:{n}\tLN:{len(s)}\n")
        for name, flag, chrom, pos, mapq, cigar, seq in RECORDS:
            f.write(f"{name}\t{flag}\t{chrom}\t{pos}\t{mapq}\t{cigar}\t*\t0\t0\t{seq}\t{'I' * len(seq)}\n")
    return fa, sam


def expected(max_coverage=300):
    """depth -> positions, unique depth -> positions (depth >= 1 only), from the read intervals."""
    reads = [(r[2], r[3], r[5], r[1], r[4]) for r in RECORDS if not r[1] & 4]
    depth, udepth = {}, {}
    import re
    for chrom, pos, cigar, flag, mapq in reads:
        span = sum(int(n) for n, op in re.findall(r"(\d+)([MDN=X])", cigar))
        uniq = not (flag & 0x100) and mapq >= 20
        for p in range(pos, pos + span):
            depth[(chrom, p)] = depth.get((chrom, p), 0) + 1
            udepth[(chrom, p)] = udepth.get((chrom, p), 0) + (1 if uniq else 0)
    counts = [0] * max_coverage
    ucounts = [0] * max_coverage
    hi = hu = 0
    for k, d in depth.items():
        if d < max_coverage:
            counts[d] += 1
        else:
            hi += 1
        u = udepth[k]
        if u < max_coverage:
            ucounts[u] += 1
        else:
            hu += 1
    counts[0] = ucounts[0] = 0      # bin 0 (empty pileups) is never printed
    return counts, ucounts, hi, hu


def text(counts, ucounts, hi, hu):
    return "".join(f"{i}\t{counts[i]}\t{ucounts[i]}\n" for i in range(1, len(counts))) + f"More\t{hi}\t{hu}\n"
