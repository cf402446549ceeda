"""An independent pure-Python restatement of the indel realigner's region logic and of the two listeners' span branches,
read from the Java -- NOT from ngsepcore_amd/csrc/realign.cpp nor from oracle/ngsep_oracle_indel.inc: test
infrastructure for tests/test_oracle_realigner_kat.py, which drives it over small pileups and compares what it does
(the pileups' spans and flags, the span allele calls, every alignment's final state, the indel / STR records) with the C
oracle's trace (NGO_REALIGN_TRACE) and VCF.  The per-call pieces (CountsHelper indel counts, clustering, callIndel,
genotype fields, moveIndelStart / realignStart / realignEnd) come from tests/indel_restatement.py, the first independent
reading.

  ReadAlignmentFileReader.loadAlignment / isMultiple / isSameAlignment / filters  alignments/io/ReadAlignmentFileReader.java:219-306
  ReadAlignment: setCigarString, collapseEqualEvents, setQualityScores,             alignments/ReadAlignment.java:581-595,747-871,
    updateAlleleCallsInfo, getAlignedReadPosition, getAlleleCall(pos | first,last),   989-1106,1222-1312,1351-1363,1471-1478
    getBaseQualityScore(s), withinIgnoreRegions, getIndelCall(s), hasIndelCalls,
    getSoftClipStart / End
  AlignmentsPileupGenerator.processAlignment / processSameStartAlns /               discovery/AlignmentsPileupGenerator.java:377-504
    startSequence / notifyEndOfAlignments / processPileups / updatePendingAlns /
    processCurrentPosition
  PileupRecord.addAlignment / getAlleleCalls(span, readGroup(s))                   discovery/PileupRecord.java:104-167
  IndelRealignerPileupListener (the whole class)                                   discovery/IndelRealignerPileupListener.java:85-578
  SingleSampleVariantsDetector.makeNonRedundantSTRs / mergeSTRs / makeSTRVariant   discovery/SingleSampleVariantsDetector.java:843-894
  AbstractLimitedSequence.getOverlapLength                                          sequences/AbstractLimitedSequence.java:376-390
  SingleSampleVariantPileupListener.onPileup (discovery), calculateReference-       discovery/SingleSampleVariantPileupListener.java:
    AlleleDiscovery, discoverVariant / discoverVariantWithSpan / discoverIndel        146-232,257-296,333-391
    (ploidy < 3), createIndelVariantPool, allelesSameLength, makeNewVariant,
    genotypeVariantSample (indel, ploidy < 3)
  MultisampleVariantsDetector.onPileup (discovery), discoverPopulationVariant-      discovery/MultisampleVariantsDetector.java:521-693
    WithSpan, discoverPopulationIndel, makeNewVariant, genotypeVariant
  NumberArrays.getIndexMaximum, HashMap<Integer, V> iteration order                math/NumberArrays.java:84-95

Only the non-SNV records are produced (the SNV fallbacks of the span branches run in the oracle; an SNV call never moves
lastIndelEnd, so the indel / STR records do not depend on them).  Java semantics kept: (byte) casts of the ignore
counts, HashMap iteration order of small Integer keys, String.toUpperCase, null references past a sequence's ends."""
from __future__ import annotations

import indel_restatement as R

H, D, I, M, P, N, S, X = range(8)
OPS = "HDIMPNSX"
BASES = "ACGT"
FLAG_PAIRED, FLAG_UNMAPPED, FLAG_REVERSE, FLAG_FIRST, FLAG_SECONDARY = 0x1, 0x4, 0x10, 0x40, 0x100
FLAG_MULTIPLE_ALN = 0x1000
DEF_REGION_BOUNDARY = 100


def count(ev, key):
    if ev is not None:
        ev[key] = ev.get(key, 0) + 1


def cref(v):
    return (v & 1) != 0


def cread(v):
    return (v & 2) != 0


def is_indel(op):
    return op == D or op == I


# ------------------------------------------------------------------------------------------------------------------
# ReadAlignment
# ------------------------------------------------------------------------------------------------------------------
def cigar_codes(text):
    """setCigarString (:1222-1266): operators by "HDIMPNSX" ('=' -> M), then collapseEqualEvents (:1296-1312)"""
    raw, n = [], 0
    for ch in text:
        if ch.isdigit():
            n = n * 10 + int(ch)
            continue
        op = OPS.find(ch)
        if op < 0 and ch == "=":
            op = M
        raw.append(8 * n + op)
        n = 0
    out, last_op, tot = [], -1, 0
    for v in raw:
        if (v & 7) != last_op:
            if tot > 0:
                out.append(8 * tot + last_op)
            tot, last_op = 0, v & 7
        tot += v // 8
    if tot > 0:
        out.append(8 * tot + last_op)
    return out


class Aln:
    def __init__(self, ident, seq, first, cigar, chars, quals, flags, rg):
        self.id, self.seq, self.first, self.flags, self.rg = ident, seq, first, flags, rg
        self.aln = cigar_codes(cigar)
        self.read_length = sum(v // 8 for v in self.aln if cread(v))
        self.last = first + sum(v // 8 for v in self.aln if cref(v)) - 1
        self.chars = chars
        self.quals = None
        if quals is not None:                                   # setQualityScores (:581-595)
            q = [38] * self.read_length
            for i, ch in enumerate(quals[:self.read_length]):
                q[i] = min(127, ord(ch))
            self.quals = q
        self.ign_start = self.ign_end = 0
        self.close = 2                                          # basesToIgnoreCloseToIndel (:115)
        self.updated = False
        self.acl = None
        self.indels = None                                      # TreeMap refPos -> (first, last, length)

    def negative(self):
        return (self.flags & FLAG_REVERSE) != 0

    def cigar(self):
        return "".join(f"{v // 8}{OPS[v & 7]}" for v in self.aln)

    # updateAlleleCallsInfo (:747-834)
    def update(self):
        if self.updated:
            return
        ref, rp = self.first, 0
        self.acl = [0] * self.read_length
        self.indels = None
        prev_indel = False
        n = len(self.aln)
        for i, v in enumerate(self.aln):
            length, op = v // 8, v & 7
            nxt_op, nxt_len, nxt_indel, nxt_read = -1, 0, False, 0
            if i < n - 1:
                nxt_op, nxt_len = self.aln[i + 1] & 7, self.aln[i + 1] // 8
                nxt_indel = is_indel(nxt_op)
                nxt_read = nxt_len if cread(nxt_op) else 0
            if cref(v):
                if cread(v):
                    for j in range(length):
                        skip = rp < self.ign_start
                        skip = skip or (self.read_length - rp) <= self.ign_end
                        skip = skip or (prev_indel and j < self.close)
                        skip = skip or (nxt_indel and j < length - 1 and j >= length - self.close)
                        skip = skip or (nxt_indel and j == length - 1 and
                                        (rp < self.close or self.read_length - rp - nxt_read < self.close))
                        after = rp + nxt_read + 1
                        skip = skip or (nxt_indel and j == length - 1 and (self.read_length - after < self.ign_end))
                        if not skip:
                            if j == length - 1 and nxt_indel:
                                ref_last = ref + 1
                                if nxt_op == I:
                                    self.acl[rp] = nxt_len + 2
                                else:
                                    self.acl[rp] = 2
                                    ref_last += nxt_len
                                if self.indels is None:
                                    self.indels = {}
                                self.indels[ref] = (ref, ref_last, nxt_len)
                            else:
                                self.acl[rp] = 1
                        ref += 1
                        rp += 1
                else:
                    ref += length
            elif cread(v):
                rp += length
            prev_indel = is_indel(op)
        self.updated = True

    # getAlignedReadPosition (:842-871)
    def read_pos(self, ref_pos):
        cur_ref, cur_read = self.first, 0
        if ref_pos < self.first or ref_pos > self.last:
            return -1
        for v in self.aln:
            length = v // 8
            if cref(v) and cread(v):
                if ref_pos < cur_ref:
                    return -1
                if cur_ref + length > ref_pos:
                    ans = cur_read + ref_pos - cur_ref
                    return -1 if ans < 0 or ans >= self.read_length else ans
            if cref(v):
                cur_ref += length
            if cread(v):
                cur_read += length
        return -1

    def allele_call(self, pos):                                 # getAlleleCall(pos) (:989-1000)
        if self.chars is None:
            return None
        rp = self.read_pos(pos)
        if rp < 0:
            return None
        self.update()
        n = self.acl[rp]
        return None if n == 0 else self.chars[rp:rp + n]

    def within_ignore(self, rf, rl):                            # withinIgnoreRegions (:1042-1044)
        return rf < self.ign_start or self.read_length - rl <= self.ign_end

    def allele_call_range(self, first, last):                   # getAlleleCall(first, last) (:1008-1016)
        if self.chars is None:
            return None
        self.update()
        rf, rl = self.read_pos(first), self.read_pos(last)
        if rf < 0 or rl < 0 or rl < rf or self.within_ignore(rf, rl):
            return None
        return self.chars[rf:rl + 1]

    def qual_at(self, pos):                                     # getBaseQualityScore (:1022-1027)
        rp = self.read_pos(pos)
        if rp < 0:
            return chr(33)
        return "+" if self.quals is None else chr(self.quals[rp])

    def quals_range(self, first, last):                         # getBaseQualityScores (:1034-1041)
        rf, rl = self.read_pos(first), self.read_pos(last)
        if rf < 0 or rl < 0 or rl < rf or self.within_ignore(rf, rl):
            return None
        if self.quals is None:
            return "+" * (rl - rf + 1)
        return "".join(chr(q) for q in self.quals[rf:rl + 1])

    def indel_calls(self):                                      # getIndelCalls (:1050-1054), TreeMap order
        self.update()
        return None if self.indels is None else dict(sorted(self.indels.items()))

    def indel_call(self, pos):                                  # getIndelCall (:1101-1106)
        self.update()
        return None if self.indels is None else self.indels.get(pos)

    def has_indel_calls(self, a, b):                            # hasIndelCalls (:1471-1478)
        calls = self.indel_calls()
        return calls is not None and any(a <= k <= b for k in calls)

    def soft_clip_start(self):                                  # :1351-1356
        return self.aln[0] // 8 if (self.aln[0] & 7) == S else 0

    def soft_clip_end(self):                                    # :1358-1363
        return self.aln[-1] // 8 if (self.aln[-1] & 7) == S else 0

    def set_ignore_start(self, v):                              # setBasesToIgnoreStart (:657-662)
        if self.ign_start != v:
            self.ign_start = v
            self.updated = False

    def set_ignore_end(self, v):                                # setBasesToIgnoreEnd (:675-680)
        if self.ign_end != v:
            self.ign_end = v
            self.updated = False

    def move_indel_start(self, old, new, ev):                   # moveIndelStart (:1114-1153)
        moved, codes = R.move_indel_start(self.first, self.aln, old, new)
        if moved and new != old:
            self.aln = codes
            self.updated = False
            count(ev, "move")
        elif not moved:
            count(ev, "move_refused")
        return moved

    def realign_start(self, new_first, first_match, ref_after, read_after, ev):   # realignStart (:1372-1418)
        fail = ref_after - (new_first + first_match) < 0 or read_after - first_match < 0
        count(ev, "realign_start_fail" if fail else "realign_start")
        f, _, codes = R.realign_start(self.first, self.last, self.aln, new_first, first_match, ref_after, read_after)
        if codes != self.aln or f != self.first:
            self.first, self.aln = f, codes
            self.updated = False

    def realign_end(self, ref_before, read_before, final_start, final_len, ev):  # realignEnd (:1427-1469)
        fail = final_start - ref_before - 1 < 0 or (self.read_length - read_before - 1) - final_len < 0
        count(ev, "realign_end_fail" if fail else "realign_end")
        _, l, codes = R.realign_end(self.first, self.last, self.aln, self.read_length, ref_before, read_before,
                                    final_start, final_len)
        if codes != self.aln or l != self.last:
            self.last, self.aln = l, codes
            self.updated = False


# ------------------------------------------------------------------------------------------------------------------
# reader (ReadAlignmentFileReader) over SAM text
# ------------------------------------------------------------------------------------------------------------------
def read_sam(path, min_mq=20, secondary=False, nonunique=False):
    """The records AlignmentsPileupGenerator.processFile sees, in file order; ids are the alignment lines' ordinals."""
    rg_ids = set()
    filt = FLAG_UNMAPPED
    if not secondary:
        filt += FLAG_SECONDARY
        if not nonunique:
            filt += FLAG_MULTIPLE_ALN
    out, prev, k = [], None, -1
    for line in open(path):
        if line.startswith("@"):
            if line.startswith("@RG"):
                for f in line.rstrip("\n").split("\t")[1:]:
                    if f.startswith("ID:"):
                        rg_ids.add(f[3:])
            continue
        f = line.rstrip("\n").split("\t")
        if len(f) < 11:
            continue
        k += 1
        flag, start = int(f[1]), int(f[3])
        key = (start, flag & FLAG_PAIRED, (flag & FLAG_FIRST) if flag & FLAG_PAIRED else 0, f[0])
        if prev == key:                                         # isSameAlignment (:292-306)
            continue
        prev = key
        tags = {t[:2]: t[5:] for t in f[11:]}
        nh = int(tags["NH"]) if "NH" in tags else None
        mapq = int(f[4])
        multiple = bool(flag & FLAG_SECONDARY) or (nh is not None and nh > 1) or (nh is None and mapq < min_mq)
        flags = flag + (FLAG_MULTIPLE_ALN if multiple else 0)
        if flag & FLAG_UNMAPPED or f[5] == "*":
            continue
        rg = tags.get("RG", "")
        rg = rg if rg in rg_ids else ""
        chars = None if f[9] == "*" else f[9].upper().replace(".", "N")
        quals = None if chars is None or f[10] == "*" else f[10]
        a = Aln(k, f[2], start, f[5], chars, quals, flags, rg)
        if chars is not None and len(chars) != a.read_length:
            continue
        if flags & filt:
            continue
        out.append(a)
    return out


# ------------------------------------------------------------------------------------------------------------------
# PileupRecord and AlignmentsPileupGenerator
# ------------------------------------------------------------------------------------------------------------------
class Pileup:
    def __init__(self, seq, pos):
        self.seq, self.pos = seq, pos
        self.alns, self.by_rg = [], {}
        self.span, self.str, self.new_str, self.embedded = 1, False, False, False

    def add(self, a):                                           # addAlignment (:154-167)
        if a.first > self.pos or a.last < self.pos:
            return
        self.alns.append(a)
        self.by_rg.setdefault(a.rg, []).append(a)

    def input_str(self):
        return self.str and not self.new_str

    def allele_calls(self, span, rgs=None):                     # getAlleleCalls (:104-152): [(allele, quals, neg)]
        if rgs is None:
            return self._calls(span, self.alns)
        out = []
        for rg in rgs:
            out += self._calls(span, self.by_rg.get(rg, []))
        return out

    def _calls(self, span, alns):
        out = []
        for a in alns:
            call = a.allele_call(self.pos)
            if call is None:
                continue
            qs = a.qual_at(self.pos)
            if span > 1:
                last = self.pos + span - 1
                call = a.allele_call_range(self.pos, last)
                if call is None:
                    continue
                qs = a.quals_range(self.pos, last)
            elif len(call) > 1:
                continue
            out.append((call, qs, a.negative()))
        return out


class Generator:
    def __init__(self, listeners, max_alns_per_start=5):
        self.listeners = listeners
        self.max_alns = max_alns_per_start
        self.seq = None
        self.pos = self.ref_last = 0
        self.last_start = -1
        self.ss_primary, self.ss_secondary, self.pending = [], [], []
        self.retired = []                                       # (the trace: alignments leaving the pending list)

    def process_alignment(self, a):                             # :377-403
        if self.seq is not None:
            same = self.seq == a.seq
            if not same or self.last_start != a.first:
                self.process_same_start()
                if not same:
                    self.process_pileups(self.ref_last + 1)
                    for l in self.listeners:
                        l.on_sequence_end(self.seq)
                    self.seq = None
                else:
                    self.process_pileups(a.first)
        if self.seq is None:                                    # startSequence (:435-444)
            self.seq, self.pos, self.ref_last = a.seq, a.first, a.last
            for l in self.listeners:
                l.on_sequence_start(self.seq)
        self.ref_last = max(self.ref_last, a.last)
        (self.ss_secondary if a.flags & FLAG_SECONDARY else self.ss_primary).append(a)
        self.last_start = a.first

    def process_same_start(self):                               # :407-433
        if self.ss_primary:
            start = self.ss_primary[0].first
        elif self.ss_secondary:
            start = self.ss_secondary[0].first
        else:
            return
        allp = self.ss_primary + self.ss_secondary
        self.ss_primary, self.ss_secondary = [], []
        per_rg = {}
        for a in allp:
            c = per_rg.get(a.rg)
            if c is None:
                per_rg[a.rg] = 1
            elif self.max_alns <= 0 or c < self.max_alns:
                per_rg[a.rg] = c + 1
            else:
                continue
            self.pending.append(a)                              # (ignore5/3 = 0: setBasesToIgnore5P/3P change nothing)

    def notify_end(self):                                       # :447-452
        self.process_same_start()
        self.process_pileups(self.ref_last + 1)
        if self.seq is not None:
            for l in self.listeners:
                l.on_sequence_end(self.seq)
        self.seq = None

    def process_pileups(self, start):                           # :453-462
        if start == self.pos:
            return
        while self.pos < start:
            if not self.process_position():
                self.update_pending()
                if not self.pending:
                    self.pos = start
        self.update_pending()

    def update_pending(self):                                   # :464-471
        keep = []
        for a in self.pending:
            (keep if a.last >= self.pos else self.retired).append(a)
        self.pending = keep

    def process_position(self):                                 # :475-498
        if not self.pending:
            self.pos += 1
            return False
        p = Pileup(self.seq, self.pos)
        for a in self.pending:
            p.add(a)
        for l in self.listeners:
            l.on_pileup(p)
        self.pos += 1
        return len(p.alns) > 0


# ------------------------------------------------------------------------------------------------------------------
# IndelRealignerPileupListener
# ------------------------------------------------------------------------------------------------------------------
def java_int_hashmap_order(keys):
    """iteration order of a java.util.HashMap<Integer, V> filled with `keys` (distinct, insertion order): table of
    16 buckets doubled whenever size exceeds 3/4 of it, bucket = (h ^ h >>> 16) & (cap - 1) with h = the value,
    insertion order inside a bucket (a resize splits a bucket's list keeping its order)"""
    cap = 16
    while len(keys) > cap * 3 // 4:
        cap *= 2

    def bucket(k):
        h = k & 0xFFFFFFFF
        return (h ^ (h >> 16)) & (cap - 1)
    idx = sorted(range(len(keys)), key=lambda i: (bucket(keys[i]), i))
    return [keys[i] for i in idx]


def hamming(a, b):
    return sum(1 for x, y in zip(a, b) if x != y)


def upper_or_none(s):
    return None if s is None else s.upper()


class Genome:
    def __init__(self, seqs):
        self.seqs = dict(seqs)

    def ref(self, name, first, last):                           # ReferenceGenome.getReference (:217-239)
        s = self.seqs.get(name)
        if s is None or first < 1 or last > len(s):
            return None
        if last < first - 1:
            raise IndexError("subSequence(begin > end)")
        return s[first - 1:last]


class Realigner:
    def __init__(self, genome, input_variants=None, events=None):
        self.g = genome
        self.ev = events                                       # {branch: times taken} (the KATs' coverage check)
        self.inputs = input_variants                           # {seq: [(first, last, type)]} in position order, or None
        self.seq_vars, self.idx = [], 0
        self.min_bp_good = 5
        self.max_bp_end = 50
        self.trace = []

    def on_sequence_start(self, seq):                           # :128-134
        if self.inputs is not None:
            self.seq_vars = self.inputs.get(seq, [])
            self.idx = 0

    def on_sequence_end(self, seq):
        pass

    def intersect(self, p):                                     # intersectWithVariants (:141-157)
        if self.inputs is not None:
            while self.idx < len(self.seq_vars):
                v = self.seq_vars[self.idx]
                if p.pos < v[0]:
                    break
                if v[0] <= p.pos <= v[1]:
                    return v
                self.idx += 1
        return None

    def on_pileup(self, p):                                     # onPileup (:85-126)
        cur = p.pos
        span = 1
        end = cur
        var = self.intersect(p)
        if var is not None:
            if var[0] == p.pos:
                if var[2] == "STR":
                    p.str = True
                span = var[1] - var[0] + 1
                end = var[1]
            else:
                p.embedded = True
                count(self.ev, "embedded")
        if var is None:
            max_len = max_span = 0
            for a in p.alns:
                ind = a.indel_call(cur)
                if ind is not None:
                    max_len = max(max_len, ind[2])
                    max_span = max(max_span, ind[1] - ind[0] + 1)
            if max_len > 0:
                end = cur + max(max_len, max_span) + 1
        if end > cur:
            c = self.conciliate(p, p.alns, end, var)
            if c > 0:
                span = c
        p.span = span
        if p.alns:                                              # (the trace: pileups with alignments only)
            self.trace.append(("P", cur, span, int(p.str), int(p.new_str), int(p.embedded)))
            if span > 1:
                for call, qs, _ in p.allele_calls(span):
                    self.trace.append(("C", call, qs))

    def conciliate(self, p, alns, end, var):                    # conciliateIndels (:165-216)
        answer = 0
        cur = p.pos
        fixed = var is not None
        votes = [0] * (end - cur + 1)
        lengths, indel_alns, max_len = self.analyze(alns, cur, end, votes)
        if not lengths:
            return answer
        count(self.ev, "conciliate")
        if fixed:
            count(self.ev, "fixed_event")
        max_i = 0
        if not fixed:
            max_i = 0                                            # NumberArrays.getIndexMaximum: the first maximum
            for i in range(1, len(votes)):
                if votes[max_i] < votes[i]:
                    max_i = i
            if len(lengths) > 1:
                new_span = self.look_for_new_str(p, indel_alns, max_len)
                if new_span > 1:
                    max_i = 0
                    answer = new_span
                    end = cur + answer - 1
                    fixed = True
                    p.str = True
                    p.new_str = True
        new_end = self.move_indel_starts(indel_alns, cur, end, max_len, max_i)
        if max_i > 0:
            count(self.ev, "max_i_moved")
            return answer
        if not fixed and new_end != end:
            end = new_end
            answer = end - cur + 1
        self.process_ends(alns, p.seq, cur, end)
        return answer

    def analyze(self, alns, start, end, votes):                 # analyzeIndels (:229-265)
        lengths, indel_alns, max_len = set(), [], 0
        for a in alns:
            found = False
            calls = a.indel_calls()
            if calls is not None:
                for k, ind in calls.items():
                    if ind[1] >= start and k <= end:
                        found = True
                        lengths.add(ind[2])
                        max_len = max(max_len, ind[2])
                        i = k - start
                        if 0 <= i < len(votes):
                            votes[i] += 1
                        break
            if found:
                indel_alns.append(a)
        return lengths, indel_alns, max_len

    def move_indel_starts(self, alns, first, last, max_len, offset):   # moveIndelStarts (:274-313)
        answer = first + 1
        for a in alns:
            calls = a.indel_calls()
            if calls is not None:
                for k, ind in calls.items():
                    if ind[1] >= first and k <= last:
                        a.move_indel_start(k, first + offset, self.ev)
                        break
            calls = a.indel_calls()
            if calls is not None:
                ref_last = first
                for k, ind in calls.items():
                    if first <= k <= ref_last + max_len:
                        ref_last = ind[1]
                if ref_last > answer:
                    answer = ref_last
        return answer

    def look_for_new_str(self, p, alns, max_len):               # lookForNewSTR (:315-349)
        new_span = 0
        cur = p.pos
        if not alns:
            return 0
        seq = self.g.ref(p.seq, cur + 1, alns[-1].last)
        length_ref = check_tandem_repeat(seq.upper()) if seq is not None else 0
        if length_ref > 0:
            count(self.ev, "new_str_ref")
            return length_ref + 2
        for a in alns:
            ind = a.indel_call(cur)
            if ind is not None and ind[2] == max_len:
                ind_span = ind[1] - ind[0] + 1
                ind_len = ind[2]
                tr = check_tandem_repeat_aln(a, cur)
                if tr > 0:
                    new_span = ind_len + 2 if ind_len >= ind_span else tr + ind_span
                    count(self.ev, "new_str_read")
                    break
        return new_span

    def process_ends(self, alns, seq, ev_first, ev_last):       # processEndsOfAlignments (:400-526)
        before = self.g.ref(seq, ev_first - DEF_REGION_BOUNDARY, ev_first)
        after = self.g.ref(seq, ev_last, ev_last + DEF_REGION_BOUNDARY)
        within = None
        if ev_first != ev_last - 1:
            within = self.g.ref(seq, ev_first + 1, ev_last - 1)
        if within is not None:
            within = within.upper()
        ref_before = upper_or_none(before)
        ref_after = upper_or_none(after)
        if ref_before is not None and within is not None:
            ref_before += within
        if ref_after is not None and within is not None:
            ref_after = within + ref_after
        ins = inserted_consensus(alns, ev_first)
        alt_before = upper_or_none(before)
        alt_after = upper_or_none(after)
        if ins is not None:
            offset = len(ins)
            if alt_before is not None:
                alt_before += ins
            if alt_before is not None and within is not None:
                alt_before += within
            if alt_after is not None and within is not None:
                alt_after = within + alt_after
            if alt_after is not None:
                alt_after = ins + alt_after
        else:
            dl = deletion_consensus_length(alns, ev_first)
            if dl > ev_last - ev_first - 1:
                dl = ev_last - ev_first - 1
                count(self.ev, "deletion_clamped")
            offset = -dl
            if alt_before is not None and within is not None:
                if dl == 0:
                    alt_before += within
                elif dl < len(within):
                    alt_before += within[dl:]
            if alt_after is not None and within is not None:
                if dl == 0:
                    alt_after = within + alt_after
                elif dl < len(within):
                    alt_after = within[dl:] + alt_after
        for a in alns:
            a_first, a_last = a.first, a.last
            before_calls = a.has_indel_calls(a_first, ev_first - 1)
            after_calls = a.has_indel_calls(ev_last + 1, a_last)
            bp_good = max(offset, self.min_bp_good)
            trim_start = ev_first - a_first < bp_good and not before_calls
            rp_after = a.read_pos(ev_last)
            if (not before_calls and ref_before is not None and alt_before is not None and rp_after >= bp_good and
                    rp_after - offset <= self.max_bp_end and rp_after < len(ref_before) and rp_after < len(alt_before) and
                    a.indel_call(ev_first) is None):
                prefix = a.chars[0:rp_after]
                ref_suffix = ref_before[len(ref_before) - rp_after:]
                d_ref = hamming(ref_suffix, prefix)
                alt_suffix = alt_before[len(alt_before) - rp_after:]
                d_alt = hamming(alt_suffix, prefix)
                new_first = ev_last - rp_after + 1 + offset
                first_match = ev_first - new_first + 1
                if d_alt < d_ref and d_alt < 3 and first_match >= self.min_bp_good:
                    a.realign_start(new_first, first_match, ev_last, rp_after, self.ev)
                    trim_start = False
            if trim_start:
                count(self.ev, "trim_start")
                ignore = ev_last - a_first + 1 + a.soft_clip_start()
                a.set_ignore_start(R.to_byte(max(a.ign_start, ignore)))
            trim_end = a_last - ev_last < bp_good and not after_calls
            rp_before = a.read_pos(ev_first)
            suffix_len = a.read_length - rp_before - 1 if rp_before >= 0 else 0
            if (not after_calls and ref_after is not None and alt_after is not None and suffix_len >= bp_good and
                    suffix_len - offset <= self.max_bp_end and suffix_len < len(ref_after) and
                    suffix_len < len(alt_after) and (a.indel_call(ev_first) is None or rp_after < 0)):
                suffix = a.chars[rp_before + 1:a.read_length]
                d_ref = hamming(ref_after[:suffix_len], suffix)
                d_alt = hamming(alt_after[:suffix_len], suffix)
                final_len = suffix_len - (offset if offset > 0 else 0)
                new_ev_last = ev_first + 1 - (offset if offset < 0 else 0)
                if d_alt < d_ref and d_alt < 3 and final_len >= self.min_bp_good:
                    a.realign_end(ev_first, rp_before, new_ev_last, final_len, self.ev)
                    trim_end = False
            if trim_end:
                count(self.ev, "trim_end")
                ignore = a_last - ev_first + 1 + a.soft_clip_end()
                a.set_ignore_end(R.to_byte(max(a.ign_end, ignore)))


def check_mono_nucleotide(seq):                                 # checkMonoNucleotide (:365-391)
    counts = [0, 0, 0, 0]
    min_len = 5
    i = 0
    while i < len(seq) and i < min_len:
        j = BASES.find(seq[i])
        if j >= 0:
            counts[j] += 1
        i += 1
    base = -1
    for j in range(4):
        if counts[j] >= i - 1:
            base = j
            break
    if base == -1 or i < min_len:
        return 0
    while i < len(seq) and counts[base] >= i - 1:
        j = BASES.find(seq[i])
        if j >= 0:
            counts[j] += 1
        i += 1
    i -= 1
    if BASES.find(seq[i - 1]) != base:
        return i - 1
    return i


def check_tandem_repeat(seq):                                   # checkTandemRepeat(String) (:359-363); dinucleotides: 0
    return check_mono_nucleotide(seq)


def check_tandem_repeat_aln(a, pos):                            # checkTandemRepeat(aln, pos) (:351-357)
    rf = a.read_pos(pos)
    if rf < 0:
        return 0
    return check_tandem_repeat(a.chars[rf + 1:].upper())


def inserted_consensus(alns, ev_first):                         # calculateInsertedConsensusSequence (:528-555)
    by_len, keys = {}, []
    for a in alns:
        if a.indel_call(ev_first) is None:
            continue
        allele = a.allele_call(ev_first)
        if allele is None:
            continue
        allele = allele[1:len(allele) - 1]
        if not allele:
            continue
        if len(allele) not in by_len:
            by_len[len(allele)] = []
            keys.append(len(allele))
        by_len[len(allele)].append(allele)
    best_n, best = 0, None
    for k in java_int_hashmap_order(keys):
        if len(by_len[k]) > best_n:
            best_n, best = len(by_len[k]), by_len[k]
    return None if best is None else R.hamming_consensus(best)


def deletion_consensus_length(alns, ev_first):                  # calculateDeletionConsensusLength (:557-578)
    counts, keys = {}, []
    for a in alns:
        call = a.indel_call(ev_first)
        if call is None:
            continue
        inner = call[1] - call[0] - 1
        if inner not in counts:
            counts[inner] = 0
            keys.append(inner)
        counts[inner] += 1
    mx = ans = 0
    for k in java_int_hashmap_order(keys):
        if mx < counts[k]:
            ans, mx = k, counts[k]
    return ans


# ------------------------------------------------------------------------------------------------------------------
# -knownSTRs: SingleSampleVariantsDetector.makeNonRedundantSTRs
# ------------------------------------------------------------------------------------------------------------------
def overlap_length(s1, s2):                                     # AbstractLimitedSequence.getOverlapLength (:376-390)
    for i in range(len(s1)):
        j, k = i, 0
        ok = True
        while j < len(s1) and k < len(s2):
            if s1[j] != s2[k]:
                ok = False
                break
            j += 1
            k += 1
        if ok and j == len(s1):
            return len(s1) - i
    return 0


def non_redundant_strs(genome, seq_order, regions):
    """regions: [(seq, first, last)] -> {seq: [(first, last, "STR")]} (makeNonRedundantSTRs :843-872, mergeSTRs
    :873-880, makeSTRVariant :883-894), each sequence's regions in (first, last) order (stable)"""
    out = {}
    for name in seq_order:
        regs = sorted([(f, l) for s, f, l in regions if s == name], key=lambda r: (r[0], r[1]))
        length = len(genome.seqs[name])
        res = []

        def emit(first, last):
            f, l = max(1, first - 1), min(last + 1, length)
            if genome.ref(name, f, l) is not None:
                res.append((f, l, "STR"))
        first = last = 0
        for rf, rl in regs:
            merge = False
            if last != 0:
                if rf - last > 5:
                    merge = False
                elif rf - last <= 2:
                    merge = True
                else:
                    r1 = genome.ref(name, max(first, last - 10), last)
                    r2 = genome.ref(name, rf, rl)
                    merge = r1 is not None and r2 is not None and overlap_length(r1.upper(), r2.upper()) > 5
            if last == 0 or not merge:
                if last > 0:
                    emit(first, last)
                first = rf
            last = rl
        if last > 0:
            emit(first, last)
        out[name] = sorted(res, key=lambda r: (r[0], r[1]))
    return out


# ------------------------------------------------------------------------------------------------------------------
# the listeners' span branches (discovery, ploidy < 3): non-SNV records
# ------------------------------------------------------------------------------------------------------------------
def reference_allele(p, genome, call_embedded, ignore_lower):   # calculateReferenceAlleleDiscovery (:191-206)
    if not call_embedded and p.embedded:
        return None
    s = genome.ref(p.seq, p.pos, p.pos + p.span - 1)
    if s is None:
        return None
    if ignore_lower and s[0].islower():
        return None
    s = s.upper()
    if p.embedded:
        s = s[:1]
        p.str = False
    return s


class SingleSampleListener:
    """SingleSampleVariantPileupListener.onPileup in discovery mode (no input variants): the indel / STR records as
    "POS REF ALT QS TYPE GT:PL:GQ:DP:ADP:ACN" (the SNV calls are not restated)"""

    def __init__(self, genome, het_rate=0.001, min_quality=40, ploidy=2, max_base_qs=30, call_embedded=False,
                 ignore_lower=False):
        self.g, self.h, self.minq, self.ploidy = genome, het_rate, min_quality, ploidy
        self.mbq, self.emb, self.lower = max_base_qs, call_embedded, ignore_lower
        self.last_indel_end = 0
        self.records = []

    def on_sequence_start(self, seq):
        self.last_indel_end = 0

    def on_sequence_end(self, seq):
        pass

    def on_pileup(self, p):
        if p.input_str() and p.pos >= self.last_indel_end:
            self.last_indel_end = p.pos + p.span - 1
        elif p.pos <= self.last_indel_end:
            p.embedded = True
        ref = reference_allele(p, self.g, self.emb, self.lower)
        if ref is None or len(ref) <= 1:
            return                                              # (span 1: discoverSNV, an SNV call or none)
        calls = p.allele_calls(len(ref))
        alleles = R.cluster_alleles([(c, q) for c, q, _ in calls], ref, self.mbq)
        hp = R.indel_helper(alleles, [(c, q) for c, q, _ in calls], self.mbq)
        r = R.call_indel(alleles, hp, self.h, p.str, p.input_str())          # callIndel (:265-361)
        if r is not None:
            al, typ, qs, c = r
            if c.undecided() or c.homref() or self.minq > c.gq:
                r = None
        if r is None:
            if not p.input_str() and p.new_str:
                p.str = p.new_str = False
            return                                              # (the SNV fallback: an SNV call or none)
        al, typ, qs, c = r
        c.update_cn(self.ploidy)                                # updateAllelesCopyNumberFromCounts(normalPloidy)
        self.records.append(f"{p.seq}\t{p.pos}\t{al[0]}\t{','.join(al[1:])}\t{qs}\t{typ}\t{R.genotype_fields(c, self.ploidy)}")
        self.last_indel_end = p.pos + len(al[0]) - 1


class PopulationListener:
    """MultisampleVariantsDetector.onPileup in discovery mode, ploidy < 3: the indel / STR records as
    "POS REF ALT QS TYPE" + every sample's GT:PL:GQ:DP:ADP:ACN (samples = [(id, [read groups in HashSet order])])"""

    def __init__(self, genome, samples, het_rate=0.001, min_quality=40, ploidy=2, max_base_qs=30, call_embedded=False,
                 ignore_lower=False):
        self.g, self.samples, self.h, self.minq, self.ploidy = genome, samples, het_rate, min_quality, ploidy
        self.mbq, self.emb, self.lower = max_base_qs, call_embedded, ignore_lower
        self.last_indel_end = 0
        self.records = []

    def on_sequence_start(self, seq):
        self.last_indel_end = 0

    def on_sequence_end(self, seq):
        pass

    def genotype(self, p, alleles):                             # genotypeVariant (:674-693) over an indel variant
        calls, vqs = [], 0
        for _, rgs in self.samples:
            sc = p.allele_calls(len(alleles[0]), rgs)
            hp = R.indel_helper(alleles, [(c, q) for c, q, _ in sc], self.mbq)
            c = R.call_indel(alleles, hp, self.h, False, False, variant=alleles)
            if isinstance(c, tuple):
                c = c[3]
            c.update_cn(self.ploidy)
            if 40 > c.gq:                                       # the fresh listener's DEF_MIN_QUALITY
                c.make_undecided()
            if not c.undecided() and not c.homref() and c.gq > vqs:
                vqs = c.gq
            calls.append(c)
        return calls, vqs

    def on_pileup(self, p):
        if p.input_str():
            self.last_indel_end = p.pos + p.span - 1
        elif p.pos <= self.last_indel_end:
            p.embedded = True
        ref = reference_allele(p, self.g, self.emb, self.lower)
        if ref is None or len(ref) <= 1:
            return
        calls = p.allele_calls(len(ref))
        alleles = R.cluster_alleles([(c, q) for c, q, _ in calls], ref, self.mbq)
        hp = R.indel_helper(alleles, [(c, q) for c, q, _ in calls], self.mbq)
        variant = None
        if len(alleles) > 1 and hp.total > 0:                   # createIndelVariantPool (:333-338)
            variant = list(alleles)
            while len(variant) > 2:                             # discoverPopulationIndel (:616-634)
                if not p.input_str() and all(len(a) == len(variant[0]) for a in variant):
                    variant = None
                    break
                gcalls, vqs = self.genotype(p, variant)
                if vqs < self.minq:
                    variant = None
                    break
                called = {variant[0]}                           # makeNewVariant (:642-656): a TreeSet
                for c in gcalls:
                    called |= {variant[k] for k in c.called}
                if len(variant) != len(called):
                    variant = [variant[0]] + [a for a in sorted(called) if a != variant[0]]
                else:
                    break
        if variant is None:
            if not p.input_str() and p.new_str:
                p.str = p.new_str = False
            return                                              # (the SNV fallback)
        typ = "STR" if p.str else "INDEL"
        gcalls, vqs = self.genotype(p, variant)
        if vqs == 0 or vqs < self.minq:
            return
        fields = "\t".join(R.genotype_fields(c, self.ploidy) for c in gcalls)
        self.records.append(f"{p.seq}\t{p.pos}\t{variant[0]}\t{','.join(variant[1:])}\t{vqs}\t{typ}\t{fields}")
        self.last_indel_end = p.pos + len(variant[0]) - 1


def run(sam, fasta_seqs, detector="single", samples=None, known_strs=None, max_alns_per_start=5, events=None, **opts):
    """SAM + reference -> (trace lines, sorted alignment lines, non-SNV records)"""
    genome = Genome(fasta_seqs)
    inputs = None
    if known_strs is not None:
        inputs = non_redundant_strs(genome, [n for n, _ in fasta_seqs], known_strs)
    real = Realigner(genome, inputs, events)
    if detector == "single":
        lst = SingleSampleListener(genome, **opts)
    else:
        lst = PopulationListener(genome, samples, **opts)
    gen = Generator([real, lst], max_alns_per_start)
    for a in read_sam(sam):
        gen.process_alignment(a)
    gen.notify_end()
    alns = sorted(gen.retired + gen.pending, key=lambda a: a.id)
    trace = ["\t".join(str(x) for x in t) for t in real.trace]
    final = [f"A\t{a.id}\t{a.first}\t{a.last}\t{a.cigar()}\t{a.ign_start}\t{a.ign_end}" for a in alns]
    return trace, final, lst.records
