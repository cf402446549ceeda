// realign.cpp -- the indel realigner's regions (realign.hpp): a replay of the pileup sweep with
// IndelRealignerPileupListener's alignment edits, the span calls' allele clusters and indel genotypes, and the
// listener's sequential span rules.  Host code: a region is a few hundred positions around reads with indels, its
// edits are sequential by nature (each pileup sees the alignments as edited so far); its span-1 columns go to
// the device with every other position's (KP).
//
//   the alignment model          alignments/ReadAlignment.java:613-644,747-871,989-1044,1101-1153,1351-1478
//   the realigner                discovery/IndelRealignerPileupListener.java:85-578
//   allele calls of a span       discovery/PileupRecord.java:126-152
//   clustering                   discovery/AlleleCallClustersBuilder.java:72-261
//   indel counts                 discovery/CountsHelper.java:96-105,253-304,384-396,410-495
//   callIndel                    discovery/VariantDiscoverySNVQAlgorithm.java:223-361
//   span rules, copy numbers     discovery/SingleSampleVariantPileupListener.java:146-273,
//                                variants/CalledGenomicVariantImpl.java:228-282
//   the record                   vcf/VCFFileWriter.java:44-308 (FORMAT GT:PL:GQ:DP:ADP:ACN)
#include "realign.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <set>

#include "engine.hpp"

namespace ngsep {

int64_t java_round(double x);
int java_phred(double p);

namespace {

enum { OP_H = 0, OP_D = 1, OP_I = 2, OP_M = 3, OP_P = 4, OP_N = 5, OP_S = 6, OP_X = 7 };
constexpr int kRegionBoundary = 100;      // DEF_REGION_BOUNDARY (IndelRealignerPileupListener.java:43)
constexpr int kMinBpGoodRefAln = 5;       // minBPForGoodRefAln (:46)
constexpr int kMaxBpRealignmentEnd = 50;  // maxBPRealignmentEnd (:47)
constexpr int kCloseIndel = 2;            // basesToIgnoreCloseToIndel (ReadAlignment.java:115)
constexpr int kNumFreq = 501;             // CountsHelper.DEF_NUM_FREQUENCIES

inline int base_index(char ch) {
    switch (ch) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}
inline char upper(char ch) { return (ch >= 'a' && ch <= 'z') ? (char)(ch - 32) : ch; }

// PhredScoreHelper.calculateProbability (math/PhredScoreHelper.java:46-51)
inline double phred_prob(int q) { return q >= 255 ? 0.0 : std::pow(10.0, -0.1 * q); }

// CountsHelper's cache entries (CountsHelper.java:147-187) the indel path reads: logProbCacheError[q][j] and
// logProbCacheGT[f][q][j] (q >= DEF_MIN_BASE_QS; computed as the caches are)
inline double log_err(int q, int j) { return -0.1 * q - (j >= 2 ? std::log10((double)(j - 1)) : 0.0); }
inline double log_gt(double af, int q, int j) {
    const double e = phred_prob(q), s = 1 - e;
    return j == 0 ? std::log10(s) : std::log10(af * s + (1 - af) * e / (j - 1));
}

// ---- ReadAlignment ----
struct IndelEv {
    int32_t first, last, len;            // GenomicVariantImpl(refPos, refLast) with setLength(opLen), keyed by refPos
};

struct Aln {
    int32_t first, last, flags, read_length;
    std::vector<int32_t> ops;
    const char* chars;                   // nullptr: no characters (read_length of them otherwise)
    const char* quals;                   // nullptr: no qualities
    int32_t ignore_start, ignore_end;
    std::vector<int16_t> acl;            // alleleCallLength per read position
    std::vector<IndelEv> indels;         // indelCalls (TreeMap by refPos)
    int16_t sample = -1;                 // multisample: sample and read-group rank (RawRead)
    uint8_t rank = 0;
    int* edits = nullptr;                // replay_region's count of updates (its indel-position marks are then redrawn)
    std::vector<uint16_t> codes;         // per read position: the span-1 column entry (update())
    bool simple = false;                 // one M item over the whole read: read position = pos - first

    // updateAlleleCallsInfo (ReadAlignment.java:747-834)
    void update() {
        if (edits) ++*edits;
        simple = ops.size() == 1 && (ops[0] & 7) == OP_M && ops[0] / 8 == read_length;
        if (simple) {
            // one M item over the whole read: no indel, so only the ignored ends make no call (the loop below, reduced)
            acl.assign((size_t)std::max(read_length, 1), 0);
            indels.clear();
            for (int r = std::max(0, ignore_start); r < read_length && read_length - r > ignore_end; r++) acl[(size_t)r] = 1;
            fill_codes();
            return;
        }
        acl.assign((size_t)std::max(read_length, 1), 0);
        indels.clear();
        int refPos = first, readPos = 0;
        bool prevIndel = false;
        const int n = (int)ops.size();
        for (int i = 0; i < n; i++) {
            const int len = ops[i] / 8, op = ops[i] & 7;
            const bool cRef = op & 1, cRead = (op & 2) != 0;
            int nextOp = -1, nextLen = 0, nextReadCons = 0;
            bool nextIsIndel = false;
            if (i < n - 1) {
                nextOp = ops[i + 1] & 7;
                nextLen = ops[i + 1] / 8;
                nextIsIndel = nextOp == OP_D || nextOp == OP_I;
                nextReadCons = (nextOp & 2) ? nextLen : 0;
            }
            if (cRef) {
                if (cRead) {
                    for (int j = 0; j < len; j++) {
                        bool skip = readPos < ignore_start || (read_length - readPos) <= ignore_end;
                        skip = skip || (prevIndel && j < kCloseIndel);
                        skip = skip || (nextIsIndel && j < len - 1 && j >= len - kCloseIndel);
                        skip = skip || (nextIsIndel && j == len - 1 &&
                                        (readPos < kCloseIndel || read_length - readPos - nextReadCons < kCloseIndel));
                        const int readPosAfterIndel = readPos + nextReadCons + 1;
                        skip = skip || (nextIsIndel && j == len - 1 && read_length - readPosAfterIndel < ignore_end);
                        if (!skip && readPos < read_length) {
                            if (j == len - 1 && nextIsIndel) {
                                acl[(size_t)readPos] = (int16_t)(nextOp == OP_I ? nextLen + 2 : 2);
                                const int refLast = refPos + 1 + (nextOp != OP_I ? nextLen : 0);
                                if (!indels.empty() && indels.back().first == refPos) indels.pop_back();   // TreeMap.put
                                indels.push_back(IndelEv{refPos, refLast, nextLen});
                            } else {
                                acl[(size_t)readPos] = 1;
                            }
                        }
                        refPos++;
                        readPos++;
                    }
                } else {
                    refPos += len;
                }
            } else if (cRead) {
                readPos += len;
            }
            prevIndel = op == OP_D || op == OP_I;
        }
        fill_codes();
    }
    // every read position's span-1 column entry (replay_region's getAlleleCalls(1)): engine.hpp's code | negative
    // strand << 8, 0xFFFF where the read makes no span-1 call there
    void fill_codes() {
        codes.assign(acl.size(), 0xFFFF);
        if (!chars) return;
        // (code_table: the code of every (quality character, read character) pair, as the branches in its comment)
        const uint8_t(*T)[256] = code_table();
        const uint16_t strand = (flags & 0x10) ? 0x100 : 0;
        const unsigned char* qs = reinterpret_cast<const unsigned char*>(quals);
        const unsigned char* cs = reinterpret_cast<const unsigned char*>(chars);
        const int16_t* ac = acl.data();
        uint16_t* out = codes.data();
        for (int r = 0; r < read_length; r++)
            if (ac[r] == 1) out[r] = (uint16_t)(T[qs ? qs[r] : '+'][cs[r]] | strand);
    }
    // code_table()[qc][ch]: q = (byte) min(30, min(qc, 127) - 33) (setQualityScores cap); q <= 3: counted | max(q, 0);
    // a character that is not A/C/G/T: counted | q; else valid | base << 5 | q (engine.hpp codes)
    static const uint8_t (*code_table())[256] {
        static const auto* t = [] {
            static uint8_t tab[256][256];
            for (int qc0 = 0; qc0 < 256; qc0++) {
                const int qc = qc0 > 127 ? 127 : qc0;
                const int q = (int8_t)std::min(30, qc - 33);
                for (int ch = 0; ch < 256; ch++) {
                    const int b = base_index((char)ch);
                    uint8_t code;
                    if (q <= 3) code = (uint8_t)(kCodeCounted | (q < 0 ? 0 : q));
                    else if (b < 0) code = (uint8_t)(kCodeCounted | q);
                    else code = (uint8_t)(kCodeValid | (b << 5) | q);
                    tab[qc0][ch] = code;
                }
            }
            return &tab;
        }();
        return *t;
    }
    // the span-1 entry at reference position pos of an alignment of the pileup (first <= pos <= last), 0xFFFF for none
    uint16_t code_at(int pos) const {
        const int r = simple ? pos - first : read_pos(pos);
        return r < 0 ? (uint16_t)0xFFFF : codes[(size_t)r];
    }
    // getAlignedReadPosition (:842-871)
    int read_pos(int refPos) const {
        if (refPos < first || refPos > last) return -1;
        int curRef = first, curRead = 0;
        for (int32_t v : ops) {
            const int len = v / 8, op = v & 7;
            const bool cRef = op & 1, cRead = (op & 2) != 0;
            if (cRef && cRead) {
                if (refPos < curRef) return -1;
                if (curRef + len > refPos) {
                    const int ans = curRead + refPos - curRef;
                    return (ans < 0 || ans >= read_length) ? -1 : ans;
                }
            }
            if (cRef) curRef += len;
            if (cRead) curRead += len;
        }
        return -1;
    }
    const IndelEv* indel_at(int pos) const {             // getIndelCall (:1101-1106)
        for (const IndelEv& e : indels) {
            if (e.first == pos) return &e;
            if (e.first > pos) break;
        }
        return nullptr;
    }
    bool has_indels(int f, int l) const {                // hasIndelCalls (:1471-1478)
        for (const IndelEv& e : indels) if (e.first >= f && e.first <= l) return true;
        return false;
    }
    int soft_clip_start() const { return !ops.empty() && (ops.front() & 7) == OP_S ? ops.front() / 8 : 0; }   // :1351-1356
    int soft_clip_end() const { return !ops.empty() && (ops.back() & 7) == OP_S ? ops.back() / 8 : 0; }       // :1358-1363
    char qual(int rp) const { return quals ? quals[rp] : '+'; }
    // getAlleleCall(pos) (:989-1000): read offset, length in *len; -1 for none
    int call1(int pos, int* len) const {
        if (!chars) return -1;
        const int rp = read_pos(pos);
        if (rp < 0) return -1;
        const int l = acl[(size_t)rp];
        if (l == 0) return -1;
        *len = l;
        return rp;
    }
    // getAlleleCall(first, last) (:1008-1016), withinIgnoreRegions (:1042-1044)
    int call_range(int f, int l, int* len) const {
        const int rf = read_pos(f), rl = read_pos(l);
        if (rf < 0 || rl < 0 || rl < rf) return -1;
        if (rf < ignore_start || read_length - rl <= ignore_end) return -1;
        *len = rl - rf + 1;
        return rf;
    }
    // moveIndelStart (:1114-1153)
    void move_indel_start(int indelRefPos, int newIndelRefPos) {
        const int displacement = newIndelRefPos - indelRefPos;
        if (displacement == 0) return;
        std::vector<int32_t> na(ops.size(), 0);
        int indelNextIdx = -1, currentRefPos = first;
        const int n = (int)ops.size();
        for (int i = 0; i < n; i++) {
            const int length = ops[i] / 8, op = ops[i] & 7;
            if ((op == OP_D || op == OP_I) && currentRefPos == indelRefPos + 1) {
                if (i == 0 || i == n - 1) return;
                const int opBefore = ops[i - 1] & 7, lenBefore = ops[i - 1] / 8;
                if (!(opBefore & 2) || !(opBefore & 1) || lenBefore <= -displacement) return;
                const int opAfter = ops[i + 1] & 7, lenAfter = ops[i + 1] / 8;
                if (!(opAfter & 2) || !(opAfter & 1) || lenAfter <= displacement) return;
                na[(size_t)i - 1] = (lenBefore + displacement) * 8 + opBefore;
                na[(size_t)i] = ops[i];
                na[(size_t)i + 1] = (lenAfter - displacement) * 8 + opAfter;
                indelNextIdx = i + 1;
            } else if (i != indelNextIdx) {
                na[(size_t)i] = ops[i];
            }
            if (op & 1) currentRefPos += length;
        }
        if (indelNextIdx < 0) return;
        ops.swap(na);
        update();
    }
    // the unknown stretch between a realigned end match and the rest: equal lengths (M), an insertion or a deletion
    static void push_unknown(std::vector<int32_t>& L, int unknownBpRead, int unknownBpRef) {
        const int difference = unknownBpRead - unknownBpRef;
        if (difference == 0) {
            if (unknownBpRead > 0) L.push_back(unknownBpRead * 8 + OP_M);
        } else if (difference > 0) {
            L.push_back(difference * 8 + OP_I);
            if (unknownBpRef > 0) L.push_back(unknownBpRef * 8 + OP_M);
        } else {
            L.push_back(-difference * 8 + OP_D);
            if (unknownBpRead > 0) L.push_back(unknownBpRead * 8 + OP_M);
        }
    }
    // realignStart (:1372-1418; the new alignment list is not collapsed)
    void realign_start(int newAlnFirst, int firstMatchLength, int refPosAfter, int alnReadPosAfter) {
        std::vector<int32_t> L{firstMatchLength * 8 + OP_M};
        const int nextRefPos = newAlnFirst + firstMatchLength;
        const int unknownBpRead = alnReadPosAfter - firstMatchLength, unknownBpRef = refPosAfter - nextRefPos;
        if (unknownBpRef < 0 || unknownBpRead < 0) return;   // "Can not realign start"
        push_unknown(L, unknownBpRead, unknownBpRef);
        int currentReadPos = 0;
        bool copy = false;
        for (int32_t v : ops) {
            const int length = v / 8, op = v & 7;
            if (copy) L.push_back(v);
            if (op & 2) {
                if (!copy && alnReadPosAfter < currentReadPos + length) {
                    copy = true;
                    L.push_back((currentReadPos + length - alnReadPosAfter) * 8 + op);
                }
                currentReadPos += length;
            }
        }
        first = newAlnFirst;
        ops.swap(L);
        update();
    }
    // realignEnd (:1427-1469)
    void realign_end(int refPosBefore, int alnPosBefore, int finalMatchRefStart, int finalMatchLength) {
        const int bpEndRead = read_length - alnPosBefore - 1;
        std::vector<int32_t> L;
        int currentReadPos = 0;
        bool copy = true;
        for (int32_t v : ops) {
            const int length = v / 8, op = v & 7;
            if (op & 2) {
                if (copy && alnPosBefore < currentReadPos + length) {
                    const int diff = currentReadPos + length - alnPosBefore - 1;
                    L.push_back((length - diff) * 8 + op);
                    copy = false;
                }
                currentReadPos += length;
            }
            if (copy) L.push_back(v);
        }
        const int unknownBpRef = finalMatchRefStart - refPosBefore - 1, unknownBpRead = bpEndRead - finalMatchLength;
        if (unknownBpRef < 0 || unknownBpRead < 0) return;   // "Can not realign end"
        push_unknown(L, unknownBpRead, unknownBpRef);
        L.push_back(finalMatchLength * 8 + OP_M);
        ops.swap(L);
        last = finalMatchRefStart + finalMatchLength - 1;
        update();
    }
};

// java.util.HashMap<Integer, V> iteration order for small non-negative keys: bucket (h ^ h >>> 16) & (cap - 1),
// capacity grown from 16 while size > 0.75 cap, insertion order inside a bucket
std::vector<int> hashmap_order(const std::vector<int>& keys) {
    int cap = 16;
    while ((int)keys.size() > cap * 3 / 4) cap *= 2;
    std::vector<int> ord(keys.size());
    for (size_t i = 0; i < ord.size(); i++) ord[i] = (int)i;
    auto bucket = [&](int k) { const unsigned u = (unsigned)k; return (u ^ (u >> 16)) & (unsigned)(cap - 1); };
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return bucket(keys[(size_t)a]) < bucket(keys[(size_t)b]); });
    return ord;
}

int hamming(const char* a, const char* b, int n) {   // HammingSequenceDistanceMeasure (sequences/:42-50)
    int d = 0;
    for (int i = 0; i < n; i++) d += a[i] != b[i];
    return d;
}
// makeHammingConsensus (AlleleCallClustersBuilder.java:79-91): per column the most frequent character, ties to the
// smallest (CountsRankHelper over a TreeMap: stable by count)
std::string hamming_consensus(const std::vector<const std::string*>& seqs) {
    const size_t l = seqs[0]->size();
    std::string out(l, ' ');
    for (size_t i = 0; i < l; i++) {
        int cnt[256] = {0};
        for (const std::string* s : seqs) cnt[(unsigned char)(*s)[i]]++;
        int best = -1;
        for (int ch = 0; ch < 256; ch++) if (cnt[ch] > 0 && (best < 0 || cnt[ch] > cnt[best])) best = ch;
        out[i] = (char)best;
    }
    return out;
}

// ---- IndelRealignerPileupListener ----
class Realigner {
public:
    Realigner(const std::string& seq) : seq_(seq) {}

    // onPileup (:85-126): the pileup's reference span
    // var: the input variant intersectWithVariants found at pos (:137-153), or null.  At its first position the span
    // is the variant's and the pileup an STR when the variant is one (:90-95); inside it the pileup is embedded
    // (:96-98, *embedded)
    int on_pileup(const std::vector<Aln*>& alns, int pos, const StrVar* var, bool* is_str, bool* is_new_str, bool* embedded) {
        int span = 1, predictedEnd = pos;
        if (var) {
            if (var->first == pos) {
                if (var->str) *is_str = true;
                span = var->last - var->first + 1;
                predictedEnd = var->last;
            } else {
                *embedded = true;
            }
        } else {
            int maxLen = 0, maxSpan = 0;
            for (const Aln* a : alns)
                if (const IndelEv* e = a->indel_at(pos)) {
                    maxLen = std::max(maxLen, e->len);
                    maxSpan = std::max(maxSpan, e->last - e->first + 1);
                }
            if (maxLen > 0) predictedEnd = pos + std::max(maxLen, maxSpan) + 1;
        }
        if (predictedEnd <= pos) return span;
        const int c = conciliate(alns, pos, predictedEnd, var != nullptr, is_str, is_new_str);
        return c > 0 ? c : span;
    }

private:
    const std::string& seq_;

    // ReferenceGenome.getReference(first, last) upper-cased; false when out of the sequence
    bool ref(int f, int l, std::string* out) const {
        if (f < 1 || l > (int)seq_.size() || l < f - 1) return false;
        out->assign(seq_, (size_t)f - 1, (size_t)(l - f + 1));
        for (char& ch : *out) ch = upper(ch);
        return true;
    }

    // checkMonoNucleotide (:365-391); checkDinucleotide is a stub returning 0 (:393-396)
    static int tandem_repeat(const char* s, int len) {
        int counts[4] = {0, 0, 0, 0};
        const int minLength = 5;
        int i = 0;
        while (i < len && i < minLength) { const int j = base_index(s[i]); if (j >= 0) counts[j]++; i++; }
        int baseIdx = -1;
        for (int j = 0; j < 4; j++) if (counts[j] >= i - 1) { baseIdx = j; break; }
        if (baseIdx == -1 || i < minLength) return 0;
        while (i < len && counts[baseIdx] >= i - 1) { const int j = base_index(s[i]); if (j >= 0) counts[j]++; i++; }
        i--;
        return base_index(s[i - 1]) != baseIdx ? i - 1 : i;
    }

    // lookForNewSTR (:315-349)
    int new_str(int pos, const std::vector<Aln*>& alns, int maxLength) const {
        if (alns.empty()) return 0;
        std::string r;
        if (ref(pos + 1, alns.back()->last, &r)) {
            const int l = tandem_repeat(r.data(), (int)r.size());
            if (l > 0) return l + 2;
        }
        for (const Aln* a : alns) {
            const IndelEv* e = a->indel_at(pos);
            if (!e || e->len != maxLength) continue;
            const int span = e->last - e->first + 1;
            int lengthTR = 0;                       // checkTandemRepeat(aln, pos) (:351-357)
            const int rf = a->read_pos(pos);
            if (rf >= 0 && a->chars) {
                std::string sub(a->chars + rf + 1, (size_t)(a->read_length - rf - 1));
                for (char& ch : sub) ch = upper(ch);
                lengthTR = tandem_repeat(sub.data(), (int)sub.size());
            }
            if (lengthTR > 0) return e->len >= span ? e->len + 2 : lengthTR + span;
        }
        return 0;
    }

    // calculateInsertedConsensusSequence (:528-555)
    static bool inserted_consensus(const std::vector<Aln*>& alns, int eventFirst, std::string* out) {
        std::vector<int> keys;
        std::vector<std::vector<std::string>> groups;
        for (const Aln* a : alns) {
            if (!a->indel_at(eventFirst)) continue;
            int len = 0;
            const int off = a->call1(eventFirst, &len);
            if (off < 0) continue;
            const int il = len - 2;
            if (il <= 0) continue;
            auto it = std::find(keys.begin(), keys.end(), il);
            size_t g = (size_t)(it - keys.begin());
            if (it == keys.end()) { keys.push_back(il); groups.emplace_back(); }
            groups[g].push_back(std::string(a->chars + off + 1, (size_t)il));
        }
        if (keys.empty()) return false;
        const std::vector<int> ord = hashmap_order(keys);
        int best = -1;
        size_t nbest = 0;
        for (int i : ord) if (groups[(size_t)i].size() > nbest) { nbest = groups[(size_t)i].size(); best = i; }
        std::vector<const std::string*> v;
        for (const std::string& s : groups[(size_t)best]) v.push_back(&s);
        *out = hamming_consensus(v);
        return true;
    }

    // calculateDeletionConsensusLength (:557-578)
    static int deletion_consensus_length(const std::vector<Aln*>& alns, int eventFirst) {
        std::vector<int> keys, counts;
        for (const Aln* a : alns) {
            const IndelEv* e = a->indel_at(eventFirst);
            if (!e) continue;
            const int inner = e->last - e->first - 1;
            auto it = std::find(keys.begin(), keys.end(), inner);
            if (it == keys.end()) { keys.push_back(inner); counts.push_back(1); }
            else counts[(size_t)(it - keys.begin())]++;
        }
        int answer = 0, max = 0;
        for (int i : hashmap_order(keys)) if (max < counts[(size_t)i]) { answer = keys[(size_t)i]; max = counts[(size_t)i]; }
        return answer;
    }

    // processEndsOfAlignments (:400-526)
    void process_ends(const std::vector<Aln*>& alns, int eventFirst, int eventLast) {
        std::string seqBefore, seqAfter, seqWithin;
        const bool hasBefore = ref(eventFirst - kRegionBoundary, eventFirst, &seqBefore);
        const bool hasAfter = ref(eventLast, eventLast + kRegionBoundary, &seqAfter);
        const bool hasWithin = eventFirst != eventLast - 1 && ref(eventFirst + 1, eventLast - 1, &seqWithin);
        const std::string refBefore = hasBefore ? seqBefore + (hasWithin ? seqWithin : "") : "";
        const std::string refAfter = hasAfter ? (hasWithin ? seqWithin : "") + seqAfter : "";
        std::string altBefore = seqBefore, altAfter = seqAfter, ins;
        int offset;
        if (inserted_consensus(alns, eventFirst, &ins)) {
            offset = (int)ins.size();
            if (hasBefore) altBefore = seqBefore + ins + (hasWithin ? seqWithin : "");
            if (hasAfter) altAfter = ins + (hasWithin ? seqWithin : "") + seqAfter;
        } else {
            int deletionLength = std::min(deletion_consensus_length(alns, eventFirst), eventLast - eventFirst - 1);
            offset = -deletionLength;
            if (hasWithin && deletionLength < (int)seqWithin.size()) {
                const std::string rest = seqWithin.substr((size_t)std::max(deletionLength, 0));
                if (hasBefore) altBefore = seqBefore + rest;
                if (hasAfter) altAfter = rest + seqAfter;
            }
        }
        const int lRefB = (int)refBefore.size(), lAltB = hasBefore ? (int)altBefore.size() : 0;
        const int lRefA = (int)refAfter.size(), lAltA = hasAfter ? (int)altAfter.size() : 0;
        const int bpGood = std::max(offset, kMinBpGoodRefAln);
        for (Aln* a : alns) {
            const int alnFirst = a->first, alnLast = a->last;
            const bool indelBefore = a->has_indels(alnFirst, eventFirst - 1);
            const bool indelAfter = a->has_indels(eventLast + 1, alnLast);
            bool trimStart = eventFirst - alnFirst < bpGood && !indelBefore;
            const int readPosAfter = a->read_pos(eventLast);
            if (!indelBefore && hasBefore && readPosAfter >= bpGood && readPosAfter - offset <= kMaxBpRealignmentEnd &&
                readPosAfter < lRefB && readPosAfter < lAltB && !a->indel_at(eventFirst) && a->chars) {
                const int refDist = hamming(refBefore.data() + lRefB - readPosAfter, a->chars, readPosAfter);
                const int altDist = hamming(altBefore.data() + lAltB - readPosAfter, a->chars, readPosAfter);
                const int newAlnFirst = eventLast - readPosAfter + 1 + offset;
                const int firstMatchLength = eventFirst - newAlnFirst + 1;
                if (altDist < refDist && altDist < 3 && firstMatchLength >= kMinBpGoodRefAln) {
                    a->realign_start(newAlnFirst, firstMatchLength, eventLast, readPosAfter);
                    trimStart = false;
                }
            }
            if (trimStart) {
                const int ignoreBP = eventLast - alnFirst + 1 + a->soft_clip_start();
                const int bp = (int8_t)std::max(a->ignore_start, ignoreBP);     // (byte) cast
                if (a->ignore_start != bp) { a->ignore_start = bp; a->update(); }
            }
            bool trimEnd = alnLast - eventLast < bpGood && !indelAfter;
            const int readPosBefore = a->read_pos(eventFirst);
            const int readSuffixLength = readPosBefore >= 0 ? a->read_length - readPosBefore - 1 : 0;
            if (!indelAfter && hasAfter && readSuffixLength >= bpGood && readSuffixLength - offset <= kMaxBpRealignmentEnd &&
                readSuffixLength < lRefA && readSuffixLength < lAltA && (!a->indel_at(eventFirst) || readPosAfter < 0) && a->chars) {
                const char* suffix = a->chars + readPosBefore + 1;
                const int refDist = hamming(refAfter.data(), suffix, readSuffixLength);
                const int altDist = hamming(altAfter.data(), suffix, readSuffixLength);
                const int finalMatchLength = readSuffixLength - (offset > 0 ? offset : 0);
                const int newEventLast = eventFirst + 1 - (offset < 0 ? offset : 0);
                if (altDist < refDist && altDist < 3 && finalMatchLength >= kMinBpGoodRefAln) {
                    a->realign_end(eventFirst, readPosBefore, newEventLast, finalMatchLength);
                    trimEnd = false;
                }
            }
            if (trimEnd) {
                const int ignoreBP = alnLast - eventFirst + 1 + a->soft_clip_end();
                const int bp = (int8_t)std::max(a->ignore_end, ignoreBP);
                if (a->ignore_end != bp) { a->ignore_end = bp; a->update(); }
            }
        }
    }

    // moveIndelStarts (:274-313)
    static int move_indel_starts(const std::vector<Aln*>& alns, int first, int last, int maxLength, int offset) {
        int answer = first + 1;
        for (Aln* a : alns) {
            for (const IndelEv e : a->indels)
                if (e.last >= first && e.first <= last) { a->move_indel_start(e.first, first + offset); break; }
            if (!a->indels.empty()) {
                int alnRefLast = first;
                for (const IndelEv& e : a->indels)
                    if (e.first >= first && e.first <= alnRefLast + maxLength) alnRefLast = e.last;
                answer = std::max(answer, alnRefLast);
            }
        }
        return answer;
    }

    // conciliateIndels (:165-216) with analyzeIndels (:229-265); the reference span if indels are called, else 0
    int conciliate(const std::vector<Aln*>& alns, int pos, int eventEnd, bool fixedEvent, bool* is_str, bool* is_new_str) {
        int answer = 0, maxLength = 0;                   // fixedEvent: varG != null (an input STR)
        const int nvotes = eventEnd - pos + 1;
        std::vector<int> votes((size_t)nvotes, 0), lengths;
        std::vector<Aln*> indelAlns;
        for (Aln* a : alns)
            for (const IndelEv& e : a->indels)
                if (e.last >= pos && e.first <= eventEnd) {
                    if (std::find(lengths.begin(), lengths.end(), e.len) == lengths.end()) lengths.push_back(e.len);
                    maxLength = std::max(maxLength, e.len);
                    const int i = e.first - pos;
                    if (i >= 0 && i < nvotes) votes[(size_t)i]++;
                    indelAlns.push_back(a);
                    break;
                }
        if (lengths.empty()) return 0;
        int maxI = 0;
        if (!fixedEvent) for (int i = 1; i < nvotes; i++) if (votes[(size_t)maxI] < votes[(size_t)i]) maxI = i;   // getIndexMaximum
        if (!fixedEvent && lengths.size() > 1) {
            const int span = new_str(pos, indelAlns, maxLength);
            if (span > 1) {
                maxI = 0;
                answer = span;
                eventEnd = pos + answer - 1;
                fixedEvent = true;
                *is_str = true;
                *is_new_str = true;
            }
        }
        const int predictedEnd = move_indel_starts(indelAlns, pos, eventEnd, maxLength, maxI);
        if (maxI > 0) return answer;
        if (!fixedEvent && predictedEnd != eventEnd) {
            eventEnd = predictedEnd;
            answer = eventEnd - pos + 1;
        }
        process_ends(alns, pos, eventEnd);
        return answer;
    }
};

// ---- allele calls of a span and their clusters ----
struct SpanCall {
    std::string allele, qual;
};

// PileupRecord.getAlleleCalls(span, null) (PileupRecord.java:126-152); span 1 keeps the one-base calls only (:143)
void span_calls(const std::vector<Aln*>& alns, int pos, int span, std::vector<SpanCall>& out) {
    out.clear();
    for (const Aln* a : alns) {
        int l1 = 0;
        const int o1 = a->call1(pos, &l1);
        if (o1 < 0) continue;
        if (span == 1) {
            if (l1 > 1) continue;
            SpanCall c;
            c.allele.assign(1, a->chars[o1]);
            c.qual.assign(1, a->qual(o1));
            out.push_back(std::move(c));
            continue;
        }
        int len = 0;
        const int off = a->call_range(pos, pos + span - 1, &len);
        if (off < 0) continue;
        SpanCall c;
        c.allele.assign(a->chars + off, (size_t)len);
        c.qual.resize((size_t)len);
        for (int i = 0; i < len; i++) c.qual[(size_t)i] = a->qual(off + i);
        out.push_back(std::move(c));
    }
}

// calculateHetPosteriors (AlleleCallClustersBuilder.java:223-261): a CountsHelper over A,C,G,T (h proportion 0.5,
// DEF_MAX_BASE_QS) per variable column, posteriors with DEF_HETEROZYGOSITY_RATE_DIPLOID
void het_posteriors(const std::vector<const SpanCall*>& calls, const std::string& consensus, int maxBaseQS, std::vector<double>& ans) {
    ans.assign(consensus.size(), 0.0);
    for (size_t i = 0; i < consensus.size(); i++) {
        const char ch = consensus[i];
        const int idxC = base_index(ch);
        if (idxC < 0) continue;
        bool variable = false;
        for (const SpanCall* c : calls) if (c->allele[i] != ch) { variable = true; break; }
        if (!variable) continue;
        // CountsHelper.updateCounts (CountsHelper.java:209-251), 4 alleles, f = g = round(0.5 * 500) = 250
        double L[4][4] = {{0}};
        for (const SpanCall* c : calls) {
            int q = c->qual[i] - 33;
            if (q > maxBaseQS) q = maxBaseQS;
            const int8_t qq = (int8_t)q;
            if (qq <= 3) continue;
            const int qc = std::min<int>(qq, 30);
            const int index = base_index(c->allele[i]);
            if (index < 0) continue;
            const double A = log_gt(0.5, qc, 0), H = log_gt(0.5, qc, 4), E = log_err(qc, 4);
            for (int a = 0; a < 4; a++) {
                L[a][a] += a == index ? A : E;
                for (int b = 0; b < 4; b++)
                    if (a != b) L[a][b] += (a == index || b == index) ? H : E;
            }
        }
        // getPosteriorProbabilities(0.001) (:410-443) + calculatePosteriorProbabilities (:472-495)
        const double h = 0.001, lph = std::log10(h / 12), lpo = std::log10((1 - h) / 4);
        double ev[16];
        int k = 0;
        for (int a = 0; a < 4; a++) {
            ev[k++] = L[a][a] + lpo;
            for (int b = 0; b < 4; b++) if (a != b) ev[k++] = L[a][b] + lph;
        }
        double logMax = 1;
        for (int t = 0; t < 16; t++) if (logMax > 0 || logMax < ev[t]) logMax = ev[t];
        double tot = 0;
        for (int t = 0; t < 16; t++) { ev[t] -= logMax; ev[t] = ev[t] < -20 ? 0.0 : std::pow(10.0, ev[t]); tot += ev[t]; }
        double post[4][4];
        k = 0;
        for (int a = 0; a < 4; a++) {
            post[a][a] = ev[k++] / tot;
            for (int b = 0; b < 4; b++) if (a != b) post[a][b] = ev[k++] / tot;
        }
        for (int b = 0; b < 4; b++) {
            const double hp = post[idxC][b] + post[b][idxC];
            if (b != idxC && hp > ans[i]) ans[i] = hp;
        }
    }
}

// CountsRankHelper<String>.selectBest(max) (math/CountsRankHelper.java:31-51): by count, ties in TreeMap order
std::vector<std::string> select_best(const std::vector<std::string>& items, int max) {
    std::map<std::string, int> cnt;
    for (const std::string& s : items) cnt[s]++;
    std::vector<std::pair<std::string, int>> v(cnt.begin(), cnt.end());
    std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
    std::vector<std::string> out;
    for (int i = 0; i < max && i < (int)v.size(); i++) out.push_back(v[(size_t)i].first);
    return out;
}

// splitAllelesByVariantSites (:165-221)
void split_alleles(const std::vector<const SpanCall*>& calls, const std::string& consensus, int maxBaseQS, std::vector<std::string>& answer) {
    std::vector<double> hp;
    het_posteriors(calls, consensus, maxBaseQS, hp);
    std::vector<int> sites;
    for (size_t i = 0; i < consensus.size(); i++) if (hp[i] >= 0.51) sites.push_back((int)i);   // DEF_MIN_HET_POSTERIOR
    if (sites.empty()) { answer.push_back(consensus); return; }
    const int m = (int)sites.size();
    std::vector<std::string> haps(calls.size());
    for (size_t i = 0; i < calls.size(); i++) {
        haps[i].resize((size_t)m);
        for (int j = 0; j < m; j++) haps[i][(size_t)j] = calls[i]->allele[(size_t)sites[(size_t)j]];
    }
    const int maxHaps = m > 3 ? std::min(10, m / 2 + 1) : 2;
    for (const std::string& sel : select_best(haps, maxHaps)) {
        std::vector<const std::string*> seqs;
        for (size_t i = 0; i < calls.size(); i++) if (haps[i] == sel) seqs.push_back(&calls[i]->allele);
        if (!seqs.empty()) answer.push_back(hamming_consensus(seqs));
    }
}

// clusterAlleleCalls (:72-141): the reference first, then the other alleles in TreeSet order
std::vector<std::string> cluster_alleles(const std::vector<SpanCall>& calls, const std::string& reference, int maxBaseQS) {
    std::vector<size_t> lens;
    for (const SpanCall& c : calls)
        if (std::find(lens.begin(), lens.end(), c.allele.size()) == lens.end()) lens.push_back(c.allele.size());
    std::vector<std::string> set;
    const double minCount = 0.2 * (double)calls.size();     // filterLengthClusters (:147-157)
    for (size_t l : lens) {
        std::vector<const SpanCall*> group;
        for (const SpanCall& c : calls) if (c.allele.size() == l) group.push_back(&c);
        if (lens.size() >= 3 && !(minCount <= (double)group.size())) continue;
        const int nsugg = l == reference.size() ? 1 : 0;
        if ((int)group.size() < 5 * nsugg) { set.push_back(reference); continue; }
        std::vector<const std::string*> al;
        for (const SpanCall* c : group) al.push_back(&c->allele);
        const std::string consensus = hamming_consensus(al);
        if (l < 4 || group.size() < 10) {
            if (nsugg) set.push_back(reference);
            set.push_back(consensus);
        } else {
            split_alleles(group, consensus, maxBaseQS, set);
        }
    }
    std::set<std::string> tree(set.begin(), set.end());
    tree.insert(reference);
    std::vector<std::string> alleles{reference};
    for (const std::string& s : tree) if (s != reference) alleles.push_back(s);
    return alleles;
}

// LogMath.logSum (math/LogMath.java:38-44)
inline double log_sum(double a, double b) {
    if (a - b > 20) return a;
    if (b - a > 20) return b;
    return a + std::log10(1 + std::pow(10.0, b - a));
}

// CountsHelper over indel alleles: calculateCountsIndel + updateCountsIndel (CountsHelper.java:96-105,253-304) with
// calculateLogCond (:384-396); logc is n x n row-major (not symmetric)
struct IndelCounts {
    int n = 0, total = 0;
    std::vector<int> counts;
    std::vector<double> logc;
};
void indel_counts_f(const std::vector<std::string>& alleles, const std::vector<SpanCall>& calls, int max_base_qs, double freq,
                    IndelCounts& h) {
    const int n = (int)alleles.size();
    const int maxBaseQS = (int8_t)max_base_qs > 0 ? (int8_t)max_base_qs : 30;
    const int f = (int)java_round(freq * kNumFreq);                    // (:256: 501, not 500)
    const double af0 = std::log10((double)f / (kNumFreq - 1)), af1 = std::log10(1 - (double)f / (kNumFreq - 1));
    const double E = std::log10(0.0001);                                  // DEF_LOG_ERROR_PROB_INDEL (:48)
    h.n = n;
    h.total = 0;
    h.counts.assign((size_t)n, 0);
    h.logc.assign((size_t)n * n, 0.0);
    std::vector<double> lca((size_t)n);
    for (const SpanCall& c : calls) {
        h.total++;
        int index = -1;
        for (int i = 0; i < n; i++) if (alleles[(size_t)i] == c.allele) { index = i; break; }
        int bestIndex = -1;
        for (int i = 0; i < n; i++) {
            if (alleles[(size_t)i].size() == c.allele.size()) {
                double lc = 0;
                for (size_t k = 0; k < c.allele.size(); k++) {
                    int q = c.qual[k] - 33;
                    if (q > maxBaseQS) q = maxBaseQS;
                    q = (int8_t)q;
                    if (q < 3) continue;                                   // DEF_MIN_BASE_QS
                    lc += alleles[(size_t)i][k] == c.allele[k] ? log_gt(0.0, q, 0) : log_err(q, 4);
                }
                lca[(size_t)i] = std::max(lc, E);
                if (lca[(size_t)i] > E && (bestIndex == -1 || lca[(size_t)bestIndex] < lca[(size_t)i])) bestIndex = i;
            } else {
                lca[(size_t)i] = E;
            }
        }
        if (index >= 0 && bestIndex >= 0 && bestIndex != index) index = std::min(index, bestIndex);
        else if (index < 0 && bestIndex >= 0) index = bestIndex;
        if (index >= 0) h.counts[(size_t)index]++;
        for (int i = 0; i < n; i++) {
            h.logc[(size_t)(i * n + i)] += lca[(size_t)i];
            for (int j = 0; j < n; j++) {
                if (i == j) continue;
                double& v = h.logc[(size_t)(i * n + j)];
                if (j == index) v += log_sum(af0 + lca[(size_t)index], af1 + E);
                else if (i == index) v += log_sum(af1 + lca[(size_t)index], af0 + E);
                else v += E;
            }
        }
    }
}

void indel_counts(const std::vector<std::string>& alleles, const std::vector<SpanCall>& calls, int max_base_qs, IndelCounts& h) {
    indel_counts_f(alleles, calls, max_base_qs, 0.5, h);
}

// CountsHelper.calculatePosteriorProbabilities (:472-495) in place
void posteriors(std::vector<double>& ev) {
    double logMax = 1, tot = 0;
    for (double v : ev) if (logMax > 0 || logMax < v) logMax = v;
    for (double& v : ev) { v -= logMax; v = v < -20 ? 0.0 : std::pow(10.0, v); tot += v; }
    for (double& v : ev) v /= tot;
}

// getPosteriorProbabilities (CountsHelper.java:410-443) + calculatePosteriorProbabilities (:472-495) over n alleles
void indel_posteriors(const IndelCounts& h, double het, std::vector<double>& post) {
    const int n = h.n;
    const double lph = std::log10(het / (n * (n - 1))), lpo = std::log10((1 - het) / n);
    std::vector<double> ev((size_t)n * n);
    post.assign((size_t)n * n, 0.0);
    int k = 0;
    for (int i = 0; i < n; i++) {
        ev[(size_t)k++] = h.logc[(size_t)(i * n + i)] + lpo;
        for (int j = 0; j < n; j++) if (i != j) ev[(size_t)k++] = h.logc[(size_t)(i * n + j)] + lph;
    }
    double logMax = 1, tot = 0;
    for (double v : ev) if (logMax > 0 || logMax < v) logMax = v;
    for (double& v : ev) { v -= logMax; v = v < -20 ? 0.0 : std::pow(10.0, v); tot += v; }
    k = 0;
    for (int i = 0; i < n; i++) {
        post[(size_t)(i * n + i)] = ev[(size_t)k++] / tot;
        for (int j = 0; j < n; j++) if (i != j) post[(size_t)(i * n + j)] = ev[(size_t)k++] / tot;
    }
}

// getIndexesMaxGenotype(post, 0) (VariantDiscoverySNVQAlgorithm.java:223-243)
void max_genotype(const std::vector<double>& post, int n, int* im0, int* im1) {
    *im0 = *im1 = 0;
    double probMax = post[0];
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            double gp = post[(size_t)(i * n + j)];
            if (i != j) gp += post[(size_t)(j * n + i)];
            if (gp > probMax + 0.01) { probMax = gp; *im0 = i; *im1 = j; }
        }
}

// calculateCountsIndel + callIndel (VariantDiscoverySNVQAlgorithm.java:265-361) with variant == null and the
// listener's filters; the VCF fields of a kept call
bool genotype_indel(const std::vector<std::string>& alleles, const std::vector<SpanCall>& calls, int pos, bool is_str,
                    bool is_input_str, const RealignParams& p, IndelCall* out) {
    const int n = (int)alleles.size();
    IndelCounts h;
    indel_counts(alleles, calls, p.max_base_qs, h);
    const std::vector<int>& counts = h.counts;
    const std::vector<double>& logc = h.logc;
    const int total = h.total;
    if (total == 0) return false;
    std::vector<double> post;
    indel_posteriors(h, p.het_rate, post);
    int im0 = 0, im1 = 0;
    max_genotype(post, n, &im0, &im1);
    int idx[3], na = 0;
    bool lengthChange = false;
    const size_t lref = alleles[0].size();
    idx[na++] = 0;
    if (im0 > 0 && im0 < n) { idx[na++] = im0; lengthChange |= alleles[(size_t)im0].size() != lref; }
    if (im1 > 0 && im1 != im0 && im1 < n) {
        idx[na++] = im1;
        lengthChange |= alleles[(size_t)im1].size() != lref;
        if (na == 3 && alleles[(size_t)im1].size() != alleles[(size_t)idx[1]].size()) lengthChange = true;
    }
    if (!lengthChange && !is_input_str) return false;                     // (:318: an input STR is called whatever its lengths)
    int ncalled, called[2];
    if (im1 != im0) { ncalled = 2; called[0] = na == 3 ? 1 : 0; called[1] = na == 3 ? 2 : 1; }
    else { ncalled = 1; called[0] = im0 == 0 ? 0 : 1; }
    double maxP = post[(size_t)(im0 * n + im1)];
    if (im0 != im1) maxP += post[(size_t)(im1 * n + im0)];
    const int gq = java_phred(1 - maxP), qs = java_phred(post[0]);
    if ((ncalled == 1 && called[0] == 0) || p.min_quality > gq) return false;   // discoverVariant (:221-227)
    // updateAllelesCopyNumberFromCounts(ploidy) (CalledGenomicVariantImpl.java:228-282)
    int acn[3] = {0, 0, 0};
    const int ploidy = p.ploidy;
    if (ploidy <= ncalled) {
        for (int i = 0; i < ncalled; i++) acn[called[i]] = 1;
    } else {
        int rc[2], trc = 0, sum = 0;
        for (int i = 0; i < ncalled; i++) { rc[i] = counts[(size_t)idx[called[i]]]; if (rc[i] == 0) rc[i] = 1; trc += rc[i]; }
        for (int i = 0; i < ncalled; i++) {
            const int64_t r = java_round((double)ploidy * rc[i] / trc);
            acn[called[i]] = (int)(r < 1 ? 1 : (int16_t)r);
            sum += acn[called[i]];
        }
        if (sum < ploidy) acn[called[0]] += ploidy - sum;
        else {
            int excess = sum - ploidy;
            for (int i = ncalled - 1; excess > 0 && i >= 0; i--) {
                const int rm = std::min(excess, acn[called[i]] - 1);
                acn[called[i]] -= rm;
                excess -= rm;
            }
        }
    }
    // the record (VCFFileWriter.printVCFRecord; FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV)
    std::string& o = out->line;
    o.clear();
    o += std::to_string(pos); o += "\t.\t"; o += alleles[0]; o += '\t';
    for (int i = 1; i < na; i++) { if (i > 1) o += ','; o += alleles[(size_t)idx[i]]; }
    o += '\t'; o += std::to_string(qs); o += "\t.\tTYPE="; o += is_str ? "STR" : "INDEL"; o += "\tGT:PL:GQ:DP:ADP:ACN\t";
    if (ncalled == 1) { o += std::to_string(called[0]); if (ploidy > 1) { o += '/'; o += std::to_string(called[0]); } }
    else { o += std::to_string(called[0]); o += '/'; o += std::to_string(called[1]); }
    o += ':';
    for (int j = 0; j < na; j++)
        for (int i = 0; i <= j; i++) {
            if (i > 0 || j > 0) o += ',';
            o += std::to_string((int)java_round(-10 * logc[(size_t)(idx[i] * n + idx[j])]));
        }
    o += ':'; o += std::to_string(gq); o += ':'; o += std::to_string(total); o += ':';
    for (int i = 0; i < na; i++) { if (i) o += ','; o += std::to_string(counts[(size_t)idx[i]]); }
    o += ':';
    if (ploidy == 0) o += '.';
    else for (int j = 0; j < na; j++) { if (j) o += ','; o += std::to_string(acn[j]); }
    o += '\n';
    out->pos = pos;
    out->last = pos + (int32_t)lref - 1;
    return true;
}

// ---- MultisampleVariantsDetector over a region (population mode) ----
// one sample's call of an indel variant (a CalledGenomicVariantImpl of SingleSampleVariantPileupListener
// .genotypeVariantSample, :361-391)
struct SampleIndelCall {
    int n_called = 0, called[2] = {0, 0}, gq = 0, dp = 0, total_cn = 0;
    bool report = false;
    std::vector<int> acn;
};

// CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts (variants/CalledGenomicVariantImpl.java:228-282)
void update_cn(SampleIndelCall& c, const std::vector<int>& counts, int total) {
    c.total_cn = total;
    std::fill(c.acn.begin(), c.acn.end(), 0);
    if (c.n_called == 0) return;
    if (c.n_called == 1 && c.called[0] == 0) { c.acn[0] = total; return; }
    const int nc = c.n_called;
    if (total <= nc) { for (int i = 0; i < nc; i++) c.acn[(size_t)c.called[i]] = 1; return; }
    if (!c.report) {
        const int def = total / nc;
        for (int i = 0; i < nc; i++) c.acn[(size_t)c.called[i]] = def;
        c.acn[(size_t)c.called[0]] += total - def * nc;
        return;
    }
    int rc[2] = {0, 0}, tr = 0;
    for (int i = 0; i < nc; i++) { rc[i] = counts[(size_t)c.called[i]]; if (rc[i] == 0) rc[i] = 1; tr += rc[i]; }
    int tc = 0;
    for (int i = 0; i < nc; i++) {
        const int64_t r = java_round((double)total * rc[i] / tr);
        c.acn[(size_t)c.called[i]] = std::max(1, (int)(int16_t)r);
        tc += c.acn[(size_t)c.called[i]];
    }
    if (tc < total) c.acn[(size_t)c.called[0]] += total - tc;
    else {
        int ex = tc - total;
        for (int i = nc - 1; ex > 0 && i >= 0; i--) {
            int& v = c.acn[(size_t)c.called[i]];
            const int rm = std::min(ex, v - 1);
            v -= rm;
            ex -= rm;
        }
    }
}

// the sample's span calls: PileupRecord.getAlleleCalls(span, sample.getReadGroups()) (:104-111) -- read groups in
// their HashSet order (rank), the pileup's order inside each
void sample_span_calls(const std::vector<Aln*>& pileup, int s, int pos, int span, std::vector<Aln*>& tmp, std::vector<SpanCall>& out) {
    tmp.clear();
    int maxrank = -1;
    for (const Aln* a : pileup) if (a->sample == s) maxrank = std::max<int>(maxrank, a->rank);
    for (int r = 0; r <= maxrank; r++)
        for (Aln* a : pileup) if (a->sample == s && a->rank == r) tmp.push_back(a);
    span_calls(tmp, pos, span, out);
}

// MultisampleVariantsDetector.genotypeVariant (:674-693) over an indel variant: genotypeVariantSample for every
// sample with a fresh listener (minQuality DEF_MIN_QUALITY 40): calculateCountsIndel over the variant's alleles,
// callIndel with the variant given (the maximum genotype's indexes taken as they are, :335-345),
// updateAllelesCopyNumberFromCounts(ploidy), makeUndecided below 40 (CalledGenomicVariantImpl.java:320-325).
// Returns the variant QS: the largest GQ of a decided, non-homozygous-reference call.
// genotypeVariantSample (SingleSampleVariantPileupListener.java:361-391) of an indel variant at ploidy < 3:
// calculateCountsIndel over the variant's alleles, callIndel with the variant given (the maximum genotype's indexes
// taken as they are, VariantDiscoverySNVQAlgorithm.java:335-345; no calls: an undecided call, :274-277),
// updateAllelesCopyNumberFromCounts(ploidy), makeUndecided below min_quality (CalledGenomicVariantImpl.java:320-325)
// genotypeVariantPool (SingleSampleVariantPileupListener.java:402-503) over an indel variant: CountsHelper
// .calculateCountsIndel per heterozygosity hypothesis (freq = k / haplotypes < 0.51, :410-414), the major allele by the
// first helper's counts (undecided, no report and no depth below `haplotypes` calls, :428-432), every other allele's
// homozygous-vs-heterozygous posteriors (:447-470), GQ and setAllelesCopyNumber (:482-498), the report from the chosen
// helper (:499-500; h = its counts and log-conditionals)
void genotype_pool_indel(const std::vector<std::string>& alleles, const std::vector<SpanCall>& sc, int haplotypes, double het,
                         int max_base_qs, SampleIndelCall& c, IndelCounts& h) {
    const int n = (int)alleles.size();
    c = SampleIndelCall();
    c.acn.assign((size_t)n, 0);
    const double step = 1.0 / (double)haplotypes;
    std::vector<double> freqs;
    for (double freq = step; freq < 0.51; freq += step) freqs.push_back(freq);
    const int nf = (int)freqs.size();
    std::vector<IndelCounts> hs((size_t)nf);
    for (int j = 0; j < nf; j++) indel_counts_f(alleles, sc, max_base_qs, freqs[(size_t)j], hs[(size_t)j]);
    const IndelCounts& h0 = hs[0];
    int major = 0;                                                       // NumberArrays.getIndexMaximum: first maximum
    for (int i = 1; i < n; i++) if (h0.counts[(size_t)major] < h0.counts[(size_t)i]) major = i;
    h = h0;
    if (h0.counts[(size_t)major] < haplotypes) {
        update_cn(c, h0.counts, haplotypes);                             // undecided.updateAllelesCopyNumberFromCounts
        return;
    }
    const double lph = std::log10(het), lpo = std::log10(1 - het);
    std::vector<double> terms((size_t)nf + 1);
    const double termHomozygous = h0.logc[(size_t)(major * n + major)] + lpo;
    double maxHetPosterior = 0, minHomoPosterior = 1, maxFreq = 0;
    int maxFreqIdx = 0, maxAlt = -1;
    for (int i = 0; i < n; i++) {
        if (i == major) continue;
        terms[0] = termHomozygous;
        for (int j = 0; j < nf; j++) terms[(size_t)j + 1] = hs[(size_t)j].logc[(size_t)(major * n + i)] + lph;
        posteriors(terms);
        int idxMax = 0;
        for (int j = 1; j <= nf; j++) if (terms[(size_t)idxMax] < terms[(size_t)j]) idxMax = j;
        if (idxMax == 0) minHomoPosterior = std::min(minHomoPosterior, terms[0]);
        else if (maxAlt == -1 || maxHetPosterior < terms[(size_t)idxMax]) {
            maxHetPosterior = terms[(size_t)idxMax];
            maxFreqIdx = idxMax - 1;
            maxFreq = freqs[(size_t)maxFreqIdx];
            maxAlt = i;
        }
    }
    if (maxAlt == -1) { c.n_called = 1; c.called[0] = major; }
    else { c.n_called = 2; c.called[0] = std::min(major, maxAlt); c.called[1] = std::max(major, maxAlt); }
    c.dp = h0.total;
    if (maxAlt == -1) {
        c.gq = java_phred(1 - minHomoPosterior);
        c.acn[(size_t)major] = haplotypes;
    } else {
        h = hs[(size_t)maxFreqIdx];
        // CountsHelper.getPosteriorProbabilities(hetRate, majorAlleleIdx) (CountsHelper.java:451-467)
        std::vector<double> ev((size_t)n);
        const double lh = std::log10(het / (n - 1)), lo = std::log10(1 - het);
        for (int j = 0; j < n; j++) ev[(size_t)j] = h.logc[(size_t)(major * n + j)] + (j == major ? lo : lh);
        posteriors(ev);
        c.gq = java_phred(1 - ev[(size_t)maxAlt]);
        int altCN = (int)(int16_t)java_round(maxFreq * haplotypes);
        if (altCN == 0) altCN++;
        else if (altCN == haplotypes) altCN--;
        c.acn[(size_t)maxAlt] = altCN;
        c.acn[(size_t)major] = haplotypes - altCN;
    }
    c.total_cn = haplotypes;                                             // setAllelesCopyNumber
    c.report = true;
    h.counts = h0.counts;
}

void genotype_indel_sample(const std::vector<std::string>& alleles, const std::vector<SpanCall>& sc, const RealignParams& p,
                           int min_quality, SampleIndelCall& c, IndelCounts& h) {
    const int n = (int)alleles.size();
    if (p.ploidy >= 3) {
        // DEF_MIN_PLOIDY_POOL_ALGORITHM: genotypeVariantPool (:378-379), makeUndecided below min_quality (:388)
        genotype_pool_indel(alleles, sc, p.ploidy, p.het_rate, p.max_base_qs, c, h);
        if ((int16_t)min_quality > c.gq) { c.n_called = 0; c.gq = 0; update_cn(c, h.counts, c.total_cn); }
        return;
    }
    c = SampleIndelCall();
    c.acn.assign((size_t)n, 0);
    indel_counts(alleles, sc, p.max_base_qs, h);
    if (h.total == 0) {
        update_cn(c, h.counts, p.ploidy);
        return;
    }
    std::vector<double> post;
    indel_posteriors(h, p.het_rate, post);
    int im0 = 0, im1 = 0;
    max_genotype(post, n, &im0, &im1);
    if (im0 > 100 || im1 > 100) c.n_called = 0;                           // GenomicVariant.MAX_NUM_ALLELES
    else if (im1 != im0) { c.n_called = 2; c.called[0] = im0; c.called[1] = im1; }
    else { c.n_called = 1; c.called[0] = im0; }
    double maxP = post[(size_t)(im0 * n + im1)];
    if (im0 != im1) maxP += post[(size_t)(im1 * n + im0)];
    c.gq = java_phred(1 - maxP);
    c.dp = h.total;
    c.report = true;                                                      // setCallReport (totalDepth > 0)
    update_cn(c, h.counts, p.ploidy);
    if ((int16_t)min_quality > c.gq) { c.n_called = 0; c.gq = 0; update_cn(c, h.counts, c.total_cn); }
}

int genotype_indel_population(const std::vector<std::string>& alleles, const std::vector<Aln*>& pileup, int pos,
                              const RealignParams& p, std::vector<SampleIndelCall>& calls, std::vector<IndelCounts>& helpers) {
    const int S = p.n_samples;
    const int span = (int)alleles[0].size();
    calls.assign((size_t)S, SampleIndelCall());
    helpers.assign((size_t)S, IndelCounts());
    std::vector<Aln*> tmp;
    std::vector<SpanCall> sc;
    int qs = 0;
    for (int s = 0; s < S; s++) {
        SampleIndelCall& c = calls[(size_t)s];
        sample_span_calls(pileup, s, pos, span, tmp, sc);
        genotype_indel_sample(alleles, sc, p, 40, c, helpers[(size_t)s]);
        const bool homref = c.n_called == 1 && c.called[0] == 0;
        if (c.n_called > 0 && !homref && c.gq > qs) qs = c.gq;
    }
    return qs;
}

// DecimalFormat("##0.0#") (main/io/ParseUtils.java:29): HALF_EVEN on the exact binary value
void app_fmt2(std::string& o, double x) {
    const double q = x * 100.0, err = std::fma(x, 100.0, -q);
    const double k = std::floor(q), fr = q - k;
    long long v = (long long)k;
    if (fr > 0.5 || (fr == 0.5 && (err > 0 || (err == 0 && (v & 1))))) v++;
    char b[48];
    if (v % 10 == 0) std::snprintf(b, sizeof b, "%lld.%lld", v / 100, (v % 100) / 10);
    else std::snprintf(b, sizeof b, "%lld.%02lld", v / 100, v % 100);
    o += b;
}

// VCFRecord.createDefaultPopulationVCFRecord (vcf/VCFRecord.java:277-282: FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV, INFO
// from DiversityStatistics.calculateDiversityStatistics(calls, false), variants/DiversityStatistics.java:123-218) as
// VCFFileWriter.printVCFRecord / printGenotypeInfo write it (:44-68,159-256); without the sequence name
void format_population_indel(int pos, const std::string& id, const std::vector<std::string>& alleles, const char* type, int qs,
                             const std::vector<SampleIndelCall>& calls, const std::vector<IndelCounts>& helpers, int ploidy,
                             std::string& o) {
    const int n = (int)alleles.size(), S = (int)calls.size();
    o.clear();
    o += std::to_string(pos); o += '\t'; o += id.empty() ? "." : id; o += '\t'; o += alleles[0]; o += '\t';
    if (n == 1) o += '.';
    for (int i = 1; i < n; i++) { if (i > 1) o += ','; o += alleles[(size_t)i]; }
    o += '\t'; o += std::to_string(qs); o += "\t.\t";
    std::vector<int> counts((size_t)n, 0);
    int sum = 0, ng = 0, nhet = 0;
    for (const SampleIndelCall& c : calls) {
        if (c.n_called == 0) continue;
        ng++;
        if (c.n_called > 1) nhet++;
        for (int i = 0; i < c.n_called; i++) { counts[(size_t)c.called[i]] += c.acn[(size_t)c.called[i]]; sum += c.acn[(size_t)c.called[i]]; }
    }
    int ncalled = 0, minAC = 0;
    for (int i = 0; i < n; i++) if (counts[(size_t)i] > 0) { ncalled++; if (minAC == 0 || minAC > counts[(size_t)i]) minAC = counts[(size_t)i]; }
    o += "NS="; o += std::to_string(ng); o += ";AN="; o += std::to_string(ncalled); o += ";AFS=";
    for (int i = 0; i < n; i++) { if (i) o += ','; o += std::to_string(counts[(size_t)i]); }
    o += ";OH="; app_fmt2(o, ng > 0 ? (double)nhet / ng : 0.0);
    if (n == 2) { o += ";MAF="; app_fmt2(o, ncalled < 2 ? 0.0 : (double)minAC / sum); }
    if (type) { o += ";TYPE="; o += type; }
    o += "\tGT:PL:GQ:DP:ADP:ACN";
    for (int s = 0; s < S; s++) {
        const SampleIndelCall& c = calls[(size_t)s];
        const IndelCounts& h = helpers[(size_t)s];
        o += '\t';
        if (c.n_called == 0) o += ploidy > 1 ? "./." : ".";
        else if (c.n_called == 1) { o += std::to_string(c.called[0]); if (ploidy > 1) { o += '/'; o += std::to_string(c.called[0]); } }
        else { o += std::to_string(c.called[0]); o += '/'; o += std::to_string(c.called[1]); }
        o += ':';
        for (int j = 0; j < n; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) o += ',';
                o += std::to_string(c.report ? (int)java_round(-10 * h.logc[(size_t)(i * n + j)]) : 0);
            }
        o += ':'; o += std::to_string(c.gq); o += ':'; o += std::to_string(c.dp); o += ':';
        for (int i = 0; i < n; i++) { if (i) o += ','; o += std::to_string(c.report ? h.counts[(size_t)i] : 0); }
        o += ':';
        if (c.total_cn == 0) o += '.';
        else for (int j = 0; j < n; j++) { if (j) o += ','; o += std::to_string((c.n_called == 0 && j == 0) ? c.total_cn : c.acn[(size_t)j]); }
    }
    o += '\n';
}

// discoverPopulationVariantWithSpan (MultisampleVariantsDetector.java:599-604) + discoverPopulationIndel (:616-634)
// + onPileup's genotypeVariant and QS test (:532-533): false for a null variant (the caller's SNV fallback), else the
// variant's record
bool population_indel(const std::vector<Aln*>& pileup, const std::vector<SpanCall>& calls, const std::string& reference,
                      int pos, bool is_str, bool input_str, const RealignParams& p, PopIndel* out) {
    std::vector<std::string> alleles = cluster_alleles(calls, reference, p.max_base_qs);
    {
        // createIndelVariantPool (SingleSampleVariantPileupListener.java:333-338): one allele, or no call -> null
        if (alleles.size() == 1) return false;
        IndelCounts h;
        indel_counts(alleles, calls, p.max_base_qs, h);
        if (h.total == 0) return false;
    }
    std::vector<SampleIndelCall> sc;
    std::vector<IndelCounts> hs;
    while (alleles.size() > 2) {
        bool same = true;                                                  // allelesSameLength (:339-345)
        for (const std::string& a : alleles) same = same && a.size() == alleles[0].size();
        if (!input_str && same) return false;
        const int qs = genotype_indel_population(alleles, pileup, pos, p, sc, hs);
        if (qs < p.min_quality) return false;
        // makeNewVariant (:642-656): a TreeSet of the reference and every sample's called alleles
        std::set<std::string> called{alleles[0]};
        for (const SampleIndelCall& c : sc)
            for (int i = 0; i < c.n_called; i++) called.insert(alleles[(size_t)c.called[i]]);
        if (called.size() == alleles.size()) break;
        std::vector<std::string> nv{alleles[0]};                           // SingleSampleVariantPileupListener.makeNewVariant
        for (const std::string& a : called) if (a != alleles[0]) nv.push_back(a);
        alleles.swap(nv);
    }
    const int qs = genotype_indel_population(alleles, pileup, pos, p, sc, hs);
    out->qs = qs;
    out->last = pos + (int32_t)alleles[0].size() - 1;
    out->pass = !(qs == 0 || qs < p.min_quality);
    out->line.clear();
    if (out->pass) format_population_indel(pos, std::string(), alleles, is_str ? "STR" : "INDEL", qs, sc, hs, p.ploidy, out->line);
    return true;
}

// GenomicVariantImpl.getVariantTypeName for the INFO TYPE of an input record: written when 2-5 (VCFFileWriter.java:47-49)
const char* type_name(int t) {
    static const char* kNames[] = {nullptr, nullptr, "MULTISNV", "EMBEDDED", "INDEL", "STR"};
    return t >= 2 && t <= 5 ? kNames[t] : nullptr;
}

// VCFFileWriter.printVCFRecord of a CalledGenomicVariantImpl over a GenomicVariantImpl, FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV
// (SingleSampleVariantsDetector.java:946-953), without the sequence name
void format_indel_record(int pos, const std::string& id, const std::vector<std::string>& alleles, int qs, const char* type,
                         const SampleIndelCall& c, const IndelCounts& h, int ploidy, std::string& o) {
    const int n = (int)alleles.size();
    o.clear();
    o += std::to_string(pos); o += '\t'; o += id.empty() ? "." : id; o += '\t'; o += alleles[0]; o += '\t';
    for (int i = 1; i < n; i++) { if (i > 1) o += ','; o += alleles[(size_t)i]; }
    o += '\t'; o += std::to_string(qs); o += "\t.\t";
    if (type) { o += "TYPE="; o += type; } else o += '.';
    o += "\tGT:PL:GQ:DP:ADP:ACN\t";
    if (c.n_called == 0) o += ploidy > 1 ? "./." : ".";
    else if (c.n_called == 1) { o += std::to_string(c.called[0]); if (ploidy > 1) { o += '/'; o += std::to_string(c.called[0]); } }
    else { o += std::to_string(c.called[0]); o += '/'; o += std::to_string(c.called[1]); }
    o += ':';
    for (int j = 0; j < n; j++)
        for (int i = 0; i <= j; i++) {
            if (i > 0 || j > 0) o += ',';
            o += std::to_string(c.report ? (int)java_round(-10 * h.logc[(size_t)(i * n + j)]) : 0);
        }
    o += ':'; o += std::to_string(c.gq); o += ':'; o += std::to_string(c.dp); o += ':';
    for (int i = 0; i < n; i++) { if (i) o += ','; o += std::to_string(c.report ? h.counts[(size_t)i] : 0); }
    o += ':';
    if (c.total_cn == 0) o += '.';
    else for (int j = 0; j < n; j++) { if (j) o += ','; o += std::to_string((c.n_called == 0 && j == 0) ? c.total_cn : c.acn[(size_t)j]); }
    o += '\n';
}

// -knownVariants, a non-SNV input variant at its first position: SingleSampleVariantsDetector's listener genotypes it in
// the one sample (genotypeVariantSample :361-391 with -minQuality) and the record carries the input's ID, alleles, QS
// and TYPE, FORMAT DEF_FORMAT_ARRAY_NGSEP_NOSNV (SingleSampleVariantsDetector.java:946-953); MultisampleVariantsDetector
// genotypes it in every sample (genotypeVariant :664-693) and writes the population record with the variant QS it sets
void known_record(const std::vector<Aln*>& pileup, int pos, const KnownRecord& kr, const RealignParams& p, std::string& o) {
    const char* type = type_name(kr.type);
    if (p.n_samples > 0) {
        std::vector<SampleIndelCall> sc;
        std::vector<IndelCounts> hs;
        const int qs = genotype_indel_population(kr.alleles, pileup, pos, p, sc, hs);
        format_population_indel(pos, kr.id, kr.alleles, type, qs, sc, hs, p.ploidy, o);
        return;
    }
    std::vector<SpanCall> calls;
    span_calls(pileup, pos, (int)kr.alleles[0].size(), calls);
    SampleIndelCall c;
    IndelCounts h;
    genotype_indel_sample(kr.alleles, calls, p, p.min_quality, c, h);
    format_indel_record(pos, kr.id, kr.alleles, kr.qs, type, c, h, p.ploidy, o);
    if (p.ploidy >= 3) {
        // the pool algorithm's copy numbers stay unless the record is its sequence's first (intersectVariantsCNVs,
        // SingleSampleVariantsDetector.java:969-991, updates that one from the counts): both lines, NUL-separated
        // (vcf.cpp format_record)
        update_cn(c, h.counts, p.ploidy);
        std::string first;
        format_indel_record(pos, kr.id, kr.alleles, kr.qs, type, c, h, p.ploidy, first);
        o += '\0';
        o += first;
    }
}

// ploidy >= 3, a span > 1 (discoverVariantWithSpan :257-273 -> discoverIndel :275-296): the clustered alleles' pool
// variant (createIndelVariantPool :333-338: none for one allele, no calls or alleles of one length), genotypeVariantPool;
// a multi-allelic variant keeps its alleles when two non-reference alleles are called, else becomes the reference and the
// called allele (makeNewVariant :346-359) and is genotyped again; an undecided, homozygous-reference or low-GQ call is
// dropped (:263, :223); a kept call's ACN from its counts (:226).  The variant keeps TYPE_UNDETERMINED and QS 0.
bool pool_indel(std::vector<std::string> alleles, const std::vector<SpanCall>& calls, int pos, const RealignParams& p, IndelCall* out) {
    {
        IndelCounts h;
        indel_counts(alleles, calls, p.max_base_qs, h);
        if (alleles.size() <= 1 || h.total == 0) return false;
    }
    auto same_len = [](const std::vector<std::string>& a) {
        for (const std::string& x : a) if (x.size() != a[0].size()) return false;
        return true;
    };
    if (same_len(alleles)) return false;
    SampleIndelCall c;
    IndelCounts h;
    genotype_pool_indel(alleles, calls, p.ploidy, p.het_rate, p.max_base_qs, c, h);
    if (alleles.size() > 2) {
        const bool homref = c.n_called == 1 && c.called[0] == 0;
        if (c.n_called == 0 || homref) return false;
        if (!(c.n_called == 2 && c.called[0] != 0)) {
            std::vector<std::string> nv{alleles[0]};                      // {reference} + the called alleles
            for (int i = 0; i < c.n_called; i++)
                if (alleles[(size_t)c.called[i]] != alleles[0]) nv.push_back(alleles[(size_t)c.called[i]]);
            if (same_len(nv)) return false;
            alleles.swap(nv);
            genotype_pool_indel(alleles, calls, p.ploidy, p.het_rate, p.max_base_qs, c, h);
        }
    }
    const bool homref = c.n_called == 1 && c.called[0] == 0;
    if (c.n_called == 0 || homref || (int16_t)p.min_quality > c.gq) return false;
    update_cn(c, h.counts, p.ploidy);                                    // discoverVariant (:226)
    format_indel_record(pos, std::string(), alleles, 0, nullptr, c, h, p.ploidy, out->line);
    out->pos = pos;
    out->last = pos + (int32_t)alleles[0].size() - 1;
    return true;
}

}  // namespace

void replay_region(const std::string& seq, int64_t first, int64_t last, std::vector<RawRead>& reads, const RealignParams& p,
                   const InputVars* inputs, const std::vector<KnownRecord>* knowns, RegionOut& out) {
    out.first = first;
    out.last = last;
    out.pos.clear();
    out.cols.clear();
    out.indels.clear();
    out.pcodes.clear();
    out.poff.clear();
    out.pindels.clear();
    out.kcalls.clear();
    const bool pop = p.n_samples > 0;
    const int S = p.n_samples;
    std::vector<Aln> alns(reads.size());
    for (size_t i = 0; i < reads.size(); i++) {
        const RawRead& r = reads[i];
        Aln& a = alns[i];
        a.first = r.first;
        a.last = r.last;
        a.flags = r.flags;
        a.ops.assign(r.ops, r.ops + r.n_ops);
        a.read_length = 0;
        for (int32_t v : a.ops) if (v & 2) a.read_length += v / 8;
        // (the characters are the read's; a CIGAR consuming more of the read than it has would index past them)
        a.chars = r.chars && r.len >= a.read_length ? r.chars : nullptr;
        a.quals = a.chars ? r.quals : nullptr;
        a.ignore_start = r.ignore_start;
        a.ignore_end = r.ignore_end;
        a.sample = r.sample;
        a.rank = r.rank;
        a.update();
    }
    // the positions where some alignment has an indel call (getIndelCall != null): elsewhere, with no input variant
    // there, the realigner's onPileup returns span 1 without looking further (its loop over the pileup finds no indel);
    // redrawn after any alignment is edited (a superset of the pileup's is all the shortcut needs)
    int edits = 0, edits_marked = -1;
    const int64_t mark_lo = first;
    std::vector<uint8_t> indel_mark((size_t)std::max<int64_t>(last - first + 1, 1), 0);
    auto remark = [&]() {
        std::fill(indel_mark.begin(), indel_mark.end(), 0);
        for (const Aln& a : alns)
            for (const IndelEv& e : a.indels)
                if (e.first >= mark_lo && e.first <= last) indel_mark[(size_t)(e.first - mark_lo)] = 1;
        edits_marked = edits;
    };
    for (Aln& a : alns) a.edits = &edits;
    {
        size_t want = 0;                                   // (the columns' entries: at most one per read and position)
        for (const Aln& a : alns) want += (size_t)std::max<int64_t>(0, std::min<int64_t>(a.last, last) - std::max<int64_t>(a.first, first) + 1);
        out.cols.reserve(want + 4 * (size_t)(last - first + 1));
        out.pos.reserve((size_t)(last - first + 1));
    }
    Realigner rl(seq);
    std::vector<int32_t> pending;          // indices into alns, admission order
    std::vector<Aln*> pileup;
    std::vector<SpanCall> calls;
    size_t next = 0;
    const int seq_len = (int)seq.size();
    // idxNextVariant at the region's first position: the first input variant that ends at or after it or starts past it
    // (every earlier one was passed at some pileup before, whatever the positions with pileups were) -- from the
    // prefix maximum of `last`; from there the listener's own loop moves it along (it never moves back)
    const std::vector<StrVar>* strs = inputs ? &inputs->v : nullptr;
    size_t vi = 0, vn = strs ? strs->size() : 0;
    if (vn) {
        const size_t a = (size_t)(std::lower_bound(inputs->pmax.begin(), inputs->pmax.end(), (int32_t)first) - inputs->pmax.begin());
        const size_t b = (size_t)(std::upper_bound(strs->begin(), strs->end(), first, [](int64_t x, const StrVar& v) { return x < (int64_t)v.first; }) - strs->begin());
        vi = std::min(a, b);
    }
    // -knownVariants: the non-SNV input variants to genotype at their first positions (kj: the first starting at or
    // after the position swept)
    size_t kj = 0;
    if (p.known && vn) kj = (size_t)(std::lower_bound(strs->begin(), strs->end(), first, [](const StrVar& v, int64_t x) { return (int64_t)v.first < x; }) - strs->begin());
    for (int64_t p64 = first; p64 <= last; p64++) {
        const int pos = (int)p64;
        while (next < alns.size() && reads[next].first <= pos) pending.push_back((int32_t)next++);   // (original starts)
        const StrVar* var = nullptr;                                       // intersectWithVariants (:137-153)
        while (vi < vn) {
            const StrVar& v = (*strs)[vi];
            if (pos < v.first) break;
            if (pos <= v.last) { var = &v; break; }
            vi++;
        }
        if (edits != edits_marked) remark();
        // the realigner's onPileup does something here only with an input variant or an indel call at pos; the pileup
        // list itself is needed by it, by the population columns and by -knownVariants
        const bool onp = var || indel_mark[(size_t)(p64 - mark_lo)];
        RegionPos rp;
        rp.pos = pos;
        if (!onp && !pop && !p.known) {
            // updatePendingAlns (AlignmentsPileupGenerator.java:464-471) and getAlleleCalls(1) in one pass: the pending
            // alignments that end before pos retire, those that start at or before it give the column's entries
            const size_t c0 = out.cols.size();
            out.cols.resize(c0 + pending.size() + 3);
            uint16_t* dst = out.cols.data() + c0;
            size_t k = 0, npile = 0;
            const uint32_t refa = (uint32_t)base_index(upper(seq[(size_t)p64 - 1]));   // (~0u: not A/C/G/T)
            uint32_t nonref = 0;
            for (int32_t i : pending) {
                const Aln* a = &alns[(size_t)i];
                if (a->last < pos) continue;
                pending[k++] = i;
                if (a->first > pos) continue;
                npile++;
                const uint16_t cd = a->code_at(pos);                       // (Aln::update's codes)
                if (cd == 0xFFFF) continue;
                *dst++ = cd;
                nonref |= (uint32_t)((cd & kCodeValid) != 0) & (uint32_t)(((cd >> 5) & 3u) != refa);
            }
            pending.resize(k);
            const size_t n = (size_t)(dst - (out.cols.data() + c0));
            if (npile == 0) { out.cols.resize(c0); continue; }
            rp.nonref = nonref != 0;
            rp.span = 1;
            rp.col_off = (int32_t)c0;
            rp.col_len = (int32_t)n;
            out.cols.resize(c0 + ((n + 3) & ~(size_t)3));
            for (size_t z = c0 + n; z < out.cols.size(); z++) out.cols[z] = 0;
        } else {
            // updatePendingAlns (AlignmentsPileupGenerator.java:464-471): alignments ending before pos retire; the
            // pileup is the pending ones that start at or before pos
            size_t k = 0;
            pileup.clear();
            for (int32_t i : pending) {
                Aln* a = &alns[(size_t)i];
                if (a->last < pos) continue;
                pending[k++] = i;
                if (a->first <= pos) pileup.push_back(a);
            }
            pending.resize(k);
            if (pileup.empty()) continue;
            if (onp) rp.span = rl.on_pileup(pileup, pos, var, &rp.str, &rp.new_str, &rp.var_embedded);
            else rp.span = 1;
            // getAlleleCalls(1): the device's column entries (engine.cpp project_read's codes)
            rp.col_off = (int32_t)out.cols.size();
            const uint32_t refa = (uint32_t)base_index(upper(seq[(size_t)p64 - 1]));
            for (const Aln* a : pileup) {
                const uint16_t cd = a->code_at(pos);                       // (Aln::update's codes)
                if (cd == 0xFFFF) continue;
                out.cols.push_back(cd);
                if ((cd & kCodeValid) && ((cd >> 5) & 3u) != refa) rp.nonref = true;
            }
            rp.col_len = (int32_t)out.cols.size() - rp.col_off;
            while (out.cols.size() % 4) out.cols.push_back(0);
        }
        if (pop) {
            // getAlleleCalls(1, sample.getReadGroups()) per sample (read-group rank, then the pileup's order) and the
            // calls of the reads of no sample (the pooled counts' getAlleleCalls(1, null) adds them): KPM's columns
            rp.pcol = (int32_t)out.poff.size();
            for (int sm = 0; sm <= S; sm++) {
                out.poff.push_back((uint32_t)out.pcodes.size());
                int maxrank = sm < S ? -1 : 0;
                if (sm < S) for (const Aln* a : pileup) if (a->sample == sm) maxrank = std::max<int>(maxrank, a->rank);
                for (int r = 0; r <= maxrank; r++)
                    for (const Aln* a : pileup) {
                        const bool mine = sm < S ? (a->sample == sm && a->rank == r) : (a->sample < 0 || a->sample >= S);
                        if (!mine) continue;
                        const uint16_t cd = a->code_at(pos);
                        if (cd != 0xFFFF) out.pcodes.push_back((uint8_t)cd);
                    }
            }
            out.poff.push_back((uint32_t)out.pcodes.size());
        }
        // discoverVariant's early exits (SingleSampleVariantPileupListener.java:191-213): no reference for the span
        // (getReference -> null), a lower-case reference base with -ignoreLowerCaseRef
        const int plast = pos + rp.span - 1;
        rp.blocked = pos < 1 || plast > seq_len || (p.ignore_lowercase && pos <= seq_len && seq[(size_t)pos - 1] >= 'a' && seq[(size_t)pos - 1] <= 'z');
        if (p.known) {
            // onPileup with input variants (SingleSampleVariantPileupListener.java:162-176, MultisampleVariantsDetector
            // .java:539-551): every input variant starting here, in list order; the SNVs are the device's (KP / KPM
            // over this position's columns), the others are genotyped here
            while (kj < vn && (*strs)[kj].first < pos) kj++;
            for (size_t q = kj; q < vn && (*strs)[q].first == pos; q++) {
                const StrVar& v = (*strs)[q];
                if (v.rec < 0 || !knowns) continue;
                KnownCall kc;
                kc.pos = pos;
                kc.known = v.known;
                known_record(pileup, pos, (*knowns)[(size_t)v.rec], p, kc.line);
                out.kcalls.push_back(std::move(kc));
            }
        } else if (rp.span > 1 && !rp.blocked) {
            std::string reference(seq, (size_t)pos - 1, (size_t)rp.span);
            for (char& ch : reference) ch = upper(ch);
            span_calls(pileup, pos, rp.span, calls);
            if (pop) {
                PopIndel pi;
                if (population_indel(pileup, calls, reference, pos, rp.str, rp.str && !rp.new_str, p, &pi)) {
                    rp.pindel = (int32_t)out.pindels.size();
                    out.pindels.push_back(std::move(pi));
                }
            } else {
                const std::vector<std::string> alleles = cluster_alleles(calls, reference, p.max_base_qs);
                IndelCall ic;
                if (p.ploidy >= 3 ? pool_indel(alleles, calls, pos, p, &ic)
                                  : genotype_indel(alleles, calls, pos, rp.str, rp.str && !rp.new_str, p, &ic)) {
                    rp.indel = (int32_t)out.indels.size();
                    out.indels.push_back(std::move(ic));
                }
            }
        }
        out.pos.push_back(rp);
    }
}

void resolve_region(const RegionOut& out, const std::vector<uint8_t>& has_snv_call, bool call_embedded, int32_t* last_indel_end,
                    std::vector<RegionDecision>& dec) {
    dec.clear();
    for (size_t i = 0; i < out.pos.size(); i++) {
        const RegionPos& rp = out.pos[i];
        // onPileup (:146-161): an input STR moves lastIndelEnd to its end, a position up to lastIndelEnd is embedded
        const bool input_str = rp.str && !rp.new_str;
        bool embedded = rp.var_embedded;
        if (input_str && rp.pos >= *last_indel_end) *last_indel_end = rp.pos + rp.span - 1;
        else if (rp.pos <= *last_indel_end) embedded = true;
        if (!call_embedded && embedded) continue;
        if (rp.blocked) continue;
        const int eff = embedded ? 1 : rp.span;
        if (eff > 1 && rp.indel >= 0) {
            dec.push_back(RegionDecision{rp.pos, 2, false, rp.indel});
            *last_indel_end = out.indels[(size_t)rp.indel].last;
            continue;
        }
        if (eff > 1 && input_str) continue;                                 // no SNV fallback for an input STR (:264)
        if (has_snv_call[i]) dec.push_back(RegionDecision{rp.pos, 1, embedded, -1});   // discoverSNV (and the fallback)
    }
}

// MultisampleVariantsDetector.onPileup (:522-538): an input STR sets lastIndelEnd to its end (no ">= lastIndelEnd"
// test, unlike the single-sample listener), a position up to lastIndelEnd is embedded; the span's indel variant is
// written when its QS passes and moves lastIndelEnd to its end; a span without one falls back to the SNV
// (discoverPopulationSNV, :605-612), except at an input STR
void resolve_population_region(const RegionOut& out, const std::vector<uint8_t>& has_snv_record, bool call_embedded,
                               int32_t* last_indel_end, std::vector<RegionDecision>& dec) {
    dec.clear();
    for (size_t i = 0; i < out.pos.size(); i++) {
        const RegionPos& rp = out.pos[i];
        const bool input_str = rp.str && !rp.new_str;
        bool embedded = rp.var_embedded;
        if (input_str) *last_indel_end = rp.pos + rp.span - 1;
        else if (rp.pos <= *last_indel_end) embedded = true;
        if (!call_embedded && embedded) continue;
        if (rp.blocked) continue;
        const int eff = embedded ? 1 : rp.span;
        if (eff > 1) {
            if (rp.pindel >= 0) {
                const PopIndel& pi = out.pindels[(size_t)rp.pindel];
                if (pi.pass) {
                    dec.push_back(RegionDecision{rp.pos, 2, false, rp.pindel});
                    *last_indel_end = pi.last;
                }
                continue;
            }
            if (input_str) continue;
        }
        if (has_snv_record[i]) dec.push_back(RegionDecision{rp.pos, 1, embedded, -1});
    }
}

}  // namespace ngsep
