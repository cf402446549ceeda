// engine.cpp -- host side of the MI355X NGSEP SNV caller.
//
//  * admission sweep: the reference's AlignmentsPileupGenerator.processAlignment /
//    processSameStartAlns (discovery/AlignmentsPileupGenerator.java:377-433) decides which
//    alignments enter the pending list and in which order;
//  * projection: ReadAlignment.updateAlleleCallsInfo / getAlignedReadPosition /
//    getAlleleCall / getBaseQualityScore (alignments/ReadAlignment.java:747-871,989-1027)
//    are evaluated once per read and stored as one code byte per covered reference position;
//  * staging: reads of every window are laid out as fixed-stride slots (SoA) in HBM;
//    the per-position pileup work is done by the kernels in kernels.hip.
#include "engine.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <mutex>
#include <unordered_map>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <cstdlib>
#include <emmintrin.h>
#include <fstream>
#include <functional>

namespace ngsep {

void* huge_alloc(size_t bytes) {
    constexpr size_t kHuge = (size_t)2 << 20;
    if (bytes < ((size_t)4 << 20)) return std::malloc(bytes);
    const size_t n = (bytes + kHuge - 1) / kHuge * kHuge;
    void* p = std::aligned_alloc(kHuge, n);
    // (measured: base pages instead cost the 200-BAM population 2.35 -> 3.7-4.0 s and chr20 0.48 -> 0.59 s, r05th)
    if (p) madvise(p, n, MADV_HUGEPAGE);
    return p;
}

int set_error(ngsep_ctx* c, int code, const std::string& msg) {
    static std::mutex mu;                        // readers of several files may fail on host threads at once
    std::lock_guard<std::mutex> lk(mu);
    if (c) c->err = msg;
    return code;
}

static inline int dna_index(char ch) {
    switch (ch) {
        case 'A': return 0;
        case 'C': return 1;
        case 'G': return 2;
        case 'T': return 3;
        default: return -1;
    }
}

// Likelihood addends exactly as CountsHelper computes its caches (CountsHelper.java:147-185).
void compute_tables(const ngsep_ctx* c, LikTables* t, GenotypeParams* g) {
    std::memset(t, 0, sizeof(*t));
    const int f = 250;   // round(0.5*500): SingleSampleVariantPileupListener.discoverSNV passes 0.5
    const double af = (double)f / 500.0;
    for (int q = 3; q <= 30; q++) {
        double e0 = -0.1 * q;
        t->E[q] = e0 - std::log10(3.0);                        // logProbCacheError[q][4]
        double errorProb = std::pow(10.0, -0.1 * q);           // PhredScoreHelper.calculateProbability
        double successProb = 1 - errorProb;
        t->A[q] = std::log10(successProb);                     // logProbCacheGT[f][q][0]
        double hetProb = af * successProb + (1 - af) * errorProb / 3;
        t->H[q] = std::log10(hetProb);                         // logProbCacheGT[f][q][4]
    }
    double h = c->het_rate;
    g->log_prior_hetero = std::log10(h / 12);                  // CountsHelper.java:415
    g->log_prior_homo = std::log10((1 - h) / 4);               // CountsHelper.java:416
    int8_t mq = (int8_t)c->params.max_base_qs;                 // byte field, CountsHelper.java:88
    g->max_q = mq > 0 ? mq : 30;
    g->min_quality = (int16_t)c->params.min_quality;
    g->dump_all = c->params.dump_all_positions;
    const char* ab = diag_env("NGSEP_ABLATE");
    g->ablate = ab ? std::atoi(ab) : 0;
    // Integer hom-ref bound.  Per valid call of quality q the differences
    // L[r][r]-L[r][x] etc. take one of the four values below; floor/ceil make the integer sums
    // lower bounds of the exact differences, so a position the bound proves hom-ref is hom-ref.
    const double K = kBoundScale;
    bool ok = true;
    for (int q = 4; q <= 30; q++) {
        const double rh = t->A[q] - t->H[q], re = t->A[q] - t->E[q], xh = t->H[q] - t->E[q];
        if (!(rh >= 0 && re >= 0 && xh >= 0)) ok = false;
        const unsigned long long wrh = (unsigned long long)std::floor(K * rh), wre = (unsigned long long)std::floor(K * re);
        const unsigned long long wxh = (unsigned long long)std::ceil(K * xh), wxa = (unsigned long long)std::ceil(K * re);
        t->wR[q] = wrh | (wre << 32);
        t->wX[q] = wxh | (wxa << 32);
    }
    // 2 P(x,y) <= P(r,r) and P(x,x) <= P(r,r) for every other genotype keeps getIndexesMaxGenotype
    // (VariantDiscoverySNVQAlgorithm.java:223-243) at ref/ref, which the listener drops (:223)
    const double t_het = g->log_prior_hetero - g->log_prior_homo + std::log10(2.0);
    t->t_het = (long long)std::floor(K * t_het) + kBoundMargin;
    t->t_homo = kBoundMargin;
    g->ploidy = c->params.ploidy;
    g->full_records = c->params.full_records || c->params.dump_all_positions ? 1 : 0;
    // the bounds prove SNVQ hom-ref calls; the pool algorithm only needs a valid non-reference call (its
    // variant needs an alternative allele count >= 1, createSNVVariantPool :313-320), the scan's candidate test
    g->use_bound = ok && !g->dump_all && std::isfinite(t_het) && g->ploidy < 3 ? 1 : 0;
    // count bound: a valid call carries q in [4, 30] (engine.hpp code), capped at max_q in the kernel
    t->c_r1 = t->c_r2 = INT64_MAX;
    t->c_x1 = t->c_x2 = 0;
    for (int q0 = 4; q0 <= 30; q0++) {
        const int q = q0 > g->max_q ? g->max_q : q0;
        t->c_r1 = std::min<long long>(t->c_r1, (long long)(t->wR[q] & 0xFFFFFFFFull));
        t->c_r2 = std::min<long long>(t->c_r2, (long long)(t->wR[q] >> 32));
        t->c_x1 = std::max<long long>(t->c_x1, (long long)(t->wX[q] & 0xFFFFFFFFull));
        t->c_x2 = std::max<long long>(t->c_x2, (long long)(t->wX[q] >> 32));
    }
    // (the test is non-decreasing in nr: c_r1, c_r2 >= 0, so the first dropping nr is found by bisection)
    auto drops = [t](long long nr, long long na) {
        return nr * t->c_r1 - na * t->c_x1 > t->t_het && nr * t->c_r2 - na * t->c_x2 > t->t_homo &&
               nr * t->c_r2 - na * t->c_x1 > t->t_het;
    };
    for (long long na = 0; na < 256; na++) {
        long long lo = 0, hi = 256;          // first nr in [lo, hi] that drops; 256: none
        while (lo < hi) {
            const long long mid = (lo + hi) / 2;
            if (drops(mid, na)) hi = mid;
            else lo = mid + 1;
        }
        t->cb_nr[na] = (int16_t)lo;
    }
    // KLM's count bound: reference calls counted only when their quality is >= kKlmQs (the rest are exceptions and
    // add nothing, a lower bound as every reference addend is >= 0), one call of another allele at its worst quality
    long long h_r1 = INT64_MAX, h_r2 = INT64_MAX;
    for (int q0 = kKlmQs; q0 <= 30; q0++) {
        const int q = q0 > g->max_q ? g->max_q : q0;
        h_r1 = std::min<long long>(h_r1, (long long)(t->wR[q] & 0xFFFFFFFFull));
        h_r2 = std::min<long long>(h_r2, (long long)(t->wR[q] >> 32));
    }
    t->cb_hi1 = 256;
    for (long long n = 0; n < 256; n++)
        if (n * h_r1 - t->c_x1 > t->t_het && n * h_r2 - t->c_x2 > t->t_homo && n * h_r2 - t->c_x1 > t->t_het) {
            t->cb_hi1 = (int32_t)n;
            break;
        }
}

// genotypeVariantPool's hypotheses (SingleSampleVariantPileupListener.java:408-416) and the CountsHelper
// caches they read (CountsHelper.java:147-185) for ploidy >= 3
void compute_pool_tables(const ngsep_ctx* c, PoolTables* pt) {
    std::memset(pt, 0, sizeof(*pt));
    const int P = c->params.ploidy;
    pt->ploidy = P;
    const double step = 1.0 / (double)P;
    int nf = 0;
    for (double freq = step; freq < 0.51 && nf < kPoolMaxFreq; freq += step) pt->freq[nf++] = freq;
    pt->nf = nf;
    auto gt = [](int f, int q, int j) {      // logProbCacheGT[f][q][j], CountsHelper.java:168-185
        const double af = (double)f / 500.0;
        const double errorProb = std::pow(10.0, -0.1 * q), successProb = 1 - errorProb;
        return j == 0 ? std::log10(successProb) : std::log10(af * successProb + (1 - af) * errorProb / (j - 1));
    };
    for (int q = 3; q <= 30; q++) {
        pt->A[q] = gt(0, q, 0);
        for (int ni = 0; ni < 3; ni++) pt->E[ni][q] = -0.1 * q - std::log10((double)(ni + 1));   // logProbCacheError[q][n]
        for (int j = 0; j < nf; j++) {
            const int f = (int)java_round(pt->freq[j] * 500), g = (int)java_round((1 - pt->freq[j]) * 500);   // :212-213
            for (int ni = 0; ni < 3; ni++) {
                pt->F[j][ni][q] = gt(f, q, ni + 2);
                pt->G[j][ni][q] = gt(g, q, ni + 2);
            }
        }
    }
    const double h = c->het_rate;
    pt->log_h = std::log10(h);
    pt->log_1h = std::log10(1 - h);
    for (int ni = 0; ni < 3; ni++) pt->log_h_n[ni] = std::log10(h / (ni + 1));
}

// ploidy >= 3: the pool tables onto the context's device before a run
int prepare_pool(ngsep_ctx* c) {
    if (c->params.ploidy < 3 || !c->dev) return NGSEP_OK;
    PoolTables pt;
    compute_pool_tables(c, &pt);
    std::string err;
    if (device_set_pool(c->dev, &pt, err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
    return NGSEP_OK;
}

// ReadAlignment.updateAlleleCallsInfo (ReadAlignment.java:747-834): allele-call length per read position.
static void allele_call_lengths(const ReadView& r, int read_length, int ignore_start, int ignore_end, int16_t* acl) {
    std::memset(acl, 0, sizeof(int16_t) * (size_t)(read_length > 0 ? read_length : 1));
    int readPos = 0;
    bool prevIndel = false;
    const int closeIndel = 2;   // basesToIgnoreCloseToIndel (:115)
    const int n = r.n_cigar;
    for (int i = 0; i < n; i++) {
        int len = r.cigar[i] / 8, op = r.cigar[i] & 7;
        bool cRef = op & 1, cRead = (op & 2) != 0;
        int nextOp = -1, nextLen = 0, nextReadCons = 0;
        bool nextIsIndel = false;
        if (i < n - 1) {
            nextOp = r.cigar[i + 1] & 7;
            nextLen = r.cigar[i + 1] / 8;
            nextIsIndel = nextOp == 1 || nextOp == 2;
            nextReadCons = (nextOp & 2) ? nextLen : 0;
        }
        if (cRef) {
            if (cRead) {
                for (int j = 0; j < len; j++) {
                    bool skip = readPos < ignore_start;
                    skip = skip || (read_length - readPos) <= ignore_end;
                    skip = skip || (prevIndel && j < closeIndel);
                    skip = skip || (nextIsIndel && j < len - 1 && j >= len - closeIndel);
                    skip = skip || (nextIsIndel && j == len - 1 &&
                                    (readPos < closeIndel || read_length - readPos - nextReadCons < closeIndel));
                    int readPosAfterIndel = readPos + nextReadCons + 1;
                    skip = skip || (nextIsIndel && j == len - 1 && (read_length - readPosAfterIndel < ignore_end));
                    if (!skip && readPos < read_length) {
                        if (j == len - 1 && nextIsIndel) acl[readPos] = (int16_t)(nextOp == 2 ? nextLen + 2 : 2);
                        else acl[readPos] = 1;
                    }
                    readPos++;
                }
            }
        } else if (cRead) {
            readPos += len;
        }
        prevIndel = (op == 1 || op == 2);
    }
}

// Projects one admitted read to one code byte per reference position in [first, last] (out holds
// last - first + 1 bytes, zero-filled here).  Equivalent to evaluating, for every covered position p,
// PileupRecord.getAlleleCalls(1)'s per-read step (PileupRecord.java:132-148) and
// CountsHelper.calculateCountsGTSNV's quality clamp (CountsHelper.java:91).
// code byte of a valid-or-counted call from its quality character and base (setQualityScores cap at 127,
// CountsHelper.java:91's min(30, q), q <= 3 or a base other than A/C/G/T counted only), for every pair
static const uint8_t* code_table() {
    static uint8_t t[256 * 256];
    static const bool init = [] {
        for (int qc0 = 0; qc0 < 256; qc0++)
            for (int b = 0; b < 256; b++) {
                const int qc = qc0 > 127 ? 127 : qc0;
                const int q = (int8_t)std::min(30, qc - 33);
                const int a = dna_index((char)b);
                uint8_t code;
                if (q <= 3) code = (uint8_t)(kCodeCounted | (q < 0 ? 0 : q));
                else if (a < 0) code = (uint8_t)(kCodeCounted | q);
                else code = (uint8_t)(kCodeValid | (a << 5) | q);
                t[qc0 * 256 + b] = code;
            }
        return true;
    }();
    (void)init;
    return t;
}

// the same codes from BAM's encoding: raw quality (0xFF = none: '+' + ... is handled by the caller) and 4-bit base
static const uint8_t* code_table_packed() {
    static uint8_t t[256 * 16];
    static const bool init = [] {
        static const char kNt[] = "=ACMGRSVTWYHKDBN";
        const uint8_t* ascii = code_table();
        for (int rq = 0; rq < 256; rq++)
            for (int nb = 0; nb < 16; nb++) t[rq * 16 + nb] = ascii[(size_t)std::min(255, rq + 33) * 256 + (uint8_t)kNt[nb]];
        return true;
    }();
    (void)init;
    return t;
}
static inline char packed_base(const char* seq, int64_t i) {
    static const char kNt[] = "=ACMGRSVTWYHKDBN";
    const uint8_t b = (uint8_t)seq[i >> 1];
    return kNt[(i & 1) ? (b & 15) : (b >> 4)];
}
// a BAM-packed read's n characters (4 bits each, high nibble first) into out: one table load per byte
static void unpack_bases(const char* seq, int32_t n, char* out) {
    static const uint16_t* tab = [] {
        static uint16_t t[256];
        static const char kNt[] = "=ACMGRSVTWYHKDBN";
        for (int b = 0; b < 256; b++) t[b] = (uint16_t)((uint8_t)kNt[b >> 4] | (uint16_t)(uint8_t)kNt[b & 15] << 8);
        return t;
    }();
    const uint8_t* s = reinterpret_cast<const uint8_t*>(seq);
    const int32_t pairs = n >> 1;
    for (int32_t k = 0; k < pairs; k++) std::memcpy(out + 2 * k, &tab[s[k]], 2);
    if (n & 1) out[n - 1] = packed_base(seq, n - 1);
}

void project_read(const ngsep_ctx* c, const ReadView& r, uint8_t* out) {
    const int64_t span = (int64_t)r.last - r.first + 1;
    if (span <= 0) return;
    if (!r.chars) { std::memset(out, 0, (size_t)span); return; }   // getAlleleCall returns null without characters
    // fast path: no I/D item and nothing ignored at the read ends -- every aligned base is a call
    // (updateAlleleCallsInfo's masks are all about indels and ignore5/3, ReadAlignment.java:747-834)
    if (r.packed && r.indel_len == 0 && c->params.ignore5 == 0 && c->params.ignore3 == 0) {
        static const uint8_t* tab = code_table_packed();
        const uint8_t* seq = reinterpret_cast<const uint8_t*>(r.chars);
        const uint8_t* quals = reinterpret_cast<const uint8_t*>(r.quals);
        int64_t o = 0, rp = 0;
        for (int32_t k = 0; k < r.n_cigar; k++) {
            const int32_t v = r.cigar[k], len = v / 8, op = v & 7;
            const bool cRef = op & 1, cRead = (op & 2) != 0;
            if (cRef && cRead) {
                const int64_t n = std::min<int64_t>(len, std::min<int64_t>(span - o, (int64_t)r.len - rp));
                int64_t j = 0;
                if (quals) {
                    if (((rp ^ 1) & 1) == 0 && n > 0) {        // odd start: the low nibble of a byte first
                        out[o] = tab[(size_t)quals[rp] * 16 + (seq[rp >> 1] & 15)];
                        j = 1;
                    }
                    for (; j + 1 < n; j += 2) {                  // whole bytes: two bases
                        const uint8_t b = seq[(rp + j) >> 1];
                        out[o + j] = tab[(size_t)quals[rp + j] * 16 + (b >> 4)];
                        out[o + j + 1] = tab[(size_t)quals[rp + j + 1] * 16 + (b & 15)];
                    }
                    for (; j < n; j++) {
                        const uint8_t b = seq[(rp + j) >> 1];
                        out[o + j] = tab[(size_t)quals[rp + j] * 16 + (((rp + j) & 1) ? (b & 15) : (b >> 4))];
                    }
                } else {
                    for (; j < n; j++) {
                        const uint8_t b = seq[(rp + j) >> 1];
                        out[o + j] = tab[(size_t)('+' - 33) * 16 + (((rp + j) & 1) ? (b & 15) : (b >> 4))];
                    }
                }
                for (j = n > 0 ? n : 0; j < len && o + j < span; j++) out[o + j] = 0;
            } else if (cRef) {
                std::memset(out + o, 0, (size_t)std::max<int64_t>(0, std::min<int64_t>(len, span - o)));
            }
            if (cRef) o += len;
            if (cRead) rp += len;
        }
        return;
    }
    if (!r.packed && r.indel_len == 0 && c->params.ignore5 == 0 && c->params.ignore3 == 0) {
        static const uint8_t* tab = code_table();
        const uint8_t* chars = reinterpret_cast<const uint8_t*>(r.chars);
        const uint8_t* quals = reinterpret_cast<const uint8_t*>(r.quals);
        int64_t o = 0, rp = 0;
        for (int32_t k = 0; k < r.n_cigar; k++) {
            const int32_t v = r.cigar[k], len = v / 8, op = v & 7;
            const bool cRef = op & 1, cRead = (op & 2) != 0;
            if (cRef && cRead) {
                const int64_t n = std::min<int64_t>(len, std::min<int64_t>(span - o, (int64_t)r.len - rp));
                if (quals)
                    for (int64_t j = 0; j < n; j++) out[o + j] = tab[(size_t)quals[rp + j] * 256 + chars[rp + j]];
                else
                    for (int64_t j = 0; j < n; j++) out[o + j] = tab[(size_t)'+' * 256 + chars[rp + j]];
                for (int64_t j = n > 0 ? n : 0; j < len && o + j < span; j++) out[o + j] = 0;
            } else if (cRef) {
                std::memset(out + o, 0, (size_t)std::max<int64_t>(0, std::min<int64_t>(len, span - o)));
            }
            if (cRef) o += len;
            if (cRead) rp += len;
        }
        return;
    }
    std::memset(out, 0, (size_t)span);
    int read_length = 0;
    for (int32_t k = 0; k < r.n_cigar; k++) if (r.cigar[k] & 2) read_length += r.cigar[k] / 8;
    // setBasesToIgnore5P/3P (ReadAlignment.java:613-644)
    const bool neg = (r.flags & 0x10) != 0;
    int ignore_start = neg ? c->params.ignore3 : c->params.ignore5;
    int ignore_end = neg ? c->params.ignore5 : c->params.ignore3;
    thread_local std::vector<int16_t> acl;
    if ((int)acl.size() < read_length + 1) acl.resize((size_t)read_length + 1);
    allele_call_lengths(r, read_length, ignore_start, ignore_end, acl.data());
    int64_t refPos = r.first, readPos = 0;
    for (int32_t k = 0; k < r.n_cigar; k++) {
        const int32_t v = r.cigar[k];
        int len = v / 8, op = v & 7;
        bool cRef = op & 1, cRead = (op & 2) != 0;
        if (cRef && cRead) {
            for (int j = 0; j < len; j++) {
                int64_t rp = readPos + j;
                int64_t o = refPos + j - r.first;
                if (rp >= read_length || o < 0 || o >= span) continue;
                if (acl[(size_t)rp] != 1) continue;   // 0: masked (getAlleleCall null); >1: skipped for span 1
                int qc = r.quals ? (unsigned char)r.quals[rp] + (r.packed ? 33 : 0) : '+';   // getBaseQualityScore
                if (qc > 127) qc = 127;                                                 // setQualityScores cap
                int q = (int8_t)std::min(30, qc - 33);
                int a = dna_index(r.packed ? packed_base(r.chars, rp) : r.chars[rp]);
                uint8_t code;
                if (q <= 3) code = (uint8_t)(kCodeCounted | (q < 0 ? 0 : q));
                else if (a < 0) code = (uint8_t)(kCodeCounted | q);
                else code = (uint8_t)(kCodeValid | (a << 5) | q);
                out[o] = code;
            }
        }
        if (cRef) refPos += len;
        if (cRead) readPos += len;
    }
}

// admission of one read into the current sequence's pending list (AlignmentsPileupGenerator
// .processSameStartAlns :428-430); its projection is deferred to project_pending (batched, parallel)
static void admit_core(ngsep_ctx* c, int32_t first, int32_t last, int32_t flags, int32_t rg, int32_t indel_len);
static void admit(ngsep_ctx* c, const ReadView& r) {
    if (!c->params.coverage_stats) {
        if (r.bidx >= 0) c->to_project.push_back(r.bidx);
        else {
            c->to_project.push_back(-1 - (int32_t)c->to_project_carried.size());
            c->to_project_carried.push_back(r);
        }
    }
    admit_core(c, r.first, r.last, r.flags, r.rg, r.indel_len);
}
// the same for the current batch's read i (no view built)
static inline void admit_index(ngsep_ctx* c, int32_t i) {
    const ngsep_read_batch* b = c->cur_batch.b;
    if (!c->params.coverage_stats) c->to_project.push_back(i);
    admit_core(c, b->first[i], c->cur_batch.last[i], b->flags[i], b->read_group ? b->read_group[i] : -1, c->cur_batch.indel[i]);
}
// the realigner's input variants of the current sequence that start at or before `upto` and open a region (the input
// STRs; with -knownVariants the records that are not SNVs) join its events (IndelRealignerPileupListener realigns
// around every input variant, :85-126), in start order among the indel reads, so they open regions of the same reach
// (carve_indel_regions, keep_raw, stream_launch); an SNV input changes nothing where no indel read reaches it
static void inject_strs(ngsep_ctx* c, int64_t upto) {
    ContigReads& cr = c->contig;
    if (cr.seq_id < 0 || (size_t)cr.seq_id >= c->strs.size()) return;
    const std::vector<StrVar>& v = c->strs[(size_t)cr.seq_id].v;
    while (c->str_next < v.size() && (int64_t)v[c->str_next].first <= upto) {
        if (v[c->str_next].event) cr.indel_reads.push_back({v[c->str_next].first, v[c->str_next].last});
        c->str_next++;
    }
}

static void admit_core(ngsep_ctx* c, int32_t first, int32_t last, int32_t flags, int32_t rg, int32_t indel_len) {
    struct { int32_t first, flags, rg, indel_len; } r{first, flags, rg, indel_len};
    ContigReads& cr = c->contig;
    if (c->params.coverage_stats) {
        // CoverageStatisticsCalculator: only [first, last] and isUnique reach the listener
        // (PileupRecord.addAlignment, :154-167); positions past the sequence end still get pileups
        cr.first.push_back(r.first);
        cr.last.push_back(last);
        cr.uniq.push_back((r.flags & 0x1000) ? 0 : 1);
        const int32_t span = last - r.first + 1;
        if (span > cr.max_span) cr.max_span = span;
        if (last >= r.first) {
            if (r.first > cr.cov_last) cr.covered += last - r.first + 1;
            else if (last > cr.cov_last) cr.covered += last - cr.cov_last;
            if (last > cr.cov_last) cr.cov_last = last;
        }
        c->stats.alignments_admitted++;
        return;
    }
    if (!c->strs.empty()) inject_strs(c, r.first);
    cr.first.push_back(r.first);
    cr.last.push_back(last);
    cr.neg.push_back((r.flags & 0x10) ? 1 : 0);
    if (c->params.multisample) {
        const bool in = r.rg >= 0 && r.rg < (int32_t)c->rg_sample.size();
        cr.sample.push_back((int16_t)(in ? c->rg_sample[r.rg] : -1));
        cr.rank.push_back((uint8_t)(in && c->rg_sample[r.rg] >= 0 ? c->rg_rank[r.rg] : 0));
    }
    if (r.indel_len > 0) cr.indel_reads.push_back({r.first, last + r.indel_len});   // the realigner's events
    int32_t span = last - r.first + 1;
    if (span > cr.max_span) cr.max_span = span;
    // union of covered positions inside the sequence (and the query range)
    int64_t lo = r.first, hi = last;
    const int64_t len = cr.seq_len;
    if (hi > len) hi = len;
    if (lo < 1) lo = 1;
    if (c->params.query_seq[0]) {
        lo = std::max<int64_t>(lo, c->params.query_first);
        hi = std::min<int64_t>(hi, c->params.query_last);
    }
    if (hi >= lo) {
        if (lo > cr.cov_last) cr.covered += hi - lo + 1;
        else if (hi > cr.cov_last) cr.covered += hi - cr.cov_last;
        if (hi > cr.cov_last) cr.cov_last = (int32_t)hi;
    }
    c->stats.alignments_admitted++;
}

// projects the admitted reads whose bytes are still pending into the sequence's byte store, on all
// host threads (every read's bytes go to its own preallocated range)
// the view of read i of the batch being admitted
static inline ReadView batch_view(const BatchRef& br, int32_t i) {
    const ngsep_read_batch* b = br.b;
    ReadView r;
    r.seq_id = b->seq_id[i];
    r.first = b->first[i];
    r.last = br.last[i];
    r.flags = b->flags[i];
    r.rg = b->read_group ? b->read_group[i] : -1;
    r.cigar = b->cigar + b->cigar_off[i];
    r.n_cigar = b->cigar_n[i];
    const int32_t sl = b->seq_len[i];
    r.len = sl > 0 ? sl : 0;
    r.chars = nullptr;
    r.quals = nullptr;
    if (sl > 0 && br.chars_at) {
        r.chars = br.chars_at[i];
        r.quals = br.quals_at[i];
    } else if (sl > 0) {
        r.chars = b->bases + b->seq_off[i];
        if (b->quals && (!b->has_quals || b->has_quals[i])) r.quals = b->quals + (br.qual_off ? br.qual_off[i] : b->seq_off[i]);
    }
    r.indel_len = br.indel[i];
    r.packed = br.packed;
    r.bidx = i;
    return r;
}

static bool realign_active(const ngsep_ctx* c);
static void keep_raw(ngsep_ctx* c, size_t b0, size_t n, const int32_t* ent, const ReadView* carried);

static void project_pending(ngsep_ctx* c) {
    std::vector<int32_t>& v = c->to_project;
    if (v.empty()) return;
    ContigReads& cr = c->contig;
    const size_t n = v.size();
    const size_t b0 = cr.bptr.size();          // the admitted reads' [first, last] are cr.first/last[b0 ...]
    std::vector<int64_t> off(n + 1, 0);
    int32_t maxlast = INT32_MIN;
    for (size_t i = 0; i < n; i++) {
        const int64_t span = (int64_t)cr.last[b0 + i] - cr.first[b0 + i] + 1;
        off[i + 1] = off[i] + (span > 0 ? span : 0);
        maxlast = std::max(maxlast, cr.last[b0 + i]);
    }
    // an uninitialised chunk for this batch's codes (a released one when it is large enough): every read
    // writes its own range
    const size_t need = (size_t)std::max<int64_t>(off[n], 1);
    HostArray<uint8_t> ch;
    for (size_t k = 0; k < c->chunk_pool.size(); k++)
        if (c->chunk_pool[k].n >= need) {
            ch = std::move(c->chunk_pool[k]);
            c->chunk_pool.erase(c->chunk_pool.begin() + (ptrdiff_t)k);
            break;
        }
    if (!ch.p) ch.alloc(need + need / 8);
    uint8_t* base = ch.p;
    cr.chunks.emplace_back(std::move(ch));
    cr.bptr.resize(b0 + n);
    for (size_t i = 0; i < n; i++) cr.bptr[b0 + i] = base + off[i];
    cr.chunk_end.push_back(b0 + n);
    cr.chunk_used.push_back(off[n]);
    cr.chunk_maxlast.push_back(maxlast);
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto t1 = std::chrono::steady_clock::now();
    const BatchRef br = c->cur_batch;
    const int32_t* ent = v.data();
    const ReadView* carried = c->to_project_carried.data();
    parallel_for((int64_t)n, 2048, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            const int32_t e = ent[i];
            if (e >= 0) project_read(c, batch_view(br, e), base + off[(size_t)i]);
            else project_read(c, carried[-1 - e], base + off[(size_t)i]);
        }
    });
    if (host_timing)
        std::fprintf(stderr, "[ngsep host] projection: %.1f ms (%u threads)\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count(), host_threads());
    if (realign_active(c)) {
        const auto t_k = std::chrono::steady_clock::now();
        keep_raw(c, b0, n, ent, carried);
        c->keep_raw_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_k).count();
    }
    v.clear();
    c->to_project_carried.clear();
}

// AlignmentsPileupGenerator.processSameStartAlns (:407-433)
static void process_same_start(ngsep_ctx* c) {
    if (c->ss_one >= 0) {                         // one primary alignment at this start (the common case): admitted
        admit_index(c, c->ss_one);
        c->ss_one = -1;
        return;
    }
    if (c->ss_secondary.empty()) {
        if (c->ss_primary.empty()) return;
        if (c->ss_primary.size() == 1) {          // one alignment at this start (the common case): admitted
            admit(c, c->ss_primary[0]);
            c->ss_primary.clear();
            return;
        }
    }
    std::pair<int32_t, int32_t> per_rg_small[8];   // (rg, count): few read groups per start
    std::vector<std::pair<int32_t, int32_t>> per_rg_big;
    int n_rg = 0;
    auto handle = [&](const ReadView& r) {
        std::pair<int32_t, int32_t>* tab = per_rg_big.empty() ? per_rg_small : per_rg_big.data();
        for (int k = 0; k < n_rg; k++) {
            if (tab[k].first == r.rg) {
                if (c->params.max_alns_per_start <= 0 || tab[k].second < c->params.max_alns_per_start) { tab[k].second++; admit(c, r); }
                return;
            }
        }
        if (n_rg == 8 && per_rg_big.empty()) per_rg_big.assign(per_rg_small, per_rg_small + 8);
        if (per_rg_big.empty()) per_rg_small[n_rg] = {r.rg, 1};
        else per_rg_big.push_back({r.rg, 1});
        n_rg++;
        admit(c, r);
    };
    for (const ReadView& r : c->ss_primary) handle(r);
    for (const ReadView& r : c->ss_secondary) handle(r);
    c->ss_primary.clear();
    c->ss_secondary.clear();
}

// flushes the current sequence: onSequenceEnd of the listener chain
static int stream_advance(ngsep_ctx* c, bool final);

static bool streaming(const ngsep_ctx* c) { return !c->staging_mode && !c->params.coverage_stats && !c->params.multisample; }

// the indel realigner runs here (realign.hpp) in streamed single-sample runs and in MultisampleVariantsDetector (run
// per sequence), at every ploidy (the pool algorithm's indel branch at >= 3), discovering or genotyping -knownVariants
// (the reference's listener chains: SingleSampleVariantsDetector.java:896-931, MultisampleVariantsDetector.java:432-450);
// elsewhere its regions are carved out and returned (params.indel_passthrough)
static bool realign_active(const ngsep_ctx* c) {
    const bool path = streaming(c) || (c->params.multisample && !c->staging_mode);
    return path && !c->params.indel_passthrough && !c->params.relative_allele_counts && !c->params.dump_all_positions;
}

// keeps the raw alignments (RawRead) a realigner region can need: those inside the reach of an indel read
// admitted so far, and those a later one could still reach (`maybe`: last + R >= the admission frontier).
// Called after each projection with the newly admitted reads b0 .. b0 + n (ent / carried: their batch views).
static void keep_raw(ngsep_ctx* c, size_t b0, size_t n, const int32_t* ent, const ReadView* carried) {
    ContigReads& cr = c->contig;
    auto& st = c->stream;
    while (st.indel_pmax.size() < cr.indel_reads.size()) {
        const size_t k = st.indel_pmax.size();
        st.indel_pmax.push_back(std::max(k ? st.indel_pmax[k - 1] : INT32_MIN, cr.indel_reads[k].second));
    }
    const int64_t R = (int64_t)cr.max_span + 100;
    auto covered = [&](int64_t f, int64_t l) {             // an indel read Y: Y.first - R <= l and Y.second + R >= f
        const size_t k = (size_t)(std::upper_bound(cr.indel_reads.begin(), cr.indel_reads.end(), l + R,
                                                   [](int64_t v, const std::pair<int32_t, int32_t>& y) { return v < (int64_t)y.first; }) -
                                  cr.indel_reads.begin());
        return k > 0 && (int64_t)st.indel_pmax[k - 1] + R >= f;
    };
    const int64_t frontier = c->last_start;                // later indel reads start here or after
    for (size_t k = st.kept_maybe_from; k < st.kept.size(); k++) {
        auto& e = st.kept[k];
        if (!e.maybe) continue;
        if (covered(e.first, e.last)) e.maybe = false;
        else if ((int64_t)e.last + R < frontier) { e.maybe = false; e.dead = true; }
    }
    // the reads to keep (decided on all host threads: 0 no, 1 covered, 2 maybe), listed in order, their entries then
    // filled on all host threads
    const size_t k0 = st.kept.size();
    std::vector<uint8_t> how(n);
    const auto& Y = cr.indel_reads;
    const size_t ny = Y.size();
    parallel_for((int64_t)n, 1 << 14, [&](int64_t lo, int64_t hi) {
        // covered(f, l) with a cursor instead of a search per read: the reads come in start order (a search again
        // where one does not), so the indel reads with first <= f + R only grow; those up to l + R are a few more
        size_t k = 0;
        int64_t fprev = INT64_MAX;
        for (int64_t i = lo; i < hi; i++) {
            const int32_t f = cr.first[b0 + (size_t)i], l = cr.last[b0 + (size_t)i];
            if ((int64_t)f < fprev)
                k = (size_t)(std::upper_bound(Y.begin(), Y.end(), (int64_t)f + R,
                                              [](int64_t v, const std::pair<int32_t, int32_t>& y) { return v < (int64_t)y.first; }) - Y.begin());
            fprev = f;
            while (k < ny && (int64_t)Y[k].first <= (int64_t)f + R) k++;
            size_t kk = k;
            while (kk < ny && (int64_t)Y[kk].first <= (int64_t)l + R) kk++;
            const bool cov = kk > 0 && (int64_t)st.indel_pmax[kk - 1] + R >= f;
            how[(size_t)i] = cov ? 1 : (int64_t)l + R >= frontier ? 2 : 0;
        }
    });
    std::vector<size_t> src;
    for (size_t i = 0; i < n; i++) if (how[i]) src.push_back(i);
    st.kept.resize(k0 + src.size());
    // one block of bytes per slice of kept reads (CIGAR items, then characters and qualities), shared by their RawReads:
    // a copy for a second region is a view, and no read costs an allocation of its own
    parallel_for((int64_t)src.size(), 512, [&](int64_t q0, int64_t q1) {
        auto view = [&](int64_t q) {
            const size_t i = src[(size_t)q];
            return ent[i] >= 0 ? batch_view(c->cur_batch, ent[i]) : carried[-1 - ent[i]];
        };
        size_t bytes = 0;
        for (int64_t q = q0; q < q1; q++) {
            const ReadView r = view(q);
            bytes += (size_t)r.n_cigar * sizeof(int32_t) + (r.chars != nullptr && r.len > 0 ? 2 * (size_t)r.len : 0);
        }
        auto blk = std::make_shared<RawBlock>();
        blk->bytes.reset(new char[std::max<size_t>(bytes, 1)]);
        char* at = blk->bytes.get();
        std::shared_ptr<const RawBlock> hold = blk;
        // (the CIGAR items of the whole slice first: int32 alignment)
        char* tail = at;
        for (int64_t q = q0; q < q1; q++) tail += (size_t)view(q).n_cigar * sizeof(int32_t);
        for (int64_t q = q0; q < q1; q++) {
            const ReadView r = view(q);
            auto& e = st.kept[k0 + (size_t)q];
            e.first = cr.first[b0 + src[(size_t)q]];
            e.last = cr.last[b0 + src[(size_t)q]];
            e.maybe = how[src[(size_t)q]] == 2;
            e.dead = false;
            RawRead& rr = e.r;
            rr.first = r.first;
            rr.last = r.last;
            rr.flags = r.flags;
            rr.n_ops = r.n_cigar;
            std::memcpy(at, r.cigar, (size_t)r.n_cigar * sizeof(int32_t));
            rr.ops = reinterpret_cast<const int32_t*>(at);
            at += (size_t)r.n_cigar * sizeof(int32_t);
            rr.len = 0;
            rr.chars = rr.quals = nullptr;
            if (r.chars != nullptr && r.len > 0) {
                rr.len = r.len;
                char* ch = tail;
                char* qu = tail + r.len;
                tail += 2 * (size_t)r.len;
                if (r.packed) unpack_bases(r.chars, r.len, ch);
                else std::memcpy(ch, r.chars, (size_t)r.len);
                rr.chars = ch;
                if (r.quals != nullptr) {
                    if (r.packed) {
                        const uint8_t* rq = reinterpret_cast<const uint8_t*>(r.quals);
                        for (int32_t k = 0; k < r.len; k++) qu[k] = (char)(rq[k] > 222 ? 255 : rq[k] + 33);
                    } else std::memcpy(qu, r.quals, (size_t)r.len);
                    rr.quals = qu;
                }
            }
            rr.hold = hold;
            const bool neg = (r.flags & 0x10) != 0;            // setBasesToIgnore5P/3P (ReadAlignment.java:613-644)
            rr.ignore_start = neg ? c->params.ignore3 : c->params.ignore5;
            rr.ignore_end = neg ? c->params.ignore5 : c->params.ignore3;
            if (c->params.multisample) {                        // the read group's sample and its rank there
                const bool in = r.rg >= 0 && r.rg < (int32_t)c->rg_sample.size();
                rr.sample = (int16_t)(in ? c->rg_sample[(size_t)r.rg] : -1);
                rr.rank = (uint8_t)(in && c->rg_sample[(size_t)r.rg] >= 0 ? c->rg_rank[(size_t)r.rg] : 0);
            }
        }
    });
    while (st.kept_maybe_from < st.kept.size() && !st.kept[st.kept_maybe_from].maybe) st.kept_maybe_from++;
    if (!streaming(c)) {
        // a whole sequence is kept until its end (multisample): the reads no region can reach leave as they die
        size_t dead = 0;
        for (size_t k = st.kept_maybe_from; k < st.kept.size(); k++) dead += st.kept[k].dead ? 1 : 0;
        if (dead > (1u << 14) && dead * 2 > st.kept.size() - st.kept_maybe_from) {
            std::remove_reference_t<decltype(st.kept)> live;
            for (auto& e : st.kept) if (!e.dead) live.push_back(std::move(e));
            st.kept.swap(live);
            st.kept_maybe_from = 0;
            while (st.kept_maybe_from < st.kept.size() && !st.kept[st.kept_maybe_from].maybe) st.kept_maybe_from++;
        }
    }
}

// the realigner's regions (carve_indel_regions' geometry with the current R) that reach [lo, hi] -- merged, so a
// region that reaches them is returned whole (as far as the indel reads admitted so far make it)
static std::vector<std::pair<int64_t, int64_t>> regions_near(const ngsep_ctx* c, int64_t lo, int64_t hi) {
    const ContigReads& cr = c->contig;
    std::vector<std::pair<int64_t, int64_t>> out;
    if (cr.indel_reads.empty()) return out;
    const int64_t R = (int64_t)cr.max_span + 100, len = (int64_t)c->seq_bases[(size_t)cr.seq_id].size();
    std::vector<std::pair<int64_t, int64_t>> iv;
    for (size_t k = c->stream.indel_lo; k < cr.indel_reads.size(); k++) {
        const int64_t a = std::max<int64_t>(1, cr.indel_reads[k].first - R), b = std::min<int64_t>(len, (int64_t)cr.indel_reads[k].second + R);
        if (a > b) continue;
        iv.push_back({a, b});
    }
    std::sort(iv.begin(), iv.end());
    std::vector<std::pair<int64_t, int64_t>> merged;
    for (const auto& x : iv) {
        if (!merged.empty() && x.first <= merged.back().second + 1) merged.back().second = std::max(merged.back().second, x.second);
        else merged.push_back(x);
    }
    for (const auto& m : merged) if (m.second >= lo && m.first <= hi) out.push_back(m);
    return out;
}

static int flush_sequence(ngsep_ctx* c) {
    if (c->cur_seq < 0) return NGSEP_OK;
    process_same_start(c);
    project_pending(c);
    if (!c->strs.empty()) inject_strs(c, INT64_MAX);      // the sequence's remaining input STRs
    int rc;
    if (streaming(c)) {
        // the sequence's remaining windows, then its genotyped-position count
        rc = stream_advance(c, true);
        c->stats.positions_genotyped += c->contig.covered - c->stream.carved_inside;
        c->stream.next_w0 = 0;
        c->stream.indel_lo = c->stream.chunk_lo = 0;
        c->stream.carved_inside = 0;
        c->stream.kept.clear();
        c->stream.kept_maybe_from = 0;
        c->stream.indel_pmax.clear();
        c->stream.last_indel_end = 0;                // SingleSampleVariantPileupListener.onSequenceStart (:186)
    } else {
        rc = stage_contig_reads(c, c->contig, !c->staging_mode);
        c->stream.kept.clear();                      // (multisample: the realigner's alignments of the sequence)
        c->stream.kept_maybe_from = 0;
        c->stream.indel_pmax.clear();
        c->stream.last_indel_end = 0;
    }
    c->contig.clear();
    c->cur_seq = -1;
    return rc;
}

// The reach the replay needs for one realigner event [y1, y2] (an indel read's [first, last + indel bases], or an input
// variant's span): IndelRealignerPileupListener realigns the alignments of the pileups at the event's positions
// (conciliateIndels, moveIndelStarts) and writes the event's record there, so the calls it can change lie inside the
// extents of the admitted alignments that overlap [y1, y2], and DEF_REGION_BOUNDARY (:43) around them.  (carved
// regions handed back keep the coarser [y1 - R, y2 + R].)  Every alignment this reach needs was admitted before
// the frontier passed y2, and an alignment keep_raw dropped ends before frontier - R at the time, which is before
// every later event's reach -- a reach drawn with a span admitted after that drop would not be (the streamed
// chr20-with-indels run lacked two alignments of such a region).
static std::pair<int64_t, int64_t> event_reach(const ContigReads& cr, int64_t y1, int64_t y2, int64_t len) {
    int64_t L = y1, M = y2;
    const int64_t ms = std::max<int32_t>(1, cr.max_span);
    size_t i = (size_t)(std::lower_bound(cr.first.begin(), cr.first.end(), (int32_t)std::max<int64_t>(INT32_MIN, y1 - ms + 1)) - cr.first.begin());
    for (; i < cr.first.size() && (int64_t)cr.first[i] <= y2; i++)
        if ((int64_t)cr.last[i] >= y1) { L = std::min<int64_t>(L, cr.first[i]); M = std::max<int64_t>(M, cr.last[i]); }
    return {std::max<int64_t>(1, L - 100), std::min<int64_t>(len, M + 100)};
}

// IndelRealignerPileupListener's reach (ngsep_gpu.h ngsep_fetch_carved_regions): every indel-bearing
// admitted alignment carves [first - R, last + indel bases + R], R = max span + 100 (DEF_REGION_BOUNDARY,
// IndelRealignerPileupListener.java:43), merged; the covered positions inside leave the genotyped count
static void carve_indel_regions(ngsep_ctx* c, ContigReads& cr) {
    if (cr.indel_reads.empty()) return;
    const bool replay = realign_active(c);              // multisample: the regions are replayed, not handed back
    const int64_t R = (int64_t)cr.max_span + 100;
    const int64_t len = (int64_t)c->seq_bases[(size_t)cr.seq_id].size();
    std::vector<std::pair<int64_t, int64_t>> iv;
    for (const auto& x : cr.indel_reads)
        iv.push_back(replay ? event_reach(cr, x.first, x.second, len)        // (replayed here: the reach the replay needs)
                            : std::pair<int64_t, int64_t>{std::max<int64_t>(1, x.first - R), std::min<int64_t>(len, (int64_t)x.second + R)});
    std::sort(iv.begin(), iv.end());
    for (const auto& x : iv) {
        if (x.first > x.second) continue;
        if (!cr.carved.empty() && x.first <= (int64_t)cr.carved.back().second + 1)
            cr.carved.back().second = (int32_t)std::max<int64_t>(cr.carved.back().second, x.second);
        else cr.carved.push_back({(int32_t)x.first, (int32_t)x.second});
    }
    // covered positions inside the carved regions (reads sorted by first), also limited to the query range
    int64_t lo_q = 1, hi_q = len;
    if (c->params.query_seq[0]) { lo_q = std::max<int64_t>(lo_q, c->params.query_first); hi_q = std::min<int64_t>(hi_q, c->params.query_last); }
    int64_t inside = 0;
    size_t r0 = 0;
    if (replay) return;
    for (const auto& cv : cr.carved) {
        const int64_t a = std::max<int64_t>(cv.first, lo_q), b = std::min<int64_t>(cv.second, hi_q);
        c->carved.push_back({cr.seq_id, {cv.first, cv.second}});
        if (a > b) continue;
        while (r0 < cr.first.size() && (int64_t)cr.first[r0] + cr.max_span < a) r0++;
        int64_t run = a - 1;
        for (size_t i = r0; i < cr.first.size() && cr.first[i] <= b; i++) {
            const int64_t f = std::max<int64_t>(cr.first[i], a), l = std::min<int64_t>(cr.last[i], b);
            if (l < f || l <= run) continue;
            inside += l - std::max(f, run + 1) + 1;
            run = l;
        }
    }
    cr.covered -= inside;
    c->stats.carved_positions += inside;
}

static int run_population_regions(ngsep_ctx* c, const ContigReads& cr, size_t from);

int stage_contig_reads(ngsep_ctx* c, ContigReads& cr, bool run_now) {
    if (cr.seq_id < 0) return NGSEP_OK;
    if (!c->params.coverage_stats) carve_indel_regions(c, cr);
    c->stats.positions_genotyped += cr.covered;
    if (!run_now || c->params.coverage_stats) {     // coverage: one device run over all sequences at the end
        c->staged_contigs.emplace_back(std::move(cr));
        cr = ContigReads();
        return NGSEP_OK;
    }
    std::vector<ContigReads> one;
    one.emplace_back(std::move(cr));
    cr = ContigReads();
    int rc = build_and_upload(c, one, false);
    if (rc != NGSEP_OK) return rc;
    double ms = 0;
    const size_t from = c->pop_sites.size();
    rc = run_device(c, &ms);
    // MultisampleVariantsDetector with the indel realigner: the regions (kept out of the run above) replayed here
    if (rc == NGSEP_OK && c->params.multisample && realign_active(c) && !one[0].carved.empty())
        rc = run_population_regions(c, one[0], from);
    device_release(c->dev);
    return rc;
}

// ---- streamed single-sample windows ----
// While the alignments are read, every window of WL positions whose reads are all admitted (and whose
// carved indel regions are known: the stream is 2 R past it) is laid out, uploaded and run on a worker
// thread, one window at a time, while admission goes on; its records join the context's list in window
// order.  The window cut changes no call (windows carry a halo of the reads' span).
static int64_t stream_window_len(const ngsep_ctx* c) {
    static const int64_t env = diag_env("NGSEP_STREAM_WINDOW") ? std::atoll(diag_env("NGSEP_STREAM_WINDOW")) : 0;   // tuning
    int64_t w = env > 0 ? env : (int64_t)1 << 22;
    if (c->params.window_positions > 0) w = std::min<int64_t>(w, c->params.window_positions);
    return std::max<int64_t>(w, 1024);
}

static void run_window_job(ngsep_ctx* c, WindowJob* j);

// joins the window in flight: its records after those already called, then the projected chunks no later
// window reads are released
static int stream_collect(ngsep_ctx* c) {
    auto& st = c->stream;
    if (!st.job) return NGSEP_OK;
    const auto t_w = std::chrono::steady_clock::now();
    st.job->th.join();
    c->window_wait_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_w).count();
    std::unique_ptr<WindowJob> j = std::move(st.job);
    if (j->rc != NGSEP_OK) return set_error(c, j->rc, j->err);
    if (j->realign) st.last_indel_end = j->last_indel_end;
    if (c->params.relative_allele_counts) {
        auto& R = c->rac;
        double np = 0;
        for (int b = 0; b < 51; b++) {
            R.prop[b] += (double)j->rac_hist[b];
            np += (double)j->rac_hist[b];
            if (j->rac_seq_slot >= 0) R.seq_prop[(size_t)j->rac_seq_slot][(size_t)b] += (double)j->rac_hist[b];
        }
        R.prop_count += np;
        R.prop_sum += j->rac_sum;
        R.prop_sum_sq += j->rac_sum_sq;
        for (int b = 0; b < 10; b++) {
            const double n = (double)j->rac_hist[51 + b], v = (double)(b + 1);
            R.nall[b] += n;
            R.nall_count += n;
            R.nall_sum += n * v;            // (integers: exact in any order)
            R.nall_sum_sq += n * v * v;
        }
    }
    if (!c->known.empty() && !j->sites.empty()) {
        // the input variant of every record (sequence, position, ALT): its QS, and input order at a shared position
        const int64_t kb = c->known_seq_begin[(size_t)j->seq_id], ke = c->known_seq_begin[(size_t)j->seq_id + 1];
        std::vector<int64_t> kidx(j->sites.size());
        std::vector<int64_t> taken;                    // known entries already matched at the current position
        for (size_t i = 0; i < j->sites.size(); i++) {
            SiteRec& o = j->sites.rec[i];
            if (i == 0 || j->sites.rec[i - 1].pos != o.pos) taken.clear();
            if (o.is_call & kRecIndel) {                   // a non-SNV input variant's record: its index kept in L[1]
                kidx[i] = __builtin_bit_cast(int64_t, o.L[1]);
                continue;
            }
            auto it = std::lower_bound(c->known.begin() + kb, c->known.begin() + ke, (int64_t)o.pos,
                                       [](const ngsep_ctx::KnownVar& v, int64_t p) { return v.pos < p; });
            int64_t k = it - c->known.begin();
            while (k < ke && c->known[(size_t)k].pos == o.pos &&
                   (c->known[(size_t)k].alt != site_alt(o) || std::find(taken.begin(), taken.end(), k) != taken.end()))
                k++;
            taken.push_back(k);
            kidx[i] = k;
            if (k < ke) o.qual = c->known[(size_t)k].qs;
        }
        for (size_t i = 1; i < j->sites.size(); i++)            // (records at one position: input order)
            for (size_t k = i; k > 0 && j->sites.rec[k - 1].pos == j->sites.rec[k].pos && kidx[k - 1] > kidx[k]; k--) {
                std::swap(j->sites.rec[k - 1], j->sites.rec[k]);
                std::swap(kidx[k - 1], kidx[k]);
            }
    }
    if (c->sites.empty()) c->sites.swap(j->sites);
    else c->sites.append(j->sites);
    ContigReads& cr = c->contig;
    // (a later window's reads start at >= its w0 - max span + 1; reads ending 2 spans before it reach no tile of it)
    const int64_t keep_from = st.next_w0 - 2 * (int64_t)std::max<int32_t>(1, cr.max_span) - 64;
    while (st.chunk_lo + 1 < cr.chunks.size() && cr.chunk_maxlast[st.chunk_lo] < keep_from) {
        HostArray<uint8_t>& ch = cr.chunks[st.chunk_lo++];
        if (c->chunk_pool.size() < 4) c->chunk_pool.push_back(std::move(ch));   // the next batches' projections reuse it
        else ch.release();
    }
    return NGSEP_OK;
}

// hands [w0, w1] of the current sequence to the worker: its reads (first in [w0 - max span + 1, w1]) in
// window coordinates, and the carved indel regions inside it (carve_indel_regions' geometry with R = 100 +
// the longest span admitted so far)
static void stream_launch(ngsep_ctx* c, int64_t w0, int64_t w1) {
    auto& st = c->stream;
    ContigReads& cr = c->contig;
    const int32_t max_span = std::max<int32_t>(1, cr.max_span);
    const int64_t lo = std::lower_bound(cr.first.begin(), cr.first.end(), (int32_t)std::max<int64_t>(INT32_MIN, w0 - max_span + 1)) - cr.first.begin();
    const int64_t hi = std::upper_bound(cr.first.begin(), cr.first.end(), (int32_t)w1) - cr.first.begin();
    const int64_t len = (int64_t)c->seq_bases[(size_t)cr.seq_id].size();
    // carved regions: reported whole (clipped to the sequence, merged with what earlier windows reported),
    // applied clipped to the window
    std::vector<std::pair<int64_t, int64_t>> cut;
    if (!cr.indel_reads.empty() && !c->params.relative_allele_counts) {   // (no realigner in that listener chain)
        const int64_t R = (int64_t)cr.max_span + 100;
        while (st.indel_lo < cr.indel_reads.size() && (int64_t)cr.indel_reads[st.indel_lo].second + R < w0) st.indel_lo++;
        std::vector<std::pair<int64_t, int64_t>> whole;
        const bool tight = realign_active(c);             // replayed here: event_reach (carved regions: [y1 - R, y2 + R])
        for (size_t k = st.indel_lo; k < cr.indel_reads.size() && (int64_t)cr.indel_reads[k].first - R <= w1; k++) {
            int64_t a = std::max<int64_t>(1, cr.indel_reads[k].first - R), b = std::min<int64_t>(len, (int64_t)cr.indel_reads[k].second + R);
            if (tight) {
                const auto r = event_reach(cr, cr.indel_reads[k].first, cr.indel_reads[k].second, len);
                a = r.first;
                b = r.second;
            }
            if (a > b) continue;
            whole.push_back({a, b});
            if (std::max(a, w0) <= std::min(b, w1)) cut.push_back({std::max(a, w0), std::min(b, w1)});
        }
        std::sort(whole.begin(), whole.end());
        for (const auto& x : whole) {
            if (realign_active(c)) break;                 // (called here: nothing handed back)
            auto& v = c->carved;
            if (!v.empty() && v.back().first == cr.seq_id && x.first <= v.back().second.second + 1) {
                v.back().second.first = std::min(v.back().second.first, x.first);
                v.back().second.second = std::max(v.back().second.second, x.second);
            } else {
                v.push_back({cr.seq_id, {x.first, x.second}});
            }
        }
        std::sort(cut.begin(), cut.end());
        std::vector<std::pair<int64_t, int64_t>> merged;
        for (const auto& x : cut) {
            if (!merged.empty() && x.first <= merged.back().second + 1) merged.back().second = std::max(merged.back().second, x.second);
            else merged.push_back(x);
        }
        cut.swap(merged);
        // covered positions inside them (the realigner's regions are called here: they stay in the count)
        int64_t inside = 0;
        if (!realign_active(c)) {
            size_t r0 = (size_t)lo;
            for (const auto& cv : cut) {
                while (r0 < (size_t)hi && (int64_t)cr.first[r0] + cr.max_span < cv.first) r0++;
                int64_t run = cv.first - 1;
                for (size_t i = r0; i < (size_t)hi && cr.first[i] <= cv.second; i++) {
                    const int64_t f = std::max<int64_t>(cr.first[i], cv.first), l = std::min<int64_t>(cr.last[i], cv.second);
                    if (l < f || l <= run) continue;
                    inside += l - std::max(f, run + 1) + 1;
                    run = l;
                }
            }
            st.carved_inside += inside;
            c->stats.carved_positions += inside;
        }
    }
    std::vector<std::vector<RawRead>> region_reads;
    std::string region_err;
    const auto t_rr = std::chrono::steady_clock::now();
    if (realign_active(c)) {
        // the regions' alignments (whole regions: stream_advance never cuts one), in pending-list order; every
        // alignment that overlaps a region must have been kept
        region_reads.resize(cut.size());
        for (size_t k = 0; k < cut.size(); k++) {
            const int64_t a = cut[k].first, b = cut[k].second;
            // (kept entries and admitted reads are in start order: only those starting in [a - max span + 1, b] can
            // overlap the region)
            const int64_t from = std::max<int64_t>(INT32_MIN, a - max_span + 1);
            auto it = std::lower_bound(st.kept.begin(), st.kept.end(), from,
                                       [](const auto& e, int64_t v) { return (int64_t)e.first < v; });
            for (; it != st.kept.end() && (int64_t)it->first <= b; ++it) {
                if (it->dead || it->last < a) continue;
                // moved when no later region and no later window reads it (it ends in this window, before the next
                // region): the kept list drops it below; copied otherwise
                const bool last_use = it->last <= w1 && (k + 1 == cut.size() || (int64_t)it->last < cut[k + 1].first);
                if (last_use) region_reads[k].push_back(std::move(it->r));
                else region_reads[k].push_back(it->r);
            }
            size_t want = 0;
            const int64_t i0 = std::max<int64_t>(lo, std::lower_bound(cr.first.begin(), cr.first.end(), (int32_t)from) - cr.first.begin());
            for (int64_t i = i0; i < hi && cr.first[(size_t)i] <= b; i++) want += cr.last[(size_t)i] >= a ? 1 : 0;
            if (want != region_reads[k].size())
                region_err = "internal error: indel realigner region " + std::to_string(a) + "-" + std::to_string(b) + " lacks " +
                             std::to_string((int64_t)want - (int64_t)region_reads[k].size()) + " alignments";
        }
        // alignments that end in this window reach no later region
        std::remove_reference_t<decltype(st.kept)> keep;
        for (auto& e : st.kept) if (!e.dead && e.last > w1) keep.push_back(std::move(e));
        st.kept.swap(keep);
        st.kept_maybe_from = 0;
        c->region_gather_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_rr).count();
    }
    if (hi <= lo) return;                       // no read reaches the window: nothing to call
    auto j = std::make_unique<WindowJob>();
    if (realign_active(c)) {
        j->realign = true;
        j->region_reads.swap(region_reads);
        j->last_indel_end = st.last_indel_end;
        if (!region_err.empty()) { j->rc = NGSEP_E_INVALID; j->err = region_err; }
    }
    if (!c->known.empty()) {
        // -knownVariants: the window's input variants at positions with a pileup (onPileup, :158-176), outside
        // the carved regions; queue code 0x80 | ref << 5 | alt << 8 | 0x400 (kernels.hip k_posterior)
        const int32_t pad_k = ((max_span + 63) / 64) * 64;
        const int64_t goff_k = pad_k - w0;
        const int64_t kb = c->known_seq_begin[(size_t)cr.seq_id], ke = c->known_seq_begin[(size_t)cr.seq_id + 1];
        auto it = std::lower_bound(c->known.begin() + kb, c->known.begin() + ke, w0,
                                   [](const ngsep_ctx::KnownVar& v, int64_t p) { return v.pos < p; });
        size_t r = (size_t)lo, ci = 0;
        int64_t maxlast = INT64_MIN;
        for (; it != c->known.begin() + ke && it->pos <= w1; ++it) {
            const int64_t p = it->pos;
            if (it->alt < 0) continue;                                    // not an SNV: genotyped in its region
            while (r < (size_t)hi && cr.first[r] <= p) { maxlast = std::max<int64_t>(maxlast, cr.last[r]); r++; }
            if (maxlast < p) continue;                                    // no pileup here
            while (ci < cut.size() && cut[ci].second < p) ci++;
            if (ci < cut.size() && cut[ci].first <= p) continue;          // a realigner region: run_regions
            j->forced.push_back((int32_t)(p + goff_k));                   // a KP queue entry (SiteQ): no column yet
            j->forced.push_back(0x80 | (it->ref << 5) | (it->alt << 8) | 0x400);
            j->forced.push_back(0);
            j->forced.push_back(-1);
        }
    }
    j->seq_id = cr.seq_id;
    j->w0 = w0;
    j->w1 = w1;
    j->max_span = max_span;
    j->carved.swap(cut);
    j->rac_seq_slot = c->rac.cur_slot;
    const int32_t pad = ((max_span + 63) / 64) * 64;
    const int64_t goff = pad - w0;              // window position p -> global p + goff
    j->reads.resize((size_t)(hi - lo));
    SRead* out = j->reads.data();
    parallel_for(hi - lo, 1 << 16, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; i++) {
            const size_t k = (size_t)(lo + i);
            out[i] = SRead{(int32_t)(cr.first[k] + goff), (int32_t)(cr.last[k] + goff), cr.bptr[k], cr.neg[k]};
        }
    });
    WindowJob* jp = j.get();
    j->th = std::thread(run_window_job, c, jp);
    st.job = std::move(j);
    st.windows++;
}

// mid-stream (after a batch): the windows that are complete, while the worker keeps up; final (end of the
// sequence): every remaining window, then the last one is joined
static int stream_advance(ngsep_ctx* c, bool final) {
    auto& st = c->stream;
    ContigReads& cr = c->contig;
    if (cr.seq_id < 0 || cr.first.empty()) return final ? stream_collect(c) : NGSEP_OK;
    const int64_t len = (int64_t)c->seq_bases[(size_t)cr.seq_id].size();
    int64_t lo = std::max<int64_t>(1, cr.first.front()), hi = std::min<int64_t>(len, cr.cov_last);
    if (c->params.query_seq[0]) { lo = std::max<int64_t>(lo, c->params.query_first); hi = std::min<int64_t>(hi, c->params.query_last); }
    if (st.next_w0 == 0) st.next_w0 = lo;
    const int64_t WL = stream_window_len(c);
    const int64_t R = (int64_t)cr.max_span + 100;
    const int64_t limit = final ? hi : std::min<int64_t>(hi, (int64_t)c->last_start - 1 - 2 * R);
    while (st.next_w0 <= limit) {
        int64_t w1 = std::min<int64_t>(st.next_w0 + WL - 1, limit);
        if (!final && w1 - st.next_w0 + 1 < WL) break;          // mid-stream: whole windows only
        if (realign_active(c) && w1 < hi) {
            // a realigner region is never cut: the window ends before it, or after it once no later indel read
            // can reach it (its end + R before the admission frontier)
            bool wait = false;
            for (const auto& r : regions_near(c, w1, w1)) {
                if (!(r.first <= w1 && r.second > w1)) continue;
                if (final || r.second + R + 1 < (int64_t)c->last_start) w1 = std::min<int64_t>(r.second, hi);
                else if (r.first - 1 >= st.next_w0) w1 = r.first - 1;
                else wait = true;
            }
            if (wait) break;
        }
        if (st.job) {
            if (!final && !st.job->done.load()) break;           // the worker is busy: after the next batch
            const int rc = stream_collect(c);
            if (rc != NGSEP_OK) return rc;
        }
        const int64_t w0 = st.next_w0;
        st.next_w0 = w1 + 1;
        stream_launch(c, w0, w1);
    }
    if (final) return stream_collect(c);
    if (st.job && st.job->done.load()) return stream_collect(c);
    return NGSEP_OK;
}

// the open same-start group outlives the caller's batch: its reads' bytes move to the carry store
static void carry_open_group(ngsep_ctx* c) {
    if (c->ss_one >= 0) {
        c->ss_primary.push_back(batch_view(c->cur_batch, c->ss_one));
        c->ss_one = -1;
    }
    if (c->ss_primary.empty() && c->ss_secondary.empty()) return;
    CarryStore& cs = c->carry[c->carry_cur ^ 1];
    size_t nc = 0, nb = 0;
    for (auto* g : {&c->ss_primary, &c->ss_secondary})
        for (const ReadView& r : *g) { nc += (size_t)r.n_cigar; nb += (size_t)r.len; }
    cs.cigar.clear(); cs.chars.clear(); cs.quals.clear();
    cs.cigar.reserve(nc); cs.chars.reserve(nb); cs.quals.reserve(nb);
    for (auto* g : {&c->ss_primary, &c->ss_secondary})
        for (ReadView& r : *g) {
            const size_t co = cs.cigar.size(), so = cs.chars.size();
            cs.cigar.insert(cs.cigar.end(), r.cigar, r.cigar + r.n_cigar);
            if (r.chars) cs.chars.append(r.chars, (size_t)r.len);
            if (r.quals) cs.quals.append(r.quals, (size_t)r.len);
            else cs.quals.append((size_t)r.len, '\0');
            r.cigar = cs.cigar.data() + co;
            if (r.chars) r.chars = cs.chars.data() + so;
            if (r.quals) r.quals = cs.quals.data() + so;
            r.bidx = -1;
        }
    c->carry_cur ^= 1;
}

// AlignmentsPileupGenerator.processAlignment + processSameStartAlns (:377-433) over whole same-start groups [from, to)
// of the current batch, all on the current sequence: each thread takes a run of groups and lists its admitted reads
// (a lone primary alignment; otherwise the primaries, then the secondaries, at most max_alns_per_start per read group
// -- process_same_start's rule), then the lists are appended in order as admit_core would one by one: the sequence's
// read arrays, the projection list, the indel events (with the input STRs before them), the covered positions (a
// running union, the chunks' entry maxima as a prefix) and the longest span.
static void admit_middle(ngsep_ctx* c, int64_t from, int64_t to) {
    const ngsep_read_batch* b = c->cur_batch.b;
    const int32_t* lastp = c->cur_batch.last;
    const int32_t* indelp = c->cur_batch.indel;
    ContigReads& cr = c->contig;
    const int maxa = c->params.max_alns_per_start;
    const int nchunk = (int)std::max<int64_t>(1, std::min<int64_t>((to - from) >> 14, 4 * (int64_t)host_threads()));
    std::vector<int64_t> cut((size_t)nchunk + 1);
    cut[0] = from;
    cut[(size_t)nchunk] = to;
    for (int k = 1; k < nchunk; k++) {
        int64_t x = from + (to - from) * k / nchunk;
        while (x < to && b->first[x] == b->first[x - 1]) x++;
        cut[(size_t)k] = std::max(x, cut[(size_t)k - 1]);
    }
    struct Part {
        std::vector<int32_t> adm;
        std::vector<std::pair<int32_t, int32_t>> indels;
        int64_t hi_max = INT64_MIN, covered = 0;
        int32_t span_max = 0, last_max = INT32_MIN;
    };
    std::vector<Part> parts((size_t)nchunk);
    const int64_t len = cr.seq_len;
    parallel_for(nchunk, 1, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; k++) {
            Part& P = parts[(size_t)k];
            const int64_t a = cut[(size_t)k], z = cut[(size_t)k + 1];
            P.adm.reserve((size_t)(z - a));
            std::pair<int32_t, int32_t> tab[64];
            for (int64_t g = a; g < z;) {
                int64_t e = g + 1;
                while (e < z && b->first[e] == b->first[g]) e++;
                if (e - g == 1 && !(b->flags[g] & 0x100)) {
                    P.adm.push_back((int32_t)g);
                } else {
                    int n_rg = 0;
                    std::vector<std::pair<int32_t, int32_t>> big;
                    auto handle = [&](int64_t i) {
                        const int32_t rg = b->read_group ? b->read_group[i] : -1;
                        std::pair<int32_t, int32_t>* t = big.empty() ? tab : big.data();
                        for (int q = 0; q < n_rg; q++)
                            if (t[q].first == rg) {
                                if (maxa <= 0 || t[q].second < maxa) { t[q].second++; P.adm.push_back((int32_t)i); }
                                return;
                            }
                        if (n_rg == 64 && big.empty()) big.assign(tab, tab + 64);
                        if (big.empty()) tab[n_rg] = {rg, 1};
                        else big.push_back({rg, 1});
                        n_rg++;
                        P.adm.push_back((int32_t)i);
                    };
                    for (int64_t i = g; i < e; i++) if (!(b->flags[i] & 0x100)) handle(i);
                    for (int64_t i = g; i < e; i++) if (b->flags[i] & 0x100) handle(i);
                }
                g = e;
            }
            for (int64_t i = a; i < z; i++) P.last_max = std::max(P.last_max, lastp[i]);
            for (int32_t i : P.adm) {
                const int32_t f = b->first[i], l = lastp[i];
                if (indelp[i] > 0) P.indels.push_back({f, l + indelp[i]});
                P.span_max = std::max(P.span_max, l - f + 1);
                const int64_t lo = std::max<int64_t>(f, 1), hi = std::min<int64_t>(l, len);
                if (hi >= lo) P.hi_max = std::max(P.hi_max, hi);
            }
        }
    });
    // offsets, the entry union maximum of every chunk, the arrays filled in parallel
    std::vector<int64_t> off((size_t)nchunk + 1, 0);
    std::vector<int64_t> m_in((size_t)nchunk + 1);
    m_in[0] = cr.cov_last;
    for (int k = 0; k < nchunk; k++) {
        off[(size_t)k + 1] = off[(size_t)k] + (int64_t)parts[(size_t)k].adm.size();
        m_in[(size_t)k + 1] = std::max<int64_t>(m_in[(size_t)k], parts[(size_t)k].hi_max);
    }
    const int64_t total = off[(size_t)nchunk];
    const size_t r0 = cr.first.size(), p0 = c->to_project.size();
    cr.first.resize(r0 + (size_t)total);
    cr.last.resize(r0 + (size_t)total);
    cr.neg.resize(r0 + (size_t)total);
    c->to_project.resize(p0 + (size_t)total);
    const bool ms = c->params.multisample != 0;          // (the read group's sample and rank, as admit_core)
    if (ms) {
        cr.sample.resize(r0 + (size_t)total);
        cr.rank.resize(r0 + (size_t)total);
    }
    parallel_for(nchunk, 1, [&](int64_t k0, int64_t k1) {
        for (int64_t k = k0; k < k1; k++) {
            Part& P = parts[(size_t)k];
            const size_t o = (size_t)off[(size_t)k];
            int64_t m = m_in[(size_t)k];
            for (size_t j = 0; j < P.adm.size(); j++) {
                const int32_t i = P.adm[j], f = b->first[i], l = lastp[i];
                cr.first[r0 + o + j] = f;
                cr.last[r0 + o + j] = l;
                cr.neg[r0 + o + j] = (b->flags[i] & 0x10) ? 1 : 0;
                c->to_project[p0 + o + j] = i;
                if (ms) {
                    const int32_t rg = b->read_group ? b->read_group[i] : -1;
                    const bool in = rg >= 0 && rg < (int32_t)c->rg_sample.size();
                    cr.sample[r0 + o + j] = (int16_t)(in ? c->rg_sample[(size_t)rg] : -1);
                    cr.rank[r0 + o + j] = (uint8_t)(in && c->rg_sample[(size_t)rg] >= 0 ? c->rg_rank[(size_t)rg] : 0);
                }
                const int64_t lo = std::max<int64_t>(f, 1), hi = std::min<int64_t>(l, len);
                if (hi >= lo) {
                    if (lo > m) P.covered += hi - lo + 1;
                    else if (hi > m) P.covered += hi - m;
                    if (hi > m) m = hi;
                }
            }
        }
    });
    for (int k = 0; k < nchunk; k++) {
        const Part& P = parts[(size_t)k];
        for (const auto& ev : P.indels) {
            if (!c->strs.empty()) inject_strs(c, ev.first);
            cr.indel_reads.push_back(ev);
        }
        cr.covered += P.covered;
        cr.max_span = std::max(cr.max_span, P.span_max);
        if (P.last_max > c->cur_last) c->cur_last = P.last_max;
    }
    if (!c->strs.empty() && total > 0) inject_strs(c, cr.first.back());
    cr.cov_last = (int32_t)std::max<int64_t>(cr.cov_last, m_in[(size_t)nchunk]);
    c->stats.alignments_admitted += total;
}

static int process_batch(ngsep_ctx* c, const ngsep_read_batch* b, bool packed, const int64_t* qual_off = nullptr,
                         const char* const* chars_at = nullptr, const char* const* quals_at = nullptr) {
    if (!b || b->n_reads < 0) return set_error(c, NGSEP_E_INVALID, "null batch");
    const int nseq = (int)c->seq_names.size();
    int rc = NGSEP_OK;
    const auto t0 = std::chrono::steady_clock::now();
    {   // the batch's admitted reads land in these: at most one (geometric) growth per batch
        ContigReads& cr = c->contig;
        const size_t k = (size_t)b->n_reads;
        auto grow = [k](auto& v) { if (v.capacity() < v.size() + k) v.reserve(std::max(v.size() + k, 2 * v.capacity())); };
        grow(c->to_project);
        grow(cr.first);
        grow(cr.last);
        if (c->params.coverage_stats) grow(cr.uniq);
        else grow(cr.neg);
        grow(cr.bptr);
    }
    // the alignments' reference ends, indel bases and read lengths from their CIGARs (all threads)
    thread_local std::vector<int32_t> lastv, indelv, rlenv;
    if (lastv.size() < (size_t)b->n_reads) {
        lastv.resize((size_t)b->n_reads);
        indelv.resize((size_t)b->n_reads);
        rlenv.resize((size_t)b->n_reads);
    }
    int32_t* lastp = lastv.data();       // (the workers see their own thread_local instances)
    int32_t* indelp = indelv.data();
    int32_t* rlenp = rlenv.data();
    parallel_for(b->n_reads, 1 << 15, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            const int32_t* cg = b->cigar + b->cigar_off[i];
            int32_t last = b->first[i] - 1, read_length = 0, indel_len = 0;
            for (int32_t k = 0; k < b->cigar_n[i]; k++) {
                const int32_t v = cg[k], op = v & 7;
                if (op == 1 || op == 2) indel_len += v / 8;
                if (v & 1) last += v / 8;
                if (v & 2) read_length += v / 8;
            }
            lastp[i] = last;
            indelp[i] = indel_len;
            rlenp[i] = read_length;
        }
    });
    c->cur_batch = BatchRef{b, lastp, indelp, packed, qual_off, chars_at, quals_at};
    int64_t n_in = 0;
    // the admission sweep (processAlignment + processSameStartAlns) over reads [from, to); false: stop the batch
    auto sweep = [&](int64_t from, int64_t to) -> bool {
    for (int64_t i = from; i < to; i++) {
        if (c->query_done) return false;
        n_in++;
        struct { int32_t seq_id, first, flags; } r{b->seq_id[i], b->first[i], b->flags[i]};
        if (r.seq_id < 0 || r.seq_id >= nseq) {
            rc = set_error(c, NGSEP_E_INVALID, "alignment on unknown sequence id " + std::to_string(r.seq_id));
            return false;
        }
        const int32_t last = lastp[i], read_length = rlenp[i];
        const int32_t sl = b->seq_len[i];
        if (sl > 0 && read_length != sl) continue;   // ReadAlignment.setReadCharacters throws -> record skipped
        // querySeq handling (AlignmentsPileupGenerator.java:342-354)
        if (c->params.query_seq[0]) {
            if (c->seq_names[r.seq_id] == c->params.query_seq) {
                c->query_found = true;
                if (r.first > c->params.query_last) { c->query_done = true; return false; }
                if (c->params.query_first > last) continue;
            } else if (c->query_found) {
                c->query_done = true;
                return false;
            } else {
                continue;
            }
        }
        // processAlignment (:377-403)
        if (c->cur_seq >= 0) {
            bool same = c->cur_seq == r.seq_id;
            if (same && r.first < c->last_start) {
                rc = set_error(c, NGSEP_E_INVALID, "alignments are not coordinate-sorted");
                return false;
            }
            if (!same || c->last_start != r.first) {
                process_same_start(c);
                if (!same) {
                    rc = flush_sequence(c);
                    if (rc != NGSEP_OK) return false;
                }
            }
        }
        if (c->cur_seq < 0) {   // startSequence (:435-444)
            c->cur_seq = r.seq_id;
            c->contig.clear();
            c->contig.seq_id = r.seq_id;
            c->contig.seq_len = (int64_t)c->seq_bases[(size_t)r.seq_id].size();
            c->cur_last = last;
            c->str_next = 0;                             // IndelRealignerPileupListener.onSequenceStart (:128-133)
            if (c->reads_hint > 0 && !c->params.coverage_stats) {
                int64_t glen = 0;
                for (const std::string& q : c->seq_bases) glen += (int64_t)q.size();
                const int64_t want = (int64_t)((double)c->reads_hint * (double)c->contig.seq_len / (double)std::max<int64_t>(glen, 1) * 1.25) + 4096;
                ContigReads& cr = c->contig;
                if ((int64_t)cr.first.capacity() < want) {
                    cr.first.reserve((size_t)want);
                    cr.last.reserve((size_t)want);
                    cr.neg.reserve((size_t)want);
                    cr.bptr.reserve((size_t)want);
                }
            }
            if (c->params.relative_allele_counts) {      // onSequenceStart (RelativeAlleleCountsCalculator.java:312-322)
                if (c->contig.seq_len > 100000) {
                    c->rac.seq_names.push_back(c->seq_names[(size_t)r.seq_id]);
                    c->rac.seq_prop.emplace_back(51, 0.0);
                    c->rac.cur_slot = (int32_t)c->rac.seq_prop.size() - 1;
                } else {
                    c->rac.cur_slot = -1;
                }
            }
        }
        if (last > c->cur_last) c->cur_last = last;
        // the open same-start group: a lone primary alignment stays an index (no view is built)
        if (!(r.flags & 0x100) && c->ss_one < 0 && c->ss_primary.empty() && c->ss_secondary.empty()) {
            c->ss_one = (int32_t)i;
        } else {
            if (c->ss_one >= 0) { c->ss_primary.push_back(batch_view(c->cur_batch, c->ss_one)); c->ss_one = -1; }
            if (r.flags & 0x100) c->ss_secondary.push_back(batch_view(c->cur_batch, (int32_t)i));
            else c->ss_primary.push_back(batch_view(c->cur_batch, (int32_t)i));
        }
        c->last_start = r.first;
    }
    return true;
    };
    // the batch's middle -- whole same-start groups of the current sequence -- admitted on all threads
    // (admit_middle); its first group (which may continue the carried one) and its last (left open) go through the
    // sweep.  Only for a sorted batch of the current sequence whose reads all carry their characters' length.
    int64_t g1 = 0, gL = 0;
    // (single-sample streamed runs and MultisampleVariantsDetector's merged batches)
    const bool middle_ok = streaming(c) || (c->params.multisample && !c->staging_mode && !c->params.coverage_stats);
    if (middle_ok && !c->params.query_seq[0] && b->n_reads >= (1 << 16) && c->cur_seq >= 0 &&
        b->seq_id[0] == c->cur_seq && b->first[0] >= c->last_start) {
        const int64_t n = b->n_reads;
        std::atomic<bool> bad{false};
        parallel_for(n, 1 << 15, [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi && !bad.load(std::memory_order_relaxed); i++) {
                const int32_t sl = b->seq_len[i];
                if (b->seq_id[i] != c->cur_seq || (i > 0 && b->first[i] < b->first[i - 1]) || (sl > 0 && rlenp[i] != sl)) bad = true;
            }
        });
        if (!bad) {
            g1 = 1;
            while (g1 < n && b->first[g1] == b->first[0]) g1++;
            gL = n - 1;
            while (gL > 0 && b->first[gL - 1] == b->first[n - 1]) gL--;
        }
    }
    if (g1 < gL) {
        if (sweep(0, g1)) {
            process_same_start(c);                       // read g1 starts another group
            admit_middle(c, g1, gL);
            n_in += gL - g1;
            c->last_start = b->first[gL - 1];
            sweep(gL, b->n_reads);
        }
    } else {
        sweep(0, b->n_reads);
    }
    c->stats.alignments_in += n_in;
    // the admitted reads' bytes are projected while the batch is alive; the open group is carried
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto t1 = std::chrono::steady_clock::now();
    // -knownSTRs: the input STRs that start at or before the open group's start join the events now, not when a read
    // at or after them is admitted: keep_raw's frontier and stream_advance's limit both take last_start as the point
    // before which nothing more can start (a coverage gap after an STR would otherwise leave it out of the window's
    // regions).  The order among the events is unchanged: admit_core injects STRs up to a read's start before it.
    if (!c->strs.empty() && c->contig.seq_id >= 0 && c->last_start > 0) inject_strs(c, c->last_start);
    project_pending(c);
    const auto t2 = std::chrono::steady_clock::now();
    if (rc == NGSEP_OK && streaming(c)) rc = stream_advance(c, false);
    const auto t3 = std::chrono::steady_clock::now();
    carry_open_group(c);
    if (host_timing)
        std::fprintf(stderr, "[ngsep host] batch of %lld: admission %.1f ms, projection %.1f ms, stream %.1f ms, carry %.1f ms\n",
                     (long long)b->n_reads, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                     std::chrono::duration<double, std::milli>(t2 - t1).count(),
                     std::chrono::duration<double, std::milli>(t3 - t2).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t3).count());
    return rc;
}

// ---- staging: fixed-stride slot layout of every window's reads ----

static inline uint8_t ref_code(const ngsep_ctx* c, char ch) {
    if (c->params.ignore_lowercase_ref && std::islower((unsigned char)ch)) return kRefInWindow;   // :198
    int a = dna_index((char)std::toupper((unsigned char)ch));                                      // :199
    if (a < 0) return kRefInWindow;    // VariantDiscoverySNVQAlgorithm.java:104-107 (N reference)
    return (uint8_t)(kRefCallable | (a << 5));
}

// reference codes of window w in global coordinates; carved indel regions get no code (no call is made there)
static void fill_ref_codes(const ngsep_ctx* c, Staged& s, const Window& w, const std::vector<std::pair<int64_t, int64_t>>& carved) {
    const std::string& ref = c->seq_bases[w.seq_id];
    uint8_t* dst = &s.h_ref[(size_t)(w.gbase + w.pad)];
    uint8_t tab[256];
    for (int ch = 0; ch < 256; ch++) tab[ch] = ref_code(c, (char)ch);
    parallel_for(w.wlen, 1 << 18, [&](int64_t lo, int64_t hi) {
        for (int64_t k = lo; k < hi; k++) dst[k] = tab[(uint8_t)ref[(size_t)(w.w0 - 1 + k)]];
    });
    for (const auto& cv : carved) {
        const int64_t a = std::max<int64_t>(cv.first, w.w0), b = std::min<int64_t>(cv.second, (int64_t)w.w0 + w.wlen - 1);
        if (a <= b) std::memset(dst + (a - w.w0), 0, (size_t)(b - a + 1));
    }
}

// ---- tile-blocked pileup (engine.hpp TileInfo) ----
// maxima of the per-position depth over blocks of 16 positions (difference array over the read table)
static std::vector<int32_t> depth_max16(const int32_t* R, int64_t nreads, int stride, int64_t g_len) {
    std::vector<int32_t> cov((size_t)g_len + 1, 0);
    for (int64_t i = 0; i < nreads; i++) {
        const int32_t a = R[i * stride], b = R[i * stride + 1];
        if (b < a) continue;
        cov[(size_t)a]++;
        cov[(size_t)b + 1]--;
    }
    std::vector<int32_t> m16((size_t)(g_len / kTileMinPos), 0);
    int32_t run = 0;
    for (int64_t p = 0; p < (int64_t)m16.size() * kTileMinPos; p++) {
        run += cov[(size_t)p];
        int32_t& m = m16[(size_t)(p / kTileMinPos)];
        if (run > m) m = run;
    }
    return m16;
}
static std::vector<int32_t> widen_max(const std::vector<int32_t>& m16, int T, int64_t ntiles) {
    std::vector<int32_t> c = m16;
    for (int t = kTileMinPos; t < T; t *= 2) {
        std::vector<int32_t> nxt((c.size() + 1) / 2);
        for (size_t i = 0; i < nxt.size(); i++) nxt[i] = std::max(c[2 * i], 2 * i + 1 < c.size() ? c[2 * i + 1] : 0);
        c.swap(nxt);
    }
    c.resize((size_t)ntiles, 0);
    return c;
}
// Tile width of the single-sample layout: KT scans bit planes of 128, 256 or 512 positions (one wavefront
// per tile, W = T/32 words per plane row).  Each width is costed as the planes' bytes (a quarter of
// sum rows_t * T) plus a fixed per-tile cost for the tile's instruction stream.  Measured on the 30x
// yeast / chr20 genomes (round 1): T = 512 scans in 0.041 / 0.144 ms vs 0.048 / 0.188 ms at T = 256.
static int choose_tile(const std::vector<int32_t>& m16, int64_t g_len, std::vector<int32_t>& rows_out) {
    int bestT = 512;
    double best_cost = -1;
    for (int T : {128, 256, 512}) {
        const int64_t ntiles = g_len / T;
        const std::vector<int32_t> r = widen_max(m16, T, ntiles);
        double bytes = 0;
        for (int64_t t = 0; t < ntiles; t++) bytes += (double)r[(size_t)t] * T;
        const double cost = bytes / 4 + 2048.0 * (double)ntiles;
        if (best_cost < 0 || cost < best_cost) { best_cost = cost; bestT = T; }
    }
    if (const char* e = diag_env("NGSEP_TILE_T")) {   // tests and tuning: a fixed tile width
        const int T = std::atoi(e);
        if (T == 128 || T == 256 || T == 512) bestT = T;
    }
    rows_out = widen_max(m16, bestT, g_len / bestT);
    return bestT;
}

// Single-sample layout: tiles of T positions; tile t has rows_t = its maximum depth
// and, at every position p, the codes of the reads covering p in pending-list order -- the order in which
// PileupRecord.getAlleleCalls (PileupRecord.java:126-152) visits them -- in ranks 0, 1, ... (rank r at p is
// the r-th covering read).  Three products per tile:
//   * the valid-call plane (KT): rank row r holds W = T/32 words of "valid call" bits; the tile's plane
//     starts at word off_t / 32;
//   * the other-allele list (KT): the tile-relative position of every valid call of another allele than
//     the reference, ascending (a position appears once per such call), at entry loff_t;
//   * the position-major byte pile (KP): position p's rows_t codes at off_t + p * rows_t, rank order;
//   * the strand bits (KP, countsStrand): bit off_t + p * rows_t + r = the rank-r read is reverse.
// Tiles are independent: built on all host threads.
static int build_single_layout(Staged& s, const RawVec<SRead>& reads, LayoutArena& arena, bool exact) {
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    auto lap = [t = std::chrono::steady_clock::now()](const char* what) mutable {
        if (!host_timing) return;
        const auto n = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngsep host]   layout %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(n - t).count());
        t = n;
    };
    const int64_t g_len = s.g_len, nreads = (int64_t)reads.size();
    std::vector<int32_t> R2((size_t)nreads * 2);
    for (int64_t i = 0; i < nreads; i++) { R2[(size_t)(2 * i)] = reads[(size_t)i].gfirst; R2[(size_t)(2 * i + 1)] = reads[(size_t)i].glast; }
    std::vector<int32_t> rows;
    const int T = choose_tile(depth_max16(R2.data(), nreads, 2, g_len), g_len, rows);
    std::vector<int32_t>().swap(R2);
    lap("depth + tile choice");
    const int64_t ntiles = g_len / T;
    s.tile = T;
    s.n_tiles = ntiles;
    s.h_tinfo.resize((size_t)ntiles);
    int64_t off = 0;
    int32_t rmax = 0;
    for (int64_t t = 0; t < ntiles; t++) {
        s.h_tinfo[(size_t)t].off = off;
        s.h_tinfo[(size_t)t].rows = rows[(size_t)t];
        s.h_tinfo[(size_t)t].pad = 0;
        off += (int64_t)rows[(size_t)t] * T;
        rmax = std::max(rmax, rows[(size_t)t]);
    }
    s.pile_bytes = off;
    s.tile_rows_max = rmax;
    // first read that can reach tile t (reads are sorted by global first position)
    auto first_read = [&](int64_t t) -> int64_t {
        const int64_t lo_pos = t * T - s.max_span;
        return std::lower_bound(reads.begin(), reads.end(), lo_pos, [](const SRead& r, int64_t v) { return (int64_t)r.gfirst <= v; }) - reads.begin();
    };
    if (!arena.ensure(off, exact)) return -2;
    s.h_cpile = arena.cpile;
    s.h_planes = arena.planes;
    s.h_cneg = arena.cneg;
    lap("tile table + alloc");
    const int W = T / 32;
    const uint8_t* ref = s.h_ref.data();
    std::atomic<int> bad{0};
    // tiles in chunks of 256 (each chunk's other-allele lists are concatenated after the parallel pass)
    const int64_t kChunk = 256, nchunk = (ntiles + kChunk - 1) / kChunk;
    std::vector<std::vector<uint16_t>> chunk_list((size_t)nchunk);
    std::vector<int32_t> tile_nl((size_t)ntiles + 1, 0);
    parallel_for(nchunk, 1, [&](int64_t c0, int64_t c1) {
        std::vector<int32_t> fill((size_t)T);
        std::vector<uint16_t> na((size_t)T);
        for (int64_t ch = c0; ch < c1; ch++) {
            const int64_t t0 = ch * kChunk, t1 = std::min(ntiles, t0 + kChunk);
            std::vector<uint16_t>& lst = chunk_list[(size_t)ch];
            int64_t r_lo = first_read(t0);
            for (int64_t t = t0; t < t1; t++) {
                const int32_t nrow = rows[(size_t)t];
                const int32_t tstart = (int32_t)(t * T), tend = tstart + T;
                while (r_lo < nreads && (int64_t)reads[(size_t)r_lo].gfirst <= (int64_t)tstart - s.max_span) r_lo++;
                if (!nrow) continue;
                const int64_t toff = s.h_tinfo[(size_t)t].off;
                uint8_t* col = s.h_cpile + toff;
                uint32_t* pl = s.h_planes + toff / 32;
                uint32_t* ng = s.h_cneg + toff / 32;
                std::memset(col, 0, (size_t)nrow * T);
                std::memset(pl, 0, (size_t)nrow * T / 8);
                std::memset(ng, 0, (size_t)nrow * T / 8);
                std::fill(fill.begin(), fill.end(), 0);
                std::fill(na.begin(), na.end(), (uint16_t)0);
                for (int64_t r = r_lo; r < nreads && reads[(size_t)r].gfirst < tend; r++) {
                    const SRead& rd = reads[(size_t)r];
                    if (rd.glast < tstart || rd.glast < rd.gfirst) continue;
                    const int32_t a = std::max(rd.gfirst, tstart) - tstart, b = std::min(rd.glast, tend - 1) - tstart;
                    const uint8_t* src = rd.bytes + (tstart + a - rd.gfirst);
                    for (int32_t p = a; p <= b; p++) {
                        const int32_t rank = fill[(size_t)p]++;
                        if (rank >= nrow) { bad = 1; continue; }
                        const uint8_t cd = src[p - a];
                        const int64_t cell = (int64_t)p * nrow + rank;
                        col[cell] = cd;
                        if (rd.neg) ng[cell >> 5] |= 1u << (cell & 31);
                        if (cd & kCodeValid) {
                            const uint8_t rc = ref[tstart + p];
                            const uint8_t ra = (rc & kRefCallable) ? (uint8_t)((rc >> 5) & 3) : 0;
                            pl[(size_t)rank * W + (p >> 5)] |= 1u << (p & 31);
                            if (((cd >> 5) & 3) != ra) na[(size_t)p]++;
                        }
                    }
                }
                // the tile's other-allele calls: their positions, ascending (one entry per call)
                const size_t before = lst.size();
                for (int32_t p = 0; p < T; p++) lst.insert(lst.end(), na[(size_t)p], (uint16_t)p);
                tile_nl[(size_t)t] = (int32_t)(lst.size() - before);
            }
        }
    });
    s.h_loff.assign((size_t)ntiles + 1, 0);
    for (int64_t t = 0; t < ntiles; t++) s.h_loff[(size_t)t + 1] = s.h_loff[(size_t)t] + tile_nl[(size_t)t];
    s.h_olist.resize((size_t)s.h_loff[(size_t)ntiles] + 64);      // + 64: KT reads a whole wave of entries
    std::vector<int64_t> cbase((size_t)nchunk + 1, 0);
    for (int64_t ch = 0; ch < nchunk; ch++) cbase[(size_t)ch + 1] = cbase[(size_t)ch] + (int64_t)chunk_list[(size_t)ch].size();
    parallel_for(nchunk, 16, [&](int64_t c0, int64_t c1) {
        for (int64_t ch = c0; ch < c1; ch++)
            if (!chunk_list[(size_t)ch].empty())
                std::memcpy(&s.h_olist[(size_t)cbase[(size_t)ch]], chunk_list[(size_t)ch].data(), chunk_list[(size_t)ch].size() * 2);
    });
    std::fill(s.h_olist.end() - 64, s.h_olist.end(), (uint16_t)0);
    lap("tiles");
    return bad ? -1 : 0;
}

// One 64-read group of a read-group layout: unit k of lane l (the read's bytes 8k .. 8k+7, XOR-ed with the reference,
// zero past its end) at dst[64 k + l].  Written one 64-byte line (8 lanes) at a time with streaming stores: a line
// written whole needs no read-for-ownership, so the layout costs its bytes once instead of twice (span 0: an empty
// lane).  The caller fences (_mm_sfence) before the layout is uploaded.
static inline void fill_group_units(uint64_t* dst, int32_t K, const uint8_t* const* src, const uint8_t* const* rf,
                                    const int64_t* span) {
    for (int32_t k = 0; k < K; k++) {
        const int64_t o = 8 * (int64_t)k;
        for (int lb = 0; lb < 64; lb += 8) {
            alignas(16) uint64_t line[8];
            for (int l = lb; l < lb + 8; l++) {
                uint64_t v = 0;
                const int64_t sp = span[l];
                if (o + 8 <= sp) {
                    uint64_t u, w;
                    std::memcpy(&u, src[l] + o, 8);
                    std::memcpy(&w, rf[l] + o, 8);
                    v = u ^ w;
                } else if (o < sp) {
                    uint8_t b8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    for (int64_t t = 0; t < sp - o; t++) b8[t] = (uint8_t)(src[l][o + t] ^ rf[l][o + t]);
                    std::memcpy(&v, b8, 8);
                }
                line[l - lb] = v;
            }
            __m128i* d = reinterpret_cast<__m128i*>(dst + o * 8 + lb);
            const __m128i* q = reinterpret_cast<const __m128i*>(line);
            _mm_stream_si128(d, _mm_load_si128(q));
            _mm_stream_si128(d + 1, _mm_load_si128(q + 1));
            _mm_stream_si128(d + 2, _mm_load_si128(q + 2));
            _mm_stream_si128(d + 3, _mm_load_si128(q + 3));
        }
    }
}

// Read-group layout (engine.hpp RGroup): the variant caller's device input.  The reads'
// projected bytes are the ones the host packer produced (one code byte per reference position of the read,
// pending-list order), stored relative to the reference (code ^ reference code, as CRAM stores bases against the
// reference): KL then needs no reference in its stream, and a gather restores the code with one byte per
// position.  Regrouped so that the scan's loads coalesce: 64 consecutive reads per group, interleaved in 8-byte
// units.  Headers: global first / last position and the strand bit.  The two
// block tables give the scan its tile's entry range and the column gather the entries that can cover a
// position.  Groups are independent: built on all host threads.
// consumed (a staged whole-genome run): called after every slice of groups with the reads whose bytes are in place, so
// the caller can return their projected chunks while the rest is filled (peak host memory ~ one copy, not two)
// device_units (streamed windows): the units are built on the device (kernels.hip k_build_units) from the reads'
// projected bytes, copied here back to back into the arena (runs of reads adjacent in their projection chunk: one copy)
// -- a copy instead of the 64-lane transposition with its reference XOR, which cost the window worker ~10 ms a window
// out[e] = max(glast of entries 0 .. e) (non-decreasing: the first entry reaching a position is a lower_bound), on all
// threads (per-chunk maxima, then the chunks' carried maxima)
template <class F>
static void prefix_max_glast(int64_t n, F&& glast, int32_t* out) {
    if (n <= 0) return;
    const int64_t kChunk = 1 << 16, nch = (n + kChunk - 1) / kChunk;
    std::vector<int32_t> cmax((size_t)nch, INT32_MIN);
    parallel_for(nch, 1, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; c++) {
            int32_t m = INT32_MIN;
            for (int64_t e = c * kChunk; e < std::min(n, (c + 1) * kChunk); e++) m = std::max<int32_t>(m, glast(e));
            cmax[(size_t)c] = m;
        }
    });
    std::vector<int32_t> carry((size_t)nch, INT32_MIN);
    for (int64_t c = 1; c < nch; c++) carry[(size_t)c] = std::max(carry[(size_t)c - 1], cmax[(size_t)c - 1]);
    parallel_for(nch, 1, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; c++) {
            int32_t m = carry[(size_t)c];
            for (int64_t e = c * kChunk; e < std::min(n, (c + 1) * kChunk); e++) out[e] = m = std::max<int32_t>(m, glast(e));
        }
    });
}

static int build_rg_layout(Staged& s, const RawVec<SRead>& reads, LayoutArena& arena, bool exact,
                           const std::function<void(int64_t)>& consumed = nullptr, bool device_units = false) {
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto t0 = std::chrono::steady_clock::now();
    const int64_t n = (int64_t)reads.size();
    const int64_t ng = (n + 63) / 64, ne = ng * 64;
    s.rg = true;
    s.tile = kKlTile;
    s.n_tiles = s.g_len / kKlTile;
    s.n_entries = ne;
    s.n_groups = ng;
    s.h_rh.resize((size_t)ne * 2);
    s.h_grp.resize((size_t)ng);
    // groups: units per read and unit offsets
    int64_t base = 0;
    for (int64_t g = 0; g < ng; g++) {
        int32_t K = 0;
        for (int64_t e = g * 64; e < std::min(n, g * 64 + 64); e++) {
            const int64_t span = (int64_t)reads[(size_t)e].glast - reads[(size_t)e].gfirst + 1;
            if (span > 0) K = std::max<int32_t>(K, (int32_t)((span + 7) / 8));
        }
        s.h_grp[(size_t)g] = RGroup{base, K, 0};
        base += (int64_t)K * 64;
    }
    s.n_units = base;
    const int32_t last_first = n ? reads[(size_t)n - 1].gfirst : 1;
    if (device_units) {
        auto span_of = [&](int64_t e) { return std::max<int64_t>(0, (int64_t)reads[(size_t)e].glast - reads[(size_t)e].gfirst + 1); };
        s.units_on_device = true;
        s.h_roff.resize((size_t)ne + 1);
        int64_t tot = 0;
        for (int64_t e = 0; e < ne; e++) {
            s.h_roff[(size_t)e] = tot;
            if (e < n) tot += span_of(e);
        }
        s.h_roff[(size_t)ne] = tot;
        s.n_rbytes = tot;
        if (!arena.ensure_units(tot / 8 + 2, exact)) return -2;
        s.h_units = arena.units;
        s.units_pinned = arena.units_pinned;
        uint8_t* dst = reinterpret_cast<uint8_t*>(arena.units);
        parallel_for(ne, 4096, [&](int64_t lo, int64_t hi) {
            for (int64_t e = lo; e < hi; e++) {
                if (e >= n) {                              // padding entry: empty
                    s.h_rh[(size_t)(2 * e)] = last_first;
                    s.h_rh[(size_t)(2 * e + 1)] = last_first - 1;
                    continue;
                }
                const SRead& rd = reads[(size_t)e];
                const int64_t span = span_of(e);
                s.h_rh[(size_t)(2 * e)] = rd.gfirst;
                s.h_rh[(size_t)(2 * e + 1)] = (int32_t)((uint32_t)(span > 0 ? rd.glast : rd.gfirst - 1) | (rd.neg ? 0x80000000u : 0u));
            }
            const int64_t top = std::min(hi, n);
            for (int64_t e = lo; e < top;) {
                const uint8_t* p = reads[(size_t)e].bytes;
                int64_t len = span_of(e), f = e + 1;
                while (f < top && (span_of(f) == 0 || reads[(size_t)f].bytes == p + len)) len += span_of(f++);
                if (len) std::memcpy(dst + s.h_roff[(size_t)e], p, (size_t)len);
                e = f;
            }
        });
        if (consumed) consumed(n);
    } else {
    if (!arena.ensure_units(base + 8, exact)) return -2;       // + 8: slack past the last unit
    s.h_units = arena.units;
    s.units_pinned = arena.units_pinned;
    uint64_t* units = s.h_units;
    const int64_t slice = consumed ? (int64_t)1 << 15 : std::max<int64_t>(ng, 1);   // groups filled between two releases
    for (int64_t sa = 0; sa < ng; sa += slice) {
    const int64_t sb = std::min(ng, sa + slice);
    parallel_for(sb - sa, 64, [&](int64_t q0, int64_t q1) {
        const int64_t g0 = sa + q0, g1 = sa + q1;
        const uint8_t* src[64];
        const uint8_t* rfs[64];
        int64_t spans[64];
        for (int64_t g = g0; g < g1; g++) {
            const RGroup G = s.h_grp[(size_t)g];
            for (int l = 0; l < 64; l++) {
                const int64_t e = g * 64 + l;
                src[l] = rfs[l] = nullptr;
                spans[l] = 0;
                if (e >= n) {                          // padding entry: empty
                    s.h_rh[(size_t)(2 * e)] = last_first;
                    s.h_rh[(size_t)(2 * e + 1)] = last_first - 1;
                    continue;
                }
                const SRead& rd = reads[(size_t)e];
                const int64_t span = std::max<int64_t>(0, (int64_t)rd.glast - rd.gfirst + 1);
                s.h_rh[(size_t)(2 * e)] = rd.gfirst;
                s.h_rh[(size_t)(2 * e + 1)] = (int32_t)((uint32_t)(span > 0 ? rd.glast : rd.gfirst - 1) | (rd.neg ? 0x80000000u : 0u));
                // reference-relative bytes: code ^ the position's reference code (0: a valid reference call of
                // quality 0 -- what the padding past the read's end holds, never an exception in KL)
                src[l] = rd.bytes;
                rfs[l] = s.h_ref.data() + rd.gfirst;
                spans[l] = span;
            }
            fill_group_units(units + G.base, G.K, src, rfs, spans);
        }
        _mm_sfence();
    });
    if (consumed) consumed(std::min(n, sb * 64));
    }
    }
    // block tables over the global coordinate (reads are sorted by gfirst).  blkA[b]: the first entry whose glast
    // reaches block b (every earlier entry ends before it), capped by blkB[b] -- the first entry with a prefix maximum of
    // glast at or past the block's start, so one long (or spliced) alignment widens only the blocks it spans, not every
    // block by the run's longest span
    const int64_t nb = (s.g_len >> kRgBlockShift) + 2;
    s.h_blkA.resize((size_t)nb);
    s.h_blkB.resize((size_t)nb);
    std::vector<int32_t> pmax((size_t)n);
    prefix_max_glast(n, [&](int64_t e) { return reads[(size_t)e].glast; }, pmax.data());
    parallel_for(nb, 1 << 14, [&](int64_t b0, int64_t b1) {
        auto first_at = [&](int64_t v) {          // first read with gfirst >= v
            return (int32_t)(std::lower_bound(reads.begin(), reads.end(), v, [](const SRead& r, int64_t x) { return (int64_t)r.gfirst < x; }) - reads.begin());
        };
        int64_t ia = std::lower_bound(pmax.begin(), pmax.end(), (int32_t)(b0 << kRgBlockShift)) - pmax.begin();
        int64_t ib = first_at(b0 << kRgBlockShift);
        for (int64_t b = b0; b < b1; b++) {
            const int64_t vb = b << kRgBlockShift;
            while (ia < n && (int64_t)pmax[(size_t)ia] < vb) ia++;
            while (ib < n && (int64_t)reads[(size_t)ib].gfirst < vb) ib++;
            s.h_blkA[(size_t)b] = (int32_t)std::min(ia, ib);
            s.h_blkB[(size_t)b] = (int32_t)ib;
        }
    });
    if (host_timing)
        std::fprintf(stderr, "[ngsep host]   read-group layout %.1f ms (%lld reads, %lld units)\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), (long long)n, (long long)base);
    return 0;
}

bool LayoutArena::ensure_units(int64_t n_units, bool exact) {
    if (units && n_units <= units_cap) return true;
    if (units_pinned) pinned_free(units);
    else std::free(units);
    units = nullptr;
    units_cap = 0;
    int64_t want = exact ? n_units : n_units + n_units / 4;
    want = std::max<int64_t>(want, 4096);
    // a whole-run layout beyond 4 GB (a staged multi-contig device run) stays pageable: the upload goes through the
    // runtime's staging buffers instead of pinning tens of GB at once (pinned_free releases either kind)
    const size_t bytes = (size_t)want * sizeof(uint64_t);
    units_pinned = bytes <= ((size_t)4 << 30);
    units = static_cast<uint64_t*>(units_pinned ? pinned_alloc(bytes) : huge_alloc(bytes));
    if (!units) return false;
    units_cap = want;
    return true;
}

bool LayoutArena::ensure(int64_t pile_bytes, bool exact) {
    if (cpile && pile_bytes <= cap) return true;
    release();
    int64_t want = exact ? pile_bytes : pile_bytes + pile_bytes / 4;
    want = (std::max<int64_t>(want, 1 << 16) + 4095) / 4096 * 4096;
    cpile = static_cast<uint8_t*>(pinned_alloc((size_t)want));
    planes = static_cast<uint32_t*>(pinned_alloc((size_t)want / 8));
    cneg = static_cast<uint32_t*>(pinned_alloc((size_t)want / 8));
    if (!cpile || !planes || !cneg) { release(); return false; }
    cap = want;
    return true;
}
void LayoutArena::release() {
    pinned_free(cpile);
    pinned_free(planes);
    pinned_free(cneg);
    if (units_pinned) pinned_free(units);
    else std::free(units);
    cpile = nullptr;
    planes = nullptr;
    cneg = nullptr;
    units = nullptr;
    cap = units_cap = 0;
}

// Population read-group layout.  MultisampleVariantsDetector genotypes every sample from its own
// read groups (PileupRecord.getAlleleCalls(span, readGroups), :104-111), so the admitted reads are split into one
// stream per (sample, read-group rank) -- the reads of no sample, which only enter the pooled counts, one stream last
// -- each in pending-list order and laid out as build_rg_layout lays out a single-sample run: 64-entry groups,
// reference-relative 8-byte units, entry headers, block tables (per stream).  The host only copies the projected
// bytes into place; KLM scans a sample's streams tile by tile on the device and KPM gathers a queued position's
// columns from them in getAlleleCalls order (rank, then pending order).
static int build_pop_rg_layout(Staged& s, LayoutArena& arena) {
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    auto t_last = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!host_timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngsep host]   population layout: %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    const int64_t n = s.n_reads;
    const int S = s.n_samples;
    const int32_t* R = s.h_reads.data();
    const int64_t* rptr = s.h_rdev.data();            // each read's projected bytes: their offset in the uploaded chunks
    const uint8_t* ref = s.h_ref.data();
    // stream keys: sample * 128 + read-group rank; the reads of no sample: S * 128
    const int64_t nkeys = (int64_t)(S + 1) * 128;
    RawVec<uint16_t> key((size_t)n);
    parallel_for(n, 1 << 16, [&](int64_t a, int64_t b) {
        for (int64_t r = a; r < b; r++) {
            const int sm = (R[r * 4 + 3] >> 8) - 1;
            key[(size_t)r] = sm < 0 || sm >= S ? (uint16_t)(S * 128) : (uint16_t)(sm * 128 + ((R[r * 4 + 3] >> 1) & 127));
        }
    });
    // a stable counting sort by key: per-chunk histograms, (key, chunk) offsets, scatter
    const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(64, n / 65536 + 1)), chl = (n + nch - 1) / nch;
    std::vector<int64_t> hist((size_t)(nch * nkeys), 0);
    parallel_for(nch, 1, [&](int64_t a, int64_t b) {
        for (int64_t c = a; c < b; c++) {
            int64_t* h = &hist[(size_t)(c * nkeys)];
            for (int64_t r = c * chl; r < std::min(n, (c + 1) * chl); r++) h[key[(size_t)r]]++;
        }
    });
    std::vector<int64_t> kcount((size_t)nkeys, 0);
    {
        int64_t run = 0;
        for (int64_t k = 0; k < nkeys; k++)
            for (int64_t c = 0; c < nch; c++) {
                int64_t& h = hist[(size_t)(c * nkeys + k)];
                const int64_t v = h;
                h = run;
                run += v;
                kcount[(size_t)k] += v;
            }
    }
    RawVec<int32_t> ord((size_t)n);
    parallel_for(nch, 1, [&](int64_t a, int64_t b) {
        for (int64_t c = a; c < b; c++) {
            int64_t* h = &hist[(size_t)(c * nkeys)];
            for (int64_t r = c * chl; r < std::min(n, (c + 1) * chl); r++) ord[(size_t)h[key[(size_t)r]]++] = (int32_t)r;
        }
    });
    decltype(key)().swap(key);
    std::vector<int64_t>().swap(hist);
    // streams (non-empty keys in key order), their entries padded to whole groups
    std::vector<int64_t> st_r0, st_n, st_e0;          // first read (in ord), reads, first entry
    s.h_samp_st.assign((size_t)S + 2, 0);
    int64_t r0 = 0, e0 = 0;
    for (int64_t k = 0; k < nkeys; k++) {
        const int sm = (int)(k / 128);
        if (k % 128 == 0) s.h_samp_st[(size_t)sm] = (int32_t)st_n.size();
        if (!kcount[(size_t)k]) continue;
        st_r0.push_back(r0);
        st_n.push_back(kcount[(size_t)k]);
        st_e0.push_back(e0);
        r0 += kcount[(size_t)k];
        e0 += (kcount[(size_t)k] + 63) / 64 * 64;
    }
    const int64_t nst = (int64_t)st_n.size();
    s.h_samp_st[(size_t)S + 1] = (int32_t)nst;
    s.n_streams = (int32_t)nst;
    const int64_t ne = e0, ng = ne / 64;
    s.n_entries = ne;
    s.n_groups = ng;
    s.h_st_end.resize((size_t)nst);
    for (int64_t st = 0; st < nst; st++) s.h_st_end[(size_t)st] = st_e0[(size_t)st] + (st_n[(size_t)st] + 63) / 64 * 64;
    // entry -> read (-1: padding) and the entry headers
    RawVec<int32_t> ent((size_t)ne);                    // (every entry written below: -1 for padding)
    s.h_rh.resize((size_t)ne * 2);
    parallel_for(nst, 1, [&](int64_t a, int64_t b) {
        for (int64_t st = a; st < b; st++) {
            const int64_t m = st_n[(size_t)st], eb = st_e0[(size_t)st];
            const int32_t last_first = R[(int64_t)ord[(size_t)(st_r0[(size_t)st] + m - 1)] * 4];
            for (int64_t i = 0; i < (m + 63) / 64 * 64; i++) {
                const int64_t e = eb + i;
                if (i >= m) {
                    ent[(size_t)e] = -1;
                    s.h_rh[(size_t)(2 * e)] = last_first;
                    s.h_rh[(size_t)(2 * e + 1)] = last_first - 1;
                    continue;
                }
                const int64_t r = ord[(size_t)(st_r0[(size_t)st] + i)];
                ent[(size_t)e] = (int32_t)r;
                const int32_t gf = R[r * 4], gl = R[r * 4 + 1];
                const bool empty = gl < gf;
                s.h_rh[(size_t)(2 * e)] = gf;
                s.h_rh[(size_t)(2 * e + 1)] = (int32_t)((uint32_t)(empty ? gf - 1 : gl) | ((R[r * 4 + 3] & 1) ? 0x80000000u : 0u));
            }
        }
    });
    lap("streams");
    // groups: units per read (on all threads: the entries' reads are scattered over R), then the unit offsets
    s.h_grp.resize((size_t)ng);
    parallel_for(ng, 1 << 12, [&](int64_t g0, int64_t g1) {
        for (int64_t g = g0; g < g1; g++) {
            int32_t K = 0;
            for (int64_t e = g * 64; e < g * 64 + 64; e++) {
                const int32_t r = ent[(size_t)e];
                if (r < 0) continue;
                const int64_t span = (int64_t)R[(int64_t)r * 4 + 1] - R[(int64_t)r * 4] + 1;
                if (span > 0) K = std::max<int32_t>(K, (int32_t)((span + 7) / 8));
            }
            s.h_grp[(size_t)g] = RGroup{0, K, 0};
        }
    });
    int64_t base = 0;
    for (int64_t g = 0; g < ng; g++) {
        s.h_grp[(size_t)g].base = base;
        base += (int64_t)s.h_grp[(size_t)g].K * 64;
    }
    s.n_units = base;
    // the units are built on the device (kernels.hip k_build_units) from the projection chunks themselves, uploaded as
    // they are (s.h_chunks, one after the other in d_rbytes): every entry gets its read's offset there (h_rdev) -- no
    // host copy (round 4's host transposition of the same bytes: 0.7-0.95 s of the chrIV 200-sample end-to-end run)
    {
        int64_t tot = 0;
        for (const auto& ch : s.h_chunks) tot += ch.second;
        s.units_on_device = true;
        s.n_rbytes = tot;
        s.h_units = nullptr;
        s.h_roff.resize((size_t)ne + 1);
        parallel_for(ne, 1 << 16, [&](int64_t a, int64_t b) {
            for (int64_t e = a; e < b; e++) {
                const int32_t r = ent[(size_t)e];
                s.h_roff[(size_t)e] = r < 0 ? 0 : s.h_rdev[(size_t)r];
            }
        });
        s.h_roff[(size_t)ne] = 0;
        (void)ref;
        (void)arena;
        (void)rptr;
    }
    lap("read bytes");
    // block tables per stream, blocks of 2^pblk_shift positions (coarser when the tables would outgrow a quarter of
    // the units; at most a KLM tile)
    int32_t shift = 6;                                 // (KPM's gather walks ~ (64 + max span) x depth / span entries)
    while (shift < 11 && ((s.g_len >> shift) + 2) * nst * 8 > std::max<int64_t>((int64_t)64 << 20, s.n_units * 2)) shift++;
    s.pblk_shift = shift;
    const int64_t nb = (s.g_len >> shift) + 2;
    s.pnblk = nb;
    s.h_blkA.resize((size_t)(nb * nst));               // (every entry written below)
    s.h_blkB.resize((size_t)(nb * nst));
    // blkA: the stream's first entry whose glast reaches the block (a running maximum of glast, as the single-sample
    // tables: one long alignment widens only the blocks it spans), capped by blkB
    parallel_for(nst, 1, [&](int64_t a, int64_t b) {
        for (int64_t st = a; st < b; st++) {
            const int64_t m = st_n[(size_t)st], eb = st_e0[(size_t)st];
            const int32_t* o = &ord[(size_t)st_r0[(size_t)st]];
            int64_t ia = 0, ib = 0;
            int64_t pm = INT64_MIN;                            // max glast of the stream's entries [0, ia)
            for (int64_t k = 0; k < nb; k++) {
                const int64_t vb = k << shift;
                while (ia < m && std::max<int64_t>(pm, (int64_t)R[(int64_t)o[ia] * 4 + 1]) < vb) {
                    pm = std::max<int64_t>(pm, (int64_t)R[(int64_t)o[ia] * 4 + 1]);
                    ia++;
                }
                while (ib < m && (int64_t)R[(int64_t)o[ib] * 4] < vb) ib++;
                s.h_blkA[(size_t)(st * nb + k)] = (int32_t)(eb + std::min(ia, ib));
                s.h_blkB[(size_t)(st * nb + k)] = (int32_t)(eb + ib);
            }
        }
    });
    // the most reads of one sample covering one position (KPM gathers each sample's column into a slot of this many
    // codes): a sweep over the sample's read starts and ends, all its streams together (a bound from the longest span
    // in the run would let one long alignment inflate every sample's slot)
    // A sample deeper than kKlmCountMaxCov somewhere also lists the KLM tiles where it is (the maximum over a tile is the
    // coverage at its first position or at one of the starts inside it): those tiles take KLM's exact-bound scan
    std::vector<int32_t> sbound((size_t)S + 1, 0);
    std::vector<std::vector<int32_t>> sdeep((size_t)S);
    parallel_for(S + 1, 1, [&](int64_t a, int64_t b) {
        std::vector<int32_t> starts, ends;
        for (int64_t sm = a; sm < b; sm++) {
            starts.clear();
            ends.clear();
            for (int32_t st = s.h_samp_st[(size_t)sm]; st < s.h_samp_st[(size_t)sm + 1]; st++) {
                const int32_t* o = &ord[(size_t)st_r0[(size_t)st]];
                for (int64_t i = 0; i < st_n[(size_t)st]; i++) {
                    starts.push_back(R[(int64_t)o[i] * 4]);
                    ends.push_back(R[(int64_t)o[i] * 4 + 1]);
                }
            }
            std::sort(starts.begin(), starts.end());
            std::sort(ends.begin(), ends.end());
            int32_t mc = 0;
            size_t j = 0;
            for (size_t i = 0; i < starts.size(); i++) {       // covering reads at starts[i]: started, not yet ended
                while (j < ends.size() && ends[j] < starts[i]) j++;
                mc = std::max<int32_t>(mc, (int32_t)(i + 1 - j));
            }
            sbound[(size_t)sm] = mc;
            if (mc <= kKlmCountMaxCov || sm == S) continue;       // (the reads of no sample are not scanned by KLM)
            const size_t n = starts.size();
            size_t ia = 0, ja = 0, ib = 0, jb = 0;
            for (int64_t t = starts[0] / kKlmTile, t1 = ends[n - 1] / kKlmTile; t <= t1; t++) {
                const int64_t T = t * kKlmTile, Tn = T + kKlmTile;
                while (ia < n && starts[ia] <= T) ia++;
                while (ja < n && ends[ja] < T) ja++;
                int64_t m = (int64_t)ia - (int64_t)ja;                 // coverage at the tile's first position
                for (; ib < n && starts[ib] < Tn; ib++) {
                    if (starts[ib] < T) continue;
                    while (jb < n && ends[jb] < starts[ib]) jb++;
                    m = std::max<int64_t>(m, (int64_t)(ib + 1) - (int64_t)jb);
                }
                if (m > kKlmCountMaxCov) sdeep[(size_t)sm].push_back((int32_t)t);
            }
        }
    });
    int32_t stride = 0;
    for (int sm = 0; sm <= S; sm++) stride = std::max(stride, sbound[(size_t)sm]);
    s.max_cov = (stride + 3) / 4 * 4;
    s.h_deep_tiles.clear();
    for (const auto& v : sdeep) s.h_deep_tiles.insert(s.h_deep_tiles.end(), v.begin(), v.end());
    std::sort(s.h_deep_tiles.begin(), s.h_deep_tiles.end());
    s.h_deep_tiles.erase(std::unique(s.h_deep_tiles.begin(), s.h_deep_tiles.end()), s.h_deep_tiles.end());
    s.prg = true;
    s.tile = kKlmTile;
    s.n_tiles = s.g_len / kKlmTile;
    s.pile_bytes = s.n_units * 8;
    lap("block tables");
    return 0;
}

int build_and_upload(ngsep_ctx* c, std::vector<ContigReads>& contigs, bool release_chunks) {
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto h0 = std::chrono::steady_clock::now();
    Staged& s = c->staged;
    s = Staged();
    int32_t max_span = 1;
    for (const ContigReads& cr : contigs) max_span = std::max(max_span, cr.max_span);
    const int32_t pad = ((max_span + 63) / 64) * 64;
    s.max_span = max_span;
    // windows: the covered span of every sequence (and the query range), cut at window_positions, laid out
    // in one global coordinate with a halo of pad >= max read span positions between windows
    int64_t g = 0;
    const int64_t W = c->params.window_positions > 0 ? c->params.window_positions : (int64_t)1 << 40;
    struct WR { size_t contig; int64_t lo, hi; };
    std::vector<WR> wr;
    for (size_t ci = 0; ci < contigs.size(); ci++) {
        const ContigReads& cr = contigs[ci];
        if (cr.first.empty()) continue;
        int64_t len = (int64_t)c->seq_bases[cr.seq_id].size();
        int64_t lo = 1, hi = len;
        if (c->params.query_seq[0]) { lo = std::max<int64_t>(lo, c->params.query_first); hi = std::min<int64_t>(hi, c->params.query_last); }
        lo = std::max<int64_t>(lo, cr.first.front());
        int64_t maxlast = 0;
        for (int32_t l : cr.last) maxlast = std::max<int64_t>(maxlast, l);
        hi = std::min<int64_t>(hi, maxlast);
        for (int64_t w0 = lo; w0 <= hi; w0 += W) {
            int64_t w1 = std::min(hi, w0 + W - 1);
            Window w;
            w.seq_id = cr.seq_id; w.w0 = (int32_t)w0; w.wlen = (int32_t)(w1 - w0 + 1);
            w.gbase = g; w.pad = pad;
            g += (int64_t)w.wlen + 2 * pad;
            s.windows.push_back(w);
            wr.push_back({ci, w0, w1});
        }
    }
    s.g_len = ((g + 64 + kRunAlign - 1) / kRunAlign) * kRunAlign;   // whole tiles, halo for 16-B reads
    if (s.g_len >= ((int64_t)1 << 31))
        return set_error(c, NGSEP_E_UNSUPPORTED, "staged genome exceeds 2^31 positions per device run; use window batching");
    // reads of every window: those starting in [w0 - max_span + 1, w1]
    std::vector<std::pair<int64_t, int64_t>> ranges(s.windows.size());
    int64_t nreads = 0, nbases = 0;
    for (size_t wi = 0; wi < s.windows.size(); wi++) {
        const ContigReads& cr = contigs[wr[wi].contig];
        const int64_t w0 = wr[wi].lo, w1 = wr[wi].hi;
        auto lo_it = std::lower_bound(cr.first.begin(), cr.first.end(), (int32_t)std::max<int64_t>(INT32_MIN, w0 - max_span + 1));
        auto hi_it = std::upper_bound(cr.first.begin(), cr.first.end(), (int32_t)w1);
        ranges[wi] = {lo_it - cr.first.begin(), hi_it - cr.first.begin()};
        nreads += ranges[wi].second - ranges[wi].first;
    }
    for (const ContigReads& cr : contigs) s.covered += cr.covered;
    // reference codes in global coordinates; carved indel regions get no code (no call is made there)
    s.h_ref.assign((size_t)s.g_len, 0);
    for (size_t wi = 0; wi < s.windows.size(); wi++) {
        const auto& cv = contigs[wr[wi].contig].carved;
        fill_ref_codes(c, s, s.windows[wi], std::vector<std::pair<int64_t, int64_t>>(cv.begin(), cv.end()));
    }
    if (host_timing)
        std::fprintf(stderr, "[ngsep host]   layout windows + reference codes %.1f ms\n",
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h0).count());
    if (!c->params.multisample) {
        // single sample: the reads' projected bytes go straight into the tile layout
        s.single = true;
        RawVec<SRead> reads((size_t)nreads);
        int64_t ri = 0;
        for (size_t wi = 0; wi < s.windows.size(); wi++) {
            Window& w = s.windows[wi];
            const ContigReads& cr = contigs[wr[wi].contig];
            w.read_begin = ri;
            const int64_t goff = w.gbase + w.pad - w.w0;   // G = pos + goff
            for (int64_t i = ranges[wi].first; i < ranges[wi].second; i++) {
                reads[(size_t)ri++] = SRead{(int32_t)(cr.first[(size_t)i] + goff), (int32_t)(cr.last[(size_t)i] + goff),
                                            cr.bptr[(size_t)i], cr.neg[(size_t)i]};
                const int64_t span = (int64_t)cr.last[(size_t)i] - cr.first[(size_t)i] + 1;
                nbases += span > 0 ? span : 0;
            }
            w.read_end = ri;
        }
        s.n_reads = nreads;
        s.n_read_bases = nbases;
        // the variant caller reads the read-group layout (KL scans it on the device); the relative allele counts
        // listener the position-major pile
        // release_chunks (ngsep_stage_finish): a sequence's projected chunks go back once every read of its windows
        // is in the layout -- the staged genome's bytes are then held about once, not twice (round 4: 114 GiB peak RSS
        // staging configs[3] on one device)
        std::vector<int64_t> contig_end(contigs.size(), 0);       // one past the sequence's last read in `reads`
        for (size_t wi = 0; wi < s.windows.size(); wi++)
            contig_end[wr[wi].contig] = std::max<int64_t>(contig_end[wr[wi].contig], s.windows[wi].read_end);
        size_t next_rel = 0;
        auto consumed = [&](int64_t done) {
            while (next_rel < contigs.size() && contig_end[next_rel] <= done) {
                std::vector<HostArray<uint8_t>>().swap(contigs[next_rel].chunks);
                next_rel++;
            }
        };
        const int lr = c->params.relative_allele_counts ? build_single_layout(s, reads, c->arena, true)
                                                        : build_rg_layout(s, reads, c->arena, true,
                                                                          release_chunks ? std::function<void(int64_t)>(consumed) : nullptr);
        if (lr == -2) return set_error(c, NGSEP_E_DEVICE, "pinned host memory for the layout could not be allocated");
        if (lr != 0) return set_error(c, NGSEP_E_INVALID, "internal error: pileup depth above the tile's row count");
        c->stats.slot_bytes = 0;
        c->stats.slot_size = 0;
    } else {
        // the reads in pending order with their projected bytes in place (no copy): the population layout reads
        // them through h_rdev, their offsets in the projection chunks as uploaded
        s.slot_size = 0;
        s.h_reads.resize((size_t)nreads * 4);
        s.h_rdev.resize((size_t)nreads);
        // the projection chunks the reads' bytes lie in, uploaded one after the other (kernels.hip device_upload): a
        // read's bytes are at h_rdev = its chunk's offset there + its offset in the chunk (ContigReads::chunk_end)
        s.h_chunks.clear();
        std::vector<std::vector<int64_t>> cdev(contigs.size());
        {
            int64_t at = 0;
            for (size_t ci = 0; ci < contigs.size(); ci++)
                for (size_t k = 0; k < contigs[ci].chunks.size(); k++) {
                    // only the bytes the chunk holds (a pooled chunk can be much larger than its batch)
                    const HostArray<uint8_t>& ch = contigs[ci].chunks[k];
                    const int64_t used = k < contigs[ci].chunk_used.size() ? contigs[ci].chunk_used[k] : (int64_t)ch.n;
                    cdev[ci].push_back(at);
                    s.h_chunks.push_back({ch.p, used});
                    at += used;
                }
        }
        std::vector<int64_t> wbase(s.windows.size() + 1, 0);
        for (size_t wi = 0; wi < s.windows.size(); wi++) wbase[wi + 1] = wbase[wi] + (ranges[wi].second - ranges[wi].first);
        for (size_t wi = 0; wi < s.windows.size(); wi++) {
            Window& w = s.windows[wi];
            const ContigReads& cr = contigs[wr[wi].contig];
            w.read_begin = wbase[wi];
            w.read_end = wbase[wi + 1];
            const int64_t goff = w.gbase + w.pad - w.w0;   // G = pos + goff
            const int64_t i0 = ranges[wi].first;
            std::atomic<int64_t> nb{0};
            const std::vector<int64_t>& cd = cdev[wr[wi].contig];
            parallel_for(ranges[wi].second - i0, 1 << 14, [&](int64_t lo, int64_t hi) {
                int64_t local = 0;
                size_t ck = (size_t)(std::upper_bound(cr.chunk_end.begin(), cr.chunk_end.end(), (size_t)(i0 + lo)) - cr.chunk_end.begin());
                for (int64_t k = lo; k < hi; k++) {
                    const int64_t i = i0 + k, ri = wbase[wi] + k;
                    while (ck < cr.chunk_end.size() && cr.chunk_end[ck] <= (size_t)i) ck++;
                    const int64_t span = (int64_t)cr.last[i] - cr.first[i] + 1;
                    s.h_reads[ri * 4 + 0] = (int32_t)(cr.first[i] + goff);
                    s.h_reads[ri * 4 + 1] = (int32_t)(cr.last[i] + goff);
                    s.h_reads[ri * 4 + 2] = 0;
                    int32_t fl = cr.neg[i];
                    if (!cr.sample.empty()) fl |= ((int32_t)cr.rank[i] << 1) | (((int32_t)cr.sample[i] + 1) << 8);
                    s.h_reads[ri * 4 + 3] = fl;
                    s.h_rdev[(size_t)ri] = ck < cd.size() && span > 0 ? cd[ck] + (cr.bptr[i] - cr.chunks[ck].p) : 0;
                    local += span > 0 ? span : 0;
                }
                nb += local;
            });
            nbases += nb.load();
        }
        s.n_reads = nreads;
        s.n_slots = 0;
        s.n_read_bases = nbases;
        s.n_samples = (int32_t)c->sample_ids.size();
        if (!c->known.empty()) {
            // -knownVariants (MultisampleVariantsDetector.onPileup :539-551): the input variants at positions with
            // a pileup (a read with first <= p <= last), in input order; queue code 0x80 | ref << 5 | alt << 8 | 0x400
            for (size_t wi = 0; wi < s.windows.size(); wi++) {
                const Window& w = s.windows[wi];
                const ContigReads& cr = contigs[wr[wi].contig];
                const int64_t goff = w.gbase + w.pad - w.w0;
                const int64_t w1 = (int64_t)w.w0 + w.wlen - 1;
                const int64_t kb = c->known_seq_begin[(size_t)cr.seq_id], ke = c->known_seq_begin[(size_t)cr.seq_id + 1];
                auto it = std::lower_bound(c->known.begin() + kb, c->known.begin() + ke, (int64_t)w.w0,
                                           [](const ngsep_ctx::KnownVar& v, int64_t p) { return v.pos < p; });
                // reads that start before the window's range end before w0, so they cannot cover an input variant
                size_t r = (size_t)ranges[wi].first, ci = 0;
                int64_t maxlast = INT64_MIN;
                const auto& cv = cr.carved;
                for (; it != c->known.begin() + ke && it->pos <= w1; ++it) {
                    const int64_t p = it->pos;
                    if (it->alt < 0) continue;                            // not an SNV: genotyped in its region
                    while (r < cr.first.size() && cr.first[r] <= p) { maxlast = std::max<int64_t>(maxlast, cr.last[r]); r++; }
                    if (maxlast < p) continue;                                    // no pileup here
                    while (ci < cv.size() && cv[ci].second < p) ci++;
                    if (ci < cv.size() && cv[ci].first <= p) continue;            // carved: the caller's own indel path
                    s.h_forced.push_back((int32_t)(p + goff));
                    s.h_forced.push_back(0x80 | (it->ref << 5) | (it->alt << 8) | 0x400);
                }
            }
            s.known = true;
        }
        const int lr = build_pop_rg_layout(s, c->arena);
        if (lr == -2) return set_error(c, NGSEP_E_DEVICE, "host memory for the population layout could not be allocated");
        if (lr != 0) return set_error(c, NGSEP_E_INVALID, "internal error: population layout");
        c->stats.slot_bytes = 0;
        c->stats.slot_size = 0;                  // (no fixed-size slots: the site-major pile is sized per tile)
    }
    c->stats.read_bases = nbases;
    c->stats.pile_bytes = s.rg || s.prg ? s.n_units * 8 : s.pile_bytes;
    c->stats.tile_positions = s.tile;
    c->stats.tile_rows_max = s.tile_rows_max;
    const auto h1 = std::chrono::steady_clock::now();
    if (!c->dev) {
        std::string err;
        if (!ensure_device(c, err)) return set_error(c, NGSEP_E_DEVICE, err);
    }
    std::string err;
    if (device_upload(c->dev, s, err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
    c->stats.global_positions = s.g_len;
    c->stats.n_tiles = s.n_tiles;
    c->stats.other_allele_calls = s.h_loff.empty() ? 0 : s.h_loff.back();
    c->stats.layout_ms = std::chrono::duration<double, std::milli>(h1 - h0).count();
    c->stats.upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h1).count();
    if (host_timing)
        std::fprintf(stderr, "[ngsep host] layout %.1f ms, device upload %.1f ms (%lld reads, %lld tiles)\n",
                     std::chrono::duration<double, std::milli>(h1 - h0).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h1).count(),
                     (long long)nreads, (long long)s.n_tiles);
    // host mirrors are not needed any more
    decltype(s.h_rdev)().swap(s.h_rdev);
    decltype(s.h_reads)().swap(s.h_reads);
    std::vector<uint8_t>().swap(s.h_ref);
    std::vector<uint8_t>().swap(s.h_pile);
    std::vector<TileInfo>().swap(s.h_tinfo);
    std::vector<uint16_t>().swap(s.h_olist);
    std::vector<int32_t>().swap(s.h_loff);
    decltype(s.h_rh)().swap(s.h_rh);
    std::vector<RGroup>().swap(s.h_grp);
    RawVec<int32_t>().swap(s.h_blkA);
    RawVec<int32_t>().swap(s.h_blkB);
    s.h_units = nullptr;
    std::vector<int32_t>().swap(s.h_samp_st);
    std::vector<int64_t>().swap(s.h_st_end);
    s.h_ppile.reset();
    std::vector<int32_t>().swap(s.h_prow);
    std::vector<int32_t>().swap(s.h_deep_tiles);
    std::vector<int64_t>().swap(s.h_pboff);
    // one-shot runs give the pinned layout buffers back (streamed windows keep theirs)
    s.h_planes = nullptr;
    s.h_cpile = nullptr;
    s.h_cneg = nullptr;
    c->arena.release();
    return NGSEP_OK;
}

// one streamed window (worker thread; the context's staged run, device and layout buffers are its own
// until stream_collect joins it): reference codes, layout, upload, kernels, records into j->sites
static int run_regions(ngsep_ctx* c, WindowJob* j, int64_t goff);

static void run_window_job(ngsep_ctx* c, WindowJob* j) {
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    if (j->rc != NGSEP_OK) { j->done = true; return; }   // (stream_launch found a fault)
    const auto h0 = std::chrono::steady_clock::now();
    Staged& s = c->staged;
    s = Staged();
    const int32_t pad = ((j->max_span + 63) / 64) * 64;
    Window w;
    w.seq_id = j->seq_id;
    w.w0 = (int32_t)j->w0;
    w.wlen = (int32_t)(j->w1 - j->w0 + 1);
    w.gbase = 0;
    w.pad = pad;
    w.read_begin = 0;
    w.read_end = (int64_t)j->reads.size();
    s.windows.push_back(w);
    s.max_span = j->max_span;
    s.g_len = (((int64_t)w.wlen + 2 * pad + 64 + kRunAlign - 1) / kRunAlign) * kRunAlign;
    s.covered = w.wlen;                 // (the dump mode's record capacity)
    if (c->params.relative_allele_counts) {
        s.h_ref.assign((size_t)s.g_len, 0);
        fill_ref_codes(c, s, w, j->carved);
    } else {
        // the reference codes are made on the device from the window's characters (kernels.hip k_ref_codes): the host
        // layout no longer reads them (its units are built there too)
        s.ref_on_device = true;
        s.h_refchars = c->seq_bases[(size_t)w.seq_id].data() + (w.w0 - 1);
        s.ref_lo = w.gbase + w.pad;
        s.ref_len = w.wlen;
        for (int ch = 0; ch < 256; ch++) s.ref_table[ch] = ref_code(c, (char)ch);
        s.h_zero.clear();
        for (const auto& cv : j->carved) {            // carved indel regions get no code (no call is made there)
            const int64_t a = std::max<int64_t>(cv.first, w.w0), b = std::min<int64_t>(cv.second, (int64_t)w.w0 + w.wlen - 1);
            if (a <= b) { s.h_zero.push_back(s.ref_lo + (a - w.w0)); s.h_zero.push_back(b - a + 1); }
        }
    }
    s.single = true;
    s.known = !c->known.empty();
    if (s.known) {
        s.h_forced.swap(j->forced);
        s.h_forced_ctr[2] = (unsigned long long)(s.h_forced.size() / 4);
    }
    s.n_reads = (int64_t)j->reads.size();
    int64_t nb = 0;
    for (const SRead& r : j->reads) nb += r.glast >= r.gfirst ? (int64_t)r.glast - r.gfirst + 1 : 0;
    s.n_read_bases = nb;
    const int lr = c->params.relative_allele_counts ? build_single_layout(s, j->reads, c->arena, false)
                                                    : build_rg_layout(s, j->reads, c->arena, false, nullptr, true);
    if (lr != 0) {
        j->rc = lr == -2 ? NGSEP_E_DEVICE : NGSEP_E_INVALID;
        j->err = lr == -2 ? "pinned host memory for the layout could not be allocated" : "internal error: pileup depth above the tile's row count";
        j->done = true;
        return;
    }
    const auto h1 = std::chrono::steady_clock::now();
    std::string err;
    if (!ensure_device(c, err) || device_upload(c->dev, s, err) != 0) {
        j->rc = NGSEP_E_DEVICE;
        j->err = err;
        j->done = true;
        return;
    }
    const auto h2 = std::chrono::steady_clock::now();
    c->stats.read_bases += nb;
    c->stats.pile_bytes += s.rg || s.prg ? s.n_units * 8 : s.pile_bytes;   // (summed over the streamed windows)
    c->stats.tile_positions = s.tile;
    c->stats.tile_rows_max = std::max(c->stats.tile_rows_max, s.tile_rows_max);
    c->stats.global_positions += s.g_len;
    c->stats.n_tiles += s.n_tiles;
    c->stats.other_allele_calls += s.h_loff.empty() ? 0 : s.h_loff.back();
    c->stats.layout_ms += std::chrono::duration<double, std::milli>(h1 - h0).count();
    c->stats.upload_ms += std::chrono::duration<double, std::milli>(h2 - h1).count();
    if (c->params.relative_allele_counts) {
        double ms = 0;
        std::string e2;
        if (device_run_rac(c->dev, s, w.gbase + w.pad, w.gbase + w.pad + w.wlen, c->params.rac_min_rd, c->params.rac_min_bq,
                           j->rac_hist, &j->rac_sum, &j->rac_sum_sq, &ms, e2) != 0) {
            j->rc = NGSEP_E_DEVICE;
            j->err = e2;
        } else {
            j->rc = NGSEP_OK;
            c->rac.kernel_ms += ms;
            c->stats.scan_ms = ms;
        }
    } else {
        j->rc = run_device_into(c, j->sites, nullptr);
        if (j->rc == NGSEP_OK && j->realign && !j->carved.empty()) j->rc = run_regions(c, j, (int64_t)pad - j->w0);
        if (j->rc != NGSEP_OK) j->err = c->err;
    }
    if (host_timing)
        std::fprintf(stderr, "[ngsep host] window %d:%lld-%lld: layout %.1f ms, upload %.1f ms, run %.1f ms (%lld reads)\n", j->seq_id,
                     (long long)j->w0, (long long)j->w1, std::chrono::duration<double, std::milli>(h1 - h0).count(),
                     std::chrono::duration<double, std::milli>(h2 - h1).count(),
                     std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h2).count(), (long long)s.n_reads);
    j->done = true;
}

// The window's realigner regions (realign.hpp): each replayed on a host thread (alignment edits, span-1 columns,
// the indel calls of longer spans); the columns genotyped on the device in one more run over the window's
// layout (KP, queue entries with their columns); the listener's span rules over both; the kept SNV and indel
// records merged into the window's, by position.  goff: window position p -> global p + goff.
static int run_regions(ngsep_ctx* c, WindowJob* j, int64_t goff) {
    using clk = std::chrono::steady_clock;
    auto ns = [](clk::time_point a, clk::time_point b) { return std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count(); };
    const std::string& seq = c->seq_bases[(size_t)j->seq_id];
    const size_t nr = j->carved.size();
    std::vector<RegionOut> outs(nr);
    RealignParams rp;
    rp.max_base_qs = c->params.max_base_qs;
    rp.min_quality = c->params.min_quality;
    rp.ploidy = c->params.ploidy;
    rp.het_rate = c->het_rate;
    rp.ignore_lowercase = c->params.ignore_lowercase_ref != 0;
    const bool known = !c->known.empty();
    rp.known = known;
    const auto t_rp = std::chrono::steady_clock::now();
    parallel_for((int64_t)nr, 1, [&](int64_t a, int64_t b) {
        for (int64_t k = a; k < b; k++)
            replay_region(seq, j->carved[(size_t)k].first, j->carved[(size_t)k].second, j->region_reads[(size_t)k], rp,
                          (size_t)j->seq_id < c->strs.size() ? &c->strs[(size_t)j->seq_id] : nullptr, &c->known_recs,
                          outs[(size_t)k]);
    });
    const auto t_q = clk::now();
    c->realign_ns += ns(t_rp, t_q);
    c->realign_regions += (int64_t)nr;
    // KP's queue: {global position, reference code, column offset / 4, entries} per callable position
    Staged& s = c->staged;
    s.known = true;
    s.h_forced.clear();
    s.h_cols.clear();
    const int64_t kb = known ? c->known_seq_begin[(size_t)j->seq_id] : 0, ke = known ? c->known_seq_begin[(size_t)j->seq_id + 1] : 0;
    // discovery: only the positions with a valid call of another allele than the reference are genotyped (DESIGN.md
    // section 5 -- any other column is hom-ref, which no listener writes), under the conditions the window's own run
    // prunes with; their columns alone are copied
    const bool prune = c->params.prune_candidates && !c->params.dump_all_positions && (c->het_rate <= 0.1 || c->params.ploidy >= 3);
    for (size_t k = 0; k < nr; k++) {
        const RegionOut& o = outs[k];
        if (!known) {
            for (const RegionPos& p : o.pos) {
                if (p.blocked || p.col_len == 0 || (prune && !p.nonref)) continue;
                const uint8_t rc = ref_code(c, seq[(size_t)p.pos - 1]);
                if (!(rc & kRefCallable)) continue;
                const size_t cb = s.h_cols.size();
                s.h_cols.insert(s.h_cols.end(), o.cols.begin() + p.col_off, o.cols.begin() + p.col_off + ((p.col_len + 3) & ~3));
                s.h_forced.push_back((int32_t)(p.pos + goff));
                s.h_forced.push_back((int32_t)rc);
                s.h_forced.push_back((int32_t)(cb / 4));
                s.h_forced.push_back(p.col_len);
            }
            continue;
        }
        const size_t cbase = s.h_cols.size();
        s.h_cols.insert(s.h_cols.end(), o.cols.begin(), o.cols.end());
        {
            // -knownVariants: the region's input SNVs at positions with a pileup, in input order, genotyped from the
            // replayed columns (queue code 0x80 | ref << 5 | alt << 8 | 0x400, as stream_launch's)
            auto it = std::lower_bound(c->known.begin() + kb, c->known.begin() + ke, o.first,
                                       [](const ngsep_ctx::KnownVar& v, int64_t p) { return v.pos < p; });
            size_t pi = 0;
            for (; it != c->known.begin() + ke && it->pos <= o.last; ++it) {
                if (it->alt < 0) continue;
                while (pi < o.pos.size() && o.pos[pi].pos < it->pos) pi++;
                if (pi == o.pos.size() || o.pos[pi].pos != it->pos) continue;       // no pileup here
                const RegionPos& p = o.pos[pi];
                s.h_forced.push_back((int32_t)(p.pos + goff));
                s.h_forced.push_back(0x80 | (it->ref << 5) | (it->alt << 8) | 0x400);
                s.h_forced.push_back((int32_t)((cbase + (size_t)p.col_off) / 4));
                s.h_forced.push_back(p.col_len);
            }
        }
    }
    std::memset(s.h_forced_ctr, 0, sizeof s.h_forced_ctr);
    s.h_forced_ctr[2] = (unsigned long long)(s.h_forced.size() / 4);
    s.h_forced_ctr[5] = (unsigned long long)(s.h_cols.size() / 4);
    SiteStore snv;
    const auto t_d = clk::now();
    c->region_setup_ns += ns(t_q, t_d);
    if (!s.h_forced.empty()) {
        const int rc = run_device_into(c, snv, nullptr);
        if (rc != NGSEP_OK) return rc;
    }
    const auto t_m = clk::now();
    c->region_device_ns += ns(t_d, t_m);
    // the listener's decisions, region by region (records and positions both ascending)
    SiteStore add;
    size_t ri = 0;
    int64_t kept = 0;
    std::vector<uint8_t> has;
    std::vector<size_t> rec_at;
    std::vector<RegionDecision> dec;
    for (size_t k = 0; k < nr && known; k++) {
        // -knownVariants: every input SNV record, and the non-SNV records genotyped by the replay (their order at a
        // shared position is the input's: stream_collect, by the known index kept in L[1])
        const RegionOut& o = outs[k];
        for (const KnownCall& kc : o.kcalls) {
            while (ri < snv.size() && snv.rec[ri].pos <= kc.pos) add.push_from(snv, ri++);
            SiteRec r;
            std::memset(&r, 0, sizeof r);
            r.seq_id = j->seq_id;
            r.pos = kc.pos;
            r.is_call = kRecCall | kRecIndel;
            add.text.push_back(kc.line);
            r.L[0] = __builtin_bit_cast(double, (int64_t)add.text.size() - 1);
            r.L[1] = __builtin_bit_cast(double, kc.known);
            add.rec.push_back(r);
            kept++;
        }
    }
    if (known) {
        while (ri < snv.size()) add.push_from(snv, ri++);
        kept += (int64_t)snv.size();
    }
    for (size_t k = 0; k < nr && !known; k++) {
        const RegionOut& o = outs[k];
        has.assign(o.pos.size(), 0);
        rec_at.assign(o.pos.size(), 0);
        for (size_t i = 0; i < o.pos.size(); i++) {
            while (ri < snv.size() && snv.rec[ri].pos < o.pos[i].pos) ri++;
            if (ri < snv.size() && snv.rec[ri].pos == o.pos[i].pos) { has[i] = 1; rec_at[i] = ri; }
        }
        resolve_region(o, has, c->params.call_embedded != 0, &j->last_indel_end, dec);
        size_t pi = 0;
        for (const RegionDecision& d : dec) {
            while (o.pos[pi].pos != d.pos) pi++;
            if (d.kind == 1) {
                add.push_from(snv, rec_at[pi], d.embedded ? kRecEmbedded : 0);
            } else {
                SiteRec r;
                std::memset(&r, 0, sizeof r);
                r.seq_id = j->seq_id;
                r.pos = d.pos;
                r.is_call = kRecCall | kRecIndel;
                add.text.push_back(o.indels[(size_t)d.idx].line);
                r.L[0] = __builtin_bit_cast(double, (int64_t)add.text.size() - 1);
                add.rec.push_back(r);
            }
            kept++;
        }
    }
    c->stats.sites_called += kept - (int64_t)snv.size();
    // merged with the window's records by position
    SiteStore merged;
    merged.rec.reserve(j->sites.size() + add.size());
    size_t a = 0, b = 0;
    while (a < j->sites.size() || b < add.size()) {
        if (b >= add.size() || (a < j->sites.size() && j->sites.rec[a].pos <= add.rec[b].pos)) merged.push_from(j->sites, a++);
        else merged.push_from(add, b++);
    }
    j->sites.swap(merged);
    s.known = false;
    s.h_forced.clear();
    s.h_cols.clear();
    c->region_merge_ns += ns(t_m, clk::now());
    return NGSEP_OK;
}

// MultisampleVariantsDetector with the indel realigner (MultisampleVariantsDetector.java:449-450): the sequence's
// realigner regions (carve_indel_regions' geometry; kept out of the sequence's run, which has just appended its records
// to pop_sites from index `from`) are replayed on the host threads (realign.cpp, population mode: alignment edits, every
// sample's span-1 columns, the span's population indel variant); the regions' positions are then genotyped by KPM from
// those columns (a queue of every replayed position in a layout of its own), onPileup's span rules resolve each region
// (resolve_population_region), and the region records join the sequence's records in position order.
static int run_population_regions(ngsep_ctx* c, const ContigReads& cr, size_t from) {
    const std::string& seq = c->seq_bases[(size_t)cr.seq_id];
    const int S = (int)c->sample_ids.size(), S1 = S + 1;
    auto& st = c->stream;
    const size_t nr = cr.carved.size();
    // every region's alignments, in admission (pending-list) order: the kept ones that overlap it, all of them
    std::vector<std::vector<RawRead>> reads(nr);
    {
        std::vector<const std::remove_reference_t<decltype(st.kept)>::value_type*> live;
        for (const auto& e : st.kept) if (!e.dead) live.push_back(&e);
        size_t lo = 0;
        for (size_t k = 0; k < nr; k++) {
            const int64_t a = cr.carved[k].first, b = cr.carved[k].second;
            while (lo < live.size() && (int64_t)live[lo]->first + cr.max_span < a) lo++;
            for (size_t i = lo; i < live.size() && live[i]->first <= b; i++)
                if (live[i]->last >= a) reads[k].push_back(live[i]->r);
            const int64_t r0 = std::lower_bound(cr.first.begin(), cr.first.end(), (int32_t)std::max<int64_t>(INT32_MIN, a - cr.max_span)) - cr.first.begin();
            size_t want = 0;
            for (int64_t i = r0; i < (int64_t)cr.first.size() && cr.first[(size_t)i] <= b; i++) want += cr.last[(size_t)i] >= a ? 1 : 0;
            if (want != reads[k].size())
                return set_error(c, NGSEP_E_INVALID, "internal error: indel realigner region " + std::to_string(a) + "-" + std::to_string(b) +
                                                     " lacks " + std::to_string((int64_t)want - (int64_t)reads[k].size()) + " alignments");
        }
    }
    std::vector<RegionOut> outs(nr);
    RealignParams rp;
    rp.max_base_qs = c->params.max_base_qs;
    rp.min_quality = c->params.min_quality;
    rp.ploidy = c->params.ploidy;
    rp.het_rate = c->het_rate;
    rp.ignore_lowercase = c->params.ignore_lowercase_ref != 0;
    rp.n_samples = S;
    const bool known = !c->known.empty();
    rp.known = known;
    const auto t_rp = std::chrono::steady_clock::now();
    parallel_for((int64_t)nr, 1, [&](int64_t a, int64_t b) {
        for (int64_t k = a; k < b; k++)
            replay_region(seq, cr.carved[(size_t)k].first, cr.carved[(size_t)k].second, reads[(size_t)k], rp,
                          (size_t)cr.seq_id < c->strs.size() ? &c->strs[(size_t)cr.seq_id] : nullptr, &c->known_recs,
                          outs[(size_t)k]);
    });
    c->realign_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_rp).count();
    c->realign_regions += (int64_t)nr;
    // KPM over the regions' positions: position v of the queue is virtual position v of a layout of its own (tiles of
    // kPopTile positions, site-major columns as build_multi_layout lays them out), discovery mode (no input alleles);
    // with -knownVariants one virtual position per input SNV at a region position with a pileup (its alleles given)
    std::vector<std::pair<uint32_t, uint32_t>> vpos;          // (region, index in its pos list) of virtual position v
    std::vector<int64_t> vknown;                              // -knownVariants: the input variant of virtual position v
    if (known) {
        const int64_t kb = c->known_seq_begin[(size_t)cr.seq_id], ke = c->known_seq_begin[(size_t)cr.seq_id + 1];
        for (size_t k = 0; k < nr; k++) {
            const RegionOut& o = outs[k];
            auto it = std::lower_bound(c->known.begin() + kb, c->known.begin() + ke, o.first,
                                       [](const ngsep_ctx::KnownVar& v, int64_t p) { return v.pos < p; });
            size_t pi = 0;
            for (; it != c->known.begin() + ke && it->pos <= o.last; ++it) {
                if (it->alt < 0) continue;
                while (pi < o.pos.size() && o.pos[pi].pos < it->pos) pi++;
                if (pi == o.pos.size() || o.pos[pi].pos != it->pos) continue;   // no pileup here
                vpos.push_back({(uint32_t)k, (uint32_t)pi});
                vknown.push_back(it - c->known.begin());
            }
        }
    } else {
        for (size_t k = 0; k < nr; k++)
            for (size_t i = 0; i < outs[k].pos.size(); i++) vpos.push_back({(uint32_t)k, (uint32_t)i});
    }
    const int64_t V = (int64_t)vpos.size();
    std::vector<int64_t> at_site((size_t)V, -1);             // v -> index of its KPM site (-1: none written)
    const ngsep_popsite_out* sites = nullptr;
    int64_t nsites = 0;
    if (V > 0) {
        Staged rs;
        rs.single = false;
        rs.known = true;                                       // the queue is given (no KTM / KQN) ...
        rs.n_samples = S;
        rs.tile = kPopTile;
        rs.g_len = ((V + kRunAlign - 1) / kRunAlign) * kRunAlign;
        rs.max_span = 1;
        rs.h_ref.assign((size_t)rs.g_len, 0);
        const int64_t ntile = rs.g_len / kPopTile;
        rs.h_prow.assign((size_t)ntile * S1, 0);
        auto col = [&](int64_t v, int s1, const uint8_t** p) -> uint32_t {
            const RegionOut& o = outs[vpos[(size_t)v].first];
            const RegionPos& q = o.pos[vpos[(size_t)v].second];
            const uint32_t b0 = o.poff[(size_t)(q.pcol + s1)], b1 = o.poff[(size_t)(q.pcol + s1 + 1)];
            *p = o.pcodes.data() + b0;
            return b1 - b0;
        };
        for (int64_t v = 0; v < V; v++)
            for (int s1 = 0; s1 < S1; s1++) {
                const uint8_t* p;
                const uint32_t n = col(v, s1, &p);
                int32_t& r = rs.h_prow[(size_t)(v / kPopTile) * S1 + s1];
                r = std::max<int32_t>(r, (int32_t)n);
            }
        rs.h_pboff.assign((size_t)ntile * S1 + 1, 0);
        std::vector<int64_t> stride((size_t)ntile, 0);
        int64_t po = 0;
        for (int64_t t = 0; t < ntile; t++) {
            int64_t so = 0;
            for (int s1 = 0; s1 < S1; s1++) { rs.h_pboff[(size_t)t * S1 + s1] = po + so; so += rs.h_prow[(size_t)t * S1 + s1]; }
            stride[(size_t)t] = so;
            po += so * kPopTile;
        }
        rs.h_pboff.back() = po;
        rs.ppile_bytes = po;
        rs.h_ppile.reset(new (std::nothrow) uint8_t[(size_t)po + 64]);
        if (!rs.h_ppile) return set_error(c, NGSEP_E_DEVICE, "host memory for the regions' population pile");
        std::memset(rs.h_ppile.get(), 0, (size_t)po + 64);
        for (int64_t v = 0; v < V; v++) {
            const int64_t t = v / kPopTile;
            for (int s1 = 0; s1 < S1; s1++) {
                const uint8_t* p;
                const uint32_t n = col(v, s1, &p);
                if (n) std::memcpy(rs.h_ppile.get() + rs.h_pboff[(size_t)t * S1 + s1] + (v - t * kPopTile) * stride[(size_t)t], p, n);
            }
            const RegionOut& o = outs[vpos[(size_t)v].first];
            const RegionPos& q = o.pos[vpos[(size_t)v].second];
            rs.h_forced.push_back((int32_t)v);                 // ... of discovery entries (no 0x400: createSNVVariantPool)
            if (known) {                                       //     or of the input SNVs (0x400: their alleles)
                const ngsep_ctx::KnownVar& kv = c->known[(size_t)vknown[(size_t)v]];
                rs.h_forced.push_back(0x80 | (kv.ref << 5) | (kv.alt << 8) | 0x400);
            } else {
                rs.h_forced.push_back(q.blocked ? 0 : (int32_t)ref_code(c, seq[(size_t)q.pos - 1]));
            }
        }
        std::string err;
        if (!ensure_device(c, err) || device_upload(c->dev, rs, err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
        LikTables t;
        GenotypeParams gp;
        compute_tables(c, &t, &gp);
        const ngsep_sample_call* calls = nullptr;
        double a = 0, b = 0, tot = 0;
        int64_t ncand = 0;
        if (device_run_multi(c->dev, rs, t, gp, S, c->params.min_allele_depth_freq, c->params.ploidy, &sites, &calls, &nsites,
                             &a, &b, &tot, &ncand, err) != 0)
            return set_error(c, NGSEP_E_DEVICE, err);
        for (int64_t i = 0; i < nsites; i++) at_site[(size_t)sites[i].seq_id] = i;   // (seq_id: the queue index)
    }
    // onPileup's rules, region by region (lastIndelEnd carried along the sequence)
    std::vector<int64_t> src;                                  // the kept SNV sites (KPM order), in output order
    std::vector<ngsep_popsite_out> add;
    std::vector<int64_t> add_text;                             // per added record: pop_text index (-1: an SNV site)
    std::vector<uint8_t> has;
    std::vector<RegionDecision> dec;
    int64_t v0 = 0;
    int32_t lie = 0;
    if (known) {
        // -knownVariants: every input SNV's record (KPM) and every non-SNV record of the replay, by position, input
        // order at a shared position (MultisampleVariantsDetector.onPileup :539-551 writes them all)
        auto text_rec = [&](const KnownCall& kc) {
            ngsep_popsite_out r;
            std::memset(&r, 0, sizeof r);
            r.multisnv_type = 3;
            for (int q = 0; q < 4; q++) r.alleles[q] = -1;
            r.seq_id = cr.seq_id;
            r.pos = kc.pos;
            add.push_back(r);
            add_text.push_back((int64_t)c->pop_text.size());
            c->pop_text.push_back(kc.line);
        };
        int64_t v = 0;
        for (size_t k = 0; k < nr; k++) {
            for (const KnownCall& kc : outs[k].kcalls) {
                while (v < V && vpos[(size_t)v].first == k && (outs[k].pos[vpos[(size_t)v].second].pos < kc.pos ||
                                                             (outs[k].pos[vpos[(size_t)v].second].pos == kc.pos && vknown[(size_t)v] < kc.known))) {
                    if (at_site[(size_t)v] >= 0) {
                        ngsep_popsite_out r = sites[at_site[(size_t)v]];
                        r.seq_id = cr.seq_id;
                        r.pos = outs[k].pos[vpos[(size_t)v].second].pos;
                        src.push_back(at_site[(size_t)v]);
                        add_text.push_back(-1);
                        add.push_back(r);
                    }
                    v++;
                }
                text_rec(kc);
            }
            while (v < V && vpos[(size_t)v].first == k) {
                if (at_site[(size_t)v] >= 0) {
                    ngsep_popsite_out r = sites[at_site[(size_t)v]];
                    r.seq_id = cr.seq_id;
                    r.pos = outs[k].pos[vpos[(size_t)v].second].pos;
                    src.push_back(at_site[(size_t)v]);
                    add_text.push_back(-1);
                    add.push_back(r);
                }
                v++;
            }
        }
    }
    for (size_t k = 0; k < nr && !known; k++) {
        const RegionOut& o = outs[k];
        has.assign(o.pos.size(), 0);
        for (size_t i = 0; i < o.pos.size(); i++) has[i] = at_site[(size_t)(v0 + (int64_t)i)] >= 0;
        resolve_population_region(o, has, c->params.call_embedded != 0, &lie, dec);
        size_t pi = 0;
        for (const RegionDecision& d : dec) {
            while (o.pos[pi].pos != d.pos) pi++;
            ngsep_popsite_out r;
            std::memset(&r, 0, sizeof r);
            if (d.kind == 1) {
                const int64_t si = at_site[(size_t)(v0 + (int64_t)pi)];
                r = sites[si];
                if (d.embedded) r.multisnv_type = 2;           // TYPE_EMBEDDED_SNV (MultisampleVariantsDetector.java:581)
                src.push_back(si);
                add_text.push_back(-1);
            } else {
                const PopIndel& pi2 = o.pindels[(size_t)d.idx];
                r.n_alleles = 0;
                r.multisnv_type = 3;                           // an indel / STR record: its text in pop_text
                r.qual = (int16_t)pi2.qs;
                for (int q = 0; q < 4; q++) r.alleles[q] = -1;
                add_text.push_back((int64_t)c->pop_text.size());
                c->pop_text.push_back(pi2.line);
            }
            r.seq_id = cr.seq_id;
            r.pos = d.pos;
            add.push_back(r);
        }
        v0 += (int64_t)o.pos.size();
    }
    // the SNV records' calls, gathered on the device into the call store (as run_device_multi's)
    std::string err;
    const size_t cfrom = c->pop_calls.size(), blk0 = cfrom / (size_t)std::max(S, 1);
    if (!src.empty()) {
        c->pop_calls.resize(cfrom + src.size() * (size_t)S);
        if (device_fetch_calls_ordered(c->dev, src.data(), (int64_t)src.size(), c->pop_calls.data() + cfrom, &c->pop_big, err) != 0)
            return set_error(c, NGSEP_E_DEVICE, err);
    }
    size_t ks = 0;
    for (size_t i = 0; i < add.size(); i++) {
        c->pop_sites.push_back(add[i]);
        c->pop_order.push_back(add_text[i] >= 0 ? add_text[i] : (int64_t)(blk0 + ks++));
    }
    c->stats.sites_called += (int64_t)add.size();
    // the sequence's records in position order (the region positions were kept out of its run: no position twice)
    const size_t n = c->pop_sites.size() - from;
    std::vector<size_t> ord(n);
    for (size_t i = 0; i < n; i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](size_t x, size_t y) { return c->pop_sites[from + x].pos < c->pop_sites[from + y].pos; });
    std::vector<ngsep_popsite_out> ps(n);
    std::vector<int64_t> po(n);
    for (size_t i = 0; i < n; i++) { ps[i] = c->pop_sites[from + ord[i]]; po[i] = c->pop_order[from + ord[i]]; }
    std::copy(ps.begin(), ps.end(), c->pop_sites.begin() + (ptrdiff_t)from);
    std::copy(po.begin(), po.end(), c->pop_order.begin() + (ptrdiff_t)from);
    return NGSEP_OK;
}

// java.lang.Math.round + PhredScoreHelper.calculatePhredScore (math/PhredScoreHelper.java:31-40)
int64_t java_round(double x) {
    if (std::isnan(x)) return 0;
    double f = std::floor(x);
    double r = (x - f >= 0.5) ? f + 1.0 : f;
    if (r >= 9.2233720368547758e18) return INT64_MAX;
    if (r <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)r;
}
int java_phred(double p) {
    if (p == 0) return 255;
    double score = -10 * std::log10(p);
    if (score > 255) return 255;
    return (int16_t)java_round(score);
}

// -csb: CountsHelper.getScoreStrandBiasFisher (CountsHelper.java:563-576), host side, emitted calls only.
static double fisher_exact(std::vector<double>& lf, int a, int b, int c, int d) {
    int n = a + b + c + d;
    if ((int)lf.size() <= n) {   // FisherExactTest.initLogFactorials (math/FisherExactTest.java:103-110)
        int m = std::max(n, 10000);
        lf.assign(m + 1, 0);
        for (int i = 2; i <= m; i++) lf[i] = lf[i - 1] + std::log10((double)i);
    }
    double ans = lf[a + b];
    ans += lf[c + d];
    ans += lf[a + c];
    ans += lf[b + d];
    ans -= lf[a];
    ans -= lf[b];
    ans -= lf[c];
    ans -= lf[d];
    ans -= lf[n];
    return std::pow(10.0, ans);
}
static double fisher_pvalue(std::vector<double>& lf, int a, int b, int c, int d) {   // FisherExactTest.java:65-101
    if (a > b) { std::swap(a, b); std::swap(c, d); }
    if (a > c) { std::swap(a, c); std::swap(b, d); }
    int e = std::min(a, d);
    double answer = 0;
    while (a >= 0 && d >= 0) {
        double p = fisher_exact(lf, a, b, c, d);
        if (e >= 10 && answer > (double)(100 * e) * p) break;
        answer += p;
        a--; b++; c++; d--; e++;
    }
    return answer;
}
static void apply_strand_bias(SiteStore& sites, size_t from) {
    std::vector<double> lf;
    for (size_t i = from; i < sites.size(); i++) {
        SiteRec& s = sites.rec[i];
        if (s.pool || s.n_alleles != 2 || s.genotype <= 0) continue;   // CalledSNV, not undecided/homRef (:218-220)
        int r = dna_index(s.ref), a = s.alt;
        int rn = s.strand[0], rp = s.strand[1], an = s.strand[2], ap = s.strand[3];
        if (s.is_call & kRecExt) {
            const ngsep_site_out& w = sites.ext[(size_t)SiteSet::ext_index(s)];
            rn = w.strand_counts[r][0]; rp = w.strand_counts[r][1]; an = w.strand_counts[a][0]; ap = w.strand_counts[a][1];
        }
        double pv = fisher_pvalue(lf, rn, an, rp, ap);
        s.strand_bias = (int8_t)std::min(100, java_phred(pv));   // MAX_STRAND_BIAS_SCORE
    }
}

// MultisampleVariantsDetector run: sites come back unordered with global positions; order them by
// position and map them to (sequence, position) (the listener writes in pileup order, :534-535)
// the emitted sites (unordered) of one pass into the context's result in position order; `fetch` brings their
// calls back in that order into the call store
template <class Fetch>
static int order_population_sites(ngsep_ctx* c, const ngsep_popsite_out* sites, int64_t n, Fetch&& fetch) {
    const size_t S = c->sample_ids.size();
    std::string err;
    std::vector<int64_t> order((size_t)n);
    for (size_t i = 0; i < order.size(); i++) order[i] = (int64_t)i;
    // position order; KPM leaves each site's queue index in seq_id, so sites of one position (input variants
    // of -knownVariants) keep the queue's (input) order
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
        return sites[a].pos != sites[b].pos ? sites[a].pos < sites[b].pos : sites[a].seq_id < sites[b].seq_id;
    });
    const std::vector<Window>& ws = c->staged.windows;
    size_t wi = 0;
    const size_t from = c->pop_sites.size();
    std::vector<int64_t> src;                   // staging index of each kept site, in output order
    src.reserve((size_t)n);
    for (int64_t i : order) {
        ngsep_popsite_out o = sites[(size_t)i];
        const int64_t gpos = o.pos;
        while (wi + 1 < ws.size() && ws[wi + 1].gbase <= gpos) wi++;
        const Window& w = ws[wi];
        const int64_t off = gpos - w.gbase - w.pad;
        if (off < 0 || off >= w.wlen) continue;
        o.seq_id = w.seq_id;
        o.pos = (int32_t)(w.w0 + off);
        c->pop_sites.push_back(o);
        src.push_back(i);
    }
    // the sites' calls: fetch puts them into the call store and sets the sites' pop_order entries
    (void)S;
    if (fetch(src.data(), (int64_t)src.size(), err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
    c->stats.sites_called += (int64_t)(c->pop_sites.size() - from);
    return NGSEP_OK;
}

static int run_device_multi(ngsep_ctx* c, const LikTables& t, const GenotypeParams& gp, double* elapsed_ms) {
    const ngsep_popsite_out* sites = nullptr;
    const ngsep_sample_call* calls = nullptr;
    int64_t n = 0;
    double scan_ms = 0, geno_ms = 0, total_ms = 0;
    int64_t ncand = 0;
    std::string err;
    const size_t S = c->sample_ids.size();
    if (device_run_multi(c->dev, c->staged, t, gp, (int32_t)S, c->params.min_allele_depth_freq, c->params.ploidy,
                         &sites, &calls, &n, &scan_ms, &geno_ms, &total_ms, &ncand, err) != 0)
        return set_error(c, NGSEP_E_DEVICE, err);
    const int rc = order_population_sites(c, sites, n, [&](const int64_t* src, int64_t m, std::string& e) {
        // gathered into output order on the device, copied straight into the (pinned) call store
        const size_t cfrom = c->pop_calls.size(), blk0 = cfrom / S;
        c->pop_calls.resize(cfrom + (size_t)m * S);
        for (int64_t k = 0; k < m; k++) c->pop_order.push_back((int64_t)blk0 + k);
        return device_fetch_calls_ordered(c->dev, src, m, c->pop_calls.data() + cfrom, &c->pop_big, e);
    });
    if (rc != NGSEP_OK) return rc;
    c->stats.candidates = ncand;
    c->stats.hard_sites = (int32_t)device_last_hard(c->dev);
    c->stats.exact_bound_passes = device_last_exact(c->dev);
    c->stats.kernel_ms = total_ms;
    c->stats.scan_ms = scan_ms;
    c->stats.genotype_ms = geno_ms;
    if (elapsed_ms) *elapsed_ms = total_ms;
    return NGSEP_OK;
}

static int finish_run(ngsep_ctx* c, size_t from, int64_t n, double scan_ms, double geno_ms, double total_ms,
                      int64_t ncand, double* elapsed_ms);

int run_device(ngsep_ctx* c, double* elapsed_ms) {
    if (c->params.multisample) {
        LikTables t;
        GenotypeParams gp;
        compute_tables(c, &t, &gp);
        if (const int rc = prepare_pool(c)) return rc;
        return run_device_multi(c, t, gp, elapsed_ms);
    }
    return run_device_into(c, c->sites, elapsed_ms);
}

static int finish_run_into(ngsep_ctx* c, SiteStore& dest, size_t from, int64_t n, double scan_ms, double geno_ms, double total_ms,
                           int64_t ncand, double* elapsed_ms);

// single sample: the staged run's records appended to dest
int run_device_into(ngsep_ctx* c, SiteStore& dest, double* elapsed_ms) {
    LikTables t;
    GenotypeParams gp;
    compute_tables(c, &t, &gp);
    if (const int rc = prepare_pool(c)) return rc;
    int64_t n = 0;
    double scan_ms = 0, geno_ms = 0, total_ms = 0;
    int64_t ncand = 0;
    std::string err;
    // exact pruning is proven for h <= 0.1 ("why pruning is exact"); the pool algorithm's
    // candidate test holds for any h
    int prune = c->params.prune_candidates && !c->params.dump_all_positions && (c->het_rate <= 0.1 || c->params.ploidy >= 3);
    const size_t from = dest.size();
    if (device_run(c->dev, c->staged, t, gp, prune, &dest, &n, &scan_ms, &geno_ms, &total_ms, &ncand, err) != 0)
        return set_error(c, NGSEP_E_DEVICE, err);
    return finish_run_into(c, dest, from, n, scan_ms, geno_ms, total_ms, ncand, elapsed_ms);
}

// records arrive sorted by global position with their (sequence, position) set by KO; windows are
// laid out in processing order, so this is (sequence order, position).
static int finish_run(ngsep_ctx* c, size_t from, int64_t n, double scan_ms, double geno_ms, double total_ms,
                      int64_t ncand, double* elapsed_ms) {
    return finish_run_into(c, c->sites, from, n, scan_ms, geno_ms, total_ms, ncand, elapsed_ms);
}
static int finish_run_into(ngsep_ctx* c, SiteStore& dest, size_t from, int64_t n, double scan_ms, double geno_ms, double total_ms,
                           int64_t ncand, double* elapsed_ms) {
    (void)n;
    if (c->params.calc_strand_bias && c->known.empty()) apply_strand_bias(dest, from);   // (genotypeSNV: none)
    c->stats.candidates = ncand;
    c->stats.hard_sites = (int32_t)device_last_hard(c->dev);
    c->stats.exact_bound_passes = device_last_exact(c->dev);
    c->stats.sites_called += (int64_t)(dest.size() - from);
    c->stats.kernel_ms = total_ms;
    c->stats.scan_ms = scan_ms;
    c->stats.genotype_ms = geno_ms;
    if (elapsed_ms) *elapsed_ms = total_ms;
    return NGSEP_OK;
}

// ---- reference loading: FastaFileReader with keepLowerCase (sequences/io/FastaFileReader.java:170-205) ----
// ---- CoverageStatisticsCalculator (discovery/CoverageStatisticsCalculator.java:108-216) ----
// The admitted reads of every sequence in one global coordinate: sequence k's region starts at gbase_k
// (position p -> gbase_k + p) and spans max(sequence length, largest last) + 2 positions, so a read's
// end never leaks into the next region.
int coverage_stage(ngsep_ctx* c, std::vector<ContigReads>& contigs) {
    std::vector<int64_t> gfirst;
    std::vector<uint32_t> spanu;
    int64_t n = 0;
    for (const auto& cr : contigs) n += (int64_t)cr.first.size();
    gfirst.reserve((size_t)n);
    spanu.reserve((size_t)n);
    int64_t gbase = 0;
    int32_t max_span = 1;
    for (const auto& cr : contigs) {
        int64_t region = cr.seq_id >= 0 ? (int64_t)c->seq_bases[(size_t)cr.seq_id].size() : 0;
        for (size_t i = 0; i < cr.first.size(); i++) {
            if (cr.first[i] < 0) return set_error(c, NGSEP_E_INVALID, "alignment with a negative first position");
            const int32_t span = std::max<int32_t>(0, cr.last[i] - cr.first[i] + 1);
            gfirst.push_back(gbase + cr.first[i]);
            spanu.push_back(((uint32_t)span << 1) | (cr.uniq[i] ? 1u : 0u));
            region = std::max<int64_t>(region, cr.last[i]);
            max_span = std::max(max_span, span);
        }
        gbase += region + 2;
    }
    if (!c->cov_dev) {
        std::string err;
        c->cov_dev = cov_create(c->device, err);
        if (!c->cov_dev) return set_error(c, NGSEP_E_DEVICE, err);
    }
    std::string err;
    if (cov_upload(c->cov_dev, gfirst, spanu, gbase, max_span, err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
    c->cov_staged = true;
    return NGSEP_OK;
}

int coverage_run(ngsep_ctx* c, double* kernel_ms) {
    if (!c->cov_dev || !c->cov_staged) return set_error(c, NGSEP_E_INVALID, "no coverage reads staged");
    const int32_t mc = c->params.max_coverage;
    std::vector<uint64_t> h((size_t)(2 * (mc + 1)), 0);
    std::string err;
    double ms = 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (cov_run(c->cov_dev, mc, h.data(), &ms, err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
    c->stats.kernel_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->stats.scan_ms = ms;
    if (c->cov_hist.size() != h.size()) c->cov_hist.assign(h.size(), 0);
    for (size_t k = 0; k < h.size(); k++) c->cov_hist[k] += h[k];
    if (kernel_ms) *kernel_ms = ms;
    return NGSEP_OK;
}

static inline char mask_base(char ch) {
    switch (ch) {
        case 'A': case 'a': case 'C': case 'c': case 'N': case 'n':
        case 'G': case 'g': case 'T': case 't': return ch;
        default: return 'N';   // DNAMaskedSequence default index
    }
}
// ReferenceGenome(filename, keepLowerCase = true) (genome/ReferenceGenome.java:40-62): the file is mapped, its lines
// cut with memchr on one thread, and the sequence lines translated (mask_base) into the sequences on all threads
int load_fasta(ngsep_ctx* c, const char* path) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return set_error(c, NGSEP_E_IO, std::string("cannot open ") + path);
    struct stat sb;
    if (fstat(fd, &sb) != 0) { ::close(fd); return set_error(c, NGSEP_E_IO, std::string("cannot stat ") + path); }
    const size_t n = (size_t)sb.st_size;
    const char* buf = nullptr;
    void* map = nullptr;
    if (n) {
        map = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
        if (map == MAP_FAILED) { ::close(fd); return set_error(c, NGSEP_E_IO, std::string("cannot map ") + path); }
        madvise(map, n, MADV_SEQUENTIAL);
        buf = static_cast<const char*>(map);
    }
    struct Seg { size_t src; int64_t dst; int64_t len; };
    struct Rec { std::string name; int64_t len = 0; size_t seg0 = 0; };
    std::vector<Rec> recs;
    std::vector<Seg> segs;
    size_t pos = 0;
    while (pos < n) {
        const char* nl = static_cast<const char*>(std::memchr(buf + pos, '\n', n - pos));
        const size_t end = nl ? (size_t)(nl - buf) : n;
        size_t l = end - pos;
        while (l > 0 && (buf[pos + l - 1] == '\r' || buf[pos + l - 1] == '\n')) l--;   // (getline + trailing CR/LF strip)
        if (l > 0 && buf[pos] == '>') {
            size_t e = 1;
            while (e < l && buf[pos + e] != ' ' && buf[pos + e] != '\t' && buf[pos + e] != '\0') e++;
            recs.push_back(Rec{std::string(buf + pos + 1, e - 1), 0, segs.size()});
        } else if (!recs.empty() && l > 0) {
            segs.push_back(Seg{pos, recs.back().len, (int64_t)l});
            recs.back().len += (int64_t)l;
        }
        pos = end + 1;
    }
    const size_t first = c->seq_bases.size();
    for (Rec& r : recs) {
        c->seq_names.push_back(r.name);
        c->seq_bases.emplace_back();
        c->seq_bases.back().resize((size_t)r.len);
    }
    std::vector<int32_t> seg_rec(segs.size());
    for (size_t k = 0; k < recs.size(); k++)
        for (size_t i = recs[k].seg0, e = k + 1 < recs.size() ? recs[k + 1].seg0 : segs.size(); i < e; i++) seg_rec[i] = (int32_t)k;
    parallel_for((int64_t)segs.size(), 1 << 12, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            const Seg& g = segs[(size_t)i];
            char* dst = &c->seq_bases[first + (size_t)seg_rec[(size_t)i]][(size_t)g.dst];
            for (int64_t k = 0; k < g.len; k++) dst[k] = mask_base(buf[g.src + (size_t)k]);
        }
    });
    if (map) munmap(map, n);
    ::close(fd);
    return NGSEP_OK;
}

}  // namespace ngsep

// ======================= C ABI (engine part) =======================
using namespace ngsep;

extern "C" int ngsep_abi_version(void) { return NGSEP_ABI_VERSION; }

extern "C" void ngsep_params_default(ngsep_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->min_mq = 20;
    p->max_alns_per_start = 5;
    p->max_base_qs = 30;
    p->min_quality = 40;
    p->ploidy = 2;
    p->het_rate = 0.001;
    p->query_first = 0;
    p->query_last = 1000000000;
    std::snprintf(p->sample_id, sizeof p->sample_id, "Sample");
    p->prune_candidates = 1;
    p->window_positions = 1 << 26;
    p->max_coverage = 300;
    p->relative_allele_counts = 0;
    p->rac_min_rd = 10;                     // RelativeAlleleCountsCalculator.DEF_MIN_RD
    p->rac_min_bq = 20;                     // DEF_MIN_BASE_QUALITY_SCORE
}

extern "C" int ngsep_open(int device, const ngsep_params* params, ngsep_ctx** out) {
    if (!out) return NGSEP_E_INVALID;
    ngsep_ctx* c = new ngsep_ctx();
    if (params) c->params = *params;
    else ngsep_params_default(&c->params);
    c->device = device;
    if (c->params.coverage_stats) {
        *out = c;
        if (c->params.max_coverage < 1 || c->params.max_coverage > 1024)
            return set_error(c, NGSEP_E_UNSUPPORTED, "maxCoverage outside [1, 1024] (LDS histograms of the coverage kernel)");
        if (c->params.multisample || c->params.query_seq[0])
            return set_error(c, NGSEP_E_INVALID, "coverage statistics take no samples and no query region");
    }
    if (c->params.relative_allele_counts) {
        *out = c;
        if (c->params.multisample || c->params.coverage_stats)
            return set_error(c, NGSEP_E_INVALID, "relative allele counts run alone (no samples, no coverage statistics)");
        if (c->params.rac_min_bq < 4 || c->params.rac_min_bq > 30)
            return set_error(c, NGSEP_E_UNSUPPORTED, "minBQ outside [4, 30] (the pile's codes clamp qualities to 30 and drop the base of q <= 3 calls)");
    }
    if (c->params.ploidy > 2 * kPoolMaxFreq) {
        *out = c;
        return set_error(c, NGSEP_E_UNSUPPORTED, "ploidy above " + std::to_string(2 * kPoolMaxFreq) +
                                                     " (the pool algorithm's hypotheses table)");
    }
    // SingleSampleVariantsDetector.run (:591-593); MultisampleVariantsDetector keeps -h as given
    c->het_rate = c->params.het_rate;
    if (!c->params.multisample && !c->params.het_rate_set && c->params.ploidy == 1) c->het_rate = 1e-6;
    *out = c;
    return NGSEP_OK;
}

// The device (HIP context, streams, code object) takes ~0.1 s to bring up: path B starts it on a thread of its
// own when the call begins, so it overlaps the FASTA-checked BAM header, decoding and the first window's layout.
void ngsep::start_device_init(ngsep_ctx* c) {
    std::lock_guard<std::mutex> lk(c->dev_mu);
    if (c->dev || c->dev_init.joinable()) return;
    c->dev_init = std::thread([c] { c->dev_init_result = device_create(c->device, c->dev_init_err); });
}

ngsep::Device* ngsep::ensure_device(ngsep_ctx* c, std::string& err) {
    std::lock_guard<std::mutex> lk(c->dev_mu);
    if (c->dev_init.joinable()) {
        c->dev_init.join();
        if (!c->dev) c->dev = c->dev_init_result;
        else if (c->dev_init_result) device_destroy(c->dev_init_result);
        c->dev_init_result = nullptr;
        if (!c->dev) err = c->dev_init_err;
    }
    if (!c->dev) c->dev = device_create(c->device, err);
    return c->dev;
}

extern "C" int ngsep_close(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    {
        std::string e;
        if (c->dev_init.joinable()) ngsep::ensure_device(c, e);
    }
    if (c->stream.job && c->stream.job->th.joinable()) c->stream.job->th.join();
    c->stream.job.reset();
    c->arena.release();
    if (c->dev) device_destroy(c->dev);
    if (c->cov_dev) cov_destroy(c->cov_dev);
    for (auto& m : c->gz_in_pool) ngsep::gz_host_free(m.first);
    for (auto& m : c->gz_chunk_pool) ngsep::gz_host_free(m.first);
    if (c->gz) ngsep::gz_destroy(c->gz);
    delete c;
    return NGSEP_OK;
}

extern "C" const char* ngsep_last_error(ngsep_ctx* c) { return c ? c->err.c_str() : "null context"; }

extern "C" int ngsep_get_stats(ngsep_ctx* c, ngsep_stats* out) {
    if (!c || !out) return NGSEP_E_INVALID;
    *out = c->stats;
    out->realign_ms = (double)c->realign_ns.load() * 1e-6;
    out->realign_regions = c->realign_regions.load();
    out->keep_raw_ms = (double)c->keep_raw_ns.load() * 1e-6;
    out->region_setup_ms = (double)c->region_setup_ns.load() * 1e-6;
    out->region_gather_ms = (double)c->region_gather_ns.load() * 1e-6;
    out->region_device_ms = (double)c->region_device_ns.load() * 1e-6;
    out->region_merge_ms = (double)c->region_merge_ns.load() * 1e-6;
    out->window_wait_ms = (double)c->window_wait_ns.load() * 1e-6;
    return NGSEP_OK;
}

extern "C" int ngsep_device_count(void) { return device_count(); }

extern "C" int ngsep_set_reference(ngsep_ctx* c, const char* name, const char* bases, int64_t len) {
    if (!c || !name || (!bases && len > 0) || len < 0) return NGSEP_E_INVALID;
    c->seq_names.emplace_back(name);
    std::string s(bases, (size_t)len);
    for (char& ch : s) ch = mask_base(ch);
    c->seq_bases.push_back(std::move(s));
    return NGSEP_OK;
}

extern "C" int ngsep_load_fasta(ngsep_ctx* c, const char* path) {
    if (!c || !path) return NGSEP_E_INVALID;
    return load_fasta(c, path);
}

extern "C" int ngsep_n_sequences(ngsep_ctx* c) { return c ? (int)c->seq_names.size() : 0; }
extern "C" const char* ngsep_sequence_name(ngsep_ctx* c, int i) {
    if (!c || i < 0 || i >= (int)c->seq_names.size()) return nullptr;
    return c->seq_names[i].c_str();
}

extern "C" int ngsep_process_alignments(ngsep_ctx* c, const ngsep_read_batch* b) {
    if (!c) return NGSEP_E_INVALID;
    c->staging_mode = false;
    return process_batch(c, b, false);
}

namespace ngsep {
int process_alignments_packed(ngsep_ctx* c, const PackedBatch* b) {
    if (!c || !b) return NGSEP_E_INVALID;
    c->staging_mode = false;
    return process_batch(c, &b->b, true, b->qual_off);
}
int process_alignments_gathered(ngsep_ctx* c, const ngsep_read_batch* b, const char* const* chars_at, const char* const* quals_at) {
    if (!c || !b || !chars_at || !quals_at) return NGSEP_E_INVALID;
    c->staging_mode = false;
    return process_batch(c, b, false, nullptr, chars_at, quals_at);
}
}  // namespace ngsep

extern "C" int ngsep_notify_end(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    int rc = flush_sequence(c);
    if (rc != NGSEP_OK || !c->params.coverage_stats || c->staging_mode) return rc;
    rc = coverage_stage(c, c->staged_contigs);
    c->staged_contigs.clear();
    if (rc == NGSEP_OK) rc = coverage_run(c, nullptr);
    cov_release(c->cov_dev);
    c->cov_staged = false;
    return rc;
}

extern "C" int ngsep_fetch_coverage(ngsep_ctx* c, int64_t* counts, int64_t* counts_unique, int64_t* high, int64_t* high_unique) {
    if (!c) return NGSEP_E_INVALID;
    if (!c->params.coverage_stats) return set_error(c, NGSEP_E_INVALID, "context not in coverage mode");
    const int32_t mc = c->params.max_coverage;
    if (c->cov_hist.size() != (size_t)(2 * (mc + 1))) c->cov_hist.assign((size_t)(2 * (mc + 1)), 0);
    for (int32_t i = 0; i < mc; i++) {
        if (counts) counts[i] = i == 0 ? 0 : (int64_t)c->cov_hist[(size_t)i];
        if (counts_unique) counts_unique[i] = i == 0 ? 0 : (int64_t)c->cov_hist[(size_t)(mc + 1 + i)];
    }
    if (high) *high = (int64_t)c->cov_hist[(size_t)mc];
    if (high_unique) *high_unique = (int64_t)c->cov_hist[(size_t)(2 * mc + 1)];
    return NGSEP_OK;
}

extern "C" int ngsep_clear_coverage(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    c->cov_hist.clear();
    return NGSEP_OK;
}

// CoverageStatisticsCalculator.printCoverageStats (:209-215)
extern "C" int ngsep_write_coverage(ngsep_ctx* c, const char* path) {
    if (!c || !path) return NGSEP_E_INVALID;
    const int32_t mc = c->params.max_coverage;
    std::vector<int64_t> a((size_t)mc), u((size_t)mc);
    int64_t hi = 0, hu = 0;
    int rc = ngsep_fetch_coverage(c, a.data(), u.data(), &hi, &hu);
    if (rc != NGSEP_OK) return rc;
    std::string out;
    char line[96];
    for (int32_t i = 1; i < mc; i++) {
        std::snprintf(line, sizeof line, "%d\t%lld\t%lld\n", i, (long long)a[(size_t)i], (long long)u[(size_t)i]);
        out += line;
    }
    std::snprintf(line, sizeof line, "More\t%lld\t%lld\n", (long long)hi, (long long)hu);
    out += line;
    const bool to_stdout = std::strcmp(path, "-") == 0;
    FILE* f = to_stdout ? stdout : std::fopen(path, "w");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot write ") + path);
    const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
    if (to_stdout) std::fflush(f); else std::fclose(f);
    return ok ? NGSEP_OK : set_error(c, NGSEP_E_IO, std::string("cannot write ") + path);
}

extern "C" int ngsep_fetch_sites(ngsep_ctx* c, ngsep_site_out* out, int64_t cap, int64_t* n_out) {
    if (!c) return NGSEP_E_INVALID;
    int64_t n = (int64_t)c->sites.size();
    if (n_out) *n_out = n;
    if (out && cap > 0)
        for (int64_t i = 0; i < std::min(n, cap); i++) out[i] = c->sites.full((size_t)i);
    return NGSEP_OK;
}

extern "C" int ngsep_clear_sites(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    c->sites.clear();
    return NGSEP_OK;
}

// SingleSampleVariantsDetector.findSNVS with -knownVariants (:896-906): VCFFileReader.loadVariants(file, true,
// true) (vcf/VCFFileReader.java:196-260,585-600) into a GenomicRegionSortedCollection over the genome.  Biallelic
// SNVs (one-base REF and ALT in ACGT) are genotyped here; ALT '.' records are skipped, as are records on
// sequences outside the reference; any other variant is refused (E_UNSUPPORTED: the indel / multi-allelic
// genotyping of genotypeVariantSample is not in this build).  path NULL or "": back to discovery.
// ---- -knownSTRs ----
// Integer.parseInt: an optional sign and decimal digits, inside the int range
static bool parse_java_int(const char* t, int32_t* out) {
    const char* q = t;
    bool neg = false;
    if (*q == '-' || *q == '+') { neg = *q == '-'; q++; }
    if (!*q) return false;
    int64_t v = 0;
    for (; *q; q++) {
        if (*q < '0' || *q > '9') return false;
        v = v * 10 + (*q - '0');
        if (v > 2147483648LL) return false;
    }
    if (neg) v = -v;
    if (v > INT32_MAX || v < INT32_MIN) return false;
    *out = (int32_t)v;
    return true;
}

// ReferenceGenome.getReference(first, last) upper-cased (ReferenceGenome.java:217-237: absent outside [1, length])
static bool ref_upper(const std::string& seq, int64_t first, int64_t last, std::string* out) {
    if (first < 1 || last > (int64_t)seq.size() || last < first - 1) return false;
    out->assign(seq, (size_t)first - 1, (size_t)(last - first + 1));
    for (char& ch : *out) if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
    return true;
}

// SingleSampleVariantsDetector.mergeSTRs (:873-881) with AbstractLimitedSequence.getOverlapLength
// (sequences/AbstractLimitedSequence.java:376-390: the longest suffix of the first that prefixes the second)
static bool merge_strs(const std::string& seq, int64_t first, int64_t last, int64_t rfirst, int64_t rlast) {
    if (rfirst - last > 5) return false;
    if (rfirst - last <= 2) return true;
    std::string a, b;
    if (!ref_upper(seq, std::max(first, last - 10), last, &a) || !ref_upper(seq, rfirst, rlast, &b)) return false;
    for (size_t i = 0; i < a.size(); i++) {
        const size_t l = a.size() - i;
        if (l <= b.size() && a.compare(i, l, b, 0, l) == 0) return l > 5;
    }
    return false;
}

extern "C" int ngsep_set_known_strs(ngsep_ctx* c, const char* path) {
    if (!c) return NGSEP_E_INVALID;
    if (c->known_given) return NGSEP_OK;   // -knownVariants set: the realigner's inputs are its records (findSNVS :897-906)
    c->strs.clear();
    if (!path || !path[0]) return NGSEP_OK;
    if (c->seq_names.empty()) return set_error(c, NGSEP_E_INVALID, "load the reference before the known STRs");
    // (an option of both variant detectors: SingleSampleVariantsDetector.findSNVS :906-912, MultisampleVariantsDetector.run
    // :439-446 -- in both the indel realigner's input variants)
    if (c->params.coverage_stats || c->params.relative_allele_counts)
        return set_error(c, NGSEP_E_INVALID, "known STRs are an option of the variant detectors only");
    std::FILE* f = std::fopen(path, "r");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot read ") + path);
    std::unordered_map<std::string, int32_t> idx;
    for (size_t i = 0; i < c->seq_names.size(); i++) idx[c->seq_names[i]] = (int32_t)i;
    // SimpleGenomicRegionFileHandler.loadRegions (genome/io/SimpleGenomicRegionFileHandler.java:57-80): fields split at
    // every space or tab; a line whose name, first or last does not parse is skipped (a warning there)
    std::vector<std::vector<StrVar>> per(c->seq_names.size());
    char* line = nullptr;
    size_t cap = 0;
    ssize_t l;
    while ((l = getline(&line, &cap, f)) >= 0) {
        while (l > 0 && (line[l - 1] == '\n' || line[l - 1] == '\r')) line[--l] = 0;
        const char* fld[3];
        int k = 0;
        char* p = line;
        while (k < 3) {
            fld[k++] = p;
            char* t = p;
            while (*t && *t != ' ' && *t != '\t') t++;
            if (!*t) break;
            *t = 0;
            p = t + 1;
        }
        int32_t a, b;
        if (k < 3 || !parse_java_int(fld[1], &a) || !parse_java_int(fld[2], &b)) continue;
        auto it = idx.find(fld[0]);
        if (it == idx.end() || b < a - 1) continue;   // (a sequence the genome lacks is never emitted; subSequence would throw)
        per[(size_t)it->second].push_back(StrVar{a, b});
    }
    std::free(line);
    std::fclose(f);
    // makeNonRedundantSTRs / makeSTRVariant (SingleSampleVariantsDetector.java:843-894): per sequence, in
    // GenomicRegionPositionComparator order (first, then last; stable), runs of mergeable regions become one variant
    // [first - 1, last + 1] clipped to the sequence (`last` is the run's LAST region's end)
    c->strs.assign(c->seq_names.size(), {});
    for (size_t sq = 0; sq < per.size(); sq++) {
        std::vector<StrVar>& v = per[sq];
        if (v.empty()) continue;
        std::stable_sort(v.begin(), v.end(), [](const StrVar& x, const StrVar& y) { return x.first != y.first ? x.first < y.first : x.last < y.last; });
        const std::string& seq = c->seq_bases[sq];
        const int64_t len = (int64_t)seq.size();
        std::vector<StrVar>& out = c->strs[sq].v;
        auto emit = [&](int64_t first, int64_t last) {
            const int64_t vf = std::max<int64_t>(1, first - 1), vl = std::min<int64_t>(last + 1, len);
            if (vf >= 1 && vl <= len && vl >= vf - 1) out.push_back(StrVar{(int32_t)vf, (int32_t)vl});
        };
        int64_t first = 0, last = 0;
        for (const StrVar& r : v) {
            if (last == 0 || !merge_strs(seq, first, last, r.first, r.last)) {
                if (last > 0) emit(first, last);
                first = r.first;
            }
            last = r.last;
        }
        if (last > 0) emit(first, last);
        std::stable_sort(out.begin(), out.end(), [](const StrVar& x, const StrVar& y) { return x.first != y.first ? x.first < y.first : x.last < y.last; });
        c->strs[sq].finish();
    }
    return NGSEP_OK;
}

extern "C" int ngsep_set_known_variants(ngsep_ctx* c, const char* vcf_path) {
    if (!c) return NGSEP_E_INVALID;
    if (c->known_given) {
        // the realigner's input variants were the previous file's records: a cleared (or refused) file leaves none,
        // as in a fresh session (-knownSTRs given before -knownVariants were dropped by it and must be set again)
        c->strs.clear();
        c->str_next = 0;
    }
    c->known.clear();
    c->known_recs.clear();
    c->known_seq_begin.clear();
    c->known_given = false;
    if (!vcf_path || !vcf_path[0]) return NGSEP_OK;
    if (c->seq_names.empty()) return set_error(c, NGSEP_E_INVALID, "load the reference before the known variants");
    if (c->params.coverage_stats || c->params.relative_allele_counts)
        return set_error(c, NGSEP_E_INVALID, "known variants are genotyped by the variant detectors only");
    std::FILE* f = std::fopen(vcf_path, "r");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot read ") + vcf_path);
    std::unordered_map<std::string, int32_t> idx;
    for (size_t i = 0; i < c->seq_names.size(); i++) idx[c->seq_names[i]] = (int32_t)i;
    std::vector<ngsep_ctx::KnownVar> v;
    std::vector<KnownRecord> recs;
    char* line = nullptr;
    size_t cap = 0;
    ssize_t l;
    int rc = NGSEP_OK;
    int64_t lineno = 0;
    // GenomicVariantImpl.getVariantTypeId names (GenomicVariant.java:32-56, GenomicVariantImpl.java:44-60)
    static const char* kNames[] = {"SNV", "MULTISNV", "EMBEDDED", "INDEL", "STR", "CNV", "REPEAT", "DEL", "INS", "INV", "DUP",
                                   "Deletion", "Insertion"};
    static const int kIds[] = {1, 2, 3, 4, 5, 10, 11, 12, 13, 14, 15, 12, 13};
    auto type_id = [&](const char* name, size_t n) {
        for (int q = 0; q < 13; q++) if (std::strlen(kNames[q]) == n && std::strncmp(kNames[q], name, n) == 0) return kIds[q];
        return 0;
    };
    while ((l = getline(&line, &cap, f)) >= 0) {
        lineno++;
        while (l > 0 && (line[l - 1] == '\n' || line[l - 1] == '\r')) line[--l] = 0;
        if (l == 0 || line[0] == '#') continue;
        const char* fld[8];
        int k = 0;
        char* p = line;
        while (k < 8) { fld[k++] = p; char* t = std::strchr(p, '\t'); if (!t) break; *t = 0; p = t + 1; }
        if (k < 6) { rc = set_error(c, NGSEP_E_FORMAT, "VCF line " + std::to_string(lineno) + " has fewer than the 6 columns CHROM to QUAL"); break; }
        if (fld[4][0] == '.') continue;                                  // a reference site (filterReferenceSitesGVCF)
        auto it = idx.find(fld[0]);
        if (it == idx.end()) continue;
        // loadInfoField (VCFFileReader.java:261-305), attribute by attribute: TYPE sets an id in (0, TYPE_INVERSION],
        // SVTYPE one >= 10, END the last position of a GenomicVariantImpl
        int type = 0;
        int32_t end = 0;
        if (k >= 8 && std::strcmp(fld[7], ".") != 0) {
            for (const char* t = fld[7]; *t;) {
                const char* e = std::strchr(t, ';');
                const size_t n = e ? (size_t)(e - t) : std::strlen(t);
                if (n > 5 && std::strncmp(t, "TYPE=", 5) == 0) { const int id = type_id(t + 5, n - 5); if (id > 0 && id <= 14) type = id; }
                if (n > 7 && std::strncmp(t, "SVTYPE=", 7) == 0) { const int id = type_id(t + 7, n - 7); if (id >= 10) type = id; }
                if (n > 4 && std::strncmp(t, "END=", 4) == 0) end = std::atoi(t + 4);
                t = e ? e + 1 : t + n;
            }
        }
        if (type >= 10) continue;                                        // structural (filterSVs)
        // loadGenomicVariant (:192-255): an SNV object for one-base A/C/G/T REF and ALT, else a GenomicVariantImpl
        // over REF and the ALT alleles (upper-cased)
        std::vector<std::string> alleles{fld[3]};
        for (const char* t = fld[4];;) {
            const char* e = std::strchr(t, ',');
            alleles.emplace_back(t, e ? (size_t)(e - t) : std::strlen(t));
            if (!e) break;
            t = e + 1;
        }
        const int a = dna_index(fld[3][0]), b = dna_index(fld[4][0]);
        const bool snv = alleles.size() == 2 && alleles[0].size() == 1 && alleles[1].size() == 1 && a >= 0 && b >= 0;
        int16_t qs = 0;
        if (fld[5][0] && fld[5][0] != '.') {
            double q = std::atof(fld[5]);
            if (q > 32767) q = 255;
            qs = (int16_t)java_round(q);
        }
        ngsep_ctx::KnownVar kv;
        kv.seq = it->second;
        kv.pos = std::atoi(fld[1]);
        kv.last = kv.pos + (int32_t)alleles[0].size() - 1;
        kv.qs = qs;
        kv.type = (int8_t)type;
        kv.rec = -1;
        if (std::strcmp(fld[2], ".") != 0) kv.id = fld[2];
        if (snv) {
            kv.ref = (int8_t)a;
            kv.alt = (int8_t)b;
        } else {
            for (std::string& x : alleles) for (char& ch : x) ch = (char)std::toupper((unsigned char)ch);
            bool all_snv = true, dup = false;                            // GenomicVariantImpl.isSNV (:254-261)
            for (size_t i = 0; i < alleles.size(); i++) {
                all_snv = all_snv && alleles[i].size() == 1 && dna_index(alleles[i][0]) >= 0;
                for (size_t j = 0; j < i; j++) dup = dup || alleles[i] == alleles[j];
            }
            if (all_snv || dup || alleles.size() > 100 || alleles[0].empty()) {
                rc = set_error(c, NGSEP_E_UNSUPPORTED, std::string("known variant ") + fld[0] + ":" + fld[1] +
                                                       (all_snv ? " is a multi-allelic SNV" : dup ? " repeats an allele" : " has too many alleles") +
                                                       " (not genotyped by this build)");
                break;
            }
            if (end > 0) kv.last = end;                                  // END of a GenomicVariantImpl (:282-289)
            kv.ref = dna_index(alleles[0][0]) >= 0 ? (int8_t)dna_index(alleles[0][0]) : 0;
            kv.alt = -1;
            kv.rec = (int32_t)recs.size();
            KnownRecord kr;
            kr.alleles = std::move(alleles);
            kr.id = kv.id;
            kr.qs = qs;
            kr.type = (int8_t)type;
            recs.push_back(std::move(kr));
        }
        v.push_back(std::move(kv));
    }
    std::free(line);
    std::fclose(f);
    if (rc != NGSEP_OK) return rc;
    c->known_given = true;
    c->strs.clear();                                   // -knownSTRs are ignored with -knownVariants (findSNVS :897-912)
    std::stable_sort(v.begin(), v.end(), [](const ngsep_ctx::KnownVar& x, const ngsep_ctx::KnownVar& y) {
        if (x.seq != y.seq) return x.seq < y.seq;
        return x.pos != y.pos ? x.pos < y.pos : x.last < y.last;   // GenomicRegionPositionComparator
    });
    c->known.swap(v);
    c->known_recs.swap(recs);
    c->known_seq_begin.assign(c->seq_names.size() + 1, 0);
    for (const auto& kv : c->known) c->known_seq_begin[(size_t)kv.seq + 1]++;
    for (size_t i = 0; i < c->seq_names.size(); i++) c->known_seq_begin[i + 1] += c->known_seq_begin[i];
    // the realigner's input variants (every record: an SNV marks its position, SingleSampleVariantsDetector.java:904)
    if (!c->known.empty()) {
        c->strs.assign(c->seq_names.size(), {});
        for (size_t k = 0; k < c->known.size(); k++) {
            const ngsep_ctx::KnownVar& kv = c->known[k];
            StrVar sv{kv.pos, kv.last};
            sv.str = kv.type == 5;                     // GenomicVariant.TYPE_STR
            sv.event = kv.alt < 0;
            sv.known = kv.alt < 0 ? (int64_t)k : -1;
            sv.rec = kv.rec;
            c->strs[(size_t)kv.seq].v.push_back(sv);
        }
        for (InputVars& iv : c->strs) iv.finish();
    }
    return NGSEP_OK;
}

// the input variant of a -knownVariants record (nullptr: none).  Records are written in order, and at one position
// in the input order (stream_collect), so a record is the first input variant of its position and ALT that no
// earlier record there took.
const ngsep_ctx::KnownVar* ngsep::known_of(const ngsep_ctx* c, const ngsep_site_out& s) { return known_at(c, s.seq_id, s.pos, site_alt(s)); }

const ngsep_ctx::KnownVar* ngsep::known_at(const ngsep_ctx* c, int32_t seq_id, int32_t pos, int alt) {
    if (c->known.empty() || seq_id < 0 || (size_t)seq_id + 1 >= c->known_seq_begin.size()) return nullptr;
    auto& st = c->vcf_known;
    if (st.seq != seq_id || st.pos != pos) { st.seq = seq_id; st.pos = pos; st.taken.clear(); }
    const int64_t kb = c->known_seq_begin[(size_t)seq_id], ke = c->known_seq_begin[(size_t)seq_id + 1];
    auto it = std::lower_bound(c->known.begin() + kb, c->known.begin() + ke, (int64_t)pos,
                               [](const ngsep_ctx::KnownVar& v, int64_t p) { return v.pos < p; });
    for (int64_t k = it - c->known.begin(); k < ke && c->known[(size_t)k].pos == pos; k++)
        if (c->known[(size_t)k].alt == alt && std::find(st.taken.begin(), st.taken.end(), k) == st.taken.end()) {
            st.taken.push_back(k);
            return &c->known[(size_t)k];
        }
    return nullptr;
}

extern "C" int ngsep_fetch_rac(ngsep_ctx* c, double* prop, double* n_alleles, double* moments) {
    if (!c) return NGSEP_E_INVALID;
    if (!c->params.relative_allele_counts) return set_error(c, NGSEP_E_INVALID, "context not in relative-allele-counts mode");
    const auto& R = c->rac;
    if (prop) std::memcpy(prop, R.prop, sizeof R.prop);
    if (n_alleles) std::memcpy(n_alleles, R.nall, sizeof R.nall);
    if (moments) {
        moments[0] = R.prop_count; moments[1] = R.prop_sum; moments[2] = R.prop_sum_sq;
        moments[3] = R.nall_count; moments[4] = R.nall_sum; moments[5] = R.nall_sum_sq;
    }
    return NGSEP_OK;
}

extern "C" int ngsep_clear_rac(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    c->rac = {};
    return NGSEP_OK;
}

namespace {
// DecimalFormat("##0.0#") (main/io/ParseUtils.java:29): HALF_EVEN on the double's exact value
std::string java_fmt2(double x) {
    const double p = x * 100.0, err = std::fma(x, 100.0, -p);
    const double k = std::floor(p), fr = p - k;
    long long n = (long long)k;
    if (fr > 0.5 || (fr == 0.5 && (err > 0 || (err == 0 && (n & 1))))) n++;
    char b[64];
    if (n % 10 == 0) std::snprintf(b, sizeof b, "%lld.%lld", n / 100, (n % 100) / 10);
    else std::snprintf(b, sizeof b, "%lld.%02lld", n / 100, n % 100);
    return b;
}
// Distribution.printDistribution (math/Distribution.java:301-345) of a distribution with no outliers
void print_distribution(std::string& o, const double* dist, int nbins, double min, double bin, double max, bool integer,
                        double count, double sum, double sum_sq) {
    const int max_idx = (int)((max - min) / bin);
    for (int i = 0; i < nbins && i <= max_idx; i++) {
        if (integer) o += std::to_string((int)(min + i * bin)) + "\t" + std::to_string((long long)java_round(dist[i])) + "\n";
        else o += java_fmt2(min + i * bin) + "\t" + java_fmt2(dist[i]) + "\n";
    }
    o += "Count\t" + std::to_string((long long)java_round(count)) + "\n";
    if (integer) o += "Sum\t" + std::to_string((long long)java_round(sum)) + "\n";
    else o += "Sum\t" + java_fmt2(sum) + "\n";
    if (count > 0) o += "Average\t" + java_fmt2(sum / count) + "\n";
    if (count > 1) {
        const double var = (sum_sq - sum * sum / count) / (count - 1);
        o += "Variance\t" + java_fmt2(var) + "\n";
        o += "STDev\t" + java_fmt2(std::sqrt(var)) + "\n";
    }
}
}  // namespace

// RelativeAlleleCountsCalculator.printResults (discovery/RelativeAlleleCountsCalculator.java:213-244)
extern "C" int ngsep_write_rac(ngsep_ctx* c, const char* out_path) {
    if (!c || !out_path) return NGSEP_E_INVALID;
    if (!c->params.relative_allele_counts) return set_error(c, NGSEP_E_INVALID, "context not in relative-allele-counts mode");
    const auto& R = c->rac;
    std::string o;
    o += "Distribution of allele proportions\n";
    print_distribution(o, R.prop, 51, 0.0, 0.01, 0.5, false, R.prop_count, R.prop_sum, R.prop_sum_sq);
    o += "Distribution of number of alleles\n";
    print_distribution(o, R.nall, 10, 1.0, 1.0, 10.0, true, R.nall_count, R.nall_sum, R.nall_sum_sq);
    if (!R.seq_names.empty()) {
        o += "Distribution of allele proportions per sequence\nProportion";
        for (const auto& n : R.seq_names) o += "\t" + n;
        o += "\n";
        double min = 0;
        for (int b = 0; b < 51; b++) {
            o += java_fmt2(min);
            for (const auto& d : R.seq_prop) o += "\t" + java_fmt2(d[(size_t)b]);
            o += "\n";
            min += 0.01;
        }
    }
    std::FILE* f = std::strcmp(out_path, "-") == 0 ? stdout : std::fopen(out_path, "w");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot write ") + out_path);
    std::fwrite(o.data(), 1, o.size(), f);
    if (f != stdout) std::fclose(f);
    else std::fflush(f);
    return NGSEP_OK;
}

extern "C" int ngsep_fetch_carved_regions(ngsep_ctx* c, int32_t* seq_id, int64_t* first, int64_t* last, int64_t cap,
                                          int64_t* n_out) {
    if (!c) return NGSEP_E_INVALID;
    const int64_t n = (int64_t)c->carved.size();
    if (n_out) *n_out = n;
    for (int64_t i = 0; i < std::min(n, cap); i++) {
        if (seq_id) seq_id[i] = c->carved[(size_t)i].first;
        if (first) first[i] = c->carved[(size_t)i].second.first;
        if (last) last[i] = c->carved[(size_t)i].second.second;
    }
    return NGSEP_OK;
}

extern "C" int ngsep_clear_carved_regions(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    c->carved.clear();
    return NGSEP_OK;
}

extern "C" int ngsep_stage_alignments(ngsep_ctx* c, const ngsep_read_batch* b) {
    if (!c) return NGSEP_E_INVALID;
    c->staging_mode = true;
    return process_batch(c, b, false);
}

extern "C" int ngsep_stage_finish(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    c->staging_mode = true;
    int rc = flush_sequence(c);
    if (rc != NGSEP_OK) return rc;
    if (c->params.relative_allele_counts || !c->known.empty()) {
        c->staged_contigs.clear();
        return set_error(c, NGSEP_E_UNSUPPORTED, "relative allele counts and known-variant genotyping run on the streaming paths "
                                                 "(ngsep_process_alignments / ngsep_call_bam / ngsep_rac_bam)");
    }
    rc = c->params.coverage_stats ? coverage_stage(c, c->staged_contigs) : build_and_upload(c, c->staged_contigs, true);
    c->staged_contigs.clear();
    return rc;
}

extern "C" int ngsep_run_staged(ngsep_ctx* c, double* elapsed_ms) {
    if (c && c->params.coverage_stats) {
        const int rc = coverage_run(c, nullptr);
        if (rc == NGSEP_OK && elapsed_ms) *elapsed_ms = c->stats.kernel_ms;
        return rc;
    }
    if (!c || !c->dev) return set_error(c, NGSEP_E_INVALID, "nothing staged");
    c->sites.clear();
    c->pop_sites.clear();
    c->pop_calls.clear();
    c->pop_big.clear();
    c->pop_order.clear();
    c->pop_text.clear();
    c->stats.sites_called = 0;
    return run_device(c, elapsed_ms);
}

// asynchronous staged runs: submit enqueues one pass (kernels + copies) and returns; collect waits for
// the oldest submitted pass and makes its calls the context's result.  At most two passes in flight,
// so the D2H and host work of one pass overlap the next pass's kernels.
extern "C" int ngsep_submit_staged(ngsep_ctx* c) {
    if (c && c->params.coverage_stats) return set_error(c, NGSEP_E_INVALID, "coverage runs are synchronous: ngsep_run_staged");
    if (!c || !c->dev) return set_error(c, NGSEP_E_INVALID, "nothing staged");
    if (c->params.multisample) {
        // population runs: kernels of one pass while the previous pass's calls are gathered and copied back; the
        // tables depend only on the options (computed once per option set)
        if (!c->tables_cached || std::memcmp(&c->tables_params, &c->params, sizeof(ngsep_params)) != 0 ||
            c->tables_het != c->het_rate) {
            compute_tables(c, &c->tables_t, &c->tables_gp);
            c->tables_params = c->params;
            c->tables_het = c->het_rate;
            c->tables_cached = true;
        }
        const LikTables& t = c->tables_t;
        const GenotypeParams& gp = c->tables_gp;
        if (const int rc = prepare_pool(c)) return rc;
        std::string err;
        if (device_submit_multi(c->dev, t, gp, (int32_t)c->sample_ids.size(), c->params.min_allele_depth_freq,
                                c->params.ploidy, err) != 0)
            return set_error(c, NGSEP_E_DEVICE, err);
        return NGSEP_OK;
    }
    if (device_inflight(c->dev) >= 2) return set_error(c, NGSEP_E_INVALID, "two staged runs already in flight: collect first");
    // the tables depend only on the options: computed once per option set
    if (!c->tables_cached || std::memcmp(&c->tables_params, &c->params, sizeof(ngsep_params)) != 0 ||
        c->tables_het != c->het_rate) {
        compute_tables(c, &c->tables_t, &c->tables_gp);
        c->tables_params = c->params;
        c->tables_het = c->het_rate;
        c->tables_cached = true;
    }
    const LikTables& t = c->tables_t;
    const GenotypeParams& gp = c->tables_gp;
    if (const int rc = prepare_pool(c)) return rc;
    const int prune = c->params.prune_candidates && !c->params.dump_all_positions && (c->het_rate <= 0.1 || c->params.ploidy >= 3);
    std::string err;
    if (device_submit(c->dev, c->staged, t, gp, prune, err) != 0) return set_error(c, NGSEP_E_DEVICE, err);
    return NGSEP_OK;
}

extern "C" int ngsep_collect_staged(ngsep_ctx* c, double* elapsed_ms) {
    if (!c || !c->dev) return set_error(c, NGSEP_E_INVALID, "nothing staged");
    if (c->params.multisample) {
        c->pop_sites.clear();
        c->pop_calls.clear();
        c->pop_big.clear();
        c->pop_order.clear();
        c->pop_text.clear();
        c->stats.sites_called = 0;
        const ngsep_popsite_out* sites = nullptr;
        int64_t n = 0, ncand = 0;
        int slot = 0;
        bool rerun = false;
        double scan_ms = 0, geno_ms = 0;
        std::string err;
        const auto t0 = std::chrono::steady_clock::now();
        if (device_collect_multi(c->dev, &sites, &n, &slot, &rerun, &scan_ms, &geno_ms, &ncand, err) != 0)
            return set_error(c, NGSEP_E_DEVICE, err);
        if (rerun) return run_device(c, elapsed_ms);    // a buffer overflowed: the pass again, synchronously (grows them)
        const auto t1 = std::chrono::steady_clock::now();
        // the slot's calls came back packed in KPM's site order: its buffers become the call store (swapped, not
        // copied) and pop_order maps the ordered sites to their blocks
        const int rc = order_population_sites(c, sites, n, [&](const int64_t* src, int64_t m, std::string&) {
            device_slot_take(c->dev, slot, n, c->pop_calls, c->pop_big);
            c->pop_order.assign(src, src + m);
            return 0;
        });
        if (rc != NGSEP_OK) return rc;
        c->stats.candidates = ncand;
        c->stats.hard_sites = (int32_t)device_last_hard(c->dev);
        c->stats.exact_bound_passes = device_last_exact(c->dev);
        c->stats.scan_ms = scan_ms;
        c->stats.genotype_ms = geno_ms;
        c->stats.kernel_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        if (elapsed_ms) *elapsed_ms = c->stats.kernel_ms;
        static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
        if (host_timing) {
            static double acc_w = 0, acc_f = 0;
            static int cnt = 0;
            acc_w += std::chrono::duration<double, std::micro>(t1 - t0).count();
            acc_f += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
            if (++cnt == 8) {
                std::fprintf(stderr, "[ngsep host] population collect: wait %.1f us, order + gather + D2H %.1f us (avg of 8)\n", acc_w / 8, acc_f / 8);
                acc_w = acc_f = 0;
                cnt = 0;
            }
        }
        return NGSEP_OK;
    }
    c->sites.clear();
    c->stats.sites_called = 0;
    int64_t n = 0, ncand = 0;
    double scan_ms = 0, geno_ms = 0, total_ms = 0;
    std::string err;
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto h0 = std::chrono::steady_clock::now();
    if (device_collect(c->dev, &c->sites, &n, &scan_ms, &geno_ms, &total_ms, &ncand, err) != 0)
        return set_error(c, NGSEP_E_DEVICE, err);
    const auto h1 = std::chrono::steady_clock::now();
    const int rc = finish_run(c, 0, n, scan_ms, geno_ms, total_ms, ncand, elapsed_ms);
    if (host_timing) {
        static double acc_c = 0, acc_f = 0;
        static int cnt = 0;
        acc_c += std::chrono::duration<double, std::micro>(h1 - h0).count();
        acc_f += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h1).count();
        if (++cnt == 20) {
            std::fprintf(stderr, "[ngsep host] collect: device_collect %.1f us, finish_run %.1f us (avg of 20)\n", acc_c / 20, acc_f / 20);
            acc_c = acc_f = 0;
            cnt = 0;
        }
    }
    return rc;
}

extern "C" int ngsep_release_staged(ngsep_ctx* c) {
    if (!c) return NGSEP_E_INVALID;
    if (c->dev) device_release(c->dev);
    if (c->cov_dev) cov_release(c->cov_dev);
    c->cov_staged = false;
    c->staged = Staged();
    return NGSEP_OK;
}

// ---- MultisampleVariantsDetector entry points ----
extern "C" int ngsep_set_samples(ngsep_ctx* c, int32_t n_samples, const char* const* sample_ids,
                                 int32_t n_read_groups, const int32_t* rg_sample, const int32_t* rg_rank) {
    if (!c || n_samples < 0 || n_read_groups < 0 || (n_samples && !sample_ids) || (n_read_groups && (!rg_sample || !rg_rank)))
        return set_error(c, NGSEP_E_INVALID, "bad sample description");
    if (n_samples > kMaxSamplesDevice)
        return set_error(c, NGSEP_E_UNSUPPORTED, "more than " + std::to_string(kMaxSamplesDevice) + " samples per device run");
    c->sample_ids.clear();
    for (int32_t i = 0; i < n_samples; i++) c->sample_ids.emplace_back(sample_ids[i] ? sample_ids[i] : "");
    c->rg_sample.assign(rg_sample, rg_sample + n_read_groups);
    c->rg_rank.assign(rg_rank, rg_rank + n_read_groups);
    c->sample_nrank.assign((size_t)n_samples, 0);
    for (int32_t g = 0; g < n_read_groups; g++) {
        const int32_t sm = rg_sample[g];
        if (sm < -1 || sm >= n_samples) return set_error(c, NGSEP_E_INVALID, "read group mapped to an unknown sample");
        if (sm >= 0) {
            if (rg_rank[g] < 0 || rg_rank[g] > 126) return set_error(c, NGSEP_E_INVALID, "read group rank out of range");
            c->sample_nrank[(size_t)sm] = (int8_t)std::max<int>(c->sample_nrank[(size_t)sm], rg_rank[g] + 1);
        }
    }
    return NGSEP_OK;
}

extern "C" int ngsep_fetch_population_sites(ngsep_ctx* c, ngsep_popsite_out* sites, ngsep_sample_call* calls,
                                            int64_t cap, int64_t* n_out) {
    if (!c || !n_out) return NGSEP_E_INVALID;
    const int64_t n = (int64_t)c->pop_sites.size();
    *n_out = n;
    const size_t S = c->sample_ids.size();
    const int64_t k = std::min<int64_t>(n, std::max<int64_t>(cap, 0));
    if (sites && k) std::memcpy(sites, c->pop_sites.data(), (size_t)k * sizeof(ngsep_popsite_out));
    if (calls && k && S)
        for (size_t i = 0; i < (size_t)k; i++)
            for (size_t j = 0; j < S; j++) {
                if (c->pop_sites[i].multisnv_type == 3) {     // an indel / STR record: ngsep_population_site_vcf_line
                    std::memset(&calls[i * S + j], 0, sizeof(ngsep_sample_call));
                    continue;
                }
                calls[i * S + j] = expand_call(c->pop_calls.data()[(size_t)c->pop_order[i] * S + j], c->pop_big.data());
            }
    return NGSEP_OK;
}
