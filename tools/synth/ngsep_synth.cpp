// ngsep_synth.cpp -- seeded synthetic FASTA / SAM / BAM (+BAI) / truth for tests and bench.py.
// Test/bench data infrastructure; the product never links it.
//
// Records are kept as a structure of arrays (one entry per BAM record, the bases and qualities in two
// shared byte arrays; PCR-duplicate and secondary copies share their original's bytes), so a human
// chromosome at 30x fits in a few GB.  The BAM writer deflates its BGZF blocks on all cores and writes
// a BAI index (SAM spec section 5) next to the file.
#include "ngsep_synth.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Rng {  // xoshiro256** seeded by splitmix64
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        for (int i = 0; i < 4; i++) {
            seed += 0x9E3779B97F4A7C15ull;
            uint64_t z = seed;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            s[i] = z ^ (z >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

struct ContigDef { const char* name; int64_t len; };
const ContigDef kYeast[] = {
    {"chrI", 230218}, {"chrII", 813184}, {"chrIII", 316620}, {"chrIV", 1531933}, {"chrV", 576874},
    {"chrVI", 270161}, {"chrVII", 1090940}, {"chrVIII", 562643}, {"chrIX", 439888}, {"chrX", 745751},
    {"chrXI", 666816}, {"chrXII", 1078177}, {"chrXIII", 924431}, {"chrXIV", 784333}, {"chrXV", 1091291},
    {"chrXVI", 948066}, {"chrM", 85779}};
const ContigDef kHuman[] = {
    {"chr1", 248956422}, {"chr2", 242193529}, {"chr3", 198295559}, {"chr4", 190214555}, {"chr5", 181538259},
    {"chr6", 170805979}, {"chr7", 159345973}, {"chr8", 145138636}, {"chr9", 138394717}, {"chr10", 133797422},
    {"chr11", 135086622}, {"chr12", 133275309}, {"chr13", 114364328}, {"chr14", 107043718}, {"chr15", 101991189},
    {"chr16", 90338345}, {"chr17", 83257441}, {"chr18", 80373285}, {"chr19", 58617616}, {"chr20", 64444167},
    {"chr21", 46709983}, {"chr22", 50818468}, {"chrX", 156040895}, {"chrY", 57227415}};

const char kBases[] = "ACGT";
const char kOps[] = "HDIMPNSX";           // NGSEP op codes (ReadAlignment.java:60-67) -> SAM letters

// error probability of a phred score, 10^(-q/10), tabulated once (the same doubles std::pow returns)
const double* err_table() {
    static double t[94];
    static bool init = [] { for (int q = 0; q < 94; q++) t[q] = std::pow(10.0, -q / 10.0); return true; }();
    (void)init;
    return t;
}

struct Snv { int32_t contig, pos; char ref, alt; int gt; };  // gt 1 het, 2 hom

// every record in BAM order (incl. those the reader filters)
struct Records {
    std::vector<int32_t> contig, pos, flags, mapq, sample, cig_n, seq_len;
    std::vector<int64_t> readno, cig_off, seq_off;
    std::vector<uint8_t> suffix, hasq;     // name suffix 0 / 'd' (PCR duplicate) / 's' (secondary)
    std::vector<int32_t> cigar;            // NGSEP codes len*8+op
    std::string bases, quals;              // quals are '!' for a record without qualities
    size_t size() const { return pos.size(); }
    void push(int32_t c, int32_t p, int32_t fl, int32_t mq, int32_t sm, int64_t no, uint8_t sfx, int64_t coff, int32_t cn,
              int64_t soff, int32_t sl, uint8_t hq) {
        contig.push_back(c); pos.push_back(p); flags.push_back(fl); mapq.push_back(mq); sample.push_back(sm);
        readno.push_back(no); suffix.push_back(sfx); cig_off.push_back(coff); cig_n.push_back(cn);
        seq_off.push_back(soff); seq_len.push_back(sl); hasq.push_back(hq);
    }
    // records [from, size()) reordered by idx (relative to from)
    void permute(size_t from, const std::vector<size_t>& idx) {
        auto perm = [&](auto& v) {
            using V = typename std::decay<decltype(v)>::type;
            V tmp(idx.size());
            for (size_t i = 0; i < idx.size(); i++) tmp[i] = v[from + idx[i]];
            std::copy(tmp.begin(), tmp.end(), v.begin() + (ptrdiff_t)from);
        };
        perm(contig); perm(pos); perm(flags); perm(mapq); perm(sample); perm(cig_n); perm(seq_len);
        perm(readno); perm(cig_off); perm(seq_off); perm(suffix); perm(hasq);
    }
};

}  // namespace

struct ngs_synth {
    ngs_synth_params p;
    std::vector<std::string> names;
    std::vector<std::string> seqs;
    Records rec;
    std::vector<Snv> truth;
    // batch view (reader-filtered records; bases/quals/cigar point into rec's arrays)
    std::vector<int32_t> b_seq, b_first, b_flags, b_rg, b_cig_n, b_seqlen;
    std::vector<int64_t> b_cig_off, b_seq_off;
    std::vector<uint8_t> b_hasq;
};

extern "C" void ngs_synth_default(ngs_synth_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->genome = NGS_GENOME_YEAST;
    p->n_contigs = 0;
    p->depth = 30;
    p->read_len = 150;
    p->seed = 2;
    p->snv_rate = 1e-3;
    p->dup_rate = 0.002;
    p->n_frac = 0.001;
}

static int sample_quality(Rng& r, int model) {
    if (model == 1) return 30;
    if (model == 2) return (int)r.below(41);
    double u = r.uniform();
    if (u < 0.02) return 2;
    if (u < 0.05) return 12;
    if (u < 0.15) return 25;
    if (u < 0.50) return 33;
    return 37;
}

static void make_population(ngs_synth* s);
static void make_batch(ngs_synth* s);
// extra reads of a collapsed repeat (hot_depth > 0) on a contig of length L, per sample
static int64_t hot_reads(const ngs_synth_params& p, int64_t L) {
    if (p.hot_depth <= 0 || p.hot_len < p.read_len || p.hot_first < 1 || p.hot_first + p.hot_len - 1 > L) return 0;
    return (int64_t)std::llround(p.hot_depth * (double)p.hot_len / p.read_len);
}

// the kept contigs of the genome table, optionally truncated (trunc_len)
static std::vector<ContigDef> kept_contigs(const ngs_synth_params& p, int* first_out, double* pa) {
    std::vector<ContigDef> defs;
    *pa = 0.31;  // P(A)=P(T)
    if (p.genome == NGS_GENOME_YEAST) defs.assign(std::begin(kYeast), std::end(kYeast));
    else if (p.genome == NGS_GENOME_HUMAN) { defs.assign(std::begin(kHuman), std::end(kHuman)); *pa = 0.295; }
    else defs.push_back({"chrS", p.custom_len});
    int first = std::max(0, p.contig_first);
    first = std::min<int>(first, (int)defs.size());
    int n = p.n_contigs > 0 ? std::min<int>(p.n_contigs, (int)defs.size() - first) : (int)defs.size() - first;
    std::vector<ContigDef> keep(defs.begin() + first, defs.begin() + first + n);
    if (p.trunc_len > 0)
        for (auto& d : keep) d.len = std::min<int64_t>(d.len, p.trunc_len);
    *first_out = first;
    return keep;
}

// reference, seed 0x4E475345 + contig index
static std::string make_reference(const ngs_synth_params& p, int contig_index, int64_t len, double pa) {
    Rng r(0x4E475345ull + (uint64_t)contig_index + (p.seed << 32));
    std::string seq((size_t)len, 'A');
    for (int64_t i = 0; i < len; i++) {
        double u = r.uniform();
        char b = u < pa ? 'A' : u < 0.5 ? 'C' : u < 1.0 - pa ? 'G' : 'T';
        if (p.lower_frac > 0 && r.uniform() < p.lower_frac) b = (char)(b - 'A' + 'a');
        seq[(size_t)i] = b;
    }
    return seq;
}

// one simulated read (and whether it gets a PCR-duplicate / secondary copy): haplotype, strand, MAPQ,
// bases with substitution errors at their phred probability and N at Q2, optional soft clip, missing
// qualities.  The order of draws from r is the generator's data contract (golden fixtures pin it).
struct GenOut { int32_t pos, flags, mapq, cn; uint8_t hq; bool dup, sec; };
static GenOut gen_read(Rng& r, const ngs_synth_params& p, const std::string& h0, const std::string& h1, int64_t L,
                       int32_t pos, const double* et, char* bases, char* quals, int32_t* cig) {
    GenOut o{};
    const int rl = p.read_len;
    const std::string& hap = r.below(2) ? h1 : h0;
    o.flags = r.below(2) ? 16 : 0;
    o.mapq = (p.lowmq_rate > 0 && r.uniform() < p.lowmq_rate) ? 5 : 60;
    for (int i = 0; i < rl; i++) {
        char b = hap[pos - 1 + i];
        int q = sample_quality(r, p.quality_model);
        if (r.uniform() < et[q]) {
            int bi = (int)(std::strchr(kBases, b) - kBases);
            b = kBases[(bi + 1 + (int)r.below(3)) % 4];
        }
        if (p.n_frac > 0 && r.uniform() < p.n_frac) { b = 'N'; q = 2; }
        bases[i] = b;
        quals[i] = (char)(33 + q);
    }
    int clip = 0, clip_end = 0;
    if (p.softclip_rate > 0 && r.uniform() < p.softclip_rate) { clip = 5 + (int)r.below(16); clip_end = (int)r.below(2); }
    if (clip && clip_end) {          // soft clip keeps the read characters
        cig[0] = (rl - clip) * 8 + 3;
        cig[1] = clip * 8 + 6;
        o.cn = 2;
    } else if (clip && pos + clip + (rl - clip) - 1 <= L) {   // a leading clip shifts the aligned start
        cig[0] = clip * 8 + 6;
        cig[1] = (rl - clip) * 8 + 3;
        o.cn = 2;
        pos += clip;
    } else {
        cig[0] = rl * 8 + 3;
        o.cn = 1;
    }
    o.hq = 1;
    if (p.noqual_rate > 0 && r.uniform() < p.noqual_rate) {
        o.hq = 0;
        std::memset(quals, '!', (size_t)rl);
    }
    o.dup = p.dup_rate > 0 && r.uniform() < p.dup_rate;
    o.sec = p.secondary_rate > 0 && r.uniform() < p.secondary_rate;
    o.pos = pos;
    return o;
}

// a donor indel: `len` bases inserted after the position, or `len` reference bases deleted from it
struct Indel { bool ins = false; int len = 0; std::string seq; };
typedef std::map<int32_t, Indel> IndelMap;
constexpr int kIndelCigar = 16;

// one read on a haplotype with indels: the read walks the donor haplotype from reference position pos and
// its CIGAR records the alignment (M runs, I for inserted bases, D for deleted reference bases); a read
// never starts with a deletion nor ends inside an insertion.  Same error/quality model as gen_read.
static GenOut gen_read_indel(Rng& r, const ngs_synth_params& p, const std::string& h0, const std::string& h1,
                             const IndelMap* ev, int64_t L, int32_t pos, const double* et, char* bases, char* quals,
                             int32_t* cig) {
    GenOut o{};
    const int rl = p.read_len;
    const int hp = r.below(2) ? 1 : 0;
    const std::string& hap = hp ? h1 : h0;
    const IndelMap& m = ev[hp];
    o.flags = r.below(2) ? 16 : 0;
    o.mapq = (p.lowmq_rate > 0 && r.uniform() < p.lowmq_rate) ? 5 : 60;
    int n = 0, nc = 0, lastop = -1;
    auto op = [&](int code, int len) {
        if (len <= 0) return;
        if (nc > 0 && lastop == code) cig[nc - 1] += len * 8;
        else if (nc < kIndelCigar) { cig[nc++] = len * 8 + code; lastop = code; }
    };
    auto emit = [&](char b) {
        int q = sample_quality(r, p.quality_model);
        if (r.uniform() < et[q]) {
            const char* pb = std::strchr(kBases, b);
            b = kBases[((pb ? (int)(pb - kBases) : 0) + 1 + (int)r.below(3)) % 4];
        }
        if (p.n_frac > 0 && r.uniform() < p.n_frac) { b = 'N'; q = 2; }
        bases[n] = b;
        quals[n] = (char)(33 + q);
        n++;
    };
    int64_t i = pos;                                       // 1-based reference position
    {   // a deletion at the start: the read starts after it
        auto it = m.find((int32_t)i);
        if (it != m.end() && !it->second.ins) i += it->second.len;
    }
    o.pos = (int32_t)i;
    while (n < rl && i <= L) {
        auto it = m.find((int32_t)i);
        if (it != m.end() && !it->second.ins && n > 0) {   // deleted reference bases
            op(1, it->second.len);
            i += it->second.len;
            continue;
        }
        emit(hap[(size_t)(i - 1)]);
        op(3, 1);
        if (it != m.end() && it->second.ins && n + it->second.len < rl) {
            for (char b : it->second.seq) emit(b);
            op(2, it->second.len);
        }
        i++;
    }
    while (n < rl) {                                       // past the contig end: pad with reference-less M
        emit('N');
        op(3, 1);
    }
    o.cn = nc;
    o.hq = 1;
    if (p.noqual_rate > 0 && r.uniform() < p.noqual_rate) {
        o.hq = 0;
        std::memset(quals, '!', (size_t)rl);
    }
    o.dup = p.dup_rate > 0 && r.uniform() < p.dup_rate;
    o.sec = p.secondary_rate > 0 && r.uniform() < p.secondary_rate;
    return o;
}

extern "C" ngs_synth* ngs_synth_create(const ngs_synth_params* pp) {
    ngs_synth* s = new ngs_synth();
    s->p = *pp;
    const ngs_synth_params& p = s->p;
    if (p.n_samples > 1) {
        make_population(s);
        make_batch(s);
        return s;
    }
    double pa;
    int first;
    const std::vector<ContigDef> keep = kept_contigs(p, &first, &pa);
    for (size_t c = 0; c < keep.size(); c++) {
        s->names.push_back(keep[c].name);
        s->seqs.push_back(make_reference(p, first + (int)c, keep[c].len, pa));
    }
    const uint64_t base_seed = p.seed * 0x9E3779B97F4A7C15ull + 17 + (uint64_t)p.sample_idx * 7919;
    Rng r(base_seed);
    const double* et = err_table();
    Records& R = s->rec;
    int64_t readno = 0;
    for (size_t c = 0; c < s->seqs.size(); c++) {
        // rng_per_contig: every contig's donor and reads come from their own streams (reads in chunks,
        // generated in parallel), so one contig generated alone (a rank's shard of the genome) equals that
        // contig of the whole-genome run
        if (p.rng_per_contig) r = Rng(base_seed + 0x632BE59BD9B4E019ull * (uint64_t)(first + (int)c + 1));
        const std::string& ref = s->seqs[c];
        int64_t L = (int64_t)ref.size();
        // donor haplotypes
        std::string h0 = ref, h1 = ref;
        for (auto& ch : h0) ch = (char)std::toupper(ch);
        for (auto& ch : h1) ch = (char)std::toupper(ch);
        for (int64_t i = 0; i < L; i++) {
            if (r.uniform() < p.snv_rate) {
                char rb = h0[i];
                int ri = (int)(std::strchr(kBases, rb) - kBases);
                int ai = (ri + 1 + (int)r.below(3)) % 4;
                int gt = r.uniform() < 2.0 / 3.0 ? 1 : 2;
                if (gt == 2) { h0[i] = kBases[ai]; h1[i] = kBases[ai]; }
                else if (r.below(2)) h1[i] = kBases[ai];
                else h0[i] = kBases[ai];
                s->truth.push_back({(int32_t)c, (int32_t)(i + 1), rb, kBases[ai], gt});
            }
        }
        // donor indels (indel_rate > 0, SURVEY.md 8(d) second dataset): 1-10 bp insertions after or
        // deletions from a reference position, on one haplotype (2/3) or both; from their own stream so the
        // SNV donor above is the same with and without them
        IndelMap ev[2];
        if (p.indel_rate > 0) {
            Rng ri(base_seed ^ 0x5851F42D4C957F2Dull ^ (uint64_t)(first + (int)c + 1) * 0x9E3779B97F4A7C15ull);
            for (int64_t i = 10; i + 20 < L; i++) {
                if (ri.uniform() >= p.indel_rate) continue;
                Indel d;
                d.ins = ri.below(2) != 0;
                d.len = 1 + (int)ri.below(10);
                for (int k = 0; k < d.len; k++) d.seq.push_back(kBases[ri.below(4)]);
                const int gt = ri.uniform() < 2.0 / 3.0 ? 1 : 2;
                const int hap = (int)ri.below(2);
                if (gt == 2 || hap == 0) ev[0][(int32_t)(i + 1)] = d;
                if (gt == 2 || hap == 1) ev[1][(int32_t)(i + 1)] = d;
                i += d.len + 5;                                   // no overlapping events
            }
        }
        int rl = p.read_len;
        size_t cstart = R.size();
        if (L < rl) continue;
        int64_t nreads = (int64_t)std::llround(p.depth * (double)L / rl);
        struct Gen { int32_t pos; int64_t order; };
        std::vector<Gen> starts(nreads);
        for (int64_t k = 0; k < nreads; k++) starts[k] = {(int32_t)(1 + r.below((uint64_t)(L - rl + 1))), k};
        // a collapsed repeat (hot_depth > 0): extra reads inside [hot_first, hot_first + hot_len)
        const int64_t hot_n = hot_reads(p, L);
        for (int64_t k = 0; k < hot_n; k++)
            starts.push_back({(int32_t)(p.hot_first + (int64_t)r.below((uint64_t)(p.hot_len - rl + 1))), nreads + k});
        nreads += hot_n;
        std::sort(starts.begin(), starts.end(), [](const Gen& a, const Gen& b) { return a.pos != b.pos ? a.pos < b.pos : a.order < b.order; });
        // read k: bases/qualities at b0 + k*rl, CIGAR at c0 + 2k (<= 2 items)
        const int64_t b0 = (int64_t)R.bases.size(), c0 = (int64_t)R.cigar.size();
        R.bases.resize((size_t)(b0 + nreads * rl));
        R.quals.resize((size_t)(b0 + nreads * rl));
        const int64_t cs = p.indel_rate > 0 ? kIndelCigar : 2;   // CIGAR items per read slot
        R.cigar.resize((size_t)(c0 + cs * nreads));
        std::vector<GenOut> outs((size_t)nreads);
        auto gen = [&](Rng& rr, int64_t k) {
            if (p.indel_rate > 0)
                outs[(size_t)k] = gen_read_indel(rr, p, h0, h1, ev, L, starts[(size_t)k].pos, et, &R.bases[(size_t)(b0 + k * rl)],
                                                 &R.quals[(size_t)(b0 + k * rl)], &R.cigar[(size_t)(c0 + cs * k)]);
            else
                outs[(size_t)k] = gen_read(rr, p, h0, h1, L, starts[(size_t)k].pos, et, &R.bases[(size_t)(b0 + k * rl)],
                                           &R.quals[(size_t)(b0 + k * rl)], &R.cigar[(size_t)(c0 + 2 * k)]);
        };
        if (p.rng_per_contig) {
            // independent streams per chunk of 65536 reads: generated on all cores
            constexpr int64_t kChunk = 65536;
            const int64_t nchunk = (nreads + kChunk - 1) / kChunk;
            const uint64_t cseed = base_seed + 0x632BE59BD9B4E019ull * (uint64_t)(first + (int)c + 1);
            std::atomic<int64_t> next{0};
            auto work = [&]() {
                for (int64_t j; (j = next.fetch_add(1)) < nchunk;) {
                    Rng rr(cseed ^ (0xD1B54A32D192ED03ull * (uint64_t)(j + 1)));
                    for (int64_t k = j * kChunk; k < std::min(nreads, (j + 1) * kChunk); k++) gen(rr, k);
                }
            };
            std::vector<std::thread> th;
            const unsigned nt = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
            for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
            work();
            for (auto& t : th) t.join();
        } else {
            for (int64_t k = 0; k < nreads; k++) gen(r, k);
        }
        for (int64_t k = 0; k < nreads; k++) {
            const GenOut& o = outs[(size_t)k];
            const int64_t no = readno++, soff = b0 + k * rl, coff = c0 + cs * k;
            R.push((int32_t)c, o.pos, o.flags, o.mapq, 0, no, 0, coff, o.cn, soff, rl, o.hq);
            if (o.dup) R.push((int32_t)c, o.pos, o.flags, o.mapq, 0, no, 'd', coff, o.cn, soff, rl, o.hq);
            if (o.sec) R.push((int32_t)c, o.pos, o.flags | 0x100, o.mapq, 0, no, 's', coff, o.cn, soff, rl, o.hq);
        }
        // keep BAM coordinate order: records were generated sorted except soft-clipped starts
        std::vector<size_t> idx(R.size() - cstart);
        std::iota(idx.begin(), idx.end(), (size_t)0);
        std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return R.pos[cstart + a] < R.pos[cstart + b]; });
        bool sorted = true;
        for (size_t i = 0; i < idx.size() && sorted; i++) sorted = idx[i] == i;
        if (!sorted) R.permute(cstart, idx);
    }
    make_batch(s);
    return s;
}

// Population of n_samples diploid individuals (the multisample configuration):
// population SNVs at snv_rate with allele frequency U(0.02, 0.98), genotypes in Hardy-Weinberg
// proportions, depth/read model per sample as for one individual.  Records of all samples are
// merged in (position, sample) order -- AlignmentsPileupGenerator's multi-file merge
// (discovery/AlignmentsPileupGenerator.java:268-289: ties go to the lowest file index) of one
// BAM per sample with equal read lengths.
static void make_population(ngs_synth* s) {
    const ngs_synth_params& p = s->p;
    double pa;
    int first;
    const std::vector<ContigDef> keep = kept_contigs(p, &first, &pa);
    const int ns = p.n_samples;
    for (size_t c = 0; c < keep.size(); c++) {
        s->names.push_back(keep[c].name);
        s->seqs.push_back(make_reference(p, first + (int)c, keep[c].len, pa));
    }
    const uint64_t base_seed = p.seed * 0x9E3779B97F4A7C15ull + 31;
    Rng r(base_seed);
    const double* et = err_table();
    Records& R = s->rec;
    int64_t readno = 0;
    for (size_t c = 0; c < s->seqs.size(); c++) {
        if (p.rng_per_contig) r = Rng(base_seed + 0x632BE59BD9B4E019ull * (uint64_t)(first + (int)c + 1));
        const std::string& ref = s->seqs[c];
        const int64_t L = (int64_t)ref.size();
        // population variants: position, alt base, per-sample allele bits (bit0 hap0, bit1 hap1)
        std::vector<int32_t> vpos;
        std::vector<char> valt;
        std::vector<uint8_t> vgt;    // vpos.size() x ns
        for (int64_t i = 0; i < L; i++) {
            if (r.uniform() >= p.snv_rate) continue;
            char rb = (char)std::toupper(ref[i]);
            const char* pr = std::strchr(kBases, rb);
            if (!pr) continue;
            int ai = ((int)(pr - kBases) + 1 + (int)r.below(3)) % 4;
            double af = 0.02 + 0.96 * r.uniform();
            vpos.push_back((int32_t)(i + 1));
            valt.push_back(kBases[ai]);
            int carriers = 0;
            for (int k = 0; k < ns; k++) {
                uint8_t g = (uint8_t)((r.uniform() < af ? 1 : 0) | (r.uniform() < af ? 2 : 0));
                vgt.push_back(g);
                carriers += g != 0;
            }
            if (carriers) s->truth.push_back({(int32_t)c, (int32_t)(i + 1), rb, kBases[ai], 1});
        }
        // population indels (indel_rate > 0): 1-10 bp insertions / deletions from their own stream (the SNV population
        // above is the same with and without them), allele frequency U(0.05, 0.95), per-sample allele bits
        std::vector<int32_t> ipos;
        std::vector<Indel> iev;
        std::vector<uint8_t> igt;    // ipos.size() x ns
        if (p.indel_rate > 0) {
            Rng ri(base_seed ^ 0x5851F42D4C957F2Dull ^ (uint64_t)(first + (int)c + 1) * 0x9E3779B97F4A7C15ull);
            for (int64_t i = 10; i + 20 < L; i++) {
                if (ri.uniform() >= p.indel_rate) continue;
                Indel d;
                d.ins = ri.below(2) != 0;
                d.len = 1 + (int)ri.below(10);
                for (int k = 0; k < d.len; k++) d.seq.push_back(kBases[ri.below(4)]);
                const double af = 0.05 + 0.9 * ri.uniform();
                for (int k = 0; k < ns; k++) igt.push_back((uint8_t)((ri.uniform() < af ? 1 : 0) | (ri.uniform() < af ? 2 : 0)));
                ipos.push_back((int32_t)(i + 1));
                iev.push_back(d);
                i += d.len + 5;                                   // no overlapping events
            }
        }
        const int rl = p.read_len;
        if (L < rl) continue;
        const int64_t nper = (int64_t)std::llround(p.depth * (double)L / rl);
        struct Gen { int32_t pos; int32_t sample; int64_t order; };
        std::vector<Gen> starts;
        starts.reserve((size_t)(nper * ns));
        for (int k = 0; k < ns; k++)
            for (int64_t j = 0; j < nper; j++) starts.push_back({(int32_t)(1 + r.below((uint64_t)(L - rl + 1))), k, j});
        const int64_t hot_n = hot_reads(p, L);               // a collapsed repeat: every sample hot_depth deeper there
        for (int k = 0; k < ns; k++)
            for (int64_t j = 0; j < hot_n; j++)
                starts.push_back({(int32_t)(p.hot_first + (int64_t)r.below((uint64_t)(p.hot_len - rl + 1))), k, nper + j});
        std::sort(starts.begin(), starts.end(), [](const Gen& a, const Gen& b) {
            if (a.pos != b.pos) return a.pos < b.pos;
            if (a.sample != b.sample) return a.sample < b.sample;
            return a.order < b.order;
        });
        R.bases.reserve(R.bases.size() + starts.size() * (size_t)rl);
        R.quals.reserve(R.quals.size() + starts.size() * (size_t)rl);
        const size_t cstart = R.size();
        for (const Gen& g : starts) {
            const int hap = (int)r.below(2);
            const int32_t flags = r.below(2) ? 16 : 0;
            const int64_t soff = (int64_t)R.bases.size();
            if (p.indel_rate > 0) {
                // the read walks sample g.sample's haplotype `hap`: its SNVs and its indel events (gen_read_indel's walk)
                auto base_at = [&](int64_t pos) {
                    char b = (char)std::toupper(ref[(size_t)(pos - 1)]);
                    const size_t v = (size_t)(std::lower_bound(vpos.begin(), vpos.end(), (int32_t)pos) - vpos.begin());
                    if (v < vpos.size() && vpos[v] == pos && ((vgt[v * ns + g.sample] >> hap) & 1)) b = valt[v];
                    return b;
                };
                auto event_at = [&](int64_t pos) -> const Indel* {
                    const size_t v = (size_t)(std::lower_bound(ipos.begin(), ipos.end(), (int32_t)pos) - ipos.begin());
                    if (v < ipos.size() && ipos[v] == pos && ((igt[v * ns + g.sample] >> hap) & 1)) return &iev[v];
                    return nullptr;
                };
                const int64_t coff = (int64_t)R.cigar.size();
                int n = 0, nc = 0, lastop = -1;
                auto op = [&](int code, int len) {
                    if (len <= 0) return;
                    if (nc > 0 && lastop == code) R.cigar.back() += len * 8;
                    else if (nc < kIndelCigar) { R.cigar.push_back(len * 8 + code); nc++; lastop = code; }
                };
                auto emit = [&](char b) {
                    int q = sample_quality(r, p.quality_model);
                    if (r.uniform() < et[q]) {
                        const char* pb = std::strchr(kBases, b);
                        b = kBases[((pb ? (int)(pb - kBases) : 0) + 1 + (int)r.below(3)) % 4];
                    }
                    if (p.n_frac > 0 && r.uniform() < p.n_frac) { b = 'N'; q = 2; }
                    R.bases.push_back(b);
                    R.quals.push_back((char)(33 + q));
                    n++;
                };
                int64_t i = g.pos;
                if (const Indel* e = event_at(i)) if (!e->ins) i += e->len;     // a deletion at the start: the read starts after it
                const int32_t start = (int32_t)i;
                while (n < rl && i <= L) {
                    const Indel* e = event_at(i);
                    if (e && !e->ins && n > 0) { op(1, e->len); i += e->len; continue; }
                    emit(base_at(i));
                    op(3, 1);
                    if (e && e->ins && n + e->len < rl) {
                        for (char b : e->seq) emit(b);
                        op(2, e->len);
                    }
                    i++;
                }
                while (n < rl) { emit('N'); op(3, 1); }
                const bool dup = p.dup_rate > 0 && r.uniform() < p.dup_rate;
                const int64_t no = readno++;
                R.push((int32_t)c, start, flags, 60, g.sample, no, 0, coff, nc, soff, rl, 1);
                if (dup) R.push((int32_t)c, start, flags, 60, g.sample, no, 'd', coff, nc, soff, rl, 1);
                continue;
            }
            size_t vi = (size_t)(std::lower_bound(vpos.begin(), vpos.end(), g.pos) - vpos.begin());
            for (int i = 0; i < rl; i++) {
                const int32_t pos = g.pos + i;
                char b = (char)std::toupper(ref[pos - 1]);
                while (vi < vpos.size() && vpos[vi] < pos) vi++;
                if (vi < vpos.size() && vpos[vi] == pos && ((vgt[vi * ns + g.sample] >> hap) & 1)) b = valt[vi];
                int q = sample_quality(r, p.quality_model);
                if (r.uniform() < et[q]) {
                    const char* pb = std::strchr(kBases, b);
                    int bi = pb ? (int)(pb - kBases) : 0;
                    b = kBases[(bi + 1 + (int)r.below(3)) % 4];
                }
                if (p.n_frac > 0 && r.uniform() < p.n_frac) { b = 'N'; q = 2; }
                R.bases.push_back(b);
                R.quals.push_back((char)(33 + q));
            }
            const int64_t coff = (int64_t)R.cigar.size();
            R.cigar.push_back(rl * 8 + 3);
            const bool dup = p.dup_rate > 0 && r.uniform() < p.dup_rate;
            const int64_t no = readno++;
            R.push((int32_t)c, g.pos, flags, 60, g.sample, no, 0, coff, 1, soff, rl, 1);
            if (dup) R.push((int32_t)c, g.pos, flags, 60, g.sample, no, 'd', coff, 1, soff, rl, 1);
        }
        if (p.indel_rate > 0) {
            // a read that starts after a deletion moved: records in (first, last, sample) order, the order in which
            // AlignmentsPileupGenerator merges the per-sample files (GenomicRegionComparator, ties to the lowest
            // file index, :268-289), each sample's file sorted by (first, last)
            const size_t m = R.size() - cstart;
            std::vector<int32_t> last(m);
            for (size_t k = 0; k < m; k++) {
                int32_t span = 0;
                for (int32_t j = 0; j < R.cig_n[cstart + k]; j++) {
                    const int32_t v = R.cigar[(size_t)(R.cig_off[cstart + k] + j)];
                    if ((v & 7) == 3 || (v & 7) == 1) span += v / 8;
                }
                last[k] = R.pos[cstart + k] + span - 1;
            }
            std::vector<size_t> idx(m);
            std::iota(idx.begin(), idx.end(), (size_t)0);
            std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) {
                if (R.pos[cstart + a] != R.pos[cstart + b]) return R.pos[cstart + a] < R.pos[cstart + b];
                if (last[a] != last[b]) return last[a] < last[b];
                return R.sample[cstart + a] < R.sample[cstart + b];
            });
            R.permute(cstart, idx);
        }
    }
}

static void make_batch(ngs_synth* s) {
    // batch view: reader filters with default options (drop secondary and MAPQ<20 without NH)
    const Records& R = s->rec;
    for (size_t i = 0; i < R.size(); i++) {
        if (R.flags[i] & 0x100) continue;
        if (R.mapq[i] < 20) continue;
        s->b_seq.push_back(R.contig[i]);
        s->b_first.push_back(R.pos[i]);
        s->b_flags.push_back(R.flags[i]);
        s->b_rg.push_back(R.sample[i]);
        s->b_cig_off.push_back(R.cig_off[i]);
        s->b_cig_n.push_back(R.cig_n[i]);
        s->b_seq_off.push_back(R.seq_off[i]);
        s->b_seqlen.push_back(R.seq_len[i]);
        s->b_hasq.push_back(R.hasq[i]);
    }
}

extern "C" void ngs_synth_free(ngs_synth* s) { delete s; }
extern "C" int ngs_synth_n_contigs(const ngs_synth* s) { return (int)s->seqs.size(); }
extern "C" const char* ngs_synth_contig_name(const ngs_synth* s, int i) { return s->names[i].c_str(); }
extern "C" int64_t ngs_synth_contig_len(const ngs_synth* s, int i) { return (int64_t)s->seqs[i].size(); }
extern "C" const char* ngs_synth_contig_seq(const ngs_synth* s, int i) { return s->seqs[i].data(); }
extern "C" int64_t ngs_synth_n_reads(const ngs_synth* s) { return (int64_t)s->b_first.size(); }
extern "C" int64_t ngs_synth_n_bases(const ngs_synth* s) {
    int64_t n = 0;
    for (int32_t l : s->b_seqlen) n += l;
    return n;
}

extern "C" int ngs_synth_batch(ngs_synth* s, ngsep_read_batch* b) {
    b->n_reads = (int64_t)s->b_first.size();
    b->seq_id = s->b_seq.data();
    b->first = s->b_first.data();
    b->flags = s->b_flags.data();
    b->read_group = s->b_rg.data();
    b->cigar_off = s->b_cig_off.data();
    b->cigar_n = s->b_cig_n.data();
    b->cigar = s->rec.cigar.data();
    b->seq_off = s->b_seq_off.data();
    b->seq_len = s->b_seqlen.data();
    b->bases = s->rec.bases.data();
    b->quals = s->rec.quals.data();
    b->has_quals = s->b_hasq.data();
    return 0;
}

extern "C" int ngs_synth_write_fasta(const ngs_synth* s, const char* path) {
    FILE* f = std::fopen(path, "w");
    if (!f) return -1;
    for (size_t c = 0; c < s->seqs.size(); c++) {
        std::fprintf(f, ">%s\n", s->names[c].c_str());
        const std::string& q = s->seqs[c];
        for (size_t i = 0; i < q.size(); i += 60) {
            std::fwrite(q.data() + i, 1, std::min<size_t>(60, q.size() - i), f);
            std::fputc('\n', f);
        }
    }
    std::fclose(f);
    return 0;
}

static std::string header_text(const ngs_synth* s) {
    std::string h = "@HD\tVN:1.6\tSO:coordinate\n";
    for (size_t c = 0; c < s->seqs.size(); c++) h += "@SQ\tSN:" + s->names[c] + "\tLN:" + std::to_string(s->seqs[c].size()) + "\n";
    const int ns = s->p.n_samples > 1 ? s->p.n_samples : 1;
    for (int k = 0; k < ns; k++) {
        char rg[64];
        std::snprintf(rg, sizeof rg, "@RG\tID:S%03d\tSM:S%03d\n", s->p.sample_idx + k, s->p.sample_idx + k);
        h += rg;
    }
    return h;
}

static std::string read_name(const Records& R, size_t i) {
    char nm[40];
    int n = std::snprintf(nm, sizeof nm, "r%09lld", (long long)R.readno[i]);
    if (R.suffix[i]) nm[n++] = (char)R.suffix[i];
    return std::string(nm, (size_t)n);
}

extern "C" int ngs_synth_write_sam(const ngs_synth* s, const char* path) {
    FILE* f = std::fopen(path, "w");
    if (!f) return -1;
    std::string h = header_text(s);
    std::fwrite(h.data(), 1, h.size(), f);
    const Records& R = s->rec;
    std::string line;
    for (size_t i = 0; i < R.size(); i++) {
        std::string cig;
        for (int32_t k = 0; k < R.cig_n[i]; k++) {
            const int32_t v = R.cigar[(size_t)(R.cig_off[i] + k)];
            cig += std::to_string(v / 8);
            cig.push_back(kOps[v & 7]);
        }
        line = read_name(R, i);
        char mid[160];
        std::snprintf(mid, sizeof mid, "\t%d\t%s\t%d\t%d\t", R.flags[i], s->names[(size_t)R.contig[i]].c_str(), R.pos[i], R.mapq[i]);
        line += mid;
        line += cig;
        line += "\t*\t0\t0\t";
        line.append(R.bases, (size_t)R.seq_off[i], (size_t)R.seq_len[i]);
        line.push_back('\t');
        if (R.hasq[i]) line.append(R.quals, (size_t)R.seq_off[i], (size_t)R.seq_len[i]);
        else line.push_back('*');
        char rg[32];
        std::snprintf(rg, sizeof rg, "\tRG:Z:S%03d\n", s->p.sample_idx + R.sample[i]);
        line += rg;
        std::fwrite(line.data(), 1, line.size(), f);
    }
    std::fclose(f);
    return 0;
}

// ---- BGZF / BAM writer (SAM spec section 4) and BAI index (section 5) ----
namespace {
constexpr size_t kBlockData = 65280;     // uncompressed bytes per BGZF block

// Deflates 64 KB blocks of a stream on all cores, in order.  Records' uncompressed offsets map to
// virtual offsets (compressed block offset << 16 | offset in block) once their block is written.
struct Bgzf {
    FILE* f;
    std::string buf;                      // uncompressed bytes not yet written
    uint64_t written_u = 0;               // uncompressed bytes already handed to blocks
    uint64_t coff = 0;                    // compressed bytes written
    std::vector<uint64_t> block_coff;     // compressed offset of every block written
    explicit Bgzf(FILE* ff) : f(ff) {}
    uint64_t upos() const { return written_u + buf.size(); }
    // raw deflate of one block at level 6 (htslib's default): libdeflate when the image has it (dlopen,
    // ~3x zlib's speed), zlib otherwise
    struct Libdeflate {
        void* (*alloc)(int) = nullptr;
        size_t (*compress)(void*, const void*, size_t, void*, size_t) = nullptr;
        void (*release)(void*) = nullptr;
        Libdeflate() {
            void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
            if (!h) return;
            alloc = (void* (*)(int))dlsym(h, "libdeflate_alloc_compressor");
            compress = (size_t (*)(void*, const void*, size_t, void*, size_t))dlsym(h, "libdeflate_deflate_compress");
            release = (void (*)(void*))dlsym(h, "libdeflate_free_compressor");
            if (!alloc || !compress || !release) alloc = nullptr;
        }
    };
    static const Libdeflate& libdeflate() { static Libdeflate l; return l; }
    static void deflate_block(const char* data, size_t n, std::vector<unsigned char>& out) {
        out.assign(n + 1024, 0);
        size_t clen = 0;
        const Libdeflate& ld = libdeflate();
        // NGS_SYNTH_LEVEL: another compression level (0 = stored blocks: an inflate-free floor for the
        // end-to-end measurement)
        static const int level = std::getenv("NGS_SYNTH_LEVEL") ? std::atoi(std::getenv("NGS_SYNTH_LEVEL")) : 6;
        if (ld.alloc && !std::getenv("NGS_SYNTH_ZLIB")) {
            thread_local struct Cmp { void* c = nullptr; ~Cmp() { if (c) libdeflate().release(c); } } cmp;
            if (!cmp.c) cmp.c = ld.alloc(level);
            clen = ld.compress(cmp.c, data, n, out.data() + 18, out.size() - 26);
        }
        if (clen == 0) {
            z_stream z{};
            deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
            z.next_in = (Bytef*)data; z.avail_in = (uInt)n;
            z.next_out = out.data() + 18; z.avail_out = (uInt)(out.size() - 26);
            deflate(&z, Z_FINISH);
            clen = z.total_out;
            deflateEnd(&z);
        }
        unsigned char* h = out.data();
        const unsigned char hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0, 0, 0};
        std::memcpy(h, hdr, 18);
        uint16_t bsize = (uint16_t)(clen + 25);
        h[16] = bsize & 0xff; h[17] = bsize >> 8;
        uint32_t crc = (uint32_t)crc32(0, (const Bytef*)data, (uInt)n);
        unsigned char* t = out.data() + 18 + clen;
        for (int i = 0; i < 4; i++) t[i] = (crc >> (8 * i)) & 0xff;
        for (int i = 0; i < 4; i++) t[4 + i] = ((uint32_t)n >> (8 * i)) & 0xff;
        out.resize(18 + clen + 8);
    }
    // compresses and writes every complete block (all blocks when final)
    void flush(bool final) {
        size_t nb = buf.size() / kBlockData;
        if (final && buf.size() % kBlockData) nb++;
        if (nb == 0) return;
        std::vector<std::vector<unsigned char>> out(nb);
        std::atomic<size_t> next{0};
        const unsigned nt = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
        auto work = [&]() {
            for (size_t b; (b = next.fetch_add(1)) < nb;) {
                const size_t o = b * kBlockData;
                deflate_block(buf.data() + o, std::min(kBlockData, buf.size() - o), out[b]);
            }
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt && t < nb; t++) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
        size_t used = 0;
        for (size_t b = 0; b < nb; b++) {
            block_coff.push_back(coff);
            std::fwrite(out[b].data(), 1, out[b].size(), f);
            coff += out[b].size();
            used += std::min(kBlockData, buf.size() - b * kBlockData);
        }
        written_u += used;
        buf.erase(0, used);
    }
    void write(const void* d, size_t n) {
        buf.append((const char*)d, n);
        if (buf.size() >= 256 * kBlockData) flush(false);
    }
    void close() {
        flush(true);
        block_coff.push_back(coff);       // the EOF block: end offset of the last record
        static const unsigned char eof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        std::fwrite(eof, 1, 28, f);
    }
    // virtual offset of uncompressed position u (u <= total)
    uint64_t voff(uint64_t u) const {
        const size_t b = (size_t)(u / kBlockData);
        return (block_coff[b] << 16) | (u % kBlockData);
    }
};
int reg2bin(int beg, int end) {
    --end;
    if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
    if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
    if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
    if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
    if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
    return 0;
}
template <class T> void put(std::string& b, T v) { b.append((const char*)&v, sizeof(T)); }

// one indexed record: reference, [beg, end) 0-based, bin and its uncompressed [start, stop) in the stream
struct IdxRec { int32_t ref, beg, end, bin; uint64_t u0, u1; };

// BAI (SAM spec 5.2): per reference the bins' chunks (merged when contiguous in the file) and the
// 16 kb linear index (smallest virtual offset of a record overlapping each window)
void write_bai(const std::string& path, const Bgzf& z, const std::vector<IdxRec>& recs, int32_t n_ref) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return;
    std::string out = "BAI\1";
    put<int32_t>(out, n_ref);
    size_t i = 0;
    for (int32_t ref = 0; ref < n_ref; ref++) {
        size_t j = i;
        while (j < recs.size() && recs[j].ref == ref) j++;
        std::vector<std::pair<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>>> bins;
        std::vector<int> bin_slot(37450, -1);
        std::vector<uint64_t> lin;
        for (size_t k = i; k < j; k++) {
            const IdxRec& r = recs[k];
            const uint64_t v0 = z.voff(r.u0), v1 = z.voff(r.u1);
            int& sl = bin_slot[(size_t)r.bin];
            if (sl < 0) { sl = (int)bins.size(); bins.push_back({(uint32_t)r.bin, {}}); }
            auto& ch = bins[(size_t)sl].second;
            if (!ch.empty() && ch.back().second == v0) ch.back().second = v1;
            else ch.push_back({v0, v1});
            const int w0 = r.beg >> 14, w1 = (r.end - 1) >> 14;
            if ((int)lin.size() <= w1) lin.resize((size_t)w1 + 1, 0);
            for (int w = w0; w <= w1; w++)
                if (lin[(size_t)w] == 0 || v0 < lin[(size_t)w]) lin[(size_t)w] = v0;
        }
        for (size_t w = 1; w < lin.size(); w++)          // empty windows: the previous window's offset
            if (lin[w] == 0) lin[w] = lin[w - 1];
        put<int32_t>(out, (int32_t)bins.size());
        for (auto& b : bins) {
            put<uint32_t>(out, b.first);
            put<int32_t>(out, (int32_t)b.second.size());
            for (auto& c : b.second) { put<uint64_t>(out, c.first); put<uint64_t>(out, c.second); }
        }
        put<int32_t>(out, (int32_t)lin.size());
        for (uint64_t v : lin) put<uint64_t>(out, v);
        i = j;
    }
    std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
}
}  // namespace

static int write_bam_impl(const ngs_synth* s, const char* path, int only_sample);
extern "C" int ngs_synth_write_bam(const ngs_synth* s, const char* path) { return write_bam_impl(s, path, -1); }
// one sample's records (and only its @RG line): the per-sample BAM files a multisample run reads
extern "C" int ngs_synth_write_bam_sample(const ngs_synth* s, const char* path, int sample) { return write_bam_impl(s, path, sample); }

static int write_bam_impl(const ngs_synth* s, const char* path, int only_sample) {
    FILE* f = std::fopen(path, "wb");
    if (!f) return -1;
    Bgzf z(f);
    std::string h = header_text(s);
    if (only_sample >= 0) {
        std::string keep;
        char want[32];
        std::snprintf(want, sizeof want, "@RG\tID:S%03d\t", s->p.sample_idx + only_sample);
        size_t p0 = 0;
        while (p0 < h.size()) {
            size_t e = h.find('\n', p0);
            std::string line = h.substr(p0, e - p0 + 1);
            if (line.compare(0, 3, "@RG") != 0 || line.compare(0, std::strlen(want), want) == 0) keep += line;
            p0 = e + 1;
        }
        h = keep;
    }
    std::string b = "BAM\1";
    put<int32_t>(b, (int32_t)h.size());
    b += h;
    put<int32_t>(b, (int32_t)s->seqs.size());
    for (size_t c = 0; c < s->seqs.size(); c++) {
        put<int32_t>(b, (int32_t)s->names[c].size() + 1);
        b += s->names[c]; b.push_back(0);
        put<int32_t>(b, (int32_t)s->seqs[c].size());
    }
    z.write(b.data(), b.size());
    static const int bam_op[8] = {5, 2, 1, 0, 6, 3, 4, 8};  // NGSEP op -> BAM op (H D I M P N S X)
    const char* nt16 = "=ACMGRSVTWYHKDBN";
    int8_t code[256];
    std::memset(code, 15, sizeof code);
    for (int k = 0; k < 16; k++) code[(unsigned char)nt16[k]] = (int8_t)k;
    const Records& R = s->rec;
    std::vector<size_t> sel;                 // records written, in order
    sel.reserve(R.size());
    for (size_t i = 0; i < R.size(); i++)
        if (only_sample < 0 || R.sample[i] == only_sample) sel.push_back(i);
    auto name_len = [&](size_t i) -> size_t {
        size_t n = 10;                       // "r%09lld"
        for (long long v = R.readno[i]; v >= 1000000000LL; v /= 10) n++;
        return n + (R.suffix[i] ? 1 : 0);
    };
    // records are serialized in chunks, each chunk's records on all cores into one buffer
    std::vector<IdxRec> idx(sel.size());
    std::vector<uint64_t> roff;
    std::string chunk;
    const unsigned nt = std::max(1u, std::min<unsigned>(std::thread::hardware_concurrency(), 16u));
    constexpr size_t kRecChunk = 1 << 18;
    for (size_t c0 = 0; c0 < sel.size(); c0 += kRecChunk) {
        const size_t c1 = std::min(sel.size(), c0 + kRecChunk);
        roff.assign(c1 - c0 + 1, 0);
        for (size_t k = c0; k < c1; k++) {
            const size_t i = sel[k];
            roff[k - c0 + 1] = roff[k - c0] + 4 + 32 + name_len(i) + 1 + 4 * (size_t)R.cig_n[i] +
                               (size_t)(R.seq_len[i] + 1) / 2 + (size_t)R.seq_len[i] + 3 + 4 + 1;
        }
        chunk.resize(roff.back());
        const uint64_t u_base = z.upos();
        std::atomic<size_t> next{c0};
        auto work = [&]() {
            for (size_t k0; (k0 = next.fetch_add(4096)) < c1;) {
                for (size_t k = k0; k < std::min(c1, k0 + 4096); k++) {
                    const size_t i = sel[k];
                    char* o = &chunk[roff[k - c0]];
                    const int l_seq = R.seq_len[i];
                    const int32_t* cig = &R.cigar[(size_t)R.cig_off[i]];
                    int reflen = 0;
                    for (int32_t j = 0; j < R.cig_n[i]; j++) if ((cig[j] & 7) & 1) reflen += cig[j] / 8;
                    const int bin = reg2bin(R.pos[i] - 1, R.pos[i] - 1 + reflen);
                    const size_t nl = name_len(i);
                    auto w32 = [&](int32_t v) { std::memcpy(o, &v, 4); o += 4; };
                    auto w16 = [&](uint16_t v) { std::memcpy(o, &v, 2); o += 2; };
                    w32((int32_t)(roff[k - c0 + 1] - roff[k - c0] - 4));
                    w32(R.contig[i]);
                    w32(R.pos[i] - 1);
                    *o++ = (char)(uint8_t)(nl + 1);
                    *o++ = (char)(uint8_t)R.mapq[i];
                    w16((uint16_t)bin);
                    w16((uint16_t)R.cig_n[i]);
                    w16((uint16_t)R.flags[i]);
                    w32(l_seq);
                    w32(-1);
                    w32(-1);
                    w32(0);
                    char nm[40];
                    std::snprintf(nm, sizeof nm, "r%09lld", (long long)R.readno[i]);
                    std::memcpy(o, nm, nl - (R.suffix[i] ? 1 : 0));
                    o += nl - (R.suffix[i] ? 1 : 0);
                    if (R.suffix[i]) *o++ = (char)R.suffix[i];
                    *o++ = 0;
                    for (int32_t j = 0; j < R.cig_n[i]; j++) w32((int32_t)((uint32_t)(cig[j] / 8) << 4 | (uint32_t)bam_op[cig[j] & 7]));
                    const char* sq = R.bases.data() + R.seq_off[i];
                    const char* ql = R.quals.data() + R.seq_off[i];
                    for (int j = 0; j < l_seq; j += 2) {
                        const int hi = code[(unsigned char)sq[j]];
                        const int lo = j + 1 < l_seq ? code[(unsigned char)sq[j + 1]] : 0;
                        *o++ = (char)(uint8_t)(hi << 4 | lo);
                    }
                    if (R.hasq[i]) for (int j = 0; j < l_seq; j++) *o++ = (char)(uint8_t)(ql[j] - 33);
                    else { std::memset(o, 0xff, (size_t)l_seq); o += l_seq; }
                    char rg[16];
                    std::snprintf(rg, sizeof rg, "RGZS%03d", s->p.sample_idx + R.sample[i]);
                    std::memcpy(o, rg, 7);
                    o += 7;
                    *o++ = 0;
                    idx[k] = {R.contig[i], R.pos[i] - 1, R.pos[i] - 1 + std::max(reflen, 1), bin, u_base + roff[k - c0],
                              u_base + roff[k - c0 + 1]};
                }
            }
        };
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; t++) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
        z.write(chunk.data(), chunk.size());
    }
    z.close();
    std::fclose(f);
    write_bai(std::string(path) + ".bai", z, idx, (int32_t)s->seqs.size());
    return 0;
}

extern "C" int ngs_synth_write_truth(const ngs_synth* s, const char* path) {
    FILE* f = std::fopen(path, "w");
    if (!f) return -1;
    std::fprintf(f, "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\tTRUTH\n");
    for (const Snv& v : s->truth)
        std::fprintf(f, "%s\t%d\t.\t%c\t%c\t.\t.\t.\tGT\t%s\n", s->names[v.contig].c_str(), v.pos, v.ref, v.alt, v.gt == 2 ? "1/1" : "0/1");
    std::fclose(f);
    return 0;
}
// ---- SAM text -> BAM (for hand-written fixtures under tests/golden) ----
// Keeps the header text verbatim, all records in file order, and the aux tags of types
// A/i/f/Z (integers written as 'i').  Test infrastructure only.
extern "C" int ngs_sam_to_bam(const char* sam_path, const char* bam_path) {
    FILE* in = std::fopen(sam_path, "r");
    if (!in) return -1;
    std::string header;
    std::vector<std::string> names;
    std::vector<int32_t> lens;
    std::vector<std::string> lines;
    char* line = nullptr;
    size_t cap = 0;
    ssize_t got;
    while ((got = getline(&line, &cap, in)) > 0) {
        std::string l(line, got);
        while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
        if (l.empty()) continue;
        if (l[0] == '@') {
            header += l + "\n";
            if (l.compare(0, 3, "@SQ") == 0) {
                std::string sn;
                int32_t ln = 0;
                size_t p = 0;
                while ((p = l.find('\t', p)) != std::string::npos) {
                    ++p;
                    if (l.compare(p, 3, "SN:") == 0) sn = l.substr(p + 3, l.find('\t', p) - p - 3);
                    if (l.compare(p, 3, "LN:") == 0) ln = std::atoi(l.c_str() + p + 3);
                }
                names.push_back(sn);
                lens.push_back(ln);
            }
        } else {
            lines.push_back(l);
        }
    }
    std::free(line);
    std::fclose(in);
    FILE* f = std::fopen(bam_path, "wb");
    if (!f) return -1;
    Bgzf z(f);
    std::string b = "BAM\1";
    put<int32_t>(b, (int32_t)header.size());
    b += header;
    put<int32_t>(b, (int32_t)names.size());
    for (size_t c = 0; c < names.size(); c++) {
        put<int32_t>(b, (int32_t)names[c].size() + 1);
        b += names[c]; b.push_back(0);
        put<int32_t>(b, lens[c]);
    }
    z.write(b.data(), b.size());
    const char* nt16 = "=ACMGRSVTWYHKDBN";
    const char* ops = "MIDNSHP=X";
    for (const std::string& l : lines) {
        std::vector<std::string> fl;
        size_t p = 0, q;
        while ((q = l.find('\t', p)) != std::string::npos) { fl.push_back(l.substr(p, q - p)); p = q + 1; }
        fl.push_back(l.substr(p));
        if (fl.size() < 11) { std::fclose(f); return -2; }
        int32_t ref = -1;
        for (size_t c = 0; c < names.size(); c++) if (names[c] == fl[2]) ref = (int32_t)c;
        int32_t pos = std::atoi(fl[3].c_str()) - 1;
        std::vector<uint32_t> cig;
        int reflen = 0;
        if (fl[5] != "*") {
            int n = 0;
            for (char ch : fl[5]) {
                if (ch >= '0' && ch <= '9') { n = n * 10 + (ch - '0'); continue; }
                const char* o = std::strchr(ops, ch);
                if (!o) { std::fclose(f); return -2; }
                int op = (int)(o - ops);
                cig.push_back((uint32_t)n << 4 | (uint32_t)op);
                if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) reflen += n;
                n = 0;
            }
        }
        std::string seq = fl[9] == "*" ? "" : fl[9];
        std::string r;
        put<int32_t>(r, ref);
        put<int32_t>(r, pos);
        put<uint8_t>(r, (uint8_t)(fl[0].size() + 1));
        put<uint8_t>(r, (uint8_t)std::atoi(fl[4].c_str()));
        put<uint16_t>(r, (uint16_t)reg2bin(pos < 0 ? 0 : pos, (pos < 0 ? 0 : pos) + (reflen ? reflen : 1)));
        put<uint16_t>(r, (uint16_t)cig.size());
        put<uint16_t>(r, (uint16_t)std::atoi(fl[1].c_str()));
        put<int32_t>(r, (int32_t)seq.size());
        put<int32_t>(r, -1);
        put<int32_t>(r, -1);
        put<int32_t>(r, 0);
        r += fl[0]; r.push_back(0);
        for (uint32_t v : cig) put<uint32_t>(r, v);
        for (size_t i = 0; i < seq.size(); i += 2) {
            const char* hi = std::strchr(nt16, std::toupper((unsigned char)seq[i]));
            const char* lo = i + 1 < seq.size() ? std::strchr(nt16, std::toupper((unsigned char)seq[i + 1])) : nt16;
            put<uint8_t>(r, (uint8_t)((hi ? hi - nt16 : 15) << 4 | (lo ? lo - nt16 : 15)));
        }
        for (size_t i = 0; i < seq.size(); i++)
            put<uint8_t>(r, fl[10] == "*" ? 0xff : (uint8_t)(fl[10][i] - 33));
        for (size_t t = 11; t < fl.size(); t++) {
            const std::string& tg = fl[t];
            if (tg.size() < 5) continue;
            r += tg.substr(0, 2);
            char ty = tg[3];
            std::string v = tg.substr(5);
            if (ty == 'i') { r.push_back('i'); put<int32_t>(r, std::atoi(v.c_str())); }
            else if (ty == 'f') { r.push_back('f'); put<float>(r, std::strtof(v.c_str(), nullptr)); }
            else if (ty == 'A') { r.push_back('A'); r.push_back(v.empty() ? ' ' : v[0]); }
            else { r.push_back('Z'); r += v; r.push_back(0); }
        }
        std::string rec;
        put<int32_t>(rec, (int32_t)r.size());
        rec += r;
        z.write(rec.data(), rec.size());
    }
    z.close();
    std::fclose(f);
    return 0;
}
