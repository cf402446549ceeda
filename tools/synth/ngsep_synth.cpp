// ngsep_synth.cpp -- seeded synthetic FASTA / SAM / BAM / truth for tests and bench.py.
// Test/bench data infrastructure; the product never links it.
#include "ngsep_synth.h"

#include <zlib.h>

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
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

struct Read {
    int32_t contig, pos, flags, mapq;
    int32_t sample = 0;             // index into the sample list (RG/SM S%03d of sample_idx + sample)
    std::string name, cigar_s;      // SAM CIGAR text
    std::vector<int32_t> cigar;     // NGSEP codes
    std::string seq, qual;          // qual empty -> '*'
};

struct Snv { int32_t contig, pos; char ref, alt; int gt; };  // gt 1 het, 2 hom

}  // namespace

struct ngs_synth {
    ngs_synth_params p;
    std::vector<std::string> names;
    std::vector<std::string> seqs;
    std::vector<Read> reads;   // all records in BAM order (incl. filtered ones)
    std::vector<Snv> truth;
    // batch storage
    std::vector<int32_t> b_seq, b_first, b_flags, b_rg, b_cig_n, b_cigar, b_seqlen;
    std::vector<int64_t> b_cig_off, b_seq_off;
    std::vector<uint8_t> b_hasq;
    std::string b_bases, b_quals;
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

extern "C" ngs_synth* ngs_synth_create(const ngs_synth_params* pp) {
    ngs_synth* s = new ngs_synth();
    s->p = *pp;
    const ngs_synth_params& p = s->p;
    if (p.n_samples > 1) {
        make_population(s);
        make_batch(s);
        return s;
    }
    std::vector<ContigDef> defs;
    double pa = 0.31;  // P(A)=P(T)
    if (p.genome == NGS_GENOME_YEAST) defs.assign(std::begin(kYeast), std::end(kYeast));
    else if (p.genome == NGS_GENOME_HUMAN) { defs.assign(std::begin(kHuman), std::end(kHuman)); pa = 0.295; }
    else defs.push_back({"chrS", p.custom_len});
    int first = std::max(0, p.contig_first);
    int n = p.n_contigs > 0 ? std::min<int>(p.n_contigs, (int)defs.size() - first) : (int)defs.size() - first;
    std::vector<ContigDef> keep(defs.begin() + first, defs.begin() + first + n);
    // reference, seed 0x4E475345 + contig index
    for (size_t c = 0; c < keep.size(); c++) {
        Rng r(0x4E475345ull + (uint64_t)(first + c) + (p.seed << 32));
        std::string seq(keep[c].len, 'A');
        for (int64_t i = 0; i < keep[c].len; i++) {
            double u = r.uniform();
            char b = u < pa ? 'A' : u < 0.5 ? 'C' : u < 1.0 - pa ? 'G' : 'T';
            if (p.lower_frac > 0 && r.uniform() < p.lower_frac) b = (char)(b - 'A' + 'a');
            seq[i] = b;
        }
        s->names.push_back(keep[c].name);
        s->seqs.push_back(std::move(seq));
    }
    Rng r(p.seed * 0x9E3779B97F4A7C15ull + 17 + (uint64_t)p.sample_idx * 7919);
    char rg[16];
    std::snprintf(rg, sizeof rg, "S%03d", p.sample_idx);
    int64_t readno = 0;
    for (size_t c = 0; c < s->seqs.size(); c++) {
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
        int rl = p.read_len;
        size_t cstart = s->reads.size();
        if (L < rl) continue;
        int64_t nreads = (int64_t)std::llround(p.depth * (double)L / rl);
        struct Gen { int32_t pos; int64_t order; };
        std::vector<Gen> starts(nreads);
        for (int64_t k = 0; k < nreads; k++) starts[k] = {(int32_t)(1 + r.below((uint64_t)(L - rl + 1))), k};
        std::sort(starts.begin(), starts.end(), [](const Gen& a, const Gen& b) { return a.pos != b.pos ? a.pos < b.pos : a.order < b.order; });
        for (int64_t k = 0; k < nreads; k++) {
            Read rd;
            rd.contig = (int32_t)c;
            rd.pos = starts[k].pos;
            const std::string& hap = r.below(2) ? h1 : h0;
            rd.flags = r.below(2) ? 16 : 0;
            rd.mapq = (p.lowmq_rate > 0 && r.uniform() < p.lowmq_rate) ? 5 : 60;
            char nm[32];
            std::snprintf(nm, sizeof nm, "r%09lld", (long long)readno++);
            rd.name = nm;
            rd.seq.resize(rl);
            rd.qual.resize(rl);
            for (int i = 0; i < rl; i++) {
                char b = hap[rd.pos - 1 + i];
                int q = sample_quality(r, p.quality_model);
                double e = std::pow(10.0, -q / 10.0);
                if (r.uniform() < e) {
                    int bi = (int)(std::strchr(kBases, b) - kBases);
                    b = kBases[(bi + 1 + (int)r.below(3)) % 4];
                }
                if (p.n_frac > 0 && r.uniform() < p.n_frac) { b = 'N'; q = 2; }
                rd.seq[i] = b;
                rd.qual[i] = (char)(33 + q);
            }
            int clip = 0, clip_end = 0;
            if (p.softclip_rate > 0 && r.uniform() < p.softclip_rate) { clip = 5 + (int)r.below(16); clip_end = (int)r.below(2); }
            if (clip) {
                // soft clip keeps the read characters, shifts the aligned start to the first M base
                char buf[64];
                if (clip_end) {
                    std::snprintf(buf, sizeof buf, "%dM%dS", rl - clip, clip);
                    rd.cigar = {(rl - clip) * 8 + 3, clip * 8 + 6};
                } else {
                    std::snprintf(buf, sizeof buf, "%dS%dM", clip, rl - clip);
                    rd.cigar = {clip * 8 + 6, (rl - clip) * 8 + 3};
                    rd.pos += clip;
                    if (rd.pos + (rl - clip) - 1 > L) { rd.pos -= clip; rd.cigar = {rl * 8 + 3}; std::snprintf(buf, sizeof buf, "%dM", rl); }
                }
                rd.cigar_s = buf;
            } else {
                rd.cigar_s = std::to_string(rl) + "M";
                rd.cigar = {rl * 8 + 3};
            }
            if (p.noqual_rate > 0 && r.uniform() < p.noqual_rate) rd.qual.clear();
            bool dup = p.dup_rate > 0 && r.uniform() < p.dup_rate;
            bool sec = p.secondary_rate > 0 && r.uniform() < p.secondary_rate;
            s->reads.push_back(rd);
            if (dup) {
                Read d = rd;
                d.name += "d";
                s->reads.push_back(d);
            }
            if (sec) {
                Read d = rd;
                d.name += "s";
                d.flags |= 0x100;
                s->reads.push_back(d);
            }
        }
        // keep BAM coordinate order: records were generated sorted except soft-clipped starts
        std::stable_sort(s->reads.begin() + (ptrdiff_t)cstart, s->reads.end(),
                         [](const Read& a, const Read& b) { return a.pos < b.pos; });
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
    std::vector<ContigDef> defs;
    double pa = 0.31;
    if (p.genome == NGS_GENOME_YEAST) defs.assign(std::begin(kYeast), std::end(kYeast));
    else if (p.genome == NGS_GENOME_HUMAN) { defs.assign(std::begin(kHuman), std::end(kHuman)); pa = 0.295; }
    else defs.push_back({"chrS", p.custom_len});
    int first = std::max(0, p.contig_first);
    int n = p.n_contigs > 0 ? std::min<int>(p.n_contigs, (int)defs.size() - first) : (int)defs.size() - first;
    const int ns = p.n_samples;
    for (int c = 0; c < n; c++) {
        const ContigDef& d = defs[first + c];
        Rng r(0x4E475345ull + (uint64_t)(first + c) + (p.seed << 32));
        std::string seq(d.len, 'A');
        for (int64_t i = 0; i < d.len; i++) {
            double u = r.uniform();
            char b = u < pa ? 'A' : u < 0.5 ? 'C' : u < 1.0 - pa ? 'G' : 'T';
            if (p.lower_frac > 0 && r.uniform() < p.lower_frac) b = (char)(b - 'A' + 'a');
            seq[i] = b;
        }
        s->names.push_back(d.name);
        s->seqs.push_back(std::move(seq));
    }
    Rng r(p.seed * 0x9E3779B97F4A7C15ull + 31);
    int64_t readno = 0;
    for (size_t c = 0; c < s->seqs.size(); c++) {
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
        const int rl = p.read_len;
        if (L < rl) continue;
        const int64_t nper = (int64_t)std::llround(p.depth * (double)L / rl);
        struct Gen { int32_t pos; int32_t sample; int64_t order; };
        std::vector<Gen> starts;
        starts.reserve((size_t)(nper * ns));
        for (int k = 0; k < ns; k++)
            for (int64_t j = 0; j < nper; j++) starts.push_back({(int32_t)(1 + r.below((uint64_t)(L - rl + 1))), k, j});
        std::sort(starts.begin(), starts.end(), [](const Gen& a, const Gen& b) {
            if (a.pos != b.pos) return a.pos < b.pos;
            if (a.sample != b.sample) return a.sample < b.sample;
            return a.order < b.order;
        });
        for (const Gen& g : starts) {
            Read rd;
            rd.contig = (int32_t)c;
            rd.pos = g.pos;
            rd.sample = g.sample;
            const int hap = (int)r.below(2);
            rd.flags = r.below(2) ? 16 : 0;
            rd.mapq = 60;
            char nm[32];
            std::snprintf(nm, sizeof nm, "r%09lld", (long long)readno++);
            rd.name = nm;
            rd.seq.resize(rl);
            rd.qual.resize(rl);
            size_t vi = (size_t)(std::lower_bound(vpos.begin(), vpos.end(), g.pos) - vpos.begin());
            for (int i = 0; i < rl; i++) {
                const int32_t pos = g.pos + i;
                char b = (char)std::toupper(ref[pos - 1]);
                while (vi < vpos.size() && vpos[vi] < pos) vi++;
                if (vi < vpos.size() && vpos[vi] == pos && ((vgt[vi * ns + g.sample] >> hap) & 1)) b = valt[vi];
                int q = sample_quality(r, p.quality_model);
                double e = std::pow(10.0, -q / 10.0);
                if (r.uniform() < e) {
                    const char* pb = std::strchr(kBases, b);
                    int bi = pb ? (int)(pb - kBases) : 0;
                    b = kBases[(bi + 1 + (int)r.below(3)) % 4];
                }
                if (p.n_frac > 0 && r.uniform() < p.n_frac) { b = 'N'; q = 2; }
                rd.seq[i] = b;
                rd.qual[i] = (char)(33 + q);
            }
            rd.cigar_s = std::to_string(rl) + "M";
            rd.cigar = {rl * 8 + 3};
            const bool dup = p.dup_rate > 0 && r.uniform() < p.dup_rate;
            s->reads.push_back(rd);
            if (dup) {
                Read d = rd;
                d.name += "d";
                s->reads.push_back(d);
            }
        }
    }
}

static void make_batch(ngs_synth* s) {
    // batch view: reader filters with default options (drop secondary and MAPQ<20 without NH)
    for (const Read& rd : s->reads) {
        if (rd.flags & 0x100) continue;
        if (rd.mapq < 20) continue;
        s->b_seq.push_back(rd.contig);
        s->b_first.push_back(rd.pos);
        s->b_flags.push_back(rd.flags);
        s->b_rg.push_back(rd.sample);
        s->b_cig_off.push_back((int64_t)s->b_cigar.size());
        s->b_cig_n.push_back((int32_t)rd.cigar.size());
        for (int32_t v : rd.cigar) s->b_cigar.push_back(v);
        s->b_seq_off.push_back((int64_t)s->b_bases.size());
        s->b_seqlen.push_back((int32_t)rd.seq.size());
        s->b_bases += rd.seq;
        if (rd.qual.empty()) { s->b_quals += std::string(rd.seq.size(), '!'); s->b_hasq.push_back(0); }
        else { s->b_quals += rd.qual; s->b_hasq.push_back(1); }
    }
}

extern "C" void ngs_synth_free(ngs_synth* s) { delete s; }
extern "C" int ngs_synth_n_contigs(const ngs_synth* s) { return (int)s->seqs.size(); }
extern "C" const char* ngs_synth_contig_name(const ngs_synth* s, int i) { return s->names[i].c_str(); }
extern "C" int64_t ngs_synth_contig_len(const ngs_synth* s, int i) { return (int64_t)s->seqs[i].size(); }
extern "C" const char* ngs_synth_contig_seq(const ngs_synth* s, int i) { return s->seqs[i].data(); }
extern "C" int64_t ngs_synth_n_reads(const ngs_synth* s) { return (int64_t)s->b_first.size(); }
extern "C" int64_t ngs_synth_n_bases(const ngs_synth* s) { return (int64_t)s->b_bases.size(); }

extern "C" int ngs_synth_batch(ngs_synth* s, ngsep_read_batch* b) {
    b->n_reads = (int64_t)s->b_first.size();
    b->seq_id = s->b_seq.data();
    b->first = s->b_first.data();
    b->flags = s->b_flags.data();
    b->read_group = s->b_rg.data();
    b->cigar_off = s->b_cig_off.data();
    b->cigar_n = s->b_cig_n.data();
    b->cigar = s->b_cigar.data();
    b->seq_off = s->b_seq_off.data();
    b->seq_len = s->b_seqlen.data();
    b->bases = s->b_bases.data();
    b->quals = s->b_quals.data();
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

extern "C" int ngs_synth_write_sam(const ngs_synth* s, const char* path) {
    FILE* f = std::fopen(path, "w");
    if (!f) return -1;
    std::string h = header_text(s);
    std::fwrite(h.data(), 1, h.size(), f);
    for (const Read& rd : s->reads) {
        std::fprintf(f, "%s\t%d\t%s\t%d\t%d\t%s\t*\t0\t0\t%s\t%s\tRG:Z:S%03d\n", rd.name.c_str(), rd.flags,
                     s->names[rd.contig].c_str(), rd.pos, rd.mapq, rd.cigar_s.c_str(), rd.seq.c_str(),
                     rd.qual.empty() ? "*" : rd.qual.c_str(), s->p.sample_idx + rd.sample);
    }
    std::fclose(f);
    return 0;
}

// ---- BGZF / BAM writer (SAM spec section 4) ----
namespace {
struct Bgzf {
    FILE* f;
    std::string buf;
    explicit Bgzf(FILE* ff) : f(ff) {}
    void block(const char* data, size_t n) {
        std::vector<unsigned char> out(n + 1024);
        z_stream z{};
        deflateInit2(&z, 6, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
        z.next_in = (Bytef*)data; z.avail_in = (uInt)n;
        z.next_out = out.data() + 18; z.avail_out = (uInt)(out.size() - 26);
        deflate(&z, Z_FINISH);
        size_t clen = z.total_out;
        deflateEnd(&z);
        unsigned char* h = out.data();
        const unsigned char hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0, 0, 0};
        std::memcpy(h, hdr, 18);
        uint16_t bsize = (uint16_t)(clen + 25);
        h[16] = bsize & 0xff; h[17] = bsize >> 8;
        uint32_t crc = (uint32_t)crc32(0, (const Bytef*)data, (uInt)n);
        unsigned char* t = out.data() + 18 + clen;
        for (int i = 0; i < 4; i++) t[i] = (crc >> (8 * i)) & 0xff;
        for (int i = 0; i < 4; i++) t[4 + i] = ((uint32_t)n >> (8 * i)) & 0xff;
        std::fwrite(out.data(), 1, 18 + clen + 8, f);
    }
    void write(const void* d, size_t n) {
        buf.append((const char*)d, n);
        while (buf.size() >= 65280) { block(buf.data(), 65280); buf.erase(0, 65280); }
    }
    void close() {
        if (!buf.empty()) block(buf.data(), buf.size());
        static const unsigned char eof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        std::fwrite(eof, 1, 28, f);
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
    for (const Read& rd : s->reads) {
        if (only_sample >= 0 && rd.sample != only_sample) continue;
        char rg[16];
        std::snprintf(rg, sizeof rg, "S%03d", s->p.sample_idx + rd.sample);
        std::string r;
        int l_seq = (int)rd.seq.size();
        int reflen = 0;
        for (int32_t v : rd.cigar) if ((v & 7) & 1) reflen += v / 8;
        put<int32_t>(r, rd.contig);
        put<int32_t>(r, rd.pos - 1);
        put<uint8_t>(r, (uint8_t)(rd.name.size() + 1));
        put<uint8_t>(r, (uint8_t)rd.mapq);
        put<uint16_t>(r, (uint16_t)reg2bin(rd.pos - 1, rd.pos - 1 + reflen));
        put<uint16_t>(r, (uint16_t)rd.cigar.size());
        put<uint16_t>(r, (uint16_t)rd.flags);
        put<int32_t>(r, l_seq);
        put<int32_t>(r, -1);
        put<int32_t>(r, -1);
        put<int32_t>(r, 0);
        r += rd.name; r.push_back(0);
        for (int32_t v : rd.cigar) put<uint32_t>(r, (uint32_t)((v / 8) << 4 | bam_op[v & 7]));
        for (int i = 0; i < l_seq; i += 2) {
            int hi = (int)(std::strchr(nt16, rd.seq[i]) - nt16);
            int lo = i + 1 < l_seq ? (int)(std::strchr(nt16, rd.seq[i + 1]) - nt16) : 0;
            put<uint8_t>(r, (uint8_t)(hi << 4 | lo));
        }
        for (int i = 0; i < l_seq; i++) put<uint8_t>(r, rd.qual.empty() ? 0xff : (uint8_t)(rd.qual[i] - 33));
        r += "RGZ"; r += rg; r.push_back(0);
        std::string rec;
        put<int32_t>(rec, (int32_t)r.size());
        rec += r;
        z.write(rec.data(), rec.size());
    }
    z.close();
    std::fclose(f);
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
