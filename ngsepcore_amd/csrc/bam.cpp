// bam.cpp -- BGZF/BAM decoding with ReadAlignmentFileReader's record semantics
// (alignments/io/ReadAlignmentFileReader.java:171-354).  htsjdk (lib/htsjdk-2.22.jar) plays this
// role in the reference; this reader reproduces the fields NGSEP takes from it:
//   getAlignmentStart/End, getFlags, getMappingQuality, CIGAR, getReadString
//   ("=ACMGRSVTWYHKDBN" decoding), getBaseQualityString (0xFF -> "*"), RG (header lookup), NH.
// Reader filters: consecutive duplicates (isSameAlignment :292-306), FLAG_MULTIPLE_ALN (:284-291),
// unmapped/secondary/multiple filter flags (AlignmentsPileupGenerator.java:363-375).
#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "engine.hpp"

struct ngsep_bam {
    ngsep_ctx* ctx = nullptr;
    std::FILE* f = nullptr;
    std::vector<uint8_t> comp;
    std::string buf;        // inflated bytes not yet consumed
    size_t pos = 0;
    bool eof = false;
    std::vector<int32_t> ref_to_seq;   // BAM refID -> ctx sequence id
    std::vector<std::string> rg_ids;   // header read groups
    std::vector<std::string> rg_sm;    // their SM tags (the read group id when absent, ReadAlignmentFileReader.java:186-188)
    std::unordered_map<std::string, int32_t> rg_index;
    int filter_flags = 0;
    int min_mq = 20;
    // previous raw record for isSameAlignment
    bool have_last = false;
    int32_t last_pos = 0;
    int last_paired = 0, last_fop = 0;
    std::string last_name;
    // batch storage
    std::vector<int32_t> b_seq, b_first, b_flags, b_rg, b_cig_n, b_cigar, b_seqlen;
    std::vector<int64_t> b_cig_off, b_seq_off;
    std::vector<uint8_t> b_hasq;
    std::string b_bases, b_quals;
};

namespace {

// inflates the next BGZF block into bam->buf; returns false at end of file
bool next_block(ngsep_bam* b, std::string& err) {
    uint8_t h[18];
    size_t n = std::fread(h, 1, 18, b->f);
    if (n == 0) return false;
    if (n < 18 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) { err = "not a BGZF file"; return false; }
    uint16_t xlen = (uint16_t)(h[10] | (h[11] << 8));
    // standard BGZF: XLEN=6 with the BC subfield
    std::vector<uint8_t> extra(xlen);
    std::memcpy(extra.data(), h + 12, std::min<size_t>(6, xlen));
    if (xlen > 6 && std::fread(extra.data() + 6, 1, xlen - 6, b->f) != (size_t)(xlen - 6)) { err = "truncated BGZF header"; return false; }
    int bsize = -1;
    for (size_t i = 0; i + 4 <= extra.size();) {
        uint16_t sl = (uint16_t)(extra[i + 2] | (extra[i + 3] << 8));
        if (extra[i] == 'B' && extra[i + 1] == 'C' && sl == 2) bsize = extra[i + 4] | (extra[i + 5] << 8);
        i += 4 + sl;
    }
    if (bsize < 0) { err = "BGZF block without BC field"; return false; }
    size_t rest = (size_t)bsize + 1 - 12 - xlen;
    b->comp.resize(rest);
    if (std::fread(b->comp.data(), 1, rest, b->f) != rest) { err = "truncated BGZF block"; return false; }
    uint32_t isize = (uint32_t)(b->comp[rest - 4] | (b->comp[rest - 3] << 8) | (b->comp[rest - 2] << 16) | ((uint32_t)b->comp[rest - 1] << 24));
    if (isize == 0) return true;
    size_t o = b->buf.size();
    b->buf.resize(o + isize);
    z_stream z{};
    inflateInit2(&z, -15);
    z.next_in = b->comp.data();
    z.avail_in = (uInt)(rest - 8);
    z.next_out = (Bytef*)&b->buf[o];
    z.avail_out = isize;
    int rc = inflate(&z, Z_FINISH);
    inflateEnd(&z);
    if (rc != Z_STREAM_END) { err = "BGZF inflate failed"; return false; }
    return true;
}

// ensures at least n unconsumed bytes; false at EOF
bool need(ngsep_bam* b, size_t n, std::string& err) {
    while (b->buf.size() - b->pos < n) {
        if (b->pos > (1u << 20)) { b->buf.erase(0, b->pos); b->pos = 0; }
        if (!next_block(b, err)) return false;
    }
    return true;
}

template <class T> T rd(const char* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }

}  // namespace

using namespace ngsep;

extern "C" int ngsep_bam_open(ngsep_ctx* c, const char* path, ngsep_bam** out) {
    if (!c || !path || !out) return NGSEP_E_INVALID;
    ngsep_bam* b = new ngsep_bam();
    b->ctx = c;
    b->f = std::fopen(path, "rb");
    if (!b->f) { delete b; return set_error(c, NGSEP_E_IO, std::string("cannot open ") + path); }
    std::string err;
    if (!need(b, 8, err) || std::memcmp(&b->buf[0], "BAM\1", 4) != 0) {
        std::fclose(b->f); delete b;
        return set_error(c, NGSEP_E_FORMAT, err.empty() ? "not a BAM file" : err);
    }
    int32_t l_text = rd<int32_t>(&b->buf[4]);
    if (!need(b, 8 + (size_t)l_text + 4, err)) { std::fclose(b->f); delete b; return set_error(c, NGSEP_E_FORMAT, "truncated BAM header"); }
    std::string text = b->buf.substr(8, (size_t)l_text);
    b->pos = 8 + (size_t)l_text;
    int32_t n_ref = rd<int32_t>(&b->buf[b->pos]);
    b->pos += 4;
    std::unordered_map<std::string, int32_t> seq_index;
    for (size_t i = 0; i < c->seq_names.size(); i++) seq_index[c->seq_names[i]] = (int32_t)i;
    // CoverageStatisticsCalculator runs without a genome (-r is optional there): the header's sequences
    const bool header_seqs = c->params.coverage_stats && c->seq_names.empty();
    for (int32_t i = 0; i < n_ref; i++) {
        if (!need(b, 4, err)) break;
        int32_t ln = rd<int32_t>(&b->buf[b->pos]);
        if (!need(b, 4 + (size_t)ln + 4, err)) break;
        std::string name(&b->buf[b->pos + 4], (size_t)(ln > 0 ? ln - 1 : 0));
        int32_t lref = rd<int32_t>(&b->buf[b->pos + 4 + ln]);
        b->pos += 8 + (size_t)ln;
        if (header_seqs && !seq_index.count(name)) {
            seq_index[name] = (int32_t)c->seq_names.size();
            c->seq_names.push_back(name);
            c->seq_bases.emplace_back();
            b->ref_to_seq.push_back(seq_index[name]);
            continue;
        }
        auto it = seq_index.find(name);
        // ReadAlignmentFileReader.loadHeader validation (:198-214)
        if (it == seq_index.end()) {
            std::fclose(b->f); delete b;
            return set_error(c, NGSEP_E_FORMAT, "Inconsistent file header. Sequence " + name + " not present in the reference sequences");
        }
        if ((int64_t)c->seq_bases[it->second].size() != lref) {
            std::fclose(b->f); delete b;
            return set_error(c, NGSEP_E_FORMAT, "Inconsistent length in file header. Sequence " + name);
        }
        b->ref_to_seq.push_back(it->second);
    }
    // @RG lines
    size_t p = 0;
    while (p < text.size()) {
        size_t e = text.find('\n', p);
        if (e == std::string::npos) e = text.size();
        std::string line = text.substr(p, e - p);
        if (line.compare(0, 3, "@RG") == 0) {
            size_t id = line.find("\tID:");
            if (id != std::string::npos) {
                size_t ie = line.find('\t', id + 4);
                std::string v = line.substr(id + 4, ie == std::string::npos ? std::string::npos : ie - id - 4);
                std::string sm = v;
                size_t sp = line.find("\tSM:");
                if (sp != std::string::npos) {
                    size_t se = line.find('\t', sp + 4);
                    sm = line.substr(sp + 4, se == std::string::npos ? std::string::npos : se - sp - 4);
                }
                if (!b->rg_index.count(v)) { b->rg_index[v] = (int32_t)b->rg_ids.size(); b->rg_ids.push_back(v); b->rg_sm.push_back(sm); }
            }
        }
        p = e + 1;
    }
    // AlignmentsPileupGenerator.createReader (:363-375)
    b->filter_flags = 0x4;
    if (!c->params.process_secondary) {
        b->filter_flags |= 0x100;
        if (!c->params.process_nonunique) b->filter_flags |= 0x1000;
    }
    b->min_mq = c->params.min_mq;
    *out = b;
    return NGSEP_OK;
}

extern "C" int ngsep_bam_next_batch(ngsep_bam* b, int64_t max_reads, ngsep_read_batch* out) {
    if (!b || !out) return NGSEP_E_INVALID;
    static const int kOp[9] = {3, 2, 1, 5, 6, 0, 4, 3, 7};   // BAM M I D N S H P = X -> NGSEP H0 D1 I2 M3 P4 N5 S6 X7
    static const char kNt[] = "=ACMGRSVTWYHKDBN";
    b->b_seq.clear(); b->b_first.clear(); b->b_flags.clear(); b->b_rg.clear(); b->b_cig_n.clear();
    b->b_cigar.clear(); b->b_seqlen.clear(); b->b_cig_off.clear(); b->b_seq_off.clear(); b->b_hasq.clear();
    b->b_bases.clear(); b->b_quals.clear();
    std::string err;
    int64_t n = 0;
    while (n < max_reads) {
        if (!need(b, 4, err)) break;
        int32_t bs = rd<int32_t>(&b->buf[b->pos]);
        if (bs < 32) return set_error(b->ctx, NGSEP_E_FORMAT, "malformed BAM record");
        if (!need(b, 4 + (size_t)bs, err)) return set_error(b->ctx, NGSEP_E_FORMAT, "truncated BAM record");
        const char* r = &b->buf[b->pos + 4];
        b->pos += 4 + (size_t)bs;
        int32_t refid = rd<int32_t>(r);
        int32_t pos0 = rd<int32_t>(r + 4);
        uint8_t l_name = (uint8_t)r[8];
        uint8_t mapq = (uint8_t)r[9];
        uint16_t n_cig = rd<uint16_t>(r + 12);
        uint16_t flag = rd<uint16_t>(r + 14);
        int32_t l_seq = rd<int32_t>(r + 16);
        const char* name = r + 32;
        const char* cig = name + l_name;
        const char* seq = cig + 4 * n_cig;
        const char* qual = seq + (l_seq + 1) / 2;
        const char* aux = qual + l_seq;
        const char* end = r + bs;
        int32_t start = pos0 + 1;
        // isSameAlignment (ReadAlignmentFileReader.java:292-306)
        int paired = (flag & 1) != 0, fop = (flag & 0x40) != 0;
        std::string nm(name, l_name ? l_name - 1 : 0);
        if (b->have_last && b->last_pos == start && b->last_paired == paired && (!paired || b->last_fop == fop) && b->last_name == nm) continue;
        b->have_last = true; b->last_pos = start; b->last_paired = paired; b->last_fop = fop; b->last_name = nm;
        if (flag & 0x4) continue;               // FLAG_READ_UNMAPPED (filtered)
        if (refid < 0 || refid >= (int32_t)b->ref_to_seq.size()) continue;
        // tags: NH and RG
        int nh = 0, nh_present = 0, rg = -1;
        for (const char* t = aux; t + 3 <= end;) {
            char t0 = t[0], t1 = t[1], ty = t[2];
            const char* v = t + 3;
            size_t sz = 0;
            long long iv = 0;
            bool isint = true;
            switch (ty) {
                case 'A': case 'c': case 'C': sz = 1; iv = ty == 'c' ? (int8_t)v[0] : (uint8_t)v[0]; break;
                case 's': sz = 2; iv = rd<int16_t>(v); break;
                case 'S': sz = 2; iv = rd<uint16_t>(v); break;
                case 'i': sz = 4; iv = rd<int32_t>(v); break;
                case 'I': sz = 4; iv = rd<uint32_t>(v); break;
                case 'f': sz = 4; isint = false; break;
                case 'Z': case 'H': { isint = false; const char* z = v; while (z < end && *z) z++; sz = (size_t)(z - v) + 1; break; }
                case 'B': {
                    isint = false;
                    char sub = v[0];
                    int32_t cnt = rd<int32_t>(v + 1);
                    int es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                    sz = 5 + (size_t)cnt * es;
                    break;
                }
                default: t = end; continue;
            }
            if (t0 == 'N' && t1 == 'H' && isint && ty != 'A') { nh = (int)iv; nh_present = 1; }
            if (t0 == 'R' && t1 == 'G' && ty == 'Z') {
                auto it = b->rg_index.find(std::string(v));
                rg = it == b->rg_index.end() ? -1 : it->second;   // getReadGroup() is null if not in header
            }
            t = v + sz;
        }
        int flags = flag;
        // isMultiple (:284-291)
        bool multiple;
        if (flag & 0x100) multiple = true;
        else if (nh_present && nh > 1) multiple = true;
        else if (nh_present && nh == 1) multiple = false;
        else multiple = mapq < b->min_mq;
        if (multiple) flags += 0x1000;
        if (n_cig == 0) continue;               // mapped read without CIGAR: setCigarString throws
        // CIGAR -> NGSEP codes with collapseEqualEvents
        int64_t coff = (int64_t)b->b_cigar.size();
        int read_len = 0;
        bool bad = false;
        int nc = 0;
        for (int i = 0; i < n_cig; i++) {
            uint32_t v = rd<uint32_t>(cig + 4 * i);
            uint32_t op = v & 15, len = v >> 4;
            if (op > 8) { bad = true; break; }
            int nop = kOp[op];
            if (nc > 0 && (b->b_cigar.back() & 7) == nop) b->b_cigar.back() += (int32_t)len * 8;
            else { b->b_cigar.push_back((int32_t)len * 8 + nop); nc++; }
            if (nop & 2) read_len += (int)len;
        }
        if (bad) { b->b_cigar.resize((size_t)coff); continue; }
        if (l_seq > 0 && l_seq != read_len) { b->b_cigar.resize((size_t)coff); continue; }   // setReadCharacters throws
        if ((flags & b->filter_flags) != 0) { b->b_cigar.resize((size_t)coff); continue; }
        b->b_seq.push_back(b->ref_to_seq[refid]);
        b->b_first.push_back(start);
        b->b_flags.push_back(flags);
        b->b_rg.push_back(rg);
        b->b_cig_off.push_back(coff);
        b->b_cig_n.push_back(nc);
        b->b_seq_off.push_back((int64_t)b->b_bases.size());
        b->b_seqlen.push_back(l_seq);
        size_t so = b->b_bases.size();
        b->b_bases.resize(so + (size_t)l_seq);
        b->b_quals.resize(so + (size_t)l_seq);
        for (int32_t i = 0; i < l_seq; i++) {
            uint8_t byte = (uint8_t)seq[i >> 1];
            b->b_bases[so + i] = kNt[(i & 1) ? (byte & 15) : (byte >> 4)];
        }
        bool hasq = l_seq > 0 && (uint8_t)qual[0] != 0xFF;
        for (int32_t i = 0; i < l_seq; i++) b->b_quals[so + i] = hasq ? (char)((uint8_t)qual[i] + 33) : '!';
        b->b_hasq.push_back(hasq ? 1 : 0);
        n++;
    }
    if (!err.empty()) return set_error(b->ctx, NGSEP_E_FORMAT, err);
    out->n_reads = n;
    out->seq_id = b->b_seq.data();
    out->first = b->b_first.data();
    out->flags = b->b_flags.data();
    out->read_group = b->b_rg.data();
    out->cigar_off = b->b_cig_off.data();
    out->cigar_n = b->b_cig_n.data();
    out->cigar = b->b_cigar.data();
    out->seq_off = b->b_seq_off.data();
    out->seq_len = b->b_seqlen.data();
    out->bases = b->b_bases.data();
    out->quals = b->b_quals.data();
    out->has_quals = b->b_hasq.data();
    return NGSEP_OK;
}

extern "C" int ngsep_bam_close(ngsep_bam* b) {
    if (!b) return NGSEP_E_INVALID;
    if (b->f) std::fclose(b->f);
    delete b;
    return NGSEP_OK;
}

namespace ngsep {
// SingleSampleVariantsDetector.findSNVS (:896-931) + onSequenceEnd/saveSequenceVariants (:933-968, :1026-1032)
int call_bam(ngsep_ctx* c, const char* bam_path, const char* out_vcf) {
    ngsep_bam* b = nullptr;
    int rc = ngsep_bam_open(c, bam_path, &b);
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_write_vcf_header(c, out_vcf);
    if (rc != NGSEP_OK) { ngsep_bam_close(b); return rc; }
    ngsep_read_batch batch;
    while (true) {
        rc = ngsep_bam_next_batch(b, 1 << 20, &batch);
        if (rc != NGSEP_OK) break;
        if (batch.n_reads == 0) break;
        rc = ngsep_process_alignments(c, &batch);
        if (rc != NGSEP_OK) break;
        if (!c->sites.empty()) { rc = ngsep_append_vcf_records(c, out_vcf); if (rc != NGSEP_OK) break; }
    }
    ngsep_bam_close(b);
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK) return rc;
    return ngsep_append_vcf_records(c, out_vcf);
}
}  // namespace ngsep

// CoverageStatisticsCalculator.processFile (discovery/CoverageStatisticsCalculator.java:99-122): the reader
// keeps secondary and non-unique alignments (processSecondaryAlignments = true), the same-start cap is 100
extern "C" int ngsep_coverage_bam(ngsep_ctx* c, const char* bam_path, const char* out_path) {
    if (!c || !bam_path) return NGSEP_E_INVALID;
    if (!c->params.coverage_stats) return set_error(c, NGSEP_E_INVALID, "ngsep_coverage_bam needs params.coverage_stats = 1");
    ngsep_bam* b = nullptr;
    int rc = ngsep_bam_open(c, bam_path, &b);
    if (rc != NGSEP_OK) return rc;
    ngsep_read_batch batch;
    while (true) {
        rc = ngsep_bam_next_batch(b, 1 << 20, &batch);
        if (rc != NGSEP_OK || batch.n_reads == 0) break;
        rc = ngsep_process_alignments(c, &batch);
        if (rc != NGSEP_OK) break;
    }
    ngsep_bam_close(b);
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK || !out_path) return rc;
    return ngsep_write_coverage(c, out_path);
}

extern "C" int ngsep_call_bam(ngsep_ctx* c, const char* bam_path, const char* out_vcf_path) {
    if (!c || !bam_path || !out_vcf_path) return NGSEP_E_INVALID;
    return ngsep::call_bam(c, bam_path, out_vcf_path);
}

// ---- MultisampleVariantsDetector.run on BAM files (discovery/MultisampleVariantsDetector.java:421-459) ----
namespace {
int32_t java_hash(const std::string& s) {
    uint32_t h = 0;
    for (unsigned char ch : s) h = 31u * h + ch;
    return (int32_t)h;
}
// iteration order of a java.util.HashSet<String> filled in the given order (variants/Sample.java:36)
std::vector<int> hashset_order(const std::vector<std::string>& ids) {
    size_t cap = 16;
    while (ids.size() > cap * 3 / 4) cap *= 2;
    std::vector<int> idx(ids.size());
    std::vector<uint32_t> bucket(ids.size());
    for (size_t i = 0; i < ids.size(); i++) {
        idx[i] = (int)i;
        const uint32_t h = (uint32_t)java_hash(ids[i]);
        bucket[i] = (h ^ (h >> 16)) & (uint32_t)(cap - 1);
    }
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return bucket[a] < bucket[b]; });
    return idx;
}
struct Cursor {
    ngsep_bam* bam = nullptr;
    ngsep_read_batch batch{};
    int64_t i = 0;
    bool done = false;
    std::vector<int32_t> rg_global;    // file read group -> global read group
    int32_t last(int64_t k) const {
        int32_t e = batch.first[k];
        for (int32_t j = 0; j < batch.cigar_n[k]; j++) { const int32_t v = batch.cigar[batch.cigar_off[k] + j]; if (v & 1) e += v / 8; }
        return e - 1;
    }
};
}  // namespace

extern "C" int ngsep_call_population_bams(ngsep_ctx* c, const char* const* bam_paths, int32_t n_files, const char* out_vcf_path) {
    if (!c || !bam_paths || n_files <= 0 || !out_vcf_path) return NGSEP_E_INVALID;
    if (!c->params.multisample) return set_error(c, NGSEP_E_INVALID, "ngsep_call_population_bams needs params.multisample = 1");
    std::vector<Cursor> cur((size_t)n_files);
    auto close_all = [&]() { for (auto& k : cur) if (k.bam) ngsep_bam_close(k.bam); };
    // loadSamplesFromAlignmentHeaders (:499-523): read group -> sample over all files, samples by id
    std::vector<std::string> rg_ids, rg_sm;
    std::unordered_map<std::string, int32_t> rg_global;
    for (int f = 0; f < n_files; f++) {
        int rc = ngsep_bam_open(c, bam_paths[f], &cur[(size_t)f].bam);
        if (rc != NGSEP_OK) { close_all(); return rc; }
        ngsep_bam* b = cur[(size_t)f].bam;
        for (size_t g = 0; g < b->rg_ids.size(); g++) {
            auto it = rg_global.find(b->rg_ids[g]);
            if (it == rg_global.end()) {
                it = rg_global.emplace(b->rg_ids[g], (int32_t)rg_ids.size()).first;
                rg_ids.push_back(b->rg_ids[g]);
                rg_sm.push_back(b->rg_sm[g]);
            } else if (rg_sm[(size_t)it->second] != b->rg_sm[g]) {
                close_all();
                return set_error(c, NGSEP_E_FORMAT, "The read group ID: " + b->rg_ids[g] + " is associated to two different samples");
            }
            cur[(size_t)f].rg_global.push_back(it->second);
        }
    }
    std::vector<std::string> samples(rg_sm);
    std::sort(samples.begin(), samples.end());
    samples.erase(std::unique(samples.begin(), samples.end()), samples.end());
    std::vector<int32_t> rg_sample(rg_ids.size(), -1), rg_rank(rg_ids.size(), 0);
    for (size_t sm = 0; sm < samples.size(); sm++) {
        std::vector<int32_t> members;
        std::vector<std::string> mids;
        for (size_t g = 0; g < rg_ids.size(); g++)
            if (rg_sm[g] == samples[sm]) { members.push_back((int32_t)g); mids.push_back(rg_ids[g]); }
        std::vector<int> ord = hashset_order(mids);
        for (size_t r = 0; r < ord.size(); r++) { rg_sample[(size_t)members[(size_t)ord[r]]] = (int32_t)sm; rg_rank[(size_t)members[(size_t)ord[r]]] = (int32_t)r; }
    }
    std::vector<const char*> sid;
    for (const auto& x : samples) sid.push_back(x.c_str());
    int rc = ngsep_set_samples(c, (int32_t)samples.size(), sid.data(), (int32_t)rg_ids.size(), rg_sample.data(), rg_rank.data());
    if (rc != NGSEP_OK) { close_all(); return rc; }
    // AlignmentsPileupGenerator.processFiles: k-way merge by GenomicRegionComparator (sequence order,
    // first, last), ties to the lowest file index (chooseNextAln, :268-289)
    auto refill = [&](Cursor& k) -> int {
        while (!k.done && k.i >= k.batch.n_reads) {
            int r = ngsep_bam_next_batch(k.bam, 1 << 18, &k.batch);
            if (r != NGSEP_OK) return r;
            k.i = 0;
            if (k.batch.n_reads == 0) k.done = true;
        }
        return NGSEP_OK;
    };
    for (auto& k : cur) { rc = refill(k); if (rc != NGSEP_OK) { close_all(); return rc; } }
    // merged batch storage
    std::vector<int32_t> m_seq, m_first, m_flags, m_rg, m_cig_n, m_cigar, m_seqlen;
    std::vector<int64_t> m_cig_off, m_seq_off;
    std::vector<uint8_t> m_hasq;
    std::string m_bases, m_quals;
    auto flush = [&]() -> int {
        if (m_first.empty()) return NGSEP_OK;
        ngsep_read_batch mb{};
        mb.n_reads = (int64_t)m_first.size();
        mb.seq_id = m_seq.data(); mb.first = m_first.data(); mb.flags = m_flags.data(); mb.read_group = m_rg.data();
        mb.cigar_off = m_cig_off.data(); mb.cigar_n = m_cig_n.data(); mb.cigar = m_cigar.data();
        mb.seq_off = m_seq_off.data(); mb.seq_len = m_seqlen.data(); mb.bases = m_bases.data(); mb.quals = m_quals.data();
        mb.has_quals = m_hasq.data();
        int r = ngsep_process_alignments(c, &mb);
        m_seq.clear(); m_first.clear(); m_flags.clear(); m_rg.clear(); m_cig_n.clear(); m_cigar.clear(); m_seqlen.clear();
        m_cig_off.clear(); m_seq_off.clear(); m_hasq.clear(); m_bases.clear(); m_quals.clear();
        return r;
    };
    while (true) {
        int best = -1;
        int32_t bs = 0, bf = 0, bl = 0;
        for (int f = 0; f < n_files; f++) {
            Cursor& k = cur[(size_t)f];
            if (k.done) continue;
            const int32_t s2 = k.batch.seq_id[k.i], f2 = k.batch.first[k.i];
            if (best >= 0 && (s2 > bs || (s2 == bs && (f2 > bf || (f2 == bf && k.last(k.i) >= bl))))) continue;
            best = f; bs = s2; bf = f2; bl = k.last(k.i);
        }
        if (best < 0) break;
        Cursor& k = cur[(size_t)best];
        const int64_t i = k.i;
        m_seq.push_back(k.batch.seq_id[i]);
        m_first.push_back(k.batch.first[i]);
        m_flags.push_back(k.batch.flags[i]);
        const int32_t lrg = k.batch.read_group ? k.batch.read_group[i] : -1;
        m_rg.push_back(lrg >= 0 && lrg < (int32_t)k.rg_global.size() ? k.rg_global[(size_t)lrg] : -1);
        m_cig_off.push_back((int64_t)m_cigar.size());
        m_cig_n.push_back(k.batch.cigar_n[i]);
        m_cigar.insert(m_cigar.end(), k.batch.cigar + k.batch.cigar_off[i], k.batch.cigar + k.batch.cigar_off[i] + k.batch.cigar_n[i]);
        m_seq_off.push_back((int64_t)m_bases.size());
        m_seqlen.push_back(k.batch.seq_len[i]);
        m_bases.append(k.batch.bases + k.batch.seq_off[i], (size_t)k.batch.seq_len[i]);
        m_quals.append(k.batch.quals + k.batch.seq_off[i], (size_t)k.batch.seq_len[i]);
        m_hasq.push_back(k.batch.has_quals ? k.batch.has_quals[i] : 1);
        k.i++;
        if (k.i >= k.batch.n_reads) {
            // the merged batch references nothing of this reader's arrays any more (copied above)
            rc = refill(k);
            if (rc != NGSEP_OK) { close_all(); return rc; }
        }
        if (m_first.size() >= (1u << 18)) { rc = flush(); if (rc != NGSEP_OK) { close_all(); return rc; } }
    }
    rc = flush();
    close_all();
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK) return rc;
    return ngsep_write_population_vcf(c, out_vcf_path);
}
