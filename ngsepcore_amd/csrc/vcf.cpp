// vcf.cpp -- VCF text exactly as SingleSampleVariantsDetector writes it:
// VCFFileHeader.makeDefaultEmptyHeader/print (vcf/VCFFileHeader.java:46-95,219-245) and
// VCFFileWriter.printVCFRecord/printGenotypeInfo (vcf/VCFFileWriter.java:44-308) for
// CalledSNV (variants/CalledSNV.java) and triallelic CalledGenomicVariantImpl calls.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>

#include "engine.hpp"

namespace ngsep {

int64_t java_round(double x);

static const char* kHeaderLines[][5] = {
    // type, id, description, number, data type (attribute order ID,Number,Type,Description: VCFHeaderLine.java:43-50)
    {"INFO", "CNV", "\"Number of samples with CNVs around this variant\"", "1", "Integer"},
    {"INFO", "TA", "\"Variant annotation based on a gene model\"", "1", "String"},
    {"INFO", "TID", "\"Id of the transcript related to the variant annotation\"", "1", "String"},
    {"INFO", "TGN", "\"Name of the gene related to the variant annotation\"", "1", "String"},
    {"INFO", "TCO", "\"One based codon position of the start of the variant. The decimal is the codon position\"", "1", "Float"},
    {"INFO", "TACH", "\"Description of the aminoacid change produced by a non-synonymous mutation. String encoded as reference aminoacid, position and mutated aminoacid\"", "1", "String"},
    {"INFO", "NS", "\"Number of samples genotyped\"", "1", "Integer"},
    {"INFO", "MAF", "\"Minor allele frequency\"", "1", "Float"},
    {"INFO", "OH", "\"Observed heterozygosity\"", "1", "Float"},
    {"INFO", "AN", "\"Number of alleles in called genotypes\"", "1", "Integer"},
    {"INFO", "AFS", "\"Allele counts over the population for all alleles, including the reference\"", "R", "Integer"},
    {"INFO", "TYPE", "\"Type of variant\"", "1", "String"},
    {"INFO", "FS", "\"Phred-scaled p-value using Fisher's exact test to detect strand bias\"", "1", "Float"},
    {"INFO", "END", "\"End position of the structural variant\"", "1", "Integer"},
    {"INFO", "SVTYPE", "\"Type of SV:DEL=Deletion, INS=Insertion, DUP=Duplication, INV=Inversion\"", "1", "String"},
    {"INFO", "SVLEN", "\"Difference in length between REF and ALT alleles\"", "1", "Integer"},
    {"FORMAT", "GT", "\"Genotype\"", "1", "String"},
    {"FORMAT", "PL", "\"Phred-scaled genotype likelihoods rounded to the closest integer\"", "G", "Integer"},
    {"FORMAT", "GQ", "\"Genotype quality\"", "1", "Integer"},
    {"FORMAT", "DP", "\"Read depth\"", "1", "Integer"},
    {"FORMAT", "ADP", "\"Counts for observed alleles, including the reference allele\"", "R", "Integer"},
    {"FORMAT", "BSDP", "\"Number of base calls (depth) for the 4 nucleotides in called SNVs sorted as A,C,G,T\"", "4", "Integer"},
    {"FORMAT", "ACN", "\"Predicted copy number of each allele taking into account the prediction of number of copies of the region surrounding the variant\"", "R", "Integer"},
};

std::string format_header(const ngsep_ctx* c) {
    c->vcf_known.last_seq = -1;                          // (a new file: its first record is the first of its sequence)
    std::string h = "##fileformat=VCFv4.2\n";
    for (const auto& l : kHeaderLines) {
        h += "##"; h += l[0]; h += "=<ID="; h += l[1]; h += ",Number="; h += l[3];
        h += ",Type="; h += l[4]; h += ",Description="; h += l[2]; h += ">\n";
    }
    if (c->params.print_sample_ploidy)
        h += "##SAMPLE=<ID=" + std::string(c->params.sample_id) + ",PL=" + std::to_string(c->params.ploidy) + ">\n";
    h += "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t";
    h += c->params.sample_id;
    h += "\n";
    return h;
}

static inline int tri(int i, int j) {   // index of L[i][j] in the upper-triangle layout of ngsep_site_out.logc
    if (i > j) { int t = i; i = j; j = t; }
    static const int base[4] = {0, 4, 7, 9};
    return base[i] + (j - i);
}

static void app(std::string& o, long long v) { o += std::to_string(v); }

// GenomicVariantImpl.getVariantTypeName of a -knownVariants record's INFO TYPE, written when 2-5 (VCFFileWriter.java:47-49)
static const char* type_name(int t) {
    static const char* kNames[] = {nullptr, nullptr, "MULTISNV", "EMBEDDED", "INDEL", "STR"};
    return t >= 2 && t <= 5 ? kNames[t] : nullptr;
}

int64_t format_site(const ngsep_ctx* c, const ngsep_site_out& s, std::string& o, bool first_of_seq) {
    static const char kB[] = "ACGT";
    const size_t start = o.size();
    const int ploidy = c->params.ploidy;
    int ri = 0;
    while (ri < 4 && kB[ri] != s.ref) ri++;
    if (ri == 4 || s.n_alleles < 2) return 0;
    const std::string& name = (s.seq_id >= 0 && s.seq_id < (int)c->seq_names.size()) ? c->seq_names[s.seq_id] : std::string("?");
    const ngsep_ctx::KnownVar* kv = known_of(c, s);   // -knownVariants: the input variant (its ID and INFO TYPE)
    const char* id = kv && !kv->id.empty() ? kv->id.c_str() : nullptr;
    const char* ktype = kv ? type_name(kv->type) : nullptr;
    if (s.pool) {
        // ploidy >= 3: genotypeVariantPool's CalledGenomicVariantImpl.  FORMAT NGSEP_NOSNV for discovery (no
        // getAllCounts), NGSEP_SNV for -knownVariants (setAllCounts) (SingleSampleVariantsDetector.java:942-946);
        // QUAL = the variant's QS (never set in discovery, the input's for known variants)
        int dna[4], n = 0;
        dna[n++] = ri;
        for (int a = 0; a < 4; a++) if (((s.pool >> a) & 1) && a != ri) dna[n++] = a;
        const bool known = !c->known.empty();
        const bool report = (s.pool & 0x10) != 0;
        auto index_of = [&](int a) { for (int i = 0; i < n; i++) if (dna[i] == a) return i; return -1; };
        const int nc = s.genotype;                       // called alleles
        const int c0 = nc > 0 ? index_of(s.alt) : -1, c1 = nc > 1 ? index_of(s.third) : -1;
        o += name; o += '\t'; app(o, s.pos); o += '\t'; o += id ? id : "."; o += '\t'; o += (char)s.ref; o += '\t';
        for (int i = 1; i < n; i++) { if (i > 1) o += ','; o += kB[dna[i]]; }
        o += '\t'; app(o, s.qual); o += "\t.\t";
        if (s.is_call & kRecEmbedded) o += "TYPE=EMBEDDED";   // an SNV inside an indel / STR (:227)
        else if (n > 2) o += "TYPE=MULTISNV";             // VCFFileWriter.java:47-49
        else if (ktype) { o += "TYPE="; o += ktype; }
        else o += '.';
        o += known ? "\tGT:PL:GQ:DP:BSDP:ACN\t" : "\tGT:PL:GQ:DP:ADP:ACN\t";
        if (nc == 0) o += "./.";
        else if (nc == 1) { app(o, c0); o += '/'; app(o, c0); }
        else { app(o, c0); o += '/'; app(o, c1); }
        o += ':';
        // PL over the report's log-conditionals (VCFFileWriter.java:200-212), upper triangle i <= j < n
        auto lt = [&](int i, int j) { return s.logc[i * n - i * (i - 1) / 2 + (j - i)]; };
        for (int j = 0; j < n; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) o += ',';
                app(o, report ? (int)java_round(-10 * lt(i, j)) : 0);
            }
        o += ':'; app(o, s.gq); o += ':'; app(o, s.dp); o += ':';
        if (known) for (int k = 0; k < 4; k++) { if (k) o += ','; app(o, s.counts[k]); }
        else for (int i = 0; i < n; i++) { if (i) o += ','; app(o, report ? s.counts[dna[i]] : 0); }
        o += ':';
        // ACN: updateAllelesCopyNumberFromCounts(ploidy) from the report's counts (discoverVariant :226,
        // intersectVariantsCNVs :975 for the first record of a sequence; CalledGenomicVariantImpl.java:228-282); an input
        // record past the first keeps the copy numbers genotypeVariantPool set (:480-498): the device keeps the first
        // called allele's in strand_bias (kernels.hip k_posterior_pool)
        int acn[4] = {0, 0, 0, 0};
        const int called[2] = {c0, c1};
        if (known && !first_of_seq && nc == 2 && s.strand_bias > 0 && s.strand_bias < ploidy) {
            acn[c0] = s.strand_bias;
            acn[c1] = ploidy - s.strand_bias;
        } else if (known && !first_of_seq && nc == 1) acn[c0] = ploidy;
        else if (nc == 1 && c0 == 0) acn[0] = ploidy;
        else if (nc > 0 && ploidy <= nc) { for (int i = 0; i < nc; i++) acn[called[i]] = 1; }
        else if (nc > 0 && !report) {
            const int def = ploidy / nc;
            for (int i = 0; i < nc; i++) acn[called[i]] = def;
            acn[called[0]] += ploidy - def * nc;
        } else if (nc > 0) {
            int rc[2], tr = 0, tc = 0;
            for (int i = 0; i < nc; i++) { rc[i] = s.counts[dna[called[i]]]; if (rc[i] == 0) rc[i] = 1; tr += rc[i]; }
            for (int i = 0; i < nc; i++) {
                const long long r = java_round((double)ploidy * rc[i] / tr);
                acn[called[i]] = (int)(r > 1 ? r : 1);
                tc += acn[called[i]];
            }
            if (tc < ploidy) acn[called[0]] += ploidy - tc;
            else {
                int ex = tc - ploidy;
                for (int i = nc - 1; ex > 0 && i >= 0; i--) {
                    const int rm = ex < acn[called[i]] - 1 ? ex : acn[called[i]] - 1;
                    acn[called[i]] -= rm;
                    ex -= rm;
                }
            }
        }
        if (nc == 0) acn[0] = ploidy;                    // undecided: ACN[0] = the copy number (VCFFileWriter.java:237)
        for (int i = 0; i < n; i++) { if (i) o += ','; app(o, acn[i]); }
        o += '\n';
        return (int64_t)(o.size() - start);
    }
    o += name; o += '\t'; app(o, s.pos); o += '\t'; o += id ? id : "."; o += '\t'; o += (char)s.ref; o += '\t';
    o += kB[(int)s.alt];
    if (s.n_alleles == 3) { o += ','; o += kB[(int)s.third]; }
    o += '\t'; app(o, s.qual); o += "\t.\t";
    // INFO: FS for CalledSNV (SingleSampleVariantsDetector.java:956-958), TYPE for non-SNV types (VCFFileWriter.java:47-49)
    bool printed = false;
    if (s.n_alleles == 2 && s.strand_bias != -1) { o += "FS="; app(o, s.strand_bias); printed = true; }
    if (s.is_call & kRecEmbedded) { if (printed) o += ';'; o += "TYPE=EMBEDDED"; printed = true; }   // -embeddedSNVs (:227)
    else if (s.n_alleles == 3) { if (printed) o += ';'; o += "TYPE=MULTISNV"; printed = true; }
    else if (ktype) { if (printed) o += ';'; o += "TYPE="; o += ktype; printed = true; }
    if (!printed) o += '.';
    o += "\tGT:PL:GQ:DP:BSDP:ACN\t";
    if (s.n_alleles == 2) {
        const int ai = s.alt;
        if (s.genotype == 2) { o += '1'; if (ploidy > 1) o += "/1"; }
        else if (s.genotype == 0) { o += '0'; if (ploidy > 1) o += "/0"; }       // (-knownVariants: hom-ref,
        else if (s.genotype < 0) { o += '.'; if (ploidy > 1) o += "/."; }        //  undecided; VCFFileWriter.java:168-185)
        else o += "0/1";
        o += ':';
        // CalledSNV keeps float log-conditionals (CalledSNV.java:42-45,259-265)
        const float hr = (float)s.logc[tri(ri, ri)], ha = (float)s.logc[tri(ai, ai)];
        const float ra = (float)s.logc[tri(ri, ai)], ar = ra;
        const bool present = (hr + ra + ar + ha) != 0;                  // CalledSNV.java:422
        const double lc[2][2] = {{hr, ra}, {ar, ha}};
        for (int j = 0; j < 2; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) o += ',';
                app(o, present ? (int)java_round(-10 * lc[i][j]) : 0);   // VCFFileWriter.java:203-211
            }
        o += ':'; app(o, s.gq); o += ':'; app(o, s.dp); o += ':';
        for (int k = 0; k < 4; k++) { if (k) o += ','; app(o, s.counts[k]); }
        o += ':';
        // CalledSNV.updateAllelesCopyNumberFromCounts (CalledSNV.java:134-158)
        int total = ploidy, refcn = 0;
        if (s.genotype == 2) refcn = 0;
        else if (s.genotype <= 0) refcn = total;    // hom-ref; undecided: ACN[0] = total (VCFFileWriter.java:237)
        else if (total <= 2) { total = 2; refcn = 1; }
        else {
            double cr = s.counts[ri], sum = cr + s.counts[ai];
            double prop = sum > 0 ? cr / sum : 0.5;
            if (prop > 1) prop = 1;
            refcn = (int16_t)java_round(prop * total);
            if (refcn == 0) refcn = 1;
            else if (refcn >= total) refcn = total - 1;
        }
        if (total == 0) o += '.';
        else { app(o, refcn); o += ','; app(o, total - refcn); }
    } else {
        const int idx[3] = {ri, s.alt, s.third};
        o += "1/2:";
        for (int j = 0; j < 3; j++)
            for (int i = 0; i <= j; i++) {
                if (i > 0 || j > 0) o += ',';
                app(o, (int)java_round(-10 * s.logc[tri(idx[i], idx[j])]));
            }
        o += ':'; app(o, s.gq); o += ':'; app(o, s.dp); o += ':';
        for (int k = 0; k < 4; k++) { if (k) o += ','; app(o, s.counts[k]); }
        o += ':';
        // CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts (:228-282), called alleles {1,2}
        if (ploidy <= 2) o += "0,1,1";
        else {
            int cnt[2], tot = 0;
            for (int i = 0; i < 2; i++) { cnt[i] = s.counts[idx[i + 1]]; if (!cnt[i]) cnt[i] = 1; tot += cnt[i]; }
            int cn[3] = {0, 0, 0}, tc = 0;
            for (int i = 0; i < 2; i++) {
                long long r = java_round((double)ploidy * cnt[i] / tot);
                cn[i + 1] = (int)(r < 1 ? 1 : r);
                tc += cn[i + 1];
            }
            if (tc < ploidy) cn[1] += ploidy - tc;
            else {
                int ex = tc - ploidy;
                for (int i = 2; ex > 0 && i >= 1; i--) { int rm = ex < cn[i] - 1 ? ex : cn[i] - 1; cn[i] -= rm; ex -= rm; }
            }
            app(o, cn[0]); o += ','; app(o, cn[1]); o += ','; app(o, cn[2]);
        }
    }
    o += '\n';
    return (int64_t)(o.size() - start);
}

// record i of the context's site list: an SNV record (format_site), or an indel / STR record's text.  A text with a
// NUL holds two lines: the second is the one written when the record is the first of its sequence (a pool -knownVariants
// record: intersectVariantsCNVs recomputes its ACN from the counts, SingleSampleVariantsDetector.java:969-991)
void format_record(const ngsep_ctx* c, size_t i, std::string& o) {
    const SiteRec& r = c->sites.rec[i];
    const bool first = c->vcf_known.last_seq != r.seq_id;
    c->vcf_known.last_seq = r.seq_id;
    if (r.is_call & kRecIndel) {
        o += (r.seq_id >= 0 && r.seq_id < (int)c->seq_names.size()) ? c->seq_names[(size_t)r.seq_id] : std::string("?");
        o += '\t';
        const std::string& t = c->sites.text[(size_t)SiteSet::ext_index(r)];
        const size_t z = t.find('\0');
        if (z == std::string::npos) o += t;
        else if (first) o.append(t, z + 1, std::string::npos);
        else o.append(t, 0, z);
        return;
    }
    format_site(c, c->sites.full(i), o, first);
}

// ---- MultisampleVariantsDetector output ----
// VCFFileHeader.print with the detector's samples (vcf/VCFFileHeader.java:219-245)
std::string format_population_header(const ngsep_ctx* c) {
    std::string h = "##fileformat=VCFv4.2\n";
    for (const auto& l : kHeaderLines) {
        h += "##"; h += l[0]; h += "=<ID="; h += l[1]; h += ",Number="; h += l[3];
        h += ",Type="; h += l[4]; h += ",Description="; h += l[2]; h += ">\n";
    }
    if (c->params.print_sample_ploidy)
        for (const std::string& id : c->sample_ids) h += "##SAMPLE=<ID=" + id + ",PL=" + std::to_string(c->params.ploidy) + ">\n";
    h += "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT";
    for (const std::string& id : c->sample_ids) { h += '\t'; h += id; }
    h += '\n';
    return h;
}

// DecimalFormat("##0.0#") (main/io/ParseUtils.java:29): HALF_EVEN rounding of the exact binary value
static void app_fmt2(std::string& o, double x) {
    const double p = x * 100.0, err = std::fma(x, 100.0, -p);
    const double k = std::floor(p), fr = p - k;
    long long n = (long long)k;
    if (fr > 0.5 || (fr == 0.5 && (err > 0 || (err == 0 && (n & 1))))) n++;
    char b[48];
    if (n % 10 == 0) std::snprintf(b, sizeof b, "%lld.%lld", n / 100, (n % 100) / 10);
    else std::snprintf(b, sizeof b, "%lld.%02lld", n / 100, n % 100);
    o += b;
}

// VCFFileWriter.printVCFRecord (:44-68) of VCFRecord.createDefaultPopulationVCFRecord: INFO from
// DiversityStatistics.calculateDiversityStatistics(calls, false) (variants/DiversityStatistics.java:123-218)
// in VCFRecord.updateDiversityStatistics order (NS, AN, AFS, OH, MAF; vcf/VCFRecord.java:288-301),
// then TYPE; FORMAT GT:PL:GQ:DP:BSDP:ACN per sample (printGenotypeInfo, :159-308)
void format_population_site(const ngsep_ctx* c, const ngsep_popsite_out& s, const ngsep_sample_call* calls, std::string& o) {
    static const char kB[] = "ACGT";
    const int S = (int)c->sample_ids.size();
    const int ploidy = c->params.ploidy;
    const std::string& name = (s.seq_id >= 0 && s.seq_id < (int)c->seq_names.size()) ? c->seq_names[s.seq_id] : std::string("?");
    // -knownVariants: the input variant's ID (MultisampleVariantsDetector.java:543-545 writes the input variant)
    const ngsep_ctx::KnownVar* kv = s.n_alleles == 2 ? known_at(c, s.seq_id, s.pos, s.alleles[1]) : nullptr;
    const char* id = kv && !kv->id.empty() ? kv->id.c_str() : nullptr;
    o += name; o += '\t'; app(o, s.pos); o += '\t'; o += id ? id : "."; o += '\t'; o += kB[(int)s.alleles[0]]; o += '\t';
    for (int i = 1; i < s.n_alleles; i++) { if (i > 1) o += ','; o += kB[(int)s.alleles[i]]; }
    o += '\t'; app(o, s.qual); o += "\t.\t";
    int counts[4] = {0, 0, 0, 0}, sum = 0, ng = 0, nhet = 0;
    for (int k = 0; k < S; k++) {
        const ngsep_sample_call& cl = calls[k];
        if (cl.n_called == 0) continue;
        ng++;
        if (cl.n_called > 1) nhet++;
        for (int i = 0; i < cl.n_called; i++) { const int j = cl.called[i]; counts[j] += cl.acn[j]; sum += cl.acn[j]; }
    }
    int ncalled = 0, minAC = 0;
    for (int i = 0; i < s.n_alleles; i++)
        if (counts[i] > 0) { ncalled++; if (minAC == 0 || minAC > counts[i]) minAC = counts[i]; }
    o += "NS="; app(o, ng); o += ";AN="; app(o, ncalled); o += ";AFS=";
    for (int i = 0; i < s.n_alleles; i++) { if (i) o += ','; app(o, counts[i]); }
    o += ";OH="; app_fmt2(o, ng > 0 ? (double)nhet / ng : 0.0);
    if (s.n_alleles == 2) { o += ";MAF="; app_fmt2(o, ncalled < 2 ? 0.0 : (double)minAC / sum); }
    if (s.multisnv_type == 2) o += ";TYPE=EMBEDDED";        // an SNV inside an indel / STR (MultisampleVariantsDetector.java:581)
    else if (s.multisnv_type) o += ";TYPE=MULTISNV";
    else if (kv && type_name(kv->type)) { o += ";TYPE="; o += type_name(kv->type); }   // an input record's TYPE
    o += "\tGT:PL:GQ:DP:BSDP:ACN";
    for (int k = 0; k < S; k++) {
        const ngsep_sample_call& cl = calls[k];
        o += '\t';
        if (cl.n_called == 0) o += ploidy > 1 ? "./." : ".";
        else if (cl.n_called == 1) { app(o, cl.called[0]); if (ploidy > 1) { o += '/'; app(o, cl.called[0]); } }
        else { app(o, cl.called[0]); o += '/'; app(o, cl.called[1]); }
        o += ':';
        const int npl = s.n_alleles * (s.n_alleles + 1) / 2;
        for (int i = 0; i < npl; i++) { if (i) o += ','; app(o, cl.pl[i]); }
        o += ':'; app(o, cl.gq); o += ':'; app(o, cl.dp); o += ':';
        for (int i = 0; i < 4; i++) { if (i) o += ','; app(o, cl.counts[i]); }
        o += ':';
        if (cl.total_cn == 0) o += '.';
        else {
            const int nal = cl.kind == 0 ? 2 : s.n_alleles;
            for (int j = 0; j < nal; j++) {
                if (j) o += ',';
                app(o, (cl.n_called == 0 && j == 0) ? cl.total_cn : cl.acn[j]);
            }
        }
    }
    o += '\n';
}

// an indel / STR population record (multisnv_type 3, the realigner regions, engine.cpp run_population_regions): its
// text appended; false for any other record
bool append_population_text(const ngsep_ctx* c, size_t i, std::string& o) {
    const ngsep_popsite_out& s = c->pop_sites[i];
    if (s.multisnv_type != 3) return false;
    o += (s.seq_id >= 0 && s.seq_id < (int)c->seq_names.size()) ? c->seq_names[(size_t)s.seq_id] : std::string("?");
    o += '\t';
    o += c->pop_text[(size_t)c->pop_order[i]];
    return true;
}

}  // namespace ngsep

using namespace ngsep;

extern "C" int64_t ngsep_population_site_vcf_line(ngsep_ctx* c, int64_t i, char* buf, int64_t cap) {
    if (!c || i < 0 || i >= (int64_t)c->pop_sites.size()) return NGSEP_E_INVALID;
    std::string o;
    if (!append_population_text(c, (size_t)i, o)) {
        const size_t S = c->sample_ids.size();
        std::vector<ngsep_sample_call> calls(S);
        for (size_t k = 0; k < S; k++) calls[k] = expand_call(c->pop_calls.data()[(size_t)c->pop_order[(size_t)i] * S + k], c->pop_big.data());
        format_population_site(c, c->pop_sites[(size_t)i], calls.data(), o);
    }
    if (buf && cap > 0) {
        const int64_t k = std::min<int64_t>((int64_t)o.size(), cap - 1);
        std::memcpy(buf, o.data(), (size_t)k);
        buf[k] = 0;
    }
    return (int64_t)o.size();
}

extern "C" int ngsep_write_population_vcf(ngsep_ctx* c, const char* path) {
    if (!c || !path) return NGSEP_E_INVALID;
    std::FILE* f = std::fopen(path, "w");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot write ") + path);
    std::string buf = format_population_header(c);
    const size_t S = c->sample_ids.size();
    std::vector<ngsep_sample_call> calls(S);
    for (size_t i = 0; i < c->pop_sites.size(); i++) {
        if (append_population_text(c, i, buf)) { if (buf.size() > (1 << 20)) { std::fwrite(buf.data(), 1, buf.size(), f); buf.clear(); } continue; }
        for (size_t k = 0; k < S; k++) calls[k] = expand_call(c->pop_calls.data()[(size_t)c->pop_order[i] * S + k], c->pop_big.data());
        format_population_site(c, c->pop_sites[i], calls.data(), buf);
        if (buf.size() > (1 << 20)) { std::fwrite(buf.data(), 1, buf.size(), f); buf.clear(); }
    }
    std::fwrite(buf.data(), 1, buf.size(), f);
    std::fclose(f);
    return NGSEP_OK;
}

extern "C" int ngsep_write_vcf_header(ngsep_ctx* c, const char* path) {
    if (!c || !path) return NGSEP_E_INVALID;
    std::FILE* f = std::fopen(path, "w");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot write ") + path);
    std::string h = format_header(c);
    std::fwrite(h.data(), 1, h.size(), f);
    std::fclose(f);
    return NGSEP_OK;
}

extern "C" int ngsep_append_vcf_records(ngsep_ctx* c, const char* path) {
    if (!c || !path) return NGSEP_E_INVALID;
    std::FILE* f = std::fopen(path, "a");
    if (!f) return set_error(c, NGSEP_E_IO, std::string("cannot write ") + path);
    std::string buf;
    buf.reserve(1 << 20);
    for (size_t i = 0; i < c->sites.size(); i++) {
        if (!(c->sites.rec[i].is_call & kRecCall)) continue;
        format_record(c, i, buf);
        if (buf.size() > (1 << 20)) { std::fwrite(buf.data(), 1, buf.size(), f); buf.clear(); }
    }
    std::fwrite(buf.data(), 1, buf.size(), f);
    std::fclose(f);
    c->sites.clear();
    return NGSEP_OK;
}

extern "C" int64_t ngsep_site_vcf_line(ngsep_ctx* c, int64_t i, char* buf, int64_t cap) {
    if (!c || i < 0 || i >= (int64_t)c->sites.size()) return NGSEP_E_INVALID;
    std::string o;
    format_record(c, (size_t)i, o);
    if (buf && cap > 0) {
        const int64_t k = std::min<int64_t>((int64_t)o.size(), cap - 1);
        std::memcpy(buf, o.data(), (size_t)k);
        buf[k] = 0;
    }
    return (int64_t)o.size();
}

extern "C" int64_t ngsep_format_site(ngsep_ctx* c, const ngsep_site_out* s, char* buf, int64_t cap) {
    if (!c || !s) return NGSEP_E_INVALID;
    std::string o;
    int64_t n = format_site(c, *s, o, true);
    if (buf && cap > 0) {
        int64_t k = std::min<int64_t>(n, cap - 1);
        std::memcpy(buf, o.data(), (size_t)k);
        buf[k] = 0;
    }
    return n;
}
