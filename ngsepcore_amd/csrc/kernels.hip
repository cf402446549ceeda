// kernels.hip -- gfx950 kernels of the NGSEP SNV pileup path.
//
//   K1  k1_candidate_scan : streams every projected read byte once (16 B per lane, fixed-stride
//                           slots, coalesced), compares it with the reference code of its position
//                           and marks positions that carry a valid non-reference call.  This is the
//                           pileup sweep of AlignmentsPileupGenerator.processCurrentPosition
//                           (discovery/AlignmentsPileupGenerator.java:475-498) reduced to the only
//                           fact that decides whether SNVQ can call a variant there.
//   K2  k2_genotype       : for each marked position, CountsHelper.calculateCountsSNV/updateCounts
//                           (discovery/CountsHelper.java:83-95,209-251) in pending-list order (bit-exact
//                           fp64 sums), getPosteriorProbabilities (:410-495), and
//                           VariantDiscoverySNVQAlgorithm.discoverSNV (:100-243) with the listener's
//                           filters (SingleSampleVariantPileupListener.java:213-232).
//   KL  kl_read_index     : per 64-position block, first read that can cover it (binary search).
//
// HBM-bound integer/byte work: no MFMA.  Memory layout is described in DESIGN.md.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "engine.hpp"

namespace ngsep {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);                   \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

struct Device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {};
    uint8_t* d_slots = nullptr;
    int32_t* d_slot_pos = nullptr;
    int4* d_reads = nullptr;
    uint8_t* d_ref = nullptr;
    uint32_t* d_bitmap = nullptr;
    int32_t* d_lb = nullptr;
    LikTables* d_tables = nullptr;
    ngsep_site_out* d_sites = nullptr;
    unsigned long long* d_counters = nullptr;
    ngsep_site_out* h_sites = nullptr;   // pinned
    unsigned long long* h_counters = nullptr;
    int64_t cap_sites = 0, cap_h_sites = 0;
    int64_t n_units = 0, n_words = 0, n_lb = 0, n_reads = 0, g_len = 0;
    int32_t slot_size = 0, max_span = 0;
};

// ------------------------------------------------------------------------------------------
// K1: candidate scan over the slot array
// ------------------------------------------------------------------------------------------
// MODE 0: valid call (code bit7) whose allele differs from a callable reference base.
// MODE 1: any counted call at an in-window position (genotype every position).
template <int MODE>
__global__ __launch_bounds__(256) void k1_candidate_scan(const u32x4* __restrict__ slots,
                                                         const int32_t* __restrict__ slot_pos,
                                                         const uint8_t* __restrict__ ref,
                                                         uint32_t* __restrict__ bitmap,
                                                         int64_t n_units, uint32_t units_per_slot,
                                                         int64_t chunk) {
    const int64_t begin = (int64_t)blockIdx.x * chunk;
    int64_t end = begin + chunk;
    if (end > n_units) end = n_units;
    int64_t u = begin + threadIdx.x;
    if (u >= end) return;
    // unit -> (slot, unit-in-slot), advanced incrementally by blockDim per step
    uint32_t slot = (uint32_t)(u / units_per_slot);
    uint32_t j = (uint32_t)(u - (int64_t)slot * units_per_slot);
    const uint32_t ds = 256u / units_per_slot, dj = 256u - ds * units_per_slot;
    const uint32_t* refw = reinterpret_cast<const uint32_t*>(ref);
    for (; u < end; u += 256) {
        const u32x4 d = __builtin_nontemporal_load(&slots[u]);
        uint32_t any = d.x | d.y | d.z | d.w;
        if (MODE == 0) any &= 0x80808080u;
        if (any) {
            const int32_t p0 = slot_pos[slot] + 16 * (int32_t)j;     // global position of byte 0
            const uint32_t* rw = refw + (p0 >> 2);
            const uint32_t sh = (uint32_t)(p0 & 3);
            const uint32_t r0 = rw[0], r1 = rw[1], r2 = rw[2], r3 = rw[3], r4 = rw[4];
            const uint32_t R[4] = {__builtin_amdgcn_alignbyte(r1, r0, sh), __builtin_amdgcn_alignbyte(r2, r1, sh),
                                   __builtin_amdgcn_alignbyte(r3, r2, sh), __builtin_amdgcn_alignbyte(r4, r3, sh)};
            const uint32_t D[4] = {d.x, d.y, d.z, d.w};
            uint32_t mask = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                uint32_t c;
                if (MODE == 0) {
                    // per byte: valid call & callable ref & allele bits differ
                    const uint32_t diff = ((D[k] ^ R[k]) & 0x60606060u) + 0x60606060u;
                    c = D[k] & R[k] & diff & 0x80808080u;
                } else {
                    const uint32_t nzd = (((D[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | D[k]) & 0x80808080u;
                    const uint32_t nzr = (((R[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | R[k]) & 0x80808080u;
                    c = nzd & nzr;
                }
                const uint32_t m = ((c >> 7) & 1u) | ((c >> 14) & 2u) | ((c >> 21) & 4u) | ((c >> 28) & 8u);
                mask |= m << (4 * k);
            }
            if (mask) {
                const uint64_t m64 = (uint64_t)mask << (p0 & 31);
                atomicOr(&bitmap[p0 >> 5], (uint32_t)m64);
                if (m64 >> 32) atomicOr(&bitmap[(p0 >> 5) + 1], (uint32_t)(m64 >> 32));
            }
        }
        j += dj;
        slot += ds;
        if (j >= units_per_slot) { j -= units_per_slot; slot++; }
    }
}

// ------------------------------------------------------------------------------------------
// KL: lb[k] = first read index whose gfirst >= 64k - max_span + 1
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void kl_read_index(const int4* __restrict__ reads, int64_t n_reads,
                                                     int32_t* __restrict__ lb, int64_t n_lb, int32_t max_span) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_lb) return;
    const int64_t key = k * 64 - max_span + 1;
    int64_t lo = 0, hi = n_reads;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((int64_t)reads[mid].x < key) lo = mid + 1;
        else hi = mid;
    }
    lb[k] = (int32_t)lo;
}

// ------------------------------------------------------------------------------------------
// K2: genotype marked positions
// ------------------------------------------------------------------------------------------
__device__ inline int64_t java_round_d(double x) {
    if (isnan(x)) return 0;
    double f = floor(x);
    return (int64_t)((x - f >= 0.5) ? f + 1.0 : f);
}
// PhredScoreHelper.calculatePhredScore (math/PhredScoreHelper.java:31-40)
__device__ inline int16_t phred_d(double p) {
    if (p == 0) return 255;
    double score = -10 * log10(p);
    if (score > 255) return 255;
    return (int16_t)java_round_d(score);
}

__global__ __launch_bounds__(256) void k2_genotype(const uint32_t* __restrict__ bitmap, int64_t n_words,
                                                   const uint8_t* __restrict__ ref, const int4* __restrict__ reads,
                                                   int64_t n_reads, const int32_t* __restrict__ lb,
                                                   const uint8_t* __restrict__ slots, int32_t S,
                                                   const LikTables* __restrict__ T, GenotypeParams gp,
                                                   ngsep_site_out* __restrict__ out, unsigned long long* counters,
                                                   int64_t cap) {
    const int64_t word = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (word >= n_words) return;
    uint32_t w = bitmap[word];
    if (w) atomicAdd(&counters[1], (unsigned long long)__popc(w));
    while (w) {
        const int b = __builtin_ctz(w);
        w &= w - 1;
        const int32_t gpos = (int32_t)(word * 32 + b);
        const uint8_t rc = ref[gpos];
        // CountsHelper.calculateCountsSNV over PileupRecord.getAlleleCalls(1) in pending order
        int32_t total = 0;
        int32_t cnt[4] = {0, 0, 0, 0};
        int32_t sc[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        double L00 = 0, L01 = 0, L02 = 0, L03 = 0, L11 = 0, L12 = 0, L13 = 0, L22 = 0, L23 = 0, L33 = 0;
        for (int64_t r = lb[gpos >> 6]; r < n_reads; r++) {
            const int4 h = reads[r];            // gfirst, glast, slot, flags
            if (h.x > gpos) break;
            if (h.y < gpos) continue;
            const int32_t off = gpos - h.x;
            const int32_t sidx = off / S;
            const uint8_t code = slots[(int64_t)(h.z + sidx) * S + (off - sidx * S)];
            if (!code) continue;                // no allele call from this read
            total++;                            // CountsHelper.java:210
            if (!(code & 0x80)) continue;       // q<=3 or not A/C/G/T (:214-221)
            const int a = (code >> 5) & 3;
            int q = code & 31;
            if (q > gp.max_q) q = gp.max_q;     // :217-219
            cnt[a]++;
            if (h.w & 1) sc[a][0]++; else sc[a][1]++;
            const double A = T->A[q], E = T->E[q], H = T->H[q];
            // updateCounts (:231-248) with f == g: the [i][j] and [j][i] sums are identical sequences
            L00 += a == 0 ? A : E;
            L11 += a == 1 ? A : E;
            L22 += a == 2 ? A : E;
            L33 += a == 3 ? A : E;
            L01 += (a == 0 || a == 1) ? H : E;
            L02 += (a == 0 || a == 2) ? H : E;
            L03 += (a == 0 || a == 3) ? H : E;
            L12 += (a == 1 || a == 2) ? H : E;
            L13 += (a == 1 || a == 3) ? H : E;
            L23 += (a == 2 || a == 3) ? H : E;
        }
        if (total == 0) continue;               // VariantDiscoverySNVQAlgorithm.java:101-103
        const bool callable = (rc & 0x80) != 0;
        int8_t genotype = -1, alt = -1, third = -1, nal = 0;
        int16_t gq = 0, qual = 0;
        bool keep = false;
        if (callable) {
            const int refIdx = (rc >> 5) & 3;
            // getPosteriorProbabilities (:410-443): events in Java order
            const double ph = gp.log_prior_homo, px = gp.log_prior_hetero;
            double ev[16] = {L00 + ph, L01 + px, L02 + px, L03 + px,
                             L11 + ph, L01 + px, L12 + px, L13 + px,
                             L22 + ph, L02 + px, L12 + px, L23 + px,
                             L33 + ph, L03 + px, L13 + px, L23 + px};
            // calculatePosteriorProbabilities (:472-495)
            double logMax = 1;
#pragma unroll
            for (int i = 0; i < 16; i++)
                if (logMax > 0 || logMax < ev[i]) logMax = ev[i];
            double totalProb = 0;
#pragma unroll
            for (int i = 0; i < 16; i++) {
                ev[i] -= logMax;
                ev[i] = ev[i] < -20 ? 0.0 : pow(10.0, ev[i]);
                totalProb += ev[i];
            }
#pragma unroll
            for (int i = 0; i < 16; i++) ev[i] = ev[i] / totalProb;
            // post(i,j) lives at 4i (diagonal) or 4i+1+j (j<i) or 4i+j (j>i)
#define POST(i, j) ev[(i) == (j) ? 4 * (i) : ((j) < (i) ? 4 * (i) + 1 + (j) : 4 * (i) + (j))]
            // getIndexesMaxGenotype (VariantDiscoverySNVQAlgorithm.java:223-243)
            int I = refIdx, J = refIdx;
            double probMax = POST(refIdx, refIdx);
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = i; j < 4; j++) {
                    double g = POST(i, j);
                    if (i != j) g += POST(j, i);
                    if (g > probMax + 0.01) { probMax = g; I = i; J = j; }
                }
            const double refProb = POST(refIdx, refIdx);
            double maxP = 0;
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (i == I && j == J) maxP = POST(i, j);
            if (I != J) {
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (i == J && j == I) maxP += POST(i, j);
            }
            gq = phred_d(1 - maxP);
            qual = phred_d(refProb);
            if (I != J && I != refIdx && J != refIdx) {
                // triallelic (:128-177)
                double pII = 0, pJJ = 0;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    if (i == I) pII = POST(i, i);
                    if (i == J) pJJ = POST(i, i);
                }
                if (pII > pJJ + 0.01) { alt = (int8_t)I; third = (int8_t)J; }
                else { alt = (int8_t)J; third = (int8_t)I; }
                nal = 3;
                genotype = 3;
                keep = true;
            } else if (I != J) {
                alt = (int8_t)(refIdx != I ? I : J);
                nal = 2;
                genotype = 1;
                keep = true;
            } else if (refIdx != I) {
                alt = (int8_t)I;
                nal = 2;
                genotype = 2;
                keep = true;
            } else {
                genotype = 0;   // homozygous reference: dropped (SingleSampleVariantPileupListener.java:223)
                nal = 1;
            }
#undef POST
            if (keep && gp.min_quality > gq) keep = false;
        }
        if (!keep && !gp.dump_all) continue;
        const unsigned long long idx = atomicAdd(&counters[0], 1ull);
        if ((int64_t)idx >= cap) continue;
        ngsep_site_out o;
        o.seq_id = -1;
        o.pos = gpos;
        o.ref = callable ? "ACGT"[(rc >> 5) & 3] : 'N';
        o.n_alleles = nal;
        o.alt = alt;
        o.third = third;
        o.genotype = genotype;
        o.strand_bias = -1;
        o.gq = gq;
        o.qual = qual;
        o.is_call = keep ? 1 : 0;
        o.dp = total;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            o.counts[i] = cnt[i];
            o.strand_counts[i][0] = sc[i][0];
            o.strand_counts[i][1] = sc[i][1];
        }
        o.logc[0] = L00; o.logc[1] = L01; o.logc[2] = L02; o.logc[3] = L03; o.logc[4] = L11;
        o.logc[5] = L12; o.logc[6] = L13; o.logc[7] = L22; o.logc[8] = L23; o.logc[9] = L33;
        out[idx] = o;
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
int device_count() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

Device* device_create(int ordinal, std::string& err) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        err = "no HIP device available (libngsep_amd requires an MI355X / gfx950 GPU)";
        return nullptr;
    }
    if (ordinal < 0 || ordinal >= n) { err = "device ordinal out of range"; return nullptr; }
    if (hipSetDevice(ordinal) != hipSuccess) { err = "hipSetDevice failed"; return nullptr; }
    Device* d = new Device();
    d->ordinal = ordinal;
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) { err = "stream"; delete d; return nullptr; }
    for (auto& e : d->ev) (void)hipEventCreate(&e);
    if (hipMalloc(&d->d_counters, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&d->h_counters, 2 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&d->d_tables, sizeof(LikTables)) != hipSuccess) {
        err = "device allocation failed";
        delete d;
        return nullptr;
    }
    return d;
}

void device_release(Device* d) {
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    (void)hipFree(d->d_slots); d->d_slots = nullptr;
    (void)hipFree(d->d_slot_pos); d->d_slot_pos = nullptr;
    (void)hipFree(d->d_reads); d->d_reads = nullptr;
    (void)hipFree(d->d_ref); d->d_ref = nullptr;
    (void)hipFree(d->d_bitmap); d->d_bitmap = nullptr;
    (void)hipFree(d->d_lb); d->d_lb = nullptr;
    d->n_units = d->n_words = d->n_lb = d->n_reads = d->g_len = 0;
}

void device_destroy(Device* d) {
    if (!d) return;
    device_release(d);
    (void)hipFree(d->d_sites);
    (void)hipFree(d->d_counters);
    (void)hipFree(d->d_tables);
    (void)hipHostFree(d->h_sites);
    (void)hipHostFree(d->h_counters);
    for (auto& e : d->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(d->stream);
    delete d;
}

int device_upload(Device* d, const Staged& s, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    device_release(d);
    const int S = s.slot_size;
    const int64_t slot_bytes = s.n_slots * (int64_t)S;
    HIP_TRY(hipMalloc(&d->d_slots, (size_t)std::max<int64_t>(slot_bytes, 16)));
    HIP_TRY(hipMalloc(&d->d_slot_pos, (size_t)std::max<int64_t>(s.n_slots, 1) * 4));
    HIP_TRY(hipMalloc(&d->d_reads, (size_t)std::max<int64_t>(s.n_reads, 1) * sizeof(int4)));
    HIP_TRY(hipMalloc(&d->d_ref, (size_t)s.g_len + 64));
    d->n_words = (s.g_len + 31) / 32 + 2;
    HIP_TRY(hipMalloc(&d->d_bitmap, (size_t)d->n_words * 4));
    d->n_lb = (s.g_len + 63) / 64 + 1;
    HIP_TRY(hipMalloc(&d->d_lb, (size_t)d->n_lb * 4));
    if (slot_bytes) HIP_TRY(hipMemcpyAsync(d->d_slots, s.h_slots.data(), (size_t)slot_bytes, hipMemcpyHostToDevice, d->stream));
    if (s.n_slots) HIP_TRY(hipMemcpyAsync(d->d_slot_pos, s.h_slot_pos.data(), (size_t)s.n_slots * 4, hipMemcpyHostToDevice, d->stream));
    if (s.n_reads) HIP_TRY(hipMemcpyAsync(d->d_reads, s.h_reads.data(), (size_t)s.n_reads * 16, hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemsetAsync(d->d_ref, 0, (size_t)s.g_len + 64, d->stream));
    HIP_TRY(hipMemcpyAsync(d->d_ref, s.h_ref.data(), (size_t)s.g_len, hipMemcpyHostToDevice, d->stream));
    d->n_units = slot_bytes / 16;
    d->n_reads = s.n_reads;
    d->g_len = s.g_len;
    d->slot_size = S;
    d->max_span = s.max_span;
    const int64_t pad = s.windows.empty() ? 64 : s.windows[0].pad;
    {
        dim3 grid((unsigned)((d->n_lb + 255) / 256));
        hipLaunchKernelGGL(kl_read_index, grid, dim3(256), 0, d->stream, d->d_reads, d->n_reads, d->d_lb, d->n_lb, (int32_t)pad);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(d->stream));
    return 0;
}

int device_run(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune,
               std::vector<ngsep_site_out>& out, double* scan_ms, double* geno_ms, double* total_ms,
               int64_t* n_candidates, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    auto t0 = std::chrono::steady_clock::now();
    // output capacity: calls are rare; dump mode needs one record per covered position
    int64_t want = g.dump_all ? std::max<int64_t>(s.covered + 1024, 1024) : std::max<int64_t>(s.g_len / 256 + 4096, 4096);
    if (want > d->cap_sites) {
        (void)hipFree(d->d_sites);
        (void)hipHostFree(d->h_sites);
        HIP_TRY(hipMalloc(&d->d_sites, (size_t)want * sizeof(ngsep_site_out)));
        HIP_TRY(hipHostMalloc(&d->h_sites, (size_t)want * sizeof(ngsep_site_out), hipHostMallocDefault));
        d->cap_sites = want;
    }
    HIP_TRY(hipMemcpyAsync(d->d_tables, &t, sizeof(LikTables), hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemsetAsync(d->d_counters, 0, 2 * sizeof(unsigned long long), d->stream));
    HIP_TRY(hipMemsetAsync(d->d_bitmap, 0, (size_t)d->n_words * 4, d->stream));
    HIP_TRY(hipEventRecord(d->ev[0], d->stream));
    if (d->n_units > 0) {
        const uint32_t ups = (uint32_t)(d->slot_size / 16);
        int64_t blocks = (d->n_units + 256 * 16 - 1) / (256 * 16);
        blocks = std::min<int64_t>(std::max<int64_t>(blocks, 1), 8192);
        int64_t chunk = (d->n_units + blocks - 1) / blocks;
        chunk = (chunk + 255) / 256 * 256;
        blocks = (d->n_units + chunk - 1) / chunk;
        if (prune)
            hipLaunchKernelGGL(k1_candidate_scan<0>, dim3((unsigned)blocks), dim3(256), 0, d->stream,
                               (const u32x4*)d->d_slots, d->d_slot_pos, d->d_ref, d->d_bitmap, d->n_units, ups, chunk);
        else
            hipLaunchKernelGGL(k1_candidate_scan<1>, dim3((unsigned)blocks), dim3(256), 0, d->stream,
                               (const u32x4*)d->d_slots, d->d_slot_pos, d->d_ref, d->d_bitmap, d->n_units, ups, chunk);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(d->ev[1], d->stream));
    {
        dim3 grid((unsigned)((d->n_words + 255) / 256));
        hipLaunchKernelGGL(k2_genotype, grid, dim3(256), 0, d->stream, d->d_bitmap, d->n_words, d->d_ref, d->d_reads,
                           d->n_reads, d->d_lb, d->d_slots, d->slot_size, d->d_tables, g, d->d_sites, d->d_counters,
                           d->cap_sites);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipEventRecord(d->ev[2], d->stream));
    HIP_TRY(hipMemcpyAsync(d->h_counters, d->d_counters, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    int64_t n = (int64_t)d->h_counters[0];
    if (n > d->cap_sites) { err = "site buffer overflow"; return -1; }
    if (n > 0) {
        HIP_TRY(hipMemcpyAsync(d->h_sites, d->d_sites, (size_t)n * sizeof(ngsep_site_out), hipMemcpyDeviceToHost, d->stream));
        HIP_TRY(hipStreamSynchronize(d->stream));
    }
    out.assign(d->h_sites, d->h_sites + n);
    auto t1 = std::chrono::steady_clock::now();
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, d->ev[0], d->ev[1]);
    (void)hipEventElapsedTime(&b, d->ev[1], d->ev[2]);
    *scan_ms = a;
    *geno_ms = b;
    *total_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    *n_candidates = (int64_t)d->h_counters[1];
    return 0;
}

}  // namespace ngsep
