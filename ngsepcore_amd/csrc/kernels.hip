// kernels.hip -- gfx950 kernels of the NGSEP SNV pileup path.
//
//   KT  k_tile_pileup : one workgroup per tile of T reference positions (global coordinates).
//        phase 1  stage the tile's read slots HBM -> LDS (global_load_lds, 16 B per lane; the slots
//                 of the reads overlapping a tile are one contiguous range) and compare every
//                 projected read byte with the reference code of its position: a position whose
//                 pileup holds a valid non-reference call becomes a candidate (LDS bitmap).  This is
//                 AlignmentsPileupGenerator.processCurrentPosition (discovery/AlignmentsPileupGenerator.java:475-498)
//                 reduced to the fact that decides whether SNVQ can call a variant there
//                 ("why pruning is exact").
//        phase 2  integer hom-ref bound of every candidate (order-independent LDS atomics).
//        phase 3  drop the candidates the bound proves hom-ref, queue the rest.
//        Tiles whose reads do not fit the LDS budget scan from global memory and queue every candidate.
//   KP  k_posterior : exact CountsHelper tally (pending-list order, bit-exact fp64), posterior and
//                 SNVQ call of the queued candidates (discovery/CountsHelper.java:83-95,209-251,410-495,
//                 VariantDiscoverySNVQAlgorithm.java:100-243, SingleSampleVariantPileupListener.java:213-232).
//   KL  kl_read_index : per 64-position block, first read that can cover it (binary search).
//   KO  ko_* : position order of the emitted records.
//
// HBM-bound integer/byte work: no MFMA.  Layout and roofline: DESIGN.md.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
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

struct QueueSite;

struct Device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {};
    uint8_t* d_slots = nullptr;
    uint8_t* d_pile = nullptr;
    int4* d_reads = nullptr;
    uint8_t* d_ref = nullptr;
    int32_t* d_lb = nullptr;
    TileInfo* d_tinfo = nullptr;
    LikTables* d_tables = nullptr;
    ngsep_site_out* d_sites = nullptr;
    ngsep_site_out* d_sorted = nullptr;
    int32_t* d_bucket = nullptr;     // counts, then starts (nb+1), then cursors (nb)
    int64_t nb_cap = 0;
    QueueSite* d_hard = nullptr;
    int64_t cap_hard = 0;
    unsigned long long* d_counters = nullptr;
    unsigned long long* h_counters = nullptr;
    int64_t cap_sites = 0;
    int64_t n_units = 0, n_slots = 0, n_lb = 0, n_reads = 0, g_len = 0, n_tiles = 0;
    int32_t slot_size = 0, max_span = 0, pad = 0, tile = 512, log2_tile = 9;
    int64_t last_n_sites = 1024;
    int64_t last_hard = 0;
    int32_t n_cu = 256;
};

// ------------------------------------------------------------------------------------------
// helpers
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

// bit 7 of the four bytes of a dword -> 4 bits
__device__ inline uint32_t nib4(uint32_t w) {
    const uint32_t c = w & 0x80808080u;
    return ((c >> 7) & 1u) | ((c >> 14) & 2u) | ((c >> 21) & 4u) | ((c >> 28) & 8u);
}
// bit k set <=> byte k of a 16-byte unit has bit 7 (a valid call)
__device__ inline uint32_t unit_valid_mask(const u32x4 d) {
    return nib4(d.x) | (nib4(d.y) << 4) | (nib4(d.z) << 8) | (nib4(d.w) << 12);
}
// byte k (0..15) of a 16-byte unit
__device__ inline uint32_t unit_byte(const u32x4 d, int k) {
    const uint32_t w = k < 8 ? (k < 4 ? d.x : d.y) : (k < 12 ? d.z : d.w);
    return (w >> (8 * (k & 3))) & 0xFFu;
}

// A candidate the tile kernel could not prove hom-ref; k_posterior genotypes it exactly
struct QueueSite {
    int32_t gpos;          // global position
    int32_t rc;            // reference code
};
static_assert(sizeof(QueueSite) == 8, "QueueSite layout");

constexpr int kCandCap = 256;   // candidates per tile with integer-bound accumulators in LDS
constexpr int kTileBlocksPerCU = 4;
constexpr int kQueueStage = 1024;    // survivors staged in LDS per tile-scan block   // persistent tile-scan blocks per CU (register-limited occupancy)

// ------------------------------------------------------------------------------------------
// KP: exact tally + posterior + SNVQ call of the queued candidates (thread per site)
// ------------------------------------------------------------------------------------------
// CountsHelper.calculateCountsSNV/updateCounts (discovery/CountsHelper.java:83-95,209-251) over the
// reads covering gpos in pending-list order (the order of the read table), so the fp64 sums are
// bit-identical to the reference's; then getPosteriorProbabilities (:410-495),
// VariantDiscoverySNVQAlgorithm.discoverSNV (:100-243) and the listener filters
// (SingleSampleVariantPileupListener.java:213-232).
__global__ __launch_bounds__(256) void k_posterior(const QueueSite* __restrict__ queue, const unsigned long long* qn,
                                                   int64_t qcap, const int4* __restrict__ reads, int64_t n_reads,
                                                   const int32_t* __restrict__ lb, const uint8_t* __restrict__ slots,
                                                   int32_t S, const LikTables* __restrict__ tabs, GenotypeParams gp,
                                                   ngsep_site_out* __restrict__ out, unsigned long long* counters,
                                                   int64_t cap) {
    __shared__ double s_t[3][32];
    if (threadIdx.x < 96)
        s_t[threadIdx.x >> 5][threadIdx.x & 31] =
            (threadIdx.x < 32 ? tabs->A : threadIdx.x < 64 ? tabs->H : tabs->E)[threadIdx.x & 31];
    __syncthreads();
    int64_t n = (int64_t)*qn;
    if (n > qcap) n = qcap;
    auto site = [&](int64_t i, ngsep_site_out& o) -> bool {
        const QueueSite qs = queue[i];
        const int32_t gpos = qs.gpos;
        const uint8_t rc = (uint8_t)qs.rc;
        int32_t total = 0;
        uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        int32_t sc[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        double L00 = 0, L01 = 0, L02 = 0, L03 = 0, L11 = 0, L12 = 0, L13 = 0, L22 = 0, L23 = 0, L33 = 0;
        // reads that can cover gpos start at lb[gpos/64] (every earlier read ends before gpos)
        bool more = true;
        for (int64_t r0 = lb[gpos >> 6]; more && r0 < n_reads; r0 += 8) {
            int4 h[8];
#pragma unroll
            for (int k = 0; k < 8; k++) h[k] = reads[r0 + k < n_reads ? r0 + k : n_reads - 1];
            uint8_t code[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const bool in = r0 + k < n_reads && h[k].x <= gpos;
                if (!in) more = false;
                const int32_t off = gpos - h[k].x;
                const bool cov = in && h[k].y >= gpos;
                const int32_t o = cov ? off : 0;
                const uint8_t cd = slots[(int64_t)(h[k].z + o / S) * S + (o % S)];
                code[k] = cov ? cd : 0;
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint8_t cd = code[k];
                total += cd != 0;                       // CountsHelper.java:210 (no call -> not counted)
                if (!(cd & 0x80)) continue;             // q<=3 or not A/C/G/T (:214-221)
                const uint32_t a = (cd >> 5) & 3;
                int q = cd & 31;
                q = q > gp.max_q ? gp.max_q : q;        // -maxBaseQS (:217-219)
                const double A = s_t[0][q], H = s_t[1][q], E = s_t[2][q];
                c0 += a == 0; c1 += a == 1; c2 += a == 2; c3 += a == 3;
                const int side = (h[k].w & 1) ? 0 : 1;  // countsStrand[idx][neg?0:1] (:226-227)
#pragma unroll
                for (int t = 0; t < 4; t++) { sc[t][0] += (t == (int)a && side == 0); sc[t][1] += (t == (int)a && side == 1); }
                // updateCounts (:231-248) with f == g: the [i][j] and [j][i] sums are identical sequences
                L00 += a == 0 ? A : E;
                L11 += a == 1 ? A : E;
                L22 += a == 2 ? A : E;
                L33 += a == 3 ? A : E;
                L01 += a <= 1 ? H : E;
                L02 += (a & 1) == 0 ? H : E;
                L03 += (a == 0 || a == 3) ? H : E;
                L12 += (a == 1 || a == 2) ? H : E;
                L13 += (a & 1) == 1 ? H : E;
                L23 += a >= 2 ? H : E;
            }
        }
        if (total == 0) return false;                   // VariantDiscoverySNVQAlgorithm.java:101-103
        const bool callable = (rc & 0x80) != 0;
        int8_t genotype = -1, alt = -1, third = -1, nal = 0;
        int16_t gq = 0, qual = 0;
        bool keep = false;
        if (callable) {
            const int refIdx = (rc >> 5) & 3;
            const double ph = gp.log_prior_homo, px = gp.log_prior_hetero;
            // getPosteriorProbabilities (CountsHelper.java:410-443): events in Java order;
            // row i holds post(i,i) at 4i and post(i,j) at 4i+1+j (j<i) or 4i+j (j>i)
            double ev[16] = {L00 + ph, L01 + px, L02 + px, L03 + px,
                             L11 + ph, L01 + px, L12 + px, L13 + px,
                             L22 + ph, L02 + px, L12 + px, L23 + px,
                             L33 + ph, L03 + px, L13 + px, L23 + px};
            // calculatePosteriorProbabilities (:472-495)
            double logMax = 1;
#pragma unroll
            for (int k = 0; k < 16; k++)
                if (logMax > 0 || logMax < ev[k]) logMax = ev[k];
            double totalProb = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const double x = ev[k] - logMax;
                ev[k] = x < -20 ? 0.0 : pow(10.0, x);
                totalProb += ev[k];
            }
#pragma unroll
            for (int k = 0; k < 16; k++) ev[k] = ev[k] / totalProb;
            auto post = [&](int a, int b) -> double {    // register-resident select, no dynamic indexing
                const int k = a == b ? 4 * a : (b < a ? 4 * a + 1 + b : 4 * a + b);
                double v = 0;
#pragma unroll
                for (int e = 0; e < 16; e++) v = (e == k) ? ev[e] : v;
                return v;
            };
            // getIndexesMaxGenotype (VariantDiscoverySNVQAlgorithm.java:223-243)
            int I = refIdx, J = refIdx;
            double probMax = post(refIdx, refIdx);
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = a; b < 4; b++) {
                    double g = ev[a == b ? 4 * a : 4 * a + b];   // post(a,b), b >= a
                    if (a != b) g += ev[4 * b + 1 + a];           // post(b,a)
                    if (g > probMax + 0.01) { probMax = g; I = a; J = b; }
                }
            const double refProb = post(refIdx, refIdx);
            double maxP = post(I, J);
            if (I != J) maxP += post(J, I);
            gq = phred_d(1 - maxP);
            qual = phred_d(refProb);
            if (I != J && I != refIdx && J != refIdx) {           // triallelic (:128-177)
                if (post(I, I) > post(J, J) + 0.01) { alt = (int8_t)I; third = (int8_t)J; }
                else { alt = (int8_t)J; third = (int8_t)I; }
                nal = 3; genotype = 3; keep = true;
            } else if (I != J) {
                alt = (int8_t)(refIdx != I ? I : J); nal = 2; genotype = 1; keep = true;
            } else if (refIdx != I) {
                alt = (int8_t)I; nal = 2; genotype = 2; keep = true;
            } else {
                genotype = 0; nal = 1;   // hom-ref: dropped (SingleSampleVariantPileupListener.java:223)
            }
            if (keep && gp.min_quality > gq) keep = false;
        }
        if (!keep && !gp.dump_all) return false;
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
        o.counts[0] = (int32_t)c0; o.counts[1] = (int32_t)c1; o.counts[2] = (int32_t)c2; o.counts[3] = (int32_t)c3;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            o.strand_counts[k][0] = sc[k][0];
            o.strand_counts[k][1] = sc[k][1];
        }
        o.logc[0] = L00; o.logc[1] = L01; o.logc[2] = L02; o.logc[3] = L03; o.logc[4] = L11;
        o.logc[5] = L12; o.logc[6] = L13; o.logc[7] = L22; o.logc[8] = L23; o.logc[9] = L33;
        return true;
    };
    // wave-uniform grid-stride loop: one output reservation per wave (ballot), not per site
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t ib = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); ib < n; ib += stride) {
        const int64_t i = ib + lane;
        ngsep_site_out o;
        const bool emit = i < n && site(i, o);
        const unsigned long long m = __ballot(emit);
        if (!m) continue;
        unsigned long long base = 0;
        if (lane == __ffsll((long long)m) - 1) base = atomicAdd(&counters[0], (unsigned long long)__popcll(m));
        base = __shfl(base, __ffsll((long long)m) - 1, 64);
        const unsigned long long idx = base + __popcll(m & ((1ull << lane) - 1ull));
        if (emit && (int64_t)idx < cap) out[idx] = o;
    }
}


// ------------------------------------------------------------------------------------------
// KT: pileup tile scan over the tile-blocked pileup matrix
// ------------------------------------------------------------------------------------------
// nonzero-allele valid bytes (MODE 0: a valid call that is not the reference allele, codes are
// allele-XOR-reference) or any counted byte (MODE 1), one bit per byte
template <int MODE>
__device__ inline uint32_t unit_hits(const u32x4 d) {
    auto f = [](uint32_t w) -> uint32_t {
        uint32_t c;
        if (MODE == 0) c = w & (((w & 0x60606060u) + 0x60606060u)) & 0x80808080u;
        else c = (((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;
        return nib4(c);
    };
    return f(d.x) | (f(d.y) << 4) | (f(d.z) << 8) | (f(d.w) << 12);
}

//   phase 1  stream the tile's block of the pileup matrix (rows_t x T bytes, one coalesced
//            16-byte load per lane and unit, kept in registers) and mark the positions whose pileup
//            holds a valid non-reference call (MODE 0) or any counted call (MODE 1): LDS bitmap,
//            restricted to callable / in-window positions.  Every other position is hom-ref
//            (DESIGN.md "why pruning is exact") or has no pileup.  This is
//            AlignmentsPileupGenerator.processCurrentPosition (discovery/AlignmentsPileupGenerator.java:475-498)
//            reduced to the fact that decides whether SNVQ can call a variant there.
//   phase 2  (MODE 0) integer hom-ref bound of every candidate: one LDS atomic per valid call at a
//            candidate position adds its fixed-point contribution to the candidate's reference or
//            allele accumulator (integer sums: order-independent, so exact).
//   phase 3  a candidate the bound proves hom-ref is dropped; the others are queued for k_posterior.
struct TileShared {
    uint32_t bits[kTileMaxPos / 32];        // candidate bitmap
    uint32_t ok[kTileMaxPos / 32];          // callable (MODE 0) / in-window (MODE 1) positions
    int32_t pref[kTileMaxPos / 32 + 1];
    unsigned long long w[2][32];            // bound addends: [0] reference call, [1] other allele
    unsigned long long acc[kCandCap * 4];   // per candidate: R, X[1..3] (indexed by allele XOR reference)
    QueueSite q[kQueueStage];               // survivors staged for one global reservation per flush
    int32_t qn;
    int32_t qbase;
    unsigned long long ncand;               // candidates seen by this block (statistics)
};

// moves the block's staged survivors to the global queue with ONE atomic (same-address global
// atomics from every tile serialise in L2 and were the scan's bottleneck)
__device__ __forceinline__ void flush_queue(TileShared& sh, QueueSite* __restrict__ queue,
                                            unsigned long long* __restrict__ counters, int64_t qcap) {
    __syncthreads();
    const int32_t n = sh.qn;
    if (n == 0) return;
    if (threadIdx.x == 0) sh.qbase = (int32_t)atomicAdd(&counters[2], (unsigned long long)n);
    __syncthreads();
    const int64_t base = sh.qbase;
    for (int i = threadIdx.x; i < n; i += kScanThreads)
        if (base + i < qcap) queue[base + i] = sh.q[i];
    __syncthreads();
    if (threadIdx.x == 0) sh.qn = 0;
    __syncthreads();
}

template <int MODE>
__device__ __forceinline__ void tile_body(TileShared& sh, const int64_t tile, const TileInfo ti,
    const u32x4* __restrict__ pile, const uint8_t* __restrict__ ref,
    int32_t log2T, const LikTables* __restrict__ tabs, const GenotypeParams& gp,
    QueueSite* __restrict__ queue, unsigned long long* __restrict__ counters, int64_t qcap) {
    uint32_t* s_bits = sh.bits;
    uint32_t* s_ok = sh.ok;
    int32_t* s_pref = sh.pref;
    unsigned long long (*s_w)[32] = sh.w;
    unsigned long long* s_acc = sh.acc;
    if (ti.rows == 0 || (gp.ablate & 4)) return;
    const int tid = threadIdx.x;
    const int32_t T = 1 << log2T;
    const int32_t tstart = (int32_t)(tile << log2T);
    const int nw = T >= 32 ? T / 32 : 1;
    const int log2U = log2T - 4;                                // units per row = T/16
    const int32_t nunits = ti.rows << log2U;
    const u32x4* blk = pile + (ti.off >> 4);

    // phase 1: issue every register-resident unit load first
    u32x4 U[kUnitsPerThread];
#pragma unroll
    for (int k = 0; k < kUnitsPerThread; k++) {
        const int32_t u = tid + k * kScanThreads;
        U[k] = u < nunits ? blk[u] : u32x4{0u, 0u, 0u, 0u};
    }
    // position masks from the reference codes: one dword (4 positions) per thread, eight
    // neighbouring lanes OR their nibbles into one bitmap word
    {
        const uint32_t* refw = reinterpret_cast<const uint32_t*>(ref + tstart);
        for (int i0 = 0; i0 < T / 4; i0 += kScanThreads) {
            const int i = i0 + tid;
            uint32_t bits = 0;
            if (i < T / 4) {
                const uint32_t v = refw[i];
                const uint32_t m = MODE == 0 ? (v & 0x80808080u) : ((((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u);
                bits = nib4(m) << (4 * (i & 7));
            }
            bits |= __shfl_xor(bits, 1, 64);
            bits |= __shfl_xor(bits, 2, 64);
            bits |= __shfl_xor(bits, 4, 64);
            if ((i & 7) == 0 && i < T / 4) {
                s_ok[i >> 3] = bits;
                s_bits[i >> 3] = 0;
            }
        }
        if (T < 32 && tid == 0) s_bits[0] = 0;
    }
    if (MODE == 0) {
        if (tid < 64) s_w[tid >> 5][tid & 31] = (tid < 32 ? tabs->wR : tabs->wX)[tid & 31];
        for (int i = tid; i < kCandCap * 4; i += kScanThreads) s_acc[i] = 0;
    }
    __syncthreads();
    const uint32_t colmask = (1u << log2U) - 1u;
    auto mark = [&](const u32x4 d, int32_t u) {
        const uint32_t m = unit_hits<MODE>(d);
        if (m) {
            const int32_t p = (int32_t)(((uint32_t)u & colmask) << 4);   // tile-relative position of byte 0
            const uint32_t sh = (uint32_t)p & 16u;
            atomicOr(&s_bits[p >> 5], (m & (s_ok[p >> 5] >> sh)) << sh);
        }
    };
#pragma unroll
    for (int k = 0; k < kUnitsPerThread; k++) {
        const int32_t u = tid + k * kScanThreads;
        if (u < nunits) mark(U[k], u);
    }
    for (int32_t u = tid + kUnitsPerThread * kScanThreads; u < nunits; u += kScanThreads) mark(blk[u], u);   // deep tiles
    __syncthreads();
    // candidate prefix counts over bitmap words (nw <= 64: one word per lane of wave 0)
    if (tid < 64) {
        const int32_t v = tid < nw ? __popc(s_bits[tid]) : 0;
        int32_t incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t n = __shfl_up(incl, o, 64);
            if (tid >= o) incl += n;
        }
        if (tid < nw) s_pref[tid] = incl - v;
        if (tid == 63) s_pref[nw] = incl;
    }
    __syncthreads();
    const int32_t ncand = s_pref[nw];
    if (ncand == 0) return;
    if (tid == 0) sh.ncand += (unsigned long long)ncand;
    if (gp.ablate & 1) return;                               // diagnostics: scan only
    const bool bound = MODE == 0 && gp.use_bound;
    if (bound) {
        // phase 2: one LDS atomic per valid call at a candidate position
        auto accumulate = [&](const u32x4 d, int32_t u) {
            const int32_t p = (int32_t)(((uint32_t)u & colmask) << 4);
            uint32_t cm = (s_bits[p >> 5] >> ((uint32_t)p & 16u)) & 0xFFFFu;
            if (!cm) return;
            cm &= unit_valid_mask(d);
            while (cm) {
                const int k = __builtin_ctz(cm);
                cm &= cm - 1;
                const int32_t pos = p + k;
                const uint32_t cd = unit_byte(d, k);
                const uint32_t a = (cd >> 5) & 3;                   // allele XOR reference allele
                int q = cd & 31;
                q = q > gp.max_q ? gp.max_q : q;
                const int w = pos >> 5;
                const int32_t ci = s_pref[w] + __popc(s_bits[w] & ((1u << (pos & 31)) - 1u));
                if (ci < kCandCap) atomicAdd(&s_acc[ci * 4 + (int)a], s_w[a == 0 ? 0 : 1][q]);
            }
        };
#pragma unroll
        for (int k = 0; k < kUnitsPerThread; k++) {
            const int32_t u = tid + k * kScanThreads;
            if (u < nunits) accumulate(U[k], u);
        }
        for (int32_t u = tid + kUnitsPerThread * kScanThreads; u < nunits; u += kScanThreads) accumulate(blk[u], u);
        __syncthreads();
    }
    // phase 3: decide every candidate.  Candidate c runs on thread (c%4)*64 + c/4 so that a tile's
    // few candidates spread over all four waves (SIMDs) instead of queueing on one.
    for (int32_t c0 = 0; c0 < ncand; c0 += kScanThreads) {
        if (c0 > 0 || sh.qn > kQueueStage - kScanThreads) flush_queue(sh, queue, counters, qcap);   // room for one chunk
        const int32_t c = c0 + (tid & 63) * 4 + (tid >> 6);
        if (c >= ncand) continue;
        int lo = 0, hi = nw - 1;              // last word whose prefix <= c
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pref[mid] <= c) lo = mid; else hi = mid - 1;
        }
        uint32_t w = s_bits[lo];
        for (int k = c - s_pref[lo]; k > 0; k--) w &= w - 1;
        const int32_t gpos = tstart + lo * 32 + __builtin_ctz(w);
        bool drop = false;
        if (bound && c < kCandCap) {
            // hom-ref if, for every other genotype G, the lower bound of L[r][r]-L[G] keeps
            // P(G) (het: P(x,y)+P(y,x)) <= P(r,r)  (DESIGN.md "hom-ref bound").  Accumulators are
            // indexed by allele XOR reference: 0 = reference, 1..3 = the three other alleles.
            const unsigned long long Rp = s_acc[c * 4];
            const long long R1 = (long long)(Rp & 0xFFFFFFFFull), R2 = (long long)(Rp >> 32);
            const unsigned long long Xa = s_acc[c * 4 + 1], Xb = s_acc[c * 4 + 2], Xc = s_acc[c * 4 + 3];
            const long long a1 = (long long)(Xa & 0xFFFFFFFFull), b1 = (long long)(Xb & 0xFFFFFFFFull);
            const long long c1 = (long long)(Xc & 0xFFFFFFFFull);
            const long long a2 = (long long)(Xa >> 32), b2 = (long long)(Xb >> 32), c2 = (long long)(Xc >> 32);
            const long long th = tabs->t_het, to = tabs->t_homo;
            // het (r,x): R1 - X1[x];  hom (x,x): R2 - X2[x];  het (x,y), x,y != r: R2 - X1[x] - X1[y]
            drop = (R1 - a1 > th) && (R1 - b1 > th) && (R1 - c1 > th) &&
                   (R2 - a2 > to) && (R2 - b2 > to) && (R2 - c2 > to) &&
                   (R2 - a1 - b1 > th) && (R2 - a1 - c1 > th) && (R2 - b1 - c1 > th);
        }
        if (drop) continue;
        sh.q[atomicAdd(&sh.qn, 1)] = QueueSite{gpos, (int32_t)ref[gpos]};
    }
}

// Persistent grid: block b works on XCD b % 8 (round-robin placement, speed only) through that
// XCD's contiguous share of the tiles, so neighbouring tiles stay in one L2.
template <int MODE>
__global__ __launch_bounds__(kScanThreads) void k_tile_pileup(
    const u32x4* __restrict__ pile, const TileInfo* __restrict__ tinfo, const uint8_t* __restrict__ ref,
    int32_t log2T, int64_t n_tiles, const LikTables* __restrict__ tabs, GenotypeParams gp,
    QueueSite* __restrict__ queue, unsigned long long* __restrict__ counters, int64_t qcap) {
    __shared__ TileShared sh;
    const int64_t nb = gridDim.x, b = blockIdx.x;
    const int64_t xcd = b % 8, j = b / 8, nbx = (nb - xcd + 7) / 8;
    const int64_t q8 = n_tiles / 8, r8 = n_tiles % 8;
    const int64_t c0 = xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8;
    const int64_t c1 = c0 + q8 + (xcd < r8 ? 1 : 0);
    if (threadIdx.x == 0) { sh.qn = 0; sh.ncand = 0; }
    __syncthreads();
    TileInfo next = c0 + j < c1 ? tinfo[c0 + j] : TileInfo{0, 0, 0};
    for (int64_t t = c0 + j; t < c1; t += nbx) {
        const TileInfo ti = next;
        if (t + nbx < c1) next = tinfo[t + nbx];   // descriptor of the next tile in flight meanwhile
        tile_body<MODE>(sh, t, ti, pile, ref, log2T, tabs, gp, queue, counters, qcap);
        __syncthreads();   // the shared tile state is reused by the next tile
    }
    flush_queue(sh, queue, counters, qcap);
    if (threadIdx.x == 0 && sh.ncand) atomicAdd(&counters[1], sh.ncand);
}

// ------------------------------------------------------------------------------------------
// KL: lb[k] = first read index whose gfirst >= 64k - pad + 1
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void kl_read_index(const int4* __restrict__ reads, int64_t n_reads,
                                                     int32_t* __restrict__ lb, int64_t n_lb, int32_t pad) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_lb) return;
    const int64_t key = k * 64 - pad + 1;
    int64_t lo = 0, hi = n_reads;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if ((int64_t)reads[mid].x < key) lo = mid + 1;
        else hi = mid;
    }
    lb[k] = (int32_t)lo;
}

// ------------------------------------------------------------------------------------------
// KO: order the emitted records by global position (counting sort on 4096-position buckets,
//     insertion sort inside a bucket: a handful of records each)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ko_hist(const ngsep_site_out* __restrict__ recs, const unsigned long long* n_ptr,
                                               int64_t cap, int32_t* __restrict__ bucket) {
    int64_t n = (int64_t)*n_ptr;
    if (n > cap) n = cap;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&bucket[recs[i].pos >> 12], 1);
}
// exclusive scan of nb bucket counts into start[0..nb] (one workgroup of 1024)
__global__ __launch_bounds__(1024) void ko_scan(const int32_t* __restrict__ bucket, int32_t* __restrict__ start,
                                                int32_t* __restrict__ cursor, int64_t nb) {
    __shared__ int32_t s_part[1024];
    const int tid = threadIdx.x;
    const int64_t per = (nb + 1023) / 1024;
    const int64_t b0 = tid * per, b1 = b0 + per < nb ? b0 + per : nb;
    int32_t sum = 0;
    for (int64_t b = b0; b < b1; b++) sum += bucket[b];
    s_part[tid] = sum;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int32_t v = tid >= o ? s_part[tid - o] : 0;
        __syncthreads();
        s_part[tid] += v;
        __syncthreads();
    }
    int32_t acc = s_part[tid] - sum;
    for (int64_t b = b0; b < b1; b++) { start[b] = acc; cursor[b] = acc; acc += bucket[b]; }
    if (tid == 1023) start[nb] = s_part[1023];
}
__global__ __launch_bounds__(256) void ko_scatter(const ngsep_site_out* __restrict__ recs, const unsigned long long* n_ptr,
                                                  int64_t cap, int32_t* __restrict__ cursor,
                                                  ngsep_site_out* __restrict__ sorted) {
    int64_t n = (int64_t)*n_ptr;
    if (n > cap) n = cap;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t slot = atomicAdd(&cursor[recs[i].pos >> 12], 1);
        sorted[slot] = recs[i];
    }
}
__global__ __launch_bounds__(256) void ko_bucket_sort(ngsep_site_out* __restrict__ sorted,
                                                      const int32_t* __restrict__ start, int64_t nb) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    const int32_t a = start[b], z = start[b + 1];
    for (int32_t i = a + 1; i < z; i++) {
        const ngsep_site_out v = sorted[i];
        int32_t k = i;
        while (k > a && sorted[k - 1].pos > v.pos) { sorted[k] = sorted[k - 1]; k--; }
        sorted[k] = v;
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
void* pinned_alloc(size_t bytes) {
    void* p = std::aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
    if (p && hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) {
        // no device (CPU-only host code paths): plain memory is fine there
    }
    return p;
}
void pinned_free(void* p) {
    if (!p) return;
    (void)hipHostUnregister(p);
    std::free(p);
}

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
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, ordinal) == hipSuccess && prop.multiProcessorCount > 0)
            d->n_cu = prop.multiProcessorCount;
    }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) { err = "stream"; delete d; return nullptr; }
    for (auto& e : d->ev) (void)hipEventCreate(&e);
    if (hipMalloc(&d->d_counters, 4 * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&d->h_counters, 4 * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess ||
        hipMalloc(&d->d_tables, sizeof(LikTables)) != hipSuccess) {
        err = "device allocation failed";
        delete d;
        return nullptr;
    }
    return d;
}

int64_t device_last_hard(const Device* d) { return d ? d->last_hard : 0; }

void device_release(Device* d) {
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    (void)hipFree(d->d_slots); d->d_slots = nullptr;
    (void)hipFree(d->d_pile); d->d_pile = nullptr;
    (void)hipFree(d->d_reads); d->d_reads = nullptr;
    (void)hipFree(d->d_ref); d->d_ref = nullptr;
    (void)hipFree(d->d_lb); d->d_lb = nullptr;
    (void)hipFree(d->d_tinfo); d->d_tinfo = nullptr;
    d->n_units = d->n_slots = d->n_lb = d->n_reads = d->g_len = d->n_tiles = 0;
}

void device_destroy(Device* d) {
    if (!d) return;
    device_release(d);
    (void)hipFree(d->d_sites);
    (void)hipFree(d->d_sorted);
    (void)hipFree(d->d_bucket);
    (void)hipFree(d->d_hard);
    (void)hipFree(d->d_counters);
    (void)hipFree(d->d_tables);
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
    const int32_t pad = s.windows.empty() ? 64 : s.windows[0].pad;
    HIP_TRY(hipMalloc(&d->d_slots, (size_t)std::max<int64_t>(slot_bytes, 16)));
    HIP_TRY(hipMalloc(&d->d_pile, (size_t)std::max<int64_t>(s.pile_bytes, 16)));
    HIP_TRY(hipMalloc(&d->d_tinfo, (size_t)std::max<int64_t>(s.n_tiles, 1) * sizeof(TileInfo)));
    HIP_TRY(hipMalloc(&d->d_reads, (size_t)std::max<int64_t>(s.n_reads, 1) * sizeof(int4)));
    HIP_TRY(hipMalloc(&d->d_ref, (size_t)s.g_len + 64));
    d->n_lb = (s.g_len + pad + 63) / 64 + 2;
    HIP_TRY(hipMalloc(&d->d_lb, (size_t)d->n_lb * 4));
    if (slot_bytes) HIP_TRY(hipMemcpyAsync(d->d_slots, s.h_slots.data(), (size_t)slot_bytes, hipMemcpyHostToDevice, d->stream));
    if (s.pile_bytes) HIP_TRY(hipMemcpyAsync(d->d_pile, s.h_pile.data(), (size_t)s.pile_bytes, hipMemcpyHostToDevice, d->stream));
    if (s.n_tiles) HIP_TRY(hipMemcpyAsync(d->d_tinfo, s.h_tinfo.data(), (size_t)s.n_tiles * sizeof(TileInfo), hipMemcpyHostToDevice, d->stream));
    if (s.n_reads) HIP_TRY(hipMemcpyAsync(d->d_reads, s.h_reads.data(), (size_t)s.n_reads * 16, hipMemcpyHostToDevice, d->stream));
    HIP_TRY(hipMemsetAsync(d->d_ref, 0, (size_t)s.g_len + 64, d->stream));
    HIP_TRY(hipMemcpyAsync(d->d_ref, s.h_ref.data(), (size_t)s.g_len, hipMemcpyHostToDevice, d->stream));
    d->n_units = slot_bytes / 16;
    d->n_slots = s.n_slots;
    d->n_reads = s.n_reads;
    d->g_len = s.g_len;
    d->slot_size = S;
    d->max_span = s.max_span;
    d->pad = pad;
    d->tile = s.tile;
    d->log2_tile = 0;
    while ((1 << d->log2_tile) < s.tile) d->log2_tile++;
    d->n_tiles = s.n_tiles;
    {
        dim3 grid((unsigned)((d->n_lb + 255) / 256));
        hipLaunchKernelGGL(kl_read_index, grid, dim3(256), 0, d->stream, d->d_reads, d->n_reads, d->d_lb, d->n_lb, pad);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipStreamSynchronize(d->stream));
    return 0;
}

int device_run(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune,
               SiteStore* out, int64_t* n_out, double* scan_ms, double* geno_ms, double* total_ms,
               int64_t* n_candidates, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    auto t0 = std::chrono::steady_clock::now();
    // output capacity: calls are rare; dump mode needs one record per covered position
    int64_t want = g.dump_all ? std::max<int64_t>(s.covered + 1024, 1024) : std::max<int64_t>(s.g_len / 256 + 4096, 4096);
    if (want > d->cap_sites) {
        (void)hipFree(d->d_sites);
        (void)hipFree(d->d_sorted);
        HIP_TRY(hipMalloc(&d->d_sites, (size_t)want * sizeof(ngsep_site_out)));
        HIP_TRY(hipMalloc(&d->d_sorted, (size_t)want * sizeof(ngsep_site_out)));
        d->cap_sites = want;
    }
    const int64_t nb = s.g_len / 4096 + 1;
    if (nb > d->nb_cap) {
        (void)hipFree(d->d_bucket);
        HIP_TRY(hipMalloc(&d->d_bucket, (size_t)(3 * nb + 1) * sizeof(int32_t)));
        d->nb_cap = nb;
    }
    // queue of candidates the tile kernel could not prove hom-ref; dump mode: every position
    int64_t qwant = g.dump_all ? std::max<int64_t>(s.covered + 1024, 1024) : std::max<int64_t>(s.g_len / 64 + 65536, 65536);
    if (qwant < d->cap_hard) qwant = d->cap_hard;
    {
        if (qwant > d->cap_hard) {
            (void)hipFree(d->d_hard);
            HIP_TRY(hipMalloc(&d->d_hard, (size_t)qwant * sizeof(QueueSite)));
            d->cap_hard = qwant;
        }
        HIP_TRY(hipMemcpyAsync(d->d_tables, &t, sizeof(LikTables), hipMemcpyHostToDevice, d->stream));
        HIP_TRY(hipMemsetAsync(d->d_counters, 0, 4 * sizeof(unsigned long long), d->stream));
        HIP_TRY(hipEventRecord(d->ev[0], d->stream));
        if (d->n_tiles > 0) {
            // persistent blocks: a few per CU, each loops over its XCD's tiles
            int per_cu = kTileBlocksPerCU;
            if (const char* e = std::getenv("NGSEP_BLOCKS_PER_CU")) per_cu = std::max(1, std::atoi(e));   // tuning
            const int64_t nblk = std::min<int64_t>(d->n_tiles, (int64_t)d->n_cu * per_cu);
            dim3 grid((unsigned)nblk);
            if (prune)
                hipLaunchKernelGGL(k_tile_pileup<0>, grid, dim3(kScanThreads), 0, d->stream, (const u32x4*)d->d_pile,
                                   d->d_tinfo, d->d_ref, d->log2_tile, d->n_tiles, d->d_tables, g, d->d_hard,
                                   d->d_counters, d->cap_hard);
            else
                hipLaunchKernelGGL(k_tile_pileup<1>, grid, dim3(kScanThreads), 0, d->stream, (const u32x4*)d->d_pile,
                                   d->d_tinfo, d->d_ref, d->log2_tile, d->n_tiles, d->d_tables, g, d->d_hard,
                                   d->d_counters, d->cap_hard);
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(d->ev[1], d->stream));
        hipLaunchKernelGGL(k_posterior, dim3(1024), dim3(256), 0, d->stream, d->d_hard, d->d_counters + 2, d->cap_hard,
                           d->d_reads, d->n_reads, d->d_lb, d->d_slots, d->slot_size, d->d_tables, g, d->d_sites,
                           d->d_counters, d->cap_sites);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(d->ev[2], d->stream));   // queue overflow is checked after the copy below
        // order the records by position on the device
        int32_t* cnt = d->d_bucket;
        int32_t* start = d->d_bucket + nb;
        int32_t* cursor = d->d_bucket + 2 * nb + 1;
        HIP_TRY(hipMemsetAsync(cnt, 0, (size_t)nb * sizeof(int32_t), d->stream));
        hipLaunchKernelGGL(ko_hist, dim3(256), dim3(256), 0, d->stream, d->d_sites, d->d_counters, d->cap_sites, cnt);
        hipLaunchKernelGGL(ko_scan, dim3(1), dim3(1024), 0, d->stream, cnt, start, cursor, nb);
        hipLaunchKernelGGL(ko_scatter, dim3(256), dim3(256), 0, d->stream, d->d_sites, d->d_counters, d->cap_sites, cursor,
                           d->d_sorted);
        hipLaunchKernelGGL(ko_bucket_sort, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, d->stream, d->d_sorted, start, nb);
        HIP_TRY(hipGetLastError());
    }
    // counters and a prefix of the ordered records in one round trip, straight into the result store
    const size_t from = out->size();
    const int64_t guess = std::min<int64_t>(d->cap_sites, d->last_n_sites + d->last_n_sites / 4 + 256);
    out->reserve(from + (size_t)guess);
    HIP_TRY(hipMemcpyAsync(d->h_counters, d->d_counters, 4 * sizeof(unsigned long long), hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipMemcpyAsync(out->buf + from, d->d_sorted, (size_t)guess * sizeof(ngsep_site_out), hipMemcpyDeviceToHost, d->stream));
    auto tq = std::chrono::steady_clock::now();
    HIP_TRY(hipStreamSynchronize(d->stream));
    auto ts = std::chrono::steady_clock::now();
    const int64_t n = (int64_t)d->h_counters[0];
    if (n > d->cap_sites) {
        // more calls than the record buffer holds (e.g. -minQuality 0): grow it and run again
        (void)hipFree(d->d_sites);
        (void)hipFree(d->d_sorted);
        d->d_sites = d->d_sorted = nullptr;
        d->cap_sites = 0;
        HIP_TRY(hipMalloc(&d->d_sites, (size_t)(n + 1024) * sizeof(ngsep_site_out)));
        HIP_TRY(hipMalloc(&d->d_sorted, (size_t)(n + 1024) * sizeof(ngsep_site_out)));
        d->cap_sites = n + 1024;
        d->last_n_sites = n;
        return device_run(d, s, t, g, prune, out, n_out, scan_ms, geno_ms, total_ms, n_candidates, err);
    }
    if ((int64_t)d->h_counters[2] > d->cap_hard) {
        // rare: more undecided candidates than the queue holds -> grow it and run again
        (void)hipFree(d->d_hard);
        d->d_hard = nullptr;
        HIP_TRY(hipMalloc(&d->d_hard, (size_t)(d->h_counters[2] + 1024) * sizeof(QueueSite)));
        d->cap_hard = (int64_t)d->h_counters[2] + 1024;
        d->last_n_sites = n;
        return device_run(d, s, t, g, prune, out, n_out, scan_ms, geno_ms, total_ms, n_candidates, err);
    }
    if (n > guess) {
        out->n = from + (size_t)guess;      // keep the records already copied when the store grows
        out->reserve(from + (size_t)n);
        HIP_TRY(hipMemcpyAsync(out->buf + from + guess, d->d_sorted + guess, (size_t)(n - guess) * sizeof(ngsep_site_out),
                               hipMemcpyDeviceToHost, d->stream));
        HIP_TRY(hipStreamSynchronize(d->stream));
    }
    d->last_n_sites = n;
    out->n = from + (size_t)n;
    *n_out = n;
    auto t1 = std::chrono::steady_clock::now();
    float a = 0, a2 = 0;
    (void)hipEventElapsedTime(&a, d->ev[0], d->ev[1]);
    (void)hipEventElapsedTime(&a2, d->ev[1], d->ev[2]);
    if (std::getenv("NGSEP_TIMING")) {
        auto us = [](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
        std::fprintf(stderr, "[ngsep timing] enqueue %.1f us, sync %.1f us, rest %.1f us, tile %.1f us, posterior %.1f us, n=%lld guess=%lld\n",
                     us(t0, tq), us(tq, ts), us(ts, t1), a * 1000.0, a2 * 1000.0, (long long)n, (long long)guess);
    }
    *scan_ms = a;
    *geno_ms = a2;
    *total_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    *n_candidates = (int64_t)d->h_counters[1];
    d->last_hard = (int64_t)d->h_counters[2];
    return 0;
}

}  // namespace ngsep
