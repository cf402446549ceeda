// kernels.hip -- gfx950 kernels of the NGSEP SNV pileup path.
//
//   KT  k_tile_pileup : one workgroup per tile of T reference positions (global coordinates).
//        phase 1  stream the tile's read slots HBM -> VGPR -> LDS (16 B per lane, coalesced; the
//                 slots of the reads overlapping a tile are one contiguous range) and, on the way,
//                 compare every projected read byte with the reference code of its position:
//                 a position whose pileup holds a valid non-reference call becomes a candidate
//                 (LDS bitmap).  This is AlignmentsPileupGenerator.processCurrentPosition
//                 (discovery/AlignmentsPileupGenerator.java:475-498) reduced to the fact that decides
//                 whether SNVQ can call a variant there ("why pruning is exact").
//        phase 2  genotype each candidate from LDS: CountsHelper.calculateCountsSNV/updateCounts
//                 (discovery/CountsHelper.java:83-95,209-251) over the reads in pending-list order
//                 (bit-exact fp64 sums), getPosteriorProbabilities (:410-495) and
//                 VariantDiscoverySNVQAlgorithm.discoverSNV (:100-243) + the listener filters
//                 (SingleSampleVariantPileupListener.java:213-232).
//        Tiles whose reads do not fit the LDS budget run the same two phases on global memory.
//   KL  kl_read_index : per 64-position block, first read that can cover it (binary search).
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

struct HardSite;

struct Device {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {};
    uint8_t* d_slots = nullptr;
    int32_t* d_slot_pos = nullptr;
    int4* d_reads = nullptr;
    uint8_t* d_ref = nullptr;
    int32_t* d_lb = nullptr;
    int4* d_tiles = nullptr;
    LikTables* d_tables = nullptr;
    ngsep_site_out* d_sites = nullptr;
    ngsep_site_out* d_sorted = nullptr;
    int32_t* d_bucket = nullptr;     // counts, then starts (nb+1), then cursors (nb)
    int64_t nb_cap = 0;
    HardSite* d_hard = nullptr;
    int64_t cap_hard = 0;
    unsigned long long* d_counters = nullptr;
    unsigned long long* h_counters = nullptr;
    int64_t cap_sites = 0;
    int64_t n_units = 0, n_slots = 0, n_lb = 0, n_reads = 0, g_len = 0, n_tiles = 0;
    int32_t slot_size = 0, max_span = 0, pad = 0, tile = 1024, tile_variant = 0;
    int64_t last_n_sites = 1024;
    int64_t last_hard = 0;
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

// 16 bytes starting at byte offset o (o >= 0) of a dword-aligned byte array
__device__ inline void load16(const uint8_t* base, int64_t o, uint32_t R[4]) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(base) + (o >> 2);
    const uint32_t sh = (uint32_t)(o & 3);
    const uint32_t r0 = w[0], r1 = w[1], r2 = w[2], r3 = w[3], r4 = w[4];
    R[0] = __builtin_amdgcn_alignbyte(r1, r0, sh);
    R[1] = __builtin_amdgcn_alignbyte(r2, r1, sh);
    R[2] = __builtin_amdgcn_alignbyte(r3, r2, sh);
    R[3] = __builtin_amdgcn_alignbyte(r4, r3, sh);
}

// candidate bits of one 16-byte unit: bit i set <=> byte i is a valid call (code bit 7) whose
// allele differs from a callable reference base (MODE 0), or any counted call at an
// in-window position (MODE 1: genotype every position)
template <int MODE>
__device__ inline uint32_t unit_candidates(const uint32_t D[4], const uint32_t R[4]) {
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t c;
        if (MODE == 0) {
            const uint32_t diff = ((D[k] ^ R[k]) & 0x60606060u) + 0x60606060u;
            c = D[k] & R[k] & diff & 0x80808080u;
        } else {
            const uint32_t nzd = (((D[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | D[k]) & 0x80808080u;
            const uint32_t nzr = (((R[k] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | R[k]) & 0x80808080u;
            c = nzd & nzr;
        }
        mask |= (((c >> 7) & 1u) | ((c >> 14) & 2u) | ((c >> 21) & 4u) | ((c >> 28) & 8u)) << (4 * k);
    }
    return mask;
}

// A candidate whose call needs the full posterior (queued by the tile kernel for k_posterior)
struct HardSite {
    double L[10];          // log-conditionals, upper triangle 00 01 02 03 11 12 13 22 23 33
    int32_t gpos, total;
    int32_t c[4];
    int32_t r_begin;       // first read that can cover gpos (global read index)
    int32_t rc;            // reference code
};
static_assert(sizeof(HardSite) == 112, "HardSite layout");

// Tally one candidate over the reads in pending-list order (CountsHelper.calculateCountsSNV /
// updateCounts, discovery/CountsHelper.java:83-95,209-251: bit-exact fp64 sums), then decide
// whether the call can be settled without the posterior: the exact hom-ref shortcut drops the
// position (SingleSampleVariantPileupListener.java:223); anything else is queued for k_posterior.
// STAGED: headers/image/tables in LDS (32-bit offsets); otherwise global memory.
template <bool STAGED>
__device__ void tally_position(int32_t gpos, uint8_t rc, int32_t r_begin, int32_t r_end,
                               const int4* __restrict__ hdr, int32_t hdr_base,
                               const uint8_t* __restrict__ img, int32_t img_slot0, int32_t S,
                               const double* __restrict__ TA, const double* __restrict__ TH,
                               const double* __restrict__ TE, const GenotypeParams& gp,
                               HardSite* __restrict__ queue, unsigned long long* counters, int64_t qcap) {
    int32_t total = 0;
    uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    double L00 = 0, L01 = 0, L02 = 0, L03 = 0, L11 = 0, L12 = 0, L13 = 0, L22 = 0, L23 = 0, L33 = 0;
    // reads [r_begin, r_end) all have gfirst <= gpos (r_end is the upper bound); batches of 4 issue
    // every LDS load of the batch before the in-order accumulation
    for (int32_t r0 = r_begin; r0 < r_end; r0 += 4) {
        uint8_t code[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int32_t r = r0 + k < r_end ? r0 + k : r_end - 1;
            const int4 h = hdr[r - hdr_base];   // gfirst, glast, slot, flags
            const int32_t off = gpos - h.x;
            const int32_t sidx = off >= S ? off / S : 0;
            uint8_t cd;
            if (STAGED) cd = img[(h.z + sidx - img_slot0) * S + (off - sidx * S)];
            else cd = img[(int64_t)(h.z + sidx) * S + (off - sidx * S)];
            code[k] = (r0 + k < r_end && h.y >= gpos) ? cd : 0;   // read must cover gpos
        }
        double tA[4], tH[4], tE[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int q = code[k] & 31;
            q = q > gp.max_q ? gp.max_q : q;
            tA[k] = TA[q];
            tH[k] = TH[q];
            tE[k] = TE[q];
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint8_t cd = code[k];
            total += cd != 0;                       // CountsHelper.java:210 (no call -> not counted)
            if (!(cd & 0x80)) continue;             // q<=3 or not A/C/G/T (:214-221)
            const uint32_t a = (cd >> 5) & 3;
            c0 += a == 0; c1 += a == 1; c2 += a == 2; c3 += a == 3;
            const double A = tA[k], H = tH[k], E = tE[k];   // q clamped to -maxBaseQS (:217-219) above
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
    if (total == 0) return;                     // VariantDiscoverySNVQAlgorithm.java:101-103
    if (gp.ablate & 2) {                        // diagnostics: keep the tally live, skip the posterior
        if (L00 + L11 + L22 + L33 + L01 + L02 + L03 + L12 + L13 + L23 == 1.0) atomicAdd(&counters[0], 1ull);
        return;
    }
    if ((rc & 0x80) && !gp.dump_all) {
        // Exact shortcut (DESIGN.md "hom-ref shortcut"): with m the largest event, every genotype
        // other than ref/ref has posterior <= 2*10^(ev-m) (CountsHelper.java:472-495 divides by a
        // total >= 1).  If that is < 0.01 for all of them, none can beat P(ref/ref)+0.01 in
        // getIndexesMaxGenotype (VariantDiscoverySNVQAlgorithm.java:223-243): hom-ref, dropped.
        const int ri = (rc >> 5) & 3;
        const double ph = gp.log_prior_homo, px = gp.log_prior_hetero;
        const double d00 = L00 + ph, d11 = L11 + ph, d22 = L22 + ph, d33 = L33 + ph;
        const double h01 = L01 + px, h02 = L02 + px, h03 = L03 + px, h12 = L12 + px, h13 = L13 + px, h23 = L23 + px;
        const double m = fmax(fmax(fmax(d00, d11), fmax(d22, d33)), fmax(fmax(fmax(h01, h02), fmax(h03, h12)), fmax(h13, h23)));
        const double lim = m - 2.4;
        const double others = fmax(fmax(fmax(h01, h02), fmax(h03, h12)), fmax(h13, h23));
        const double homo_other = fmax(fmax(ri == 0 ? -INFINITY : d00, ri == 1 ? -INFINITY : d11),
                                       fmax(ri == 2 ? -INFINITY : d22, ri == 3 ? -INFINITY : d33));
        if (others < lim && homo_other < lim) return;
    }
    const unsigned long long qi = atomicAdd(&counters[2], 1ull);
    if ((int64_t)qi >= qcap) return;            // host re-runs with a larger queue
    HardSite hs;
    hs.L[0] = L00; hs.L[1] = L01; hs.L[2] = L02; hs.L[3] = L03; hs.L[4] = L11;
    hs.L[5] = L12; hs.L[6] = L13; hs.L[7] = L22; hs.L[8] = L23; hs.L[9] = L33;
    hs.gpos = gpos;
    hs.total = total;
    hs.c[0] = (int32_t)c0; hs.c[1] = (int32_t)c1; hs.c[2] = (int32_t)c2; hs.c[3] = (int32_t)c3;
    hs.r_begin = r_begin;
    hs.rc = rc;
    queue[qi] = hs;
}

// ------------------------------------------------------------------------------------------
// KP: posterior + SNVQ call for queued candidates (thread per site)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_posterior(const HardSite* __restrict__ queue, const unsigned long long* qn,
                                                   int64_t qcap, const int4* __restrict__ reads, int64_t n_reads,
                                                   const uint8_t* __restrict__ slots, int32_t S, GenotypeParams gp,
                                                   ngsep_site_out* __restrict__ out, unsigned long long* counters,
                                                   int64_t cap) {
    int64_t n = (int64_t)*qn;
    if (n > qcap) n = qcap;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const HardSite hs = queue[i];
        const uint8_t rc = (uint8_t)hs.rc;
        const double L00 = hs.L[0], L01 = hs.L[1], L02 = hs.L[2], L03 = hs.L[3], L11 = hs.L[4];
        const double L12 = hs.L[5], L13 = hs.L[6], L22 = hs.L[7], L23 = hs.L[8], L33 = hs.L[9];
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
        if (!keep && !gp.dump_all) continue;
        const unsigned long long idx = atomicAdd(&counters[0], 1ull);
        if ((int64_t)idx >= cap) continue;
        ngsep_site_out o;
        o.seq_id = -1;
        o.pos = hs.gpos;
        o.ref = callable ? "ACGT"[(rc >> 5) & 3] : 'N';
        o.n_alleles = nal;
        o.alt = alt;
        o.third = third;
        o.genotype = genotype;
        o.strand_bias = -1;
        o.gq = gq;
        o.qual = qual;
        o.is_call = keep ? 1 : 0;
        o.dp = hs.total;
#pragma unroll
        for (int k = 0; k < 4; k++) o.counts[k] = hs.c[k];
        // CountsHelper.countsStrand (:226-227), recounted for emitted records only
        int32_t sc[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        for (int64_t r = hs.r_begin; r < n_reads; r++) {
            const int4 h = reads[r];
            if (h.x > hs.gpos) break;
            if (h.y < hs.gpos) continue;
            const int32_t off = hs.gpos - h.x;
            const uint8_t code = slots[(int64_t)(h.z + off / S) * S + (off % S)];
            if (!(code & 0x80)) continue;
            const int a = (code >> 5) & 3;
            const int side = (h.w & 1) ? 0 : 1;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                sc[k][0] += (k == a && side == 0);
                sc[k][1] += (k == a && side == 1);
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            o.strand_counts[k][0] = sc[k][0];
            o.strand_counts[k][1] = sc[k][1];
        }
#pragma unroll
        for (int k = 0; k < 10; k++) o.logc[k] = hs.L[k];
        out[idx] = o;
    }
}

// ------------------------------------------------------------------------------------------
// KT: fused pileup tile
// ------------------------------------------------------------------------------------------
// tile descriptor: {first read, end read, first slot, end slot} of the reads overlapping the tile
template <int MODE, int IMG_BYTES, int MAX_READS, int MAX_SLOTS, int MAX_POS>
__global__ __launch_bounds__(256, 2) void k_tile_pileup(
    const u32x4* __restrict__ slots, const int32_t* __restrict__ slot_pos, const int4* __restrict__ reads,
    const int4* __restrict__ tiles, const uint8_t* __restrict__ ref, const int32_t* __restrict__ lb,
    int32_t T, int32_t S, int32_t max_span, int64_t n_tiles, const LikTables* __restrict__ tabs, GenotypeParams gp,
    HardSite* __restrict__ queue, unsigned long long* __restrict__ counters, int64_t qcap) {
    __shared__ __attribute__((aligned(16))) uint8_t s_img[IMG_BYTES];
    __shared__ int4 s_hdr[MAX_READS];
    __shared__ int32_t s_spos[MAX_SLOTS];                      // position of byte 0 of every staged slot
    __shared__ __attribute__((aligned(16))) uint8_t s_ref[MAX_POS + 64];
    __shared__ uint32_t s_bits[MAX_POS / 32];
    __shared__ int32_t s_pref[MAX_POS / 32 + 1];
    __shared__ double s_tab[3][32];                            // A, H, E likelihood addends

    // XCD-aware tile order: consecutive tiles (which share boundary reads) run on one XCD
    const int64_t b = blockIdx.x;
    const int64_t q8 = n_tiles / 8, r8 = n_tiles % 8, xcd = b % 8, idx = b / 8;
    const int64_t tile = xcd < r8 ? xcd * (q8 + 1) + idx : r8 * (q8 + 1) + (xcd - r8) * q8 + idx;
    const int32_t tstart = (int32_t)(tile * T);
    const int32_t tend = tstart + T;
    const int tid = threadIdx.x;
    const int4 td = tiles[tile];
    const int32_t rlo = td.x, rhi = td.y, s0 = td.z, s1 = td.w;
    if (rhi <= rlo) return;
    const int32_t nslot = s1 - s0;
    const bool staged = (int64_t)nslot * S <= IMG_BYTES && nslot <= MAX_SLOTS && (rhi - rlo) <= MAX_READS;
    const uint32_t ups = (uint32_t)(S / 16);

    // reference codes of the tile, zero outside [tstart, tend): outside positions are never candidates
    {
        const uint32_t* refw = reinterpret_cast<const uint32_t*>(ref);
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_ref);
        for (int i = tid; i < (T + 64) / 4; i += 256) {
            const int32_t g = tstart - 16 + 4 * i;
            uint32_t v = (g >= tstart && g + 3 < tend) ? refw[g >> 2] : 0u;
            dst[i] = v;
        }
    }
    for (int i = tid; i < T / 32; i += 256) s_bits[i] = 0;
    if (tid < 96) s_tab[tid >> 5][tid & 31] = (tid < 32 ? tabs->A : tid < 64 ? tabs->H : tabs->E)[tid & 31];
    if (staged) {
        for (int i = tid; i < rhi - rlo; i += 256) s_hdr[i] = reads[rlo + i];
        for (int i = tid; i < nslot; i += 256) s_spos[i] = slot_pos[s0 + i];
        __syncthreads();
        // phase 1a: LDS-DMA of every 16-byte unit that overlaps the tile (lane-masked, all in flight)
        const int32_t nunits = nslot * (int32_t)ups;
        const int wave = tid >> 6, lane = tid & 63;
        for (int32_t base = wave * 64; base < nunits; base += 256) {
            const int32_t uu = base + lane;
            bool need = false;
            if (uu < nunits) {
                const int32_t sl = uu / (int32_t)ups, jj = uu - sl * (int32_t)ups;
                const int32_t p0 = s_spos[sl] + 16 * jj;
                need = p0 + 15 >= tstart && p0 < tend;
            }
            if (need)
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(&slots[(int64_t)s0 * ups + uu]),
                                                 (__attribute__((address_space(3))) void*)(&s_img[base * 16]),
                                                 16, 0, 0);
        }
        __syncthreads();   // drains the LDS-DMA (vmcnt(0)) before anyone reads the image
        // phase 1b: scan units from LDS, mark candidates
        for (int32_t uu = tid; uu < nunits; uu += 256) {
            const int32_t sl = uu / (int32_t)ups, jj = uu - sl * (int32_t)ups;
            const int32_t p0 = s_spos[sl] + 16 * jj;
            if (!(p0 + 15 >= tstart && p0 < tend)) continue;
            const u32x4 d = *reinterpret_cast<const u32x4*>(&s_img[uu * 16]);
            uint32_t any = d.x | d.y | d.z | d.w;
            if (MODE == 0) any &= 0x80808080u;
            if (!any) continue;
            const uint32_t D[4] = {d.x, d.y, d.z, d.w};
            uint32_t R[4];
            load16(s_ref, p0 - tstart + 16, R);
            const uint32_t m = unit_candidates<MODE>(D, R);
            if (m) {
                const int32_t o = p0 - tstart;
                if (o >= 0) {
                    const uint64_t m64 = (uint64_t)m << (o & 31);
                    atomicOr(&s_bits[o >> 5], (uint32_t)m64);
                    if ((m64 >> 32) && ((o >> 5) + 1) < T / 32) atomicOr(&s_bits[(o >> 5) + 1], (uint32_t)(m64 >> 32));
                } else {
                    atomicOr(&s_bits[0], m >> (-o));
                }
            }
        }
    } else {
        // oversized tile: the same scan straight from global memory
        __syncthreads();
        const int64_t u0 = (int64_t)s0 * ups, u1 = (int64_t)s1 * ups;
        for (int64_t u = u0 + tid; u < u1; u += 256) {
            const int64_t sl = u / ups;
            const int32_t p0 = slot_pos[sl] + 16 * (int32_t)(u - sl * ups);
            if (!(p0 + 15 >= tstart && p0 < tend)) continue;
            const u32x4 d = slots[u];
            uint32_t any = d.x | d.y | d.z | d.w;
            if (MODE == 0) any &= 0x80808080u;
            if (!any) continue;
            const uint32_t D[4] = {d.x, d.y, d.z, d.w};
            uint32_t R[4];
            load16(s_ref, p0 - tstart + 16, R);
            const uint32_t m = unit_candidates<MODE>(D, R);
            if (m) {
                const int32_t o = p0 - tstart;
                if (o >= 0) {
                    const uint64_t m64 = (uint64_t)m << (o & 31);
                    atomicOr(&s_bits[o >> 5], (uint32_t)m64);
                    if ((m64 >> 32) && ((o >> 5) + 1) < T / 32) atomicOr(&s_bits[(o >> 5) + 1], (uint32_t)(m64 >> 32));
                } else {
                    atomicOr(&s_bits[0], m >> (-o));
                }
            }
        }
    }
    __syncthreads();
    // candidate prefix counts over bitmap words
    const int nw = T / 32;
    if (tid < 64) {
        // wave-wide exclusive scan of popcounts (nw <= 128: two words per lane)
        const int w0 = 2 * tid, w1 = 2 * tid + 1;
        const int32_t c0 = w0 < nw ? __popc(s_bits[w0]) : 0, c1 = w1 < nw ? __popc(s_bits[w1]) : 0;
        int32_t v = c0 + c1, incl = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t n = __shfl_up(incl, o, 64);
            if (tid >= o) incl += n;
        }
        const int32_t excl = incl - v;
        if (w0 < nw) s_pref[w0] = excl;
        if (w1 < nw) s_pref[w1] = excl + c0;
        if (tid == 63) s_pref[nw] = incl;
    }
    __syncthreads();
    const int32_t ncand = s_pref[nw];
    if (tid == 0 && ncand) atomicAdd(&counters[1], (unsigned long long)ncand);
    // phase 2: tally candidates.  Candidate c runs on thread (c%4)*64 + c/4 so that a tile's few
    // candidates spread over all four waves (SIMDs) instead of queueing on one.
    for (int32_t c = (gp.ablate & 1) ? ncand : ((tid & 63) * 4 + (tid >> 6)); c < ncand; c += 256) {
        int lo = 0, hi = nw - 1;              // last word whose prefix <= c
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pref[mid] <= c) lo = mid; else hi = mid - 1;
        }
        uint32_t w = s_bits[lo];
        for (int k = c - s_pref[lo]; k > 0; k--) w &= w - 1;
        const int32_t gpos = tstart + lo * 32 + __builtin_ctz(w);
        const uint8_t rc = s_ref[gpos - tstart + 16];
        if (staged) {
            // first read that can cover gpos: gfirst >= gpos - max_span + 1 (headers sorted by gfirst)
            int a = 0, z = rhi - rlo;
            const int32_t key = gpos - max_span + 1;
            while (a < z) {
                const int m = (a + z) >> 1;
                if (s_hdr[m].x < key) a = m + 1; else z = m;
            }
            int e = a;                            // first read starting after gpos
            z = rhi - rlo;
            while (e < z) {
                const int m = (e + z) >> 1;
                if (s_hdr[m].x <= gpos) e = m + 1; else z = m;
            }
            tally_position<true>(gpos, rc, rlo + a, rlo + e, s_hdr, rlo, s_img, s0, S, s_tab[0], s_tab[1], s_tab[2], gp,
                                 queue, counters, qcap);
        } else {
            int32_t rb = lb[gpos >> 6];
            if (rb < rlo) rb = rlo;
            int32_t re = rb, z = rhi;             // first read starting after gpos
            while (re < z) {
                const int32_t m = (re + z) >> 1;
                if (reads[m].x <= gpos) re = m + 1; else z = m;
            }
            tally_position<false>(gpos, rc, rb, re, reads, 0, reinterpret_cast<const uint8_t*>(slots), 0, S,
                                  s_tab[0], s_tab[1], s_tab[2], gp, queue, counters, qcap);
        }
    }
}

// tile descriptors from the read index
__global__ __launch_bounds__(256) void kt_tile_info(const int4* __restrict__ reads, int64_t n_reads, int64_t n_slots,
                                                    const int32_t* __restrict__ lb, int64_t n_lb, int32_t T, int32_t pad,
                                                    int64_t n_tiles, int4* __restrict__ tiles) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_tiles) return;
    const int64_t tstart = t * T, tend = tstart + T;
    const int64_t rlo = lb[tstart >> 6];
    int64_t k = (tend + pad) >> 6;
    if (k >= n_lb) k = n_lb - 1;
    const int64_t rhi = lb[k];
    tiles[t] = make_int4((int)rlo, (int)rhi, (int)(rlo < n_reads ? reads[rlo].z : n_slots),
                         (int)(rhi < n_reads ? reads[rhi].z : n_slots));
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
    (void)hipFree(d->d_slot_pos); d->d_slot_pos = nullptr;
    (void)hipFree(d->d_reads); d->d_reads = nullptr;
    (void)hipFree(d->d_ref); d->d_ref = nullptr;
    (void)hipFree(d->d_lb); d->d_lb = nullptr;
    (void)hipFree(d->d_tiles); d->d_tiles = nullptr;
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
    HIP_TRY(hipMalloc(&d->d_slot_pos, (size_t)std::max<int64_t>(s.n_slots, 1) * 4));
    HIP_TRY(hipMalloc(&d->d_reads, (size_t)std::max<int64_t>(s.n_reads, 1) * sizeof(int4)));
    HIP_TRY(hipMalloc(&d->d_ref, (size_t)s.g_len + 64));
    d->n_lb = (s.g_len + pad + 63) / 64 + 2;
    HIP_TRY(hipMalloc(&d->d_lb, (size_t)d->n_lb * 4));
    if (slot_bytes) HIP_TRY(hipMemcpyAsync(d->d_slots, s.h_slots.data(), (size_t)slot_bytes, hipMemcpyHostToDevice, d->stream));
    if (s.n_slots) HIP_TRY(hipMemcpyAsync(d->d_slot_pos, s.h_slot_pos.data(), (size_t)s.n_slots * 4, hipMemcpyHostToDevice, d->stream));
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
    d->tile_variant = s.tile_variant;
    d->n_tiles = (s.g_len + s.tile - 1) / s.tile;
    {
        dim3 grid((unsigned)((d->n_lb + 255) / 256));
        hipLaunchKernelGGL(kl_read_index, grid, dim3(256), 0, d->stream, d->d_reads, d->n_reads, d->d_lb, d->n_lb, pad);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMalloc(&d->d_tiles, (size_t)std::max<int64_t>(d->n_tiles, 1) * sizeof(int4)));
        dim3 gt((unsigned)((d->n_tiles + 255) / 256));
        hipLaunchKernelGGL(kt_tile_info, gt, dim3(256), 0, d->stream, d->d_reads, d->n_reads, d->n_slots, d->d_lb, d->n_lb,
                           d->tile, pad, d->n_tiles, d->d_tiles);
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
    // queue of candidates that need the full posterior: ~2% of candidates; dump mode: every position
    int64_t qwant = g.dump_all ? std::max<int64_t>(s.covered + 1024, 1024) : std::max<int64_t>(s.g_len / 64 + 65536, 65536);
    if (qwant < d->cap_hard) qwant = d->cap_hard;
    {
        if (qwant > d->cap_hard) {
            (void)hipFree(d->d_hard);
            HIP_TRY(hipMalloc(&d->d_hard, (size_t)qwant * sizeof(HardSite)));
            d->cap_hard = qwant;
        }
        HIP_TRY(hipMemcpyAsync(d->d_tables, &t, sizeof(LikTables), hipMemcpyHostToDevice, d->stream));
        HIP_TRY(hipMemsetAsync(d->d_counters, 0, 4 * sizeof(unsigned long long), d->stream));
        HIP_TRY(hipEventRecord(d->ev[0], d->stream));
        if (d->n_tiles > 0) {
            dim3 grid((unsigned)d->n_tiles);
#define NGSEP_LAUNCH_TILE(MODE, B)                                                                                     \
    hipLaunchKernelGGL((k_tile_pileup<MODE, B.img_bytes, B.max_reads, B.max_slots, B.max_pos>), grid, dim3(256), 0,  \
                       d->stream, (const u32x4*)d->d_slots, d->d_slot_pos, d->d_reads, d->d_tiles, d->d_ref, d->d_lb, \
                       d->tile, d->slot_size, d->max_span, d->n_tiles, d->d_tables, g, d->d_hard, d->d_counters,       \
                       d->cap_hard)
            if (d->tile_variant == 0) {
                if (prune) NGSEP_LAUNCH_TILE(0, kTileSmall); else NGSEP_LAUNCH_TILE(1, kTileSmall);
            } else {
                if (prune) NGSEP_LAUNCH_TILE(0, kTileLarge); else NGSEP_LAUNCH_TILE(1, kTileLarge);
            }
#undef NGSEP_LAUNCH_TILE
            HIP_TRY(hipGetLastError());
        }
        HIP_TRY(hipEventRecord(d->ev[1], d->stream));
        hipLaunchKernelGGL(k_posterior, dim3(1024), dim3(256), 0, d->stream, d->d_hard, d->d_counters + 2, d->cap_hard,
                           d->d_reads, d->n_reads, d->d_slots, d->slot_size, g, d->d_sites, d->d_counters, d->cap_sites);
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
    if (n > d->cap_sites) { err = "site buffer overflow"; return -1; }
    if ((int64_t)d->h_counters[2] > d->cap_hard) {
        // rare: more undecided candidates than the queue holds -> grow it and run again
        (void)hipFree(d->d_hard);
        d->d_hard = nullptr;
        HIP_TRY(hipMalloc(&d->d_hard, (size_t)(d->h_counters[2] + 1024) * sizeof(HardSite)));
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
