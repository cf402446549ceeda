// kernels.hip -- gfx950 kernels of the NGSEP SNV pileup path.
//
//   KL  k_read_scan<T, U> : single-sample scan straight from the read-group layout (1 B per read base, engine.hpp
//        RGroup), one workgroup per tile of T positions: coverage from an LDS difference array, per-position
//        exception / other-allele counters from SWAR over the reads' 8-byte units, the candidates (a valid
//        non-reference call at a callable position) and the count bound as a table; survivors queued with their
//        column space.  This is AlignmentsPileupGenerator.processCurrentPosition
//        (discovery/AlignmentsPileupGenerator.java:475-498) reduced to the fact that decides whether SNVQ can call a
//        variant there ("why pruning is exact").
//   KG  k_gather_kl / k_gather_cols : the queued sites' columns (PileupRecord.getAlleleCalls(1) in pending order)
//        gathered from the read-group layout, the queue compacted.
//   KQ  k_queue_all : every in-window position queued (dump mode, runs without the exact pruning).
//   KP  k_posterior : exact CountsHelper tally (pending-list order, bit-exact fp64), posterior and
//        SNVQ call of the queued candidates (discovery/CountsHelper.java:83-95,209-251,410-495,
//        VariantDiscoverySNVQAlgorithm.java:100-243, SingleSampleVariantPileupListener.java:213-232);
//        records go to position buckets.
//   KO  ko_fused : position order of the records (rank per bucket) and their (sequence, position).
//   KLM / KQN / KPM k_scan_pop / k_queue_need / k_posterior_multi : MultisampleVariantsDetector.
//   KR  k_rac : RelativeAlleleCountsCalculator over the tile-blocked byte pile (engine.cpp build_single_layout).
//
// HBM-bound integer/byte work: no MFMA.  Layout and roofline: DESIGN.md.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "engine.hpp"
#include <sys/mman.h>

namespace ngsep {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ablation bits (GenotypeParams.ablate, NGSEP_ABLATE) exist only in diagnostic builds (make DIAG=1): a release
// build compiles every ablated branch out
#ifdef NGSEP_DIAG
#define ABLATE(mask, bit) ((((mask) & (bit)) != 0))
#else
#define ABLATE(mask, bit) false
#endif

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#expr) + " (kernels.hip:" + std::to_string(__LINE__) + "): " + \
                  hipGetErrorString(e_);                                                 \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

struct QueueSite;
struct SiteQ;

// counter set of a single-sample run: [0] records | fullest bucket << 40, [1] candidates (KQ), [2] KP's queue
// length, [3] spare, [4] whole records, [5] column space reserved by KG (units of 4 entries), then KL's shards:
// shard t at kCtrShard0 + kCtrShardStride t = {queue sites, column space, candidates} (one 128-B line each)
constexpr int kKlShards = 64;
constexpr int kCtrShard0 = 8, kCtrShardStride = 16;
constexpr int kCtrWords = kCtrShard0 + kCtrShardStride * kKlShards;

struct RunSlot {                     // one in-flight single-sample run (see device_submit)
    hipStream_t stream = nullptr;            // its compute stream (runs of the two slots overlap)
    SiteQ* d_hard = nullptr;                 // KL (KQ, -knownVariants) -> KG queue (KL: kKlShards segments)
    SiteQ* d_hard2 = nullptr;                // KG -> KP queue (compact)
    int64_t cap_hard = 0;
    uint16_t* d_cols = nullptr;              // the queued sites' columns (KL / KG -> KP), u16 entries
    int64_t cap_cols = 0;
    SiteRec* d_brec = nullptr;               // KP's records by position bucket: bucket b = d_brec[b * bcap ..]
    ngsep_site_out* d_ext = nullptr;         // KP's whole records (multi-allelic, pool, dump mode, full_records)
    int64_t cap_ext = 0, guess_ext = 0;
    int32_t* d_bcount = nullptr;             // records per bucket (zeroed by KT)
    int64_t nb_cap = 0, brec_cap = 0;
    LikTables* d_tables = nullptr;
    LikTables h_tables{};                    // last uploaded tables
    bool tables_valid = false;
    SiteRec* d_sorted = nullptr;
    int64_t cap = 0;
    unsigned long long* d_ctr = nullptr;     // its counter set (kCtrWords, see above)
    unsigned long long* h_ctr = nullptr;     // pinned copy
    SiteSet host;                            // pinned D2H destination of the ordered records and the whole ones
    hipEvent_t ev[6] = {};                   // KT start, KT end, KP end, after KO, copies done, KP start
    int64_t guess = 0;
    bool busy = false;
    bool scan_timed = false;                     // this run recorded ev[0] / ev[1] around its scan (KL or KQ)
    int prune = 0;
    GenotypeParams g{};
    LikTables tabs{};
    const Staged* staged = nullptr;
    std::chrono::steady_clock::time_point t0;
};

// KPM's two stages (k_stage_a, then k_posterior_multi over its queue): KLM's (position, sample) pairs of the columns it could not prove hom-ref,
// in kKlShards segments of pseg; KQN's queue index of every need word's first bit; per queued position a 256-bit sample
// mask (zeroed once: the first stage clears what it read); the second stage's queue
struct PopStage {
    uint2* pairs = nullptr;
    int64_t pseg = 0;
    int32_t* qword = nullptr;
    int64_t cap_qword = 0;
    uint32_t* pmask = nullptr;
    QueueSite* qB = nullptr;
    int64_t cap = 0;                         // queue entries of pmask and qB
    void release() {
        (void)hipFree(pairs); (void)hipFree(qword); (void)hipFree(pmask); (void)hipFree(qB);
        pairs = nullptr; qword = nullptr; pmask = nullptr; qB = nullptr;
        pseg = cap_qword = cap = 0;
    }
    hipError_t ensure(int64_t qcap, int64_t nwords, hipStream_t st);   // for a queue of qcap positions over nwords words
};

struct MultiSlot {                   // one in-flight multisample run (device_submit_multi / device_collect_multi)
    QueueSite* d_hard = nullptr;             // KQN -> KPM queue
    int64_t cap_hard = 0;
    uint32_t* d_need = nullptr;              // open positions (a bit per global position)
    int64_t cap_need = 0;                    // words
    bool need_clean = false;                 // d_need is all zero (cleared by the last pass's k_stage_a)
    ngsep_popsite_out* d_psites = nullptr;   // KPM's sites (unordered) and their per-sample calls
    ngsep_sample_call* d_pcalls = nullptr;
    int64_t cap_psites = 0;
    ngsep_popsite_out* h_psites = nullptr;   // pinned D2H destination of the sites
    int64_t cap_h_psites = 0, guess = 0;
    hipEvent_t ev[6] = {};                   // KTM start, KQN end, (unused), KPM end, copies done, calls packed
    bool busy = false;
    PopCall32* d_pack = nullptr;             // KPM's calls packed in KPM's (unordered) site order
    PinnedStore<PopCall32> h_pack;           // pinned D2H destination (handed to the context at collect)
    ngsep_sample_call* d_big = nullptr;      // the calls a PopCall32 cannot hold
    PinnedStore<ngsep_sample_call> h_big;
    int64_t cap_pack = 0;                    // sites
    int64_t guess_big = 0, cap_big = 0;
    PopStage stage;
};

struct Device {
    int ordinal = 0;
    MultiSlot mslot[2];
    int mnext = 0, mfirst = 0, minflight = 0;
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;
    RunSlot slot[2];
    int64_t n_submitted = 0, n_collected = 0;
    // an event between KP and KO costs a few microseconds of idle GPU per pass: recorded only when
    // the posterior kernel's duration is asked for (NGSEP_TIME_POSTERIOR, diagnostics)
    bool time_posterior = env_hook("NGSEP_TIME_POSTERIOR") != nullptr;
    bool time_scan = diag_env("NGSEP_NO_SCAN_TIMING") == nullptr;   // diagnostics: without KT's events
    hipEvent_t ev[4] = {};
    uint8_t* d_pile = nullptr;       // single sample: position-major byte pile; multisample: per-sample blocks
    uint32_t* d_planes = nullptr;    // single sample: valid-call plane of the pile (KT)
    uint16_t* d_olist = nullptr;     // single sample: other-allele call positions per tile (KT)
    int32_t* d_loff = nullptr;       // their per-tile ranges
    size_t cap_olist = 0, cap_loff = 0;
    uint32_t* d_cneg = nullptr;      // single sample: strand bits of the pile's cells (KP)
    int4* d_wins = nullptr;          // windows {global start of w0, w0, seq_id, wlen}, ascending (KO maps records)
    // single-sample buffers are kept from run to run (streamed windows) and grown when a run needs more
    size_t cap_pile = 0, cap_planes = 0, cap_cneg = 0, cap_ref = 0, cap_tinfo = 0, cap_wins = 0;
    int32_t n_wins = 0;
    int32_t planes_W = 0;            // words per plane row (T / 32)
    uint8_t* d_ref = nullptr;
    TileInfo* d_tinfo = nullptr;
    // single-sample variant calling: the read-group layout (engine.hpp RGroup) KL scans
    uint64_t* d_units = nullptr;
    int2* d_rh = nullptr;
    RGroup* d_grp = nullptr;
    int32_t* d_blkA = nullptr;
    int32_t* d_blkB = nullptr;
    size_t cap_units = 0, cap_rh = 0, cap_grp = 0, cap_blk = 0, cap_blkB = 0;
    uint8_t* d_rbytes = nullptr;     // k_build_units' input: the reads' projected bytes back to back, and entry offsets
    int64_t* d_roff = nullptr;
    size_t cap_rbytes = 0, cap_roff = 0;
    char* d_refchars = nullptr;      // k_ref_codes' input: a window's reference characters, and the carved ranges
    int64_t* d_zero = nullptr;
    size_t cap_refchars = 0, cap_zero = 0;
    int64_t n_entries = 0;
    bool rg = false;
    // multisample: the population read-group layout (the units / headers / groups above, engine.hpp Staged::prg)
    bool prg = false;
    int32_t* d_samp_st = nullptr;    //   streams of each sample
    int64_t* d_st_end = nullptr;     //   one past each stream's last entry
    int32_t n_streams = 0, pblk_shift = kRgBlockShift, pop_stride = 0;
    int64_t pnblk = 0;
    int32_t* d_deep_tiles = nullptr; //   KLM tiles some sample covers deeper than kKlmCountMaxCov (k_scan_pop<false>)
    int64_t n_deep_tiles = 0;
    uint8_t* d_deep_flag = nullptr;  //   ... as a byte per tile (k_scan_pop<true> skips them)
    uint8_t* d_gcol = nullptr;       //   KPM / k_stage_a columns when they do not fit LDS (kPopGatherCap)
    size_t cap_gcol = 0;
    uint32_t* d_need = nullptr;      //   open positions, a bit per global position
    bool need_clean = false;         //   d_need is all zero (cleared by the last run's k_stage_a)
    PopStage pstage;                 //   KPM's two stages (device_run_multi)
    ngsep_popsite_out* h_psites = nullptr;      // multisample: pinned staging of the emitted sites and calls
    ngsep_sample_call* h_pcalls = nullptr;
    int64_t cap_h_psites = 0, cap_h_pcalls = 0;
    uint8_t* d_ppile = nullptr;      // multisample: KPM's site-major per-tile pile
    int32_t* d_prow = nullptr;       //   rows per block
    int64_t* d_pboff = nullptr;      //   block offsets
    int32_t n_samples = 0;
    ngsep_popsite_out* d_psites = nullptr;
    ngsep_sample_call* d_pcalls = nullptr;
    QueueSite* d_mforced = nullptr;              // multisample -knownVariants: the input variants to genotype (KPM's queue)
    unsigned long long* d_mforced_ctr = nullptr; //   [2] = their count (KPM's queue length)
    int64_t n_mforced = -1;                      //   -1: discovery (KTM + KQN build the queue)
    PopCall32* d_pcalls_ord = nullptr;           // the kept sites' calls in output order, packed (k_gather_calls)
    ngsep_sample_call* d_pbig = nullptr;         // the calls a PopCall32 cannot hold (+ their counter)
    int64_t cap_pcalls_ord = 0;                  // records
    int64_t* d_csrc = nullptr;                   // staging index of each kept site, in output order
    int64_t* h_csrc = nullptr;                   // (pinned)
    int64_t cap_csrc = 0;
    int64_t cap_psites = 0;
    unsigned long long* d_stamps = nullptr;   // diagnostics (NGSEP_TIMING)
    void* d_rac = nullptr;           // RelativeAlleleCounts: histograms + per-block sums (device, pinned host)
    void* h_rac = nullptr;
    LikTables* d_tables = nullptr;
    PoolTables* d_pool = nullptr;    // ploidy >= 3: the pool algorithm's tables (device_set_pool)
    // host -> device copies of pageable host memory go through these pinned buffers (h2d): the DMA engines only
    // ever read pinned memory
    uint8_t* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_ev[2] = {nullptr, nullptr};
    bool stage_busy[2] = {false, false};
    int stage_k = 0;
    PoolTables h_pool{};             // their last upload
    bool pool_valid = false;
    int32_t ko_shift = 14, ko_bcap = 64;   // 2^ko_shift positions per bucket (grown on overflow)
    QueueSite* d_hard = nullptr;
    int64_t cap_hard = 0;
    unsigned long long* d_counters = nullptr;
    unsigned long long* h_counters = nullptr;
    int64_t cap_sites = 0;
    int64_t n_reads = 0, g_len = 0, n_tiles = 0;
    int32_t max_span = 0, pad = 0, tile = 512, log2_tile = 9;
    int64_t last_n_sites = 1024;
    int64_t last_n_ext = 0;
    int64_t last_hard = 0;
    int64_t last_cols = 0;      // column entries the last run reserved
    int64_t last_exact = 0;     // wave passes of KT's exact integer bound in the last run
    int kt_blocks_per_cu[2] = {0, 0};
    int kt_planes_per_cu[3] = {0, 0, 0};
    LikTables h_tables;         // last uploaded tables (pinned copy source)
    bool tables_valid = false;
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

// A single-sample site for KP: its position and reference code (-knownVariants: the input alleles, kernels.hip
// k_posterior) and its column -- the nonzero codes of the reads covering it in pending-list order, u16 entries
// code | negative strand << 8 at cols[4 coff ..], rows of them (-1: not gathered yet, KG does it; -2: the column
// buffer overflowed, the host grows it and runs the pass again)
struct SiteQ {
    int32_t gpos;
    int32_t rc;
    int32_t coff;          // in units of 4 entries
    int32_t rows;
};
static_assert(sizeof(SiteQ) == 16, "SiteQ layout");


// ------------------------------------------------------------------------------------------
// KP: exact tally + posterior + SNVQ call of the queued candidates -- one lane per site
// ------------------------------------------------------------------------------------------
// The codes of the reads covering gpos are one contiguous column of the position-major byte pile,
// already in pending-list rank order (engine.cpp build_single_layout), and their strands the matching
// bits of the strand array.  A lane walks its site's column in rank order and runs
// CountsHelper.calculateCountsSNV/updateCounts (discovery/CountsHelper.java:83-95,209-251): the ten
// fp64 log-likelihood sums get their addends in the reference's order, so they are bit-identical; then
// getPosteriorProbabilities / calculatePosteriorProbabilities (:410-495, events in Java's order, the
// normaliser summed in that order), VariantDiscoverySNVQAlgorithm.discoverSNV / getIndexesMaxGenotype
// (:100-243) and the listener filters (SingleSampleVariantPileupListener.java:213-232).  No cross-lane
// work: every lane of the wave does useful fp64 work on its own site.  An emitted record goes to the
// bucket of its position (KO orders the buckets).
__device__ inline double pow10_j(double x) { return pow(10.0, x); }   // Math.pow(10.0, x)
// getPosteriorProbabilities' 16 events (row i: (i,i), then (i,j), j != i ascending) take L[min][max]: event (j,i) has
// the exponent of the earlier event (i,j).  The earlier one's index (0: none): 5->1, 9->2, 10->6, 13->3, 14->7, 15->11
__device__ __forceinline__ int ev_partner(int k) {
    constexpr unsigned long long kTab = (1ull << 20) | (2ull << 36) | (6ull << 40) | (3ull << 52) | (7ull << 56) | (11ull << 60);
    return (int)((kTab >> (4 * k)) & 15ull);
}

// One emitted site into its bucket slot: the 64-B SiteRec (engine.hpp) from the record's header dwords h
// (ngsep_site_out layout: seq, gpos, ref|n_alleles|alt|third, genotype|strand_bias|gq, qual|is_call|pool, dp,
// counts[4], strand_counts[4][2]) and its ten log-conditionals L.  A record the 64 B cannot hold (whole =
// multi-allelic / pool / dump / full_records, or counts past 65535) goes whole to ext, the SiteRec pointing to it.
__device__ inline void put_site(SiteRec* __restrict__ slot, ngsep_site_out* __restrict__ ext, unsigned long long* ext_n,
                                int64_t ext_cap, const uint32_t (&h)[18], const double (&L)[10], bool whole, int ri, int ai) {
    uint32_t big = 0;
#pragma unroll
    for (int t = 6; t < 18; t++) big |= h[t];
    whole = whole || big > 0xFFFFu || ri < 0 || ri > 3 || ai < 0 || ai > 3;
    auto pick = [&](int k) {                           // L[k] without dynamic register indexing
        double v = 0;
#pragma unroll
        for (int e = 0; e < 10; e++) v = e == k ? L[e] : v;
        return v;
    };
    auto tri = [](int i, int j) {
        const int a = i < j ? i : j, b = i < j ? j : i;
        return (a == 0 ? 0 : a == 1 ? 4 : a == 2 ? 7 : 9) + (b - a);
    };
    auto sel = [&](int k) {                            // h[k] for k in 10..17
        uint32_t v = 0;
#pragma unroll
        for (int e = 10; e < 18; e++) v = e == k ? h[e] : v;
        return v;
    };
    uint32_t w[16];
    w[0] = h[0]; w[1] = h[1]; w[2] = h[2]; w[3] = h[3];
    w[4] = h[4] | (whole ? (uint32_t)kRecExt << 16 : 0u);
    w[5] = h[5];
    w[6] = (h[6] & 0xFFFFu) | h[7] << 16;
    w[7] = (h[8] & 0xFFFFu) | h[9] << 16;
    double d0 = 0, d1 = 0, d2 = 0;
    if (whole) {
        w[8] = w[9] = 0;
        const unsigned long long e = atomicAdd(ext_n, 1ull);
        if ((int64_t)e < ext_cap) {
            uint32_t* o = reinterpret_cast<uint32_t*>(ext + e);
#pragma unroll
            for (int t = 0; t < 18; t++) o[t] = h[t];
#pragma unroll
            for (int t = 0; t < 10; t++) {
                const unsigned long long bits = __builtin_bit_cast(unsigned long long, L[t]);
                o[18 + 2 * t] = (uint32_t)bits;
                o[19 + 2 * t] = (uint32_t)(bits >> 32);
            }
        }
        d0 = __builtin_bit_cast(double, (long long)e);
    } else {
        w[8] = (sel(10 + 2 * ri) & 0xFFFFu) | sel(11 + 2 * ri) << 16;
        w[9] = (sel(10 + 2 * ai) & 0xFFFFu) | sel(11 + 2 * ai) << 16;
        d0 = pick(tri(ri, ri));
        d1 = pick(tri(ri, ai));
        d2 = pick(tri(ai, ai));
    }
    const unsigned long long b0 = __builtin_bit_cast(unsigned long long, d0), b1 = __builtin_bit_cast(unsigned long long, d1),
                             b2 = __builtin_bit_cast(unsigned long long, d2);
    w[10] = (uint32_t)b0; w[11] = (uint32_t)(b0 >> 32);
    w[12] = (uint32_t)b1; w[13] = (uint32_t)(b1 >> 32);
    w[14] = (uint32_t)b2; w[15] = (uint32_t)(b2 >> 32);
    uint4* o = reinterpret_cast<uint4*>(slot);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    o[2] = make_uint4(w[8], w[9], w[10], w[11]);
    o[3] = make_uint4(w[12], w[13], w[14], w[15]);
}

constexpr int kPostThreads = 256;
__global__ __launch_bounds__(kPostThreads) void k_posterior(const SiteQ* __restrict__ queue, const unsigned long long* qn,
                                                   int64_t qcap, const uint16_t* __restrict__ cols,
                                                   const LikTables* __restrict__ tabs, GenotypeParams gp,
                                                   SiteRec* __restrict__ brec, int32_t* __restrict__ bcount,
                                                   int shift, int32_t bcap, ngsep_site_out* __restrict__ ext,
                                                   unsigned long long* ext_n, int64_t ext_cap) {
    __shared__ double s_t[3][32];   // A (log10(1-e)), H (heterozygous), E (error) per capped quality
    __shared__ double s_ev[16][kPostThreads];   // each lane's 16 genotype events (posterior phase)
    if (threadIdx.x < 96)
        s_t[threadIdx.x >> 5][threadIdx.x & 31] =
            (threadIdx.x < 32 ? tabs->A : threadIdx.x < 64 ? tabs->H : tabs->E)[threadIdx.x & 31];
    __syncthreads();
    int64_t n = (int64_t)*qn;
    if (n > qcap) n = qcap;
    const int64_t stride = (int64_t)gridDim.x * kPostThreads;
    for (int64_t i = (int64_t)blockIdx.x * kPostThreads + threadIdx.x; i < n; i += stride) {
        const SiteQ qs = queue[i];
        const int32_t gpos = qs.gpos;
        const uint32_t rc = (uint32_t)qs.rc;
        const int32_t rows = qs.rows;
        if (rows < 0) continue;                    // no column: an overflowed pass, which the host runs again
        // tally in rank (= pending-list) order
        int32_t total = 0;
        int32_t cnt[4] = {0, 0, 0, 0};
        int32_t sc[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        // L00 L01 L02 L03 L11 L12 L13 L22 L23 L33 (upper triangle, ngsep_site_out.logc order)
        double L[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        // the column's entries in order (rank r = entry r: two per dword) through a window of 8 dwords in flight
        // (the column buffer has 64 bytes of slack, so the loads past the column need no guard); a small loop, so
        // the kernel's code stays in the instruction cache
        {
            const uint32_t* cw = reinterpret_cast<const uint32_t*>(cols) + ((int64_t)qs.coff << 1);
            const int nd = (rows + 1) >> 1;
            uint32_t q0 = cw[0], q1 = cw[1], q2 = cw[2], q3 = cw[3], q4 = cw[4], q5 = cw[5], q6 = cw[6], q7 = cw[7];
            for (int k = 0; k < nd; k++) {
                const uint32_t d = q0;
                q0 = q1; q1 = q2; q2 = q3; q3 = q4; q4 = q5; q5 = q6; q6 = q7;
                q7 = cw[k + 8];
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const int r = 2 * k + e;                               // rank of this entry
                    const uint32_t ent = r < rows ? (d >> (16 * e)) & 0xFFFFu : 0u;
                    const uint32_t cd = ent & 0xFFu;
                    if (cd == 0) continue;
                    total++;                                              // CountsHelper.java:210
                    if (!(cd & 0x80u)) continue;                          // q<=3 or not A/C/G/T (:214-221)
                    const int a = (int)((cd >> 5) & 3u);
                    int q = (int)(cd & 31u);
                    q = q > gp.max_q ? gp.max_q : q;                      // -maxBaseQS (:217-219)
                    const int neg = (int)((ent >> 8) & 1u);
#pragma unroll
                    for (int t = 0; t < 4; t++) {                         // constant indices: registers, not scratch
                        cnt[t] += a == t ? 1 : 0;
                        sc[t][0] += (a == t && neg) ? 1 : 0;              // countsStrand[idx][neg?0:1] (:226-227)
                        sc[t][1] += (a == t && !neg) ? 1 : 0;
                    }
                    const double A = s_t[0][q], H = s_t[1][q], E = s_t[2][q];
                    // updateCounts (:231-248): [i][i] += i==idx ? A : E; [i][j] += (i==idx || j==idx) ? H : E
                    L[0] += a == 0 ? A : E;
                    L[1] += (a == 0 || a == 1) ? H : E;
                    L[2] += (a == 0 || a == 2) ? H : E;
                    L[3] += (a == 0 || a == 3) ? H : E;
                    L[4] += a == 1 ? A : E;
                    L[5] += (a == 1 || a == 2) ? H : E;
                    L[6] += (a == 1 || a == 3) ? H : E;
                    L[7] += a == 2 ? A : E;
                    L[8] += (a == 2 || a == 3) ? H : E;
                    L[9] += a == 3 ? A : E;
                }
            }
        }
        const bool known = (rc & 0x400u) != 0;     // -knownVariants site: ref (bits 5-6) and alt (bits 8-9) given
        if ((total == 0 && !known) || ABLATE(gp.ablate, 8)) continue;        // VariantDiscoverySNVQAlgorithm.java:101-103
        const bool callable = (rc & 0x80u) != 0;
        int8_t genotype = -1, alt = -1, third = -1, nal = 0;
        int16_t gq = 0, qual = 0;
        bool keep = false;
        if (known) {
            // genotypeVariantSample (SingleSampleVariantPileupListener.java:361-391) -> genotypeSNV
            // (VariantDiscoverySNVQAlgorithm.java:21-62): hom-ref, hom-alt (+0.01), het (+0.01) over the input
            // alleles; GQ 0 or below -minQuality: undecided.  No calls at all: undecided, no log-conditionals.
            const int r = (int)((rc >> 5) & 3u), a = (int)((rc >> 8) & 3u);
            nal = 2;
            alt = (int8_t)a;
            keep = true;
            if (total > 0) {
                constexpr int kEv[16] = {0, 1, 2, 3, 4, 1, 5, 6, 7, 2, 5, 8, 9, 3, 6, 8};
                double ev[16];
#pragma unroll
                for (int k = 0; k < 16; k++) ev[k] = L[kEv[k]] + ((k & 3) == 0 ? gp.log_prior_homo : gp.log_prior_hetero);
                double logMax = 1;
#pragma unroll
                for (int k = 0; k < 16; k++)
                    if (logMax > 0 || logMax < ev[k]) logMax = ev[k];
                uint32_t act = 0;
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const double x = ev[k] - logMax;
                    const bool on = !(x < -20);
                    act |= on ? 1u << k : 0u;
                    s_ev[k][threadIdx.x] = on ? x : 0.0;
                }
                double totalProb = 0;
                for (uint32_t rem = act; rem; rem &= rem - 1) {
                    const int k = __builtin_ctz(rem);
                    const int src = ev_partner(k);
                    const double pk = src ? s_ev[src][threadIdx.x] : pow10_j(s_ev[k][threadIdx.x]);
                    totalProb += pk;
                    s_ev[k][threadIdx.x] = pk;
                }
                for (uint32_t rem = act; rem; rem &= rem - 1) {
                    const int k = __builtin_ctz(rem);
                    s_ev[k][threadIdx.x] = s_ev[k][threadIdx.x] / totalProb;
                }
                auto post = [&](int i, int j) -> double {
                    return s_ev[i == j ? 4 * i : 4 * i + (j < i ? j + 1 : j)][threadIdx.x];
                };
                double pMax = post(r, r);
                int gt = 0;
                if (post(a, a) > pMax + 0.01) { pMax = post(a, a); gt = 2; }
                const double pHet = post(r, a) + post(a, r);
                if (pHet > pMax + 0.01) { pMax = pHet; gt = 1; }
                gq = phred_d(1 - pMax);
                if (gq == 0) gt = -1;
                if (gp.min_quality > gq) { gt = -1; gq = 0; }           // makeUndecided (:388)
                genotype = (int8_t)gt;
            }
        } else if (callable) {
            const int refIdx = (int)((rc >> 5) & 3u);
            // getPosteriorProbabilities (CountsHelper.java:410-443): events in Java's order -- row i holds
            // (i,i) then (i,j) for j != i ascending; L is symmetric
            constexpr int kEv[16] = {0, 1, 2, 3, 4, 1, 5, 6, 7, 2, 5, 8, 9, 3, 6, 8};   // event -> L index
            double ev[16];
#pragma unroll
            for (int k = 0; k < 16; k++) ev[k] = L[kEv[k]] + ((k & 3) == 0 ? gp.log_prior_homo : gp.log_prior_hetero);
            // calculatePosteriorProbabilities (:472-495).  Events more than 20 below the maximum are 0 and add
            // nothing to the normaliser, so only the others take a pow and a division -- each lane walks its
            // own active events in Java's order, so the normaliser is summed exactly as the reference does.
            // The lane's 16 events live in LDS (column tid), so the walk indexes them without scratch memory.
            double logMax = 1;
#pragma unroll
            for (int k = 0; k < 16; k++)
                if (logMax > 0 || logMax < ev[k]) logMax = ev[k];
            uint32_t act = 0;
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const double x = ev[k] - logMax;
                const bool on = !(x < -20);
                act |= on ? 1u << k : 0u;
                s_ev[k][threadIdx.x] = on ? x : 0.0;
            }
            double totalProb = 0;
            for (uint32_t rem = act; rem; rem &= rem - 1) {
                const int k = __builtin_ctz(rem);
                const int src = ev_partner(k);              // (j, i) repeats (i, j)'s exponent: its pow is reused
                const double pk = src ? s_ev[src][threadIdx.x] : pow10_j(s_ev[k][threadIdx.x]);
                totalProb += pk;
                s_ev[k][threadIdx.x] = pk;
            }
            for (uint32_t rem = act; rem; rem &= rem - 1) {
                const int k = __builtin_ctz(rem);
                s_ev[k][threadIdx.x] = s_ev[k][threadIdx.x] / totalProb;
            }
#pragma unroll
            for (int k = 0; k < 16; k++) ev[k] = s_ev[k][threadIdx.x];
            // post(i, j) is event 4i + (j < i ? j + 1 : j) for j != i, 4i for j == i
            auto post = [&](int i, int j) -> double {
                return s_ev[i == j ? 4 * i : 4 * i + (j < i ? j + 1 : j)][threadIdx.x];
            };
            // getIndexesMaxGenotype (VariantDiscoverySNVQAlgorithm.java:223-243), default index = reference
            int I = refIdx, J = refIdx;
            const double refProb = post(refIdx, refIdx);
            double probMax = refProb;
#pragma unroll
            for (int pi = 0; pi < 4; pi++)
#pragma unroll
                for (int pj = pi; pj < 4; pj++) {
                    const int k1 = pi == pj ? 4 * pi : 4 * pi + pj;          // (pi, pj), pj > pi
                    const int k2 = 4 * pj + pi + 1;                          // (pj, pi), pi < pj
                    double g = ev[k1];
                    if (pi != pj) g += ev[k2];
                    if (g > probMax + 0.01) { probMax = g; I = pi; J = pj; }
                }
            gq = phred_d(1 - probMax);
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
        // the record goes to its position bucket (KO orders each bucket)
        const int32_t bk = gpos >> shift;
        const int32_t k = atomicAdd(&bcount[bk], 1);
        if (k >= bcap) continue;                       // overflow: the host grows the buckets and reruns
        uint32_t h[18];
        h[0] = 0xFFFFFFFFu;
        h[1] = (uint32_t)gpos;
        const uint32_t ref = callable ? (uint32_t)(uint8_t)"ACGT"[(rc >> 5) & 3] : (uint32_t)'N';
        h[2] = ref | (uint32_t)(uint8_t)nal << 8 | (uint32_t)(uint8_t)alt << 16 | (uint32_t)(uint8_t)third << 24;
        h[3] = (uint32_t)(uint8_t)genotype | 0xFF00u | (uint32_t)(uint16_t)gq << 16;
        h[4] = (uint32_t)(uint16_t)qual | (uint32_t)(keep ? 1 : 0) << 16;
        h[5] = (uint32_t)total;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            h[6 + t] = (uint32_t)cnt[t];
            h[10 + 2 * t] = (uint32_t)sc[t][0];
            h[11 + 2 * t] = (uint32_t)sc[t][1];
        }
        const int ri = callable ? (int)((rc >> 5) & 3u) : -1;
        put_site(brec + (int64_t)bk * bcap + k, ext, ext_n, ext_cap, h, L, gp.full_records != 0 || nal != 2, ri, alt);
    }
}


// ------------------------------------------------------------------------------------------
// KPP: ploidy >= 3 -- the pool algorithm over the queued candidates, one lane per site
// ------------------------------------------------------------------------------------------
// SingleSampleVariantPileupListener.discoverSNV's pool branch (:238-254): createSNVVariantPool (:297-332)
// picks the variant's alleles from the SNV counts (count >= max(1, 0.5/ploidy * sum)), genotypeVariantPool
// (:402-503) scores one homozygous and nf heterozygous-frequency hypotheses per alternative allele, a
// multi-allelic variant called {0, k} or {k} is re-genotyped as the biallelic {ref, k}; -knownVariants sites
// (genotypeVariantSample, :361-391) genotype the input's two alleles.  Every likelihood sum is the
// CountsHelper.updateCounts addend sequence (CountsHelper.java:209-251) over the site's column in rank
// order, so each sum is bit-identical; only the entries the decision reads are formed: the major allele's
// row for each hypothesis, then the report's upper triangle at the chosen hypothesis.
struct PoolResult {
    int n_called, c0, c1;       // called allele indexes into the variant's alleles (ascending)
    int gq, dp;                 // dp: setTotalReadDepth (0 for the undecided low-count call)
    bool report;                // VariantCallReport present
    int acn[4];                 // setAllelesCopyNumber of genotypeVariantPool (:480-497) over the variant's alleles
    double L[10];               // report log-conditionals, upper triangle over the variant's alleles
};

// one pass over a site's column: f(allele index into dna[] or -1, capped q) for every counted call
// (q <= 3: lowBaseQualityCount only, not passed).  A column is code bytes (KPM's pile) or u16 entries whose low
// byte is the code (KP's columns)
template <class C, class F>
__device__ inline void pool_walk(const C* __restrict__ col, int32_t rows, const int* dna, int n, int32_t max_q, F&& f) {
    for (int32_t r = 0; r < rows; r++) {
        const uint32_t cd = col[r] & 0xFFu;
        if (!(cd & 0x80u)) continue;                   // no call, or q <= 3 / not A,C,G,T: no likelihood update
        const int a = (int)((cd >> 5) & 3u);
        int q = (int)(cd & 31u);
        q = q > max_q ? max_q : q;
        int idx = -1;                                  // alleles.indexOf(allele)
        for (int i = 0; i < n; i++) idx = (idx < 0 && dna[i] == a) ? i : idx;
        if (idx >= 0) f(idx, q);
    }
}

// genotypeVariantPool for the variant dna[0..n) (reference first); cnt4 = the column's A,C,G,T valid counts
template <class C>
__device__ PoolResult pool_genotype(const C* __restrict__ col, int32_t rows, int32_t total, const int* cnt4,
                                    const int* dna, int n, const PoolTables* __restrict__ pt, int32_t max_q) {
    PoolResult R;
    R.n_called = 0; R.c0 = -1; R.c1 = -1; R.gq = 0; R.dp = 0; R.report = false;
    R.acn[0] = R.acn[1] = R.acn[2] = R.acn[3] = 0;
    for (int k = 0; k < 10; k++) R.L[k] = 0;
    const int P = pt->ploidy, nf = pt->nf, ni = n - 2;
    int major = 0;                                     // NumberArrays.getIndexMaximum: the first maximum
    for (int i = 1; i < n; i++) major = cnt4[dna[major]] < cnt4[dna[i]] ? i : major;
    if (cnt4[dna[major]] < P) return R;                // undecided, no report (:436-440)
    // the major allele's row L_j[major][*] of every hypothesis j
    double Lr[kPoolMaxFreq][4];
    for (int j = 0; j < nf; j++) {
        double l0 = 0, l1 = 0, l2 = 0, l3 = 0;
        pool_walk(col, rows, dna, n, max_q, [&](int idx, int q) {
            const double A = pt->A[q], E = pt->E[ni][q], Fv = pt->F[j][ni][q], Gv = pt->G[j][ni][q];
            // [m][m] += idx == m ? A : E;  [m][k] += k == idx ? F : (m == idx ? G : E)
            const double v0 = major == 0 ? (idx == 0 ? A : E) : (idx == 0 ? Fv : (major == idx ? Gv : E));
            const double v1 = major == 1 ? (idx == 1 ? A : E) : (idx == 1 ? Fv : (major == idx ? Gv : E));
            const double v2 = major == 2 ? (idx == 2 ? A : E) : (idx == 2 ? Fv : (major == idx ? Gv : E));
            const double v3 = major == 3 ? (idx == 3 ? A : E) : (idx == 3 ? Fv : (major == idx ? Gv : E));
            l0 += v0; l1 += v1;
            if (n > 2) l2 += v2;
            if (n > 3) l3 += v3;
        });
        Lr[j][0] = l0; Lr[j][1] = l1; Lr[j][2] = l2; Lr[j][3] = l3;
    }
    const double termHomozygous = Lr[0][major] + pt->log_1h;
    double maxHetPosterior = 0, minHomoPosterior = 1;
    int maxFreqIdx = 0, maxAlt = -1;
    for (int i = 0; i < n; i++) {
        if (i == major) continue;
        // calculatePosteriorProbabilities over {homozygous, hypothesis 0..nf-1} (CountsHelper.java:472-495)
        double logMax = 1;
        for (int j = -1; j < nf; j++) {
            const double x = j < 0 ? termHomozygous : Lr[j][i] + pt->log_h;
            if (logMax > 0 || logMax < x) logMax = x;
        }
        double totalProb = 0;
        for (int j = -1; j < nf; j++) {
            const double x = (j < 0 ? termHomozygous : Lr[j][i] + pt->log_h) - logMax;
            totalProb += x < -20 ? 0.0 : pow10_j(x);
        }
        int idxMax = 0;
        double best = 0, post0 = 0;
        for (int j = -1; j < nf; j++) {
            const double x = (j < 0 ? termHomozygous : Lr[j][i] + pt->log_h) - logMax;
            const double pj = (x < -20 ? 0.0 : pow10_j(x)) / totalProb;
            if (j < 0) { post0 = pj; best = pj; }
            else if (best < pj) { best = pj; idxMax = j + 1; }
        }
        if (idxMax == 0) minHomoPosterior = post0 < minHomoPosterior ? post0 : minHomoPosterior;
        else if (maxAlt == -1 || maxHetPosterior < best) { maxHetPosterior = best; maxFreqIdx = idxMax - 1; maxAlt = i; }
    }
    if (maxAlt == -1) { R.n_called = 1; R.c0 = major; }
    else { R.n_called = 2; R.c0 = major < maxAlt ? major : maxAlt; R.c1 = major < maxAlt ? maxAlt : major; }
    R.dp = total;
    const int jr = maxAlt == -1 ? 0 : maxFreqIdx;      // the report's hypothesis
    auto set_acn = [&](int k, int v) {
#pragma unroll
        for (int e = 0; e < 4; e++) R.acn[e] = e == k ? v : R.acn[e];
    };
    if (maxAlt == -1) {
        R.gq = phred_d(1 - minHomoPosterior);
        set_acn(major, P);
    } else {
        int altCN = (int)(int16_t)java_round_d(pt->freq[maxFreqIdx] * P);
        if (altCN == 0) altCN++;
        else if (altCN == P) altCN--;
        set_acn(maxAlt, altCN);
        set_acn(major, P - altCN);
        // getPosteriorProbabilities(h, major) (CountsHelper.java:451-467) over the chosen hypothesis' row
        const double lph = pt->log_h_n[ni];
        double logMax = 1;
        for (int k = 0; k < n; k++) {
            const double x = Lr[jr][k] + (k == major ? pt->log_1h : lph);
            if (logMax > 0 || logMax < x) logMax = x;
        }
        double totalProb = 0, pAlt = 0;
        for (int k = 0; k < n; k++) {
            const double x = Lr[jr][k] + (k == major ? pt->log_1h : lph) - logMax;
            const double pk = x < -20 ? 0.0 : pow10_j(x);
            totalProb += pk;
            if (k == maxAlt) pAlt = pk;
        }
        R.gq = phred_d(1 - pAlt / totalProb);
    }
    // the report: the chosen helper's log-conditionals, upper triangle
    R.report = true;
    double L[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    pool_walk(col, rows, dna, n, max_q, [&](int idx, int q) {
        const double A = pt->A[q], E = pt->E[ni][q], Fv = pt->F[jr][ni][q], Gv = pt->G[jr][ni][q];
        int k = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = i; j < 4; j++) {
                if (j < n) {
                    // [i][i] += i == idx ? A : E;  [i][j] += j == idx ? F : (i == idx ? G : E)
                    const double v = i == j ? (i == idx ? A : E) : (j == idx ? Fv : (i == idx ? Gv : E));
                    L[k] += v;
                }
                k++;
            }
    });
    // repack the 4x4 upper triangle into the n-allele upper triangle
    int o = 0, k = 0;
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = i; j < 4; j++) {
            if (j < n) R.L[o++] = L[k];
            k++;
        }
    return R;
}

__global__ __launch_bounds__(kPostThreads) void k_posterior_pool(const SiteQ* __restrict__ queue, const unsigned long long* qn,
                                                        int64_t qcap, const uint16_t* __restrict__ cols,
                                                        const PoolTables* __restrict__ pt, GenotypeParams gp,
                                                        SiteRec* __restrict__ brec, int32_t* __restrict__ bcount,
                                                        int shift, int32_t bcap, ngsep_site_out* __restrict__ ext,
                                                        unsigned long long* ext_n, int64_t ext_cap) {
    int64_t nq = (int64_t)*qn;
    if (nq > qcap) nq = qcap;
    const int64_t stride = (int64_t)gridDim.x * kPostThreads;
    for (int64_t i = (int64_t)blockIdx.x * kPostThreads + threadIdx.x; i < nq; i += stride) {
        const SiteQ qs = queue[i];
        const int32_t gpos = qs.gpos;
        const uint32_t rc = (uint32_t)qs.rc;
        const int32_t rows = qs.rows;
        if (rows < 0) continue;                    // no column: an overflowed pass, which the host runs again
        const uint16_t* col = cols + ((int64_t)qs.coff << 2);
        // the SNV tally of calculateCountsSNV (CountsHelper.java:83-95): totals, A,C,G,T and strand counts
        int32_t total = 0;
        int cnt[4] = {0, 0, 0, 0};
        int32_t sc[4][2] = {{0, 0}, {0, 0}, {0, 0}, {0, 0}};
        for (int32_t r = 0; r < rows; r++) {
            const uint32_t ent = col[r];
            const uint32_t cd = ent & 0xFFu;
            if (cd == 0) continue;
            total++;
            if (!(cd & 0x80u)) continue;
            const int a = (int)((cd >> 5) & 3u);
            const int neg = (int)((ent >> 8) & 1u);
#pragma unroll
            for (int t = 0; t < 4; t++) {
                cnt[t] += a == t ? 1 : 0;
                sc[t][0] += (a == t && neg) ? 1 : 0;
                sc[t][1] += (a == t && !neg) ? 1 : 0;
            }
        }
        const bool known = (rc & 0x400u) != 0;
        const bool callable = (rc & 0x80u) != 0;
        int dna[4] = {0, 0, 0, 0};
        int n = 0;
        bool keep = false, multi = false;
        PoolResult R;
        R.n_called = 0; R.c0 = -1; R.c1 = -1; R.gq = 0; R.dp = 0; R.report = false;
        if (known) {
            dna[0] = (int)((rc >> 5) & 3u);
            dna[1] = (int)((rc >> 8) & 3u);
            n = 2;
            R = pool_genotype(col, rows, total, cnt, dna, n, pt, gp.max_q);
            if (gp.min_quality > R.gq) { R.n_called = 0; R.c0 = R.c1 = -1; R.gq = 0; }   // makeUndecided (:388)
            keep = true;
        } else if (callable && total > 0) {
            // createSNVVariantPool(pileup, helperSNV, reference, 0.5 / ploidy)
            const int refIdx = (int)((rc >> 5) & 3u);
            const int sum = cnt[0] + cnt[1] + cnt[2] + cnt[3];
            double minCount = (0.5 / (double)pt->ploidy) * sum;
            minCount = minCount < 1 ? 1 : minCount;
            dna[n++] = refIdx;
            for (int t = 0; t < 4; t++)
                if (cnt[t] >= minCount && t != refIdx) dna[n++] = t;
            if (n >= 2) {
                multi = n > 2;
                R = pool_genotype(col, rows, total, cnt, dna, n, pt, gp.max_q);
                bool ok = true;
                if (multi) {
                    if (R.n_called == 0 || (R.n_called == 1 && R.c0 == 0)) ok = false;
                    else if (!(R.n_called == 2 && R.c0 != 0)) {
                        // makeNewVariant(variant, {ref} + called alleles) (:346-359): the biallelic SNV
                        const int alt = R.n_called == 1 ? dna[R.c0] : dna[R.c1];
                        dna[1] = alt;
                        n = 2;
                        multi = false;
                        R = pool_genotype(col, rows, total, cnt, dna, n, pt, gp.max_q);
                    }
                }
                // discoverVariant (:221-227): undecided, hom-ref and GQ below -minQuality are dropped
                keep = ok && R.n_called > 0 && !(R.n_called == 1 && R.c0 == 0) && !(gp.min_quality > R.gq);
            }
        }
        if (!keep) continue;
        const int32_t bk = gpos >> shift;
        const int32_t k = atomicAdd(&bcount[bk], 1);
        if (k >= bcap) continue;                       // overflow: the host grows the buckets and reruns
        uint32_t mask = 0;
        for (int t = 0; t < n; t++) mask |= 1u << dna[t];
        const int a0 = R.c0 >= 0 ? dna[R.c0] : -1, a1 = R.c1 >= 0 ? dna[R.c1] : -1;
        uint32_t h[18];
        h[0] = 0xFFFFFFFFu;
        h[1] = (uint32_t)gpos;
        const uint32_t ref = (uint32_t)(uint8_t)"ACGT"[dna[0]];
        h[2] = ref | (uint32_t)(uint8_t)n << 8 | (uint32_t)(uint8_t)(int8_t)a0 << 16 | (uint32_t)(uint8_t)(int8_t)a1 << 24;
        // -knownVariants: genotypeVariantPool's copy number of the first called allele of a heterozygous call (the
        // writer keeps it past the sequence's first record, vcf.cpp format_site) in the strand-bias byte; -1 otherwise
        int acn0 = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) acn0 = e == R.c0 ? R.acn[e] : acn0;
        const uint32_t sb = (known && R.n_called == 2) ? (uint32_t)(uint8_t)acn0 : 0xFFu;
        h[3] = (uint32_t)(uint8_t)R.n_called | sb << 8 | (uint32_t)(uint16_t)R.gq << 16;
        h[4] = 1u << 16 | (mask | (R.report ? 0x10u : 0u)) << 24;
        h[5] = (uint32_t)R.dp;
#pragma unroll
        for (int t = 0; t < 4; t++) {
            h[6 + t] = (uint32_t)cnt[t];
            h[10 + 2 * t] = (uint32_t)sc[t][0];
            h[11 + 2 * t] = (uint32_t)sc[t][1];
        }
        put_site(brec + (int64_t)bk * bcap + k, ext, ext_n, ext_cap, h, R.L, true, dna[0], -1);
        (void)multi;
    }
}


// ------------------------------------------------------------------------------------------
// KL: the single-sample scan over the read-group layout -- one workgroup per tile of T positions
// ------------------------------------------------------------------------------------------
// AlignmentsPileupGenerator.processCurrentPosition (discovery/AlignmentsPileupGenerator.java:475-498) reduced to
// what decides whether SNVQ can call a variant at a position, straight from the packed
// reads (engine.hpp RGroup: 1 B per read base, 8 B per read header):
//   * coverage: every read segment inside the tile adds +1 / -1 to an LDS difference array (2 atomics per read);
//   * exceptions: a wave takes a group of 64 reads, lane = read, and streams its 8-byte units (512 contiguous
//     bytes per wave load, kKlUnroll loads in flight per lane); a byte is an exception when its position is
//     callable and it is not a valid call of the reference allele (SWAR against the tile's reference codes in
//     LDS).  Exceptions (a few % of the bytes) add to the position's LDS counter: low half = exceptions, high
//     half = valid calls of another allele (na);
//   * candidates: callable positions with na > 0; the reference calls are nr = coverage - exceptions, and the
//     count bound (table cb_nr) drops those whose counts prove them hom-ref.  A position
//     deeper than 65535 reads (the halves could carry into each other) is queued whenever it is callable;
//   * survivors: queued for KP with their column space reserved (rows = -3 - coverage); KG gathers the columns.
//     The workgroup's queue slots and column space come from one atomic each (a block scan orders them).
// No MFMA: byte SWAR and integer counters.
constexpr int kKlThreads = 256;
#ifndef NGSEP_KL_UNROLL
#define NGSEP_KL_UNROLL 4
#endif
constexpr int kKlUnroll = NGSEP_KL_UNROLL;
// units allocated past a layout's last group: KL's and KLM's next-batch loads are unconditional and may read up to
// 2 x 4 - 1 rows past a read's last unit, the last group's included (never used, only loaded)
constexpr int64_t kUnitSlack = 8 + 64 * 8;
static_assert(NGSEP_KL_UNROLL <= 4, "kUnitSlack covers batches of at most 4 units");

// PileupRecord.getAlleleCalls(1) at global position p over the read-group layout: the nonzero codes of the reads
// covering p, in pending-list (entry) order, as u16 entries code | negative strand << 8 (WRITE), one wave.  e0 is
// at or before the first entry that can cover p (blkA).  Returns the entries written; *cov = the covering reads.
template <bool WRITE>
__device__ inline int32_t wave_gather(int32_t p, int64_t e0, int64_t n_entries, const int2* __restrict__ rh,
                                      const RGroup* __restrict__ grp, const uint64_t* __restrict__ units,
                                      uint32_t refcode, uint16_t* __restrict__ dst, int32_t* cov_out) {
    const int lane = threadIdx.x & 63;
    int32_t n = 0, cov = 0;
    int64_t e = e0 & ~(int64_t)63;
    int2 h = e < n_entries ? rh[e + lane] : make_int2(0x7FFFFFFF, 0);
    for (; e < n_entries; e += 64) {
        const int2 hn = e + 64 < n_entries ? rh[e + 64 + lane] : make_int2(0x7FFFFFFF, 0);   // next chunk in flight
        const int32_t gf = h.x, gl = h.y & 0x7FFFFFFF;
        const bool covers = gf <= p && p <= gl;
        cov += (int32_t)__popcll(__ballot(covers));
        if (WRITE) {
            uint32_t code = 0;
            if (covers) {
                const RGroup G = grp[e >> 6];
                const int32_t o = p - gf;
                const uint64_t u = units[G.base + (int64_t)(o >> 3) * 64 + lane];
                code = ((uint32_t)(u >> (8 * (o & 7))) & 0xFFu) ^ refcode;   // (the layout is reference-relative)
            }
            const unsigned long long m = __ballot(code != 0);
            if (code) {
                const int rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                dst[n + rk] = (uint16_t)(code | (((uint32_t)h.y >> 31) << 8));
            }
            n += (int32_t)__popcll(m);
        }
        if (__ballot(gf > p)) break;                       // entries are sorted by gfirst: none later covers p
        h = hn;
    }
    if (cov_out) *cov_out = cov;
    return n;
}

// KL's flags from reference-relative bytes y = code ^ reference code (bit 7 of byte k):
__device__ __forceinline__ uint32_t kl_exc(uint32_t y) {
    // not a valid call of the reference's allele (bits 5-7 differ); at a callable position an exception
    return ((((y >> 5) & 0x07070707u) + 0x7F7F7F7Fu) & 0x80808080u);
}
__device__ __forceinline__ uint32_t kl_nonref(uint32_t y) {
    // a valid call (code bit 7 = reference bit 7) of another allele (bits 5-6 differ)
    return ((((y >> 5) & 0x03030303u) + 0x7F7F7F7Fu) & ~y & 0x80808080u);
}

// KL's read stream over the tile's groups (wave w: groups g_lo + w, g_lo + w + 4, ...).  A lane takes its read's
// units from the first one inside the tile in batches of kKlUnroll, the next batch's loads issued before the
// current batch's counter adds (software pipelined: 4-8 loads in flight per lane at 64 VGPRs, 8 waves per SIMD), and
// the next group's headers and unit offset fetched a group ahead; the bytes are reference-relative (engine.hpp
// RGroup), so the stream reads no reference and no LDS: its counter adds never hold it up.
//   !DEEP: per position a 16-bit counter, exceptions in the low byte, other-allele calls in the high byte; a
//          unit's 8 positions take five 32-bit LDS adds -- exact while no position of the tile is deeper than
//          255 reads (the kernel checks, and reruns the stream DEEP).  Counter of tile position i: halfword 8 + i;
//   DEEP:  one 32-bit counter per position (exceptions | other-allele << 16) at word 8 + i, one add per exception.
// Counts at positions outside the tile (margins) are never read; they are bounded by the tile's own depth (a read
// that reaches them covers the tile's first or last position), so they cannot carry into the tile's counters.
template <int T, bool DEEP, int U>
__device__ __forceinline__ void kl_stream(const uint64_t* __restrict__ units, const int2* __restrict__ rh,
                                          const RGroup* __restrict__ grp, int64_t e_lo, int64_t e_hi, int32_t tstart,
                                          int32_t* s_diff, uint32_t* s_cnt, bool do_diff, int32_t ablate, uint32_t& sink) {
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform: in SGPRs)
    const int64_t g_lo = e_lo >> 6, g_hi = (e_hi + 63) >> 6;
    const bool no_counts = ABLATE(ablate, 128), no_units = ABLATE(ablate, 256);   // diagnostics
    int64_t g = g_lo + wv;
    int2 h = g < g_hi ? rh[g * 64 + lane] : make_int2(0, 0);
    RGroup Gc = g < g_hi ? grp[g] : RGroup{0, 0, 0};
    for (; g < g_hi; g += kKlThreads / 64) {
        const int64_t e = g * 64 + lane;
        const int2 hn = g + kKlThreads / 64 < g_hi ? rh[e + kKlThreads] : make_int2(0, 0);   // the next group's headers in flight
        const RGroup G = Gc;                                // and its unit offset
        Gc = g + kKlThreads / 64 < g_hi ? grp[g + kKlThreads / 64] : RGroup{0, 0, 0};
        const int32_t gf = h.x, gl = h.y & 0x7FFFFFFF;
        const int32_t a = max(gf, tstart), b = min(gl, tstart + T - 1);
        const bool act = e >= e_lo && e < e_hi && a <= b;
        if (do_diff && act) {
            atomicAdd(&s_diff[a - tstart], 1);
            atomicAdd(&s_diff[b - tstart + 1], -1);
        }
        const int32_t k0 = act ? (a - gf) >> 3 : 0, kn = act && !no_units ? ((b - gf) >> 3) - k0 : -1;   // units k0 .. k0 + kn
        const int32_t ob0 = gf - tstart + 8 * k0 + 8;     // counter index of unit k0's byte 0 (>= 1)
        // !DEEP: the unit's first halfword at byte (ob0 & 1) << 1 of its dword; fs: the funnel shift that takes the flags'
        // >> 7 and that alignment at once; cb: unit k0's first counter dword (unit k0 + k's: 4 k dwords further)
        const uint32_t fs = 7u + 16u * (uint32_t)(ob0 & 1);
        uint32_t* const cb = s_cnt + ((ob0 + 1) >> 1) - 1;
        const uint64_t* ub = units + G.base + lane + (int64_t)k0 * 64;
        // a lane's own trip count (the wave runs while any lane has units left); loads are unconditional (a
        // batch's slots past the read's last unit repeat it) so that each unit waits for its own load only
#define KL_LOAD(q) (q)                                    // (nontemporal loads measured no change)
        // (the next batch's loads unconditional, past the read's end too -- other reads' rows or the buffer's slack,
        // never used: a load under a lane condition made the compiler wait for every outstanding load, the next
        // batch's included, before the current batch)
        // (clamped to the read's last unit: a slot past it reloads that unit's line, a cache hit -- FETCH_SIZE 2.51 ->
        // 2.25 GB per configs[2] launch, 1.02x the algorithmic bytes, at the same time, r05c2)
        // (the clamp on byte offsets, 512 per unit: one min and one add per load)
        const int32_t limb = (kn < 0 ? 0 : kn) << 9;
        const char* const ubb = reinterpret_cast<const char*>(ub);
        auto load = [&](int32_t k) { return *reinterpret_cast<const uint64_t*>(ubb + (uint32_t)min(k << 9, limb)); };
        uint64_t u[U];
#pragma unroll
        for (int i = 0; i < U; i++) u[i] = KL_LOAD(load(i));
        for (int32_t j = 0; j <= kn; j += U) {
            uint64_t v[U];
#pragma unroll
            for (int i = 0; i < U; i++) v[i] = KL_LOAD(load(j + U + i));
#pragma unroll
            for (int i = 0; i < U; i++) {
                if (j + i > kn) continue;
                const uint32_t ylo = (uint32_t)u[i], yhi = (uint32_t)(u[i] >> 32);
                // the flags from x = y & 0x7F per byte and b = x + 0x60 (bit 7: x >= 32, allele bits 5-6 set): an
                // exception is y >= 32 (y's bit 7 or b's), another allele's valid call b's bit 7 without y's -- three
                // operations per dword for the test, one more for the other allele (kl_exc / kl_nonref take seven)
                const uint32_t blo = (ylo & 0x7F7F7F7Fu) + 0x60606060u, bhi = (yhi & 0x7F7F7F7Fu) + 0x60606060u;
                const uint32_t elo = (ylo | blo) & 0x80808080u, ehi = (yhi | bhi) & 0x80808080u;
                if (no_counts) { sink += elo + ehi + kl_nonref(ylo) + kl_nonref(yhi); continue; }
                if (!(elo | ehi) && !ABLATE(ablate, 2048)) continue;   // (2048, diagnostics: every lane adds)
                const uint32_t nlo = blo & ~ylo & 0x80808080u, nhi = bhi & ~yhi & 0x80808080u;   // (kl_nonref)
                const int32_t ob = ob0 + 8 * (j + i);     // counter index of the unit's byte 0
                if (!DEEP) {
                    // (exception, other-allele) byte pairs of the 8 positions, then shifted to the halfword
                    // (measured and not kept: one halfword add per exception, the wave looping as often as its busiest
                    // lane -- KL 0.460 against 0.399 ms on configs[2], r05ex)
                    // (the flag bytes, bit 7 each, interleaved; the >> 7 rides on the funnel shifts below)
                    const uint32_t w0 = __builtin_amdgcn_perm(nlo, elo, 0x05010400u), w1 = __builtin_amdgcn_perm(nlo, elo, 0x07030602u);
                    const uint32_t w2 = __builtin_amdgcn_perm(nhi, ehi, 0x05010400u), w3 = __builtin_amdgcn_perm(nhi, ehi, 0x07030602u);
                    uint32_t* c = cb + 4 * (j + i);              // (ob even: the first add is of 0)
                    if (ABLATE(ablate, 512)) {                   // diagnostics: stores instead of adds
                        c[0] = __builtin_amdgcn_alignbit(w0, 0u, fs);
                        c[1] = __builtin_amdgcn_alignbit(w1, w0, fs);
                        c[2] = __builtin_amdgcn_alignbit(w2, w1, fs);
                        c[3] = __builtin_amdgcn_alignbit(w3, w2, fs);
                        c[4] = __builtin_amdgcn_alignbit(0u, w3, fs);
                        continue;
                    }
                    if (ABLATE(ablate, 1024)) { atomicAdd(c, w0 + w1 + w2 + w3); continue; }   // diagnostics: one add
                    if (ABLATE(ablate, 8192) && i != 0) continue;   // diagnostics: a batch's first unit only
                    if (ABLATE(ablate, 16384)) { sink += atomicAdd(c, w0 + w1 + w2 + w3); continue; }   // diagnostics: returning add
                    atomicAdd(c, __builtin_amdgcn_alignbit(w0, 0u, fs));
                    atomicAdd(c + 1, __builtin_amdgcn_alignbit(w1, w0, fs));
                    atomicAdd(c + 2, __builtin_amdgcn_alignbit(w2, w1, fs));
                    atomicAdd(c + 3, __builtin_amdgcn_alignbit(w3, w2, fs));
                    atomicAdd(c + 4, __builtin_amdgcn_alignbit(0u, w3, fs));
                } else {
                    uint64_t ex = (uint64_t)elo | (uint64_t)ehi << 32;
                    const uint64_t nr = (uint64_t)nlo | (uint64_t)nhi << 32;
                    while (ex) {
                        const int bit = __builtin_ctzll(ex);
                        ex &= ex - 1ull;
                        atomicAdd(&s_cnt[ob + (bit >> 3)], 1u + ((uint32_t)(nr >> bit) & 1u) * 0x10000u);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < U; i++) u[i] = v[i];
        }
#undef KL_LOAD
        h = hn;
    }
}

// 8 waves per SIMD: the pipelined stream's registers capped at 64
#define KL_WPE_ATTR __attribute__((amdgpu_waves_per_eu(8)))
template <int T, int U>
__global__ __launch_bounds__(kKlThreads) KL_WPE_ATTR void k_read_scan(
    const uint64_t* __restrict__ units, const int2* __restrict__ rh, const RGroup* __restrict__ grp,
    const int32_t* __restrict__ blkA, const int32_t* __restrict__ blkB, int64_t n_entries,
    const uint8_t* __restrict__ ref, const LikTables* __restrict__ tabs, GenotypeParams gp,
    SiteQ* __restrict__ queue, unsigned long long* __restrict__ counters, int64_t qseg,
    int64_t cseg4, int32_t* __restrict__ bcount, int64_t nb) {
    constexpr int PT = T / kKlThreads;                 // positions per thread in the candidate phase
    constexpr int NC = T / 2 + 16;                     // counter words (halfword per position, margins 8 and 24)
    static_assert(PT == 8 || PT == 16, "candidate phase: whole 16-byte counter words per thread");
    __shared__ alignas(16) int32_t s_diff[T + 32];     // coverage differences; then DEEP's counters (word 8 + i)
    __shared__ alignas(16) uint32_t s_ref[T / 4];
    __shared__ alignas(16) uint32_t s_cnt[NC];
    __shared__ int16_t s_cb[256];
    __shared__ int32_t s_wsum[kKlThreads / 64], s_wmax[kKlThreads / 64];
    __shared__ unsigned long long s_wscan[kKlThreads / 64], s_ncand[kKlThreads / 64], s_colbase, s_qbase;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int32_t tstart = (int32_t)((int64_t)blockIdx.x * T);
    (void)n_entries;
    for (int64_t i = (int64_t)blockIdx.x * kKlThreads + tid; i < nb; i += (int64_t)gridDim.x * kKlThreads) bcount[i] = 0;
    for (int i = tid; i <= T; i += kKlThreads) s_diff[i] = 0;
    for (int i = tid; i < NC; i += kKlThreads) s_cnt[i] = 0;
    {
        const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ref + tstart);
        for (int i = tid; i < T / 4; i += kKlThreads) s_ref[i] = r32[i];
    }
    s_cb[tid] = tabs->cb_nr[tid];
    const int64_t e_lo = blkA[tstart >> kRgBlockShift], e_hi = blkB[(tstart + T) >> kRgBlockShift];
    __syncthreads();
    uint32_t sink = 0;
    kl_stream<T, false, U>(units, rh, grp, e_lo, e_hi, tstart, s_diff, s_cnt, true, gp.ablate, sink);
    __syncthreads();
    // ---- coverage (prefix of the difference array)
    int32_t loc[PT];
    int32_t run = 0;
#pragma unroll
    for (int j = 0; j < PT; j++) { run += s_diff[PT * tid + j]; loc[j] = run; }
    int32_t incl = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t v = __shfl_up(incl, o, 64);
        if (lane >= o) incl += v;
    }
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    int32_t off = incl - run;
    for (int w = 0; w < wv; w++) off += s_wsum[w];
    int32_t cmax = 0;
#pragma unroll
    for (int j = 0; j < PT; j++) { loc[j] += off; cmax = max(cmax, loc[j]); }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cmax = max(cmax, __shfl_xor(cmax, o, 64));
    if (lane == 0) s_wmax[wv] = cmax;
    __syncthreads();
    const bool deep = max(max(s_wmax[0], s_wmax[1]), max(s_wmax[2], s_wmax[3])) > 255;
    uint32_t* s_deep = reinterpret_cast<uint32_t*>(s_diff);   // (the coverage is in registers now)
    if (deep) {                                          // byte counters could carry: stream again, 32-bit counters
        for (int i = tid; i < T + 32; i += kKlThreads) s_deep[i] = 0;
        __syncthreads();
        kl_stream<T, true, U>(units, rh, grp, e_lo, e_hi, tstart, s_diff, s_deep, false, gp.ablate, sink);
        __syncthreads();
    }
    if (sink == 0xFFFFFFFFu) s_cnt[0] = sink;            // keeps the diagnostics' work alive
    // ---- candidates and the count bound
    const bool bound = gp.use_bound != 0 && !ABLATE(gp.ablate, 1);
    uint32_t rwv[PT / 4];                                // the thread's positions' reference codes
#pragma unroll
    for (int k = 0; k < PT / 4; k += 2) {
        const uint2 v = *reinterpret_cast<const uint2*>(&s_ref[PT / 4 * tid + k]);
        rwv[k] = v.x;
        rwv[k + 1] = v.y;
    }
    uint32_t ncand = 0, need_bits = 0;
    uint64_t mine = 0;                                   // survivors << 40 | column space (units of 4 entries)
    uint32_t cwv[PT / 2];                                // !deep: the positions' counters (halfwords PT tid + 8 ..)
#pragma unroll
    for (int k = 0; k < PT / 2; k += 4) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (!deep) v = *reinterpret_cast<const uint4*>(&s_cnt[PT / 2 * tid + 4 + k]);
        cwv[k] = v.x; cwv[k + 1] = v.y; cwv[k + 2] = v.z; cwv[k + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < PT; j++) {
        const int32_t cov = loc[j];
        const uint32_t rc = (rwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        int32_t exc, na;
        if (!deep) {
            const uint32_t word = cwv[j >> 1];
            const uint32_t hw = word >> (16 * (j & 1));
            exc = (int32_t)(hw & 0xFFu);
            na = (int32_t)((hw >> 8) & 0xFFu);
        } else {
            const uint32_t cn = s_deep[PT * tid + j + 8];
            exc = (int32_t)(cn & 0xFFFFu);
            na = (int32_t)(cn >> 16);
        }
        bool need;
        if (cov > 0xFFFF) {                              // (the 16-bit halves could carry)
            need = (rc & 0x80u) != 0;
            ncand += need ? 1u : 0u;
        } else {
            const bool cand = (rc & 0x80u) && na > 0;
            ncand += cand ? 1u : 0u;
            need = cand && !(bound && na <= 255 && cov - exc >= (int32_t)s_cb[na]);
        }
        if (ABLATE(gp.ablate, 1)) need = false;
        if (need) {
            need_bits |= 1u << j;
            mine += (1ull << 40) + (uint64_t)((cov + 3) >> 2);
        }
    }
    // block scan of (survivors, column space): queue slots and column offsets in position order
    uint64_t sc = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t v = __shfl_up(sc, o, 64);
        if (lane >= o) sc += v;
    }
    unsigned long long nc = ncand;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) nc += __shfl_xor(nc, o, 64);
    if (lane == 63) s_wscan[wv] = sc;
    if (lane == 0) s_ncand[wv] = nc;
    __syncthreads();
    // the workgroup's queue slots and column space: one atomic each on its shard's counters (a counter that
    // every workgroup adds to serializes them: ~88 adds per microsecond on one word)
    const int shard = blockIdx.x % kKlShards;
    unsigned long long* sctr = counters + kCtrShard0 + kCtrShardStride * shard;
    if (tid == 0) {
        unsigned long long tnc = 0, tot = 0;
        for (int w = 0; w < kKlThreads / 64; w++) { tnc += s_ncand[w]; tot += s_wscan[w]; }
        if (tnc) atomicAdd(&sctr[2], tnc);
        const unsigned long long ns = tot >> 40, c4 = tot & ((1ull << 40) - 1ull);
        s_qbase = ns ? atomicAdd(&sctr[0], ns) : 0ull;
        s_colbase = ns ? atomicAdd(&sctr[1], c4) : 0ull;
    }
    __syncthreads();
    if (!need_bits) return;
    uint64_t ex = sc - mine;
    for (int w = 0; w < wv; w++) ex += s_wscan[w];
    int64_t qi = (int64_t)s_qbase + (int64_t)(ex >> 40);                        // in the shard's segment
    int64_t c4 = (int64_t)s_colbase + (int64_t)(ex & ((1ull << 40) - 1ull));
#pragma unroll
    for (int j = 0; j < PT; j++) {
        if (!((need_bits >> j) & 1u)) continue;
        const int32_t cov = loc[j];
        const uint32_t rc = (rwv[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        const int32_t rows = (c4 << 2) + cov <= (cseg4 << 2) ? -3 - cov : -2;   // -2: the shard's columns are full (rerun)
        if (qi < qseg) queue[shard * qseg + qi] = SiteQ{tstart + PT * tid + j, (int32_t)rc, (int32_t)(shard * cseg4 + c4), rows};
        qi++;
        c4 += (cov + 3) >> 2;
    }
}

// KG's segment table: s_pre[k] = sites in segments before k (each segment's count capped at qseg), s_pre[nshard]
// = all; block 0 stores the total in counters[2].  The first wave loads the counts in parallel (a scan).
__device__ __forceinline__ void kg_segments(const unsigned long long* __restrict__ qcnt, int stride, int nshard, int64_t qseg,
                                            int64_t* s_pre, unsigned long long* __restrict__ counters) {
    static_assert(kKlShards <= 64, "one lane per segment");
    if (threadIdx.x < 64) {
        const int k = threadIdx.x;
        const int64_t c = k < nshard ? min((int64_t)qcnt[(int64_t)k * stride], qseg) : 0;
        int64_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t v = __shfl_up(incl, o, 64);
            if (k >= o) incl += v;
        }
        if (k < nshard) s_pre[k] = incl - c;
        if (k == nshard - 1) {
            s_pre[nshard] = incl;
            if (blockIdx.x == 0) counters[2] = (unsigned long long)incl;   // (KP runs after this kernel)
        }
    }
    __syncthreads();
}

// KG: the queued sites' columns, and the compact queue KP reads.  The input queue is nshard segments of qseg
// entries (segment t holds qcnt[t * stride] sites: KL's shards; one segment otherwise); qout gets them in segment
// order and counters[2] their number.  rows <= -3: space for -3 - rows entries reserved at coff (KL's survivors);
// rows == -1: none reserved (-knownVariants, dump mode / no pruning): a counting pass and a reservation first.
// One wave per site.
__global__ __launch_bounds__(256) void k_gather_cols(const SiteQ* __restrict__ qin, const unsigned long long* __restrict__ qcnt,
                                                     int stride, int nshard, int64_t qseg, SiteQ* __restrict__ qout,
                                                     const int2* __restrict__ rh, const RGroup* __restrict__ grp,
                                                     const uint64_t* __restrict__ units, const int32_t* __restrict__ blkA,
                                                     const uint8_t* __restrict__ ref,
                                                     int64_t n_entries, uint16_t* __restrict__ cols, int64_t col_cap,
                                                     unsigned long long* __restrict__ counters) {
    __shared__ int64_t s_pre[kKlShards + 1];
    const int lane = threadIdx.x & 63;
    kg_segments(qcnt, stride, nshard, qseg, s_pre, counters);
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t total = s_pre[nshard];
    for (int64_t i = w0; i < total; i += nw) {
        int k = 0;                                       // the segment of compact index i (binary search)
        for (int step = kKlShards; step > 0; step >>= 1)
            if (k + step < nshard && s_pre[k + step] <= i) k += step;
        const int64_t j = i - s_pre[k];
        {
            SiteQ q = qin[(int64_t)k * qseg + j];
            if (q.rows < 0 && q.rows != -2) {
                const int32_t p = q.gpos;
                const int64_t e0 = blkA[p >> kRgBlockShift];
                int64_t c4;
                int32_t cov;
                if (q.rows == -1) {
                    wave_gather<false>(p, e0, n_entries, rh, grp, units, 0u, nullptr, &cov);
                    unsigned long long r = 0;
                    if (lane == 0) r = atomicAdd(&counters[5], (unsigned long long)((cov + 3) >> 2));
                    c4 = (int64_t)__shfl(r, 0, 64);
                } else {
                    cov = -3 - q.rows;
                    c4 = q.coff;
                }
                int32_t r = -2;
                if ((c4 << 2) + cov <= col_cap) r = wave_gather<true>(p, e0, n_entries, rh, grp, units, (uint32_t)ref[p], cols + (c4 << 2), nullptr);
                q.coff = (int32_t)c4;
                q.rows = r;
            }
            if (lane == 0) qout[i] = q;
        }
    }
}

// KG for KL's queue (every site's column space reserved: rows <= -3, or -2 when the shard's columns were full):
// a wave gathers kKgSites sites at once, their chunk loads interleaved (one site's gather is a chain of dependent
// loads -- block table, headers, units -- so a wave per site leaves the chip waiting).  Compacts like k_gather_cols.
template <int kKgSites>
__global__ __launch_bounds__(256) void k_gather_kl(const SiteQ* __restrict__ qin, const unsigned long long* __restrict__ qcnt,
                                                   int stride, int nshard, int64_t qseg, SiteQ* __restrict__ qout,
                                                   const int2* __restrict__ rh, const RGroup* __restrict__ grp,
                                                   const uint64_t* __restrict__ units, const int32_t* __restrict__ blkA,
                                                   const uint8_t* __restrict__ ref, int64_t n_entries,
                                                   uint16_t* __restrict__ cols, unsigned long long* __restrict__ counters) {
    __shared__ int64_t s_pre[kKlShards + 1];
    const int lane = threadIdx.x & 63;
    kg_segments(qcnt, stride, nshard, qseg, s_pre, counters);
    const int64_t total = s_pre[nshard];
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
    const int64_t w0 = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (int64_t i0 = w0 * kKgSites; i0 < total; i0 += nw * kKgSites) {
        SiteQ q[kKgSites];
        int64_t e[kKgSites];
        int32_t n[kKgSites];
        uint32_t rcode[kKgSites];
        bool live[kKgSites];
#pragma unroll
        for (int t = 0; t < kKgSites; t++) {
            const int64_t i = i0 + t;
            live[t] = false;
            n[t] = 0;
            e[t] = 0;
            rcode[t] = 0;
            q[t] = SiteQ{0, 0, 0, -2};
            if (i >= total) continue;
            int k = 0;
            for (int step = kKlShards; step > 0; step >>= 1)
                if (k + step < nshard && s_pre[k + step] <= i) k += step;
            q[t] = qin[(int64_t)k * qseg + (i - s_pre[k])];
            live[t] = q[t].rows <= -3;
        }
#pragma unroll
        for (int t = 0; t < kKgSites; t++)
            if (live[t]) {
                e[t] = (int64_t)blkA[q[t].gpos >> kRgBlockShift] & ~(int64_t)63;
                rcode[t] = ref[q[t].gpos];
            }
        // chunk steps: every live site reads its next 64 entries' headers, then the covering ones' units (loading the
        // next chunk's headers while this chunk's units are in flight measured no change, DESIGN.md 3 KG)
        for (;;) {
            bool any = false;
#pragma unroll
            for (int t = 0; t < kKgSites; t++) any |= live[t];
            if (!any) break;
            int2 h[kKgSites];
            int64_t gb[kKgSites];
#pragma unroll
            for (int t = 0; t < kKgSites; t++) {
                const bool l = live[t] && e[t] < n_entries;
                h[t] = l ? rh[e[t] + lane] : make_int2(0x7FFFFFFF, 0);
                gb[t] = l ? grp[e[t] >> 6].base : 0;
            }
            uint64_t u[kKgSites];
            int32_t o[kKgSites];
#pragma unroll
            for (int t = 0; t < kKgSites; t++) {
                const int32_t p = q[t].gpos, gf = h[t].x, gl = h[t].y & 0x7FFFFFFF;
                const bool covers = live[t] && gf <= p && p <= gl;
                o[t] = covers ? p - gf : -1;
                u[t] = covers ? units[gb[t] + (int64_t)(o[t] >> 3) * 64 + lane] : 0ull;
            }
#pragma unroll
            for (int t = 0; t < kKgSites; t++) {
                if (!live[t]) continue;
                const int32_t p = q[t].gpos;
                const uint32_t code = o[t] >= 0 ? (((uint32_t)(u[t] >> (8 * (o[t] & 7))) & 0xFFu) ^ rcode[t]) : 0u;
                const unsigned long long m = __ballot(code != 0);
                if (code) {
                    const int rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    cols[((int64_t)q[t].coff << 2) + n[t] + rk] = (uint16_t)(code | (((uint32_t)h[t].y >> 31) << 8));
                }
                n[t] += (int32_t)__popcll(m);
                e[t] += 64;
                if (__ballot(h[t].x > p) || e[t] >= n_entries) {   // entries are sorted by gfirst: none later covers p
                    live[t] = false;
                    q[t].rows = n[t];
                }
            }
        }
#pragma unroll
        for (int t = 0; t < kKgSites; t++)
            if (lane == t && i0 + t < total) qout[i0 + t] = q[t];
    }
}

__global__ __launch_bounds__(256) void k_zero_i32(int32_t* __restrict__ p, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0;
}

// ------------------------------------------------------------------------------------------
// KQ: every in-window position queued (dump mode, and runs without the exact pruning: -h > 0.1 or
//     prune_candidates = 0); KP skips positions without a pileup (VariantDiscoverySNVQAlgorithm.java:101-103)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_queue_all(const uint8_t* __restrict__ ref, int64_t g_len, SiteQ* __restrict__ queue,
                                                   unsigned long long* __restrict__ counters, int64_t qcap,
                                                   int32_t* __restrict__ bcount, int64_t nb) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nb; i += stride) bcount[i] = 0;
    const int64_t nwave = (g_len + 63) / 64;
    for (int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; w < nwave; w += stride >> 6) {
        const int64_t g = w * 64 + lane;
        const uint32_t rc = g < g_len ? (uint32_t)ref[g] : 0u;
        const unsigned long long m = __ballot(rc != 0);
        if (!m) continue;
        unsigned long long base = 0;
        if (lane == 0) base = atomicAdd(&counters[2], (unsigned long long)__popcll(m));
        base = __shfl(base, 0, 64);
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (rc != 0 && (int64_t)(base + rank) < qcap) queue[base + rank] = SiteQ{(int32_t)g, (int32_t)rc, 0, -1};
        if (lane == 0) atomicAdd(&counters[1], (unsigned long long)__popcll(m));
    }
}

// KQN: the open positions (a bit per global position) into the KPM queue, {position, reference code}
__global__ __launch_bounds__(256) void k_queue_need(const uint32_t* __restrict__ need, const uint8_t* __restrict__ ref, int64_t nwords,
                                                    QueueSite* __restrict__ queue, unsigned long long* __restrict__ counters, int64_t qcap,
                                                    int32_t* __restrict__ qword) {
    const int lane = threadIdx.x & 63;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < nwords; base += stride) {
        const int64_t i = base + threadIdx.x;
        uint32_t m = i < nwords ? need[i] : 0u;
        const uint32_t c = (uint32_t)__popc(m);
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(incl, o, 64);
            if (lane >= o) incl += v;
        }
        const uint32_t tot = __shfl(incl, 63, 64);
        if (!tot) continue;
        unsigned long long q0 = 0;
        if (lane == 63) q0 = atomicAdd(&counters[2], (unsigned long long)tot);
        q0 = __shfl(q0, 63, 64);
        int64_t at = (int64_t)q0 + (incl - c);
        if (qword && m) qword[i] = (int32_t)at;           // (KPM's first stage: the queue index of the word's first bit)
        while (m) {
            const int b = __builtin_ctz(m);
            m &= m - 1u;
            const int64_t g = i * 32 + b;
            if (at < qcap) queue[at] = QueueSite{(int32_t)g, (int32_t)ref[g]};
            at++;
        }
    }
}

// ------------------------------------------------------------------------------------------
// KLM: the multisample scan over the population read-group layout -- one wavefront per (sample, tile of kKlmTile
//      positions), four samples per workgroup
// ------------------------------------------------------------------------------------------
// A sample without a valid call of another allele than the reference at a position cannot make a decided
// non-reference call there, and one whose valid calls the exact integer bound (§5) proves hom-ref cannot either
// (SingleSampleVariantPileupListener.genotypeVariantSample, :361-391); a position where every sample is so proven
// gets variant QS 0, which MultisampleVariantsDetector.onPileup never writes (:534).  Per sample tile:
//   pass 1: the wave streams the sample's units over the tile (its read-group streams in turn; lane = read, as KL).
//           COUNT: per position two byte counters, the valid reference calls of quality >= kKlmQs (a batch of units in
//           2 U + 1 LDS adds, every lane) and the valid calls of another allele (three adds per unit on the lanes whose
//           unit has one; SWAR flags, klm_flags).  !COUNT: the positions holding a valid call of another allele marked
//           in an LDS bitmap;
//   count:  COUNT, a callable position with one call of another allele is a candidate the count bound may drop: its
//           counted reference calls reaching cb_hi1 make it hom-ref for this sample (about 97 % of the candidate
//           columns at 10x); positions with two or three stay for the exact bound, with four or more open as they are;
//           COUNT's exact bound is an in-wave walk (below); !COUNT:
//   slots:  the positions still marked get LDS slots in position order;
//   pass 2: every lane adds the weights of its read's valid calls at the slotted positions it covers (one 8-byte
//           reload each) into its slot's {ref, alt 1, alt 2, alt 3} sums -- the exact integer bound;
//   pass 3: a slot the bound cannot prove hom-ref -- or holding more than kMcMaxCalls valid calls, or past
//           kKlmSlots -- keeps its position open: one bit per global position (atomicOr); KQN queues them for KPM.
// COUNT needs every sample's coverage over the tile below 128 (the host's per-tile bound, engine.cpp build_pop_rg_layout):
// the byte counters cannot carry.  The tiles where some sample is deeper (collapsed repeats,
// rDNA, deep populations) run !COUNT, launched over those tiles only: every marked position takes the exact bound.
// The reads of no sample only enter the pooled counts: not scanned.  No block barrier after the tables: every wave's
// state is its own.
constexpr int kKlmThreads = 256;
// the population layout's padding past a read's last position (k_build_units): zero bytes = a reference call of quality
// 0 relative to any reference code, which KLM's counters (quality >= kKlmQs) and marks ignore (no per-unit mask of the
// read's end)
constexpr uint64_t kPopPadUnit = 0ull;
constexpr int kKlmWords = kKlmTile / 32 + 2;   // tile bitmap words, a 32-position margin on either side
constexpr uint32_t kKlmDirectN = 4;            // COUNT: columns with this many calls of another allele open unwalked
constexpr int kKlmUnroll = 4;                  // pass 1: unit loads per batch, the next batch issued before the current
                                               // batch's marks (pipelined 4: 1.368-1.372 ms vs 8 unpipelined 1.393-1.395)
constexpr int kKlmCntBytes = kKlmTile + 48;    // COUNT, per wave: counted reference calls, byte counters (byte i + 8:
                                               // tile position i; a batch's adds reach 31 positions past the tile)
constexpr int kKlmDifBytes = kKlmCntBytes;    // COUNT, per wave: valid calls of another allele, byte counters (the same)
constexpr int kKlmWaveLds = kKlmCntBytes + kKlmDifBytes;   // the exact bound's slots reuse it after the count
static_assert(kKlmTile == 2048 && kRunAlign % kKlmTile == 0, "KLM tile: one bitmap word per lane");
static_assert(kKlmSlots * (32 + 4 + 2) <= kKlmWaveLds, "KLM slots within the wave's counter space");

__device__ __forceinline__ uint32_t nib4_byte7(uint32_t w) {   // bit 7 of the four bytes -> 4 bits
    return ((w >> 7) & 1u) | ((w >> 14) & 2u) | ((w >> 21) & 4u) | ((w >> 28) & 8u);
}
// the same for a word holding nothing but those four bits (w & 0x80808080 == w), in five full-rate operations: bytes 0-2
// gathered by one 24-bit multiply (bit 8k of w >> 7 times 2^(14 - 7k) lands on bit 14 + k, the cross terms on distinct
// bits below 14 or above 16, so nothing carries into 14-16), byte 3 shifted down (KLM A/B: 1.005 -> 0.994 ms)
__device__ __forceinline__ uint32_t nib4_of_b7(uint32_t w) {
    return ((__umul24((w >> 7) & 0x010101u, 0x4081u) >> 14) & 7u) | ((w >> 28) & 8u);
}
// KLM's two flags of a reference-relative dword y, bit 7 of byte k: r, a valid call of the reference's allele of quality
// >= kKlmQs (y in [kKlmQs, 31]); n, a valid call of another allele (y in [32, 127], kl_nonref).  Six operations: with
// x = y & 0x7F per byte, x + (128 - Qs) and x + 96 reach bit 7 iff x >= Qs / x >= 32 and never carry out of the byte.
__device__ __forceinline__ void klm_flags(uint32_t y, uint32_t& r, uint32_t& n) {
    const uint32_t x = y & 0x7F7F7F7Fu;
    const uint32_t b = x + 0x60606060u;
    r = (x + 0x01010101u * (uint32_t)(128 - kKlmQs)) & ~(b | y) & 0x80808080u;
    n = b & ~y & 0x80808080u;
}
// adds a unit's eight flag bytes (bit 7 each, lo = bytes 0-3) as 0 / 1 to the byte counters from byte o1 + 1 on, p =
// the counters' dword o1 >> 2, fs = 31 - 8 (o1 & 3): three funnel shifts take the >> 7 and the byte alignment at once
// (the first add is of zero when o1 + 1 is aligned)
__device__ __forceinline__ void klm_add8(uint32_t* p, uint32_t fs, uint32_t lo, uint32_t hi) {
    atomicAdd(p, __builtin_amdgcn_alignbit(lo, 0u, fs));
    atomicAdd(p + 1, __builtin_amdgcn_alignbit(hi, lo, fs));
    atomicAdd(p + 2, __builtin_amdgcn_alignbit(0u, hi, fs));
}

template <bool COUNT>
__global__ __launch_bounds__(kKlmThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_scan_pop(
    const uint64_t* __restrict__ units, const int2* __restrict__ rh, const RGroup* __restrict__ grp,
    const int32_t* __restrict__ samp_st, const int32_t* __restrict__ blkA, const int32_t* __restrict__ blkB,
    int64_t nblk, int32_t shift, int32_t n_samples, const uint8_t* __restrict__ ref, const LikTables* __restrict__ tabs,
    GenotypeParams gp, uint32_t* __restrict__ need, unsigned long long* __restrict__ counters, uint2* __restrict__ pairs,
    int64_t pseg, const int64_t* __restrict__ st_end, const uint8_t* __restrict__ deep_flag,
    const int32_t* __restrict__ deep_tiles) {
    // deep_flag (COUNT): tiles some sample covers deeper than kKlmCountMaxCov are skipped here -- the !COUNT launch over
    // deep_tiles (its grid: those tiles only) scans them
    const int nsg = (n_samples + 3) >> 2;
    // COUNT: one sample group's consecutive tiles on one XCD at about the same time (the blocks b, b + 8, ... share an
    // XCD: the bijective remap of cdna_hip_programming.md T1, then sample-group-major order), even tiles streaming their
    // rounds forward and odd tiles backward -- so the 128-B lines that hold units of both tiles at a tile edge are read
    // by the two workgroups close together, the second read an L2 hit
    int64_t tile, sgi;
    if (COUNT) {
        const uint32_t N = gridDim.x, bid = blockIdx.x, q = N >> 3, r = N & 7, x = bid & 7;
        const uint32_t lid = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
        const uint32_t ntile = N / (uint32_t)nsg;
        sgi = lid / ntile;
        tile = lid - (uint32_t)sgi * ntile;
    } else {
        sgi = (int64_t)blockIdx.x % nsg;
        tile = deep_tiles ? (int64_t)deep_tiles[blockIdx.x / nsg] : (int64_t)blockIdx.x / nsg;
    }
    if (COUNT && deep_flag && deep_flag[tile]) return;      // (the whole workgroup: no barrier has been reached)
    __shared__ unsigned long long w[2][32];
    __shared__ uint32_t s_call[kKlmTile / 32];         // callable positions of the tile
    constexpr int kBmWords = COUNT ? 1 : kKlmWords;   // (COUNT keeps its columns in registers)
    __shared__ uint32_t s_bm[4][kBmWords];             // !COUNT: marked positions, then those the exact bound takes
    __shared__ uint16_t s_wb[4][kBmWords];             // !COUNT: slot of each bitmap word's first slotted position
    __shared__ alignas(16) uint32_t s_wave[4][kKlmWaveLds / 4];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // (wave-uniform: in SGPRs)
    if (threadIdx.x < 64) w[threadIdx.x >> 5][threadIdx.x & 31] = (threadIdx.x < 32 ? tabs->wR : tabs->wX)[threadIdx.x & 31];
    {
        // 8 positions' callable bits per thread (bit 7 of the reference code), four threads per word
        const uint2 r = reinterpret_cast<const uint2*>(ref + tile * kKlmTile)[threadIdx.x];
        uint32_t v = (nib4_byte7(r.x) | nib4_byte7(r.y) << 4) << (8 * (threadIdx.x & 3));
        v |= __shfl_xor(v, 1, 64);
        v |= __shfl_xor(v, 2, 64);
        if ((threadIdx.x & 3) == 0) s_call[threadIdx.x >> 2] = v;
    }
    const int s = (int)sgi * 4 + wv;
    uint32_t* bm = s_bm[wv];
    uint32_t* rc32 = s_wave[wv];                        // COUNT: reference calls of quality >= kKlmQs
    uint32_t* nc32 = s_wave[wv] + kKlmCntBytes / 4;     // COUNT: valid calls of another allele
    if (s < n_samples) {
        if (COUNT)
            for (int i = lane; i < kKlmWaveLds / 4; i += 64) s_wave[wv][i] = 0u;
        else
            for (int i = lane; i < kKlmWords; i += 64) bm[i] = 0u;
    }
    __syncthreads();
    if (s >= n_samples) return;
    const int32_t tstart = (int32_t)(tile * kKlmTile), tlast = tstart + kKlmTile - 1;
    const int st0 = samp_st[s], st1 = samp_st[s + 1];
    uint32_t sink = 0;                                  // (diagnostics)
    // ---- pass 1: COUNT the two counters, !COUNT the marks
    for (int st = st0; st < st1; st++) {
        const int64_t e_lo = blkA[(int64_t)st * nblk + (tstart >> shift)];
        const int64_t e_hi = blkB[(int64_t)st * nblk + (tlast >> shift) + 1];
        // rounds of 64 consecutive entries (lane = entry e0 + lane, whatever its group): every lane busy but in the
        // last round, where a read's units are split over f = 64 / m lanes (m entries left, m <= 32); the next round's
        // header and group base in flight
        // (COUNT, odd tiles: the rounds in reverse, the last one first -- round v0 streams entries phys(v0) ..)
        const int64_t last0 = e_lo + (((e_hi - e_lo - 1) >> 6) << 6);
        const bool rev = COUNT && (tile & 1);
        auto phys = [&](int64_t v) { return rev ? e_lo + last0 - v : v; };
        int2 h = phys(e_lo) + lane < e_hi && e_lo < e_hi ? rh[phys(e_lo) + lane] : make_int2(0, -1);
        int64_t gbase = phys(e_lo) + lane < e_hi && e_lo < e_hi ? grp[(phys(e_lo) + lane) >> 6].base : 0;
        for (int64_t v0 = e_lo; v0 < e_hi; v0 += 64) {
            const int64_t e0 = phys(v0);
            int64_t e = e0 + lane;
            const int64_t en = phys(v0 + 64) + lane;           // the next round's entry
            const bool nx = v0 + 64 < e_hi && en < e_hi;
            const int2 hn = nx ? rh[en] : make_int2(0, -1);
            const int64_t gbn = nx ? grp[en >> 6].base : 0;
            const int32_t m = (int32_t)min(e_hi - e0, (int64_t)64);   // (wave-uniform)
            int32_t f = 1, part = 0;
            if (m <= 32) {
                const int32_t src = lane % m;
                f = 64 / m;
                part = lane / m;                                // (>= f: no part, the lane idles)
                h.x = __shfl(h.x, src, 64);
                h.y = __shfl(h.y, src, 64);
                gbase = (int64_t)(((uint64_t)(uint32_t)__shfl((int)(uint32_t)((uint64_t)gbase >> 32), src, 64) << 32) |
                                  (uint32_t)__shfl((int)(uint32_t)gbase, src, 64));
                e = e0 + src;
            }
            const int32_t gf = h.x, gl = h.y & 0x7FFFFFFF;
            const int32_t a = max(gf, tstart), b = min(gl, tlast);
            const bool act = e < e_hi && a <= b && part < f;
            int32_t k0 = act ? (a - gf) >> 3 : 0, kn = act ? ((b - gf) >> 3) - k0 : -1;
            if (f > 1 && act) {                                 // part `part` of the read's kn + 1 units
                const int32_t chunk = (kn + f) / f, ks = part * chunk;
                if (ks > kn) kn = -1;                           // nothing left for this part (its loads: unit k0)
                else { k0 += ks; kn = min(kn - ks, chunk - 1); }
            }
            const uint64_t* ub = units + gbase + (e & 63) + (int64_t)k0 * 64;
            const int32_t ti0 = gf + 8 * k0 - tstart + 32;   // bitmap index of unit k0's byte 0 (>= 25); COUNT: its
                                                              // counter byte is ti0 - 24 (>= 1)
            // (the read's last unit holds padding past its last position: zero bytes in the population layout -- reference
            // calls of quality 0, neither counted nor marked -- so nothing is masked here; k_build_units)
            const int32_t o1 = ti0 - 25;                        // COUNT: counter byte of unit k0's byte 0, minus 1 (>= 0);
            uint32_t* const rcp = rc32 + (o1 >> 2);             // unit k0 + k's adds start 2 k dwords further
            uint32_t* const ncp = nc32 + (o1 >> 2);
            const uint32_t fs = 31u - 8u * (uint32_t)(o1 & 3);
            // (every batch's loads are issued unconditionally: a load under a lane condition made the compiler wait for
            // every outstanding load, the next batch's included, before the current batch)
            // (clamped to the read's last unit, as KL's are: a slot past it reloads that unit's line, a cache hit.  Round
            // 5's VALU-bound kernel lost 1.5 % to the clamp's address arithmetic; once the counters above cut its VALU
            // by half, the unclamped loads' lines -- 1.53x the algorithmic bytes -- were what it waited on)
            // (the clamp on byte offsets, 512 per unit: one min and one add per load)
            const int32_t limb = (kn < 0 ? 0 : kn) << 9;
            const char* const ubb = reinterpret_cast<const char*>(ub);
            auto load = [&](int32_t k) { return *reinterpret_cast<const uint64_t*>(ubb + (uint32_t)min(k << 9, limb)); };
            uint64_t u[kKlmUnroll];
#pragma unroll
            for (int i = 0; i < kKlmUnroll; i++) u[i] = load(i);
            for (int32_t j = 0; j <= kn; j += kKlmUnroll) {
                uint64_t v[kKlmUnroll];
#pragma unroll
                for (int i = 0; i < kKlmUnroll; i++) v[i] = load(j + kKlmUnroll + i);
                if constexpr (COUNT) {
                    // the batch's reference calls in 2 U + 1 adds (one funnel shift each) instead of 3 per unit: a
                    // wave's LDS add costs its transfer and its bank conflicts whatever its lanes hold (KLM 0.746 ->
                    // 0.738 ms); the units past the read's last one (their loads repeat it) add zeros; the other
                    // allele's calls per unit.  (Round 5 marked those calls with returning ORs into a marked /
                    // marked-twice bitmap pair and counted exceptions and coverage differences: KLM 0.826-0.847 ms;
                    // exceptions, other-allele calls and coverage differences in three planes, every add on the lanes
                    // whose unit has one: bank conflicts 122 -> 51 M cycles, but 6 waves per SIMD and VALU +25 %,
                    // 0.830 ms, r06o)
                    uint32_t rf[2 * kKlmUnroll];
#pragma unroll
                    for (int i = 0; i < kKlmUnroll; i++) {
                        const bool in = j + i <= kn;
                        const uint32_t ylo = (uint32_t)u[i], yhi = (uint32_t)(u[i] >> 32);
                        uint32_t r0, n0, r1, n1;
                        klm_flags(ylo, r0, n0);
                        klm_flags(yhi, r1, n1);
                        rf[2 * i] = in ? r0 : 0u;
                        rf[2 * i + 1] = in ? r1 : 0u;
                        if (in && (n0 | n1)) klm_add8(ncp + 2 * (j + i), fs, n0, n1);
                    }
                    uint32_t* const p = rcp + 2 * j;
                    atomicAdd(p, __builtin_amdgcn_alignbit(rf[0], 0u, fs));
#pragma unroll
                    for (int t = 1; t < 2 * kKlmUnroll; t++) atomicAdd(p + t, __builtin_amdgcn_alignbit(rf[t], rf[t - 1], fs));
                    atomicAdd(p + 2 * kKlmUnroll, __builtin_amdgcn_alignbit(0u, rf[2 * kKlmUnroll - 1], fs));
                }
#pragma unroll
                for (int i = 0; i < kKlmUnroll; i++) {
                    if (COUNT || j + i > kn) continue;
                    const uint32_t ylo = (uint32_t)u[i], yhi = (uint32_t)(u[i] >> 32);
                    if (ABLATE(gp.ablate, 524288)) { sink += ylo ^ yhi; continue; }   // (diagnostics: loads only)
                    {
                        const uint32_t nlo = kl_nonref(ylo), nhi = kl_nonref(yhi);
                        if (!(nlo | nhi)) continue;
                        const uint32_t m = nib4_of_b7(nlo) | nib4_of_b7(nhi) << 4;
                        const int32_t ti = ti0 + 8 * (j + i);
                        const uint64_t mv = (uint64_t)m << (ti & 31);
                        const uint32_t m0 = (uint32_t)mv, m1 = (uint32_t)(mv >> 32);
                        if (m0) atomicOr(&bm[ti >> 5], m0);
                        if (m1) atomicOr(&bm[(ti >> 5) + 1], m1);
                    }
                }
#pragma unroll
                for (int i = 0; i < kKlmUnroll; i++) u[i] = v[i];
            }
            h = hn;
            gbase = gbn;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- candidates: the callable positions holding a valid call of another allele (lane: positions 32 lane ..
    //      32 lane + 31); COUNT drops those the count bound proves hom-ref
    const bool bound_on = gp.use_bound != 0;
    uint32_t word, ncand, many = 0u;                    // many (COUNT): kKlmDirectN or more calls of another allele
    if constexpr (COUNT) {
        // per dword of four positions, bit 7 of byte k: n >= 1, n >= 2, r >= cb_hi1 (every counter is below 128 and
        // adding at most 128 to one never carries out of its byte)
        const int32_t cb = max(tabs->cb_hi1, 0);
        const uint32_t kc = 0x01010101u * (uint32_t)(cb < 128 ? 128 - cb : 0);   // (cb >= 128: nothing reaches it)
        uint32_t cand = 0u, drop = 0u;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t rw = rc32[8 * lane + 2 + q], nw = nc32[8 * lane + 2 + q];   // positions 32 lane + 4q ..
            const uint32_t ge1 = (nw + 0x7F7F7F7Fu) & 0x80808080u;
            const uint32_t dr = (rw + kc) & ~(nw + 0x7E7E7E7Eu) & ge1;               // one such call, r >= cb
            cand |= nib4_of_b7(ge1) << (4 * q);
            drop |= nib4_of_b7(dr) << (4 * q);
            many |= nib4_of_b7((nw + (0x80u - kKlmDirectN) * 0x01010101u) & 0x80808080u) << (4 * q);
        }
        word = cand & s_call[lane];
        ncand = (uint32_t)__popc(word);
        if (bound_on) word &= ~drop;
    } else {
        word = bm[1 + lane] & s_call[lane];
        ncand = (uint32_t)__popc(word);
    }
    if (sink == 0xFFFFFFFFu) word |= 1u;                // keeps the diagnostics' work alive
    if (ABLATE(gp.ablate, 262144)) word = 0u;           // (diagnostics: no exact pass)
    if (COUNT) {
        // ---- the exact bound for the count bound's survivors, eight lanes per column: each lane takes every eighth
        //      entry of the sample's streams from the column's block-table entry on, the covering reads' units loaded as
        //      their headers arrive, the valid calls summed into {reference, alt 1-3} weights and reduced across the
        //      eight; a column the bound cannot prove hom-ref (or with more than kMcMaxCalls valid calls) opens its
        //      position and, with pairs, is listed for KPM's first stage.  The gathers' latency hides behind the other
        //      waves' streams (a separate kernel over the same columns: 0.109-0.166 ms after KLM, r05w2 / r05x).
        const int sh = (int)(blockIdx.x % kKlShards);
        unsigned long long* sc = counters + kCtrShard0 + kCtrShardStride * sh;
        // a column with kKlmDirectN or more calls of another allele opens without the walk (at 10x nearly every one is
        // a carrier the exact bound cannot prove hom-ref: 61 % of the walked columns opened, r06cnt); opening a column
        // only hands one more (position, sample) pair to KPM's first stage, which genotypes it exactly.  configs[4]:
        // walked columns 329 K -> 158 K at 4 (queued positions 4860 -> 4864), KLM -0.5 %; at 3: 141 K, but 5918 queued
        // positions cost KPM's first stage +10 us (r06ae / r06af)
        const uint32_t direct = bound_on ? word & many : 0u;
        if (__ballot(direct != 0u)) {
            word &= ~direct;
            const uint32_t dc = (uint32_t)__popc(direct);
            for (uint32_t wd = direct; wd; wd &= wd - 1u) {
                const int32_t p = tstart + 32 * lane + __builtin_ctz(wd);
                atomicOr(&need[p >> 5], 1u << (p & 31));
            }
            if (pairs) {
                uint32_t dincl = dc;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t x = __shfl_up(dincl, o, 64);
                    if (lane >= o) dincl += x;
                }
                const uint32_t dtot = (uint32_t)__shfl((int)dincl, 63, 64);
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(&sc[2], (unsigned long long)dtot);
                base = __shfl(base, 0, 64);
                int64_t kp = (int64_t)base + (dincl - dc);
                for (uint32_t wd = direct; wd; wd &= wd - 1u, kp++)
                    if (kp < pseg) pairs[(int64_t)sh * pseg + kp] = make_uint2((uint32_t)(tstart + 32 * lane + __builtin_ctz(wd)), (uint32_t)s);
            }
        }
        const uint32_t c = (uint32_t)__popc(word);
        uint32_t incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t x = __shfl_up(incl, o, 64);
            if (lane >= o) incl += x;
        }
        const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
        unsigned long long tcand = ncand;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tcand += __shfl_xor(tcand, o, 64);
        if (lane == 0) {
            if (tcand) atomicAdd(&sc[0], tcand);
            if (tot) atomicAdd(&sc[1], (unsigned long long)tot);
        }
        if (tot == 0) return;
        // the wave's columns in position order (tile offsets; its counters' LDS is free by now)
        uint16_t* cpos = reinterpret_cast<uint16_t*>(s_wave[wv]);
        {
            uint32_t k = incl - c;
            for (uint32_t wd = word; wd; wd &= wd - 1u) cpos[k++] = (uint16_t)(32 * lane + __builtin_ctz(wd));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int j = lane & 7;
        const int32_t maxq = gp.max_q;
        const long long th = tabs->t_het, to = tabs->t_homo;
        for (uint32_t c0 = 0; c0 < tot; c0 += 8) {
            const uint32_t ci = c0 + (uint32_t)(lane >> 3);
            const bool have = ci < tot;
            const int32_t p = have ? tstart + cpos[ci] : 0;
            unsigned long long a0 = 0ull, a1 = 0ull, a2 = 0ull, a3 = 0ull;
            uint32_t sn = 0;
            if (have) {
                for (int st = st0; st < st1; st++) {
                    const int64_t end = st_end[st];
                    for (int64_t e = blkA[(int64_t)st * nblk + (p >> shift)] + j;; e += 8) {
                        const int2 h = e < end ? rh[e] : make_int2(0x7FFFFFFF, 0);
                        const int32_t gf = h.x, gl = h.y & 0x7FFFFFFF;
                        if (gf <= p && p <= gl) {
                            const int64_t o = p - gf;
                            const uint64_t u = units[grp[e >> 6].base + (o >> 3) * 64 + (e & 63)];
                            const uint32_t y = (uint32_t)(u >> (8 * (o & 7))) & 0xFFu;   // (reference-relative)
                            if (!(y & 0x80u)) {                                          // a valid call
                                const uint32_t al = (y >> 5) & 3u;
                                int q = (int)(y & 31u);
                                q = q > maxq ? maxq : q;
                                const unsigned long long wq = w[al == 0 ? 0 : 1][q];
                                a0 += al == 0 ? wq : 0ull;
                                a1 += al == 1 ? wq : 0ull;
                                a2 += al == 2 ? wq : 0ull;
                                a3 += al == 3 ? wq : 0ull;
                                sn++;
                            }
                        }
                        // entries are sorted by gfirst: the eight stop once every one's entry starts past p
                        const unsigned long long mb = __ballot(gf <= p);
                        if (!((mb >> (lane & ~7)) & 0xFFull)) break;
                    }
                }
            }
#pragma unroll
            for (int o = 4; o > 0; o >>= 1) {
                a0 += __shfl_xor(a0, o, 64); a1 += __shfl_xor(a1, o, 64);
                a2 += __shfl_xor(a2, o, 64); a3 += __shfl_xor(a3, o, 64);
                sn += __shfl_xor(sn, o, 64);
            }
            bool open = false;
            if (have && j == 0) {
                const long long R1 = (long long)(a0 & 0xFFFFFFFFull), R2 = (long long)(a0 >> 32);
                const long long x1 = (long long)(a1 & 0xFFFFFFFFull), y1 = (long long)(a2 & 0xFFFFFFFFull);
                const long long z1 = (long long)(a3 & 0xFFFFFFFFull);
                const long long x2 = (long long)(a1 >> 32), y2 = (long long)(a2 >> 32), z2 = (long long)(a3 >> 32);
                const bool drop = (R1 - x1 > th) && (R1 - y1 > th) && (R1 - z1 > th) &&
                                  (R2 - x2 > to) && (R2 - y2 > to) && (R2 - z2 > to) &&
                                  (R2 - x1 - y1 > th) && (R2 - x1 - z1 > th) && (R2 - y1 - z1 > th);
                open = !bound_on || sn > (uint32_t)kMcMaxCalls || !drop;
                if (open) atomicOr(&need[p >> 5], 1u << (p & 31));
            }
            if (pairs) {
                const unsigned long long m = __ballot(open);
                if (m) {
                    unsigned long long base = 0;
                    if (lane == 0) base = atomicAdd(&sc[2], (unsigned long long)__popcll(m));
                    base = __shfl(base, 0, 64);
                    if (open) {
                        const int64_t kp = (int64_t)base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                        if (kp < pseg) pairs[(int64_t)sh * pseg + kp] = make_uint2((uint32_t)p, (uint32_t)s);
                    }
                }
            }
        }
        return;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bm[1 + lane] = word;
    if (lane == 0) { bm[0] = 0u; bm[kKlmWords - 1] = 0u; }
    // ---- slots: the tile's remaining positions in order
    uint16_t* wb = s_wb[wv];
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(s_wave[wv]);
    uint32_t* sn = s_wave[wv] + 2 * 4 * kKlmSlots;
    uint16_t* spos = reinterpret_cast<uint16_t*>(sn + kKlmSlots);
    const uint32_t c = (uint32_t)__popc(word);
    uint32_t incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t x = __shfl_up(incl, o, 64);
        if (lane >= o) incl += x;
    }
    const uint32_t nslot = __shfl(incl, 63, 64);
    unsigned long long tcand = ncand;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tcand += __shfl_xor(tcand, o, 64);
    const uint32_t nkeep = min(nslot, (uint32_t)kKlmSlots);
    if (lane == 0) {                                   // candidate and exactly bounded columns (one add per wave)
        unsigned long long* sc = counters + kCtrShard0 + kCtrShardStride * (int)(blockIdx.x % kKlShards);
        if (tcand) atomicAdd(&sc[0], tcand);
        if (nkeep) atomicAdd(&sc[1], (unsigned long long)nkeep);
    }
    if (nslot == 0) return;
    const uint32_t ex = incl - c;
    wb[1 + lane] = (uint16_t)min(ex, 65535u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t i = lane; i < nkeep; i += 64) {
        acc[4 * i] = 0ull; acc[4 * i + 1] = 0ull; acc[4 * i + 2] = 0ull; acc[4 * i + 3] = 0ull;
        sn[i] = 0u;
    }
    {
        uint32_t wd = word, sl = ex;
        while (wd) {
            const int bit = __builtin_ctz(wd);
            wd &= wd - 1u;
            const int32_t ti = 32 * lane + bit;
            if (sl < (uint32_t)kKlmSlots) spos[sl] = (uint16_t)ti;
            else {                                        // past the slots: kept open
                const int32_t gpos = tstart + ti;
                atomicOr(&need[gpos >> 5], 1u << (gpos & 31));
                if (pairs) {                              // (and not proven hom-ref: a pair for KPM's first stage)
                    const int sh = (int)(blockIdx.x % kKlShards);
                    const unsigned long long k = atomicAdd(&counters[kCtrShard0 + kCtrShardStride * sh + 2], 1ull);
                    if ((int64_t)k < pseg) pairs[(int64_t)sh * pseg + (int64_t)k] = make_uint2((uint32_t)gpos, (uint32_t)s);
                }
            }
            sl++;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- pass 2: each lane's valid calls at the slotted positions its read covers, into the slots' sums (one 8-byte
    //      unit load per position, software-pipelined: a position's load issued before the previous one's sums are
    //      added; the next group's header and base fetched a group ahead)
    const int32_t maxq = gp.max_q;
    for (int st = st0; st < st1; st++) {
        const int64_t e_lo = blkA[(int64_t)st * nblk + (tstart >> shift)];
        const int64_t e_hi = blkB[(int64_t)st * nblk + (tlast >> shift) + 1];
        const int64_t g_hi = (e_hi + 63) >> 6;
        int64_t g = e_lo >> 6;
        int2 hc = g < g_hi ? rh[g * 64 + lane] : make_int2(0, -1);
        int64_t gbc = g < g_hi ? grp[g].base : 0;
        for (; g < g_hi; g++) {
            const int64_t e = g * 64 + lane;
            const int2 h = hc;
            const int64_t gbase = gbc;
            hc = g + 1 < g_hi ? rh[e + 64] : make_int2(0, -1);
            gbc = g + 1 < g_hi ? grp[g + 1].base : 0;
            const int32_t gf = h.x, gl = h.y & 0x7FFFFFFF;
            const int32_t a = max(gf, tstart), b = min(gl, tlast);
            if (!(e >= e_lo && e < e_hi && a <= b)) continue;
            const uint64_t* ub = units + gbase + lane;
            const int32_t A = a - tstart + 32, B = b - tstart + 32;
            uint64_t qu = 0ull;                                 // the position in flight: unit, byte shift, slot
            uint32_t qsh = 0u, qs = 0u;
            bool pend = false;
            auto add = [&]() {
                const uint32_t y = (uint32_t)(qu >> qsh) & 0xFFu;
                if (y & 0x80u) return;                          // not a valid call (the position is callable)
                const uint32_t al = (y >> 5) & 3u;
                int q = (int)(y & 31u);
                q = q > maxq ? maxq : q;
                atomicAdd(&acc[4 * qs + al], w[al == 0 ? 0 : 1][q]);
                atomicAdd(&sn[qs], 1u);
            };
            for (int32_t wi = A >> 5; wi <= (B >> 5); wi++) {
                uint32_t wd = bm[wi];
                if (wi == (A >> 5)) wd &= ~0u << (A & 31);
                if (wi == (B >> 5) && (B & 31) != 31) wd &= (1u << ((B & 31) + 1)) - 1u;
                if (!wd) continue;
                const uint32_t full = bm[wi];
                const uint32_t sbase = wb[wi];
                while (wd) {
                    const int bit = __builtin_ctz(wd);
                    wd &= wd - 1u;
                    const uint32_t sl = sbase + (uint32_t)__popc(full & ((1u << bit) - 1u));
                    if (sl >= (uint32_t)kKlmSlots) continue;
                    const int32_t o = wi * 32 + bit - 32 + tstart - gf;   // byte offset in the read
                    const uint64_t nu = ub[(int64_t)(o >> 3) * 64];
                    if (pend) add();
                    qu = nu; qsh = 8u * (uint32_t)(o & 7); qs = sl; pend = true;
                }
            }
            if (pend) add();
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- pass 3: the exact bound per slot.  A column it cannot prove hom-ref opens its position and, with pairs,
    //      is listed (position, sample) for KPM's first stage: the columns a decided non-reference call can come from
    const long long th = tabs->t_het, to = tabs->t_homo;
    for (uint32_t i0 = 0; i0 < nkeep; i0 += 64) {
        const uint32_t i = i0 + lane;
        bool open = false;
        if (i < nkeep) {
            const unsigned long long a0 = acc[4 * i], a1 = acc[4 * i + 1], a2 = acc[4 * i + 2], a3 = acc[4 * i + 3];
            const long long R1 = (long long)(a0 & 0xFFFFFFFFull), R2 = (long long)(a0 >> 32);
            const long long x1 = (long long)(a1 & 0xFFFFFFFFull), y1 = (long long)(a2 & 0xFFFFFFFFull);
            const long long z1 = (long long)(a3 & 0xFFFFFFFFull);
            const long long x2 = (long long)(a1 >> 32), y2 = (long long)(a2 >> 32), z2 = (long long)(a3 >> 32);
            const bool drop = (R1 - x1 > th) && (R1 - y1 > th) && (R1 - z1 > th) &&
                              (R2 - x2 > to) && (R2 - y2 > to) && (R2 - z2 > to) &&
                              (R2 - x1 - y1 > th) && (R2 - x1 - z1 > th) && (R2 - y1 - z1 > th);
            open = !bound_on || sn[i] > (uint32_t)kMcMaxCalls || !drop;
        }
        const int32_t gpos = i < nkeep ? tstart + spos[i] : 0;
        if (open) atomicOr(&need[gpos >> 5], 1u << (gpos & 31));
        if (pairs) {
            const unsigned long long m = __ballot(open);
            if (m) {
                const int sh = (int)(blockIdx.x % kKlShards);
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(&counters[kCtrShard0 + kCtrShardStride * sh + 2], (unsigned long long)__popcll(m));
                base = __shfl(base, 0, 64);
                if (open) {
                    const int64_t k = (int64_t)base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                    if (k < pseg) pairs[(int64_t)sh * pseg + k] = make_uint2((uint32_t)gpos, (uint32_t)s);
                }
            }
        }
    }
}

// KPM's first stage, its per-position sample masks: pair (position, sample) -> bit sample of the position's queue entry
// (KQN's word bases: qword[w] = the queue index of word w's first open position).  A segment past its capacity sets
// counters[3] bit 62: the first stage then passes every position to the second.
__global__ __launch_bounds__(256) void k_pair_mask(const uint2* __restrict__ pairs, int64_t pseg, const uint32_t* __restrict__ need,
                                                   const int32_t* __restrict__ qword, uint32_t* __restrict__ pmask, int64_t qcap,
                                                   unsigned long long* __restrict__ counters) {
    const int sh = (int)blockIdx.y;
    const unsigned long long n = counters[kCtrShard0 + kCtrShardStride * sh + 2];
    if ((int64_t)n > pseg) {
        if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(&counters[3], 1ull << 62);
        return;
    }
    for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < (int64_t)n; k += (int64_t)gridDim.x * blockDim.x) {
        const uint2 pr = pairs[(int64_t)sh * pseg + k];
        const uint32_t gpos = pr.x, w = gpos >> 5;
        const int64_t q = (int64_t)qword[w] + __popc(need[w] & ((1u << (gpos & 31)) - 1u));
        if (q < qcap) atomicOr(&pmask[q * 8 + (pr.y >> 5)], 1u << (pr.y & 31));
    }
}

// ------------------------------------------------------------------------------------------
// KPM: population genotyping of the queued positions -- one workgroup per position
// ------------------------------------------------------------------------------------------
// MultisampleVariantsDetector.onPileup (discovery/MultisampleVariantsDetector.java:522-558) for an
// SNV pileup: the reads covering the position are gathered in pending order into LDS; the pooled
// counts give the candidate alleles (SingleSampleVariantPileupListener.createSNVVariantPool, :297-332);
// thread s tallies sample s in its read-group order (PileupRecord.getAlleleCalls, :104-111; the fp64
// sums in the reference's order) and genotypes it (genotypeVariantSample, :361-391, with
// VariantDiscoverySNVQAlgorithm.genotypeSNV, :21-97); the multi-allelic loop (discoverPopulationSNV,
// :585-597, makeNewVariant :642-656) and the variant QS (genotypeVariant, :674-693) are block reductions.
constexpr int kPopThreads = 256;
constexpr int kPopTileLog2 = 7;
static_assert((1 << kPopTileLog2) == kPopTile, "KPM pile tile");
static_assert(kPopThreads >= kMaxSamplesDevice, "one thread per sample");

struct PopCall {
    int kind, n_called, c0, c1, gq, total_cn;
    // copy numbers of alleles 0-3, four 16-bit fields of one register pair (indexed fields, even as separate
    // scalars, were folded into an indexed load and kept the struct in scratch); a field never goes below 0
    uint64_t acnp;
    __device__ __forceinline__ int acn(int j) const { return (int)(int16_t)(uint16_t)(acnp >> (16 * j)); }
    __device__ __forceinline__ void add_acn(int j, int v) { acnp += (uint64_t)(int64_t)v << (16 * j); }
    __device__ __forceinline__ void set_acn(int j, int v) {
        acnp = (acnp & ~(0xFFFFull << (16 * j))) | ((uint64_t)(uint16_t)v << (16 * j));
    }
    __device__ __forceinline__ void clear_acn() { acnp = 0; }
};

__device__ inline int tri_d(int i, int j) {      // upper-triangle index of L[i][j] (symmetric, f == g)
    const int a = i < j ? i : j, b = i < j ? j : i;
    return (a == 0 ? 0 : a == 1 ? 4 : a == 2 ? 7 : 9) + (b - a);
}
// a thread's ten log-conditionals kept in LDS (column-major, conflict-free) once its tally is done: KPM's genotyping and
// PL phases read them from there, so the 20 VGPRs they held are free for the fp64 posterior (the 4-wave build spilled)
struct LdsRow {
    const double* p;
    __device__ double operator[](int k) const { return p[k * kPopThreads]; }
};
template <class LA>
__device__ inline double sel10(const LA& L, int k) {
    double v = 0;
#pragma unroll
    for (int e = 0; e < 10; e++) v = e == k ? L[e] : v;
    return v;
}
// element k of a 4-entry register array (static indexes only: a dynamic one sends the array to scratch)
// (written without loops: SROA runs before the unroller, and a loop index there keeps the array in scratch)
__device__ __forceinline__ void set4i(int* a, int k, int v) {
    if (k == 0) a[0] = v;
    else if (k == 1) a[1] = v;
    else if (k == 2) a[2] = v;
    else a[3] = v;
}
__device__ __forceinline__ int sel4i(const int* a, int k) {
    return k == 0 ? a[0] : k == 1 ? a[1] : k == 2 ? a[2] : a[3];
}

// CalledSNV.updateAllelesCopyNumberFromCounts (variants/CalledSNV.java:134-158)
__device__ __forceinline__ void csnv_cn(int genotype, int cref, int calt, int total, int* tot_out, int* ref_out) {
    int ref = 0;
    if (genotype == -1) { *tot_out = total; *ref_out = 0; return; }
    if (genotype == 0) ref = total;
    else if (genotype == 2) ref = 0;
    else if (total <= 2) { total = 2; ref = 1; }
    else {
        const double sum = (double)cref + (double)calt;
        double prop = sum > 0 ? (double)cref / sum : 0.5;
        if (prop > 1) prop = 1;
        ref = (int16_t)java_round_d(prop * total);
        if (ref == 0) ref = 1;
        else if (ref >= total) ref = total - 1;
    }
    *tot_out = total;
    *ref_out = ref;
}
// CalledGenomicVariantImpl.updateAllelesCopyNumberFromCounts (variants/CalledGenomicVariantImpl.java:228-282)
__device__ __forceinline__ void cgv_cn(PopCall& c, int total, const int* rcounts, bool report) {
    c.total_cn = total;
    c.clear_acn();
    if (c.n_called == 0) return;
    const int called[2] = {c.c0, c.c1};
    if (c.n_called == 1 && c.c0 == 0) { c.set_acn(0, total); return; }
    const int nc = c.n_called;
    auto addcn = [&](int j, int v) { c.add_acn(j, v); };
    auto getcn = [&](int j) -> int { return c.acn(j); };
    // (loops over the at most two called alleles unrolled: static indexes)
    if (total <= nc) {
#pragma unroll
        for (int i = 0; i < 2; i++) if (i < nc) addcn(called[i], 1);
        return;
    }
    if (!report) {
        const int def = total / nc;
#pragma unroll
        for (int i = 0; i < 2; i++) if (i < nc) addcn(called[i], def);
        addcn(called[0], total - def * nc);
        return;
    }
    int rc[2] = {0, 0}, tr = 0;
#pragma unroll
    for (int i = 0; i < 2; i++) if (i < nc) { rc[i] = sel4i(rcounts, called[i]); if (rc[i] == 0) rc[i] = 1; tr += rc[i]; }
    int tc = 0;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        if (i >= nc) continue;
        const long long r = java_round_d((double)total * rc[i] / tr);
        const int v = (int)(r > 1 ? r : 1);
        addcn(called[i], v - getcn(called[i]));
        tc += v;
    }
    if (tc < total) addcn(called[0], total - tc);
    else {
        int ex = tc - total;
#pragma unroll
        for (int i = 1; i >= 0; i--) {                     // i = nc - 1 .. 0 while ex > 0
            if (i >= nc || ex <= 0) continue;
            const int cur = getcn(called[i]);
            const int rm = ex < cur - 1 ? ex : cur - 1;
            addcn(called[i], -rm);
            ex -= rm;
        }
    }
}

// genotypeVariantSample with a fresh listener (minQuality = DEF_MIN_QUALITY 40) + genotypeSNV
template <class LA>
__device__ __forceinline__ PopCall genotype_sample_d(const LA& L, const int* cnt, int total, int nal, const int* idx,
                                     const GenotypeParams& gp, int ploidy) {
    PopCall c;
    c.kind = 1; c.n_called = 0; c.c0 = 0; c.c1 = 0; c.gq = 0; c.total_cn = ploidy;
    c.clear_acn();
    if (total == 0) return c;                   // undecided CalledGenomicVariantImpl(variant, new byte[0])
    const double ph = gp.log_prior_homo, px = gp.log_prior_hetero;
    if (nal == 2) {
        // the biallelic case without the 16-entry posterior array (registers: KPM's 4-wave build spilled here): the
        // same sums in the same order, keeping only the four posteriors the call reads and the six exponents the
        // symmetric genotypes reuse
        constexpr int LI[16] = {0, 1, 2, 3, 4, 1, 5, 6, 7, 2, 5, 8, 9, 3, 6, 8};   // ev[k] = L[LI[k]] + prior
        const int r = idx[0], a = idx[1];
        auto kof = [](int x, int y) { return x == y ? 4 * x : (y < x ? 4 * x + 1 + y : 4 * x + y); };
        const int k_rr = kof(r, r), k_aa = kof(a, a), k_ra = kof(r, a), k_ar = kof(a, r);
        double logMax = 1;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const double x = L[LI[k]] + ((k & 3) == 0 ? ph : px);
            if (logMax > 0 || logMax < x) logMax = x;
        }
        double totalProb = 0, v_rr = 0, v_aa = 0, v_ra = 0, v_ar = 0;
        double s1 = 0, s2 = 0, s3 = 0, s6 = 0, s7 = 0, s11 = 0;
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int src = ev_partner(k);
            double val;
            if (src) val = src == 1 ? s1 : src == 2 ? s2 : src == 3 ? s3 : src == 6 ? s6 : src == 7 ? s7 : s11;
            else {
                const double x = (L[LI[k]] + ((k & 3) == 0 ? ph : px)) - logMax;
                val = x < -20 ? 0.0 : pow(10.0, x);
            }
            if (k == 1) s1 = val;
            if (k == 2) s2 = val;
            if (k == 3) s3 = val;
            if (k == 6) s6 = val;
            if (k == 7) s7 = val;
            if (k == 11) s11 = val;
            totalProb += val;
            v_rr = k == k_rr ? val : v_rr;
            v_aa = k == k_aa ? val : v_aa;
            v_ra = k == k_ra ? val : v_ra;
            v_ar = k == k_ar ? val : v_ar;
        }
        double pMax = v_rr / totalProb;
        int genotype = 0;
        const double pHomoAlt = v_aa / totalProb;
        if (pHomoAlt > pMax + 0.01) { pMax = pHomoAlt; genotype = 2; }
        const double pHetero = v_ra / totalProb + v_ar / totalProb;
        if (pHetero > pMax + 0.01) { pMax = pHetero; genotype = 1; }
        int gq = phred_d(1 - pMax);
        if (gq == 0) genotype = -1;
        c.kind = 0;
        int tot = 0, ref = 0;
        csnv_cn(genotype, sel4i(cnt, r), sel4i(cnt, a), ploidy, &tot, &ref);
        if (40 > gq) { genotype = -1; gq = 0; ref = 0; }      // makeUndecided (CalledSNV.java:279-285)
        c.gq = gq;
        c.total_cn = tot;
        if (genotype == -1) c.n_called = 0;
        else if (genotype == 0) { c.n_called = 1; c.c0 = 0; }
        else if (genotype == 2) { c.n_called = 1; c.c0 = 1; }
        else { c.n_called = 2; c.c0 = 0; c.c1 = 1; }
        c.clear_acn();
        c.set_acn(0, genotype == -1 ? 0 : ref);
        c.set_acn(1, genotype == -1 ? 0 : tot - ref);
        return c;
    }
    double ev[16] = {L[0] + ph, L[1] + px, L[2] + px, L[3] + px,
                     L[4] + ph, L[1] + px, L[5] + px, L[6] + px,
                     L[7] + ph, L[2] + px, L[5] + px, L[8] + px,
                     L[9] + ph, L[3] + px, L[6] + px, L[8] + px};
    double logMax = 1;
#pragma unroll
    for (int k = 0; k < 16; k++)
        if (logMax > 0 || logMax < ev[k]) logMax = ev[k];
    double totalProb = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const double x = ev[k] - logMax;
        const int src = ev_partner(k);                        // (j, i) repeats (i, j)'s exponent: its pow is reused
        ev[k] = src ? ev[src] : (x < -20 ? 0.0 : pow(10.0, x));
        totalProb += ev[k];
    }
#pragma unroll
    for (int k = 0; k < 16; k++) ev[k] = ev[k] / totalProb;
    auto post = [&](int a, int b) -> double {
        const int k = a == b ? 4 * a : (b < a ? 4 * a + 1 + b : 4 * a + b);
        double v = 0;
#pragma unroll
        for (int e = 0; e < 16; e++) v = (e == k) ? ev[e] : v;
        return v;
    };
    if (nal == 2) {
        const int r = idx[0], a = idx[1];
        double pMax = post(r, r);
        int genotype = 0;
        const double pHomoAlt = post(a, a);
        if (pHomoAlt > pMax + 0.01) { pMax = pHomoAlt; genotype = 2; }
        const double pHetero = post(r, a) + post(a, r);
        if (pHetero > pMax + 0.01) { pMax = pHetero; genotype = 1; }
        int gq = phred_d(1 - pMax);
        if (gq == 0) genotype = -1;
        c.kind = 0;
        int tot = 0, ref = 0;
        csnv_cn(genotype, sel4i(cnt, r), sel4i(cnt, a), ploidy, &tot, &ref);
        if (40 > gq) { genotype = -1; gq = 0; ref = 0; }      // makeUndecided (CalledSNV.java:279-285)
        c.gq = gq;
        c.total_cn = tot;
        if (genotype == -1) c.n_called = 0;
        else if (genotype == 0) { c.n_called = 1; c.c0 = 0; }
        else if (genotype == 2) { c.n_called = 1; c.c0 = 1; }
        else { c.n_called = 2; c.c0 = 0; c.c1 = 1; }
        c.clear_acn();
        c.set_acn(0, genotype == -1 ? 0 : ref);
        c.set_acn(1, genotype == -1 ? 0 : tot - ref);
        return c;
    }
    int rcounts[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 4; i++) rcounts[i] = i < nal ? sel4i(cnt, idx[i]) : 0;
    int bi = 0, bj = 0;                                       // getIndexesMaxGenotype(report, 0)
    double probMax = post(idx[0], idx[0]);
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (!(i < nal && j >= i && j < nal)) continue;
            double g = post(idx[i], idx[j]);
            if (i != j) g += post(idx[j], idx[i]);
            if (g > probMax + 0.01) { probMax = g; bi = i; bj = j; }
        }
    double maxP = post(sel4i(idx, bi), sel4i(idx, bj));
    if (bi != bj) { maxP += post(sel4i(idx, bj), sel4i(idx, bi)); c.n_called = 2; c.c0 = bi; c.c1 = bj; }
    else { c.n_called = 1; c.c0 = bi; }
    c.gq = phred_d(1 - maxP);
    c.kind = 1;
    cgv_cn(c, ploidy, rcounts, true);
    if (40 > c.gq) { c.n_called = 0; c.gq = 0; cgv_cn(c, c.total_cn, rcounts, true); }   // makeUndecided
    return c;
}

// KPM's gather from the population read-group layout (engine.hpp Staged::prg): PileupRecord.getAlleleCalls(1,
// readGroups) of sample s at global position p -- the nonzero codes of the reads covering p, stream (read-group rank)
// after stream, pending order inside -- into dst (at most cap codes; the host sizes cap by the sample's coverage
// bound).  Entries are walked from the stream's block-table entry eight headers at a time (their two possible
// groups' bases loaded alongside), the covering ones' unit loads issued together.
// The next header batch is loaded while this batch's unit dwords are in flight (configs[4] KPM 0.484-0.485 ->
// 0.423-0.425 ms A/B on one box, tools/history/gpu_r4_klmabn.sh).
#ifndef NGSEP_KPM_GBATCH
#define NGSEP_KPM_GBATCH 8   // entry headers a gathering thread loads at once
#endif
struct PopGather {
    const uint64_t* units;
    const int2* rh;
    const RGroup* grp;
    const int32_t* samp_st;     // streams of sample s: [samp_st[s], samp_st[s + 1]) (s = S: the reads of no sample)
    const int64_t* st_end;      // one past each stream's last entry
    const int32_t* blkA;        // [stream * nblk + (p >> shift)]: the stream's first entry that can cover p
    const uint8_t* ref;
    int64_t nblk;
    int32_t shift, stride;      // stride: codes per sample column
    uint8_t* gcol;              // GCOL kernels: the columns in this device scratch (a workgroup's own part), not in LDS
};
template <int kGatherBatch>                      // entry headers a gathering thread loads at once
__device__ inline int32_t pop_gather(const PopGather& pg, int32_t p, int s, uint8_t* dst, int32_t cap) {
    int32_t rows = 0;
    const uint32_t rc = pg.ref[p];
    const int st1 = pg.samp_st[s + 1];
    for (int st = pg.samp_st[s]; st < st1; st++) {
        int64_t e = pg.blkA[(int64_t)st * pg.nblk + (p >> pg.shift)];
        const int64_t end = pg.st_end[st];
        bool done = false;
        // the next batch's headers are loaded while this batch's unit dwords are in flight (when this batch's last
        // header still starts at or before p, i.e. the next batch can hold covering reads)
        int2 hn[kGatherBatch];
#pragma unroll
        for (int i = 0; i < kGatherBatch; i++) hn[i] = e + i < end ? pg.rh[e + i] : make_int2(0x7FFFFFFF, 0);
        while (!done && e < end) {
            int2 h[kGatherBatch];
#pragma unroll
            for (int i = 0; i < kGatherBatch; i++) h[i] = hn[i];
            const int64_t g0 = e >> 6;
            const int64_t gb0 = pg.grp[g0].base;
            const int64_t gb1 = ((e + kGatherBatch - 1) >> 6) != g0 && ((g0 + 1) << 6) < end ? pg.grp[g0 + 1].base : gb0;
            uint32_t u[kGatherBatch];
#pragma unroll
            for (int i = 0; i < kGatherBatch; i++) {
                const int32_t gf = h[i].x, gl = h[i].y & 0x7FFFFFFF;
                u[i] = 0;
                if (gf <= p && p <= gl) {
                    const int64_t ei = e + i, o = p - gf;
                    // the covering byte's dword of its unit
                    const uint32_t* uw = reinterpret_cast<const uint32_t*>(pg.units + ((ei >> 6) == g0 ? gb0 : gb1) + (o >> 3) * 64 + (ei & 63));
                    u[i] = uw[(o >> 2) & 1];
                }
            }
            if (h[kGatherBatch - 1].x <= p) {
#pragma unroll
                for (int i = 0; i < kGatherBatch; i++)
                    hn[i] = e + kGatherBatch + i < end ? pg.rh[e + kGatherBatch + i] : make_int2(0x7FFFFFFF, 0);
            }
#pragma unroll
            for (int i = 0; i < kGatherBatch; i++) {
                const int32_t gf = h[i].x, gl = h[i].y & 0x7FFFFFFF;
                if (gf > p) done = true;                  // entries are sorted by gfirst: none later covers p
                if (!(gf <= p && p <= gl)) continue;
                const uint32_t code = ((u[i] >> (8 * ((p - gf) & 3))) & 0xFFu) ^ rc;   // (reference-relative)
                if (!code) continue;
                if (rows < cap) dst[rows] = (uint8_t)code;
                rows++;
            }
            e += kGatherBatch;
        }
    }
    return rows;
}

// KPM's first stage (two-stage discovery: ploidy < 3, no -knownVariants, minAlleleDepthFrequency 0, the bounds on) -- one
// wavefront per queued position, lane j = the j-th sample KLM could not prove hom-ref there (pmask, from KLM's pairs):
// only those columns are gathered and genotyped.  Every other sample is hom-ref for any allele set,
// so it adds no called allele and nothing to the variant QS; its other-allele calls only add alleles that no sample
// calls, which the multi-allelic loop (discoverPopulationSNV :590-595, makeNewVariant) removes before the QS is final.
// A position whose QS passes (onPileup :534) -- or with more than 64 such samples, or after a pair segment overflowed --
// goes to qB, the second stage's queue (k_posterior_multi over every column); the others are done.  (The first version,
// k_posterior_multi over the masked columns with one workgroup per position, measured 0.45 against one stage's 0.42 ms on
// configs[4]: a position's chain of dependent gathers, not its columns, sets a workgroup's time.)
struct LdsRow64 {
    const double* p;
    __device__ double operator[](int k) const { return p[k * 64]; }
};
__device__ __forceinline__ int nth_set_bit(uint32_t w, int r) {   // the r-th (0-based) set bit of w
    for (int k = 0; k < r; k++) w &= w - 1u;
    return __builtin_ctz(w);
}
// GCOL: the lanes' columns in pg.gcol (blockIdx.x's 64 x stride bytes) -- a population too deep for them in LDS
template <bool GCOL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4))) void k_stage_a(
    const QueueSite* __restrict__ queue, const unsigned long long* qn, int64_t qcap, const PopGather pg,
    const LikTables* __restrict__ tabs, GenotypeParams gp, int32_t ploidy, uint32_t* __restrict__ pmask,
    QueueSite* __restrict__ qB, unsigned long long* __restrict__ qB_n, int64_t qB_cap, unsigned long long* counters,
    uint32_t* __restrict__ need_clear, int64_t need_words) {
    __shared__ double s_t[3][32];
    __shared__ double s_L[10][64];
    // the pass's open-position bits are read for the last time by k_pair_mask, before this kernel: cleared here for the
    // slot's next pass (no memset dispatch of their own)
    for (int64_t w = (int64_t)blockIdx.x * 64 + threadIdx.x; w < need_words; w += (int64_t)gridDim.x * 64) need_clear[w] = 0u;
    extern __shared__ uint8_t s_gcol[];                  // the lanes' columns, pg.stride codes each
    const int lane = threadIdx.x;
    for (int k = lane; k < 96; k += 64) s_t[k >> 5][k & 31] = (k < 32 ? tabs->A : k < 64 ? tabs->H : tabs->E)[k & 31];
    __syncthreads();
    int64_t n = (int64_t)*qn;
    if (n > qcap) n = qcap;
    const bool passall = ((counters[3] >> 62) & 1ull) != 0;   // (a pair segment past its capacity)
    auto pass_on = [&](const QueueSite& q) {
        if (lane == 0) {
            const unsigned long long k = atomicAdd(qB_n, 1ull);
            if ((int64_t)k < qB_cap) qB[k] = q;
        }
    };
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        const QueueSite qs = queue[i];
        const uint32_t mw = lane < 8 ? pmask[i * 8 + lane] : 0u;
        if (lane < 8) pmask[i * 8 + lane] = 0u;          // (cleared for the next pass)
        if (passall) { pass_on(qs); continue; }
        uint32_t incl = (uint32_t)__popc(mw);
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            const uint32_t x = __shfl_up(incl, o, 64);
            if (lane >= o) incl += x;
        }
        const uint32_t nmask = (uint32_t)__shfl((int)incl, 7, 64);
        if (nmask > 64u) { pass_on(qs); continue; }
        int s = -1;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t wk = (uint32_t)__shfl((int)mw, k, 64), ik = (uint32_t)__shfl((int)incl, k, 64);
            const uint32_t ek = ik - (uint32_t)__popc(wk);
            if ((uint32_t)lane >= ek && (uint32_t)lane < ik) s = 32 * k + nth_set_bit(wk, lane - (int)ek);
        }
        const int32_t gpos = qs.gpos;
        const uint32_t rc = (uint32_t)qs.rc;
        uint8_t* col = GCOL ? pg.gcol + ((int64_t)blockIdx.x * 64 + lane) * pg.stride : s_gcol + (int64_t)lane * pg.stride;
        int32_t rows = 0;
        if (s >= 0) {
            rows = pop_gather<NGSEP_KPM_GBATCH>(pg, gpos, s, col, pg.stride);
            if (rows > pg.stride) {                      // (the host's coverage bound makes this unreachable)
                atomicOr(&counters[3], 1ull << 63);
                rows = pg.stride;
            }
        }
        // the sample's counts and log-conditionals (CountsHelper, as k_posterior_multi)
        int total = 0;
        int cnt[4] = {0, 0, 0, 0};
        double L[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int32_t r = 0; r < rows; r++) {
            const uint32_t cd = col[r];
            total += cd != 0;
            if (!(cd & 0x80u)) continue;
            const uint32_t a = (cd >> 5) & 3u;
            cnt[0] += a == 0; cnt[1] += a == 1; cnt[2] += a == 2; cnt[3] += a == 3;
            int q = (int)(cd & 31u);
            q = q > gp.max_q ? gp.max_q : q;
            const double A = s_t[0][q], H = s_t[1][q], E = s_t[2][q];
            L[0] += a == 0 ? A : E;
            L[4] += a == 1 ? A : E;
            L[7] += a == 2 ? A : E;
            L[9] += a == 3 ? A : E;
            L[1] += a <= 1 ? H : E;
            L[2] += (a & 1) == 0 ? H : E;
            L[3] += (a == 0 || a == 3) ? H : E;
            L[5] += (a == 1 || a == 2) ? H : E;
            L[6] += (a & 1) == 1 ? H : E;
            L[8] += a >= 2 ? H : E;
        }
#pragma unroll
        for (int k = 0; k < 10; k++) s_L[k][lane] = L[k];
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const LdsRow64 Lr{&s_L[0][lane]};
        int pc[4] = {cnt[0], cnt[1], cnt[2], cnt[3]};
        int tt = total;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            pc[0] += __shfl_xor(pc[0], o, 64); pc[1] += __shfl_xor(pc[1], o, 64);
            pc[2] += __shfl_xor(pc[2], o, 64); pc[3] += __shfl_xor(pc[3], o, 64);
            tt += __shfl_xor(tt, o, 64);
        }
        if (tt == 0) continue;                                   // createSNVVariantPool: totalCount 0
        if (!(rc & 0x80u)) continue;                             // N (or masked) reference: no variant
        const int refIdx = (int)((rc >> 5) & 3u);
        int idx[4] = {refIdx, 0, 0, 0};
        int nal = 1;
#pragma unroll
        for (int a = 0; a < 4; a++)                              // minAlleleDepthFrequency 0: a count of 1
            if (a != refIdx && sel4i(pc, a) >= 1) { set4i(idx, nal < 4 ? nal : 3, a); nal++; }
        if (nal < 2) continue;
        int qsv = 0;
        for (;;) {
            const PopCall call = genotype_sample_d(Lr, cnt, total, nal, idx, gp, ploidy);
            const bool homref = call.n_called == 1 && call.c0 == 0;
            int q = call.n_called > 0 && !homref ? call.gq : 0;
            int bits = 0;
            if (call.n_called >= 1) bits |= 1 << sel4i(idx, call.c0 & 3);
            if (call.n_called == 2) bits |= 1 << sel4i(idx, call.c1 & 3);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                q = max(q, __shfl_xor(q, o, 64));
                bits |= __shfl_xor(bits, o, 64);
            }
            qsv = q;
            const int set = bits | (1 << refIdx);
            if (nal <= 2) break;
            if (__popc(set) == nal) break;
            nal = 1;
#pragma unroll
            for (int a = 0; a < 4; a++) if (a != refIdx && (set >> a & 1)) { set4i(idx, nal, a); nal++; }
            if (nal < 2) break;
        }
        if (nal < 2) continue;                                   // only the reference allele is left
        if (qsv == 0 || qsv < gp.min_quality) continue;          // MultisampleVariantsDetector.java:534
        pass_on(qs);
    }
}

// POOL: ploidy >= 3 (the pool branch's report arrays would otherwise cost every run registers and scratch).
// GATHER, where the columns come from: 0 a site-major pile (the realigner's region positions, engine.cpp
// run_population_regions; ppile / prow / pboff); 1 the population read-group layout, gathered here into dynamic LDS
// (measured and not kept: a separate gather kernel, one thread per (position, sample) at 8 waves per SIMD, into
// columns KPM then read with the next position's in flight -- 0.64 against 0.52 ms for gather + KPM on configs[4]:
// the gather's cost is its scattered lines, ~10 per sample column, not latency KPM fails to hide)
// GCOL (GATHER 1): the columns in pg.gcol (blockIdx.x's (S + 1) x stride bytes), not LDS -- a population whose per-sample
// coverage bound times S + 1 exceeds kPopGatherCap (MultisampleVariantsDetector genotypes at any depth, :522-558)
template <bool POOL, int WPE, int GATHER, bool GCOL>
__global__ __launch_bounds__(kPopThreads) __attribute__((amdgpu_waves_per_eu(WPE))) void k_posterior_multi(
    const QueueSite* __restrict__ queue, const unsigned long long* qn, int64_t qcap,
    const uint8_t* __restrict__ ppile, const int32_t* __restrict__ prow, const int64_t* __restrict__ pboff,
    const PopGather pg, const LikTables* __restrict__ tabs, GenotypeParams gp,
    int32_t n_samples, double min_adf, int32_t ploidy, const PoolTables* __restrict__ pt,
    ngsep_popsite_out* __restrict__ sites, ngsep_sample_call* __restrict__ calls,
    unsigned long long* counters, int64_t cap, unsigned long long* __restrict__ stamps) {
    // stamps (diagnostics, NGSEP_TIMING): s_memtime at the phase ends of block 0's first site
    auto stamp = [&](int k) {
        if (stamps && blockIdx.x == 0 && threadIdx.x == 0) stamps[k] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);
    __shared__ double s_t[3][32];
    __shared__ double s_L[10][kPopThreads];             // each thread's log-conditionals after its tally (LdsRow)
    __shared__ int32_t s_pc[4], s_tot;
    __shared__ int32_t s_called, s_qs;
    __shared__ unsigned long long s_base;
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < 96) s_t[tid >> 5][tid & 31] = (tid < 32 ? tabs->A : tid < 64 ? tabs->H : tabs->E)[tid & 31];
    int64_t n = (int64_t)*qn;
    if (n > qcap) n = qcap;
    // thread s's column of a queued position: its rows and first code (site-major tile, engine.hpp: the S + 1 columns
    // of gpos are one contiguous run of stride bytes).  The next position's entry and column are fetched while the
    // current one is genotyped.
    auto column_of = [&](int64_t qi, int32_t gpos, int32_t& rows, const uint8_t*& col) {
        rows = 0;
        col = nullptr;
        if (tid > n_samples) return;
        (void)qi;
        const int64_t b0 = (int64_t)(gpos >> kPopTileLog2) * (n_samples + 1), bi = b0 + tid;
        const int64_t stride = (pboff[b0 + n_samples + 1] - pboff[b0]) >> kPopTileLog2;
        rows = prow[bi];
        col = ppile + pboff[bi] + (int64_t)(gpos & (kPopTile - 1)) * stride;
    };
    extern __shared__ uint8_t s_gcol[];                  // GATHER: the position's columns, pg.stride codes per sample
    QueueSite qs_next{0, 0};
    int32_t rows_next = 0;
    const uint8_t* col_next = nullptr;
    if ((int64_t)blockIdx.x < n) {
        qs_next = queue[blockIdx.x];
        if (GATHER != 1) column_of(blockIdx.x, qs_next.gpos, rows_next, col_next);
    }
    for (int64_t i = blockIdx.x; i < n; i += gridDim.x) {
        __syncthreads();
        const QueueSite qs = qs_next;
        const int32_t gpos = qs.gpos;
        const uint32_t rc = (uint32_t)qs.rc;
        const int64_t inext = i + gridDim.x;
        if (inext < n) qs_next = queue[inext];
        if (tid == 0) { s_pc[0] = s_pc[1] = s_pc[2] = s_pc[3] = 0; s_tot = 0; s_called = 0; s_qs = 0; }
        __syncthreads();
        // 1-3. thread s walks sample s's column of the pile (read-group rank order, pending order inside:
        //      PileupRecord.getAlleleCalls(span, readGroups), :104-111), 8 codes in flight; thread n_samples
        //      walks the column of the reads of no sample, which only enter the pooled counts
        //      (getAlleleCalls(1, null))
        int total = 0;
        int cnt[4] = {0, 0, 0, 0};
        double L[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        constexpr bool pool = POOL;
        int32_t rows = rows_next;
        const uint8_t* col = col_next;
        if (GATHER == 1 && tid <= n_samples) {
            uint8_t* dst = GCOL ? pg.gcol + ((int64_t)blockIdx.x * (n_samples + 1) + tid) * pg.stride
                                : s_gcol + (int64_t)tid * pg.stride;
            rows = pop_gather<NGSEP_KPM_GBATCH>(pg, gpos, tid, dst, pg.stride);
            if (rows > pg.stride) {                          // (the host's coverage bound makes this unreachable)
                atomicOr(&counters[3], 1ull << 63);
                rows = pg.stride;
            }
            col = dst;
        }
        if (tid <= n_samples) {
            const bool tally = tid < n_samples && !pool;        // (the pool algorithm walks the column itself)
            for (int32_t r0 = 0; r0 < rows; r0 += 8) {
                uint32_t code[8];
#pragma unroll
                for (int k = 0; k < 8; k++) code[k] = r0 + k < rows ? (uint32_t)col[r0 + k] : 0u;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t cd = code[k];
                    total += cd != 0;                                  // CountsHelper.java:210
                    if (!(cd & 0x80u)) continue;                       // q<=3 or not A/C/G/T (:214-221)
                    const uint32_t a = (cd >> 5) & 3u;
                    cnt[0] += a == 0; cnt[1] += a == 1; cnt[2] += a == 2; cnt[3] += a == 3;
                    if (!tally) continue;
                    int q = (int)(cd & 31u);
                    q = q > gp.max_q ? gp.max_q : q;                   // -maxBaseQS (:217-219)
                    const double A = s_t[0][q], H = s_t[1][q], E = s_t[2][q];
                    L[0] += a == 0 ? A : E;
                    L[4] += a == 1 ? A : E;
                    L[7] += a == 2 ? A : E;
                    L[9] += a == 3 ? A : E;
                    L[1] += a <= 1 ? H : E;
                    L[2] += (a & 1) == 0 ? H : E;
                    L[3] += (a == 0 || a == 3) ? H : E;
                    L[5] += (a == 1 || a == 2) ? H : E;
                    L[6] += (a & 1) == 1 ? H : E;
                    L[8] += a >= 2 ? H : E;
                }
            }
        }
        if (i == blockIdx.x) stamp(1);
#pragma unroll
        for (int k = 0; k < 10; k++) s_L[k][tid] = L[k];
        __atomic_signal_fence(__ATOMIC_SEQ_CST);             // (read back from LDS below: the registers are released)
        const LdsRow Lr{&s_L[0][tid]};
        if (GATHER != 1 && inext < n) column_of(inext, qs_next.gpos, rows_next, col_next);   // (in flight during the genotyping)
        // pooled counts: the sum over every sample and the reads of no sample
        {
            int c0 = cnt[0], c1 = cnt[1], c2 = cnt[2], c3 = cnt[3], tt = total;
            for (int o = 32; o > 0; o >>= 1) {
                c0 += __shfl_xor(c0, o, 64); c1 += __shfl_xor(c1, o, 64);
                c2 += __shfl_xor(c2, o, 64); c3 += __shfl_xor(c3, o, 64);
                tt += __shfl_xor(tt, o, 64);
            }
            if (lane == 0) {
                atomicAdd(&s_pc[0], c0); atomicAdd(&s_pc[1], c1); atomicAdd(&s_pc[2], c2); atomicAdd(&s_pc[3], c3);
                atomicAdd(&s_tot, tt);
            }
        }
        if (tid == n_samples) { total = 0; cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0; }
        __syncthreads();
        if (i == blockIdx.x) stamp(2);
        // -knownVariants (MultisampleVariantsDetector.onPileup :539-551): the input variant's own alleles, every
        // sample genotyped (genotypeVariant :674-693) and the record written whatever its QS
        const bool known = (rc & 0x400u) != 0;
        if (s_tot == 0 && !known) continue;                       // createSNVVariantPool: totalCount 0
        if (ABLATE(gp.ablate, 64)) continue;                             // diagnostics: tallies only
        // 4. candidate alleles from the pooled counts (createSNVVariantPool)
        if (!(rc & 0x80u)) continue;                               // N (or masked) reference: no variant
        const int refIdx = (int)((rc >> 5) & 3u);
        const int pc[4] = {s_pc[0], s_pc[1], s_pc[2], s_pc[3]};
        const int sum = pc[0] + pc[1] + pc[2] + pc[3];
        double minCount = min_adf * sum;
        if (minCount < 1) minCount = 1;
        int idx[4] = {refIdx, 0, 0, 0};
        int nal = 1;
        if (known) {
            idx[1] = (int)((rc >> 8) & 3u);
            nal = 2;
        } else {
            for (int a = 0; a < 4; a++)
                if (a != refIdx && pc[a] >= minCount) { set4i(idx, nal < 4 ? nal : 3, a); nal++; }
        }
        if (nal < 2) continue;
        int multisnv = nal > 2;
        // 5. genotype every sample; shrink a multi-allelic variant to the called alleles
        PopCall call;
        PoolResult pr;
        int qsv = 0;
        for (;;) {
            if (tid == 0) { s_called = 0; s_qs = 0; }
            __syncthreads();
            if (tid < n_samples && pool) {
                // genotypeVariantSample's pool branch (SingleSampleVariantPileupListener.java:368-371): genotypeVariantPool
                // over the sample's calls, setAllCounts, makeUndecided below the fresh listener's minQuality (40)
                pr = pool_genotype(col, rows, total, cnt, idx, nal, pt, gp.max_q);
                call.kind = 1; call.n_called = pr.n_called; call.c0 = pr.c0 < 0 ? 0 : pr.c0; call.c1 = pr.c1 < 0 ? 0 : pr.c1;
                call.gq = pr.gq; call.total_cn = ploidy;
                call.clear_acn();
                call.set_acn(0, pr.acn[0]); call.set_acn(1, pr.acn[1]); call.set_acn(2, pr.acn[2]); call.set_acn(3, pr.acn[3]);
                if (40 > call.gq) {
                    call.n_called = 0; call.gq = 0;
                    call.clear_acn();
                }
            }
            if (tid < n_samples) {
                if (!pool) call = genotype_sample_d(Lr, cnt, total, nal, idx, gp, ploidy);
                const bool homref = call.n_called == 1 && call.c0 == 0;
                if (call.n_called > 0 && !homref) atomicMax(&s_qs, call.gq);
                int bits = 0;
                if (call.n_called >= 1) bits |= 1 << sel4i(idx, call.c0 & 3);
                if (call.n_called == 2) bits |= 1 << sel4i(idx, call.c1 & 3);
                if (bits) atomicOr(&s_called, bits);
            }
            __syncthreads();
            qsv = s_qs;
            const int set = s_called | (1 << refIdx);
            __syncthreads();                                       // everyone has read before the next reset
            if (nal <= 2) break;
            if (__popc(set) == nal) break;
            nal = 1;
            for (int a = 0; a < 4; a++) if (a != refIdx && (set >> a & 1)) { set4i(idx, nal, a); nal++; }
            multisnv = 0;                                          // makeNewVariant: SNV or GenomicVariantImpl (no TYPE)
            if (nal < 2) break;
        }
        if (i == blockIdx.x) stamp(5);
        if (nal < 2) continue;                                     // only the reference allele is left
        if (!known && (qsv == 0 || qsv < gp.min_quality)) continue;   // MultisampleVariantsDetector.java:534
        // 6. emit the site and its calls
        __syncthreads();
        if (tid == 0) s_base = atomicAdd(&counters[0], 1ull);
        __syncthreads();
        const unsigned long long at = s_base;
        if ((int64_t)at >= cap) continue;
        if (tid == 0) {
            ngsep_popsite_out o;
            o.seq_id = (int32_t)i; o.pos = gpos; o.n_alleles = (int8_t)nal;   // (seq_id: the queue index, host order)
            for (int k = 0; k < 4; k++) o.alleles[k] = (int8_t)(k < nal ? idx[k] : -1);
            o.multisnv_type = (int8_t)multisnv; o.qual = (int16_t)qsv; o.pad = 0;
            sites[at] = o;
        }
        if (tid < n_samples) {
            // the call's 19 dwords stored as they are computed (a whole record held in registers pushed KPM's
            // 4-wave build into scratch)
            uint32_t* o = reinterpret_cast<uint32_t*>(calls + (int64_t)at * n_samples + tid);
            static_assert(sizeof(ngsep_sample_call) == 76, "ngsep_sample_call: 19 dwords");
            o[0] = (uint32_t)(uint8_t)call.kind | (uint32_t)(uint8_t)call.n_called << 8 | (uint32_t)(uint8_t)call.c0 << 16 |
                   (uint32_t)(uint8_t)call.c1 << 24;
            o[1] = (uint32_t)(uint16_t)call.gq | (uint32_t)(uint16_t)call.total_cn << 16;
            o[2] = (uint32_t)(pool ? pr.dp : total);
#pragma unroll
            for (int k = 0; k < 4; k++) o[3 + k] = (uint32_t)cnt[k];
            o[7] = (uint32_t)call.acnp;                              // (int16 acn[0], acn[1])
            o[8] = (uint32_t)(call.acnp >> 32);                      // (acn[2], acn[3])
            uint32_t* pl = o + 9;
            int npl = 0;                                           // PL values written (the rest are 0)
            // PL (VCFFileWriter.java:200-212) from the call report
            if (pool) {
                if (pr.report) {
                    for (int j = 0; j < nal; j++)
                        for (int ii = 0; ii <= j; ii++)
                            pl[npl++] = (uint32_t)(int32_t)java_round_d(-10 * sel10(pr.L, ii * nal - ii * (ii - 1) / 2 + (j - ii)));
                }
            } else if (call.kind == 0) {
                const float hr = (float)sel10(Lr, tri_d(idx[0], idx[0])), ha = (float)sel10(Lr, tri_d(idx[1], idx[1]));
                const float ra = (float)sel10(Lr, tri_d(idx[0], idx[1])), ar = ra;
                const bool present = (hr + ra + ar + ha) != 0;     // CalledSNV.java:422 (float sum)
                if (present) {
                    pl[0] = (uint32_t)(int32_t)java_round_d(-10 * (double)hr);
                    pl[1] = (uint32_t)(int32_t)java_round_d(-10 * (double)ra);
                    pl[2] = (uint32_t)(int32_t)java_round_d(-10 * (double)ha);
                    npl = 3;
                }
            } else if (total > 0) {
                for (int j = 0; j < nal; j++)
                    for (int ii = 0; ii <= j; ii++)
                        pl[npl++] = (uint32_t)(int32_t)java_round_d(-10 * sel10(Lr, tri_d(sel4i(idx, ii), sel4i(idx, j))));
            }
            for (int k = npl; k < 10; k++) pl[k] = 0u;
        }
    }
}

// ------------------------------------------------------------------------------------------
// KO: order the emitted records by global position.  KP appended every record to the bucket of its
//     position (2^shift positions per bucket, bcap records each).  Each KO workgroup sums the (capped)
//     counts of the buckets before its 16 for their output offsets (an L2-resident read: no separate
//     scan launch), block 0 writes the record count and the fullest bucket; one wave per bucket ranks
//     its keys and copies the records in order.
// ------------------------------------------------------------------------------------------

constexpr int kKofBuckets = 16;                // one wave per bucket, 16 waves per workgroup
__global__ __launch_bounds__(1024) void ko_fused(const SiteRec* __restrict__ brec, const int32_t* __restrict__ bcount,
                                                 int64_t nb, int32_t bcap, unsigned long long* __restrict__ counters,
                                                 SiteRec* __restrict__ sorted, int64_t cap,
                                                 const int4* __restrict__ wins, int32_t n_wins, int32_t bucket_span) {
    __shared__ uint32_t s_pos[kKofBuckets][1024];   // crowded buckets only (> 64 records)
    __shared__ int32_t s_red[16], s_cnt[kKofBuckets];
    __shared__ int32_t s_mx[16];
    __shared__ long long s_raw[16];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int64_t b0 = (int64_t)blockIdx.x * kKofBuckets;
    // the output offset of this block's buckets: the (capped) records of every bucket before them, then a prefix
    // over its own 16; block 0 also totals every record KP emitted and the fullest bucket (above bcap the host
    // grows the buckets and reruns)
    {
        int32_t part = 0, mx = 0;
        long long raw = 0;
        const int64_t lim = blockIdx.x == 0 ? nb : b0;
        for (int64_t b = tid; b < lim; b += 1024) {
            const int32_t c = bcount[b];
            if (b < b0) part += c < bcap ? c : bcap;
            raw += c;
            mx = c > mx ? c : mx;
        }
        for (int o = 32; o > 0; o >>= 1) {
            part += __shfl_xor(part, o, 64);
            raw += __shfl_xor(raw, o, 64);
            const int32_t m2 = __shfl_xor(mx, o, 64);
            mx = m2 > mx ? m2 : mx;
        }
        if (lane == 0) { s_red[wv] = part; s_mx[wv] = mx; s_raw[wv] = raw; }
        if (tid < kKofBuckets) {
            const int32_t c = b0 + tid < nb ? bcount[b0 + tid] : 0;
            s_cnt[tid] = c < bcap ? c : bcap;
        }
        __syncthreads();
        if (blockIdx.x == 0 && tid == 0) {
            int32_t m = 0;
            long long total = 0;
            for (int k = 0; k < 16; k++) { m = s_mx[k] > m ? s_mx[k] : m; total += s_raw[k]; }
            counters[0] = (unsigned long long)total | ((unsigned long long)m << 40);
        }
    }
    const int64_t b = b0 + wv;
    if (b >= nb) return;
    const int32_t c = s_cnt[wv];
    if (c == 0) return;
    const SiteRec* src = brec + b * bcap;
    int64_t off = 0;
    for (int k = 0; k < 16; k++) off += s_red[k];
    for (int k = 0; k < wv; k++) off += s_cnt[k];
    // the last window starting at or before the bucket (wave-uniform); a record's window is that one or
    // (rarely) a later one.  Records only arise in window bodies, where the reference is non-zero.
    int32_t wb = 0;
    {
        const int32_t b0pos = (int32_t)(b * bucket_span);
        int32_t hi = n_wins - 1;
        while (wb < hi) {
            const int32_t mid = (wb + hi + 1) >> 1;
            if (wins[mid].x <= b0pos) wb = mid;
            else hi = mid - 1;
        }
    }
    constexpr int W = sizeof(SiteRec) / 4;          // 16 dwords
    // rank (position, then arrival) and the mapped (sequence, 1-based position) of record k, on lane k
    // (c <= 64) or in rounds (crowded buckets)
    for (int k0 = 0; k0 < c; k0 += 64) {
        const int k = k0 + lane;
        int32_t rank = 0, seq = 0, pos1 = 0;
        uint32_t mine = 0;
        if (k < c) {
            mine = (uint32_t)src[k].pos;
            int32_t wi = wb;
            while (wi + 1 < n_wins && wins[wi + 1].x <= (int32_t)mine) wi++;
            const int4 wd = wins[wi];                 // {global start of w0, w0, seq_id, wlen}
            seq = wd.z;
            pos1 = wd.y + ((int32_t)mine - wd.x);
        }
        if (c <= 64) {
            for (int m = 0; m < c; m++) {
                const uint32_t o = (uint32_t)__shfl((int)mine, m, 64);
                rank += (o < mine || (o == mine && m < k)) ? 1 : 0;
            }
        } else {
            if (k0 == 0) {                            // stage every key once
                for (int m = lane; m < c; m += 64) s_pos[wv][m] = (uint32_t)src[m].pos;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            if (k < c)
                for (int m = 0; m < c; m++) {
                    const uint32_t o = s_pos[wv][m];
                    rank += (o < mine || (o == mine && m < k)) ? 1 : 0;
                }
        }
        // cooperative copy of this round's records: 16 consecutive lanes per record, coalesced
        const int nr = min(64, c - k0);
        for (int i0 = 0; i0 < nr * W; i0 += 64) {     // wave-uniform trip count: the shuffles see every lane
            const int idx = i0 + lane;
            const int r = min(idx / W, 63), w = idx - (idx / W) * W;
            const int32_t rk = __shfl(rank, r, 64);
            const int32_t sq = __shfl(seq, r, 64);
            const int32_t p1 = __shfl(pos1, r, 64);
            if (idx < nr * W) {
                const int64_t to = off + rk;
                const uint32_t v = w == 0 ? (uint32_t)sq : w == 1 ? (uint32_t)p1
                                                                  : reinterpret_cast<const uint32_t*>(src + k0 + r)[w];
                if (to < cap) reinterpret_cast<uint32_t*>(sorted + to)[w] = v;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// a launch's error; with NGSEP_SYNC_CHECK (diagnostics) the device is drained after every launch, so a fault
// is reported at the launch (HIP_TRY's line) that caused it
static hipError_t launch_check() {
    static const bool sync = diag_env("NGSEP_SYNC_CHECK") != nullptr;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || !sync) return e;
    return hipDeviceSynchronize();
}

// ---- pinned host memory and the DMA endpoint registry (engine.hpp) ----
// Round 3's intermittent "illegal memory access" faults all surfaced at host <-> device copies whose host side was
// pageable memory (std::vector / new[] arrays of the uploads, freed right after each upload, engine.cpp
// release_staged).  For a pageable copy above GPU_PINNED_MIN_XFER_SIZE the HIP runtime pins the host range in place
// (hsa_amd_memory_lock_to_pool, a KFD userptr mapping) and keeps the pin cached after the copy returns; the freed
// range comes back from glibc at the same address for the next window / contig / test's same-sized array, so a later
// copy could go through a pin whose pages had been unmapped.  Hence the invariant: no copy's host endpoint is ever
// pageable.  Pageable sources are memcpy'd into two hipHostMalloc'd staging buffers (h2d); every other host endpoint
// must lie in a block recorded below, which dma_copy checks before it enqueues the copy.
namespace {
struct PinBlock { size_t bytes; int kind; };       // kind 1: aligned_alloc + hipHostRegister, 2: hipHostMalloc
std::mutex g_pin_mu;
std::map<uintptr_t, PinBlock> g_pins;
int host_device_count() {
    static const int n = [] { int k = 0; return hipGetDeviceCount(&k) == hipSuccess ? k : 0; }();
    return n;
}
void pin_record(void* p, size_t bytes, int kind) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pins[(uintptr_t)p] = PinBlock{bytes, kind};
}
int pin_forget(void* p) {                          // the block's kind (0: not recorded)
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.find((uintptr_t)p);
    if (it == g_pins.end()) return 0;
    const int k = it->second.kind;
    g_pins.erase(it);
    return k;
}
}  // namespace

bool pinned_covers(const void* p, size_t bytes) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pins.upper_bound(a);
    if (it == g_pins.begin()) return false;
    --it;
    return a >= it->first && a + bytes <= it->first + it->second.bytes;
}

// runtime-allocated pinned host buffers (hipHostMalloc), recorded for dma_copy
static hipError_t host_pinned_malloc(void** p, size_t bytes) {
    const hipError_t e = hipHostMalloc(p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) pin_record(*p, bytes, 2);
    return e;
}
static void host_pinned_free(void* p) {
    if (!p) return;
    (void)pin_forget(p);
    (void)hipHostFree(p);                          // (the runtime waits for the device's streams)
}

void* pinned_alloc(size_t bytes) {
    const size_t rounded = (std::max<size_t>(bytes, 1) + 4095) / 4096 * 4096;
    if (host_device_count() <= 0) return std::malloc(rounded);     // host-only code paths: nothing is copied
    void* p = nullptr;
    if (rounded >= ((size_t)64 << 20)) {
        // a large block: transparent huge pages, faulted in on all host threads before the registration pins them
        // (4 KB pages faulted one by one inside hipHostRegister took ~0.5 s for a 3 GB population layout)
        constexpr size_t kHuge = (size_t)2 << 20;
        const size_t n = (rounded + kHuge - 1) / kHuge * kHuge;
        p = std::aligned_alloc(kHuge, n);
        if (p) {
            madvise(p, n, MADV_HUGEPAGE);
            char* c = static_cast<char*>(p);
            parallel_for((int64_t)(n / kHuge), 16, [&](int64_t a, int64_t b) {
                for (int64_t k = a; k < b; k++) c[(size_t)k * kHuge] = 0;
            });
        }
    } else {
        p = std::aligned_alloc(4096, rounded);
    }
    if (p && hipHostRegister(p, rounded, hipHostRegisterDefault) == hipSuccess) {
        pin_record(p, rounded, 1);
        return p;
    }
    std::free(p);
    // registration refused (locked-memory limit, an overlapping registration): runtime-allocated pinned memory
    void* q = nullptr;
    if (host_pinned_malloc(&q, rounded) == hipSuccess) return q;
    return nullptr;
}
void pinned_free(void* p) {
    if (!p) return;
    const int kind = pin_forget(p);
    if (kind == 0) { std::free(p); return; }       // (host-only code paths)
    // no copy may still be reading the block when it is unregistered (an upload whose run launched nothing after it
    // is not waited for by the run's own synchronisation)
    (void)hipDeviceSynchronize();
    if (kind == 2) { (void)hipHostFree(p); return; }
    (void)hipHostUnregister(p);
    std::free(p);
}

int dma_copy(void* dst, const void* src, size_t bytes, int kind, void* stream, bool sync, std::string& err, const char* file, int line) {
    if (!bytes) return 0;
    const void* host = kind == 0 ? src : static_cast<const void*>(dst);
    const std::string where = std::string(file) + ":" + std::to_string(line);
    if (!pinned_covers(host, bytes)) {
        err = "internal error: the host side of the device copy at " + where + " is not registered pinned memory";
        return -1;
    }
    const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost;
    const hipError_t e = sync ? hipMemcpy(dst, src, bytes, k) : hipMemcpyAsync(dst, src, bytes, k, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) { err = "device copy at " + where + ": " + hipGetErrorString(e); return -1; }
    return 0;
}
#define DMA(dst, src, bytes, kind, st) do { if (dma_copy((dst), (src), (bytes), (kind), (st), false, err, "kernels.hip", __LINE__) != 0) return -1; } while (0)
#define DMA_SYNC(dst, src, bytes, kind) do { if (dma_copy((dst), (src), (bytes), (kind), nullptr, true, err, "kernels.hip", __LINE__) != 0) return -1; } while (0)

// host -> device copy of pageable host memory: chunks memcpy'd (all host threads) into the device's two pinned
// staging buffers, each DMA'd on `st` while the next is filled.  Returns once the source has been read (it may be
// freed); the last chunk's DMA may still run, and a staging buffer is reused only after its event.  One thread at a
// time drives a device (the window worker, or the caller's thread), so the staging state needs no lock.
constexpr size_t kStageBytes = (size_t)64 << 20;
static int h2d(Device* d, void* dst, const void* src, size_t bytes, hipStream_t st, std::string& err) {
    if (!bytes) return 0;
    for (int k = 0; k < 2; k++)
        if (!d->stage[k]) {
            HIP_TRY(host_pinned_malloc((void**)&d->stage[k], kStageBytes));
            HIP_TRY(hipEventCreateWithFlags(&d->stage_ev[k], hipEventDisableTiming));
            d->stage_busy[k] = false;
        }
    const uint8_t* in = static_cast<const uint8_t*>(src);
    uint8_t* out = static_cast<uint8_t*>(dst);
    for (size_t off = 0; off < bytes;) {
        const size_t n = std::min(kStageBytes, bytes - off);
        const int k = d->stage_k;
        if (d->stage_busy[k]) HIP_TRY(hipEventSynchronize(d->stage_ev[k]));
        uint8_t* buf = d->stage[k];
        if (n >= ((size_t)4 << 20))
            parallel_for((int64_t)((n + (1 << 20) - 1) >> 20), 1, [&](int64_t a, int64_t b) {
                const size_t lo = (size_t)a << 20, hi = std::min(n, (size_t)b << 20);
                std::memcpy(buf + lo, in + off + lo, hi - lo);
            });
        else std::memcpy(buf, in + off, n);
        HIP_TRY(hipMemcpyAsync(out + off, buf, n, hipMemcpyHostToDevice, st));
        HIP_TRY(hipEventRecord(d->stage_ev[k], st));
        d->stage_busy[k] = true;
        d->stage_k ^= 1;
        off += n;
    }
    return 0;
}
#define H2D(dst, src, bytes, st) do { if (h2d(d, (dst), (src), (bytes), (st), err) != 0) return -1; } while (0)

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
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&d->copy_stream, hipStreamNonBlocking) != hipSuccess) { err = "stream"; delete d; return nullptr; }
    for (auto& e : d->ev) (void)hipEventCreate(&e);
    // both slots' runs go to the device stream: with a stream per slot (NGSEP_SLOT_STREAMS=1) the next
    // run's KT overlaps this run's KP/KO, measured slower (KT shares the CUs: 70 -> 60 G positions/s)
    const bool one_stream = diag_env("NGSEP_SLOT_STREAMS") == nullptr;
    for (auto& sl : d->slot) {
        if (one_stream) sl.stream = d->stream;
        else if (hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking) != hipSuccess) { err = "stream"; return nullptr; }
        if (hipMalloc(&sl.d_tables, sizeof(LikTables)) != hipSuccess) { err = "device allocation failed"; return nullptr; }
        for (int k = 0; k < 6; k++)     // 0-2 and 5 time the kernels; 3-4 only order the streams
            (void)hipEventCreateWithFlags(&sl.ev[k], (k < 3 || k == 5) ? hipEventDefault : hipEventDisableTiming);
    }
    if (hipMalloc(&d->d_counters, kCtrWords * sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(d->d_counters, 0, kCtrWords * sizeof(unsigned long long)) != hipSuccess ||
        host_pinned_malloc((void**)&d->h_counters, kCtrWords * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&d->d_tables, sizeof(LikTables)) != hipSuccess) {
        err = "device allocation failed";
        delete d;
        return nullptr;
    }
    // the code object is loaded now (an empty launch), not inside the first run
    hipLaunchKernelGGL(k_zero_i32, dim3(1), dim3(256), 0, d->stream, (int32_t*)nullptr, (int64_t)0);
    (void)hipStreamSynchronize(d->stream);
    for (int k = 0; k < 2; k++) {
        if (hipMalloc(&d->slot[k].d_ctr, kCtrWords * sizeof(unsigned long long)) != hipSuccess ||
            hipMemset(d->slot[k].d_ctr, 0, kCtrWords * sizeof(unsigned long long)) != hipSuccess ||
            host_pinned_malloc((void**)&d->slot[k].h_ctr, kCtrWords * sizeof(unsigned long long)) != hipSuccess) {
            err = "pinned allocation failed";
            return nullptr;
        }
        (void)hipEventRecord(d->slot[k].ev[4], d->copy_stream);  // a fresh slot is free
    }
    return d;
}

int64_t device_last_hard(const Device* d) { return d ? d->last_hard : 0; }
int64_t device_last_exact(const Device* d) { return d ? d->last_exact : 0; }

void device_release(Device* d) {
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    (void)hipDeviceSynchronize();                    // uncollected runs are dropped
    for (auto& sl : d->slot) sl.busy = false;
    d->n_collected = d->n_submitted;
    (void)hipFree(d->d_pile); d->d_pile = nullptr;
    (void)hipFree(d->d_planes); d->d_planes = nullptr;
    (void)hipFree(d->d_olist); d->d_olist = nullptr;
    (void)hipFree(d->d_loff); d->d_loff = nullptr;
    d->cap_olist = d->cap_loff = 0;
    (void)hipFree(d->d_cneg); d->d_cneg = nullptr;
    (void)hipFree(d->d_wins); d->d_wins = nullptr;
    d->n_wins = 0;
    d->planes_W = 0;
    (void)hipFree(d->d_ref); d->d_ref = nullptr;
    (void)hipFree(d->d_tinfo); d->d_tinfo = nullptr;
    (void)hipFree(d->d_units); d->d_units = nullptr;
    (void)hipFree(d->d_rbytes); d->d_rbytes = nullptr;
    (void)hipFree(d->d_roff); d->d_roff = nullptr;
    d->cap_rbytes = d->cap_roff = 0;
    (void)hipFree(d->d_refchars); d->d_refchars = nullptr;
    (void)hipFree(d->d_zero); d->d_zero = nullptr;
    d->cap_refchars = d->cap_zero = 0;
    (void)hipFree(d->d_rh); d->d_rh = nullptr;
    (void)hipFree(d->d_grp); d->d_grp = nullptr;
    (void)hipFree(d->d_blkA); d->d_blkA = nullptr;
    (void)hipFree(d->d_blkB); d->d_blkB = nullptr;
    d->cap_units = d->cap_rh = d->cap_grp = d->cap_blk = d->cap_blkB = 0;
    d->n_entries = 0;
    d->rg = false;
    (void)hipFree(d->d_samp_st); d->d_samp_st = nullptr;
    (void)hipFree(d->d_st_end); d->d_st_end = nullptr;
    d->prg = false;
    d->n_streams = 0;
    d->pop_stride = 0;
    (void)hipFree(d->d_deep_tiles); d->d_deep_tiles = nullptr;
    (void)hipFree(d->d_deep_flag); d->d_deep_flag = nullptr;
    d->n_deep_tiles = 0;
    (void)hipFree(d->d_need); d->d_need = nullptr;
    d->pstage.release();
    for (auto& m : d->mslot) m.stage.release();
    (void)hipFree(d->d_mforced); d->d_mforced = nullptr;
    (void)hipFree(d->d_mforced_ctr); d->d_mforced_ctr = nullptr;
    d->n_mforced = -1;
    (void)hipFree(d->d_ppile); d->d_ppile = nullptr;
    (void)hipFree(d->d_prow); d->d_prow = nullptr;
    (void)hipFree(d->d_pboff); d->d_pboff = nullptr;
    d->n_samples = 0;
    d->n_reads = d->g_len = d->n_tiles = 0;
    d->cap_pile = d->cap_planes = d->cap_cneg = d->cap_ref = d->cap_tinfo = d->cap_wins = 0;
}

// a device buffer of at least `bytes` (kept when it is large enough; grown by a quarter otherwise)
template <class T>
static int ensure_dev(T** p, size_t* cap, size_t bytes, bool slack, std::string& err) {
    if (*p && *cap >= bytes) return 0;
    (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t want = slack ? bytes + bytes / 4 : bytes;
    HIP_TRY(hipMalloc(p, want));
    *cap = want;
    return 0;
}

void device_destroy(Device* d) {
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    // a fault of work no run waited for is reported here, against the context that launched it
    const hipError_t pending = hipDeviceSynchronize();
    if (pending != hipSuccess) std::fprintf(stderr, "[ngsep] device error pending at close: %s\n", hipGetErrorString(pending));
    device_release(d);
    (void)hipDeviceSynchronize();
    (void)hipFree(d->d_rac);
    if (d->h_rac) host_pinned_free(d->h_rac);
    for (auto& sl : d->slot) {
        (void)hipFree(sl.d_brec);
        (void)hipFree(sl.d_bcount);
        (void)hipFree(sl.d_hard);
        (void)hipFree(sl.d_hard2);
        (void)hipFree(sl.d_ctr);
        (void)hipFree(sl.d_cols);
        (void)hipFree(sl.d_tables);
        if (sl.stream && sl.stream != d->stream) (void)hipStreamDestroy(sl.stream);
        (void)hipFree(sl.d_sorted);
        (void)hipFree(sl.d_ext);
        host_pinned_free(sl.h_ctr);
        for (auto& e : sl.ev) (void)hipEventDestroy(e);
    }
    (void)hipFree(d->d_psites);
    (void)hipFree(d->d_pcalls);
    (void)hipFree(d->d_gcol);
    (void)hipFree(d->d_pcalls_ord);
    (void)hipFree(d->d_mforced);
    (void)hipFree(d->d_mforced_ctr);
    (void)hipFree(d->d_pbig);
    for (auto& m : d->mslot) {
        (void)hipFree(m.d_hard); (void)hipFree(m.d_need); (void)hipFree(m.d_psites); (void)hipFree(m.d_pcalls);
        if (m.h_psites) host_pinned_free(m.h_psites);
        (void)hipFree(m.d_pack); (void)hipFree(m.d_big);
        m.stage.release();
        for (auto& e : m.ev) if (e) (void)hipEventDestroy(e);
    }
    (void)hipFree(d->d_csrc);
    if (d->h_csrc) host_pinned_free(d->h_csrc);
    if (d->h_psites) host_pinned_free(d->h_psites);
    if (d->h_pcalls) host_pinned_free(d->h_pcalls);
    (void)hipFree(d->d_hard);
    (void)hipFree(d->d_counters);
    (void)hipFree(d->d_tables);
    (void)hipFree(d->d_pool);
    host_pinned_free(d->h_counters);
    for (int k = 0; k < 2; k++) {
        if (d->stage[k]) host_pinned_free(d->stage[k]);
        if (d->stage_ev[k]) (void)hipEventDestroy(d->stage_ev[k]);
    }
    for (auto& e : d->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(d->stream);
    (void)hipStreamDestroy(d->copy_stream);
    delete d;
}

// A streamed window's reference codes on the device (engine.cpp run_window_job): global position i in [lo, lo + len)
// gets t[the window's character i - lo] (engine.cpp ref_code as a 256-entry table), every other position 0 -- the
// host's fill_ref_codes; k_zero_ranges then clears the carved indel regions (one workgroup per {start, length} pair)
struct RefTable {
    uint8_t t[256];
};
__global__ __launch_bounds__(256) void k_ref_codes(const uint8_t* __restrict__ chars, int64_t lo, int64_t len, int64_t g_len,
                                                   const RefTable t, uint8_t* __restrict__ ref) {
    __shared__ uint8_t s_t[256];
    s_t[threadIdx.x] = t.t[threadIdx.x];
    __syncthreads();
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < g_len; i += (int64_t)gridDim.x * blockDim.x)
        ref[i] = (i >= lo && i < lo + len) ? s_t[chars[i - lo]] : (uint8_t)0;
}
__global__ __launch_bounds__(256) void k_zero_ranges(const int64_t* __restrict__ ranges, uint8_t* __restrict__ ref) {
    const int64_t a = ranges[2 * blockIdx.x], n = ranges[2 * blockIdx.x + 1];
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) ref[a + i] = 0;
}

// The read-group layout's units built on the device (streamed windows: engine.cpp build_rg_layout device_units) --
// one wavefront per 64-read group, lane = entry: unit k of the lane's read = its projected bytes 8k .. 8k+7 XOR-ed
// with the reference codes of the same positions, zero past the read's end (the host's fill_group_units, byte for
// byte).  Each lane walks its read and the reference with aligned 8-byte loads, the unaligned unit funnel-shifted
// from two of them (every load lies inside the read's bytes + 15 and the reference + 15: both buffers carry 64 bytes
// of slack); the stores of one k are one 512-byte line run per wave.
__global__ __launch_bounds__(256) void k_build_units(const uint8_t* __restrict__ rb, const int64_t* __restrict__ roff,
                                                     const int2* __restrict__ rh, const RGroup* __restrict__ grp,
                                                     const uint8_t* __restrict__ ref, int64_t n_groups,
                                                     uint64_t* __restrict__ units, uint64_t pad) {
    const int lane = threadIdx.x & 63;
    const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (g >= n_groups) return;
    const RGroup G = grp[g];
    const int64_t e = g * 64 + lane;
    const int2 h = rh[e];
    const int32_t gf = h.x, gl = h.y & 0x7FFFFFFF;
    const int64_t span = gl >= gf ? (int64_t)gl - gf + 1 : 0;
    uint64_t* out = units + G.base + lane;
    if (span == 0) {
        for (int32_t k = 0; k < G.K; k++) out[(int64_t)k * 64] = 0ull;
        return;
    }
    const uintptr_t sa = (uintptr_t)(rb + roff[e]), ra = (uintptr_t)(ref + gf);
    const uint64_t* sp = reinterpret_cast<const uint64_t*>(sa & ~(uintptr_t)7);
    const uint64_t* rp = reinterpret_cast<const uint64_t*>(ra & ~(uintptr_t)7);
    const uint32_t ss = 8u * (uint32_t)(sa & 7), rs = 8u * (uint32_t)(ra & 7);
    uint64_t s0 = sp[0], r0 = rp[0];
    for (int32_t k = 0; k < G.K; k++) {
        const int64_t o = 8 * (int64_t)k;
        uint64_t v = 0ull;
        if (o < span) {
            const uint64_t s1 = sp[k + 1], r1 = rp[k + 1];
            const uint64_t su = ss ? (s0 >> ss) | (s1 << (64u - ss)) : s0;
            const uint64_t ru = rs ? (r0 >> rs) | (r1 << (64u - rs)) : r0;
            v = su ^ ru;
            if (span - o < 8) {                          // past the read's last position: the layout's padding bytes
                const uint64_t m = (1ull << (8 * (span - o))) - 1ull;
                v = (v & m) | (pad & ~m);
            }
            s0 = s1;
            r0 = r1;
        }
        out[(int64_t)k * 64] = v;
    }
}

int device_upload(Device* d, const Staged& s, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    const int32_t pad = s.windows.empty() ? 64 : s.windows[0].pad;
    // single sample (a streamed window or a whole run): buffers kept across runs while large enough; the
    // multisample run starts from nothing
    const bool keep = s.single && d->d_ppile == nullptr && !d->prg;
    if (!keep) {
        // (a fault of earlier work is reported as such, not against this upload's copies)
        const hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) { err = std::string("device fault pending before the upload (earlier work): ") + hipGetErrorString(e); return -1; }
        device_release(d);
    }
    else HIP_TRY(hipDeviceSynchronize());          // the previous run is done reading them
    if (ensure_dev(&d->d_ref, &d->cap_ref, (size_t)s.g_len + 64, keep, err)) return -1;
    HIP_TRY(hipMemsetAsync(d->d_ref + s.g_len, 0, 64, d->stream));
    if (s.ref_on_device) {
        if (ensure_dev(&d->d_refchars, &d->cap_refchars, (size_t)std::max<int64_t>(s.ref_len, 1), keep, err)) return -1;
        if (s.ref_len) H2D(d->d_refchars, s.h_refchars, (size_t)s.ref_len, d->stream);
        RefTable t;
        std::memcpy(t.t, s.ref_table, 256);
        const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((s.g_len + 255) / 256, (int64_t)d->n_cu * 16));
        hipLaunchKernelGGL(k_ref_codes, dim3((unsigned)blocks), dim3(256), 0, d->stream, (const uint8_t*)d->d_refchars,
                           s.ref_lo, s.ref_len, s.g_len, t, d->d_ref);
        HIP_TRY(launch_check());
        const int64_t nz = (int64_t)s.h_zero.size() / 2;
        if (nz) {
            if (ensure_dev(&d->d_zero, &d->cap_zero, s.h_zero.size() * sizeof(int64_t), keep, err)) return -1;
            H2D(d->d_zero, s.h_zero.data(), s.h_zero.size() * sizeof(int64_t), d->stream);
            hipLaunchKernelGGL(k_zero_ranges, dim3((unsigned)nz), dim3(256), 0, d->stream, (const int64_t*)d->d_zero, d->d_ref);
            HIP_TRY(launch_check());
        }
    } else {
        H2D(d->d_ref, s.h_ref.data(), (size_t)s.g_len, d->stream);
    }
    d->rg = s.rg;
    if (s.rg) {
        // the read-group layout: units, entry headers, group table, block tables (KL, KG)
        const size_t nblk = (size_t)(s.g_len >> kRgBlockShift) + 2;
        if (ensure_dev(&d->d_units, &d->cap_units, (size_t)(s.n_units + kUnitSlack) * sizeof(uint64_t), keep, err) ||
            ensure_dev(&d->d_rh, &d->cap_rh, (size_t)std::max<int64_t>(s.n_entries, 64) * sizeof(int2), keep, err) ||
            ensure_dev(&d->d_grp, &d->cap_grp, (size_t)std::max<int64_t>(s.n_groups, 1) * sizeof(RGroup), keep, err) ||
            ensure_dev(&d->d_blkA, &d->cap_blk, nblk * sizeof(int32_t), keep, err) ||
            ensure_dev(&d->d_blkB, &d->cap_blkB, nblk * sizeof(int32_t), keep, err))
            return -1;
        if (s.units_on_device) {
            // the reads' bytes back to back and their entry offsets; k_build_units lays the units out below
            if (ensure_dev(&d->d_rbytes, &d->cap_rbytes, (size_t)s.n_rbytes + 64, keep, err) ||
                ensure_dev(&d->d_roff, &d->cap_roff, (size_t)(s.n_entries + 1) * sizeof(int64_t), keep, err))
                return -1;
            if (s.n_rbytes) {
                if (pinned_covers(s.h_units, (size_t)s.n_rbytes)) DMA(d->d_rbytes, s.h_units, (size_t)s.n_rbytes, 0, d->stream);
                else H2D(d->d_rbytes, s.h_units, (size_t)s.n_rbytes, d->stream);
            }
            H2D(d->d_roff, s.h_roff.data(), (size_t)(s.n_entries + 1) * sizeof(int64_t), d->stream);
        } else if (s.n_units) {
            // a pinned arena is copied directly; a pageable one (a layout beyond 4 GB) through the staging buffers
            if (pinned_covers(s.h_units, (size_t)s.n_units * sizeof(uint64_t))) DMA(d->d_units, s.h_units, (size_t)s.n_units * sizeof(uint64_t), 0, d->stream);
            else H2D(d->d_units, s.h_units, (size_t)s.n_units * sizeof(uint64_t), d->stream);
        }
        HIP_TRY(hipMemsetAsync(d->d_units + s.n_units, 0, kUnitSlack * sizeof(uint64_t), d->stream));
        if (s.n_entries) H2D(d->d_rh, s.h_rh.data(), (size_t)s.n_entries * sizeof(int2), d->stream);
        else {
            int32_t empty[128];
            for (int k = 0; k < 64; k++) { empty[2 * k] = 1; empty[2 * k + 1] = 0; }
            H2D(d->d_rh, empty, sizeof empty, d->stream);
        }
        if (s.n_groups) H2D(d->d_grp, s.h_grp.data(), (size_t)s.n_groups * sizeof(RGroup), d->stream);
        if (s.units_on_device && s.n_groups) {
            if (s.h_roff.size() != (size_t)s.n_entries + 1 || s.n_entries != s.n_groups * 64) {
                err = "internal error: device unit build without its entry offsets";
                return -1;
            }
            hipLaunchKernelGGL(k_build_units, dim3((unsigned)((s.n_groups + 3) / 4)), dim3(256), 0, d->stream,
                               (const uint8_t*)d->d_rbytes, (const int64_t*)d->d_roff, (const int2*)d->d_rh,
                               (const RGroup*)d->d_grp, (const uint8_t*)d->d_ref, s.n_groups, d->d_units, 0ull);
            HIP_TRY(launch_check());
        }
        H2D(d->d_blkA, s.h_blkA.data(), nblk * sizeof(int32_t), d->stream);
        H2D(d->d_blkB, s.h_blkB.data(), nblk * sizeof(int32_t), d->stream);
        d->n_entries = std::max<int64_t>(s.n_entries, 64);
    } else if (s.single) {
        if (ensure_dev(&d->d_pile, &d->cap_pile, (size_t)s.pile_bytes + 64, keep, err) ||      // + 64: KP loads whole dwords of a column
            ensure_dev(&d->d_tinfo, &d->cap_tinfo, (size_t)std::max<int64_t>(s.n_tiles, 1) * sizeof(TileInfo), keep, err))
            return -1;
        if (s.n_tiles && !s.h_tinfo.empty()) H2D(d->d_tinfo, s.h_tinfo.data(), (size_t)s.n_tiles * sizeof(TileInfo), d->stream);
        // single sample: planes (KT), the position-major pile and its strand bits (KP)
        const size_t ncw = (size_t)(s.pile_bytes / 32);
        if (ensure_dev(&d->d_planes, &d->cap_planes, (size_t)std::max<int64_t>(s.pile_bytes / 8, 16), keep, err) ||
            ensure_dev(&d->d_olist, &d->cap_olist, std::max<size_t>(s.h_olist.size(), 64) * sizeof(uint16_t), keep, err) ||
            ensure_dev(&d->d_loff, &d->cap_loff, std::max<size_t>(s.h_loff.size(), 2) * sizeof(int32_t), keep, err) ||
            ensure_dev(&d->d_cneg, &d->cap_cneg, (ncw + 4) * sizeof(uint32_t), keep, err))    // + 4: KP's strand-word window
            return -1;
        HIP_TRY(hipMemsetAsync(d->d_cneg + ncw, 0, 4 * sizeof(uint32_t), d->stream));
        if (s.pile_bytes) {
            // (the pinned arena is copied directly; H2D stages it should a registration have been refused)
            if (pinned_covers(s.h_cpile, (size_t)s.pile_bytes)) DMA(d->d_pile, s.h_cpile, (size_t)s.pile_bytes, 0, d->stream);
            else H2D(d->d_pile, s.h_cpile, (size_t)s.pile_bytes, d->stream);
            if (pinned_covers(s.h_planes, (size_t)(s.pile_bytes / 8))) DMA(d->d_planes, s.h_planes, (size_t)(s.pile_bytes / 8), 0, d->stream);
            else H2D(d->d_planes, s.h_planes, (size_t)(s.pile_bytes / 8), d->stream);
            if (pinned_covers(s.h_cneg, ncw * sizeof(uint32_t))) DMA(d->d_cneg, s.h_cneg, ncw * sizeof(uint32_t), 0, d->stream);
            else H2D(d->d_cneg, s.h_cneg, ncw * sizeof(uint32_t), d->stream);
        }
        if (!s.h_olist.empty()) H2D(d->d_olist, s.h_olist.data(), s.h_olist.size() * sizeof(uint16_t), d->stream);
        if (!s.h_loff.empty()) H2D(d->d_loff, s.h_loff.data(), s.h_loff.size() * sizeof(int32_t), d->stream);
        d->planes_W = s.tile / 32;
    } else {
        HIP_TRY(hipMalloc(&d->d_need, (size_t)(s.g_len / 32 + 1) * sizeof(uint32_t)));
        d->need_clean = false;
        if (s.prg) {
            // multisample: the population read-group layout (KLM scans it, KPM gathers its columns)
            const size_t nblk = (size_t)(s.pnblk * s.n_streams);
            // (+ kUnitSlack: KLM's unconditional next-batch loads may run past the last group)
            HIP_TRY(hipMalloc(&d->d_units, (size_t)(s.n_units + kUnitSlack) * sizeof(uint64_t)));
            HIP_TRY(hipMalloc(&d->d_rh, (size_t)std::max<int64_t>(s.n_entries, 64) * sizeof(int2)));
            HIP_TRY(hipMalloc(&d->d_grp, (size_t)std::max<int64_t>(s.n_groups, 1) * sizeof(RGroup)));
            HIP_TRY(hipMalloc(&d->d_blkA, std::max<size_t>(nblk, 1) * sizeof(int32_t)));
            HIP_TRY(hipMalloc(&d->d_blkB, std::max<size_t>(nblk, 1) * sizeof(int32_t)));
            HIP_TRY(hipMalloc(&d->d_samp_st, s.h_samp_st.size() * sizeof(int32_t)));
            HIP_TRY(hipMalloc(&d->d_st_end, std::max<size_t>(s.h_st_end.size(), 1) * sizeof(int64_t)));
            if (s.units_on_device) {
                // the reads' bytes and entry offsets; k_build_units lays the units out once the headers are there
                if (s.h_roff.size() != (size_t)s.n_entries + 1 || s.n_entries != s.n_groups * 64) {
                    err = "internal error: device unit build without its entry offsets";
                    return -1;
                }
                HIP_TRY(hipMalloc(&d->d_rbytes, (size_t)s.n_rbytes + 64));
                d->cap_rbytes = (size_t)s.n_rbytes + 64;
                HIP_TRY(hipMalloc(&d->d_roff, (size_t)(s.n_entries + 1) * sizeof(int64_t)));
                d->cap_roff = (size_t)(s.n_entries + 1) * sizeof(int64_t);
                int64_t at = 0;                            // the projection chunks, one after the other
                for (const auto& ch : s.h_chunks) {
                    H2D(d->d_rbytes + at, ch.first, (size_t)ch.second, d->stream);
                    at += ch.second;
                }
                H2D(d->d_roff, s.h_roff.data(), (size_t)(s.n_entries + 1) * sizeof(int64_t), d->stream);
            } else if (s.n_units) {
                if (pinned_covers(s.h_units, (size_t)s.n_units * sizeof(uint64_t))) DMA(d->d_units, s.h_units, (size_t)s.n_units * sizeof(uint64_t), 0, d->stream);
                else H2D(d->d_units, s.h_units, (size_t)s.n_units * sizeof(uint64_t), d->stream);
            }
            HIP_TRY(hipMemsetAsync(d->d_units + s.n_units, 0, kUnitSlack * sizeof(uint64_t), d->stream));
            if (s.n_entries) H2D(d->d_rh, s.h_rh.data(), (size_t)s.n_entries * sizeof(int2), d->stream);
            if (s.n_groups) H2D(d->d_grp, s.h_grp.data(), (size_t)s.n_groups * sizeof(RGroup), d->stream);
            if (s.units_on_device && s.n_groups) {
                hipLaunchKernelGGL(k_build_units, dim3((unsigned)((s.n_groups + 3) / 4)), dim3(256), 0, d->stream,
                                   (const uint8_t*)d->d_rbytes, (const int64_t*)d->d_roff, (const int2*)d->d_rh,
                                   (const RGroup*)d->d_grp, (const uint8_t*)d->d_ref, s.n_groups, d->d_units,
                                   kPopPadUnit);
                HIP_TRY(launch_check());
                // (the bytes are not needed past the build: released once it is done)
                HIP_TRY(hipStreamSynchronize(d->stream));
                (void)hipFree(d->d_rbytes); d->d_rbytes = nullptr;
                (void)hipFree(d->d_roff); d->d_roff = nullptr;
                d->cap_rbytes = d->cap_roff = 0;
            }
            if (nblk) {
                H2D(d->d_blkA, s.h_blkA.data(), nblk * sizeof(int32_t), d->stream);
                H2D(d->d_blkB, s.h_blkB.data(), nblk * sizeof(int32_t), d->stream);
            }
            H2D(d->d_samp_st, s.h_samp_st.data(), s.h_samp_st.size() * sizeof(int32_t), d->stream);
            if (!s.h_st_end.empty()) H2D(d->d_st_end, s.h_st_end.data(), s.h_st_end.size() * sizeof(int64_t), d->stream);
            d->n_entries = s.n_entries;
            d->prg = true;
            d->n_streams = s.n_streams;
            d->pblk_shift = s.pblk_shift;
            d->pnblk = s.pnblk;
            d->pop_stride = std::max<int32_t>(s.max_cov, 1);
            d->n_deep_tiles = (int64_t)s.h_deep_tiles.size();
            if (d->n_deep_tiles) {
                const int64_t ntile = s.g_len / kKlmTile;
                std::vector<uint8_t> flag((size_t)ntile, 0);
                for (int32_t t : s.h_deep_tiles) flag[(size_t)t] = 1;
                HIP_TRY(hipMalloc(&d->d_deep_tiles, (size_t)d->n_deep_tiles * sizeof(int32_t)));
                HIP_TRY(hipMalloc(&d->d_deep_flag, (size_t)ntile));
                H2D(d->d_deep_tiles, s.h_deep_tiles.data(), (size_t)d->n_deep_tiles * sizeof(int32_t), d->stream);
                H2D(d->d_deep_flag, flag.data(), (size_t)ntile, d->stream);
            }
        } else {
            // the realigner's region positions: a site-major pile (KPM)
            HIP_TRY(hipMalloc(&d->d_ppile, (size_t)s.ppile_bytes + 64));
            HIP_TRY(hipMalloc(&d->d_prow, std::max<size_t>(s.h_prow.size(), 1) * sizeof(int32_t)));
            HIP_TRY(hipMalloc(&d->d_pboff, std::max<size_t>(s.h_pboff.size(), 1) * sizeof(int64_t)));
            H2D(d->d_ppile, s.h_ppile.get(), (size_t)s.ppile_bytes + 64, d->stream);
            if (!s.h_prow.empty()) H2D(d->d_prow, s.h_prow.data(), s.h_prow.size() * sizeof(int32_t), d->stream);
            if (!s.h_pboff.empty()) H2D(d->d_pboff, s.h_pboff.data(), s.h_pboff.size() * sizeof(int64_t), d->stream);
        }
        if (s.known) {
            // -knownVariants: the input variants at covered positions are KPM's whole queue (no scan)
            const int64_t nf = (int64_t)s.h_forced.size() / 2;
            unsigned long long hc[8] = {0, 0, (unsigned long long)nf, 0, 0, 0, 0, 0};
            HIP_TRY(hipMalloc(&d->d_mforced, (size_t)std::max<int64_t>(nf, 1) * sizeof(QueueSite)));
            HIP_TRY(hipMalloc(&d->d_mforced_ctr, 8 * sizeof(unsigned long long)));
            if (nf) H2D(d->d_mforced, s.h_forced.data(), (size_t)nf * sizeof(QueueSite), d->stream);
            H2D(d->d_mforced_ctr, hc, sizeof hc, d->stream);
            d->n_mforced = nf;
        }
        HIP_TRY(hipStreamSynchronize(d->stream));       // the host layout is freed after the upload
        d->n_samples = s.n_samples;
    }
    d->n_reads = s.n_reads;
    d->g_len = s.g_len;
    d->max_span = s.max_span;
    d->pad = pad;
    d->tile = s.tile;
    d->log2_tile = 0;
    while ((1 << d->log2_tile) < s.tile) d->log2_tile++;
    d->n_tiles = s.n_tiles;
    {
        std::vector<int4> wins;
        for (const Window& w : s.windows) wins.push_back(int4{(int)(w.gbase + w.pad), w.w0, w.seq_id, w.wlen});
        if (wins.empty()) wins.push_back(int4{0, 0, -1, 0});
        if (ensure_dev(&d->d_wins, &d->cap_wins, wins.size() * sizeof(int4), false, err)) return -1;
        H2D(d->d_wins, wins.data(), wins.size() * sizeof(int4), d->stream);
        HIP_TRY(hipStreamSynchronize(d->stream));
        d->n_wins = (int32_t)wins.size();
    }
    HIP_TRY(hipStreamSynchronize(d->stream));
    return 0;
}

// ------------------------------------------------------------------------------------------
// single-sample runs: submit (kernels + D2H enqueued) and collect (wait, finish) so that a run's
// copies and host post-processing overlap the next run's kernels.  Two result slots; slot s owns
// its ordered-record buffer, its counter set and a pinned host store.  Compute stream: [wait slot
// free] KT KP KO; copy stream: [wait KO] D2H counters + records, clear the counter set.
// ------------------------------------------------------------------------------------------
static int grow_slot(Device* d, RunSlot& sl, int64_t sites, int64_t queue, std::string& err, int64_t cols = 0) {
    if (sites > d->cap_sites) d->cap_sites = sites;     // the slots' ordered-record buffers follow
    if (queue > sl.cap_hard) {
        (void)hipFree(sl.d_hard);
        (void)hipFree(sl.d_hard2);
        sl.d_hard = sl.d_hard2 = nullptr;
        HIP_TRY(hipMalloc(&sl.d_hard, (size_t)queue * sizeof(SiteQ)));
        HIP_TRY(hipMalloc(&sl.d_hard2, (size_t)queue * sizeof(SiteQ)));
        sl.cap_hard = queue;
    }
    if (cols > sl.cap_cols) {                            // + 64 entries: KP's dword window reads past a column
        (void)hipFree(sl.d_cols);
        sl.d_cols = nullptr;
        HIP_TRY(hipMalloc(&sl.d_cols, (size_t)(cols + 64) * sizeof(uint16_t)));
        HIP_TRY(hipMemset(sl.d_cols, 0, (size_t)(cols + 64) * sizeof(uint16_t)));
        sl.cap_cols = cols;
    }
    return 0;
}

// enqueues one run into slot sl (kernels on the compute stream, copies on the copy stream)
static int enqueue_run(Device* d, RunSlot& sl, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune,
                       bool idle, std::string& err) {
    // capacities (shared buffers only change while nothing runs): calls are rare; dump mode needs one
    // record per covered position
    const int64_t nforced = (int64_t)s.h_forced.size() / 4;     // -knownVariants: the sites to genotype (SiteQ)
    int64_t want = g.dump_all ? std::max<int64_t>(s.covered + 1024, 1024) : std::max<int64_t>(s.g_len / 256 + 4096, 4096);
    int64_t qwant = (g.dump_all || !prune) ? s.g_len + 1024 : std::max<int64_t>(s.g_len / 64 + 65536, 65536);
    want = std::max<int64_t>(want, nforced + 1024);
    qwant = std::max<int64_t>(qwant, nforced + 1024);
    // the queued sites' columns (u16 entries): the survivors are ~1 in 1000 positions at 30x; every covered
    // position in dump mode (the read bases bound it); grown when a run overflows
    int64_t cwant = std::max<int64_t>(std::max<int64_t>(1 << 20, s.g_len / 16), d->last_cols + d->last_cols / 4);
    if (g.dump_all || !prune) cwant = std::max<int64_t>(cwant, s.n_read_bases + 4 * s.g_len);
    cwant = std::max<int64_t>(cwant, (int64_t)s.h_cols.size() + 1024);         // the realigner regions' columns
    if (want > d->cap_sites || qwant > sl.cap_hard || cwant > sl.cap_cols) {
        if (!idle) HIP_TRY(hipStreamSynchronize(sl.stream));
        if (grow_slot(d, sl, want, qwant, err, cwant) != 0) return -1;
    }
    if (sl.cap < d->cap_sites) {
        HIP_TRY(hipEventSynchronize(sl.ev[4]));
        (void)hipFree(sl.d_sorted);
        sl.d_sorted = nullptr;
        HIP_TRY(hipMalloc(&sl.d_sorted, (size_t)d->cap_sites * sizeof(SiteRec)));
        sl.cap = d->cap_sites;
    }
    // whole records: every record in dump mode / with full_records, else the rare multi-allelic and pool calls
    const int64_t ewant = g.full_records ? d->cap_sites : std::max<int64_t>(4096, d->cap_sites / 64);
    if (ewant > sl.cap_ext) {
        HIP_TRY(hipEventSynchronize(sl.ev[4]));
        if (!idle) HIP_TRY(hipStreamSynchronize(sl.stream));
        (void)hipFree(sl.d_ext);
        sl.d_ext = nullptr;
        HIP_TRY(hipMalloc(&sl.d_ext, (size_t)ewant * sizeof(ngsep_site_out)));
        sl.cap_ext = ewant;
    }
    // position buckets of the ordering pass: a few records each (dump mode: 16 positions, so 16
    // records at most; calls: 4096 positions and room for 64, grown when a run overflows)
    const int shift = g.dump_all ? 4 : d->ko_shift;
    const int32_t bcap = g.dump_all ? 16 : d->ko_bcap;
    const int64_t nb = (s.g_len >> shift) + 1;
    if (nb > sl.nb_cap || nb * bcap > sl.brec_cap) {
        if (!idle) HIP_TRY(hipStreamSynchronize(sl.stream));
        if (nb > sl.nb_cap) {
            (void)hipFree(sl.d_bcount);
            sl.d_bcount = nullptr;
            HIP_TRY(hipMalloc(&sl.d_bcount, (size_t)nb * sizeof(int32_t)));
            sl.nb_cap = nb;
        }
        if (nb * bcap > sl.brec_cap) {
            (void)hipFree(sl.d_brec);
            sl.d_brec = nullptr;
            HIP_TRY(hipMalloc(&sl.d_brec, (size_t)(nb * bcap) * sizeof(SiteRec)));
            sl.brec_cap = nb * bcap;
        }
    }
    unsigned long long* ctr = sl.d_ctr;
    sl.t0 = std::chrono::steady_clock::now();
    // the slot's previous copies (and the reset of its counter set) are done before it is reused
    if (hipEventQuery(sl.ev[4]) != hipSuccess) HIP_TRY(hipStreamWaitEvent(sl.stream, sl.ev[4], 0));
    if (!sl.tables_valid || std::memcmp(&sl.h_tables, &t, sizeof(LikTables)) != 0) {
        HIP_TRY(hipStreamSynchronize(sl.stream));     // the previous upload may still read h_tables
        sl.h_tables = t;
        H2D(sl.d_tables, &sl.h_tables, sizeof(LikTables), sl.stream);
        sl.tables_valid = true;
    }
    // KT is timed by events bound to its dispatch (hipExtLaunchKernelGGL): the kernel's own start and end
    hipEvent_t k0 = d->time_scan ? sl.ev[0] : nullptr, k1 = d->time_scan ? sl.ev[1] : nullptr;
    if (!d->rg) { err = "no read-group layout resident"; return -1; }
    int64_t kg_sites = 0;                                        // KG's sites (estimate)
    bool kl_run = false;                                         // KL's sharded queue (else one segment, count at [2])
    sl.scan_timed = false;
    if (s.known) {
        // -knownVariants: no scan, the input variants' sites (covered, in window order) are KP's queue
        if (nforced > 0) H2D(sl.d_hard, s.h_forced.data(), (size_t)nforced * sizeof(SiteQ), sl.stream);
        if (!s.h_cols.empty())                                   // entries with their columns (realigner regions)
            H2D(sl.d_cols, s.h_cols.data(), s.h_cols.size() * sizeof(uint16_t), sl.stream);
        H2D(ctr, s.h_forced_ctr, 8 * sizeof(unsigned long long), sl.stream);
        hipLaunchKernelGGL(k_zero_i32, dim3((unsigned)std::min<int64_t>((nb + 255) / 256, 4096)), dim3(256), 0, sl.stream, sl.d_bcount, nb);
        HIP_TRY(launch_check());
        d->last_hard = nforced;
        kg_sites = nforced;
    } else if (d->n_tiles > 0 && prune) {
        // KL: one workgroup per tile of kKlTile positions, straight from the read-group layout
        // (measured on chr20 30x: 2048-position tiles beat 4096; batches of 8 unpipelined beat 16 and 24; batches
        // of 4 pipelined at 8 waves per SIMD beat 8 unpipelined by 2 %, tools/gpu_r4_abn.sh)
        hipExtLaunchKernelGGL(k_read_scan<kKlTile, kKlUnroll>, dim3((unsigned)(s.g_len / kKlTile)), dim3(kKlThreads), 0, sl.stream, k0, k1, 0,
                              (const uint64_t*)d->d_units, (const int2*)d->d_rh, (const RGroup*)d->d_grp, (const int32_t*)d->d_blkA,
                              (const int32_t*)d->d_blkB, d->n_entries, (const uint8_t*)d->d_ref, (const LikTables*)sl.d_tables, g,
                              sl.d_hard, ctr, sl.cap_hard / kKlShards, (sl.cap_cols >> 2) / kKlShards, sl.d_bcount, nb);
        HIP_TRY(launch_check());
        sl.scan_timed = k0 != nullptr;
        kg_sites = d->last_hard + d->last_hard / 8;              // KL's survivors (sized from the previous run)
        kl_run = true;
    } else {
        // dump mode / no pruning: every in-window position goes to KP
        const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>((s.g_len + 255) / 256, (int64_t)d->n_cu * 8));
        hipExtLaunchKernelGGL(k_queue_all, dim3((unsigned)nblk), dim3(256), 0, sl.stream, k0, k1, 0, (const uint8_t*)d->d_ref,
                              s.g_len, sl.d_hard, ctr, sl.cap_hard, sl.d_bcount, nb);
        HIP_TRY(launch_check());
        sl.scan_timed = k0 != nullptr;
        kg_sites = s.g_len;
    }
    {
        // KG: the queued sites' columns, one wave per site (grid-stride past the estimate)
        const int64_t nblk = std::max<int64_t>(d->n_cu, std::min<int64_t>((kg_sites + 3) / 4, (int64_t)d->n_cu * 32));
        static const int kg_env = diag_env("NGSEP_KG_SITES") ? std::atoi(diag_env("NGSEP_KG_SITES")) : 4;   // tuning
        const int kgs = kg_env == 8 ? 8 : kg_env == 2 ? 2 : 4;
        if (kl_run)
            hipLaunchKernelGGL(kgs == 8 ? k_gather_kl<8> : kgs == 2 ? k_gather_kl<2> : k_gather_kl<4>,
                               dim3((unsigned)std::max<int64_t>(d->n_cu, std::min<int64_t>((kg_sites + 4 * kgs - 1) / (4 * kgs), (int64_t)d->n_cu * 32))),
                               dim3(256), 0, sl.stream, (const SiteQ*)sl.d_hard, (const unsigned long long*)(ctr + kCtrShard0), kCtrShardStride,
                               kKlShards, sl.cap_hard / kKlShards, sl.d_hard2, (const int2*)d->d_rh, (const RGroup*)d->d_grp,
                               (const uint64_t*)d->d_units, (const int32_t*)d->d_blkA, (const uint8_t*)d->d_ref, d->n_entries, sl.d_cols, ctr);
        else
        hipLaunchKernelGGL(k_gather_cols, dim3((unsigned)nblk), dim3(256), 0, sl.stream, (const SiteQ*)sl.d_hard,
                           (const unsigned long long*)(kl_run ? ctr + kCtrShard0 : ctr + 2), kl_run ? kCtrShardStride : 1,
                           kl_run ? kKlShards : 1, kl_run ? sl.cap_hard / kKlShards : sl.cap_hard, sl.d_hard2,
                           (const int2*)d->d_rh, (const RGroup*)d->d_grp,
                           (const uint64_t*)d->d_units, (const int32_t*)d->d_blkA, (const uint8_t*)d->d_ref, d->n_entries, sl.d_cols,
                           sl.cap_cols, ctr);
        HIP_TRY(launch_check());
    }
    // one lane per queued site: enough workgroups for the queue (the count is on the device; sized from the
    // previous run's survivors, grid-stride beyond)
    static const int kp_env = diag_env("NGSEP_KP_GRID") ? std::max(1, std::atoi(diag_env("NGSEP_KP_GRID"))) : 0;   // tuning
    const int kp_grid = kp_env ? kp_env : (int)std::max<int64_t>(d->n_cu, std::min<int64_t>((d->last_hard + kPostThreads - 1) / kPostThreads, 8 * (int64_t)d->n_cu));
    if (g.ploidy >= 3 && !g.dump_all) {
        if (!d->pool_valid) { err = "ploidy >= 3 without pool tables (device_set_pool)"; return -1; }
        hipExtLaunchKernelGGL(k_posterior_pool, dim3(kp_grid), dim3(kPostThreads), 0, sl.stream,
                              d->time_posterior ? sl.ev[5] : nullptr, d->time_posterior ? sl.ev[2] : nullptr, 0,
                              (const SiteQ*)sl.d_hard2, (const unsigned long long*)(ctr + 2), sl.cap_hard, (const uint16_t*)sl.d_cols,
                              (const PoolTables*)d->d_pool, g, sl.d_brec, sl.d_bcount, shift, bcap, sl.d_ext, ctr + 4, sl.cap_ext);
    } else {
        hipExtLaunchKernelGGL(k_posterior, dim3(kp_grid), dim3(kPostThreads), 0, sl.stream,
                              d->time_posterior ? sl.ev[5] : nullptr, d->time_posterior ? sl.ev[2] : nullptr, 0,
                              (const SiteQ*)sl.d_hard2, (const unsigned long long*)(ctr + 2), sl.cap_hard, (const uint16_t*)sl.d_cols,
                              (const LikTables*)sl.d_tables, g, sl.d_brec, sl.d_bcount, shift, bcap, sl.d_ext, ctr + 4, sl.cap_ext);
    }
    HIP_TRY(launch_check());
    // order the records by position on the device (one kernel; counters[0] = records | max bucket << 40)
    hipLaunchKernelGGL(ko_fused, dim3((unsigned)((nb + kKofBuckets - 1) / kKofBuckets)), dim3(64 * kKofBuckets), 0, sl.stream, sl.d_brec,
                       (const int32_t*)sl.d_bcount, nb, bcap, ctr, sl.d_sorted, sl.cap, d->d_wins, d->n_wins, 1 << shift);
    HIP_TRY(launch_check());
    // copies: counters and a prefix of the ordered records (sized from the previous run) straight into
    // the slot's pinned store, then the counter set is cleared for the slot's next run.  On the copy
    // stream (ordered after KO by ev[3]) or, with NGSEP_COPY_ON_COMPUTE=1, on the compute stream
    static const bool on_compute = diag_env("NGSEP_COPY_ON_COMPUTE") != nullptr;   // diagnostics
    hipStream_t cs = on_compute ? sl.stream : d->copy_stream;
    if (!on_compute) HIP_TRY(hipEventRecord(sl.ev[3], sl.stream));
    sl.guess = std::min<int64_t>(d->cap_sites, d->last_n_sites + d->last_n_sites / 64 + 64);
    sl.guess_ext = std::min<int64_t>(sl.cap_ext, d->last_n_ext + d->last_n_ext / 64 + 16);
    sl.host.rec.reserve((size_t)sl.guess);
    sl.host.ext.reserve((size_t)sl.guess_ext);
    if (!on_compute) HIP_TRY(hipStreamWaitEvent(cs, sl.ev[3], 0));
    DMA(sl.h_ctr, ctr, kCtrWords * sizeof(unsigned long long), 1, cs);
    DMA(sl.host.rec.buf, sl.d_sorted, (size_t)sl.guess * sizeof(SiteRec), 1, cs);
    if (sl.guess_ext > 0)
        DMA(sl.host.ext.buf, sl.d_ext, (size_t)sl.guess_ext * sizeof(ngsep_site_out), 1, cs);
    HIP_TRY(hipMemsetAsync(ctr, 0, kCtrWords * sizeof(unsigned long long), cs));
    HIP_TRY(hipEventRecord(sl.ev[4], cs));
    sl.g = g;
    sl.prune = prune;
    sl.tabs = t;
    sl.staged = &s;
    return 0;
}

// the pool algorithm's tables (ploidy >= 3): uploaded when they change, after the runs that read the old ones
int device_set_pool(Device* d, const PoolTables* pt, std::string& err) {
    if (!pt) return 0;
    if (d->pool_valid && std::memcmp(&d->h_pool, pt, sizeof(PoolTables)) == 0) return 0;
    HIP_TRY(hipSetDevice(d->ordinal));
    HIP_TRY(hipDeviceSynchronize());
    if (!d->d_pool) HIP_TRY(hipMalloc(&d->d_pool, sizeof(PoolTables)));
    H2D(d->d_pool, pt, sizeof(PoolTables), d->stream);
    HIP_TRY(hipStreamSynchronize(d->stream));
    d->h_pool = *pt;
    d->pool_valid = true;
    return 0;
}

int device_submit(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    RunSlot& sl = d->slot[d->n_submitted % 2];
    if (sl.busy) { err = "both result slots hold uncollected runs"; return -1; }
    if (enqueue_run(d, sl, s, t, g, prune, d->n_submitted == d->n_collected, err) != 0) return -1;
    sl.busy = true;
    d->n_submitted++;
    return 0;
}

// waits for the oldest submitted run and moves its position-ordered records into out (appended at
// out->size(); swapped in when out is empty).  Returns 1 when the run overflowed a buffer: the
// buffers have been grown and the caller runs it again.
int device_collect(Device* d, SiteStore* out, int64_t* n_out, double* scan_ms, double* geno_ms, double* total_ms,
                   int64_t* n_candidates, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    if (d->n_collected == d->n_submitted) { err = "no run to collect"; return -1; }
    RunSlot& sl = d->slot[d->n_collected % 2];
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto h0 = std::chrono::steady_clock::now();
    HIP_TRY(hipEventSynchronize(sl.ev[4]));
    if (host_timing) {
        static double acc = 0;
        static int cnt = 0;
        acc += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
        if (++cnt == 20) { std::fprintf(stderr, "[ngsep host] event wait %.1f us\n", acc / 20); acc = 0; cnt = 0; }
    }
    constexpr unsigned long long kNMask = (1ull << 40) - 1;
    int64_t n, mx, q, ne, nc, ncand;
    bool qfull, cfull;
    auto read_ctr = [&]() {
        const unsigned long long* h = sl.h_ctr;
        n = (int64_t)(h[0] & kNMask);
        mx = (int64_t)(h[0] >> 40);                      // fullest position bucket
        ne = (int64_t)h[4];
        // KL's shards (the queue and column segments of cap / kKlShards each), then KG's reservations
        int64_t qs = 0, qmax = 0, cs4 = 0, cmax4 = 0;
        ncand = (int64_t)h[1];
        for (int t = 0; t < kKlShards; t++) {
            const unsigned long long* c = h + kCtrShard0 + kCtrShardStride * t;
            qs += (int64_t)c[0];
            qmax = std::max<int64_t>(qmax, (int64_t)c[0]);
            cs4 += (int64_t)c[1];
            cmax4 = std::max<int64_t>(cmax4, (int64_t)c[1]);
            ncand += (int64_t)c[2];
        }
        q = qs > 0 ? qs : (int64_t)h[2];
        nc = (cs4 + (int64_t)h[5]) * 4;                  // column entries reserved
        qfull = q > sl.cap_hard || qmax > sl.cap_hard / kKlShards;
        cfull = (int64_t)h[5] * 4 > sl.cap_cols || cmax4 > (sl.cap_cols >> 2) / kKlShards;
        if (qs > 0) {                                    // sized for the fullest shard
            q = std::max<int64_t>(q, qmax * kKlShards);
            nc = std::max<int64_t>(nc, cmax4 * 4 * kKlShards);
        }
    };
    read_ctr();
    for (int attempt = 0; n > d->cap_sites || qfull || ne > sl.cap_ext || cfull ||
                          (!sl.g.dump_all && mx > d->ko_bcap); attempt++) {
        // more calls or undecided candidates than the buffers hold (e.g. -minQuality 0): drain, grow
        // and run this slot again in place (a later run in the other slot keeps its own results)
        if (attempt == 3) { err = "result buffers kept overflowing"; return -1; }
        HIP_TRY(hipDeviceSynchronize());
        if (grow_slot(d, sl, std::max(d->cap_sites, n + 1024), qfull ? std::max(sl.cap_hard, q + q / 4 + 1024) : sl.cap_hard, err,
                      cfull ? std::max(sl.cap_cols, nc + nc / 4 + 1024) : sl.cap_cols) != 0) return -1;
        if (ne > sl.cap_ext) {
            (void)hipFree(sl.d_ext);
            sl.d_ext = nullptr;
            HIP_TRY(hipMalloc(&sl.d_ext, (size_t)(ne + 1024) * sizeof(ngsep_site_out)));
            sl.cap_ext = ne + 1024;
        }
        if (!sl.g.dump_all && mx > d->ko_bcap) {
            // crowded buckets (e.g. -minQuality 0 calls most positions): room for the fullest one, up to
            // the 1024 keys a KO wave ranks; past that, 16-position buckets that cannot overflow
            if (mx <= 1024) while (d->ko_bcap < mx) d->ko_bcap *= 2;
            else { d->ko_shift = 4; d->ko_bcap = 16; }
        }
        d->last_n_sites = n;
        if (enqueue_run(d, sl, *sl.staged, sl.tabs, sl.g, sl.prune, true, err) != 0) return -1;
        HIP_TRY(hipEventSynchronize(sl.ev[4]));
        read_ctr();
    }
    d->last_cols = nc;
    sl.busy = false;
    d->n_collected++;
    if (n > sl.guess) {
        sl.host.rec.n = (size_t)sl.guess;             // keep the records already copied when the store grows
        sl.host.rec.reserve((size_t)n);
        DMA_SYNC(sl.host.rec.buf + sl.guess, sl.d_sorted + sl.guess, (size_t)(n - sl.guess) * sizeof(SiteRec), 1);
    }
    if (ne > sl.guess_ext) {
        sl.host.ext.n = (size_t)sl.guess_ext;
        sl.host.ext.reserve((size_t)ne);
        DMA_SYNC(sl.host.ext.buf + sl.guess_ext, sl.d_ext + sl.guess_ext, (size_t)(ne - sl.guess_ext) * sizeof(ngsep_site_out), 1);
    }
    sl.host.rec.n = (size_t)n;
    sl.host.ext.n = (size_t)ne;
    d->last_n_sites = n;
    d->last_n_ext = ne;
    if (out->size() == 0) out->swap(sl.host);
    else out->append(sl.host);
    sl.host.clear();
    *n_out = n;
    float a = 0, a2 = 0;
    // (only events this run recorded: a -knownVariants run has no scan, and the elapsed time of events never recorded
    // is an error the next launch check would report)
    if (d->time_scan && sl.scan_timed) (void)hipEventElapsedTime(&a, sl.ev[0], sl.ev[1]);
    if (d->time_posterior) (void)hipEventElapsedTime(&a2, sl.ev[5], sl.ev[2]);
    *scan_ms = a;
    *geno_ms = a2;
    *total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - sl.t0).count();
    *n_candidates = ncand;
    d->last_hard = (int64_t)sl.h_ctr[2];
    d->last_exact = (int64_t)sl.h_ctr[3];
    return 0;
}

int64_t device_inflight(const Device* d) { return d ? d->n_submitted - d->n_collected : 0; }

int device_run(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune,
               SiteStore* out, int64_t* n_out, double* scan_ms, double* geno_ms, double* total_ms,
               int64_t* n_candidates, std::string& err) {
    while (d->n_collected < d->n_submitted) {        // finish anything asynchronous first (results dropped)
        SiteStore drop;
        int64_t nn = 0; double a = 0, b = 0, c2 = 0; int64_t nc = 0;
        if (device_collect(d, &drop, &nn, &a, &b, &c2, &nc, err) != 0) return -1;
    }
    if (device_submit(d, s, t, g, prune, err) != 0) return -1;
    return device_collect(d, out, n_out, scan_ms, geno_ms, total_ms, n_candidates, err);
}

// ------------------------------------------------------------------------------------------
// KR: RelativeAlleleCountsCalculator.onPileup (discovery/RelativeAlleleCountsCalculator.java:246-294) over
// every position of the run's window -- one lane per position, its column of the position-major byte pile
// (the rows of the reads covering it, rank order).  A nonzero code is an allele call of getAlleleCalls(1);
// a call of quality >= minBaseQualityScore counts for its base (A, C, G, T from a valid code, any other
// character as 'N' from a counted one: min_bq is in [4, 30], so the code's clamped quality decides it and
// q <= 3 calls, whose base the code drops, never count).  Positions with >= minRD calls and >= 1 counted
// allele add their number of alleles and the proportion of the second most frequent allele (TreeMap order
// A < C < G < N < T, strict maxima) to the histograms of math.Distribution (bins (int)((v - min) / len)).
// The proportion's sums are kept per block in grid-stride order (the host adds the blocks in order).
// ------------------------------------------------------------------------------------------
constexpr int kRacThreads = 256;
constexpr int kRacBlocks = 1024;
constexpr int kRacPropBins = 51, kRacNallBins = 10;
__global__ __launch_bounds__(kRacThreads) void k_rac(const uint8_t* __restrict__ cpile, const TileInfo* __restrict__ tinfo,
                                                     int32_t log2T, int64_t g0, int64_t g1, int32_t min_rd, int32_t min_bq,
                                                     unsigned long long* __restrict__ hist, double* __restrict__ part) {
    __shared__ uint32_t s_h[kRacPropBins + kRacNallBins];
    __shared__ double s_sum[kRacThreads], s_sq[kRacThreads];
    for (int i = threadIdx.x; i < kRacPropBins + kRacNallBins; i += kRacThreads) s_h[i] = 0;
    __syncthreads();
    const int32_t Tm = (1 << log2T) - 1;
    double sum = 0, sq = 0;
    for (int64_t g = g0 + (int64_t)blockIdx.x * kRacThreads + threadIdx.x; g < g1; g += (int64_t)gridDim.x * kRacThreads) {
        const TileInfo ti = tinfo[g >> log2T];
        const int32_t rows = ti.rows;
        if (rows == 0) continue;
        const int64_t base = ti.off + (int64_t)(g & Tm) * rows;
        const int64_t c0 = base & ~(int64_t)3;
        const uint32_t* cw = reinterpret_cast<const uint32_t*>(cpile) + (c0 >> 2);
        const int sh = (int)(base - c0);
        const int nd = (rows + sh + 3) >> 2;
        int32_t calls = 0, cA = 0, cC = 0, cG = 0, cT = 0, cN = 0;
        for (int k = 0; k < nd; k++) {
            const uint32_t d = cw[k];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const int r = 4 * k + e - sh;
                const uint32_t cd = (r >= 0 && r < rows) ? (d >> (8 * e)) & 0xFFu : 0u;
                if (cd == 0) continue;
                calls++;
                if ((int32_t)(cd & 31u) < min_bq) continue;
                if (cd & 0x80u) {
                    const uint32_t a = (cd >> 5) & 3u;
                    cA += a == 0; cC += a == 1; cG += a == 2; cT += a == 3;
                } else {
                    cN++;
                }
            }
        }
        if (calls < min_rd) continue;
        const int32_t c[5] = {cA, cC, cG, cN, cT};      // TreeMap<String> order
        int32_t nz = 0, mx = -1, mc = -1;
#pragma unroll
        for (int k = 0; k < 5; k++) {
            nz += c[k] > 0;
            if (c[k] > 0 && (mx < 0 || mc < c[k])) { mx = k; mc = c[k]; }
        }
        if (nz == 0) continue;
        atomicAdd(&s_h[kRacPropBins + (int)((double)(nz - 1) / 1.0)], 1u);
        int32_t s2 = -1, sc = 0;
#pragma unroll
        for (int k = 0; k < 5; k++)
            if (k != mx && c[k] > 0 && (s2 < 0 || sc < c[k])) { s2 = k; sc = c[k]; }
        const double prop = (double)sc / (double)(mc + sc);
        atomicAdd(&s_h[(int)((prop - 0.0) / 0.01)], 1u);
        sum += prop;
        sq += prop * prop;
    }
    s_sum[threadIdx.x] = sum;
    s_sq[threadIdx.x] = sq;
    __syncthreads();
    if (threadIdx.x == 0) {                          // the block's partial sums in thread order
        double a = 0, b = 0;
        for (int i = 0; i < kRacThreads; i++) { a += s_sum[i]; b += s_sq[i]; }
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
    for (int i = threadIdx.x; i < kRacPropBins + kRacNallBins; i += kRacThreads)
        if (s_h[i]) atomicAdd(&hist[i], (unsigned long long)s_h[i]);
}

// one RelativeAlleleCounts pass over positions [g0, g1) of the resident single-sample layout: the 51 + 10
// histogram counts, the proportion's sum and sum of squares (blocks added in order)
int device_run_rac(Device* d, const Staged& s, int64_t g0, int64_t g1, int32_t min_rd, int32_t min_bq,
                   unsigned long long* hist_out, double* sum, double* sum_sq, double* kernel_ms, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    if (!s.single || !d->d_pile || !d->d_tinfo) { err = "no single-sample layout resident"; return -1; }
    if (g0 < 0 || g1 > s.g_len || g1 < g0 || (g1 > 0 && ((g1 - 1) >> d->log2_tile) >= d->n_tiles)) { err = "position range outside the layout"; return -1; }
    if (!d->d_rac) {
        HIP_TRY(hipMalloc(&d->d_rac, 64 * sizeof(unsigned long long) + 2 * kRacBlocks * sizeof(double)));
        HIP_TRY(host_pinned_malloc((void**)&d->h_rac, 64 * sizeof(unsigned long long) + 2 * kRacBlocks * sizeof(double)));
    }
    unsigned long long* hist = reinterpret_cast<unsigned long long*>(d->d_rac);
    double* part = reinterpret_cast<double*>(reinterpret_cast<char*>(d->d_rac) + 64 * sizeof(unsigned long long));
    HIP_TRY(hipMemsetAsync(d->d_rac, 0, 64 * sizeof(unsigned long long), d->stream));
    hipExtLaunchKernelGGL(k_rac, dim3(kRacBlocks), dim3(kRacThreads), 0, d->stream, d->ev[0], d->ev[1], 0,
                          (const uint8_t*)d->d_pile, (const TileInfo*)d->d_tinfo, d->log2_tile, g0, g1, min_rd, min_bq, hist, part);
    HIP_TRY(launch_check());
    DMA(d->h_rac, d->d_rac, 64 * sizeof(unsigned long long) + 2 * kRacBlocks * sizeof(double), 1, d->stream);
    HIP_TRY(hipStreamSynchronize(d->stream));
    const unsigned long long* hh = reinterpret_cast<const unsigned long long*>(d->h_rac);
    const double* pp = reinterpret_cast<const double*>(reinterpret_cast<const char*>(d->h_rac) + 64 * sizeof(unsigned long long));
    for (int i = 0; i < kRacPropBins + kRacNallBins; i++) hist_out[i] = hh[i];
    double a = 0, b = 0;
    for (int i = 0; i < kRacBlocks; i++) { a += pp[2 * i]; b += pp[2 * i + 1]; }
    *sum = a;
    *sum_sq = b;
    float ms = 0;
    (void)hipEventElapsedTime(&ms, d->ev[0], d->ev[1]);
    *kernel_ms = ms;
    return 0;
}

// KPM's variant and grid: 3 waves per SIMD -- 139 VGPRs, no scratch at all (round 4: the log-conditionals read back
// from LDS, the biallelic posterior without its 16-entry array, the copy numbers in one register pair, static indexes
// only); the 4-wave build spills 10 VGPRs, which wrote 113 MB per configs[4] launch against 45 MB at 3 waves for
// the same time (`tools/gpu_r4_kpmab.sh`) -- and 16384 workgroups looping over the queue
#ifndef NGSEP_KPM_WPE                          // (build-time override: A/B builds only)
#define NGSEP_KPM_WPE 3
#endif
constexpr int kKpmWavesPerEu = NGSEP_KPM_WPE;
constexpr unsigned kKpmGrid = 16384;
// KPM's grid: one workgroup per slot the occupancy leaves (3 waves per SIMD, 4-wave workgroups: 3 per CU), each looping
// over the queue -- configs[4] KPM 0.302 -> 0.256 ms against 16384 workgroups (the empty ones' dispatch was the
// difference; 512 / 1024 / 1536 per 256 CUs: 0.283 / 0.259 / 0.283 ms, tools/gpu_r5_indel.sh).  (DIAG builds:
// NGSEP_KPM_GRID / NGSEP_STA_GRID override the two grids.)
static unsigned kpm_grid(const Device* d) {
    static const char* e = diag_env("NGSEP_KPM_GRID");
    return e ? std::max(1u, (unsigned)std::atoi(e)) : (unsigned)std::max(1, d->n_cu * 3);
}
static unsigned sta_grid() {
    static const unsigned g = diag_env("NGSEP_STA_GRID") ? std::max(1u, (unsigned)std::atoi(diag_env("NGSEP_STA_GRID"))) : kKpmGrid;
    return g;
}
static auto kpm_kernel(int ploidy, int gather, bool gcol) {
    if (gather == 1 && gcol)
        return ploidy >= 3 ? k_posterior_multi<true, kKpmWavesPerEu, 1, true> : k_posterior_multi<false, kKpmWavesPerEu, 1, true>;
    if (gather == 1)
        return ploidy >= 3 ? k_posterior_multi<true, kKpmWavesPerEu, 1, false> : k_posterior_multi<false, kKpmWavesPerEu, 1, false>;
    return ploidy >= 3 ? k_posterior_multi<true, kKpmWavesPerEu, 0, false> : k_posterior_multi<false, kKpmWavesPerEu, 0, false>;
}

// Where KPM's and k_stage_a's gathered columns live: LDS while the bytes of one workgroup's columns ((S + 1) x the
// per-sample coverage bound for KPM, 64 x it for the first stage) stay within kPopGatherCap, else the device scratch
// d_gcol, a part per workgroup -- the grid then shrinks so that the scratch stays within kPopGatherCap's budget
// (kPopGcolBudget).  No depth is refused (MultisampleVariantsDetector genotypes a position at whatever depth it has,
// :522-558, :674-693).  NGSEP_POP_GCOL=1 (test hook) takes the scratch at any depth.
struct PopCols {
    bool kpm_gcol = false, sta_gcol = false;
    unsigned kpm_grid = 1, sta_grid = 1;
};
static PopCols pop_cols(Device* d, std::string& err, bool* fail) {
    const bool force = env_hook("NGSEP_POP_GCOL") != nullptr;     // (read every run)
    PopCols c;
    *fail = false;
    const int64_t stride = std::max<int32_t>(d->pop_stride, 1);
    const int64_t kpm_wg = (int64_t)(d->n_samples + 1) * stride, sta_wg = 64 * stride;
    c.kpm_gcol = d->prg && (force || kpm_wg > kPopGatherCap);
    c.sta_gcol = d->prg && (force || sta_wg > kPopGatherCap);
    c.kpm_grid = kpm_grid(d);
    c.sta_grid = sta_grid();
    if (c.kpm_gcol) c.kpm_grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(c.kpm_grid, kPopGcolBudget / kpm_wg));
    if (c.sta_gcol) c.sta_grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(c.sta_grid, kPopGcolBudget / sta_wg));
    const size_t need = std::max<size_t>(c.kpm_gcol ? (size_t)c.kpm_grid * (size_t)kpm_wg : 0,
                                         c.sta_gcol ? (size_t)c.sta_grid * (size_t)sta_wg : 0);
    if (need && ensure_dev(&d->d_gcol, &d->cap_gcol, need, false, err)) *fail = true;
    return c;
}

// KLM over every (sample, tile) of the resident population layout, then KQN (shared by the two multisample paths)
// (need_clean: the open-position bits are already zero -- the previous pass's k_stage_a cleared them)
static hipError_t launch_pop_scan(Device* d, const GenotypeParams& g, uint32_t* need, QueueSite* queue, int64_t qcap,
                                  unsigned long long* ctr, hipEvent_t ev_start, hipEvent_t ev_end, PopStage* stage,
                                  bool need_clean) {
    const int64_t nwords = d->g_len / 32 + 1;
    hipError_t e = need_clean ? hipSuccess : hipMemsetAsync(need, 0, (size_t)nwords * sizeof(uint32_t), d->stream);
    if (e != hipSuccess) return e;
    const int64_t ntile = d->g_len / kKlmTile;
    const int64_t nblk = std::max<int64_t>(1, ntile * ((d->n_samples + 3) / 4));
    if (nblk >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    // the count bound needs every sample's coverage over a tile below 128 (byte counters): the tiles where some sample
    // is deeper take the exact bound at every marked position (k_scan_pop<false>, a launch over those tiles only)
    const int64_t ndeep = d->n_deep_tiles;
    const int64_t nsg = (d->n_samples + 3) / 4;
    const bool counting = ndeep == 0 || ndeep < ntile;
    if (counting) {
        hipExtLaunchKernelGGL(k_scan_pop<true>, dim3((unsigned)nblk), dim3(kKlmThreads), 0, d->stream, ev_start, nullptr, 0,
                              (const uint64_t*)d->d_units, (const int2*)d->d_rh, (const RGroup*)d->d_grp,
                              (const int32_t*)d->d_samp_st, (const int32_t*)d->d_blkA, (const int32_t*)d->d_blkB, d->pnblk,
                              d->pblk_shift, d->n_samples, (const uint8_t*)d->d_ref, (const LikTables*)d->d_tables, g, need, ctr,
                              stage ? stage->pairs : nullptr, stage ? stage->pseg : (int64_t)0, (const int64_t*)d->d_st_end,
                              (const uint8_t*)(ndeep ? d->d_deep_flag : nullptr), (const int32_t*)nullptr);
        if ((e = launch_check()) != hipSuccess) return e;
    }
    if (ndeep) {
        hipExtLaunchKernelGGL(k_scan_pop<false>, dim3((unsigned)(ndeep * nsg)), dim3(kKlmThreads), 0, d->stream,
                              counting ? nullptr : ev_start, nullptr, 0,
                              (const uint64_t*)d->d_units, (const int2*)d->d_rh, (const RGroup*)d->d_grp,
                              (const int32_t*)d->d_samp_st, (const int32_t*)d->d_blkA, (const int32_t*)d->d_blkB, d->pnblk,
                              d->pblk_shift, d->n_samples, (const uint8_t*)d->d_ref, (const LikTables*)d->d_tables, g, need, ctr,
                              stage ? stage->pairs : nullptr, stage ? stage->pseg : (int64_t)0, (const int64_t*)d->d_st_end,
                              (const uint8_t*)nullptr, (const int32_t*)d->d_deep_tiles);
        if ((e = launch_check()) != hipSuccess) return e;
    }
    const int64_t qblk = std::max<int64_t>(1, std::min<int64_t>((nwords + 255) / 256, (int64_t)d->n_cu * 4));
    hipExtLaunchKernelGGL(k_queue_need, dim3((unsigned)qblk), dim3(256), 0, d->stream, nullptr, ev_end, 0,
                          (const uint32_t*)need, (const uint8_t*)d->d_ref, nwords, queue, ctr, qcap, stage ? stage->qword : nullptr);
    if ((e = launch_check()) != hipSuccess) return e;
    if (stage) {                                       // KPM's first stage's sample masks
        hipLaunchKernelGGL(k_pair_mask, dim3(16, kKlShards), dim3(256), 0, d->stream, (const uint2*)stage->pairs, stage->pseg,
                           (const uint32_t*)need, (const int32_t*)stage->qword, stage->pmask, qcap, ctr);
        e = launch_check();
    }
    return e;
}

hipError_t PopStage::ensure(int64_t qcap, int64_t nwords, hipStream_t st) {
    hipError_t e = hipSuccess;
    if (qcap > cap) {
        (void)hipFree(pmask); (void)hipFree(qB); (void)hipFree(pairs);
        pmask = nullptr; qB = nullptr; pairs = nullptr;
        if ((e = hipMalloc(&pmask, (size_t)qcap * 8 * sizeof(uint32_t))) != hipSuccess) return e;
        if ((e = hipMemsetAsync(pmask, 0, (size_t)qcap * 8 * sizeof(uint32_t), st)) != hipSuccess) return e;
        if ((e = hipMalloc(&qB, (size_t)qcap * sizeof(QueueSite))) != hipSuccess) return e;
        pseg = std::max<int64_t>(4096, qcap / 4);           // (segments past this: the first stage passes everything on)
        if ((e = hipMalloc(&pairs, (size_t)pseg * kKlShards * sizeof(uint2))) != hipSuccess) return e;
        cap = qcap;
    }
    if (nwords > cap_qword) {
        (void)hipFree(qword);
        qword = nullptr;
        if ((e = hipMalloc(&qword, (size_t)nwords * sizeof(int32_t))) != hipSuccess) return e;
        cap_qword = nwords;
    }
    return e;
}

// KPM's two stages apply to discovery without minAlleleDepthFrequency (the first stage's allele set is the called
// alleles'), ploidy < 3 and the hom-ref bounds on (the samples they prove hom-ref are hom-ref for any allele set)
static bool pop_two_stage(const Device* d, const GenotypeParams& g, double min_adf, int ploidy, bool mknown) {
    const bool off = env_hook("NGSEP_KPM_ONE_STAGE") != nullptr;   // (test hook: the one-stage path; read every run)
    return !off && !mknown && d->prg && ploidy < 3 && min_adf == 0.0 && g.use_bound != 0;
}
static PopGather pop_gather_of(const Device* d, bool gcol) {
    PopGather pg{};
    if (!d->prg) return pg;
    pg.units = d->d_units; pg.rh = d->d_rh; pg.grp = d->d_grp; pg.samp_st = d->d_samp_st; pg.st_end = d->d_st_end;
    pg.blkA = d->d_blkA; pg.ref = d->d_ref; pg.nblk = d->pnblk; pg.shift = d->pblk_shift; pg.stride = d->pop_stride;
    pg.gcol = gcol ? d->d_gcol : nullptr;
    return pg;
}
// KPM's first stage over KQN's queue (k_stage_a, one wavefront per position): the positions whose QS can pass -> the
// stage's queue (counter 7), which the second stage (k_posterior_multi) genotypes in full
static hipError_t launch_stage_a(Device* d, const PopCols& pc, const GenotypeParams& g, int ploidy, const QueueSite* queue,
                                 const unsigned long long* qn, int64_t qcap, PopStage& st, unsigned long long* ctr,
                                 uint32_t* need_clear, int64_t need_words) {
    hipLaunchKernelGGL(pc.sta_gcol ? k_stage_a<true> : k_stage_a<false>, dim3(pc.sta_grid), dim3(64),
                       pc.sta_gcol ? (size_t)0 : (size_t)64 * (size_t)d->pop_stride, d->stream, queue, qn, qcap,
                       pop_gather_of(d, pc.sta_gcol), (const LikTables*)d->d_tables, g, (int32_t)ploidy, st.pmask, st.qB, ctr + 7,
                       st.cap, ctr, need_clear, need_words);
    return launch_check();
}
// KPM over a queue (mode 1: columns gathered from the population layout; 0: the realigner regions' site-major pile)
static hipError_t launch_kpm(Device* d, const PopCols& pc, int mode, const GenotypeParams& g, int ploidy, double min_adf,
                             const QueueSite* queue, const unsigned long long* qn, int64_t qcap, ngsep_popsite_out* sites,
                             ngsep_sample_call* calls, unsigned long long* ctr, int64_t cap, unsigned long long* stamps,
                             hipEvent_t ev_end) {
    const bool gcol = mode == 1 && pc.kpm_gcol;
    const size_t lds = mode == 1 && !gcol ? (size_t)(d->n_samples + 1) * (size_t)d->pop_stride : 0;
    hipExtLaunchKernelGGL(kpm_kernel(ploidy, mode, gcol), dim3(mode == 1 ? pc.kpm_grid : kpm_grid(d)), dim3(kPopThreads), lds,
                          d->stream, nullptr, ev_end, 0, queue, qn, qcap, (const uint8_t*)d->d_ppile, (const int32_t*)d->d_prow,
                          (const int64_t*)d->d_pboff, pop_gather_of(d, gcol), (const LikTables*)d->d_tables, g, d->n_samples,
                          min_adf, (int32_t)ploidy, (const PoolTables*)(ploidy >= 3 ? d->d_pool : nullptr), sites, calls, ctr,
                          cap, stamps);
    return launch_check();
}
// the shard counters' sums: KLM's candidate columns and bounded columns
static void pop_scan_counts(const unsigned long long* h, int64_t* cand, int64_t* bounded) {
    int64_t a = 0, b = 0;
    for (int t = 0; t < kKlShards; t++) { a += (int64_t)h[kCtrShard0 + kCtrShardStride * t]; b += (int64_t)h[kCtrShard0 + kCtrShardStride * t + 1]; }
    *cand = a;
    *bounded = b;
}

// MultisampleVariantsDetector run: KLM over every (sample, tile), KQN, KPM over the queued positions,
// D2H of the emitted sites and their per-sample calls (unordered; the host orders them)
int device_run_multi(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g,
                     int32_t n_samples, double min_adf, int ploidy,
                     const ngsep_popsite_out** sites, const ngsep_sample_call** calls, int64_t* n_sites,
                     double* scan_ms, double* geno_ms, double* total_ms, int64_t* n_candidates, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    auto t0 = std::chrono::steady_clock::now();
    const int32_t S = d->n_samples;
    if (S <= 0 || n_samples != S) { err = "multisample run without samples (ngsep_set_samples)"; return -1; }
    if (S > kMaxSamplesDevice) { err = "too many samples for one device run"; return -1; }
    const bool timing = diag_env("NGSEP_TIMING") != nullptr;
    if (timing && !d->d_stamps) HIP_TRY(hipMalloc(&d->d_stamps, 16 * sizeof(unsigned long long)));
    if (timing) HIP_TRY(hipMemsetAsync(d->d_stamps, 0, 16 * sizeof(unsigned long long), d->stream));
    int64_t want = std::max<int64_t>(d->last_n_sites + d->last_n_sites / 4 + 1024, 4096);
    if (want > d->cap_psites) {
        (void)hipFree(d->d_psites);
        (void)hipFree(d->d_pcalls);
        d->d_psites = nullptr;
        d->d_pcalls = nullptr;
        HIP_TRY(hipMalloc(&d->d_psites, (size_t)want * sizeof(ngsep_popsite_out)));
        HIP_TRY(hipMalloc(&d->d_pcalls, (size_t)want * S * sizeof(ngsep_sample_call)));
        d->cap_psites = want;
    }
    int64_t qwant = std::max<int64_t>(s.g_len / 64 + 65536, 65536);
    if (qwant > d->cap_hard) {
        (void)hipFree(d->d_hard);
        HIP_TRY(hipMalloc(&d->d_hard, (size_t)qwant * sizeof(QueueSite)));
        d->cap_hard = qwant;
    }
    if (!d->tables_valid || std::memcmp(&d->h_tables, &t, sizeof(LikTables)) != 0) {
        d->h_tables = t;
        H2D(d->d_tables, &d->h_tables, sizeof(LikTables), d->stream);
        d->tables_valid = true;
    }
    unsigned long long* ctr = d->d_counters;
    HIP_TRY(hipMemsetAsync(ctr, 0, kCtrWords * sizeof(unsigned long long), d->stream));
    // KLM + KQN, timed together by events bound to their dispatches (ev 0-1), KPM by ev 1-2
    const bool mknown = d->n_mforced >= 0;             // -knownVariants (and the realigner's regions): the queue is given
    const bool two = pop_two_stage(d, g, min_adf, ploidy, mknown);
    if (two) HIP_TRY(d->pstage.ensure(d->cap_hard, d->g_len / 32 + 1, d->stream));
    if (mknown || !d->prg) {
        HIP_TRY(hipEventRecord(d->ev[0], d->stream));
        HIP_TRY(hipEventRecord(d->ev[1], d->stream));
    } else {
        const bool clean = d->need_clean;
        d->need_clean = false;
        HIP_TRY(launch_pop_scan(d, g, d->d_need, d->d_hard, d->cap_hard, ctr, d->ev[0], d->ev[1], two ? &d->pstage : nullptr, clean));
    }
    if (ploidy >= 3 && !d->pool_valid) { err = "ploidy >= 3 without pool tables (device_set_pool)"; return -1; }
    // (no start event on KPM: a start event between KQN and KPM was measured to idle the device; KPM's time is
    // taken from KQN's end)
    if (!mknown && !d->prg) { err = "multisample run without a population layout"; return -1; }
    const int mode = d->prg ? 1 : 0;
    bool cfail = false;
    const PopCols pc = pop_cols(d, err, &cfail);
    if (cfail) return -1;
    if (two) {
        const bool scanned = !mknown && d->prg;
        HIP_TRY(launch_stage_a(d, pc, g, ploidy, d->d_hard, ctr + 2, d->cap_hard, d->pstage, ctr, scanned ? d->d_need : nullptr,
                               scanned ? d->g_len / 32 + 1 : 0));
        d->need_clean = scanned;
    }
    HIP_TRY(launch_kpm(d, pc, mode, g, ploidy, min_adf, (const QueueSite*)(mknown ? d->d_mforced : two ? d->pstage.qB : d->d_hard),
                       (const unsigned long long*)(mknown ? d->d_mforced_ctr + 2 : two ? ctr + 7 : ctr + 2),
                       mknown ? std::max<int64_t>(d->n_mforced, 1) : two ? d->pstage.cap : d->cap_hard, d->d_psites, d->d_pcalls,
                       ctr, d->cap_psites, d->d_stamps, d->ev[2]));
    DMA(d->h_counters, ctr, kCtrWords * sizeof(unsigned long long), 1, d->stream);
    HIP_TRY(hipStreamSynchronize(d->stream));
    const unsigned long long c3 = d->h_counters[3];
    if (c3 >> 63) { err = "internal error: a gathered population column exceeds its coverage bound"; return -1; }
    int64_t cand = 0, bounded = 0;
    pop_scan_counts(d->h_counters, &cand, &bounded);
    const int64_t n = (int64_t)d->h_counters[0];
    if ((int64_t)d->h_counters[2] > d->cap_hard) {
        (void)hipFree(d->d_hard);
        d->d_hard = nullptr;
        HIP_TRY(hipMalloc(&d->d_hard, (size_t)(d->h_counters[2] + 1024) * sizeof(QueueSite)));
        d->cap_hard = (int64_t)d->h_counters[2] + 1024;
        return device_run_multi(d, s, t, g, n_samples, min_adf, ploidy, sites, calls, n_sites, scan_ms, geno_ms, total_ms, n_candidates, err);
    }
    if (n > d->cap_psites) {
        d->last_n_sites = n;
        d->cap_psites = 0;
        return device_run_multi(d, s, t, g, n_samples, min_adf, ploidy, sites, calls, n_sites, scan_ms, geno_ms, total_ms, n_candidates, err);
    }
    if (n > d->cap_h_psites || n * S > d->cap_h_pcalls) {          // pinned staging, grown geometrically
        if (d->h_psites) host_pinned_free(d->h_psites);
        if (d->h_pcalls) host_pinned_free(d->h_pcalls);
        d->h_psites = nullptr;
        d->h_pcalls = nullptr;
        d->cap_h_psites = std::max<int64_t>(n + n / 2, 1024);
        d->cap_h_pcalls = d->cap_h_psites * S;
        HIP_TRY(host_pinned_malloc((void**)&d->h_psites, (size_t)d->cap_h_psites * sizeof(ngsep_popsite_out)));
        HIP_TRY(host_pinned_malloc((void**)&d->h_pcalls, (size_t)d->cap_h_pcalls * sizeof(ngsep_sample_call)));
    }
    if (n) {
        // the sites only: their calls come back in output order through device_fetch_calls_ordered
        DMA(d->h_psites, d->d_psites, (size_t)n * sizeof(ngsep_popsite_out), 1, d->stream);
        HIP_TRY(hipStreamSynchronize(d->stream));
    }
    *sites = d->h_psites;
    *calls = nullptr;
    *n_sites = n;
    d->last_n_sites = n;
    d->last_hard = (int64_t)d->h_counters[2];
    d->last_exact = bounded;
    if (timing) {
        unsigned long long* st = nullptr;                        // (a pinned endpoint, as every copy's)
        HIP_TRY(host_pinned_malloc((void**)&st, 16 * sizeof(unsigned long long)));
        DMA_SYNC(st, d->d_stamps, 16 * sizeof(unsigned long long), 1);
        std::fprintf(stderr, "[ngsep timing] KPM block 0 phases (cycles): tally %lld, pooled %lld, genotype %lld\n",
                     (long long)(st[1] - st[0]), (long long)(st[2] - st[1]), (long long)(st[5] - st[2]));
        host_pinned_free(st);
    }
    float a = 0, a2 = 0;
    (void)hipEventElapsedTime(&a, d->ev[0], d->ev[1]);
    (void)hipEventElapsedTime(&a2, d->ev[1], d->ev[2]);
    *scan_ms = a;
    *geno_ms = a2;
    *total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    *n_candidates = cand;                   // candidate columns (sample, position) the scan marked
    return 0;
}

// the kept sites' per-sample calls gathered into output order and packed into PopCall32 (engine.hpp); a call a
// field of which does not fit goes whole to big[], its record holding big_base + its index there
__global__ __launch_bounds__(256) void k_gather_calls(const ngsep_sample_call* __restrict__ calls, const int64_t* __restrict__ src,
                                                      int64_t m, int64_t S, PopCall32* __restrict__ out,
                                                      ngsep_sample_call* __restrict__ big, unsigned long long* nbig,
                                                      int64_t big_cap, int64_t big_base, int force_big) {
    const int64_t total = m * S;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = i / S, smp = i - k * S;
        const ngsep_sample_call c = calls[src[k] * S + smp];
        bool fit = c.kind >= 0 && c.kind <= 1 && c.n_called >= 0 && c.n_called <= 3 && c.called[0] >= -1 && c.called[0] <= 14 &&
                   c.called[1] >= -1 && c.called[1] <= 14 && c.gq >= 0 && c.gq <= 255 && c.dp >= 0 && c.dp <= 65535;
#pragma unroll
        for (int t = 0; t < 4; t++) fit = fit && c.counts[t] >= 0 && c.counts[t] <= 65535 && c.acn[t] >= -128 && c.acn[t] <= 127;
#pragma unroll
        for (int t = 0; t < 10; t++) fit = fit && (t < 6 ? (c.pl[t] >= 0 && c.pl[t] <= 65535) : c.pl[t] == 0);
        fit = fit && !force_big;
        PopCall32 o;
        if (fit) {
            o.flags = (uint8_t)(c.kind | c.n_called << 1);
            o.called = (uint8_t)((c.called[0] + 1) | (c.called[1] + 1) << 4);
            o.gq = (uint8_t)c.gq;
            o.pad0 = 0;
            o.total_cn = c.total_cn;
            o.dp = (uint16_t)c.dp;
#pragma unroll
            for (int t = 0; t < 4; t++) { o.counts[t] = (uint16_t)c.counts[t]; o.acn[t] = (int8_t)c.acn[t]; }
#pragma unroll
            for (int t = 0; t < 6; t++) o.pl[t] = (uint16_t)c.pl[t];
        } else {
            const unsigned long long b = atomicAdd(nbig, 1ull);
            if ((int64_t)b < big_cap) big[b] = c;
            const unsigned long long gi = (unsigned long long)big_base + b;
            o = PopCall32{};
            o.flags = 0x80;
            o.pl[0] = (uint16_t)(gi & 0xFFFFu);
            o.pl[1] = (uint16_t)(gi >> 16);
        }
        out[i] = o;
    }
}

// after device_run_multi: the calls of the m kept sites (staging indexes src, output order) gathered and packed on
// the device and copied straight into dst (pinned host memory of the context's call store); the calls that do not
// fit a PopCall32 are appended whole to big
int device_fetch_calls_from(Device* d, const ngsep_sample_call* calls, hipStream_t stream, const int64_t* src, int64_t m,
                            PopCall32* dst, PinnedStore<ngsep_sample_call>* big, std::string& err);
int device_fetch_calls_ordered(Device* d, const int64_t* src, int64_t m, PopCall32* dst, PinnedStore<ngsep_sample_call>* big, std::string& err) {
    return device_fetch_calls_from(d, d->d_pcalls, d->stream, src, m, dst, big, err);
}

int device_fetch_calls_from(Device* d, const ngsep_sample_call* calls, hipStream_t stream, const int64_t* src, int64_t m,
                            PopCall32* dst, PinnedStore<ngsep_sample_call>* big, std::string& err) {
    if (m <= 0) return 0;
    HIP_TRY(hipSetDevice(d->ordinal));
    const int64_t S = d->n_samples;
    if (m > d->cap_csrc) {
        (void)hipFree(d->d_csrc);
        if (d->h_csrc) host_pinned_free(d->h_csrc);
        d->d_csrc = nullptr;
        d->h_csrc = nullptr;
        d->cap_csrc = std::max<int64_t>(m + m / 2, 4096);
        HIP_TRY(hipMalloc(&d->d_csrc, (size_t)d->cap_csrc * sizeof(int64_t)));
        HIP_TRY(host_pinned_malloc((void**)&d->h_csrc, (size_t)(d->cap_csrc + 1) * sizeof(int64_t)));
    }
    if (m * S > d->cap_pcalls_ord) {
        (void)hipFree(d->d_pcalls_ord);
        (void)hipFree(d->d_pbig);
        d->d_pcalls_ord = nullptr;
        d->d_pbig = nullptr;
        d->cap_pcalls_ord = std::max<int64_t>(m * S + m * S / 2, 4096 * S);
        HIP_TRY(hipMalloc(&d->d_pcalls_ord, (size_t)d->cap_pcalls_ord * sizeof(PopCall32)));
        HIP_TRY(hipMalloc(&d->d_pbig, (size_t)d->cap_pcalls_ord * sizeof(ngsep_sample_call) + 8));
    }
    // the big-record counter sits after the records
    unsigned long long* d_nbig = reinterpret_cast<unsigned long long*>(d->d_pbig + d->cap_pcalls_ord);
    std::memcpy(d->h_csrc, src, (size_t)m * sizeof(int64_t));
    DMA(d->d_csrc, d->h_csrc, (size_t)m * sizeof(int64_t), 0, stream);
    HIP_TRY(hipMemsetAsync(d_nbig, 0, sizeof(unsigned long long), stream));
    const int64_t nblk = std::max<int64_t>(1, std::min<int64_t>((m * S + 255) / 256, (int64_t)d->n_cu * 8));
    hipLaunchKernelGGL(k_gather_calls, dim3((unsigned)nblk), dim3(256), 0, stream, calls, (const int64_t*)d->d_csrc, m, S,
                       d->d_pcalls_ord, d->d_pbig, d_nbig, d->cap_pcalls_ord, (int64_t)big->size(),
                       env_hook("NGSEP_POP_ALL_BIG") ? 1 : 0);   // (tests: every call through the whole-record list)
    HIP_TRY(launch_check());
    DMA(dst, d->d_pcalls_ord, (size_t)(m * S) * sizeof(PopCall32), 1, stream);
    unsigned long long* h_nbig = reinterpret_cast<unsigned long long*>(d->h_csrc + d->cap_csrc);
    DMA(h_nbig, d_nbig, sizeof(unsigned long long), 1, stream);
    HIP_TRY(hipStreamSynchronize(stream));
    const int64_t nb = (int64_t)*h_nbig;
    if (nb > 0) {
        const size_t b0 = big->size();
        big->resize(b0 + (size_t)nb);
        DMA_SYNC(big->data() + b0, d->d_pbig, (size_t)nb * sizeof(ngsep_sample_call), 1);
    }
    return 0;
}

// KPM's calls packed in place of order (no site permutation: the host orders the packed records), the emitted
// site count read from the device counter; the calls that do not fit go whole to big[] (index = their slot there)
__global__ __launch_bounds__(256) void k_pack_calls(const ngsep_sample_call* __restrict__ calls, const unsigned long long* nsites,
                                                    int64_t cap_sites, int64_t S, PopCall32* __restrict__ out,
                                                    ngsep_sample_call* __restrict__ big, unsigned long long* nbig, int64_t big_cap,
                                                    int force_big) {
    int64_t n = (int64_t)*nsites;
    if (n > cap_sites) n = cap_sites;
    const int64_t total = n * S;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const ngsep_sample_call c = calls[i];
        bool fit = c.kind >= 0 && c.kind <= 1 && c.n_called >= 0 && c.n_called <= 3 && c.called[0] >= -1 && c.called[0] <= 14 &&
                   c.called[1] >= -1 && c.called[1] <= 14 && c.gq >= 0 && c.gq <= 255 && c.dp >= 0 && c.dp <= 65535;
#pragma unroll
        for (int t = 0; t < 4; t++) fit = fit && c.counts[t] >= 0 && c.counts[t] <= 65535 && c.acn[t] >= -128 && c.acn[t] <= 127;
#pragma unroll
        for (int t = 0; t < 10; t++) fit = fit && (t < 6 ? (c.pl[t] >= 0 && c.pl[t] <= 65535) : c.pl[t] == 0);
        fit = fit && !force_big;
        PopCall32 o;
        if (fit) {
            o.flags = (uint8_t)(c.kind | c.n_called << 1);
            o.called = (uint8_t)((c.called[0] + 1) | (c.called[1] + 1) << 4);
            o.gq = (uint8_t)c.gq;
            o.pad0 = 0;
            o.total_cn = c.total_cn;
            o.dp = (uint16_t)c.dp;
#pragma unroll
            for (int t = 0; t < 4; t++) { o.counts[t] = (uint16_t)c.counts[t]; o.acn[t] = (int8_t)c.acn[t]; }
#pragma unroll
            for (int t = 0; t < 6; t++) o.pl[t] = (uint16_t)c.pl[t];
        } else {
            const unsigned long long b = atomicAdd(nbig, 1ull);
            if ((int64_t)b < big_cap) big[b] = c;
            o = PopCall32{};
            o.flags = 0x80;
            o.pl[0] = (uint16_t)(b & 0xFFFFu);
            o.pl[1] = (uint16_t)(b >> 16);
        }
        out[i] = o;
    }
}

// Asynchronous multisample runs: submit enqueues KTM + KQN + KPM of one pass into a slot of its own and the D2H of
// its counters and (a guess of) its sites; collect waits for the oldest pass, and device_fetch_calls_from gathers
// its calls on the copy stream, so the gather and the big D2H of one pass overlap the next pass's kernels.
int device_submit_multi(Device* d, const LikTables& t, const GenotypeParams& g, int32_t n_samples, double min_adf,
                        int ploidy, std::string& err) {
    HIP_TRY(hipSetDevice(d->ordinal));
    const int32_t S = d->n_samples;
    if (S <= 0 || n_samples != S) { err = "multisample run without samples (ngsep_set_samples)"; return -1; }
    if (S > kMaxSamplesDevice) { err = "too many samples for one device run"; return -1; }
    if (ploidy >= 3 && !d->pool_valid) { err = "ploidy >= 3 without pool tables (device_set_pool)"; return -1; }
    if (d->minflight >= 2) { err = "two staged runs already in flight: collect first"; return -1; }
    MultiSlot& m = d->mslot[d->mnext];
    // capacities from the synchronous run's counts (device_run_multi grows them); a pass that still overflows is
    // rerun synchronously by the collect
    const int64_t want = std::max<int64_t>(d->last_n_sites + d->last_n_sites / 4 + 1024, 4096);
    if (want > m.cap_psites) {
        (void)hipFree(m.d_psites);
        (void)hipFree(m.d_pcalls);
        m.d_psites = nullptr;
        m.d_pcalls = nullptr;
        HIP_TRY(hipMalloc(&m.d_psites, (size_t)want * sizeof(ngsep_popsite_out)));
        HIP_TRY(hipMalloc(&m.d_pcalls, (size_t)want * S * sizeof(ngsep_sample_call)));
        m.cap_psites = want;
    }
    if (want > m.cap_h_psites) {
        if (m.h_psites) host_pinned_free(m.h_psites);
        m.h_psites = nullptr;
        HIP_TRY(host_pinned_malloc((void**)&m.h_psites, (size_t)want * sizeof(ngsep_popsite_out)));
        m.cap_h_psites = want;
    }
    const int64_t qwant = std::max<int64_t>(std::max<int64_t>(d->g_len / 64 + 65536, d->last_hard + 1024), 65536);
    if (qwant > m.cap_hard) {
        (void)hipFree(m.d_hard);
        m.d_hard = nullptr;
        HIP_TRY(hipMalloc(&m.d_hard, (size_t)qwant * sizeof(QueueSite)));
        m.cap_hard = qwant;
    }
    const int64_t nwords = d->g_len / 32 + 1;
    if (nwords > m.cap_need) {
        (void)hipFree(m.d_need);
        m.d_need = nullptr;
        HIP_TRY(hipMalloc(&m.d_need, (size_t)nwords * sizeof(uint32_t)));
        m.cap_need = nwords;
        m.need_clean = false;
    }
    if (!m.ev[0])
        for (int k = 0; k < 5; k++) HIP_TRY(hipEventCreateWithFlags(&m.ev[k], k < 4 ? hipEventDefault : hipEventDisableTiming));
    if (!d->tables_valid || std::memcmp(&d->h_tables, &t, sizeof(LikTables)) != 0) {
        HIP_TRY(hipStreamSynchronize(d->stream));     // an earlier upload may still read h_tables
        d->h_tables = t;
        H2D(d->d_tables, &d->h_tables, sizeof(LikTables), d->stream);
        d->tables_valid = true;
    }
    unsigned long long* ctr = d->slot[d->mnext].d_ctr;
    HIP_TRY(hipMemsetAsync(ctr, 0, kCtrWords * sizeof(unsigned long long), d->stream));
    const bool mknown = d->n_mforced >= 0;             // -knownVariants: the input variants are the queue
    if (!mknown && !d->prg) { err = "multisample run without a population layout"; return -1; }
    const bool two = pop_two_stage(d, g, min_adf, ploidy, mknown);
    if (two) HIP_TRY(m.stage.ensure(m.cap_hard, nwords, d->stream));
    if (mknown) {
        HIP_TRY(hipEventRecord(m.ev[0], d->stream));
        HIP_TRY(hipEventRecord(m.ev[1], d->stream));
    } else {
        const bool clean = m.need_clean;
        m.need_clean = false;
        HIP_TRY(launch_pop_scan(d, g, m.d_need, m.d_hard, m.cap_hard, ctr, m.ev[0], m.ev[1], two ? &m.stage : nullptr, clean));
    }
    const int mode = d->prg ? 1 : 0;
    bool cfail = false;
    const PopCols pc = pop_cols(d, err, &cfail);
    if (cfail) return -1;
    if (two) {
        HIP_TRY(launch_stage_a(d, pc, g, ploidy, m.d_hard, ctr + 2, m.cap_hard, m.stage, ctr, mknown ? nullptr : m.d_need,
                               mknown ? 0 : nwords));
        m.need_clean = !mknown;
    }
    HIP_TRY(launch_kpm(d, pc, mode, g, ploidy, min_adf, (const QueueSite*)(mknown ? d->d_mforced : two ? m.stage.qB : m.d_hard),
                       (const unsigned long long*)(mknown ? d->d_mforced_ctr + 2 : two ? ctr + 7 : ctr + 2),
                       mknown ? std::max<int64_t>(d->n_mforced, 1) : two ? m.stage.cap : m.cap_hard, m.d_psites, m.d_pcalls,
                       ctr, m.cap_psites, (unsigned long long*)nullptr, m.ev[3]));
    // the calls packed right behind KPM on the compute stream; the copies (counters, a guess of the sites, their
    // packed calls and whole records) on the copy stream, so the next pass's kernels do not wait for them
    if (m.cap_pack < m.cap_psites) {
        (void)hipFree(m.d_pack);
        (void)hipFree(m.d_big);
        m.d_pack = nullptr;
        m.d_big = nullptr;
        HIP_TRY(hipMalloc(&m.d_pack, (size_t)m.cap_psites * S * sizeof(PopCall32)));
        m.cap_big = std::max<int64_t>(4096, m.cap_psites * S / 8);
        HIP_TRY(hipMalloc(&m.d_big, (size_t)m.cap_big * sizeof(ngsep_sample_call)));
        m.cap_pack = m.cap_psites;
    }
    // (stores handed back by the context keep their capacity: no reallocation once warm)
    m.h_pack.clear();
    m.h_pack.reserve((size_t)(m.cap_psites * S));
    m.h_big.clear();
    m.h_big.reserve((size_t)m.cap_big);
    if (!m.ev[5]) HIP_TRY(hipEventCreateWithFlags(&m.ev[5], hipEventDisableTiming));
    unsigned long long* d_nbig = ctr + 5;             // (zero: the pass's kernels before k_pack_calls leave counter 5 alone)
    const int64_t pblk = std::max<int64_t>(1, std::min<int64_t>((m.cap_psites * S + 255) / 256, (int64_t)d->n_cu * 8));
    hipLaunchKernelGGL(k_pack_calls, dim3((unsigned)pblk), dim3(256), 0, d->stream, (const ngsep_sample_call*)m.d_pcalls,
                       (const unsigned long long*)ctr, m.cap_psites, (int64_t)S, m.d_pack, m.d_big, d_nbig, m.cap_big,
                       env_hook("NGSEP_POP_ALL_BIG") ? 1 : 0);   // (tests: every call through the whole-record list)
    HIP_TRY(launch_check());
    HIP_TRY(hipEventRecord(m.ev[5], d->stream));
    HIP_TRY(hipStreamWaitEvent(d->copy_stream, m.ev[5], 0));
    hipStream_t cs = d->copy_stream;
    DMA(d->slot[d->mnext].h_ctr, ctr, kCtrWords * sizeof(unsigned long long), 1, cs);
    m.guess = std::min<int64_t>(m.cap_psites, d->last_n_sites + d->last_n_sites / 16 + 64);
    DMA(m.h_psites, m.d_psites, (size_t)m.guess * sizeof(ngsep_popsite_out), 1, cs);
    DMA(m.h_pack.data(), m.d_pack, (size_t)(m.guess * S) * sizeof(PopCall32), 1, cs);
    m.guess_big = std::min<int64_t>(m.cap_big, 4096);
    DMA(m.h_big.data(), m.d_big, (size_t)m.guess_big * sizeof(ngsep_sample_call), 1, cs);
    HIP_TRY(hipEventRecord(m.ev[4], cs));
    m.busy = true;
    d->mnext ^= 1;
    d->minflight++;
    return 0;
}

// the oldest submitted multisample pass: its sites (unordered, pinned) and the slot holding its calls.  *rerun = true
// when the pass overflowed a buffer (the caller reruns it synchronously through device_run_multi)
int device_collect_multi(Device* d, const ngsep_popsite_out** sites, int64_t* n_sites, int* slot, bool* rerun,
                         double* scan_ms, double* geno_ms, int64_t* n_candidates, std::string& err) {
    if (d->minflight <= 0) { err = "no run to collect"; return -1; }
    HIP_TRY(hipSetDevice(d->ordinal));
    const int k = d->mfirst;
    MultiSlot& m = d->mslot[k];
    d->mfirst ^= 1;
    d->minflight--;
    m.busy = false;
    HIP_TRY(hipEventSynchronize(m.ev[4]));
    const unsigned long long* hc = d->slot[k].h_ctr;
    const unsigned long long c3 = hc[3];
    if (c3 >> 63) { err = "internal error: a gathered population column exceeds its coverage bound"; return -1; }
    int64_t cand = 0, bounded = 0;
    pop_scan_counts(hc, &cand, &bounded);
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    static std::atomic<int> told{0};
    if (host_timing && told.fetch_add(1) < 2) {
        int64_t pairs = 0;
        for (int t = 0; t < kKlShards; t++) pairs += (int64_t)hc[kCtrShard0 + kCtrShardStride * t + 2];
        std::fprintf(stderr, "[ngsep host] population pass: candidate columns %lld, exact-bound columns %lld, opened (pairs) %lld, "
                     "queued positions %lld, second-stage positions %lld, sites %lld\n", (long long)cand, (long long)bounded,
                     (long long)pairs, (long long)hc[2], (long long)hc[7], (long long)hc[0]);
    }
    const int64_t n = (int64_t)hc[0];
    *rerun = (int64_t)hc[2] > m.cap_hard || n > m.cap_psites || (int64_t)hc[5] > m.cap_big;
    *slot = k;
    if (*rerun) return 0;
    const int64_t S = d->n_samples;
    if (n > m.guess) {
        DMA_SYNC(m.h_psites + m.guess, m.d_psites + m.guess, (size_t)(n - m.guess) * sizeof(ngsep_popsite_out), 1);
        DMA_SYNC(m.h_pack.data() + m.guess * S, m.d_pack + m.guess * S, (size_t)((n - m.guess) * S) * sizeof(PopCall32), 1);
    }
    const int64_t nb = (int64_t)hc[5];
    if (nb > m.guess_big)
        DMA_SYNC(m.h_big.data() + m.guess_big, m.d_big + m.guess_big, (size_t)(nb - m.guess_big) * sizeof(ngsep_sample_call), 1);
    *sites = m.h_psites;
    *n_sites = n;
    d->last_n_sites = n;
    d->last_hard = (int64_t)hc[2];
    d->last_exact = bounded;
    float a = 0, a2 = 0;
    (void)hipEventElapsedTime(&a, m.ev[0], m.ev[1]);
    (void)hipEventElapsedTime(&a2, m.ev[1], m.ev[3]);
    *scan_ms = a;
    *geno_ms = a2;
    *n_candidates = cand;
    return 0;
}

void device_slot_take(Device* d, int slot, int64_t n_sites, PinnedStore<PopCall32>& calls, PinnedStore<ngsep_sample_call>& big) {
    MultiSlot& m = d->mslot[slot];
    m.h_pack.n = (size_t)(n_sites * d->n_samples);
    m.h_big.n = (size_t)d->slot[slot].h_ctr[5];
    calls.swap(m.h_pack);
    big.swap(m.h_big);
    // the slot keeps what the context handed back, grown here (on the collect that makes the swap) rather than in
    // a later submit: from the second collect on, no pinned allocation happens in the pipeline
    m.h_pack.clear();
    m.h_pack.reserve((size_t)(m.cap_psites * d->n_samples));
    m.h_big.clear();
    m.h_big.reserve((size_t)m.cap_big);
}

int device_multi_inflight(const Device* d) { return d->minflight; }

}  // namespace ngsep
