// engine.hpp -- internal types of libngsep_amd.so (not part of the C ABI).
//
// Host side mirrors the reference's AlignmentsPileupGenerator admission sweep
// (discovery/AlignmentsPileupGenerator.java:377-452) and ReadAlignment's allele-call
// projection (alignments/ReadAlignment.java:747-871); the per-position work
// (PileupRecord -> CountsHelper -> VariantDiscoverySNVQAlgorithm) runs in kernels.hip.
#pragma once

#include <algorithm>
#include <cstdint>
#include <deque>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <sched.h>
#include <thread>
#include <vector>
#include <atomic>
#include <mutex>
#include <condition_variable>
#include <functional>
#include <utility>

#include "../../include/ngsep_gpu.h"
#include "realign.hpp"

namespace ngsep {

// ---- projected read-base code (one byte per reference position a read covers) ----
//   0x00                  : no allele call (deletion/skip, masked base, base before an indel, padding)
//   0x20 | q              : counted call that does not update likelihoods (q<=3 or not A/C/G/T)
//   0x80 | a<<5 | q       : valid call, allele a (0..3 = A,C,G,T), q = min(30, phred) > 3
// q is CountsHelper.java:91's min(DEF_MAX_BASE_QS, qual-33); the -maxBaseQS cap (:217-219)
// is applied in the kernel.
constexpr uint8_t kCodeCounted = 0x20;
constexpr uint8_t kCodeValid = 0x80;

// ---- reference code per position (global coordinate) ----
//   0x00 : padding between windows (outside any window)
//   0x01 : inside a window, not callable (N, lower case with -ignoreLowerCaseRef)
//   0x80 | a<<5 : callable reference base a
constexpr uint8_t kRefInWindow = 0x01;
constexpr uint8_t kRefCallable = 0x80;

// Tile-blocked pileup matrix ("pile"), the layout the scan kernel streams:
// the positions are cut into tiles of T (power of two) positions; tile t stores rows_t x T code
// bytes, row-major, where every row holds non-overlapping reads clipped to the tile (greedy
// interval colouring, rows_t = the tile's maximum depth).  Codes are stored with the allele
// XOR-ed with the reference allele, so a valid non-reference call is a valid byte with nonzero
// allele bits and the scan needs no reference lookup.
struct TileInfo {
    int64_t off;     // byte offset of the tile's block in the pile (16-B aligned)
    int32_t rows;    // rows_t (0 = no reads overlap the tile)
    int32_t pad;
};
static_assert(sizeof(TileInfo) == 16, "TileInfo layout");
constexpr int kScanThreads = 256;          // threads per tile-scan workgroup (one tile per wavefront)
constexpr int kScanRegUnits = 64 * 24;     // tile-size budget: 16-byte units per tile (deeper tiles are rare)
constexpr int kTileMaxPos = 1024;          // largest tile (positions): <= 64 units per row
constexpr int kTileMinPos = 16;
constexpr int kPopTile = 128;              // positions per KPM pile tile
constexpr int kRunAlign = 4096;            // a run's global coordinate is a whole number of these (KL tiles)

// Read-group layout of the single-sample variant caller: the admitted reads of a run
// in pending-list order are its entries; 64 consecutive entries form a group, and the group's reads'
// projected code bytes (one per reference position of [gfirst, glast]), each XOR-ed with its position's
// reference code (reference-relative: 0 is a valid reference call of quality 0), are interleaved in 8-byte
// units: unit k of entry 64 g + l is units[base_g + 64 k + l] (bytes 8k .. 8k+7 of the read, zero past its end).
// A wavefront that reads unit k of its 64 reads loads 512 contiguous bytes.  Entry header: {gfirst,
// glast | negative-strand << 31}; padding entries are empty (glast = gfirst - 1, gfirst = the last real one).
struct RGroup {
    int64_t base;    // unit offset of the group
    int32_t K;       // units per read (the group's longest span / 8, rounded up)
    int32_t pad;
};
static_assert(sizeof(RGroup) == 16, "RGroup layout");
constexpr int kRgBlockShift = 8;           // entry index tables per 256 positions (blkA / blkB)
constexpr int kKlTile = 2048;              // positions per KL tile (one workgroup each; divides kRunAlign)
constexpr int kMcMaxCalls = 254;           // multisample candidate column: valid calls the bounds take (sums fit 32 bits)
constexpr int kKlmTile = 2048;             // positions per KLM sample tile (one wavefront each; divides kRunAlign)
constexpr int kKlmSlots = 96;              // KLM: candidate columns a sample tile bounds exactly in LDS (more: kept open)
constexpr int kKlmQs = 10;                 // KLM's count bound counts the reference calls of quality >= kKlmQs
constexpr int kKlmCountMaxCov = 127;       // ... when no sample is deeper than this (its byte counters cannot carry)
constexpr int kPopGatherCap = 40960;       // KPM (gather): LDS bytes for one position's columns ((S + 1) x the per-sample bound);
                                           // with KPM's 21 KB of static LDS, within the 64 KB a workgroup is given.  Deeper
                                           // populations gather into a device scratch buffer instead (kernels.hip, GCOL)
constexpr int64_t kPopGcolBudget = (int64_t)1 << 30;   // ... of at most this many bytes (fewer KPM workgroups past it)

// the (first) alternative allele of a record as a DNA index: a pool record keeps its variant's alleles in
// the mask bits (ngsep_site_out.pool), an SNVQ record in .alt
template <class R>
inline int site_alt(const R& s) {
    if (!s.pool) return s.alt;
    for (int a = 0; a < 4; a++)
        if (((s.pool >> a) & 1) && "ACGT"[a] != s.ref) return a;
    return -1;
}

// K2 output record (device layout == ngsep_site_out, with gpos in .pos)
static_assert(sizeof(ngsep_site_out) == 152, "site record layout");
static_assert(sizeof(ngsep_sample_call) == 76, "sample call layout");
static_assert(sizeof(ngsep_popsite_out) == 20, "population site layout");
constexpr int kMaxSamplesDevice = 255;     // samples genotyped by one workgroup (one thread each, one for reads of no sample)

// Likelihood addends for the SNV model with n=4 alleles and f=g=250
// (CountsHelper.java:147-185 with heterozygousProportion 0.5, SingleSampleVariantPileupListener.java:236)
struct LikTables {
    double A[32];   // log10(1-e)                     logProbCacheGT[f][q][0]
    double H[32];   // log10(0.5(1-e)+0.5 e/3)        logProbCacheGT[250][q][4]
    double E[32];   // -0.1 q - log10(3)              logProbCacheError[q][4]
    // Integer hom-ref bound (DESIGN.md "hom-ref bound"), fixed point with kBoundScale units:
    //   wR[q] = floor(K(A-H)) | floor(K(A-E)) << 32   added once per reference-allele call
    //   wX[q] =  ceil(K(H-E)) |  ceil(K(A-E)) << 32   added once per call of a non-reference allele
    unsigned long long wR[32];
    unsigned long long wX[32];
    long long t_het;      // floor(K (log10 h/12 - log10 (1-h)/4 + log10 2)) + margin
    long long t_homo;     // margin
    // count bound (kernels.hip phase 2): extreme addends over the qualities a valid call can carry
    long long c_r1, c_r2; // min over q of the low / high half of wR
    long long c_x1, c_x2; // max over q of the low / high half of wX
    // the count bound as a table: with na other-allele calls, nr >= cb_nr[na] reference calls drop
    // the candidate (the three inequalities are non-decreasing in nr); 256: never (nr, na <= 255)
    int16_t cb_nr[256];
    // KLM's count bound (multisample): a sample column with ONE valid call of another allele and
    // at least cb_hi1 valid reference calls of quality >= kKlmQs is hom-ref (the reference addends at their minimum
    // over q in [kKlmQs, 30], the other allele's at its maximum); 256: never
    int32_t cb_hi1;
};
constexpr double kBoundScale = 1048576.0;   // 2^20: a tile holds <= 512 reads -> sums < 2^31
constexpr long long kBoundMargin = 64;      // 6e-5 in log10 units, >> fp64 rounding of the sums

// Pool genotyping (ploidy >= 3, SingleSampleVariantPileupListener.genotypeVariantPool :402-503): the
// hypotheses' frequencies, accumulated as the reference does (freq = step; freq < 0.51; freq += step), and
// the CountsHelper caches they index (CountsHelper.java:135-187) for variants of n = 2..4 alleles
constexpr int kPoolMaxFreq = 64;           // ploidy <= 128
struct PoolTables {
    int32_t ploidy, nf;                     // haplotypes, number of frequency hypotheses
    double freq[kPoolMaxFreq];              // hypothesis j's heterozygous proportion
    double A[32];                           // logProbCacheGT[*][q][0] = log10(1-e)
    double E[3][32];                        // logProbCacheError[q][n], n = 2, 3, 4
    double F[kPoolMaxFreq][3][32];          // logProbCacheGT[round(500 freq_j)][q][n]
    double G[kPoolMaxFreq][3][32];          // logProbCacheGT[round(500 (1-freq_j))][q][n]
    double log_h, log_1h;                   // log10(h), log10(1-h) (:446-447)
    double log_h_n[3];                      // log10(h/(n-1)), n = 2, 3, 4 (CountsHelper.java:451-467)
};

struct GenotypeParams {
    double log_prior_homo;     // log10((1-h)/4), CountsHelper.java:416
    double log_prior_hetero;   // log10(h/12),    CountsHelper.java:415
    int32_t max_q;             // effective -maxBaseQS cap
    int32_t min_quality;       // -minQuality
    int32_t dump_all;          // emit a record for every position with DP>0
    int32_t ablate;            // diagnostics only (env NGSEP_ABLATE): 1 scan only (no bound, no queue),
                               // 8 tally without posterior, 16 posterior kernel reads the queue only,
                               // 32 population kernel gathers only, 64 population kernel stops after the tallies,
                               // 128 KL without the exception counters, 256 KL without the read bases,
                               // 32768 KTM without the column bounds
    int32_t use_bound;         // 1: candidates proven hom-ref by the integer bound are dropped in the tile kernel
    int32_t full_records;      // 1: every record whole (ngsep_params.full_records); dump mode implies it
    int32_t ploidy;            // >= 3: KP runs the pool algorithm (k_posterior_pool), KT queues every
                               // position with a valid non-reference call (the pool variant needs one)
};

struct Window {            // a contiguous range of one sequence, resident in HBM
    int32_t seq_id;
    int32_t w0;            // first 1-based position
    int32_t wlen;          // number of positions
    int64_t gbase;         // global coordinate of position w0 is gbase + pad
    int32_t pad;           // halo positions on each side (>= max read span)
    int64_t read_begin, read_end;    // index range in the global read table
};

// uninitialised host array, filled in parallel (no serial zero-fill of GB-sized layouts)
// malloc for host arrays of the streamed path: blocks of 4 MB and more come 2 MB-aligned with transparent huge pages
// requested (madvise), so filling them takes 512x fewer page faults (engine.cpp)
void* huge_alloc(size_t bytes);

template <class T>
struct HostArray {
    T* p = nullptr;
    size_t n = 0;
    HostArray() = default;
    HostArray(const HostArray&) = delete;
    HostArray& operator=(const HostArray&) = delete;
    HostArray(HostArray&& o) noexcept : p(o.p), n(o.n) { o.p = nullptr; o.n = 0; }
    HostArray& operator=(HostArray&& o) noexcept { if (this != &o) { release(); p = o.p; n = o.n; o.p = nullptr; o.n = 0; } return *this; }
    ~HostArray() { release(); }
    void alloc(size_t k) { release(); n = k; p = k ? static_cast<T*>(huge_alloc(k * sizeof(T))) : nullptr; }
    void release() { std::free(p); p = nullptr; n = 0; }
};

// huge_alloc's pages with the elements a resize adds left uninitialised: for arrays whose every element the caller
// writes itself, on all threads (the serial zero fill of a value-initialising resize was ~0.3 s of the 200-sample
// population layout's 1.2 GB of index arrays)
template <class T>
struct RawAllocator {
    using value_type = T;
    RawAllocator() = default;
    template <class U> RawAllocator(const RawAllocator<U>&) {}
    T* allocate(size_t n) {
        void* p = huge_alloc(n * sizeof(T));
        if (!p) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { std::free(p); }
    template <class U> void construct(U* p) noexcept { ::new ((void*)p) U; }
    template <class U, class... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
    template <class U> bool operator==(const RawAllocator<U>&) const { return true; }
    template <class U> bool operator!=(const RawAllocator<U>&) const { return false; }
};
template <class T> using RawVec = std::vector<T, RawAllocator<T>>;

// Admitted reads of one sequence in pending order (AlignmentsPileupGenerator.pendingAlignments)
struct ContigReads {
    int32_t seq_id = -1;
    int64_t seq_len = 0;               // the sequence's length
    RawVec<int32_t> first, last;       // (resized, then written in full on all threads: no zero fill)
    RawVec<uint8_t> neg;               // 1 = negative strand
    std::vector<uint8_t> uniq;         // coverage mode: 1 = ReadAlignment.isUnique (no FLAG_MULTIPLE_ALN)
    std::vector<int16_t> sample;       // multisample: sample of the read's group (-1 none)
    std::vector<uint8_t> rank;         // multisample: rank of the read group in its sample's set
    RawVec<const uint8_t*> bptr;       // the read's projected codes over [first, last]
    std::vector<HostArray<uint8_t>> chunks;   // their storage: one uninitialised chunk per projected batch
    // indel-bearing admitted reads: [first, last + indel bases]; widened by the realigner's reach and merged
    // into `carved` when the sequence is staged (engine.cpp carve_indel_regions)
    std::vector<std::pair<int32_t, int32_t>> indel_reads;
    std::vector<std::pair<int32_t, int32_t>> carved;
    std::vector<size_t> chunk_end;     // reads [chunk_end[k-1], chunk_end[k]) have their bytes in chunks[k]
    std::vector<int64_t> chunk_used;   // the bytes chunks[k] holds (a pooled chunk may be larger)
    std::vector<int32_t> chunk_maxlast;   // their largest last position (streamed windows release the chunk after)
    int32_t max_span = 0;
    int64_t covered = 0;               // union of [first,last] (positions with a pileup)
    int32_t cov_last = 0;              // running max of last (for `covered`)
    void clear() {
        first.clear(); last.clear(); neg.clear(); uniq.clear(); sample.clear(); rank.clear(); bptr.clear(); chunks.clear();
        indel_reads.clear(); carved.clear(); chunk_end.clear(); chunk_used.clear(); chunk_maxlast.clear();
        max_span = 0; covered = 0; cov_last = 0; seq_id = -1;
    }
};

// One alignment as the admission sweep sees it: a view into the caller's batch, or into the context's
// carry storage when its same-start group is still open at the end of a batch
struct ReadView {
    int32_t seq_id, first, last, flags, rg;
    const int32_t* cigar;
    int32_t n_cigar;
    const char* chars;     // nullptr = no characters (getReadCharacters() == null)
    const char* quals;     // nullptr = no qualities ('*')
    int32_t len;
    int32_t indel_len;     // bases in the CIGAR's I/D items (0: SNV-only alignment)
    bool packed;           // BAM encoding (ngsep_call_bam's reader): chars = 4-bit bases, 2 per byte (high nibble
                           // first, "=ACMGRSVTWYHKDBN"), quals = raw Phred values (no +33)
    int32_t bidx;          // index in the batch being processed (-1: a carried read, in the carry store)
};
// the batch being admitted (engine.cpp process_batch): its reads are referenced by index until projected
struct BatchRef {
    const ngsep_read_batch* b = nullptr;
    const int32_t* last = nullptr;      // per read: reference end, indel bases (from the CIGAR)
    const int32_t* indel = nullptr;
    bool packed = false;
    const int64_t* qual_off = nullptr;  // packed batches: the qualities' offsets (else seq_off)
    const char* const* chars_at = nullptr;   // merged batches: each read's bases and qualities where they lie (else
    const char* const* quals_at = nullptr;   // bases / quals + seq_off); a null quals_at[i]: no qualities
};
// bam.cpp's BAM-encoded batches (ReadView::packed): bases and qualities read in place in the reader's decoded chunk
// (bases = quals = its start, a record's 4-bit bases at seq_off[i], its qualities at qual_off[i]), valid until the
// batch after next is read
struct PackedBatch {
    ngsep_read_batch b{};
    const int64_t* qual_off = nullptr;
};
struct CarryStore {        // owned copies of the open same-start group's reads
    std::vector<int32_t> cigar;
    std::string chars, quals;
};

// Environment.  A release build reads only: the host thread count (NGSEP_THREADS, OMP_NUM_THREADS); timing switches
// that add stderr lines or kernel events (NGSEP_HOST_TIMING, NGSEP_TIME_POSTERIOR); and test hooks that force an
// equivalent code path whose output the tests compare with the default one (NGSEP_ZLIB, NGSEP_PCUT_MISS,
// NGSEP_POP_STREAM, NGSEP_POP_ALL_BIG, NGSEP_BGZF_READ, NGSEP_KPM_ONE_STAGE); NGSEP_GPU_INFLATE selects the device inflate
// for the single-sample BAM readers (same bytes).  Tuning overrides and ablations (which may change launches or results) exist
// only in diagnostic builds (make DIAG=1 defines NGSEP_DIAG): elsewhere diag_env is always null.
inline const char* env_hook(const char* name) { return std::getenv(name); }
#ifdef NGSEP_DIAG
inline const char* diag_env(const char* name) { return std::getenv(name); }
#else
inline const char* diag_env(const char*) { return nullptr; }
#endif

// host worker threads: NGSEP_THREADS; else this process's share of the cores it may run on -- the affinity mask
// divided among the node's ranks (LOCAL_WORLD_SIZE, one process per GPU), at most OMP_NUM_THREADS when that is above 1
// (the GPU box's CPU share; torch.distributed.run sets 1 for its children by default, which is not a share)
inline unsigned host_threads() {
    static const unsigned n = [] {
        if (const char* e = std::getenv("NGSEP_THREADS")) return (unsigned)std::max(1L, std::min(std::atol(e), 64L));
        long cores = (long)std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0 && CPU_COUNT(&set) > 0) cores = CPU_COUNT(&set);
        const char* lw = std::getenv("LOCAL_WORLD_SIZE");
        const long ranks = lw ? std::max(1L, std::atol(lw)) : 1L;
        long v = std::max(1L, cores / ranks);
        const char* omp = std::getenv("OMP_NUM_THREADS");
        if (omp && std::atol(omp) > 1) v = std::min(v, std::atol(omp));
        return (unsigned)std::max(1L, std::min(v, 64L));
    }();
    return n;
}
// The host worker pool: host_threads() - 1 persistent workers shared by every parallel_for, whichever thread calls
// it (the BGZF decoder, the batch reader, the admission sweep and the layouts run concurrently; threads created per
// call oversubscribed the cores).  A call queues helper tickets and works itself; on finishing it cancels the
// tickets no worker has taken and waits only for the taken ones, so nested and concurrent calls cannot deadlock.
class HostPool {
public:
    struct Job {
        std::function<void()> work;
        std::unique_ptr<std::atomic<int>[]> state;   // per ticket: 0 queued, 1 taken, 2 done, 3 cancelled
        int n = 0;
        std::mutex mu;
        std::condition_variable cv;
    };
    static HostPool& get() {
        static HostPool* p = new HostPool((int)host_threads() - 1);   // (never destroyed: workers outlive statics)
        return *p;
    }
    int workers() const { return (int)th_.size(); }
    void submit(const std::shared_ptr<Job>& job) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            for (int k = 0; k < job->n; k++) q_.emplace_back(job, k);
        }
        if (job->n == 1) cv_.notify_one();
        else cv_.notify_all();
    }
private:
    explicit HostPool(int n) {
        for (int k = 0; k < n; k++) th_.emplace_back([this] { loop(); });
        for (auto& t : th_) t.detach();
    }
    void loop() {
        for (;;) {
            std::pair<std::shared_ptr<Job>, int> tk;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return !q_.empty(); });
                tk = std::move(q_.front());
                q_.pop_front();
            }
            Job& j = *tk.first;
            int expect = 0;
            if (!j.state[tk.second].compare_exchange_strong(expect, 1)) continue;   // cancelled: the call is done
            j.work();
            {
                std::lock_guard<std::mutex> lk(j.mu);
                j.state[tk.second].store(2);
            }
            j.cv.notify_all();
        }
    }
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::pair<std::shared_ptr<Job>, int>> q_;
    std::vector<std::thread> th_;
};

// fn(lo, hi) over [0, n) in chunks of >= grain on the host threads (inline below 2 chunks)
template <class F>
void parallel_for(int64_t n, int64_t grain, F&& fn) {
    if (n <= 0) return;
    const int64_t nt = std::min<int64_t>(host_threads(), (n + grain - 1) / std::max<int64_t>(grain, 1));
    if (nt <= 1) { fn((int64_t)0, n); return; }
    const int64_t chunk = std::max<int64_t>(grain, (n + nt * 4 - 1) / (nt * 4));
    std::atomic<int64_t> next{0};
    auto work = [&]() {
        for (int64_t lo; (lo = next.fetch_add(chunk)) < n;) fn(lo, std::min(n, lo + chunk));
    };
    HostPool& pool = HostPool::get();
    const int helpers = (int)std::min<int64_t>(nt - 1, pool.workers());
    if (helpers <= 0) { work(); return; }
    auto job = std::make_shared<HostPool::Job>();
    job->work = work;
    job->n = helpers;
    job->state.reset(new std::atomic<int>[(size_t)helpers]);
    for (int k = 0; k < helpers; k++) job->state[k].store(0);
    pool.submit(job);
    work();
    for (int k = 0; k < helpers; k++) {
        int expect = 0;
        job->state[k].compare_exchange_strong(expect, 3);
    }
    std::unique_lock<std::mutex> lk(job->mu);
    job->cv.wait(lk, [&] {
        for (int k = 0; k < helpers; k++)
            if (job->state[k].load() == 1) return false;
        return true;
    });
}

struct Device;   // kernels.hip
struct CovDevice;   // coverage.hip
struct GzDevice;    // inflate.hip

// Pinned host memory (kernels.hip).  Every host address a device copy reads or writes lies in a block recorded in
// one registry: pinned_alloc's blocks (a page-aligned block registered with hipHostRegister, or hipHostMalloc when
// the registration is refused) and the runtime-allocated buffers of kernels.hip / coverage.hip.  The copies check
// their host endpoint against it (dma_copy); pageable sources go through the staging buffers (DESIGN.md section 4,
// "Uploads": the runtime's pin-in-place path for pageable copies is what faulted in round 3).  With a device present
// pinned_alloc returns pinned memory or nullptr; without one (host-only code paths) plain memory.
void* pinned_alloc(size_t bytes);
void pinned_free(void* p);
bool pinned_covers(const void* p, size_t bytes);      // [p, p + bytes) inside one registered block
// a device copy whose host endpoint must be registered (kind 0: host -> device, 1: device -> host); `stream` is a
// hipStream_t, nullptr with sync = true is the synchronous hipMemcpy.  Returns 0, or -1 with err set (an
// unregistered host endpoint is an internal error, never copied).
int dma_copy(void* dst, const void* src, size_t bytes, int kind, void* stream, bool sync, std::string& err, const char* file, int line);

// Record lists backed by pinned host memory, so a D2H copy lands in place without a staging copy:
// the called sites (SingleSampleVariantPileupListener.calledVariants) and the population calls.
template <class T>
struct PinnedStore {
    T* buf = nullptr;
    size_t n = 0, cap = 0;
    PinnedStore() = default;
    PinnedStore(const PinnedStore&) = delete;
    PinnedStore& operator=(const PinnedStore&) = delete;
    ~PinnedStore() { if (buf) pinned_free(buf); }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
    void clear() { n = 0; }
    T* data() { return buf; }
    const T* data() const { return buf; }
    T& operator[](size_t i) { return buf[i]; }
    const T& operator[](size_t i) const { return buf[i]; }
    const T* begin() const { return buf; }
    const T* end() const { return buf + n; }
    void reserve(size_t want) {
        if (want <= cap) return;
        size_t nc = cap ? cap : 4096;
        while (nc < want) nc *= 2;
        auto* nb = static_cast<T*>(pinned_alloc(nc * sizeof(T)));
        if (!nb) throw std::bad_alloc();
        if (n) std::memcpy(nb, buf, n * sizeof(T));
        if (buf) pinned_free(buf);
        buf = nb;
        cap = nc;
    }
    void resize(size_t want) { reserve(want); n = want; }          // new records are not initialised
    void push_back(const T& o) { reserve(n + 1); buf[n++] = o; }
    void swap(PinnedStore& o) { std::swap(buf, o.buf); std::swap(n, o.n); std::swap(cap, o.cap); }
};
// Device -> host record of one site: 64 B, what the reference's CalledSNV keeps
// (variants/CalledSNV.java:42-45,259-265: genotype, GQ, QUAL, DP, the base counts, log-conditionals of the
// called pair, the strand-bias inputs).  A record that needs more (multi-allelic / pool calls, dump mode,
// params.full_records, counts past 65535) is whole in the set's `ext` list: is_call bit 1 set and L[0]'s bits
// hold its index there; its header fields below are filled as well.
struct SiteRec {
    int32_t seq_id;
    int32_t pos;               // KP: the global position; KO: the 1-based position
    int8_t ref, n_alleles, alt, third, genotype, strand_bias;
    int16_t gq;
    int16_t qual;
    int8_t is_call;            // bit 0: passes the listener filters; bit 1: whole record in ext; bit 2: an SNV inside
                               // a called indel (TYPE=EMBEDDED); bit 3: an indel / STR call, its VCF text in the
                               // set's `text` list (L[0]'s bits hold its index)
    uint8_t pool;
    int32_t dp;
    uint16_t counts[4];        // A,C,G,T
    uint16_t strand[4];        // reference negative / positive, alternative negative / positive
    double L[3];               // logc (ref,ref), (ref,alt), (alt,alt)
};
static_assert(sizeof(SiteRec) == 64, "site record layout");
constexpr int8_t kRecCall = 1, kRecExt = 2, kRecEmbedded = 4, kRecIndel = 8;

inline int site_tri(int i, int j) {   // index of L[i][j] in ngsep_site_out.logc
    if (i > j) std::swap(i, j);
    static const int base[4] = {0, 4, 7, 9};
    return base[i] + (j - i);
}

// the called sites of a run or a whole detector: the records (pinned: the device copies into them) and the
// whole records they point to
// One sample's call at a population site as it comes back from the device and is kept (32 B instead of the
// 76-B ngsep_sample_call): flags = kind | n_called << 1 | whole << 7, called = (c0 + 1) | (c1 + 1) << 4.  A call
// a field of which does not fit (GQ > 255, DP / counts / PL > 65535, |ACN| > 127, more than six PL values) is
// kept whole in pop_big, pl[0] | pl[1] << 16 its index.
struct PopCall32 {
    uint8_t flags, called, gq, pad0;
    int16_t total_cn;
    uint16_t dp;
    uint16_t counts[4];
    int8_t acn[4];
    uint16_t pl[6];
};
static_assert(sizeof(PopCall32) == 32, "PopCall32 layout");

inline ngsep_sample_call expand_call(const PopCall32& p, const ngsep_sample_call* big) {
    if (p.flags & 0x80) return big[(size_t)p.pl[0] | ((size_t)p.pl[1] << 16)];
    ngsep_sample_call o;
    o.kind = (int8_t)(p.flags & 1);
    o.n_called = (int8_t)((p.flags >> 1) & 3);
    o.called[0] = (int8_t)((int)(p.called & 15) - 1);
    o.called[1] = (int8_t)((int)(p.called >> 4) - 1);
    o.gq = (int16_t)p.gq;
    o.total_cn = p.total_cn;
    o.dp = (int32_t)p.dp;
    for (int k = 0; k < 4; k++) { o.counts[k] = (int32_t)p.counts[k]; o.acn[k] = (int16_t)p.acn[k]; }
    for (int k = 0; k < 10; k++) o.pl[k] = k < 6 ? (int32_t)p.pl[k] : 0;
    return o;
}

struct SiteSet {
    PinnedStore<SiteRec> rec;
    PinnedStore<ngsep_site_out> ext;
    std::vector<std::string> text;     // indel / STR records: the VCF line after the sequence name
    size_t size() const { return rec.size(); }
    bool empty() const { return rec.empty(); }
    void clear() { rec.clear(); ext.clear(); text.clear(); }
    void swap(SiteSet& o) { rec.swap(o.rec); ext.swap(o.ext); text.swap(o.text); }
    static int64_t ext_index(const SiteRec& r) { return __builtin_bit_cast(int64_t, r.L[0]); }
    // o's records after ours (ext / text indexes rebased)
    void append(const SiteSet& o) {
        if (o.empty()) return;
        const size_t from = rec.size(), ebase = ext.size(), tbase = text.size();
        rec.reserve(from + o.rec.size());
        std::memcpy(rec.buf + from, o.rec.buf, o.rec.size() * sizeof(SiteRec));
        rec.n = from + o.rec.size();
        if (!o.ext.empty()) {
            ext.reserve(ebase + o.ext.size());
            std::memcpy(ext.buf + ebase, o.ext.buf, o.ext.size() * sizeof(ngsep_site_out));
            ext.n = ebase + o.ext.size();
        }
        text.insert(text.end(), o.text.begin(), o.text.end());
        if (ebase || tbase)
            for (size_t i = from; i < rec.size(); i++) {
                if (rec[i].is_call & kRecExt) rec[i].L[0] = __builtin_bit_cast(double, ext_index(rec[i]) + (int64_t)ebase);
                else if (rec[i].is_call & kRecIndel) rec[i].L[0] = __builtin_bit_cast(double, ext_index(rec[i]) + (int64_t)tbase);
            }
    }
    // record i of o after ours (its ext / text entry copied)
    void push_from(const SiteSet& o, size_t i, int8_t extra_flags = 0) {
        SiteRec r = o.rec[i];
        if (r.is_call & kRecExt) {
            ext.push_back(o.ext[(size_t)ext_index(r)]);
            r.L[0] = __builtin_bit_cast(double, (int64_t)ext.size() - 1);
        } else if (r.is_call & kRecIndel) {
            text.push_back(o.text[(size_t)ext_index(r)]);
            r.L[0] = __builtin_bit_cast(double, (int64_t)text.size() - 1);
        }
        r.is_call = (int8_t)(r.is_call | extra_flags);
        rec.push_back(r);
    }
    // the ABI record of site i (ngsep_site_out)
    ngsep_site_out full(size_t i) const {
        const SiteRec& r = rec[i];
        ngsep_site_out o;
        if (r.is_call & kRecExt) {
            o = ext[(size_t)ext_index(r)];
        } else {
            std::memset(&o, 0, sizeof o);
            o.ref = r.ref; o.n_alleles = r.n_alleles; o.alt = r.alt; o.third = r.third; o.genotype = r.genotype;
            o.gq = r.gq; o.dp = r.dp; o.pool = r.pool;
            for (int k = 0; k < 4; k++) o.counts[k] = r.counts[k];
            int ri = 0;
            while (ri < 4 && "ACGT"[ri] != r.ref) ri++;
            if (ri < 4 && r.alt >= 0 && r.alt < 4) {
                o.strand_counts[ri][0] = r.strand[0]; o.strand_counts[ri][1] = r.strand[1];
                o.strand_counts[(int)r.alt][0] = r.strand[2]; o.strand_counts[(int)r.alt][1] = r.strand[3];
                o.logc[site_tri(ri, ri)] = r.L[0];
                o.logc[site_tri(ri, r.alt)] = r.L[1];
                o.logc[site_tri(r.alt, r.alt)] = r.L[2];
            }
        }
        if (r.is_call & kRecIndel) std::memset(&o, 0, sizeof o);   // (the record is its text)
        o.seq_id = r.seq_id; o.pos = r.pos; o.qual = r.qual; o.strand_bias = r.strand_bias;
        o.is_call = (int8_t)(r.is_call & (kRecCall | kRecEmbedded | kRecIndel));
        return o;
    }
};
using SiteStore = SiteSet;

// a read of the single-sample layout: global [gfirst, glast] and its projected bytes
struct SRead {
    int32_t gfirst, glast;
    const uint8_t* bytes;
    uint8_t neg;                        // negative strand
};

struct Staged {            // everything resident for one run
    std::vector<Window> windows;
    int64_t g_len = 0;                  // global coordinate length
    int64_t n_reads = 0, n_slots = 0, n_read_bases = 0, covered = 0;
    int32_t slot_size = 0;
    int32_t max_span = 0;
    int32_t tile = 512;                 // positions per pileup tile (T)
    int32_t tile_rows_max = 0;          // largest rows_t
    int64_t n_tiles = 0;
    int64_t pile_bytes = 0;
    // host mirrors (freed after upload)
    RawVec<int64_t> h_rdev;             // multisample: each read's bytes in the uploaded projection chunks (h_chunks): each read's projected bytes (the sequence's chunks, in place)
    std::vector<uint8_t> h_pile;
    std::vector<TileInfo> h_tinfo;
    RawVec<int32_t> h_reads;            // 4 ints per read: gfirst, glast, slot, flags
                                        //   flags: bit0 negative strand, bits 1-7 read-group rank,
                                        //   bits 8-23 sample + 1 (0: no sample) -- multisample only
    int32_t n_samples = 0;
    // the realigner's region positions (engine.cpp run_population_regions): KPM's site-major pile -- per tile of
    // kPopTile positions, position p's columns of samples 0 .. S (the reads of no sample last) back to back, each
    // rows(t, s) code bytes in getAlleleCalls order -- column (p, s) at pboff[t * (S + 1) + s] + (p % kPopTile) *
    // stride_t, stride_t = the tile's rows summed over its samples
    std::unique_ptr<uint8_t[]> h_ppile;
    std::vector<int32_t> h_prow;        // rows per (tile, sample): h_prow[t * (S + 1) + s]
    std::vector<int64_t> h_pboff;       // block offsets, same index (+ the total at the end)
    int64_t ppile_bytes = 0;
    std::vector<uint8_t> h_ref;
    // single-sample layout (engine.cpp build_single_layout): the valid-call plane, position-major byte
    // pile in pending-list rank order, strand bits of its cells -- in the context's pinned LayoutArena --
    // and the per-tile lists of other-allele call positions
    std::vector<uint16_t> h_olist;
    std::vector<int32_t> h_loff;        // tile t's entries: h_olist[h_loff[t] .. h_loff[t+1])
    uint32_t* h_planes = nullptr;
    uint8_t* h_cpile = nullptr;
    uint32_t* h_cneg = nullptr;
    bool single = false;                // the single-sample layout (else the multisample one)
    // read-group layout (engine.cpp build_rg_layout; the variant caller's device input): units in the
    // context's pinned arena, entry headers, group table and the entry index of every 256-position block:
    // blkA[b] = first entry with gfirst >= 256 b - max_span + 1 (the first that can cover the block),
    // blkB[b] = first entry with gfirst >= 256 b
    bool rg = false;
    int64_t n_entries = 0, n_groups = 0, n_units = 0;
    uint64_t* h_units = nullptr;
    bool units_pinned = true;           // h_units is the arena's pinned block (false: pageable, copied synchronously)
    // units built on the device (kernels.hip k_build_units): h_units then holds the reads' projected bytes back to
    // back (n_rbytes), entry e's from h_roff[e] (padding entries: the total)
    bool units_on_device = false;
    int64_t n_rbytes = 0;
    RawVec<int64_t> h_roff;
    // reference codes made on the device (streamed windows, kernels.hip k_ref_codes): global [ref_lo, ref_lo + ref_len)
    // from the characters at h_refchars through ref_table (engine.cpp ref_code), 0 elsewhere and on the h_zero ranges
    // (global start, length pairs)
    std::vector<std::pair<const uint8_t*, int64_t>> h_chunks;   // population: the projection chunks d_rbytes is made of
    bool ref_on_device = false;
    const char* h_refchars = nullptr;
    int64_t ref_lo = 0, ref_len = 0;
    uint8_t ref_table[256] = {};
    std::vector<int64_t> h_zero;
    RawVec<int32_t> h_rh;               // 2 per entry (every one written by the layout builders)
    std::vector<RGroup> h_grp;
    RawVec<int32_t> h_blkA, h_blkB;     // (written in full by the layout builders)
    // -knownVariants: the run genotypes these sites (KP queue entries {global position, code}: code =
    // 0x80 | ref << 5 | alt << 8 | 0x400) instead of scanning; counters preset to their number
    bool known = false;
    std::vector<int32_t> h_forced;
    unsigned long long h_forced_ctr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // the realigner's regions (realign.hpp): their queue entries carry their columns (rows >= 0), uploaded
    // here (u16 entries, h_forced_ctr[5] = their size / 4)
    std::vector<uint16_t> h_cols;
    // population read-group layout (engine.cpp build_pop_rg_layout; MultisampleVariantsDetector's device input):
    // the read-group layout above with one stream of entries per (sample, read-group rank), in (sample, rank)
    // order, the reads of no sample last; each stream's entries in pending-list order, padded to whole groups.
    // Block tables per stream: h_blkA / h_blkB[st * pnblk + b] over blocks of 2^pblk_shift positions (global entry
    // indexes); h_samp_st[s] .. h_samp_st[s + 1] = the streams of sample s (s = S: the reads of no sample);
    // h_st_end[st] = one past the stream's last entry (its padding included)
    bool prg = false;
    int32_t n_streams = 0, pblk_shift = kRgBlockShift, max_cov = 0;
    int64_t pnblk = 0;
    std::vector<int32_t> h_samp_st;
    std::vector<int64_t> h_st_end;
    // KLM tiles (kKlmTile positions) where some sample's coverage exceeds kKlmCountMaxCov: KLM's byte counters cannot
    // carry there, so those tiles take the exact-bound scan (k_scan_pop<false>) and every other tile the counting one
    std::vector<int32_t> h_deep_tiles;
};

// Pinned host buffers of the single-sample layout, reused run after run (streamed windows: no page faults,
// DMA-speed uploads).  Grown geometrically; sized by the pile bytes (valid-call plane and strand bits = / 8).
struct LayoutArena {
    uint8_t* cpile = nullptr;
    uint32_t* planes = nullptr;
    uint32_t* cneg = nullptr;
    int64_t cap = 0;
    uint64_t* units = nullptr;          // read-group layout units
    int64_t units_cap = 0;
    bool units_pinned = false;          // false: a pageable block (a layout beyond 4 GB, engine.cpp ensure_units)
    bool ensure(int64_t pile_bytes, bool exact);
    bool ensure_units(int64_t n_units, bool exact);
    void release();
    ~LayoutArena() { release(); }
};

// One streamed window of a sequence (single-sample calls while the alignments are still being read,
// engine.cpp stream_advance): its reads in window coordinates and the carved indel regions inside it,
// laid out, uploaded and run on the context's worker thread; its records come back in `sites`.
struct WindowJob {
    int32_t seq_id = -1;
    int64_t w0 = 0, w1 = 0;
    int32_t max_span = 1;
    RawVec<SRead> reads;                                    // global coordinates (window at pad)
    std::vector<std::pair<int64_t, int64_t>> carved;        // 1-based, inside [w0, w1]
    // the indel realigner's regions (whole inside the window, = carved) and their alignments; the listener's
    // lastIndelEnd before and after the window
    bool realign = false;
    std::vector<std::vector<RawRead>> region_reads;
    int32_t last_indel_end = 0;
    std::vector<int32_t> forced;                            // -knownVariants: KP queue entries (global position, code)
    SiteStore sites;
    // RelativeAlleleCounts mode: the window's histograms and proportion sums; its sequence's slot in the
    // per-sequence distributions (-1: a sequence of <= 100000 bp)
    unsigned long long rac_hist[61] = {};
    double rac_sum = 0, rac_sum_sq = 0;
    int32_t rac_seq_slot = -1;
    int rc = 0;
    std::string err;
    std::atomic<bool> done{false};
    std::thread th;
};

}  // namespace ngsep

struct ngsep_ctx {
    ngsep_params params;
    int device = 0;
    std::string err;
    double het_rate = 0.001;
    // compute_tables cache of the staged-run entry points (keyed by the options)
    bool tables_cached = false;
    ngsep_params tables_params{};
    double tables_het = 0;
    ngsep::LikTables tables_t{};
    ngsep::GenotypeParams tables_gp{};
    // reference
    std::vector<std::string> seq_names;
    std::vector<std::string> seq_bases;      // case kept, masked to AaCcNngGtT
    // admission sweep state
    int32_t cur_seq = -1;
    int32_t last_start = 0;
    int32_t cur_last = 0;
    std::vector<ngsep::ReadView> ss_primary, ss_secondary;   // the open same-start group
    ngsep::CarryStore carry[2];                               // its reads' bytes across batches
    int carry_cur = 0;
    // admitted reads whose projection is pending (batch end): >= 0 an index in the current batch,
    // < 0 entry -1 - k of to_project_carried
    std::vector<int32_t> to_project;
    std::vector<ngsep::ReadView> to_project_carried;
    ngsep::BatchRef cur_batch;
    int32_t ss_one = -1;                                     // the open group's only read, by batch index (or -1)
    std::vector<ngsep::HostArray<uint8_t>> chunk_pool;       // released projection chunks, reused
    ngsep::ContigReads contig;
    bool query_found = false;
    bool query_done = false;
    bool staging_mode = false;
    // windows collected for a staged run
    std::vector<ngsep::ContigReads> staged_contigs;
    ngsep::Staged staged;
    ngsep::LayoutArena arena;
    // -knownVariants (ngsep_set_known_variants): the input variants to genotype instead of discovering, in
    // GenomicRegionSortedCollection order (sequence, first, last; input order at equal keys).  A biallelic SNV has
    // ref / alt DNA codes; any other record alt = -1 and its alleles in known_recs[rec] (genotyped on the host, in the
    // realigner's regions); type: its INFO TYPE id
    struct KnownVar { int32_t seq, pos, last; int8_t ref, alt, type; int16_t qs; int32_t rec; std::string id; };
    std::vector<KnownVar> known;
    std::vector<ngsep::KnownRecord> known_recs;
    std::vector<int64_t> known_seq_begin;                    // per sequence: first entry (size n_seq + 1)
    bool known_given = false;                                // a -knownVariants file was set (its -knownSTRs are ignored)
    // the indel realigner's input variants per sequence (IndelRealignerPileupListener.setInputVariants): the known
    // variants when given, else the -knownSTRs (ngsep_set_known_strs); str_next: the next event of the current
    // sequence to enter its realigner regions (engine.cpp inject_strs)
    std::vector<ngsep::InputVars> strs;
    size_t str_next = 0;
    // path B: the alignments the BAM is expected to hold (its size / 40 B, an upper estimate); a sequence's read
    // arrays reserve their share up front (virtual memory, touched only as they fill: no regrowth copies)
    int64_t reads_hint = 0;
    // known_at: the position written; last_seq: the sequence of the last record written (the first record of a sequence
    // is the one intersectVariantsCNVs updates, SingleSampleVariantsDetector.java:969-991)
    mutable struct { int32_t seq = -1, pos = -1, last_seq = -1; std::vector<int64_t> taken; } vcf_known;
    // RelativeAlleleCountsCalculator mode (params.relative_allele_counts): its Distributions
    struct {
        double prop[51] = {}, prop_count = 0, prop_sum = 0, prop_sum_sq = 0;
        double nall[10] = {}, nall_count = 0, nall_sum = 0, nall_sum_sq = 0;
        std::vector<std::string> seq_names;                  // sequences longer than 100000 bp, in order
        std::vector<std::vector<double>> seq_prop;           // their proportion bins
        int32_t cur_slot = -1;                               // the current sequence's slot
        double kernel_ms = 0;
    } rac;
    // streamed single-sample windows of the current sequence (run_now paths)
    struct {
        int64_t next_w0 = 0;                      // first position not yet handed to a window (0: not started)
        size_t indel_lo = 0;                      // indel reads before this index reach no later window
        size_t chunk_lo = 0;                      // projected chunks before this index are released
        int64_t carved_inside = 0;                // covered positions inside carved regions (this sequence)
        // the indel realigner (params.indel_passthrough = 0): admitted alignments kept for its regions' replays --
        // those inside a known region's reach and those a later indel read could still reach (`maybe`)
        struct Kept { int32_t first, last; bool maybe, dead; ngsep::RawRead r; };
        std::vector<Kept> kept;
        size_t kept_maybe_from = 0;               // entries before this one are not `maybe`
        std::vector<int32_t> indel_pmax;          // running max of indel_reads[k].second (the regions' ends)
        int32_t last_indel_end = 0;               // SingleSampleVariantPileupListener.lastIndelEnd (this sequence)
        std::unique_ptr<ngsep::WindowJob> job;    // in flight on its own thread
        int64_t windows = 0;                      // windows run (diagnostics)
    } stream;
    ngsep::Device* dev = nullptr;
    // path B: BGZF blocks inflated on the device (inflate.hip) by the single-sample readers of this context, one
    // reader at a time (gz_busy); pinned input / decoded-chunk buffers (pointer, capacity) kept across readers
    ngsep::GzDevice* gz = nullptr;
    std::atomic<bool> gz_busy{false};
    std::vector<std::pair<void*, size_t>> gz_in_pool, gz_chunk_pool;
    // path B: the device is created on a thread of its own while the input is read (start_device_init), adopted
    // by the first device step (ensure_device)
    std::thread dev_init;
    ngsep::Device* dev_init_result = nullptr;
    std::string dev_init_err;
    std::mutex dev_mu;
    // CoverageStatisticsCalculator mode (params.coverage_stats)
    ngsep::CovDevice* cov_dev = nullptr;
    bool cov_staged = false;
    std::vector<uint64_t> cov_hist;          // 2 x (max_coverage + 1), accumulated over runs
    // multisample (ngsep_set_samples)
    std::vector<std::string> sample_ids;
    std::vector<int32_t> rg_sample, rg_rank;
    std::vector<int8_t> sample_nrank;        // read groups per sample
    // outputs
    ngsep::SiteStore sites;
    // regions around indel-bearing alignments the device path did not call (the indel realigner's reach,
    // ngsep_fetch_carved_regions): (sequence, first, last), 1-based inclusive, in processing order
    std::vector<std::pair<int32_t, std::pair<int64_t, int64_t>>> carved;
    int pending_sync = 0;                         // multisample runs submitted, not yet collected
    std::vector<ngsep_popsite_out> pop_sites;     // (sequence, position) order
    ngsep::PinnedStore<ngsep::PopCall32> pop_calls;     // pop_sites.size() x n_samples (compact; expand_call)
    ngsep::PinnedStore<ngsep_sample_call> pop_big;      // the calls a PopCall32 cannot hold, whole
    std::vector<int64_t> pop_order;                     // site i's calls: pop_calls[pop_order[i] * n_samples ..]
                                                        // (an indel / STR record, multisnv_type 3: pop_text[pop_order[i]])
    std::vector<std::string> pop_text;                  // indel / STR population records (realigner regions), no sequence name
    ngsep_stats stats{};
    std::atomic<int64_t> realign_ns{0}, realign_regions{0};   // region replays (worker threads): stats.realign_*
    std::atomic<int64_t> keep_raw_ns{0}, region_setup_ns{0}, region_device_ns{0}, region_merge_ns{0}, window_wait_ns{0}, region_gather_ns{0};   // stats
};

namespace ngsep {
// engine.cpp
int set_error(ngsep_ctx* c, int code, const std::string& msg);
// ngsep_process_alignments for a batch in BAM encoding (ReadView::packed; bam.cpp's call_bam)
int process_alignments_packed(ngsep_ctx* c, const PackedBatch* b);
// ngsep_process_alignments for a batch whose reads' bytes stay in their own files' batches (bam.cpp's population
// merge): read i's bases at chars_at[i], its qualities at quals_at[i] (b->bases / quals / seq_off unused)
int process_alignments_gathered(ngsep_ctx* c, const ngsep_read_batch* b, const char* const* chars_at, const char* const* quals_at);
void project_read(const ngsep_ctx* c, const ReadView& r, uint8_t* out);
int stage_contig_reads(ngsep_ctx* c, ContigReads& cr, bool run_now);
int build_and_upload(ngsep_ctx* c, std::vector<ContigReads>& contigs, bool release_chunks);
int run_device_into(ngsep_ctx* c, SiteStore& dest, double* elapsed_ms);
int run_device(ngsep_ctx* c, double* elapsed_ms);
void compute_tables(const ngsep_ctx* c, LikTables* t, GenotypeParams* g);
int prepare_pool(ngsep_ctx* c);
int64_t java_round(double x);
// kernels.hip
Device* device_create(int ordinal, std::string& err);
void start_device_init(ngsep_ctx* c);            // engine.cpp
Device* ensure_device(ngsep_ctx* c, std::string& err);
void device_destroy(Device* d);
int device_upload(Device* d, const Staged& s, std::string& err);
// runs the tile + posterior kernels and copies the position-ordered records into out->buf[out->n ...]
int device_run(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune,
               SiteStore* out, int64_t* n_out, double* scan_ms, double* geno_ms, double* total_ms,
               int64_t* n_candidates, std::string& err);
void device_release(Device* d);
// ploidy >= 3: the pool algorithm's tables for the next runs (uploaded when they change; NULL: unchanged)
int device_set_pool(Device* d, const PoolTables* pt, std::string& err);
// asynchronous single-sample runs (two result slots): submit enqueues kernels and copies; collect
// waits for the oldest run (an overflowed run is grown and re-run in place)
int device_submit(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g, int prune, std::string& err);
int device_collect(Device* d, SiteStore* out, int64_t* n_out, double* scan_ms, double* geno_ms, double* total_ms,
                   int64_t* n_candidates, std::string& err);
int64_t device_inflight(const Device* d);
// multisample: scan over the candidate columns + population genotyping of the queued positions; the
// sites (global positions, unordered) and their calls (n_samples per site) in the device's pinned
// staging buffers, valid until the next run
// the kept sites' calls gathered into output order and packed on the device (dst: m x S PopCall32; the calls that
// do not fit are appended whole to big, the records index it from big->size())
int device_fetch_calls_ordered(Device* d, const int64_t* src, int64_t m, PopCall32* dst, PinnedStore<ngsep_sample_call>* big, std::string& err);
int device_submit_multi(Device* d, const LikTables& t, const GenotypeParams& g, int32_t n_samples, double min_adf,
                        int ploidy, std::string& err);
int device_collect_multi(Device* d, const ngsep_popsite_out** sites, int64_t* n_sites, int* slot, bool* rerun,
                         double* scan_ms, double* geno_ms, int64_t* n_candidates, std::string& err);
// the collected slot's packed calls (KPM's site order) and whole records handed over to the context's stores (the
// buffers are swapped, nothing is copied)
void device_slot_take(Device* d, int slot, int64_t n_sites, PinnedStore<PopCall32>& calls, PinnedStore<ngsep_sample_call>& big);
int device_multi_inflight(const Device* d);
int device_run_multi(Device* d, const Staged& s, const LikTables& t, const GenotypeParams& g,
                     int32_t n_samples, double min_adf, int ploidy,
                     const ngsep_popsite_out** sites, const ngsep_sample_call** calls, int64_t* n_sites,
                     double* scan_ms, double* geno_ms, double* total_ms, int64_t* n_candidates, std::string& err);
// RelativeAlleleCountsCalculator over positions [g0, g1) of the resident single-sample layout: hist_out[0..51)
// the proportion bins, [51..61) the number-of-alleles bins; the proportion's sum and sum of squares
int device_run_rac(Device* d, const Staged& s, int64_t g0, int64_t g1, int32_t min_rd, int32_t min_bq,
                   unsigned long long* hist_out, double* sum, double* sum_sq, double* kernel_ms, std::string& err);
int64_t device_last_hard(const Device* d);
int64_t device_last_exact(const Device* d);
int device_count();
// coverage.hip
CovDevice* cov_create(int ordinal, std::string& err);
void cov_release(CovDevice* d);
void cov_destroy(CovDevice* d);
int cov_upload(CovDevice* d, const std::vector<int64_t>& gfirst, const std::vector<uint32_t>& spanu, int64_t g_len,
               int32_t max_span, std::string& err);
int cov_run(CovDevice* d, int32_t max_cov, uint64_t* hist_out, double* kernel_ms, std::string& err);
// inflate.hip: BGZF blocks inflated on the device (bam.cpp's decoder; two slots in flight)
struct GzDevice;
GzDevice* gz_create(int ordinal, std::string& err);
void gz_destroy(GzDevice* d);
int gz_wave_blocks(const GzDevice* d);          // blocks a batch should hold at most (one wave of workgroups)
void* gz_host_alloc(size_t n);                   // pinned host memory
void gz_host_free(void* p);
int gz_submit(GzDevice* d, int slot, const uint8_t* in, size_t in_n, const size_t* boff, const size_t* bclen,
              const uint32_t* bisize, const size_t* dout, size_t nb, uint8_t* out, size_t out_n, std::string& err);
int gz_wait(GzDevice* d, int slot, std::string& err);
// engine.cpp
int coverage_stage(ngsep_ctx* c, std::vector<ContigReads>& contigs);
int coverage_run(ngsep_ctx* c, double* kernel_ms);
// engine.cpp: the ID of a -knownVariants record's input variant (nullptr: '.')
const ngsep_ctx::KnownVar* known_of(const ngsep_ctx* c, const ngsep_site_out& s);
const ngsep_ctx::KnownVar* known_at(const ngsep_ctx* c, int32_t seq_id, int32_t pos, int alt);
// vcf.cpp
std::string format_header(const ngsep_ctx* c);
int64_t format_site(const ngsep_ctx* c, const ngsep_site_out& s, std::string& out, bool first_of_seq);
std::string format_population_header(const ngsep_ctx* c);
void format_population_site(const ngsep_ctx* c, const ngsep_popsite_out& s, const ngsep_sample_call* calls, std::string& out);
// bam.cpp
int call_bam(ngsep_ctx* c, const char* bam_path, const char* out_vcf);
}  // namespace ngsep
