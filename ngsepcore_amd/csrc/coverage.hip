// coverage.hip -- CoverageStatisticsCalculator on gfx950 (discovery/CoverageStatisticsCalculator.java:108-216).
//
// The reference listener bins, for every pileup the generator emits, PileupRecord.getNumAlignments() and
// getNumUniqueAlns() (PileupRecord.java:154-177) into coverageCounts[0, maxCoverage) + "More".  Both counts
// are interval depths over the admitted alignments [first, last], so no allele call is touched: the device
// sees 12 bytes per admitted read (global first position, span and the unique bit) and the positions are
// implicit.
//
// Layout: admitted reads of all sequences in one global coordinate (sequence regions back to back),
// ascending first position (pending order).  Positions are cut into tiles (index: 4096 positions).
//   KCI kc_tile_index : tstart[t] = first read whose tile(first) >= t           (one thread per read)
//   KCH kc_tile_hist  : persistent workgroups over tiles of 4096 positions: the reads that can overlap the tile (tiles back to
//                       lo_tile = tile(t0 - max_span + 1)) add +/-(1 | unique << 32) to an LDS
//                       difference array, a workgroup prefix sum turns it into packed (depth, unique
//                       depth) per position (modular u64 arithmetic: the packed sums are exact because
//                       every final depth is >= 0 and < 2^32), and run-length-compressed LDS histogram
//                       updates bin both depths in LDS; each workgroup flushes its bins with global atomics once.
// HBM traffic: 12 B per read (+ the lookback of one tile of reads) and the histogram; the kernel is bound
// by its LDS work (atomics + scan over the tile's positions) and load latency, not by HBM.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdint>
#include <climits>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>
#include "engine.hpp"

namespace ngsep {

constexpr int kCovLog2Tile = 12;                     // tile index granularity (KCI) = the largest tile
constexpr int kCovThreads = 256;                     // 4 wavefronts
constexpr int kCovMaxBins = 1024;                    // largest maxCoverage: 4 private bin sets + 16 KB <= 64 KB LDS

#define COV_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            err = std::string(#expr) + ": " + hipGetErrorString(e_);                   \
            return -1;                                                                 \
        }                                                                              \
    } while (0)

struct CovDevice {
    int ordinal = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev[2] = {};
    int64_t* d_gfirst = nullptr;      // global first position per read (ascending)
    uint32_t* d_spanu = nullptr;      // span << 1 | unique
    int64_t* d_tstart = nullptr;      // n_tiles + 1
    unsigned long long* d_hist = nullptr;   // 2 x (max_cov + 1): depth bins, unique-depth bins (index max_cov = More)
    int64_t n_reads = 0, g_len = 0, n_tiles = 0;
    int32_t max_span = 1;
    int32_t hist_cap = 0;
    int32_t n_cu = 256;
};

// KCI: tile start index of the read list (tiles with no read starting in them point at the next read)
__global__ void kc_tile_index(const int64_t* __restrict__ gfirst, int64_t n, int64_t n_tiles, int64_t* __restrict__ tstart) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const int64_t tp = i == 0 ? -1 : (gfirst[i - 1] >> kCovLog2Tile);
    const int64_t tc = i == n ? n_tiles : (gfirst[i] >> kCovLog2Tile);
    for (int64_t t = tp + 1; t <= tc; t++) tstart[t] = i;
}

// KCH: persistent workgroups, each walks tiles of 2^LOG2T positions with a grid stride (LOG2T <=
// kCovLog2Tile; the read range comes from the 4096-position index).  Histogram bins live in LDS for the
// workgroup's whole life, private per wavefront (4 copies: the run-length updates of different waves never
// hit the same LDS word), and are summed and flushed to the global histogram once at the end -- measured:
// zeroing and flushing the bins per tile cost more than the tile's own work (71-125 us vs 4096/2048-position
// workgroup-per-tile launches on the yeast 30x genome).
template <int LOG2T>
__global__ void __launch_bounds__(kCovThreads)
kc_tile_hist(const int64_t* __restrict__ gfirst, const uint32_t* __restrict__ spanu, const int64_t* __restrict__ tstart,
             int64_t g_len, int64_t n_tl, int32_t max_span, int32_t max_cov, unsigned long long* __restrict__ hist) {
    constexpr int T = 1 << LOG2T;
    constexpr int PER = T / kCovThreads;               // consecutive positions per thread
    __shared__ unsigned long long diff[T + 1];
    __shared__ unsigned long long wave_tot[kCovThreads / 64];
    extern __shared__ uint32_t bins[];                 // 4 waves x 2 x (max_cov + 1)
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int nb = 2 * (max_cov + 1);
    uint32_t* wb = bins + wave * nb;
    for (int k = tid; k < 4 * nb; k += kCovThreads) bins[k] = 0u;
    // read range of a tile: reads whose first lies in [t0 - max_span + 1, t0 + T)
    auto range = [&](int64_t t, int64_t& r0, int64_t& r1) {
        const int64_t t0 = t << LOG2T;
        const int64_t lo_pos = t0 - (int64_t)max_span + 1;
        const int64_t lo_tile = lo_pos <= 0 ? 0 : (lo_pos >> kCovLog2Tile);
        r0 = tstart[lo_tile];
        r1 = tstart[((t0 + T - 1) >> kCovLog2Tile) + 1];
    };
    int64_t r0 = 0, r1 = 0;
    if ((int64_t)blockIdx.x < n_tl) range(blockIdx.x, r0, r1);
    for (int64_t t = blockIdx.x; t < n_tl; t += gridDim.x) {
        const int64_t t0 = t << LOG2T;
        // this tile's reads in flight in batches of kCovBatch per thread (independent loads), and the next
        // tile's range, before the LDS work
        constexpr int kCovBatch = 4;
        int64_t f[kCovBatch];
        uint32_t su[kCovBatch];
        int64_t r = r0 + tid;
#pragma unroll
        for (int j = 0; j < kCovBatch; j++) {
            const int64_t rj = r + (int64_t)j * kCovThreads;
            f[j] = rj < r1 ? gfirst[rj] : INT64_MAX;
            su[j] = rj < r1 ? spanu[rj] : 0u;
        }
        const int64_t cur1 = r1;
        if (t + gridDim.x < n_tl) range(t + gridDim.x, r0, r1);
        for (int k = tid; k <= T; k += kCovThreads) diff[k] = 0ull;
        __syncthreads();
        while (true) {
#pragma unroll
            for (int j = 0; j < kCovBatch; j++) {
                if (f[j] >= t0 + T) continue;          // past the tile (the index is coarser) or no read
                const int64_t l = f[j] + (int64_t)(su[j] >> 1) - 1;
                if (l < t0) continue;
                const unsigned long long inc = 1ull | ((unsigned long long)(su[j] & 1u) << 32);
                const int64_t a = (f[j] > t0 ? f[j] : t0) - t0;
                const int64_t b = l + 1 - t0;
                atomicAdd(&diff[a], inc);
                if (b < T) atomicAdd(&diff[b], 0ull - inc);
            }
            r += (int64_t)kCovBatch * kCovThreads;
            if (r >= cur1) break;                      // deep tiles: the next batch
#pragma unroll
            for (int j = 0; j < kCovBatch; j++) {
                const int64_t rj = r + (int64_t)j * kCovThreads;
                f[j] = rj < cur1 ? gfirst[rj] : INT64_MAX;
                su[j] = rj < cur1 ? spanu[rj] : 0u;
            }
        }
        __syncthreads();
        // workgroup prefix sum: PER consecutive positions per thread, wavefront scan of the thread sums
        const int base = tid * PER;
        unsigned long long v[PER];
        unsigned long long s = 0;
#pragma unroll
        for (int k = 0; k < PER; k++) { s += diff[base + k]; v[k] = s; }
        unsigned long long inc_scan = s;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const unsigned long long o = __shfl_up(inc_scan, d, 64);
            if (lane >= d) inc_scan += o;
        }
        if (lane == 63) wave_tot[wave] = inc_scan;
        __syncthreads();
        unsigned long long carry = inc_scan - s;
        for (int w = 0; w < wave; w++) carry += wave_tot[w];
        // histogram with run-length compression (depth changes only at read ends)
        const int64_t p_end = g_len - t0;              // positions of this tile inside the coordinate space
        uint32_t run_d = 0xffffffffu, run_u = 0xffffffffu, cnt_d = 0, cnt_u = 0;
#pragma unroll
        for (int k = 0; k < PER; k++) {
            if (base + k >= p_end) continue;           // (no break: the loop stays unrolled, v[] in registers)
            const unsigned long long pk = v[k] + carry;
            uint32_t dd = (uint32_t)pk, du = (uint32_t)(pk >> 32);
            dd = dd < (uint32_t)max_cov ? dd : (uint32_t)max_cov;
            du = du < (uint32_t)max_cov ? du : (uint32_t)max_cov;
            if (dd != run_d) { if (cnt_d) atomicAdd(&wb[run_d], cnt_d); run_d = dd; cnt_d = 0; }
            if (du != run_u) { if (cnt_u) atomicAdd(&wb[max_cov + 1 + run_u], cnt_u); run_u = du; cnt_u = 0; }
            cnt_d++;
            cnt_u++;
        }
        if (cnt_d) atomicAdd(&wb[run_d], cnt_d);
        if (cnt_u) atomicAdd(&wb[max_cov + 1 + run_u], cnt_u);
        __syncthreads();                               // diff and wave_tot are reused by the next tile
    }
    __syncthreads();                                   // (a workgroup without tiles: the zeroed bins)
    for (int k = tid; k < nb; k += kCovThreads) {
        const unsigned long long c = (unsigned long long)bins[k] + bins[nb + k] + bins[2 * nb + k] + bins[3 * nb + k];
        if (c) atomicAdd(&hist[k], c);
    }
}

CovDevice* cov_create(int ordinal, std::string& err) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        err = "no HIP device available (libngsep_amd requires an MI355X / gfx950 GPU)";
        return nullptr;
    }
    if (ordinal < 0 || ordinal >= n) { err = "device ordinal out of range"; return nullptr; }
    if (hipSetDevice(ordinal) != hipSuccess) { err = "hipSetDevice failed"; return nullptr; }
    CovDevice* d = new CovDevice();
    d->ordinal = ordinal;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, ordinal) == hipSuccess && prop.multiProcessorCount > 0) d->n_cu = prop.multiProcessorCount;
    }
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) { err = "stream"; delete d; return nullptr; }
    for (auto& e : d->ev) (void)hipEventCreate(&e);
    return d;
}

void cov_release(CovDevice* d) {
    if (!d) return;
    (void)hipSetDevice(d->ordinal);
    (void)hipStreamSynchronize(d->stream);
    (void)hipFree(d->d_gfirst); d->d_gfirst = nullptr;
    (void)hipFree(d->d_spanu); d->d_spanu = nullptr;
    (void)hipFree(d->d_tstart); d->d_tstart = nullptr;
    d->n_reads = d->g_len = d->n_tiles = 0;
}

void cov_destroy(CovDevice* d) {
    if (!d) return;
    cov_release(d);
    (void)hipFree(d->d_hist);
    for (auto& e : d->ev) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(d->stream);
    delete d;
}

int cov_upload(CovDevice* d, const std::vector<int64_t>& gfirst, const std::vector<uint32_t>& spanu, int64_t g_len,
               int32_t max_span, std::string& err) {
    cov_release(d);
    COV_TRY(hipSetDevice(d->ordinal));
    const int64_t n = (int64_t)gfirst.size();
    if ((int64_t)spanu.size() != n) { err = "coverage read arrays differ in length"; return -1; }
    for (int64_t i = 1; i < n; i++)
        if (gfirst[i] < gfirst[i - 1]) { err = "coverage reads not in ascending global order"; return -1; }
    if (n && (gfirst[0] < 0 || gfirst[n - 1] >= g_len)) { err = "coverage read outside the coordinate space"; return -1; }
    d->n_reads = n;
    d->g_len = g_len;
    d->n_tiles = (g_len + (1 << kCovLog2Tile) - 1) >> kCovLog2Tile;
    d->max_span = max_span > 0 ? max_span : 1;
    COV_TRY(hipMalloc(&d->d_gfirst, sizeof(int64_t) * (size_t)(n > 0 ? n : 1)));
    COV_TRY(hipMalloc(&d->d_spanu, sizeof(uint32_t) * (size_t)(n > 0 ? n : 1)));
    COV_TRY(hipMalloc(&d->d_tstart, sizeof(int64_t) * (size_t)(d->n_tiles + 1)));
    if (n) {
        // (no copy's host side is pageable memory, kernels.hip "pinned host memory": the arrays go through a
        // pinned block)
        const size_t bg = sizeof(int64_t) * (size_t)n, bs = sizeof(uint32_t) * (size_t)n;
        uint8_t* h = static_cast<uint8_t*>(pinned_alloc(bg + bs));
        if (!h) { err = "pinned allocation failed"; return -1; }
        std::memcpy(h, gfirst.data(), bg);
        std::memcpy(h + bg, spanu.data(), bs);
        int rc = dma_copy(d->d_gfirst, h, bg, 0, d->stream, false, err, "coverage.hip", __LINE__);
        if (rc == 0) rc = dma_copy(d->d_spanu, h + bg, bs, 0, d->stream, false, err, "coverage.hip", __LINE__);
        const hipError_t e = hipStreamSynchronize(d->stream);
        pinned_free(h);
        if (rc != 0) return -1;
        COV_TRY(e);
    }
    const int64_t blocks = (n + 1 + 255) / 256;
    kc_tile_index<<<dim3((unsigned)blocks), dim3(256), 0, d->stream>>>(d->d_gfirst, n, d->n_tiles, d->d_tstart);
    COV_TRY(hipGetLastError());
    COV_TRY(hipStreamSynchronize(d->stream));
    return 0;
}

// one pass over the uploaded reads: hist_out[0 .. max_cov] = depth bins (max_cov = More),
// hist_out[max_cov + 1 .. 2 max_cov + 1] = unique-depth bins
int cov_run(CovDevice* d, int32_t max_cov, uint64_t* hist_out, double* kernel_ms, std::string& err) {
    if (max_cov < 1 || max_cov > kCovMaxBins) { err = "maxCoverage outside [1, 1024]"; return -1; }
    COV_TRY(hipSetDevice(d->ordinal));
    const int nb = 2 * (max_cov + 1);
    if (nb > d->hist_cap) {
        (void)hipFree(d->d_hist);
        d->d_hist = nullptr;
        COV_TRY(hipMalloc(&d->d_hist, sizeof(unsigned long long) * (size_t)nb));
        d->hist_cap = nb;
    }
    COV_TRY(hipMemsetAsync(d->d_hist, 0, sizeof(unsigned long long) * (size_t)nb, d->stream));
    float ms = 0.f;
    if (d->n_tiles > 0) {
        if (d->n_tiles > 0x7fffffff) { err = "coordinate space too large for one launch"; return -1; }
        // tile width 4096 (NGSEP_COV_TILE=2048 selects the narrow tile, diagnostics); as many workgroups as are
        // co-resident, each walking tiles with a grid stride
        const size_t lds = sizeof(uint32_t) * 4 * (size_t)nb;
        static const bool narrow_env = diag_env("NGSEP_COV_TILE") && std::atoi(diag_env("NGSEP_COV_TILE")) == 2048;
        const bool narrow = narrow_env || lds > 32768;
        const int64_t ntl = narrow ? (d->g_len + 2047) >> 11 : d->n_tiles;
        int per_cu = 0;
        if (narrow) COV_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kc_tile_hist<11>, kCovThreads, lds));
        else COV_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kc_tile_hist<12>, kCovThreads, lds));
        const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(ntl, (int64_t)d->n_cu * std::max(1, per_cu)));
        if (narrow)
            hipExtLaunchKernelGGL(kc_tile_hist<11>, dim3((unsigned)grid), dim3(kCovThreads), lds, d->stream, d->ev[0], d->ev[1],
                                  0, d->d_gfirst, d->d_spanu, d->d_tstart, d->g_len, ntl, d->max_span, max_cov, d->d_hist);
        else
            hipExtLaunchKernelGGL(kc_tile_hist<12>, dim3((unsigned)grid), dim3(kCovThreads), lds, d->stream, d->ev[0], d->ev[1],
                                  0, d->d_gfirst, d->d_spanu, d->d_tstart, d->g_len, ntl, d->max_span, max_cov, d->d_hist);
        COV_TRY(hipGetLastError());
    }
    {
        const size_t bytes = sizeof(unsigned long long) * (size_t)nb;
        void* h = pinned_alloc(bytes);
        if (!h) { err = "pinned allocation failed"; return -1; }
        const int rc = dma_copy(h, d->d_hist, bytes, 1, d->stream, false, err, "coverage.hip", __LINE__);
        const hipError_t e = hipStreamSynchronize(d->stream);
        if (rc == 0 && e == hipSuccess) std::memcpy(hist_out, h, bytes);
        pinned_free(h);
        if (rc != 0) return -1;
        COV_TRY(e);
    }
    if (d->n_tiles > 0) COV_TRY(hipEventElapsedTime(&ms, d->ev[0], d->ev[1]));
    if (kernel_ms) *kernel_ms = ms;
    return 0;
}

}  // namespace ngsep
