// bam.cpp -- BGZF/BAM decoding with ReadAlignmentFileReader's record semantics
// (alignments/io/ReadAlignmentFileReader.java:171-354).  htsjdk (lib/htsjdk-2.22.jar) plays this
// role in the reference; this reader reproduces the fields NGSEP takes from it:
//   getAlignmentStart/End, getFlags, getMappingQuality, CIGAR, getReadString
//   ("=ACMGRSVTWYHKDBN" decoding), getBaseQualityString (0xFF -> "*"), RG (header lookup), NH.
// Reader filters: consecutive duplicates (isSameAlignment :292-306), FLAG_MULTIPLE_ALN (:284-291),
// unmapped/secondary/multiple filter flags (AlignmentsPileupGenerator.java:363-375).
//
// Host pipeline: a decoder thread reads the compressed file in 32 MB chunks,
// inflates their BGZF blocks on all host threads (libdeflate through dlopen when the image has it, zlib
// otherwise) and hands the decoded bytes over a bounded queue; ngsep_bam_next_batch cuts the records
// (one pass over the block_size chain) and decodes them into the batch arrays in parallel.  A BAI index
// (path.bai, SAM spec 5.2) gives random access: ngsep_bam_set_region seeks to the first chunk of a
// region (ngsep_call_region_bam, the sharded callers).
#include <dlfcn.h>
#include <zlib.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "engine.hpp"

namespace {

// raw-deflate decompression of one BGZF block: libdeflate when present (dlopen, ~2-3x zlib), zlib otherwise
struct Inflater {
    void* (*alloc)() = nullptr;
    int (*decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
    void (*release)(void*) = nullptr;
    Inflater() {
        if (ngsep::env_hook("NGSEP_ZLIB")) return;     // diagnostics: force zlib
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
        decompress = (int (*)(void*, const void*, size_t, void*, size_t, size_t*))dlsym(h, "libdeflate_deflate_decompress");
        release = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
        if (!alloc || !decompress || !release) alloc = nullptr;
    }
    static const Inflater& get() { static Inflater i; return i; }
    // inflates in[0, n) into exactly out_n bytes
    bool run(const uint8_t* in, size_t n, uint8_t* out, size_t out_n) const {
        if (alloc) {
            thread_local struct D { void* d = nullptr; ~D() { if (d) Inflater::get().release(d); } } dd;
            if (!dd.d) dd.d = alloc();
            size_t got = 0;
            return decompress(dd.d, in, n, out, out_n, &got) == 0 && got == out_n;
        }
        z_stream z{};
        if (inflateInit2(&z, -15) != Z_OK) return false;
        z.next_in = const_cast<Bytef*>(in);
        z.avail_in = (uInt)n;
        z.next_out = out;
        z.avail_out = (uInt)out_n;
        const int rc = inflate(&z, Z_FINISH);
        inflateEnd(&z);
        return rc == Z_STREAM_END && z.total_out == out_n;
    }
};

// growable array without value-initialisation (batch and chunk buffers are overwritten in parallel); pinned: page-locked
// host memory (gz_host_alloc) the device inflate copies into and out of at the link's rate
template <class T>
struct RawBuf {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    bool pinned = false;
    RawBuf() = default;
    RawBuf(const RawBuf&) = delete;
    RawBuf& operator=(const RawBuf&) = delete;
    RawBuf(RawBuf&& o) noexcept : p(o.p), n(o.n), cap(o.cap), pinned(o.pinned) { o.p = nullptr; o.n = o.cap = 0; }
    RawBuf& operator=(RawBuf&& o) noexcept {
        std::swap(p, o.p); std::swap(n, o.n); std::swap(cap, o.cap); std::swap(pinned, o.pinned);
        return *this;
    }
    ~RawBuf() { release(); }
    void release() {
        if (pinned) ngsep::gz_host_free(p);
        else std::free(p);
        p = nullptr;
        n = cap = 0;
    }
    // takes over a pinned allocation (p, cap)
    void adopt_pinned(void* q, size_t c) { release(); p = static_cast<T*>(q); cap = c / sizeof(T); pinned = true; }
    void resize(size_t k) {
        if (k > cap) {
            const size_t c = std::max(k, cap + cap / 2);
            T* q = static_cast<T*>(pinned ? ngsep::gz_host_alloc(c * sizeof(T)) : ngsep::huge_alloc(c * sizeof(T)));
            if (!q) throw std::bad_alloc();
            if (n) std::memcpy(q, p, n * sizeof(T));
            if (pinned) ngsep::gz_host_free(p);
            else std::free(p);
            p = q;
            cap = c;
        }
        n = k;
    }
    T* data() { return p; }
    T& operator[](size_t i) { return p[i]; }
};

constexpr size_t kChunkHead = (size_t)4 << 20;   // headroom before a chunk's bytes for the previous chunk's tail

struct Chunk {                 // decoded bytes of whole BGZF blocks at mem.p + kChunkHead
    RawBuf<uint8_t> mem;
    size_t len = 0;
    bool eof = false;
    std::string err;
};

// BAI (SAM spec 5.2): per reference, the bins' chunks and the 16 kb linear index
struct BaiRef {
    std::unordered_map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
    std::vector<uint64_t> lin;
};

}  // namespace

struct ngsep_bam {
    ngsep_ctx* ctx = nullptr;
    std::FILE* f = nullptr;
    std::string path;
    // decoder thread -> consumer queue
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Chunk> q;
    std::vector<RawBuf<uint8_t>> pool;   // consumed chunk buffers, reused by the decoder (no page faults / unmaps)
    bool stop = false, producer_done = false;
    // consumer side: the current decoded buffer; bytes [pos, end) not yet consumed
    RawBuf<uint8_t> mem;
    uint8_t* buf = nullptr;
    size_t end = 0, pos = 0;
    bool eof = false;
    std::vector<int32_t> ref_to_seq;   // BAM refID -> ctx sequence id
    std::vector<std::string> ref_names;
    std::vector<int64_t> ref_lens;     // (their @SQ lengths)
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
    // region (ngsep_bam_set_region): stop at the first record past it
    int32_t region_ref = -1;
    int64_t region_last = 0;
    bool region_done = false;
    // index
    bool bai_loaded = false;
    std::vector<BaiRef> bai;
    // batch storage (filled in parallel, never value-initialised): two sets used in turn, so a batch stays
    // valid while the next one is decoded (call_bam decodes batch k+1 while batch k is admitted)
    struct BatchStore {
        RawBuf<int32_t> b_seq, b_first, b_flags, b_rg, b_cig_n, b_cigar, b_seqlen;
        RawBuf<int64_t> b_cig_off, b_seq_off;
        RawBuf<uint8_t> b_hasq;
        RawBuf<char> b_bases, b_quals;
        RawBuf<int64_t> b_qual_off;                // packed batches: the qualities' offsets in the chunk
    } store[2];
    int store_cur = 0;
    // packed batches reference the decoded chunk in place: a chunk the reader leaves while filling batch j can still be
    // read by batch j - 1 (admitted meanwhile), so it is recycled only when batch j + 1 starts (for_each_batch admits
    // batch k while batch k + 1 is read, and k is done before k + 2 is read)
    int64_t batch_seq = 0;
    std::vector<std::pair<int64_t, RawBuf<uint8_t>>> retired;
    // inflate on the device (the context's GzDevice, borrowed while the reader is open), else on the host threads
    bool gpu_inflate = false;
    // fill_batch's per record state (reused batch after batch)
    struct Rec { int32_t keep, ncig, lseq, flags, rg, seq, first; };
    RawBuf<Rec> rec_buf;
    // NGSEP_HOST_TIMING diagnostics: seconds in the decoder's inflate, the record cut, parse and emit
    double t_inflate = 0, t_wait = 0, t_need = 0, t_cut = 0, t_parse = 0, t_emit = 0;
    double t_read = 0, t_pin = 0;               // device inflate: the decoder's file reads, its pinned allocations
    int64_t n_pcut = 0, n_pcut_serial = 0;      // parallel cuts, and their segments walked sequentially
    double t_pcut_walk = 0, t_pcut_merge = 0;
};

namespace {

using ngsep::parallel_for;

// the whole BGZF blocks at the start of comp[0, n) (SAM spec 4.1.1): their raw deflate data (offset, length) and
// decoded sizes; returns the bytes they span (a block cut off by n stays for the next read)
size_t scan_bgzf(const uint8_t* comp, size_t n, std::vector<size_t>& boff, std::vector<size_t>& bclen,
                 std::vector<uint32_t>& bisize, std::string& err) {
    boff.clear();
    bclen.clear();
    bisize.clear();
    size_t p = 0;
    while (p + 18 <= n) {
        const uint8_t* h = comp + p;
        if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) { err = "not a BGZF file"; break; }
        const uint16_t xlen = (uint16_t)(h[10] | (h[11] << 8));
        if (p + 12 + xlen > n) break;
        int bsize = -1;
        for (size_t i = 0; i + 4 <= xlen;) {
            const uint8_t* x = h + 12 + i;
            const uint16_t sl = (uint16_t)(x[2] | (x[3] << 8));
            if (x[0] == 'B' && x[1] == 'C' && sl == 2) bsize = x[4] | (x[5] << 8);
            i += 4 + sl;
        }
        if (bsize < 0) { err = "BGZF block without BC field"; break; }
        const size_t total = (size_t)bsize + 1;
        if (total < 12 + (size_t)xlen + 8) { err = "malformed BGZF block"; break; }
        if (p + total > n) break;
        const uint8_t* t = h + total - 4;
        boff.push_back(p + 12 + xlen);
        bclen.push_back(total - 12 - xlen - 8);
        bisize.push_back((uint32_t)(t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24)));
        p += total;
    }
    return p;
}

// decoder thread, device inflate (inflate.hip): 32 MB of the file at a time into a pinned buffer, its whole blocks
// inflated by KZ into a pinned chunk; two reads in flight (the file read of one overlaps the copies and kernel of the
// previous), the chunk handed over when its batch is done
void decoder_loop_gpu(ngsep_bam* b) {
    // (NGSEP_BGZF_READ: a smaller read, test hook -- many batches and blocks cut across reads on small files; never
    // below one whole BGZF block, 64 KB + its header: this buffer holds at most kRead bytes and must fit a block)
    const char* rh = ngsep::env_hook("NGSEP_BGZF_READ");
    const size_t kRead = rh ? std::max<size_t>((size_t)std::atoll(rh), (size_t)65536 + 256) : (size_t)32 << 20;
    ngsep_ctx* c = b->ctx;
    RawBuf<uint8_t> comp[2];
    for (int i = 0; i < 2; i++) {
        if (!c->gz_in_pool.empty()) { comp[i].adopt_pinned(c->gz_in_pool.back().first, c->gz_in_pool.back().second); c->gz_in_pool.pop_back(); }
        else comp[i].pinned = true;
    }
    std::vector<size_t> boff, bclen, dout;
    std::vector<uint32_t> bisize;
    const uint8_t* tail = nullptr;
    size_t tail_n = 0;
    bool file_eof = false;
    int sl = 0;
    Chunk pend;
    bool have_pend = false;
    int pend_slot = -1;
    std::string gerr;
    if (!c->gz) c->gz = ngsep::gz_create(c->device, gerr);
    auto hand_over = [&](Chunk&& ch) {
        {
            std::lock_guard<std::mutex> lk(b->mu);
            b->q.push_back(std::move(ch));
        }
        b->cv.notify_all();
    };
    auto finish_pending = [&]() {
        if (pend_slot < 0) return;
        const auto tw = std::chrono::steady_clock::now();
        std::string e;
        if (ngsep::gz_wait(c->gz, pend_slot, e) != 0 && pend.err.empty()) pend.err = e.empty() ? "BGZF inflate failed" : e;
        b->t_inflate += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count();
        pend_slot = -1;
    };
    while (true) {
        {
            std::unique_lock<std::mutex> lk(b->mu);
            b->cv.wait(lk, [&] { return b->stop || b->q.size() < 3; });
            if (b->stop) break;
        }
        Chunk ch;
        RawBuf<uint8_t>& cb = comp[sl];
        size_t total = 0;
        if (!c->gz) ch.err = "BGZF inflate device: " + gerr;
        else {
            cb.n = 0;
            cb.resize(tail_n + kRead + 256);
            if (tail_n) std::memmove(cb.data(), tail, tail_n);
            total = tail_n;
            if (!file_eof && tail_n < kRead) {             // (the buffer holds kRead bytes at most: carries cannot pile up)
                const auto tr = std::chrono::steady_clock::now();
                const size_t want = kRead - tail_n;
                const size_t got = std::fread(cb.data() + tail_n, 1, want, b->f);
                b->t_read += std::chrono::duration<double>(std::chrono::steady_clock::now() - tr).count();
                total += got;
                if (got < want) file_eof = true;
            }
        }
        size_t p = ch.err.empty() ? scan_bgzf(cb.data(), total, boff, bclen, bisize, ch.err) : 0;
        // at most one wave of KZ workgroups a batch (a batch a few blocks past it would take a second block latency):
        // the blocks past it are carried to the next read
        const size_t cap = (size_t)ngsep::gz_wave_blocks(c->gz);
        if (ch.err.empty() && boff.size() > cap) {
            p = boff[cap - 1] + bclen[cap - 1] + 8;
            boff.resize(cap);
            bclen.resize(cap);
            bisize.resize(cap);
        }
        if (ch.err.empty() && p < total && file_eof && boff.empty()) ch.err = "truncated BGZF block";
        tail = cb.data() + p;
        tail_n = ch.err.empty() ? total - p : 0;
        dout.assign(boff.size() + 1, 0);
        for (size_t k = 0; k < boff.size(); k++) dout[k + 1] = dout[k] + bisize[k];
        {
            std::lock_guard<std::mutex> lk(b->mu);
            if (!b->pool.empty()) { ch.mem = std::move(b->pool.back()); b->pool.pop_back(); }
        }
        if (!ch.mem.pinned) {
            ch.mem.release();
            if (!c->gz_chunk_pool.empty()) { ch.mem.adopt_pinned(c->gz_chunk_pool.back().first, c->gz_chunk_pool.back().second); c->gz_chunk_pool.pop_back(); }
            else ch.mem.pinned = true;
        }
        ch.mem.n = 0;
        const auto tp = std::chrono::steady_clock::now();
        ch.mem.resize(kChunkHead + dout.back());
        b->t_pin += std::chrono::duration<double>(std::chrono::steady_clock::now() - tp).count();
        ch.len = dout.back();
        if (ch.err.empty() && !boff.empty() &&
            ngsep::gz_submit(c->gz, sl, cb.data(), total, boff.data(), bclen.data(), bisize.data(), dout.data(), boff.size(),
                             ch.mem.data() + kChunkHead, ch.len, ch.err) == 0) {
            // (submitted: finished by the next round's finish_pending)
        }
        ch.eof = file_eof && tail_n == 0;
        const bool last = ch.eof || !ch.err.empty();
        finish_pending();                                  // the previous read's chunk
        if (have_pend) hand_over(std::move(pend));
        pend = std::move(ch);
        have_pend = true;
        pend_slot = boff.empty() || !pend.err.empty() ? -1 : sl;
        if (last) {
            finish_pending();
            hand_over(std::move(pend));
            pend = Chunk();
            break;
        }
        sl ^= 1;
    }
    finish_pending();                                      // (stopped: the in-flight batch drains before its buffers go)
    pend = Chunk();
    for (int i = 0; i < 2; i++)
        if (comp[i].p && comp[i].pinned) {
            c->gz_in_pool.emplace_back(comp[i].p, comp[i].cap);
            comp[i].p = nullptr;
            comp[i].cap = comp[i].n = 0;
        }
    std::lock_guard<std::mutex> lk(b->mu);
    b->producer_done = true;
    b->cv.notify_all();
}

// decoder thread: 32 MB of compressed blocks at a time, inflated on all host threads
void decoder_loop(ngsep_bam* b) {
    if (b->gpu_inflate) return decoder_loop_gpu(b);
    // (NGSEP_BGZF_READ: a smaller read, test hook -- blocks cut across reads on small files)
    const char* rh = ngsep::env_hook("NGSEP_BGZF_READ");
    const size_t kRead = rh ? std::max<size_t>((size_t)std::atoll(rh), 4096) : (size_t)32 << 20;
    // the compressed bytes: one buffer reused read after read (never value-initialised -- a vector's resize zeroed 32 MB
    // a read, 200 x 32 MB for a population's files), a block cut off by the read moved to its front
    RawBuf<uint8_t> comp;
    size_t have = 0;                                   // bytes of a cut block at comp's front
    bool file_eof = false;
    while (true) {
        {
            std::unique_lock<std::mutex> lk(b->mu);
            b->cv.wait(lk, [&] { return b->stop || b->q.size() < 3; });
            if (b->stop) break;
        }
        Chunk ch;
        size_t total = have;
        if (!file_eof) {
            comp.n = have;                             // (a growth keeps the cut block)
            comp.resize(have + kRead);
            const size_t got = std::fread(comp.data() + have, 1, kRead, b->f);
            total += got;
            if (got < kRead) file_eof = true;
        }
        // whole blocks in comp: offsets and decoded sizes
        std::vector<size_t> boff, bclen;
        std::vector<uint32_t> bisize;
        const size_t p = scan_bgzf(comp.data(), total, boff, bclen, bisize, ch.err);
        size_t carry_n = 0;
        if (ch.err.empty() && p < total) {
            if (file_eof && boff.empty()) ch.err = "truncated BGZF block";
            carry_n = total - p;
        }
        std::vector<size_t> dout(boff.size() + 1, 0);
        for (size_t k = 0; k < boff.size(); k++) dout[k + 1] = dout[k] + bisize[k];
        {
            std::lock_guard<std::mutex> lk(b->mu);
            if (!b->pool.empty()) { ch.mem = std::move(b->pool.back()); b->pool.pop_back(); }
        }
        ch.mem.n = 0;                       // nothing to keep when a recycled buffer grows
        ch.mem.resize(kChunkHead + dout.back());
        ch.len = dout.back();
        uint8_t* dst = ch.mem.data() + kChunkHead;
        std::atomic<int> bad{0};
        const Inflater& inf = Inflater::get();
        const auto ti0 = std::chrono::steady_clock::now();
        parallel_for((int64_t)boff.size(), 16, [&](int64_t lo, int64_t hi) {
            for (int64_t k = lo; k < hi; k++)
                if (bisize[(size_t)k] && !inf.run(comp.data() + boff[(size_t)k], bclen[(size_t)k], dst + dout[(size_t)k], bisize[(size_t)k]))
                    bad = 1;
        });
        b->t_inflate += std::chrono::duration<double>(std::chrono::steady_clock::now() - ti0).count();
        if (bad && ch.err.empty()) ch.err = "BGZF inflate failed";
        if (carry_n) std::memmove(comp.data(), comp.data() + p, carry_n);   // (the inflate is done with comp)
        have = carry_n;
        ch.eof = file_eof && carry_n == 0;
        const bool last = ch.eof || !ch.err.empty();
        {
            std::lock_guard<std::mutex> lk(b->mu);
            b->q.push_back(std::move(ch));
        }
        b->cv.notify_all();
        if (last) break;
    }
    std::lock_guard<std::mutex> lk(b->mu);
    b->producer_done = true;
    b->cv.notify_all();
}

void stop_decoder(ngsep_bam* b) {
    if (b->th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(b->mu);
            b->stop = true;
        }
        b->cv.notify_all();
        b->th.join();
    }
    b->q.clear();
    b->stop = false;
    b->producer_done = false;
}

void start_decoder(ngsep_bam* b) {
    stop_decoder(b);
    b->eof = false;
    b->th = std::thread(decoder_loop, b);
}

// ensures at least n unconsumed bytes; false at EOF (err set on a format error).  The unconsumed tail moves
// into the next chunk's headroom (no copy of the chunk itself).
bool need(ngsep_bam* b, size_t n, std::string& err) {
    struct T { ngsep_bam* b; std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
               ~T() { b->t_need += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); } } tm{b};
    while (b->end - b->pos < n) {
        if (b->eof) return false;
        Chunk ch;
        const auto tw0 = std::chrono::steady_clock::now();
        {
            std::unique_lock<std::mutex> lk(b->mu);
            b->cv.wait(lk, [&] { return !b->q.empty() || b->producer_done; });
            if (b->q.empty()) { b->eof = true; return false; }
            ch = std::move(b->q.front());
            b->q.pop_front();
        }
        b->t_wait += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw0).count();
        b->cv.notify_all();
        if (!ch.err.empty()) { err = ch.err; b->eof = true; return false; }
        const size_t rem = b->end - b->pos;
        if (rem <= kChunkHead) {
            uint8_t* start = ch.mem.data() + kChunkHead - rem;
            if (rem) std::memcpy(start, b->buf + b->pos, rem);
            b->mem = std::move(ch.mem);
            b->buf = start;
            b->pos = 0;
            b->end = rem + ch.len;
        } else {                                   // a record longer than the headroom: one copy
            RawBuf<uint8_t> m;
            m.resize(rem + ch.len);
            std::memcpy(m.data(), b->buf + b->pos, rem);
            std::memcpy(m.data() + rem, ch.mem.data() + kChunkHead, ch.len);
            b->mem = std::move(m);
            b->buf = b->mem.data();
            b->pos = 0;
            b->end = rem + ch.len;
            ch.mem = std::move(m);         // the consumed buffer (now in m) goes back to the pool below
        }
        if (ch.mem.cap) b->retired.emplace_back(b->batch_seq, std::move(ch.mem));   // (recycled by fill_batch)
        if (ch.eof) b->eof = true;
    }
    return true;
}

template <class T> T rd(const uint8_t* p) { T v; std::memcpy(&v, p, sizeof(T)); return v; }

// BAI of a BAM: path + ".bai", else the path with ".bam" replaced by ".bai"
bool load_bai(ngsep_bam* b) {
    if (b->bai_loaded) return !b->bai.empty();
    b->bai_loaded = true;
    std::string p1 = b->path + ".bai", p2;
    if (b->path.size() > 4 && b->path.compare(b->path.size() - 4, 4, ".bam") == 0) p2 = b->path.substr(0, b->path.size() - 4) + ".bai";
    std::FILE* f = std::fopen(p1.c_str(), "rb");
    if (!f && !p2.empty()) f = std::fopen(p2.c_str(), "rb");
    if (!f) return false;
    std::vector<uint8_t> d;
    uint8_t tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) d.insert(d.end(), tmp, tmp + got);
    std::fclose(f);
    size_t o = 0;
    auto ok = [&](size_t k) { return o + k <= d.size(); };
    if (!ok(8) || std::memcmp(d.data(), "BAI\1", 4) != 0) return false;
    o = 4;
    const int32_t n_ref = rd<int32_t>(&d[o]);
    o += 4;
    std::vector<BaiRef> refs((size_t)std::max(n_ref, 0));
    for (int32_t r = 0; r < n_ref; r++) {
        if (!ok(4)) return false;
        const int32_t n_bin = rd<int32_t>(&d[o]);
        o += 4;
        for (int32_t k = 0; k < n_bin; k++) {
            if (!ok(8)) return false;
            const uint32_t bin = rd<uint32_t>(&d[o]);
            const int32_t n_chunk = rd<int32_t>(&d[o + 4]);
            o += 8;
            if (!ok((size_t)n_chunk * 16)) return false;
            auto& v = refs[(size_t)r].bins[bin];
            for (int32_t c = 0; c < n_chunk; c++) v.push_back({rd<uint64_t>(&d[o + 16 * c]), rd<uint64_t>(&d[o + 16 * c + 8])});
            o += (size_t)n_chunk * 16;
        }
        if (!ok(4)) return false;
        const int32_t n_intv = rd<int32_t>(&d[o]);
        o += 4;
        if (!ok((size_t)n_intv * 8)) return false;
        refs[(size_t)r].lin.resize((size_t)n_intv);
        for (int32_t k = 0; k < n_intv; k++) refs[(size_t)r].lin[(size_t)k] = rd<uint64_t>(&d[o + 8 * k]);
        o += (size_t)n_intv * 8;
    }
    b->bai.swap(refs);
    return true;
}

// bins overlapping [beg, end) (SAM spec 5.3 reg2bins)
void reg2bins(int64_t beg, int64_t end, std::vector<uint32_t>& out) {
    out.clear();
    --end;
    out.push_back(0);
    for (int64_t k = 1 + (beg >> 26); k <= 1 + (end >> 26); k++) out.push_back((uint32_t)k);
    for (int64_t k = 9 + (beg >> 23); k <= 9 + (end >> 23); k++) out.push_back((uint32_t)k);
    for (int64_t k = 73 + (beg >> 20); k <= 73 + (end >> 20); k++) out.push_back((uint32_t)k);
    for (int64_t k = 585 + (beg >> 17); k <= 585 + (end >> 17); k++) out.push_back((uint32_t)k);
    for (int64_t k = 4681 + (beg >> 14); k <= 4681 + (end >> 14); k++) out.push_back((uint32_t)k);
}

}  // namespace

using namespace ngsep;

namespace {
bool gpu_inflate_wanted(const ngsep_ctx* c) {
    return c->sample_ids.empty() && ngsep::env_hook("NGSEP_GPU_INFLATE") != nullptr;
}
// a closing reader's pinned chunk buffers go back to its context, and the context's inflate device is free again
void give_back_inflate(ngsep_bam* b) {
    if (!b->gpu_inflate) return;
    ngsep_ctx* c = b->ctx;
    auto keep = [&](RawBuf<uint8_t>& m) {
        if (m.p && m.pinned && c->gz_chunk_pool.size() < 6) {
            c->gz_chunk_pool.emplace_back(m.p, m.cap);
            m.p = nullptr;
            m.n = m.cap = 0;
        }
    };
    for (auto& m : b->pool) keep(m);
    b->pool.clear();
    keep(b->mem);
    b->buf = nullptr;
    b->gpu_inflate = false;
    c->gz_busy = false;
}
}  // namespace

extern "C" int ngsep_bam_open(ngsep_ctx* c, const char* path, ngsep_bam** out) {
    if (!c || !path || !out) return NGSEP_E_INVALID;
    ngsep_bam* b = new ngsep_bam();
    b->ctx = c;
    b->path = path;
    b->f = std::fopen(path, "rb");
    if (!b->f) { delete b; return set_error(c, NGSEP_E_IO, std::string("cannot open ") + path); }
    // single-sample readers inflate on the device, one reader of the context at a time (a population's hundreds of
    // open readers stay on the host threads)
    b->gpu_inflate = gpu_inflate_wanted(c) && !c->gz_busy.exchange(true);
    start_decoder(b);
    auto fail = [&](int code, const std::string& m) {
        stop_decoder(b);
        give_back_inflate(b);
        std::fclose(b->f);
        delete b;
        return set_error(c, code, m);
    };
    std::string err;
    if (!need(b, 8, err) || std::memcmp(&b->buf[0], "BAM\1", 4) != 0) return fail(NGSEP_E_FORMAT, err.empty() ? "not a BAM file" : err);
    int32_t l_text = rd<int32_t>(&b->buf[4]);
    if (!need(b, 8 + (size_t)l_text + 4, err)) return fail(NGSEP_E_FORMAT, "truncated BAM header");
    std::string text((const char*)&b->buf[8], (size_t)l_text);
    b->pos = 8 + (size_t)l_text;
    int32_t n_ref = rd<int32_t>(&b->buf[b->pos]);
    b->pos += 4;
    std::unordered_map<std::string, int32_t> seq_index;
    for (size_t i = 0; i < c->seq_names.size(); i++) seq_index[c->seq_names[i]] = (int32_t)i;
    // CoverageStatisticsCalculator and RelativeAlleleCountsCalculator run without a genome (-r is optional
    // there): the header's sequences (for the latter with their lengths, as N bases: it reads no reference)
    const bool header_seqs = (c->params.coverage_stats || c->params.relative_allele_counts) && c->seq_names.empty();
    for (int32_t i = 0; i < n_ref; i++) {
        if (!need(b, 4, err)) break;
        int32_t ln = rd<int32_t>(&b->buf[b->pos]);
        if (!need(b, 4 + (size_t)ln + 4, err)) break;
        std::string name((const char*)&b->buf[b->pos + 4], (size_t)(ln > 0 ? ln - 1 : 0));
        int32_t lref = rd<int32_t>(&b->buf[b->pos + 4 + ln]);
        b->pos += 8 + (size_t)ln;
        b->ref_names.push_back(name);
        b->ref_lens.push_back(lref);
        if (header_seqs && !seq_index.count(name)) {
            seq_index[name] = (int32_t)c->seq_names.size();
            c->seq_names.push_back(name);
            if (c->params.relative_allele_counts) c->seq_bases.emplace_back((size_t)std::max(lref, 0), 'N');
            else c->seq_bases.emplace_back();
            b->ref_to_seq.push_back(seq_index[name]);
            continue;
        }
        auto it = seq_index.find(name);
        // ReadAlignmentFileReader.loadHeader validation (:198-214)
        if (it == seq_index.end()) return fail(NGSEP_E_FORMAT, "Inconsistent file header. Sequence " + name + " not present in the reference sequences");
        if ((int64_t)c->seq_bases[it->second].size() != lref) return fail(NGSEP_E_FORMAT, "Inconsistent length in file header. Sequence " + name);
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

// Positions the reader at the first record that can overlap seq:first-last (1-based) through the BAI
// index; records come in file order from there and next_batch stops after the last record starting at
// or before `last` on that sequence.  Returns NGSEP_E_IO without an index, NGSEP_E_INVALID for an
// unknown sequence.
extern "C" int ngsep_bam_set_region(ngsep_bam* b, const char* seq_name, int64_t first, int64_t last) {
    if (!b || !seq_name) return NGSEP_E_INVALID;
    int32_t ref = -1;
    for (size_t i = 0; i < b->ref_names.size(); i++) if (b->ref_names[i] == seq_name) ref = (int32_t)i;
    if (ref < 0) return set_error(b->ctx, NGSEP_E_INVALID, std::string("sequence not in the BAM header: ") + seq_name);
    if (!load_bai(b)) return set_error(b->ctx, NGSEP_E_IO, "no BAI index for " + b->path);
    if (first < 1) first = 1;
    if (last < first) last = first;
    // the smallest record offset of a chunk that can hold records overlapping the region: chunks of the
    // region's bins ending after the linear-index offset of its first 16 kb window, entered no earlier
    // than that offset (every record before it ends before the window)
    uint64_t start = UINT64_MAX;
    if ((size_t)ref < b->bai.size()) {
        const BaiRef& br = b->bai[(size_t)ref];
        const int64_t w = (first - 1) >> 14;
        const uint64_t min_off = br.lin.empty() ? 0 : br.lin[(size_t)std::min<int64_t>(w, (int64_t)br.lin.size() - 1)];
        std::vector<uint32_t> bins;
        reg2bins(first - 1, std::min<int64_t>(last, (int64_t)1 << 29), bins);
        for (uint32_t bin : bins) {
            auto it = br.bins.find(bin);
            if (it == br.bins.end()) continue;
            for (const auto& ch : it->second)
                if (ch.second > min_off) start = std::min(start, std::max(ch.first, min_off));
        }
    }
    stop_decoder(b);
    b->buf = nullptr;
    b->end = b->pos = 0;
    b->have_last = false;
    b->region_ref = ref;
    b->region_last = last;
    b->region_done = start == UINT64_MAX;       // no chunk: the region holds no record
    if (b->region_done) { b->eof = true; return NGSEP_OK; }
    if (std::fseek(b->f, (long)(start >> 16), SEEK_SET) != 0) return set_error(b->ctx, NGSEP_E_IO, "seek failed in " + b->path);
    start_decoder(b);
    std::string err;
    if (!need(b, (size_t)(start & 0xFFFF), err)) return set_error(b->ctx, NGSEP_E_FORMAT, err.empty() ? "region start past the end of the file" : err);
    b->pos = (size_t)(start & 0xFFFF);
    return NGSEP_OK;
}

namespace {

// A plausible record start at o (block_size, refID, pos, the NUL-terminated printable read name, the fixed fields'
// sizes within block_size, next refID): where a parallel cut segment starts its own walk
bool plausible_record(const ngsep_bam* b, const uint8_t* buf, size_t o, size_t hi) {
    if (o + 40 > hi) return false;
    const int32_t bs = rd<int32_t>(buf + o);
    if (bs < 34 || bs > (1 << 22) || o + 4 + (size_t)bs > hi) return false;
    const int32_t nref = (int32_t)b->ref_to_seq.size();
    const int32_t refid = rd<int32_t>(buf + o + 4), pos0 = rd<int32_t>(buf + o + 8), nref2 = rd<int32_t>(buf + o + 24);
    if (refid < -1 || refid >= nref || pos0 < -1 || nref2 < -1 || nref2 >= nref) return false;
    const int l_name = buf[o + 12];
    const int n_cig = rd<uint16_t>(buf + o + 16);
    const int32_t l_seq = rd<int32_t>(buf + o + 20);
    if (l_name < 2 || l_seq < 0) return false;
    if (32 + (int64_t)l_name + 4 * (int64_t)n_cig + (l_seq + 1) / 2 + (int64_t)l_seq > bs) return false;
    const uint8_t* nm = buf + o + 36;
    for (int k = 0; k + 1 < l_name; k++)
        if (nm[k] < 33 || nm[k] > 126 || nm[k] == '@') return false;
    return nm[l_name - 1] == 0;
}

// The record chain over the whole decoded buffer [b->pos, b->end), cut on all host threads: segment t > 0 walks
// its own chain from the first position that looks like two consecutive records, and the merge takes a segment's
// offsets only from the record at which the true chain (walked from b->pos) enters it -- a chain is determined by
// any one of its records, so the result equals the sequential walk; a segment whose walk never meets the true
// chain is walked sequentially.  Stops at max_reads, at a record past the buffer's end, or at a malformed record
// (left for the sequential cut to report).
void parallel_cut(ngsep_bam* b, int64_t max_reads, size_t span, std::vector<size_t>& roff) {
    const uint8_t* buf = b->buf;
    const size_t lo = b->pos, hi = b->pos + span;            // (a record past hi is left to the sequential cut)
    constexpr int T = 32;
    size_t bnd[T + 1];
    for (int t = 0; t <= T; t++) bnd[t] = lo + (hi - lo) / T * (size_t)t;
    bnd[T] = hi;
    std::vector<size_t> seg[T];
    size_t seg_end[T] = {};
    const auto tw0 = std::chrono::steady_clock::now();
    // (tests: NGSEP_PCUT_MISS=1 makes every odd segment's own walk start one byte off the chain, so the merge walks it)
    static const bool miss = env_hook("NGSEP_PCUT_MISS") != nullptr;
    parallel_for(T, 1, [&](int64_t t0, int64_t t1) {
        for (int64_t t = t0; t < t1; t++) {
            size_t o = bnd[t];
            if (miss && (t & 1)) {
                const int32_t bs0 = rd<int32_t>(buf + o);
                if (bs0 < 32) continue;
                o += 1;
            } else if (t > 0) {
                const size_t lim = std::min(bnd[t + 1], bnd[t] + ((size_t)1 << 20));
                while (o < lim && !(plausible_record(b, buf, o, hi) && plausible_record(b, buf, o + 4 + (size_t)rd<int32_t>(buf + o), hi))) o++;
                if (o >= lim) continue;
            }
            std::vector<size_t>& v = seg[t];
            v.reserve((bnd[t + 1] - bnd[t]) / 200 + 16);
            while (o < bnd[t + 1] && o + 4 <= hi) {
                const int32_t bs = rd<int32_t>(buf + o);
                if (bs < 32 || o + 4 + (size_t)bs > hi) break;
                if (o + 4096 < hi) __builtin_prefetch(buf + o + 4096);
                v.push_back(o);
                o += 4 + (size_t)bs;
            }
            seg_end[t] = o;                                  // the record after the segment's last one
        }
    });
    const auto tw1 = std::chrono::steady_clock::now();
    size_t cur = lo;
    bool stop = false;
    for (int t = 0; t < T && !stop; t++) {
        const std::vector<size_t>& v = seg[t];
        auto it = std::lower_bound(v.begin(), v.end(), cur);
        if (cur < bnd[t + 1] && it != v.end() && *it == cur) {
            // the segment's offsets from cur on, in bulk (no record is touched again)
            const size_t j = (size_t)(it - v.begin());
            const size_t take = std::min(v.size() - j, (size_t)(max_reads - (int64_t)roff.size()));
            const size_t at = roff.size();
            roff.resize(at + take);
            for (size_t k = 0; k < take; k++) roff[at + k] = v[j + k] + 4;
            if (j + take < v.size()) { cur = v[j + take]; stop = true; }
            else cur = seg_end[t];
        }
        if (!stop && cur < bnd[t + 1]) b->n_pcut_serial++;
        while (!stop && cur < bnd[t + 1]) {                 // (the segment's own walk missed the chain, or stopped)
            if ((int64_t)roff.size() >= max_reads || cur + 4 > hi) { stop = true; break; }
            const int32_t bs = rd<int32_t>(buf + cur);
            if (bs < 32 || cur + 4 + (size_t)bs > hi) { stop = true; break; }
            roff.push_back(cur + 4);
            cur += 4 + (size_t)bs;
        }
    }
    b->pos = cur;
    b->n_pcut++;
    b->t_pcut_walk += std::chrono::duration<double>(tw1 - tw0).count();
    b->t_pcut_merge += std::chrono::duration<double>(std::chrono::steady_clock::now() - tw1).count();
}

// one batch of up to max_reads kept records into B (ngsep_bam_next_batch)
// packed: BAM encoding read in place (bases = quals = the chunk, *qual_off = the qualities' offsets; PackedBatch)
int fill_batch(ngsep_bam* b, ngsep_bam::BatchStore& B, int64_t max_reads, ngsep_read_batch* out, bool* retry, bool packed,
               const int64_t** qual_off) {
    *retry = false;
    static const int kOp[9] = {3, 2, 1, 5, 6, 0, 4, 3, 7};   // BAM M I D N S H P = X -> NGSEP H0 D1 I2 M3 P4 N5 S6 X7

    static const char kNt[] = "=ACMGRSVTWYHKDBN";
    std::string err;
    // 1. cut up to max_reads whole records (their offsets in buf), sequentially along the block_size chain
    std::vector<size_t> roff;
    roff.reserve((size_t)std::min<int64_t>(max_reads, 1 << 20));
    const auto tc0 = std::chrono::steady_clock::now();
    // (more decoded bytes are only pulled in while no record is cut: pulling compacts the buffer)
    while ((int64_t)roff.size() < max_reads && !b->region_done) {
        if (b->end - b->pos < 4) {
            if (!roff.empty()) break;
            if (!need(b, 4, err)) break;
        }
        const int32_t bs = rd<int32_t>(&b->buf[b->pos]);
        if (bs < 32) return set_error(b->ctx, NGSEP_E_FORMAT, "malformed BAM record");
        if (b->end - b->pos < 4 + (size_t)bs) {
            // the rest of this record is in the next chunk: decode the records cut so far first
            if (!roff.empty()) break;
            if (!need(b, 4 + (size_t)bs, err)) return set_error(b->ctx, NGSEP_E_FORMAT, err.empty() ? "truncated BAM record" : err);
        }
        // a decoded chunk's worth of records (bounded by max_reads at 512 B a record): cut on all threads; the
        // sequential walk below picks up where it stopped
        // (only when the span holds the record at b->pos: a single record longer than the span, e.g. an ultra-long
        // read, would leave the cut empty and b->pos unmoved; the sequential walk takes it)
        const size_t span = std::min(b->end - b->pos, (size_t)max_reads * 512);
        if (roff.empty() && b->region_ref < 0 && span >= ((size_t)8 << 20) && 4 + (size_t)bs <= span) {
            parallel_cut(b, max_reads, span, roff);
            if (!roff.empty()) continue;
        }
        const uint8_t* r = &b->buf[b->pos + 4];
        // the record chain is a dependent walk through freshly inflated memory: pull the lines a few
        // records ahead (the chain only moves forward)
        if (b->end - b->pos > 4096) __builtin_prefetch(&b->buf[b->pos + 4096]);
        if (b->region_ref >= 0) {
            const int32_t refid = rd<int32_t>(r), pos0 = rd<int32_t>(r + 4);
            if (refid != b->region_ref || (int64_t)pos0 + 1 > b->region_last) { b->region_done = true; break; }
        }
        roff.push_back(b->pos + 4);
        b->pos += 4 + (size_t)bs;
    }
    if (!err.empty()) return set_error(b->ctx, NGSEP_E_FORMAT, err);
    const int64_t n = (int64_t)roff.size();
    const auto tc1 = std::chrono::steady_clock::now();
    // 2. per record: filters (isSameAlignment against the previous raw record, isMultiple, filter flags,
    //    malformed CIGAR / read length) and output sizes -- in parallel
    // (per record state in a buffer the reader keeps: no 14 MB zero fill a batch; every record's keep is written)
    using Rec = ngsep_bam::Rec;
    RawBuf<Rec>& recb = b->rec_buf;
    recb.n = 0;
    recb.resize((size_t)n);
    Rec* rec = recb.data();
    const uint8_t* base = b->buf;
    auto name_of = [&](size_t o) { return std::make_pair((const char*)base + o + 32, (size_t)(base[o + 8] ? base[o + 8] - 1 : 0)); };
    parallel_for(n, 4096, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            const uint8_t* r = base + roff[(size_t)i];
            const int32_t refid = rd<int32_t>(r), pos0 = rd<int32_t>(r + 4);
            const uint8_t l_name = r[8], mapq = r[9];
            const uint16_t n_cig = rd<uint16_t>(r + 12), flag = rd<uint16_t>(r + 14);
            const int32_t l_seq = rd<int32_t>(r + 16);
            const int32_t bs = rd<int32_t>(r - 4);
            Rec& o = rec[(size_t)i];
            o.keep = 0;
            o.first = pos0 + 1;
            // isSameAlignment (ReadAlignmentFileReader.java:292-306) with the previous raw record
            const int paired = (flag & 1) != 0, fop = (flag & 0x40) != 0;
            bool same;
            if (i == 0) {
                same = b->have_last && b->last_pos == pos0 + 1 && b->last_paired == paired && (!paired || b->last_fop == fop) &&
                       b->last_name.size() == (size_t)(l_name ? l_name - 1 : 0) &&
                       std::memcmp(b->last_name.data(), r + 32, b->last_name.size()) == 0;
            } else {
                const uint8_t* pr = base + roff[(size_t)i - 1];
                const uint16_t pflag = rd<uint16_t>(pr + 14);
                const int pp = (pflag & 1) != 0, pf = (pflag & 0x40) != 0;
                same = rd<int32_t>(pr + 4) == pos0 && pp == paired && (!paired || pf == fop) && pr[8] == l_name &&
                       std::memcmp(pr + 32, r + 32, l_name) == 0;
            }
            if (same) continue;
            if (flag & 0x4) continue;               // FLAG_READ_UNMAPPED (filtered)
            if (refid < 0 || refid >= (int32_t)b->ref_to_seq.size()) continue;
            const uint8_t* end = r + bs;
            const uint8_t* cig = r + 32 + l_name;
            const uint8_t* seq = cig + 4 * n_cig;
            const uint8_t* qual = seq + (l_seq + 1) / 2;
            const uint8_t* aux = qual + l_seq;
            if (aux > end) continue;
            // tags: NH and RG
            int nh = 0, nh_present = 0, rg = -1;
            for (const uint8_t* t = aux; t + 3 <= end;) {
                const char t0 = (char)t[0], t1 = (char)t[1], ty = (char)t[2];
                const uint8_t* v = t + 3;
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
                    case 'Z': case 'H': { isint = false; const uint8_t* z = v; while (z < end && *z) z++; sz = (size_t)(z - v) + 1; break; }
                    case 'B': {
                        isint = false;
                        const char sub = (char)v[0];
                        const int32_t cnt = rd<int32_t>(v + 1);
                        const int es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2 : 4;
                        sz = 5 + (size_t)cnt * es;
                        break;
                    }
                    default: t = end; continue;
                }
                if (t0 == 'N' && t1 == 'H' && isint && ty != 'A') { nh = (int)iv; nh_present = 1; }
                if (t0 == 'R' && t1 == 'G' && ty == 'Z') {
                    // getReadGroup() is null if not in the header (a few groups: compared in place)
                    rg = -1;
                    if (b->rg_ids.size() <= 16) {
                        for (size_t g = 0; g < b->rg_ids.size(); g++)
                            if (std::strcmp(b->rg_ids[g].c_str(), (const char*)v) == 0) { rg = (int32_t)g; break; }
                    } else {
                        auto it = b->rg_index.find(std::string((const char*)v));
                        if (it != b->rg_index.end()) rg = it->second;
                    }
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
            int read_len = 0, nc = 0, prev = -1;
            bool bad = false;
            for (int k = 0; k < n_cig; k++) {
                const uint32_t v = rd<uint32_t>(cig + 4 * k);
                const uint32_t op = v & 15;
                if (op > 8) { bad = true; break; }
                const int nop = kOp[op];
                if (nop != prev) { nc++; prev = nop; }
                if (nop & 2) read_len += (int)(v >> 4);
            }
            if (bad) continue;
            if (l_seq > 0 && l_seq != read_len) continue;   // setReadCharacters throws
            if ((flags & b->filter_flags) != 0) continue;
            o.keep = 1;
            o.ncig = nc;
            o.lseq = l_seq;
            o.flags = flags;
            o.rg = rg;
            o.seq = b->ref_to_seq[(size_t)refid];
        }
    });
    if (n > 0) {        // the last raw record of this batch is the next batch's "previous"
        const uint8_t* r = base + roff[(size_t)n - 1];
        const uint16_t flag = rd<uint16_t>(r + 14);
        b->have_last = true;
        b->last_pos = rd<int32_t>(r + 4) + 1;
        b->last_paired = (flag & 1) != 0;
        b->last_fop = (flag & 0x40) != 0;
        auto nm = name_of(roff[(size_t)n - 1]);
        b->last_name.assign(nm.first, nm.second);
    }
    const auto tc2 = std::chrono::steady_clock::now();
    // 3. output offsets of the kept records (a chunked scan: per-chunk totals in parallel, the chunks' starts
    //    serially, each chunk's records walked from its start), then their fields in parallel
    constexpr int64_t kEmitChunk = 4096;
    const int64_t nch = (n + kEmitChunk - 1) / kEmitChunk;
    struct Offs { int64_t k, c, q; };              // kept records, CIGAR elements, sequence bytes before a chunk
    std::vector<Offs> cst((size_t)nch + 1, Offs{0, 0, 0});
    parallel_for(nch, 1, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; c++) {
            Offs t{0, 0, 0};
            for (int64_t i = c * kEmitChunk; i < std::min(n, (c + 1) * kEmitChunk); i++) {
                const Rec& o = rec[(size_t)i];
                if (!o.keep) continue;
                t.k++;
                t.c += o.ncig;
                t.q += o.lseq;
            }
            cst[(size_t)c + 1] = t;
        }
    });
    for (int64_t c = 0; c < nch; c++) {
        cst[(size_t)c + 1].k += cst[(size_t)c].k;
        cst[(size_t)c + 1].c += cst[(size_t)c].c;
        cst[(size_t)c + 1].q += cst[(size_t)c].q;
    }
    const int64_t nk = cst[(size_t)nch].k;
    B.b_seq.resize((size_t)nk); B.b_first.resize((size_t)nk); B.b_flags.resize((size_t)nk); B.b_rg.resize((size_t)nk);
    B.b_cig_off.resize((size_t)nk); B.b_cig_n.resize((size_t)nk); B.b_seq_off.resize((size_t)nk); B.b_seqlen.resize((size_t)nk);
    B.b_hasq.resize((size_t)nk);
    B.b_cigar.resize((size_t)cst[(size_t)nch].c);
    if (packed) {
        B.b_qual_off.resize((size_t)nk);
    } else {
        B.b_bases.resize((size_t)cst[(size_t)nch].q);
        B.b_quals.resize((size_t)cst[(size_t)nch].q);
    }
    parallel_for(nch, 1, [&](int64_t c0, int64_t c1) {
      for (int64_t c = c0; c < c1; c++) {
        Offs at = cst[(size_t)c];
        for (int64_t i = c * kEmitChunk; i < std::min(n, (c + 1) * kEmitChunk); i++) {
            const Rec& o = rec[(size_t)i];
            if (!o.keep) continue;
            const size_t k = (size_t)at.k;
            const int64_t cig_at = at.c, seq_at = at.q;
            at.k++;
            at.c += o.ncig;
            at.q += o.lseq;
            const uint8_t* r = base + roff[(size_t)i];
            const uint8_t l_name = r[8];
            const uint16_t n_cig = rd<uint16_t>(r + 12);
            const int32_t l_seq = o.lseq;
            const uint8_t* cig = r + 32 + l_name;
            const uint8_t* seq = cig + 4 * n_cig;
            const uint8_t* qual = seq + (l_seq + 1) / 2;
            B.b_seq[k] = o.seq;
            B.b_first[k] = o.first;
            B.b_flags[k] = o.flags;
            B.b_rg[k] = o.rg;
            B.b_cig_off[k] = cig_at;
            B.b_cig_n[k] = o.ncig;
            int32_t* cd = &B.b_cigar[(size_t)cig_at];
            int nc = 0;
            for (int c2 = 0; c2 < n_cig; c2++) {
                const uint32_t v = rd<uint32_t>(cig + 4 * c2);
                const int nop = kOp[v & 15];
                if (nc > 0 && (cd[nc - 1] & 7) == nop) cd[nc - 1] += (int32_t)(v >> 4) * 8;
                else cd[nc++] = (int32_t)(v >> 4) * 8 + nop;
            }
            B.b_seqlen[k] = l_seq;
            const bool hasq = l_seq > 0 && qual[0] != 0xFF;
            if (packed) {
                // BAM's own encoding (ReadView::packed): the 4-bit bases and the raw qualities where they are
                B.b_seq_off[k] = (int64_t)(seq - base);
                B.b_qual_off[k] = (int64_t)(qual - base);
            } else {
                B.b_seq_off[k] = seq_at;
                char* bs = &B.b_bases[(size_t)seq_at];
                char* qs = &B.b_quals[(size_t)seq_at];
                static const uint16_t* pair = [] {    // one byte of two bases -> their two characters
                    static uint16_t t[256];
                    for (int v = 0; v < 256; v++) t[v] = (uint16_t)((uint8_t)kNt[v >> 4] | ((uint16_t)(uint8_t)kNt[v & 15] << 8));
                    return t;
                }();
                for (int32_t j = 0; j + 1 < l_seq; j += 2) std::memcpy(bs + j, &pair[seq[j >> 1]], 2);
                if (l_seq & 1) bs[l_seq - 1] = kNt[seq[(l_seq - 1) >> 1] >> 4];
                if (hasq) for (int32_t j = 0; j < l_seq; j++) qs[j] = (char)(qual[j] + 33);
                else std::memset(qs, '!', (size_t)l_seq);
            }
            B.b_hasq[k] = hasq ? 1 : 0;
        }
      }
    });
    const auto tc3 = std::chrono::steady_clock::now();
    b->t_cut += std::chrono::duration<double>(tc1 - tc0).count();
    b->t_parse += std::chrono::duration<double>(tc2 - tc1).count();
    b->t_emit += std::chrono::duration<double>(tc3 - tc2).count();
    out->n_reads = nk;
    out->seq_id = B.b_seq.data();
    out->first = B.b_first.data();
    out->flags = B.b_flags.data();
    out->read_group = B.b_rg.data();
    out->cigar_off = B.b_cig_off.data();
    out->cigar_n = B.b_cig_n.data();
    out->cigar = B.b_cigar.data();
    out->seq_off = B.b_seq_off.data();
    out->seq_len = B.b_seqlen.data();
    out->bases = packed ? reinterpret_cast<const char*>(base) : B.b_bases.data();
    out->quals = packed ? reinterpret_cast<const char*>(base) : B.b_quals.data();
    if (qual_off) *qual_off = packed ? B.b_qual_off.data() : nullptr;
    out->has_quals = B.b_hasq.data();
    // a batch with every record filtered is not the end of the file: the caller stops at n_reads == 0
    *retry = nk == 0 && n > 0;
    return NGSEP_OK;
}

}  // namespace

static int next_batch(ngsep_bam* b, int64_t max_reads, ngsep_read_batch* out, bool packed, const int64_t** qual_off = nullptr) {
    if (!b || !out) return NGSEP_E_INVALID;
    ngsep_bam::BatchStore& B = b->store[b->store_cur];
    b->store_cur ^= 1;
    {   // this batch's number; the chunks left while reading an earlier batch go back to the decoder (the batch before
        // this one is done: see ngsep_bam::retired)
        const int64_t j = ++b->batch_seq;
        std::lock_guard<std::mutex> lk(b->mu);
        size_t w = 0;
        for (size_t k = 0; k < b->retired.size(); k++) {
            if (b->retired[k].first < j) {
                if (b->pool.size() < 6) b->pool.push_back(std::move(b->retired[k].second));
            } else {
                if (w != k) b->retired[w] = std::move(b->retired[k]);
                w++;
            }
        }
        b->retired.resize(w);
    }
    bool retry = true;
    int rc = NGSEP_OK;
    while (retry && rc == NGSEP_OK) rc = fill_batch(b, B, max_reads, out, &retry, packed, qual_off);
    return rc;
}

extern "C" int ngsep_bam_next_batch(ngsep_bam* b, int64_t max_reads, ngsep_read_batch* out) {
    return next_batch(b, max_reads, out, false);
}

extern "C" int ngsep_bam_close(ngsep_bam* b) {
    if (!b) return NGSEP_E_INVALID;
    stop_decoder(b);
    if (env_hook("NGSEP_HOST_TIMING"))
        std::fprintf(stderr, "[ngsep host] bam: inflate %.3f s (decoder thread%s), consumer wait %.3f s, need %.3f s, cut %.3f s (incl. wait; %lld parallel: walks %.3f s, merge %.3f s, %lld segments walked sequentially), parse %.3f s, emit %.3f s\n",
                     b->t_inflate, b->gpu_inflate ? ", waiting on the device" : "", b->t_wait, b->t_need, b->t_cut, (long long)b->n_pcut, b->t_pcut_walk, b->t_pcut_merge,
                     (long long)b->n_pcut_serial, b->t_parse, b->t_emit);
    if (env_hook("NGSEP_HOST_TIMING") && b->gpu_inflate)
        std::fprintf(stderr, "[ngsep host] bam (device inflate): file reads %.3f s, pinned allocations %.3f s\n", b->t_read, b->t_pin);
    give_back_inflate(b);
    if (b->f) std::fclose(b->f);
    delete b;
    return NGSEP_OK;
}

// BGZF decompression on the context's device (inflate.hip), the decoder's device path as one call: every block of
// in[0, n) (which must end on a block boundary) -> out[0, *out_n).  NGSEP_E_INVALID (with *out_n the size needed) when
// cap is too small.
extern "C" int ngsep_bgzf_inflate(ngsep_ctx* c, const uint8_t* in, int64_t n, uint8_t* out, int64_t cap, int64_t* out_n) {
    if (!c || (!in && n) || n < 0 || cap < 0 || !out_n) return NGSEP_E_INVALID;
    std::vector<size_t> boff, bclen, dout;
    std::vector<uint32_t> bisize;
    std::string err;
    const size_t p = scan_bgzf(in, (size_t)n, boff, bclen, bisize, err);
    if (!err.empty()) return set_error(c, NGSEP_E_FORMAT, err);
    if (p != (size_t)n) return set_error(c, NGSEP_E_FORMAT, "truncated BGZF block");
    dout.assign(boff.size() + 1, 0);
    for (size_t k = 0; k < boff.size(); k++) dout[k + 1] = dout[k] + bisize[k];
    *out_n = (int64_t)dout.back();
    if ((int64_t)dout.back() > cap) return set_error(c, NGSEP_E_INVALID, "output buffer too small");
    if (boff.empty()) return NGSEP_OK;
    if (c->gz_busy.exchange(true)) return set_error(c, NGSEP_E_INVALID, "the context's inflate device is in use by an open reader");
    struct Release { ngsep_ctx* c; ~Release() { c->gz_busy = false; } } rel{c};
    if (!c->gz) c->gz = ngsep::gz_create(c->device, err);
    if (!c->gz) return set_error(c, NGSEP_E_DEVICE, err);
    RawBuf<uint8_t> pin_in, pin_out;
    pin_in.pinned = pin_out.pinned = true;
    pin_in.resize((size_t)n);
    pin_out.resize(std::max<size_t>(dout.back(), 1));
    std::memcpy(pin_in.data(), in, (size_t)n);
    if (ngsep::gz_submit(c->gz, 0, pin_in.data(), (size_t)n, boff.data(), bclen.data(), bisize.data(), dout.data(), boff.size(),
                         pin_out.data(), dout.back(), err) != 0 ||
        ngsep::gz_wait(c->gz, 0, err) != 0)
        return set_error(c, NGSEP_E_FORMAT, err);
    std::memcpy(out, pin_out.data(), dout.back());
    return NGSEP_OK;
}

namespace ngsep {
// the reader's batches through fn in order, the next batch decoding (its own storage set) while fn runs on
// the current one; stops at the end of the file, at an error, or once the query region is done
template <class F>
static int for_each_batch(ngsep_ctx* c, ngsep_bam* b, F&& fn) {
    // (BAM-encoded batches: bases and qualities are not re-encoded, ReadView::packed)
    ngsep::PackedBatch batch[2];
    int cur = 0;
    int rc = next_batch(b, 1 << 20, &batch[0].b, true, &batch[0].qual_off);
    while (rc == NGSEP_OK && batch[cur].b.n_reads > 0 && !c->query_done) {
        int rc_next = NGSEP_OK;
        std::thread th([&] { rc_next = next_batch(b, 1 << 20, &batch[cur ^ 1].b, true, &batch[cur ^ 1].qual_off); });
        rc = fn(batch[cur]);
        th.join();
        if (rc == NGSEP_OK) rc = rc_next;
        cur ^= 1;
    }
    return rc;
}

// SingleSampleVariantsDetector.findSNVS (:896-931) + onSequenceEnd/saveSequenceVariants (:933-968, :1026-1032).
// With -querySeq the reader jumps to the region through the BAI index when there is one (the reference
// decodes the file from its start, AlignmentsPileupGenerator.java:310-322, 342-354); reading stops once the
// query region is done either way.
int call_bam(ngsep_ctx* c, const char* bam_path, const char* out_vcf) {
    start_device_init(c);
    {
        struct stat sb;
        if (!c->params.query_seq[0] && stat(bam_path, &sb) == 0) c->reads_hint = (int64_t)sb.st_size / 40;
    }
    ngsep_bam* b = nullptr;
    int rc = ngsep_bam_open(c, bam_path, &b);
    if (rc != NGSEP_OK) return rc;
    if (c->params.query_seq[0]) {
        const int r = ngsep_bam_set_region(b, c->params.query_seq, std::max<int64_t>(1, c->params.query_first), c->params.query_last);
        if (r != NGSEP_OK && r != NGSEP_E_IO) { ngsep_bam_close(b); return r; }   // no index: stream from the start
    }
    rc = ngsep_write_vcf_header(c, out_vcf);
    if (rc != NGSEP_OK) { ngsep_bam_close(b); return rc; }
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    const auto t0 = std::chrono::steady_clock::now();
    rc = for_each_batch(c, b, [&](const ngsep::PackedBatch& batch) {
        int r = process_alignments_packed(c, &batch);
        if (r == NGSEP_OK && !c->sites.empty()) r = ngsep_append_vcf_records(c, out_vcf);
        return r;
    });
    const auto t1 = std::chrono::steady_clock::now();
    ngsep_bam_close(b);
    if (rc != NGSEP_OK) return rc;
    const auto t2 = std::chrono::steady_clock::now();
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK) return rc;
    const auto t3 = std::chrono::steady_clock::now();
    rc = ngsep_append_vcf_records(c, out_vcf);
    if (host_timing)
        std::fprintf(stderr, "[ngsep host] call_bam: batches %.3f s, close %.3f s, end of alignments %.3f s, last records %.3f s\n",
                     std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count(),
                     std::chrono::duration<double>(t3 - t2).count(),
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t3).count());
    return rc;
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
    rc = for_each_batch(c, b, [&](const ngsep::PackedBatch& batch) { return process_alignments_packed(c, &batch); });
    ngsep_bam_close(b);
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK || !out_path) return rc;
    return ngsep_write_coverage(c, out_path);
}

// RelativeAlleleCountsCalculator.run (discovery/RelativeAlleleCountsCalculator.java:183-211): the generator over
// the BAM (maxAlnsPerStartPos = maxRD and secondaryAlns come with the context's params), printResults' text
extern "C" int ngsep_rac_bam(ngsep_ctx* c, const char* bam_path, const char* out_path) {
    if (!c || !bam_path) return NGSEP_E_INVALID;
    if (!c->params.relative_allele_counts) return set_error(c, NGSEP_E_INVALID, "ngsep_rac_bam needs params.relative_allele_counts = 1");
    ngsep_bam* b = nullptr;
    int rc = ngsep_bam_open(c, bam_path, &b);
    if (rc != NGSEP_OK) return rc;
    rc = for_each_batch(c, b, [&](const ngsep::PackedBatch& batch) { return process_alignments_packed(c, &batch); });
    ngsep_bam_close(b);
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK || !out_path) return rc;
    return ngsep_write_rac(c, out_path);
}

extern "C" int ngsep_call_bam(ngsep_ctx* c, const char* bam_path, const char* out_vcf_path) {
    if (!c || !bam_path || !out_vcf_path) return NGSEP_E_INVALID;
    return ngsep::call_bam(c, bam_path, out_vcf_path);
}

// findSNVS restricted to seq:first-last (-querySeq/-first/-last) through the BAI index: the per-region
// caller of the sharded drivers (every rank reads only its sequences' blocks of the BAM)
extern "C" int ngsep_call_region_bam(ngsep_ctx* c, const char* bam_path, const char* seq, int64_t first, int64_t last,
                                     const char* out_vcf_path) {
    if (!c || !bam_path || !seq || !out_vcf_path || std::strlen(seq) >= sizeof c->params.query_seq) return NGSEP_E_INVALID;
    if (c->cur_seq >= 0 || c->query_found) return set_error(c, NGSEP_E_INVALID, "ngsep_call_region_bam needs a context without alignments");
    const ngsep_params saved = c->params;
    std::snprintf(c->params.query_seq, sizeof c->params.query_seq, "%s", seq);
    c->params.query_first = (int32_t)std::max<int64_t>(0, std::min<int64_t>(first, INT32_MAX));
    c->params.query_last = (int32_t)std::max<int64_t>(0, std::min<int64_t>(last, INT32_MAX));
    const int rc = ngsep::call_bam(c, bam_path, out_vcf_path);
    c->params = saved;
    c->query_found = c->query_done = false;
    return rc;
}

// A window boundary for the sharded drivers: the first position p >= pos that no realigner event can
// reach.  Events are the alignments with I/D (IndelRealignerPileupListener opens one at an indel start, :101-118) and
// the realigner's input variants that open regions (-knownSTRs, non-SNV -knownVariants); an event edits only the
// alignments of its pileup (conciliateIndels :165-216), which end within one alignment span of it, and the calls it
// makes end inside [first, last + indel bases] of its reads, so with M = 2 x the longest span around pos + 100 a position
// outside every [first - M, last + indel + M] has the same realigner and listener state (lastIndelEnd, idxNextVariant)
// whatever happened before it.  A run of seq from p - lead (querySeq first: the alignments that start before it and
// reach p are then admitted as in a whole run, maxAlnsPerStartPos included) therefore calls every position >= p as the
// whole run does, and a run to p - 1 calls every position < p as it does.  The alignments are those of every file
// (all reader-filtered records, whatever maxAlnsPerStartPos admits: more events only move the cut right); *cut =
// sequence length + 1 when no such position exists before the sequence end.  Deterministic in (files, seq, pos), so
// neighbouring ranks agree on their shared boundary.
extern "C" int ngsep_clean_cut(ngsep_ctx* c, const char* const* bam_paths, int32_t n_files, const char* seq, int64_t pos,
                               int64_t* cut, int64_t* lead) {
    if (!c || !bam_paths || n_files < 1 || !seq || !cut || !lead) return NGSEP_E_INVALID;
    int32_t sid = -1;
    for (size_t i = 0; i < c->seq_names.size(); i++) if (c->seq_names[i] == seq) { sid = (int32_t)i; break; }
    if (sid < 0) return set_error(c, NGSEP_E_INVALID, std::string("sequence not in the reference: ") + seq);
    const int64_t len = (int64_t)c->seq_bases[(size_t)sid].size();
    if (pos < 1) pos = 1;
    if (pos > len) { *cut = len + 1; *lead = 0; return NGSEP_OK; }
    for (int64_t W = (int64_t)1 << 16;; W *= 4) {
        const int64_t lo = std::max<int64_t>(1, pos - W), hi = pos + W;
        std::vector<std::pair<int64_t, int64_t>> ev;      // [first, last + indel bases] of the events
        int64_t maxspan = 1, maxind = 0;
        for (int32_t fi = 0; fi < n_files; fi++) {
            ngsep_bam* b = nullptr;
            int rc = ngsep_bam_open(c, bam_paths[fi], &b);
            if (rc != NGSEP_OK) return rc;
            rc = ngsep_bam_set_region(b, seq, lo, hi);
            ngsep_read_batch batch{};
            while (rc == NGSEP_OK) {
                rc = ngsep_bam_next_batch(b, 1 << 16, &batch);
                if (rc != NGSEP_OK || batch.n_reads == 0) break;
                for (int64_t i = 0; i < batch.n_reads; i++) {
                    if (batch.seq_id[i] != sid) continue;
                    int64_t last = batch.first[i] - 1, indel = 0;
                    for (int32_t k = 0; k < batch.cigar_n[i]; k++) {
                        const int32_t v = batch.cigar[batch.cigar_off[i] + k], op = v & 7;
                        if (v & 1) last += v / 8;
                        if (op == 1 || op == 2) indel += v / 8;
                    }
                    if (last < lo || batch.first[i] > hi) continue;
                    maxspan = std::max<int64_t>(maxspan, last - batch.first[i] + 1);
                    maxind = std::max<int64_t>(maxind, indel);
                    if (indel > 0) ev.push_back({batch.first[i], last + indel});
                }
            }
            ngsep_bam_close(b);
            if (rc != NGSEP_OK) return rc;
        }
        if ((size_t)sid < c->strs.size())
            for (const StrVar& v : c->strs[(size_t)sid].v)
                if (v.event && v.last >= lo - W && v.first <= hi + W) ev.push_back({v.first, v.last});
        const int64_t M = 2 * maxspan + 100;
        std::sort(ev.begin(), ev.end());
        int64_t p = pos;                                  // the first uncovered position >= pos
        for (const auto& e : ev) {
            if (e.first - M > p) break;
            if (e.second + M >= p) p = e.second + M + 1;
        }
        // decided when no alignment outside [lo, hi] can cover p: those past hi start their intervals after hi - M,
        // those before lo end theirs before lo + M + their indel bases.  The left margin takes the most indel bases
        // any alignment of the neighbourhood carries on top of 4 M: an alignment before lo with more insertion bases
        // than 2 M + that (an insertion longer than twice the longest span seen, a long read's) is assumed absent
        const bool right = p <= hi - M || hi >= len, left = lo == 1 || pos - lo >= 4 * M + maxind;
        if (right && left) { *cut = std::min<int64_t>(p, len + 1); *lead = M + maxspan; return NGSEP_OK; }
        if (W > ((int64_t)1 << 34)) { *cut = len + 1; *lead = M + maxspan; return NGSEP_OK; }
    }
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
    ngsep_read_batch pending{};        // the batch after `batch`, read ahead by the whole-file probe
    bool has_pending = false;
    int64_t i = 0;
    bool done = false;
    std::vector<int32_t> rg_global;    // file read group -> global read group
    int32_t last(int64_t k) const {
        int32_t e = batch.first[k];
        for (int32_t j = 0; j < batch.cigar_n[k]; j++) { const int32_t v = batch.cigar[batch.cigar_off[k] + j]; if (v & 1) e += v / 8; }
        return e - 1;
    }
};

// AlignmentsPileupGenerator.processFiles over files read whole: the merged order (sequence, first, last, then
// the lowest file index -- chooseNextAln, :268-289) built in parallel.  Split keys cut every file at the same key
// (lower_bound), so each key range is an independent k-way merge; the records are then gathered into one merged
// SoA by all host threads and handed to the sweep in batches of 2^18.
int merge_whole_files(ngsep_ctx* c, std::vector<Cursor>& cur, int n_files) {
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    auto t_0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
        if (!host_timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngsep host] population merge: %s %.3f s\n", what, std::chrono::duration<double>(t - t_0).count());
        t_0 = t;
    };
    struct Key { int32_t seq, first, last; };
    auto kless = [](const Key& a, const Key& b) {
        if (a.seq != b.seq) return a.seq < b.seq;
        if (a.first != b.first) return a.first < b.first;
        return a.last < b.last;
    };
    std::vector<std::vector<Key>> keys((size_t)n_files);
    int64_t n_total = 0, fmax = 0;
    for (int f = 0; f < n_files; f++) {
        const int64_t n = cur[(size_t)f].done ? 0 : cur[(size_t)f].batch.n_reads;
        keys[(size_t)f].resize((size_t)n);
        n_total += n;
        if (n > (cur[(size_t)fmax].done ? 0 : cur[(size_t)fmax].batch.n_reads)) fmax = f;
    }
    if (n_total == 0) return NGSEP_OK;
    ngsep::parallel_for(n_files, 1, [&](int64_t lo, int64_t hi) {
        for (int64_t f = lo; f < hi; f++) {
            const Cursor& k = cur[(size_t)f];
            for (size_t i = 0; i < keys[(size_t)f].size(); i++)
                keys[(size_t)f][i] = Key{k.batch.seq_id[i], k.batch.first[i], k.last((int64_t)i)};
        }
    });
    // split keys: quantiles of the largest file (a key range holds every file's records of those keys)
    const std::vector<Key>& kf = keys[(size_t)fmax];
    const int64_t parts = std::max<int64_t>(1, std::min<int64_t>(1024, n_total / 32768));
    std::vector<Key> split;
    for (int64_t q = 1; q < parts; q++) {
        const Key x = kf[(size_t)((int64_t)kf.size() * q / parts)];
        if (split.empty() || kless(split.back(), x)) split.push_back(x);
    }
    const int64_t np = (int64_t)split.size() + 1;
    lap("keys");
    // cut[f][p] = first record of file f in range p (np + 1 entries per file)
    std::vector<std::vector<int64_t>> cut((size_t)n_files, std::vector<int64_t>((size_t)np + 1));
    ngsep::parallel_for(n_files, 1, [&](int64_t lo, int64_t hi) {
        for (int64_t f = lo; f < hi; f++) {
            const auto& v = keys[(size_t)f];
            auto& ct = cut[(size_t)f];
            ct[0] = 0;
            for (int64_t p = 1; p < np; p++)
                ct[(size_t)p] = std::lower_bound(v.begin(), v.end(), split[(size_t)p - 1], kless) - v.begin();
            ct[(size_t)np] = (int64_t)v.size();
        }
    });
    // per range: the merged order (file, record) and its CIGAR / base totals
    std::vector<std::vector<std::pair<int32_t, int32_t>>> order((size_t)np);
    std::vector<int64_t> n_rec((size_t)np + 1, 0), n_cig((size_t)np + 1, 0);
    ngsep::parallel_for(np, 1, [&](int64_t lo, int64_t hi) {
        struct Head { Key k; int32_t file; int64_t i; };
        std::vector<Head> heap;
        auto before = [&](const Head& a, const Head& b) {
            if (kless(a.k, b.k)) return true;
            if (kless(b.k, a.k)) return false;
            return a.file < b.file;
        };
        auto sift_down = [&](size_t i) {
            const size_t n = heap.size();
            while (true) {
                size_t m = i;
                const size_t l = 2 * i + 1, r = l + 1;
                if (l < n && before(heap[l], heap[m])) m = l;
                if (r < n && before(heap[r], heap[m])) m = r;
                if (m == i) return;
                std::swap(heap[i], heap[m]);
                i = m;
            }
        };
        for (int64_t p = lo; p < hi; p++) {
            heap.clear();
            int64_t tot = 0;
            for (int f = 0; f < n_files; f++) {
                const int64_t a = cut[(size_t)f][(size_t)p], b = cut[(size_t)f][(size_t)p + 1];
                tot += b - a;
                if (a < b) heap.push_back(Head{keys[(size_t)f][(size_t)a], f, a});
            }
            for (size_t i = heap.size() / 2; i-- > 0;) sift_down(i);
            auto& ord = order[(size_t)p];
            ord.reserve((size_t)tot);
            int64_t nc = 0;
            while (!heap.empty()) {
                const int32_t f = heap[0].file;
                const int64_t i = heap[0].i;
                ord.emplace_back(f, (int32_t)i);
                nc += cur[(size_t)f].batch.cigar_n[i];
                if (i + 1 < cut[(size_t)f][(size_t)p + 1]) {
                    heap[0].i = i + 1;
                    heap[0].k = keys[(size_t)f][(size_t)i + 1];
                } else {
                    heap[0] = heap.back();
                    heap.pop_back();
                }
                if (!heap.empty()) sift_down(0);
            }
            n_rec[(size_t)p + 1] = (int64_t)ord.size();
            n_cig[(size_t)p + 1] = nc;
        }
    });
    lap("ordered ranges");
    for (int64_t p = 0; p < np; p++) {
        n_rec[(size_t)p + 1] += n_rec[(size_t)p];
        n_cig[(size_t)p + 1] += n_cig[(size_t)p];
    }
    const int64_t N = n_rec[(size_t)np];
    // (uninitialised storage: the pages are first touched by the parallel gather).  The reads' bases and qualities
    // stay in their files' batches (two bytes per read base: copying them here, ~6 GB for configs[4], and releasing
    // the copy cost ~0.4 s); the merged batches point at them.
    RawBuf<int32_t> m_seq, m_first, m_flags, m_rg, m_cig_n, m_seqlen, m_cigar;
    RawBuf<int64_t> m_cig_off;
    RawBuf<const char*> m_chars, m_qp;
    for (auto* v : {&m_seq, &m_first, &m_flags, &m_rg, &m_cig_n, &m_seqlen}) v->resize((size_t)N);
    m_cigar.resize((size_t)std::max<int64_t>(1, n_cig[(size_t)np]));
    m_cig_off.resize((size_t)N);
    m_chars.resize((size_t)N);
    m_qp.resize((size_t)N);
    ngsep::parallel_for(np, 1, [&](int64_t lo, int64_t hi) {
        for (int64_t p = lo; p < hi; p++) {
            int64_t r = n_rec[(size_t)p], co = n_cig[(size_t)p];
            for (const auto& fi : order[(size_t)p]) {
                const Cursor& k = cur[(size_t)fi.first];
                const int64_t i = fi.second;
                m_seq[(size_t)r] = k.batch.seq_id[i];
                m_first[(size_t)r] = k.batch.first[i];
                m_flags[(size_t)r] = k.batch.flags[i];
                const int32_t lrg = k.batch.read_group ? k.batch.read_group[i] : -1;
                m_rg[(size_t)r] = lrg >= 0 && lrg < (int32_t)k.rg_global.size() ? k.rg_global[(size_t)lrg] : -1;
                const int32_t cn = k.batch.cigar_n[i];
                m_cig_off[(size_t)r] = co;
                m_cig_n[(size_t)r] = cn;
                std::memcpy(&m_cigar[(size_t)co], k.batch.cigar + k.batch.cigar_off[i], (size_t)cn * sizeof(int32_t));
                co += cn;
                m_seqlen[(size_t)r] = k.batch.seq_len[i];
                m_chars[(size_t)r] = k.batch.bases + k.batch.seq_off[i];
                const bool hq = k.batch.quals && (!k.batch.has_quals || k.batch.has_quals[i]);
                m_qp[(size_t)r] = hq ? k.batch.quals + k.batch.seq_off[i] : nullptr;
                r++;
            }
        }
    });
    lap("gather");
    keys.clear();
    order.clear();
    const int64_t kBatch = (int64_t)1 << 18;
    for (int64_t s0 = 0; s0 < N && !c->query_done; s0 += kBatch) {
        ngsep_read_batch mb{};
        mb.n_reads = std::min(kBatch, N - s0);
        mb.seq_id = m_seq.data() + s0; mb.first = m_first.data() + s0; mb.flags = m_flags.data() + s0;
        mb.read_group = m_rg.data() + s0; mb.cigar_off = m_cig_off.data() + s0; mb.cigar_n = m_cig_n.data() + s0;
        mb.cigar = m_cigar.data(); mb.seq_len = m_seqlen.data() + s0;
        const int r = ngsep::process_alignments_gathered(c, &mb, m_chars.data() + s0, m_qp.data() + s0);
        if (r != NGSEP_OK) return r;
    }
    lap("sweep of the merged batches");
    return NGSEP_OK;
}
}  // namespace

extern "C" int ngsep_call_population_bams(ngsep_ctx* c, const char* const* bam_paths, int32_t n_files, const char* out_vcf_path) {
    if (!c || !bam_paths || n_files <= 0 || !out_vcf_path) return NGSEP_E_INVALID;
    if (!c->params.multisample) return set_error(c, NGSEP_E_INVALID, "ngsep_call_population_bams needs params.multisample = 1");
    start_device_init(c);
    static const bool pop_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    auto tp = std::chrono::steady_clock::now();
    auto plap = [&](const char* what) {
        if (!pop_timing) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[ngsep host] population: %s %.3f s\n", what, std::chrono::duration<double>(t - tp).count());
        tp = t;
    };
    std::vector<Cursor> cur((size_t)n_files);
    auto close_all = [&]() { for (auto& k : cur) if (k.bam) ngsep_bam_close(k.bam); };
    // loadSamplesFromAlignmentHeaders (:499-523): read group -> sample over all files, samples by id
    std::vector<std::string> rg_ids, rg_sm;
    std::unordered_map<std::string, int32_t> rg_global;
    // the files are opened (header read, decoder started) on all host threads; errors reported in file order
    {
        std::vector<int> orc((size_t)n_files, NGSEP_OK);
        ngsep::parallel_for(n_files, 1, [&](int64_t lo, int64_t hi) {
            for (int64_t f = lo; f < hi; f++) {
                ngsep_bam* b = nullptr;
                int r = ngsep_bam_open(c, bam_paths[f], &b);
                if (r == NGSEP_OK && c->params.query_seq[0]) {   // -querySeq: every file read from the region's index chunks
                    r = ngsep_bam_set_region(b, c->params.query_seq, std::max<int64_t>(1, c->params.query_first), c->params.query_last);
                    if (r == NGSEP_E_IO) r = NGSEP_OK;
                }
                cur[(size_t)f].bam = b;
                orc[(size_t)f] = r;
            }
        });
        for (int f = 0; f < n_files; f++)
            if (orc[(size_t)f] != NGSEP_OK) {
                // the first failing file's message, deterministically: its open repeated alone
                close_all();
                ngsep_bam* b = nullptr;
                const int r = ngsep_bam_open(c, bam_paths[f], &b);
                if (r == NGSEP_OK) ngsep_bam_close(b);
                return orc[(size_t)f];
            }
    }
    for (int f = 0; f < n_files; f++) {
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
    plap("open");
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
    plap("samples");
    // AlignmentsPileupGenerator.processFiles: k-way merge by GenomicRegionComparator (sequence order,
    // first, last), ties to the lowest file index (chooseNextAln, :268-289)
    auto refill = [&](Cursor& k) -> int {
        while (!k.done && k.i >= k.batch.n_reads) {
            if (k.has_pending) {
                k.batch = k.pending;
                k.has_pending = false;
            } else {
                int r = ngsep_bam_next_batch(k.bam, 1 << 18, &k.batch);
                if (r != NGSEP_OK) return r;
            }
            k.i = 0;
            if (k.batch.n_reads == 0) k.done = true;
        }
        return NGSEP_OK;
    };
    // every file read whole when it fits one batch of kWhole records (the reader keeps two batches, so the probe
    // for a second one leaves the first valid): the merge then runs in parallel over key ranges
    const int64_t kWhole = (int64_t)1 << 22;
    bool whole = true;
    const auto tl0 = std::chrono::steady_clock::now();
    {
        std::vector<int> brc((size_t)n_files, NGSEP_OK);
        ngsep::parallel_for(n_files, 1, [&](int64_t lo, int64_t hi) {
            for (int64_t f = lo; f < hi; f++) {
                Cursor& k = cur[(size_t)f];
                int r = ngsep_bam_next_batch(k.bam, kWhole, &k.batch);
                if (r == NGSEP_OK && k.batch.n_reads > 0) {
                    r = ngsep_bam_next_batch(k.bam, kWhole, &k.pending);
                    k.has_pending = r == NGSEP_OK && k.pending.n_reads > 0;
                }
                k.i = 0;
                if (k.batch.n_reads == 0) k.done = true;
                brc[(size_t)f] = r;
            }
        });
        for (int f = 0; f < n_files; f++) {
            if (brc[(size_t)f] != NGSEP_OK) { close_all(); return brc[(size_t)f]; }
            if (cur[(size_t)f].has_pending) whole = false;
        }
    }
    if (env_hook("NGSEP_HOST_TIMING"))
        std::fprintf(stderr, "[ngsep host] population: %d files opened and read in %.3f s\n", n_files,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - tl0).count());
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
    if (env_hook("NGSEP_POP_STREAM")) whole = false;     // diagnostics / tests: the streaming merge
    plap("open + whole-file reads");
    if (whole && !c->query_done) {
        rc = merge_whole_files(c, cur, n_files);
        plap("merge + sweep");
        // nothing references the files' batches any more: they are closed (decoders joined, buffers freed) on
        // a thread of their own while the population layout and the device run proceed
        std::thread closer(close_all);
        if (rc == NGSEP_OK) {
            rc = ngsep_notify_end(c);
            plap("end of alignments (layout, device run)");
        }
        if (rc == NGSEP_OK) {
            rc = ngsep_write_population_vcf(c, out_vcf_path);
            plap("VCF");
        }
        closer.join();
        return rc;
    }
    // the files' next records in a binary min-heap on (sequence, first, last, file index): log2(files)
    // comparisons per record instead of a scan over every file
    struct Head { int32_t seq, first, last, file; };
    auto before = [](const Head& a, const Head& b) {
        if (a.seq != b.seq) return a.seq < b.seq;
        if (a.first != b.first) return a.first < b.first;
        if (a.last != b.last) return a.last < b.last;
        return a.file < b.file;
    };
    std::vector<Head> heap;
    heap.reserve((size_t)n_files);
    auto head_of = [&](int f) {
        const Cursor& k = cur[(size_t)f];
        return Head{k.batch.seq_id[k.i], k.batch.first[k.i], k.last(k.i), f};
    };
    auto sift_down = [&](size_t i) {
        const size_t n = heap.size();
        while (true) {
            size_t m = i;
            const size_t l = 2 * i + 1, r = l + 1;
            if (l < n && before(heap[l], heap[m])) m = l;
            if (r < n && before(heap[r], heap[m])) m = r;
            if (m == i) return;
            std::swap(heap[i], heap[m]);
            i = m;
        }
    };
    static const bool host_timing = env_hook("NGSEP_HOST_TIMING") != nullptr;   // diagnostics
    double t_refill = 0, t_flush = 0;
    const auto tm0 = std::chrono::steady_clock::now();
    auto secs = [](std::chrono::steady_clock::time_point a) {
        return std::chrono::duration<double>(std::chrono::steady_clock::now() - a).count();
    };
    for (int f = 0; f < n_files; f++)
        if (!cur[(size_t)f].done) heap.push_back(head_of(f));
    for (size_t i = heap.size() / 2; i-- > 0;) sift_down(i);
    while (!c->query_done && !heap.empty()) {
        const int best = heap[0].file;
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
            const auto tr = std::chrono::steady_clock::now();
            rc = refill(k);
            t_refill += secs(tr);
            if (rc != NGSEP_OK) { close_all(); return rc; }
        }
        if (k.done) {
            heap[0] = heap.back();
            heap.pop_back();
        } else {
            heap[0] = head_of(best);
        }
        if (!heap.empty()) sift_down(0);
        if (m_first.size() >= (1u << 18)) {
            const auto tf = std::chrono::steady_clock::now();
            rc = flush();
            t_flush += secs(tf);
            if (rc != NGSEP_OK) { close_all(); return rc; }
        }
    }
    if (host_timing)
        std::fprintf(stderr, "[ngsep host] population merge of %d files: %.3f s (refills %.3f s, admission of the merged batches %.3f s)\n",
                     n_files, secs(tm0), t_refill, t_flush);
    rc = flush();
    close_all();
    if (rc != NGSEP_OK) return rc;
    rc = ngsep_notify_end(c);
    if (rc != NGSEP_OK) return rc;
    return ngsep_write_population_vcf(c, out_vcf_path);
}

// MultisampleVariantsDetector restricted to seq:first-last (-querySeq/-first/-last), every file read from the region's
// index chunks: the per-sequence caller of the sharded population driver (sharding.call_population_sharded), one
// context per rank -- reference, known variants and device kept from sequence to sequence.  Writes the VCF header and
// the region's population records to out_vcf_path.
extern "C" int ngsep_call_population_region_bams(ngsep_ctx* c, const char* const* bam_paths, int32_t n_files, const char* seq,
                                                 int64_t first, int64_t last, const char* out_vcf_path) {
    if (!c || !bam_paths || n_files <= 0 || !seq || !out_vcf_path || std::strlen(seq) >= sizeof c->params.query_seq) return NGSEP_E_INVALID;
    if (c->cur_seq >= 0 || c->query_found)
        return set_error(c, NGSEP_E_INVALID, "ngsep_call_population_region_bams needs a context without alignments");
    const ngsep_params saved = c->params;
    std::snprintf(c->params.query_seq, sizeof c->params.query_seq, "%s", seq);
    c->params.query_first = (int32_t)std::max<int64_t>(0, std::min<int64_t>(first, INT32_MAX));
    c->params.query_last = (int32_t)std::max<int64_t>(0, std::min<int64_t>(last, INT32_MAX));
    const int rc = ngsep_call_population_bams(c, bam_paths, n_files, out_vcf_path);
    c->params = saved;
    c->query_found = c->query_done = false;
    // the region's records are in its file; the next region starts from an empty population store
    c->pop_sites.clear();
    c->pop_calls.clear();
    c->pop_big.clear();
    c->pop_order.clear();
    c->pop_text.clear();
    return rc;
}

// ---- several devices from one process ----
// The windows of ngsep_clean_cut (AlignmentsPileupGenerator.java:242-254,310-322: each window a querySeq region run from
// its cut minus the lead-in) handed to one host thread per context from an in-process queue; each thread drives its own
// context -- its device, HIP streams and pinned buffers -- and keeps the records inside its window; the blocks are
// written in (sequence, window) order.  The output equals the one-context run (tests/test_gpu_multi.py).
namespace {
struct MultiUnit { int32_t seq; int64_t first, last, lead; };

// the windows of every header sequence the reference holds (window <= 0: whole sequences), cut points monotone
int plan_windows(ngsep_ctx* const* ctxs, int32_t n_ctx, const char* const* bams, int32_t n_files, int64_t window,
                 std::vector<MultiUnit>& units) {
    ngsep_ctx* c0 = ctxs[0];
    ngsep_bam* b = nullptr;
    int rc = ngsep_bam_open(c0, bams[0], &b);
    if (rc != NGSEP_OK) return rc;
    std::vector<std::pair<int32_t, int64_t>> seqs;      // (sequence id, @SQ length) in header order
    for (size_t i = 0; i < b->ref_names.size(); i++) {
        int32_t sid = -1;
        for (size_t k = 0; k < c0->seq_names.size(); k++) if (c0->seq_names[k] == b->ref_names[i]) { sid = (int32_t)k; break; }
        if (sid >= 0) seqs.push_back({sid, std::min<int64_t>(b->ref_lens[i], (int64_t)c0->seq_bases[(size_t)sid].size())});
    }
    ngsep_bam_close(b);
    struct Cut { size_t seq; int64_t pos, cut = 0, lead = 0; };
    std::vector<Cut> cuts;
    for (size_t q = 0; q < seqs.size(); q++)
        if (window > 0)
            for (int64_t p = 1 + window; p <= seqs[q].second; p += window) cuts.push_back({q, p});
    // the cuts on every context's thread (each reads the BAI neighbourhood of its positions)
    std::atomic<size_t> next{0};
    std::atomic<int> bad{NGSEP_OK};
    std::vector<std::string> errs((size_t)n_ctx);
    auto work = [&](int t) {
        for (size_t i; (i = next.fetch_add(1)) < cuts.size() && bad.load() == NGSEP_OK;) {
            Cut& x = cuts[i];
            const int r = ngsep_clean_cut(ctxs[t], bams, n_files, ctxs[t]->seq_names[(size_t)seqs[x.seq].first].c_str(), x.pos,
                                          &x.cut, &x.lead);
            if (r != NGSEP_OK) { errs[(size_t)t] = ctxs[t]->err; bad.store(r); }
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < n_ctx; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    if (bad.load() != NGSEP_OK) {
        for (const std::string& e : errs) if (!e.empty()) return set_error(c0, bad.load(), e);
        return bad.load();
    }
    size_t k = 0;
    for (size_t q = 0; q < seqs.size(); q++) {
        const int64_t len = seqs[q].second;
        std::vector<int64_t> bnd{1}, lead{0};
        for (; k < cuts.size() && cuts[k].seq == q; k++) {
            bnd.push_back(std::max(bnd.back(), std::min(cuts[k].cut, len + 1)));
            lead.push_back(cuts[k].lead);
        }
        bnd.push_back(len + 1);
        for (size_t i = 0; i + 1 < bnd.size(); i++)
            if (bnd[i] < bnd[i + 1]) units.push_back({seqs[q].first, bnd[i], bnd[i + 1] - 1, lead[i]});
    }
    return NGSEP_OK;
}

// the records of a VCF file with first <= POS <= last (its header into *header when that is empty)
bool keep_window(const std::string& path, int64_t first, int64_t last, std::string* header, std::string& recs) {
    std::FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    char* line = nullptr;
    size_t cap = 0;
    ssize_t l;
    const bool want_header = header->empty();
    while ((l = getline(&line, &cap, f)) >= 0) {
        if (line[0] == '#') {
            if (want_header) header->append(line, (size_t)l);
            continue;
        }
        const char* t = std::strchr(line, '\t');
        if (!t) continue;
        const long long pos = std::atoll(t + 1);
        if (pos >= first && pos <= last) recs.append(line, (size_t)l);
    }
    std::free(line);
    std::fclose(f);
    return true;
}

int multi_run(ngsep_ctx* const* ctxs, int32_t n_ctx, const char* const* bams, int32_t n_files, const char* out_vcf,
              int64_t window, bool population) {
    if (!ctxs || n_ctx < 1 || !bams || n_files < 1 || !out_vcf) return NGSEP_E_INVALID;
    for (int32_t t = 0; t < n_ctx; t++) if (!ctxs[t]) return NGSEP_E_INVALID;
    ngsep_ctx* c0 = ctxs[0];
    if (c0->seq_names.empty()) return set_error(c0, NGSEP_E_INVALID, "load the reference into the first context");
    for (int32_t t = 1; t < n_ctx; t++) {
        ngsep_ctx* c = ctxs[t];
        for (int32_t u = 0; u < t; u++)
            if (ctxs[u] == c) return set_error(c0, NGSEP_E_INVALID, "a context is listed twice (one host thread drives each)");
        ngsep_params a = c0->params, b = c->params;
        if (std::memcmp(&a, &b, sizeof a) != 0) return set_error(c0, NGSEP_E_INVALID, "the contexts' parameters differ");
        if (c->seq_names.empty()) {                    // the first context's reference and input variants (a copy per
                                                       // context: N devices hold N references on the host)
            c->seq_names = c0->seq_names;
            c->seq_bases = c0->seq_bases;
            c->known = c0->known;
            c->known_recs = c0->known_recs;
            c->known_seq_begin = c0->known_seq_begin;
            c->known_given = c0->known_given;
            c->strs = c0->strs;
            c->het_rate = c0->het_rate;
        } else if (c->seq_names != c0->seq_names) {
            return set_error(c0, NGSEP_E_INVALID, "the contexts' references differ");
        }
    }
    // pass-through mode carves with the run's own longest span: whole sequences only (sharding.call_bam_sharded)
    if (c0->params.indel_passthrough) window = 0;
    std::vector<MultiUnit> units;
    int rc = plan_windows(ctxs, n_ctx, bams, n_files, window, units);
    if (rc != NGSEP_OK) return rc;
    std::vector<std::string> blocks(units.size()), headers((size_t)n_ctx), errs((size_t)n_ctx);
    std::atomic<size_t> next{0};
    std::atomic<int> bad{NGSEP_OK};
    const std::string tmp_base = std::string(out_vcf) + ".part";
    auto work = [&](int t) {
        ngsep_ctx* c = ctxs[t];
        const std::string tmp = tmp_base + std::to_string(t);
        for (size_t i; (i = next.fetch_add(1)) < units.size() && bad.load() == NGSEP_OK;) {
            const MultiUnit& u = units[i];
            const char* seq = c->seq_names[(size_t)u.seq].c_str();
            const int64_t from = std::max<int64_t>(1, u.first - u.lead);
            const int r = population ? ngsep_call_population_region_bams(c, bams, n_files, seq, from, u.last, tmp.c_str())
                                     : ngsep_call_region_bam(c, bams[0], seq, from, u.last, tmp.c_str());
            if (r != NGSEP_OK) { errs[(size_t)t] = c->err; bad.store(r); break; }
            if (!keep_window(tmp, u.first, u.last, &headers[(size_t)t], blocks[i])) {
                errs[(size_t)t] = "cannot read " + tmp;
                bad.store(NGSEP_E_IO);
                break;
            }
        }
        std::remove(tmp.c_str());
    };
    std::vector<std::thread> th;
    for (int t = 1; t < n_ctx; t++) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    if (bad.load() != NGSEP_OK) {
        for (const std::string& e : errs) if (!e.empty()) return set_error(c0, bad.load(), e);
        return bad.load();
    }
    std::string header;
    for (const std::string& h : headers) if (!h.empty()) { header = h; break; }
    if (header.empty()) {                               // no window anywhere: the header of the run's options
        if (!population) {
            if ((rc = ngsep_write_vcf_header(c0, out_vcf)) != NGSEP_OK) return rc;
            std::FILE* f = std::fopen(out_vcf, "r");
            if (!f) return set_error(c0, NGSEP_E_IO, std::string("cannot read ") + out_vcf);
            char buf[1 << 16];
            size_t n;
            while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) header.append(buf, n);
            std::fclose(f);
        } else if (!c0->seq_names.empty()) {
            const std::string tmp = tmp_base + "h";
            rc = ngsep_call_population_region_bams(c0, bams, n_files, c0->seq_names[0].c_str(), 1, 1, tmp.c_str());
            std::string none;
            if (rc == NGSEP_OK) keep_window(tmp, 1, 0, &header, none);
            std::remove(tmp.c_str());
            if (rc != NGSEP_OK) return rc;
        }
    }
    std::FILE* f = std::fopen(out_vcf, "w");
    if (!f) return set_error(c0, NGSEP_E_IO, std::string("cannot write ") + out_vcf);
    std::fwrite(header.data(), 1, header.size(), f);
    for (const std::string& b : blocks) std::fwrite(b.data(), 1, b.size(), f);
    const bool ok = std::fclose(f) == 0;
    if (!ok) return set_error(c0, NGSEP_E_IO, std::string("cannot write ") + out_vcf);
    // pass-through mode: every context's carved regions, in sequence then position order, on the first context
    if (c0->params.indel_passthrough) {
        for (int32_t t = 1; t < n_ctx; t++) {
            c0->carved.insert(c0->carved.end(), ctxs[t]->carved.begin(), ctxs[t]->carved.end());
            ctxs[t]->carved.clear();
        }
        std::vector<int32_t> order(c0->seq_names.size(), 0);
        {
            ngsep_bam* b = nullptr;
            if (ngsep_bam_open(c0, bams[0], &b) == NGSEP_OK) {
                for (size_t i = 0; i < b->ref_names.size(); i++)
                    for (size_t k = 0; k < c0->seq_names.size(); k++) if (c0->seq_names[k] == b->ref_names[i]) order[k] = (int32_t)i;
                ngsep_bam_close(b);
            }
        }
        std::sort(c0->carved.begin(), c0->carved.end(), [&](const auto& x, const auto& y) {
            if (order[(size_t)x.first] != order[(size_t)y.first]) return order[(size_t)x.first] < order[(size_t)y.first];
            return x.second < y.second;
        });
    }
    return NGSEP_OK;
}
}  // namespace

extern "C" int ngsep_call_bam_multi(ngsep_ctx* const* ctxs, int32_t n_ctx, const char* bam_path, const char* out_vcf_path,
                                    int64_t window) {
    const char* bams[1] = {bam_path};
    if (!bam_path) return NGSEP_E_INVALID;
    return multi_run(ctxs, n_ctx, bams, 1, out_vcf_path, window, false);
}

extern "C" int ngsep_call_population_bams_multi(ngsep_ctx* const* ctxs, int32_t n_ctx, const char* const* bam_paths,
                                                int32_t n_files, const char* out_vcf_path, int64_t window) {
    return multi_run(ctxs, n_ctx, bam_paths, n_files, out_vcf_path, window, true);
}

extern "C" int ngsep_plan_windows(ngsep_ctx* c, const char* const* bam_paths, int32_t n_files, int64_t window, int32_t* seq_id,
                                  int64_t* first, int64_t* last, int64_t* lead, int64_t cap, int64_t* n_out) {
    if (!c || !bam_paths || n_files < 1 || !n_out) return NGSEP_E_INVALID;
    if (c->seq_names.empty()) return set_error(c, NGSEP_E_INVALID, "load the reference before planning windows");
    std::vector<MultiUnit> units;
    ngsep_ctx* one[1] = {c};
    const int rc = plan_windows(one, 1, bam_paths, n_files, c->params.indel_passthrough ? 0 : window, units);
    if (rc != NGSEP_OK) return rc;
    *n_out = (int64_t)units.size();
    for (int64_t i = 0; i < (int64_t)units.size() && i < cap; i++) {
        if (seq_id) seq_id[i] = units[(size_t)i].seq;
        if (first) first[i] = units[(size_t)i].first;
        if (last) last[i] = units[(size_t)i].last;
        if (lead) lead[i] = units[(size_t)i].lead;
    }
    return NGSEP_OK;
}
