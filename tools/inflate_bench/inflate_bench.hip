// inflate_bench: KZ (ngsepcore_amd/csrc/inflate.hip) on the first BGZF blocks of a file -- whole batches and
// single-block launches timed with events (per-block latency vs throughput), output checked against zlib.
#include "../../ngsepcore_amd/csrc/inflate.hip"
#include <zlib.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

using namespace ngsep;

static bool zinf(const uint8_t* in, size_t n, uint8_t* out, size_t on) {
    z_stream z{};
    if (inflateInit2(&z, -15) != Z_OK) return false;
    z.next_in = const_cast<Bytef*>(in); z.avail_in = (uInt)n; z.next_out = out; z.avail_out = (uInt)on;
    const int rc = inflate(&z, Z_FINISH);
    inflateEnd(&z);
    return rc == Z_STREAM_END && z.total_out == on;
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: inflate_bench file.bam [MB]\n"); return 2; }
    const size_t want = (size_t)(argc > 2 ? std::atof(argv[2]) : 32.0) * (1 << 20);
    std::FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> comp(want);
    comp.resize(std::fread(comp.data(), 1, want, f));
    std::fclose(f);
    std::vector<size_t> boff, bclen, dout;
    std::vector<uint32_t> bisize;
    size_t p = 0;
    while (p + 18 <= comp.size()) {
        const uint8_t* h = comp.data() + p;
        const uint16_t xlen = (uint16_t)(h[10] | (h[11] << 8));
        const int bsize = h[16] | (h[17] << 8);
        const size_t total = (size_t)bsize + 1;
        if (p + total > comp.size()) break;
        const uint8_t* t = h + total - 4;
        boff.push_back(p + 12 + xlen);
        bclen.push_back(total - 12 - xlen - 8);
        bisize.push_back((uint32_t)(t[0] | (t[1] << 8) | (t[2] << 16) | ((uint32_t)t[3] << 24)));
        p += total;
    }
    dout.assign(boff.size() + 1, 0);
    for (size_t k = 0; k < boff.size(); k++) dout[k + 1] = dout[k] + bisize[k];
    std::printf("%zu blocks, %.1f MB compressed -> %.1f MB\n", boff.size(), p / 1e6, dout.back() / 1e6);
    std::string err;
    GzDevice* d = gz_create(0, err);
    if (!d) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
    uint8_t *pin_in = (uint8_t*)gz_host_alloc(p + 256), *pin_out = (uint8_t*)gz_host_alloc(dout.back() + 16);
    std::memcpy(pin_in, comp.data(), p);
    for (int rep = 0; rep < 3; rep++) {
        const auto t0 = std::chrono::steady_clock::now();
        if (gz_submit(d, 0, pin_in, p, boff.data(), bclen.data(), bisize.data(), dout.data(), boff.size(), pin_out, dout.back(), err) ||
            gz_wait(d, 0, err)) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
        std::printf("batch: %.3f ms (H2D + KZ + D2H)\n", std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    // the kernel alone, whole batch and k blocks
    GzSlot& s = d->slot[0];
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    for (int64_t nb : {(int64_t)boff.size(), (int64_t)1024, (int64_t)256, (int64_t)64, (int64_t)1}) {
        if (nb > (int64_t)boff.size()) continue;
        (void)hipEventRecord(e0, s.stream);
        hipLaunchKernelGGL(k_inflate, dim3((unsigned)nb), dim3(kZThreads), sizeof(ZLds), s.stream, (const uint8_t*)s.d_in,
                           (uint64_t)p, (const ZBlock*)s.d_blk, nb, s.d_out, s.d_err);
        (void)hipEventRecord(e1, s.stream);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::printf("KZ over %lld blocks: %.3f ms (%.1f us a block, %.2f GB/s out)\n", (long long)nb, ms, 1000.0 * ms / nb,
                    dout[(size_t)nb] / (ms * 1e6));
    }
    // check against zlib
    std::vector<uint8_t> ref(dout.back());
    size_t bad = 0;
    for (size_t k = 0; k < boff.size(); k++)
        if (!zinf(comp.data() + boff[k], bclen[k], ref.data() + dout[k], bisize[k])) bad++;
    std::printf("zlib failures %zu, device output %s\n", bad, std::memcmp(ref.data(), pin_out, dout.back()) == 0 ? "identical" : "DIFFERS");
    gz_destroy(d);
    return 0;
}
