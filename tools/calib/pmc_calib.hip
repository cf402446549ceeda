// pmc_calib.hip -- PMC FETCH_SIZE calibration for streaming reads of a known size at 4, 8 and 16 bytes per lane
// (MI355X_MICROARCH.md's x2 correction is stated for 16-B wide reads only).  Each kernel reads a 1 GiB buffer
// (past the 256 MiB Infinity Cache) exactly once with coalesced loads of one width; run under
// `rocprofv3 --pmc FETCH_SIZE --kernel-trace` and divide the bytes read by FETCH_SIZE (KiB) x 1024.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <class V>
__device__ inline uint32_t fold(const V& v) { return (uint32_t)v ^ (uint32_t)((uint64_t)v >> 32); }
template <>
__device__ inline uint32_t fold<uint4>(const uint4& v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <class V>
__global__ __launch_bounds__(256) void k_read(const V* __restrict__ p, size_t n, uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc ^= fold(p[i]);
    if (acc == 0x9E3779B9u) out[0] = acc;        // (never true for the fill below: keeps the loads)
}

int main() {
    const size_t bytes = (size_t)1 << 30;
    void* buf = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) { std::fprintf(stderr, "alloc failed\n"); return 1; }
    if (hipMemset(buf, 0x11, bytes) != hipSuccess) return 1;
    int ncu = 256;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    const dim3 grid(ncu * 8), block(256);
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_read<uint32_t>, grid, block, 0, 0, (const uint32_t*)buf, bytes / 4, out);
        hipLaunchKernelGGL(k_read<uint64_t>, grid, block, 0, 0, (const uint64_t*)buf, bytes / 8, out);
        hipLaunchKernelGGL(k_read<uint4>, grid, block, 0, 0, (const uint4*)buf, bytes / 16, out);
    }
    if (hipDeviceSynchronize() != hipSuccess) { std::fprintf(stderr, "kernel failed\n"); return 1; }
    std::printf("bytes_per_launch %zu\n", bytes);
    hipFree(buf);
    hipFree(out);
    return 0;
}
