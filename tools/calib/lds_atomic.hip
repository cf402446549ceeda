// LDS atomic throughput on gfx950 (tools/calib, diagnostics): cycles per ds_add_u32 wave-instruction for
// several address patterns and active-lane counts, ds_write_b32 beside it.  One line per case on stdout.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int kIters = 4096;

// mode 0 ds_add distinct (lane), 1 ds_add 1/4 lanes active, 2 ds_add pseudo-random over 2048 words,
// 3 ds_add 4 lanes per address, 4 ds_write distinct, 5 ds_add random with 16 lanes active, 6 ds_add lane*2 (2-way banks)
__global__ __launch_bounds__(256) void k_lds(int mode, uint32_t* out) {
    __shared__ uint32_t s[4096];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 4096; i += 256) s[i] = 0;
    __syncthreads();
    uint32_t x = 2654435761u * (tid + 1) + blockIdx.x;
    const int wbase = (tid >> 6) * 1024;
    int ad[8];
    bool act = true;
    for (int k = 0; k < 8; k++) {
        x = x * 1664525u + 1013904223u;
        switch (mode) {
            case 0: ad[k] = wbase + lane + 64 * k; break;
            case 1: ad[k] = wbase + lane + 64 * k; act = (lane & 3) == 0; break;
            case 2: ad[k] = (x >> 8) & 2047; break;
            case 3: ad[k] = wbase + (lane >> 2) + 64 * k; break;
            case 4: ad[k] = wbase + lane + 64 * k; break;
            case 5: ad[k] = (x >> 8) & 2047; act = (lane & 3) == 0; break;
            default: ad[k] = wbase + 2 * lane; break;
        }
    }
    if (act) {
        for (int it = 0; it < kIters / 8; it++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (mode == 4) s[ad[k]] = it;
                else atomicAdd(&s[ad[k]], 1u);
            }
        }
    }
    __syncthreads();
    uint32_t acc = 0;
    for (int i = tid; i < 4096; i += 256) acc += s[i];
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    uint32_t* out;
    hipMalloc(&out, 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev = 0, clk = 0, ncu = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    const char* names[] = {"add distinct 64", "add distinct 16 active", "add random 64", "add 4 lanes/addr",
                           "write distinct 64", "add random 16 active", "add stride 2"};
    for (int mode = 0; mode < 7; mode++) {
        for (int wg_per_cu : {1, 4, 8}) {
            const int grid = ncu * wg_per_cu;
            hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, 0, mode, out);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_lds, dim3(grid), dim3(256), 0, 0, mode, out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_cu = (double)wg_per_cu * 4 * kIters;   // wave-instructions per CU
            const double cyc = ms * 1e-3 * clk * 1e3 / instr_per_cu;
            std::printf("%-24s wg/cu %d  %.3f ms  %.2f cycles per wave-instruction per CU\n", names[mode], wg_per_cu, ms, cyc);
        }
    }
    return 0;
}
