// Microbenchmark (GPU box): LDS read forms for the 2-bins-per-lane merge.
//   mode 0: ds_read_b64 8-byte aligned      mode 1: ds_read_b64 at 4 mod 8
//   mode 2: ds_read2_b32 (two dwords)       mode 3: 2 x ds_read_b32 (64-lane slots)
// Each thread sums NREP x 8 reads; checks the unaligned values against b32 reads.
// Build: hipcc --offload-arch=gfx950 -O3 -Xclang -target-feature -Xclang +unaligned-access-mode
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
typedef float f2a __attribute__((ext_vector_type(2), aligned(8)));
constexpr int NREP = 2048;

template <int MODE>
__global__ __launch_bounds__(512) void bench(float* out, int s)
{
    __shared__ __attribute__((aligned(16))) float d[16384 + 256];
    for (int i = threadIdx.x; i < 16384 + 256; i += 512) d[i] = (float)(i & 1023);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float acc = 0.f;
    int base = wave * 1040;
    typedef float f2 __attribute__((ext_vector_type(2)));
    for (int it = 0; it < NREP; ++it) {
        f2 v[8];
        const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + s + 2 * lane);
        const unsigned addr1 = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + s + lane);
        if (MODE == 0 || MODE == 1) {
            asm volatile("ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:512\n\tds_read_b64 %2, %8 offset:1024\n\t"
                         "ds_read_b64 %3, %8 offset:1536\n\tds_read_b64 %4, %8 offset:2048\n\tds_read_b64 %5, %8 offset:2560\n\t"
                         "ds_read_b64 %6, %8 offset:3072\n\tds_read_b64 %7, %8 offset:3584\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]), "=v"(v[4]), "=v"(v[5]), "=v"(v[6]), "=v"(v[7])
                         : "v"(addr));
        } else if (MODE == 2) {
            asm volatile("ds_read2_b32 %0, %8 offset1:1\n\tds_read2_b32 %1, %8 offset0:128 offset1:129\n\t"
                         "ds_read2_b32 %2, %9 offset1:1\n\tds_read2_b32 %3, %9 offset0:128 offset1:129\n\t"
                         "ds_read2_b32 %4, %10 offset1:1\n\tds_read2_b32 %5, %10 offset0:128 offset1:129\n\t"
                         "ds_read2_b32 %6, %11 offset1:1\n\tds_read2_b32 %7, %11 offset0:128 offset1:129\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]), "=v"(v[4]), "=v"(v[5]), "=v"(v[6]), "=v"(v[7])
                         : "v"(addr), "v"(addr + 1024), "v"(addr + 2048), "v"(addr + 3072));
        } else {
            // the same 1024 bytes per pair as 2 x ds_read_b32 per 64-lane slot
            asm volatile("ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:256\n\tds_read_b32 %2, %8 offset:512\n\t"
                         "ds_read_b32 %3, %8 offset:768\n\tds_read_b32 %4, %8 offset:1024\n\tds_read_b32 %5, %8 offset:1280\n\t"
                         "ds_read_b32 %6, %8 offset:1536\n\tds_read_b32 %7, %8 offset:1792\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(v[0].x), "=v"(v[0].y), "=v"(v[1].x), "=v"(v[1].y), "=v"(v[2].x), "=v"(v[2].y), "=v"(v[3].x), "=v"(v[3].y)
                         : "v"(addr1));
            asm volatile("ds_read_b32 %0, %8 offset:2048\n\tds_read_b32 %1, %8 offset:2304\n\tds_read_b32 %2, %8 offset:2560\n\t"
                         "ds_read_b32 %3, %8 offset:2816\n\tds_read_b32 %4, %8 offset:3072\n\tds_read_b32 %5, %8 offset:3328\n\t"
                         "ds_read_b32 %6, %8 offset:3584\n\tds_read_b32 %7, %8 offset:3840\n\ts_waitcnt lgkmcnt(0)"
                         : "=v"(v[4].x), "=v"(v[4].y), "=v"(v[5].x), "=v"(v[5].y), "=v"(v[6].x), "=v"(v[6].y), "=v"(v[7].x), "=v"(v[7].y)
                         : "v"(addr1));
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y;
        base = (base + 8) & 4095;
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

__global__ void check(float* out, int s)
{
    __shared__ float d[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) d[i] = (float)i;
    __syncthreads();
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 v;
    const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + s + 2 * threadIdx.x);
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr));
    out[2 * threadIdx.x] = v.x;
    out[2 * threadIdx.x + 1] = v.y;
}

int main()
{
    float* out;
    hipMalloc(&out, 256 * 8 * 512 * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // correctness of the unaligned b64 form
    hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, out, 1);
    std::vector<float> h(128);
    hipMemcpy(h.data(), out, 128 * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 128; ++i) bad += h[i] != (float)(i + 1);
    printf("unaligned b64 check: %s\n", bad ? "WRONG" : "ok");
    const int grid = 256 * 2;
    auto run = [&](int mode, int s) {
        float ms = 0;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            if (mode == 0) hipLaunchKernelGGL(bench<0>, dim3(grid), dim3(512), 0, 0, out, s);
            if (mode == 1) hipLaunchKernelGGL(bench<1>, dim3(grid), dim3(512), 0, 0, out, s);
            if (mode == 2) hipLaunchKernelGGL(bench<2>, dim3(grid), dim3(512), 0, 0, out, s);
            if (mode == 3) hipLaunchKernelGGL(bench<3>, dim3(grid), dim3(512), 0, 0, out, s);
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ms, a, b);
        }
        // bytes read per CU per cycle at 2.4 GHz
        const double bytes = (double)grid * 512 * NREP * 8 * 8;
        printf("mode %d s %d: %.3f ms  %.1f B/clk/CU\n", mode, s, ms, bytes / (ms * 1e-3) / 2.4e9 / 256);
    };
    run(0, 0);
    run(1, 1);
    run(2, 1);
    run(3, 0);
    return 0;
}
