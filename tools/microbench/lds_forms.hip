// Microbenchmark (GPU box): LDS instruction throughput and unaligned-access
// behaviour on gfx950, for the merge-loop design.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/lds_forms.hip -o /tmp/lds_forms && /tmp/lds_forms
// Every mode: 512-thread workgroups, 2 per CU, 8 LDS instructions per loop
// iteration per wave (independent), reported as bytes per clock per CU at an
// assumed 2.4 GHz and as ns per wave-instruction per CU.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

constexpr int NREP = 4096;
constexpr int LDSF = 16384;   // floats of LDS per workgroup (64 KiB)

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512, 4) void bench(float* out, int mis)
{
    __shared__ __attribute__((aligned(16))) float d[LDSF + 1024];
    for (int i = threadIdx.x; i < LDSF + 1024; i += 512) d[i] = (float)(i & 1023);
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float acc = 0.f;
    int base = wave * 1600;
    for (int it = 0; it < NREP; ++it) {
        // element offset of this lane: `mis` floats past the natural alignment
        if constexpr (MODE == 0) {   // ds_read_b32, 64 consecutive dwords per instruction
            const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + mis + lane);
            float v[8];
            asm volatile(
                "ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:256\n\tds_read_b32 %2, %8 offset:512\n\t"
                "ds_read_b32 %3, %8 offset:768\n\tds_read_b32 %4, %8 offset:1024\n\tds_read_b32 %5, %8 offset:1280\n\t"
                "ds_read_b32 %6, %8 offset:1536\n\tds_read_b32 %7, %8 offset:1792\n\ts_waitcnt lgkmcnt(0)"
                : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]), "=v"(v[4]), "=v"(v[5]), "=v"(v[6]), "=v"(v[7])
                : "v"(addr));
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k];
        } else if constexpr (MODE == 1) {   // ds_read_b64, 128 consecutive dwords
            const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + mis + 2 * lane);
            f2 v[8];
            asm volatile(
                "ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:512\n\tds_read_b64 %2, %8 offset:1024\n\t"
                "ds_read_b64 %3, %8 offset:1536\n\tds_read_b64 %4, %8 offset:2048\n\tds_read_b64 %5, %8 offset:2560\n\t"
                "ds_read_b64 %6, %8 offset:3072\n\tds_read_b64 %7, %8 offset:3584\n\ts_waitcnt lgkmcnt(0)"
                : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]), "=v"(v[4]), "=v"(v[5]), "=v"(v[6]), "=v"(v[7])
                : "v"(addr));
#pragma unroll
            for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y;
        } else if constexpr (MODE == 2) {   // ds_read_b128, 256 consecutive dwords
            const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + mis + 4 * lane);
            f4 v[4];
            asm volatile(
                "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\tds_read_b128 %2, %4 offset:2048\n\t"
                "ds_read_b128 %3, %4 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3])
                : "v"(addr));
#pragma unroll
            for (int k = 0; k < 4; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
        } else if constexpr (MODE == 3) {   // ds_write_b32
            const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + mis + lane);
            const float x = acc + (float)it;
            asm volatile(
                "ds_write_b32 %0, %1\n\tds_write_b32 %0, %1 offset:256\n\tds_write_b32 %0, %1 offset:512\n\t"
                "ds_write_b32 %0, %1 offset:768\n\tds_write_b32 %0, %1 offset:1024\n\tds_write_b32 %0, %1 offset:1280\n\t"
                "ds_write_b32 %0, %1 offset:1536\n\tds_write_b32 %0, %1 offset:1792\n\ts_waitcnt lgkmcnt(0)"
                :
                : "v"(addr), "v"(x)
                : "memory");
            acc += 1.0f;
        } else if constexpr (MODE == 4) {   // ds_write_b64
            const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + mis + 2 * lane);
            f2 x;
            x.x = acc + (float)it;
            x.y = acc;
            asm volatile(
                "ds_write_b64 %0, %1\n\tds_write_b64 %0, %1 offset:512\n\tds_write_b64 %0, %1 offset:1024\n\t"
                "ds_write_b64 %0, %1 offset:1536\n\tds_write_b64 %0, %1 offset:2048\n\tds_write_b64 %0, %1 offset:2560\n\t"
                "ds_write_b64 %0, %1 offset:3072\n\tds_write_b64 %0, %1 offset:3584\n\ts_waitcnt lgkmcnt(0)"
                :
                : "v"(addr), "v"(x)
                : "memory");
            acc += 1.0f;
        } else if constexpr (MODE == 5) {   // merge-like: 2 x ds_read_b32 + ds_write_b32 per 64 bins
            const unsigned a1 = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + lane);
            const unsigned a2 = a1 + 4u * (unsigned)(300 + mis);
            const unsigned a3 = a1 + 4u * 6000u;
            float h[4], t[4];
            asm volatile(
                "ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:256\n\tds_read_b32 %2, %8 offset:512\n\t"
                "ds_read_b32 %3, %8 offset:768\n\tds_read_b32 %4, %9\n\tds_read_b32 %5, %9 offset:256\n\t"
                "ds_read_b32 %6, %9 offset:512\n\tds_read_b32 %7, %9 offset:768\n\ts_waitcnt lgkmcnt(0)"
                : "=v"(h[0]), "=v"(h[1]), "=v"(h[2]), "=v"(h[3]), "=v"(t[0]), "=v"(t[1]), "=v"(t[2]), "=v"(t[3])
                : "v"(a1), "v"(a2));
            float o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = h[k] + t[k];
            asm volatile(
                "ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:256\n\tds_write_b32 %0, %3 offset:512\n\t"
                "ds_write_b32 %0, %4 offset:768\n\ts_waitcnt lgkmcnt(0)"
                :
                : "v"(a3), "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3])
                : "memory");
            acc += o[0];
        } else if constexpr (MODE == 6) {   // merge-like with b64: 2 x ds_read_b64 + ds_write_b64 per 128 bins
            const unsigned a1 = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + 2 * lane);
            const unsigned a2 = a1 + 4u * (unsigned)(300 + mis);
            const unsigned a3 = a1 + 4u * 6000u;
            f2 h[2], t[2];
            asm volatile(
                "ds_read_b64 %0, %4\n\tds_read_b64 %1, %4 offset:512\n\t"
                "ds_read_b64 %2, %5\n\tds_read_b64 %3, %5 offset:512\n\ts_waitcnt lgkmcnt(0)"
                : "=v"(h[0]), "=v"(h[1]), "=v"(t[0]), "=v"(t[1])
                : "v"(a1), "v"(a2));
            f2 o[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) o[k] = h[k] + t[k];
            asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %2 offset:512\n\ts_waitcnt lgkmcnt(0)"
                         :
                         : "v"(a3), "v"(o[0]), "v"(o[1])
                         : "memory");
            acc += o[0].x;
        } else if constexpr (MODE == 7) {   // two-level fused with b64: 4 x read_b64 + 1 write_b64 per 128 bins
            const unsigned a1 = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + base + 2 * lane);
            const unsigned a2 = a1 + 4u * (unsigned)(300 + mis);
            const unsigned a3 = a1 + 4u * (unsigned)(2000 + mis);
            const unsigned a4 = a1 + 4u * (unsigned)(3000 + mis);
            const unsigned a5 = a1 + 4u * 6000u;
            f2 h[2], t[2], u[2], w[2];
            asm volatile(
                "ds_read_b64 %0, %8\n\tds_read_b64 %1, %8 offset:512\n\t"
                "ds_read_b64 %2, %9\n\tds_read_b64 %3, %9 offset:512\n\t"
                "ds_read_b64 %4, %10\n\tds_read_b64 %5, %10 offset:512\n\t"
                "ds_read_b64 %6, %11\n\tds_read_b64 %7, %11 offset:512\n\ts_waitcnt lgkmcnt(0)"
                : "=v"(h[0]), "=v"(h[1]), "=v"(t[0]), "=v"(t[1]), "=v"(u[0]), "=v"(u[1]), "=v"(w[0]), "=v"(w[1])
                : "v"(a1), "v"(a2), "v"(a3), "v"(a4));
            f2 o[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) o[k] = (h[k] + t[k]) + (u[k] + w[k]);
            asm volatile("ds_write_b64 %0, %1\n\tds_write_b64 %0, %2 offset:512\n\ts_waitcnt lgkmcnt(0)"
                         :
                         : "v"(a5), "v"(o[0]), "v"(o[1])
                         : "memory");
            acc += o[0].x;
        }
        base = (base + 8) & 4095;
    }
    out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// unaligned ds_read_b64 / ds_write_b64 / ds_read_b128 correctness
__global__ void check(float* out, int mis)
{
    __shared__ __attribute__((aligned(16))) float d[2048];
    const int t = threadIdx.x;
    for (int i = t; i < 2048; i += 64) d[i] = (float)i;
    __syncthreads();
    f2 v;
    f4 q;
    const unsigned addr = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + mis + 2 * t);
    const unsigned addr4 = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + mis + 4 * t);
    asm volatile("ds_read_b64 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)" : "=v"(v), "=v"(q) : "v"(addr), "v"(addr4));
    out[2 * t] = v.x;
    out[2 * t + 1] = v.y;
    out[128 + 4 * t] = q.x;
    out[128 + 4 * t + 1] = q.y;
    out[128 + 4 * t + 2] = q.z;
    out[128 + 4 * t + 3] = q.w;
    __syncthreads();
    f2 w;
    w.x = -1.0f - (float)(2 * t);
    w.y = -2.0f - (float)(2 * t);
    const unsigned wa = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)(d + 1024 + mis + 2 * t);
    asm volatile("ds_write_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(wa), "v"(w) : "memory");
    __syncthreads();
    for (int i = t; i < 256; i += 64) out[512 + i] = d[1024 + i];
}

template <int MODE>
double run(float* out, int mis, int blocks, const char* name, double bytes_per_iter_wave)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(512), 0, 0, out, mis);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(512), 0, 0, out, mis);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double waves = (double)blocks * 8;
    const double bytes = waves * NREP * bytes_per_iter_wave;
    const double bpc = bytes / (ms * 1e-3) / 2.4e9 / 256.0;
    printf("%-34s mis=%d  %.3f ms  %.1f B/clk/CU\n", name, mis, ms, bpc);
    return bpc;
}

int main()
{
    float* out;
    hipMalloc(&out, 256 * 8 * 512 * sizeof(float) * 2);
    const int blocks = 256 * 2 * 8;
    for (int mis = 0; mis < 4; ++mis) {
        float* dout;
        hipMalloc(&dout, 1024 * sizeof(float));
        hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, dout, mis);
        std::vector<float> h(1024);
        hipMemcpy(h.data(), dout, 1024 * sizeof(float), hipMemcpyDeviceToHost);
        int bad_r = 0, bad_q = 0, bad_w = 0;
        for (int i = 0; i < 128; ++i) bad_r += h[i] != (float)(mis + i);
        for (int i = 0; i < 256; ++i) bad_q += h[128 + i] != (float)(mis + i);
        for (int i = 0; i < 128; ++i) bad_w += h[512 + mis + i] != -1.0f - (float)i;
        printf("misalign %d floats: read_b64 %s, read_b128 %s, write_b64 %s\n", mis, bad_r ? "WRONG" : "ok",
               bad_q ? "WRONG" : "ok", bad_w ? "WRONG" : "ok");
        hipFree(dout);
    }
    for (int mis : {0, 1}) {
        run<0>(out, mis, blocks, "ds_read_b32", 8 * 256.0);
        run<1>(out, mis, blocks, "ds_read_b64", 8 * 512.0);
        run<2>(out, mis, blocks, "ds_read_b128", 4 * 1024.0);
        run<2>(out, mis + 2, blocks, "ds_read_b128 (+2)", 4 * 1024.0);
        run<3>(out, mis, blocks, "ds_write_b32", 8 * 256.0);
        run<4>(out, mis, blocks, "ds_write_b64", 8 * 512.0);
    }
    // merge-like loops: bytes = merge adds x 4 (one per output element)
    for (int mis : {0, 1}) {
        run<5>(out, mis, blocks, "merge b32 (adds*4B)", 4 * 256.0);
        run<6>(out, mis, blocks, "merge b64 (adds*4B)", 2 * 512.0);
        run<7>(out, mis, blocks, "merge2 b64 (level-adds*4B)", 2 * 2 * 512.0);
    }
    return 0;
}
