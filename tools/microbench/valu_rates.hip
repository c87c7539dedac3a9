// Microbenchmark (GPU box): issue cost of the fused ladder's VALU forms on
// gfx950 -- the float64 multiply / add / floor / fract /
// conversions of the window bounds against plain and packed float32 adds.
// One wave per SIMD (256-thread workgroups, one per CU), 8 independent chains
// of one instruction per loop iteration; reports shader-clock cycles per
// wave-instruction (s_memtime around the loop, wave 0 of each workgroup,
// median over workgroups).
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/valu_rates.hip -o /tmp/valu_rates && /tmp/valu_rates
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int NREP = 2048;

#define OP8_D(INS)                                                                                      \
    asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS " %4, %4\n\t" \
                 INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"                                      \
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]))
#define OP8_D2(INS)                                                                                     \
    asm volatile(INS " %0, %0, %0\n\t" INS " %1, %1, %1\n\t" INS " %2, %2, %2\n\t" INS " %3, %3, %3\n\t" \
                 INS " %4, %4, %4\n\t" INS " %5, %5, %5\n\t" INS " %6, %6, %6\n\t" INS " %7, %7, %7"     \
                 : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]), "+v"(d[4]), "+v"(d[5]), "+v"(d[6]), "+v"(d[7]))
#define OP8_F2(INS)                                                                                     \
    asm volatile(INS " %0, %0, %0\n\t" INS " %1, %1, %1\n\t" INS " %2, %2, %2\n\t" INS " %3, %3, %3\n\t" \
                 INS " %4, %4, %4\n\t" INS " %5, %5, %5\n\t" INS " %6, %6, %6\n\t" INS " %7, %7, %7"     \
                 : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]))
// conversions: float64 source, 32-bit destination (and back)
#define CVT8(INS, DST, SRC)                                                                             \
    asm volatile(INS " %0, %8\n\t" INS " %1, %9\n\t" INS " %2, %10\n\t" INS " %3, %11\n\t" INS " %4, %12\n\t" \
                 INS " %5, %13\n\t" INS " %6, %14\n\t" INS " %7, %15"                                  \
                 : "=v"(DST[0]), "=v"(DST[1]), "=v"(DST[2]), "=v"(DST[3]), "=v"(DST[4]), "=v"(DST[5]),   \
                   "=v"(DST[6]), "=v"(DST[7])                                                           \
                 : "v"(SRC[0]), "v"(SRC[1]), "v"(SRC[2]), "v"(SRC[3]), "v"(SRC[4]), "v"(SRC[5]), "v"(SRC[6]), \
                   "v"(SRC[7]))

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void bench(float* out, unsigned long long* cyc)
{
    double d[8];
    float f[8];
    unsigned u[8];
    f2 p[8];
    for (int i = 0; i < 8; ++i) {
        d[i] = 1.0 + threadIdx.x + i;
        f[i] = 1.0f + threadIdx.x + i;
        u[i] = threadIdx.x + i;
        p[i] = f2{f[i], f[i]};
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < NREP; ++it) {
        if constexpr (MODE == 0) OP8_F2("v_add_f32");
        if constexpr (MODE == 1) OP8_D2("v_add_f64");
        if constexpr (MODE == 2) OP8_D2("v_mul_f64");
        if constexpr (MODE == 3) OP8_D("v_floor_f64");
        if constexpr (MODE == 4) OP8_D("v_fract_f64");
        if constexpr (MODE == 5) OP8_D("v_trunc_f64");
        if constexpr (MODE == 6) { CVT8("v_cvt_u32_f64", u, d); asm volatile("" : "+v"(d[0]) : "v"(u[0])); }
        if constexpr (MODE == 7) { CVT8("v_cvt_f64_u32", d, u); asm volatile("" : "+v"(u[0]) : "v"(d[0])); }
        if constexpr (MODE == 8) { CVT8("v_cvt_f32_f64", f, d); asm volatile("" : "+v"(d[0]) : "v"(f[0])); }
        if constexpr (MODE == 9)
            asm volatile("v_pk_add_f32 %0, %0, %0\n\tv_pk_add_f32 %1, %1, %1\n\tv_pk_add_f32 %2, %2, %2\n\t"
                         "v_pk_add_f32 %3, %3, %3\n\tv_pk_add_f32 %4, %4, %4\n\tv_pk_add_f32 %5, %5, %5\n\t"
                         "v_pk_add_f32 %6, %6, %6\n\tv_pk_add_f32 %7, %7, %7"
                         : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7]));
        if constexpr (MODE == 10) { CVT8("v_cvt_f32_u32", f, u); asm volatile("" : "+v"(u[0]) : "v"(f[0])); }
        if constexpr (MODE == 11) OP8_F2("v_mul_f32");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += (float)d[i] + f[i] + (float)u[i] + p[i].x + p[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(const char* name, float* d_out, unsigned long long* d_cyc, int blocks)
{
    hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc);
    hipLaunchKernelGGL(bench<MODE>, dim3(blocks), dim3(256), 0, 0, d_out, d_cyc);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); return; }
    std::vector<unsigned long long> c(blocks);
    (void)hipMemcpy(c.data(), d_cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double per = (double)c[blocks / 2] / (NREP * 8.0);
    std::printf("{\"op\": \"%s\", \"cycles_per_wave_instr\": %.3f}\n", name, per);
}

int main()
{
    const int blocks = 256;
    float* d_out;
    unsigned long long* d_cyc;
    if (hipMalloc(&d_out, blocks * 256 * sizeof(float)) != hipSuccess) return 1;
    if (hipMalloc(&d_cyc, blocks * sizeof(unsigned long long)) != hipSuccess) return 1;
    run<0>("v_add_f32", d_out, d_cyc, blocks);
    run<11>("v_mul_f32", d_out, d_cyc, blocks);
    run<9>("v_pk_add_f32", d_out, d_cyc, blocks);
    run<1>("v_add_f64", d_out, d_cyc, blocks);
    run<2>("v_mul_f64", d_out, d_cyc, blocks);
    run<3>("v_floor_f64", d_out, d_cyc, blocks);
    run<4>("v_fract_f64", d_out, d_cyc, blocks);
    run<5>("v_trunc_f64", d_out, d_cyc, blocks);
    run<6>("v_cvt_u32_f64", d_out, d_cyc, blocks);
    run<7>("v_cvt_f64_u32", d_out, d_cyc, blocks);
    run<8>("v_cvt_f32_f64", d_out, d_cyc, blocks);
    run<10>("v_cvt_f32_u32", d_out, d_cyc, blocks);
    (void)hipFree(d_out);
    (void)hipFree(d_cyc);
    return 0;
}
