// Microbenchmark (GPU box): the FFA merge level loop in isolation -- LDS
// rows of p = 260 bins, 66 rows, random head/tail/shift descriptors, NLEV
// levels per launch, two 512-thread workgroups per CU -- to separate the LDS
// read, write, VALU and barrier costs of one level.
//   mode 0: full level (reads, adds, barrier, write-back, barrier)
//   mode 1: no write-back        mode 2: no barriers
//   mode 3: reads + adds only (no write-back, no barriers)
//   mode 4: head read only (no tail read, no select)
//   mode 5: full level, write-back with ds_write_addtid_b32
//   mode 6: full level, wrap select with one v_cmp per row and SALU slot masks
//   mode 7: modes 5 + 6
//   mode 8: bin-pair layout (stride Q = 262): ds_read_b64 heads, two
//           ds_read_b32 tails per pair, ds_write_b64 write-back
//   mode 9: mode 8 with the heads as two ds_read_b32
// Build: hipcc --offload-arch=gfx950 -O3 -o merge_loop merge_loop.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int P = 260, ROWS = 66, SMAX = 5, RW = 9, NLEV = 64, BLOCK = 512;
typedef const __attribute__((address_space(3))) float* lds_cptr;

typedef float f2 __attribute__((ext_vector_type(2), aligned(8)));
typedef const __attribute__((address_space(3))) f2* lds_cptr2;
__device__ __forceinline__ float ldv(lds_cptr p) { return *(const volatile __attribute__((address_space(3))) float*)p; }
__device__ __forceinline__ f2 ldv2(lds_cptr2 p) { return *(const volatile __attribute__((address_space(3))) f2*)p; }
constexpr int Q = 262;

template <int MODE>
__global__ __launch_bounds__(BLOCK, 4) void pair_bench(float* out, const unsigned* descs)
{
    __shared__ __attribute__((aligned(16))) float data[17408 + 128];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 17408 + 128; i += BLOCK) data[i] = (float)(i % 97) * 0.25f;
    __syncthreads();
    const int nr = (ROWS - wave + 7) / 8;
    for (int lev = 0; lev < NLEV; ++lev) {
        uint32_t d = 0;
        if (lane < nr) d = descs[(lev * ROWS + wave + 8 * lane) & 4095];
        float v[RW][SMAX];
        const lds_cptr l2 = (lds_cptr)data + 2 * lane, l1 = (lds_cptr)data + lane;
#pragma unroll
        for (int i = 0; i < RW; ++i) {
            const uint32_t dw = (uint32_t)__builtin_amdgcn_readlane((int)d, i);
            const int h = (int)(dw & 1023u) % ROWS, t = (int)((dw >> 10) & 1023u) % ROWS, sft = (int)(dw >> 20) % P;
            const int thr = P - sft;
            lds_cptr ta2 = l2 + (t * Q + sft), tw2 = ta2 - P;
            lds_cptr ta1 = l1 + (t * Q + sft), tw1 = ta1 - P;
            asm("" : "+v"(ta2), "+v"(tw2), "+v"(ta1), "+v"(tw1));
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const lds_cptr tp = 2 * lane >= thr - 128 * k ? tw2 : ta2;
                const float x0 = ldv(tp + 128 * k), x1 = ldv(tp + 128 * k + 1);
                float h0, h1;
                if (MODE == 8) {
                    const f2 hv = ldv2((lds_cptr2)(l2 + h * Q) + 64 * k);
                    h0 = hv.x;
                    h1 = hv.y;
                } else {
                    h0 = ldv(l2 + h * Q + 128 * k);
                    h1 = ldv(l2 + h * Q + 128 * k + 1);
                }
                v[i][2 * k] = __fadd_rn(h0, x0);
                v[i][2 * k + 1] = __fadd_rn(h1, x1);
            }
            const lds_cptr tp = lane >= thr - 256 ? tw1 : ta1;
            v[i][4] = __fadd_rn(ldv(l1 + h * Q + 256), ldv(tp + 256));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
#pragma unroll
        for (int i = 0; i < RW; ++i)
            if (i < nr) {
                float* orow = data + (wave + 8 * i) * Q;
                float* o2 = orow + 2 * lane;
                *reinterpret_cast<f2*>(o2) = f2{v[i][0], v[i][1]};
                *reinterpret_cast<f2*>(o2 + 128) = f2{v[i][2], v[i][3]};
                if (lane < P - 256) orow[256 + lane] = v[i][4];
                if (lane == 0) orow[P] = v[i][0];
            }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    out[blockIdx.x * BLOCK + tid] = data[tid];
}

template <int MODE>
__global__ __launch_bounds__(BLOCK, 4) void merge_bench(float* out, const unsigned* descs)
{
    __shared__ __attribute__((aligned(16))) float data[17408 + 128];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < 17408 + 128; i += BLOCK) data[i] = (float)(i % 97) * 0.25f;
    __syncthreads();
    const int nr = (ROWS - wave + 7) / 8;
    float acc = 0.f;
    for (int lev = 0; lev < NLEV; ++lev) {
        uint32_t d = 0;
        if (lane < nr) d = descs[(lev * ROWS + wave + 8 * lane) & 4095];
        float v[RW][SMAX];
        const lds_cptr l1 = (lds_cptr)data + lane;
#pragma unroll
        for (int i = 0; i < RW; ++i) {
            const uint32_t dw = (uint32_t)__builtin_amdgcn_readlane((int)d, i);
            const int h = (int)(dw & 1023u) % ROWS, t = (int)((dw >> 10) & 1023u) % ROWS, sft = (int)(dw >> 20) % P;
            const lds_cptr hrow = l1 + h * P;
            lds_cptr ta = l1 + (t * P + sft);
            lds_cptr tw = ta - P;
            asm("" : "+v"(ta), "+v"(tw));
            const int thr = P - sft;
            if (MODE == 6 || MODE == 7) {
                const int kw = thr >> 6;                                   // slot holding the wrap point
                const unsigned long long m = __builtin_amdgcn_ballot_w64(lane >= thr - 64 * kw);
#pragma unroll
                for (int k = 0; k < SMAX; ++k) {
                    const unsigned long long mk = k < kw ? 0ull : (k > kw ? ~0ull : m);
                    const bool sel = (mk >> lane) & 1ull;
                    const lds_cptr tp = sel ? tw : ta;
                    v[i][k] = __fadd_rn(hrow[64 * k], tp[64 * k]);
                }
            } else {
#pragma unroll
            for (int k = 0; k < SMAX; ++k) {
                if (MODE == 4) {
                    v[i][k] = hrow[64 * k];
                } else {
                    const lds_cptr tp = lane >= thr - 64 * k ? tw : ta;
                    v[i][k] = __fadd_rn(hrow[64 * k], tp[64 * k]);
                }
            }
            }
        }
        if (MODE == 0 || MODE == 1 || MODE >= 5) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        }
        if (MODE == 5 || MODE == 7) {
            const unsigned dbase = (unsigned)(size_t)(const __attribute__((address_space(3))) float*)data;
#pragma unroll
            for (int i = 0; i < RW; ++i)
                if (i < nr) {
                    const unsigned rb = __builtin_amdgcn_readfirstlane(dbase + (unsigned)((wave + 8 * i) * P) * 4u);
                    // rows of this test stay below 64 KiB + 1 KiB of offsets
                    asm volatile("s_mov_b32 m0, %5\n\ts_nop 0\n\tds_write_addtid_b32 %0\n\tds_write_addtid_b32 %1 offset:256\n\t"
                                 "ds_write_addtid_b32 %2 offset:512\n\tds_write_addtid_b32 %3 offset:768"
                                 : : "v"(v[i][0]), "v"(v[i][1]), "v"(v[i][2]), "v"(v[i][3]), "v"(v[i][4]), "s"(rb) : "memory");
                    if (lane < P - 256) data[(wave + 8 * i) * P + 256 + lane] = v[i][4];
                }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        } else if (MODE == 0 || MODE == 2 || MODE == 6) {
#pragma unroll
            for (int i = 0; i < RW; ++i)
                if (i < nr) {
                    float* orow = data + (wave + 8 * i) * P + lane;
#pragma unroll
                    for (int k = 0; k < SMAX; ++k)
                        if (64 * (k + 1) <= P || lane + 64 * k < P) orow[64 * k] = v[i][k];
                }
        } else {
#pragma unroll
            for (int i = 0; i < RW; ++i)
#pragma unroll
                for (int k = 0; k < SMAX; ++k) acc += v[i][k];
        }
        if (MODE == 0 || MODE == 1 || MODE >= 5) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        }
    }
    out[blockIdx.x * BLOCK + tid] = acc + data[tid];
}

int main()
{
    float* out;
    unsigned* descs;
    (void)hipMalloc(&out, 4096 * BLOCK * sizeof(float));
    (void)hipMalloc(&descs, 4096 * sizeof(unsigned));
    unsigned h[4096];
    unsigned x = 12345;
    for (int i = 0; i < 4096; ++i) {
        x = x * 1103515245u + 12345u;
        h[i] = x;
    }
    (void)hipMemcpy(descs, h, sizeof(h), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int grid = 256 * 2 * 8;
    auto run = [&](int mode) {
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(a);
            if (mode == 0) hipLaunchKernelGGL(merge_bench<0>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 1) hipLaunchKernelGGL(merge_bench<1>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 2) hipLaunchKernelGGL(merge_bench<2>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 3) hipLaunchKernelGGL(merge_bench<3>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 4) hipLaunchKernelGGL(merge_bench<4>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 5) hipLaunchKernelGGL(merge_bench<5>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 6) hipLaunchKernelGGL(merge_bench<6>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 7) hipLaunchKernelGGL(merge_bench<7>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 8) hipLaunchKernelGGL(pair_bench<8>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            if (mode == 9) hipLaunchKernelGGL(pair_bench<9>, dim3(grid), dim3(BLOCK), 0, 0, out, descs);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            (void)hipEventElapsedTime(&ms, a, b);
        }
        // row-levels per CU: grid / 256 workgroups x NLEV levels x ROWS rows
        const double rl = (double)grid / 256 * NLEV * ROWS;
        printf("mode %d: %.3f ms  %.1f cycles per row-level per CU (2.4 GHz)\n", mode, ms, ms * 1e-3 * 2.4e9 / rl);
    };
    for (int m = 0; m <= 9; ++m) run(m);
    return 0;
}
