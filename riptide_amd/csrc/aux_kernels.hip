// Auxiliary HIP kernels of the hot path: standalone boxcar S/N (snr1/snr2
// entry points), exact running median, dereddening (scrunch -> running median
// -> linear interpolation -> subtract) and fp64 normalisation, plus the small
// kernel-API helpers (rollback, fused_rollback_add, circular_prefix_sum).
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <cmath>

#include "common.hpp"
#include "kernels.hpp"

namespace rt {

__device__ __forceinline__ double wave_scan_d(double v, int lane)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const double y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

__device__ __forceinline__ float wave_max_f(float v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}

// ---------------------------------------------------------------------------
// Boxcar S/N over rows of a block (snr.hpp:37-65).  Two launches: (1) fp64
// circular prefix sums of each row into `cps` + the row sum, (2) per-width
// maximum of c[i+w] - c[i].  One wave per row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void snr_prefix_kernel(const float* __restrict__ x, uint64_t rows,
                                                         uint32_t cols, float* __restrict__ cps,
                                                         float* __restrict__ sums)
{
    const int lane = threadIdx.x & 63;
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* xr = x + r * cols;
    float* cr = cps + r * cols;
    const uint32_t c = (cols + 63) / 64;
    const uint32_t j0 = min(lane * c, cols), j1 = min(j0 + c, cols);
    double part = 0.0;
    for (uint32_t j = j0; j < j1; ++j) part += (double)xr[j];
    const double incl = wave_scan_d(part, lane);
    double acc = __shfl_up(incl, 1, 64);
    if (lane == 0) acc = 0.0;
    for (uint32_t j = j0; j < j1; ++j) {
        acc += (double)xr[j];
        cr[j] = (float)acc;
    }
    const float total = __shfl((float)acc, (int)((cols - 1) / c), 64);
    if (lane == 0) sums[r] = total;
}

__global__ __launch_bounds__(256) void snr_width_kernel(const float* __restrict__ cps, const float* __restrict__ sums,
                                                        uint64_t rows, uint32_t cols,
                                                        const uint32_t* __restrict__ widths, uint32_t nw,
                                                        float stdnoise, float* __restrict__ out)
{
    const int lane = threadIdx.x & 63;
    const uint64_t r = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (r >= rows) return;
    const float* cr = cps + r * cols;
    const float sum = sums[r];
    const uint32_t c = (cols + 63) / 64;
    const uint32_t j0 = min(lane * c, cols), j1 = min(j0 + c, cols);
    for (uint32_t iw = 0; iw < nw; ++iw) {
        const uint32_t w = widths[iw];
        float dmax = -INFINITY;
        for (uint32_t i = j0; i < j1; ++i) {
            const uint32_t k = i + w;
            const float ck = k < cols ? cr[k] : __fadd_rn(cr[k - cols], sum);
            dmax = fmaxf(dmax, __fsub_rn(ck, cr[i]));
        }
        dmax = wave_max_f(dmax);
        if (lane == 0) {
            const float h = sqrtf((float)(cols - w) / (float)((uint64_t)cols * w));
            const float b = (float)w / (float)(cols - w) * h;
            out[r * nw + iw] = ((h + b) * dmax - b * sum) / stdnoise;
        }
    }
}

hipError_t launch_snr_rows(const float* x, uint64_t rows, uint32_t cols, const uint32_t* d_widths,
                           uint32_t nw, float stdnoise, float* cps_scratch, float* out, hipStream_t s)
{
    if (!rows) return hipSuccess;
    const uint32_t blocks = (uint32_t)((rows + 3) / 4);
    float* sums = cps_scratch + rows * cols;
    hipLaunchKernelGGL(snr_prefix_kernel, dim3(blocks), dim3(256), 0, s, x, rows, cols, cps_scratch, sums);
    hipLaunchKernelGGL(snr_width_kernel, dim3(blocks), dim3(256), 0, s, cps_scratch, sums, rows, cols,
                       d_widths, nw, stdnoise, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Running median (running_median.hpp:100-132): out[i] = the (w/2)-th order
// statistic of x[clamp(i - w/2 + j, 0, n-1)], j in [0, w).  Exact: the result
// is one of the window's values, as with the reference's quickselect.
// ---------------------------------------------------------------------------
constexpr int kRmedTile = 256;
constexpr int kRmedSmallMax = 255;

// Small windows: the block stages its span in LDS; one thread per output
// counts, for each candidate, how many window values are < and <= it.
__global__ __launch_bounds__(kRmedTile) void rmed_small_kernel(const float* __restrict__ x, uint64_t n, int width,
                                                               float* __restrict__ out, uint64_t x_stride,
                                                               uint64_t out_stride)
{
    __shared__ float span[kRmedTile + kRmedSmallMax];
    x += (uint64_t)blockIdx.y * x_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    const int half = width / 2;
    const int64_t i0 = (int64_t)blockIdx.x * kRmedTile;
    for (int k = threadIdx.x; k < kRmedTile + width - 1; k += kRmedTile) {
        int64_t idx = i0 - half + k;
        idx = idx < 0 ? 0 : (idx >= (int64_t)n ? (int64_t)n - 1 : idx);
        span[k] = x[idx];
    }
    __syncthreads();
    const int64_t i = i0 + threadIdx.x;
    if (i >= (int64_t)n) return;
    const float* win = span + threadIdx.x;
    float res = win[half];
    for (int j = 0; j < width; ++j) {
        const float v = win[j];
        int less = 0, leq = 0;
        for (int k = 0; k < width; ++k) {
            const float u = win[k];
            less += u < v;
            leq += u <= v;
        }
        if (less <= half && half < leq) { res = v; break; }
    }
    out[i] = res;
}

// outputs per thread of rmed_run_kernel (odd: the 64 lanes' LDS reads at
// stride kRmedRun land on distinct banks)
constexpr int kRmedRun = 3;   // 3 / 5 / 7 / 9: 197 / 202 / 234 / 264 us (profiles/r05p7_prep_rmed_run.log)

__device__ __forceinline__ void rank_of(const float* win, int width, float v, int& less, int& leq)
{
    // four independent counter pairs: the window's LDS reads go out four at
    // a time instead of one read-compare-add chain
    int l0 = 0, l1 = 0, l2 = 0, l3 = 0, q0 = 0, q1 = 0, q2 = 0, q3 = 0;
    int k = 0;
    for (; k + 4 <= width; k += 4) {
        const float u0 = win[k], u1 = win[k + 1], u2 = win[k + 2], u3 = win[k + 3];
        l0 += u0 < v; q0 += u0 <= v;
        l1 += u1 < v; q1 += u1 <= v;
        l2 += u2 < v; q2 += u2 <= v;
        l3 += u3 < v; q3 += u3 <= v;
    }
    for (; k < width; ++k) {
        const float u = win[k];
        l0 += u < v;
        q0 += u <= v;
    }
    less = (l0 + l1) + (l2 + l3);
    leq = (q0 + q1) + (q2 + q3);
}

// One pass over the window: the rank of v (values < v, values <= v) and its
// neighbours in sorted order (the largest value below v, the smallest above).
__device__ __forceinline__ void rank_nb(const float* win, int width, float v, int& less, int& leq, float& below,
                                        float& above)
{
    int l0 = 0, l1 = 0, q0 = 0, q1 = 0;
    float b0 = -INFINITY, b1 = -INFINITY, a0 = INFINITY, a1 = INFINITY;
    int k = 0;
    for (; k + 2 <= width; k += 2) {
        const float u0 = win[k], u1 = win[k + 1];
        l0 += u0 < v; q0 += u0 <= v;
        l1 += u1 < v; q1 += u1 <= v;
        b0 = (u0 < v && u0 > b0) ? u0 : b0;
        b1 = (u1 < v && u1 > b1) ? u1 : b1;
        a0 = (u0 > v && u0 < a0) ? u0 : a0;
        a1 = (u1 > v && u1 < a1) ? u1 : a1;
    }
    if (k < width) {
        const float u = win[k];
        l0 += u < v; q0 += u <= v;
        b0 = (u < v && u > b0) ? u : b0;
        a0 = (u > v && u < a0) ? u : a0;
    }
    less = l0 + l1;
    leq = q0 + q1;
    below = b0 > b1 ? b0 : b1;
    above = a0 < a1 ? a0 : a1;
}

// Small windows, kRmedRun consecutive outputs per thread, each found by a
// walk in sorted order from a starting value m: one pass gives m's rank and
// its two neighbours; m is the median when its rank interval holds w/2,
// else the walk moves to the neighbour on the median's side.  The first
// output starts from the window value closest to the window's mean (for
// noise-like data a few places from the median; the previous round's full
// counting search tried ~w/2 candidates at w reads each), each next one from
// the previous median (one sample leaves, one enters: at most one step).  A
// walk longer than kRmedMaxSteps or one that runs off the window's values
// (NaN / infinite data) takes the full counting search.  The value returned
// is the window's first element equal to the median (the element the full
// search returns: the median value is unique, and of equal values it picks
// the first in window order -- +0.0 / -0.0 included).  kRmedRun is odd, so
// the 64 lanes' LDS reads (stride kRmedRun) land on distinct banks.
constexpr int kRmedMaxSteps = 48;

template <int RUN>
__global__ __launch_bounds__(kRmedTile) void rmed_run_kernel(const float* __restrict__ x, uint64_t n, int width,
                                                             float* __restrict__ out, uint64_t x_stride,
                                                             uint64_t out_stride)
{
    __shared__ float span[kRmedTile * RUN + kRmedSmallMax];
    x += (uint64_t)blockIdx.y * x_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    const int half = width / 2;
    const int64_t i0 = (int64_t)blockIdx.x * (kRmedTile * RUN);
    for (int k = threadIdx.x; k < kRmedTile * RUN + width - 1; k += kRmedTile) {
        int64_t idx = i0 - half + k;
        idx = idx < 0 ? 0 : (idx >= (int64_t)n ? (int64_t)n - 1 : idx);
        span[k] = x[idx];
    }
    __syncthreads();
    const int64_t ib = i0 + (int64_t)threadIdx.x * RUN;
    float m = 0.0f;
    bool have = false;
    for (int r = 0; r < RUN; ++r) {
        if (ib + r >= (int64_t)n) return;
        const float* win = span + threadIdx.x * RUN + r;
        if (!have) {
            // the window value closest to the window's mean
            float s0 = 0.0f, s1 = 0.0f;
            int k = 0;
            for (; k + 2 <= width; k += 2) {
                s0 += win[k];
                s1 += win[k + 1];
            }
            if (k < width) s0 += win[k];
            const float mean = (s0 + s1) / (float)width;
            m = win[half];
            float bd = fabsf(m - mean);
            for (k = 0; k < width; ++k) {
                const float d = fabsf(win[k] - mean);
                if (d < bd) {
                    bd = d;
                    m = win[k];
                }
            }
        }
        bool found = false;
        for (int step = 0; step < kRmedMaxSteps; ++step) {
            int less, leq;
            float below, above;
            rank_nb(win, width, m, less, leq, below, above);
            if (less <= half && half < leq) {
                found = true;
                break;
            }
            const float c = less > half ? below : above;
            if (!(c > -INFINITY && c < INFINITY)) break;
            m = c;
        }
        if (found) {
            // the window's first element equal to the median
            int k = 0;
            while (k < width && !(win[k] == m)) ++k;
            if (k < width) m = win[k];
            else found = false;
        }
        if (!found) {
            // the full counting search (rmed_small_kernel)
            float res = win[half];
            for (int j = 0; j < width; ++j) {
                const float v = win[j];
                int less, leq;
                rank_of(win, width, v, less, leq);
                if (less <= half && half < leq) { res = v; break; }
            }
            m = res;
        }
        have = true;
        out[ib + r] = m;
    }
}

__device__ __forceinline__ uint32_t float_key(float v)
{
    const uint32_t b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ float key_float(uint32_t k)
{
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// Large windows: one block per output, radix select on order-preserving keys.
__global__ __launch_bounds__(256) void rmed_large_kernel(const float* __restrict__ x, uint64_t n, int width,
                                                         float* __restrict__ out, uint64_t x_stride,
                                                         uint64_t out_stride)
{
    __shared__ int wsum[4];
    x += (uint64_t)blockIdx.y * x_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    const int64_t i = blockIdx.x;
    const int half = width / 2;
    uint32_t prefix = 0, mask = 0;
    int k = half;
    for (int bit = 31; bit >= 0; --bit) {
        const uint32_t b = 1u << bit;
        int cnt = 0;
        for (int j = threadIdx.x; j < width; j += 256) {
            int64_t idx = i - half + j;
            idx = idx < 0 ? 0 : (idx >= (int64_t)n ? (int64_t)n - 1 : idx);
            const uint32_t key = float_key(x[idx]);
            cnt += ((key & mask) == prefix) && !(key & b);
        }
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
        __syncthreads();
        const int zeros = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        __syncthreads();
        if (k >= zeros) {
            k -= zeros;
            prefix |= b;
        }
        mask |= b;
    }
    if (threadIdx.x == 0) out[i] = key_float(prefix);
}

hipError_t launch_running_median(const float* x, uint64_t n, uint32_t width, float* out, uint64_t x_stride,
                                 uint64_t out_stride, uint32_t batch, hipStream_t s)
{
    if (!n || !batch) return hipSuccess;
    if (width <= (uint32_t)kRmedSmallMax && std::getenv("RIPTIDE_AMD_RMED_COUNTING")) {
        // A/B: one counting search per output
        hipLaunchKernelGGL(rmed_small_kernel, dim3((uint32_t)((n + kRmedTile - 1) / kRmedTile), batch),
                           dim3(kRmedTile), 0, s, x, n, (int)width, out, x_stride, out_stride);
    } else if (width <= (uint32_t)kRmedSmallMax) {
        // read per launch (like RIPTIDE_AMD_RMED_COUNTING), so one process
        // can test every run length
        const char* e = std::getenv("RIPTIDE_AMD_RMED_RUN");
        const int run = e ? std::atoi(e) : kRmedRun;
        auto go = [&](auto kern, int r) {
            const uint64_t per = (uint64_t)kRmedTile * r;
            hipLaunchKernelGGL(kern, dim3((uint32_t)((n + per - 1) / per), batch), dim3(kRmedTile), 0, s, x, n,
                               (int)width, out, x_stride, out_stride);
        };
        if (run == 5) go(rmed_run_kernel<5>, 5);
        else if (run == 7) go(rmed_run_kernel<7>, 7);
        else if (run == 9) go(rmed_run_kernel<9>, 9);
        else go(rmed_run_kernel<kRmedRun>, kRmedRun);
    } else {
        hipLaunchKernelGGL(rmed_large_kernel, dim3((uint32_t)n, batch), dim3(256), 0, s, x, n, (int)width,
                           out, x_stride, out_stride);
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Dereddening (time_series.py:93-122, running_medians.py:40-83)
// ---------------------------------------------------------------------------
// numpy float32 pairwise summation (the add-reduce inner loop used by
// ndarray.mean over a contiguous axis): blocks of <= 128 with 8 accumulators,
// recursive halving at multiples of 8 above that; the reduction starts from 0.
__device__ float np_pairwise_leaf(const float* a, int n)
{
    if (n < 8) {
        float r = 0.0f;
        for (int i = 0; i < n; ++i) r = __fadd_rn(r, a[i]);
        return r;
    }
    float r0 = a[0], r1 = a[1], r2 = a[2], r3 = a[3], r4 = a[4], r5 = a[5], r6 = a[6], r7 = a[7];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
        r0 = __fadd_rn(r0, a[i + 0]); r1 = __fadd_rn(r1, a[i + 1]);
        r2 = __fadd_rn(r2, a[i + 2]); r3 = __fadd_rn(r3, a[i + 3]);
        r4 = __fadd_rn(r4, a[i + 4]); r5 = __fadd_rn(r5, a[i + 5]);
        r6 = __fadd_rn(r6, a[i + 6]); r7 = __fadd_rn(r7, a[i + 7]);
    }
    float res = __fadd_rn(__fadd_rn(__fadd_rn(r0, r1), __fadd_rn(r2, r3)),
                          __fadd_rn(__fadd_rn(r4, r5), __fadd_rn(r6, r7)));
    for (; i < n; ++i) res = __fadd_rn(res, a[i]);
    return res;
}

__device__ float np_pairwise_sum(const float* a, int n)
{
    if (n <= 128) return np_pairwise_leaf(a, n);
    int offs[24], ns[24], st[24];
    float left[24];
    int sp = 0;
    offs[0] = 0; ns[0] = n; st[0] = 0;
    float ret = 0.0f;
    while (sp >= 0) {
        const int off = offs[sp], nn = ns[sp];
        if (nn <= 128) {
            ret = np_pairwise_leaf(a + off, nn);
            --sp;
            continue;
        }
        int n2 = nn / 2;
        n2 -= n2 % 8;
        if (st[sp] == 0) {
            st[sp] = 1;
            ++sp; offs[sp] = off; ns[sp] = n2; st[sp] = 0;
        } else if (st[sp] == 1) {
            left[sp] = ret;
            st[sp] = 2;
            ++sp; offs[sp] = off + n2; ns[sp] = nn - n2; st[sp] = 0;
        } else {
            ret = __fadd_rn(left[sp], ret);
            --sp;
        }
    }
    return ret;
}

// np_pairwise_sum for the counts whose halving tree has one level (n <= 128,
// or both halves <= 128: np_pairwise_split2), without the general form's
// explicit stack (private arrays indexed at run time live in scratch memory)
__host__ __device__ inline bool np_pairwise_split2(int n)
{
    int n2 = n / 2;
    n2 -= n2 % 8;
    return n <= 128 || n - n2 <= 128;
}

__device__ __forceinline__ float np_pairwise_sum2(const float* a, int n)
{
    if (n <= 128) return np_pairwise_leaf(a, n);
    int n2 = n / 2;
    n2 -= n2 % 8;
    const float left = np_pairwise_leaf(a, n2);
    return __fadd_rn(left, np_pairwise_leaf(a + n2, n - n2));
}

// scrunch_kernel for np_pairwise_split2(factor) <= kScrunchMaxFactor: 64
// outputs per block, their 64 * factor input samples staged in LDS by the
// block's four waves with coalesced (16-byte where aligned) loads -- one
// thread per output reading its own block straight from global memory
// touched 64 cache lines per load instruction and re-fetched them from L2 --
// then one lane per output sums its block from LDS in numpy's pairwise order.
constexpr uint32_t kScrunchMaxFactor = 256;

__global__ __launch_bounds__(256) void scrunch2_kernel(const float* __restrict__ x, uint64_t n_out, uint32_t factor,
                                                       float* __restrict__ out, uint64_t x_stride, uint64_t out_stride,
                                                       int vec)
{
    extern __shared__ float stage[];
    const uint64_t i0 = (uint64_t)blockIdx.x * 64;
    const uint32_t rows = (uint32_t)min<uint64_t>(64, n_out - i0);
    const uint32_t len = rows * factor;
    const float* src = x + (uint64_t)blockIdx.y * x_stride + i0 * factor;
    if (vec) {   // src 16-byte aligned (launch: x, x_stride and 64 * factor)
        const uint32_t n4 = len / 4;
        for (uint32_t k = threadIdx.x; k < n4; k += 256)
            reinterpret_cast<float4*>(stage)[k] = reinterpret_cast<const float4*>(src)[k];
        for (uint32_t k = 4 * n4 + threadIdx.x; k < len; k += 256) stage[k] = src[k];
    } else {
        for (uint32_t k = threadIdx.x; k < len; k += 256) stage[k] = src[k];
    }
    __syncthreads();
    if (threadIdx.x >= rows) return;
    const float sum = np_pairwise_sum2(stage + threadIdx.x * factor, (int)factor);
    out[(uint64_t)blockIdx.y * out_stride + i0 + threadIdx.x] = (float)((double)sum / (double)factor);
}

// scrunch(): mean of consecutive blocks of `factor` samples; numpy divides the
// float32 sum by an np.intp count, i.e. in float64, then casts to float32.
__global__ __launch_bounds__(256) void scrunch_kernel(const float* __restrict__ x, uint64_t n_out, uint32_t factor,
                                                      float* __restrict__ out, uint64_t x_stride, uint64_t out_stride)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_out) return;
    x += (uint64_t)blockIdx.y * x_stride + i * factor;
    out += (uint64_t)blockIdx.y * out_stride;
    const float s = np_pairwise_sum(x, (int)factor);
    out[i] = (float)((double)s / (double)factor);
}

hipError_t launch_scrunch(const float* x, uint64_t n_out, uint32_t factor, float* out, uint64_t x_stride,
                          uint64_t out_stride, uint32_t batch, hipStream_t s)
{
    if (!n_out || !batch) return hipSuccess;
    if (factor <= kScrunchMaxFactor && np_pairwise_split2((int)factor)) {
        const int vec = ((uintptr_t)x % 16) == 0 && x_stride % 4 == 0 && (64 * factor) % 4 == 0;
        hipLaunchKernelGGL(scrunch2_kernel, dim3((uint32_t)((n_out + 63) / 64), batch), dim3(256),
                           64 * factor * sizeof(float), s, x, n_out, factor, out, x_stride, out_stride, vec);
    }
    else
        hipLaunchKernelGGL(scrunch_kernel, dim3((uint32_t)((n_out + 255) / 256), batch), dim3(256), 0, s,
                           x, n_out, factor, out, x_stride, out_stride);
    return hipGetLastError();
}

// np.interp(i, xp, fp) (compiled_base.c arr_interp) for xp[j] = j*factor +
// (factor-1)/2, fp = rmed_lo: slope*(x - xp[j]) + fp[j], unfused, in float64.
__device__ double np_interp_at(uint64_t i, const float* __restrict__ fp, uint64_t n_lo, uint32_t factor)
{
    const double c = 0.5 * ((double)factor - 1.0);
    const double xv = (double)i;
    auto xp = [&](int64_t j) { return (double)(j * (int64_t)factor) + c; };
    const int64_t last = (int64_t)n_lo - 1;
    if (n_lo == 1 || xv < xp(0)) return (double)fp[0];
    if (xv > xp(last)) return (double)fp[last];
    int64_t j = (int64_t)floor((xv - c) / (double)factor);
    if (j < 0) j = 0;
    if (j > last) j = last;
    while (j > 0 && xp(j) > xv) --j;
    while (j < last && xp(j + 1) <= xv) ++j;
    if (j == last || xp(j) == xv) return (double)fp[j];
    const double y0 = (double)fp[j], y1 = (double)fp[j + 1];
    const double slope = __ddiv_rn(__dsub_rn(y1, y0), __dsub_rn(xp(j + 1), xp(j)));
    return __dadd_rn(__dmul_rn(slope, __dsub_rn(xv, xp(j))), y0);
}

// The segment slopes of np_interp_at, computed once per segment instead of
// once per sample: slope[j] = (fp[j + 1] - fp[j]) / (xp[j + 1] - xp[j]), the
// same float64 operations.
__global__ __launch_bounds__(256) void interp_slope_kernel(const float* __restrict__ fp, uint64_t n_lo, uint32_t factor,
                                                           double* __restrict__ slope, uint64_t lo_stride)
{
    const uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (j + 1 >= n_lo) return;
    fp += (uint64_t)blockIdx.y * lo_stride;
    slope += (uint64_t)blockIdx.y * lo_stride;
    const double c = 0.5 * ((double)factor - 1.0);
    const double x0 = (double)(j * (uint64_t)factor) + c, x1 = (double)((j + 1) * (uint64_t)factor) + c;
    slope[j] = __ddiv_rn(__dsub_rn((double)fp[j + 1], (double)fp[j]), __dsub_rn(x1, x0));
}

// np_interp_at with 32-bit indices (series below 2^31 samples: every double
// below is an exact small integer or half-integer), the segment index by
// integer arithmetic (xp[j] = j * factor + c, c = (factor - 1) / 2: j =
// floor((2i - factor + 1) / (2 factor)) for xv >= xp[0], exact; the guards of
// np_interp_at kept) and the slope from the table: the same float64 result.
__device__ __forceinline__ double np_interp_fast(uint32_t i, const float* __restrict__ fp,
                                                 const double* __restrict__ slope, uint32_t n_lo, uint32_t factor)
{
    const double c = 0.5 * ((double)factor - 1.0);
    const double xv = (double)i;
    auto xp = [&](uint32_t j) { return (double)(j * factor) + c; };
    const uint32_t last = n_lo - 1;
    if (n_lo == 1 || xv < c) return (double)fp[0];
    if (xv > xp(last)) return (double)fp[last];
    uint32_t j = (2u * i + 1u - factor) / (2u * factor);
    if (j > last) j = last;
    while (j > 0 && xp(j) > xv) --j;
    while (j < last && xp(j + 1) <= xv) ++j;
    if (j == last || xp(j) == xv) return (double)fp[j];
    return __dadd_rn(__dmul_rn(slope[j], __dsub_rn(xv, xp(j))), (double)fp[j]);
}

// out[i] = float32(x[i] - interp(i))  (time_series.py:118-122), the slopes
// from interp_slope_kernel (factor > 1, n < 2^30).  STATS: the block's sums
// of out and out^2 in float64 (partials[2 * (y * gridDim.x + x) + {0, 1}])
// for the normalisation that follows (norm_stats_finalize_kernel), saving
// its two read passes of the series.
constexpr uint32_t kDeredGroups = 4;   // deredden_slope_kernel: 16 samples per thread, 4096 per block

template <bool STATS>
__global__ __launch_bounds__(256) void deredden_slope_kernel(const float* __restrict__ x, uint32_t n,
                                                             const float* __restrict__ fp, const double* __restrict__ slope,
                                                             uint32_t n_lo, uint32_t factor, float* __restrict__ out,
                                                             uint64_t x_stride, uint64_t lo_stride, uint64_t out_stride,
                                                             double* __restrict__ partials)
{
    // kDeredGroups groups of four consecutive samples per thread (16-byte
    // loads and stores: the launch checks the strides and bases), the
    // block's groups interleaved for coalescing
    x += (uint64_t)blockIdx.y * x_stride;
    fp += (uint64_t)blockIdx.y * lo_stride;
    slope += (uint64_t)blockIdx.y * lo_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    double sum = 0.0, sq = 0.0;
#pragma unroll
    for (uint32_t g = 0; g < kDeredGroups; ++g) {
        const uint32_t i0 = 4u * (blockIdx.x * 256u * kDeredGroups + g * 256u + threadIdx.x);
        if (i0 < n) {
            if (i0 + 4 <= n && factor >= 4) {
                const float4 v = *reinterpret_cast<const float4*>(x + i0);
                // the segment j of sample i0 from a float estimate corrected
                // by np_interp_fast's exact tests, on xj = xp[j] carried by
                // adding / subtracting factor (exact: integers and
                // half-integers below 2^31); factor >= 4, so i0 .. i0 + 3 lie
                // in segment j or j + 1, whose fp / slope loads go out once,
                // ahead of the four samples
                const double c = 0.5 * ((double)factor - 1.0), df = (double)factor;
                const uint32_t last = n_lo - 1;
                const double xlast = (double)(last * factor) + c;
                const double x0 = (double)i0;
                const float est = ((float)(2u * i0 + 1u) - (float)factor) / (float)(2u * factor);
                uint32_t j = est > 0.0f ? min((uint32_t)est, last) : 0u;
                double xj = (double)(j * factor) + c;
                while (j > 0 && xj > x0) {
                    --j;
                    xj -= df;
                }
                while (j < last && xj + df <= x0) {
                    ++j;
                    xj += df;
                }
                const uint32_t j1 = min(j + 1, last);
                const double fa = (double)fp[j], fb = (double)fp[j1];
                const double sa = slope[min(j, last - 1)], sb = slope[min(j1, last - 1)];
                float rr[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const double xv = x0 + (double)t;
                    double y;
                    if (xv < c) {
                        y = (double)fp[0];
                    } else if (xv > xlast) {
                        y = (double)fp[last];
                    } else {
                        const bool nx = j < last && xj + df <= xv;
                        const uint32_t jj = nx ? j1 : j;
                        const double xp = nx ? xj + df : xj, fv = nx ? fb : fa, sl = nx ? sb : sa;
                        y = (jj == last || xp == xv) ? fv : __dadd_rn(__dmul_rn(sl, __dsub_rn(xv, xp)), fv);
                    }
                    const float xs = t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w;
                    rr[t] = (float)__dsub_rn((double)xs, y);
                    if (STATS) {
                        const double e = (double)rr[t];
                        sum += e;
                        sq += e * e;
                    }
                }
                *reinterpret_cast<float4*>(out + i0) = make_float4(rr[0], rr[1], rr[2], rr[3]);
            } else {
                for (uint32_t i = i0; i < min(i0 + 4, n); ++i) {
                    const float r = (float)__dsub_rn((double)x[i], np_interp_fast(i, fp, slope, n_lo, factor));
                    out[i] = r;
                    if (STATS) {
                        sum += (double)r;
                        sq += (double)r * (double)r;
                    }
                }
            }
        }
    }
    if (STATS) {
        __shared__ double sh[8];
        for (int o = 32; o > 0; o >>= 1) {
            sum += __shfl_xor(sum, o, 64);
            sq += __shfl_xor(sq, o, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            sh[threadIdx.x >> 6] = sum;
            sh[4 + (threadIdx.x >> 6)] = sq;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double* p = partials + 2 * ((uint64_t)blockIdx.y * gridDim.x + blockIdx.x);
            p[0] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
            p[1] = (sh[4] + sh[5]) + (sh[6] + sh[7]);
        }
    }
}

// mean = sum / n and var = sumsq / n - mean^2 of one trial (blockIdx.x) from
// deredden_slope_kernel<true>'s per-block partials, into stats[2b], [2b + 1]
// as norm_finalize_kernel leaves them.  The dereddened series has mean ~0
// (the running median is subtracted), so the one-pass variance loses nothing
// to cancellation at float64 precision.
__global__ __launch_bounds__(256) void norm_stats_finalize_kernel(const double* __restrict__ partials, uint32_t nblocks,
                                                                  uint64_t n, double* __restrict__ stats)
{
    __shared__ double sh[8];
    double s = 0.0, q = 0.0;
    const double* p = partials + 2 * (uint64_t)blockIdx.x * nblocks;
    for (uint32_t i = threadIdx.x; i < nblocks; i += 256) {
        s += p[2 * i];
        q += p[2 * i + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        q += __shfl_xor(q, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        sh[threadIdx.x >> 6] = s;
        sh[4 + (threadIdx.x >> 6)] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const double mean = ((sh[0] + sh[1]) + (sh[2] + sh[3])) / (double)n;
        const double msq = ((sh[4] + sh[5]) + (sh[6] + sh[7])) / (double)n;
        stats[2 * blockIdx.x] = mean;
        stats[2 * blockIdx.x + 1] = fmax(msq - mean * mean, 0.0);
    }
}

// the one-sample-per-thread form (rows not 16-byte aligned)
__global__ __launch_bounds__(256) void deredden_slope1_kernel(const float* __restrict__ x, uint32_t n,
                                                              const float* __restrict__ fp, const double* __restrict__ slope,
                                                              uint32_t n_lo, uint32_t factor, float* __restrict__ out,
                                                              uint64_t x_stride, uint64_t lo_stride, uint64_t out_stride)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    x += (uint64_t)blockIdx.y * x_stride;
    fp += (uint64_t)blockIdx.y * lo_stride;
    slope += (uint64_t)blockIdx.y * lo_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    out[i] = (float)__dsub_rn((double)x[i], np_interp_fast(i, fp, slope, n_lo, factor));
}

// out[i] = float32(x[i] - interp(i))  (time_series.py:118-122)
__global__ __launch_bounds__(256) void deredden_subtract_kernel(const float* __restrict__ x, uint64_t n,
                                                                const float* __restrict__ fp, uint64_t n_lo,
                                                                uint32_t factor, float* __restrict__ out,
                                                                uint64_t x_stride, uint64_t lo_stride,
                                                                uint64_t out_stride)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    x += (uint64_t)blockIdx.y * x_stride;
    fp += (uint64_t)blockIdx.y * lo_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    out[i] = (float)__dsub_rn((double)x[i], np_interp_at(i, fp, n_lo, factor));
}

hipError_t launch_deredden_subtract(const float* x, uint64_t n, const float* rmed_lo, uint64_t n_lo,
                                    uint32_t factor, float* out, uint64_t x_stride, uint64_t lo_stride,
                                    uint64_t out_stride, uint32_t batch, hipStream_t s, double* slopes)
{
    if (!n || !batch) return hipSuccess;
    if (slopes && factor > 1 && n_lo > 1 && n < (1ull << 31) && !std::getenv("RIPTIDE_AMD_INTERP_PER_SAMPLE")) {
        hipLaunchKernelGGL(interp_slope_kernel, dim3((uint32_t)((n_lo + 255) / 256), batch), dim3(256), 0, s, rmed_lo,
                           n_lo, factor, slopes, lo_stride);
        const bool vec = ((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0 && x_stride % 4 == 0 &&
                         out_stride % 4 == 0 && n < (1ull << 30);
        if (vec)
            hipLaunchKernelGGL(deredden_slope_kernel<false>, dim3((uint32_t)dered_norm_blocks(n), batch), dim3(256), 0,
                               s, x, (uint32_t)n, rmed_lo, (const double*)slopes, (uint32_t)n_lo, factor, out, x_stride,
                               lo_stride, out_stride, nullptr);
        else
            hipLaunchKernelGGL(deredden_slope1_kernel, dim3((uint32_t)((n + 255) / 256), batch), dim3(256), 0, s, x,
                               (uint32_t)n, rmed_lo, (const double*)slopes, (uint32_t)n_lo, factor, out, x_stride,
                               lo_stride, out_stride);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(deredden_subtract_kernel, dim3((uint32_t)((n + 255) / 256), batch), dim3(256), 0, s,
                       x, n, rmed_lo, n_lo, factor, out, x_stride, lo_stride, out_stride);
    return hipGetLastError();
}

// fast_running_median output (running_medians.py:81-83): the interpolated
// running median itself, float64.
__global__ __launch_bounds__(256) void interp_kernel(uint64_t n, const float* __restrict__ fp, uint64_t n_lo,
                                                     uint32_t factor, double* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) out[i] = np_interp_at(i, fp, n_lo, factor);
}

hipError_t launch_interp(uint64_t n, const float* rmed_lo, uint64_t n_lo, uint32_t factor, double* out,
                         hipStream_t s)
{
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(interp_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, n, rmed_lo, n_lo,
                       factor, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Normalisation (time_series.py:66-90): mean and variance in float64 (two
// passes, as numpy's var), then float32((x - mean) / sqrt(var)).
// ---------------------------------------------------------------------------
constexpr int kNormBlock = 256;

__device__ __forceinline__ double block_sum_d(double v, double* sh)
{
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    if (threadIdx.x == 0) t = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    __syncthreads();
    return t;
}

// mode 0: partial sums of x; mode 1: partial sums of (x - mean)^2, mean = stats[2*b]
__global__ __launch_bounds__(kNormBlock) void norm_partial_kernel(const float* __restrict__ x, uint64_t n,
                                                                  uint64_t x_stride, double* __restrict__ partials,
                                                                  const double* __restrict__ stats, int mode)
{
    __shared__ double sh[4];
    x += (uint64_t)blockIdx.y * x_stride;
    const double mean = mode ? stats[2 * blockIdx.y] : 0.0;
    double acc = 0.0;
    for (uint64_t i = (uint64_t)blockIdx.x * kNormBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kNormBlock) {
        const double v = (double)x[i];
        if (mode) {
            const double d = v - mean;
            acc += d * d;
        } else {
            acc += v;
        }
    }
    const double t = block_sum_d(acc, sh);
    if (threadIdx.x == 0) partials[(uint64_t)blockIdx.y * gridDim.x + blockIdx.x] = t;
}

// norm_partial_kernel with 16-byte loads, two per iteration (16-byte aligned
// rows): the same float64 sums in another order (a per-thread order; numpy's
// pairwise order is matched by neither, the tests hold the result to 2e-6).
__global__ __launch_bounds__(kNormBlock) void norm_partial4_kernel(const float* __restrict__ x, uint64_t n,
                                                                   uint64_t x_stride, double* __restrict__ partials,
                                                                   const double* __restrict__ stats, int mode)
{
    __shared__ double sh[4];
    x += (uint64_t)blockIdx.y * x_stride;
    const double mean = mode ? stats[2 * blockIdx.y] : 0.0;
    double a0 = 0.0, a1 = 0.0;
    const uint64_t n4 = n >> 2;
    const uint64_t step = (uint64_t)gridDim.x * kNormBlock;
    auto add4 = [&](const float4 v, double& acc) {
        const double e[4] = {(double)v.x, (double)v.y, (double)v.z, (double)v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (mode) {
                const double d = e[k] - mean;
                acc += d * d;
            } else {
                acc += e[k];
            }
        }
    };
    uint64_t i = (uint64_t)blockIdx.x * kNormBlock + threadIdx.x;
    for (; i + step < n4; i += 2 * step) {
        const float4 v0 = reinterpret_cast<const float4*>(x)[i];
        const float4 v1 = reinterpret_cast<const float4*>(x)[i + step];
        add4(v0, a0);
        add4(v1, a1);
    }
    if (i < n4) add4(reinterpret_cast<const float4*>(x)[i], a0);
    // the n mod 4 tail: block 0
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const double v = (double)x[4 * n4 + threadIdx.x];
        if (mode) {
            const double d = v - mean;
            a1 += d * d;
        } else {
            a1 += v;
        }
    }
    const double t = block_sum_d(a0 + a1, sh);
    if (threadIdx.x == 0) partials[(uint64_t)blockIdx.y * gridDim.x + blockIdx.x] = t;
}

__global__ __launch_bounds__(kNormBlock) void norm_finalize_kernel(const double* __restrict__ partials, uint32_t nblocks,
                                                                   uint64_t n, double* __restrict__ stats, int mode)
{
    __shared__ double sh[4];
    double acc = 0.0;
    for (uint32_t i = threadIdx.x; i < nblocks; i += kNormBlock) acc += partials[(uint64_t)blockIdx.x * nblocks + i];
    const double t = block_sum_d(acc, sh);
    if (threadIdx.x == 0) stats[2 * blockIdx.x + mode] = t / (double)n;
}

// four samples per thread (16-byte aligned rows; norm_apply_kernel otherwise).
// x and out may be the same buffer (launch_deredden_normalise applies in
// place), so neither is __restrict__.
__global__ __launch_bounds__(256) void norm_apply4_kernel(const float* x, uint64_t n,
                                                          const double* __restrict__ stats, float* out,
                                                          uint64_t x_stride, uint64_t out_stride)
{
    const uint64_t i0 = 4 * ((uint64_t)blockIdx.x * 256 + threadIdx.x);
    if (i0 >= n) return;
    const double mean = stats[2 * blockIdx.y], var = stats[2 * blockIdx.y + 1];
    const double norm = sqrt(var);
    x += (uint64_t)blockIdx.y * x_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    if (i0 + 4 <= n) {
        const float4 v = *reinterpret_cast<const float4*>(x + i0);
        float4 r;
        r.x = (float)__ddiv_rn(__dsub_rn((double)v.x, mean), norm);
        r.y = (float)__ddiv_rn(__dsub_rn((double)v.y, mean), norm);
        r.z = (float)__ddiv_rn(__dsub_rn((double)v.z, mean), norm);
        r.w = (float)__ddiv_rn(__dsub_rn((double)v.w, mean), norm);
        *reinterpret_cast<float4*>(out + i0) = r;
    } else {
        for (uint64_t i = i0; i < n; ++i) out[i] = (float)__ddiv_rn(__dsub_rn((double)x[i], mean), norm);
    }
}

__global__ __launch_bounds__(256) void norm_apply_kernel(const float* __restrict__ x, uint64_t n,
                                                         const double* __restrict__ stats, float* __restrict__ out,
                                                         uint64_t x_stride, uint64_t out_stride)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double mean = stats[2 * blockIdx.y], var = stats[2 * blockIdx.y + 1];
    const double norm = sqrt(var);
    out[(uint64_t)blockIdx.y * out_stride + i] =
        (float)__ddiv_rn(__dsub_rn((double)x[(uint64_t)blockIdx.y * x_stride + i], mean), norm);
}

// d_partials must hold batch * nblocks + 2 * batch doubles.
hipError_t launch_normalise(const float* x, uint64_t n, float* out, double* d_partials, uint32_t nblocks,
                            uint64_t x_stride, uint64_t out_stride, uint32_t batch, hipStream_t s)
{
    if (!n || !batch) return hipSuccess;
    double* stats = d_partials + (uint64_t)batch * nblocks;
    const bool vec_in = ((uintptr_t)x % 16) == 0 && x_stride % 4 == 0 && !std::getenv("RIPTIDE_AMD_NORM_SCALAR");
    for (int mode = 0; mode < 2; ++mode) {
        if (vec_in)
            hipLaunchKernelGGL(norm_partial4_kernel, dim3(nblocks, batch), dim3(kNormBlock), 0, s, x, n, x_stride,
                               d_partials, stats, mode);
        else
            hipLaunchKernelGGL(norm_partial_kernel, dim3(nblocks, batch), dim3(kNormBlock), 0, s, x, n, x_stride,
                               d_partials, stats, mode);
        hipLaunchKernelGGL(norm_finalize_kernel, dim3(batch), dim3(kNormBlock), 0, s, d_partials, nblocks, n,
                           stats, mode);
    }
    if (((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0 && x_stride % 4 == 0 && out_stride % 4 == 0)
        hipLaunchKernelGGL(norm_apply4_kernel, dim3((uint32_t)((n + 1023) / 1024), batch), dim3(256), 0, s, x, n,
                           stats, out, x_stride, out_stride);
    else
        hipLaunchKernelGGL(norm_apply_kernel, dim3((uint32_t)((n + 255) / 256), batch), dim3(256), 0, s, x, n, stats,
                           out, x_stride, out_stride);
    return hipGetLastError();
}

bool dered_norm_fusable(const float* x, uint64_t n, uint64_t n_lo, uint32_t factor, const float* out,
                        uint64_t x_stride, uint64_t out_stride)
{
    return factor > 1 && n_lo > 1 && n < (1ull << 30) && ((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
           x_stride % 4 == 0 && out_stride % 4 == 0 && !std::getenv("RIPTIDE_AMD_INTERP_PER_SAMPLE") &&
           !std::getenv("RIPTIDE_AMD_NORM_UNFUSED");
}

hipError_t launch_deredden_normalise(const float* x, uint64_t n, const float* rmed_lo, uint64_t n_lo,
                                     uint32_t factor, float* out, uint64_t x_stride, uint64_t lo_stride,
                                     uint64_t out_stride, uint32_t batch, hipStream_t s, double* slopes,
                                     double* partials, double* stats)
{
    if (!n || !batch) return hipSuccess;
    const uint32_t nb = (uint32_t)dered_norm_blocks(n);
    hipLaunchKernelGGL(interp_slope_kernel, dim3((uint32_t)((n_lo + 255) / 256), batch), dim3(256), 0, s, rmed_lo,
                       n_lo, factor, slopes, lo_stride);
    hipLaunchKernelGGL(deredden_slope_kernel<true>, dim3(nb, batch), dim3(256), 0, s, x, (uint32_t)n, rmed_lo,
                       (const double*)slopes, (uint32_t)n_lo, factor, out, x_stride, lo_stride, out_stride, partials);
    hipLaunchKernelGGL(norm_stats_finalize_kernel, dim3(batch), dim3(256), 0, s, (const double*)partials, nb, n, stats);
    hipLaunchKernelGGL(norm_apply4_kernel, dim3((uint32_t)((n + 1023) / 1024), batch), dim3(256), 0, s, out, n,
                       (const double*)stats, out, out_stride, out_stride);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Kernel-API helpers (kernels.hpp:19-38, :73-101)
// ---------------------------------------------------------------------------
// out[i] = (y ? x[i] + y[(i + shift) mod n] : x[(i + shift) mod n])
__global__ __launch_bounds__(256) void rollback_kernel(const float* __restrict__ x, uint64_t n, uint64_t shift,
                                                       const float* __restrict__ y, float* __restrict__ out)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t j = i + shift % n;
    if (j >= n) j -= n;
    out[i] = y ? __fadd_rn(x[i], y[j]) : x[j];
}

hipError_t launch_rollback(const float* x, uint64_t n, uint64_t shift, const float* y, float* out, hipStream_t s)
{
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(rollback_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, x, n, shift, y, out);
    return hipGetLastError();
}

// One wave: fp64 prefix over the first min(n, nsum) elements.
__global__ __launch_bounds__(64) void cps_scan_kernel(const float* __restrict__ x, uint64_t n, uint64_t nsum,
                                                      float* __restrict__ out, float* __restrict__ total)
{
    const int lane = threadIdx.x;
    const uint64_t c = (n + 63) / 64;
    const uint64_t j0 = min((uint64_t)lane * c, n), j1 = min(j0 + c, n);
    double part = 0.0;
    for (uint64_t j = j0; j < j1; ++j) part += (double)x[j];
    const double incl = wave_scan_d(part, lane);
    double acc = __shfl_up(incl, 1, 64);
    if (lane == 0) acc = 0.0;
    for (uint64_t j = j0; j < j1; ++j) {
        acc += (double)x[j];
        if (j < nsum) out[j] = (float)acc;
    }
    const float t = __shfl((float)acc, (int)((n - 1) / c), 64);
    if (lane == 0) *total = t;
}

__global__ __launch_bounds__(256) void cps_wrap_kernel(uint64_t n, uint64_t nsum, float* __restrict__ out,
                                                       const float* __restrict__ total)
{
    const uint64_t i = n + (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= nsum) return;
    const uint64_t q = i / n;
    out[i] = __fadd_rn(out[i - q * n], __fmul_rn((float)q, *total));
}

hipError_t launch_circular_prefix_sum(const float* x, uint64_t n, uint64_t nsum, float* out, hipStream_t s)
{
    if (!n || !nsum) return hipSuccess;
    float* total = out + nsum;   // caller provides one extra float
    hipLaunchKernelGGL(cps_scan_kernel, dim3(1), dim3(64), 0, s, x, n, nsum, out, total);
    if (nsum > n)
        hipLaunchKernelGGL(cps_wrap_kernel, dim3((uint32_t)((nsum - n + 255) / 256)), dim3(256), 0, s, n, nsum,
                           out, total);
    return hipGetLastError();
}

}  // namespace rt
