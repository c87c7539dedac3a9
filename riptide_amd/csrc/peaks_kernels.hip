// Peak detection on the device (riptide/peak_detection.py:37-142), the two
// data-parallel stages of find_peaks over a batch of periodograms:
//
//   segment_order_stats_kernel: for every (trial, width, frequency segment),
//     the order statistics np.percentile(..., (25, 50, 75)) interpolates
//     between (peak_detection.py:81-83): the segment's S/N values are sorted
//     in LDS (bitonic, +inf padded) and the requested ranks written out.  The
//     host finishes the percentiles with numpy's own lerp expressions, the
//     control points and np.polyfit (a few thousand points per width).
//   threshold_select_kernel: the dynamic threshold poly(log f) (np.polyval's
//     Horner loop, fp64, no contraction) and the selection mask
//     (s > thr) & (s > smin) (peak_detection.py:131-133), compacted into
//     index lists per (trial, width).  The host sorts each list (np.where
//     order) and clusters it (cluster1d), which touches only selected points.
//
// Both kernels read the periodogram in the engine's [trial][L][W] layout.
#include <hip/hip_runtime.h>

#include <mutex>

#include <cstdint>

#include "kernels.hpp"

namespace rt {

constexpr int kPeakBlock = 256;

struct SegRanks {           // ranks of the order statistics, passed by value
    uint32_t r[kMaxSegmentRanks];
};

// One block per (segment, width, trial).  The requested order statistics
// are selected, not sorted for: the segment's values (dynamic LDS, n2 =
// per_seg rounded up to a power of two) are binned by value between their
// minimum and maximum into nb = min(n2, kSelBins) bins -- (x - min) * scale
// truncated is monotone in x, so every value of a lower bin is smaller than
// every value of a higher one -- the bins' counts prefix-summed, and each
// rank found in its bin's few values (a counting select among them).  About
// five passes over the segment instead of the log2(n2)^2 / 2 compare-exchange
// stages of a bitonic sort.  The bitonic sort (+inf padded) stays as the
// fallback for segments the binning cannot split: a NaN-free segment with an
// infinite value, a single distinct value, or more than cap values in a
// selected bin (a far outlier crowding the rest into few bins).
constexpr int kSelBins = 4096;
constexpr int kSelLists = kMaxSegmentRanks;

template <int BLOCK>
__device__ void bitonic_ascending(float* key, uint32_t n2)
{
    for (uint32_t k = 2; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = threadIdx.x; i < n2; i += BLOCK) {
                const uint32_t ixj = i ^ j;
                if (ixj > i) {
                    const float a = key[i], b = key[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        key[i] = b;
                        key[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
}

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void segment_order_stats_kernel(
    const float* __restrict__ snrs, uint64_t snr_stride, uint32_t W, uint32_t per_seg, uint32_t n2,
    SegRanks ranks, uint32_t nranks, float* __restrict__ out)
{
    constexpr int kWaves = BLOCK / 64;
    extern __shared__ __attribute__((aligned(16))) float key[];        // n2 values, then nb bins
    __shared__ float wmin[kWaves], wmax[kWaves];
    __shared__ uint32_t wsum[kWaves];
    __shared__ uint32_t tbin[kSelLists], tbase[kSelLists], lid[kSelLists], lcnt[kSelLists], win[kSelLists];
    const uint32_t seg = blockIdx.x, iw = blockIdx.y, trial = blockIdx.z;
    const uint32_t nseg = gridDim.x;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float* s = snrs + (uint64_t)trial * snr_stride + (uint64_t)seg * per_seg * W + iw;
    float* o = out + (((uint64_t)trial * W + iw) * nseg + seg) * nranks;
    uint32_t* hist = reinterpret_cast<uint32_t*>(key + n2);
    const uint32_t nb = n2 < (uint32_t)kSelBins ? n2 : (uint32_t)kSelBins;
    int nan_seen = 0;
    float mn = INFINITY, mx = -INFINITY;
    for (uint32_t i = tid; i < n2; i += BLOCK) {
        float v = INFINITY;
        if (i < per_seg) {
            v = s[(uint64_t)i * W];
            nan_seen |= v != v;
            mn = fminf(mn, v);
            mx = fmaxf(mx, v);
        }
        key[i] = v;
    }
    for (uint32_t i = tid; i < nb; i += BLOCK) hist[i] = 0u;
    for (int d = 32; d >= 1; d >>= 1) {
        mn = fminf(mn, __shfl_xor(mn, d));
        mx = fmaxf(mx, __shfl_xor(mx, d));
    }
    if (lane == 0) {
        wmin[wave] = mn;
        wmax[wave] = mx;
    }
    const int has_nan = __syncthreads_or(nan_seen);
    if (has_nan) {
        if (tid < nranks) o[tid] = NAN;
        return;
    }
    mn = wmin[0];
    mx = wmax[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) {
        mn = fminf(mn, wmin[w]);
        mx = fmaxf(mx, wmax[w]);
    }
    const float scale = (float)nb / (mx - mn);
    // block-uniform: the binning splits the segment (finite, distinct values)
    bool binned = per_seg > 64 && mn > -INFINITY && mx < INFINITY && mx > mn && scale > 0.f && scale < 3.0e38f;
    if (binned) {
        for (uint32_t i = tid; i < per_seg; i += BLOCK) {
            const uint32_t b = min((uint32_t)((key[i] - mn) * scale), nb - 1u);
            atomicAdd(&hist[b], 1u);
        }
        __syncthreads();
        // exclusive prefix sum of the bins: a thread's run of consecutive
        // bins, then the runs' totals scanned across the block
        const uint32_t per = (nb + BLOCK - 1) / BLOCK;
        const uint32_t b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
        uint32_t run = 0;
        for (uint32_t b = b0; b < b1; ++b) run += hist[b];
        uint32_t incl = run;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(incl, d);
            if ((int)lane >= d) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        if (tid < kSelLists) {
            lcnt[tid] = 0u;
            win[tid] = 0xFFFFFFFFu;
            tbin[tid] = 0xFFFFFFFFu;
        }
        __syncthreads();
        uint32_t base = incl - run;
        for (int w = 0; w < (int)wave; ++w) base += wsum[w];
        // the bin of every rank: cum[b] <= r < cum[b] + count[b]
        for (uint32_t b = b0; b < b1; ++b) {
            const uint32_t c = hist[b];
            for (uint32_t q = 0; q < nranks; ++q) {
                const uint32_t r = ranks.r[q];
                if (r >= base && r < base + c) {
                    tbin[q] = b;
                    tbase[q] = base;
                }
            }
            base += c;
        }
        __syncthreads();
        int unset = 0;      // a rank past the segment (the bitonic path's +inf padding)
        for (uint32_t q = 0; q < nranks; ++q) unset |= tbin[q] == 0xFFFFFFFFu;
        if (tid == 0) {
            for (uint32_t q = 0; q < nranks; ++q) {
                uint32_t l = q;
                for (uint32_t e = 0; e < q; ++e)
                    if (tbin[e] == tbin[q]) {
                        l = lid[e];
                        break;
                    }
                lid[q] = l;
            }
        }
        __syncthreads();
        // the selected bins' values, one list per distinct bin, in the bin area
        const uint32_t cap = nb / (uint32_t)kSelLists;
        for (uint32_t i = tid; i < per_seg; i += BLOCK) {
            const float v = key[i];
            const uint32_t b = min((uint32_t)((v - mn) * scale), nb - 1u);
            for (uint32_t q = 0; q < nranks; ++q) {
                if (lid[q] == q && b == tbin[q]) {
                    const uint32_t pos = atomicAdd(&lcnt[q], 1u);
                    if (pos < cap) reinterpret_cast<float*>(hist)[q * cap + pos] = v;
                }
            }
        }
        __syncthreads();
        int over = unset;
        for (uint32_t q = 0; q < nranks && !unset; ++q) over |= lcnt[lid[q]] > cap;
        binned = !over;
        if (binned) {
            // rank r - cum[bin] within its bin's list: the value with that
            // many smaller ones (ties: the lowest list position)
            const float* lists = reinterpret_cast<const float*>(hist);
            for (uint32_t q = 0; q < nranks; ++q) {
                const uint32_t l = lid[q], m = lcnt[l], k = ranks.r[q] - tbase[q];
                const float* L = lists + l * cap;
                for (uint32_t t = tid; t < m; t += BLOCK) {
                    const float e = L[t];
                    uint32_t lt = 0, eq = 0;
                    for (uint32_t j = 0; j < m; ++j) {
                        lt += L[j] < e;
                        eq += L[j] == e;
                    }
                    if (lt <= k && k < lt + eq) atomicMin(&win[q], t);
                }
            }
            __syncthreads();
            if (tid < nranks) o[tid] = lists[lid[tid] * cap + win[tid]];
            return;
        }
    }
    // fallback: bitonic sort of the padded segment, ascending
    __syncthreads();
    bitonic_ascending<BLOCK>(key, n2);
    if (tid < nranks) o[tid] = key[ranks.r[tid]];
}

__global__ __launch_bounds__(kPeakBlock) void threshold_select_kernel(
    const float* __restrict__ snrs, uint64_t snr_stride, uint32_t L, uint32_t W, const double* __restrict__ logf,
    const double* __restrict__ coeffs, uint32_t ncoef, double smin, uint32_t* __restrict__ counts,
    uint32_t* __restrict__ idx, uint32_t cap)
{
    const uint32_t i = blockIdx.x * kPeakBlock + threadIdx.x;
    const uint32_t iw = blockIdx.y, trial = blockIdx.z;
    if (i >= L) return;
    const double s = (double)snrs[(uint64_t)trial * snr_stride + (uint64_t)i * W + iw];
    const double* c = coeffs + ((uint64_t)trial * W + iw) * ncoef;
    const double x = logf[i];
    double y = 0.0;                                  // np.polyval: y = y * x + pv
    for (uint32_t k = 0; k < ncoef; ++k) y = __dadd_rn(__dmul_rn(y, x), c[k]);
    if (s > y && s > smin) {
        const uint32_t list = trial * W + iw;
        const uint32_t pos = atomicAdd(&counts[list], 1u);
        if (pos < cap) idx[(uint64_t)list * cap + pos] = i;
    }
}

hipError_t launch_segment_order_stats(const float* snrs, uint64_t snr_stride, uint32_t batch, uint32_t W,
                                      uint32_t nseg, uint32_t per_seg, const uint32_t* ranks, uint32_t nranks,
                                      float* out, hipStream_t s)
{
    if (!batch || !W || !nseg) return hipSuccess;
    if (per_seg > (uint32_t)kMaxSegmentPoints || nranks > (uint32_t)kMaxSegmentRanks) return hipErrorInvalidValue;
    SegRanks rk{};
    for (uint32_t i = 0; i < nranks; ++i) rk.r[i] = ranks[i];
    uint32_t n2 = 1;
    while (n2 < per_seg) n2 <<= 1;
    const size_t lds = ((size_t)n2 + (n2 < (uint32_t)kSelBins ? n2 : (uint32_t)kSelBins)) * sizeof(float);
    if (n2 <= 4096) {
        hipLaunchKernelGGL(segment_order_stats_kernel<kPeakBlock>, dim3(nseg, W, batch), dim3(kPeakBlock), lds, s,
                           snrs, snr_stride, W, per_seg, n2, rk, nranks, out);
    } else {
        // > 64 KiB of dynamic LDS: opt in once per device (the attribute is
        // per device; a mutex so concurrent host threads do not race)
        static std::mutex mu;
        static uint64_t done = 0;   // bit d: device d opted in
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        {
            std::lock_guard<std::mutex> lk(mu);
            if (dev >= 64 || !(done >> dev & 1)) {
                e = hipFuncSetAttribute(reinterpret_cast<const void*>(segment_order_stats_kernel<1024>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize,
                                        (int)((kMaxSegmentPoints + kSelBins) * sizeof(float)));
                if (e != hipSuccess) return e;
                if (dev < 64) done |= 1ull << dev;
            }
        }
        hipLaunchKernelGGL(segment_order_stats_kernel<1024>, dim3(nseg, W, batch), dim3(1024), lds, s, snrs,
                           snr_stride, W, per_seg, n2, rk, nranks, out);
    }
    return hipGetLastError();
}

hipError_t launch_threshold_select(const float* snrs, uint64_t snr_stride, uint32_t batch, uint32_t L, uint32_t W,
                                   const double* logf, const double* coeffs, uint32_t ncoef, double smin,
                                   uint32_t* counts, uint32_t* idx, uint32_t cap, hipStream_t s)
{
    if (!batch || !W || !L) return hipSuccess;
    hipLaunchKernelGGL(threshold_select_kernel, dim3((L + kPeakBlock - 1) / kPeakBlock, W, batch), dim3(kPeakBlock), 0,
                       s, snrs, snr_stride, L, W, logf, coeffs, ncoef, smin, counts, idx, cap);
    return hipGetLastError();
}

// 8-bit SIGPROC samples -> float32 (riptide/time_series.py:352-357: numpy
// astype(np.float32) of int8 / uint8 values, exact).  4 samples per thread.
__global__ __launch_bounds__(256) void convert_samples_kernel(const uint8_t* __restrict__ raw, uint64_t n,
                                                              int is_signed, float* __restrict__ out)
{
    const uint64_t i = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (i + 3 < n) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(raw + i);
        float4 v;
        if (is_signed) {
            v = make_float4((float)(int8_t)(w & 0xFF), (float)(int8_t)((w >> 8) & 0xFF),
                            (float)(int8_t)((w >> 16) & 0xFF), (float)(int8_t)(w >> 24));
        } else {
            v = make_float4((float)(w & 0xFF), (float)((w >> 8) & 0xFF), (float)((w >> 16) & 0xFF), (float)(w >> 24));
        }
        out[i] = v.x;
        out[i + 1] = v.y;
        out[i + 2] = v.z;
        out[i + 3] = v.w;
    } else {
        for (uint64_t k = i; k < n; ++k) out[k] = is_signed ? (float)(int8_t)raw[k] : (float)raw[k];
    }
}

hipError_t launch_convert_samples(const void* raw, uint64_t n, int is_signed, float* out, hipStream_t s)
{
    if (!n) return hipSuccess;
    const uint64_t blocks = (n + 1023) / 1024;
    hipLaunchKernelGGL(convert_samples_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, (const uint8_t*)raw, n,
                       is_signed, out);
    return hipGetLastError();
}

}  // namespace rt
