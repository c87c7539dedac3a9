// FFA periodogram hot path for MI355X (gfx950): downsampling ladder, LDS cone
// kernel (several FFA merge levels per HBM pass), fused boxcar S/N epilogue.
//
// Exactness: every float operation that the reference performs is performed
// here on the same operands in the same association (explicit *_rn intrinsics
// where hipcc would otherwise contract into FMA), so the FFA transform is
// bit-identical to riptide::transform (transforms.hpp:30-61) and downsample is
// bit-identical to the strict restatement of downsample.hpp:44-82.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"

namespace rt {

template <int N> struct IntC { static constexpr int value = N; };

// ---------------------------------------------------------------------------
// Downsampling ladder (downsample.hpp:44-82; periodogram.hpp:162-168)
// ---------------------------------------------------------------------------
// wmin * w[0] + w[1] + ... + w[cnt - 1], added one by one in that order
// (downsample.hpp:44-82).  The reads go out eight at a time ahead of their
// additions (a plain loop waited for every LDS read in turn: at f ~ 100 the
// ladder was bound by that latency); the elements past cnt - 1 of the last
// group add -0.0, an exact no-op (x + (-0.0) == x).
__device__ __forceinline__ float window_sum(const float* w, float wmin, uint32_t cnt)
{
    float acc = __fmul_rn(wmin, w[0]);
    uint32_t i = 1;
    for (; i + 8 <= cnt; i += 8) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = w[i + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = __fadd_rn(acc, v[j]);
    }
    if (i < cnt) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = i + j < cnt ? w[i + j] : -0.0f;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc = __fadd_rn(acc, v[j]);
    }
    return acc;
}

// One block = up to 256 consecutive outputs of one rung of one trial (fewer for
// large f, so the block's input span fits the LDS stage).  The span is loaded
// with coalesced loads, then each thread sums its window from LDS in the
// reference's order.  Rungs are flattened along blockIdx.x through a per-rung
// first-block table; blockIdx.y = trial.
__global__ __launch_bounds__(256) void downsample_ladder_kernel(
    const float* __restrict__ x, uint64_t n_in, uint64_t x_stride,
    const DsRung* __restrict__ rungs, uint32_t num_rungs,
    float* __restrict__ out, uint64_t out_stride)
{
    __shared__ float span[kDsSpanFloats];
    uint32_t lo = 0, hi = num_rungs - 1;
    const uint32_t b = blockIdx.x;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (rungs[mid].first_block <= b) lo = mid; else hi = mid - 1;
    }
    const DsRung r = rungs[lo];
    const uint64_t k0 = (uint64_t)(b - r.first_block) * r.per_block;
    const uint64_t k1 = min(k0 + r.per_block, r.n);
    x += (uint64_t)blockIdx.y * x_stride;
    out += (uint64_t)blockIdx.y * out_stride + r.out_off;
    const uint64_t k = k0 + threadIdx.x;
    if (r.identity) {           // f == 1: the rung searches the data at its own resolution
        if (k < k1) out[k] = x[k];
        return;
    }
    const double f = r.f;
    const double last = (double)n_in - 1.0;
    // input span of the block: [imin(k0), imax(k1 - 1)]
    const uint64_t s0 = (uint64_t)floor(__dmul_rn((double)k0, f));
    double e1 = floor(__dadd_rn(__dmul_rn((double)(k1 - 1), f), f));
    if (e1 > last) e1 = last;
    const uint64_t s1 = (uint64_t)e1;
    const float* src = x + s0;
    if (r.staged) {
        const uint32_t len = (uint32_t)(s1 - s0 + 1);
        for (uint32_t i = threadIdx.x; i < len; i += 256) span[i] = x[s0 + i];
        __syncthreads();
        src = span;
    }
    if (k >= k1) return;
    const double start = __dmul_rn((double)k, f);
    const double end = __dadd_rn(start, f);
    const uint64_t imin = (uint64_t)floor(start);
    double dmax = floor(end);
    if (dmax > last) dmax = last;
    const uint64_t imax = (uint64_t)dmax;
    const float wmin = (float)__dsub_rn((double)(imin + 1), start);
    const float wmax = (float)__dsub_rn(end, (double)imax);
    const float* w = src + (imin - s0);
    const uint32_t cnt = (uint32_t)(imax - imin);
    out[k] = __fadd_rn(window_sum(w, wmin, cnt), __fmul_rn(wmax, w[cnt]));
}

// Fused ladder: one block per input span (and trial pair) computes the
// outputs of EVERY rung whose window starts in the span, so the series is
// read from HBM once instead of once per rung (57 rungs at cfg2).  The span
// plus a margin (the plan's: ceil(f) + 2 for its largest fused rung, rounded
// up to 64, <= kDsFusedMargin) is staged in LDS, kDsPairSpan samples in
// all; each output is the same sequential window sum as the per-rung kernel.

// first output k of a rung whose window start floor(k f) is >= s
__device__ __forceinline__ uint64_t ds_first_output(double f, uint64_t s)
{
    uint64_t k = (uint64_t)ceil((double)s / f);
    while (k > 0 && (uint64_t)floor(__dmul_rn((double)(k - 1), f)) >= s) --k;
    while ((uint64_t)floor(__dmul_rn((double)k, f)) < s) ++k;
    return k;
}

// The first output of a rung whose window start floor(k f) is >= s, clipped
// to the rung's length: k_lo of a block's span [s0, s_end) at s = s0, k_hi
// at s = s_end (s_end = n_in for the last block: every remaining output).
__device__ __forceinline__ uint32_t ds_rung_bound(const DsRung& r, uint64_t s, uint64_t n_in)
{
    if (r.identity) return (uint32_t)min(s, r.n);
    return (uint32_t)(s >= n_in ? r.n : min(ds_first_output(r.f, s), r.n));
}

// Every rung's window sums over one staged span.  Indices are 32-bit (the
// planner keeps every series below 2^29 samples), the start / end / floor
// arithmetic is the reference's in float64 (downsample.hpp:53-75: (imin + 1)
// - start is (floor(start) + 1.0) - start exactly, end - imax is end -
// min(floor(end), N - 1)), and each rung's output range in the span is
// computed once per block by one lane per rung instead of by every thread.
//
// The span is staged as overlapping pairs: pair i holds samples s0 + i and
// s0 + i + 1, 8-byte aligned, so a window's consecutive samples from ANY
// start come in ds_read_b64 reads at immediate offsets (2 LDS cycles per 64
// lanes x 2 samples, 64 banks) -- with single samples (ds_read_b32 or the
// compiler's ds_read2_b32, 32 banks) the reads took twice the LDS cycles
// and, the window starts of adjacent outputs lying f apart, conflicted
// alike (tools/ladder_conflicts.py).  Volatile reads: the
// compiler would fuse two of them into ds_read2_b64 (8 cycles).
typedef float ds_pair __attribute__((ext_vector_type(2), aligned(8)));
// A workgroup runs NT = 2 trials of one span: each output's float64 bounds
// (most of the VALU work at f < 12) are computed once for both trials'
// windows.  1024 threads: 2 x 32 KiB of pairs allow two workgroups per CU,
// sixteen waves each (the CU's 32; 512 threads left it half full).
// RT_DS_THREADS / RT_DS_TRIALS: geometry A/B builds.
#ifndef RT_DS_THREADS
#define RT_DS_THREADS 1024
#endif
#ifndef RT_DS_TRIALS
#define RT_DS_TRIALS 2
#endif
constexpr uint32_t kDsFusedThreads = RT_DS_THREADS;
constexpr uint32_t kDsFusedTrials = RT_DS_TRIALS;
static_assert((kDsFusedThreads & (kDsFusedThreads - 1)) == 0 && kDsFusedThreads >= 64, "whole waves, power of two");
static_assert(kDsFusedTrials == 1 || kDsFusedTrials == 2, "trials per workgroup");
// samples staged per trial (pairs): two trials' pairs and the rung table fill
// just under half the CU's 160 KiB, so two workgroups stay resident
// (RT_DS_PAIRS: A/B builds)
#ifndef RT_DS_PAIRS
#define RT_DS_PAIRS 4864
#endif
constexpr uint32_t kDsPairSpan = RT_DS_PAIRS;
static_assert(kDsPairSpan >= 4 * kDsFusedMargin && kDsPairSpan % 64 == 0, "span: whole waves, margin <= a quarter");
static_assert(2 * (kDsFusedTrials * kDsPairSpan * 8 + 8 * kDsMaxRungs) <= 160 * 1024, "two workgroups per CU");
typedef const volatile __attribute__((address_space(3))) ds_pair* ds_pptr;

__global__ __launch_bounds__(kDsFusedThreads) void downsample_fused_kernel(
    const float* __restrict__ x, uint64_t n_in, uint64_t x_stride,
    const DsRung* __restrict__ rungs, uint32_t num_rungs,
    float* __restrict__ out, uint64_t out_stride, uint32_t batch, uint32_t span)
{
    constexpr uint32_t NT = kDsFusedTrials;
    __shared__ ds_pair pairs[NT * kDsPairSpan];
    __shared__ uint32_t kr[2 * kDsMaxRungs];
    const uint64_t s0 = (uint64_t)blockIdx.x * span;
    const uint64_t s_end = min(s0 + (uint64_t)span, n_in);             // window starts owned by this block
    const uint64_t l_end = min(s0 + (uint64_t)kDsPairSpan, n_in);    // staged input
    // trials t0 .. t0 + nt - 1 (a last workgroup of an odd batch stages its
    // one trial twice and stores the same values twice)
    const uint32_t t0 = blockIdx.y * NT;
    const uint32_t nt = min(NT, batch - t0);
    // Only a block staged up to the end of the series can hold windows that
    // min(floor(end), N - 1) clips (otherwise end < s_end + margin <= l_end
    // < N); every other block stages all kDsPairSpan pairs, sample
    // s0 + kDsPairSpan included.  Its loads go out together, ahead of the
    // rung ranges (one lane per rung bound, k_lo and k_hi in two waves:
    // float64 divisions and loops), so the two latencies overlap.
    const bool tail = l_end >= n_in;
    static_assert(2 * kDsMaxRungs <= kDsFusedThreads, "one lane per rung bound");
    const uint32_t r_hi = threadIdx.x / kDsMaxRungs, r_i = threadIdx.x % kDsMaxRungs;
    const bool has_rung = r_hi < 2 && r_i < num_rungs;
    DsRung rr{};
    if (has_rung) rr = rungs[r_i];
    constexpr uint32_t SU = (kDsPairSpan + kDsFusedThreads - 1) / kDsFusedThreads;
    float sa[NT][SU], sb[NT][SU];
    if (!tail) {
#pragma unroll
        for (uint32_t q = 0; q < NT; ++q) {
            const float* xs = x + (uint64_t)(t0 + min(q, nt - 1)) * x_stride + s0 + threadIdx.x;
#pragma unroll
            for (uint32_t u = 0; u < SU; ++u) {
                if (kDsPairSpan % kDsFusedThreads == 0 || threadIdx.x + u * kDsFusedThreads < kDsPairSpan) {
                    sa[q][u] = xs[u * kDsFusedThreads];
                    sb[q][u] = xs[u * kDsFusedThreads + 1];
                }
            }
        }
    }
    if (has_rung) kr[2 * r_i + r_hi] = ds_rung_bound(rr, r_hi ? s_end : s0, n_in);
    if (!tail) {
#pragma unroll
        for (uint32_t q = 0; q < NT; ++q)
#pragma unroll
            for (uint32_t u = 0; u < SU; ++u)
                if (kDsPairSpan % kDsFusedThreads == 0 || threadIdx.x + u * kDsFusedThreads < kDsPairSpan)
                    pairs[q * kDsPairSpan + threadIdx.x + u * kDsFusedThreads] = ds_pair{sa[q][u], sb[q][u]};
    } else {
        for (uint32_t q = 0; q < NT; ++q) {
            const float* xq = x + (uint64_t)(t0 + min(q, nt - 1)) * x_stride;
            for (uint64_t i = s0 + threadIdx.x; i < l_end; i += kDsFusedThreads)
                pairs[q * kDsPairSpan + (i - s0)] = ds_pair{xq[i], i + 1 < n_in ? xq[i + 1] : 0.0f};
        }
    }
    __syncthreads();
    const double last = (double)n_in - 1.0;
    const uint32_t b0 = (uint32_t)s0;
    // lp[s] (+ q kDsPairSpan for trial q): the pair of sample s (pointer
    // arithmetic, so the compiler folds a window's pair offsets, and the
    // second trial's 32 KiB, into the reads' immediate offsets)
    const ds_pptr lp = (ds_pptr)pairs - b0;
    // A non-clipping block has cnt = floor(f) or floor(f) + 1 (floor and
    // rounding are monotone and start + floor(f) is exact), so with F =
    // floor(f) its samples w[1 .. F - 1] all add, w[F] adds when cnt = F + 1
    // (else -0.0, an exact no-op) and w[cnt] is a select of w[F] and w[F + 1]
    // (inside the staged margin: the plan's >= ceil(f) + 2); the clipping
    // block takes the general sum.  The non-clipping bounds come from fract
    // and truncation: (floor(start) + 1) - start is 1 - frac(start) rounded
    // once, as 1.0 - fract(start) is (fract is exact for start >= 0);
    // end - floor(end) is fract(end) exactly (Sterbenz); the uint32
    // truncations are the floors.
    //
    // F < 12 (most of the ladder's outputs: f ~ 1.5-10 at cfg2): one template
    // instance per F, every read at an immediate offset.
    // trial q's rung output (a missing second trial: the first's, whose
    // values it recomputes from the same staged samples -- no branch)
    float* oq[NT];
    // vo: the output's byte offset (32 bits: a rung holds < 2^29 outputs),
    // one offset for both trials' stores (global_store with an SGPR base)
    auto put = [&](uint32_t q, uint32_t vo, float v) { *(float*)((char*)oq[q] + vo) = v; };
    // kd: the output index k as float64 (exact), the window start's operand
    auto output_small = [&](auto ff, double f, double kd, uint32_t vo) {
        constexpr int F = decltype(ff)::value;
        const double start = __dmul_rn(kd, f);
        const double end = __dadd_rn(start, f);
        const uint32_t imin = (uint32_t)start, imax = (uint32_t)end;
        const float wmin = (float)__dsub_rn(1.0, __builtin_amdgcn_fract(start));
        const float wmax = (float)__builtin_amdgcn_fract(end);
        const bool full = imax - imin > (uint32_t)F;
        const ds_pptr w = lp + imin;
        // every read of both trials first (volatile reads issue in program
        // order), then the two independent sums
        float v[NT][F + 3];
#pragma unroll
        for (uint32_t q = 0; q < NT; ++q)
#pragma unroll
            for (int j = 0; j <= F + 1; j += 2) {
                const ds_pair p = w[q * kDsPairSpan + j];
                v[q][j] = p.x;
                v[q][j + 1] = p.y;
            }
#pragma unroll
        for (uint32_t q = 0; q < NT; ++q) {
            float acc = __fmul_rn(wmin, v[q][0]);
#pragma unroll
            for (int j = 1; j < F; ++j) acc = __fadd_rn(acc, v[q][j]);
            acc = __fadd_rn(acc, full ? v[q][F] : -0.0f);
            put(q, vo, __fadd_rn(acc, __fmul_rn(wmax, full ? v[q][F + 1] : v[q][F])));
        }
    };
    // F >= 12: the same sum with uniform trip counts (F is the rung's), four
    // pair reads ahead of their eight additions
    auto output_large = [&](double f, uint32_t F, double kd, uint32_t vo) {
        const double start = __dmul_rn(kd, f);
        const double end = __dadd_rn(start, f);
        const uint32_t imin = (uint32_t)start, imax = (uint32_t)end;
        const float wmin = (float)__dsub_rn(1.0, __builtin_amdgcn_fract(start));
        const float wmax = (float)__builtin_amdgcn_fract(end);
        const bool full = imax - imin > F;
        const ds_pptr w = lp + imin;
        // both trials' sums side by side (independent chains)
        float acc[NT];
#pragma unroll
        for (uint32_t q = 0; q < NT; ++q) {
            const ds_pair p = w[q * kDsPairSpan];
            acc[q] = __fadd_rn(__fmul_rn(wmin, p.x), p.y);
        }
        uint32_t e = 2;
        for (; e + 8 <= F; e += 8) {
            ds_pair g[NT][4];
#pragma unroll
            for (uint32_t q = 0; q < NT; ++q)
#pragma unroll
                for (int i = 0; i < 4; ++i) g[q][i] = w[q * kDsPairSpan + e + 2 * i];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (uint32_t q = 0; q < NT; ++q) acc[q] = __fadd_rn(__fadd_rn(acc[q], g[q][i].x), g[q][i].y);
        }
        for (; e + 2 <= F; e += 2)
#pragma unroll
            for (uint32_t q = 0; q < NT; ++q) {
                const ds_pair p = w[q * kDsPairSpan + e];
                acc[q] = __fadd_rn(__fadd_rn(acc[q], p.x), p.y);
            }
        if (e < F)
#pragma unroll
            for (uint32_t q = 0; q < NT; ++q) acc[q] = __fadd_rn(acc[q], w[q * kDsPairSpan + e].x);
#pragma unroll
        for (uint32_t q = 0; q < NT; ++q) {
            const ds_pair p = w[q * kDsPairSpan + F];
            const float a = __fadd_rn(acc[q], full ? p.x : -0.0f);
            put(q, vo, __fadd_rn(a, __fmul_rn(wmax, full ? p.y : p.x)));
        }
    };
    // the clipping block: the reference's bounds with min(floor(end), N - 1)
    // and the window sum sample by sample
    auto output_tail = [&](double f, double kd, uint32_t vo) {
        const double start = __dmul_rn(kd, f);
        const double end = __dadd_rn(start, f);
        const double fs = floor(start);
        double dmax = floor(end);
        if (dmax > last) dmax = last;
        const uint32_t imin = (uint32_t)fs, imax = (uint32_t)dmax;
        const float wmin = (float)__dsub_rn(__dadd_rn(fs, 1.0), start);
        const float wmax = (float)__dsub_rn(end, dmax);
        for (uint32_t q = 0; q < NT; ++q) {
            const ds_pptr w = lp + q * kDsPairSpan + imin;
            float acc = __fmul_rn(wmin, w[0].x);
            for (uint32_t j = 1; j < imax - imin; ++j) acc = __fadd_rn(acc, w[j].x);
            put(q, vo, __fadd_rn(acc, __fmul_rn(wmax, w[imax - imin].x)));
        }
    };
    // the rung table in lanes: lane l of every wave holds rung c + l's output
    // range and parameters (one LDS read and one global load per 64 rungs),
    // taken per rung with v_readlane -- a per-rung LDS read and scalar load
    // were a memory wait per rung and wave (57 rungs at cfg2)
    const uint32_t lane = threadIdx.x & 63;
    // Work balance: the rungs' outputs tile the waves in turn -- output
    // k_lo + i of a rung goes to thread (rot + i) mod T, rot advancing by
    // each rung's output count rounded up to whole waves -- so the short
    // rungs (f > 7: fewer than T outputs in a span) land on successive waves
    // instead of all on the first ones, and the workgroup's waves finish
    // together (its LDS frees for the next one only when the last does).  A
    // wave's lanes stay consecutive outputs; a wave without outputs in a
    // rung skips it on scalar compares.
    const uint32_t wbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x & ~63u));
    uint32_t rot = 0;
    for (uint32_t c = 0; c < num_rungs; c += 64) {
        const uint32_t rl = min(c + lane, num_rungs - 1);
        const int my_lo = (int)kr[2 * rl], my_hi = (int)kr[2 * rl + 1];
        const DsRung mr = rungs[rl];
        const long long my_f = __double_as_longlong(mr.f);
        const int my_f_lo = (int)(uint32_t)my_f, my_f_hi = (int)(uint32_t)((uint64_t)my_f >> 32);
        const int my_o_lo = (int)(uint32_t)mr.out_off, my_o_hi = (int)(uint32_t)(mr.out_off >> 32);
        const int my_id = (int)mr.identity;
        const uint32_t nr = min(64u, num_rungs - c);
        for (uint32_t j = 0; j < nr; ++j) {
            const uint32_t k_lo = (uint32_t)__builtin_amdgcn_readlane(my_lo, (int)j);
            const uint32_t k_hi = (uint32_t)__builtin_amdgcn_readlane(my_hi, (int)j);
            const uint32_t nk = k_hi - k_lo;
            const uint32_t wfirst = (wbase - rot) & (kDsFusedThreads - 1);
            const uint32_t i0 = (threadIdx.x - rot) & (kDsFusedThreads - 1);
            rot = (rot + ((nk + 63) & ~63u)) & (kDsFusedThreads - 1);
            if (wfirst >= nk) continue;          // rot: a multiple of 64
            const uint64_t off = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(my_o_lo, (int)j) |
                                 ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(my_o_hi, (int)j) << 32);
#pragma unroll
            for (uint32_t q = 0; q < NT; ++q) oq[q] = out + (uint64_t)(t0 + min(q, nt - 1)) * out_stride + off;
            if (__builtin_amdgcn_readlane(my_id, (int)j)) {
                for (uint32_t k = k_lo + i0; k < k_hi; k += kDsFusedThreads)
#pragma unroll
                    for (uint32_t q = 0; q < NT; ++q) put(q, 4u * k, lp[q * kDsPairSpan + k].x);
                continue;
            }
            const double f = __longlong_as_double(
                (long long)((uint64_t)(uint32_t)__builtin_amdgcn_readlane(my_f_lo, (int)j) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(my_f_hi, (int)j) << 32)));
            // this thread's outputs k = k_lo + i0, + T, ... < k_hi of the rung, as
            // (k as float64, byte offset 4 k): the loop runs on those two alone
            auto outputs = [&](auto body) {
                const double kend = (double)k_hi;
                double kd = (double)(k_lo + i0);
                for (uint32_t vo = 4u * (k_lo + i0); kd < kend; kd += (double)kDsFusedThreads, vo += 4u * kDsFusedThreads)
                    body(kd, vo);
            };
            if (tail) {
                outputs([&](double kd, uint32_t vo) { output_tail(f, kd, vo); });
                continue;
            }
            auto rung = [&](auto ff) {
                outputs([&](double kd, uint32_t vo) { output_small(ff, f, kd, vo); });
            };
            const uint32_t F = (uint32_t)f;
            switch (F) {
            case 1: rung(IntC<1>{}); break;
            case 2: rung(IntC<2>{}); break;
            case 3: rung(IntC<3>{}); break;
            case 4: rung(IntC<4>{}); break;
            case 5: rung(IntC<5>{}); break;
            case 6: rung(IntC<6>{}); break;
            case 7: rung(IntC<7>{}); break;
            case 8: rung(IntC<8>{}); break;
            case 9: rung(IntC<9>{}); break;
            case 10: rung(IntC<10>{}); break;
            case 11: rung(IntC<11>{}); break;
            default:
                // F >= 12 (F = 0 does not occur: f > 1 off the identity rung)
                if (F >= 12)
                    outputs([&](double kd, uint32_t vo) { output_large(f, F, kd, vo); });
                else
                    outputs([&](double kd, uint32_t vo) { output_tail(f, kd, vo); });
                break;
            }
        }
    }
}

hipError_t launch_downsample_fused(const float* x, uint64_t n_in, uint64_t x_stride, const DsRung* d_rungs,
                                   uint32_t num_rungs, uint32_t margin, float* out, uint64_t out_stride,
                                   uint32_t batch, hipStream_t s)
{
    if (!num_rungs || !batch || !n_in) return hipSuccess;
    if (margin < 2 || margin > kDsFusedMargin) return hipErrorInvalidValue;
    const uint32_t span = kDsPairSpan - margin;
    const uint64_t blocks = (n_in + span - 1) / span;
    hipLaunchKernelGGL(downsample_fused_kernel, dim3((uint32_t)blocks, (batch + kDsFusedTrials - 1) / kDsFusedTrials),
                       dim3(kDsFusedThreads), 0, s, x, n_in, x_stride, d_rungs, num_rungs, out, out_stride, batch,
                       span);
    return hipGetLastError();
}

hipError_t launch_downsample_ladder(const float* x, uint64_t n_in, uint64_t x_stride,
                                    const DsRung* d_rungs, uint32_t num_rungs, uint32_t total_blocks,
                                    float* out, uint64_t out_stride, uint32_t batch, hipStream_t s)
{
    if (!num_rungs || !total_blocks || !batch) return hipSuccess;
    hipLaunchKernelGGL(downsample_ladder_kernel, dim3(total_blocks, batch), dim3(256), 0, s,
                       x, n_in, x_stride, d_rungs, num_rungs, out, out_stride);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Cone kernel
// ---------------------------------------------------------------------------
// A work unit = one work item (UnitDesc) of one trial: `levels` merge levels
// of the FFA recursion for the rows of one tile (or one whole node), in LDS.
//   1. begin: the unit's view (one scalar load of its UnitDesc); the bottom
//      level is LDS-DMA'd from the transform block (a whole unit: one run of
//      16-byte chunks; a tile unit: one run per range of its dependency cone,
//      listed in the host-built blob, which is DMA'd alongside: rows per
//      level, the row-descriptor table of every level, the bottom rows' LDS
//      offsets -- build_tile_blob, plan.cpp)
//   2. merge levels, deepest first (transforms.hpp:13-27), one row per wave
//      and one phase bin per lane, two levels per LDS round trip where no
//      level holds size-1 nodes:
//          out[r][j] = H[h(r)][j] + T[t(r)][(j + shift(r)) mod p]
//      Lane i holds the descriptor of the wave's i-th row as LDS offsets;
//      the row loop takes them with v_readlane.  Bins j = lane + 64k use
//      immediate offsets, so a 64-bin slot is one ds_read per operand
//      (consecutive lanes -> consecutive banks) and one ds_write.  A step's
//      outputs are staged in registers between two barriers (in place).
//   3. a non-final pass stores its last level straight from the registers;
//      a final pass runs the fused boxcar S/N epilogue (snr.hpp:37-65) on it.
// Whole units compute their descriptors on the fly (node partition
// arithmetic, no table).

// Cache policy bits (gfx950: 1 sc0, 2 nt, 16 sc1) of the fill's LDS-DMA
// loads, of the merge passes' output stores and of the S/N stores.  A/B,
// same box, cone ms per trial (profiles/r03zg_ab_*.log): nt stores cfg2
// 7.663 -> 7.616, cfg3 1.907 -> 1.883 (the next pass reads them from HBM
// anyway); nt fills 7.86 / 1.94, slower (adjacent tiles' cones overlap and
// share their L2 lines) -- stores nt, fills default.  Only the whole-slot
// stores (64 consecutive words per wave instruction) are nt: the short-row
// stores (4-byte scattered per lane) took cfg4 from 0.776 to 1.306 ms per
// trial with nt (r03zh_ab_cfg4.log) and keep the default.
constexpr int kFillCpol = 0, kStoreCpol = 2, kSnrCpol = 0;

// LDS-only workgroup barrier: orders LDS accesses without waiting for the
// global loads or stores that are still in flight.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

template <class T>
__device__ __forceinline__ T* uni_ptr(T* p)
{
    return reinterpret_cast<T*>(uni64(reinterpret_cast<uint64_t>(p)));
}

// Wave-uniform view of one unit (scalar registers).
struct UnitView {
    int item, trial;
    int node_start, node_size, s0, s1, levels, mode, src, dst;
    int p, m, rows_eval;
    uint64_t src_off, buf_off, snr_row;
    float stdnoise;
    uint32_t blob;            // word offset of the host-built blob (kNoBlob: none)
    int nruns, entries, nb, slot_words, run_off;   // its header counts
    int fill_chunks;          // 16-byte chunks of the bottom-level fill
    int zero_row;             // LDS float offset of the unit's -0.0 row (0: none; kHdrZero)
};

typedef const __attribute__((address_space(4))) uint32_t* const_u32_ptr;

__device__ __forceinline__ UnitView unit_view(const ConeArgs& a, int item, int trial)
{
    UnitView v;
    v.item = uni(item);
    v.trial = uni(trial);
    // constant address space: scalar (SMEM) loads, counted in lgkmcnt, so
    // they never wait behind the vector-memory queue (DMA fills, stores)
    const const_u32_ptr w = (const_u32_ptr)(uintptr_t)(a.items + v.item);
    uint32_t x[sizeof(UnitDesc) / 4];
#pragma unroll
    for (int i = 0; i < (int)(sizeof(UnitDesc) / 4); ++i) x[i] = w[i];
    UnitDesc d;
    __builtin_memcpy(&d, x, sizeof d);
    v.node_start = uni((int)d.node_start);
    v.node_size = uni((int)d.node_size);
    v.s0 = uni((int)d.s0);
    v.s1 = uni((int)d.s1);
    v.levels = uni((int)d.levels);
    v.mode = uni((int)d.mode);
    v.src = uni((int)d.src);
    v.dst = uni((int)d.dst);
    v.p = uni((int)d.p);
    v.m = uni((int)d.m);
    v.rows_eval = uni((int)d.rows_eval);
    v.src_off = uni64(d.src_off);
    v.buf_off = uni64(d.buf_off);
    v.snr_row = uni64(d.snr_row);
    v.stdnoise = __int_as_float(uni(__float_as_int(d.stdnoise)));
    v.blob = (uint32_t)uni((int)d.pad);
    v.nruns = uni((int)d.nruns);
    v.entries = uni((int)d.entries);
    v.nb = uni((int)d.nb);
    v.slot_words = uni((int)d.slot_words);
    v.run_off = uni((int)d.run_off);
    v.fill_chunks = uni((int)d.fill_chunks);
    v.zero_row = uni((int)d.zero_row);
    return v;
}

// Per-unit context (wave-uniform) and its LDS metadata: for tile units the
// blob (kBlobHeader words of header, the DMA runs, the descriptor table, the
// bottom-row offsets) DMA'd into `aux`.
constexpr int kAuxWords = kBlobHeader + kDescEntries + kMaxRows + kSlotWords;
static_assert(kAuxWords == kAuxMetaWords, "metadata area");
struct UnitCtx {
    UnitView U;
    bool tile;                // a tile unit (else: a whole node)
    bool table;               // the host-built blob is in aux (every tile unit, most whole units)
    int al;                   // whole units: 16-byte phase (floats) of the block
    bool slots;               // the blob holds row-slot tables (merge_step_slots)
    int nruns, entries, nb;   // blob header counts
    const uint32_t* aux;      // the blob's LDS part in LDS
    const uint32_t* aux0;     // the workgroup's metadata area (roll table at kLut4Off)
    uint4 sv;                 // tile units: this wave's DMA segments (lane i: segment wave + 8i), the
    int mine;                 // same for every trial; `mine` of them
};

__device__ __forceinline__ int rows_at(const UnitCtx& C, int l)
{
    return C.table ? uni((int)C.aux[kHdrRows + l]) : C.U.node_size;
}
__device__ __forceinline__ int desc_offset(const UnitCtx& C, int l) { return uni((int)C.aux[kHdrDesc + l]); }
__device__ __forceinline__ const uint32_t* desc_table(const UnitCtx& C) { return C.aux + kBlobHeader; }
// the row-slot table of the merge step whose output level is lo: its slot
// count, then one word per slot
__device__ __forceinline__ const uint32_t* slot_table(const UnitCtx& C, int lo)
{
    return C.aux + uni((int)C.aux[kHdrSlotOff + lo]);
}
__device__ __forceinline__ const int* bottom_offsets(const UnitCtx& C)
{
    return reinterpret_cast<const int*>(desc_table(C) + C.entries);
}

// Raw buffer resource over `bytes` bytes at p (gfx9 dword3: 32-bit data
// format); out-of-range buffer loads return 0 and stores are dropped.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(uni_ptr(const_cast<void*>(p)), (short)0, uni((int)bytes), 0x00020000);
}

// LDS DMA of `nch` 16-byte chunks from byte offset `goff` of resource rs
// into lds[0 .. 4 nch) (floats), by the waves `wave0 .. W - 1` of the
// workgroup in steps of `wstep` waves: a wave instruction moves 64
// consecutive chunks (destination M0 + 16 lane); lanes past the end are
// exec-masked off and write nothing.
__device__ __forceinline__ void dma_run(__amdgpu_buffer_rsrc_t rs, uint32_t goff, int nch, float* lds, int wave,
                                        int wstep, int lane)
{
    for (int c0 = wave * 64; c0 < nch; c0 += wstep * 64) {
        const int c = c0 + lane;
        if (c < nch)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + 4 * c0), 16,
                                                     (int)(goff + 16u * (uint32_t)c), 0, 0, kFillCpol);
    }
}

// Source block (the transform's rows in the leaf buffer or ping / pong) of a
// unit's bottom level for `trial`, as a buffer resource over the block.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t unit_src(const ConeArgs& a, const UnitView& U, int trial)
{
    const float* src;
    if (U.src == kSelLeaves) src = a.leaves + (uint64_t)trial * a.leaves_stride + U.src_off;
    else src = (U.src == kSelPing ? a.ping : a.pong) + (uint64_t)trial * a.buf_stride + U.buf_off;
    // transform blocks start 16-byte aligned and are padded to 4 floats
    return buffer_rsrc(src, (((uint32_t)U.m * (uint32_t)U.p + 3u) & ~3u) * 4u);
}

// Issues the LDS DMA of a unit's bottom level for `trial` into `buf` (a whole
// unit: one run of 16-byte chunks; a tile unit: the host-built DMA segments,
// one vector load, lane i of wave w holding segment w + 8i) and, with
// `blob_too`, the blob's LDS part (header, descriptors, bottom-row offsets,
// slot tables) into the metadata area.  Nothing is waited for.
template <int SMAX>
__device__ __forceinline__ void unit_fill(const ConeArgs& a, const UnitCtx& C, int trial, float* buf, int tid,
                                          bool blob_too)
{
    const int lane = tid & 63, wave = tid >> 6;
    const UnitView& U = C.U;
    const int p = U.p;
    const __amdgpu_buffer_rsrc_t rs = unit_src(a, U, trial);
    if (!C.table) {
        const int nch = (U.node_size * p + C.al + 3) >> 2;
        dma_run(rs, ((uint32_t)U.node_start * (uint32_t)p - (uint32_t)C.al) * 4u, nch, buf, wave, kConeWaves, lane);
        return;
    }
    const int words = U.run_off;   // the LDS part: header .. slot tables
    // the wave's DMA segments (unit_segments, loaded once per workgroup)
    const uint4 sv = C.sv;
    const int mine = C.mine;
    if (blob_too && wave == kConeWaves - 1) {
        const __amdgpu_buffer_rsrc_t rb = buffer_rsrc(a.blob + U.blob, (uint32_t)words * 4u);
        dma_run(rb, 0u, words >> 2, (float*)const_cast<uint32_t*>(C.aux), 0, 1, lane);
    }
    for (int i = 0; i < mine; ++i) {
        const int c0 = __builtin_amdgcn_readlane((int)sv.x, i);
        const int n = __builtin_amdgcn_readlane((int)sv.y, i);
        const uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)sv.z, i);
        if (lane < n && 4 * (c0 + n) <= kLdsBufFloats && !(a.flags & kConeDiagNoFill))
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(buf + 4 * c0), 16,
                                                     (int)((g + (uint32_t)lane) * 16u), 0, 0, kFillCpol);
    }
}

// The wave's DMA segments of a tile unit: wave w issues segments w, w + 8,
// ...; its lane i holds segment w + 8i (one coalesced vector load; wave-major
// table, build_tile_blob: the wave's segments are consecutive).  Trial-
// independent: kept in registers for every trial of the workgroup.
__device__ __forceinline__ void unit_segments(const ConeArgs& a, UnitCtx& C, int tid)
{
    const int lane = tid & 63, wave = tid >> 6;
    const uint4* const segs = reinterpret_cast<const uint4*>(a.blob + C.U.blob + C.U.run_off);
    C.mine = uni(C.nruns > wave ? (C.nruns - wave + kConeWaves - 1) / kConeWaves : 0);
    C.sv = make_uint4(0u, 0u, 0u, 0u);
    const int K = (C.nruns + kConeWaves - 1) / kConeWaves;
    if (lane < C.mine) C.sv = segs[wave * K + lane];
}

// Starts the unit of `item` at trial `trial`: its view (one scalar load of
// its UnitDesc) and, with `dma`, the LDS DMA of its blob into `aux` and of its
// bottom level into `buf` (unit_fill).  Nothing is waited for: the caller
// waits (vmcnt) and barriers before reading LDS.  `ok` = the kernel instance
// can run the unit (the host validates every schedule, validate_exec_plan;
// this guards the error flag): LDS buffer and register rows, the metadata
// area, rows of exactly SMAX slots for SMAX <= 5 (unmasked full slots;
// kPack2: the p <= 32 rows).
template <int SMAX, int RW>
__device__ __forceinline__ UnitCtx unit_begin(const ConeArgs& a, uint32_t item, uint32_t trial, uint32_t* aux,
                                              float* buf, int tid, bool dma, bool& ok, unsigned long long* ts = nullptr)
{
    UnitCtx C;
    C.U = unit_view(a, (int)item, (int)trial);
    const UnitView& U = C.U;
#ifdef RT_STAMPS
    if (ts) ts[0] = __builtin_amdgcn_s_memtime() + (U.p & 0);
#endif
    C.tile = U.mode == kModeTile;
    C.table = U.blob != kNoBlob;
    C.aux = aux;
    C.aux0 = aux;
    const int p = U.p;
    const int slots = merge_slots((uint32_t)p);
    ok = U.levels <= kMaxLevels && p > 0 &&
         ((SMAX <= 5 || SMAX == kPack2) ? slots == SMAX : (slots <= SMAX && slots != kPack2));
    const int cap = min(lds_row_capacity((uint32_t)p, SMAX), kConeWaves * RW * row_pack(SMAX));
    if (!C.table) {
        // short-row units always carry a blob, 4/5-slot units slot tables
        ok = ok && SMAX != kPack2 && (!resolved_slots(SMAX) || U.levels == 0);
        C.al = (int)(((uint32_t)U.node_start * (uint32_t)p) & 3u);
        C.slots = false;
        C.nruns = C.entries = C.nb = 0;
        const int nch = (U.node_size * p + C.al + 3) >> 2;
        ok = ok && !C.tile && U.node_size <= cap && 4 * nch <= kLdsBufFloats;
    } else {
        C.al = 0;
        // the blob's header counts come with the view (UnitDesc); its DMA
        // runs with one vector load -- the unit's DMA is issued two memory
        // round trips after the workgroup starts (a scalar load per run took
        // ~10K cycles for a 16-run tile)
        C.nruns = U.nruns;
        C.entries = U.entries;
        C.nb = U.nb;
        C.slots = U.slot_words != 0;
        const int words = U.run_off;   // the LDS part: header .. slot tables
        if constexpr (SMAX == kPack2) {
            // at the end of the level buffer, above the fill and every level
            // (validate_exec_plan; pack_blob_words)
            C.aux = reinterpret_cast<uint32_t*>(buf + kLdsBufFloats) - words;
            ok = ok && C.nb <= cap && 4 * U.fill_chunks + words <= kLdsBufFloats &&
                 C.nb * pack_stride(p) + words <= kLdsBufFloats;
        } else {
            ok = ok && C.nb <= cap && C.entries <= kDescEntries && words <= kAuxWords;
            // the 4-slot roll table lies past the blob's LDS part
            if (SMAX == 4 && C.slots) ok = ok && words <= kLut4Off;
            // the 4/5-slot instances run row-slot steps only (merge_levels)
            if (resolved_slots(SMAX)) ok = ok && (U.levels == 0 || (C.slots && (a.flags & kConeFuse2)));
            // the zero row of an all-fused whole unit: past its fill, inside the level buffer
            if (U.zero_row)
                ok = ok && resolved_slots(SMAX) && !C.tile && U.zero_row >= 4 * U.fill_chunks &&
                     U.zero_row + 64 * SMAX <= kLdsDataFloats;
        }
        ok = ok && words >= kBlobHeader + C.entries + C.nb && C.nruns <= 64 * kConeWaves && (words & 3) == 0;
    }
#ifdef RT_STAMPS
    if (ts) ts[1] = __builtin_amdgcn_s_memtime() + (ok ? 0 : 0);
#endif
    C.sv = make_uint4(0u, 0u, 0u, 0u);
    C.mine = 0;
    if (ok && dma) {
        if (C.table) unit_segments(a, C, tid);
        unit_fill<SMAX>(a, C, (int)trial, buf, tid, true);
    }
#ifdef RT_STAMPS
    if (ts) ts[2] = __builtin_amdgcn_s_memtime();
#endif
    return C;
}

// x mod p for 0 <= x < 2^22 and p >= 1 (roll shifts: x = s - t(s) < node
// size): a float-reciprocal quotient, off by at most one, then corrected --
// ~8 VALU instead of the ~35 of an integer remainder by a run-time p.
__device__ __forceinline__ int mod_small(int x, int p)
{
    const int q = (int)((float)x * __builtin_amdgcn_rcpf((float)p));
    int r = x - (int)__umul24((unsigned)q, (unsigned)p);
    r = r < 0 ? r + p : r;
    return r >= p ? r - p : r;
}

// Row descriptor (head row, tail row, roll shift) of output row r at level
// l of a whole unit (the node partition of its split tree), as row indices
// of the level below; t = -1 for a carried leaf (size-1 node).
__device__ __forceinline__ void row_desc(int node_size, int l, int r, int p, int& h, int& t, int& sh)
{
    int a0 = 0, sz = node_size;
    for (int d = 0; d < l; ++d) {
        if (sz > 1) {
            const int hs = sz >> 1;
            if (r - a0 < hs) sz = hs;
            else {
                a0 += hs;
                sz -= hs;
            }
        }
    }
    if (sz <= 1) {
        h = r;
        t = -1;
        sh = 0;
    } else {
        const int s = r - a0;
        const uint32_t hs = (uint32_t)sz >> 1, ts = (uint32_t)sz - hs;
        const int hh = (int)merge_index(merge_coef(hs, (uint32_t)sz), (uint32_t)s);
        const int tt = (int)merge_index(merge_coef(ts, (uint32_t)sz), (uint32_t)s);
        h = a0 + hh;
        t = a0 + (int)hs + tt;
        sh = mod_small(s - tt, p);
    }
}

// Packed row descriptor: head row | tail row << 10 | shift << 20 (tail row
// kCarried: a size-1 node carried unchanged).  Rows < 1023, shift < 4096.
constexpr uint32_t kCarried = kCarriedRow;

__device__ __forceinline__ uint32_t pack_desc(int h, int t, int sh)
{
    return (uint32_t)h | ((t < 0 ? kCarried : (uint32_t)t) << 10) | ((uint32_t)sh << 20);
}

// Descriptor of output row r of level l: the tile table, or the node partition.
__device__ __forceinline__ uint32_t unit_desc(const UnitCtx& C, int l, int r, int p)
{
    if (C.table) return desc_table(C)[desc_offset(C, l) + r];
    int h, t, sh;
    row_desc(C.U.node_size, l, r, p, h, t, sh);
    return pack_desc(h, t, sh);
}

typedef const __attribute__((address_space(3))) float* lds_cptr;

// LDS reads the compiler must not pair into ds_read2_b32 / ds_read2st64_b32
// (those issue at a lower rate than separate ds_read_b32 on gfx950,
// tools/microbench/lds_b64.hip): volatile accesses are never merged.
__device__ __forceinline__ float lds_ld(lds_cptr p) { return *(const volatile __attribute__((address_space(3))) float*)p; }

// Outputs of level l (rows wave + 8i) into v, from the level below in dense
// rows of stride p at `src`:
//   out[j] = H[j] + T[(j + s) mod p]
// Bins j = lane + 64k: one ds_read_b32 of H and one of T per slot, T[j + s]
// before the wrap point p - s and T[j + s - p] from it on (two opaque
// per-row bases and a compare/select per slot; the slot offset 256k an
// immediate).  Per row the descriptor is one v_readlane of the packed word
// (unpacked in SALU).  The additions are the reference's, element by
// element.  CARRIED: the level may hold size-1 nodes (whole units near their
// leaves), whose rows add -0.0 to H (x + (-0.0) == x exactly, as the
// reference's copy).  Branch-free over rows and slots: rows i >= nr and bins
// past p read in-bounds garbage that is never written back.
template <int SMAX, int RW, bool CARRIED>
__device__ __forceinline__ void merge_level_dense(const UnitCtx& C, const float* src, int p, int l, int lane,
                                                  int wave, int nr, float (&v)[RW][SMAX], const int* loff)
{
    const int S = (p + 63) >> 6;
    // lane i unpacks the descriptor of the wave's i-th row into LDS float
    // offsets (head row, tail row + shift) and the shift; the row loop takes
    // them with v_readlane, so no per-row scalar unpacking or multiplies
    int ho = 0, to = 0, sh = 0, car = 0;
    if (lane < nr) {
        const uint32_t d = unit_desc(C, l, wave + kConeWaves * lane, p);
        const uint32_t tc = (d >> 10) & 1023u;
        sh = (int)(d >> 20);
        // source rows: dense (stride p), or the bottom level's fill layout
        ho = loff ? loff[d & 1023u] : (int)(d & 1023u) * p;
        to = (tc == kCarried ? ho : (loff ? loff[tc] : (int)tc * p)) + sh;
        car = tc == kCarried;
    }
    const lds_cptr l1 = (lds_cptr)src + lane;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        const int hoi = __builtin_amdgcn_readlane(ho, i);
        const int toi = __builtin_amdgcn_readlane(to, i);
        const int si = __builtin_amdgcn_readlane(sh, i);
        uint32_t keep = 0xFFFFFFFFu, neg0 = 0u;
        if (CARRIED) {
            keep = __builtin_amdgcn_readlane(car, i) ? 0u : 0xFFFFFFFFu;
            neg0 = ~keep & 0x80000000u;
        }
        const lds_cptr hrow = l1 + hoi;
        lds_cptr ta = l1 + toi;
        lds_cptr tw = ta - p;
        asm("" : "+v"(ta), "+v"(tw));
        const int ls = lane + si;               // bin j = lane + 64k wraps when ls >= p - 64k
#pragma unroll
        for (int k = 0; k < SMAX; ++k) {
            if (SMAX <= 5 || k < S) {
                const lds_cptr tp = ls >= p - 64 * k ? tw : ta;
                float x = lds_ld(tp + 64 * k);
                if (CARRIED) x = __uint_as_float((__float_as_uint(x) & keep) | neg0);
                v[i][k] = __fadd_rn(hrow[64 * k], x);
            }
        }
    }
}

// Two merge levels in one LDS round trip: the outputs of level l from the
// rows of level l + 2 (the level l + 1 in between is never stored).  Output
// row r of level l is H[h] + roll(T[t], sh) with H, T rows of level l + 1,
// and H[h] = HH[hh] + roll(HT[ht], sH), T[t] = TH[th] + roll(TT[tt], sT) from
// level l + 2, so bin j is
//     (HH[hh][j] + HT[ht][(j + sH) mod p])
//   + (TH[th][(j + sh) mod p] + TT[tt][(j + sh + sT) mod p])
// -- the reference's float additions on the same operands in the same
// association (transforms.hpp:13-27 applied twice), so bit-exact.  Per
// 64-bin slot: 4 ds_read_b32 + 1 ds_write_b32 per two levels instead of 4 + 2.
// Only levels whose nodes all have >= 2 rows (no carried size-1 nodes at
// level l + 1) are fused.
template <int SMAX, int RW>
__device__ __forceinline__ void merge_level2_dense(const UnitCtx& C, const float* src, int p, int l, int lane,
                                                   int wave, int nr, float (&v)[RW][SMAX], const int* loff)
{
    const int S = (p + 63) >> 6;
    int o0 = 0, o1 = 0, o2 = 0, o3 = 0, s1 = 0, s2 = 0, s3 = 0;
    if (lane < nr) {
        const uint32_t d0 = unit_desc(C, l, wave + kConeWaves * lane, p);
        const uint32_t dh = unit_desc(C, l + 1, (int)(d0 & 1023u), p);
        const uint32_t dt = unit_desc(C, l + 1, (int)((d0 >> 10) & 1023u), p);
        const int sh = (int)(d0 >> 20), sH = (int)(dh >> 20), sT = (int)(dt >> 20);
        int sTT = sh + sT;
        sTT = sTT >= p ? sTT - p : sTT;
        // source rows: dense (stride p), or the bottom level's fill layout
        const uint32_t r0 = dh & 1023u, r1 = (dh >> 10) & 1023u, r2 = dt & 1023u, r3 = (dt >> 10) & 1023u;
        o0 = (loff ? loff[r0] : (int)r0 * p);
        o1 = (loff ? loff[r1] : (int)r1 * p) + sH;
        o2 = (loff ? loff[r2] : (int)r2 * p) + sh;
        o3 = (loff ? loff[r3] : (int)r3 * p) + sTT;
        s1 = sH;
        s2 = sh;
        s3 = sTT;
    }
    const lds_cptr l1 = (lds_cptr)src + lane;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        const lds_cptr hrow = l1 + __builtin_amdgcn_readlane(o0, i);
        lds_cptr b1 = l1 + __builtin_amdgcn_readlane(o1, i);
        lds_cptr b2 = l1 + __builtin_amdgcn_readlane(o2, i);
        lds_cptr b3 = l1 + __builtin_amdgcn_readlane(o3, i);
        lds_cptr w1 = b1 - p, w2 = b2 - p, w3 = b3 - p;
        asm("" : "+v"(b1), "+v"(w1), "+v"(b2), "+v"(w2), "+v"(b3), "+v"(w3));
        const int ls1 = lane + __builtin_amdgcn_readlane(s1, i);
        const int ls2 = lane + __builtin_amdgcn_readlane(s2, i);
        const int ls3 = lane + __builtin_amdgcn_readlane(s3, i);
#pragma unroll
        for (int k = 0; k < SMAX; ++k) {
            if (SMAX <= 5 || k < S) {
                const int wk = p - 64 * k;
                const float x1 = lds_ld((ls1 >= wk ? w1 : b1) + 64 * k);
                const float x2 = lds_ld((ls2 >= wk ? w2 : b2) + 64 * k);
                const float x3 = lds_ld((ls3 >= wk ? w3 : b3) + 64 * k);
                v[i][k] = __fadd_rn(__fadd_rn(hrow[64 * k], x1), __fadd_rn(x2, x3));
            }
        }
    }
}

// Output level l == 0 of a non-final pass: straight from the staging
// registers to global memory at byte offset st_o0 (the tile's rows are one
// contiguous segment).
template <int SMAX, int RW>
__device__ __forceinline__ void store_rows(const float (&v)[RW][SMAX], int p, int lane, int wave, int nr,
                                           __amdgpu_buffer_rsrc_t rs, uint32_t st_o0)
{
    const int S = (p + 63) >> 6;
    const bool tail_ok = lane + 64 * (SMAX - 1) < p;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (i < nr) {
            const uint32_t ob = st_o0 + (uint32_t)((wave + kConeWaves * i) * p + lane) * 4u;
#pragma unroll
            for (int k = 0; k < SMAX; ++k) {
                if constexpr (SMAX <= 5) {
                    // rows of exactly SMAX slots: the last slot's lanes past p
                    // store out of the buffer's range, which drops them
                    const uint32_t o = k < SMAX - 1 ? ob + 256u * (uint32_t)k
                                                    : (tail_ok ? ob + 256u * (uint32_t)k : 0x80000000u);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][k]), rs, (int)o, 0, kStoreCpol);
                } else if (64 * (k + 1) <= p || (k < S && lane + 64 * k < p)) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][k]), rs,
                                                          (int)(ob + 256u * (uint32_t)k), 0, kStoreCpol);
                }
            }
        }
    }
}

// Write-back of a level's staged rows into the dense LDS rows at `base`.
// SMAX <= 5 kernels run rows of exactly SMAX slots: all but the last are
// full; the last slot's lanes past p write to a dummy word in the LDS pad
// (an address select instead of an exec-mask save/restore per row).
template <int SMAX, int RW>
__device__ __forceinline__ void write_rows(float* base, float* dummy, const float (&v)[RW][SMAX], int p, int lane,
                                           int wave, int nr)
{
    const int S = (p + 63) >> 6;
    const bool tail_ok = lane + 64 * (SMAX - 1) < p;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (i < nr) {
            float* orow = base + (wave + kConeWaves * i) * p + lane;
#pragma unroll
            for (int k = 0; k < SMAX; ++k) {
                if constexpr (SMAX <= 5) {
                    if (k < SMAX - 1) orow[64 * k] = v[i][k];
                    else *(tail_ok ? orow + 64 * k : dummy) = v[i][k];
                } else {
                    if (64 * (k + 1) <= p || (k < S && lane + 64 * k < p)) orow[64 * k] = v[i][k];
                }
            }
        }
    }
}

// Row-slot merge steps (units with a blob, SMAX <= 5 rows of exactly SMAX
// slots; common.hpp kSlotPair).  A wave's slot q fills register rows 2q and
// 2q + 1: one output row, two independent rows, or a row pair r, r + 1 with
// the same head and tail rows and roll shifts s, s + 1.  The pair's second
// row reuses the first's terms: with H = the head term and T the rolled tail
// term of row r (fused: H = HH + roll(HT, sH), T = roll(TH, s) +
// roll(TT, s + sT)), row r + 1 is H[j] + T[(j + 1) mod p] -- the same float
// operands in the same association as computing it directly, so bit-exact --
// taken with one DPP lane shift (wave_shl:1) per 64-bin slot, the slot's
// lane 63 from lane 0 of the next slot, and bin p - 1 from bin 0.  Half the
// LDS reads of the pair.
//
// Per-row terms from the row's scalars (SGPRs): r0 head row offset, r1..r3
// the rolled rows' offsets (+ their rolls), t1..t3 the rolls, c1 carried.
// HEAD false (row B of a kSlotHalf): only the tail term; hs is row A's.
template <int SMAX, bool TWO, bool HEAD = true>
__device__ __forceinline__ void row_terms_s(lds_cptr l1, int p, int lane, int r0, int r1, int r2, int r3, int t1,
                                            int t2, int t3, int c1, float (&hs)[SMAX], float (&ts)[SMAX])
{
    if constexpr (TWO && !HEAD) {
        lds_cptr b2 = l1 + r2;
        lds_cptr b3 = l1 + r3;
        lds_cptr w2 = b2 - p, w3 = b3 - p;
        asm("" : "+v"(b2), "+v"(w2), "+v"(b3), "+v"(w3));
        const int ls2 = lane + t2;
        const int ls3 = lane + t3;
#pragma unroll
        for (int k = 0; k < SMAX; ++k) {
            const int wk = p - 64 * k;
            const float x2 = lds_ld((ls2 >= wk ? w2 : b2) + 64 * k);
            const float x3 = lds_ld((ls3 >= wk ? w3 : b3) + 64 * k);
            ts[k] = __fadd_rn(x2, x3);
        }
    } else if constexpr (TWO) {
        const lds_cptr hrow = l1 + r0;
        lds_cptr b1 = l1 + r1;
        lds_cptr b2 = l1 + r2;
        lds_cptr b3 = l1 + r3;
        lds_cptr w1 = b1 - p, w2 = b2 - p, w3 = b3 - p;
        asm("" : "+v"(b1), "+v"(w1), "+v"(b2), "+v"(w2), "+v"(b3), "+v"(w3));
        const int ls1 = lane + t1;
        const int ls2 = lane + t2;
        const int ls3 = lane + t3;
#pragma unroll
        for (int k = 0; k < SMAX; ++k) {
            const int wk = p - 64 * k;
            const float x1 = lds_ld((ls1 >= wk ? w1 : b1) + 64 * k);
            const float x2 = lds_ld((ls2 >= wk ? w2 : b2) + 64 * k);
            const float x3 = lds_ld((ls3 >= wk ? w3 : b3) + 64 * k);
            hs[k] = __fadd_rn(lds_ld(hrow + 64 * k), x1);
            ts[k] = __fadd_rn(x2, x3);
        }
    } else if constexpr (!HEAD) {
        // single step, row B of a half: its tail only (never carried)
        lds_cptr ta = l1 + r1;
        lds_cptr tw = ta - p;
        asm("" : "+v"(ta), "+v"(tw));
        const int ls = lane + t1;
#pragma unroll
        for (int k = 0; k < SMAX; ++k) ts[k] = lds_ld((ls >= p - 64 * k ? tw : ta) + 64 * k);
    } else {
        // r0 head row, r1 tail row + shift, t1 shift, c1 carried (size-1 node:
        // the tail term is -0.0, x + (-0.0) == x exactly)
        const lds_cptr hrow = l1 + r0;
        lds_cptr ta = l1 + r1;
        lds_cptr tw = ta - p;
        asm("" : "+v"(ta), "+v"(tw));
        const int ls = lane + t1;
        const uint32_t keep = c1 ? 0u : 0xFFFFFFFFu;
        const uint32_t neg0 = ~keep & 0x80000000u;
#pragma unroll
        for (int k = 0; k < SMAX; ++k) {
            const float x = lds_ld((ls >= p - 64 * k ? tw : ta) + 64 * k);
            hs[k] = lds_ld(hrow + 64 * k);
            ts[k] = __uint_as_float((__float_as_uint(x) & keep) | neg0);
        }
    }
}

// Roll table (4-slot rows, p = 193..256): a rolled read of a
// row at roll t takes bin j = lane + 64k from T[(lane + t + 64k) mod p].
// Entry x = lane + t (x < p + 64) of a per-unit LDS table holds the four
// byte offsets 4 ((x + 64k) mod p), k = 0..3, as 16-bit halves of 8 bytes:
// one conflict-free ds_read_b64 per rolled row (consecutive lanes,
// consecutive entries), then one address add per slot from the row's start
// (an SGPR) -- instead of a compare and a select per slot against the wrap
// point.  Same LDS words, same additions: bit-exact.  The table sits at the
// end of the unit's metadata area (kLut4Off, past every blob's LDS part:
// validate_exec_plan) and is rebuilt by every unit of a 4-slot instance.
typedef const __attribute__((address_space(3))) unsigned long long* lut_cptr;
typedef const __attribute__((address_space(3))) char* lds_ccptr;

// rolled row whose roll-table entry is e and whose row starts at byte `rb`
// of LDS (uniform)
__device__ __forceinline__ void rolled_lut4(lds_ccptr rb, unsigned long long e, float (&x)[4])
{
    const uint32_t e0 = (uint32_t)e, e1 = (uint32_t)(e >> 32);
    x[0] = lds_ld((lds_cptr)(rb + (e0 & 0xFFFFu)));
    x[1] = lds_ld((lds_cptr)(rb + (e0 >> 16)));
    x[2] = lds_ld((lds_cptr)(rb + (e1 & 0xFFFFu)));
    x[3] = lds_ld((lds_cptr)(rb + (e1 >> 16)));
}

// row_terms_s with the roll table: s0 the level's rows (uniform), r0 the head
// row's offset, q1..q3 the rolled rows' offsets WITHOUT their rolls t1..t3.
// The table entries are read first (plain loads, free to move) and the head
// row before the rolled rows (the volatile reads keep their order), so the
// head reads are in flight while the entries return.
template <bool TWO, bool HEAD = true>
__device__ __forceinline__ void row_terms_lut(lds_cptr l1, lds_cptr s0, lut_cptr lutl, int r0, int q1, int q2, int q3,
                                              int t1, int t2, int t3, int c1, float (&hs)[4], float (&ts)[4])
{
    const lds_ccptr b = (lds_ccptr)s0;
    if constexpr (TWO) {
        const unsigned long long e1 = HEAD ? lutl[t1] : 0ull;
        const unsigned long long e2 = lutl[t2], e3 = lutl[t3];
        float h[4], x1[4], x2[4], x3[4];
        if constexpr (HEAD) {
#pragma unroll
            for (int k = 0; k < 4; ++k) h[k] = lds_ld(l1 + r0 + 64 * k);
            rolled_lut4(b + 4 * q1, e1, x1);
        }
        rolled_lut4(b + 4 * q2, e2, x2);
        rolled_lut4(b + 4 * q3, e3, x3);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if constexpr (HEAD) hs[k] = __fadd_rn(h[k], x1[k]);
            ts[k] = __fadd_rn(x2[k], x3[k]);
        }
    } else {
        const unsigned long long e = lutl[t1];
        float x[4];
        if constexpr (HEAD) {
#pragma unroll
            for (int k = 0; k < 4; ++k) hs[k] = lds_ld(l1 + r0 + 64 * k);
        }
        rolled_lut4(b + 4 * q1, e, x);
        if constexpr (HEAD) {
            // c1: a carried size-1 node (its tail term is -0.0, x + (-0.0) == x)
            const uint32_t keep = c1 ? 0u : 0xFFFFFFFFu;
            const uint32_t neg0 = ~keep & 0x80000000u;
#pragma unroll
            for (int k = 0; k < 4; ++k) ts[k] = __uint_as_float((__float_as_uint(x[k]) & keep) | neg0);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) ts[k] = x[k];
        }
    }
}

// Builds the roll table of rows of p bins (4-slot instances) at `lut`:
// entry x < p + 64 = {4 (x mod p) | 4 ((x + 64) mod p) << 16,
//                     4 ((x + 128) mod p) | 4 ((x + 192) mod p) << 16}.
__device__ __forceinline__ void build_roll_lut4(uint32_t* lut, int p, int tid)
{
    for (int w = tid; w < 2 * (p + 64); w += kConeBlock) {
        const int x = (w >> 1) + 128 * (w & 1);
        int y0 = x, y1 = x + 64;
        // y < p + 256 < 3p (p >= 193): at most two subtractions
        y0 -= y0 >= p ? p : 0;
        y0 -= y0 >= p ? p : 0;
        y1 -= y1 >= p ? p : 0;
        y1 -= y1 >= p ? p : 0;
        lut[w] = (uint32_t)(4 * y0) | ((uint32_t)(4 * y1) << 16);
    }
}

// Per-row terms of the row whose resolved descriptor sits in lane i
// (unpacked per lane: o0 .. o3, s1 .. s3; seven v_readlane per row).
template <int SMAX, bool TWO, bool HEAD = true>
__device__ __forceinline__ void row_terms(lds_cptr l1, int p, int lane, int i, int o0, int o1, int o2, int o3, int s1,
                                          int s2, int s3, float (&hs)[SMAX], float (&ts)[SMAX],
                                          lds_cptr s0 = nullptr, lut_cptr lutl = nullptr)
{
    if constexpr (SMAX == 4) {
        // o1 .. o3 are the rolled rows' offsets without their rolls here
        if constexpr (TWO) {
            if constexpr (HEAD) {
                int r0 = __builtin_amdgcn_readlane(o0, i), q1 = __builtin_amdgcn_readlane(o1, i);
                int q2 = __builtin_amdgcn_readlane(o2, i), q3 = __builtin_amdgcn_readlane(o3, i);
                int t1 = __builtin_amdgcn_readlane(s1, i), t2 = __builtin_amdgcn_readlane(s2, i);
                int t3 = __builtin_amdgcn_readlane(s3, i);
                asm volatile("" : "+s"(r0), "+s"(q1), "+s"(q2), "+s"(q3), "+s"(t1), "+s"(t2), "+s"(t3));
                row_terms_lut<true>(l1, s0, lutl, r0, q1, q2, q3, t1, t2, t3, 0, hs, ts);
            } else {
                int q2 = __builtin_amdgcn_readlane(o2, i), q3 = __builtin_amdgcn_readlane(o3, i);
                int t2 = __builtin_amdgcn_readlane(s2, i), t3 = __builtin_amdgcn_readlane(s3, i);
                asm volatile("" : "+s"(q2), "+s"(q3), "+s"(t2), "+s"(t3));
                row_terms_lut<true, false>(l1, s0, lutl, 0, 0, q2, q3, 0, t2, t3, 0, hs, ts);
            }
        } else {
            if constexpr (HEAD) {
                int r0 = __builtin_amdgcn_readlane(o0, i), q1 = __builtin_amdgcn_readlane(o1, i);
                int t1 = __builtin_amdgcn_readlane(s1, i), c1 = __builtin_amdgcn_readlane(o2, i);
                asm volatile("" : "+s"(r0), "+s"(q1), "+s"(t1), "+s"(c1));
                row_terms_lut<false>(l1, s0, lutl, r0, q1, 0, 0, t1, 0, 0, c1, hs, ts);
            } else {
                int q1 = __builtin_amdgcn_readlane(o1, i), t1 = __builtin_amdgcn_readlane(s1, i);
                asm volatile("" : "+s"(q1), "+s"(t1));
                row_terms_lut<false, false>(l1, s0, lutl, 0, q1, 0, 0, t1, 0, 0, 0, hs, ts);
            }
        }
        return;
    }
    // all of the row's scalars first, in distinct SGPRs: a v_readlane result
    // read by the next VALU instruction costs s_nop wait states
    if constexpr (TWO) {
        if constexpr (HEAD) {
            int r0 = __builtin_amdgcn_readlane(o0, i), r1 = __builtin_amdgcn_readlane(o1, i);
            int r2 = __builtin_amdgcn_readlane(o2, i), r3 = __builtin_amdgcn_readlane(o3, i);
            int t1 = __builtin_amdgcn_readlane(s1, i), t2 = __builtin_amdgcn_readlane(s2, i);
            int t3 = __builtin_amdgcn_readlane(s3, i);
            asm volatile("" : "+s"(r0), "+s"(r1), "+s"(r2), "+s"(r3), "+s"(t1), "+s"(t2), "+s"(t3));
            row_terms_s<SMAX, true>(l1, p, lane, r0, r1, r2, r3, t1, t2, t3, 0, hs, ts);
        } else {
            int r2 = __builtin_amdgcn_readlane(o2, i), r3 = __builtin_amdgcn_readlane(o3, i);
            int t2 = __builtin_amdgcn_readlane(s2, i), t3 = __builtin_amdgcn_readlane(s3, i);
            asm volatile("" : "+s"(r2), "+s"(r3), "+s"(t2), "+s"(t3));
            row_terms_s<SMAX, true, false>(l1, p, lane, 0, 0, r2, r3, 0, t2, t3, 0, hs, ts);
        }
    } else {
        if constexpr (HEAD) {
            int r0 = __builtin_amdgcn_readlane(o0, i), r1 = __builtin_amdgcn_readlane(o1, i);
            int t1 = __builtin_amdgcn_readlane(s1, i), c1 = __builtin_amdgcn_readlane(o2, i);
            asm volatile("" : "+s"(r0), "+s"(r1), "+s"(t1), "+s"(c1));
            row_terms_s<SMAX, false>(l1, p, lane, r0, r1, 0, 0, t1, 0, 0, c1, hs, ts);
        } else {
            int r1 = __builtin_amdgcn_readlane(o1, i), t1 = __builtin_amdgcn_readlane(s1, i);
            asm volatile("" : "+s"(r1), "+s"(t1));
            row_terms_s<SMAX, false, false>(l1, p, lane, 0, r1, 0, 0, t1, 0, 0, 0, hs, ts);
        }
    }
}

template <int SMAX, int RW, bool TWO>
__device__ __forceinline__ void merge_step_slots(const UnitCtx& C, const float* src, int p, int lo, int lane,
                                                 int wave, float (&v)[RW][SMAX], const int* loff, uint32_t& sw,
                                                 int& nq)
{
    constexpr int Q = (RW + 1) / 2;
    static_assert(Q <= 32, "row slots: one lane per slot row");
    const uint32_t* st = slot_table(C, lo);
    const int ns = uni((int)st[0]);
    nq = uni(ns > wave ? (ns - wave + kConeWaves - 1) / kConeWaves : 0);
    // lane i < 32 resolves row A of the wave's slot i, lane 32 + i its row B
    const int qi = lane & 31;
    int o0 = 0, o1 = 0, o2 = 0, o3 = 0, s1 = 0, s2 = 0, s3 = 0;
    if constexpr (resolved_slots(SMAX)) {
        // host-resolved rows: one 16-byte entry per lane (the slot's row A in
        // lanes 0-31 with the slot word, row B in lanes 32-63)
        // wave-major halves (build_tile_blob): the 32 lanes of a half read
        // consecutive 16-byte entries; lanes past Q re-read entry Q - 1
        const int qc = qi < Q ? qi : Q - 1;
        const uint4 e = reinterpret_cast<const uint4*>(st)[1 + (lane >> 5) * (kConeWaves * Q) + wave * Q + qc];
        sw = lane < 32 ? e.w : 0u;
        s1 = (int)(e.z & 1023u);
        // the roll table path takes the rolled rows' offsets without rolls
        constexpr int roll_in = SMAX == 4 ? 0 : 1;
        if constexpr (TWO) {
            s2 = (int)((e.z >> 10) & 1023u);
            s3 = (int)((e.z >> 20) & 1023u);
            o0 = (int)(e.x & 0xFFFFu);
            o1 = (int)(e.x >> 16) + roll_in * s1;
            o2 = (int)(e.y & 0xFFFFu) + roll_in * s2;
            o3 = (int)(e.y >> 16) + roll_in * s3;
        } else {
            o0 = (int)(e.x & 0xFFFFu);
            o1 = (int)(e.x >> 16) + roll_in * s1;
            o2 = (int)((e.z >> 30) & 1u);
        }
        (void)loff;
    } else {
    sw = qi < nq ? st[1 + wave + kConeWaves * qi] : 0u;
    const bool act = qi < nq && (lane < 32 || (sw >> 20) == kSlotTwo || (sw >> 20) == kSlotHalf);
    const int r = lane < 32 ? (int)(sw & 1023u) : (int)((sw >> 10) & 1023u);
    const uint32_t* const desc = desc_table(C);
    // the first step reads the bottom level through its row offsets
    const bool use_loff = loff != nullptr;
    if (act) {
        if constexpr (TWO) {
            const uint32_t d0 = desc[desc_offset(C, lo) + r];
            const uint32_t dh = desc[desc_offset(C, lo + 1) + (int)(d0 & 1023u)];
            const uint32_t dt = desc[desc_offset(C, lo + 1) + (int)((d0 >> 10) & 1023u)];
            const int sh = (int)(d0 >> 20), sH = (int)(dh >> 20), sT = (int)(dt >> 20);
            int sTT = sh + sT;
            sTT = sTT >= p ? sTT - p : sTT;
            const uint32_t r0 = dh & 1023u, r1 = (dh >> 10) & 1023u, r2 = dt & 1023u, r3 = (dt >> 10) & 1023u;
            o0 = (use_loff ? loff[r0] : (int)__umul24(r0, (uint32_t)p));
            o1 = (use_loff ? loff[r1] : (int)__umul24(r1, (uint32_t)p)) + sH;
            o2 = (use_loff ? loff[r2] : (int)__umul24(r2, (uint32_t)p)) + sh;
            o3 = (use_loff ? loff[r3] : (int)__umul24(r3, (uint32_t)p)) + sTT;
            s1 = sH;
            s2 = sh;
            s3 = sTT;
        } else {
            const uint32_t d = desc[desc_offset(C, lo) + r];
            const uint32_t tc = (d >> 10) & 1023u;
            s1 = (int)(d >> 20);
            o0 = use_loff ? loff[d & 1023u] : (int)__umul24(d & 1023u, (uint32_t)p);
            o1 = (tc == kCarried ? o0 : (use_loff ? loff[tc] : (int)__umul24(tc, (uint32_t)p))) + s1;
            o2 = tc == kCarried;
        }
    }
    }
    const lds_cptr l1 = (lds_cptr)src + lane;
    const lds_cptr s0 = (lds_cptr)src;
    const lut_cptr lutl = (lut_cptr)(C.aux0 + kLut4Off) + lane;
    const int jl = p - 1 - 64 * (SMAX - 1);   // lane of bin p - 1 in the last slot
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        if (q < nq) {
            const uint32_t kq = (uint32_t)__builtin_amdgcn_readlane((int)sw, q) >> 20;
            float hs[SMAX], ts[SMAX];
            row_terms<SMAX, TWO>(l1, p, lane, q, o0, o1, o2, o3, s1, s2, s3, hs, ts, s0, lutl);
#pragma unroll
            for (int k = 0; k < SMAX; ++k) v[2 * q][k] = __fadd_rn(hs[k], ts[k]);
            const int qb = 2 * q + 1 < RW ? 2 * q + 1 : RW - 1;   // row B's register row (q < Q: in range)
            if (2 * q + 1 < RW) {
                if (kq == kSlotPair) {
#ifdef RT_PAIR_SELECT
                    int n0[SMAX];
#pragma unroll
                    for (int k = 0; k < SMAX; ++k) n0[k] = __builtin_amdgcn_readlane(__float_as_int(ts[(k + 1) % SMAX]), 0);
#pragma unroll
                    for (int k = 0; k < SMAX; ++k) {
                        // wave_shl:1 -- lane L takes lane L + 1 (lane 63: bound_ctrl 0, replaced)
                        float x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(ts[k]), 0x130, 0xF, 0xF, true));
                        x = lane == (k + 1 < SMAX ? 63 : jl) ? __int_as_float(n0[k]) : x;
                        v[qb][k] = __fadd_rn(hs[k], x);
                    }
#else
                    // bin j + 1 of the rolled tail term: slot k's lanes 0-62
                    // from lanes 1-63 (wave_shl:1, bound_ctrl off: lane 63 has
                    // no source and keeps the old value), lane 63 from lane 0
                    // of slot k + 1 (the old value: wave_rol:1 of slot k + 1);
                    // the last slot's bin p - 1 (lane jl) takes bin 0 (lane 0
                    // of slot 0) by v_writelane -- two or three VALU per slot
                    // instead of a v_readlane, a move and a select each
                    const int w0 = __builtin_amdgcn_readlane(__float_as_int(ts[0]), 0);
#pragma unroll
                    for (int k = 0; k < SMAX; ++k) {
                        int x;
                        if (k + 1 < SMAX) {
                            const int nx = __builtin_amdgcn_mov_dpp(__float_as_int(ts[k + 1]), 0x134, 0xF, 0xF, false);
                            x = __builtin_amdgcn_update_dpp(nx, __float_as_int(ts[k]), 0x130, 0xF, 0xF, false);
                        } else {
                            x = __builtin_amdgcn_mov_dpp(__float_as_int(ts[k]), 0x130, 0xF, 0xF, true);
                            // lane select in M0 (gfx9: one SGPR operand per VALU instruction)
                            asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(x) : "s"(w0), "s"(jl)
                                         : "m0");
                        }
                        v[qb][k] = __fadd_rn(hs[k], __int_as_float(x));
                    }
#endif
                } else if (kq == kSlotHalf) {
                    // row B shares row A's head term: only its tail term
                    float tb[SMAX];
                    row_terms<SMAX, TWO, false>(l1, p, lane, 32 + q, o0, o1, o2, o3, s1, s2, s3, hs, tb, s0, lutl);
#pragma unroll
                    for (int k = 0; k < SMAX; ++k) v[qb][k] = __fadd_rn(hs[k], tb[k]);
                } else if (kq == kSlotTwo) {
                    row_terms<SMAX, TWO>(l1, p, lane, 32 + q, o0, o1, o2, o3, s1, s2, s3, hs, ts, s0, lutl);
#pragma unroll
                    for (int k = 0; k < SMAX; ++k) v[qb][k] = __fadd_rn(hs[k], ts[k]);
                }
            }
        }
    }
}

// Slot-step write-back into the dense LDS rows at base / store to global
// memory (a non-final pass's output level): register rows 2q, 2q + 1 to the
// slot's rows A and B (row stride q: p, or a final pass's S/N stride).
#ifndef RT_NO_ADDTID_WRITES
// A row's full 64-bin slots (all but the last) by ds_write_addtid_b32: the
// address is M0 + offset + 4 lane (no address VGPR), 2 LDS cycles per wave
// instruction instead of ds_write_b32's 4.  M0 holds 16 bits: rows past
// 64 KiB - 1 KiB take M0 = a - 32 KiB and offsets from 32 KiB.  Same-box
// A/B, cone ms per trial (profiles/r05q_ab_*.log): cfg2 6.56-6.58 vs
// 6.59-6.62, cfg3 1.658-1.693 vs 1.670-1.697 (RT_NO_ADDTID_WRITES: the
// ds_write_b32 form).
template <int SMAX>
__device__ __forceinline__ void write_row_addtid(uint32_t a, const float (&x)[SMAX])
{
    static_assert(SMAX == 4 || SMAX == 5, "4/5-slot rows");
    if (a <= 0xFFFFu - 256u * (SMAX - 2)) {
        if constexpr (SMAX == 4)
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tds_write_addtid_b32 %1\n\tds_write_addtid_b32 %2 offset:256\n\t"
                         "ds_write_addtid_b32 %3 offset:512"
                         :: "s"(a), "v"(x[0]), "v"(x[1]), "v"(x[2]) : "memory", "m0");
        else
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tds_write_addtid_b32 %1\n\tds_write_addtid_b32 %2 offset:256\n\t"
                         "ds_write_addtid_b32 %3 offset:512\n\tds_write_addtid_b32 %4 offset:768"
                         :: "s"(a), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]) : "memory", "m0");
    } else {
        const uint32_t b = a - 32768u;
        if constexpr (SMAX == 4)
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tds_write_addtid_b32 %1 offset:32768\n\t"
                         "ds_write_addtid_b32 %2 offset:33024\n\tds_write_addtid_b32 %3 offset:33280"
                         :: "s"(b), "v"(x[0]), "v"(x[1]), "v"(x[2]) : "memory", "m0");
        else
            asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tds_write_addtid_b32 %1 offset:32768\n\t"
                         "ds_write_addtid_b32 %2 offset:33024\n\tds_write_addtid_b32 %3 offset:33280\n\t"
                         "ds_write_addtid_b32 %4 offset:33536"
                         :: "s"(b), "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]) : "memory", "m0");
    }
}
#endif

template <int SMAX, int RW>
__device__ __forceinline__ void write_rows_slots(float* base, float* dummy, const float (&v)[RW][SMAX], int p,
                                                 int lane, uint32_t sw, int nq, int q)
{
    const bool tail_ok = lane + 64 * (SMAX - 1) < p;
#ifndef RT_NO_ADDTID_WRITES
    if constexpr (resolved_slots(SMAX)) {
        typedef __attribute__((address_space(3))) float* lds_fptr;
        const uint32_t b0 = (uint32_t)(uintptr_t)(lds_fptr)base;
#pragma unroll
        for (int i = 0; i < RW; ++i) {
            if (i / 2 < nq) {
                const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)sw, i / 2);
                if (i % 2 == 0 || (w >> 20) != kSlotOne) {
                    const int row = (int)((i % 2 == 0 ? w : w >> 10) & 1023u);
                    write_row_addtid<SMAX>(b0 + 4u * (uint32_t)(row * q), v[i]);
                    float* orow = base + row * q + lane;
                    *(tail_ok ? orow + 64 * (SMAX - 1) : dummy) = v[i][SMAX - 1];
                }
            }
        }
        return;
    }
#endif
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (i / 2 < nq) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)sw, i / 2);
            if (i % 2 == 0 || (w >> 20) != kSlotOne) {
                const int row = (int)((i % 2 == 0 ? w : w >> 10) & 1023u);
                float* orow = base + row * q + lane;
#pragma unroll
                for (int k = 0; k < SMAX; ++k) {
                    if (k < SMAX - 1) orow[64 * k] = v[i][k];
                    else *(tail_ok ? orow + 64 * k : dummy) = v[i][k];
                }
            }
        }
    }
}

template <int SMAX, int RW>
__device__ __forceinline__ void store_rows_slots(const float (&v)[RW][SMAX], int p, int lane, uint32_t sw, int nq,
                                                 __amdgpu_buffer_rsrc_t rs, uint32_t st_o0)
{
    const bool tail_ok = lane + 64 * (SMAX - 1) < p;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (i / 2 < nq) {
            const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)sw, i / 2);
            if (i % 2 == 0 || (w >> 20) != kSlotOne) {
                const int row = (int)((i % 2 == 0 ? w : w >> 10) & 1023u);
                const uint32_t ob = st_o0 + (uint32_t)(row * p + lane) * 4u;
#pragma unroll
                for (int k = 0; k < SMAX; ++k) {
                    const uint32_t o = k < SMAX - 1 ? ob + 256u * (uint32_t)k
                                                    : (tail_ok ? ob + 256u * (uint32_t)k : 0x80000000u);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][k]), rs, (int)o, 0, kStoreCpol);
                }
            }
        }
    }
}

// kPack2 merge step (p <= 32; units always with a blob): register row i of
// wave w holds two adjacent output rows, 2(w + 8i) in lanes 0-31 and
// 2(w + 8i) + 1 in lanes 32-63, bin j = lane & 31 (adjacent rows: the two
// halves of a read or write hit disjoint banks -- rows 8 apart, as before,
// collided on every bank at p = 16 or 32).  Every lane resolves its own row's
// descriptor (the two halves read different table words; lanes of a half
// read the same word) and computes its bin's wrapped indices itself: no
// v_readlane and no per-row scalar work, so a wave instruction does the
// work of two rows at the cost of one.  TWO: two levels per step, the
// additions of merge_level2_dense; otherwise one level (carried size-1 nodes
// add -0.0).  Rows past nrows and bins past p compute in-bounds garbage that
// is never written back.
template <int RW, bool TWO, bool FIRST>
__device__ __forceinline__ void merge_step_lanes(const UnitCtx& C, const float* src, int p, int lo, int lane, int wave,
                                                 int nrows, float (&v)[RW][1], const int* loff)
{
    // an opaque copy of the lane, so per-row addresses are not hoisted out of
    // the level loop into 2 x RW long-lived registers (spills)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    // bins past p read bin 0's words (a broadcast, no extra bank cycles)
    const int h = ln >> 5, j = (ln & 31) < p ? (ln & 31) : 0;
    const uint32_t* const desc = desc_table(C);
    const int dl = TWO ? 0 : desc_offset(C, lo);
    const uint2* const step = reinterpret_cast<const uint2*>(TWO ? slot_table(C, lo) : C.aux);
    const lds_cptr sp = (lds_cptr)src;
    // groups of G register rows without a branch between them, so the
    // descriptor chains (2-4 dependent LDS reads per row) of a group overlap
    constexpr int G = 4;
    auto rowidx = [&](int i) {
        const int r = 2 * (wave + kConeWaves * i) + h;
        return r < nrows ? r : nrows - 1;
    };
    // the next row's entry is read before this row's (volatile) data reads:
    // LDS reads complete in order, so a descriptor read issued after them
    // waited for all of them (lgkmcnt(0)) before its decode could start
    uint2 enext = make_uint2(0u, 0u);
    auto row = [&](int i, bool pre) {
        const int r = rowidx(i);
        if constexpr (TWO) {
            // the host-resolved row: source rows q0..q3 of level lo + 2, rolls
            const uint2 e = enext;
            if (pre) enext = step[rowidx(i + 1)];
            const uint32_t q0 = e.x & 1023u, q1 = (e.x >> 10) & 1023u, q2 = (e.x >> 20) & 1023u, q3 = e.y & 1023u;
            const int sH = (int)((e.y >> 10) & 63u), sh = (int)((e.y >> 16) & 63u), sTT = (int)((e.y >> 22) & 63u);
            const int o0 = FIRST ? loff[q0] : (int)__umul24(q0, (uint32_t)p);
            const int o1 = FIRST ? loff[q1] : (int)__umul24(q1, (uint32_t)p);
            const int o2 = FIRST ? loff[q2] : (int)__umul24(q2, (uint32_t)p);
            const int o3 = FIRST ? loff[q3] : (int)__umul24(q3, (uint32_t)p);
            // (j + s) mod p for j, s < p: min of the sum and the sum - p as
            // unsigned (the latter wraps to a huge value below p)
            uint32_t u1 = (uint32_t)(j + sH), u2 = (uint32_t)(j + sh), u3 = (uint32_t)(j + sTT);
            const int i1 = (int)min(u1, u1 - (uint32_t)p), i2 = (int)min(u2, u2 - (uint32_t)p);
            const int i3 = (int)min(u3, u3 - (uint32_t)p);
            const float x0 = lds_ld(sp + o0 + j);
            const float x1 = lds_ld(sp + o1 + i1);
            const float x2 = lds_ld(sp + o2 + i2);
            const float x3 = lds_ld(sp + o3 + i3);
            v[i][0] = __fadd_rn(__fadd_rn(x0, x1), __fadd_rn(x2, x3));
        } else {
            const uint32_t d = desc[dl + r];
            const uint32_t tc = (d >> 10) & 1023u;
            const bool car = tc == kCarried;
            const int sh = (int)(d >> 20);
            const int ho = FIRST ? loff[d & 1023u] : (int)__umul24(d & 1023u, (uint32_t)p);
            const int to = car ? ho : (FIRST ? loff[tc & 1023u] : (int)__umul24(tc, (uint32_t)p));
            const uint32_t u1 = (uint32_t)(j + sh);
            const int i1 = (int)min(u1, u1 - (uint32_t)p);
            const float x0 = lds_ld(sp + ho + j);
            float x1 = lds_ld(sp + to + i1);
            x1 = car ? -0.0f : x1;
            v[i][0] = __fadd_rn(x0, x1);
        }
    };
#pragma unroll
    for (int g = 0; g < RW; g += G) {
        if (2 * (wave + kConeWaves * g) < nrows) {
            const int ge = g + G < RW ? g + G : RW;
            if constexpr (TWO) enext = step[rowidx(g)];
#pragma unroll
            for (int i = g; i < ge; ++i) row(i, i + 1 < ge);
        }
    }
}

template <int RW>
__device__ __forceinline__ void write_rows_lanes(float* base, float* dummy, const float (&v)[RW][1], int p, int lane,
                                                 int wave, int nrows)
{
    // an opaque copy of the lane, so per-row addresses are not hoisted out of
    // the level loop into 2 x RW long-lived registers (spills)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int h = ln >> 5, j = ln & 31;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (2 * (wave + kConeWaves * i) < nrows) {
            const int r = 2 * (wave + kConeWaves * i) + h;
            *((r < nrows && j < p) ? base + (int)__umul24((uint32_t)r, (uint32_t)p) + j : dummy) = v[i][0];
        }
    }
}

template <int RW>
__device__ __forceinline__ void store_rows_lanes(const float (&v)[RW][1], int p, int lane, int wave, int nrows,
                                                 __amdgpu_buffer_rsrc_t rs, uint32_t st_o0)
{
    // an opaque copy of the lane, so per-row addresses are not hoisted out of
    // the level loop into 2 x RW long-lived registers (spills)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int h = ln >> 5, j = ln & 31;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (2 * (wave + kConeWaves * i) < nrows) {
            const int r = 2 * (wave + kConeWaves * i) + h;
            const uint32_t o = (r < nrows && j < p) ? st_o0 + (__umul24((uint32_t)r, (uint32_t)p) + (uint32_t)j) * 4u : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][0]), rs, (int)o, 0, 0);
        }
    }
}

// kPack2 rows of p >= 8 bins as (row, 8-bin segment) tasks, one per lane
// (merge_step_tasks): task t = tid + kConeBlock * i is row t / segs, segment
// t % segs, bins j0 .. j0 + 7 with j0 = min(8 * seg, p - 8) (the last
// segment of a row overlaps the one before it when 8 does not divide p:
// those bins are computed twice, identically, and written twice with the
// same value).  A lane resolves its row's entry once for its 8 bins, the
// head read is the row plus an immediate offset, and a rolled read picks one
// of two bases (before / after the wrap point) per bin: a third of the VALU
// of the lane-per-bin layout, where every lane decoded its row's entry and
// wrapped its own index.  Tasks past the level's rows redo the last task
// (same values, same addresses).  Levels above the fill at the odd stride
// qs = p | 1 (the 32-lane halves of a read or write then hit distinct banks
// for distinct rows).
constexpr int kPackSeg = 8;
constexpr int kPackTasks = 3;                 // tasks per lane: kMaxRows rows x 4 segments
static_assert(kMaxRows * 4 <= kPackTasks * kConeBlock, "short-row tasks per lane");
RT_HD inline int pack_segments(int p) { return (p + kPackSeg - 1) / kPackSeg; }

// task -> (row, first bin); segs in 1..4, t < 2^11
__device__ __forceinline__ void pack_task(int t, int segs, int p, int& r, int& j0)
{
    const uint32_t m = segs == 1 ? (1u << 20) : (segs == 2 ? (1u << 19) : (segs == 3 ? 349526u : (1u << 18)));
    r = (int)(__umul24((uint32_t)t, m) >> 20);
    j0 = min((t - r * segs) * kPackSeg, p - kPackSeg);
}

// The same from the short-row roll table: entry x = j0 + s
// (x < 2p <= 64) holds the byte offsets 4 ((x + e) mod p) of the segment's
// eight elements as bytes: one conflict-free ds_read_b64 per rolled segment,
// then one address add per element (byte select) instead of a compare and a
// select.  Same LDS words: bit-exact.  The table lives in the metadata area,
// which short-row units do not use (their blob is in their level buffer).
__device__ __forceinline__ void pack_rolled_lut(lds_cptr sp, int o, unsigned long long e, float (&x)[kPackSeg])
{
    const lds_ccptr rb = (lds_ccptr)(sp + o);
    const uint32_t e0 = (uint32_t)e, e1 = (uint32_t)(e >> 32);
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = lds_ld((lds_cptr)(rb + ((e0 >> (8 * k)) & 0xFFu)));
#pragma unroll
    for (int k = 0; k < 4; ++k) x[4 + k] = lds_ld((lds_cptr)(rb + ((e1 >> (8 * k)) & 0xFFu)));
}

// Interleaved short-row tasks (SEGS = segs >= 2, every step whose output
// stays in LDS): lane (row, segment s) takes bins s + SEGS * k, k < 8, so the
// segs lanes of a row read consecutive words of each source row (shared
// words broadcast) and a 32-lane group of a read touches few distinct rows'
// words per bank; with the per-p strides of pack_stride the steps' reads run
// at 1.05-1.34 x the conflict-free LDS cycles instead of 1.08-2.25 x (host
// simulation of the cfg4 schedule).  Bins past p (8 * SEGS > p) are computed
// from in-bounds words and written into the row's padding (pack_stride >=
// 8 * SEGS): never read as data.  The interleaved roll table at
// kPackLutI: entry x = s + roll (x < p + SEGS) holds the byte offsets
// 4 ((x + SEGS * e) mod p), e < 8.  The HBM-bound last step of a merge-only
// pass keeps the contiguous tasks (16-byte stores).
constexpr int kPackLutI = 128;                // word offset: past the contiguous table's 4p <= 128 words
static_assert(kPackLutI + 2 * (32 + 4) <= kAuxWords, "short-row roll tables");

__device__ __forceinline__ void build_pack_lut(uint32_t* lut, int p, int tid)
{
    for (int w = tid; w < 4 * p; w += kConeBlock) {
        const int x = (w >> 1) + 4 * (w & 1);
        uint32_t word = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            int y = x + i;                        // < 2p + 8 <= 3p (p >= 8)
            y -= y >= p ? p : 0;
            y -= y >= p ? p : 0;
            word |= (uint32_t)(4 * y) << (8 * i);
        }
        lut[w] = word;
    }
    const int segs = pack_segments(p);
    if (segs >= 2)
        for (int w = tid; w < 2 * (p + segs); w += kConeBlock) {
            const int x = w >> 1, e0 = 4 * (w & 1);
            uint32_t word = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int y = x + segs * (e0 + i);      // < p + 8 segs <= 2p + 7 < 3p
                y -= y >= p ? p : 0;
                y -= y >= p ? p : 0;
                word |= (uint32_t)(4 * y) << (8 * i);
            }
            lut[kPackLutI + w] = word;
        }
}

// task -> (row, segment) of the interleaved layout
template <int SEGS>
__device__ __forceinline__ void pack_task_i(int t, int& r, int& seg)
{
    r = t / SEGS;
    seg = t - r * SEGS;
}

// SEGS = 0: contiguous tasks; SEGS = segs >= 2: interleaved tasks
template <bool TWO, bool FIRST, int SEGS>
__device__ __forceinline__ void merge_step_tasks(const UnitCtx& C, const float* src, int p, int qs, int lo, int tid,
                                                 int nrows, float (&v)[kPackTasks][kPackSeg], const int* loff)
{
    const lut_cptr plut = (lut_cptr)(C.aux0 + (SEGS ? kPackLutI : 0));
    const int segs = SEGS ? SEGS : pack_segments(p);
    constexpr int ES = SEGS ? SEGS : 1;           // word stride of a task's bins
    const int ntask = nrows * segs;
    const uint32_t* const desc = desc_table(C);
    const int dl = TWO ? 0 : desc_offset(C, lo);
    const uint2* const step = reinterpret_cast<const uint2*>(TWO ? slot_table(C, lo) : C.aux);
    const lds_cptr sp = (lds_cptr)src;
    // waves whose tasks all lie past the level skip the block (per wave:
    // a partly filled block would otherwise run every wave)
    const int wave0 = tid & ~63;
#pragma unroll
    for (int i = 0; i < kPackTasks; ++i) {
        if (kConeBlock * i + wave0 < ntask) {
            int r, j0;
            if constexpr (SEGS) pack_task_i<SEGS>(min(tid + kConeBlock * i, ntask - 1), r, j0);   // j0: the segment
            else pack_task(min(tid + kConeBlock * i, ntask - 1), segs, p, r, j0);
            float x0[kPackSeg], x1[kPackSeg];
            if constexpr (TWO) {
                // the host-resolved row: source rows q0..q3 of level lo + 2, rolls
                const uint2 e = step[r];
                const uint32_t q0 = e.x & 1023u, q1 = (e.x >> 10) & 1023u, q2 = (e.x >> 20) & 1023u, q3 = e.y & 1023u;
                const int sH = (int)((e.y >> 10) & 63u), sh = (int)((e.y >> 16) & 63u), sTT = (int)((e.y >> 22) & 63u);
                const int o0 = FIRST ? loff[q0] : (int)__umul24(q0, (uint32_t)qs);
                const int o1 = FIRST ? loff[q1] : (int)__umul24(q1, (uint32_t)qs);
                const int o2 = FIRST ? loff[q2] : (int)__umul24(q2, (uint32_t)qs);
                const int o3 = FIRST ? loff[q3] : (int)__umul24(q3, (uint32_t)qs);
                float x2[kPackSeg], x3[kPackSeg];
                const lds_cptr h0 = sp + o0 + j0;
                // table entries first (plain loads), then the volatile reads
                const unsigned long long e1 = plut[j0 + sH], e2 = plut[j0 + sh], e3 = plut[j0 + sTT];
#pragma unroll
                for (int k = 0; k < kPackSeg; ++k) x0[k] = lds_ld(h0 + ES * k);
                pack_rolled_lut(sp, o1, e1, x1);
                pack_rolled_lut(sp, o2, e2, x2);
                pack_rolled_lut(sp, o3, e3, x3);
#pragma unroll
                for (int k = 0; k < kPackSeg; ++k) v[i][k] = __fadd_rn(__fadd_rn(x0[k], x1[k]), __fadd_rn(x2[k], x3[k]));
            } else {
                const uint32_t d = desc[dl + r];
                const uint32_t tc = (d >> 10) & 1023u;
                const bool car = tc == kCarried;
                const int sh = (int)(d >> 20);
                const int ho = FIRST ? loff[d & 1023u] : (int)__umul24(d & 1023u, (uint32_t)qs);
                const int to = car ? ho : (FIRST ? loff[tc & 1023u] : (int)__umul24(tc, (uint32_t)qs));
                const lds_cptr h0 = sp + ho + j0;
                const unsigned long long e1 = plut[j0 + (car ? 0 : sh)];
#pragma unroll
                for (int k = 0; k < kPackSeg; ++k) x0[k] = lds_ld(h0 + ES * k);
                pack_rolled_lut(sp, to, e1, x1);
                // a carried size-1 node adds -0.0 (x + (-0.0) == x: the reference's copy)
#pragma unroll
                for (int k = 0; k < kPackSeg; ++k) v[i][k] = __fadd_rn(x0[k], car ? -0.0f : x1[k]);
            }
        }
    }
}

// short-row tasks stored to HBM with 16-byte stores: a wave instruction
// writes 1 KiB of contiguous rows instead of 64 words 8 apart.  A/B, same
// box, cone ms per cfg4 trial (profiles/r03zi_ab_cfg4.log): 0.771 / 0.772
// with eight 4-byte stores per task, 0.679 / 0.679 with two 16-byte ones,
// S/N identical.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <bool GLOBAL, int SEGS>
__device__ __forceinline__ void put_tasks(float* base, int q, const float (&v)[kPackTasks][kPackSeg], int p, int tid,
                                          int nrows, __amdgpu_buffer_rsrc_t rs, uint32_t st_o0)
{
    static_assert(!(GLOBAL && SEGS), "HBM stores take the contiguous tasks");
    const int segs = SEGS ? SEGS : pack_segments(p);
    constexpr int ES = SEGS ? SEGS : 1;
    const int ntask = nrows * segs;
    const int wave0 = tid & ~63;
#pragma unroll
    for (int i = 0; i < kPackTasks; ++i) {
        if (kConeBlock * i + wave0 < ntask) {
            int r, j0;
            if constexpr (SEGS) pack_task_i<SEGS>(min(tid + kConeBlock * i, ntask - 1), r, j0);
            else pack_task(min(tid + kConeBlock * i, ntask - 1), segs, p, r, j0);
            if constexpr (GLOBAL) {
                const uint32_t ob = st_o0 + (uint32_t)(r * p + j0) * 4u;
                // the task's 8 bins as two 16-byte stores (dword-aligned
                // multi-dword buffer stores)
#pragma unroll
                for (int k = 0; k < kPackSeg; k += 4) {
                    const v4u w = {__float_as_uint(v[i][k]), __float_as_uint(v[i][k + 1]),
                                   __float_as_uint(v[i][k + 2]), __float_as_uint(v[i][k + 3])};
                    __builtin_amdgcn_raw_buffer_store_b128(w, rs, (int)(ob + 4u * k), 0, 0);
                }
            } else {
                float* const o = base + r * q + j0;
#pragma unroll
                for (int k = 0; k < kPackSeg; ++k) o[ES * k] = v[i][k];
            }
        }
    }
}

// All merge levels of one unit, deepest first, in place in the dense rows
// at `base`.  SMAX >= ceil(p/64) slots per row, RW rows per wave
// (lds_row_capacity(p, SMAX) guarantees ceil(rows/8) <= RW at every level).
// Each level's outputs are staged in registers between two barriers, then
// written back.  With `st` set (a non-final pass), the output level goes from
// the staging registers straight to global memory instead of back into LDS.
// pre_store(): called by every wave after the last merge step's LDS reads
// and before its output level is stored from registers (st): the level
// buffer is then free for the next trial's fill.  A final pass's output
// level (row-slot steps) starts oshift floats past base.
template <int SMAX, int RW, class PreStore>
__device__ __forceinline__ void merge_levels(const UnitCtx& C, float* base, int p, int L, int tid, bool st,
                                             __amdgpu_buffer_rsrc_t rs, uint32_t st_o0, uint32_t flags, float* dummy,
                                             int qout, int oshift, PreStore&& pre_store)
{
    const int lane = tid & 63, wave = tid >> 6;
    const bool tile = C.tile;
    const int node_size = C.U.node_size;
    // the first step reads the bottom level in its fill layout: through the
    // blob's bottom-row offsets, or (whole unit without a blob) as dense rows
    // at the block's 16-byte phase; every later level is dense rows (stride
    // p) at base
    const int* const loff = C.table ? bottom_offsets(C) : nullptr;
    float* const src0 = C.table ? base : base + C.al;
    // deepest first; two levels per step (merge_level2_dense) once no level
    // below the step's output holds size-1 nodes, single steps before that
    // and for a last odd level
    const bool fuse = (flags & kConeFuse2) != 0;
    if constexpr (SMAX == kPack2) {
        if (p >= kPackSeg) {
            const int qs = pack_stride(p);
            for (int l = L - 1; l >= 0;) {
                const bool two = fuse && l >= 1 && (tile || (node_size >> l) >= 2);
                const int lo = two ? l - 1 : l;
                const int nrows = rows_at(C, lo);
                float v[kPackTasks][kPackSeg];
                const bool first = l == L - 1;
                const float* src = first ? src0 : base;
                // interleaved tasks unless the step's output goes to HBM
                const int segs = pack_segments(p);
                const int inter = (segs >= 2 && !(lo == 0 && st)) ? segs : 0;
                auto step = [&](auto sc) {
                    constexpr int S = decltype(sc)::value;
                    if (first) {
                        if (two) merge_step_tasks<true, true, S>(C, src, p, qs, lo, tid, nrows, v, loff);
                        else merge_step_tasks<false, true, S>(C, src, p, qs, lo, tid, nrows, v, loff);
                    } else {
                        if (two) merge_step_tasks<true, false, S>(C, src, p, qs, lo, tid, nrows, v, nullptr);
                        else merge_step_tasks<false, false, S>(C, src, p, qs, lo, tid, nrows, v, nullptr);
                    }
                };
                if (inter == 2) step(IntC<2>{});
                else if (inter == 3) step(IntC<3>{});
                else if (inter == 4) step(IntC<4>{});
                else step(IntC<0>{});
                l = lo - 1;
                if (lo == 0 && st) {
                    pre_store();
                    put_tasks<true, 0>(base, qs, v, p, tid, nrows, rs, st_o0);
                    return;
                }
                if (!(flags & kConeDiagNoBarrier)) lds_barrier();
                // the output level (lo == 0) at the caller's stride qout
                if (!(flags & kConeDiagNoWrite)) {
                    const int qw = lo == 0 ? qout : qs;
                    if (inter == 2) put_tasks<false, 2>(base, qw, v, p, tid, nrows, rs, st_o0);
                    else if (inter == 3) put_tasks<false, 3>(base, qw, v, p, tid, nrows, rs, st_o0);
                    else if (inter == 4) put_tasks<false, 4>(base, qw, v, p, tid, nrows, rs, st_o0);
                    else put_tasks<false, 0>(base, qw, v, p, tid, nrows, rs, st_o0);
                }
                if (!(flags & kConeDiagNoBarrier)) lds_barrier();
            }
            return;
        }
        for (int l = L - 1; l >= 0;) {
            const bool two = fuse && l >= 1 && (tile || (node_size >> l) >= 2);
            const int lo = two ? l - 1 : l;
            const int nrows = rows_at(C, lo);
            float v[RW][1];
            const bool first = l == L - 1;
            const float* src = first ? src0 : base;
            const int* lo_src = first ? loff : nullptr;
            if (first) {
                if (two) merge_step_lanes<RW, true, true>(C, src, p, lo, lane, wave, nrows, v, lo_src);
                else merge_step_lanes<RW, false, true>(C, src, p, lo, lane, wave, nrows, v, lo_src);
            } else {
                if (two) merge_step_lanes<RW, true, false>(C, src, p, lo, lane, wave, nrows, v, lo_src);
                else merge_step_lanes<RW, false, false>(C, src, p, lo, lane, wave, nrows, v, lo_src);
            }
            l = lo - 1;
            if (lo == 0 && st) {
                pre_store();
                store_rows_lanes<RW>(v, p, lane, wave, nrows, rs, st_o0);
                return;
            }
            if (!(flags & kConeDiagNoBarrier)) lds_barrier();
            if (!(flags & kConeDiagNoWrite)) write_rows_lanes<RW>(base, dummy, v, p, lane, wave, nrows);
            if (!(flags & kConeDiagNoBarrier)) lds_barrier();
        }
        return;
    }
    if constexpr (SMAX <= 5) {
        // the 4/5-slot instances (p = 193-320) run only row-slot steps: every
        // unit of theirs carries slot tables (validate_exec_plan; unit_begin
        // refuses a unit without them), so the dense per-level paths below are
        // compiled out of these, the hottest instances
        if (resolved_slots(SMAX) || (C.slots && fuse)) {
            // row-slot steps (the host's slot tables follow this step order;
            // a unit with a zero row fuses every step)
            const bool all2 = C.U.zero_row != 0;
            for (int l = L - 1; l >= 0;) {
                const bool two = l >= 1 && (tile || all2 || (node_size >> l) >= 2);
                const int lo = two ? l - 1 : l;
                float v[RW][SMAX];
                const bool first = l == L - 1;
                const float* src = first ? src0 : base;
                const int* lo_src = first ? loff : nullptr;
                uint32_t sw;
                int nq;
                if (two) merge_step_slots<SMAX, RW, true>(C, src, p, lo, lane, wave, v, lo_src, sw, nq);
                else merge_step_slots<SMAX, RW, false>(C, src, p, lo, lane, wave, v, lo_src, sw, nq);
                l = lo - 1;
                if (lo == 0 && st) {
                    pre_store();
                    store_rows_slots<SMAX, RW>(v, p, lane, sw, nq, rs, st_o0);
                    return;
                }
                if (!(flags & kConeDiagNoBarrier)) lds_barrier();
                // the output level of a final pass at row stride qout (the S/N's)
                if (!(flags & kConeDiagNoWrite))
                    write_rows_slots<SMAX, RW>(lo == 0 ? base + oshift : base, dummy, v, p, lane, sw, nq,
                                               lo == 0 ? qout : p);
                if (!(flags & kConeDiagNoBarrier)) lds_barrier();
            }
            return;
        }
    }
    if constexpr (!resolved_slots(SMAX)) {
    for (int l = L - 1; l >= 0;) {
        // size-1 nodes exist at depth l only in whole units with node_size >> l < 2
        const bool two = fuse && l >= 1 && (tile || (node_size >> l) >= 2);
        const int lo = two ? l - 1 : l;          // output level of this step
        const int orows = rows_at(C, lo);
        const int nr = uni(orows > wave ? (orows - wave + kConeWaves - 1) / kConeWaves : 0);
        constexpr int S = slot_count(SMAX);
        float v[RW][S];
        const bool carried = !tile && (node_size >> l) < 2;
        const bool first = l == L - 1;
        const float* src = first ? src0 : base;
        const int* lo_src = first ? loff : nullptr;
        if (two)
            merge_level2_dense<S, RW>(C, src, p, lo, lane, wave, nr, v, lo_src);
        else if (carried)
            merge_level_dense<S, RW, true>(C, src, p, l, lane, wave, nr, v, lo_src);
        else
            merge_level_dense<S, RW, false>(C, src, p, l, lane, wave, nr, v, lo_src);
        l = lo - 1;
        if (lo == 0 && st) {
            pre_store();
            store_rows<S, RW>(v, p, lane, wave, nr, rs, st_o0);
            return;
        }
        if (!(flags & kConeDiagNoBarrier)) lds_barrier();
        if (!(flags & kConeDiagNoWrite)) {
            write_rows<S, RW>(base, dummy, v, p, lane, wave, nr);
        }
        if (!(flags & kConeDiagNoBarrier)) lds_barrier();
    }
    }
}

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v)
{
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

// row_shr:d within 16-lane rows: lane g (of a G-lane group, G <= 16) takes
// lane g - d of its group when g >= d.
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d_rows(double v)
{
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Inclusive scan over each G-lane group (G = 2 .. 64): row_shr steps inside
// 16-lane rows, then row_bcast:15 / row_bcast:31 across rows.  The partial
// sums start at +0.0 and are never -0.0, so adding the +0.0 that masked
// lanes receive is an exact no-op.
template <int G>
__device__ __forceinline__ double seg_scan_dpp(double v, int lane)
{
    const int g = lane & (G < 16 ? G - 1 : 15);     // position inside the group's part of the 16-lane row
    double y = dpp_d<0x111>(v);
    v = g >= 1 ? v + y : v;
    if (G >= 4) {
        y = dpp_d<0x112>(v);
        v = g >= 2 ? v + y : v;
    }
    if (G >= 8) {
        y = dpp_d<0x114>(v);
        v = g >= 4 ? v + y : v;
    }
    if (G >= 16) {
        y = dpp_d<0x118>(v);
        v = g >= 8 ? v + y : v;
    }
    if (G >= 32) v = v + dpp_d_rows<0x142, 0xA>(v);   // rows 1, 3 += lane 15 of rows 0, 2
    if (G >= 64) v = v + dpp_d_rows<0x143, 0xC>(v);   // rows 2, 3 += lane 31
    return v;
}

// diff_max (kernels.hpp:50-60) of width W over the lane's columns (cp[i] =
// +inf past the lane's chunk, so those differences are -inf).
// v_sub_f32 / v_max3_f32 as volatile asm: the width's work stays inside its
// switch case (from plain code the compiler evaluated every case -- all
// kSnrWin widths -- ahead of the width loop in every row pass).  v_max3_f32
// (IEEE mode) never returns a quiet-NaN operand over a number, as diff_max's
// comparison (kernels.hpp:50-60).
template <int CH, int W>
__device__ __forceinline__ float window_max(const float (&z)[CH + kSnrWin], const float (&cp)[CH])
{
    float dm = -INFINITY;
#pragma unroll
    for (int i = 0; i + 1 < CH; i += 2) {
        float t0, t1;
        asm volatile("v_sub_f32 %1, %3, %4\n\tv_sub_f32 %2, %5, %6\n\tv_max3_f32 %0, %0, %1, %2"
                     : "+v"(dm), "=&v"(t0), "=&v"(t1)
                     : "v"(z[i + W]), "v"(cp[i]), "v"(z[i + 1 + W]), "v"(cp[i + 1]));
    }
    if constexpr (CH & 1) {
        float t0;
        asm volatile("v_sub_f32 %1, %2, %3\n\tv_max_f32 %0, %0, %1"
                     : "+v"(dm), "=&v"(t0)
                     : "v"(z[CH - 1 + W]), "v"(cp[CH - 1]));
    }
    return dm;
}

// width dispatch: one switch (a jump, not a chain of scalar compares)
template <int CH>
__device__ __forceinline__ float window_dispatch(int w, const float (&z)[CH + kSnrWin], const float (&cp)[CH])
{
    static_assert(kSnrWin == 12, "cases below");
    switch (w) {
    case 1: return window_max<CH, 1>(z, cp);
    case 2: return window_max<CH, 2>(z, cp);
    case 3: return window_max<CH, 3>(z, cp);
    case 4: return window_max<CH, 4>(z, cp);
    case 5: return window_max<CH, 5>(z, cp);
    case 6: return window_max<CH, 6>(z, cp);
    case 7: return window_max<CH, 7>(z, cp);
    case 8: return window_max<CH, 8>(z, cp);
    case 9: return window_max<CH, 9>(z, cp);
    case 10: return window_max<CH, 10>(z, cp);
    case 11: return window_max<CH, 11>(z, cp);
    case 12: return window_max<CH, 12>(z, cp);
    default: return -INFINITY;
    }
}

// The standard ladder of small boxcar widths: generate_width_trials
// (ffautils.py:3-10) with wtsp 1.5 always starts 1, 2, 3, 4, 6, 9 (every
// BASELINE config: W = 6 or 10 from 240 bins).  When a plan's widths begin
// with it, the S/N evaluates those six window maxima in one straight block
// (independent v_max3 chains the compiler may interleave, no width switch,
// one interleaved DPP all-reduce), instead of one switch case and one
// all-reduce per width.  Same float operations, same results.
constexpr int kStdWidths[6] = {1, 2, 3, 4, 6, 9};

template <int CH, int W>
__device__ __forceinline__ float window_max_nv(const float (&z)[CH + kSnrWin], const float (&cp)[CH])
{
    // diff_max (kernels.hpp:50-60) as window_max, without volatile: the six
    // widths' chains are independent and may be interleaved
    float dm = -INFINITY;
#pragma unroll
    for (int i = 0; i + 1 < CH; i += 2) {
        float t0, t1;
        asm("v_sub_f32 %1, %3, %4\n\tv_sub_f32 %2, %5, %6\n\tv_max3_f32 %0, %0, %1, %2"
            : "+v"(dm), "=&v"(t0), "=&v"(t1)
            : "v"(z[i + W]), "v"(cp[i]), "v"(z[i + 1 + W]), "v"(cp[i + 1]));
    }
    if constexpr (CH & 1) {
        float t0;
        asm("v_sub_f32 %1, %2, %3\n\tv_max_f32 %0, %0, %1" : "+v"(dm), "=&v"(t0) : "v"(z[CH - 1 + W]), "v"(cp[CH - 1]));
    }
    return dm;
}

// one v_max_f32 with a DPP source per value and step, six values interleaved
// (each DPP reads a register written six instructions earlier: no wait states)
#define RT_MAX6_STEP(CTRL)                                                                                  \
    asm volatile("v_max_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %4, %4, %4 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %5, %5, %5 " CTRL " row_mask:0xf bank_mask:0xf"                              \
                 : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]), "+v"(m[3]), "+v"(m[4]), "+v"(m[5]))

// The six standard widths' row maxima all-reduced over each G-lane group
// (grp_allmax for six values at once); lane g of a group then keeps width g.
template <int CH, int G>
__device__ __forceinline__ float snr_std6(const float (&z)[CH + kSnrWin], const float (&cp)[CH], int g)
{
    static_assert(G == 8 || G == 16, "one DPP row per group");
    float m[6] = {window_max_nv<CH, 1>(z, cp), window_max_nv<CH, 2>(z, cp), window_max_nv<CH, 3>(z, cp),
                  window_max_nv<CH, 4>(z, cp), window_max_nv<CH, 6>(z, cp), window_max_nv<CH, 9>(z, cp)};
    asm volatile("s_nop 1" ::: "memory");
    RT_MAX6_STEP("quad_perm:[1,0,3,2]");
    RT_MAX6_STEP("quad_perm:[2,3,0,1]");
    RT_MAX6_STEP("row_half_mirror");
    if constexpr (G >= 16) RT_MAX6_STEP("row_mirror");
    float r = m[0];
#pragma unroll
    for (int i = 1; i < 6; ++i) r = g == i ? m[i] : r;
    return r;
}
#undef RT_MAX6_STEP

// The short rows' standard ladder 1, 2, 3 (generate_width_trials from 16-32
// bins: BASELINE configs[3]) in 4-lane groups: three independent window
// maxima and one interleaved quad all-reduce (each DPP reads a register
// written three instructions earlier), instead of a width switch and an
// all-reduce with its wait states per width.  Same float operations.
#define RT_MAX3_STEP(CTRL)                                                                                  \
    asm volatile("v_max_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf\n\t"                        \
                 "v_max_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf"                              \
                 : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]))

template <int CH>
__device__ __forceinline__ float snr_std3(const float (&z)[CH + kSnrWin], const float (&cp)[CH], int g)
{
    float m[3] = {window_max_nv<CH, 1>(z, cp), window_max_nv<CH, 2>(z, cp), window_max_nv<CH, 3>(z, cp)};
    asm volatile("s_nop 1" ::: "memory");
    RT_MAX3_STEP("quad_perm:[1,0,3,2]");
    RT_MAX3_STEP("quad_perm:[2,3,0,1]");
    return g == 0 ? m[0] : (g == 1 ? m[1] : m[2]);
}
#undef RT_MAX3_STEP


#ifdef RT_STAMPS
#define RT_SNR_MARK(i)                                                           \
    do {                                                                         \
        if (tid == 0 && base == 0 && tl) tl[i] = __builtin_amdgcn_s_memtime();   \
    } while (0)
#else
#define RT_SNR_MARK(i) do { } while (0)
#endif

// Per-width constants of the S/N formula (snr.hpp:37-65): h + b and b of
// width w over p bins.
__device__ __forceinline__ void snr_width_consts(int w, int p, float* out)
{
    const float h = sqrtf((float)(p - w) / (float)(p * w));
    const float b = (float)w / (float)(p - w) * h;
    out[0] = h + b;
    out[1] = b;
}

// max over each G-lane group (G = 2 .. 64, groups aligned), in every lane
// of the group: quad swaps, then the half-row and row mirrors, then (G >= 32)
// cross-row exchanges (max never returns a NaN operand over a number, as
// diff_max's comparison)
template <int G>
__device__ __forceinline__ float grp_allmax(float v)
{
    static_assert(G == 2 || G == 4 || G == 8 || G == 16 || G == 32 || G == 64, "lane groups");
    // v_max_f32 with a DPP source (no canonicalising moves around a
    // separate DPP move); s_nop 1: the DPP read of a VGPR written by the
    // previous VALU instruction
    asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(v));
    if constexpr (G >= 4)
        asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(v));
    if constexpr (G >= 8)
        asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf" : "+v"(v));
    if constexpr (G >= 16)
        asm volatile("s_nop 1\n\tv_max_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(v));
    // 32- and 64-lane groups: lane i <-> i ^ 16 by ds_swizzle (xor mask 16
    // inside 32 lanes), lane i <-> i ^ 32 by ds_bpermute
    if constexpr (G >= 32) v = fmaxf(v, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x401F)));
    if constexpr (G == 64) v = fmaxf(v, __shfl_xor(v, 32, 64));
    return v;
}

// Fused boxcar S/N (snr.hpp:37-65) of the output rows s < rows_eval held in
// LDS (row stride q): G lanes per row, each lane a chunk of c <= CH columns
// held in registers (c odd: the G chunks of a row start on distinct banks).
// fp64 prefix: sequential in the chunk + log2(G)-step segmented scan
// (kernels.hpp:73-86).  For G <= 16 (one DPP row) the scan and the width
// maxima's all-reduce run on DPP row shifts (VALU, no LDS round trip); each
// lane then reads its window c[j0 .. j0 + CH + kSnrWin) (the wrap c[p + j] =
// c[j] + sum applied once per element) and evaluates every width w <= kSnrWin
// from registers.  Wider widths read LDS per width.  Transposed emit: the
// row's max of width iw goes to every lane of its group (DPP all-reduce) and
// lane g keeps widths g, g + G, ...; one S/N formula (one fp32 division) and
// one store per lane and slot after the widths, the stores of a row
// consecutive.  Row passes without workgroup barriers: a row's G <= 64 lanes
// are one wave, and a wave's LDS accesses complete in order.
// (kSnrWin, kSnrMaxChunk: common.hpp)
template <int CH, int G, bool WIDE = false>
__device__ __forceinline__ void snr_rows(const ConeArgs& a, const UnitView& U, float* data, int q, const int* wl,
                                         int nev, int c, int tid, const float* whb, unsigned long long* tl)
{
    const int lane = tid & 63;
    const int p = U.p;
    const int g = lane & (G - 1);
    // rows with room for the wrapped prefix extension (final-pass output
    // levels at the S/N stride); only the register-window path uses it
    const bool ext = CH <= kSnrMaxChunk && q >= p + kSnrWin;
    // WIDE (the caller checked snr_wide_ok): every width past the register
    // window read as a plain LDS window, the wrapped prefix stored up to
    // p + wmax
    const int next = WIDE ? wl[kMaxWidths] : kSnrWin;   // wrapped prefix words stored past p
    // rows with room past p for a lane's whole CH-column prefix write
    const bool wfull = q >= p + CH;
    // lanes past the row keep their natural chunk start g * c (their
    // columns are masked) where the row stride holds every lane's chunk:
    // clamped to p they read the banks of another row's lane (a 2-way
    // conflict on every chunk and window read at p = 240-254)
    const bool natural = ext && wfull && (G - 1) * c + CH <= q;
    int j0 = natural ? g * c : min(g * c, p);
    int cnt = max(min(j0 + c, p) - j0, 0);        // columns of this lane (may be 0)
    const int owner = (p - 1) / c;
    constexpr int rows_per_pass = kConeBlock / G;
    constexpr int writer = G - 1;
    (void)writer;
    const uint32_t nw = a.num_widths;
    float* snr = a.snr + (uint64_t)U.trial * a.snr_stride + (U.snr_row + (uint64_t)U.s0) * (uint64_t)nw;
    const __amdgpu_buffer_rsrc_t srs = buffer_rsrc(snr, (uint32_t)nev * nw * 4u);
    // the widths in lanes (lane i: width i), taken per width by v_readlane
    // instead of an LDS read and its wait
    const int wlane = wl[min(lane, (int)nw - 1)];
    // the plan's widths begin with the standard ladder 1, 2, 3, 4, 6, 9
    bool std6 = nw >= 6;
#pragma unroll
    for (int i = 0; i < 6; ++i) std6 = std6 && __builtin_amdgcn_readlane(wlane, i) == kStdWidths[i];
    // ... or begin 1, 2, 3 in 4-lane groups (short rows)
    bool std3 = G == 4 && nw >= 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) std3 = std3 && __builtin_amdgcn_readlane(wlane, i) == kStdWidths[i];
    for (int base = 0; base < nev; base += rows_per_pass) {
        // opaque per row pass: the column masks (i < cnt, j0 + k >= p) are
        // recomputed by one v_cmp each instead of being hoisted out of the
        // loop into SGPR pairs that spill (two v_readlane per use)
        asm volatile("" : "+v"(j0), "+v"(cnt));
        const int r = base + (tid / G);
        const bool active = r < nev;
        float* const row = data + min(r, nev - 1) * q + j0;
        float cp[CH];
        // every lane reads CH columns at immediate offsets (past its chunk:
        // the next chunk, the next row or the LDS pad), masked to 0
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const float x = row[i];
            cp[i] = i < cnt ? x : 0.0f;
            // the select on the float, before the fp64 conversion (else two
            // selects on the converted halves)
            asm("" : "+v"(cp[i]));
        }
        // fp64 prefix: the masked columns add +0.0 (the partial sums start at
        // +0.0 and are never -0.0, so the additions are exact no-ops)
        double part = 0.0;
#pragma unroll
        for (int i = 0; i < CH; ++i) part = part + (double)cp[i];
        double acc = dpp_d<0x138>(seg_scan_dpp<G>(part, lane));   // wave_shr:1 -- lane g takes lane g - 1
        if (g == 0) acc = 0.0;
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            acc = acc + (double)cp[i];
            cp[i] = (float)acc;
        }
        const float sum = __shfl((float)acc, owner, G);
        {
            // columns past the lane's chunk (and rows past nev) go to dummy
            // words in the LDS pad: a base select per column (the column an
            // immediate offset) instead of exec masks
            typedef __attribute__((address_space(3))) float* lds_ptr;
            if (wfull) {
                // every lane of an active row writes all CH columns, last
                // column first: a column past the lane's chunk is the next
                // lane's column i - c, which that lane writes later (a
                // wave's LDS writes land in order), or lies past the row
                // inside its stride (q >= p + CH)
                if (active) {
                    // volatile: the compiler keeps the descending order
                    volatile __attribute__((address_space(3))) float* const rk =
                        (volatile __attribute__((address_space(3))) float*)row;
#pragma unroll
                    for (int i = CH - 1; i >= 0; --i) rk[i] = cp[i];
                }
            } else {
                // one dummy word per lane and column (the same word for
                // every lane serialised those stores on one bank)
                const lds_ptr dummy = (lds_ptr)(data + kLdsDataFloats + 4 + lane);
                int cw = active ? cnt : 0;
                asm("" : "+v"(cw));
                const lds_ptr rk = (lds_ptr)row;
#pragma unroll
                for (int i = 0; i < CH; ++i) {
                    lds_ptr b = i < cw ? rk : dummy;
                    asm("" : "+v"(b));
                    b[i] = cp[i];
                }
            }
        }
        // rows at a stride q >= p + kSnrWin: the wrapped prefix c[p + j] =
        // c[j] + sum (kernels.hpp:88-97, j < kSnrWin, or j < wmax on the wide
        // stride) stored after the row by its own lanes (the wave's LDS
        // accesses complete in order), so the window reads below take
        // c[j0 .. j0 + CH + kSnrWin) -- and c[j0 + w ..] -- without a wrap
        const float* const crow = data + min(r, nev - 1) * q;
        if (ext) {
            float* const rb = data + min(r, nev - 1) * q;
            auto put = [&](int e) {
                if (active && e < next)
                    *(volatile __attribute__((address_space(3))) float*)(rb + p + e) =
                        __fadd_rn(lds_ld((lds_cptr)(rb + e)), sum);
            };
            if constexpr (WIDE) {
                for (int e0 = 0; e0 < next; e0 += G) put(e0 + g);
            } else {
#pragma unroll
                for (int e0 = 0; e0 < kSnrWin; e0 += G) put(e0 + g);
            }
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) cp[i] = i < cnt ? cp[i] : INFINITY;
        RT_SNR_MARK(7);
        // a row's lanes are one wave: its prefix writes are seen by its
        // window reads below without a workgroup barrier (a compiler barrier
        // only), so the waves of a unit run their row passes independently
        __asm__ __volatile__("" ::: "memory");
        RT_SNR_MARK(8);
        constexpr int NSEL = (kMaxWidths + G - 1) / G;
        float sel[NSEL] = {};
        auto emit = [&](uint32_t iw, float dmax) {
            const float dm = grp_allmax<G>(dmax);
#pragma unroll
            for (int sl = 0; sl < NSEL; ++sl)
                if (sl * G < (int)nw) sel[sl] = (int)iw == g + sl * G ? dm : sel[sl];
        };
        if constexpr (CH <= kSnrMaxChunk) {
            // widths <= kSnrWin from the register window c[j0 .. j0 + CH + kSnrWin)
            float z[CH + kSnrWin];
            // two opaque bases (row and row - p), slot offsets immediate; one
            // volatile read per element from the selected base (a plain read
            // of each base was sunk into a branch per element, each with its
            // own s_waitcnt lgkmcnt(0): 29 serialised LDS round trips per row
            // pass)
            lds_cptr za = (lds_cptr)(crow + j0);
            lds_cptr zb = za - p;
            asm("" : "+v"(za), "+v"(zb));
            if (ext) {
                // past the row: its wrapped extension (or, past that, words
                // only differences with masked columns read)
#pragma unroll
                for (int t = 0; t < CH + kSnrWin; ++t) z[t] = lds_ld(za + t);
            } else {
                // the wrap term as an addend (+0.0 before the wrap point: the
                // prefix values are never -0.0, so x + 0.0 == x exactly), so
                // no compare mask lives across the reads
                float x[CH + kSnrWin], ad[CH + kSnrWin];
#pragma unroll
                for (int t = 0; t < CH + kSnrWin; ++t) {
                    const bool wrap = j0 + t >= p;
                    ad[t] = wrap ? sum : 0.0f;
                    x[t] = lds_ld((wrap ? zb : za) + t);
                }
#pragma unroll
                for (int t = 0; t < CH + kSnrWin; ++t) z[t] = __fadd_rn(x[t], ad[t]);
            }
            RT_SNR_MARK(9);
            uint32_t iw0 = 0;
            if constexpr (G == 8 || G == 16) {
                if (std6) {
                    // widths 0-5 are the standard ladder: lane g < 6 keeps width g
                    sel[0] = snr_std6<CH, G>(z, cp, g);
                    iw0 = 6;
                }
            }
            if constexpr (G == 4) {
                if (std3) {
                    // widths 0-2 are 1, 2, 3: lane g < 3 keeps width g
                    sel[0] = snr_std3<CH>(z, cp, g);
                    iw0 = 3;
                }
            }
            for (uint32_t iw = iw0; iw < nw; ++iw) {
                const int w = __builtin_amdgcn_readlane(wlane, (int)iw);
                if (w <= kSnrWin) emit(iw, window_dispatch<CH>(w, z, cp));
            }
        }
        // wider widths: the window c[j0 + w ..] read from LDS per width
        for (uint32_t iw = 0; iw < nw; ++iw) {
            const int w = __builtin_amdgcn_readlane(wlane, (int)iw);
            if (CH <= kSnrMaxChunk && w <= kSnrWin) continue;
            if constexpr (CH <= kSnrMaxChunk) {
                // c[j0 + w + t] for the lane's columns t at immediate offsets:
                // WIDE, inside the row or its stored extension; else the wrap
                // (j >= p) as a second base za - p and the addend sum (+0.0
                // before the wrap point: exact, the prefix values are never
                // -0.0).  Columns past the chunk read words whose differences
                // with cp = +inf are dropped.
                lds_cptr za = (lds_cptr)(crow + j0 + w);
                lds_cptr zb = za - p;
                asm("" : "+v"(za), "+v"(zb));
                float d[CH];
                if constexpr (WIDE) {
#pragma unroll
                    for (int t = 0; t < CH; ++t) d[t] = __fsub_rn(lds_ld(za + t), cp[t]);   // diff_max, kernels.hpp:50-60
                } else {
                    const int tw = p - j0 - w;        // first wrapped column
                    float x[CH], ad[CH];
#pragma unroll
                    for (int t = 0; t < CH; ++t) {
                        const bool wrap = t >= tw;
                        ad[t] = wrap ? sum : 0.0f;
                        x[t] = lds_ld((wrap ? zb : za) + t);
                    }
#pragma unroll
                    for (int t = 0; t < CH; ++t) d[t] = __fsub_rn(__fadd_rn(x[t], ad[t]), cp[t]);
                }
                float m = d[0];
#pragma unroll
                for (int t = 1; t + 1 < CH; t += 2) m = fmaxf(m, fmaxf(d[t], d[t + 1]));
                if constexpr (CH % 2 == 0) m = fmaxf(m, d[CH - 1]);
                emit(iw, m);
                continue;
            }
            const int last = max(cnt - 1, 0);
            float dmax = -INFINITY;
            float lv[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int j = j0 + min(t, last) + w;
                lv[t] = crow[j >= p ? j - p : j];
            }
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                const bool wrap = j0 + min(i, last) + w >= p;
                const float ck = wrap ? __fadd_rn(lv[i], sum) : lv[i];
                dmax = fmaxf(dmax, __fsub_rn(ck, cp[i]));  // diff_max, kernels.hpp:50-60
            }
            emit(iw, dmax);
        }
#pragma unroll
        for (int sl = 0; sl < NSEL; ++sl) {
            if (sl * G < (int)nw) {
                const int iw = g + sl * G;
                const int iwc = min(iw, (int)nw - 1);
                const float hpb = whb[2 * iwc], b = whb[2 * iwc + 1];
                const float v = (hpb * sel[sl] - b * sum) / U.stdnoise;
                const uint32_t o = (active && iw < (int)nw) ? ((uint32_t)r * nw + (uint32_t)iw) * 4u : 0x80000000u;
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), srs, (int)o, 0, kSnrCpol);
            }
        }
        RT_SNR_MARK(10);
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

// diff_max (kernels.hpp:50-60) of width W over the S = 2 K + 1 window starts
// of a segment, c[0 .. S + W) in K + 5 register pairs P (P[k] = c[2k],
// c[2k + 1]) and, for odd W, the shifted pairs H[k] = c[2k + 1], c[2k + 2]:
// max_i c[i + W] - c[i], two differences per v_pk_add_f32 (negated second
// operand: x + (-y) == x - y, signed zeros included) and one v_max3_f32.
template <int K, int W>
__device__ __forceinline__ float seg_window_max(const f2v (&P)[K + 5], const f2v (&H)[K + 4])
{
    float dm = -INFINITY;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const f2v hi = (W & 1) ? H[k + (W - 1) / 2] : P[k + W / 2];
        f2v d;
        asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(d) : "v"(hi), "v"(P[k]));
        asm("v_max3_f32 %0, %0, %1, %2" : "+v"(dm) : "v"(d.x), "v"(d.y));
    }
    // the last start, 2K
    constexpr int e = 2 * K + W;
    const float ce = (e & 1) ? P[e / 2].y : P[e / 2].x;
    float t;
    asm("v_sub_f32 %1, %2, %3\n\tv_max_f32 %0, %0, %1" : "+v"(dm), "=&v"(t) : "v"(ce), "v"(P[K].x));
    return dm;
}

// Segmented boxcar S/N (snr.hpp:37-65, kernels.hpp:50-101) of a final level
// of <= 64 rows of 240-264 bins, row r at slot + r * kSnrSegStride + r0 (r0 =
// 8 S - p <= 24 columns of slack in front of the row): lane = row, wave w =
// slot columns [w S, w S + S).  The slack columns count as +0.0 samples and
// +inf prefix values (selects in wave 0 only), so they add nothing to the
// sums and never start a window.
//   A. the segment's S samples and the next segment's first E (the last
//      segment: the row's first E) into registers; the segment's fp64 sum to
//      the exchange area (kSnrSegExch floats at the end of the level buffer);
//   B. the segment's offset (the sums of the segments before it, in order),
//      the row total, the segment's fp64 running sum cast per column
//      (circular_prefix_sum, kernels.hpp:62-80), and the next segment's first
//      E prefix values the same way from offset + this segment's sum -- the
//      very additions the next wave makes -- (the last segment: the wrap
//      c[p + e] = c[e] + sum, kernels.hpp:88-97, c[e] from the row's first
//      samples from +0.0, as wave 0 does);
//   C. every width's window maximum over the segment's starts, to a maxima
//      area below the exchange area (the rows' samples are all in registers
//      by then: the phase-A barrier);
//   D. width iw on wave iw (mod 8): the 8 segment maxima, the S/N formula,
//      one store per row.
// Each lane works on its own row throughout: no shuffles or scans, and no
// prefix values exchanged (2 workgroup barriers).
template <int SMAX>
__device__ __forceinline__ void snr_segments(const ConeArgs& a, const UnitView& U, float* slot, const int* wl,
                                             int nrows, int tid, const float* whb)
{
    constexpr int S = kSnrSegCols;
    constexpr int E = kSnrSegWmax;
    constexpr int K = S / 2;
    constexpr int q = kSnrSegStride;
    constexpr int kMax = 8 * E * 64;          // maxima area: [segment][width - 1][lane]
    static_assert(S == 2 * K + 1 && 2 * (K + 5) >= S + E && 8 * S - 24 > 0, "segment shape");
    static_assert(kSnrSegRows <= 64 && kLdsBufFloats - kSnrSegExch - kMax >= 0, "segmented S/N areas");
    // an opaque thread index (as snr_epilogue)
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63;
    const int wave = uni(tid >> 6);
    const int p = U.p;
    const int nev = (int)min((int64_t)nrows, (int64_t)U.rows_eval - (int64_t)U.s0);
    if (nev <= 0) return;
    const uint32_t nw = a.num_widths;
    const int r0 = 8 * S - p;                 // slack columns in front of the row (0 .. 24)
    // r0 in a VGPR: the slack selects of wave 0 as v_cmp + v_cndmask (uniform
    // masks per column were hoisted into SGPR pairs that spill)
    int r0v = r0;
    asm volatile("" : "+v"(r0v));
    uint32_t wmask = 0;
    for (uint32_t iw = 0; iw < nw; ++iw) wmask |= 1u << uni(wl[iw]);
    double* const exch = reinterpret_cast<double*>(slot + kLdsBufFloats - kSnrSegExch);
    float* const maxa = slot + kLdsBufFloats - kSnrSegExch - kMax;
    float* const snr = a.snr + (uint64_t)U.trial * a.snr_stride + (U.snr_row + (uint64_t)U.s0) * (uint64_t)nw;
    const __amdgpu_buffer_rsrc_t srs = buffer_rsrc(snr, (uint32_t)nev * nw * 4u);
    // one block of <= 64 rows (snr_seg_ok); rows past nev compute the values
    // of row nev - 1 again and do not store
    const int r = lane;
    const bool act = r < nev;
    float* const row = slot + min(r, nev - 1) * q;
    const float* const seg = row + wave * S;
    float c[S], n[E];
    // A: samples (this segment, then the next one's first E) and the sum
#pragma unroll
    for (int g = 0; g < S; ++g) c[g] = lds_ld((lds_cptr)(seg + g));
    {
        const lds_cptr nx = (lds_cptr)(wave < 7 ? seg + S : row + r0);
#pragma unroll
        for (int e = 0; e < E; ++e) n[e] = lds_ld(nx + e);
    }
    if (wave == 0) {
        asm volatile("" : "+v"(r0v));
#pragma unroll
        for (int g = 0; g < 24; ++g) c[g] = g < r0v ? 0.0f : c[g];
    }
    // (the first addition of 0.0 dropped: a -0.0 sum is made +0.0 by the
    // offsets' and the total's +0.0 starts)
    double part = (double)c[0];
#pragma unroll
    for (int g = 1; g < S; ++g) part = part + (double)c[g];
    exch[wave * 64 + lane] = part;
    lds_barrier();
    // B: offset, total, prefix values of this segment and of the next one's
    // first E columns
    double off = 0.0, tot = 0.0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
        const double pv = exch[w * 64 + lane];
        if (w < wave) off = off + pv;
        tot = tot + pv;
    }
    const float sumx = (float)tot;
    double acc = off;
#pragma unroll
    for (int g = 0; g < S; ++g) {
        acc = acc + (double)c[g];
        c[g] = (float)acc;
    }
    {
        // the next wave's offset is ((p_0 + p_1) + ...) + p_wave: off + part,
        // the same additions; the last wave starts the row over from +0.0
        double an = wave < 7 ? off + part : 0.0;
#pragma unroll
        for (int e = 0; e < E; ++e) {
            an = an + (double)n[e];
            n[e] = (float)an;
        }
        if (wave == 7) {
#pragma unroll
            for (int e = 0; e < E; ++e) n[e] = __fadd_rn(n[e], sumx);
        }
    }
    // C: the window maxima; prefix values as pairs P[k] = c[2k], c[2k + 1]
    // (wave 0: +inf at the slack starts), c[S + e] = n[e]
    f2v P[K + 5], H[K + 4];
#pragma unroll
    for (int k = 0; k < K; ++k) P[k] = f2v{c[2 * k], c[2 * k + 1]};
    P[K] = f2v{c[2 * K], n[0]};
#pragma unroll
    for (int k = K + 1; k < K + 5; ++k) P[k] = f2v{n[2 * (k - K) - 1], n[2 * (k - K)]};
    if (wave == 0) {
        asm volatile("" : "+v"(r0v));
#pragma unroll
        for (int g = 0; g < 24; ++g) {
            if (g & 1) P[g / 2].y = g < r0v ? INFINITY : P[g / 2].y;
            else P[g / 2].x = g < r0v ? INFINITY : P[g / 2].x;
        }
    }
#pragma unroll
    for (int k = 0; k < K + 4; ++k) H[k] = f2v{P[k].y, P[k + 1].x};
    float m[E + 1];
#pragma unroll
    for (int w = 0; w <= E; ++w) m[w] = -INFINITY;
    constexpr uint32_t kStdMask = (1u << 1) | (1u << 2) | (1u << 3) | (1u << 4) | (1u << 6) | (1u << 9);
    if (wmask == kStdMask) {
        // the standard ladder 1, 2, 3, 4, 6, 9 in one block: six independent
        // max chains for the scheduler to interleave
        m[1] = seg_window_max<K, 1>(P, H);
        m[2] = seg_window_max<K, 2>(P, H);
        m[3] = seg_window_max<K, 3>(P, H);
        m[4] = seg_window_max<K, 4>(P, H);
        m[6] = seg_window_max<K, 6>(P, H);
        m[9] = seg_window_max<K, 9>(P, H);
    } else {
        if (wmask & (1u << 1)) m[1] = seg_window_max<K, 1>(P, H);
        if (wmask & (1u << 2)) m[2] = seg_window_max<K, 2>(P, H);
        if (wmask & (1u << 3)) m[3] = seg_window_max<K, 3>(P, H);
        if (wmask & (1u << 4)) m[4] = seg_window_max<K, 4>(P, H);
        if (wmask & (1u << 5)) m[5] = seg_window_max<K, 5>(P, H);
        if (wmask & (1u << 6)) m[6] = seg_window_max<K, 6>(P, H);
        if (wmask & (1u << 7)) m[7] = seg_window_max<K, 7>(P, H);
        if (wmask & (1u << 8)) m[8] = seg_window_max<K, 8>(P, H);
        if (wmask & (1u << 9)) m[9] = seg_window_max<K, 9>(P, H);
    }
#pragma unroll
    for (int w = 1; w <= E; ++w)
        if (wmask & (1u << w)) maxa[(wave * E + w - 1) * 64 + lane] = m[w];
    lds_barrier();
    // D: width iw on wave iw (mod 8)
    for (int iw = wave; iw < (int)nw; iw += 8) {
        const int w = uni(wl[iw]);
        const lds_cptr mx = (lds_cptr)(maxa + (w - 1) * 64 + lane);
        float dm = lds_ld(mx);
#pragma unroll
        for (int k = 1; k < 8; ++k) dm = fmaxf(dm, lds_ld(mx + E * 64 * k));
        const float hpb = whb[2 * iw], b = whb[2 * iw + 1];
        const float v = (hpb * dm - b * sumx) / U.stdnoise;
        const uint32_t o = act ? ((uint32_t)r * nw + (uint32_t)iw) * 4u : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), srs, (int)o, 0, kSnrCpol);
    }
}

// Phase-bin range [lo, hi] a cone kernel variant runs, and the S/N lane-group
// size G of a row of p bins: the epilogue instantiates only the row shapes its
// variant can meet (smaller kernels; the rest is compiled out).
// The wide variants' slot widths are the register staging's breakpoints
// (merge_rows_per_wave = 45 / slots rows per wave): 11 slots stage 4 rows
// per wave (32-row units at p = 513-704, where 16 slots staged 2), 22 slots
// 2 (16-row units at p = 1025-1408, where 45 slots staged 1).
constexpr int variant_pmin(int smax)
{
    return smax == kPack2 ? 1
                          : (smax <= 5 ? 64 * (smax - 1) + 1
                                       : (smax == 8 ? 321 : (smax == 11 ? 513 : (smax == 16 ? 705 : (smax == 22 ? 1025 : 1409)))));
}
constexpr int variant_pmax(int smax) { return smax == kPack2 ? 32 : 64 * smax; }
constexpr bool variant_has_group(int smax, int G)
{
    return snr_group(variant_pmin(smax)) <= G && G <= snr_group(variant_pmax(smax));
}

// S/N lane-group size of the short-row variant (kPack2, p <= 32).  A/B, same
// box, cone ms per cfg4 trial (profiles/r03zf_ab_cfg4.log): G = 8 0.837 /
// 0.837, G = 4 0.777 / 0.778, G = 2 0.796 / 0.797, S/N identical -- 4.
constexpr int kSnrShortG = 4;

// register chunk of a short row's S/N lane (snr_epilogue's kPack2 case)
__device__ __forceinline__ int snr_short_ch(int p)
{
    const int cs = ((p + kSnrShortG - 1) / kSnrShortG) | 1;
    return cs <= 5 ? 5 : (cs <= 9 ? 9 : kSnrMaxChunk);
}

// Row stride of a short-row final pass's output level: room for the S/N's
// whole-chunk prefix writes and its wrapped prefix extension (snr_rows'
// wfull / ext / natural paths: no per-column dummy selects, no wrap selects
// in the window reads), and = 4 (mod 8), so the 8 rows x 4 chunks of a 32-lane
// LDS group (chunk stride c odd) start on 32 distinct banks (at the odd merge
// stride p | 1 they collided).
__device__ __forceinline__ int snr_short_stride(int p)
{
    const int cs = ((p + kSnrShortG - 1) / kSnrShortG) | 1;
    const int ch = snr_short_ch(p);
    const int q0 = max(p + max(ch, kSnrWin), (kSnrShortG - 1) * cs + ch);
    return q0 + ((4 - q0) & 7);
}

template <int SMAX, bool WIDE = false>
__device__ __forceinline__ void snr_epilogue(const ConeArgs& a, const UnitView& U, float* data, int q, const int* wl,
                                             int nrows, int tid, float* whb, unsigned long long* tl)
{
    // an opaque thread index: nothing lane-derived of the S/N is hoisted out
    // of the kernel's trial loop into registers live across the merge
    asm volatile("" : "+v"(tid));
    const int lane = tid & 63, wave = tid >> 6;
    const int p = U.p;
    const int nev = (int)min((int64_t)nrows, (int64_t)U.rows_eval - (int64_t)U.s0);
    if (nev <= 0) return;
    // G lanes per row: the smallest power of two >= 8 whose chunks fit
    // kSnrMaxChunk columns; chunk lengths odd (the G chunks of a row start
    // on distinct banks)
    int G = 8;
    while (G < 64 && (((p + G - 1) / G) | 1) > kSnrMaxChunk) G <<= 1;
    int c = (p + G - 1) / G;
    if (c < kSnrMaxChunk) c |= 1;
    const uint32_t nw = a.num_widths;
    float* snr = a.snr + (uint64_t)U.trial * a.snr_stride + (U.snr_row + (uint64_t)U.s0) * (uint64_t)nw;
    if constexpr (SMAX == kPack2) {
        // short rows (p <= 32): kSnrShortG lanes per row, so a pass covers
        // 512 / G rows (cfg4's ~380-row final units: 3 passes at G = 4
        // instead of 6 at G = 8)
        constexpr int GS = kSnrShortG;
        const int cs = ((p + GS - 1) / GS) | 1;
        if (cs <= 5) snr_rows<5, GS>(a, U, data, q, wl, nev, cs, tid, whb, tl);
        else if (cs <= 9) snr_rows<9, GS>(a, U, data, q, wl, nev, cs, tid, whb, tl);
        else snr_rows<kSnrMaxChunk, GS>(a, U, data, q, wl, nev, cs, tid, whb, tl);
        return;
    }
    if (c <= kSnrMaxChunk) {
        // short rows (p <= 40 / 72): register chunks sized to the row, not 17
        if constexpr (variant_has_group(SMAX, 8)) {
            if (G == 8) {
                if (c <= 5) snr_rows<5, 8>(a, U, data, q, wl, nev, c, tid, whb, tl);
                else if (c <= 9) snr_rows<9, 8>(a, U, data, q, wl, nev, c, tid, whb, tl);
                else snr_rows<kSnrMaxChunk, 8>(a, U, data, q, wl, nev, c, tid, whb, tl);
                return;
            }
        }
        if constexpr (variant_has_group(SMAX, 16)) {
            if (G == 16) {
                if constexpr (WIDE) {
                    if (snr_wide_ok(p, q, wl[kMaxWidths])) {
                        snr_rows<kSnrMaxChunk, 16, true>(a, U, data, q, wl, nev, c, tid, whb, tl);
                        return;
                    }
                }
                snr_rows<kSnrMaxChunk, 16>(a, U, data, q, wl, nev, c, tid, whb, tl);
                return;
            }
        }
        if constexpr (variant_has_group(SMAX, 32)) {
            if (G == 32) {
                snr_rows<kSnrMaxChunk, 32>(a, U, data, q, wl, nev, c, tid, whb, tl);
                return;
            }
        }
        if constexpr (variant_has_group(SMAX, 64)) snr_rows<kSnrMaxChunk, 64>(a, U, data, q, wl, nev, c, tid, whb, tl);
    } else if (c <= kSnrChunk) {
        if constexpr (variant_has_group(SMAX, 64)) snr_rows<kSnrChunk, 64>(a, U, data, q, wl, nev, c, tid, whb, tl);
    } else if constexpr (variant_pmax(SMAX) > 64 * kSnrChunk) {
        // very wide rows (p > 64 * kSnrChunk): one wave per row, chunks from LDS
        const int g = lane;
        const int j0 = min(g * c, p);
        const int cnt = min(j0 + c, p) - j0;
        const int owner = (p - 1) / c;
        for (int base = 0; base < nev; base += kConeWaves) {
            const int r = base + wave;
            const bool active = r < nev;
            float* row = data + min(r, nev - 1) * q;
            double part = 0.0;
            for (int j = j0; j < j0 + cnt; ++j) part += (double)row[j];
            double incl = part;
            for (int d = 1; d < 64; d <<= 1) {
                const double y = __shfl_up(incl, d, 64);
                if (g >= d) incl += y;
            }
            double acc = __shfl_up(incl, 1, 64);
            if (g == 0) acc = 0.0;
            lds_barrier();
            if (active)
                for (int j = j0; j < j0 + cnt; ++j) {
                    acc += (double)row[j];
                    row[j] = (float)acc;
                }
            const float sum = __shfl((float)acc, owner, 64);
            lds_barrier();
            for (uint32_t iw = 0; iw < nw; ++iw) {
                const int w = uni(wl[iw]);
                float dmax = -INFINITY;
                for (int i = j0; i < j0 + cnt; ++i) {
                    const int k = i + w;
                    const float ck = k < p ? row[k] : __fadd_rn(row[k - p], sum);
                    dmax = fmaxf(dmax, __fsub_rn(ck, row[i]));
                }
                for (int o = 32; o > 0; o >>= 1) dmax = fmaxf(dmax, __shfl_xor(dmax, o, 64));
                if (active && g == 0) {
                    const float h = sqrtf((float)(p - w) / (float)(p * w));
                    const float b = (float)w / (float)(p - w) * h;
                    snr[(uint64_t)r * nw + iw] = ((h + b) * dmax - b * sum) / U.stdnoise;
                }
            }
            lds_barrier();
        }
    }
}

// Diagnostic build only (make stamps, -DRT_STAMPS): thread 0 of every unit
// writes one record of s_memtime marks at phase boundaries to a.stamps +
// kStampRecWords * u (the host offsets a.stamps per launch; no atomics, so
// the timing is not perturbed by contention).
#ifdef RT_STAMPS
#define RT_MARK(i)                                                               \
    do {                                                                         \
        if (tid == 0) tl[i] = __builtin_amdgcn_s_memtime();                      \
    } while (0)
#else
#define RT_MARK(i) do { } while (0)
#endif

// One kernel per merge slot width SMAX (units with ceil(p/64) <= SMAX), so each
// gets its own register allocation; one workgroup per unit u = blockIdx.x
// (unit u = item u / batch, trial u % batch; items are sorted longest first),
// two workgroups per CU: a unit's DMA is waited for at its start, the CU's
// other workgroup filling the wait.
//   begin(u) [DMA] | wait | merge(u) | store or S/N(u)
// SNR: the launch's units all end in the fused S/N (final passes) -- or none
// does (the merge-only passes store their output level): separate instances,
// so a merge-only launch carries no S/N code and no S/N register floor.
// WIDE: final units whose S/N takes the widths past its register window as
// plain LDS windows (snr_wide_ok; a separate instantiation, so the plans
// without such widths run code without it)
// instances whose workgroups run several trials of an item (ConeArgs::
// trials_per_wg); the others one trial each
#ifdef RT_NO_TRIAL_LOOP
template <int SMAX> constexpr bool kTrialLoop = false;   // A/B build: one trial per workgroup everywhere
#else
template <int SMAX> constexpr bool kTrialLoop = SMAX >= 4;
#endif

template <int SMAX, int RWT, bool WIDE, bool SNR>
__global__ __launch_bounds__(kConeBlock, kConeWavesPerSimd) void cone_kernel(ConeArgs a)
{
    constexpr int RW = RWT ? RWT : merge_rows_per_wave(SMAX);   // register rows per wave
    __shared__ __attribute__((aligned(16))) float data[kLdsBufFloats + kLdsPadFloats];
    __shared__ __attribute__((aligned(16))) uint32_t aux[kAuxWords + kLutPad];   // the host blob (+ roll table)
    // boxcar widths (LDS reads never wait on the S/N stores in flight), then
    // the widest of them
    __shared__ int wl[kMaxWidths + 1];
    __shared__ float whb[2 * kMaxWidths];   // S/N: h + b and b per width

    const int tid = threadIdx.x;
#ifdef RT_STAMPS
    unsigned long long t_entry = __builtin_amdgcn_s_memtime();
    unsigned long long r_entry = __builtin_amdgcn_s_memrealtime();
    unsigned long long t_begin[3] = {};
#endif
    // workgroup -> (item, its trials t0 .. t0 + tn - 1); the 1-3-slot
    // instances (p = 33-192, no BASELINE config) run one trial per workgroup
    // (launch_cone): their trial loop would spill
    const uint32_t tpw = (kTrialLoop<SMAX> && a.trials_per_wg) ? a.trials_per_wg : 1u;
    const uint32_t groups = cone_trial_groups(a.batch, tpw);
    const uint32_t total = a.num_items * groups;
    if (blockIdx.x >= total) return;
    const uint32_t item = blockIdx.x / groups;
    const uint32_t t0 = (blockIdx.x - item * groups) * tpw;
    const int tn = (int)min(tpw, a.batch - t0);
    if (tid < (int)a.num_widths) wl[tid] = (int)a.widths[tid];   // visible after the first barrier
    if (tid == 0) {
        uint32_t wm = 0;
        for (uint32_t i = 0; i < a.num_widths; ++i) wm = max(wm, a.widths[i]);
        wl[kMaxWidths] = (int)wm;
    }
    const bool dma = !(a.flags & kConeDiagNoLand);
    bool ok;
#ifdef RT_STAMPS
    UnitCtx C = unit_begin<SMAX, RW>(a, item, t0, aux, data, tid, dma, ok, t_begin);
    unsigned long long tl[kStampMarks] = {};
    tl[0] = __builtin_amdgcn_s_memtime();
#else
    UnitCtx C = unit_begin<SMAX, RW>(a, item, t0, aux, data, tid, dma, ok);
#endif
    const UnitView& U = C.U;
    const int p = U.p;
    const int L = U.levels;
    float* const buf = data;
    // the launch kind is the unit's (the planner splits final and merge-only
    // launches; validate_exec_plan)
    ok = ok && ((U.dst == kSelSnr) == SNR);
    // a final pass's per-width S/N constants, published by the barrier below
    // (the S/N row passes have no barrier of their own)
    if (SNR && tid < (int)a.num_widths) snr_width_consts(wl[tid], p, whb + 2 * tid);
    // the roll table of a 4-slot unit (past its blob's LDS part, which the
    // DMA may still be writing), published by the barrier below
    if constexpr (SMAX == 4)
        if (C.slots && ok) build_roll_lut4(aux + kLut4Off, p, tid);
    // the -0.0 row of an all-fused whole unit (past the fill: no trial's DMA
    // or merge level writes it, so once per workgroup)
    if constexpr (resolved_slots(SMAX))
        if (ok && U.zero_row)
            for (int j = tid; j < 64 * SMAX; j += kConeBlock) data[U.zero_row + j] = -0.0f;
    // the short-row roll table in the unused metadata area
    if constexpr (SMAX == kPack2)
        if (ok && p >= kPackSeg) build_pack_lut(aux, p, tid);
    // every wave waits for its own DMA, the barrier publishes all of them
    __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
    lds_barrier();
    RT_MARK(1);
    RT_MARK(2);
    if (!ok) {
        if (tid == 0 && a.error_flag) atomicOr(a.error_flag, 1);
        return;
    }
    // merge levels, deepest first; a non-final pass stores its output level
    // straight from registers (st), a final pass keeps it in LDS for the S/N
    // epilogue
    constexpr bool st = !SNR;
    const bool st_regs = st && (a.flags & kConeStoreFromRegs);
    const uint32_t o0 = (uint32_t)(U.node_start + U.s0) * (uint32_t)p * 4u;
    const int n0 = rows_at(C, 0);
    // a final pass's output level at a row stride = 16 (mod 32): the S/N
    // epilogue's lane groups (two rows of 16 lanes per 32-lane LDS group, odd
    // chunk strides) then read and write on distinct banks (at stride p they
    // collided on up to 10 of 32 banks)
    int qout = p;
    // the segmented S/N (snr_segments): rows of 240-264 bins, widths <= 9,
    // <= 64 rows in slots of kSnrSegStride floats (feature bit kConeSnrSeg)
    // (not in the WIDE instances: widths past kSnrWin exclude it, and their
    // code stays free of its registers)
    const bool seg_snr = SNR && !WIDE && resolved_slots(SMAX) && (a.flags & kConeSnrSeg) && L > 0 && C.slots &&
                         snr_seg_ok(p, wl[kMaxWidths], n0);
    // short rows keep their blob's LDS part at the end of the level buffer,
    // which a final pass's output level (at the S/N stride) and its S/N's
    // dummy words may overwrite: every trial's fill then re-DMAs it -- unless
    // the output level at the short-row S/N stride ends below the blob (set
    // below: that stride takes the S/N's whole-chunk path, which writes no
    // dummy words, only the rows [0, n0 q) and their wrapped extensions)
    bool blob_clobbered = SMAX == kPack2 && SNR;
    // short rows in (row, segment) tasks: every level above the fill at the
    // odd stride pack_stride(p)
    if constexpr (SMAX == kPack2) {
        if (L > 0) qout = pack_stride(p);
        // a final pass's output level at the short-row S/N stride where the
        // unit's rows fit (over the blob: the blob is dead once the last
        // merge step has read its table, a barrier before the level's
        // write-back)
        if (SNR && L > 0 && p >= kPackSeg && (a.flags & kConeSnrStride)) {
            const int qf = snr_short_stride(p);
            if (n0 * qf <= kLdsDataFloats) qout = qf;
            // the blob survives the S/N: loaded once per workgroup, not per
            // trial (cfg4's final units re-read ~12 KB of
            // blob per trial, 0.1 GB of its 1.34 GB)
            if (qout == qf && n0 * qf + U.run_off <= kLdsBufFloats) blob_clobbered = false;
        }
    }
    if constexpr (SMAX <= 5 && SMAX != kPack2) {
        // = 16 (mod 32) and >= p + kSnrMaxChunk (room for the S/N's whole-
        // chunk prefix writes and its wrapped prefix extension), else >=
        // p + kSnrWin (the extension only)
        const int qa = p + kSnrMaxChunk + ((16 - ((p + kSnrMaxChunk) & 31)) & 31);
        const int qb = p + kSnrWin + ((16 - ((p + kSnrWin) & 31)) & 31);
        if (seg_snr) {
            qout = kSnrSegStride;
        } else if (!st && L > 0 && C.slots && (a.flags & kConeFuse2) && (a.flags & kConeSnrStride)) {
            qout = n0 * qa <= kLdsDataFloats ? qa : (n0 * qb <= kLdsDataFloats ? qb : p);
            // widths past the register window: a stride with room for their
            // plain-LDS windows (snr_wide_stride), = 16 (mod 32) where that
            // fits too
            const int wmax = wl[kMaxWidths];
            if (WIDE && snr_group(p) == 16 && wmax > kSnrWin && wmax < p) {
                const int qw = snr_wide_stride(p, wmax);
                const int qwp = qw + ((16 - (qw & 31)) & 31);
                if (n0 * qwp <= kLdsDataFloats) qout = qwp;
                else if (n0 * qw <= kLdsDataFloats) qout = qw;
            }
        }
    }
    // the trials of this workgroup, one after the other: trial k's level
    // buffer is free once its last merge step has read it (merge-only units
    // store that step from registers: the next trial's fill is issued before
    // those stores) or once its S/N has read it (final units)
    for (int k = 0;;) {
        const int trial = C.U.trial;
        const float* dst = (U.dst == kSelPing ? a.ping : a.pong) + (uint64_t)trial * a.buf_stride + U.buf_off;
        const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(dst, (((uint32_t)U.m * (uint32_t)p + 3u) & ~3u) * 4u);
        const bool more = k + 1 < tn;
        bool next_issued = false;
        auto fill_next = [&]() {
            if (more) {
                lds_barrier();           // every wave is past its last read of the level buffer
                if (dma) unit_fill<SMAX>(a, C, trial + 1, buf, tid, blob_clobbered);
            }
            next_issued = true;
        };
        if (L > 0 && !(a.flags & kConeDiagNoMerge))
            merge_levels<SMAX, RW>(C, buf, p, L, tid, st_regs, rs, o0, a.flags, buf + kLdsBufFloats + 4 + (tid & 63),
                                   qout, seg_snr ? 8 * kSnrSegCols - p : 0, fill_next);
        RT_MARK(3);
        // the output level: dense rows from the buffer start, or (no merge
        // level) the single bottom row where the DMA left it
        float* const obase = L > 0 ? buf : buf + (C.table ? uni(bottom_offsets(C)[0]) : C.al);
        if (st) {
            if (L == 0 || !st_regs) {
                const int qst = L > 0 ? qout : p;    // the merged level's LDS row stride
                for (int r = 0; r < n0; ++r)
                    for (int j = tid; j < p; j += kConeBlock)
                        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(obase[r * qst + j]), rs,
                                                              (int)(o0 + (uint32_t)(r * p + j) * 4u), 0, kStoreCpol);
            }
        } else if constexpr (SNR) {
            if (seg_snr) {
                if constexpr (resolved_slots(SMAX) && !WIDE)
                    if (!(a.flags & kConeDiagNoSnr)) snr_segments<SMAX>(a, C.U, buf, wl, n0, tid, whb);
            } else {
#ifdef RT_STAMPS
                if (!(a.flags & kConeDiagNoSnr)) snr_epilogue<SMAX, WIDE>(a, C.U, obase, qout, wl, n0, tid, whb, tl);
#else
                if (!(a.flags & kConeDiagNoSnr)) snr_epilogue<SMAX, WIDE>(a, C.U, obase, qout, wl, n0, tid, whb, nullptr);
#endif
            }
        }
#ifdef RT_STAMPS
        lds_barrier();
        RT_MARK(4);
        tl[5] = t_entry;
        tl[11] = t_begin[0];
        tl[12] = t_begin[1];
        tl[13] = t_begin[2];
        RT_MARK(6);
        tl[14] = r_entry;
        tl[15] = __builtin_amdgcn_s_memrealtime();
        if (tid == 0 && a.stamps) {
            unsigned long long* e = a.stamps + (uint64_t)kStampRecWords * ((uint64_t)item * a.batch + (uint32_t)trial);
            const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_REG_HW_ID
            const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
            e[0] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
#pragma unroll
            for (int i = 0; i < kStampMarks; ++i) e[1 + i] = tl[i];
            e[1 + kStampMarks] = (unsigned long long)p | ((unsigned long long)L << 16) |
                                 ((unsigned long long)U.mode << 24) | ((unsigned long long)rows_at(C, 0) << 32) |
                                 ((unsigned long long)(U.dst == kSelSnr) << 48);
        }
#endif
        if (!kTrialLoop<SMAX> || !more) break;
        // final units (and merge-only units not stored from registers): the
        // next trial's fill once every wave is done with the level buffer
        if (!next_issued) fill_next();
        // a final unit's output level (at the S/N stride) may have covered the
        // zero row: rewritten for the next trial (its first step reads it)
        if constexpr (resolved_slots(SMAX) && SNR)
            if (U.zero_row)
                for (int j = tid; j < 64 * SMAX; j += kConeBlock) data[U.zero_row + j] = -0.0f;
        ++k;
        C.U.trial = trial + 1;
#ifdef RT_STAMPS
        t_entry = __builtin_amdgcn_s_memtime();
        r_entry = __builtin_amdgcn_s_memrealtime();
        t_begin[0] = t_begin[1] = t_begin[2] = t_entry;
        tl[0] = t_entry;
#endif
        // the next trial's fill (and this trial's stores, which count in the
        // same in-order counter) landed; the barrier publishes every wave's
        __builtin_amdgcn_s_waitcnt(0x0F70);          // vmcnt(0)
        lds_barrier();
        RT_MARK(1);
        RT_MARK(2);
    }
    // every DMA was waited for before its trial, and the stores need no wait
    // before the end of the program
}

// One workgroup per unit: the hardware dispatcher keeps both of a CU's
// workgroup slots busy to the end of the launch (measured: 10.37 vs 11.55 ms
// per cfg2 trial against a persistent grid, round 1).
template <int SMAX, int RW = 0>
static hipError_t launch_kind(const ConeArgs& args, dim3 g, dim3 b, bool wide_snr, bool snr, hipStream_t s)
{
    if (!snr) {
        if (wide_snr) return hipErrorInvalidValue;
        hipLaunchKernelGGL((cone_kernel<SMAX, RW, false, false>), g, b, 0, s, args);
    } else if (wide_snr && SMAX >= 3 && SMAX <= 5 && RW == 0) {
        // (the register-row-class instances have no WIDE form: their S/N
        // reads the wide widths through the general per-width path)
        if constexpr (SMAX >= 3 && SMAX <= 5 && RW == 0) hipLaunchKernelGGL((cone_kernel<SMAX, 0, true, true>), g, b, 0, s, args);
    } else {
        hipLaunchKernelGGL((cone_kernel<SMAX, RW, false, true>), g, b, 0, s, args);
    }
    return hipSuccess;
}

hipError_t launch_cone(const ConeArgs& args_in, uint32_t smax, uint32_t rw, bool wide_snr, bool snr, hipStream_t s)
{
    if (!args_in.num_items || !args_in.batch) return hipSuccess;
    ConeArgs args = args_in;
#ifdef RT_NO_TRIAL_LOOP
    args.trials_per_wg = 1;
#else
    if (smax < 4) args.trials_per_wg = 1;    // kTrialLoop: one trial per workgroup
#endif
    const uint64_t total = (uint64_t)args.num_items * cone_trial_groups(args.batch, args.trials_per_wg);
    if (total > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const dim3 g((uint32_t)total), b(kConeBlock);
    hipError_t e = hipErrorInvalidValue;
    // one instance per slot width: every unit runs the variant's default
    // register rows (the planner no longer splits launches by node size)
    if (rw != 0) return hipErrorInvalidValue;
    switch (smax) {
    case 1: e = launch_kind<1>(args, g, b, wide_snr, snr, s); break;
    case 2: e = launch_kind<2>(args, g, b, wide_snr, snr, s); break;
    case 3: e = launch_kind<3>(args, g, b, wide_snr, snr, s); break;
    case 4: e = launch_kind<4>(args, g, b, wide_snr, snr, s); break;
    case 5: e = launch_kind<5>(args, g, b, wide_snr, snr, s); break;
    case 8: e = launch_kind<8>(args, g, b, wide_snr, snr, s); break;
    case 11: e = launch_kind<11>(args, g, b, wide_snr, snr, s); break;
    case 16: e = launch_kind<16>(args, g, b, wide_snr, snr, s); break;
    case 22: e = launch_kind<22>(args, g, b, wide_snr, snr, s); break;
    case kMaxSlots: e = launch_kind<kMaxSlots>(args, g, b, wide_snr, snr, s); break;
    case kPack2: e = launch_kind<kPack2>(args, g, b, wide_snr, snr, s); break;
    default: return hipErrorInvalidValue;
    }
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace rt

namespace rt {

// ---------------------------------------------------------------------------
// Fallback for rows too wide for the LDS cone kernel (ffa2 with p > ~11k):
// one launch per tree depth, one workgroup per output row, global memory.
// nodes[] = (start, size) of every node at this depth, sorted by start.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void ffa_level_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                        const uint2* __restrict__ nodes, uint32_t num_nodes,
                                                        uint32_t p)
{
    const uint32_t u = blockIdx.x;
    uint32_t lo = 0, hi = num_nodes - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (nodes[mid].x <= u) lo = mid; else hi = mid - 1;
    }
    const uint2 nd = nodes[lo];
    const float* hrow;
    const float* trow = nullptr;
    uint32_t shift = 0;
    if (nd.y <= 1) {
        hrow = in + (uint64_t)u * p;
    } else {
        const uint32_t s = u - nd.x, sh = nd.y >> 1, st = nd.y - sh;
        const uint32_t h = merge_index(merge_coef(sh, nd.y), s);
        const uint32_t t = merge_index(merge_coef(st, nd.y), s);
        hrow = in + (uint64_t)(nd.x + h) * p;
        trow = in + (uint64_t)(nd.x + sh + t) * p;
        shift = (s - t) % p;
    }
    float* o = out + (uint64_t)u * p;
    for (uint32_t j = threadIdx.x; j < p; j += 256) {
        float v = hrow[j];
        if (trow) {
            uint32_t c = j + shift;
            if (c >= p) c -= p;
            v = __fadd_rn(v, trow[c]);
        }
        o[j] = v;
    }
}

hipError_t launch_ffa_level(const float* in, float* out, const uint2* d_nodes, uint32_t num_nodes,
                            uint32_t rows, uint32_t p, hipStream_t s)
{
    hipLaunchKernelGGL(ffa_level_kernel, dim3(rows), dim3(256), 0, s, in, out, d_nodes, num_nodes, p);
    return hipGetLastError();
}

}  // namespace rt
