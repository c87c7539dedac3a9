// FFA periodogram hot path for MI355X (gfx950): downsampling ladder, LDS cone
// kernel (several FFA merge levels per HBM pass), fused boxcar S/N epilogue.
//
// Exactness: every float operation that the reference performs is performed
// here on the same operands in the same association (explicit *_rn intrinsics
// where hipcc would otherwise contract into FMA), so the FFA transform is
// bit-identical to riptide::transform (transforms.hpp:30-61) and downsample is
// bit-identical to the strict restatement of downsample.hpp:44-82.
#include <hip/hip_runtime.h>

#include "common.hpp"
#include "kernels.hpp"

namespace rt {

// ---------------------------------------------------------------------------
// Downsampling ladder (downsample.hpp:44-82; periodogram.hpp:162-168)
// ---------------------------------------------------------------------------
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
    float acc = __fmul_rn(wmin, w[0]);
    for (uint32_t i = 1; i < cnt; ++i)
        acc = __fadd_rn(acc, w[i]);
    acc = __fadd_rn(acc, __fmul_rn(wmax, w[cnt]));
    out[k] = acc;
}

// Fused ladder: one block per input span (and trial) computes the outputs of
// EVERY rung whose window starts in the span, so the series is read from HBM
// once instead of once per rung (57 rungs at cfg2).  The span plus a margin
// of kDsFusedMargin floats (>= ceil(f) + 2 for every fused rung) is staged in
// LDS; each output is the same sequential window sum as the per-rung kernel.
constexpr uint32_t kDsFusedSpan = kDsSpanFloats - kDsFusedMargin;

// first output k of a rung whose window start floor(k f) is >= s
__device__ __forceinline__ uint64_t ds_first_output(double f, uint64_t s)
{
    uint64_t k = (uint64_t)ceil((double)s / f);
    while (k > 0 && (uint64_t)floor(__dmul_rn((double)(k - 1), f)) >= s) --k;
    while ((uint64_t)floor(__dmul_rn((double)k, f)) < s) ++k;
    return k;
}

__global__ __launch_bounds__(256) void downsample_fused_kernel(
    const float* __restrict__ x, uint64_t n_in, uint64_t x_stride,
    const DsRung* __restrict__ rungs, uint32_t num_rungs,
    float* __restrict__ out, uint64_t out_stride)
{
    __shared__ float span[kDsSpanFloats];
    const uint64_t s0 = (uint64_t)blockIdx.x * kDsFusedSpan;
    const uint64_t s_end = min(s0 + (uint64_t)kDsFusedSpan, n_in);     // window starts owned by this block
    const uint64_t l_end = min(s0 + (uint64_t)kDsSpanFloats, n_in);    // staged input
    x += (uint64_t)blockIdx.y * x_stride;
    out += (uint64_t)blockIdx.y * out_stride;
    for (uint64_t i = s0 + threadIdx.x; i < l_end; i += 256) span[i - s0] = x[i];
    __syncthreads();
    const double last = (double)n_in - 1.0;
    for (uint32_t ri = 0; ri < num_rungs; ++ri) {
        const DsRung r = rungs[ri];
        float* o = out + r.out_off;
        if (r.identity) {
            for (uint64_t k = s0 + threadIdx.x; k < min(s_end, r.n); k += 256) o[k] = span[k - s0];
            continue;
        }
        const double f = r.f;
        const uint64_t k_lo = ds_first_output(f, s0);
        const uint64_t k_hi = min(s_end >= n_in ? r.n : ds_first_output(f, s_end), r.n);
        for (uint64_t k = k_lo + threadIdx.x; k < k_hi; k += 256) {
            const double start = __dmul_rn((double)k, f);
            const double end = __dadd_rn(start, f);
            const uint64_t imin = (uint64_t)floor(start);
            double dmax = floor(end);
            if (dmax > last) dmax = last;
            const uint64_t imax = (uint64_t)dmax;
            const float wmin = (float)__dsub_rn((double)(imin + 1), start);
            const float wmax = (float)__dsub_rn(end, (double)imax);
            const float* w = span + (imin - s0);
            const uint32_t cnt = (uint32_t)(imax - imin);
            float acc = __fmul_rn(wmin, w[0]);
            for (uint32_t i = 1; i < cnt; ++i) acc = __fadd_rn(acc, w[i]);
            acc = __fadd_rn(acc, __fmul_rn(wmax, w[cnt]));
            o[k] = acc;
        }
    }
}

hipError_t launch_downsample_fused(const float* x, uint64_t n_in, uint64_t x_stride, const DsRung* d_rungs,
                                   uint32_t num_rungs, float* out, uint64_t out_stride, uint32_t batch, hipStream_t s)
{
    if (!num_rungs || !batch || !n_in) return hipSuccess;
    const uint64_t blocks = (n_in + kDsFusedSpan - 1) / kDsFusedSpan;
    hipLaunchKernelGGL(downsample_fused_kernel, dim3((uint32_t)blocks, batch), dim3(256), 0, s, x, n_in, x_stride,
                       d_rungs, num_rungs, out, out_stride);
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
// One workgroup (512 threads, 77 KiB of LDS: two workgroups per CU) per work
// unit = one work item (UnitDesc) of one trial: `levels` merge levels of the
// FFA recursion for the rows of one tile (or one whole node), held in LDS.
// Phases:
//   1. setup: unit view, rows per level, range tree of tile units (the
//      planner guarantees 2^l ranges at cone level l)
//   2. fill of the bottom level (dense rows, stride p): 16-byte buffer loads
//      into registers; while they are in flight, the row descriptors of
//      every level are built into a table; then landed in LDS
//   3. merge levels, deepest first (transforms.hpp:13-27), one row per wave
//      and one phase bin per lane:
//          out[r][j] = H[h(r)][j] + T[t(r)][(j + shift(r)) mod p]
//      Lane i unpacks the descriptor of the wave's i-th row into LDS offsets;
//      the row loop takes them with v_readlane.  Bins j = lane + 64k use
//      immediate offsets, so a 64-bin slot is one ds_read for H, one for T
//      (consecutive lanes -> consecutive banks) and one ds_write.  A level's
//      outputs are staged in registers between two barriers (in place).
//   4. a non-final pass stores its last level straight from the registers;
//      a final pass runs the fused boxcar S/N epilogue (snr.hpp:37-65) on it.
// The other workgroup on the CU overlaps its latency-bound phases (setup,
// fill wait) with this one's LDS and VALU work; the kernel as a whole is
// bound by the CU's LDS, VALU and scalar issue.
struct Range {          // rows [lo, hi] of one node of the split tree
    int size;           // rows of the node
    int lo, hi;         // node-local rows
    int start;          // first row of the node within the transform
    int base;           // first LDS row of this range in its level's packed layout
};


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

__device__ __forceinline__ int wave_incl_scan_int(int v, int lane)
{
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

// Wave-uniform view of one unit (scalar registers).
struct UnitView {
    int item, trial;
    int node_start, node_size, s0, s1, levels, mode, src, dst;
    int p, m, rows_eval;
    uint64_t src_off, buf_off, snr_row;
    float stdnoise;
};

// Per-unit metadata in LDS (double-buffered): the unit's view, rows per level
// and the range tree of tile units.  Everything the merge and the epilogue of
// a unit need is read from here, never from global memory, so no vmcnt wait
// (which would also wait for the next unit's DMA) is needed after setup.
struct UnitMeta {
    UnitView view;
    int nrows[kMaxLevels + 1];       // rows of every level (0 = output level)
    int doff[kMaxLevels + 1];        // first descriptor-table entry of every level
    Range ranges[kMaxRanges];        // tile units: level l holds 2^l ranges at (1 << l) - 1
};

__device__ __forceinline__ UnitView read_view(const UnitMeta& M)
{
    UnitView v;
    v.item = uni(M.view.item);
    v.trial = uni(M.view.trial);
    v.node_start = uni(M.view.node_start);
    v.node_size = uni(M.view.node_size);
    v.s0 = uni(M.view.s0);
    v.s1 = uni(M.view.s1);
    v.levels = uni(M.view.levels);
    v.mode = uni(M.view.mode);
    v.src = uni(M.view.src);
    v.dst = uni(M.view.dst);
    v.p = uni(M.view.p);
    v.m = uni(M.view.m);
    v.rows_eval = uni(M.view.rows_eval);
    v.src_off = uni64(M.view.src_off);
    v.buf_off = uni64(M.view.buf_off);
    v.snr_row = uni64(M.view.snr_row);
    v.stdnoise = __int_as_float(uni(__float_as_int(M.view.stdnoise)));
    return v;
}

__device__ __forceinline__ UnitView unit_view(const ConeArgs& a, int item, int trial)
{
    UnitView v;
    v.item = uni(item);
    v.trial = uni(trial);
    const UnitDesc d = a.items[v.item];
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
    return v;
}

// Metadata of unit u into M (+ the source-row table of its bottom level).
// Every thread calls it; it ends with a barrier.
__device__ __forceinline__ void setup_unit(const ConeArgs& a, int item, int trial, UnitMeta& M, int* src_row, int tid)
{
    const int lane = tid & 63, wave = tid >> 6;
    const UnitView U = unit_view(a, item, trial);
    if (tid == 0) M.view = U;
    const int L = U.levels;
    if (U.mode == kModeTile) {
        // level l (wave l): lane i walks the head/tail path i (MSB first) from
        // the tile; the planner guarantees every node above the bottom level
        // has >= 2 rows, so level l has exactly 2^l ranges
        if (wave <= L) {
            const int l = wave;
            const int nr = 1 << l;
            Range R{0, 0, -1, 0, 0};
            if (lane < nr) {
                uint32_t size = (uint32_t)U.node_size, lo = (uint32_t)U.s0, hi = (uint32_t)U.s1 - 1;
                int start = U.node_start;
                for (int d = 0; d < l; ++d) {
                    const uint32_t sh = size >> 1, st = size - sh;
                    const bool tail = (lane >> (l - 1 - d)) & 1;
                    const uint32_t cs = tail ? st : sh;
                    const float k = merge_coef(cs, size);
                    lo = merge_index(k, lo);
                    hi = merge_index(k, hi);
                    if (tail) start += (int)sh;
                    size = cs;
                }
                R.size = (int)size;
                R.lo = (int)lo;
                R.hi = (int)hi;
                R.start = start;
            }
            const int c = R.hi - R.lo + 1;
            const int incl = wave_incl_scan_int(lane < nr ? c : 0, lane);
            if (lane < nr) {
                R.base = incl - c;
                M.ranges[nr - 1 + lane] = R;
            }
            if (lane == 63) M.nrows[l] = incl;
        }
        lds_barrier();
        if (tid == 0) {
            int o = 0;
            for (int l = 0; l <= L; ++l) {
                M.doff[l] = o;
                o += M.nrows[l];
            }
        }
        const int nb = uni(M.nrows[L]);
        const Range* lv = &M.ranges[(1 << L) - 1];
        for (int r = tid; r < nb; r += kConeBlock) {
            int lo = 0;
            for (int step = (1 << L) >> 1; step > 0; step >>= 1)
                if (lv[lo + step].base <= r) lo += step;
            const Range R = lv[lo];
            src_row[r] = R.start + R.lo + (r - R.base);
        }
    } else if (tid <= L) {
        M.nrows[tid] = U.node_size;
        M.doff[tid] = tid * U.node_size;
    }
    lds_barrier();
}

// Raw buffer resource over `bytes` bytes at p (gfx9 dword3: 32-bit data
// format); out-of-range buffer loads return 0 and stores are dropped.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buffer_rsrc(const void* p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(uni_ptr(const_cast<void*>(p)), (short)0, uni((int)bytes), 0x00020000);
}

// Fill of a unit's bottom level into dense rows (stride p): 16-byte aligned
// global loads into registers
// (issued before the descriptor build, so their latency overlaps it), then
// landed in LDS.  A whole unit is
// one contiguous block of rows; a tile unit is read row by row (its rows come
// from 2^L separate ranges).  Chunk k of a thread holds elements
// e[k] .. e[k] + 3 of the LDS segment starting at lo[k]; elements outside
// [0, len) are dropped.
struct Fill {
    float4 v[kFillChunks];
    int lo[kFillChunks], e[kFillChunks];
    int len;
    int al;             // whole units: the level buffer starts at data + al (LDS 16-B phase = global phase)
};

__device__ __forceinline__ void fill_issue(const ConeArgs& a, const UnitMeta& M, const UnitView& U,
                                           const int* src_row, int tid, Fill& F)
{
    const int p = U.p;
    const int nb = uni(M.nrows[U.levels]);
    const float* src;
    if (U.src == kSelLeaves) src = a.leaves + (uint64_t)U.trial * a.leaves_stride + U.src_off;
    else src = (U.src == kSelPing ? a.ping : a.pong) + (uint64_t)U.trial * a.buf_stride + U.buf_off;
    // transform blocks start 16-byte aligned and are padded to 4 floats
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(src, (((uint32_t)U.m * (uint32_t)p + 3u) & ~3u) * 4u);
    if (U.mode != kModeTile) {
        const uint32_t g0 = (uint32_t)U.node_start * (uint32_t)p;
        const int al = (int)(g0 & 3u);
        const int n = nb * p;
        const int nchunks = (n + al + 3) >> 2;
        F.len = n;
        F.al = al;
#pragma unroll
        for (int k = 0; k < kFillChunks; ++k) {
            const int c = tid + k * kConeBlock;
            F.lo[k] = 0;
            F.e[k] = c < nchunks ? 4 * c - al : n;
            // chunks past the level load from an out-of-range offset (the
            // buffer returns zeros; never landed): no exec-mask branch
            const uint32_t off = c < nchunks ? (g0 - (uint32_t)al + 4u * (uint32_t)c) * 4u : 0x80000000u;
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
            F.v[k] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                                 __uint_as_float(q[3]));
        }
    } else {
        const int amax = (p & 3) == 0 ? 0 : ((p & 1) == 0 ? 2 : 3);
        const int nch = (p + amax + 3) >> 2;                 // chunks per row (upper bound)
        const int totalc = nb * nch;
        F.len = p;
        F.al = 0;
        int r = tid / nch;
        int c = tid - r * nch;
        const int dr = kConeBlock / nch, dc = kConeBlock - dr * nch;
#pragma unroll
        for (int k = 0; k < kFillChunks; ++k) {
            const bool on = k * kConeBlock + tid < totalc;
            const int rr = min(r, nb - 1);
            const uint32_t g = (uint32_t)src_row[rr] * (uint32_t)p;
            const int al = (int)(g & 3u);
            const int e = 4 * c - al;
            F.lo[k] = rr * p;
            F.e[k] = on ? e : p;
            const uint32_t off = (on && e < p) ? (g - (uint32_t)al + 4u * (uint32_t)c) * 4u : 0x80000000u;
            const auto q = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0);
            F.v[k] = make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]),
                                 __uint_as_float(q[3]));
            r += dr;
            c += dc;
            if (c >= nch) {
                c -= nch;
                ++r;
            }
        }
    }
}

// Lands the staged chunks at base = data + F.al.  A chunk whose LDS address is
// 16-byte aligned and lies wholly inside its segment is one ds_write_b128
// (8x8-lane groups over 32 banks: conflict-free); the others (segment ends,
// tile rows of odd phase) are written element-wise.
__device__ __forceinline__ void fill_land(const Fill& F, float* base)
{
    const unsigned len = (unsigned)F.len;
    const int al = F.al;
#pragma unroll
    for (int k = 0; k < kFillChunks; ++k) {
        const int e = F.e[k];
        float* row = base + F.lo[k];
        const bool vec = e >= 0 && e + 3 < (int)len && ((F.lo[k] + e + al) & 3) == 0;
        if (vec) {
            *reinterpret_cast<float4*>(row + e) = F.v[k];
        } else {
            if ((unsigned)e < len) row[e] = F.v[k].x;
            if ((unsigned)(e + 1) < len) row[e + 1] = F.v[k].y;
            if ((unsigned)(e + 2) < len) row[e + 2] = F.v[k].z;
            if ((unsigned)(e + 3) < len) row[e + 3] = F.v[k].w;
        }
    }
}

// Row descriptor (head row, tail row, roll shift) of output row r at level
// l, as row indices of the level below; t = -1 for a carried leaf (size-1
// node).
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

__device__ __forceinline__ void row_desc(const UnitMeta& M, bool tile, int node_size, int l, int r, int p, int& h,
                                         int& t, int& sh)
{
    if (tile) {
        // the last of the level's 2^l ranges starting at or before r: l
        // halving steps (uniform trip count)
        const Range* lv = &M.ranges[(1 << l) - 1];
        int lo = 0;
        for (int step = (1 << l) >> 1; step > 0; step >>= 1)
            if (lv[lo + step].base <= r) lo += step;
        const Range R = lv[lo];
        const int u = R.lo + (r - R.base);
        const Range H = M.ranges[(2 << l) - 1 + 2 * lo];
        const Range T = M.ranges[(2 << l) + 2 * lo];
        const uint32_t hs = (uint32_t)R.size >> 1, ts = (uint32_t)R.size - hs;
        const int hh = (int)merge_index(merge_coef(hs, (uint32_t)R.size), (uint32_t)u);
        const int tt = (int)merge_index(merge_coef(ts, (uint32_t)R.size), (uint32_t)u);
        h = H.base + hh - H.lo;
        t = T.base + tt - T.lo;
        sh = mod_small(u - tt, p);
    } else {
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
}

// Packed row descriptor: head row | tail row << 10 | shift << 20 (tail row
// kCarried: a size-1 node carried unchanged).  Rows < 1023, shift < 4096.
constexpr uint32_t kCarried = 1023;

__device__ __forceinline__ uint32_t pack_desc(int h, int t, int sh)
{
    return (uint32_t)h | ((t < 0 ? kCarried : (uint32_t)t) << 10) | ((uint32_t)sh << 20);
}

// First table entry of level l: levels 0..l-1 precede it.
__device__ __forceinline__ int desc_offset(const UnitMeta& M, int l) { return uni(M.doff[l]); }

// Descriptors of every output row of levels 0..L-1 (thread per entry).
__device__ __forceinline__ void build_desc_table(const UnitMeta& M, uint32_t* desc, int entries, int p, int L,
                                                 bool tile, int node_size, int tid)
{
    for (int idx = tid; idx < entries; idx += kConeBlock) {
        int l = 0, r = idx;
        while (r >= uni(M.nrows[l])) {
            r -= uni(M.nrows[l]);
            ++l;
        }
        int h, t, sh;
        row_desc(M, tile, node_size, l, r, p, h, t, sh);
        desc[idx] = pack_desc(h, t, sh);
    }
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
__device__ __forceinline__ void merge_level_dense(const UnitMeta& M, const float* src, const uint32_t* desc,
                                                  bool use_table, int p, int l, bool tile, int node_size, int lane,
                                                  int wave, int nr, float (&v)[RW][SMAX])
{
    const int S = (p + 63) >> 6;
    // lane i unpacks the descriptor of the wave's i-th row into LDS float
    // offsets (head row, tail row + shift) and the shift; the row loop takes
    // them with v_readlane, so no per-row scalar unpacking or multiplies
    int ho = 0, to = 0, sh = 0, car = 0;
    if (lane < nr) {
        const int r = wave + kConeWaves * lane;
        uint32_t d;
        if (use_table) {
            d = desc[desc_offset(M, l) + r];
        } else {
            int h, t, s;
            row_desc(M, tile, node_size, l, r, p, h, t, s);
            d = pack_desc(h, t, s);
        }
        const uint32_t tc = (d >> 10) & 1023u;
        sh = (int)(d >> 20);
        ho = (int)(d & 1023u) * p;
        to = (tc == kCarried ? 0 : (int)tc * p) + sh;
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
__device__ __forceinline__ void merge_level2_dense(const UnitMeta& M, const float* src, const uint32_t* desc,
                                                   bool use_table, int p, int l, bool tile, int node_size, int lane,
                                                   int wave, int nr, float (&v)[RW][SMAX])
{
    const int S = (p + 63) >> 6;
    int o0 = 0, o1 = 0, o2 = 0, o3 = 0, s1 = 0, s2 = 0, s3 = 0;
    if (lane < nr) {
        const int r = wave + kConeWaves * lane;
        uint32_t d0, dh, dt;
        if (use_table) {
            d0 = desc[desc_offset(M, l) + r];
            const int b1 = desc_offset(M, l + 1);
            dh = desc[b1 + (int)(d0 & 1023u)];
            dt = desc[b1 + (int)((d0 >> 10) & 1023u)];
        } else {
            int h, t, sh;
            row_desc(M, tile, node_size, l, r, p, h, t, sh);
            d0 = pack_desc(h, t, sh);
            row_desc(M, tile, node_size, l + 1, h, p, h, t, sh);
            dh = pack_desc(h, t, sh);
            row_desc(M, tile, node_size, l + 1, (int)((d0 >> 10) & 1023u), p, h, t, sh);
            dt = pack_desc(h, t, sh);
        }
        const int sh = (int)(d0 >> 20), sH = (int)(dh >> 20), sT = (int)(dt >> 20);
        int sTT = sh + sT;
        sTT = sTT >= p ? sTT - p : sTT;
        o0 = (int)(dh & 1023u) * p;
        o1 = (int)((dh >> 10) & 1023u) * p + sH;
        o2 = (int)(dt & 1023u) * p + sh;
        o3 = (int)((dt >> 10) & 1023u) * p + sTT;
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

// kPack2 variant (p <= 32): register row i of a wave holds two output rows,
// the wave's row 2i in lanes 0-31 and row 2i + 1 in lanes 32-63 (bin j =
// lane & 31), so a wave instruction does the work of two rows instead of
// leaving 32-48 of its 64 lanes idle.  Each half takes its row's offsets with
// its own v_readlane and a select; otherwise as merge_level_dense (same
// additions, same -0.0 carry masking).
template <int RW, bool CARRIED>
__device__ __forceinline__ void merge_level_packed(const UnitMeta& M, const float* src, const uint32_t* desc,
                                                   bool use_table, int p, int l, bool tile, int node_size, int lane,
                                                   int wave, int nr, float (&v)[RW][1])
{
    int ho = 0, to = 0, sh = 0, car = 0;
    if (lane < nr) {
        const int r = wave + kConeWaves * lane;
        uint32_t d;
        if (use_table) {
            d = desc[desc_offset(M, l) + r];
        } else {
            int h, t, s;
            row_desc(M, tile, node_size, l, r, p, h, t, s);
            d = pack_desc(h, t, s);
        }
        const uint32_t tc = (d >> 10) & 1023u;
        sh = (int)(d >> 20);
        ho = (int)(d & 1023u) * p;
        to = (tc == kCarried ? 0 : (int)tc * p) + sh;
        car = tc == kCarried;
    }
    const bool hi = lane >= 32;
    const int j = lane & 31;
    const lds_cptr l1 = (lds_cptr)src + j;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        const int hoi = hi ? __builtin_amdgcn_readlane(ho, 2 * i + 1) : __builtin_amdgcn_readlane(ho, 2 * i);
        const int toi = hi ? __builtin_amdgcn_readlane(to, 2 * i + 1) : __builtin_amdgcn_readlane(to, 2 * i);
        const int si = hi ? __builtin_amdgcn_readlane(sh, 2 * i + 1) : __builtin_amdgcn_readlane(sh, 2 * i);
        uint32_t keep = 0xFFFFFFFFu, neg0 = 0u;
        if (CARRIED) {
            const int ci = hi ? __builtin_amdgcn_readlane(car, 2 * i + 1) : __builtin_amdgcn_readlane(car, 2 * i);
            keep = ci ? 0u : 0xFFFFFFFFu;
            neg0 = ~keep & 0x80000000u;
        }
        const lds_cptr hrow = l1 + hoi;
        lds_cptr ta = l1 + toi;
        lds_cptr tw = ta - p;
        asm("" : "+v"(ta), "+v"(tw));
        float x = lds_ld(j + si >= p ? tw : ta);
        if (CARRIED) x = __uint_as_float((__float_as_uint(x) & keep) | neg0);
        v[i][0] = __fadd_rn(hrow[0], x);
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
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][k]), rs, (int)o, 0, 0);
                } else if (64 * (k + 1) <= p || (k < S && lane + 64 * k < p)) {
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][k]), rs,
                                                          (int)(ob + 256u * (uint32_t)k), 0, 0);
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

// kPack2 store / write-back: lane half h of register row i is the wave's row
// 2i + h; halves past nr and bins past p store out of the buffer's range
// (dropped) or to the LDS dummy word.
template <int RW>
__device__ __forceinline__ void store_rows_packed(const float (&v)[RW][1], int p, int lane, int wave, int nr,
                                                  __amdgpu_buffer_rsrc_t rs, uint32_t st_o0)
{
    const int hi = lane >> 5, j = lane & 31;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (2 * i < nr) {
            const int k = 2 * i + hi;
            const uint32_t o = (k < nr && j < p) ? st_o0 + (uint32_t)((wave + kConeWaves * k) * p + j) * 4u
                                                 : 0x80000000u;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v[i][0]), rs, (int)o, 0, 0);
        }
    }
}

template <int RW>
__device__ __forceinline__ void write_rows_packed(float* base, float* dummy, const float (&v)[RW][1], int p, int lane,
                                                  int wave, int nr)
{
    const int hi = lane >> 5, j = lane & 31;
#pragma unroll
    for (int i = 0; i < RW; ++i) {
        if (2 * i < nr) {
            const int k = 2 * i + hi;
            *((k < nr && j < p) ? base + (wave + kConeWaves * k) * p + j : dummy) = v[i][0];
        }
    }
}

// All merge levels of one unit, deepest first, in place in the dense rows
// at `base`.  SMAX >= ceil(p/64) slots per row, RW rows per wave
// (lds_row_capacity(p, SMAX) guarantees ceil(rows/8) <= RW at every level).
// Each level's outputs are staged in registers between two barriers, then
// written back.  With `st` set (a non-final pass), the output level goes from
// the staging registers straight to global memory instead of back into LDS.
template <int SMAX, int RW>
__device__ __forceinline__ void merge_levels(const UnitMeta& M, float* base, const uint32_t* desc, bool use_table,
                                             int p, int L, bool tile, int node_size, int tid, bool st,
                                             __amdgpu_buffer_rsrc_t rs, uint32_t st_o0, uint32_t flags, float* dummy)
{
    const int lane = tid & 63, wave = tid >> 6;
    // deepest first; two levels per step (merge_level2_dense) once no level
    // below the step's output holds size-1 nodes, single steps before that
    // and for a last odd level
    const bool fuse = (flags & kConeFuse2) && SMAX != kPack2;
    for (int l = L - 1; l >= 0;) {
        // size-1 nodes exist at depth l only in whole units with node_size >> l < 2
        const bool two = fuse && l >= 1 && (tile || (node_size >> l) >= 2);
        const int lo = two ? l - 1 : l;          // output level of this step
        const int orows = uni(M.nrows[lo]);
        const int nr = uni(orows > wave ? (orows - wave + kConeWaves - 1) / kConeWaves : 0);
        constexpr int S = slot_count(SMAX);
        float v[RW][S];
        const bool carried = !tile && (node_size >> l) < 2;
        if constexpr (SMAX == kPack2) {
            if (carried)
                merge_level_packed<RW, true>(M, base, desc, use_table, p, l, tile, node_size, lane, wave, nr, v);
            else
                merge_level_packed<RW, false>(M, base, desc, use_table, p, l, tile, node_size, lane, wave, nr, v);
        } else {
            if (two)
                merge_level2_dense<S, RW>(M, base, desc, use_table, p, lo, tile, node_size, lane, wave, nr, v);
            else if (carried)
                merge_level_dense<S, RW, true>(M, base, desc, use_table, p, l, tile, node_size, lane, wave, nr, v);
            else
                merge_level_dense<S, RW, false>(M, base, desc, use_table, p, l, tile, node_size, lane, wave, nr, v);
        }
        l = lo - 1;
        if (lo == 0 && st) {
            if constexpr (SMAX == kPack2) store_rows_packed<RW>(v, p, lane, wave, nr, rs, st_o0);
            else store_rows<S, RW>(v, p, lane, wave, nr, rs, st_o0);
            return;
        }
        if (!(flags & kConeDiagNoBarrier)) lds_barrier();
        if (!(flags & kConeDiagNoWrite)) {
            if constexpr (SMAX == kPack2) write_rows_packed<RW>(base, dummy, v, p, lane, wave, nr);
            else write_rows<S, RW>(base, dummy, v, p, lane, wave, nr);
        }
        if (!(flags & kConeDiagNoBarrier)) lds_barrier();
    }
}

// Fused boxcar S/N (snr.hpp:37-65) of the output rows s < rows_eval held in LDS
// (row stride p): G lanes per row, each lane a chunk of c <= CH columns held
// in registers (c odd: the G chunks of a row start on distinct banks).
// fp64 prefix: sequential in the chunk + log2(G)-step segmented scan
// (kernels.hpp:73-86).  For G <= 16 (one DPP row) the scan, the per-width
// max and the neighbour exchange run on DPP row shifts (VALU, no LDS
// round trip); each lane then reads its window c[j0 .. j0 + CH + kSnrWin)
// (the wrap c[p + j] = c[j] + sum applied once per element) and evaluates
// every width w <= kSnrWin from registers.  Wider rows and wider widths use
// the general path (shuffles, LDS reads per width).
constexpr int kSnrWin = 12;
// S/N chunk columns per lane held in registers (and the window path), by the
// register budget of the block size
constexpr int kSnrMaxChunk = kConeBlock >= 1024 || kConeWgsPerCu == 3 ? 9 : 17;

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, true));
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

// Inclusive scan over each G-lane group (G = 8 .. 64): row_shr steps inside
// 16-lane rows, then row_bcast:15 / row_bcast:31 across rows.  The partial
// sums start at +0.0 and are never -0.0, so adding the +0.0 that masked
// lanes receive is an exact no-op.
template <int G>
__device__ __forceinline__ double seg_scan_dpp(double v, int lane)
{
    const int g = lane & (G < 16 ? G - 1 : 15);     // position inside the group's part of the 16-lane row
    double y = dpp_d<0x111>(v);
    v = g >= 1 ? v + y : v;
    y = dpp_d<0x112>(v);
    v = g >= 2 ? v + y : v;
    y = dpp_d<0x114>(v);
    v = g >= 4 ? v + y : v;
    if (G >= 16) {
        y = dpp_d<0x118>(v);
        v = g >= 8 ? v + y : v;
    }
    if (G >= 32) v = v + dpp_d_rows<0x142, 0xA>(v);   // rows 1, 3 += lane 15 of rows 0, 2
    if (G >= 64) v = v + dpp_d_rows<0x143, 0xC>(v);   // rows 2, 3 += lane 31
    return v;
}

// row_shr:d keeping the lane's own value where the source is outside the
// 16-lane row (bound_ctrl off, old = v)
template <int CTRL>
__device__ __forceinline__ float dpp_keep(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}

template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_keep_rows(float v)
{
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWS, 0xF, false));
}

// max over the G lanes of a group, valid in lane g == G - 1.  fmaxf never
// returns a NaN operand over a number, as diff_max's comparison.
template <int G>
__device__ __forceinline__ float seg_max_dpp(float v, int lane)
{
    if constexpr (G >= 16) {
        v = fmaxf(v, dpp_keep<0x111>(v));
        v = fmaxf(v, dpp_keep<0x112>(v));
        v = fmaxf(v, dpp_keep<0x114>(v));
        v = fmaxf(v, dpp_keep<0x118>(v));
        if (G >= 32) v = fmaxf(v, dpp_keep_rows<0x142, 0xA>(v));
        if (G >= 64) v = fmaxf(v, dpp_keep_rows<0x143, 0xC>(v));
    } else {
        const int g = lane & 7;
        float y = dpp_keep<0x111>(v);
        v = g >= 1 ? fmaxf(v, y) : v;
        y = dpp_keep<0x112>(v);
        v = g >= 2 ? fmaxf(v, y) : v;
        y = dpp_keep<0x114>(v);
        v = g >= 4 ? fmaxf(v, y) : v;
    }
    return v;
}

// diff_max (kernels.hpp:50-60) of width W over the lane's columns (cp[i] =
// +inf past the lane's chunk, so those differences are -inf)
template <int CH, int W>
__device__ __forceinline__ float window_max(const float (&z)[CH + kSnrWin], const float (&cp)[CH])
{
    float dm = -INFINITY;
#pragma unroll
    for (int i = 0; i < CH; ++i) dm = fmaxf(dm, __fsub_rn(z[i + W], cp[i]));
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

#ifdef RT_STAMPS
#define RT_SNR_MARK(i)                                                           \
    do {                                                                         \
        if (tid == 0 && base == 0 && tl) tl[i] = __builtin_amdgcn_s_memtime();   \
    } while (0)
#else
#define RT_SNR_MARK(i) do { } while (0)
#endif

template <int CH, int G>
__device__ __forceinline__ void snr_rows(const ConeArgs& a, const UnitView& U, float* data, int q, const int* wl,
                                         int nev, int c, int tid, const float* whb, unsigned long long* tl)
{
    constexpr bool kDpp = true;
    const int lane = tid & 63;
    const int p = U.p;
    const int g = lane & (G - 1);
    int j0 = min(g * c, p);
    int cnt = min(j0 + c, p) - j0;                // columns of this lane (may be 0)
    const int owner = (p - 1) / c;
    const int rows_per_pass = kConeBlock / G;
    const int writer = kDpp ? G - 1 : 0;
    const uint32_t nw = a.num_widths;
    float* snr = a.snr + (uint64_t)U.trial * a.snr_stride + (U.snr_row + (uint64_t)U.s0) * (uint64_t)nw;
    const __amdgpu_buffer_rsrc_t srs = buffer_rsrc(snr, (uint32_t)nev * nw * 4u);
    for (int base = 0; base < nev; base += rows_per_pass) {
        // opaque per row pass: the column masks (i < cnt, j0 + k >= p) are
        // recomputed by one v_cmp each instead of being hoisted out of the
        // loop into SGPR pairs that spill (two v_readlane per use)
        asm volatile("" : "+v"(j0), "+v"(cnt));
        const int r = base + (tid / G);
        const bool active = r < nev;
        float* row = data + min(r, nev - 1) * q + j0;
        float cp[CH];
        // every lane reads CH columns at immediate offsets (past its chunk:
        // the next chunk, the next row or the LDS pad), masked to 0
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const float x = row[i];
            cp[i] = i < cnt ? x : 0.0f;
        }
        // fp64 prefix: the masked columns add +0.0 (the partial sums start at
        // +0.0 and are never -0.0, so the additions are exact no-ops)
        double part = 0.0;
#pragma unroll
        for (int i = 0; i < CH; ++i) part = part + (double)cp[i];
        double acc;
        if constexpr (kDpp) {
            const double incl = seg_scan_dpp<G>(part, lane);
            acc = dpp_d<0x138>(incl);               // wave_shr:1 -- lane g takes lane g - 1
        } else {
            double incl = part;
            for (int d = 1; d < G; d <<= 1) {
                const double y = __shfl_up(incl, d, G);
                if (g >= d) incl += y;
            }
            acc = __shfl_up(incl, 1, G);
        }
        if (g == 0) acc = 0.0;
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            acc = acc + (double)cp[i];
            cp[i] = (float)acc;
        }
        const float sum = __shfl((float)acc, owner, G);
        {
            // columns past the lane's chunk (and rows past nev) go to a dummy
            // word in the LDS pad: an address select instead of exec masks
            float* const dummy = data + kLdsDataFloats + 4 + lane;
#pragma unroll
            for (int i = 0; i < CH; ++i) *((active && i < cnt) ? row + i : dummy) = cp[i];
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) cp[i] = i < cnt ? cp[i] : INFINITY;
        RT_SNR_MARK(7);
        lds_barrier();                        // prefix rows visible to all lanes
        RT_SNR_MARK(8);
        const float* crow = data + min(r, nev - 1) * q;
        // one lane per row stores; the others store out of the buffer's
        // range, which drops them (no exec-mask save/restore)
        const uint32_t so = (active && g == writer) ? (uint32_t)r * nw * 4u : 0x80000000u;
        auto emit = [&](uint32_t iw, int w, float dmax) {
            (void)w;
            dmax = seg_max_dpp<G>(dmax, lane);
            // h + b and b of this width (per unit, in LDS: uniform reads)
            const float hpb = __int_as_float(uni(__float_as_int(whb[2 * iw])));
            const float b = __int_as_float(uni(__float_as_int(whb[2 * iw + 1])));
            const float v = (hpb * dmax - b * sum) / U.stdnoise;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), srs, (int)(so + iw * 4u), 0, 0);
        };
        if constexpr (CH <= kSnrMaxChunk) {
            // widths <= kSnrWin from the register window c[j0 .. j0 + CH + kSnrWin)
            float z[CH + kSnrWin];
            {
                // two opaque bases (row and row - p), slot offsets immediate
                lds_cptr za = (lds_cptr)(crow + j0);
                lds_cptr zb = za - p;
                asm("" : "+v"(za), "+v"(zb));
#pragma unroll
                for (int k = 0; k < CH + kSnrWin; ++k) {
                    const bool wrap = j0 + k >= p;
                    const float va = za[k], vb = zb[k];
                    z[k] = wrap ? __fadd_rn(vb, sum) : va;
                }
            }
            RT_SNR_MARK(9);
            for (uint32_t iw = 0; iw < nw; ++iw) {
                const int w = uni(wl[iw]);
                if (w <= kSnrWin) emit(iw, w, window_dispatch<CH>(w, z, cp));
            }
        }
        // wider widths: the window c[j0 + w ..] read from LDS per width
        for (uint32_t iw = 0; iw < nw; ++iw) {
            const int w = uni(wl[iw]);
            if (CH <= kSnrMaxChunk && w <= kSnrWin) continue;
            float dmax = -INFINITY;
            const int last = max(cnt - 1, 0);
            float lv[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int k = j0 + min(t, last) + w;
                lv[t] = crow[k >= p ? k - p : k];
            }
#pragma unroll
            for (int i = 0; i < CH; ++i) {
                const bool wrap = j0 + min(i, last) + w >= p;
                const float ck = wrap ? __fadd_rn(lv[i], sum) : lv[i];
                dmax = fmaxf(dmax, __fsub_rn(ck, cp[i]));  // diff_max, kernels.hpp:50-60
            }
            emit(iw, w, dmax);
        }
        RT_SNR_MARK(10);
    }
}

// Phase-bin range [lo, hi] a cone kernel variant runs, and the S/N lane-group
// size G of a row of p bins: the epilogue instantiates only the row shapes its
// variant can meet (smaller kernels; the rest is compiled out).
constexpr int snr_group(int p)
{
    int G = 8;
    while (G < 64 && ((((p + G - 1) / G) | 1) > kSnrMaxChunk)) G <<= 1;
    return G;
}
constexpr int variant_pmin(int smax) { return smax == kPack2 ? 1 : (smax <= 5 ? 64 * (smax - 1) + 1 : (smax == 8 ? 321 : (smax == 16 ? 513 : 1025))); }
constexpr int variant_pmax(int smax) { return smax == kPack2 ? 32 : (smax <= 5 ? 64 * smax : (smax == 8 ? 512 : (smax == 16 ? 1024 : 64 * kMaxSlots))); }
constexpr bool variant_has_group(int smax, int G)
{
    return snr_group(variant_pmin(smax)) <= G && G <= snr_group(variant_pmax(smax));
}

template <int SMAX>
__device__ __forceinline__ void snr_epilogue(const ConeArgs& a, const UnitView& U, float* data, int q, const int* wl,
                                             int nrows, int tid, float* whb, unsigned long long* tl)
{
    const int lane = tid & 63, wave = tid >> 6;
    const int p = U.p;
    const int nev = (int)min((int64_t)nrows, (int64_t)U.rows_eval - (int64_t)U.s0);
    if (nev <= 0) return;
    // per-width constants of the S/N formula (snr.hpp:37-65), once per unit;
    // visible to every wave after the first barrier of the row passes
    if (tid < (int)a.num_widths) {
        const int w = wl[tid];
        const float h = sqrtf((float)(p - w) / (float)(p * w));
        const float b = (float)w / (float)(p - w) * h;
        whb[2 * tid] = h + b;
        whb[2 * tid + 1] = b;
    }
    // G lanes per row: the smallest power of two >= 8 whose chunks fit
    // kSnrMaxChunk columns (17 at G = 64); chunk lengths odd
    int G = 8;
    while (G < 64 && (((p + G - 1) / G) | 1) > kSnrMaxChunk) G <<= 1;
    int c = (p + G - 1) / G;
    if (c < kSnrChunk) c |= 1;
    const uint32_t nw = a.num_widths;
    float* snr = a.snr + (uint64_t)U.trial * a.snr_stride + (U.snr_row + (uint64_t)U.s0) * (uint64_t)nw;
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
// gets its own register allocation.  min 4 waves per SIMD: <= 128 VGPRs, two
// workgroups per CU.
template <int SMAX, int RWT = 0>
__global__ __launch_bounds__(kConeBlock, kConeWavesPerSimd) void cone_kernel(ConeArgs a)
{
    constexpr int RW = RWT ? RWT : merge_rows_per_wave(SMAX);   // register rows per wave
#ifdef RT_STAMPS
    unsigned long long tl[kStampMarks] = {};
    tl[0] = __builtin_amdgcn_s_memtime();
#endif
    __shared__ __attribute__((aligned(16))) float data[kLdsDataFloats + kLdsPadFloats];
    __shared__ UnitMeta M;
    __shared__ uint32_t desc[kDescEntries];
    __shared__ int src_row[kMaxRows];
    __shared__ int wl[kMaxWidths];   // boxcar widths: LDS reads never wait on the S/N stores in flight
    __shared__ float whb[2 * kMaxWidths];   // S/N: h + b and b per width

    const int tid = threadIdx.x;
    // grid (items, trials): no division to split a flat unit index
    const int item = (int)blockIdx.x, trial = (int)blockIdx.y;
    if (item >= (int)a.num_items || trial >= (int)a.batch) return;
    const int u = trial * (int)a.num_items + item;   // unit record index (diagnostic stamps)
    (void)u;
    if (tid < (int)a.num_widths) wl[tid] = (int)a.widths[tid];   // visible after setup's barriers
    setup_unit(a, item, trial, M, src_row, tid);
    RT_MARK(1);
    const UnitView U = read_view(M);
    const int p = U.p;
    const int L = U.levels;
    const bool tile = U.mode == kModeTile;
    bool ok = uni(M.nrows[L]) * p <= kLdsDataFloats;
    // SMAX <= 5 variants assume rows of exactly SMAX slots (unmasked full slots)
    // (kPack2 runs exactly the p <= 32 rows)
    ok = ok && ((SMAX <= 5 || SMAX == kPack2) ? merge_slots((uint32_t)p) == SMAX
                                              : (merge_slots((uint32_t)p) <= SMAX && merge_slots((uint32_t)p) != kPack2));
    for (int l = 0; l <= L; ++l)
        ok = ok && uni(M.nrows[l]) <= lds_row_capacity((uint32_t)p, SMAX) &&
             uni(M.nrows[l]) <= kConeWaves * RW * row_pack(SMAX);
    if (!ok) {
        if (tid == 0 && a.error_flag) atomicOr(a.error_flag, 1);
        return;
    }
    Fill F;
    fill_issue(a, M, U, src_row, tid, F);
    RT_MARK(2);
    // row descriptors of every level while the loads are in flight
    const int entries = desc_offset(M, L);
    const bool use_table = entries <= kDescEntries;
    if (use_table && !(a.flags & kConeDiagNoDesc)) build_desc_table(M, desc, entries, p, L, tile, U.node_size, tid);
    RT_MARK(3);
    float* const base = data + uni(F.al);   // the filled level: dense rows, stride p
    if (!(a.flags & kConeDiagNoLand)) fill_land(F, base);
    else if (F.v[0].x == 12345.678f) base[tid] = F.v[0].y;   // keep the loads alive
    lds_barrier();
    RT_MARK(4);
    // ---- merge levels, deepest first; a non-final pass stores its output
    // level straight from registers (st), a final pass keeps it in LDS for
    // the S/N epilogue
    const bool st = U.dst != kSelSnr;
    const bool st_regs = st && (a.flags & kConeStoreFromRegs);
    const float* dst = (U.dst == kSelPing ? a.ping : a.pong) + (uint64_t)U.trial * a.buf_stride + U.buf_off;
    const __amdgpu_buffer_rsrc_t rs = buffer_rsrc(dst, (((uint32_t)U.m * (uint32_t)p + 3u) & ~3u) * 4u);
    const uint32_t o0 = (uint32_t)(U.node_start + U.s0) * (uint32_t)p * 4u;
    if (L > 0 && !(a.flags & kConeDiagNoMerge))
        merge_levels<SMAX, RW>(M, base, desc, use_table, p, L, tile, U.node_size, tid, st_regs,
                                                      rs, o0, a.flags, data + kLdsDataFloats + 4 + (tid & 63));
    RT_MARK(5);
    const int n0 = uni(M.nrows[0]);
    // the output level, in place in the dense rows at base
    float* const obuf = base;
    const int ostride = p;
    if (st) {
        if (L == 0 || !st_regs) {
            // ---- store the output level from LDS (a single leaf row, or A/B)
            for (int r = 0; r < n0; ++r)
                for (int j = tid; j < p; j += kConeBlock)
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(obuf[r * ostride + j]), rs,
                                                          (int)(o0 + (uint32_t)(r * p + j) * 4u), 0, 0);
        }
    } else {
#ifdef RT_STAMPS
        if (!(a.flags & kConeDiagNoSnr)) snr_epilogue<SMAX>(a, U, obuf, ostride, wl, n0, tid, whb, tl);
#else
        if (!(a.flags & kConeDiagNoSnr)) snr_epilogue<SMAX>(a, U, obuf, ostride, wl, n0, tid, whb, nullptr);
#endif
    }
#ifdef RT_STAMPS
    if (tid == 0 && a.stamps) {
        RT_MARK(6);
        unsigned long long* e = a.stamps + (uint64_t)kStampRecWords * (uint64_t)u;
        const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (31 << 11));     // HW_REG_HW_ID
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg(20 | (31 << 11));   // HW_REG_XCC_ID
        e[0] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
#pragma unroll
        for (int i = 0; i < kStampMarks; ++i) e[1 + i] = tl[i];
        e[1 + kStampMarks] = (unsigned long long)p | ((unsigned long long)L << 16) |
                             ((unsigned long long)U.mode << 24) | ((unsigned long long)n0 << 32) |
                             ((unsigned long long)(U.dst == kSelSnr) << 48);
    }
#endif
}

hipError_t launch_cone(const ConeArgs& args, uint32_t smax, uint32_t rw, hipStream_t s)
{
    if (!args.num_items || !args.batch) return hipSuccess;
    const dim3 g(args.num_items, args.batch), b(kConeBlock);
    switch (smax) {
    case 1:
        switch (rw) {
        case 12: hipLaunchKernelGGL((cone_kernel<1, 12>), g, b, 0, s, args); break;
        case 16: hipLaunchKernelGGL((cone_kernel<1, 16>), g, b, 0, s, args); break;
        case 20: hipLaunchKernelGGL((cone_kernel<1, 20>), g, b, 0, s, args); break;
        default: hipLaunchKernelGGL(cone_kernel<1>, g, b, 0, s, args); break;
        }
        break;
    case 2: hipLaunchKernelGGL(cone_kernel<2>, g, b, 0, s, args); break;
    case 3: hipLaunchKernelGGL(cone_kernel<3>, g, b, 0, s, args); break;
    case 4:
        switch (rw) {
        case 5: hipLaunchKernelGGL((cone_kernel<4, 5>), g, b, 0, s, args); break;
        case 6: hipLaunchKernelGGL((cone_kernel<4, 6>), g, b, 0, s, args); break;
        case 7: hipLaunchKernelGGL((cone_kernel<4, 7>), g, b, 0, s, args); break;
        case 8: hipLaunchKernelGGL((cone_kernel<4, 8>), g, b, 0, s, args); break;
        default: hipLaunchKernelGGL(cone_kernel<4>, g, b, 0, s, args); break;
        }
        break;
    case 5:
        switch (rw) {
        case 5: hipLaunchKernelGGL((cone_kernel<5, 5>), g, b, 0, s, args); break;
        case 6: hipLaunchKernelGGL((cone_kernel<5, 6>), g, b, 0, s, args); break;
        case 7: hipLaunchKernelGGL((cone_kernel<5, 7>), g, b, 0, s, args); break;
        case 8: hipLaunchKernelGGL((cone_kernel<5, 8>), g, b, 0, s, args); break;
        default: hipLaunchKernelGGL(cone_kernel<5>, g, b, 0, s, args); break;
        }
        break;
    case 8: hipLaunchKernelGGL(cone_kernel<8>, g, b, 0, s, args); break;
    case 16: hipLaunchKernelGGL(cone_kernel<16>, g, b, 0, s, args); break;
    case kMaxSlots: hipLaunchKernelGGL(cone_kernel<kMaxSlots>, g, b, 0, s, args); break;
    case kPack2: hipLaunchKernelGGL(cone_kernel<kPack2>, g, b, 0, s, args); break;
    default: return hipErrorInvalidValue;
    }
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
