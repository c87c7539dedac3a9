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
// One workgroup = one ConeItem: `levels` merge levels of the FFA recursion for
// the rows of one tile (or one whole node), held entirely in LDS.
//
//   level l (0 = target node, `levels` = deepest) is a packed list of row
//   ranges, one per node of the split tree at that depth that the tile depends
//   on.  Each merge step computes level l from level l+1 into registers
//   (flattened over rows x phase bins, 34 values per thread), then overwrites
//   the LDS level buffer.  The merge is transforms.hpp:13-27:
//       out[u][j] = H[h(u)][j] + T[t(u)][(j + u - t(u)) mod p]
//
// LDS: 136 KiB level buffer + 8 KiB row descriptors + range tree = ~147 KiB,
// i.e. one workgroup per CU.
struct Range {          // rows [lo, hi] of one node of the split tree
    int size;           // rows of the node
    int lo, hi;         // node-local rows
    int start;          // first row of the node within the transform
    int base;           // first LDS row of this range in its level's packed layout
    int child;          // index of the first child range (next level)
};

__device__ __forceinline__ int div_rows(int e, int p, float inv_p)
{
    int r = (int)((float)e * inv_p);
    if (r * p > e) --r;
    else if ((r + 1) * p <= e) ++r;
    return r;
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

// Index of the last range in [first, first+count) whose base <= r.
__device__ __forceinline__ int find_range(const Range* ranges, int first, int count, int r)
{
    int lo = first, hi = first + count - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (ranges[mid].base <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Diagnostic build only (make stamps, -DRT_STAMPS): thread 0 adds the cycles of
// each phase of the item to a.stamps[phase] (s_memtime; phases end at barriers).
#ifdef RT_STAMPS
#define RT_STAMP(i)                                                              \
    do {                                                                         \
        if (tid == 0) {                                                          \
            const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
            atomicAdd(&a.stamps[i], t_ - t_stamp);                               \
            t_stamp = t_;                                                        \
        }                                                                        \
    } while (0)
#else
#define RT_STAMP(i) do { } while (0)
#endif

__global__ __launch_bounds__(kConeBlock) void cone_kernel(ConeArgs a)
{
#ifdef RT_STAMPS
    unsigned long long t_stamp = __builtin_amdgcn_s_memtime();
#endif
    __shared__ float4 data4[kLdsDataFloats / 4];   // 16-byte aligned level buffer
    float* const data = reinterpret_cast<float*>(data4);
    __shared__ int2 desc[kMaxRows];
    __shared__ Range ranges[kMaxRanges];
    __shared__ int lv_first[kMaxTileLevels + 1];
    __shared__ int lv_count[kMaxTileLevels + 1];
    __shared__ int lv_rows[kMaxTileLevels + 1];
    __shared__ int wl[kMaxWidths];           // boxcar widths, staged in LDS (DS ops wait by count)

    const ConeItem it = a.items[blockIdx.x];
    const FfaXform X = a.xf[it.xform];
    const int p = (int)X.p;
    const float inv_p = 1.0f / (float)p;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int L = it.levels;
    const bool tile = it.mode == kModeTile;
    const uint64_t trial = blockIdx.y;
    if (tid < kMaxWidths) wl[tid] = (int)a.widths[tid];
    const int p4 = lds_row_stride((uint32_t)p);          // LDS row stride (floats)
    const int qpr = p4 >> 2;                               // quads per LDS row
    // LDS row of -0.0f after the largest level the planner allows (lds_row_capacity)
    const int zrow = (kLdsDataFloats / p4 - 1) * p4;

    const float* src;
    if (it.src == kSelLeaves) src = a.leaves + trial * a.leaves_stride + X.src_off;
    else src = (it.src == kSelPing ? a.ping : a.pong) + trial * a.buf_stride + X.buf_off;

    int nrows;
    if (tile) {
        // ---- dependency cone of the tile: top-down range tree, one lane per range (wave 0)
        if (wave == 0) {
            if (lane == 0) {
                Range r0;
                r0.size = (int)it.node_size;
                r0.lo = (int)it.s0;
                r0.hi = (int)it.s1 - 1;
                r0.start = (int)it.node_start;
                r0.base = 0;
                r0.child = 0;
                ranges[0] = r0;
                lv_first[0] = 0;
                lv_count[0] = 1;
                lv_rows[0] = r0.hi - r0.lo + 1;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            int first = 0, count = 1;
            for (int l = 0; l < L; ++l) {
                const int nfirst = first + count;
                Range r, h, t;
                int nchild = 0, c0 = 0, c1 = 0;
                if (lane < count) {
                    r = ranges[first + lane];
                    if (r.size <= 1) {          // a leaf is carried unchanged
                        nchild = 1;
                        h = r;
                        c0 = r.hi - r.lo + 1;
                    } else {
                        nchild = 2;
                        const int sh = r.size >> 1, st = r.size - sh;
                        const float kh = merge_coef((uint32_t)sh, (uint32_t)r.size);
                        const float kt = merge_coef((uint32_t)st, (uint32_t)r.size);
                        h.size = sh;
                        h.lo = (int)merge_index(kh, (uint32_t)r.lo);
                        h.hi = (int)merge_index(kh, (uint32_t)r.hi);
                        h.start = r.start;
                        t.size = st;
                        t.lo = (int)merge_index(kt, (uint32_t)r.lo);
                        t.hi = (int)merge_index(kt, (uint32_t)r.hi);
                        t.start = r.start + sh;
                        c0 = h.hi - h.lo + 1;
                        c1 = t.hi - t.lo + 1;
                    }
                }
                const int pos_incl = wave_incl_scan_int(nchild, lane);
                const int rows_incl = wave_incl_scan_int(c0 + c1, lane);
                const int total = __shfl(pos_incl, 63, 64);
                const int total_rows = __shfl(rows_incl, 63, 64);
                if (lane < count) {
                    const int pos = nfirst + pos_incl - nchild;
                    const int rbase = rows_incl - (c0 + c1);
                    h.base = rbase;
                    h.child = 0;
                    ranges[pos] = h;
                    if (nchild == 2) {
                        t.base = rbase + c0;
                        t.child = 0;
                        ranges[pos + 1] = t;
                    }
                    ranges[first + lane].child = pos;
                }
                if (lane == 0) {
                    lv_first[l + 1] = nfirst;
                    lv_count[l + 1] = total;
                    lv_rows[l + 1] = total_rows;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                first = nfirst;
                count = total;
            }
        }
        __syncthreads();
        nrows = lv_rows[L];
        if (nrows > kMaxRows || nrows * p4 > zrow) {
            if (tid == 0 && a.error_flag) atomicOr(a.error_flag, 1);
            return;
        }
        // ---- bottom level: source row of every LDS row, then the load
        const int bf = lv_first[L], bc = lv_count[L];
        for (int r = tid; r < nrows; r += kConeBlock) {
            const Range R = ranges[find_range(ranges, bf, bc, r)];
            desc[r].x = R.start + R.lo + (r - R.base);
        }
        __syncthreads();
    } else {
        nrows = (int)it.node_size;
        if (nrows > kMaxRows || nrows * p4 > zrow) {
            if (tid == 0 && a.error_flag) atomicOr(a.error_flag, 2);
            return;
        }
    }
    RT_STAMP(0);
    // ---- fill the bottom level with 16-byte loads.  Row r is global row
    // grow(r), floats [grow*p, grow*p + p) of a 16-byte aligned buffer, covered
    // by at most nch aligned float4 chunks: chunk c holds elements
    // e = 4c + j - al (al = grow*p & 3), kept when 0 <= e < p.  Every thread
    // issues all its loads before the first LDS write.
    {
        const int amax = (p & 3) == 0 ? 0 : ((p & 1) == 0 ? 2 : 3);
        const int nch = (p + amax + 3) >> 2;                 // chunks per row (upper bound)
        const int totalc = nrows * nch;
        float4 v[kFillChunks];
        int lo[kFillChunks], e0[kFillChunks];
        int r = div_rows(tid, nch, 1.0f / (float)nch);
        int c = tid - r * nch;
        asm volatile("" : "+v"(r), "+v"(c));
        const int dr = kConeBlock / nch, dc = kConeBlock - (kConeBlock / nch) * nch;
#pragma unroll
        for (int k = 0; k < kFillChunks; ++k) {
            const int rr = min(r, nrows - 1);
            const int grow = tile ? desc[rr].x : (int)it.node_start + rr;
            const uint64_t g = (uint64_t)grow * p;
            const int al = (int)(g & 3);
            int e = 4 * c - al;
            if (k * kConeBlock + tid >= totalc) e = p;       // inactive chunk
            if (e < p) v[k] = *reinterpret_cast<const float4*>(src + (g - al) + 4 * c);
            lo[k] = rr * p4;
            e0[k] = e;
            r += dr;
            c += dc;
            if (c >= nch) {
                c -= nch;
                ++r;
            }
        }
#pragma unroll
        for (int k = 0; k < kFillChunks; ++k) {
            const int e = e0[k];
            float* row = data + lo[k];
            if ((unsigned)e < (unsigned)p) row[e] = v[k].x;
            if ((unsigned)(e + 1) < (unsigned)p) row[e + 1] = v[k].y;
            if ((unsigned)(e + 2) < (unsigned)p) row[e + 2] = v[k].z;
            if ((unsigned)(e + 3) < (unsigned)p) row[e + 3] = v[k].w;
        }
    }
    __syncthreads();
    RT_STAMP(1);

    // ---- merge levels, deepest first.  Two barriers per level: the row
    // descriptors of level l-1 are built while level l is written back.
    // Descriptor of output row r of level l: (head row | tail row << 16) in
    // floats, and the roll shift (transforms.hpp:13-27).
    auto build_desc = [&](int l) {
        const int orows = tile ? lv_rows[l] : (int)it.node_size;
        for (int r = tid; r < orows; r += kConeBlock) {
            int hrow, trow = -1, shift = 0;
            if (tile) {
                const Range R = ranges[find_range(ranges, lv_first[l], lv_count[l], r)];
                const int u = R.lo + (r - R.base);
                const Range H = ranges[R.child];
                if (R.size <= 1) {
                    hrow = H.base + (u - H.lo);
                } else {
                    const Range T = ranges[R.child + 1];
                    const int sh = R.size >> 1, st = R.size - sh;
                    const int h = (int)merge_index(merge_coef((uint32_t)sh, (uint32_t)R.size), (uint32_t)u);
                    const int t = (int)merge_index(merge_coef((uint32_t)st, (uint32_t)R.size), (uint32_t)u);
                    hrow = H.base + (h - H.lo);
                    trow = T.base + (t - T.lo);
                    shift = (u - t) % p;
                }
            } else {
                int a0 = 0, sz = (int)it.node_size;
                for (int d = 0; d < l; ++d) {
                    if (sz > 1) {
                        const int hs = sz >> 1;
                        if (r - a0 < hs) sz = hs;
                        else { a0 += hs; sz -= hs; }
                    }
                }
                if (sz <= 1) {
                    hrow = r;
                } else {
                    const int s = r - a0;
                    const int sh = sz >> 1, st = sz - sh;
                    const int h = (int)merge_index(merge_coef((uint32_t)sh, (uint32_t)sz), (uint32_t)s);
                    const int t = (int)merge_index(merge_coef((uint32_t)st, (uint32_t)sz), (uint32_t)s);
                    hrow = a0 + h;
                    trow = a0 + sh + t;
                    shift = (s - t) % p;
                }
            }
            const int ho = hrow * p4;
            const int to = trow < 0 ? zrow : trow * p4;
            desc[r] = make_int2(ho | (to << 16), shift);
        }
    };
    for (int i = tid; i < p4; i += kConeBlock) data[zrow + i] = -0.0f;
    if (L > 0) build_desc(L - 1);
    __syncthreads();
    RT_STAMP(2);
    for (int l = L - 1; l >= 0; --l) {
        const int orows = tile ? lv_rows[l] : (int)it.node_size;
        // Quads: lane-owned groups of 4 consecutive phase bins of one row (rows
        // are padded to p4).  H is one aligned ds_read_b128, the rolled T four
        // ds_read_b32, the result one ds_write_b128; pad columns carry garbage
        // that only ever flows into pad columns.
        const int totalq = orows * qpr;
        float4 v[kQuadsPerThread];
        int r = div_rows(tid, qpr, 1.0f / (float)qpr);
        int q = tid - r * qpr;
        // opaque per level: stops LICM from hoisting all per-quad indices out
        // of the level loop (which spills the register file)
        asm volatile("" : "+v"(r), "+v"(q));
        const int dr = kConeBlock / qpr, dq = kConeBlock - (kConeBlock / qpr) * qpr;
        const int last_row = orows - 1;
#pragma unroll
        for (int g = 0; g < kQuadsPerThread; g += kMergeGroup) {
            if (g * kConeBlock < totalq) {         // uniform: whole group inactive otherwise
#pragma unroll
                for (int j = 0; j < kMergeGroup && g + j < kQuadsPerThread; ++j) {
                    const int2 d = desc[min(r, last_row)];
                    const int ho = d.x & 0xFFFF;
                    const int to = (int)((unsigned)d.x >> 16);
                    const int col = q << 2;
                    const float4 hv = data4[(ho + col) >> 2];   // ho, col multiples of 4
                    int c0 = col + d.y;
                    c0 = c0 >= p ? c0 - p : c0;
                    int c1 = c0 + 1, c2 = c0 + 2, c3 = c0 + 3;
                    c1 = c1 >= p ? c1 - p : c1;
                    c2 = c2 >= p ? c2 - p : c2;
                    c3 = c3 >= p ? c3 - p : c3;
                    // carried rows point `to` at the -0.0 row: x + (-0.0) == x exactly
                    v[g + j] = make_float4(__fadd_rn(hv.x, data[to + c0]), __fadd_rn(hv.y, data[to + c1]),
                                           __fadd_rn(hv.z, data[to + c2]), __fadd_rn(hv.w, data[to + c3]));
                    r += dr;
                    q += dq;
                    const bool wrap = q >= qpr;
                    q = wrap ? q - qpr : q;
                    r = wrap ? r + 1 : r;
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < kQuadsPerThread; g += kMergeGroup) {
            if (g * kConeBlock < totalq) {
#pragma unroll
                for (int j = 0; j < kMergeGroup && g + j < kQuadsPerThread; ++j) {
                    const int qi = (g + j) * kConeBlock + tid;
                    if (qi < totalq) data4[qi] = v[g + j];
                }
            }
        }
        if (l > 0) build_desc(l - 1);
        __syncthreads();
        RT_STAMP(3);
        nrows = orows;
    }

    // ---- output: tile rows [s0, s0 + nrows) of the node, one contiguous
    // global segment written in aligned float4 chunks (segment-end chunks
    // element-wise).  Chunk c holds segment elements e = 4c + j - al.
    if (it.dst != kSelSnr) {
        const uint64_t g0 = (uint64_t)(it.node_start + it.s0) * p;
        const int al = (int)(g0 & 3);
        float* dst = (it.dst == kSelPing ? a.ping : a.pong) + trial * a.buf_stride + X.buf_off + (g0 - al);
        const int total = nrows * p;
        const int totalc = (total + al + 3) >> 2;
        float4 v[kFillChunks];
        // (row, col) of element e = 4*tid - al, stepped by 4*kConeBlock per chunk
        int e = 4 * tid - al;
        int r = e < 0 ? -1 : div_rows(e, p, inv_p);
        int col = e - r * p;
        asm volatile("" : "+v"(r), "+v"(col));
        constexpr int kStep = 4 * kConeBlock;
        const int dr = kStep / p, dc = kStep - (kStep / p) * p;
#pragma unroll
        for (int k = 0; k < kFillChunks; ++k) {
            if (k * kConeBlock + tid < totalc) {
                float x[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    int cj = col + j, rj = r;
                    if (cj >= p) {
                        cj -= p;
                        ++rj;
                    }
                    if (p < 4) {                 // uniform: several wraps inside a chunk
                        while (cj >= p) {
                            cj -= p;
                            ++rj;
                        }
                    }
                    const int ej = e + j;
                    x[j] = data[((unsigned)ej < (unsigned)total) ? rj * p4 + cj : 0];
                }
                v[k] = make_float4(x[0], x[1], x[2], x[3]);
            }
            e += kStep;
            r += dr;
            col += dc;
            if (col >= p) {
                col -= p;
                ++r;
            }
        }
#pragma unroll
        for (int k = 0; k < kFillChunks; ++k) {
            const int ci = k * kConeBlock + tid;
            if (ci < totalc) {
                const int eb = 4 * ci - al;
                if (eb >= 0 && eb + 3 < total) {
                    *reinterpret_cast<float4*>(dst + 4 * ci) = v[k];
                } else {
                    if ((unsigned)eb < (unsigned)total) dst[4 * ci] = v[k].x;
                    if ((unsigned)(eb + 1) < (unsigned)total) dst[4 * ci + 1] = v[k].y;
                    if ((unsigned)(eb + 2) < (unsigned)total) dst[4 * ci + 2] = v[k].z;
                    if ((unsigned)(eb + 3) < (unsigned)total) dst[4 * ci + 3] = v[k].w;
                }
            }
        }
        RT_STAMP(4);
#ifdef RT_STAMPS
        if (tid == 0) atomicAdd(&a.stamps[7], 1ull);
#endif
        return;
    }

    // ---- fused boxcar S/N epilogue (snr.hpp:37-65) on the root's rows s < rows_eval
    const int nev = (int)min((int64_t)nrows, (int64_t)X.rows_eval - (int64_t)it.s0);
    if (nev <= 0) return;
    // G lanes per row (G in 8..64, the smallest with ceil(p/G) <= kSnrChunk),
    // each lane a chunk of c <= kSnrChunk columns held in registers; c is odd so
    // the G chunks of a row hit distinct LDS banks.  fp64 prefix: sequential in
    // the chunk + log2(G)-step segmented scan (kernels.hpp:73-86).
    int G = 8;
    while (G < 64 && ((((p + G - 1) / G) | 1) > kSnrChunk)) G <<= 1;
    int c = (p + G - 1) / G;
    if (c < kSnrChunk) c |= 1;
    const int g = lane & (G - 1);
    const int j0 = min(g * c, p);
    const int cnt = min(j0 + c, p) - j0;          // columns of this lane (may be 0)
    const int owner = (p - 1) / c;
    const int rows_per_pass = kConeBlock / G;
    const uint32_t nw = a.num_widths;
    float* snr = a.snr + trial * a.snr_stride + (X.snr_row + it.s0) * (uint64_t)nw;
    if (c <= kSnrChunk) {
        for (int base = 0; base < nev; base += rows_per_pass) {
            const int r = base + (tid / G);
            const bool active = r < nev;
            float* row = data + min(r, nev - 1) * p4 + j0;
            const int last = max(cnt - 1, 0);
            float cp[kSnrChunk];
            // branch-free: every lane issues all kSnrChunk reads (clamped to its
            // chunk), values past the chunk are masked
#pragma unroll
            for (int i = 0; i < kSnrChunk; ++i) {
                const float x = row[min(i, last)];
                cp[i] = i < cnt ? x : 0.0f;
            }
            double part = 0.0;
#pragma unroll
            for (int i = 0; i < kSnrChunk; ++i) {
                const double t = part + (double)cp[i];
                part = i < cnt ? t : part;
            }
            double incl = part;
            for (int d = 1; d < G; d <<= 1) {
                const double y = __shfl_up(incl, d, G);
                if (g >= d) incl += y;
            }
            double acc = __shfl_up(incl, 1, G);
            if (g == 0) acc = 0.0;
#pragma unroll
            for (int i = 0; i < kSnrChunk; ++i) {
                const double t = acc + (double)cp[i];
                acc = i < cnt ? t : acc;
                cp[i] = (float)acc;
            }
            const float sum = __shfl((float)acc, owner, G);
            if (active) {
#pragma unroll
                for (int i = 0; i < kSnrChunk; ++i)
                    if (i < cnt) row[i] = cp[i];
            }
            __syncthreads();                      // prefix rows visible to all lanes
            const float* crow = data + min(r, nev - 1) * p4;
            for (uint32_t iw = 0; iw < nw; ++iw) {
                const int w = wl[iw];
                float dmax = -INFINITY;
                constexpr int kB = 11;                    // reads in flight per batch
                static_assert(kSnrChunk % kB == 0, "batching");
#pragma unroll
                for (int b0 = 0; b0 < kSnrChunk; b0 += kB) {
                    float lv[kB];
#pragma unroll
                    for (int t = 0; t < kB; ++t) {
                        const int k = j0 + min(b0 + t, last) + w;
                        lv[t] = crow[k >= p ? k - p : k];
                    }
#pragma unroll
                    for (int t = 0; t < kB; ++t) {
                        const int i = b0 + t;
                        const bool wrap = j0 + min(i, last) + w >= p;
                        const float ck = wrap ? __fadd_rn(lv[t], sum) : lv[t];
                        const float d = __fsub_rn(ck, cp[i]);
                        dmax = (i < cnt && d > dmax) ? d : dmax;  // diff_max, kernels.hpp:50-60
                    }
                }
                for (int o = G >> 1; o > 0; o >>= 1) {
                    const float y = __shfl_xor(dmax, o, G);
                    dmax = y > dmax ? y : dmax;
                }
                if (active && g == 0) {
                    const float h = sqrtf((float)(p - w) / (float)(p * w));
                    const float b = (float)w / (float)(p - w) * h;
                    snr[(uint64_t)r * nw + iw] = ((h + b) * dmax - b * sum) / X.stdnoise;
                }
            }
        }
    } else {
        // very wide rows (p > 64 * kSnrChunk): one wave per row, chunks from LDS
        for (int base = 0; base < nev; base += kConeBlock / 64) {
            const int r = base + wave;
            const bool active = r < nev;
            float* row = data + min(r, nev - 1) * p4;
            double part = 0.0;
            for (int j = j0; j < j0 + cnt; ++j) part += (double)row[j];
            double incl = part;
            for (int d = 1; d < 64; d <<= 1) {
                const double y = __shfl_up(incl, d, 64);
                if (g >= d) incl += y;
            }
            double acc = __shfl_up(incl, 1, 64);
            if (g == 0) acc = 0.0;
            __syncthreads();
            if (active)
                for (int j = j0; j < j0 + cnt; ++j) {
                    acc += (double)row[j];
                    row[j] = (float)acc;
                }
            const float sum = __shfl((float)acc, owner, 64);
            __syncthreads();
            for (uint32_t iw = 0; iw < nw; ++iw) {
                const int w = (int)a.widths[iw];
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
                    snr[(uint64_t)r * nw + iw] = ((h + b) * dmax - b * sum) / X.stdnoise;
                }
            }
            __syncthreads();
        }
    }
    RT_STAMP(5);
#ifdef RT_STAMPS
    if (tid == 0) atomicAdd(&a.stamps[7], 1ull);
#endif
}

hipError_t launch_cone(const ConeArgs& args, uint32_t batch, hipStream_t s)
{
    if (!args.num_items || !batch) return hipSuccess;
    hipLaunchKernelGGL(cone_kernel, dim3(args.num_items, batch), dim3(kConeBlock), 0, s, args);
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
