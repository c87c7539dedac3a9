// Launch wrappers of the HIP kernels (host-callable, stream-ordered, no sync).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "common.hpp"

namespace rt {

constexpr uint32_t kDsSpanFloats = 4096;   // LDS input stage of the ladder kernels (16 KiB)
constexpr uint32_t kDsFusedMargin = 512;   // fused ladder: staged floats past the span (rungs with ceil(f) + 2 <= margin)
constexpr uint32_t kDsMaxRungs = 256;      // fused ladder: rungs per plan (per-block rung ranges in LDS)

struct DsRung {
    double f;
    uint64_t n;          // output samples of this rung
    uint64_t out_off;    // float offset in the per-trial leaf buffer
    uint32_t first_block;
    uint32_t identity;   // f == 1: plain copy
    uint32_t per_block;  // outputs per block (input span of a block <= kDsSpanFloats)
    uint32_t staged;     // 0: f too large to stage a block's span in LDS, read global memory
};

// Outputs per block of the ladder kernel for factor f (0: cannot stage).
inline uint32_t ds_per_block(double f)
{
    const double o = std::floor((double)(kDsSpanFloats - 4) / (f + 1.0)) - 1.0;
    if (o < 1.0) return 0;
    return o > 256.0 ? 256u : (uint32_t)o;
}

// A block stages its span in LDS when that leaves it >= 32 outputs (f below
// ~123); a wider rung's block of 256 outputs reads each window from global
// memory (a staged block of 1-31 outputs left 225-255 of its threads idle
// behind one span load: cfg5's long range, f up to ~1950).
inline void ds_configure(DsRung& r)
{
    const uint32_t o = r.identity ? 256u : ds_per_block(r.f);
    r.staged = o >= 32;
    r.per_block = r.staged ? o : 256u;
}

// ffa_kernels.hip
hipError_t launch_downsample_ladder(const float* x, uint64_t n_in, uint64_t x_stride,
                                    const DsRung* d_rungs, uint32_t num_rungs, uint32_t total_blocks,
                                    float* out, uint64_t out_stride, uint32_t batch, hipStream_t s);
// all rungs of a periodogram from one read of the series; margin: samples
// staged past each span, ds_fused_margin(rungs) (every rung: ceil(f) + 2 <= margin <= kDsFusedMargin)
hipError_t launch_downsample_fused(const float* x, uint64_t n_in, uint64_t x_stride, const DsRung* d_rungs,
                                   uint32_t num_rungs, uint32_t margin, float* out, uint64_t out_stride,
                                   uint32_t batch, hipStream_t s);

// The fused ladder's margin for a plan's rungs: ceil(f) + 2 of the largest
// non-identity rung, rounded up to 64 samples (0: a rung needs more than
// kDsFusedMargin -- not fusable).
inline uint32_t ds_fused_margin(const DsRung* rungs, size_t num_rungs)
{
    double need = 2.0;
    for (size_t i = 0; i < num_rungs; ++i)
        if (!rungs[i].identity) need = std::fmax(need, std::ceil(rungs[i].f) + 2.0);
    if (need > (double)kDsFusedMargin) return 0;
    const uint32_t m = ((uint32_t)need + 63u) & ~63u;
    return m < kDsFusedMargin ? m : kDsFusedMargin;
}
// smax: merge_slots() bucket covering every transform of the launch
hipError_t launch_cone(const ConeArgs& args, uint32_t smax, uint32_t rw, bool wide_snr, bool snr,
                       hipStream_t s);   // grid (num_items, batch); rw, wide_snr, snr: the Launch's
hipError_t launch_ffa_level(const float* in, float* out, const uint2* d_nodes, uint32_t num_nodes,
                            uint32_t rows, uint32_t p, hipStream_t s);

// peaks_kernels.hip
constexpr int kMaxSegmentPoints = 32768;  // rows of one peak-detection segment sorted in LDS (128 KiB)
constexpr int kMaxSegmentRanks = 8;       // order statistics per segment (host ranks array)
hipError_t launch_segment_order_stats(const float* snrs, uint64_t snr_stride, uint32_t batch, uint32_t W,
                                      uint32_t nseg, uint32_t per_seg, const uint32_t* ranks, uint32_t nranks,
                                      float* out, hipStream_t s);
hipError_t launch_threshold_select(const float* snrs, uint64_t snr_stride, uint32_t batch, uint32_t L, uint32_t W,
                                   const double* logf, const double* coeffs, uint32_t ncoef, double smin,
                                   uint32_t* counts, uint32_t* idx, uint32_t cap, hipStream_t s);

hipError_t launch_convert_samples(const void* raw, uint64_t n, int is_signed, float* out, hipStream_t s);

// aux_kernels.hip
hipError_t launch_snr_rows(const float* x, uint64_t rows, uint32_t cols, const uint32_t* d_widths,
                           uint32_t nw, float stdnoise, float* cps_scratch, float* out, hipStream_t s);
hipError_t launch_running_median(const float* x, uint64_t n, uint32_t width, float* out, uint64_t x_stride,
                                 uint64_t out_stride, uint32_t batch, hipStream_t s);
hipError_t launch_scrunch(const float* x, uint64_t n_out, uint32_t factor, float* out, uint64_t x_stride,
                          uint64_t out_stride, uint32_t batch, hipStream_t s);
hipError_t launch_deredden_subtract(const float* x, uint64_t n, const float* rmed_lo, uint64_t n_lo,
                                    uint32_t factor, float* out, uint64_t x_stride, uint64_t lo_stride,
                                    uint64_t out_stride, uint32_t batch, hipStream_t s, double* slopes = nullptr);
// dereddening + normalisation with the normalisation's statistics summed by
// the dereddening kernel (no read pass of their own).  Applies when
// dered_norm_fusable(); partials: batch * 2 * dered_norm_blocks(n) doubles,
// stats: 2 * batch doubles.
inline uint64_t dered_norm_blocks(uint64_t n) { return (n + 4095) / 4096; }   // 4096 samples per block
bool dered_norm_fusable(const float* x, uint64_t n, uint64_t n_lo, uint32_t factor, const float* out,
                        uint64_t x_stride, uint64_t out_stride);
hipError_t launch_deredden_normalise(const float* x, uint64_t n, const float* rmed_lo, uint64_t n_lo,
                                     uint32_t factor, float* out, uint64_t x_stride, uint64_t lo_stride,
                                     uint64_t out_stride, uint32_t batch, hipStream_t s, double* slopes,
                                     double* partials, double* stats);
hipError_t launch_interp(uint64_t n, const float* rmed_lo, uint64_t n_lo, uint32_t factor, double* out,
                         hipStream_t s);
hipError_t launch_normalise(const float* x, uint64_t n, float* out, double* d_partials, uint32_t nblocks,
                            uint64_t x_stride, uint64_t out_stride, uint32_t batch, hipStream_t s);
hipError_t launch_rollback(const float* x, uint64_t n, uint64_t shift, const float* y, float* out, hipStream_t s);
hipError_t launch_circular_prefix_sum(const float* x, uint64_t n, uint64_t nsum, float* out, hipStream_t s);

}  // namespace rt
