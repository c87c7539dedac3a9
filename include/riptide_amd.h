/*
 * riptide_amd.h -- C ABI of the MI355X-native FFA periodogram engine.
 *
 * This is the drop-in boundary for riptide's native module `riptide.libcpp`
 * (pybind11, /root/reference/riptide/cpp/python_bindings.cpp:213-267).  Each
 * host-buffer entry point below replaces one binding of that module, with the
 * same argument meaning, output shape/dtype and error text; the Python shim
 * riptide_amd/libcpp.py (or the ctypes stub in INTEGRATION.md) maps them onto
 * the reference's function names.  All compute runs in HIP kernels on the
 * current device; there is no CPU compute path.
 *
 * Conventions
 *  - Return value: RT_OK (0) on success; RT_EINVAL for the cases where the
 *    reference throws std::invalid_argument / std::domain_error (Python
 *    ValueError); RT_EHIP for a HIP runtime failure; RT_EINTERNAL otherwise.
 *    rt_last_error() returns the message of the calling thread's last failure
 *    (the reference's exception text for RT_EINVAL).
 *  - "host" pointers are ordinary CPU memory (numpy buffers); "device"
 *    pointers are HIP device memory; `stream` is a hipStream_t (NULL = the
 *    library's own stream).  Host-buffer calls are synchronous.
 *  - Widths are uint64 (size_t in the reference).
 */
#ifndef RIPTIDE_AMD_H
#define RIPTIDE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_EINVAL 1
#define RT_EHIP 2
#define RT_EINTERNAL 3

const char* rt_last_error(void);
/* Version string of the engine and the gfx target it was built for. */
const char* rt_version(void);
/* Select the HIP device used by subsequent host-buffer calls of this thread. */
int rt_set_device(int device);

/* ---------------- host-buffer drop-ins for riptide.libcpp ----------------- */

/* python_bindings.cpp:32-40  rollback(x, shift): out = roll(x, -shift) */
int rt_rollback(const float* x, size_t size, size_t shift, float* out);

/* python_bindings.cpp:43-58  fused_rollback_add(x, y, shift): out = x + roll(y, -shift) */
int rt_fused_rollback_add(const float* x, const float* y, size_t size, size_t shift, float* out);

/* python_bindings.cpp:61-69  circular_prefix_sum(x, nsum): out has nsum elements */
int rt_circular_prefix_sum(const float* x, size_t size, size_t nsum, float* out);

/* python_bindings.cpp:72-84  ffa2(data[rows, cols]) -> out[rows, cols] */
int rt_ffa2(const float* in, size_t rows, size_t cols, float* out);

/* python_bindings.cpp:87-106  benchmark_ffa2(rows, cols, loops) -> seconds per loop
 * (device-resident zero input, HIP-event timed) */
int rt_benchmark_ffa2(size_t rows, size_t cols, size_t loops, double* seconds);

/* python_bindings.cpp:109-126  snr1(data[size], widths, stdnoise) -> out[num_widths] */
int rt_snr1(const float* x, size_t size, const uint64_t* widths, size_t num_widths, float stdnoise, float* out);

/* python_bindings.cpp:129-148  snr2(data[rows, cols], widths, stdnoise) -> out[rows, num_widths] */
int rt_snr2(const float* x, size_t rows, size_t cols, const uint64_t* widths, size_t num_widths,
            float stdnoise, float* out);

/* downsample.hpp:21-24  floor(size / f) */
size_t rt_downsampled_size(size_t size, double f);

/* python_bindings.cpp:151-165  downsample(data, factor) -> out[rt_downsampled_size(size, factor)] */
int rt_downsample(const float* x, size_t size, double factor, float* out);
/* Row-wise downsampling of a rows x size array by the same factor: rows x
 * downsampled_size(size, f) floats (the batched form folding.py's
 * downsample_vertical needs; same arithmetic as rt_downsample). */
int rt_downsample_rows(const float* x, size_t rows, size_t size, double f, float* out);

/* periodogram.hpp:63-109  number of trial periods (validates arguments) */
int rt_periodogram_length(size_t size, double tsamp, double period_min, double period_max,
                          size_t bins_min, size_t bins_max, size_t* length);

/* python_bindings.cpp:168-197  periodogram(data, tsamp, widths, period_min, period_max,
 * bins_min, bins_max) -> periods[L] (f64), foldbins[L] (u32), snrs[L, num_widths] (f32) */
int rt_periodogram(const float* data, size_t size, double tsamp, const uint64_t* widths, size_t num_widths,
                   double period_min, double period_max, size_t bins_min, size_t bins_max,
                   double* periods, uint32_t* foldbins, float* snrs);

/* python_bindings.cpp:200-210  running_median(data, width) -> out[size] */
int rt_running_median(const float* x, size_t size, size_t width, float* out);

/* running_medians.py:49-83 fast_running_median(data, width_samples, min_points) for a
 * scrunch factor > 1: float32 block means, exact running median of width
 * min_points, np.interp back to full resolution -> out[size] (float64).  A
 * scrunch factor of 1 is rt_running_median (the reference returns float32 then). */
int rt_fast_running_median(const float* x, size_t size, size_t width_samples, size_t min_points, double* out);

/* time_series.py:93-122 + :66-90 (TimeSeries.deredden(width_samples, minpts) then
 * .normalise()), one series; either stage may be skipped. width_samples is
 * int(round(rmed_width / tsamp)) computed by the caller (Python round). */
int rt_deredden_normalise(const float* x, size_t size, size_t width_samples, size_t min_points,
                          int deredden, int normalise, float* out);

/* periodogram.hpp:190-194  trial-period grid only (host computation, no device) */
int rt_periodogram_grid(size_t size, double tsamp, double period_min, double period_max, size_t bins_min,
                        size_t bins_max, double* periods, uint32_t* foldbins);

/* Host-only: build the FFA pass schedule for a periodogram and verify its
 * invariants (tiles inside nodes, LDS budget, final pass covers every row). */
int rt_schedule_check(size_t size, double tsamp, size_t num_widths, double period_min, double period_max,
                      size_t bins_min, size_t bins_max, uint64_t* transforms, uint64_t* items,
                      uint64_t* launches, double* alg_bytes_per_trial, double* moved_bytes_per_trial,
                      uint64_t* cells_per_trial);

/* Host-only: the downsampling-ladder kernel a periodogram plan of these
 * parameters runs (periodogram.hpp:162-168 restated per rung): *fused = 1
 * for the one-read fused ladder (32-bit sample indices: series below 2^29
 * samples, every rung's window inside its staging margin), 2 for the fused
 * ladder over the rungs inside the margin plus the per-rung kernel for the
 * wider ones, 0 for the per-rung kernel alone (64-bit indices); *rungs =
 * rungs that feed a transform.  Either pointer may be NULL. */
int rt_ladder_check(size_t size, double tsamp, double period_min, double period_max, size_t bins_min,
                    size_t bins_max, int* fused, uint64_t* rungs);

/* The pass schedule rt_ffa2 runs for one rows x cols transform, built and
 * validated on the host only (validate_exec_plan: tiles, LDS budgets, unit
 * blobs, DMA segments, row slots); no device needed.  *launches may be NULL. */
int rt_ffa_schedule_check(size_t rows, size_t cols, uint64_t* launches);

/* ------------------ device-resident batched hot path ---------------------- */

typedef struct rt_plan rt_plan;

/* Build the periodogram plan (ladder, grid, pass schedule) once per
 * (size, tsamp, widths, period range, bins range).  Validates like
 * periodogram.hpp:25-40 and snr.hpp:21-31 (widths < bins_min). */
int rt_plan_create(size_t size, double tsamp, const uint64_t* widths, size_t num_widths,
                   double period_min, double period_max, size_t bins_min, size_t bins_max,
                   rt_plan** plan);
void rt_plan_destroy(rt_plan* plan);
/* L (number of trial periods) and W (number of widths). */
int rt_plan_shape(const rt_plan* plan, size_t* length, size_t* num_widths);
/* Host copy of the trial-period grid (bit-exact with the reference). */
int rt_plan_grid(const rt_plan* plan, double* periods, uint32_t* foldbins);
/* Device workspace bytes needed to process `batch` trials per call. */
int rt_plan_workspace_bytes(const rt_plan* plan, size_t batch, size_t* bytes);

/* Periodogram S/N of `batch` series resident in device memory.
 *   d_data  : batch x size floats, series b at d_data + b * data_stride
 *   d_snrs  : batch x (L * W) floats, trial b at d_snrs + b * snr_stride
 * The series must already be dereddened/normalised as the caller wants
 * (rt_deredden_normalise_device).  Stream-ordered, no host synchronisation. */
int rt_periodogram_device(const rt_plan* plan, const float* d_data, size_t batch, size_t data_stride,
                          float* d_snrs, size_t snr_stride, void* d_workspace, size_t workspace_bytes,
                          void* stream);
/* rt_periodogram_device in two stream-ordered halves, so a pipelined caller
 * can run batch k + 1's downsampling ladder (periodogram.hpp:162-168) on one
 * stream while batch k's FFA passes + S/N run on another: the ladder fills
 * the workspace's leaf buffer, the passes read it (same workspace, same
 * batch).  ladder then passes == rt_periodogram_device. */
int rt_periodogram_ladder_device(const rt_plan* plan, const float* d_data, size_t batch, size_t data_stride,
                                 void* d_workspace, size_t workspace_bytes, void* stream);
int rt_periodogram_passes_device(const rt_plan* plan, size_t batch, float* d_snrs, size_t snr_stride,
                                 void* d_workspace, size_t workspace_bytes, void* stream);

/* Device error flag of a plan: the cone kernel refuses (and leaves unwritten)
 * any work unit that breaks its LDS / register budget and raises the plan's
 * sticky flag.  Reads it on `stream` (synchronising that stream), clears it,
 * and returns RT_EINTERNAL if it was set.  The reference has no such state
 * (a CPU transform cannot run out of LDS); the host entry point
 * rt_periodogram checks it itself, as riptide::periodogram
 * (periodogram.hpp:117-201) would raise. */
int rt_plan_check(const rt_plan* plan, void* stream);

/* Device workspace bytes for rt_deredden_normalise_device. */
int rt_deredden_workspace_bytes(size_t size, size_t width_samples, size_t min_points, size_t batch,
                                size_t* bytes);
/* Batched dereddening + normalisation in device memory (d_out may equal d_in
 * only when deredden == 0). */
int rt_deredden_normalise_device(const float* d_in, size_t size, size_t batch, size_t in_stride,
                                 size_t width_samples, size_t min_points, int deredden, int normalise,
                                 float* d_out, size_t out_stride, void* d_workspace, size_t workspace_bytes,
                                 void* stream);

/* ------------------------- peak detection (device) ------------------------ */
/* The data-parallel stages of riptide.peak_detection.find_peaks
 * (peak_detection.py:37-142) over a batch of device periodograms in the
 * rt_periodogram_device layout (trial b at d_snrs + b * snr_stride, L x W
 * row-major).  The host finishes each stage with numpy's own expressions
 * (percentile lerp, polyfit, cluster1d), so the peaks are identical.
 *
 * Order statistics of every (trial, width, segment): segment k covers rows
 * [k * per_seg, (k + 1) * per_seg) (segment_stats, peak_detection.py:71-82);
 * d_out[((b * W + iw) * nseg + k) * nranks + r] = the ranks[r]-th smallest S/N
 * of the segment (NaN if the segment holds a NaN).  per_seg <= 32768. */
int rt_segment_order_stats_device(const float* d_snrs, size_t batch, size_t snr_stride, size_t length,
                                  size_t num_widths, size_t nseg, size_t per_seg, const uint32_t* ranks,
                                  size_t nranks, float* d_out, void* stream);
/* Threshold selection (peak_detection.py:131-133): row i of (trial b, width
 * iw) is selected when s > polyval(coeffs[b][iw], logf[i]) and s > smin
 * (fp64, s = float64 of the S/N).  d_coeffs: batch x W x ncoef doubles,
 * highest degree first (np.poly1d order); d_logf: L doubles (np.log of the
 * trial frequencies).  Selected rows are appended, in no particular order, to
 * d_idx[(b * W + iw) * cap ...] and counted in d_counts[b * W + iw] (zeroed
 * by the call); a count above cap means the list was truncated. */
int rt_threshold_select_device(const float* d_snrs, size_t batch, size_t snr_stride, size_t length,
                               size_t num_widths, const double* d_logf, const double* d_coeffs, size_t ncoef,
                               double smin, uint32_t* d_counts, uint32_t* d_idx, size_t cap, void* stream);

/* --------------------------- file input (device) --------------------------- */
/* 8-bit SIGPROC samples (riptide/time_series.py:352-357) to float32 in device
 * memory: d_raw holds n bytes, int8 when is_signed else uint8; exact as
 * numpy's astype(np.float32).  d_raw must be 4-byte aligned. */
int rt_convert_samples_device(const void* d_raw, size_t n, int is_signed, float* d_out, void* stream);

/* ----------------------------- profiling ---------------------------------- */
/* When enabled, rt_periodogram_device records HIP events around every cone
 * (FFA pass) launch and accumulates their time and algorithmic bytes
 * (4mp read + 4mp or 4*rows_eval*W written per pass). */
int rt_profile_enable(int on);
/* kind: 0 = FFA cone passes, 1 = downsample ladder.  Synchronises the events. */
int rt_profile_read(int kind, double* milliseconds, double* alg_bytes, double* moved_bytes, uint64_t* launches);
int rt_profile_reset(void);

/* Diagnostics (meaningful in the -DRT_STAMPS build, libriptide_amd_stamps.so):
 * cone-kernel cycles per phase summed over work items -- [0] prologue,
 * [1] bottom-level fill, [2] row descriptors, [3] merge levels, [4] store,
 * [5] fused S/N, [7] items.  The first call allocates the counters. */
int rt_diag_stamps(uint64_t* out8, int reset);
/* Diagnostic builds: per-unit timeline records (8 words each: hw id | xcc << 32,
 * start, setup done, fill landed, merge done, end, unit, shape), up to cap. */
int rt_diag_timeline(uint64_t* out, uint64_t cap, uint64_t* count);
/* Diagnostic builds: index of each cone launch's first timeline record (one
 * entry per launch since the last rt_diag_stamps reset), up to cap. */
int rt_diag_launches(uint64_t* out, uint64_t cap, uint64_t* count);

/* Plan statistics: transforms, work items, passes, cone launches per trial. */
int rt_plan_stats(const rt_plan* plan, uint64_t* transforms, uint64_t* items, uint64_t* launches,
                  double* alg_bytes_per_trial, double* moved_bytes_per_trial, uint64_t* cells_per_trial);


#ifdef __cplusplus
}
#endif

#endif /* RIPTIDE_AMD_H */
