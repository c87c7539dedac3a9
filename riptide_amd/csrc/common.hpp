// Shared host/device definitions of the MI355X FFA periodogram engine.
//
// Data model: a periodogram is a ladder of rungs (downsampling
// factors f); each rung contributes one FFA transform per phase-bin count
// B in [bins_min, bstop].  A transform of m rows x p (= B) columns is evaluated
// as a sequence of *passes*; each pass is one launch of the cone kernel over a
// list of work items (one workgroup each).
//
//   pass 0  ("whole" items): every node of the FFA split tree at depth d_b is
//           small enough (<= C rows) to be transformed entirely in LDS, from
//           the leaves (rows of the downsampled series) up.
//   pass k  ("tile" items):  K consecutive output rows of a node at depth d,
//           computed from the rows they depend on L levels below (their
//           dependency cone), again entirely in LDS.
//
// The last pass of a transform fuses the boxcar S/N scan (snr.hpp:37-65) on the
// rows it produced, so the transform output never returns to HBM.
#pragma once
#include <cstddef>
#include <cstdint>

#if defined(__HIPCC__)
#define RT_HD __host__ __device__
#else
#define RT_HD
#endif

namespace rt {

// ---- cone kernel geometry (gfx950: 160 KiB LDS per CU, one workgroup per CU)
constexpr int kConeBlock = 512;             // 8 waves, 2 workgroups per CU
constexpr int kLdsDataFloats = 16384;       // 64 KiB level buffer
constexpr int kMaxRows = 512;               // rows per level held in LDS (row descriptors)
constexpr int kMaxTileLevels = 6;           // L for tile items
constexpr int kMaxRanges = (1 << (kMaxTileLevels + 1)) - 1;
constexpr int kMaxWholeLevels = 11;         // ceil(log2(kMaxRows)) + 1
constexpr int kMaxWidths = 32;           // boxcar widths handled by the fused S/N epilogue
constexpr int kRegsPerThread = (kLdsDataFloats + kConeBlock - 1) / kConeBlock;
constexpr int kSnrChunk = 33;             // S/N epilogue: columns per lane held in registers
constexpr int kMergeGroup = 8;             // elements per thread with LDS reads in flight together

constexpr int kQuadsPerThread = (kLdsDataFloats / 4 + kConeBlock - 1) / kConeBlock;
// float4 chunks per thread of the fill/store phases: a level of n rows of
// stride p4 spans at most n*p4/4 + n aligned chunks (one extra per row for
// misalignment), n*p4 < kLdsDataFloats and n <= kMaxRows.
constexpr int kFillChunks = (kLdsDataFloats / 4 + kMaxRows + kConeBlock - 1) / kConeBlock;

// LDS rows are padded to a multiple of 4 floats (16-byte aligned rows) so the
// merge can move 4 phase bins per lane with ds_read_b128 / ds_write_b128.
RT_HD inline int lds_row_stride(uint32_t p) { return (int)((p + 3) & ~3u); }

// Row capacity of the LDS level buffer for p phase bins (one row is kept free
// for the -0.0 row that carried leaves add).
RT_HD inline int lds_row_capacity(uint32_t p)
{
    const int c = kLdsDataFloats / lds_row_stride(p) - 1;
    return c < kMaxRows ? c : kMaxRows;
}

// One FFA transform of a plan ((rung, bins) step of periodogram.hpp:223-269).
struct FfaXform {
    uint32_t p;          // phase bins (= columns)
    uint32_t m;          // rows (= n / p)
    uint32_t rows_eval;  // rows whose S/N is evaluated (periodogram.hpp:253)
    uint32_t rung;
    uint64_t src_off;    // float offset of the leaf rows in the per-trial leaf buffer
    uint64_t buf_off;    // float offset of the scratch rows in ping/pong
    uint64_t snr_row;    // first S/N output row (prefix sum of rows_eval)
    float stdnoise;      // periodogram.hpp:251
    uint32_t pad;
};
static_assert(sizeof(FfaXform) == 48, "FfaXform layout");

enum : uint8_t { kModeWhole = 0, kModeTile = 1 };
enum : uint8_t { kSelLeaves = 0, kSelPing = 1, kSelPong = 2, kSelSnr = 3 };

// One workgroup of one pass.
struct ConeItem {
    uint32_t xform;
    uint32_t node_start;  // first row (within the transform) of the target node
    uint32_t node_size;   // rows of the target node
    uint32_t s0, s1;      // output tile [s0, s1) in node-local rows
    uint8_t levels;       // merge levels evaluated by this item
    uint8_t mode;         // kModeWhole / kModeTile
    uint8_t src;          // kSelLeaves / kSelPing / kSelPong
    uint8_t dst;          // kSelPing / kSelPong / kSelSnr
    uint32_t pad;
};
static_assert(sizeof(ConeItem) == 28, "ConeItem layout");

// Arguments of one cone-kernel launch.  Per-trial strides are in floats.
struct ConeArgs {
    const FfaXform* xf;
    const ConeItem* items;
    uint32_t num_items;
    uint32_t num_widths;
    const float* leaves;
    uint64_t leaves_stride;
    float* ping;
    float* pong;
    uint64_t buf_stride;
    float* snr;
    uint64_t snr_stride;
    uint32_t widths[kMaxWidths];  // boxcar widths (bins)
    int* error_flag;      // set non-zero if a work item violates the LDS budget
    unsigned long long* stamps;   // RT_STAMPS diagnostic builds only: per-phase cycles
};

// Merge index of the FFA recursion (transforms.hpp:17-22): the reference build
// evaluates (size_t)(k * s + 0.5f) with k = (child_rows - 1.0f) / (rows - 1.0f)
// in float32; the fused and unfused forms agree for every rows < 2e5
// (tests/test_oracle_golden.py::test_ffa2_bit_exact).  The fused form is used.
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t merge_index(float k, uint32_t s)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)__builtin_fmaf(k, (float)s, 0.5f);
#else
    return (uint32_t)__builtin_fmaf(k, (float)s, 0.5f);
#endif
}

#if defined(__HIPCC__)
__host__ __device__
#endif
inline float merge_coef(uint32_t child_rows, uint32_t rows)
{
    return ((float)child_rows - 1.0f) / ((float)rows - 1.0f);
}

}  // namespace rt
